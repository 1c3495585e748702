// Device implementation of the temporal-blocked stencil (see stencil_tb.hip
// for the design notes). Included by the per-(dtype, vector width)
// instantiation units tb_*.hip so they compile in parallel.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>
#include <cstdlib>
#include <mutex>
#include <map>

#include "heat2d/kernels.hpp"

namespace heat2d {
namespace kern {
namespace tbimpl {

template <typename T>
struct Vec16;
template <>
struct Vec16<float> {
  using type = float __attribute__((ext_vector_type(4)));
  static constexpr int n = 4;
};
template <>
struct Vec16<double> {
  using type = double __attribute__((ext_vector_type(2)));
  static constexpr int n = 2;
};

// DPP wave shifts (GFX9 family). wave_shr:1 -> lane i reads lane i-1;
// wave_shl:1 -> lane i reads lane i+1. Lanes without a source get 0 (garbage
// by construction: they lie in the strip's redundant halo columns).
constexpr int kDppWaveShl1 = 0x130;
constexpr int kDppWaveShr1 = 0x138;

// bound_ctrl = true: source-less lanes read 0 and no `old` operand has to be
// materialised (saves a v_mov per DPP move).
template <int CTRL>
__device__ __forceinline__ int dpp_mov(int x) {
  return __builtin_amdgcn_mov_dpp(x, CTRL, 0xF, 0xF, true);
}
__device__ __forceinline__ float from_lower(float x) { return __int_as_float(dpp_mov<kDppWaveShr1>(__float_as_int(x))); }
__device__ __forceinline__ float from_upper(float x) { return __int_as_float(dpp_mov<kDppWaveShl1>(__float_as_int(x))); }
__device__ __forceinline__ double from_lower(double x) {
  const long long b = __double_as_longlong(x);
  const int lo = dpp_mov<kDppWaveShr1>((int)(b & 0xffffffffLL));
  const int hi = dpp_mov<kDppWaveShr1>((int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ double from_upper(double x) {
  const long long b = __double_as_longlong(x);
  const int lo = dpp_mov<kDppWaveShl1>((int)(b & 0xffffffffLL));
  const int hi = dpp_mov<kDppWaveShl1>((int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

struct TbArgs {
  int64_t pitch;
  int64_t ncols;
  int64_t col_lo;  // allocation column bounds [col_lo, col_hi)
  int64_t col_hi;
  int64_t row_begin, row_end;
  int64_t nstrips;
  int64_t nbands;  // row bands (work item = band x strip)
  int64_t nwaves;  // launched waves (grid-stride over items)
  int64_t fixed_lo, fixed_hi;  // local rows outside [fixed_lo, fixed_hi) are Dirichlet
};

template <typename T, int NV, int K>
struct TbShape {
  static constexpr int VM = Vec16<T>::n;          // elements per 16-B vector
  static constexpr int V = NV * VM;               // elements per lane
  static constexpr int KA = (K + V - 1) / V * V;  // halo columns: whole lanes (vector stores stay aligned)
  static constexpr int W = 64 * V;
  static constexpr int U = W - 2 * KA;
  static_assert(U > 0, "temporal depth too large for the strip width");
};

// Branch-free memory access: every row load / store goes through a raw buffer
// descriptor whose base is the (wave-uniform) row address; lanes that must not
// touch memory carry an out-of-range voffset, so the hardware range check
// returns 0 / drops the store instead of an exec-masked branch. With no
// memory op under control flow, hipcc's waitcnt pass can count the prefetch
// ring precisely (vmcnt(N>0)) instead of draining it every row.
constexpr int32_t kOob = (int32_t)0x80000000u;


template <typename T>
struct Bits;
template <>
struct Bits<float> {
  using U = unsigned int;
};
template <>
struct Bits<double> {
  using U = unsigned long long;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}

// PF: prefetch depth in units of 3 rows (PF = 2 -> 6 rows in flight per wave).
template <typename T, int NV, int K, bool EDGE, int PF>
struct March {
  using S = TbShape<T, NV, K>;
  static constexpr int V = S::V;
  static constexpr int VM = S::VM;
  using VT = typename Vec16<T>::type;
  using U4 = unsigned int __attribute__((ext_vector_type(4)));

  const char* srow;  // byte address of (row 0, column -cpad) in src   [wave-uniform]
  char* drow;        // same in dst                                      [wave-uniform]
  int64_t pitch_b;   // bytes per row                                    [wave-uniform]
  uint32_t nrec;     // descriptor size (= pitch_b)
  T r;
  int64_t t0, t1;    // output rows
  int64_t fixed_lo, fixed_hi;
  int64_t me;        // end of level-0 rows
  int32_t ld_off;    // per-lane load byte offset (kOob outside the allocation)
  int32_t st_off;    // per-lane vector store offset (kOob unless all V columns are owned output)
  int32_t st_e[EDGE ? V : 1];  // EDGE: per-element store offsets
  unsigned fixmask;  // EDGE: per-element Dirichlet column bits

  T X[3][K][V];      // level state: 3-phase rotating window (SSA after unroll)
  // level-0 prefetch ring: 3*PFJ rows in flight; row m sits in Lb[m%3][0]
  // when consumed, the slot's older entries shift down, row m+3*PFJ lands last
  VT Lb[3][PF][NV];

  template <int PH>
  __device__ __forceinline__ void prefetch_advance(int64_t m) {
#pragma unroll
    for (int j = 0; j + 1 < PF; ++j)
#pragma unroll
      for (int v = 0; v < NV; ++v) Lb[PH][j][v] = Lb[PH][j + 1][v];
    const int64_t nxt = m + 3 * PF;
    load_row(nxt < me ? nxt : me - 1, Lb[PH][PF - 1]);
  }

  __device__ __forceinline__ void prefetch_prime(int64_t mb) {
#pragma unroll
    for (int q = 0; q < 3 * PF; ++q) load_row(mb + q < me ? mb + q : me - 1, Lb[q % 3][q / 3]);
  }

  __device__ __forceinline__ void load_row(int64_t m, VT (&out)[NV]) const {
    const __amdgpu_buffer_rsrc_t rs = row_rsrc(srow + m * pitch_b, nrec);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      U4 b = __builtin_amdgcn_raw_buffer_load_b128(rs, ld_off + v * 16, 0, 0);
      out[v] = __builtin_bit_cast(VT, b);
    }
  }

  __device__ __forceinline__ void store_row(int64_t row, const T (&out)[V]) const {
    const __amdgpu_buffer_rsrc_t rs = row_rsrc(drow + row * pitch_b, nrec);
    if (!EDGE) {
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        VT w;
#pragma unroll
        for (int e = 0; e < VM; ++e) w[e] = out[v * VM + e];
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(U4, w), rs, st_off + v * 16, 0, 0);
      }
    } else {
#pragma unroll
      for (int e = 0; e < V; ++e) {
        if constexpr (sizeof(T) == 4)
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned int, out[e]), rs, st_e[e], 0, 0);
        else
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(unsigned int __attribute__((ext_vector_type(2))), out[e]), rs, st_e[e], 0, 0);
      }
    }
  }

  template <int PH, bool STORE>
  __device__ __forceinline__ void step(int64_t m) {
    constexpr int PO = PH, PQ = (PH + 1) % 3, PN = (PH + 2) % 3;
    // level 0: consume the prefetched row m, refill the slot with row m+3
    // (clamped to the last row: a harmless re-read keeps the loop branch-free)
#pragma unroll
    for (int v = 0; v < NV; ++v)
#pragma unroll
      for (int e = 0; e < VM; ++e) X[PN][0][v * VM + e] = Lb[PH][0][v][e];
    prefetch_advance<PH>(m);
#pragma unroll
    for (int s = 1; s <= K; ++s) {
      const T* o = X[PO][s - 1];  // row m-s-1 (north, x-1)
      const T* q = X[PQ][s - 1];  // row m-s   (centre)
      const T* n = X[PN][s - 1];  // row m-s+1 (south, x+1)
      const T west0 = from_lower(q[V - 1]);
      const T eastL = from_upper(q[0]);
      T out[V];
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const T west = e > 0 ? q[e - 1] : west0;
        const T east = e < V - 1 ? q[e + 1] : eastL;
        // reference order: T(x+1,y) + T(x,y+1) + T(x-1,y) + T(x,y-1) - 4*T(x,y).
        // sum - 4c as fma(-4, c, sum) is bitwise identical (4c is exact) and
        // saves one fp op; c + r*(...) stays unfused, as in the reference.
        const T sum = ((n[e] + east) + o[e]) + west;
        T val = q[e] + r * __builtin_fma(T(-4), q[e], sum);
        if (EDGE && ((fixmask >> e) & 1u)) val = q[e];
        out[e] = val;
      }
      const int64_t row = m - s;
      if (EDGE && (row < fixed_lo || row >= fixed_hi)) {  // Dirichlet row (global frame): keep
#pragma unroll
        for (int e = 0; e < V; ++e) out[e] = q[e];
      }
      if (s < K) {
#pragma unroll
        for (int e = 0; e < V; ++e) X[PN][s][e] = out[e];
      } else if (STORE) {
        store_row(row, out);
      }
    }
  }

  // Levels are primed for 2K rows (no output yet), then every row m in
  // [t0+K, t1+K) emits output row m-K.
  __device__ __forceinline__ void run() {
    const int64_t mb = t0 - K;
    me = t1 + K;
    prefetch_prime(mb);
    int64_t m = mb;
#pragma unroll 1
    for (int i = 0; i < (2 * K) / 3; ++i) {
      step<0, false>(m++);
      step<1, false>(m++);
      step<2, false>(m++);
    }
    constexpr int P0 = (2 * K) % 3;
    if constexpr (P0 >= 1) step<0, false>(m++);
    if constexpr (P0 >= 2) step<1, false>(m++);
    // main loop: m in [t0+K, me), at least one row (t1 > t0)
    for (;;) {
      step<P0, true>(m);
      if (++m >= me) break;
      step<(P0 + 1) % 3, true>(m);
      if (++m >= me) break;
      step<(P0 + 2) % 3, true>(m);
      if (++m >= me) break;
    }
  }
};

// Skew-2 pipeline. Level s computes row m-2s at march row m (instead of m-s),
// so within one row iteration the K levels read only rows produced in EARLIER
// iterations: the K level updates are mutually independent (ILP = K*V instead
// of V; the skew-1 pipeline chains all K levels through the freshly computed
// south neighbour, a 6-deep fp dependency per level). Levels are evaluated
// from K down to 1 so each level reads its 3 input rows before the level below
// overwrites the oldest of them: 3 rows per level, ring index (row mod 3).
template <typename T, int NV, int K, bool EDGE, int PF>
struct March2 : March<T, NV, K, EDGE, PF> {
  using B = March<T, NV, K, EDGE, PF>;
  using B::r;
  using B::X;
  using B::Lb;
  using B::me;
  using B::t0;
  using B::t1;
  static constexpr int V = B::V;
  static constexpr int VM = B::VM;
  int64_t mend;  // end of march rows (t1 + 2K)

  template <int PH, bool STORE>
  __device__ __forceinline__ void step2(int64_t m) {
#pragma unroll
    for (int s = K; s >= 1; --s) {
      // level s-1 rows m-2s-1 (north), m-2s (centre), m-2s+1 (south); slot = row mod 3
      constexpr int dummy = 0;
      (void)dummy;
      const int so = ((PH - 2 * s - 1) % 3 + 3) % 3;
      const int sq = ((PH - 2 * s) % 3 + 3) % 3;
      const int sn = ((PH - 2 * s + 1) % 3 + 3) % 3;
      const T* o = X[so][s - 1];
      const T* q = X[sq][s - 1];
      const T* n = X[sn][s - 1];
      const T west0 = from_lower(q[V - 1]);
      const T eastL = from_upper(q[0]);
      T out[V];
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const T west = e > 0 ? q[e - 1] : west0;
        const T east = e < V - 1 ? q[e + 1] : eastL;
        const T sum = ((n[e] + east) + o[e]) + west;
        T val = q[e] + r * __builtin_fma(T(-4), q[e], sum);
        if (EDGE && ((B::fixmask >> e) & 1u)) val = q[e];
        out[e] = val;
      }
      const int64_t row = m - 2 * s;
      if (EDGE && (row < B::fixed_lo || row >= B::fixed_hi)) {
#pragma unroll
        for (int e = 0; e < V; ++e) out[e] = q[e];
      }
      if (s < K) {
        const int sw = ((PH - 2 * s) % 3 + 3) % 3;  // slot of row m-2s
#pragma unroll
        for (int e = 0; e < V; ++e) X[sw][s][e] = out[e];
      } else if (STORE) {
        B::store_row(row, out);
      }
    }
    // level 0: row m lands in slot (m mod 3) = PH (level 1 has consumed row m-3)
#pragma unroll
    for (int v = 0; v < NV; ++v)
#pragma unroll
      for (int e = 0; e < VM; ++e) X[PH][0][v * VM + e] = Lb[PH][0][v][e];
    B::template prefetch_advance<PH>(m);
  }

  // level-0 rows [t0-K, t1+K); march rows [t0-K, t1+2K); output row m-2K for
  // m >= t0+2K (the first 3K rows only prime the levels)
  __device__ __forceinline__ void run() {
    const int64_t mb = t0 - K;
    me = t1 + K;
    mend = t1 + 2 * K;
    B::prefetch_prime(mb);
    int64_t m = mb;
    // phase PH = (m - mb) mod 3 (mb plays the role of row 0 for the rings)
#pragma unroll 1
    for (int i = 0; i < K; ++i) {  // 3K priming rows
      step2<0, false>(m++);
      step2<1, false>(m++);
      step2<2, false>(m++);
    }
    for (;;) {
      step2<0, true>(m);
      if (++m >= mend) break;
      step2<1, true>(m);
      if (++m >= mend) break;
      step2<2, true>(m);
      if (++m >= mend) break;
    }
  }
};

template <typename T, int NV, int K, bool EDGE, int SK, int PF>
__device__ __forceinline__ void march(const T* src, T* dst, const TbArgs& a, T r, int64_t strip, int64_t t0,
                                      int64_t t1, int lane) {
  using S = TbShape<T, NV, K>;
  constexpr int V = S::V;
  constexpr int ES = (int)sizeof(T);
  const int64_t u0 = strip * S::U;
  const int64_t c0 = u0 - S::KA;
  const int64_t mycol = c0 + (int64_t)lane * V;
  const int64_t ustop = min(u0 + (int64_t)S::U, a.ncols);
  using M = typename std::conditional<SK == 2, March2<T, NV, K, EDGE, PF>, March<T, NV, K, EDGE, PF>>::type;
  M w;
  // row base = column col_lo (= -cpad) of row 0; offsets are relative to it
  w.srow = reinterpret_cast<const char*>(src + a.col_lo);
  w.drow = reinterpret_cast<char*>(dst + a.col_lo);
  w.pitch_b = a.pitch * ES;
  w.nrec = (uint32_t)(a.pitch * ES);
  w.r = r;
  w.t0 = t0;
  w.t1 = t1;
  w.fixed_lo = a.fixed_lo;
  w.fixed_hi = a.fixed_hi;
  const int32_t off = (int32_t)((mycol - a.col_lo) * ES);
  const bool in_alloc = (mycol >= a.col_lo) && (mycol + V <= a.col_hi);
  w.ld_off = in_alloc ? off : kOob;
  const bool full = (mycol >= u0) && (mycol + V <= ustop);
  w.st_off = full ? off : kOob;
  unsigned fm = 0;
  if constexpr (EDGE) {
#pragma unroll
    for (int e = 0; e < V; ++e) {
      const int64_t c = mycol + e;
      if (c < 0 || c >= a.ncols) fm |= 1u << e;
      w.st_e[e] = (c >= u0 && c < ustop) ? off + e * ES : kOob;
    }
  }
  w.fixmask = fm;
  w.run();
}

template <typename T, int NV, int K, int SK, int PF>
__global__ __launch_bounds__(256) void tb_kernel(const T* __restrict__ src, T* __restrict__ dst, TbArgs a,
                                                 T r) {
  using S = TbShape<T, NV, K>;
  const int lane = threadIdx.x & 63;
  // readfirstlane: make the wave id (and everything derived from it: strip, rows,
  // row addresses) provably wave-uniform -> SGPRs and scalar buffer descriptors
  const int64_t wid = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  if (wid >= a.nwaves) return;  // whole wave exits; no barriers in this kernel
  // Work items = (row band, strip), band-major: consecutive waves take adjacent
  // strips of the same band, so the waves in flight stream whole contiguous
  // rows (HBM page locality) and all march in step.
  const int64_t rows = a.row_end - a.row_begin;
  const int64_t items = a.nbands * a.nstrips;
  for (int64_t it = wid; it < items; it += a.nwaves) {
    const int64_t band = it / a.nstrips;
    const int64_t strip = it - band * a.nstrips;
    const int64_t r0 = band * rows / a.nbands;
    const int64_t r1 = (band + 1) * rows / a.nbands;
    if (r1 <= r0) continue;
    // safe path: the strip reaches a Dirichlet/pad column, or the march's
    // rows [t0-K, t1+K) reach a Dirichlet row; everything else runs mask-free
    const int64_t c0 = strip * S::U - S::KA;
    const int64_t t0 = a.row_begin + r0, t1 = a.row_begin + r1;
    const bool edge = (c0 < 0) || (c0 + S::W > a.ncols) || (t0 - K < a.fixed_lo) || (t1 + K > a.fixed_hi);
    if (edge)
      march<T, NV, K, true, SK, PF>(src, dst, a, r, strip, t0, t1, lane);
    else
      march<T, NV, K, false, SK, PF>(src, dst, a, r, strip, t0, t1, lane);
  }
}

template <typename T, int NV, int K, int SK, int PF>
constexpr auto kernel_ptr() {
  return &tb_kernel<T, NV, K, SK, PF>;
}

// Resident 256-thread workgroups per CU for one kernel instance (occupancy
// API; these kernels use ~44 SGPRs, inside the range where the API is exact).
template <typename T, int NV, int K, int SK, int PF>
int blocks_per_cu() {
  static std::mutex mu;
  static std::map<int, int> cache;  // device -> blocks/CU
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find(dev);
  if (it != cache.end()) return it->second;
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, reinterpret_cast<const void*>(kernel_ptr<T, NV, K, SK, PF>()), 256, 0) !=
          hipSuccess ||
      nb <= 0)
    nb = 1;
  cache[dev] = nb;
  return nb;
}

// Per-(T, NV) entry points, explicitly instantiated in tb_<dtype>_nv<NV>.hip
// (one translation unit each, compiled in parallel).
template <typename T, int NV, int SK, int PF>
void dispatch(int k, unsigned nblocks, const T* src, T* dst, const TbArgs& a, T r, hipStream_t s);
template <typename T, int NV, int SK, int PF>
int occupancy_blocks(int k);

#define H2D_TB_CASE(T, NV, SK, PF, KK)                                                              \
  case KK:                                                                                          \
    hipLaunchKernelGGL((tb_kernel<T, NV, KK, SK, PF>), dim3(nblocks), dim3(256), 0, s, src, dst, a, r); \
    return;
#define H2D_OCC_CASE(T, NV, SK, PF, KK) \
  case KK:                              \
    return blocks_per_cu<T, NV, KK, SK, PF>();

}  // namespace tbimpl
}  // namespace kern
}  // namespace heat2d
