// Temporal-blocked 5-point FTCS stencil for gfx950 (CDNA4).
//
// Replaces reference K1 `heat_eqn` (fortran/hip/heat_kernel.cpp:31-45: one
// thread per point, 5 scalar loads, 128x4 blocks) and K12, the per-step
// full-field D2D copy (fortran/hip/heat.F90:243).
//
// Design (wave64, no LDS, no barriers):
//   * one WAVE owns a column strip of 64*V columns (V = 16 B / sizeof(T)) and a
//     tile of output rows; it marches down the rows, loading each input row
//     exactly once with one 16-B load per lane (1 KiB per wave instruction);
//   * K time levels are pipelined in registers: at march row m the wave loads
//     row m of level 0 and computes row m-s of level s for s = 1..K, so K time
//     steps cost ONE HBM read + ONE HBM write per point (the single-step
//     roofline is 16 B/pt fp64; at K = 8 the kernel needs 2 B/pt);
//   * east/west neighbours come from the adjacent lane through DPP
//     wave_shr:1 / wave_shl:1 (VALU modifiers, no LDS traffic); the strip's
//     outer K columns are redundant halo work (shrinking valid region);
//   * the 3-row window per level rotates through a 3-phase unrolled loop, so no
//     register moves are needed for the rotation;
//   * the arithmetic order is exactly the reference's
//     c + r*((((E + N) + W) + S) - 4c) (fortran/hip/heat_kernel.cpp:43) and the
//     file is built with -ffp-contract=off: results are bitwise identical to the
//     CPU reference and to an unblocked K=1 run.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "heat2d/kernels.hpp"

namespace heat2d {
namespace kern {
namespace {

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

__device__ __forceinline__ float from_lower(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), kDppWaveShr1, 0xF, 0xF, false));
}
__device__ __forceinline__ float from_upper(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), kDppWaveShl1, 0xF, 0xF, false));
}
__device__ __forceinline__ double from_lower(double x) {
  long long b = __double_as_longlong(x);
  int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffLL), kDppWaveShr1, 0xF, 0xF, false);
  int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), kDppWaveShr1, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ double from_upper(double x) {
  long long b = __double_as_longlong(x);
  int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffLL), kDppWaveShl1, 0xF, 0xF, false);
  int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), kDppWaveShl1, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

struct TbArgs {
  int64_t pitch;
  int64_t ncols;
  int64_t col_lo;  // allocation column bounds [col_lo, col_hi)
  int64_t col_hi;
  int64_t row_begin, row_end;
  int64_t tile_rows;
  int64_t nstrips, ntiles;
  int64_t fixed_lo, fixed_hi;  // local rows outside [fixed_lo, fixed_hi) are Dirichlet
};

template <typename T, int K>
struct TbShape {
  static constexpr int V = Vec16<T>::n;
  static constexpr int KA = (K + V - 1) / V * V;  // halo columns, vector aligned
  static constexpr int W = 64 * V;
  static constexpr int U = W - 2 * KA;
  static_assert(U > 0, "temporal depth too large for the strip width");
};

template <typename T, int K, bool EDGE>
struct March {
  using S = TbShape<T, K>;
  static constexpr int V = S::V;
  using VT = typename Vec16<T>::type;

  const T* __restrict__ src;
  T* __restrict__ dst;
  T r;
  int64_t pitch;
  int64_t t0, t1;      // output rows
  int64_t fixed_lo, fixed_hi;
  int64_t mycol;       // first column held by this lane
  int64_t me;          // end of level-0 rows
  bool ld_ok;          // lane inside the allocation
  bool st_full;        // lane's V columns all produced & owned (non-edge fast path)
  unsigned fixmask;    // EDGE: per-element Dirichlet column bits
  unsigned stmask;     // EDGE: per-element store bits

  T X[3][K][V];        // level state: 3-phase rotating window (SSA after unroll)
  VT Lb[3];            // level-0 prefetch ring (3 rows ahead)

  __device__ __forceinline__ VT load_row(int64_t m) const {
    if (ld_ok) return *reinterpret_cast<const VT*>(src + m * pitch + mycol);
    return VT{};
  }

  template <int PH>
  __device__ __forceinline__ void step(int64_t m) {
    constexpr int PO = PH, PQ = (PH + 1) % 3, PN = (PH + 2) % 3;
    // level 0: consume the prefetched row m, refill the slot with row m+3
    {
      VT v = Lb[PH];
#pragma unroll
      for (int e = 0; e < V; ++e) X[PN][0][e] = v[e];
      if (m + 3 < me) Lb[PH] = load_row(m + 3);
    }
#pragma unroll
    for (int s = 1; s <= K; ++s) {
      // rows of level s computed before m >= t0-K+2s are outside its valid
      // (shrinking) window: skip them (wave-uniform branch).
      if (m < t0 - K + 2 * s) continue;
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
        // reference order: T(x+1,y) + T(x,y+1) + T(x-1,y) + T(x,y-1) - 4*T(x,y)
        const T sum = ((n[e] + east) + o[e]) + west;
        T val = q[e] + r * (sum - T(4) * q[e]);
        if (EDGE && ((fixmask >> e) & 1u)) val = q[e];
        out[e] = val;
      }
      const int64_t row = m - s;
      if (row < fixed_lo || row >= fixed_hi) {  // Dirichlet row (global frame): keep
#pragma unroll
        for (int e = 0; e < V; ++e) out[e] = q[e];
      }
      if (s < K) {
#pragma unroll
        for (int e = 0; e < V; ++e) X[PN][s][e] = out[e];
      } else if (row >= t0 && row < t1) {
        T* p = dst + row * pitch + mycol;
        if (!EDGE) {
          if (st_full) {
            VT w;
#pragma unroll
            for (int e = 0; e < V; ++e) w[e] = out[e];
            *reinterpret_cast<VT*>(p) = w;
          }
        } else {
#pragma unroll
          for (int e = 0; e < V; ++e)
            if ((stmask >> e) & 1u) p[e] = out[e];
        }
      }
    }
  }

  __device__ __forceinline__ void run() {
    const int64_t mb = t0 - K;
    me = t1 + K;
#pragma unroll
    for (int q = 0; q < 3; ++q) Lb[q] = (mb + q < me) ? load_row(mb + q) : VT{};
    int64_t m = mb;
    for (;;) {
      step<0>(m);
      if (++m >= me) break;
      step<1>(m);
      if (++m >= me) break;
      step<2>(m);
      if (++m >= me) break;
    }
  }
};

template <typename T, int K>
__global__ __launch_bounds__(256) void tb_kernel(const T* __restrict__ src, T* __restrict__ dst,
                                                 TbArgs a, T r) {
  using S = TbShape<T, K>;
  constexpr int V = S::V;
  const int lane = threadIdx.x & 63;
  const int64_t wid = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (wid >= a.nstrips * a.ntiles) return;  // whole wave exits; no barriers in this kernel
  const int64_t strip = wid % a.nstrips;
  const int64_t tile = wid / a.nstrips;
  const int64_t t0 = a.row_begin + tile * a.tile_rows;
  const int64_t t1 = min(t0 + a.tile_rows, a.row_end);
  const int64_t u0 = strip * S::U;
  const int64_t c0 = u0 - S::KA;
  const int64_t mycol = c0 + (int64_t)lane * V;
  const int64_t ustop = min(u0 + (int64_t)S::U, a.ncols);
  const bool edge = (c0 < 0) || (c0 + S::W > a.ncols);
  const bool ld_ok = (mycol >= a.col_lo) && (mycol + V <= a.col_hi);

  if (!edge) {
    March<T, K, false> w;
    w.src = src; w.dst = dst; w.r = r; w.pitch = a.pitch; w.t0 = t0; w.t1 = t1;
    w.fixed_lo = a.fixed_lo; w.fixed_hi = a.fixed_hi; w.mycol = mycol; w.ld_ok = ld_ok;
    w.st_full = (mycol >= u0) && (mycol + V <= ustop);
    w.fixmask = 0; w.stmask = 0;
    w.run();
  } else {
    March<T, K, true> w;
    w.src = src; w.dst = dst; w.r = r; w.pitch = a.pitch; w.t0 = t0; w.t1 = t1;
    w.fixed_lo = a.fixed_lo; w.fixed_hi = a.fixed_hi; w.mycol = mycol; w.ld_ok = ld_ok;
    w.st_full = false;
    unsigned fm = 0, sm = 0;
#pragma unroll
    for (int e = 0; e < V; ++e) {
      const int64_t c = mycol + e;
      if (c < 0 || c >= a.ncols) fm |= 1u << e;
      if (c >= u0 && c < ustop) sm |= 1u << e;
    }
    w.fixmask = fm; w.stmask = sm;
    w.run();
  }
}

template <typename T>
int useful_width(int k) {
  constexpr int V = Vec16<T>::n;
  const int ka = (k + V - 1) / V * V;
  return 64 * V - 2 * ka;
}

template <typename T, int K>
void launch_k(const TbPlan& p, const T* src, T* dst, const TbArgs& a, T r, hipStream_t s) {
  hipLaunchKernelGGL((tb_kernel<T, K>), dim3((unsigned)p.nblocks), dim3(256), 0, s, src, dst, a, r);
}

template <typename T>
void dispatch(const TbPlan& p, const T* src, T* dst, const TbArgs& a, T r, hipStream_t s) {
  switch (p.k) {
#define H2D_CASE(KK) \
  case KK:           \
    launch_k<T, KK>(p, src, dst, a, r, s); \
    break;
    H2D_CASE(1) H2D_CASE(2) H2D_CASE(3) H2D_CASE(4) H2D_CASE(5) H2D_CASE(6) H2D_CASE(7) H2D_CASE(8)
    H2D_CASE(9) H2D_CASE(10) H2D_CASE(11) H2D_CASE(12) H2D_CASE(13) H2D_CASE(14) H2D_CASE(15) H2D_CASE(16)
#undef H2D_CASE
    default:
      HEAT2D_REQUIRE(false, "temporal depth out of range");
  }
}

}  // namespace

TbPlan plan_tb(DType dt, const SlabLayout& L, int64_t row_begin, int64_t row_end, int k,
               int64_t tile_rows) {
  HEAT2D_REQUIRE(k >= 1 && k <= kMaxTB, "k must be in [1, kMaxTB]");
  HEAT2D_REQUIRE(row_begin >= 0 && row_end <= L.nrows && row_begin < row_end, "bad row range");
  TbPlan p{};
  p.k = k;
  p.vec = dt == DType::F32 ? 4 : 2;
  p.strip_w = 64 * p.vec;
  p.useful_w = dt == DType::F32 ? useful_width<float>(k) : useful_width<double>(k);
  p.nstrips = (L.ncols + p.useful_w - 1) / p.useful_w;
  const int64_t rows = row_end - row_begin;
  if (tile_rows <= 0) {
    // fill the chip: aim for >= 8192 waves (256 CUs x 32 wave slots), tiles
    // long enough that the 2k-row march overhead stays small.
    const int64_t target_waves = 8192;
    tile_rows = (rows * p.nstrips + target_waves - 1) / target_waves;
    tile_rows = std::max<int64_t>(tile_rows, 8 * (int64_t)k);
    tile_rows = std::max<int64_t>(tile_rows, 32);
    tile_rows = std::min<int64_t>(tile_rows, 512);
  }
  p.tile_rows = std::min<int64_t>(tile_rows, rows);
  p.ntiles = (rows + p.tile_rows - 1) / p.tile_rows;
  p.nwaves = p.nstrips * p.ntiles;
  p.nblocks = (p.nwaves + 3) / 4;
  return p;
}

void launch_tb(DType dt, const void* src, void* dst, const SlabLayout& L, int64_t row_begin,
               int64_t row_end, int k, double r, hipStream_t stream, int64_t tile_rows) {
  HEAT2D_REQUIRE(k <= L.halo, "temporal depth exceeds the halo depth");
  HEAT2D_REQUIRE(L.cpad >= 16, "column padding too small for the strip halo");
  if (row_end <= row_begin) return;
  const TbPlan p = plan_tb(dt, L, row_begin, row_end, k, tile_rows);
  TbArgs a{};
  a.pitch = L.pitch;
  a.ncols = L.ncols;
  a.col_lo = -L.cpad;
  a.col_hi = L.col_hi();
  a.row_begin = row_begin;
  a.row_end = row_end;
  a.tile_rows = p.tile_rows;
  a.nstrips = p.nstrips;
  a.ntiles = p.ntiles;
  a.fixed_lo = -L.row0;
  a.fixed_hi = L.nrows_global - L.row0;
  const int64_t o = L.origin();
  if (dt == DType::F32) {
    dispatch<float>(p, static_cast<const float*>(src) + o, static_cast<float*>(dst) + o, a, (float)r, stream);
  } else {
    dispatch<double>(p, static_cast<const double*>(src) + o, static_cast<double*>(dst) + o, a, r, stream);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) fail(__FILE__, __LINE__, std::string("tb_kernel launch: ") + hipGetErrorString(e));
}

}  // namespace kern
}  // namespace heat2d
