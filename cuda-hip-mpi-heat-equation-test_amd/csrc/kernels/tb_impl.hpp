// Device implementation of the temporal-blocked stencil (see stencil_tb.hip
// for the design notes). Included by the per-(dtype, vector width, prefetch
// ring) instantiation units tb_*.hip so they compile in parallel.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>
#include <type_traits>
#include <utility>

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

// Precision-preserving fma: __builtin_fma is the DOUBLE builtin — on floats it
// silently promotes the whole update to fp64 (v_cvt_f64_f32 + fp64 VALU at half
// rate, and a different rounding than the fp32 reference).
__device__ __forceinline__ float fma_t(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
__device__ __forceinline__ double fma_t(double a, double b, double c) { return __builtin_fma(a, b, c); }

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

// Single fp32 adds for the two across-lane sums of the packed march
// (MarchF32). Written plainly, the backend merges such scalar adds with their
// neighbours into v_pk_add_f32 on re-assembled register pairs (2 extra moves
// per pair); an empty asm that takes the sum as an in/out operand keeps each
// add scalar, so the two halves of a pair are produced in place and the DPP
// move folds into the add (v_add_f32_dpp, by the compiler's DPP combine, which
// also inserts the DPP read hazard waits — a hand-written asm add needed an
// s_nop per DPP and measured the same: profiles/packed_fp32.md).
__device__ __forceinline__ float fence_v(float r) {
  asm("" : "+v"(r));
  return r;
}
__device__ __forceinline__ float sadd(float a, float b) { return fence_v(a + b); }
__device__ __forceinline__ float sadd_from_upper(float a, float x) { return fence_v(a + from_upper(x)); }
__device__ __forceinline__ float sadd_from_lower(float a, float x) { return fence_v(a + from_lower(x)); }

// Kernel arguments: the work is up to kMaxRects rectangles (output rows x
// strips), each cut into `nb` row bands; a work item is one (band, strip) of
// one rectangle. item0 = index of the rectangle's first item.
constexpr int kMaxRects = kMaxPlanRects;
constexpr int kMainRects = 4;  // interior (MAIN) kernels: frame-strip rects or the boundary bands
struct TbRectArg {
  int64_t r0, r1;  // output rows [r0, r1)
  int64_t s0, s1;  // strips [s0, s1)
  int64_t nb;      // row bands
  int64_t item0;
};
struct TbArgs {
  int64_t pitch;
  int64_t ncols;
  int64_t col_lo;  // allocation column bounds [col_lo, col_hi)
  int64_t col_hi;
  int64_t nitems;  // total items over all rects
  int64_t nwaves;  // launched waves (grid-stride over items)
  int64_t fixed_lo, fixed_hi;  // local rows outside [fixed_lo, fixed_hi) are Dirichlet
  int32_t nrect;
  int32_t pad0;
  TbRectArg rect[kMaxRects];
  double* partials;   // ST kernels: per-wave statistics, partials[j * nwaves + wave] (kNStatFused = 6 values)
  // Diagnostics (HEAT2D_WAVE_TIMES, kern::wave_times): per launched wave
  // {start, end (wall clock, 100 MHz), first item, its edge kind}; nullptr off
  uint64_t* wtimes;
  // arith 3 (any r): scaled-level coefficients, computed on the host in
  // double for this launch's depth k: fb = (1 - 4r) / r (the centre weight of
  // a level carried as T / r^level), fu = r^k (unscales the stored level),
  // fu1 = r^(k-1) (level k-1, the statistics' residual)
  double fb, fu, fu1;
  // Dynamic item queue (SplitPlan::flags & kPlanDynamic): {next item beyond the first
  // round, waves finished}; a wave takes its first item statically (wid) and
  // then the next free one, so waves that run faster take more items. The
  // last wave to finish resets both counters for the next launch. nullptr:
  // static grid stride.
  uint32_t* queue;
};

// Fused statistics of the stored (last) level (ST kernels): sum T, sum T^2,
// min T, max T, sum (T_K - T_{K-1})^2, max |T_K - T_{K-1}| over the owned
// points — T_K - T_{K-1} is the one-step residual of the cycle's last step,
// whatever the depth. Accumulated in fp64 per lane, reduced per wave with a
// fixed butterfly, one partial per wave: deterministic for a given plan.
constexpr int kNStatFused = 6;
struct StatAcc {
  double s = 0.0, ss = 0.0, mn = __builtin_huge_val(), mx = -__builtin_huge_val(), dd = 0.0, md = 0.0;
  __device__ __forceinline__ void add(bool ok, double v, double c) {
    const double d = v - c;
    s += ok ? v : 0.0;
    ss += ok ? v * v : 0.0;
    mn = fmin(mn, ok ? v : __builtin_huge_val());
    mx = fmax(mx, ok ? v : -__builtin_huge_val());
    dd += ok ? d * d : 0.0;
    md = fmax(md, ok ? fabs(d) : 0.0);
  }
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
// touch memory carry an out-of-range voffset, and a store whose row is not an
// output row gets a descriptor with num_records = 0, so the hardware range
// check returns 0 / drops the access instead of an exec-masked branch. With no
// memory op under control flow, the waitcnt pass counts the prefetch ring
// precisely (vmcnt(N>0)) instead of draining it every row.
constexpr int32_t kOob = (int32_t)0x80000000u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}

// One wave marching UP a column strip (decreasing row index) with K time
// levels pipelined in registers.
//
// At march row m the wave loads level-0 row m and computes row m+s of level s
// (s = 1..K) from level s-1 rows m+s+1 (south, x+1: the OLDEST, produced two
// iterations ago), m+s (centre) and m+s-1 (north, x-1: produced earlier in
// THIS iteration). The reference sums T(x+1,y) + T(x,y+1) + T(x-1,y) + T(x,y-1)
// (fortran/hip/heat_kernel.cpp:43) — south first — so marching upward lets the
// partial (S + E) be formed from the oldest row BEFORE that row's register is
// overwritten by the level's new row. Each level therefore keeps 2 rows of
// state (ring indexed by iteration parity) instead of 3, and the dependency
// chain from the fresh row is 5 ops instead of 6 — both with the reference's
// exact operation order (bitwise identical results).
//
// Level 0 lives directly in the RING-slot load ring (row m in slot
// phase(m) = (mtop - m) mod RING): a slot is refilled as soon as its row has
// been used as a south neighbour, so RING - 2 rows are in flight and no
// register ever receives a copy of a value with a pending load (which would
// force a vmcnt drain). The loop is unrolled RING times so every slot is a
// fixed register set. Row indices are 32-bit so every row test is a scalar
// compare (gfx9 has no 64-bit scalar less-than).
// Frame handling by edge kind EK (bit 0: the march reaches a Dirichlet ROW of
// the global frame, bit 1: the strip reaches a Dirichlet / pad COLUMN). A
// pinned point must keep its value at every level: the update C + r*x is done
// with r = 0 there, so pinning costs no instruction in kinds 1 and 2 —
// kind 1 zeroes the wave-uniform scalar r for frame rows (SALU select), kind 2
// multiplies by a per-lane r vector with zeros in frame columns. Only kind 3
// (corner items, both) pays a select per element and level; the kernel runs
// those items in two half-height pieces so they do not become the tail.
// (0 * x is +-0 and C + +-0 == C for the finite values the march carries.)
//
// Arithmetic AR (SolverConfig::arith): 0 = the reference expression with every
// operation rounded, C + r*(sum - 4C) (-ffp-contract=off; bitwise equal to the
// CPU twin and the NumPy golden); 1 = the same expression contracted to
// fma(r, sum - 4C, C) — what hipcc's default -ffp-contract=fast makes of the
// reference's own kernel line (fortran/hip/heat_kernel.cpp:43): one VALU op
// fewer per point (5 fp64 ops + 2 DPP moves instead of 6 + 2) for a kernel that
// is VALU-co-bound. When r is a power of two (sigma = 0.25 in every shipped
// input) r*x is exact and both forms round identically (normal range).
// 2 = r == 1/4 exactly (sigma = 0.25: the reference configuration): the centre
// weight 1 - 4r is zero and the update is T' = (((S + E) + N) + W) / 4, the
// reference's own sum with one exact multiply. Kind-0 items (no pinned point:
// the bulk of every launch) carry level s scaled by 4^s, so a level is the
// plain sum — 3 adds + 2 DPP moves per point instead of 5 + 2 — and multiply by
// 4^-K once, at the store (powers of two: exact, so the stored bits equal the
// per-level /4 form for |T| < 2^(emax - 2K)). Pinned kinds (re = 0 where
// pinned) compute unscaled: kind 1 fma(ke, C, re * sum) with scalar ke = 1 -
// 4 re (2 ops, as arith 1), kinds 2 / 3 re * sum + (C - 4 re C) (3 ops); the
// added term is exactly 0 at updated points and C at pinned ones — the same
// bits. Where every (sum, 4C)
// pair lies within a factor of two (smooth positive data, e.g. the reference IC
// with values in [1, 2]), sum - 4C is exact (Sterbenz) and the reference
// rounding gives the same bits too.
// 3 = any r (SolverConfig::arith 3, "fast"): the same scaling with 1 / r in
// place of 4. With X_s = T_s / r^s the update T' = (1 - 4r) C + r (S+E+N+W)
// becomes X_{s+1} = fma(b, X_s(C), ((S + E) + N) + W), b = (1 - 4r) / r: 3 adds
// + 1 fma per point and level instead of 5 ops (arith 1); the stored level is
// multiplied by r^K once. Kind-0 items only; pinned kinds (the frame must stay
// bit-exact) run arith 2's unscaled forms with the centre weight ke = 1 - 4r
// instead of 0: kind 1 fma(ke, C, r * sum), kinds 2 / 3 r * sum + (C - 4rC)
// as two fmas. Not the
// reference's rounding: within a stated bound of it (tests/test_arith_fast.py,
// |T_fast - T_exact| <= 16 n u max|T_0| after n steps, u the unit roundoff),
// and, since interior and pinned items round differently, the bits depend on
// the launch plan. At r = 1/4 (b = 0, r^K a power of two) it IS arith 2.
template <typename T>
constexpr T inv_pow4(int l) {
  T s = T(1);
  for (int i = 0; i < l; ++i) s *= T(0.25);
  return s;
}
// Dependency chains of the march (CL levels per chain). Level s computes
// row m + off(s) while the march is at level-0 row m. Inside a chain (delta 1)
// level s reads level s-1's row of THIS iteration — a serial dependency, K
// levels deep per row in the single-chain march (CL = K). At a chain boundary
// (delta 2: s = 1 + j*CL, j >= 1) level s reads only rows of level s-1 from the
// three previous iterations, so the K/CL chains of an iteration are
// independent: instruction-level parallelism for a wave that is alone on its
// SIMD (small grids, thin-slab boundary bands), paid with one more register
// row for the level below each boundary (a 3-slot ring) and one more march
// row per boundary. Same operations, same order per point: bitwise identical.
// Measured: profiles/chained_march.md.
template <int K, int CL>
struct ChainShape {
  static constexpr int delta(int s) { return (s > 1 && (s - 1) % CL == 0) ? 2 : 1; }
  static constexpr int off(int s) { return s + (s >= 1 ? (s - 1) / CL : 0); }
  // ring size of stored level j (1 .. K-1): 2 rows, 3 below a boundary
  static constexpr int ring(int j) { return (j >= 1 && j < K) ? delta(j + 1) + 1 : 2; }
  static constexpr int boundaries = K >= 1 ? (K - 1) / CL : 0;
  // loop-body length: whole level-0 rings and whole 2- (and 3-) slot level rings
  static constexpr int unroll(int ring0) {
    return boundaries == 0 ? ring0 : (ring0 % 3 == 0 ? (ring0 % 2 == 0 ? ring0 : 2 * ring0) : (ring0 % 2 == 0 ? 3 * ring0 : 6 * ring0));
  }
  // slot of the row level j computed `back` iterations before phase ph
  static constexpr int slot(int ph, int back, int j) { return ((ph - back) % ring(j) + ring(j)) % ring(j); }
  // Priming: at march iteration i (0 = the top row), level s computes row
  // mtop - i + off(s), which some output needs only once i >= off(s) + s; in
  // the first iterations the deep levels would compute rows above the band's
  // dependency cone (about K^2 wasted level-rows per work item, 18 % of a
  // 64-row item at K = 16). Levels needed at iteration i:
  static __device__ __forceinline__ int32_t levels_at(int32_t i) {
    int32_t n = 0;
#pragma unroll
    for (int s = 1; s <= K; ++s) n += (off(s) + s <= i) ? 1 : 0;
    return n;
  }
  static constexpr int prime_iters = off(K) + K;  // from here on every level is needed
};

// Default chain length per dtype (build flags HEAT2D_CHAIN_F32 / _F64; 0 = one
// chain of K levels) for depths >= HEAT2D_CHAIN_MIN_K. Measured with fixed
// plans (profiles/chained_march.md): chains of 4 speed up the deep fp64 passes
// (32768^2 K = 20: 6.78 -> 6.56 ms per cycle), are neutral for fp64 K = 14
// and fp32 K = 16 on big grids, and cost 6 % on the 4096^2 fp32 grid — so only
// fp64 K = 17..20 (the one-pass depths of short runs) uses them.
#ifndef HEAT2D_CHAIN_F32
#define HEAT2D_CHAIN_F32 0
#endif
#ifndef HEAT2D_CHAIN_F64
#define HEAT2D_CHAIN_F64 4
#endif
#ifndef HEAT2D_CHAIN_MIN_K
#define HEAT2D_CHAIN_MIN_K 17
#endif
// above K = 20 the chains' extra rows push the fp64 interior kernel to 1 wave/SIMD
#ifndef HEAT2D_CHAIN_MAX_K
#define HEAT2D_CHAIN_MAX_K 20
#endif
template <typename T, int K>
constexpr int chain_len() {
  constexpr int c = std::is_same<T, float>::value ? HEAT2D_CHAIN_F32 : HEAT2D_CHAIN_F64;
  return (c <= 0 || c >= K || K < HEAT2D_CHAIN_MIN_K || K > HEAT2D_CHAIN_MAX_K) ? K : c;
}

// Cache-policy bits of the march's 16-B row stores: 2 = nt (streaming). The
// output rows are written once and read by the next pass only, so marking them
// streaming leaves more of the XCD's L2 to the halo columns neighbouring strips
// re-read: rocprof FETCH_SIZE per pass 1.160 -> 1.138x the field (fp64 32768^2,
// K = 16), 1.130 -> 1.124x (fp32); 480-step fp64 bench +0.7 % in 6 of 6
// interleaved pairs (profiles/hbm_model_check.md). Build with
// -DHEAT2D_STORE_AUX=0 for the default policy.
#ifndef HEAT2D_STORE_AUX
#define HEAT2D_STORE_AUX 2
#endif

template <typename T, int NV, int K, int EK, int RING, int AR, bool ST = false, int CL = K>
struct March {
  using S = TbShape<T, NV, K>;
  static constexpr int V = S::V;
  static constexpr int VM = S::VM;
  static constexpr int KX = K > 1 ? K - 1 : 1;  // levels 1..K-1 kept in X
  using VT = typename Vec16<T>::type;
  using U4 = unsigned int __attribute__((ext_vector_type(4)));
  static_assert(RING % 2 == 0 && RING >= 4, "ring must be even (parity-indexed level rings) and >= 4");

  const char* srow;  // byte address of (row 0, column -cpad) in src   [wave-uniform]
  char* drow;        // same in dst                                      [wave-uniform]
  // Row pointers of the steady march, stepped by one row per march row: the
  // prefetch row (m + 2 - RING) and the stored row (m + off(K)). A row address
  // recomputed from its index costs ~12 scalar ops (64-bit multiply, sign,
  // descriptor) per access — with one wave per SIMD every one an issue slot
  // the VALU loses (31 SALU per march row against 136 VALU at fp32 K = 16,
  // rocprofv3 SQ_INSTS_SALU, profiles/r3/pairprof/).
  const char* lp;
  char* sp;
  // ... except in the fp64 K >= 20 ring-4 kernels, where the two loop-carried
  // pointers push the interior kernel past 256 VGPRs (SGPR spills into VGPR
  // lanes: 1 wave/SIMD instead of 2); those keep the per-row recomputation
  static constexpr bool kIncPtr = !(std::is_same<T, double>::value && K >= 20 && RING == 4);
  int64_t pitch_b;   // bytes per row                                    [wave-uniform]
  uint32_t nrec;     // descriptor size (= pitch_b)
  T r;
  int32_t t0, t1;    // output rows [t0, t1)
  int32_t fixed_lo, fixed_hi;  // EK & 1: rows outside [fixed_lo, fixed_hi) are frame rows
  int32_t mlo;       // lowest march row (t0 - off(K))
  int32_t mload;     // lowest level-0 row loaded (t0 - K)
  int32_t ld_off;    // per-lane load byte offset (kOob outside the allocation)
  int32_t st_off;    // per-lane vector store offset (kOob unless the lane holds output columns)
  T rl[(EK & 2) ? V : 1];  // EK & 2: r per element, 0 in Dirichlet / pad columns
  T fb, fu, fu1;           // AR 3: TbArgs::fb / fu / fu1
  T fk;                    // AR 3: the centre weight 1 - 4r of the unscaled pinned kinds
  static constexpr bool kScaled = (AR == 2 || AR == 3) && EK == 0;  // levels carried scaled (AR 2: x 4^level, 3: / r^level)

  using Ch = ChainShape<K, CL>;
  static constexpr int L = Ch::unroll(RING);  // march rows per loop body
  T X[3][KX][V];     // levels 1..K-1: X[slot][level-1][elem] (slot 2 only below chain boundaries)
  VT Lb[RING][NV];   // level 0: load ring
  StatAcc acc;       // ST: statistics of the stored rows
  uint32_t colmask;  // ST: bit e = element e is an owned output column of this lane

  __device__ __forceinline__ void load_row(int32_t m, VT (&out)[NV]) const { load_row_p(srow + (int64_t)m * pitch_b, true, out); }
  // live == false: a row below the item's lowest loaded row (it only feeds
  // priming values): num_records 0, the load returns 0 without a memory access
  __device__ __forceinline__ void load_row_p(const char* p, bool live, VT (&out)[NV]) const {
    const __amdgpu_buffer_rsrc_t rs = row_rsrc(p, live ? nrec : 0u);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      U4 b = __builtin_amdgcn_raw_buffer_load_b128(rs, ld_off + v * 16, 0, 0);
      out[v] = __builtin_bit_cast(VT, b);
    }
  }

  // live == false (priming rows): num_records 0 drops the whole store.
  __device__ __forceinline__ void store_row(char* p, bool live, const T (&out)[V]) const {
    const __amdgpu_buffer_rsrc_t rs = row_rsrc(p, live ? nrec : 0u);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      VT w;
#pragma unroll
      for (int e = 0; e < VM; ++e) w[e] = out[v * VM + e];
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(U4, w), rs, st_off + v * 16, 0, HEAT2D_STORE_AUX);
    }
  }

  __device__ __forceinline__ void unpack(const VT (&x)[NV], T (&out)[V]) const {
#pragma unroll
    for (int v = 0; v < NV; ++v)
#pragma unroll
      for (int e = 0; e < VM; ++e) out[v * VM + e] = x[v][e];
  }

  // part = S + E(C): the first partial sum of the reference order, from the
  // level's oldest row S and the east neighbours of its centre row C.
  __device__ __forceinline__ void partial(const T (&Sx)[V], const T (&C)[V], T (&part)[V]) const {
    const T eastL = from_upper(C[0]);
#pragma unroll
    for (int e = 0; e < V; ++e) part[e] = Sx[e] + (e < V - 1 ? C[e + 1] : eastL);
  }

  // ((part + N) + W) then C + r*(sum - 4C), pinned columns / rows kept.
  __device__ __forceinline__ void update(const T (&part)[V], const T (&C)[V], const T (&N)[V], int32_t row,
                                         T (&out)[V]) const {
    const T west0 = from_lower(C[V - 1]);
    const bool frame_row = (EK & 1) && ((uint32_t)(row - fixed_lo) >= (uint32_t)(fixed_hi - fixed_lo));  // wave-uniform
    const T rs = frame_row ? T(0) : r;                                      // EK 1: scalar select
#pragma unroll
    for (int e = 0; e < V; ++e) {
      const T west = e > 0 ? C[e - 1] : west0;
      // reference order: ((S + E) + N) + W - 4C; sum - 4C as fma(-4, C, sum)
      // is bitwise identical (4C is exact) and saves one op; C + r*(...)
      // stays unfused, as in the reference.
      const T sum = (part[e] + N[e]) + west;
      T re;
      if constexpr (EK == 0) re = r;
      else if constexpr (EK == 1) re = rs;
      else if constexpr (EK == 2) re = rl[e];
      else re = frame_row ? T(0) : rl[e];
      if constexpr (AR == 3 && EK == 0) {
        out[e] = fma_t(fb, C[e], sum);  // scaled: T / r^s
      } else if constexpr (AR == 2 || AR == 3) {
        // scaled kind 0: the plain sum (4^s T). Pinned kinds (re = 0 where
        // pinned), unscaled: kind 1 (frame rows: wave-uniform) fma(ke, C, re *
        // sum) with scalar ke = 1 - 4 re; kinds 2 / 3 (per-element re)
        // re * sum + (C - 4 re C). The added term is exactly 0 at updated
        // points (re = 1/4) and C at pinned ones. (AR 3: ke = 1 - 4r at
        // updated rows; at r = 1/4 the same bits as AR 2.)
        if constexpr (EK == 0) out[e] = sum;
        else if constexpr (EK == 1) out[e] = fma_t(frame_row ? T(1) : (AR == 3 ? fk : T(0)), C[e], re * sum);
        else out[e] = fma_t(re, sum, fma_t(re, T(-4) * C[e], C[e]));
      } else if constexpr (AR == 1) {
        out[e] = fma_t(re, fma_t(T(-4), C[e], sum), C[e]);
      } else {
        out[e] = C[e] + re * fma_t(T(-4), C[e], sum);
      }
    }
  }

  // One march row at phase PH (0 .. L-1; level-0 ring slot PH % RING, level-j
  // ring slot PH % ring(j)).
  // PRIME: only levels 1..nl (levels_at of this iteration) are computed.
  template <int PH, bool PRIME = false>
  __device__ __forceinline__ void step(int32_t m, int32_t nl = K) {
    constexpr int P0 = PH % RING;
    constexpr int sN = P0, sC = (P0 + RING - 1) % RING, sS = (P0 + RING - 2) % RING;  // level-0 slots
    T part[V];
    T C0[V], N0[V];
    {
      T S0[V];
      unpack(Lb[sS], S0);
      unpack(Lb[sC], C0);
      partial(S0, C0, part);  // level 1's S+E
    }
    {  // row m+2 is dead: refill its slot with row m+2-RING (clamped: a harmless re-read).
      // The scheduling fence keeps the load below the slot's last use: hoisted
      // above it, the load would need a fresh register and a copy at the loop
      // latch (which waits for the load and serialises the ring).
      const int32_t nxt = m + 2 - RING;
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (kIncPtr) {
        load_row_p(lp, nxt >= mload, Lb[sS]);
        lp -= pitch_b;
      } else {
        load_row(nxt >= mload ? nxt : mload, Lb[sS]);
      }
    }
    unpack(Lb[sN], N0);
#pragma unroll
    for (int s = 1; s <= K; ++s) {
      // PRIME: deeper levels are not needed yet (wave-uniform guard; a `break`
      // here would keep the loop from unrolling into constant register indices)
      if (PRIME && s > nl) continue;
      T C[V], N[V], out[V], nxtpart[V];
      const int d = Ch::delta(s);
      const int j = s > 1 ? s - 1 : 1;  // the level read (s - 1), when stored
#pragma unroll
      for (int e = 0; e < V; ++e) {
        // delta 1: N = level s-1's row of this iteration (fresh), C one back;
        // delta 2: N one back, C two back (independent of this iteration)
        C[e] = s == 1 ? C0[e] : X[Ch::slot(PH, d, j)][j - 1][e];
        N[e] = s == 1 ? N0[e] : X[Ch::slot(PH, d - 1, j)][j - 1][e];
      }
      const int ps = Ch::slot(PH, 0, s < K ? s : 1);  // this level's slot of this iteration
      // level s+1's S+E from level s's S (the slot about to be overwritten) and C
      if (s < K) partial(X[ps][s - 1], X[Ch::slot(PH, Ch::delta(s + 1), s)][s - 1], nxtpart);
      update(part, C, N, m + Ch::off(s), out);
      if (s < K) {
#pragma unroll
        for (int e = 0; e < V; ++e) X[ps][s - 1][e] = out[e];
#pragma unroll
        for (int e = 0; e < V; ++e) part[e] = nxtpart[e];
      } else {
        const int32_t row = m + Ch::off(K);
        const bool live = (uint32_t)(row - t0) < (uint32_t)(t1 - t0);  // row in [t0, t1), wave-uniform
        if constexpr (kScaled) {
          const T u = AR == 2 ? inv_pow4<T>(K) : fu;
#pragma unroll
          for (int e = 0; e < V; ++e) out[e] *= u;
        }
        store_row(kIncPtr ? sp : drow + (int64_t)row * pitch_b, live, out);
        if constexpr (ST) {
          if (live) {
            const T cu = kScaled ? (AR == 2 ? inv_pow4<T>(K - 1) : fu1) : T(1);  // level K-1 scale
#pragma unroll
            for (int e = 0; e < V; ++e) acc.add((colmask >> e) & 1u, (double)out[e], (double)(C[e] * cu));
          }
        }
      }
    }
    if constexpr (kIncPtr) sp -= pitch_b;
  }

  template <int... I>
  __device__ __forceinline__ void body(int32_t m, std::integer_sequence<int, I...>) {
    (step<I>(m - I), ...);
  }
  template <int... I>
  __device__ __forceinline__ void body_prime(int32_t m, int32_t i, std::integer_sequence<int, I...>) {
    (step<I, true>(m - I, Ch::levels_at(i + I)), ...);
  }

  // March rows m = t1+K-1 down to t0-off(K) (level-0 rows [t0-K, t1+K) are
  // loaded; below t0-K the loads are clamped: those rows only feed priming
  // values). Level K row m+off(K) is an output row once it is < t1: the first
  // iterations only prime the levels (their stores are dropped by the
  // descriptor). The trip count is rounded up to whole L-row bodies (the
  // extra rows' stores are dropped too): a loop body with a single exit, so
  // no load can be sunk past a mid-body exit (which would serialise the ring).
  // PS: skip the levels the first march rows do not need (priming). The
  // interior kernels use it (fp64 too since round 5: +5-8 % per pass at
  // depths 13..20 although it costs some of them an occupancy level,
  // profiles/r5/i/, r5/j/); the general kernels do not (4-5 % slower for the
  // 1-wave/SIMD fp32 small grid, profiles/priming_skip.md).
  template <bool PS = false>
  __device__ __forceinline__ void run() {
    mload = t0 - K;
    mlo = t0 - Ch::off(K);
    const int32_t mtop = t1 + K - 1;
    lp = srow + (int64_t)(mtop + 2 - RING) * pitch_b;
    sp = drow + (int64_t)(mtop + Ch::off(K)) * pitch_b;
    // slots 0..RING-3: rows mtop, mtop-1, ...; slots RING-2 / RING-1 stand for
    // rows mtop+2 / mtop+1 (priming only: their results are never stored)
#pragma unroll
    for (int q = 0; q < RING - 2; ++q) load_row(mtop - q >= mload ? mtop - q : mload, Lb[q]);
#pragma unroll
    for (int q = RING - 2; q < RING; ++q)
#pragma unroll
      for (int v = 0; v < NV; ++v) Lb[q][v] = VT{};
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int s = 0; s < KX; ++s)
#pragma unroll
        for (int e = 0; e < V; ++e) X[p][s][e] = T(0);
    const int32_t iters = mtop - mlo + 1;
    const int32_t bodies = (iters + L - 1) / L;
    // priming bodies (deep levels skipped while not needed), then the steady loop
    const int32_t pb = PS ? min(bodies, (int32_t)((Ch::prime_iters + L - 1) / L)) : 0;
    int32_t m = mtop;
    int32_t b = 0;
#pragma unroll 1
    for (; b < pb; ++b) {
      body_prime(m, b * L, std::make_integer_sequence<int, L>{});
      m -= L;
    }
#pragma unroll 1
    for (; b < bodies; ++b) {
      body(m, std::make_integer_sequence<int, L>{});
      m -= L;
    }
  }
};

// fp32 march on PACKED math (v_pk_add_f32 / v_pk_fma_f32 / v_pk_mul_f32: two
// fp32 lanes per VALU op, the fp32 rate CDNA4 quotes). A lane's 16-B vector
// (columns c0..c3) is kept as an even/odd pair of register pairs
// a = (c0, c2), b = (c1, c3), so the in-lane east/west neighbours of a whole
// pair are the other pair (east of a is b, west of b is a) and only the
// across-lane ones are built half by half with single fp32 adds (sadd*, the
// DPP shift folded into v_add_f32_dpp):
//   east of b = (c2, c0 of lane+1),   west of a = (c3 of lane-1, c1).
// Per row and level: 8 packed ops + 4 single adds for 4 points (12 VALU ops).
// With the element-wise layout March<float> uses, the compiler had to
// rebuild misaligned pairs for every packed op (~4.9 VALU ops per point and
// ~2x the registers: 209 VGPRs at K = 10). Same operation order and rounding
// per element as March (bitwise identical); the loads / stores / ring /
// descriptors / edge kinds are March's.
template <int K, int EK, int RING, int AR, bool ST = false, int CL = K>
struct MarchF32 {
  using F2 = float __attribute__((ext_vector_type(2)));
  using VT = float __attribute__((ext_vector_type(4)));
  using U4 = unsigned int __attribute__((ext_vector_type(4)));
  static constexpr int KX = K > 1 ? K - 1 : 1;
  static_assert(RING % 2 == 0 && RING >= 4, "ring must be even and >= 4");
  struct Row {
    F2 a, b;  // a = (c0, c2), b = (c1, c3)
  };

  const char* srow;
  char* drow;
  const char* lp;  // steady-march row pointers (see March)
  char* sp;
  int64_t pitch_b;
  uint32_t nrec;
  float r;
  int32_t t0, t1;
  int32_t fixed_lo, fixed_hi;
  int32_t mlo;    // lowest march row (t0 - off(K))
  int32_t mload;  // lowest level-0 row loaded (t0 - K)
  int32_t ld_off;
  int32_t st_off;
  Row rl;  // EK & 2: r per element (0 in Dirichlet / pad columns)
  float fb, fu, fu1;  // AR 3: TbArgs::fb / fu / fu1
  float fk;           // AR 3: the centre weight 1 - 4r of the unscaled pinned kinds (see March)
  static constexpr bool kScaled = (AR == 2 || AR == 3) && EK == 0;  // levels carried scaled (see March)
  using Ch = ChainShape<K, CL>;
  static constexpr int L = Ch::unroll(RING);
  Row X[3][KX];  // slot 2 only below chain boundaries (see March)
  StatAcc acc;       // ST: statistics of the stored rows
  uint32_t colmask;  // ST: bit e = element e (memory order) is an owned output column
  // Level-0 ring. A slot holds a row in memory order (a = (c0, c1),
  // b = (c2, c3)) from its load until its first use (as the north row), where
  // it is rearranged IN PLACE to the even/odd form: one swap per row instead
  // of a rebuild at each of its three uses.
  Row Lb[RING];

  __device__ __forceinline__ void load_row(int32_t m, Row& out) const { load_row_p(srow + (int64_t)m * pitch_b, true, out); }
  // live == false: below the item's lowest loaded row (priming values only): returns 0
  __device__ __forceinline__ void load_row_p(const char* p, bool live, Row& out) const {
    const __amdgpu_buffer_rsrc_t rs = row_rsrc(p, live ? nrec : 0u);
    const VT v = __builtin_bit_cast(VT, __builtin_amdgcn_raw_buffer_load_b128(rs, ld_off, 0, 0));
    out = Row{F2{v.x, v.y}, F2{v.z, v.w}};
  }
  __device__ __forceinline__ void store_row(bool live, const VT& w) const {
    const __amdgpu_buffer_rsrc_t rs = row_rsrc(sp, live ? nrec : 0u);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(U4, w), rs, st_off, 0, HEAT2D_STORE_AUX);
  }
  static __device__ __forceinline__ Row split(const Row& v) { return Row{F2{v.a.x, v.b.x}, F2{v.a.y, v.b.y}}; }

  // part = S + E(C) (first partial sum of the reference order)
  static __device__ __forceinline__ Row partial(const Row& S, const Row& C) {
    return Row{S.a + C.b, F2{sadd(S.b.x, C.a.y), sadd_from_upper(S.b.y, C.a.x)}};
  }
  // ((part + N) + W): the reference's sum
  static __device__ __forceinline__ Row sum4(const Row& part, const Row& C, const Row& N) {
    const F2 ta = part.a + N.a;
    return Row{F2{sadd_from_lower(ta.x, C.b.y), sadd(ta.y, C.b.x)}, (part.b + N.b) + C.a};
  }
  // AR 2, pinned kinds: re * sum + (C - 4 re C) (see March::update)
  static __device__ __forceinline__ F2 pin2(F2 re, F2 sum, F2 c) {
    const F2 m4 = {-4.f, -4.f};
    return __builtin_elementwise_fma(re, sum, __builtin_elementwise_fma(re, m4 * c, c));
  }
  static __device__ __forceinline__ float pin1(float re, float sum, float c) {
    return __builtin_fmaf(re, sum, __builtin_fmaf(re, -4.f * c, c));
  }
  // sum - 4C (in) and the per-element r (re) of the update C + r*(sum - 4C)
  __device__ __forceinline__ void terms(const Row& part, const Row& C, const Row& N, int32_t row, Row& in,
                                        Row& re) const {
    const Row sum = sum4(part, C, N);
    const F2 m4 = {-4.f, -4.f};
    in = Row{__builtin_elementwise_fma(m4, C.a, sum.a), __builtin_elementwise_fma(m4, C.b, sum.b)};
    const bool frame_row = (EK & 1) && ((uint32_t)(row - fixed_lo) >= (uint32_t)(fixed_hi - fixed_lo));  // wave-uniform
    if constexpr (EK == 0) {
      re = Row{F2{r, r}, F2{r, r}};
    } else if constexpr (EK == 1) {
      const float rs = frame_row ? 0.f : r;
      re = Row{F2{rs, rs}, F2{rs, rs}};
    } else if constexpr (EK == 2) {
      re = rl;
    } else {
      const F2 z = {0.f, 0.f};
      re = frame_row ? Row{z, z} : rl;
    }
  }
  __device__ __forceinline__ Row update(const Row& part, const Row& C, const Row& N, int32_t row) const {
    if constexpr (AR == 3 && EK == 0) {  // scaled: fma(b, C, sum) on packed pairs
      const Row sum = sum4(part, C, N);
      const F2 b2 = {fb, fb};
      return Row{__builtin_elementwise_fma(b2, C.a, sum.a), __builtin_elementwise_fma(b2, C.b, sum.b)};
    }
    if constexpr (AR == 2 || AR == 3) {  // (AR 3, kind 0: above)
      const Row sum = sum4(part, C, N);
      if constexpr (EK == 0) return sum;  // scaled: 4^s T
      const bool frame_row = (EK & 1) && ((uint32_t)(row - fixed_lo) >= (uint32_t)(fixed_hi - fixed_lo));  // wave-uniform
      if constexpr (EK == 1) {  // fma(ke, C, re * sum), scalar (re, ke) (see March::update)
        const float k0 = frame_row ? 1.f : (AR == 3 ? fk : 0.f);
        const F2 re = {frame_row ? 0.f : r, frame_row ? 0.f : r}, ke = {k0, k0};
        return Row{__builtin_elementwise_fma(ke, C.a, re * sum.a), __builtin_elementwise_fma(ke, C.b, re * sum.b)};
      }
      const F2 z = {0.f, 0.f};
      const Row re = (EK == 3 && frame_row) ? Row{z, z} : rl;
      return Row{pin2(re.a, sum.a, C.a), pin2(re.b, sum.b, C.b)};
    }
    Row in, re;
    terms(part, C, N, row, in, re);
    if constexpr (AR == 1)
      return Row{__builtin_elementwise_fma(re.a, in.a, C.a), __builtin_elementwise_fma(re.b, in.b, C.b)};
    else
      return Row{C.a + re.a * in.a, C.b + re.b * in.b};
  }
  static __device__ __forceinline__ float fin(float re, float in, float c) {
    if constexpr (AR == 1) return __builtin_fmaf(re, in, c);
    else return c + re * in;
  }
  // The stored (last) level: its 4 final ops as scalar fp32 ops writing the
  // store vector in memory order (c0, c1, c2, c3) — a packed op would produce
  // the even/odd pairs and need a transpose before the 16-B store.
  __device__ __forceinline__ VT update_last(const Row& part, const Row& C, const Row& N, int32_t row) const {
    if constexpr (AR == 3 && EK == 0) {  // scaled level K, unscaled by r^K at the store
      const Row sum = sum4(part, C, N);
      return VT{__builtin_fmaf(fb, C.a.x, sum.a.x) * fu, __builtin_fmaf(fb, C.b.x, sum.b.x) * fu,
                __builtin_fmaf(fb, C.a.y, sum.a.y) * fu, __builtin_fmaf(fb, C.b.y, sum.b.y) * fu};
    }
    if constexpr (AR == 2 || AR == 3) {  // (AR 3, kind 0: above)
      const Row sum = sum4(part, C, N);
      if constexpr (EK == 0) {
        // unscale 4^K T once, at the store (exact)
        constexpr float u = inv_pow4<float>(K);
        return VT{sum.a.x * u, sum.b.x * u, sum.a.y * u, sum.b.y * u};
      }
      const bool frame_row = (EK & 1) && ((uint32_t)(row - fixed_lo) >= (uint32_t)(fixed_hi - fixed_lo));  // wave-uniform
      if constexpr (EK == 1) {
        const float re = frame_row ? 0.f : r, ke = frame_row ? 1.f : (AR == 3 ? fk : 0.f);
        return VT{__builtin_fmaf(ke, C.a.x, re * sum.a.x), __builtin_fmaf(ke, C.b.x, re * sum.b.x),
                  __builtin_fmaf(ke, C.a.y, re * sum.a.y), __builtin_fmaf(ke, C.b.y, re * sum.b.y)};
      }
      const F2 z = {0.f, 0.f};
      const Row re = (EK == 3 && frame_row) ? Row{z, z} : rl;
      return VT{pin1(re.a.x, sum.a.x, C.a.x), pin1(re.b.x, sum.b.x, C.b.x), pin1(re.a.y, sum.a.y, C.a.y),
                pin1(re.b.y, sum.b.y, C.b.y)};
    }
    Row in, re;
    terms(part, C, N, row, in, re);
    return VT{fin(re.a.x, in.a.x, C.a.x), fin(re.b.x, in.b.x, C.b.x), fin(re.a.y, in.a.y, C.a.y),
              fin(re.b.y, in.b.y, C.b.y)};
  }

  template <int PH, bool PRIME = false>
  __device__ __forceinline__ void step(int32_t m, int32_t nl = K) {
    constexpr int P0 = PH % RING;
    constexpr int sN = P0, sC = (P0 + RING - 1) % RING, sS = (P0 + RING - 2) % RING;
    const Row C0 = Lb[sC];
    Row part = partial(Lb[sS], C0);
    {
      const int32_t nxt = m + 2 - RING;
      __builtin_amdgcn_sched_barrier(0);
      load_row_p(lp, nxt >= mload, Lb[sS]);
      lp -= pitch_b;
    }
    Lb[sN] = split(Lb[sN]);  // first use of this row: to even/odd form, in place
    const Row N0 = Lb[sN];
#pragma unroll
    for (int s = 1; s <= K; ++s) {
      if (PRIME && s > nl) continue;  // wave-uniform guard (see March)
      const int d = Ch::delta(s);
      const int j = s > 1 ? s - 1 : 1;
      const Row C = s == 1 ? C0 : X[Ch::slot(PH, d, j)][j - 1];
      const Row N = s == 1 ? N0 : X[Ch::slot(PH, d - 1, j)][j - 1];
      if (s < K) {
        const int i = s < K ? s - 1 : 0;
        const int ps = Ch::slot(PH, 0, s < K ? s : 1);
        const Row nxtpart = partial(X[ps][i], X[Ch::slot(PH, Ch::delta(s + 1), s < K ? s : 1)][i]);
        X[ps][i] = update(part, C, N, m + Ch::off(s));
        part = nxtpart;
      } else {
        const int32_t row = m + Ch::off(K);
        const bool live = (uint32_t)(row - t0) < (uint32_t)(t1 - t0);  // row in [t0, t1), wave-uniform
        const VT w = update_last(part, C, N, row);
        store_row(live, w);
        if constexpr (ST) {
          if (live) {  // C in even/odd form: a = (c0, c2), b = (c1, c3)
            const float cu = kScaled ? (AR == 2 ? inv_pow4<float>(K - 1) : fu1) : 1.f;  // level K-1 scale
            acc.add(colmask & 1u, (double)w.x, (double)(C.a.x * cu));
            acc.add((colmask >> 1) & 1u, (double)w.y, (double)(C.b.x * cu));
            acc.add((colmask >> 2) & 1u, (double)w.z, (double)(C.a.y * cu));
            acc.add((colmask >> 3) & 1u, (double)w.w, (double)(C.b.y * cu));
          }
        }
      }
    }
    sp -= pitch_b;
  }

  template <int... I>
  __device__ __forceinline__ void body(int32_t m, std::integer_sequence<int, I...>) {
    (step<I>(m - I), ...);
  }
  template <int... I>
  __device__ __forceinline__ void body_prime(int32_t m, int32_t i, std::integer_sequence<int, I...>) {
    (step<I, true>(m - I, Ch::levels_at(i + I)), ...);
  }

  // PS: skip the levels the first march rows do not need (priming). The
  // interior kernels use it (fp64 too since round 5: +5-8 % per pass at
  // depths 13..20 although it costs some of them an occupancy level,
  // profiles/r5/i/, r5/j/); the general kernels do not (4-5 % slower for the
  // 1-wave/SIMD fp32 small grid, profiles/priming_skip.md).
  template <bool PS = false>
  __device__ __forceinline__ void run() {
    mload = t0 - K;
    mlo = t0 - Ch::off(K);
    const int32_t mtop = t1 + K - 1;
    lp = srow + (int64_t)(mtop + 2 - RING) * pitch_b;
    sp = drow + (int64_t)(mtop + Ch::off(K)) * pitch_b;
#pragma unroll
    for (int q = 0; q < RING - 2; ++q) load_row(mtop - q >= mload ? mtop - q : mload, Lb[q]);
#pragma unroll
    for (int q = RING - 2; q < RING; ++q) Lb[q] = Row{F2{0.f, 0.f}, F2{0.f, 0.f}};
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int s = 0; s < KX; ++s) X[p][s] = Row{F2{0.f, 0.f}, F2{0.f, 0.f}};
    const int32_t iters = mtop - mlo + 1;
    const int32_t bodies = (iters + L - 1) / L;
    // priming bodies (deep levels skipped while not needed), then the steady loop
    const int32_t pb = PS ? min(bodies, (int32_t)((Ch::prime_iters + L - 1) / L)) : 0;
    int32_t m = mtop;
    int32_t b = 0;
#pragma unroll 1
    for (; b < pb; ++b) {
      body_prime(m, b * L, std::make_integer_sequence<int, L>{});
      m -= L;
    }
#pragma unroll 1
    for (; b < bodies; ++b) {
      body(m, std::make_integer_sequence<int, L>{});
      m -= L;
    }
  }
};

// Packed fp32 march (MarchF32) for the 16-B-per-lane float kernels; set
// HEAT2D_NO_PACKED_F32 at build time to compile the element-wise March instead
// (A/B builds).
#ifndef HEAT2D_NO_PACKED_F32
template <typename T, int NV>
constexpr bool kPackedF32 = std::is_same<T, float>::value && NV == 1;
#else
template <typename T, int NV>
constexpr bool kPackedF32 = false;
#endif

template <typename T, int NV, int K, int EK, int RING, int AR, bool ST = false, bool PS = false, int CLX = 0>
__device__ __forceinline__ void march(const T* src, T* dst, const TbArgs& a, T r, int64_t strip, int64_t t0,
                                      int64_t t1, int lane, StatAcc* acc = nullptr) {
  using S = TbShape<T, NV, K>;
  constexpr int V = S::V;
  constexpr int ES = (int)sizeof(T);
  const int64_t u0 = strip * S::U;
  const int64_t c0 = u0 - S::KA;
  const int64_t mycol = c0 + (int64_t)lane * V;
  const int64_t ustop = min(u0 + (int64_t)S::U, a.ncols);
  // the fused-statistics variant keeps one chain: its accumulators on top of
  // the chains' extra rows spill at fp64 K >= 21
  // (CLX > 0: an explicit chain length — the boundary-band kernel)
  constexpr int CL = CLX > 0 ? (CLX < K ? CLX : K) : (ST ? K : chain_len<T, K>());
  using W = typename std::conditional<kPackedF32<T, NV>, MarchF32<K, EK, RING, AR, ST, CL>,
                                      March<T, NV, K, EK, RING, AR, ST, CL>>::type;
  W w;
  // row base = column col_lo (= -cpad) of row 0; offsets are relative to it
  w.srow = reinterpret_cast<const char*>(src + a.col_lo);
  w.drow = reinterpret_cast<char*>(dst + a.col_lo);
  w.pitch_b = a.pitch * ES;
  w.nrec = (uint32_t)(a.pitch * ES);
  w.r = r;
  if constexpr (AR == 3) {
    w.fk = (T)(1.0 - 4.0 * (double)r);
    w.fb = (T)a.fb;
    w.fu = (T)a.fu;
    w.fu1 = (T)a.fu1;
  }
  w.t0 = (int32_t)t0;
  w.t1 = (int32_t)t1;
  w.fixed_lo = (int32_t)a.fixed_lo;
  w.fixed_hi = (int32_t)a.fixed_hi;
  const int32_t off = (int32_t)((mycol - a.col_lo) * ES);
  const bool in_alloc = (mycol >= a.col_lo) && (mycol + V <= a.col_hi);
  w.ld_off = in_alloc ? off : kOob;
  // Strip boundaries u0 are multiples of V, so a lane holds either only halo
  // columns or only useful ones — except the lane straddling ncols, whose
  // vector also covers the Dirichlet column / right pad. Those elements are
  // pinned (r = 0) at every level, so storing the whole vector writes them
  // back unchanged: one 16-B store per lane, no per-element stores. (dst's
  // frame equals src's frame by construction.)
  const bool useful = (mycol >= u0) && (mycol < ustop);
  w.st_off = useful && in_alloc ? off : kOob;
  if constexpr ((EK & 2) != 0) {
    auto rcol = [&](int e) { return (mycol + e < 0 || mycol + e >= a.ncols) ? T(0) : r; };
    if constexpr (kPackedF32<T, NV>) {
      w.rl.a = {rcol(0), rcol(2)};
      w.rl.b = {rcol(1), rcol(3)};
    } else {
#pragma unroll
      for (int e = 0; e < V; ++e) w.rl[e] = rcol(e);
    }
  }
  if constexpr (ST) {
    uint32_t mask = 0;
#pragma unroll
    for (int e = 0; e < V; ++e) mask |= (useful && mycol + e >= 0 && mycol + e < a.ncols) ? (1u << e) : 0u;
    w.colmask = mask;
    w.acc = *acc;
    w.run();
    *acc = w.acc;
  } else {
    w.template run<PS>();
  }
}

// Work item `it` -> a range [lin, lin_end) of its rect's strip-major row
// sequence (lin = strip_local * rows + row_local), marched piece by piece, one
// piece per strip it touches.
//   nb > 0: row bands — item = (band, strip), band-major; one piece.
//   nb < 0: -nb equal segments of the whole sequence — item = segment; a
//           segment may cross strip ends (1-2 pieces when segments are shorter
//           than a strip). Every wave gets the same row count whatever the
//           strip count, which bands (whole rows x whole strips) cannot give a
//           thin slab: profiles/thin_slab.md.
// Only (it, lin) are carried across a march (the rest is recomputed from the
// kernarg per piece): more loop-carried SGPRs spill into VGPR lanes and cost
// the deep fp64 interior kernels a wave per SIMD. lin < 2^31 (host-checked).
struct TbSpan {
  int32_t lin, lin_end, rows;
  int64_t r0, s0;
};
// floor(a * b / c) for 0 <= a, b and 0 < c with a result below 2^31 (host
// checks: strip rows < 2^31): a double-precision quotient corrected to the
// exact one (its error is below 1), instead of a 64-bit integer division —
// ~100 scalar ops each, four per item lookup, on waves that are alone on
// their SIMD.
__device__ __forceinline__ int64_t muldiv(int64_t a, int64_t b, int64_t c) {
  const int64_t p = a * b;
  int64_t q = (int64_t)((double)p / (double)c);
  while (q > 0 && q * c > p) --q;
  while ((q + 1) * c <= p) ++q;
  return q;
}
// NR: rects the kernel instance can be handed (the interior kernels take at
// most 4: a larger scan costs the deep fp64 ones SGPRs that spill to scratch).
template <int NR = kMaxRects>
__device__ __forceinline__ TbSpan tb_span(const TbArgs& a, int64_t it) {
  // select the rect with constant indices only (a dynamic index into the
  // by-value kernarg struct would be lowered to a private-memory copy)
  TbRectArg R = a.rect[0];
#pragma unroll
  for (int i = 1; i < NR; ++i)
    if (i < a.nrect && it >= a.rect[i].item0) R = a.rect[i];
  const int64_t local = it - R.item0;
  const int64_t ns = R.s1 - R.s0;
  const int64_t rows = R.r1 - R.r0;
  TbSpan g{0, 0, (int32_t)rows, R.r0, R.s0};
  if (R.nb > 0) {
    const int64_t band = muldiv(local, 1, ns), sl = local - band * ns;
    g.lin = (int32_t)(sl * rows + muldiv(band, rows, R.nb));
    g.lin_end = (int32_t)(sl * rows + muldiv(band + 1, rows, R.nb));
  } else {
    const int64_t total = ns * rows, nseg = -R.nb;
    g.lin = (int32_t)muldiv(local, total, nseg);
    g.lin_end = (int32_t)muldiv(local + 1, total, nseg);
  }
  return g;
}
// The piece of item `it` starting at lin -> (strip, output rows [t0, t1));
// false when lin is past the item. Advance with lin += t1 - t0.
template <int NR = kMaxRects>
__device__ __forceinline__ bool tb_piece(const TbArgs& a, int64_t it, int32_t lin, int64_t& strip, int64_t& t0,
                                         int64_t& t1) {
  const TbSpan g = tb_span<NR>(a, it);
  if (lin >= g.lin_end) return false;
  const int32_t sl = lin / g.rows, row = lin - sl * g.rows;
  strip = g.s0 + sl;
  t0 = g.r0 + row;
  t1 = t0 + min(g.rows - row, g.lin_end - lin);
  return true;
}

// MAIN = true: the caller guarantees no item reaches a frame ROW (the slab
// interior of the split schedule): items are kind 0, or kind 2 on the
// frame-column strips — two code paths, fewer registers than the general
// kernel (no per-level row tests, no corner selects). MAIN = false: the general
// kernel classifies each item (edge kinds 0..3, see March).
// Occupancy floor handed to the register allocator: the fp64 interior kernels
// with ring 4 keep 2 waves/SIMD at K = 17 and 21..24 under a floor; at K =
// 18..20 a floor spills since the priming skip (their ring-6 twins fit 226-247
// VGPRs, which the autotuner weighs; round 4's fma K = 11 floor of 4 waves
// spills with the skip too). (The packed fp32 march with the single
// across-lane adds spills under a 3-wave floor from K = 12 on, so it has none.)
// The fp32 interior kernels at K = 17..20 (ring 4) keep 2 waves/SIMD under a
// floor. Checked per build: ScratchSize = 0 in the ISA (tools/isa_report.py,
// tests/test_isa.py).
template <typename T, int NV, int K, int RING, bool MAIN, int AR>
constexpr int kMinWaves = (std::is_same<T, double>::value && MAIN && RING == 4 && (K == 17 || K >= 21))   ? 2
                          : (std::is_same<T, float>::value && MAIN && RING == 4 && K >= 17)                        ? 2
                                                                                                                  : 1;

// wave-wide sum / min / max (fixed xor butterfly: every lane ends with the
// same bits, lane 0's are written)
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_min(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ bool lane_id_is0() { return (threadIdx.x & 63) == 0; }

// The wave's next work item after `it` (static grid stride, or the dynamic queue).
__device__ __forceinline__ int64_t next_item(const TbArgs& a, int64_t it) {
  if (!a.queue) return it + a.nwaves;
  uint32_t v = 0;
  if (lane_id_is0()) v = __hip_atomic_fetch_add(a.queue, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return a.nwaves + (int64_t)__builtin_amdgcn_readfirstlane(v);
}
__device__ __forceinline__ void queue_exit(const TbArgs& a) {
  if (!a.queue || !lane_id_is0()) return;
  const uint32_t d = __hip_atomic_fetch_add(a.queue + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (d + 1u == (uint32_t)a.nwaves) {  // every wave has taken its last item: reset for the next launch
    __hip_atomic_store(a.queue, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(a.queue + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Kernel variants (VAR): 0 plain; 1 fused statistics (StatAcc; general kernel).
// (A latency-oriented variant for the boundary-band launch — priming skip +
// dependency chains — measured slower everywhere and was removed:
// profiles/edge_kernel.md. So was the fused-cycle interior kernel, whose
// first items were the bands the exchange sends: one such launch ran 720 us
// where band launch + interior take 647 (edge-first) or 610 (lead order),
// profiles/r4/lead/.)
constexpr int kVarPlain = 0, kVarStats = 1;

template <typename T, int NV, int K, int RING, bool MAIN, int AR, int VAR = kVarPlain>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(VAR == kVarPlain ? kMinWaves<T, NV, K, RING, MAIN, AR> : 1))) void tb_kernel(const T* __restrict__ src, T* __restrict__ dst, TbArgs a, T r) {
  constexpr bool ST = VAR == kVarStats;
  static_assert(VAR != kVarStats || !MAIN, "the statistics variant uses the general kernel");
  using S = TbShape<T, NV, K>;
  const int lane = threadIdx.x & 63;
  // readfirstlane: make the wave id (and everything derived from it: strip, rows,
  // row addresses) provably wave-uniform -> SGPRs and scalar buffer descriptors
  // (Blocks are dealt round-robin over the 8 XCDs; numbering them so that each
  // XCD owns a contiguous run of strips cut the strip-halo re-fetch from 1.14x
  // to 1.07x of the field but cost 6 % fp64 / 3 % fp32 — the round-robin
  // numbering streams HBM better: profiles/README.md §8. Removed in round 5.)
  const int64_t wid = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  if (wid >= a.nwaves) return;  // whole wave exits; no barriers in this kernel
  if (a.wtimes && lane_id_is0()) a.wtimes[wid * 4] = wall_clock64();
  // Band items are band-major within a rect: consecutive waves take adjacent
  // strips of the same band, so the waves in flight stream whole contiguous
  // rows (HBM page locality) and all march in step.
  StatAcc acc;
  // one flat loop over the pieces of items wid, wid + nwaves, ... (a nested
  // piece loop around the march costs the deep fp64 kernels registers)
  constexpr int NR = MAIN ? kMainRects : kMaxRects;
  int64_t it = wid;
  int32_t lin = tb_span<NR>(a, it).lin;
  while (it < a.nitems) {
    int64_t strip, t0, t1;
    if (!tb_piece<NR>(a, it, lin, strip, t0, t1)) {
      it = next_item(a, it);
      if (it < a.nitems) lin = tb_span<NR>(a, it).lin;
      continue;
    }
    lin += (int32_t)(t1 - t0);
    const int64_t c0 = strip * S::U - S::KA;
    if constexpr (ST) {
      const int ek = (((t0 - K < a.fixed_lo) || (t1 + K > a.fixed_hi)) ? 1 : 0) |
                     (((c0 < 0) || (c0 + S::W > a.ncols)) ? 2 : 0);
      switch (ek) {
        case 0: march<T, NV, K, 0, RING, AR, true>(src, dst, a, r, strip, t0, t1, lane, &acc); break;
        case 1: march<T, NV, K, 1, RING, AR, true>(src, dst, a, r, strip, t0, t1, lane, &acc); break;
        case 2: march<T, NV, K, 2, RING, AR, true>(src, dst, a, r, strip, t0, t1, lane, &acc); break;
        default: march<T, NV, K, 3, RING, AR, true>(src, dst, a, r, strip, t0, t1, lane, &acc); break;
      }
    } else if constexpr (MAIN) {
      if ((c0 < 0) || (c0 + S::W > a.ncols))
        march<T, NV, K, 2, RING, AR, false, true>(src, dst, a, r, strip, t0, t1, lane);
      else
        march<T, NV, K, 0, RING, AR, false, true>(src, dst, a, r, strip, t0, t1, lane);
    } else {
      const int ek = (((t0 - K < a.fixed_lo) || (t1 + K > a.fixed_hi)) ? 1 : 0) |
                     (((c0 < 0) || (c0 + S::W > a.ncols)) ? 2 : 0);
      switch (ek) {
        case 0: march<T, NV, K, 0, RING, AR>(src, dst, a, r, strip, t0, t1, lane); break;
        case 1: march<T, NV, K, 1, RING, AR>(src, dst, a, r, strip, t0, t1, lane); break;
        case 2: march<T, NV, K, 2, RING, AR>(src, dst, a, r, strip, t0, t1, lane); break;
        default: march<T, NV, K, 3, RING, AR>(src, dst, a, r, strip, t0, t1, lane); break;
      }
    }
  }
  queue_exit(a);
  if (a.wtimes && lane_id_is0()) {
    a.wtimes[wid * 4 + 1] = wall_clock64();
    a.wtimes[wid * 4 + 2] = (uint64_t)wid;
  }
  if constexpr (ST) {
    const double v[kNStatFused] = {wave_sum(acc.s), wave_sum(acc.ss), wave_min(acc.mn),
                                   wave_max(acc.mx), wave_sum(acc.dd), wave_max(acc.md)};
    if (lane == 0) {
#pragma unroll
      for (int j = 0; j < kNStatFused; ++j) a.partials[j * a.nwaves + wid] = v[j];
    }
  }
}

template <typename T, int NV, int K, int RING, bool MAIN, int AR, int VAR = kVarPlain>
constexpr auto kernel_ptr() {
  return &tb_kernel<T, NV, K, RING, MAIN, AR, VAR>;
}

// Resident 256-thread workgroups per CU for one kernel instance (occupancy API).
template <typename T, int NV, int K, int RING, bool MAIN, int AR, int VAR = kVarPlain>
int blocks_per_cu() {
  static std::mutex mu;
  static std::map<int, int> cache;  // device -> blocks/CU
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find(dev);
  if (it != cache.end()) return it->second;
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, reinterpret_cast<const void*>(kernel_ptr<T, NV, K, RING, MAIN, AR, VAR>()),
                                                   256, 0) != hipSuccess ||
      nb <= 0)
    nb = 1;
  cache[dev] = nb;
  return nb;
}

// Per-(T, RING, MAIN, AR) entry points (16 B per lane), explicitly instantiated in
// tb_<dtype>_r<RING>_<main|gen>[_fma].hip (one translation unit each, compiled in parallel).
template <typename T, int RING, bool MAIN, int AR>
void dispatch(int k, unsigned nblocks, const T* src, T* dst, const TbArgs& a, T r, hipStream_t s);
template <typename T, int RING, bool MAIN, int AR>
int occupancy_blocks(int k);
// fused-statistics kernels: general kernel, ring 4 (tb_<dtype>_stats.hip)
template <typename T, int AR>
void dispatch_stats(int k, unsigned nblocks, const T* src, T* dst, const TbArgs& a, T r, hipStream_t s);
template <typename T, int AR>
int occupancy_blocks_stats(int k);
#define H2D_TB_CASE(T, RING, MAIN, AR, KK)                                                                    \
  case KK:                                                                                                    \
    hipLaunchKernelGGL((tb_kernel<T, 1, KK, RING, MAIN, AR>), dim3(nblocks), dim3(256), 0, s, src, dst, a, r); \
    return;
#define H2D_OCC_CASE(T, RING, MAIN, AR, KK) \
  case KK:                                  \
    return blocks_per_cu<T, 1, KK, RING, MAIN, AR>();

// Instantiate dispatch/occupancy for K = 1..16 of one (T, RING, MAIN, AR).
#define H2D_TB_CASES(M, T, RING, MAIN, AR)                                                             \
  M(T, RING, MAIN, AR, 1) M(T, RING, MAIN, AR, 2) M(T, RING, MAIN, AR, 3) M(T, RING, MAIN, AR, 4)       \
  M(T, RING, MAIN, AR, 5) M(T, RING, MAIN, AR, 6) M(T, RING, MAIN, AR, 7) M(T, RING, MAIN, AR, 8)       \
  M(T, RING, MAIN, AR, 9) M(T, RING, MAIN, AR, 10) M(T, RING, MAIN, AR, 11) M(T, RING, MAIN, AR, 12)    \
  M(T, RING, MAIN, AR, 13) M(T, RING, MAIN, AR, 14) M(T, RING, MAIN, AR, 15) M(T, RING, MAIN, AR, 16)
// fp32: K = 17..24 (kMaxTBF32, common.hpp): the big fp32 grids are HBM-bound
// at K = 16-20, and the packed interior march fits K = 24 in 2 waves/SIMD
#define H2D_TB_CASES_F32DEEP(M, T, RING, MAIN, AR)                                                     \
  M(T, RING, MAIN, AR, 17) M(T, RING, MAIN, AR, 18) M(T, RING, MAIN, AR, 19) M(T, RING, MAIN, AR, 20)   \
  M(T, RING, MAIN, AR, 21) M(T, RING, MAIN, AR, 22) M(T, RING, MAIN, AR, 23) M(T, RING, MAIN, AR, 24)
// fp64 only: K = 17..24 (kMaxTB)
#define H2D_TB_CASES_DEEP(M, T, RING, MAIN, AR)                                                        \
  M(T, RING, MAIN, AR, 17) M(T, RING, MAIN, AR, 18) M(T, RING, MAIN, AR, 19) M(T, RING, MAIN, AR, 20)   \
  M(T, RING, MAIN, AR, 21) M(T, RING, MAIN, AR, 22) M(T, RING, MAIN, AR, 23) M(T, RING, MAIN, AR, 24)
#define H2D_NO_CASES(M, T, RING, MAIN, AR)
#define H2D_TB_UNIT_IMPL(T, RING, MAIN, AR, DEEP)                                                       \
  template <>                                                                                           \
  void dispatch<T, RING, MAIN, AR>(int k, unsigned nblocks, const T* src, T* dst, const TbArgs& a, T r, \
                                   hipStream_t s) {                                                     \
    switch (k) {                                                                                        \
      H2D_TB_CASES(H2D_TB_CASE, T, RING, MAIN, AR)                                                      \
      DEEP(H2D_TB_CASE, T, RING, MAIN, AR)                                                              \
      default:                                                                                          \
        break;                                                                                          \
    }                                                                                                   \
    HEAT2D_REQUIRE(false, "temporal depth not instantiated for this variant");                          \
  }                                                                                                     \
  template <>                                                                                           \
  int occupancy_blocks<T, RING, MAIN, AR>(int k) {                                                      \
    switch (k) {                                                                                        \
      H2D_TB_CASES(H2D_OCC_CASE, T, RING, MAIN, AR)                                                     \
      DEEP(H2D_OCC_CASE, T, RING, MAIN, AR)                                                             \
      default:                                                                                          \
        break;                                                                                          \
    }                                                                                                   \
    return 1;                                                                                           \
  }
#define H2D_TB_UNIT(T, RING, MAIN, AR) H2D_TB_UNIT_IMPL(T, RING, MAIN, AR, H2D_NO_CASES)
#define H2D_TB_UNIT_F64(T, RING, MAIN, AR) H2D_TB_UNIT_IMPL(T, RING, MAIN, AR, H2D_TB_CASES_DEEP)
#define H2D_TB_UNIT_F32(T, RING, MAIN, AR) H2D_TB_UNIT_IMPL(T, RING, MAIN, AR, H2D_TB_CASES_F32DEEP)
#define H2D_ST_CASE(T, RING, MAIN, AR, KK)                                                                        \
  case KK:                                                                                                        \
    hipLaunchKernelGGL((tb_kernel<T, 1, KK, 4, false, AR, kVarStats>), dim3(nblocks), dim3(256), 0, s, src, dst, a, \
                       r);                                                                                        \
    return;
#define H2D_ST_OCC_CASE(T, RING, MAIN, AR, KK) \
  case KK:                                     \
    return blocks_per_cu<T, 1, KK, 4, false, AR, kVarStats>();
#define H2D_ST_UNIT(T, AR, DEEP)                                                                              \
  template <>                                                                                                 \
  void dispatch_stats<T, AR>(int k, unsigned nblocks, const T* src, T* dst, const TbArgs& a, T r,             \
                             hipStream_t s) {                                                                 \
    switch (k) {                                                                                              \
      H2D_TB_CASES(H2D_ST_CASE, T, 4, false, AR)                                                              \
      DEEP(H2D_ST_CASE, T, 4, false, AR)                                                                      \
      default:                                                                                                \
        break;                                                                                                \
    }                                                                                                         \
    HEAT2D_REQUIRE(false, "temporal depth not instantiated for the statistics kernel");                       \
  }                                                                                                           \
  template <>                                                                                                 \
  int occupancy_blocks_stats<T, AR>(int k) {                                                                  \
    switch (k) {                                                                                              \
      H2D_TB_CASES(H2D_ST_OCC_CASE, T, 4, false, AR)                                                          \
      DEEP(H2D_ST_OCC_CASE, T, 4, false, AR)                                                                  \
      default:                                                                                                \
        break;                                                                                                \
    }                                                                                                         \
    return 1;                                                                                                 \
  }


}  // namespace tbimpl
}  // namespace kern
}  // namespace heat2d
