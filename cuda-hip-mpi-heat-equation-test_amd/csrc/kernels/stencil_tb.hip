// Temporal-blocked 5-point FTCS stencil for gfx950 (CDNA4): host-side
// planning and launch. Device code: tb_impl.hpp; instantiations: tb_*.hip.
//
// Replaces reference K1 `heat_eqn` (fortran/hip/heat_kernel.cpp:31-45: one
// thread per point, 5 scalar loads, 128x4 blocks) and K12, the per-step
// full-field D2D copy (fortran/hip/heat.F90:243).
//
// Design (wave64, no LDS, no barriers):
//   * one WAVE owns a column strip of 64*V columns (V = NV * 16 B / sizeof(T))
//     and marches UP a run of rows, loading each input row exactly once with
//     NV 16-B loads per lane (1 KiB per wave instruction);
//   * K time levels are pipelined in registers: at march row m the wave loads
//     row m of level 0 and computes row m+s of level s for s = 1..K, so K time
//     steps cost ONE HBM read + ONE HBM write per point (the single-step
//     roofline is 16 B/pt fp64; at K = 8 the kernel needs 2 B/pt);
//   * marching upward puts the OLDEST row first in the reference's summation
//     order, so each level needs only 2 rows of register state (parity ring)
//     and a 5-op dependency chain from the freshly computed row;
//   * east/west neighbours come from the adjacent lane through DPP
//     wave_shr:1 / wave_shl:1 (VALU modifiers, no LDS traffic); the strip's
//     outer K columns are redundant halo work (shrinking valid region);
//   * loads/stores are raw buffer ops on per-row descriptors with out-of-range
//     voffsets for masked lanes (and num_records = 0 for priming rows): no
//     memory op under control flow, so the RING-row prefetch is waited for
//     with counted vmcnt(N);
//   * persistent grid: as many waves as the chip holds resident
//     (occupancy API x CUs), work items = (row band, strip), band-major;
//   * the arithmetic order is exactly the reference's
//     c + r*((((S + E) + N) + W) - 4c) (fortran/hip/heat_kernel.cpp:43, with
//     S = T(x+1,y), E = T(x,y+1), N = T(x-1,y), W = T(x,y-1)) and the file is
//     built with -ffp-contract=off: results are bitwise identical to the CPU
//     reference and to an unblocked K=1 run, in fp64 and in fp32. arith = 1
//     selects the contracted form fma(r, sum - 4c, c) (one op fewer per point;
//     bitwise equal to its CPU twin; equal to arith 0 when r is a power of two).
//     arith = 2 (r == 1/4 only): ((((S + E) + N) + W)) / 4, the update with its
//     zero centre weight folded away — 3 adds + 2 DPP moves per interior point
//     and level (levels carried scaled by 4^level, tb_impl.hpp); bitwise equal
//     to its CPU twin, and to arith 0 on data where sum - 4c is exact.
#include <cmath>
#include <type_traits>

#include "tb_impl.hpp"

namespace heat2d {
namespace kern {
namespace {
using namespace tbimpl;

int cu_count() {
  static std::mutex mu;
  static std::map<int, int> cache;
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find(dev);
  if (it != cache.end()) return it->second;
  int n = 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  cache[dev] = n;
  return n;
}

int vec_elems(DType dt) { return dt == DType::F32 ? 4 : 2; }

// halo columns per strip side (whole lanes) and useful strip width; must match TbShape
int halo_cols(DType dt, int k) {
  const int v = vec_elems(dt);
  return (k + v - 1) / v * v;
}
int useful_width(DType dt, int k) { return 64 * vec_elems(dt) - 2 * halo_cols(dt, k); }

// Level-0 row ring per wave (RING - 2 rows in flight; the march loop is
// unrolled RING times). Override: HEAT2D_TB_RING=4|6.
int default_ring(DType dt, int k) {
  if (const char* env = std::getenv("HEAT2D_TB_RING")) {
    const int r = std::atoi(env);
    if (r == 4 || r == 6 || r == 8) return r;
  }
  // measured on MI355X (bench/sweep.py, 32768^2, profiles/sweep_split_32768.txt)
  if (dt == DType::F64) return k <= 10 ? 6 : 4;
  return (k == 10 || k == 11) ? 6 : 4;  // (K > 16: ring 4, see ring_ok)
}

// fp32 K = 17..20 exist with ring 4 only (ring 6 needs > 256 VGPRs there and
// spilled in the general kernel): every plan of those depths uses ring 4.
// Ring 8 (6 rows in flight) exists only for the fp32 general kernel at K <= 16,
// for single launches (plan_single): one wave per SIMD there, whose loads wait
// on memory ~20 % of its life with 4 rows in flight (SQ_WAIT_ANY,
// profiles/r3/pairprof/); other plans fall back to ring 6.
// (Ring 10, and ring 8 for the fp64 general kernel, measured no better:
// profiles/r3/ring10/.)
int ring_ok(DType dt, int k, int ring, bool single = false) {
  if (dt == DType::F32 && k > 16) return 4;
  if (ring == 8 && !(single && k <= 16 && dt == DType::F32)) return 6;
  return ring;
}
bool ring_valid(int r) { return r == 4 || r == 6 || r == 8; }

// arith code -> the kernels' AR template argument (0 reference rounding,
// 1 contracted fma, 2 r = 1/4, 3 any r with scaled levels: tb_impl.hpp); f is
// called with std::integral_constant<int, AR>.
template <class F>
decltype(auto) with_ar(int arith, F&& f) {
  HEAT2D_REQUIRE(arith >= 0 && arith <= 3, "arith must be 0 (exact), 1 (fma), 2 (r = 1/4) or 3 (fast)");
  if (arith == 3) return f(std::integral_constant<int, 3>{});
  if (arith == 2) return f(std::integral_constant<int, 2>{});
  if (arith == 1) return f(std::integral_constant<int, 1>{});
  return f(std::integral_constant<int, 0>{});
}
template <typename T, int AR>
int occupancy_t(int ring, bool main, int k) {
  if (ring == 4) return main ? occupancy_blocks<T, 4, true, AR>(k) : occupancy_blocks<T, 4, false, AR>(k);
  if constexpr (std::is_same<T, float>::value) {
    if (ring == 8) {
      HEAT2D_REQUIRE(!main && k <= 16, "ring 8: fp32 general kernel, K <= 16");
      return occupancy_blocks<T, 8, false, AR>(k);
    }
  }
  HEAT2D_REQUIRE(ring == 6, "ring must be 4, 6 (8: fp32 general kernel of single launches)");
  return main ? occupancy_blocks<T, 6, true, AR>(k) : occupancy_blocks<T, 6, false, AR>(k);
}

int occupancy_stats(DType dt, int k, int arith) {
  return with_ar(arith, [&](auto ar) {
    constexpr int AR = decltype(ar)::value;
    return dt == DType::F32 ? occupancy_blocks_stats<float, AR>(k) : occupancy_blocks_stats<double, AR>(k);
  });
}

int occupancy(DType dt, int ring, bool main, int k, int arith) {
  return with_ar(arith, [&](auto ar) {
    constexpr int AR = decltype(ar)::value;
    return dt == DType::F32 ? occupancy_t<float, AR>(ring, main, k) : occupancy_t<double, AR>(ring, main, k);
  });
}

template <typename T, int AR>
void dispatch_ar(int ring, bool main, int k, unsigned nblocks, const T* s, T* d, const TbArgs& a, T r,
                 hipStream_t st) {
  if constexpr (std::is_same<T, float>::value) {
    if (ring == 8) {
      HEAT2D_REQUIRE(!main && k <= 16, "ring 8: fp32 general kernel, K <= 16");
      dispatch<T, 8, false, AR>(k, nblocks, s, d, a, r, st);
      return;
    }
  }
  if (ring == 4) {
    if (main) dispatch<T, 4, true, AR>(k, nblocks, s, d, a, r, st);
    else dispatch<T, 4, false, AR>(k, nblocks, s, d, a, r, st);
  } else {
    if (main) dispatch<T, 6, true, AR>(k, nblocks, s, d, a, r, st);
    else dispatch<T, 6, false, AR>(k, nblocks, s, d, a, r, st);
  }
}

template <typename T>
void dispatch_t(int ring, bool main, int arith, int k, unsigned nblocks, const T* s, T* d, const TbArgs& a, T r,
                hipStream_t st) {
  with_ar(arith, [&](auto ar) { dispatch_ar<T, decltype(ar)::value>(ring, main, k, nblocks, s, d, a, r, st); });
}

void check_layout(DType dt, const SlabLayout& L, int k) {
  HEAT2D_REQUIRE(k >= 1 && k <= max_tb(dt), "k must be in [1, max_tb(dtype)] (24)");
  HEAT2D_REQUIRE(k <= L.halo, "temporal depth exceeds the halo depth");
  HEAT2D_REQUIRE(L.cpad >= (k + 1) / 2 * 2 + 4, "column padding too small for the strip halo");
  // the march keeps row indices in 32 bits (scalar compares)
  HEAT2D_REQUIRE(L.nrows_global + 2 * L.halo < (int64_t(1) << 31) && L.row0 < (int64_t(1) << 31),
                 "row count exceeds the 32-bit row index of the stencil kernel");
}

// Row-band count for `rows` x `ns` strips on `simds` balance units: minimise
// (rounds of items per SIMD, the most-loaded SIMD sets the launch time) x
// (band rows + priming rows). Balanced per SIMD, not per resident-wave slot:
// one march wave keeps its SIMD's VALU ~80 % busy, so a second wave on the
// same SIMD adds little throughput (rocprofv3 SQ counters, 4096^2 fp32:
// profiles/small_grid/) — 1197 items on 1024 SIMDs ran 1.5x slower than 1007
// would. fp64 balances over resident wave slots instead: there 2-3 waves per
// SIMD do add throughput (A/B: profiles/band_balance.md). Several rounds when
// the strips alone leave many units idle.
// prime_rows: march rows of overhead per band (2k; the fp32 interior kernel
// skips the levels its priming rows do not need, which costs ~k - 1).
// units the band chooser balances items over: SIMDs for fp32, resident wave slots for fp64
int64_t balance_units(DType dt, int cus, int bpc) {
  const int64_t c = (int64_t)(cus > 0 ? cus : cu_count());
  return dt == DType::F32 ? c * 4 : c * bpc * 4;
}

// HEAT2D_WAVE_TIMES=1 (diagnostics, eager runs only): every tb_kernel launch
// records per-wave start / end times into one device buffer (the last launch
// wins); kern::wave_times copies it out.
struct WaveTimes {
  uint64_t* buf = nullptr;
  int64_t cap = 0, n = 0;
};
WaveTimes& wave_times_state() {
  static WaveTimes w;
  return w;
}
uint64_t* wave_times_buf(int64_t nwaves) {
  static const bool on = [] {
    const char* e = std::getenv("HEAT2D_WAVE_TIMES");
    return e && std::atoi(e) != 0;
  }();
  if (!on) return nullptr;
  WaveTimes& w = wave_times_state();
  if (w.cap < nwaves) {
    if (w.buf) (void)hipFree(w.buf);
    w.cap = std::max<int64_t>(nwaves, 65536);
    if (hipMalloc(reinterpret_cast<void**>(&w.buf), (size_t)w.cap * 4 * sizeof(uint64_t)) != hipSuccess) {
      w.buf = nullptr;
      w.cap = 0;
      return nullptr;
    }
  }
  w.n = nwaves;
  return w.buf;
}

int64_t choose_bands(int64_t rows, int64_t ns, int64_t simds, int k, int64_t prime_rows = -1) {
  const int64_t slots = std::max<int64_t>(simds, 1);
  if (prime_rows < 0) prime_rows = 2 * (int64_t)k;
  const int64_t min_rows = std::max<int64_t>(2 * prime_rows, 16);
  const int64_t nb_max = std::max<int64_t>(1, std::min<int64_t>(rows / min_rows, 64 * slots / std::max<int64_t>(ns, 1) + 1));
  int64_t best = 1;
  double best_cost = 1e300;
  for (int64_t nb = 1; nb <= nb_max; ++nb) {
    const int64_t items = nb * ns;
    const int64_t rounds = (items + slots - 1) / slots;
    const double idle = (double)(rounds * slots) / (double)items;
    const double prime = 1.0 + (double)prime_rows * (double)nb / (double)rows;
    const double cost = idle * prime;
    if (cost < best_cost - 1e-9) {
      best_cost = cost;
      best = nb;
    }
  }
  return best;
}

// Launch `rects` (item counts from their nb and strip ranges) on `nwaves` waves.
// partials != nullptr: the fused-statistics kernel (general, ring 4). Returns the waves launched.
int64_t launch_rects(DType dt, const void* src, void* dst, const SlabLayout& L, int k, int ring, bool main,
                     const TbRect* rects, int nrect, int64_t nwaves, double r, hipStream_t stream, int arith,
                     double* partials = nullptr, uint32_t* queue = nullptr) {
  HEAT2D_REQUIRE(nrect >= 1 && nrect <= (main ? kMainRects : kMaxRects), "bad rect count");
  TbArgs a{};
  a.pitch = L.pitch;
  a.ncols = L.ncols;
  a.col_lo = -L.cpad;
  a.col_hi = L.col_hi();
  a.fixed_lo = -L.row0;
  a.fixed_hi = L.nrows_global - L.row0;
  int64_t items = 0;
  int q = 0;
  for (int i = 0; i < nrect; ++i) {
    const TbRect& R = rects[i];
    if (R.r1 <= R.r0 || R.s1 <= R.s0 || R.nb == 0) continue;
    HEAT2D_REQUIRE(R.r0 >= 0 && R.r1 <= L.nrows, "rect rows outside the slab");
    a.rect[q] = TbRectArg{R.r0, R.r1, R.s0, R.s1, R.nb, items};
    // nb < 0: -nb segments of the strip-major row sequence (tb_range)
    HEAT2D_REQUIRE(R.nb > 0 || -R.nb <= (R.r1 - R.r0) * (R.s1 - R.s0), "more segments than strip rows");
    HEAT2D_REQUIRE((R.r1 - R.r0) * (R.s1 - R.s0) < (int64_t(1) << 31), "rect exceeds 2^31 strip rows");
    items += R.nb > 0 ? R.nb * (R.s1 - R.s0) : -R.nb;
    ++q;
  }
  if (q == 0) return 0;
  a.nrect = q;
  a.pad0 = 0;
  a.nitems = items;
  a.nwaves = std::max<int64_t>(1, std::min<int64_t>(nwaves, items));
  a.partials = partials;
  a.wtimes = wave_times_buf(a.nwaves);
  if (arith == 3) {  // scaled levels (tb_impl.hpp AR 3): coefficients of this depth, in double
    HEAT2D_REQUIRE(r > 0.0, "arith 3 (fast) needs r > 0");
    a.fb = (1.0 - 4.0 * r) / r;
    a.fu = std::pow(r, (double)k);
    a.fu1 = std::pow(r, (double)(k - 1));
  }
  // the dynamic queue only pays with more items than waves (interior and
  // single launches; not the statistics kernel)
  a.queue = (queue && !partials && items > a.nwaves) ? queue : nullptr;
  const unsigned nblocks = (unsigned)((a.nwaves + 3) / 4);
  const int64_t o = L.origin();
  if (partials) {
    HEAT2D_REQUIRE(a.nwaves <= max_stats_waves(), "statistics partials buffer too small");
    const float* s32 = static_cast<const float*>(src) + o;
    const double* s64 = static_cast<const double*>(src) + o;
    with_ar(arith, [&](auto ar) {
      constexpr int AR = decltype(ar)::value;
      if (dt == DType::F32) dispatch_stats<float, AR>(k, nblocks, s32, static_cast<float*>(dst) + o, a, (float)r, stream);
      else dispatch_stats<double, AR>(k, nblocks, s64, static_cast<double*>(dst) + o, a, r, stream);
    });
  } else if (dt == DType::F32) {
    dispatch_t<float>(ring, main, arith, k, nblocks, static_cast<const float*>(src) + o, static_cast<float*>(dst) + o, a,
                      (float)r, stream);
  } else {
    dispatch_t<double>(ring, main, arith, k, nblocks, static_cast<const double*>(src) + o, static_cast<double*>(dst) + o,
                       a, r, stream);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) fail(__FILE__, __LINE__, std::string("tb_kernel launch: ") + hipGetErrorString(e));
  return a.nwaves;
}

}  // namespace

TbPlan plan_tb(DType dt, const SlabLayout& L, int64_t row_begin, int64_t row_end, int k, int64_t tile_rows,
               int cus, int arith) {
  check_layout(dt, L, k);
  HEAT2D_REQUIRE(row_begin >= 0 && row_end <= L.nrows && row_begin < row_end, "bad row range");
  TbPlan p{};
  p.k = k;
  p.skew = 1;
  p.vec = vec_elems(dt);
  p.strip_w = 64 * p.vec;
  p.useful_w = useful_width(dt, k);
  p.nstrips = (L.ncols + p.useful_w - 1) / p.useful_w;
  const int64_t rows = row_end - row_begin;
  p.prefetch = ring_ok(dt, k, default_ring(dt, k));
  p.main = 0;
  const int bpc = occupancy(dt, p.prefetch, false, k, arith);
  p.blocks_per_cu = bpc;
  const int64_t slots = (int64_t)(cus > 0 ? cus : cu_count()) * bpc * 4;  // resident waves
  if (tile_rows < 0) {  // -tile_rows segments of the strip-major row sequence (TbRect nb < 0)
    const int64_t nseg = std::min<int64_t>(-tile_rows, rows * p.nstrips);
    p.ntiles = -nseg;
    p.nwaves = std::min<int64_t>(nseg, std::max<int64_t>(slots, 1));
    p.tile_rows = (rows * p.nstrips + nseg - 1) / nseg;
    p.nblocks = (p.nwaves + 3) / 4;
    return p;
  }
  int64_t nbands;
  if (tile_rows > 0) {
    nbands = (rows + tile_rows - 1) / tile_rows;
  } else {
    nbands = choose_bands(rows, p.nstrips, balance_units(dt, cus, bpc), k);
  }
  nbands = std::max<int64_t>(1, std::min<int64_t>(nbands, rows));
  const int64_t items = nbands * p.nstrips;
  p.ntiles = nbands;
  p.nwaves = std::min<int64_t>(items, std::max<int64_t>(slots, 1));
  p.tile_rows = (rows + nbands - 1) / nbands;
  p.nblocks = (p.nwaves + 3) / 4;
  return p;
}

void launch_tb(DType dt, const void* src, void* dst, const SlabLayout& L, int64_t row_begin, int64_t row_end, int k,
               double r, hipStream_t stream, int64_t tile_rows, int cus, int arith) {
  launch_tb2(dt, src, dst, L, row_begin, row_end, 0, 0, k, r, stream, tile_rows, cus, arith);
}

void launch_tb2(DType dt, const void* src, void* dst, const SlabLayout& L, int64_t rb0, int64_t re0, int64_t rb1,
                int64_t re1, int k, double r, hipStream_t stream, int64_t tile_rows, int cus, int arith) {
  check_layout(dt, L, k);
  const int64_t n0 = std::max<int64_t>(0, re0 - rb0), n1 = std::max<int64_t>(0, re1 - rb1);
  if (n0 + n1 == 0) return;
  // plan over the concatenated rows, then give each range its share of bands
  const TbPlan p = plan_tb(dt, L, 0, std::min<int64_t>(n0 + n1, L.nrows), k, tile_rows, cus, arith);
  TbRect rects[2];
  int nr = 0;
  if (p.ntiles < 0) {  // segments, shared out over the two ranges by rows
    const int64_t ns = -p.ntiles;
    const int64_t s0 = n1 == 0 ? ns : (n0 == 0 ? 0 : std::max<int64_t>(1, (ns * n0 + (n0 + n1) / 2) / (n0 + n1)));
    if (n0 > 0) rects[nr++] = TbRect{rb0, re0, 0, p.nstrips, -std::min<int64_t>(s0, n0 * p.nstrips)};
    if (n1 > 0) rects[nr++] = TbRect{rb1, re1, 0, p.nstrips, -std::min<int64_t>(std::max<int64_t>(1, ns - s0), n1 * p.nstrips)};
    launch_rects(dt, src, dst, L, k, p.prefetch, false, rects, nr, p.nwaves, r, stream, arith);
    return;
  }
  const int64_t nb = std::max<int64_t>(p.ntiles, (n0 > 0) + (n1 > 0));
  const int64_t nb0 = n1 == 0 ? nb : (n0 == 0 ? 0 : std::min<int64_t>(nb - 1, std::max<int64_t>(1, (nb * n0 + (n0 + n1) / 2) / (n0 + n1))));
  if (n0 > 0) rects[nr++] = TbRect{rb0, re0, 0, p.nstrips, std::min<int64_t>(nb0, n0)};
  if (n1 > 0) rects[nr++] = TbRect{rb1, re1, 0, p.nstrips, std::min<int64_t>(nb - nb0, n1)};
  const int64_t slots = (int64_t)(cus > 0 ? cus : cu_count()) * p.blocks_per_cu * 4;
  launch_rects(dt, src, dst, L, k, p.prefetch, false, rects, nr, slots, r, stream, arith);
}

// r = 1/4 kernels (arith 2): an interior item costs 3 adds + 2 DPP moves per
// point and level (fp32: 8 VALU ops per 4 points, fp64: 10 per 2), a
// frame-column strip's item (edge kinds 2 / 3: the unscaled 3-op update) w =
// 1.75x (fp32: 14) / 1.6x (fp64: 16) that. Launched as equals, the two
// frame-column strips' items end last — with one item per wave the launch
// lasts as long as its slowest wave (4096^2 fp32 K = 15: 69 us per cycle
// against 66 for arith 1, whose kinds all cost ~12). Weighted: the first and
// last strip get rects of their own whose items cost what an interior one
// does, priming rows (2k per item) included: (Le + 2k) w = Li + 2k. A plan
// whose segments tile every strip exactly keeps doing so (a segment crossing
// a strip end pays a second priming), with as many interior segments per
// strip as fit the original item count. plan.rects[] / plan.nrects hold the
// rects; plan.main keeps the unweighted rect that describes the plan.
//
// Frame ROWS likewise: an item whose march reaches the global top / bottom row
// (edge kind 1: the unscaled 2-op form, fp32 12 VALU ops per 4 points against
// 8, fp64 14 per 2 against 10) runs ~1.4-1.5x an interior item per march row.
// In a single-launch plan (plan_single: the small grid's, where every wave
// holds one item and the launch lasts as long as its slowest wave) those are
// the first and last item of every strip. When the rect's marches reach a
// frame row, the interior strips get a top / bottom rect of one short band
// each, (h + 2k) w1 = Li + 2k, and the segments / bands in between: 5 rects.
double pinned_weight(DType dt, bool row, bool single, int ring) {
  // Measured: fp32 columns 1.4 best over 1.0-2.3 (4096^2 K = 16, 1007
  // segments: 58.7-59.1 us per cycle against 60.1 at 1.5 and 60.7 at 1.75,
  // profiles/r3/sweep5/); rows from per-wave timelines (tools/wave_times.py,
  // profiles/r3/wt2/): fp32 1.3 puts the frame-row items at 45.8 us against
  // 46.9 for the interior ones (1.5: 40.5); fp64 4096^2 K = 12 at 1.4 / 1.6
  // left the frame rows at 68 and the frame columns at 61 us against 75. A
  // wave alone on its SIMD hides part of the pinned kinds' extra ops in its own
  // stalls; in the 2-waves/SIMD interior launch of a split plan they cost their
  // full VALU ratio: fp64 columns 1.6 there (32768^2 K = 20: 4310-4332 Gpts/s
  // against 4071-4153 at 1.3, same box, profiles/r3/abwcol/)
  // The fp32 ring-8 general kernel (294 VGPRs at K = 16) runs interior items
  // 8 % faster than ring 6 but its pinned kinds not (ring8/: 43.7 us interior,
  // 53.5 frame rows, 47.5 frame columns at 1.3 / 1.4): 1.6 / 1.55 there
  if (dt == DType::F32 && ring == 8) return row ? 1.6 : 1.55;
  if (row) return 1.3;
  if (dt == DType::F32) return 1.4;
  return single ? 1.3 : 1.6;
}

int weighted_main(DType dt, int k, const TbRect& R, const SlabLayout& L, TbRect out[kMaxPlanRects], bool single,
                  int ring) {
  const int64_t ns = R.s1 - R.s0, rows = R.r1 - R.r0;
  if (ns < 3 || rows < 2) return 0;
  const double w = pinned_weight(dt, false, single, ring), w1 = pinned_weight(dt, true, single, ring), prime = 2.0 * k;
  auto edge_items = [&](double li) {  // items of one frame strip for interior items of li rows
    const double le = std::max(8.0, (li + prime) / w - prime);
    return std::min<int64_t>(rows, (int64_t)std::ceil((double)rows / le));
  };
  // frame rows within the marches of the rect's first / last rows (the
  // kernel's edge-kind test: t0 - k < fixed_lo, t1 + k > fixed_hi)
  const bool ftop = L.row0 + R.r0 < k, fbot = L.row0 + R.r1 + k > L.nrows_global;
  // rows of the top / bottom band for interior items of li rows: as costly as
  // one of those, and at least k (so the next item is kind 0)
  auto frame_rows = [&](double li) {
    return std::max<int64_t>(k, (int64_t)std::floor((li + prime) / w1 - prime));
  };
  int64_t hT = 0, hB = 0;  // rows carved out at the top / bottom of the interior strips
  int64_t ne, ni;
  if (R.nb < 0) {
    const int64_t S = -R.nb;
    if (S % ns == 0) {  // strip-aligned segments: q per interior strip, as many as fit S items
      const int nf = (ftop ? 1 : 0) + (fbot ? 1 : 0);
      auto fit = [&](int64_t q, int64_t* qe, int64_t* ht, int64_t* hb) {
        // frame bands of the interior strips, sized for the segments between them
        *ht = *hb = 0;
        if (nf > 0) {
          const int64_t h = frame_rows((double)rows / (q + nf));
          if (rows - nf * h >= std::max<int64_t>(q * 2 * (int64_t)k, 1)) {
            const int64_t h2 = frame_rows((double)(rows - nf * h) / q);
            *ht = ftop ? h2 : 0;
            *hb = fbot ? h2 : 0;
            if (rows - *ht - *hb < std::max<int64_t>(q * 2 * (int64_t)k, 1)) *ht = *hb = 0;
          }
        }
        *qe = edge_items((double)(rows - *ht - *hb) / q);
        return (ns - 2) * (q + (*ht > 0) + (*hb > 0)) + 2 * *qe;
      };
      int64_t q = S / ns, qe = 0;
      while (q > 1 && fit(q, &qe, &hT, &hB) > S) --q;
      fit(q, &qe, &hT, &hB);
      ni = (ns - 2) * q;
      ne = qe;
    } else {  // segments already cross strip ends: carve the frame strips out
      ne = edge_items((double)rows * (double)ns / (double)S);
      ni = std::max<int64_t>(1, S - 2 * ne);
    }
    ni = -std::min<int64_t>(ni, (rows - hT - hB) * (ns - 2));
    ne = -ne;
  } else {  // bands: more (shorter) bands on the frame strips, one short band per frame side
    ni = R.nb;
    const double li = (double)rows / R.nb;
    if (R.nb >= 2) {
      const int64_t h = frame_rows(li);
      if (rows - (ftop + fbot) * h >= R.nb * 2 * (int64_t)k) {
        hT = ftop ? h : 0;
        hB = fbot ? h : 0;
      }
    }
    ne = std::max<int64_t>(R.nb, edge_items(li));
  }
  int n = 0;
  out[n++] = TbRect{R.r0, R.r1, R.s0, R.s0 + 1, ne};
  if (hT > 0) out[n++] = TbRect{R.r0, R.r0 + hT, R.s0 + 1, R.s1 - 1, 1};
  out[n++] = TbRect{R.r0 + hT, R.r1 - hB, R.s0 + 1, R.s1 - 1, ni};
  if (hB > 0) out[n++] = TbRect{R.r1 - hB, R.r1, R.s0 + 1, R.s1 - 1, 1};
  out[n++] = TbRect{R.r0, R.r1, R.s1 - 1, R.s1, ne};
  return n;
}

int64_t rect_items(const TbRect& R) { return R.nb > 0 ? R.nb * (R.s1 - R.s0) : -R.nb; }

// arith 2: put the weighted rects of p.main into p.rects (see weighted_main)
void weight_main(DType dt, const SlabLayout& L, SplitPlan& p, int arith, int64_t slots, bool single) {
  if (arith != 2) return;
  const int n = weighted_main(dt, p.k, p.main, L, p.rects, single, p.ring);
  if (n == 0) return;
  p.nrects = n;
  p.main_items = 0;
  for (int i = 0; i < n; ++i) p.main_items += rect_items(p.rects[i]);
  p.main_waves = std::min<int64_t>(p.main_items, slots);
}

SplitPlan plan_split(DType dt, const SlabLayout& L, int k, int64_t band, int cus, int spare_waves,
                     int ring_override, int64_t main_bands, int arith) {
  check_layout(dt, L, k);
  SplitPlan p{};
  p.k = k;
  p.ring = ring_ok(dt, k, (ring_override == 4 || ring_override == 6) ? ring_override : default_ring(dt, k));
  const int64_t n = L.nrows, B = std::max<int64_t>(band, k);
  const int64_t U = useful_width(dt, k);
  const int64_t ns = (L.ncols + U - 1) / U;
  const int64_t rows_m = n - 2 * B;
  if (rows_m < 4 * k) return p;  // valid = 0: too thin to split
  // MAIN: the interior rows, all strips, persistent (one item per resident wave)
  const int bpc = occupancy(dt, p.ring, true, k, arith);
  const int64_t slots = (int64_t)(cus > 0 ? cus : cu_count()) * bpc * 4;
  const int64_t mw = std::max<int64_t>(4, slots - std::max(0, spare_waves));
  // the fp32 interior kernel skips unneeded priming levels (tb_impl.hpp run<PS>)
  int64_t nb_m = choose_bands(rows_m, ns, dt == DType::F32 ? balance_units(dt, cus, bpc) : mw, k,
                              dt == DType::F32 ? std::max(1, k - 1) : -1);
  if (main_bands > 0) nb_m = std::min<int64_t>(main_bands, std::max<int64_t>(1, rows_m / (2 * (int64_t)k)));
  if (main_bands < 0) nb_m = -std::min<int64_t>(-main_bands, std::max<int64_t>(1, rows_m * ns / (2 * (int64_t)k)));
  p.main = TbRect{B, n - B, 0, ns, nb_m};
  p.main_items = nb_m > 0 ? nb_m * ns : -nb_m;
  p.main_waves = std::min<int64_t>(p.main_items, mw);  // > one item per wave if main_bands asks for it
  weight_main(dt, L, p, arith, mw, false);
  // EDGE: the two boundary bands (one band each), general kernel. Short
  // (B + 2k march rows per item): beside MAIN where wave slots allow, else
  // right after it — either way the halo exchange that follows overlaps the
  // NEXT cycle's MAIN, which does not wait for it.
  p.edge[0] = TbRect{0, B, 0, ns, 1};
  p.edge[1] = TbRect{n - B, n, 0, ns, 1};
  p.nedge = 2;
  p.edge_items = 2 * ns;
  const int bpc_e = occupancy(dt, p.ring, false, k, arith);
  p.edge_waves = std::min<int64_t>(p.edge_items, (int64_t)cu_count() * bpc_e * 4);
  p.valid = 1;
  return p;
}

SplitPlan with_edge_bands(DType dt, const SplitPlan& p, int64_t nb, int arith) {
  SplitPlan q = p;
  if (!(p.valid == 1 || p.valid == 3) || nb < 1) return q;
  q.edge_items = 0;
  for (int i = 0; i < q.nedge; ++i) {
    TbRect& e = q.edge[i];
    e.nb = std::max<int64_t>(1, std::min<int64_t>(nb, e.r1 - e.r0));
    q.edge_items += e.nb * (e.s1 - e.s0);
  }
  const int bpc_e = occupancy(dt, q.ring, false, q.k, arith);
  q.edge_waves = std::min<int64_t>(q.edge_items, (int64_t)cu_count() * bpc_e * 4);
  return q;
}

SplitPlan plan_single(DType dt, const SlabLayout& L, int k, int cus, int ring_override, int64_t bands, int arith) {
  check_layout(dt, L, k);
  SplitPlan p{};
  p.k = k;
  p.ring = ring_ok(dt, k, ring_valid(ring_override) ? ring_override : default_ring(dt, k), true);
  const int64_t U = useful_width(dt, k);
  const int64_t ns = (L.ncols + U - 1) / U;
  const int bpc = occupancy(dt, p.ring, false, k, arith);
  const int64_t slots = (int64_t)(cus > 0 ? cus : cu_count()) * bpc * 4;
  int64_t nb = choose_bands(L.nrows, ns, balance_units(dt, cus, bpc), k);
  if (bands > 0) nb = std::min<int64_t>(bands, std::max<int64_t>(1, L.nrows / (2 * (int64_t)k)));
  if (bands < 0) nb = -std::min<int64_t>(-bands, std::max<int64_t>(1, L.nrows * ns / (2 * (int64_t)k)));
  p.main = TbRect{0, L.nrows, 0, ns, nb};
  p.main_items = nb > 0 ? nb * ns : -nb;
  p.main_waves = std::min<int64_t>(p.main_items, slots);
  weight_main(dt, L, p, arith, slots, true);
  p.nedge = 0;
  p.valid = 2;
  return p;
}

int64_t wave_times(uint64_t* out, int64_t max_waves) {
  WaveTimes& w = wave_times_state();
  if (!w.buf || w.n == 0) return 0;
  HEAT2D_REQUIRE(hipDeviceSynchronize() == hipSuccess, "wave_times: device synchronisation failed");
  const int64_t n = std::min(w.n, max_waves);
  HEAT2D_REQUIRE(hipMemcpy(out, w.buf, (size_t)n * 4 * sizeof(uint64_t), hipMemcpyDeviceToHost) == hipSuccess,
                 "wave_times: copy failed");
  return n;
}

int64_t max_stats_waves() { return (int64_t)cu_count() * 32; }  // 8 x 256-thread blocks per CU

void launch_tb_stats(DType dt, const void* src, void* dst, const SlabLayout& L, int k, double r, double* partials,
                     double* out6, hipStream_t stream, int arith) {
  check_layout(dt, L, k);
  HEAT2D_REQUIRE(partials && out6, "statistics buffers required");
  const int64_t U = useful_width(dt, k);
  const int64_t ns = (L.ncols + U - 1) / U;
  const int64_t slots = (int64_t)cu_count() * occupancy_stats(dt, k, arith) * 4;
  const int64_t nb = std::max<int64_t>(
      1, std::min<int64_t>(choose_bands(L.nrows, ns, balance_units(dt, 0, occupancy_stats(dt, k, arith)), k), L.nrows));
  const TbRect rect{0, L.nrows, 0, ns, nb};
  const int64_t nw = launch_rects(dt, src, dst, L, k, 4, false, &rect, 1, slots, r, stream, arith, partials);
  launch_reduce_partials(partials, nw, out6, stream);
}

// Boundary-band rects of a slab whose bands stay clear of the global frame
// rows (every middle rank of a row decomposition): the interior kernel marches
// them (item kinds 0 / 2 only), at its 2 waves per SIMD instead of the general
// kernel's 1 (fp64 K = 20: 249 vs 374 + 118 acc VGPRs; fp32 480-step slab
// rehearsal 8838 -> 9233 Gpts/s, profiles/r4/lead/).
bool edges_on_main(const SlabLayout& L, int k, const TbRect* R, int n) {
  if (n < 1 || n > kMainRects) return false;
  for (int i = 0; i < n; ++i)
    if (R[i].r1 > R[i].r0 && (R[i].r0 - k < -L.row0 || R[i].r1 + k > L.nrows_global - L.row0)) return false;
  return true;
}

bool edges_on_main(const SlabLayout& L, const SplitPlan& p) {
  return (p.valid == 1 || p.valid == 3) && edges_on_main(L, p.k, p.edge, p.nedge);
}

bool edge_rect_on_main(const SlabLayout& L, const SplitPlan& p, int i) {
  return i >= 0 && i < p.nedge && edges_on_main(L, p.k, &p.edge[i], 1);
}

void launch_edge_rect(DType dt, const void* src, void* dst, const SlabLayout& L, const SplitPlan& p, int i, double r,
                      hipStream_t stream, int arith) {
  HEAT2D_REQUIRE(i >= 0 && i < p.nedge, "edge rect index");
  const TbRect& R = p.edge[i];
  const bool on_main = edges_on_main(L, p.k, &R, 1);
  const int64_t items = R.nb > 0 ? R.nb * (R.s1 - R.s0) : -R.nb;
  const int64_t slots = (int64_t)cu_count() * occupancy(dt, p.ring, on_main, p.k, arith) * 4;
  launch_rects(dt, src, dst, L, p.k, p.ring, on_main, &R, 1, std::min<int64_t>(items, slots), r, stream, arith);
}

void launch_split(DType dt, const void* src, void* dst, const SlabLayout& L, const SplitPlan& p, bool main_part,
                  double r, hipStream_t stream, int arith, uint32_t* queue) {
  // (SplitPlan::flags & kPlanDynamic: the main part takes its items from the dynamic queue)
  uint32_t* q = (p.flags & kPlanDynamic) ? queue : nullptr;
  HEAT2D_REQUIRE(p.valid, "invalid split plan");
  // the main part: p.main, or its frame-strip-weighted rects (weight_main)
  const TbRect* mr = p.nrects > 0 ? p.rects : &p.main;
  const int nm = p.nrects > 0 ? p.nrects : 1;
  if (p.valid == 2) {  // single general launch over the whole slab (no edge part)
    if (main_part)
      launch_rects(dt, src, dst, L, p.k, p.ring, false, mr, nm, p.main_waves, r, stream, arith, nullptr, q);
    return;
  }
  if (main_part)
    launch_rects(dt, src, dst, L, p.k, p.ring, true, mr, nm, p.main_waves, r, stream, arith, nullptr, q);
  else
    launch_rects(dt, src, dst, L, p.k, p.ring, edges_on_main(L, p.k, p.edge, p.nedge), p.edge, p.nedge, p.edge_waves,
                 r, stream, arith);
}

}  // namespace kern
}  // namespace heat2d
