// Temporal-blocked 5-point FTCS stencil for gfx950 (CDNA4): host-side
// planning and launch. Device code: tb_impl.hpp; instantiations: tb_*.hip.
//
// Replaces reference K1 `heat_eqn` (fortran/hip/heat_kernel.cpp:31-45: one
// thread per point, 5 scalar loads, 128x4 blocks) and K12, the per-step
// full-field D2D copy (fortran/hip/heat.F90:243).
//
// Design (wave64, no LDS, no barriers):
//   * one WAVE owns a column strip of 64*V columns (V = NV * 16 B / sizeof(T))
//     and marches down a run of rows, loading each input row exactly once with
//     NV 16-B loads per lane (1 KiB per wave instruction);
//   * K time levels are pipelined in registers: at march row m the wave loads
//     row m of level 0 and computes row m-s of level s for s = 1..K, so K time
//     steps cost ONE HBM read + ONE HBM write per point (the single-step
//     roofline is 16 B/pt fp64; at K = 8 the kernel needs 2 B/pt);
//   * east/west neighbours come from the adjacent lane through DPP
//     wave_shr:1 / wave_shl:1 (VALU modifiers, no LDS traffic); the strip's
//     outer K columns are redundant halo work (shrinking valid region);
//   * the 3-row window per level rotates through a 3-phase unrolled loop, so no
//     register moves are needed for the rotation;
//   * loads/stores are raw buffer ops on per-row descriptors with out-of-range
//     voffsets for masked lanes: no memory op under control flow, so the
//     prefetch ring (3 rows ahead) is waited for with counted vmcnt(N);
//   * persistent, balanced schedule: exactly as many waves as the chip holds
//     resident (occupancy API x CUs); wave w owns the contiguous row-units
//     [w*R/S, (w+1)*R/S) of the strip-major list of R = strips x rows, so all
//     waves finish together (no partial last round) and every march is long
//     (the 2K-row start-up of a march is amortised);
//   * the arithmetic order is exactly the reference's
//     c + r*((((E + N) + W) + S) - 4c) (fortran/hip/heat_kernel.cpp:43) and the
//     file is built with -ffp-contract=off: results are bitwise identical to the
//     CPU reference and to an unblocked K=1 run.
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

template <typename T, int NV>
int useful_width(int k) {
  constexpr int V = NV * Vec16<T>::n;
  const int ka = (k + V - 1) / V * V;  // must match TbShape::KA
  return 64 * V - 2 * ka;
}


// Vector width (16-B vectors per lane). 2 halves the strip-halo redundancy
// but doubles the register state; instantiated for K <= 8 only.
// Override: HEAT2D_TB_NV=1|2.
int default_nv(DType dt, int k) {
  const char* env = std::getenv("HEAT2D_TB_NV");  // read per plan: tunable at run time
  (void)dt;
  if (env) return (std::atoi(env) == 2 && k <= 8) ? 2 : 1;
  // measured on MI355X (bench/sweep.py, 32768^2): 32 B/lane wins for fp64 while
  // the kernel is still bandwidth-bound (k <= 6); beyond that the register
  // state costs more occupancy than the halved halo redundancy returns
  return (dt == DType::F64 && k <= 6) ? 2 : 1;
}

// Level pipeline skew (1: levels chained within a row iteration; 2: levels
// independent, more ILP, +1 row of state per level). Override: HEAT2D_TB_SKEW.
int default_skew(DType dt, int k) {
  const char* env = std::getenv("HEAT2D_TB_SKEW");
  (void)dt;
  (void)k;
  if (env) return std::atoi(env) == 2 ? 2 : 1;
  return 1;  // skew-2's extra row of state per level costs more occupancy than its ILP returns (measured)
}

// Prefetch depth (units of 3 rows). 6 rows in flight hides the HBM latency
// of the compute-heavier deep pipelines; instantiated for 16 B/lane, skew 1.
// Override: HEAT2D_TB_PF=1|2.
int default_pf(DType dt, int k, int nv, int sk) {
  if (nv != 1 || sk != 1) return 1;
  const char* env = std::getenv("HEAT2D_TB_PF");
  if (env) return std::atoi(env) == 2 ? 2 : 1;
  return (dt == DType::F64 ? k >= 7 : k >= 9) ? 2 : 1;  // measured (bench/sweep.py, A/B in one box)
}

template <typename T>
int occupancy(int nv, int sk, int pf, int k) {
  if (nv == 1) {
    if (sk == 2) return occupancy_blocks<T, 1, 2, 1>(k);
    return pf == 2 ? occupancy_blocks<T, 1, 1, 2>(k) : occupancy_blocks<T, 1, 1, 1>(k);
  }
  return sk == 2 ? occupancy_blocks<T, 2, 2, 1>(k) : occupancy_blocks<T, 2, 1, 1>(k);
}

template <typename T>
void dispatch_variant(int nv, int sk, int pf, int k, unsigned nblocks, const T* s, T* d, const TbArgs& a, T r,
                      hipStream_t st) {
  if (nv == 1) {
    if (sk == 2) dispatch<T, 1, 2, 1>(k, nblocks, s, d, a, r, st);
    else if (pf == 2) dispatch<T, 1, 1, 2>(k, nblocks, s, d, a, r, st);
    else dispatch<T, 1, 1, 1>(k, nblocks, s, d, a, r, st);
  } else {
    if (sk == 2) dispatch<T, 2, 2, 1>(k, nblocks, s, d, a, r, st);
    else dispatch<T, 2, 1, 1>(k, nblocks, s, d, a, r, st);
  }
}

}  // namespace

TbPlan plan_tb(DType dt, const SlabLayout& L, int64_t row_begin, int64_t row_end, int k, int64_t tile_rows,
               int cus) {
  HEAT2D_REQUIRE(k >= 1 && k <= kMaxTB, "k must be in [1, kMaxTB]");
  HEAT2D_REQUIRE(row_begin >= 0 && row_end <= L.nrows && row_begin < row_end, "bad row range");
  TbPlan p{};
  p.k = k;
  const int nv = default_nv(dt, k);
  p.skew = default_skew(dt, k);
  const int vm = dt == DType::F32 ? 4 : 2;
  p.vec = nv * vm;
  p.strip_w = 64 * p.vec;
  if (dt == DType::F32)
    p.useful_w = nv == 1 ? useful_width<float, 1>(k) : useful_width<float, 2>(k);
  else
    p.useful_w = nv == 1 ? useful_width<double, 1>(k) : useful_width<double, 2>(k);
  p.nstrips = (L.ncols + p.useful_w - 1) / p.useful_w;
  const int64_t rows = row_end - row_begin;
  p.prefetch = 3 * default_pf(dt, k, nv, p.skew);
  const int pf = p.prefetch / 3;
  const int bpc = dt == DType::F32 ? occupancy<float>(nv, p.skew, pf, k) : occupancy<double>(nv, p.skew, pf, k);
  p.blocks_per_cu = bpc;
  const int64_t slots = (int64_t)(cus > 0 ? cus : cu_count()) * bpc * 4;  // resident waves
  int64_t nbands;
  if (tile_rows > 0) {
    nbands = (rows + tile_rows - 1) / tile_rows;
  } else {
    // persistent: one (band, strip) item per resident wave, bands >= ~4k rows
    const int64_t min_rows = std::max<int64_t>(4 * (int64_t)k, 16);
    nbands = std::max<int64_t>(1, slots / p.nstrips);
    nbands = std::min<int64_t>(nbands, std::max<int64_t>(1, rows / min_rows));
  }
  nbands = std::max<int64_t>(1, std::min<int64_t>(nbands, rows));
  const int64_t items = nbands * p.nstrips;
  const int64_t nwaves = std::min<int64_t>(items, std::max<int64_t>(slots, 1));
  p.ntiles = nbands;
  p.nwaves = nwaves;
  p.tile_rows = (rows + nbands - 1) / nbands;
  p.nblocks = (nwaves + 3) / 4;
  return p;
}

void launch_tb(DType dt, const void* src, void* dst, const SlabLayout& L, int64_t row_begin, int64_t row_end, int k,
               double r, hipStream_t stream, int64_t tile_rows, int cus) {
  HEAT2D_REQUIRE(k <= L.halo, "temporal depth exceeds the halo depth");
  HEAT2D_REQUIRE(L.cpad >= 16, "column padding too small for the strip halo");
  if (row_end <= row_begin) return;
  const TbPlan p = plan_tb(dt, L, row_begin, row_end, k, tile_rows, cus);
  TbArgs a{};
  a.pitch = L.pitch;
  a.ncols = L.ncols;
  a.col_lo = -L.cpad;
  a.col_hi = L.col_hi();
  a.row_begin = row_begin;
  a.row_end = row_end;
  a.nstrips = p.nstrips;
  a.nbands = p.ntiles;
  a.nwaves = p.nwaves;
  a.fixed_lo = -L.row0;
  a.fixed_hi = L.nrows_global - L.row0;
  const int64_t o = L.origin();
  const int nv = p.vec / (dt == DType::F32 ? 4 : 2);
  if (dt == DType::F32) {
    const float* s = static_cast<const float*>(src) + o;
    float* d = static_cast<float*>(dst) + o;
    dispatch_variant<float>(nv, p.skew, p.prefetch / 3, p.k, (unsigned)p.nblocks, s, d, a, (float)r, stream);
  } else {
    const double* s = static_cast<const double*>(src) + o;
    double* d = static_cast<double*>(dst) + o;
    dispatch_variant<double>(nv, p.skew, p.prefetch / 3, p.k, (unsigned)p.nblocks, s, d, a, r, stream);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) fail(__FILE__, __LINE__, std::string("tb_kernel launch: ") + hipGetErrorString(e));
}

}  // namespace kern
}  // namespace heat2d
