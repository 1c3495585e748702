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
//   * persistent schedule: as many waves as the chip holds resident
//     (occupancy API x CUs), work items = (row band, strip), band-major;
//   * the arithmetic order is exactly the reference's
//     c + r*((((S + E) + N) + W) - 4c) (fortran/hip/heat_kernel.cpp:43, with
//     S = T(x+1,y), E = T(x,y+1), N = T(x-1,y), W = T(x,y-1)) and the file is
//     built with -ffp-contract=off: results are bitwise identical to the CPU
//     reference and to an unblocked K=1 run, in fp64 and in fp32.
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
// (and the DPP moves per point) but doubles the register state.
// Override: HEAT2D_TB_NV=1|2 (read per plan: tunable at run time).
int default_nv(DType dt, int k) {
  if (const char* env = std::getenv("HEAT2D_TB_NV")) return std::atoi(env) == 2 ? 2 : 1;
  (void)dt;
  (void)k;
  return 1;
}

// Level-0 row ring per wave (RING - 2 rows in flight; the march loop is
// unrolled RING times). Override: HEAT2D_TB_RING=4|6|8 (8 only for 16 B/lane).
int default_ring(DType dt, int k, int nv) {
  if (const char* env = std::getenv("HEAT2D_TB_RING")) {
    const int r = std::atoi(env);
    if (r == 4 || r == 6 || (r == 8 && nv == 1)) return r;
  }
  // measured on MI355X (bench/sweep.py, 32768^2, profiles/sweep_ring_tight_32768.txt)
  if (dt == DType::F64) return k <= 10 ? 6 : 4;
  return k <= 9 ? 4 : 6;
}

// Register budget: tight (occupancy target tight_waves()) or the compiler's
// own. Override: HEAT2D_TB_TIGHT=0|1.
bool default_tight(DType dt, int k, int nv, int ring) {
  if (const char* env = std::getenv("HEAT2D_TB_TIGHT")) return std::atoi(env) != 0;
  (void)dt;
  (void)k;
  (void)nv;
  (void)ring;
  return true;
}

template <typename T>
int occupancy(int nv, int ring, int k, bool tight) {
  if (nv == 2) return ring == 4 ? occupancy_blocks<T, 2, 4>(k, tight) : occupancy_blocks<T, 2, 6>(k, tight);
  return ring == 4   ? occupancy_blocks<T, 1, 4>(k, tight)
         : ring == 6 ? occupancy_blocks<T, 1, 6>(k, tight)
                     : occupancy_blocks<T, 1, 8>(k, tight);
}

template <typename T>
void dispatch_variant(int nv, int ring, bool tight, int k, unsigned nblocks, const T* s, T* d, const TbArgs& a,
                      T r, hipStream_t st) {
  if (nv == 2) {
    if (ring == 4) dispatch<T, 2, 4>(k, tight, nblocks, s, d, a, r, st);
    else dispatch<T, 2, 6>(k, tight, nblocks, s, d, a, r, st);
  } else {
    if (ring == 4) dispatch<T, 1, 4>(k, tight, nblocks, s, d, a, r, st);
    else if (ring == 6) dispatch<T, 1, 6>(k, tight, nblocks, s, d, a, r, st);
    else dispatch<T, 1, 8>(k, tight, nblocks, s, d, a, r, st);
  }
}

}  // namespace

TbPlan plan_tb(DType dt, const SlabLayout& L, int64_t row_begin, int64_t row_end, int k, int64_t tile_rows,
               int cus) {
  HEAT2D_REQUIRE(k >= 1 && k <= kMaxTB, "k must be in [1, kMaxTB]");
  HEAT2D_REQUIRE(row_begin >= 0 && row_end <= L.nrows && row_begin < row_end, "bad row range");
  HEAT2D_REQUIRE(L.cpad >= 16, "column padding too small for the strip halo");
  TbPlan p{};
  p.k = k;
  const int nv = default_nv(dt, k);
  p.skew = 1;
  const int vm = dt == DType::F32 ? 4 : 2;
  p.vec = nv * vm;
  p.strip_w = 64 * p.vec;
  if (dt == DType::F32)
    p.useful_w = nv == 1 ? useful_width<float, 1>(k) : useful_width<float, 2>(k);
  else
    p.useful_w = nv == 1 ? useful_width<double, 1>(k) : useful_width<double, 2>(k);
  p.nstrips = (L.ncols + p.useful_w - 1) / p.useful_w;
  const int64_t rows = row_end - row_begin;
  p.prefetch = default_ring(dt, k, nv);
  p.tight = default_tight(dt, k, nv, p.prefetch) ? 1 : 0;
  const int bpc = dt == DType::F32 ? occupancy<float>(nv, p.prefetch, k, p.tight)
                                   : occupancy<double>(nv, p.prefetch, k, p.tight);
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
  launch_tb2(dt, src, dst, L, row_begin, row_end, 0, 0, k, r, stream, tile_rows, cus);
}

void launch_tb2(DType dt, const void* src, void* dst, const SlabLayout& L, int64_t rb0, int64_t re0, int64_t rb1,
                int64_t re1, int k, double r, hipStream_t stream, int64_t tile_rows, int cus) {
  HEAT2D_REQUIRE(k <= L.halo, "temporal depth exceeds the halo depth");
  HEAT2D_REQUIRE(L.cpad >= 16, "column padding too small for the strip halo");
  // the march keeps row indices in 32 bits (scalar compares)
  HEAT2D_REQUIRE(L.nrows_global + 2 * L.halo < (int64_t(1) << 31) && L.row0 < (int64_t(1) << 31),
                 "row count exceeds the 32-bit row index of the stencil kernel");
  if (re0 <= rb0) {  // range 1 only
    rb0 = rb1;
    re0 = re1;
    rb1 = re1 = 0;
  }
  if (re0 <= rb0) return;
  const int64_t n0 = re0 - rb0, n1 = re1 > rb1 ? re1 - rb1 : 0;
  HEAT2D_REQUIRE(n1 == 0 || rb1 >= 0 && re1 <= L.nrows, "bad second row range");
  // plan over the concatenated rows, then give each range its share of bands
  TbPlan p = plan_tb(dt, L, 0, n0 + n1, k, tile_rows, cus);
  int64_t nb0 = p.ntiles;
  if (n1 > 0) {
    const int64_t nb = std::max<int64_t>(p.ntiles, 2);
    nb0 = std::min<int64_t>(nb - 1, std::max<int64_t>(1, (nb * n0 + (n0 + n1) / 2) / (n0 + n1)));
    const int64_t slots = (int64_t)(cus > 0 ? cus : cu_count()) * p.blocks_per_cu * 4;
    p.ntiles = nb;
    p.nwaves = std::max<int64_t>(1, std::min<int64_t>(nb * p.nstrips, slots));
    p.nblocks = (p.nwaves + 3) / 4;
  }
  TbArgs a{};
  a.pitch = L.pitch;
  a.ncols = L.ncols;
  a.col_lo = -L.cpad;
  a.col_hi = L.col_hi();
  a.row_begin = rb0;
  a.row_end = re0;
  a.row_begin1 = rb1;
  a.row_end1 = n1 > 0 ? re1 : rb1;
  a.nstrips = p.nstrips;
  a.nbands = p.ntiles;
  a.nbands0 = nb0;
  a.nwaves = p.nwaves;
  a.fixed_lo = -L.row0;
  a.fixed_hi = L.nrows_global - L.row0;
  const int64_t o = L.origin();
  const int nv = p.vec / (dt == DType::F32 ? 4 : 2);
  if (dt == DType::F32) {
    const float* s = static_cast<const float*>(src) + o;
    float* d = static_cast<float*>(dst) + o;
    dispatch_variant<float>(nv, p.prefetch, p.tight != 0, p.k, (unsigned)p.nblocks, s, d, a, (float)r, stream);
  } else {
    const double* s = static_cast<const double*>(src) + o;
    double* d = static_cast<double*>(dst) + o;
    dispatch_variant<double>(nv, p.prefetch, p.tight != 0, p.k, (unsigned)p.nblocks, s, d, a, r, stream);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) fail(__FILE__, __LINE__, std::string("tb_kernel launch: ") + hipGetErrorString(e));
}

}  // namespace kern
}  // namespace heat2d
