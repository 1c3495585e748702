// heat2d — MI355X-native 2-D heat-equation framework.
// Common types, error handling and the slab memory layout shared by kernels,
// the runtime and the C ABI.
//
// Layout (replaces the x-fastest, 1-ghost, 32-bit-indexed layout of
// reference fortran/hip/heat_kernel.cpp:26 `idx(i,j)`):
//   * row-major T[i][j]; i = x index (slow, decomposed across ranks exactly as
//     the reference splits x, fortran/hip/heat.F90:147), j = y index (fast);
//   * `halo` ghost rows above and below the owned rows (>= temporal-block depth),
//     so a halo exchange is a contiguous block of rows (zero-copy for RCCL);
//   * `cpad` padding columns on the left (column -1 is the Dirichlet column),
//     pitch rounded so every row starts 256-B aligned;
//   * all offsets int64 (a 288 GB HBM field holds ~3.6e10 fp64 points).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>

namespace heat2d {

enum class DType : int32_t { F32 = 0, F64 = 1 };

inline size_t dtype_size(DType d) { return d == DType::F32 ? 4 : 8; }
inline const char* dtype_name(DType d) { return d == DType::F32 ? "fp32" : "fp64"; }

struct Error : std::runtime_error {
  using std::runtime_error::runtime_error;
};

[[noreturn]] inline void fail(const char* file, int line, const std::string& msg) {
  throw Error(std::string(file) + ":" + std::to_string(line) + ": " + msg);
}

#define HEAT2D_REQUIRE(cond, msg)                                              \
  do {                                                                         \
    if (!(cond)) ::heat2d::fail(__FILE__, __LINE__, std::string("requirement failed: ") + #cond + " — " + (msg)); \
  } while (0)

// Column padding on the left of every row (elements). Must be >= the largest
// temporal-block depth (rounded to the vector width) and keep rows aligned.
constexpr int64_t kColPad = 32;
// Largest supported temporal-block depth (time steps fused per HBM pass):
// 24 for both dtypes (max_tb). The fp64 interior kernel keeps 2 waves/SIMD up
// to K = 24 with ring 4, so a short run can take one HBM pass; the packed fp32
// interior kernel keeps 2 waves/SIMD up to K = 24 with ring 4 (a floor:
// tb_impl.hpp kMinWaves) — deeper passes for the HBM-bound big fp32 grids (one
// read + one write of the field per K steps: the 240 GB grid's 64 steps in 3
// passes instead of 4, +13.8 %, profiles/r4/deep32/).
constexpr int kMaxTB = 24;
constexpr int kMaxTBF32 = 24;
inline int max_tb(DType dt) { return dt == DType::F64 ? kMaxTB : kMaxTBF32; }
// Default halo depth (ghost rows per side). Must be >= temporal depth used.
constexpr int64_t kDefaultHalo = kMaxTB;

// Memory layout of one rank's slab. POD so it can cross the C ABI.
struct SlabLayout {
  int64_t nrows;         // owned rows on this slab (local nx)
  int64_t ncols;         // owned columns (ny)
  int64_t halo;          // ghost rows above and below
  int64_t cpad;          // padding columns left of column 0
  int64_t pitch;         // elements per row
  int64_t row0;          // global row index of local row 0
  int64_t nrows_global;  // global owned rows (n)

  __host__ __device__ int64_t rows_alloc() const { return nrows + 2 * halo; }
  __host__ __device__ int64_t elems() const { return rows_alloc() * pitch; }
  // offset of element (i, j), i in [-halo, nrows+halo), j in [-cpad, pitch-cpad)
  __host__ __device__ int64_t offset(int64_t i, int64_t j) const { return (i + halo) * pitch + (j + cpad); }
  __host__ __device__ int64_t origin() const { return offset(0, 0); }
  __host__ __device__ int64_t col_hi() const { return pitch - cpad; }  // exclusive upper column bound
};

// Pitch rule: left pad + owned + >=1 Dirichlet column, rounded up to 64
// elements (256 B fp32 / 512 B fp64 row alignment).
inline int64_t make_pitch(int64_t ncols, int64_t cpad) {
  int64_t need = cpad + ncols + kColPad;  // right pad: room for the widest strip overrun
  return (need + 63) / 64 * 64;
}

inline SlabLayout make_layout(int64_t nrows, int64_t ncols, int64_t halo, int64_t row0,
                              int64_t nrows_global) {
  SlabLayout L{};
  L.nrows = nrows;
  L.ncols = ncols;
  L.halo = halo;
  L.cpad = kColPad;
  L.pitch = make_pitch(ncols, L.cpad);
  L.row0 = row0;
  L.nrows_global = nrows_global;
  return L;
}

// 1-D slab decomposition of `n` global rows over `nranks` ranks, remainder
// spread over the first ranks (the reference silently drops n mod P,
// fortran/hip/heat.F90:147 `nx = n/nblocks(1)`).
//
// edge_shift > 0 (nranks >= 3): the two edge slabs (rank 0 and nranks - 1,
// the global frame rows on one side) each give `edge_shift` rows to the
// middle ones, spread evenly (remainder to the first middle ranks). An edge
// slab's cycle costs more per row than a middle one's — its frame-side band
// runs on the general kernel in the interior's tail (profiles/r6/b/: 40-55 us
// of a 0.62 ms one-cycle step at N = 8) — and a multi-rank step lasts as long
// as its slowest rank; bench.py measures the excess and picks the shift
// (SolverConfig::edge_shift). Clamped to a quarter of the uniform slab.
struct SlabRange {
  int64_t row0;
  int64_t nrows;
};
inline int64_t slab_rows(int64_t n, int nranks, int rank, int64_t edge_shift) {
  const int64_t base = n / nranks, rem = n % nranks;
  int64_t rows = base + (rank < rem ? 1 : 0);
  const int64_t e = nranks >= 3 ? std::max<int64_t>(0, std::min<int64_t>(edge_shift, base / 4)) : 0;
  if (e == 0) return rows;
  if (rank == 0 || rank == nranks - 1) return rows - e;
  const int64_t mid = nranks - 2, give = 2 * e;
  return rows + give / mid + (rank - 1 < give % mid ? 1 : 0);
}
inline SlabRange decompose(int64_t n, int nranks, int rank, int64_t edge_shift = 0) {
  HEAT2D_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, "bad rank/nranks");
  int64_t row0 = 0;
  for (int r = 0; r < rank; ++r) row0 += slab_rows(n, nranks, r, edge_shift);
  return {row0, slab_rows(n, nranks, rank, edge_shift)};
}

}  // namespace heat2d
