// heat2d device-kernel launchers (gfx950). Every launcher is capture-safe:
// no allocation, no synchronisation, only kernel launches on `stream`.
#pragma once

#include <hip/hip_runtime.h>

#include "heat2d/common.hpp"

namespace heat2d {
namespace kern {

// Tiling of one temporal-block launch. Filled by plan_tb(); exposed so tests
// and the autotuner can inspect / override it.
struct TbPlan {
  int32_t k;          // time steps fused in this launch (1..kMaxTB)
  int32_t vec;        // elements per lane (16 B: 4 fp32 / 2 fp64)
  int32_t strip_w;    // columns loaded per wave (64 * vec)
  int32_t useful_w;   // columns produced per wave (strip_w - 2*ceil(k, vec))
  int64_t tile_rows;  // output rows per wave tile
  int64_t nstrips;
  int64_t ntiles;
  int64_t nwaves;
  int64_t nblocks;    // 256-thread workgroups (4 independent waves each)
  int32_t skew;       // level pipeline skew (always 1: upward march, see tb_impl.hpp)
  int32_t blocks_per_cu;  // resident workgroups per CU (occupancy API)
  int32_t prefetch;   // level-0 row ring per wave (RING; RING-2 rows in flight)
  int32_t main;       // 1: interior-only (MAIN) kernel instance
};

// Plan a launch that advances rows [row_begin, row_end) of the slab by k steps.
// tile_rows == 0 selects the occupancy-driven row bands, > 0 bands of that many
// rows, < 0 -tile_rows segments (TbRect nb < 0; ntiles = -segments); cus > 0 plans for a
// stream restricted to that many CUs (comm-reserving CU mask).
// arith: 0 = reference arithmetic (every op rounded), 1 = contracted fma form,
// 2 = r == 1/4: (S + E + N + W) / 4 (tb_impl.hpp, March); every launcher below
// takes it last.
TbPlan plan_tb(DType dt, const SlabLayout& L, int64_t row_begin, int64_t row_end, int k,
               int64_t tile_rows = 0, int cus = 0, int arith = 0);

// dst(rows [row_begin,row_end)) = k FTCS steps of src. `src`/`dst` are
// allocation bases laid out per `L`. Requires k <= L.halo and the k ghost rows
// on both sides of the range to hold valid data at time t (Dirichlet rows are
// recognised from L.row0 / L.nrows_global and kept fixed).
void launch_tb(DType dt, const void* src, void* dst, const SlabLayout& L, int64_t row_begin,
               int64_t row_end, int k, double r, hipStream_t stream, int64_t tile_rows = 0, int cus = 0,
               int arith = 0);
// Same for TWO disjoint row ranges [rb0, re0) and [rb1, re1) in one launch.
void launch_tb2(DType dt, const void* src, void* dst, const SlabLayout& L, int64_t rb0, int64_t re0, int64_t rb1,
                int64_t re1, int k, double r, hipStream_t stream, int64_t tile_rows = 0, int cus = 0,
                int arith = 0);

// Split schedule of one cycle (k steps over the whole slab) into two launches
// on two streams:
//   MAIN: rows [band, n-band), all strips — the interior kernel (no frame-row
//         code: fewer registers), a persistent grid on all wave slots;
//   EDGE: the two boundary bands (all strips), general kernel.
// The caller orders them with events (solver.cpp). valid = 0: slab too thin
// or narrow for the split (use launch_tb on the whole slab); valid = 2: a
// single-launch plan (plan_single); valid = 3: the split run edge-first — the
// band launch alone, then the interior, both on the compute stream, with the
// halo exchange beside the interior (the autotuner's choice for slabs where
// the interior would otherwise share the chip with the band waves).
// nb > 0: nb row bands per strip (nb x strips work items); nb < 0: -nb equal
// segments of the strip-major row sequence (one work item each, crossing strip
// ends where they fall: equal rows per wave for any strip count).
struct TbRect {
  int64_t r0, r1, s0, s1, nb;
};
// rects of one launch (SplitPlan::rects, the kernel's TbArgs::rect)
constexpr int kMaxPlanRects = 6;
constexpr int32_t kPlanDynamic = 2;  // SplitPlan::flags
constexpr int32_t kPlanLead = 4;     // SplitPlan::flags (valid = 1)
struct SplitPlan {
  int32_t k, ring, valid, nedge;
  TbRect main;
  TbRect edge[4];
  int64_t main_waves, edge_waves, main_items, edge_items;
  // nrects > 0 (arith 2): `main` cut into frame-strip-weighted rects,
  // launched instead of `main` (stencil_tb.hip weight_main).
  // flags & kPlanDynamic: the main launch takes its items from a dynamic
  // queue (more items than waves; TbArgs::queue). flags & kPlanLead (valid 1,
  // exchanging slabs): the concurrent order with the band launch issued
  // FIRST — its waves take their slots before the interior's, the interior's
  // last-dispatched waves (its one-item waves) start behind them, and the
  // exchange follows the bands on the comm stream.
  int32_t nrects, flags;
  TbRect rects[kMaxPlanRects];
};
// The same plan with its boundary-band (EDGE) rects cut into `nb` row bands
// each (valid = 1 / 3; default 1): more, shorter band items — nb x as many
// waves for the latency-bound band launch, each marching B/nb + 2k rows
// instead of B + 2k.
SplitPlan with_edge_bands(DType dt, const SplitPlan& p, int64_t nb, int arith = 0);
// ring_override: 4 | 6 (0: default); main_bands: MAIN row bands (0: persistent default;
// < 0: -main_bands segments, TbRect)
SplitPlan plan_split(DType dt, const SlabLayout& L, int k, int64_t band, int cus = 0, int spare_waves = 0,
                     int ring_override = 0, int64_t main_bands = 0, int arith = 0);
// The alternative the autotuner weighs against the split (valid = 2): ONE
// general launch over the whole slab (no edge part), e.g. for small grids
// where the second launch costs more than it saves.
SplitPlan plan_single(DType dt, const SlabLayout& L, int k, int cus = 0, int ring_override = 0, int64_t bands = 0,
                      int arith = 0);
// Whether the plan's boundary-band launch runs on the interior kernel (its
// bands clear of the global frame rows: every middle rank) rather than the
// general one (1 wave/SIMD at deep fp64 depths).
bool edges_on_main(const SlabLayout& L, const SplitPlan& p);
// One boundary-band rect of the plan alone, on the interior kernel where it
// stays clear of the global frame rows, else the general one (edge ranks).
bool edge_rect_on_main(const SlabLayout& L, const SplitPlan& p, int i);
void launch_edge_rect(DType dt, const void* src, void* dst, const SlabLayout& L, const SplitPlan& p, int i, double r,
                      hipStream_t stream, int arith = 0);
// queue: 2 device counters (zeroed once) for plans with flags & kPlanDynamic (dynamic items)
void launch_split(DType dt, const void* src, void* dst, const SlabLayout& L, const SplitPlan& p, bool main_part,
                  double r, hipStream_t stream, int arith = 0, uint32_t* queue = nullptr);

// Initial / boundary condition kinds (covers every IC of the reference
// variants, see models/presets.py for the mapping).
enum class IcKind : int32_t {
  Uniform = 0,   // interior = a, Dirichlet frame = b   (fortran/hip/heat.F90:274-282)
  Box = 1,       // a inside [x0,x1]x[y0,y1] (frame included), else b (fortran/serial/heat.f90:40-48)
  IndexBox = 2,  // a for global frame-index ranges [i0,i1) x [j0,j1), else b (python/serial/heat.py:25)
  Sine = 3,      // a * sin(kx*pi*(x-x0)/(x1-x0)) * sin(ky*pi*(y-y0)/(y1-y0)), frame = 0 (analytic oracle)
  Const = 4,     // a everywhere
};

struct IcParams {
  int32_t kind;
  double a, b;
  double x0, x1, y0, y1;     // box / sine extents
  int64_t i0, i1, j0, j1;    // index box (frame-inclusive global indices: frame row = 0)
  double kx, ky;             // sine mode numbers
  double pad;                // value for allocation padding outside the frame
};

// Fill the whole allocation (owned points, Dirichlet frame, ghost/pad rows)
// from the IC. `xcoord` has nrows_global+2 entries (frame-inclusive, entry 0
// is global row -1), `ycoord` has ncols+2 entries — both device arrays.
void launch_init(DType dt, void* field, const SlabLayout& L, const IcParams& ic,
                 const double* xcoord, const double* ycoord, hipStream_t stream);

// Statistics over the owned region: [sum, sum_sq, min, max, sum_sq_diff, max_abs_diff]
// (diff terms vs `other`, zero if other == nullptr). Deterministic two-pass
// reduction; `work` must hold stats_work_elems() doubles; result (6 doubles)
// written to `out` (device).
int64_t stats_work_elems();
void launch_stats(DType dt, const void* field, const void* other, const SlabLayout& L,
                  double* work, double* out, hipStream_t stream);

// One cycle of k steps over the whole slab (one general launch, like
// plan_single) that also reduces the statistics of the NEW field and its
// one-step residual T_k - T_{k-1} — [sum, sum_sq, min, max, sum_sq_diff,
// max_abs_diff], the launch_stats layout — fused into the march's stored
// level (no extra pass over the field): per-wave partials in `partials`
// (>= kNStat * max_stats_waves() doubles), then a fixed-order reduce into
// out6 (device). Deterministic for a given slab and device.
int64_t max_stats_waves();
// Diagnostics: per-wave {start, end, wave id, 0} (wall clock ticks) of the
// last tb_kernel launch when HEAT2D_WAVE_TIMES=1; returns the waves copied.
int64_t wave_times(uint64_t* out, int64_t max_waves);
void launch_tb_stats(DType dt, const void* src, void* dst, const SlabLayout& L, int k, double r, double* partials,
                     double* out6, hipStream_t stream, int arith = 0);
void launch_reduce_partials(const double* partials, int64_t nparts, double* out6, hipStream_t stream);

// Field comparison (the bench's check of its timed field against an
// independent engine): rows [ra, ra + nrows) of `a` (layout La) against rows
// [rb, rb + nrows) of `b` (layout Lb), owned columns (La.ncols == Lb.ncols).
// out2 (device) = {max |a - b|, number of elements whose bit patterns differ}
// (NaN anywhere: max = NaN). `work` >= 2 * compare_work_blocks() doubles.
int64_t compare_work_blocks();
void launch_compare(DType dt, const void* a, const SlabLayout& La, int64_t ra, const void* b, const SlabLayout& Lb,
                    int64_t rb, int64_t nrows, double* work, double* out2, hipStream_t stream);

// Vectorised streaming copy / read (bandwidth roof probes; copy-swap mode).
void launch_copy(void* dst, const void* src, int64_t bytes, hipStream_t stream, int blocks = 0);
void launch_read(const void* src, int64_t bytes, unsigned* sink, hipStream_t stream, int blocks = 0);

// Pack/unpack `nrows` rows starting at local row `row` into / from a
// contiguous buffer of nrows*ncols elements (the owned columns only). Used for
// generic transports and host staging; the RCCL path sends rows in place.
void launch_pack_rows(DType dt, const void* field, const SlabLayout& L, int64_t row,
                      int64_t nrows, void* buf, hipStream_t stream);
void launch_unpack_rows(DType dt, void* field, const SlabLayout& L, int64_t row, int64_t nrows,
                        const void* buf, hipStream_t stream);

// IPC transport ordering (kernels/ipc_sync.hip): one 64-B slot per rank in
// host-shared memory; `ctrl` = {abort word, timed-out rank + 1}.
struct IpcSlot {
  uint64_t ready, done;
  uint64_t pad[6];
};
void launch_ipc_arrive(IpcSlot* slots, uint64_t* ctrl, int me, int p0, int p1, uint64_t timeout_ticks,
                       hipStream_t stream);
void launch_ipc_depart(IpcSlot* slots, int me, hipStream_t stream);

}  // namespace kern
}  // namespace heat2d
