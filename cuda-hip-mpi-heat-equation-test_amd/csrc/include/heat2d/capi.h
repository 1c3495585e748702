/* heat2d C ABI — consumed by the Python package through ctypes and by any
 * other host language. Replaces the reference's Fortran<->C++ `bind(c)`
 * launcher interface (fortran/hip/heat.F90:48-102 -> heat_kernel.cpp:48-150)
 * with a complete engine API. Every function returns 0 on success, non-zero on
 * error; heat2d_last_error() gives the message (thread-local). */
#ifndef HEAT2D_CAPI_H
#define HEAT2D_CAPI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct heat2d_layout {
  int64_t nrows, ncols, halo, cpad, pitch, row0, nrows_global;
} heat2d_layout;

typedef struct heat2d_ic {
  int32_t kind;
  double a, b;
  double x0, x1, y0, y1;
  int64_t i0, i1, j0, j1;
  double kx, ky;
  double pad;
} heat2d_ic;

typedef struct heat2d_config {
  int64_t n_rows, n_cols;
  int32_t dtype, backend;
  double r;
  int32_t tb, overlap, copy_swap, managed, device, use_graph;
  int64_t tile_rows, halo;
  int32_t comm_cus, autotune;
  int32_t engine, arith; /* arith: 0 reference rounding, 1 contracted fma, 2 jacobi (r = 1/4) */
  int32_t edge_shift; /* rows each edge slab gives the middle ones (common.hpp decompose) */
  int64_t slab_row0, slab_rows_global; /* 1-rank rehearsal of a middle slab (0: the slab is the grid) */
} heat2d_config;

typedef struct heat2d_tb_plan {
  int32_t k, vec, strip_w, useful_w;
  int64_t tile_rows, nstrips, ntiles, nwaves, nblocks;
  int32_t skew, blocks_per_cu, prefetch, main;
} heat2d_tb_plan;

typedef struct heat2d_rect {
  int64_t r0, r1, s0, s1, nb;
} heat2d_rect;

typedef struct heat2d_split_plan {
  int32_t k, ring, valid, nedge;
  heat2d_rect main;
  heat2d_rect edge[4];
  int64_t main_waves, edge_waves, main_items, edge_items;
  int32_t nrects, flags;  // flags & 2: dynamic item queue, & 4: lead order
  heat2d_rect rects[6];
} heat2d_split_plan;

typedef int (*heat2d_exchange_fn)(void* ctx, void* send_lo, void* send_hi, void* recv_lo,
                                  void* recv_hi, int64_t count, int32_t dtype);
typedef int (*heat2d_allreduce_fn)(void* ctx, double* vals, int32_t n, int32_t op);
typedef int (*heat2d_barrier_fn)(void* ctx);

const char* heat2d_last_error(void);
/* print a native backtrace to stderr on SIGABRT / SIGSEGV / SIGBUS / SIGFPE / SIGILL, then chain to the
   previous handler (idempotent) */
int heat2d_install_crash_handler(void);
int heat2d_version(void);
int heat2d_max_tb(void);
int heat2d_device_count(int* n);
// Device limits the reference's PyCUDA program queries (python/cuda/cuda.py:16-27):
// out = [max_block_dim_x, _y, _z, max_grid_dim_x, _y, _z, total_constant_memory,
//        max_threads_per_block, warp_size, multiprocessor_count]
int heat2d_device_limits(int device, int64_t* out10);
// Diagnostics (HEAT2D_WAVE_TIMES=1): per-wave {start, end, wave, 0} wall-clock
// ticks of the last stencil launch; *n = waves copied.
int heat2d_wave_times(uint64_t* out, int64_t max_waves, int64_t* n);

int heat2d_make_layout(int64_t nrows, int64_t ncols, int64_t halo, int64_t row0,
                       int64_t nrows_global, heat2d_layout* out);
int heat2d_decompose(int64_t n, int nranks, int rank, int64_t* row0, int64_t* nrows);
/* the same with the edge slabs' rows shifted to the middle ones (common.hpp) */
int heat2d_decompose_shifted(int64_t n, int nranks, int rank, int64_t edge_shift, int64_t* row0, int64_t* nrows);
/* MAIN + EDGE split of one cycle (the overlapped schedule's two launches) */
int heat2d_plan_split(int dtype, const heat2d_layout* L, int k, int64_t band, heat2d_split_plan* out);
int heat2d_plan_tb(int dtype, const heat2d_layout* L, int64_t rb, int64_t re, int k,
                   int64_t tile_rows, heat2d_tb_plan* out);

/* input.dat parsing (C++ twin of utils/config.py): out = {n, sigma, nu, dom_len, ntime, soln, nfields} */
int heat2d_parse_input(const char* text, double* out7);

/* Raw ops on caller-owned memory (device pointers for the HIP ops; host for cpu_*).
 * `stream` is a hipStream_t (e.g. torch.cuda.current_stream().cuda_stream). */
int heat2d_tb(int dtype, const void* src, void* dst, const heat2d_layout* L, int64_t rb,
              int64_t re, int k, double r, void* stream, int64_t tile_rows, int arith);
int heat2d_init_field(int dtype, void* field, const heat2d_layout* L, const heat2d_ic* ic,
                      const double* xcoord_dev, const double* ycoord_dev, void* stream);
int heat2d_stats(int dtype, const void* field, const void* other, const heat2d_layout* L,
                 double* work_dev, double* out_dev, void* stream);
int64_t heat2d_stats_work_elems(void);
int heat2d_copy(void* dst, const void* src, int64_t bytes, void* stream, int blocks);
int heat2d_read(const void* src, int64_t bytes, void* sink, void* stream, int blocks);
int heat2d_pack_rows(int dtype, const void* field, const heat2d_layout* L, int64_t row,
                     int64_t nrows, void* buf, void* stream);
int heat2d_unpack_rows(int dtype, void* field, const heat2d_layout* L, int64_t row,
                       int64_t nrows, const void* buf, void* stream);

int heat2d_cpu_tb(int dtype, const void* src, void* dst, const heat2d_layout* L, int64_t rb,
                  int64_t re, int k, double r, int arith);
int heat2d_cpu_init_field(int dtype, void* field, const heat2d_layout* L, const heat2d_ic* ic,
                          const double* xcoord, const double* ycoord);
int heat2d_cpu_stats(int dtype, const void* field, const void* other, const heat2d_layout* L,
                     double* out6);

/* Transports (opaque handles). */
int heat2d_rccl_unique_id(void* out128);
int heat2d_transport_self(void** out);
int heat2d_transport_rccl(const void* uid128, int rank, int size, int device, void** out);
/* 1-rank periodic self-exchange over RCCL: perf rehearsal of the multi-GPU schedule on one GPU */
int heat2d_transport_rccl_loop(int device, void** out);
int heat2d_transport_callback(heat2d_exchange_fn ex, heat2d_allreduce_fn ar, heat2d_barrier_fn br,
                              void* ctx, int rank, int size, void** out);
typedef int (*heat2d_allgather_fn)(void* ctx, const void* mine, void* all, int64_t bytes);
// IPC transport (process per GPU, no RCCL): host collectives through the callbacks.
int heat2d_transport_ipc(heat2d_allgather_fn ag, heat2d_allreduce_fn ar, heat2d_barrier_fn br, void* ctx, int rank,
                         int size, int device, void** out);
int heat2d_transport_ipc_loop(int device, void** out);
int heat2d_transport_free(void* t);
/* what the fabric reports for this rank: {kind (0 host/self, 1 RCCL, 2 IPC), nranks, rank, device}
   (RCCL: ncclCommCount / ncclCommUserRank / ncclCommCuDevice) */
int heat2d_transport_info(void* t, int32_t* out4);
/* hipDeviceGetPCIBusId of a device ordinal ("dddd:bb:dd.f") */
int heat2d_device_pci_bus_id(int device, char* out, int64_t cap);
/* fail fast: abort the transport's fabric (RCCL: ncclCommAbort); its solver's next synchronisation raises */
int heat2d_transport_abort(void* t, const char* reason);
/* watchdog mechanism self-test (no GPU): mode 0 = progress for progress_polls polls then a hang,
   1 = idle (must not fire), 2 = fabric error. fired_after_s = -1 if it did not fire within wait_s. */
int heat2d_watchdog_selftest(double timeout_s, int mode, int progress_polls, double wait_s, double* fired_after_s,
                             char* reason, int64_t cap);

/* Solver. */
int heat2d_solver_create(const heat2d_config* cfg, void* transport, void** out);
int heat2d_solver_free(void* s);
int heat2d_solver_init(void* s, const heat2d_ic* ic, const double* xg, const double* yg);
int heat2d_solver_step(void* s, int64_t n);
/* step(n) with the global statistics of T_n and its one-step residual fused into the last cycle:
   out6 = {sum, sum_sq, min, max, sum (T_n - T_{n-1})^2, max |T_n - T_{n-1}|} */
int heat2d_solver_step_stats(void* s, int64_t n, double* out6);
/* depth of the balanced cycles step() runs when no measured schedule applies */
int heat2d_solver_pref_depth(void* s, int32_t* out);
int heat2d_solver_sync(void* s);
int heat2d_solver_stats(void* s, double* out6, int residual);
int heat2d_solver_download(void* s, void* host, int64_t ld);
// memory-fit planner (runtime.hpp solver_footprint / plan_max_grid): out3 =
// {field bytes, workspace bytes, total} of a Solver of cfg on rank of nranks
int heat2d_solver_footprint(const heat2d_config* cfg, int rank, int nranks, int64_t* out3);
// the largest n x n grid of dtype on nranks ranks whose largest slab fits budget_bytes
int heat2d_plan_max_grid(int dtype, int nranks, int64_t budget_bytes, int64_t* n);
// hipMemGetInfo of device
int heat2d_mem_info(int device, int64_t* free_bytes, int64_t* total_bytes);
// s's current field, local rows [r0, r0 + nrows), against other's, rows
// [other_r0, ...): out2 = {max |a - b| (NaN if any), differing bit patterns}
int heat2d_solver_compare(void* s, void* other, int64_t r0, int64_t nrows, int64_t other_r0, double* out2);
int heat2d_solver_upload(void* s, const void* host, int64_t ld);
int heat2d_solver_layout(void* s, heat2d_layout* out);
/* run-time specialised FTCS step (hipRTC; python/cuda/cuda.py parity) */
int heat2d_jit_create(int dtype, const heat2d_layout* L, double r, int device, int arith, void** out);
int heat2d_jit_free(void* j);
int heat2d_jit_step(void* j, const void* src, void* dst, void* stream);
int heat2d_jit_render(int dtype, const heat2d_layout* L, double r, int arith, char* buf, int64_t cap, int64_t* len);
int heat2d_jit_compile_check(const char* source, const char* arch, int64_t* code_bytes);
/* phase timers (hipEvents): on/off; read = [main ms, edge ms, exchange ms, cycle ms, cycles], then reset */
int heat2d_solver_timing(void* s, int on);
int heat2d_solver_phase_times(void* s, double* out5);
/* plan / autotune every cycle depth a step(n) will use (keep planning out of timed regions) */
int heat2d_solver_prepare(void* s, int64_t n);
/* split plan used for depth k (planned / autotuned on first use); tuned_ms = autotuned cycle time or 0 */
int heat2d_solver_plan(void* s, int k, heat2d_split_plan* out, float* tuned_ms);
/* number of split plans made so far (first uses of a depth; a prepare()d run adds none) */
int heat2d_solver_plans_made(void* s, int64_t* out);
int heat2d_solver_info(void* s, int32_t* tb, int64_t* band, int64_t* steps, void** field,
                       void** stream);

/* Loopback group: P slabs on one device (or host). */
int heat2d_group_create(const heat2d_config* cfg, int nranks, void** out);
int heat2d_group_free(void* g);
int heat2d_group_init(void* g, const heat2d_ic* ic, const double* xg, const double* yg);
int heat2d_group_step(void* g, int64_t n);
int heat2d_group_download(void* g, void* host, int64_t ld);
/* whole global owned region -> the members' slabs, then a loopback halo exchange */
int heat2d_group_upload(void* g, const void* host, int64_t ld);
/* member i's solver (borrowed handle: valid while the group lives; plan / info / hist queries) */
int heat2d_group_member(void* g, int i, void** solver);
/* cycles step() launched since the last reset, by depth: out[k], k = 0..heat2d_max_tb() (n >= max_tb + 1) */
int heat2d_solver_cycle_hist(void* s, int64_t* out, int n, int reset);
/* the measured cycle schedule prepare(n) chose for step(n): depths in out[0..min(cap, len)); len = -1 if none
   (step(n) then runs balanced cycles of the preferred depth) */
int heat2d_solver_schedule(void* s, int64_t n, int32_t* out, int64_t cap, int64_t* len);
/* *out = 1 if step(n) replays its measured schedule as one captured hipGraph, else 0 (eager launches) */
int heat2d_solver_schedule_replayed(void* s, int64_t n, int32_t* out);
// Cycle depths step(n) runs from the solver's current state (len = count; out may be null).
int heat2d_solver_step_cycles(void* s, int64_t n, int32_t* out, int64_t cap, int64_t* len);
// Halo rows exchanged per side since the last reset (sum over cycles).
int heat2d_solver_halo_rows(void* s, int reset, int64_t* out);
// Valid ghost rows of the current buffer (the last exchange's depth).
int heat2d_solver_ghost_rows(void* s, int32_t* out);
// Plans / schedules the solver took from the persistent plan cache; the cache file path.
int heat2d_solver_plan_cache_hits(void* s, int64_t* out);
// Depths autotuned in this process and candidate plans screened for them.
int heat2d_solver_tune_stats(void* s, int64_t* depths, int64_t* candidates);
int heat2d_plan_cache_path(char* buf, int64_t cap);
// The plan cache's own entry points (format tests): reload $HEAT2D_PLAN_CACHE,
// put / get one plan (found = 0 on a miss or a refused entry) and one schedule
// (count = -1 on a miss).
int heat2d_plan_cache_reload(void);
int heat2d_plan_cache_put(const char* ctx, int k, int64_t band, const heat2d_split_plan* p, float ms);
int heat2d_plan_cache_get(const char* ctx, int k, int64_t band, heat2d_split_plan* p, float* ms, int32_t* found);
int heat2d_plan_cache_put_schedule(const char* ctx, int64_t n, const int32_t* depths, int64_t count);
int heat2d_plan_cache_get_schedule(const char* ctx, int64_t n, int32_t* depths, int64_t cap, int64_t* count);
// Where the depth-k split plan came from: 0 planned (not autotuned), 1 autotuned in
// this process, 2 the plan cache (re-validated), -1 not planned yet.
int heat2d_solver_plan_origin(void* s, int k, int32_t* out);
// Autotune / measured-schedule eligibility of a decomposition (the same on every rank).
int heat2d_autotune_slabs(int64_t n_rows, int64_t n_cols, int nranks, int autotune, int32_t* out);
/* the schedule search itself on given cycle times t_ms[k] (k = 1..kmax; t_ms[0] unused): depths in out */
// schedule search (runtime.hpp, schedule.cpp), on per-depth cost arrays t_ms[0..kmax] (< 0: unusable):
// dp_schedule: the exact least-cost schedule of n steps (*total its cost)
int heat2d_dp_schedule(int64_t n, int kmax, const double* t_ms, int32_t* out, int64_t cap, int64_t* len,
                       double* total);
// near_schedules: balanced candidates within tol of the best, concatenated in out, lengths / costs per candidate
int heat2d_near_schedules(int64_t n, int kmax, const double* t_ms, double tol, int m, int32_t* out, int64_t cap,
                          int64_t* lens, double* costs, int32_t* count);
// search_schedule with prescan(k) = pre_ms[k] and tune(k) = tuned_ms[k] (arrays of kmax + 1): the
// chosen schedule, its cost and the depths prescanned / tuned, in order (each array >= kmax entries)
int heat2d_search_schedule(int64_t n, int kmax, const double* pre_ms, const double* tuned_ms, int32_t* out,
                           int64_t cap, int64_t* len, double* cost, int32_t* prescanned, int32_t* nprescanned,
                           int32_t* tuned, int32_t* ntuned);

/* I/O (io.cpp). */
int heat2d_write_xyz(const char* path, int dtype, const void* host, int64_t nrows, int64_t ncols,
                     int64_t ld, const double* x, const double* y, int append);
int heat2d_write_npy(const char* path, int dtype, const void* host, int64_t nrows, int64_t ncols,
                     int64_t ld);

#ifdef __cplusplus
}
#endif

#endif /* HEAT2D_CAPI_H */
