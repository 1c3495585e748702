// heat2d native runtime: slab solver, transports, CPU twin kernels.
//
// Replaces the reference's host drivers (fortran/hip/heat.F90 setup/swap/
// heat_eqn, fortran/mpi+cuda/heat.F90) with one engine that
//   * keeps two pitched fields (ping-pong, no per-step D2D copy),
//   * advances K steps per HBM pass (temporal blocking, kernels.hpp),
//   * splits each cycle into boundary bands + interior: the bands and their
//     halo exchange (RCCL send/recv, zero-copy rows) run on a comm stream
//     beside the interior kernel, ordered only by hipEvents (solver.cpp),
//   * runs the same schedule on a CPU backend (for CPU-only CI with gloo) and
//     on a loopback group (P slabs on one GPU, bitwise == P=1).
#pragma once

#include <hip/hip_runtime.h>

#include <functional>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "heat2d/common.hpp"
#include "heat2d/jit.hpp"
#include "heat2d/kernels.hpp"

namespace heat2d {

enum class Backend : int32_t { Hip = 0, Cpu = 1 };

// POD config (crosses the C ABI).
struct SolverConfig {
  int64_t n_rows;      // global owned rows (x points)
  int64_t n_cols;      // owned columns (y points)
  int32_t dtype;       // DType
  int32_t backend;     // Backend
  double r;            // FTCS coefficient nu*dt/delta^2
  int32_t tb;          // temporal-block depth K (steps per HBM pass)
  int32_t overlap;     // 1: boundary/interior split + comm stream (P>1)
  int32_t copy_swap;   // 1: reference-parity mode, full D2D copy each step (K forced to 1)
  int32_t managed;     // 1: hipMallocManaged fields (parity with fortran/cuda_kernel/heat_managed.F90)
  int32_t device;      // HIP device ordinal (-1: current)
  int32_t use_graph;   // 1: replay cycles from a captured hipGraph
  int64_t tile_rows;   // 0: auto
  int64_t halo;        // 0: auto (= kMaxTB)
  int32_t comm_cus;    // P>1 overlap: >0 CUs masked off the compute stream; 0 soft (interior planned for ncu-2); -1 none
  int32_t autotune;    // split schedule: time candidate (ring, bands) plans once per depth and keep the fastest
                       // (-1 auto: on for slabs >= 2^24 points, 0 off, 1 on)
  int32_t engine;      // 0: temporal-blocked kernels; 1: run-time specialised hipRTC kernel (K = 1, jit.hpp)
  int32_t arith;       // 0: reference arithmetic, every op rounded (bitwise == NumPy golden);
                       // 1: contracted fma(r, sum - 4c, c) (one op fewer per point, kernels.hpp);
                       // 2: r == 1/4 only: r * sum (zero centre weight: 3 adds per point, tb_impl.hpp)
  int32_t edge_shift;  // rows each edge slab gives to the middle ones (decompose(); bench.py measures it)
  // 1-rank rehearsal of a MIDDLE slab (slab_rows_global > 0): this solver owns
  // rows [slab_row0, slab_row0 + n_rows) of a grid of slab_rows_global rows,
  // so its bands are interior bands, as on rank 3 of 8 (0: the slab is the grid)
  int64_t slab_row0;
  int64_t slab_rows_global;
};

// ---------------------------------------------------------------- transports

class Transport {
 public:
  virtual ~Transport() = default;
  virtual int rank() const = 0;
  virtual int size() const = 0;
  // Halo exchange of k rows of `field` (allocation base, layout L): rows
  // [0,k) -> rank-1, rows [nrows-k,nrows) -> rank+1; receive into [-k,0) from
  // rank-1 and [nrows,nrows+k) from rank+1. on_device: `field` is device
  // memory and the exchange is enqueued on `stream`; otherwise host memory,
  // synchronous.
  virtual void exchange(void* field, const SlabLayout& L, DType dt, int64_t k, hipStream_t stream,
                        bool on_device) = 0;
  // Blocking all-reduce of host doubles (op 0 = sum, 1 = max, 2 = min).
  virtual void allreduce(double* vals, int n, int op) = 0;
  virtual void barrier() = 0;
  virtual std::string name() const = 0;
  virtual bool capturable() const { return false; }  // safe inside hipGraph capture
  // allreduce() / barrier() really meet the other ranks (false for the
  // loopback, whose members share one host thread: its group agrees instead)
  virtual bool collective() const { return true; }
  // a graph with this transport's exchanges captured in it was launched on `stream`
  // (failure detection tracks the replay as a whole)
  virtual void graph_launched(hipStream_t /*stream*/) {}
  // true if exchange() moves data (size > 1, or a 1-rank periodic rehearsal)
  virtual bool exchanges() const { return size() > 1; }
  // Failure detection: raise if the fabric reported an asynchronous error
  // (RCCL: ncclCommGetAsyncError). Polled at every synchronisation point.
  virtual void check() {}
  // Two-phase cycles (transports whose ranks share one process, e.g. the
  // loopback): every rank post()s the field its cycle is writing and the
  // event that marks that field's boundary bands written BEFORE any rank's
  // exchange() of the same cycle is enqueued (LoopbackGroup drives this
  // order). Fabrics with their own rendezvous (RCCL) ignore it.
  virtual void post(void* /*field*/, const SlabLayout& /*L*/, hipEvent_t /*bands_ready*/) {}
  // Fail fast: abort the fabric (RCCL: ncclCommAbort) so that every blocked
  // operation of this rank returns, and make check() raise `reason`. Called by
  // the transport's own watchdog (hang / async error) or by a driver whose
  // other rank failed. Thread-safe, idempotent.
  virtual void abort(const std::string& /*reason*/) {}
  virtual bool aborted() const { return false; }
  // I/O phase (serial per-rank output turns, checkpoint writes, restart
  // reads): barriers / all-reduces issued while it is on may wait on a peer's
  // host I/O for long; failure detection does not treat them as a hung fabric
  // (RCCL: not tracked by the watchdog; host hubs: no barrier timeout).
  // Nested on/off pairs; every rank brackets the same phase.
  virtual void io_phase(bool /*on*/) {}
  // The solver's two field buffers (allocation bases, layout L): transports
  // that map their peers' fields once (IPC) do it here. Collective.
  virtual void attach(void* /*buf0*/, void* /*buf1*/, const SlabLayout& /*L*/, DType /*dt*/) {}
  // Bytes to allocate for a field buffer of `bytes` (the solver's two
  // fields): a transport that exports them to its peers may need more (IPC).
  virtual size_t field_alloc_bytes(size_t bytes) const { return bytes; }
  // What the fabric itself reports about this rank — the proof that a
  // multi-GPU run really put N ranks on N devices (the reference prints
  // "MPI rank r using GPU d", fortran/hip/heat.F90:125). kind: 0 host / self,
  // 1 RCCL (ncclCommCount / ncclCommUserRank / ncclCommCuDevice), 2 IPC (its
  // rank / size and the device it mapped its peers on); device -1: none.
  struct FabricInfo {
    int32_t kind, nranks, rank, device;
  };
  virtual FabricInfo fabric_info() { return {0, size(), rank(), -1}; }
};

// RAII bracket of Transport::io_phase.
struct IoPhase {
  Transport& t;
  explicit IoPhase(Transport& tr) : t(tr) { t.io_phase(true); }
  ~IoPhase() { t.io_phase(false); }
  IoPhase(const IoPhase&) = delete;
  IoPhase& operator=(const IoPhase&) = delete;
};

// The messages of one halo exchange, shared by every transport (RCCL sends
// and receives exactly these; the loopback copies them): k whole padded rows
// per message, contiguous in the slab layout, so no pack / unpack.
//   to / from rank-1: send rows [0, k),          receive into [-k, 0)
//   to / from rank+1: send rows [nrows-k, nrows), receive into [nrows, nrows+k)
// (the reference's two MPI_Sendrecv per step, fortran/hip/heat.F90:212-213)
struct HaloMsg {
  int peer;
  int64_t send_row, recv_row;
};
inline int halo_msgs(int rank, int size, const SlabLayout& L, int64_t k, HaloMsg out[2]) {
  int n = 0;
  if (rank > 0) out[n++] = HaloMsg{rank - 1, 0, -k};
  if (rank < size - 1) out[n++] = HaloMsg{rank + 1, L.nrows - k, L.nrows};
  return n;
}
inline size_t halo_row_bytes(const SlabLayout& L, int64_t row, size_t es) {
  return (size_t)((row + L.halo) * L.pitch) * es;
}
inline size_t halo_msg_bytes(const SlabLayout& L, int64_t k, size_t es) { return (size_t)(k * L.pitch) * es; }

std::shared_ptr<Transport> make_self_transport();
// P ranks of one process (one device, or host memory): halos move by
// device-to-device copies on the receiving rank's exchange stream, ordered by
// events against the neighbours' band kernels (transport.cpp). make_loopback_
// transports returns the P member transports of one group.
std::vector<std::shared_ptr<Transport>> make_loopback_transports(int nranks);
// P ranks as host threads of one process, host-memory fields (CPU backend):
// barrier-synchronised zero-copy row exchange, fixed-order all-reduce;
// barriers time out (HEAT2D_COMM_TIMEOUT) and abort() wakes every waiter.
std::vector<std::shared_ptr<Transport>> make_thread_transports(int nranks);
// P ranks as threads of one process with device fields, no RCCL: halos pulled
// by device-to-device copies out of the neighbours' fields (peer access between
// GPUs), ordered by events + host-side waits (transport.cpp PeerTransport).
std::vector<std::shared_ptr<Transport>> make_peer_transports(int nranks);
// RCCL over xGMI. `uid` = 128-byte ncclUniqueId produced by rccl_unique_id()
// on rank 0 and broadcast out of band (torch.distributed store, file, or a
// shared variable for thread-per-GPU).
std::shared_ptr<Transport> make_rccl_transport(const void* uid, int rank, int size, int device);
void rccl_unique_id(void* out128);
// 1-rank RCCL communicator whose exchange sends the slab's boundary rows to
// ITSELF (periodic wrap) — a performance rehearsal of the multi-GPU schedule
// (bands + RCCL kernels + CU-masked interior) on one GPU. Not for physics:
// it overwrites the Dirichlet frame rows.
std::shared_ptr<Transport> make_rccl_loop_transport(int device);
// Host callbacks (Python / gloo, tests). Buffers passed are host pointers to
// packed rows (k*ncols elements): send_lo/send_hi may be null at domain ends.
struct CallbackOps {
  void* ctx;
  int (*exchange)(void* ctx, void* send_lo, void* send_hi, void* recv_lo, void* recv_hi,
                  int64_t count, int32_t dtype);
  int (*allreduce)(void* ctx, double* vals, int32_t n, int32_t op);
  int (*barrier)(void* ctx);
};
std::shared_ptr<Transport> make_callback_transport(const CallbackOps& ops, int rank, int size);
// Process-per-GPU (or processes sharing a GPU) without RCCL: neighbours'
// fields mapped once via hipIpc handles, halos pulled by device copies,
// ordered by stream-side counters in host-shared memory (ipc_transport.cpp);
// capturable into hipGraphs. Host collectives through these callbacks
// (Python: torch.distributed gloo). Collective construction-free: the handle
// exchange happens in attach() (Solver constructor, every rank).
struct IpcOps {
  void* ctx;
  int (*allgather)(void* ctx, const void* mine, void* all, int64_t bytes);
  int (*allreduce)(void* ctx, double* vals, int32_t n, int32_t op);
  int (*barrier)(void* ctx);
};
std::shared_ptr<Transport> make_ipc_transport(const IpcOps& ops, int rank, int size, int device);
// 1-rank IPC transport exchanging the slab's boundary rows with itself
// (periodic wrap, like make_rccl_loop_transport): a rehearsal of one rank's
// IPC cycle on one GPU. Not physics (it overwrites the frame rows).
std::shared_ptr<Transport> make_ipc_loop_transport(int device);

// ---------------------------------------------------------------- CPU twins

namespace cpu {
void tb(DType dt, const void* src, void* dst, const SlabLayout& L, int64_t row_begin,
        int64_t row_end, int k, double r, int arith = 0);
void init(DType dt, void* field, const SlabLayout& L, const kern::IcParams& ic,
          const double* xcoord, const double* ycoord);
void stats(DType dt, const void* field, const void* other, const SlabLayout& L, double out[6]);
void pack_rows(DType dt, const void* field, const SlabLayout& L, int64_t row, int64_t nrows, void* buf);
void unpack_rows(DType dt, void* field, const SlabLayout& L, int64_t row, int64_t nrows, const void* buf);
int num_threads();
}  // namespace cpu

// ---------------------------------------------------------------- solver

// Cycle schedules (runtime/schedule.cpp): how n steps are cut into HBM passes
// of depth <= kmax from per-depth cycle costs (ms; < 0: unusable depth).
// The exact schedule minimising the summed cost (unbounded-knapsack DP;
// ties: fewer cycles, deeper first), deepest cycles first; empty if n cannot be
// reached. *total = its cost (or -1).
std::vector<int> dp_schedule(int64_t n, int kmax, const std::function<double(int)>& cost, double* total = nullptr);
// Balanced candidates (depths b and b + 1), one per base depth b, whose cost is
// within tol (relative) of the best of them, best first, at most m: (cost, schedule).
std::vector<std::pair<double, std::vector<int>>> near_schedules(int64_t n, int kmax, const std::function<double(int)>& cost,
                                                                 double tol, int m);
struct ScheduleSearchOptions {
  double stop_ratio = 1.25;    // prescan stops once the per-step cost is this much worse than the best
  double prescan_tol = 0.20;   // depths of the prescan schedules within this of the best are tuned ...
  int prescan_bases = 4;       // ... at most this many base depths
  int64_t walk_min_cycles = 8;  // runs of at least this many cycles walk beyond the tuned depths
  int walk_patience = 2;       // a walk ends after this many tunings in a row that did not lower the cost
  double walk_tol = 0.08;      // ... and whose per-step cost was more than this much above the best's
  double near_tol = 0.03;      // near ties returned for timing
  int near_max = 3;
};
struct ScheduleSearch {
  std::vector<int> best;   // the chosen schedule (deepest cycles first), empty if none
  double cost = -1.0;      // its summed tuned cost (ms)
  std::vector<std::pair<double, std::vector<int>>> near;  // best first, then tuned near ties
  std::vector<int> prescanned, tuned;                     // depths measured, in order
};
// The measured-schedule search of Solver::prepare (stages in schedule.cpp):
// prescan(k) = default-plan cycle time, tune(k) = autotuned cycle time, each
// called at most once per depth, in a deterministic order given their values
// (the solver passes max-over-ranks measurements: every rank searches alike).
ScheduleSearch search_schedule(int64_t n, int kmax, const std::function<double(int)>& prescan,
                               const std::function<double(int)>& tune, const ScheduleSearchOptions& o = {});
// Whether slabs of this decomposition get autotuned split plans and measured
// cycle schedules (SolverConfig::autotune, -1 = auto). A function of the
// GLOBAL problem only — the smallest slab (n_rows / P rows) decides — so every
// rank takes the same branch of prepare()'s collectives (uneven slabs that
// straddle the 2^24-point threshold, e.g. 5793^2 on 2 ranks, would otherwise
// split into ranks that all-reduce and ranks that do not).
bool autotune_slabs(int64_t n_rows, int64_t n_cols, int nranks, int autotune);
// Exchange depth after cycle i of a cycle sequence: the depth of the cycle that
// follows (the ghost rows it reads); after the last one, `next` (the depth
// the caller expects next, e.g. the sequence's own first depth when step(n)
// repeats).
inline int exchange_depth(const std::vector<int>& seq, size_t i, int next) {
  return i + 1 < seq.size() ? seq[i + 1] : next;
}

// The slab layout a Solver of config `cfg` uses on `rank` of `nranks` (uneven
// decompose() slabs, or the 1-rank middle-slab rehearsal), ghost bands of
// cfg.halo (0: kDefaultHalo) rows, pitched columns.
SlabLayout solver_layout(const SolverConfig& cfg, int rank, int nranks);
// Device bytes that Solver allocates for its state: both pitched fields with
// their ghost bands (field_bytes) plus the statistics / partials / item-queue
// workspaces (work_bytes; HIP backend) — exactly the constructor's hipMallocs
// (tests/test_memory_plan.py compares them with hipMemGetInfo). Not counted:
// the transport's own buffers and the runtime (the planner's reserve).
struct Footprint {
  int64_t field_bytes, work_bytes, total_bytes;
};
Footprint solver_footprint(const SolverConfig& cfg, int rank, int nranks);
// Memory-fit planner: the largest n such that an n x n grid of `dtype` on
// `nranks` ranks fits budget_bytes per GPU (the largest slab, rank 0's,
// decides). The reference sizes nothing: its grid is input.dat's n, with a
// whole-field host mirror (fortran/hip/heat.F90:161-176); here the IC is made
// on the device, so only the two device fields count.
int64_t plan_max_grid(int dtype, int nranks, int64_t budget_bytes, int64_t halo = 0);

class Solver {
 public:
  Solver(const SolverConfig& cfg, std::shared_ptr<Transport> tr, hipStream_t external_stream = nullptr);
  ~Solver();
  Solver(const Solver&) = delete;
  Solver& operator=(const Solver&) = delete;

  // IC on the device. xg: n_rows+2 frame-inclusive global x coordinates,
  // yg: n_cols+2 y coordinates. Ghost rows come from the global IC (no exchange).
  void init(const kern::IcParams& ic, const double* xg, const double* yg);
  // Advance n time steps (asynchronous on the HIP backend).
  void step(int64_t n);
  // Plan (and autotune, if enabled) every cycle depth a step(n) will use, so
  // that no planning happens inside a timed step(n). On slabs whose split
  // plans are autotuned it also picks step(n)'s cycle schedule by
  // measurement: the number of cycles c (depths balanced within c) with the
  // smallest sum of measured cycle times — the max over ranks, so every rank
  // runs the same schedule. E.g. 20 steps at 32768^2 fp64: one depth-20 pass
  // (6.4 ms) instead of two depth-10 passes (7.6 ms).
  void prepare(int64_t n);
  // The measured schedule step(n) will run (nullptr: balanced cycles of
  // pref_depth()).
  const std::vector<int>* schedule(int64_t n) const;
  // whether step(n) replays its schedule as one captured graph (prepare(n)
  // decides: short-cycle schedules only, replay_schedule)
  bool schedule_replayed(int64_t n) const {
    auto it = sched_replay_.find(n);
    return it != sched_replay_.end() && it->second;
  }
  // depth of the balanced cycles when no measured schedule applies (the
  // steady-state best: fp64 14, fp32 16 unless --tb is given)
  int pref_depth() const { return k_pref_; }
  void synchronize();
  // Global statistics over all ranks: sum, sum_sq, min, max of the current
  // field (a separate pass over it); residual = true adds sum (T_n - T_{n-1})^2
  // and max |T_n - T_{n-1}| when the last cycle had depth 1 (the other buffer
  // then holds T_{n-1}), else NaN — use step_stats for a residual at any depth.
  void stats(double out[6], bool residual);
  // step(n), with the statistics of T_n and its ONE-STEP residual T_n - T_{n-1}
  // (layout of stats()) fused into the last cycle's stencil launch — no extra
  // pass over the field (HIP engine; the CPU twin, copy-swap and jit modes run
  // n-1 steps, one step, and stats(residual)). Reduced over ranks.
  void step_stats(int64_t n, double out[6]);
  // Owned region <-> host (rows x n_cols, leading dimension ld elements).
  void download(void* host, int64_t ld);
  void upload(const void* host, int64_t ld);  // followed by a halo exchange
  // Any rectangle of the current buffer (local rows [r0,r1), cols [c0,c1),
  // ghost/frame included) -> host.
  void download_region(int64_t r0, int64_t r1, int64_t c0, int64_t c1, void* host, int64_t ld);
  // This rank's current field, local rows [r0, r0 + nrows), against `other`'s
  // current field, local rows [other_r0, other_r0 + nrows) (same device, same
  // dtype and width; e.g. an independent engine's run of the same problem):
  // out = {max |a - b| (NaN if any), elements whose bit patterns differ}.
  // Local to this rank (callers reduce over ranks); synchronises both solvers.
  void compare(Solver& other, int64_t r0, int64_t nrows, int64_t other_r0, double out[2]);

  // Phase API. One cycle of depth k = cycle_launch(k, x) (kernels, the event
  // that marks the bands written, Transport::post) then cycle_finish() (halo
  // exchange of x rows of the new field, buffer swap). step() runs the two back
  // to back; LoopbackGroup runs every member's launch before any member's finish.
  // x = the depth of the NEXT cycle (the ghost rows it will read; 0: k): the
  // exchange moves x rows, and the boundary bands are max(k, x) rows — not the
  // largest depth the halo allows. The current buffer must hold >= k valid
  // ghost rows (ghost_rows(); topup() first otherwise).
  void cycle_launch(int k, int x = 0);
  void cycle_finish();
  void cycle_compute(int k);   // whole-slab compute cur -> nxt (no exchange)
  void cycle_swap();
  void exchange_post();        // Transport::post of the current buffer (two-phase transports)
  void exchange_now(int k = 0);  // exchange k (0: band) halo rows of the current buffer on the compute stream
  // Rows of the current buffer's ghost bands that hold valid neighbour data
  // (band() after init / upload; the last exchange's depth after a cycle).
  int ghost_rows() const { return ghost_; }
  // Make ghost_rows() >= k with one blocking exchange of k rows (collective:
  // every rank tops up at the same point; a no-op where nothing is exchanged).
  void topup(int k);
  bool needs_topup(int k) const { return tr_->exchanges() && ghost_ < k; }
  // The cycle depths step(n) will run from the current state (measured
  // schedule, graph pairs, balanced cycles), in order.
  std::vector<int> step_cycles(int64_t n) const;
  // Halo rows each cycle exchanged since the last reset (sum over cycles).
  int64_t halo_rows_exchanged(bool reset);
  void upload_owned(const void* host, int64_t ld);  // upload() without the halo exchange
  // Cycles launched by step() since the last reset, by depth: hist[k] for
  // k = 0..kMaxTB (graph replays count their two cycles each).
  void cycle_hist(int64_t out[kMaxTB + 1], bool reset);

  const SlabLayout& layout() const { return L_; }
  const SolverConfig& config() const { return cfg_; }
  DType dtype() const { return (DType)cfg_.dtype; }
  void* field() const { return buf_[cur_]; }
  void* other_field() const { return buf_[cur_ ^ 1]; }
  int64_t steps_done() const { return steps_; }
  int rank() const { return tr_->rank(); }
  int size() const { return tr_->size(); }
  hipStream_t stream() const { return s_compute_; }
  Transport& transport() { return *tr_; }
  int64_t band() const { return band_; }
  // Split plan in use for depth k (planned / autotuned on first use).
  const kern::SplitPlan& plan_for(int k) { return split_plan(k); }
  float tuned_ms(int k) const { return k >= 0 && k <= kMaxTB ? tuned_ms_[k] : 0.f; }
  // split plans planned so far (each a first use of a depth; autotuned on big slabs)
  int64_t plans_made() const { return plans_made_; }
  // plans and schedules taken from the persistent plan cache (plan_cache.hpp)
  int64_t plan_cache_hits() const { return plan_cache_hits_; }
  // origin of the depth-k split plan: -1 not planned, 0 planned (no autotune),
  // 1 autotuned here, 2 taken from the plan cache (re-validated)
  int plan_origin(int k) const { return k >= 1 && k <= kMaxTB ? plan_origin_[k] : -1; }
  // depths autotuned in this process and candidate plans screened for them
  int64_t depths_tuned() const {
    int64_t n = 0;
    for (int k = 1; k <= kMaxTB; ++k) n += plan_origin_[k] == 1;
    return n;
  }
  int64_t tune_trials() const { return tune_trials_; }
  int spare_waves() const;
  // Phase timers (hipEvents on the GPU timeline) for every cycle while
  // enabled: [main ms, edge ms, exchange ms, whole-cycle ms (serial schedule),
  // cycles]. phase_times() synchronises, sums the recorded cycles and resets.
  void set_timing(bool on);
  void phase_times(double out[5]);

 private:
  void launch_overlap(int k, int64_t B);
  void launch_serial(int k);
  void launch_stats_cycle(int k);
  void reduce_global(const double loc[6], double out[6]);
  const kern::SplitPlan& split_plan(int k);
  // depth-k plan with boundary bands of B >= k rows: split_plan(k)'s choice
  // (order, ring, interior bands) re-cut for the wider bands
  const kern::SplitPlan& split_plan_banded(int k, int64_t B);
  void autotune_split(int k);
  // exposed-exchange estimate added to a candidate's trial time (exchanging slabs)
  float exchange_penalty(const kern::SplitPlan& c, float trial_ms) const;
  void cycle_copy_swap();
  void launch_tb(const void* src, void* dst, int64_t rb, int64_t re, int k);
  void exchange_on(void* field, int64_t k, hipStream_t s);
  // every rank must hold the same value (cycle sequence, exchange depths):
  // all-reduced and compared, a mismatch fails naming each rank's value
  void agree(uint64_t h, const std::string& what);
  uint64_t sequence_hash(int64_t n) const;
  struct CycleRun {
    int k;
    int64_t pairs;  // > 0: `pairs` replays of the two-cycle depth-k graph
  };
  std::vector<CycleRun> step_runs(int64_t n, int par) const;
  bool pair_graphs() const;
  void run_graph_cycles(int64_t npairs);
  void ensure_pair_graph();
  bool measured_schedules() const;
  void trial_cycle(const kern::SplitPlan& c);
  bool schedule_graphs() const;
  bool replay_schedule(int64_t n);
  void capture_schedule(int64_t n);
  float time_trial_schedule(const std::vector<int>& sc, int reps = 1);  // ms: the fastest of reps graph replays of sc
  float time_trial_eager(const std::vector<int>& sc, int reps);  // ms: the fastest of reps eager launches of sc
  void prepare_plans(int64_t n);  // prepare()'s planning / autotune / measured schedule (HIP split engine)
  float time_plan(const kern::SplitPlan& c, int kTimed);  // steady-state ms per trial cycle
  std::string cache_ctx() const;   // plan-cache key of this slab (plan_cache.hpp)
  std::string sched_ctx() const;   // ... of the decomposition's schedules
  bool cached_split(int k);        // plan of depth k from the cache, re-validated
  bool cached_schedule(int64_t n); // measured schedule of n steps from the cache (collective)
  void run_schedule_graph(int64_t n);
  float depth_ms(int k);
  float prescan_ms(int k);  // default-plan cycle time of depth k, max over ranks (schedule prescan)
  ScheduleSearch choose_schedule(int64_t n);

  SolverConfig cfg_;
  std::shared_ptr<Transport> tr_;
  SlabLayout L_{};
  bool hip_ = true;
  void* buf_[2] = {nullptr, nullptr};
  int cur_ = 0;
  int64_t steps_ = 0;
  int64_t band_ = 0;     // largest boundary band / halo exchange depth (= K)
  int ghost_ = 0;        // valid ghost rows of buf_[cur_] (see ghost_rows)
  int pend_x_ = 0;       // exchange depth of the pending cycle
  int last_x_[2] = {0, 0};  // rows of buf_[b] its last exchange moved (peers may still be pulling them)
  int64_t halo_rows_ = 0;  // rows exchanged per side, summed over cycles (metrics)
  std::map<std::pair<int, int64_t>, kern::SplitPlan> banded_;  // split_plan_banded cache
  hipStream_t s_compute_ = nullptr, s_comm_ = nullptr;
  bool own_streams_ = false;
  bool first_cycle_ = false;  // the next launch_overlap is a step() call's first cycle (lead_first)
  hipEvent_t ev_bnd_ = nullptr, ev_comm_ = nullptr, ev_int_ = nullptr;
  // an edge rank's first-cycle frame-side band (cycle_finish): its own event,
  // so ev_bnd_ — which receiver-driven transports wait on after post() — keeps
  // marking only the bands the exchange sends
  hipEvent_t ev_frame_ = nullptr;
  // fork / join of every stream capture (pair graph, measured schedules,
  // schedule trials): created once and destroyed after the streams, so no
  // event a capture recorded is freed while a stream may still name it
  hipEvent_t ev_fork_ = nullptr, ev_join_ = nullptr;
  double* d_work_ = nullptr;   // stats workspace + 6 results
  bool timing_ = false;
  struct PhaseEvents {
    hipEvent_t ev[6];  // main begin/end, edge begin/end, exchange begin/end
    int kind;          // 0: split cycle, 1: serial cycle (ev[0..1] only)
  };
  std::vector<PhaseEvents> phase_ev_;   // recorded, not yet summed
  std::vector<PhaseEvents> phase_pool_;  // reusable
  double phase_acc_[5] = {};
  PhaseEvents* phase_begin(int kind);
  // the launched, not yet finished cycle (cycle_launch -> cycle_finish)
  enum class Pending { None, Serial, Concurrent, EdgeFirst };
  Pending pend_ = Pending::None;
  int pend_frame_ = -1;  // edge-rank lead cycle: the frame-side band rect cycle_finish launches after the exchange
  int64_t pend_frame_b_ = 0;  // ... of the plan split_plan_banded(pend_k_, pend_frame_b_)
  int pend_k_ = 0;
  int64_t pend_pe_ = -1;  // index into phase_ev_ (timing) or -1
  int64_t hist_[kMaxTB + 1] = {};
  int k_pref_ = 1;
  int last_k_ = 0;            // depth of the last finished cycle
  bool stats_next_ = false;   // the next cycle_launch is the fused-statistics cycle
  double* d_part_ = nullptr;  // fused statistics: per-wave partials
  std::map<int64_t, std::vector<int>> sched_;  // measured schedules by step count
  std::map<int64_t, bool> sched_replay_;       // step(n) replays its schedule as a graph
  // use_graph + a capturable transport: each measured schedule captured whole
  // (both streams), keyed by (steps, starting buffer parity)
  std::map<std::pair<int64_t, int>, hipGraphExec_t> sched_graph_;
  float depth_ms_[kMaxTB + 1] = {};            // cycle ms per depth, max over ranks (schedule search)
  float pre_ms_[kMaxTB + 1] = {};              // default-plan cycle ms per depth, max over ranks (prescan)
  int64_t tune_trials_ = 0;                    // candidate plans the autotuner screened
  int compute_cus_ = 0;  // CUs of the (possibly CU-masked) compute stream; 0 = all
  kern::SplitPlan split_[kMaxTB + 1] = {};  // per temporal depth (k == 0: not planned yet)
  float tuned_ms_[kMaxTB + 1] = {};           // autotuned cycle time (ms), 0 if not tuned
  int64_t plans_made_ = 0;
  int64_t plan_cache_hits_ = 0;
  int plan_origin_[kMaxTB + 1];           // plan_origin(), initialised to -1
  uint32_t* d_queue_ = nullptr;           // dynamic item queue of the main launches (SplitPlan::pair bit 1)
  hipEvent_t ev_t0_ = nullptr, ev_t1_ = nullptr;  // time_plan
  hipGraphExec_t graph_exec_ = nullptr;  // two cycles (A->B->A) at depth K
  int graph_k_ = 0;
  std::vector<char> host_stage_;  // CPU-backend / callback staging
  std::unique_ptr<JitStencil> jit_;  // engine 1
};

// P slabs of one domain on ONE device (or host), each a full Solver with its
// own compute / comm streams, split plans and autotuner, exchanging halos
// through the loopback transport (the same messages RCCL moves): the whole
// multi-rank schedule — overlapped split cycles in either order, balanced
// depths, the event protocol across streams — runs with real exchanges on one
// GPU and must be bitwise identical to P = 1.
class LoopbackGroup {
 public:
  LoopbackGroup(const SolverConfig& cfg, int nranks);
  ~LoopbackGroup();
  void init(const kern::IcParams& ic, const double* xg, const double* yg);
  void step(int64_t n);
  void synchronize();
  void download(void* host, int64_t ld);  // whole global owned region
  void upload(const void* host, int64_t ld);  // whole global owned region, then a halo exchange
  int nranks() const { return (int)members_.size(); }
  Solver& member(int i) { return *members_[i]; }

 private:
  std::vector<std::unique_ptr<Solver>> members_;
};

}  // namespace heat2d
