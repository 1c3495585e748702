// Slab solver: the time loop of fortran/hip/heat.F90:232-254 (heat_eqn) and
// fortran/mpi+cuda/heat.F90:197-223, re-designed for MI355X.
//
// Reference, per step: full-field D2D copy; stencil kernel; device sync;
// pack; sync; 2 D2H; 2 blocking MPI_Sendrecv; 2 H2D; unpack (+sync) — all
// serialised on the null stream.
//
// Here, per cycle of k <= K steps (one HBM pass), src -> dst (ping-pong, no
// copy), split into two concurrent launches (kern::plan_split):
//   MAIN (compute stream): rows [B, n-B) x the strips that reach no frame
//        column — the lean interior-only kernel on most wave slots;
//   EDGE (comm stream): the two B-row boundary bands and the frame-column
//        strips, cut into short items, on the remaining slots; then (P > 1)
//        the RCCL grouped send/recv of the B band rows.
//   compute: wait(ev_bnd: EDGE c-1) -> MAIN c -> record(ev_int)
//   comm:    wait(ev_int: MAIN c-1) -> EDGE c -> record(ev_bnd) -> exchange
//            -> record(ev_comm)
// MAIN never reads ghost rows (only owned rows [0, n)), so it never waits for
// an exchange: MAIN launches run back to back while EDGE and the halo exchange
// of the same cycle proceed beside them — also at P = 1, where the split keeps
// the frame-handling code out of the main kernel (its registers and its tail).
// Ordering is carried entirely by events; the host never synchronises inside
// the loop. Hazards covered (cycle c, src_c = dst_{c-1}):
//   * MAIN c reads src_c cells written by EDGE c-1, and overwrites dst_c cells
//     that EDGE c-1 read                                     -> wait ev_bnd
//   * EDGE c reads src_c cells written by MAIN c-1, and overwrites dst_c
//     cells that MAIN c-1 read                               -> wait ev_int
//   * EDGE c reads ghost rows received by exchange c-1       -> comm-stream order
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <thread>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "heat2d/plan_cache.hpp"
#include "heat2d/runtime.hpp"
#include "heat2d/watchdog.hpp"

#include <rocprofiler-sdk-roctx/roctx.h>

namespace heat2d {

#define H2D_HIP(expr)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess) fail(__FILE__, __LINE__, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

namespace {
void* host_alloc(size_t bytes) {
  const size_t a = 256;
  void* p = std::aligned_alloc(a, (bytes + a - 1) / a * a);
  HEAT2D_REQUIRE(p != nullptr, "host allocation failed");
  return p;
}
}  // namespace

SlabLayout solver_layout(const SolverConfig& cfg, int rank, int nranks) {
  const int64_t halo = cfg.halo > 0 ? cfg.halo : kDefaultHalo;
  if (cfg.slab_rows_global > 0) {  // 1-rank rehearsal of a middle slab of a bigger grid
    HEAT2D_REQUIRE(nranks == 1, "slab_rows_global: single-rank rehearsal only");
    HEAT2D_REQUIRE(cfg.slab_row0 >= 0 && cfg.slab_row0 + cfg.n_rows <= cfg.slab_rows_global, "slab outside the grid");
    return make_layout(cfg.n_rows, cfg.n_cols, halo, cfg.slab_row0, cfg.slab_rows_global);
  }
  const SlabRange sr = decompose(cfg.n_rows, nranks, rank, cfg.edge_shift);
  return make_layout(sr.nrows, cfg.n_cols, halo, sr.row0, cfg.n_rows);
}

Footprint solver_footprint(const SolverConfig& cfg, int rank, int nranks) {
  const SlabLayout L = solver_layout(cfg, rank, nranks);
  Footprint f{};
  f.field_bytes = 2 * L.elems() * (int64_t)dtype_size((DType)cfg.dtype);
  if (cfg.backend == (int32_t)Backend::Hip)
    f.work_bytes = (kern::stats_work_elems() + 8) * 8 + 6 * kern::max_stats_waves() * 8 + 2 * 4;
  f.total_bytes = f.field_bytes + f.work_bytes;
  return f;
}

int64_t plan_max_grid(int dtype, int nranks, int64_t budget_bytes, int64_t halo) {
  HEAT2D_REQUIRE(nranks >= 1 && budget_bytes > 0, "plan_max_grid needs nranks >= 1 and a positive budget");
  SolverConfig c{};
  c.dtype = dtype;
  c.backend = (int32_t)Backend::Hip;
  c.halo = halo;
  // the largest slab is rank 0's (decompose() gives the remainder to the first ranks)
  auto fits = [&](int64_t n) {
    c.n_rows = c.n_cols = n;
    return solver_footprint(c, 0, nranks).total_bytes <= budget_bytes;
  };
  int64_t lo = 0, hi = 1;
  while (fits(hi) && hi < (int64_t(1) << 31)) hi *= 2;  // the footprint grows with n
  while (hi - lo > 1) {
    const int64_t mid = lo + (hi - lo) / 2;
    (fits(mid) ? lo : hi) = mid;
  }
  HEAT2D_REQUIRE(lo >= nranks, "no grid of at least one row per rank fits the budget");
  return lo;
}

Solver::Solver(const SolverConfig& cfg, std::shared_ptr<Transport> tr, hipStream_t external_stream)
    : cfg_(cfg), tr_(std::move(tr)) {
  HEAT2D_REQUIRE(tr_ != nullptr, "transport required");
  HEAT2D_REQUIRE(cfg_.n_rows >= 1 && cfg_.n_cols >= 1, "empty grid");
  HEAT2D_REQUIRE(cfg_.dtype == 0 || cfg_.dtype == 1, "dtype must be 0 (fp32) or 1 (fp64)");
  hip_ = cfg_.backend == (int32_t)Backend::Hip;
  std::fill(plan_origin_, plan_origin_ + kMaxTB + 1, -1);
  const int P = tr_->size(), rank = tr_->rank();
  HEAT2D_REQUIRE(cfg_.n_rows >= P, "fewer rows than ranks");

  // tb <= 0: the measured best depth of the HIP engine (bench.py sweeps on
  // MI355X, profiles/README.md §11: fp64 14 — equal to 12 on a whole 32768²
  // grid, 3-6 % faster on the slabs of 2/4/8-rank runs — fp32 16 with the
  // packed fp32 march); 8 on the CPU twin.
  // tb <= 0 on the HIP engine: depths up to max_tb (fp64 24, fp32 20) are
  // available to the measured schedules of prepare(); the balanced fallback
  // uses the steady-state best.
  const bool tb_given = cfg_.tb > 0;
  const int tb_pref = hip_ ? (cfg_.dtype == 1 ? 14 : 16) : 8;
  const int tb_auto = hip_ ? max_tb(dtype()) : 8;
  int K = std::max(1, std::min<int>(tb_given ? cfg_.tb : tb_auto, max_tb(dtype())));
  if (cfg_.copy_swap) K = 1;
  HEAT2D_REQUIRE(cfg_.engine == 0 || cfg_.engine == 1, "engine must be 0 (temporal-blocked) or 1 (jit)");
  if (cfg_.arith < 0) {
    // auto: the contracted form when it is bitwise identical to the reference
    // rounding — r an exact power of two (sigma = 0.25 in every shipped
    // input.dat), where r*x is exact (normal range) — else the reference form
    int e = 0;
    cfg_.arith = (cfg_.r > 0 && std::frexp(cfg_.r, &e) == 0.5) ? 1 : 0;
  }
  HEAT2D_REQUIRE(cfg_.arith >= 0 && cfg_.arith <= 3,
                 "arith must be 0 (reference rounding), 1 (fma), 2 (jacobi, r = 1/4), 3 (fast) or -1 (auto)");
  HEAT2D_REQUIRE(cfg_.arith != 2 || cfg_.r == 0.25, "arith 2 (jacobi) needs r == 1/4 exactly (sigma = 0.25)");
  HEAT2D_REQUIRE(cfg_.arith != 3 || cfg_.r > 0, "arith 3 (fast) needs r > 0");
  if (cfg_.engine == 1) {
    HEAT2D_REQUIRE(hip_, "the jit engine runs on the HIP backend");
    HEAT2D_REQUIRE(!cfg_.copy_swap, "the jit engine has no copy-swap mode");
    K = 1;  // one step per launch, like the reference's JIT program
  }
  if (cfg_.arith == 3 && cfg_.r < 0.25) {
    // scaled levels carry T / r^s: keep r^K and max|T| / r^K well inside the
    // exponent range (fp32: r^K >= 2^-60; fp64: 2^-480), shallower passes else
    const double lim = cfg_.dtype == 0 ? -60.0 : -480.0;
    const int kmax = (int)std::floor(lim / std::log2(cfg_.r));
    K = std::max(1, std::min(K, kmax));
  }
  // every rank must own >= K rows so a neighbour's K ghost rows come from one rank
  K = (int)std::min<int64_t>(K, cfg_.n_rows / P);
  cfg_.tb = K;
  band_ = K;
  k_pref_ = tb_given ? K : std::min(K, tb_pref);
  HEAT2D_REQUIRE((cfg_.halo > 0 ? cfg_.halo : kDefaultHalo) >= K, "halo must be >= temporal depth");
  L_ = solver_layout(cfg_, rank, P);

  const size_t bytes = (size_t)L_.elems() * dtype_size(dtype());
  if (hip_) {
    if (cfg_.device >= 0) H2D_HIP(hipSetDevice(cfg_.device));
    else H2D_HIP(hipGetDevice(&cfg_.device));
    const size_t alloc = tr_->field_alloc_bytes(bytes);  // (IPC: see IpcTransport::field_alloc_bytes)
    for (int b = 0; b < 2; ++b) {
      if (cfg_.managed) H2D_HIP(hipMallocManaged(&buf_[b], alloc));
      else H2D_HIP(hipMalloc(&buf_[b], alloc));
    }
    // (solver_footprint() counts exactly these allocations: keep them in step)
    H2D_HIP(hipMalloc(reinterpret_cast<void**>(&d_work_), (size_t)(kern::stats_work_elems() + 8) * sizeof(double)));
    H2D_HIP(hipMalloc(reinterpret_cast<void**>(&d_part_), (size_t)(6 * kern::max_stats_waves()) * sizeof(double)));
    H2D_HIP(hipMalloc(reinterpret_cast<void**>(&d_queue_), 2 * sizeof(uint32_t)));
    H2D_HIP(hipMemset(d_queue_, 0, 2 * sizeof(uint32_t)));
    if (external_stream) {
      s_compute_ = s_comm_ = external_stream;
      cfg_.overlap = 0;
    } else {
      int ncu = 0;
      H2D_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, cfg_.device));
      const int want = cfg_.comm_cus;
      const bool ovl = tr_->exchanges() && cfg_.overlap;
      if (ovl && want > 0 && want < ncu) {
        // Hard reservation: `want` CUs, spread over the XCDs, out of the
        // compute stream's CU mask. Measured on MI355X (rehearsal, 4096 x 32768
        // fp64 slab, profiles/overlap_rehearsal.md): 8 masked CUs cost the
        // interior ~20 %, far more than 8/256 — kept as an option only.
        std::vector<uint32_t> mask((size_t)(ncu + 31) / 32, 0u);
        for (int i = 0; i < ncu; ++i) mask[(size_t)i / 32] |= 1u << (i % 32);
        for (int j = 0; j < want; ++j) {
          const int i = (int)((int64_t)j * ncu / want);
          mask[(size_t)i / 32] &= ~(1u << (i % 32));
        }
        H2D_HIP(hipExtStreamCreateWithCUMask(&s_compute_, (uint32_t)mask.size(), mask.data()));
        compute_cus_ = ncu - want;
      } else {
        // Soft reservation (default): no mask; the split plan sizes the
        // persistent interior grid to leave wave slots for the edge launch
        // and RCCL's workgroups (kern::plan_split).
        H2D_HIP(hipStreamCreateWithFlags(&s_compute_, hipStreamNonBlocking));
      }
      // (A high-priority comm stream did not get the band waves dispatched
      // first in steady-state cycles, nor change the small grid: profiles/r4/lead/, r4/m/.)
      H2D_HIP(hipStreamCreateWithFlags(&s_comm_, hipStreamNonBlocking));
      own_streams_ = true;
    }
    H2D_HIP(hipEventCreateWithFlags(&ev_bnd_, hipEventDisableTiming));
    H2D_HIP(hipEventCreateWithFlags(&ev_comm_, hipEventDisableTiming));
    H2D_HIP(hipEventCreateWithFlags(&ev_int_, hipEventDisableTiming));
    H2D_HIP(hipEventCreateWithFlags(&ev_frame_, hipEventDisableTiming));
    H2D_HIP(hipEventCreateWithFlags(&ev_fork_, hipEventDisableTiming));
    H2D_HIP(hipEventCreateWithFlags(&ev_join_, hipEventDisableTiming));
    H2D_HIP(hipEventRecord(ev_comm_, s_comm_));
    H2D_HIP(hipEventRecord(ev_bnd_, s_comm_));
    H2D_HIP(hipEventRecord(ev_int_, s_compute_));
    if (cfg_.engine == 1) {
      jit_.reset(new JitStencil(dtype(), L_, cfg_.r, cfg_.device, cfg_.arith));
      cfg_.overlap = 0;
      cfg_.use_graph = 0;
    }
  } else {
    for (int b = 0; b < 2; ++b) buf_[b] = host_alloc(bytes);
    cfg_.overlap = 0;
    cfg_.use_graph = 0;
  }
  tr_->attach(buf_[0], buf_[1], L_, dtype());
}

Solver::~Solver() {
  if (hip_) {
    (void)hipSetDevice(cfg_.device);
    if (s_compute_) (void)hipStreamSynchronize(s_compute_);
    if (s_comm_ && s_comm_ != s_compute_) (void)hipStreamSynchronize(s_comm_);
    if (graph_exec_) (void)hipGraphExecDestroy(graph_exec_);
    for (auto& g : sched_graph_) (void)hipGraphExecDestroy(g.second);
    for (auto& b : buf_)
      if (b) (void)hipFree(b);
    if (d_work_) (void)hipFree(d_work_);
    if (d_part_) (void)hipFree(d_part_);
    if (d_queue_) (void)hipFree(d_queue_);
    // the streams go before the events recorded on them (captures included)
    if (own_streams_) {
      (void)hipStreamDestroy(s_compute_);
      (void)hipStreamDestroy(s_comm_);
    }
    for (hipEvent_t e : {ev_bnd_, ev_comm_, ev_int_, ev_frame_, ev_fork_, ev_join_, ev_t0_, ev_t1_})
      if (e) (void)hipEventDestroy(e);
    for (auto* v : {&phase_ev_, &phase_pool_})
      for (auto& pe : *v)
        for (auto& e : pe.ev) (void)hipEventDestroy(e);
    (void)hipGetLastError();  // teardown errors must not surface as the next launch's
  } else {
    for (auto& b : buf_) std::free(b);
  }
}

void Solver::init(const kern::IcParams& ic, const double* xg, const double* yg) {
  // xg covers the whole grid's rows (frame-inclusive)
  const size_t nx = (size_t)(std::max(cfg_.n_rows, cfg_.slab_rows_global) + 2), ny = (size_t)(cfg_.n_cols + 2);
  if (hip_) {
    H2D_HIP(hipSetDevice(cfg_.device));
    double* d = nullptr;
    H2D_HIP(hipMalloc(reinterpret_cast<void**>(&d), (nx + ny) * sizeof(double)));
    H2D_HIP(hipMemcpyAsync(d, xg, nx * sizeof(double), hipMemcpyHostToDevice, s_compute_));
    H2D_HIP(hipMemcpyAsync(d + nx, yg, ny * sizeof(double), hipMemcpyHostToDevice, s_compute_));
    for (int b = 0; b < 2; ++b) kern::launch_init(dtype(), buf_[b], L_, ic, d, d + nx, s_compute_);
    H2D_HIP(hipStreamSynchronize(s_compute_));
    H2D_HIP(hipFree(d));
  } else {
    for (int b = 0; b < 2; ++b) cpu::init(dtype(), buf_[b], L_, ic, xg, yg);
  }
  // ghost rows are filled from the global IC directly: no exchange needed
  cur_ = 0;
  steps_ = 0;
  ghost_ = (int)band_;
  last_x_[0] = last_x_[1] = 0;
  last_k_ = 0;
}

void Solver::launch_tb(const void* src, void* dst, int64_t rb, int64_t re, int k) {
  if (re <= rb) return;
  if (hip_)
    kern::launch_tb(dtype(), src, dst, L_, rb, re, k, cfg_.r, s_compute_, cfg_.tile_rows, compute_cus_, cfg_.arith);
  else
    cpu::tb(dtype(), src, dst, L_, rb, re, k, cfg_.r, cfg_.arith);
}

void Solver::exchange_on(void* field, int64_t k, hipStream_t s) {
  if (!tr_->exchanges()) return;
  HEAT2D_REQUIRE(k >= 1 && k <= band_, "halo exchange depth outside [1, band]");
  tr_->exchange(field, L_, dtype(), k, s, hip_);
  halo_rows_ += k;
}

int64_t Solver::halo_rows_exchanged(bool reset) {
  const int64_t v = halo_rows_;
  if (reset) halo_rows_ = 0;
  return v;
}

void Solver::cycle_compute(int k) {
  if (jit_) {
    jit_->step(buf_[cur_], buf_[cur_ ^ 1], s_compute_);  // k == 1
    return;
  }
  launch_tb(buf_[cur_], buf_[cur_ ^ 1], 0, L_.nrows, k);
}

void Solver::cycle_swap() {
  cur_ ^= 1;
}

void Solver::exchange_post() {
  if (!tr_->exchanges()) return;
  if (hip_) H2D_HIP(hipEventRecord(ev_bnd_, s_compute_));
  tr_->post(buf_[cur_], L_, hip_ ? ev_bnd_ : nullptr);
}

void Solver::exchange_now(int k) {
  const int64_t d = k > 0 ? k : band_;
  exchange_on(buf_[cur_], d, s_compute_);
  ghost_ = (int)d;
  last_x_[cur_] = std::max<int>(last_x_[cur_], (int)d);
}

// One blocking exchange of k rows of the current buffer, between cycles: the
// previous cycle's kernels on both streams have finished (synchronize), so
// every band row sent is final, and the next cycle starts after the copies
// landed. Used where a cycle needs deeper ghost rows than the last exchange
// moved (a step(n) whose first depth exceeds the previous call's last
// exchange); prepare(n) does it outside timed regions.
void Solver::topup(int k) {
  if (!needs_topup(k)) return;
  HEAT2D_REQUIRE(k <= band_, "top-up deeper than the halo band");
  synchronize();
  exchange_post();
  exchange_now(k);
  synchronize();
}

void Solver::cycle_launch(int k, int x) {
  HEAT2D_REQUIRE(pend_ == Pending::None, "cycle_launch: previous cycle not finished");
  HEAT2D_REQUIRE(k >= 1 && k <= cfg_.tb, "cycle depth outside [1, tb]");
  if (x <= 0 || !tr_->exchanges()) x = k;
  HEAT2D_REQUIRE(x <= band_, "exchange depth outside [1, band]");
  HEAT2D_REQUIRE(!tr_->exchanges() || ghost_ >= k,
                 "cycle of depth " + std::to_string(k) + " on " + std::to_string(ghost_) +
                     " valid ghost rows (rank " + std::to_string(tr_->rank()) + "): topup() first");
  if (stats_next_ && hip_ && !jit_) {
    first_cycle_ = false;
    launch_stats_cycle(k);
  }
  // Boundary bands: the rows the exchange sends (x) must be written by the
  // band launch, and MAIN must not touch rows a receiver-driven transport
  // (loopback, peer, IPC pulls) may still be reading: the previous exchange
  // of this cycle's destination buffer moved last_x_ rows of it, and only the
  // band launch is ordered after that exchange's pulls (the concurrent order's
  // MAIN waits for the previous EDGE only).
  else if (cfg_.overlap && hip_) launch_overlap(k, std::max({k, x, last_x_[cur_ ^ 1]}));
  else launch_serial(k);
  stats_next_ = false;
  pend_k_ = k;
  pend_x_ = x;
}

// The fused-statistics cycle: one general launch over the whole slab on the
// compute stream, after the previous cycle's EDGE and exchange (ev_bnd /
// ev_comm), the per-wave partials reduced right behind it into the tail of
// d_work_; the exchange of its bands follows on the comm stream (overlap) or
// the compute stream (serial), as for an edge-first / serial cycle.
void Solver::launch_stats_cycle(int k) {
  roctxRangePushA("heat2d.cycle.stats");
  H2D_HIP(hipStreamWaitEvent(s_compute_, ev_bnd_, 0));
  H2D_HIP(hipStreamWaitEvent(s_compute_, ev_comm_, 0));
  kern::launch_tb_stats(dtype(), buf_[cur_], buf_[cur_ ^ 1], L_, k, cfg_.r, d_part_,
                        d_work_ + kern::stats_work_elems(), s_compute_, cfg_.arith);
  H2D_HIP(hipEventRecord(ev_bnd_, s_compute_));
  H2D_HIP(hipEventRecord(ev_int_, s_compute_));
  if (tr_->exchanges()) tr_->post(buf_[cur_ ^ 1], L_, ev_bnd_);
  pend_ = (cfg_.overlap && s_comm_ != s_compute_) ? Pending::EdgeFirst : Pending::Serial;
  pend_pe_ = -1;
}

void Solver::cycle_finish() {
  HEAT2D_REQUIRE(pend_ != Pending::None, "cycle_finish without cycle_launch");
  void* dst = buf_[cur_ ^ 1];
  PhaseEvents* pe = pend_pe_ >= 0 ? &phase_ev_[(size_t)pend_pe_] : nullptr;
  if (pend_ == Pending::Serial) {
    exchange_on(dst, pend_x_, s_compute_);
    if (pe) H2D_HIP(hipEventRecord(pe->ev[1], s_compute_));
  } else {
    // both split orders: the exchange of the new bands runs on the comm
    // stream (concurrent: right behind the EDGE launch there; edge-first:
    // behind the bands, which ran first on the compute stream)
    if (pend_ == Pending::EdgeFirst) H2D_HIP(hipStreamWaitEvent(s_comm_, ev_bnd_, 0));
    exchange_on(dst, pend_x_, s_comm_);
    if (pe) H2D_HIP(hipEventRecord(pe->ev[5], s_comm_));
    if (pend_frame_ >= 0) {  // the edge rank's frame-side band (launch_overlap), after the exchange
      kern::launch_edge_rect(dtype(), buf_[cur_], dst, L_, split_plan_banded(pend_k_, pend_frame_b_), pend_frame_, cfg_.r,
                             s_comm_, cfg_.arith);
      // the next cycle's compute-stream work waits for it (and so for the
      // exchange ahead of it); ev_bnd_, posted to the transport, is left alone
      H2D_HIP(hipEventRecord(ev_frame_, s_comm_));
      H2D_HIP(hipStreamWaitEvent(s_compute_, ev_frame_, 0));
      pend_frame_ = -1;
    }
    H2D_HIP(hipEventRecord(ev_comm_, s_comm_));
  }
  roctxRangePop();
  pend_ = Pending::None;
  pend_pe_ = -1;
  steps_ += pend_k_;
  hist_[pend_k_] += 1;
  last_k_ = pend_k_;
  ghost_ = pend_x_;
  if (tr_->exchanges()) last_x_[cur_ ^ 1] = pend_x_;
  cycle_swap();
}

void Solver::cycle_hist(int64_t out[kMaxTB + 1], bool reset) {
  for (int i = 0; i <= kMaxTB; ++i) out[i] = hist_[i];
  if (reset)
    for (auto& h : hist_) h = 0;
}

void Solver::launch_serial(int k) {
  roctxRangePushA("heat2d.cycle.serial");
  PhaseEvents* pe = (timing_ && hip_) ? phase_begin(1) : nullptr;
  if (pe) H2D_HIP(hipEventRecord(pe->ev[0], s_compute_));
  cycle_compute(k);
  if (pe) H2D_HIP(hipEventRecord(pe->ev[4], s_compute_));
  if (tr_->exchanges()) {
    if (hip_) H2D_HIP(hipEventRecord(ev_bnd_, s_compute_));
    tr_->post(buf_[cur_ ^ 1], L_, hip_ ? ev_bnd_ : nullptr);
  }
  pend_ = Pending::Serial;
  pend_pe_ = pe ? (int64_t)phase_ev_.size() - 1 : -1;
}

Solver::PhaseEvents* Solver::phase_begin(int kind) {
  if (phase_pool_.empty()) {
    PhaseEvents pe{};
    for (auto& e : pe.ev) H2D_HIP(hipEventCreate(&e));
    phase_pool_.push_back(pe);
  }
  phase_ev_.push_back(phase_pool_.back());
  phase_pool_.pop_back();
  phase_ev_.back().kind = kind;
  return &phase_ev_.back();
}

void Solver::set_timing(bool on) {
  if (!hip_) return;
  timing_ = on;
}

void Solver::phase_times(double out[5]) {
  if (hip_ && !phase_ev_.empty()) {
    synchronize();
    auto el = [](hipEvent_t a, hipEvent_t b) {
      float ms = 0.f;
      H2D_HIP(hipEventElapsedTime(&ms, a, b));
      return (double)ms;
    };
    for (auto& pe : phase_ev_) {
      if (pe.kind == 0) {
        phase_acc_[0] += el(pe.ev[0], pe.ev[1]);  // main (compute stream)
        phase_acc_[1] += el(pe.ev[2], pe.ev[3]);  // edge (comm stream, from its wait)
        phase_acc_[2] += el(pe.ev[3], pe.ev[5]);  // halo exchange
        // cycle: from the first record to the last (edge-first plans start with the bands)
        phase_acc_[3] += std::max({el(pe.ev[0], pe.ev[1]), el(pe.ev[2], pe.ev[5]), el(pe.ev[2], pe.ev[1])});
      } else {
        phase_acc_[0] += el(pe.ev[0], pe.ev[4]);  // compute
        phase_acc_[2] += el(pe.ev[4], pe.ev[1]);  // exchange
        phase_acc_[3] += el(pe.ev[0], pe.ev[1]);
      }
      phase_acc_[4] += 1.0;
      phase_pool_.push_back(pe);
    }
    phase_ev_.clear();
  }
  for (int i = 0; i < 5; ++i) out[i] = phase_acc_[i];
  for (double& v : phase_acc_) v = 0.0;
}

const kern::SplitPlan& Solver::split_plan(int k) {
  kern::SplitPlan& p = split_[k];
  if (p.k != k) {
    // room for RCCL's workgroups beside the two stencil launches when exchanging
    const int spare = spare_waves();
    // bands of k rows (split_plan_banded widens them when a deeper exchange follows)
    p = kern::plan_split(dtype(), L_, k, k, compute_cus_, spare, 0, 0, cfg_.arith);
    p.k = k;
    ++plans_made_;
    plan_origin_[k] = 0;
    if (p.valid && autotune_slabs(cfg_.n_rows, cfg_.n_cols, tr_->size(), cfg_.autotune)) {
      if (cached_split(k)) plan_origin_[k] = 2;
      else {
        autotune_split(k);
        plan_origin_[k] = 1;
      }
    }
    // HEAT2D_SPLIT_ORDER=edge-first | concurrent overrides the split's ordering (tests, A/B);
    // HEAT2D_SPLIT_ORDER=single forces one general launch per cycle (no exchange only)
    if (const char* env = std::getenv("HEAT2D_SPLIT_ORDER")) {
      const std::string o = env;
      if (o == "edge-first" && p.valid == 1) p.valid = 3;
      if (o == "concurrent" && p.valid == 3) p.valid = 1;
      if (o == "concurrent") p.flags &= ~kern::kPlanLead;
      if (o == "lead" && (p.valid == 1 || p.valid == 3) && tr_->exchanges()) {
        p.valid = 1;
        p.flags |= kern::kPlanLead;
      }
      if (o == "single" && !tr_->exchanges()) {
        p = kern::plan_single(dtype(), L_, k, compute_cus_, 0, 0, cfg_.arith);
        p.k = k;
      }
    }
    // HEAT2D_SEGMENTS=n / HEAT2D_BANDS=n re-plan the interior (or the single
    // launch) as n segment work items / n row bands, keeping the order and ring
    // (tests, A/B)
    const char* env_seg = std::getenv("HEAT2D_SEGMENTS");
    const char* env_bands = std::getenv("HEAT2D_BANDS");
    if (env_seg || env_bands) {
      const int64_t nseg = env_seg ? std::atoll(env_seg) : -std::atoll(env_bands);  // < 0: bands
      if (nseg != 0 && p.valid) {
        const int valid = p.valid, ring = p.ring;
        p = valid == 2 ? kern::plan_single(dtype(), L_, k, compute_cus_, ring, -nseg, cfg_.arith)
                       : kern::plan_split(dtype(), L_, k, k, compute_cus_, spare, ring, -nseg, cfg_.arith);
        if (p.valid) p.valid = valid;
        p.k = k;
      }
    }
    // HEAT2D_EDGE_BANDS=n: the boundary-band rects cut into n row bands each (tests, A/B)
    if (const char* e = std::getenv("HEAT2D_EDGE_BANDS"); e && std::atoll(e) > 0 && (p.valid == 1 || p.valid == 3))
      p = kern::with_edge_bands(dtype(), p, std::atoll(e), cfg_.arith);
    // HEAT2D_MAX_WAVES=n: at most n waves for the main launch (tests: several items per wave)
    if (const char* e = std::getenv("HEAT2D_MAX_WAVES"); e && std::atoll(e) > 0 && p.valid >= 1 && p.valid <= 3)
      p.main_waves = std::min<int64_t>(p.main_waves, std::atoll(e));
    // HEAT2D_DYNAMIC=1: the main launch takes its items from the dynamic queue (tests, A/B)
    if (const char* e = std::getenv("HEAT2D_DYNAMIC"); e && std::atoi(e) == 1 && p.valid >= 1 && p.valid <= 3)
      p.flags |= kern::kPlanDynamic;
  }
  return p;
}

const kern::SplitPlan& Solver::split_plan_banded(int k, int64_t B) {
  const kern::SplitPlan& base = split_plan(k);
  if (B <= k || !base.valid || base.valid == 2) return base;
  auto it = banded_.find({k, B});
  if (it != banded_.end()) return it->second;
  // the same choice (order, ring, interior bands / segments) over the interior
  // left between B-row bands; too thin for that: valid = 0 (serial cycle)
  kern::SplitPlan d = kern::plan_split(dtype(), L_, k, B, compute_cus_, spare_waves(), base.ring, base.main.nb,
                                       cfg_.arith);
  if (d.valid) {
    if (base.nedge > 0 && base.edge[0].nb > 1) d = kern::with_edge_bands(dtype(), d, base.edge[0].nb, cfg_.arith);
    d.flags = base.flags;
    d.valid = base.valid;
    d.main_waves = std::min<int64_t>(d.main_items, std::max<int64_t>(1, base.main_waves));
  }
  d.k = k;
  return banded_.emplace(std::make_pair(k, B), d).first->second;
}

// Time candidate split plans (ring 4/6 x MAIN band counts) in the steady
// state of the real loop — consecutive cycles on the real buffers, same
// stream/event protocol, no exchange — and keep the fastest. Every trial
// cycle reads the CURRENT buffer and writes the other one without swapping
// (the same kernels and traffic as the ping-pong loop; the timing does not
// depend on the values), so the solution is untouched and no backup copy is
// needed — the full-HBM grid (two fields ~ 240 GB) is tuned too. Measured on MI355X the cycle time at 32768^2 swings by up to ~25%
// between band counts of the same depth (DRAM page / channel locality of the
// waves marching in lockstep, and the item-per-wave tail), which no static
// rule captured; a single isolated cycle mispredicts the loop, hence the
// steady-state measurement (profiles/autotune.md).
// Wave slots the interior grid leaves free for RCCL's kernels when the slab
// exchanges halos (8: more cost the interior more than the bands gain,
// profiles/thin_slab.md §2).
int Solver::spare_waves() const {
  if (!tr_->exchanges()) return 0;
  return 8;
}

static int device_cus_of(int device) {
  int ncu = 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || ncu <= 0) ncu = 256;
  return ncu;
}

// Dynamic-queue candidates (HEAT2D_DYNAMIC=0 keeps them out of the autotuner;
// =1 forces the queue on plans with more items than waves). With 2 waves per
// SIMD the older wave issues first: on the headline's interior launch the
// first 1024 of 2048 equal waves end at 3.67 ms, the other 1024 at 5.43 ms,
// which then run alone on their SIMDs (profiles/r3/dyn/). A queue lets the
// early waves take more items: 32768^2 fp64 20 steps 4358 -> 4820 Gpts/s on
// one box.
static bool dynamic_candidates() {
  static const bool on = [] {
    const char* e = std::getenv("HEAT2D_DYNAMIC");
    return !e || std::atoi(e) != 0;
  }();
  return on;
}

// The first cycle of a step() call on an exchanging slab runs in the lead
// order whatever its plan's split order (HEAT2D_LEAD_FIRST=0: the plan's
// order): issued onto an idle GPU, the band launch gets its wave slots before
// the interior's, which follows without waiting for it — the band launch (and
// the exchange behind it) off the cycle's critical path. In steady-state
// cycles both streams' launches become ready together and the band waves can
// lose that race (then the bands end with the interior and the exchange
// follows), so later cycles keep the autotuned order. A one-cycle step (the
// 8-rank 20-step strong-scaling run) is all first cycle: 4096-row fp64 slab
// rehearsal, kernel span 647 -> 610 us per cycle (profiles/r4/h/).
static bool lead_first() {  // (read per call: tests toggle it within one process)
  const char* e = std::getenv("HEAT2D_LEAD_FIRST");
  return !e || std::atoi(e) != 0;
}

// smallest steady-state cycle (ms) for which edge-first split plans are tried
constexpr float kEdgeFirstMinCycleMs = 0.4f;

// One trial cycle of plan c (autotuner, prepare's clock warm-up): the real
// kernels and traffic of a cycle, reading the CURRENT buffer and writing the
// other one without a swap or an exchange, so the solution is untouched.
void Solver::trial_cycle(const kern::SplitPlan& c) {
  void* src = buf_[cur_];
  void* dst = buf_[cur_ ^ 1];
  last_k_ = 0;  // the other buffer no longer holds T_{n-1}: stats(residual) reports NaN
  if (c.valid == 3) {  // edge-first: both parts in order on the compute stream
    H2D_HIP(hipStreamWaitEvent(s_compute_, ev_bnd_, 0));
    kern::launch_split(dtype(), src, dst, L_, c, false, cfg_.r, s_compute_, cfg_.arith);
    kern::launch_split(dtype(), src, dst, L_, c, true, cfg_.r, s_compute_, cfg_.arith, d_queue_);
    H2D_HIP(hipEventRecord(ev_int_, s_compute_));
    H2D_HIP(hipEventRecord(ev_bnd_, s_compute_));
    return;
  }
  H2D_HIP(hipStreamWaitEvent(s_compute_, ev_bnd_, 0));
  H2D_HIP(hipStreamWaitEvent(s_comm_, ev_int_, 0));
  if (c.flags & kern::kPlanLead) {  // lead: the band launch issued first
    kern::launch_split(dtype(), src, dst, L_, c, false, cfg_.r, s_comm_, cfg_.arith);
    kern::launch_split(dtype(), src, dst, L_, c, true, cfg_.r, s_compute_, cfg_.arith, d_queue_);
    H2D_HIP(hipEventRecord(ev_int_, s_compute_));
    H2D_HIP(hipEventRecord(ev_bnd_, s_comm_));
    return;
  }
  kern::launch_split(dtype(), src, dst, L_, c, true, cfg_.r, s_compute_, cfg_.arith, d_queue_);
  H2D_HIP(hipEventRecord(ev_int_, s_compute_));
  kern::launch_split(dtype(), src, dst, L_, c, false, cfg_.r, s_comm_, cfg_.arith);
  H2D_HIP(hipEventRecord(ev_bnd_, s_comm_));
}

// Steady-state ms per cycle of plan c: one warm-up trial cycle, then
// kTimed back-to-back trial cycles between two events (both streams, the real
// event protocol, no exchange; the solution is untouched).
float Solver::time_plan(const kern::SplitPlan& c, int kTimed) {
  constexpr int kWarm = 1;
  if (!ev_t0_) {
    H2D_HIP(hipEventCreate(&ev_t0_));
    H2D_HIP(hipEventCreate(&ev_t1_));
  }
  H2D_HIP(hipEventRecord(ev_int_, s_compute_));
  H2D_HIP(hipEventRecord(ev_bnd_, s_comm_));
  for (int i = 0; i < kWarm; ++i) trial_cycle(c);
  H2D_HIP(hipStreamWaitEvent(s_compute_, ev_bnd_, 0));
  H2D_HIP(hipEventRecord(ev_t0_, s_compute_));
  for (int i = 0; i < kTimed; ++i) trial_cycle(c);
  H2D_HIP(hipStreamWaitEvent(s_compute_, ev_bnd_, 0));
  H2D_HIP(hipEventRecord(ev_t1_, s_compute_));
  H2D_HIP(hipEventSynchronize(ev_t1_));
  float ms = 0.f;
  H2D_HIP(hipEventElapsedTime(&ms, ev_t0_, ev_t1_));
  return ms / kTimed;
}

// The environment knobs that shape the autotuner's candidate set or the plans
// it returns (a run with any of them set must neither reuse plans tuned without
// it nor leave plans for runs without it): an FNV-1a hash of their values,
// part of every cache key.
static uint64_t plan_env_hash() {
  static const uint64_t h = [] {
    uint64_t v = 1469598103934665603ull;
    for (const char* name : {"HEAT2D_DYNAMIC", "HEAT2D_TB_RING",
                             "HEAT2D_SPLIT_ORDER", "HEAT2D_SEGMENTS", "HEAT2D_BANDS", "HEAT2D_MAX_WAVES",
                             "HEAT2D_EDGE_BANDS", "HEAT2D_GRAPH_MAX_CYCLE_US"}) {
      const char* e = std::getenv(name);
      const std::string kv = std::string(name) + "=" + (e ? e : "<unset>") + ";";
      for (unsigned char c : kv) v = (v ^ c) * 1099511628211ull;
    }
    return v;
  }();
  return h;
}

// Plan-cache context of this slab: what a tuned plan's timing depends on
// besides the depth (plan_cache.hpp), including the transport (its name and
// whether it gates: the fused candidates exist only for gating transports)
// and the plan-shaping environment knobs.
std::string Solver::cache_ctx() const {
  hipDeviceProp_t prop{};
  std::string arch = "unknown";
  int ncu = 0;
  if (hipGetDeviceProperties(&prop, cfg_.device) == hipSuccess) {
    arch = prop.gcnArchName;
    ncu = prop.multiProcessorCount;
  }
  const int pos = (L_.row0 == 0 ? 1 : 0) | (L_.row0 + L_.nrows == L_.nrows_global ? 2 : 0);
  char b[640];
  std::snprintf(b, sizeof(b), "%s|cu%d|%s|ar%d|%lldx%lld|p%lld|h%lld|pos%d|ccu%d|sp%d|x%d|tr=%s|env%016llx",
                arch.c_str(), ncu, dtype_name(dtype()), cfg_.arith, (long long)L_.nrows, (long long)L_.ncols,
                (long long)L_.pitch, (long long)L_.halo, pos, compute_cus_, spare_waves(), tr_->exchanges() ? 1 : 0,
                tr_->name().c_str(), (unsigned long long)plan_env_hash());
  return b;
}

// The cached autotuned plan of depth k for this slab, re-validated by one
// short re-time (5 trial cycles): kept if within 10 % of the cached time.
bool Solver::cached_split(int k) {
  if (!hip_ || !plancache::enabled()) return false;
  kern::SplitPlan c{};
  float ms = 0.f;
  if (!plancache::get_plan(cache_ctx(), k, k, &c, &ms) || ms <= 0.f) return false;
  // geometry must match this slab (defensive: the key already pins it)
  const kern::SplitPlan fresh = kern::plan_split(dtype(), L_, k, k, compute_cus_, spare_waves(), c.ring,
                                                 c.main.nb, cfg_.arith);
  if (!c.valid || (c.valid != 2 && !fresh.valid) || c.main.r1 > L_.nrows || c.nedge > 4) return false;
  // semantic checks on top of the key: a plan kind this run may not use
  // (the dynamic queue is off under HEAT2D_DYNAMIC=0; a single launch cannot
  // exchange; the lead order is for exchanging slabs)
  if ((c.flags & kern::kPlanDynamic) && !dynamic_candidates()) return false;
  if (c.valid == 2 && tr_->exchanges()) return false;
  if ((c.flags & kern::kPlanLead) && (c.valid != 1 || !tr_->exchanges())) return false;
  // HEAT2D_PLAN_CACHE_TRUST=1: no re-time (bench.py --measure-hbm's profiled
  // re-runs, whose counter collection would distort the timing: they must
  // run the parent run's plans as they are)
  if (const char* e = std::getenv("HEAT2D_PLAN_CACHE_TRUST"); e && std::atoi(e) != 0) {
    c.k = k;
    split_[k] = c;
    tuned_ms_[k] = ms;
    ++plan_cache_hits_;
    return true;
  }
  synchronize();
  const float t = time_plan(c, 4);
  H2D_HIP(hipEventRecord(ev_int_, s_compute_));
  H2D_HIP(hipEventRecord(ev_bnd_, s_comm_));
  synchronize();
  if (std::fabs(t - ms) > 0.10f * ms) return false;
  c.k = k;
  split_[k] = c;
  tuned_ms_[k] = t;
  ++plan_cache_hits_;
  return true;
}

// Staged screening (round 3 timed every candidate over 4 cycles and the 4
// best over 12, twice the trial cycles): stage A times every candidate over ONE cycle
// (after one warm-up cycle; up to 4 for cycles under 1 ms, where one sample is
// noisy and cheap), stage B the 6 best of A over 4, stage C the 3 best
// of B over 12 — about half the trial cycles at the same winner (the leaders
// are 1-2 % apart, which stage C resolves). Cycles longer than kLongCycleMs
// (the full-HBM grids: ~50 ms per pass) screen a reduced candidate family.
constexpr float kLongCycleMs = 8.0f;

// HEAT2D_TUNE_LOG=1: every screening stage's ranking on stderr (diagnostics)
static bool tune_log() {
  static const bool on = [] {
    const char* e = std::getenv("HEAT2D_TUNE_LOG");
    return e && std::atoi(e) != 0;
  }();
  return on;
}

// The trial cycles cannot run the halo exchange (it is collective, and the
// ranks' candidate lists differ), so on an exchanging slab each candidate is
// ranked by its trial time plus the part of the exchange its order cannot
// hide: the concurrent order starts the exchange only after its band launch,
// which runs beside the interior and ends with it (phase timers of the 4096-row
// rehearsal: interior 0.61 ms, bands 0.66 ms) — the whole exchange is exposed;
// the edge-first and fused orders run it beside the interior. The exchange is
// modelled at 50 GB/s per message (an xGMI link, one direction) + 10 us.
// Without it the no-exchange trials picked the concurrent order for the
// 8-rank fp64 slab by 0.5 %, and the exchanging rehearsal ran 18 % slower than
// with the edge-first order (profiles/r4/b/).
float Solver::exchange_penalty(const kern::SplitPlan& c, float trial_ms) const {
  if (!tr_->exchanges()) return 0.f;
  const double bytes = (double)halo_msg_bytes(L_, c.k, dtype_size(dtype()));
  const float tx = (float)(bytes / 50e6 + 0.010);  // ms
  if (c.valid == 3 || (c.valid == 1 && (c.flags & kern::kPlanLead)))
    return std::max(0.f, tx - 0.8f * trial_ms);
  return tx;
}

void Solver::autotune_split(int k) {
  const int spare = spare_waves();
  synchronize();
  kern::SplitPlan best = split_[k];
  const float base_ms = time_plan(best, 2);
  const bool long_cycles = base_ms > kLongCycleMs;
  auto finish = [&](kern::SplitPlan b, float ms) {
    synchronize();
    b.k = k;
    split_[k] = b;
    tuned_ms_[k] = ms;
    if (plancache::enabled()) plancache::put_plan(cache_ctx(), k, k, b, ms);
    // restore the event protocol: both streams idle, events recorded
    H2D_HIP(hipEventRecord(ev_int_, s_compute_));
    H2D_HIP(hipEventRecord(ev_bnd_, s_comm_));
    synchronize();
  };
  // Long cycles (the full-HBM grids, ~50 ms per pass): a neighbouring depth
  // (k -/+ 1) tuned in this process lends its choice — order, ring, interior
  // bands / segments, queue, edge bands — re-planned for k and timed once: a
  // balanced schedule mixes depths k and k + 1, and a second full screening
  // costs ~10 s there (240 GB fp32 grid, 64 steps: depths 21 and 22 —
  // prepare 21 s, profiles/r4/t/).
  if (long_cycles) {
    for (int nk : {k - 1, k + 1}) {
      if (nk < 1 || nk > kMaxTB || (plan_origin_[nk] != 1 && plan_origin_[nk] != 2)) continue;
      const kern::SplitPlan& q = split_[nk];
      if (q.k != nk || !q.valid) continue;
      kern::SplitPlan c = q.valid == 2
                              ? kern::plan_single(dtype(), L_, k, compute_cus_, q.ring, q.main.nb, cfg_.arith)
                              : kern::plan_split(dtype(), L_, k, k, compute_cus_, spare, q.ring, q.main.nb, cfg_.arith);
      if (!c.valid) continue;
      c.valid = q.valid;
      c.flags = q.flags;
      if ((c.valid == 1 || c.valid == 3) && q.nedge > 0 && q.edge[0].nb > 1)
        c = kern::with_edge_bands(dtype(), c, q.edge[0].nb, cfg_.arith);
      const float t = time_plan(c, 2);
      ++tune_trials_;
      // kept only if it beats this depth's default plan on the same score
      // (trial + the exchange its order cannot hide); else the default plan
      // stays — no second screening of ~50 ms cycles either way
      if (t + exchange_penalty(c, t) <= base_ms + exchange_penalty(best, base_ms)) finish(c, t);
      else finish(best, base_ms);
      return;
    }
  }
  const int64_t nb0 = best.main.nb;
  // without an exchange to hide, a single general launch per cycle competes too
  const bool single_ok = !tr_->exchanges();
  const int64_t nb1 = single_ok ? kern::plan_single(dtype(), L_, k, compute_cus_, 0, 0, cfg_.arith).main.nb : 0;
  // mode 1: split, interior and bands concurrently on two streams; mode 2
  // (no exchange): one general launch; mode 3 (exchange): edge-first split —
  // the short band launch first on the whole chip, then the interior, with the
  // exchange of the bands running beside the interior (valid = 3)
  std::vector<kern::SplitPlan> cands{best};
  auto add = [&](const kern::SplitPlan& c) {
    cands.push_back(c);
    // more items than waves: also with the dynamic item queue (faster waves
    // take more items; per-wave timelines of the 32768^2 fp64 interior showed
    // a bimodal spread of up to 25 % between equal items: profiles/r3/wt3/)
    if (dynamic_candidates() && c.main_items > c.main_waves && c.valid >= 1 && c.valid <= 3) {
      kern::SplitPlan d = c;
      d.flags |= kern::kPlanDynamic;
      cands.push_back(d);
    }
  };
  if (dynamic_candidates() && best.main_items > best.main_waves && best.valid >= 1 && best.valid <= 3) {
    kern::SplitPlan d = best;
    d.flags |= kern::kPlanDynamic;
    cands.push_back(d);
  }
  const std::vector<double> factors = long_cycles ? std::vector<double>{1.0, 0.5, 2.0}
                                                  : std::vector<double>{1.0, 0.9, 0.8, 0.7, 0.6, 0.5, 1.25, 1.5, 2.0};
  for (int mode : {1, 2, 3}) {
    if (mode == 2 && !single_ok) continue;
    // the trials run without the exchange, which the edge-first order puts
    // beside the WHOLE interior: only where the interior is long enough to
    // hide it (measured on the 1-rank RCCL rehearsal, profiles/multi_gpu_rehearsal_v4.md:
    // fp64 slabs of 4096-16384 rows +2-4 %; a 4096-row fp32 slab, whose
    // interior cycle is 0.28 ms, lost 7 % to an exposed exchange)
    if (mode == 3 && (single_ok || best.valid != 1 || base_ms < kEdgeFirstMinCycleMs)) continue;
    // ring 8 (6 rows in flight): fp32 single launches only (stencil_tb.hip ring_ok)
    const std::vector<int> rings = (mode == 2 && dtype() == DType::F32 && k <= 16) ? std::vector<int>{4, 6, 8}
                                                                                     : std::vector<int>{4, 6};
    for (int ring : rings) {
      for (double f : factors) {
        const int64_t nb = std::max<int64_t>(1, (int64_t)((mode == 2 ? nb1 : nb0) * f + 0.5));
        if (mode == 1 && ring == best.ring && nb == best.main.nb) continue;
        kern::SplitPlan c = mode == 2 ? kern::plan_single(dtype(), L_, k, compute_cus_, ring, nb, cfg_.arith)
                                      : kern::plan_split(dtype(), L_, k, k, compute_cus_, spare, ring, nb,
                                                         cfg_.arith);
        if (!c.valid) continue;
        if (mode == 3) c.valid = 3;
        if (mode == 1)  // more items than waves only via explicit band counts above the default
          c.main_waves = std::min<int64_t>(c.main_items, std::max<int64_t>(c.main_waves, best.main_waves));
        add(c);
      }
      // segment work items (TbRect nb < 0): the interior cut into equal runs of
      // strip rows, 1/2 .. 2 per persistent wave — balanced whatever the strip
      // count (thin slabs: profiles/thin_slab.md).
      // fp32: single launches only — split plans over segments won 4-cycle trials
      // by noise and then ran 1.7 % slower than bands on 32768^2 (interleaved A/B,
      // profiles/thin_slab.md §4), while single launches over segments win 4096^2
      if (dtype() == DType::F32 && mode != 2) continue;
      const int64_t w0 = mode == 2 ? kern::plan_single(dtype(), L_, k, compute_cus_, ring, 0, cfg_.arith).main_waves
                                   : best.main_waves;
      std::vector<int64_t> segs;
      for (double f : long_cycles ? std::vector<double>{1.0} : std::vector<double>{0.5, 1.0, 1.5, 2.0})
        segs.push_back(std::max<int64_t>(1, (int64_t)(w0 * f + 0.5)));
      if (dynamic_candidates()) segs.push_back(4 * w0);  // (timed with the dynamic queue too, add())
      if (mode == 2 && cfg_.arith == 2 && !long_cycles) {
        // r = 1/4 single launches: strip-aligned segment counts too (a whole
        // number per strip), whose frame-row items the plan can weight
        // (stencil_tb.hip weighted_main) — one per SIMD and one per wave
        const int64_t ns = kern::plan_single(dtype(), L_, k, compute_cus_, ring, 0, cfg_.arith).main.s1;
        const int64_t simds = (int64_t)(compute_cus_ > 0 ? compute_cus_ : device_cus_of(cfg_.device)) * 4;
        for (int64_t target : {simds, w0, 2 * simds}) {
          const int64_t q = target / std::max<int64_t>(ns, 1);
          if (q >= 2) segs.push_back(q * ns);
        }
      }
      std::sort(segs.begin(), segs.end());
      segs.erase(std::unique(segs.begin(), segs.end()), segs.end());
      for (int64_t nseg : segs) {
        kern::SplitPlan c = mode == 2 ? kern::plan_single(dtype(), L_, k, compute_cus_, ring, -nseg, cfg_.arith)
                                      : kern::plan_split(dtype(), L_, k, k, compute_cus_, spare, ring, -nseg,
                                                         cfg_.arith);
        if (!c.valid) continue;
        if (mode == 3) c.valid = 3;
        add(c);
      }
    }
  }
  // screening: (cycles per trial, candidates kept) per stage; stage A times
  // short cycles over up to 4 (a single ~50 us cycle is noisy; they are cheap)
  using Stage = std::pair<int, size_t>;
  const int a_cycles = std::max(1, std::min(4, (int)std::ceil(1.0f / std::max(base_ms, 1e-3f))));
  const std::vector<Stage> stages{{a_cycles, 6}, {4, 3}, {12, 1}};
  struct Timed {
    float score, ms;  // ranking score (trial + exposed exchange), trial ms per cycle
    kern::SplitPlan plan;
  };
  std::vector<Timed> timed;
  for (const auto& c : cands) timed.push_back(Timed{0.f, 0.f, c});
  for (const Stage& st : stages) {
    for (auto& t : timed) {
      t.ms = time_plan(t.plan, st.first);
      t.score = t.ms + exchange_penalty(t.plan, t.ms);
    }
    std::stable_sort(timed.begin(), timed.end(), [](const Timed& x, const Timed& y) { return x.score < y.score; });
    if (tune_log())
      for (const auto& t : timed)
        std::fprintf(stderr, "heat2d tune k=%d cycles=%d: order %d ring %d bands %lld items %lld waves %lld dyn %d ms %.4f score %.4f\n",
                     k, st.first, t.plan.valid, t.plan.ring, (long long)t.plan.main.nb, (long long)t.plan.main_items,
                     (long long)t.plan.main_waves, (t.plan.flags & kern::kPlanDynamic) ? 1 : 0, t.ms, t.score);
    timed.resize(std::min(timed.size(), st.second));
  }
  best = timed.front().plan;
  float best_score = timed.front().score, best_ms = timed.front().ms;
  // the winner's boundary bands cut into 2..4 row bands each: the band launch
  // is latency-bound (one wave per strip and band, ~1 wave per SIMD, each
  // marching B + 2k rows) — more, shorter items where the split leaves the
  // chip room (its time is on the cycle's critical path in the edge-first order)
  if (best.valid == 1 || best.valid == 3) {
    for (int64_t nb : {2, 3, 4}) {
      const kern::SplitPlan c = kern::with_edge_bands(dtype(), best, nb, cfg_.arith);
      if (c.edge_items == best.edge_items) continue;
      const float t = time_plan(c, 12);
      const float score = t + exchange_penalty(c, t);
      ++tune_trials_;
      if (score < best_score) {
        best_score = score;
        best_ms = t;
        best = c;
      }
    }
  }
  tune_trials_ += (int64_t)cands.size();
  finish(best, best_ms);
}

void Solver::launch_overlap(int k, int64_t B) {
  void* src = buf_[cur_];
  void* dst = buf_[cur_ ^ 1];
  const kern::SplitPlan& sp = split_plan_banded(k, B);
  HEAT2D_REQUIRE(sp.valid != 2 || !tr_->exchanges(), "single-launch plan with a halo exchange");
  roctxRangePushA("heat2d.cycle.split");
  PhaseEvents* pe = timing_ ? phase_begin(0) : nullptr;
  pend_pe_ = pe ? (int64_t)phase_ev_.size() - 1 : -1;
  // (the first cycle leads only where the band launch runs on the interior
  // kernel: a slab at the global frame (the first / last rank) bands on the
  // general kernel, whose 1-wave/SIMD waves issued first hold the register
  // files of ~750 SIMDs against the interior — 850 us instead of 615 for its
  // one-cycle step, edge-first 640: profiles/r5/ad/)
  const bool lead = (sp.valid == 1 || sp.valid == 3) &&
                    ((sp.flags & kern::kPlanLead) ||
                     (first_cycle_ && tr_->exchanges() && lead_first() && kern::edges_on_main(L_, sp)));
  // An edge rank's first cycle: its two bands apart. The far band (the one
  // the exchange sends, clear of the global frame) leads on the interior
  // kernel as on a middle rank; the frame-side band — which no exchange
  // reads — goes on the general kernel behind the exchange on the comm
  // stream (cycle_finish), into the wave slots the interior's last round of
  // items leaves free.
  int frame_rect = -1;
  if (!lead && (sp.valid == 1 || sp.valid == 3) && first_cycle_ && tr_->exchanges() && lead_first() &&
      sp.nedge == 2 && kern::edge_rect_on_main(L_, sp, 0) != kern::edge_rect_on_main(L_, sp, 1))
    frame_rect = kern::edge_rect_on_main(L_, sp, 0) ? 1 : 0;
  first_cycle_ = false;
  if (frame_rect >= 0) {
    H2D_HIP(hipStreamWaitEvent(s_compute_, ev_bnd_, 0));  // edge part c-1
    H2D_HIP(hipStreamWaitEvent(s_comm_, ev_int_, 0));     // main part c-1
    if (pe) H2D_HIP(hipEventRecord(pe->ev[2], s_comm_));
    kern::launch_edge_rect(dtype(), src, dst, L_, sp, 1 - frame_rect, cfg_.r, s_comm_, cfg_.arith);
    if (pe) H2D_HIP(hipEventRecord(pe->ev[0], s_compute_));
    kern::launch_split(dtype(), src, dst, L_, sp, true, cfg_.r, s_compute_, cfg_.arith, d_queue_);
    if (pe) H2D_HIP(hipEventRecord(pe->ev[1], s_compute_));
    H2D_HIP(hipEventRecord(ev_int_, s_compute_));
    if (pe) H2D_HIP(hipEventRecord(pe->ev[3], s_comm_));
    H2D_HIP(hipEventRecord(ev_bnd_, s_comm_));
    if (tr_->exchanges()) tr_->post(dst, L_, ev_bnd_);
    pend_ = Pending::Concurrent;
    pend_frame_ = frame_rect;
    pend_frame_b_ = B;
    return;
  }
  if (sp.valid == 3 && !lead) {
    // edge-first: compute stream = [exchange c-1 landed] bands(c) -> interior(c);
    // comm stream (cycle_finish) = [bands(c) done] exchange(c), beside the interior.
    H2D_HIP(hipStreamWaitEvent(s_compute_, ev_comm_, 0));
    if (pe) H2D_HIP(hipEventRecord(pe->ev[2], s_compute_));
    kern::launch_split(dtype(), src, dst, L_, sp, false, cfg_.r, s_compute_, cfg_.arith);
    if (pe) H2D_HIP(hipEventRecord(pe->ev[3], s_compute_));
    H2D_HIP(hipEventRecord(ev_bnd_, s_compute_));
    if (tr_->exchanges()) tr_->post(dst, L_, ev_bnd_);
    if (pe) H2D_HIP(hipEventRecord(pe->ev[0], s_compute_));
    kern::launch_split(dtype(), src, dst, L_, sp, true, cfg_.r, s_compute_, cfg_.arith, d_queue_);
    if (pe) H2D_HIP(hipEventRecord(pe->ev[1], s_compute_));
    H2D_HIP(hipEventRecord(ev_int_, s_compute_));
    pend_ = Pending::EdgeFirst;
    return;
  }
  H2D_HIP(hipStreamWaitEvent(s_compute_, ev_bnd_, 0));  // edge part c-1 (record not yet replaced)
  H2D_HIP(hipStreamWaitEvent(s_comm_, ev_int_, 0));     // main part c-1
  if (pe) H2D_HIP(hipEventRecord(pe->ev[2], s_comm_));
  if (lead) {
    // lead: the band launch first (comm stream), then the interior beside it
    kern::launch_split(dtype(), src, dst, L_, sp, false, cfg_.r, s_comm_, cfg_.arith);
    if (pe) H2D_HIP(hipEventRecord(pe->ev[0], s_compute_));
    kern::launch_split(dtype(), src, dst, L_, sp, true, cfg_.r, s_compute_, cfg_.arith, d_queue_);
    if (pe) H2D_HIP(hipEventRecord(pe->ev[1], s_compute_));
    H2D_HIP(hipEventRecord(ev_int_, s_compute_));
  } else if (sp.valid) {
    if (pe) H2D_HIP(hipEventRecord(pe->ev[0], s_compute_));
    kern::launch_split(dtype(), src, dst, L_, sp, true, cfg_.r, s_compute_, cfg_.arith, d_queue_);
    if (pe) H2D_HIP(hipEventRecord(pe->ev[1], s_compute_));
    H2D_HIP(hipEventRecord(ev_int_, s_compute_));
    kern::launch_split(dtype(), src, dst, L_, sp, false, cfg_.r, s_comm_, cfg_.arith);
  } else {  // slab too thin / narrow to split: all of it beside the exchange
    if (pe) {
      H2D_HIP(hipEventRecord(pe->ev[0], s_compute_));
      H2D_HIP(hipEventRecord(pe->ev[1], s_compute_));
    }
    kern::launch_tb(dtype(), src, dst, L_, 0, L_.nrows, k, cfg_.r, s_comm_, 0, 0, cfg_.arith);
  }
  if (pe) H2D_HIP(hipEventRecord(pe->ev[3], s_comm_));
  H2D_HIP(hipEventRecord(ev_bnd_, s_comm_));
  if (tr_->exchanges()) tr_->post(dst, L_, ev_bnd_);
  pend_ = Pending::Concurrent;
}

void Solver::cycle_copy_swap() {
  // Reference-parity schedule (fortran/hip/heat.F90:243-249): T_old <- T (full
  // D2D copy), T <- stencil(T_old), halo swap into T. No pointer swap.
  void* cur = buf_[cur_];
  void* old = buf_[cur_ ^ 1];
  const size_t bytes = (size_t)L_.elems() * dtype_size(dtype());
  if (hip_) kern::launch_copy(old, cur, (int64_t)bytes, s_compute_);
  else std::memcpy(old, cur, bytes);
  launch_tb(old, cur, 0, L_.nrows, 1);
  exchange_on(cur, 1, s_compute_);
  ghost_ = 1;
  if (tr_->exchanges()) last_x_[0] = last_x_[1] = 1;
  last_k_ = 1;
}

void Solver::run_graph_cycles(int64_t npairs) {
  ensure_pair_graph();
  first_cycle_ = false;  // the replay is this call's first cycle: any eager cycle after it is not
  const int K = k_pref_;
  const bool ovl = cfg_.overlap != 0;
  if (ovl) {  // the graph starts only when the eager work on both streams is done
    H2D_HIP(hipStreamWaitEvent(s_compute_, ev_bnd_, 0));
    H2D_HIP(hipStreamWaitEvent(s_compute_, ev_comm_, 0));
  }
  // the graph was captured for buffer parity 0 -> 1 -> 0
  for (int64_t i = 0; i < npairs; ++i) H2D_HIP(hipGraphLaunch(graph_exec_, s_compute_));
  if (npairs > 0 && tr_->exchanges()) tr_->graph_launched(s_compute_);
  hist_[K] += 2 * npairs;
  if (npairs > 0) {
    last_k_ = K;
    ghost_ = K;  // both captured cycles exchange K rows
    if (tr_->exchanges()) {
      last_x_[0] = last_x_[1] = K;
      halo_rows_ += 2 * npairs * K;
    }
  }
  if (ovl) {  // eager cycles after the graph order against its end
    H2D_HIP(hipEventRecord(ev_int_, s_compute_));
    H2D_HIP(hipEventRecord(ev_bnd_, s_compute_));
    H2D_HIP(hipEventRecord(ev_comm_, s_compute_));
    H2D_HIP(hipStreamWaitEvent(s_comm_, ev_comm_, 0));
  }
}

// Capture + instantiate the two-cycle graph of depth pref_depth (parity 0 ->
// 1 -> 0) unless it exists: called by prepare(), so that instantiation (~ms)
// stays out of timed step()s.
void Solver::ensure_pair_graph() {
  const int K = k_pref_;
  const bool ovl = cfg_.overlap != 0;
  if (ovl) (void)split_plan(K);  // plan / autotune (synchronising) before any capture
  if (!graph_exec_ || graph_k_ != K) {
    if (graph_exec_) {
      hipGraphExec_t old = graph_exec_;
      graph_exec_ = nullptr;  // (a failure below must not leave the destructor a destroyed exec)
      H2D_HIP(hipGraphExecDestroy(old));
    }
    hipGraph_t g = nullptr;
    const hipEvent_t fork = ev_fork_, join = ev_join_;  // (the solver's own: see runtime.hpp)
    const int saved = cur_, saved_ghost = ghost_, saved_last = last_k_;
    const int64_t saved_steps = steps_, saved_hist = hist_[K], saved_halo = halo_rows_;
    ghost_ = (int)band_;  // replays start after step()'s top-up
    const int saved_lx0 = last_x_[0], saved_lx1 = last_x_[1];
    if (tr_->exchanges()) last_x_[0] = last_x_[1] = (int)band_;  // whatever a replay follows
    first_cycle_ = false;  // captured cycles keep their plans' order, whatever ran before
    if (!ovl) {
      H2D_HIP(hipStreamBeginCapture(s_compute_, hipStreamCaptureModeThreadLocal));
      for (int c = 0; c < 2; ++c) {
        cycle_launch(K);
        cycle_finish();
      }
    } else {
      // Two-stream capture: fork the comm stream off the capture, record the
      // two overlapped cycles (their event protocol becomes graph edges), join.
      // Cross-cycle overlap inside the graph is kept; at graph boundaries the
      // launches serialise (the next graph's first cycle needs this one's
      // second anyway, except the exchange, which then is not hidden).
      H2D_HIP(hipStreamBeginCapture(s_compute_, hipStreamCaptureModeThreadLocal));
      H2D_HIP(hipEventRecord(fork, s_compute_));
      H2D_HIP(hipStreamWaitEvent(s_comm_, fork, 0));
      H2D_HIP(hipEventRecord(ev_int_, s_compute_));  // in-capture records replace the external ones
      H2D_HIP(hipEventRecord(ev_bnd_, s_comm_));
      H2D_HIP(hipEventRecord(ev_comm_, s_comm_));  // edge-first cycles wait on it
      const bool timing = timing_;
      timing_ = false;  // no timing events inside graphs
      for (int c = 0; c < 2; ++c) {
        cycle_launch(K);
        cycle_finish();
      }
      timing_ = timing;
      H2D_HIP(hipEventRecord(join, s_comm_));
      H2D_HIP(hipStreamWaitEvent(s_compute_, join, 0));
      H2D_HIP(hipStreamEndCapture(s_compute_, &g));
    }
    cur_ = saved;
    steps_ = saved_steps;
    hist_[K] = saved_hist;
    ghost_ = saved_ghost;
    last_k_ = saved_last;
    halo_rows_ = saved_halo;
    last_x_[0] = saved_lx0;
    last_x_[1] = saved_lx1;
    if (!g) H2D_HIP(hipStreamEndCapture(s_compute_, &g));
    H2D_HIP(hipGraphInstantiate(&graph_exec_, g, nullptr, nullptr, 0));
    H2D_HIP(hipGraphDestroy(g));
    H2D_HIP(hipGraphUpload(graph_exec_, s_compute_));  // (not in the first timed launch)
    graph_k_ = K;
    if (ovl) {  // the events were recorded inside the capture only: re-establish them
      H2D_HIP(hipEventRecord(ev_int_, s_compute_));
      H2D_HIP(hipEventRecord(ev_bnd_, s_comm_));
      H2D_HIP(hipEventRecord(ev_comm_, s_comm_));
    }
  }
}

bool Solver::pair_graphs() const {
  return cfg_.use_graph && hip_ && (!tr_->exchanges() || tr_->capturable());
}

// step(n)'s cycles from buffer parity `par`: the measured schedule if prepare()
// chose one, else graph pairs of depth pref_depth (parity 0 only, the parity
// the pair graph was captured for) and balanced cycles: ceil(left / K) cycles
// of depth base or base + 1 rather than full-depth cycles plus one short
// remainder cycle (a K = 4 cycle runs ~3x slower per step than K = 12: 100
// steps = 8 x 11 + 12, not 8 x 12 + 4).
std::vector<Solver::CycleRun> Solver::step_runs(int64_t n, int par) const {
  std::vector<CycleRun> runs;
  if (n <= 0) return runs;
  if (const std::vector<int>* sc = schedule(n)) {
    for (int k : *sc) runs.push_back({k, 0});
    return runs;
  }
  const int K = k_pref_;
  int64_t left = n;
  while (left > 0) {
    if (pair_graphs() && left >= 2 * K && par == 0) {
      const int64_t pairs = left / (2 * K);
      runs.push_back({K, pairs});
      left -= pairs * 2 * K;
      continue;
    }
    const int64_t ncyc = (left + K - 1) / K;
    const int k = (int)(left / ncyc + (left % ncyc ? 1 : 0));
    runs.push_back({k, 0});
    left -= k;
    par ^= 1;
  }
  return runs;
}

std::vector<int> Solver::step_cycles(int64_t n) const {
  if (cfg_.copy_swap) return std::vector<int>((size_t)std::max<int64_t>(0, n), 1);
  std::vector<int> seq;
  for (const CycleRun& r : step_runs(n, cur_)) seq.insert(seq.end(), (size_t)(r.pairs > 0 ? 2 * r.pairs : 1), r.k);
  return seq;
}

void Solver::step(int64_t n) {
  if (n <= 0) return;
  if (hip_) H2D_HIP(hipSetDevice(cfg_.device));
  if (cfg_.copy_swap) {
    for (int64_t i = 0; i < n; ++i) cycle_copy_swap();
    steps_ += n;
    return;
  }
  const std::vector<CycleRun> runs = step_runs(n, cur_);
  first_cycle_ = true;
  // each cycle's exchange moves the rows the NEXT cycle reads; the last one
  // those of this call's first cycle (a repeated step(n) — bench, the CLI's
  // chunks — then never tops up)
  const int first = runs.front().k;
  topup(first);
  if (schedule(n) && replay_schedule(n)) {
    run_schedule_graph(n);
    return;
  }
  for (size_t i = 0; i < runs.size(); ++i) {
    if (runs[i].pairs > 0) {
      run_graph_cycles(runs[i].pairs);
      steps_ += runs[i].pairs * 2 * runs[i].k;
      continue;
    }
    cycle_launch(runs[i].k, i + 1 < runs.size() ? runs[i + 1].k : first);
    cycle_finish();
  }
}

// Same decision on every rank (autotune_slabs: the global problem decides).
bool Solver::measured_schedules() const {
  if (!hip_ || !cfg_.overlap || cfg_.copy_swap || jit_) return false;
  if (cfg_.use_graph && tr_->exchanges() && !tr_->capturable()) return false;  // graphs of the pair kind
  return autotune_slabs(cfg_.n_rows, cfg_.n_cols, tr_->size(), cfg_.autotune);
}

std::string Solver::sched_ctx() const {
  // the schedule is the ranks' common choice: the whole decomposition is its key
  return cache_ctx() + "|P" + std::to_string(tr_->size()) + "|N" + std::to_string(cfg_.n_rows) + "|kmax" +
         std::to_string(cfg_.tb) + "|g" + std::to_string(schedule_graphs() ? 1 : 0);
}

// A cached measured schedule for step(n), used only if EVERY rank has the
// same one (min/max of its hash all-reduced): a hit on some ranks only must
// not let them skip the collectives of the schedule search the others run.
bool Solver::cached_schedule(int64_t n) {
  if (!hip_ || !plancache::enabled()) return false;
  std::vector<int> s;
  const bool hit = plancache::get_schedule(sched_ctx(), n, &s);
  uint64_t h = 1469598103934665603ull;
  for (int d : s) h = (h ^ (uint64_t)d) * 1099511628211ull;
  const double hv = (double)(h >> 12);
  if (tr_->exchanges() && tr_->collective()) {
    double v[3] = {hit ? 1.0 : 0.0, hv, -hv};
    tr_->allreduce(v, 3, 2);  // min
    if (v[0] != 1.0 || v[1] != -v[2]) return false;
  } else if (!hit) {
    return false;
  }
  sched_[n] = std::move(s);
  ++plan_cache_hits_;
  return true;
}

bool autotune_slabs(int64_t n_rows, int64_t n_cols, int nranks, int autotune) {
  if (autotune >= 0) return autotune > 0;
  const int64_t min_rows = n_rows / std::max(1, nranks);  // the thinnest slab of decompose()
  return min_rows * n_cols >= (int64_t(1) << 24);
}

// FNV-1a over the cycles step(n) runs from the current parity and the
// exchange depth after each: what RCCL pairs by order across ranks.
uint64_t Solver::sequence_hash(int64_t n) const {
  uint64_t h = 1469598103934665603ull;
  auto mix = [&](int64_t v) {
    for (int b = 0; b < 8; ++b) {
      h ^= (uint64_t)((v >> (8 * b)) & 0xff);
      h *= 1099511628211ull;
    }
  };
  mix(n);
  mix(band_);
  mix(cfg_.copy_swap);
  const std::vector<int> seq = step_cycles(n);
  for (size_t i = 0; i < seq.size(); ++i) {
    mix(seq[i]);
    mix(exchange_depth(seq, i, seq.front()));
  }
  return h;
}

void Solver::agree(uint64_t h, const std::string& what) {
  if (!tr_->exchanges() || !tr_->collective() || tr_->size() <= 1) return;
  const int P = tr_->size(), me = tr_->rank();
  const double hv = (double)(h >> 12);  // 52 bits: exact in a double, exact under a sum with zeros
  if (P <= 64) {
    std::vector<double> v((size_t)P, 0.0);
    v[(size_t)me] = hv;
    tr_->allreduce(v.data(), P, 0);
    bool same = true;
    for (int r = 1; r < P; ++r) same = same && v[(size_t)r] == v[0];
    if (same) return;
    std::string msg = "ranks disagree on " + what + " (a collective would mismatch): ";
    char b[64];
    for (int r = 0; r < P; ++r) {
      std::snprintf(b, sizeof(b), "%srank %d: %013llx", r ? ", " : "", r, (unsigned long long)v[(size_t)r]);
      msg += b;
    }
    fail(__FILE__, __LINE__, msg + " (this is rank " + std::to_string(me) + ")");
  }
  double mm[2] = {hv, -hv};
  tr_->allreduce(mm, 2, 1);
  if (mm[0] != -mm[1])
    fail(__FILE__, __LINE__, "ranks disagree on " + what + " (rank " + std::to_string(me) + " of " +
                                 std::to_string(P) + ")");
}

// Autotuned steady-state cycle time of depth k, max over ranks (0: no tuned
// split plan for this depth, e.g. a slab too thin to split).
float Solver::depth_ms(int k) {
  if (depth_ms_[k] == 0.f) {
    (void)split_plan(k);
    double v = tuned_ms_[k];
    tr_->allreduce(&v, 1, 1);
    depth_ms_[k] = v > 0 ? (float)v : -1.f;
    if (tune_log()) std::fprintf(stderr, "heat2d sched depth k=%d tuned ms %.4f\n", k, depth_ms_[k]);
  }
  return depth_ms_[k];
}

float Solver::prescan_ms(int k) {
  if (pre_ms_[k] == 0.f) {
    double v = 0.0;
    if (tuned_ms_[k] > 0.f) {
      v = tuned_ms_[k];
    } else {
      const kern::SplitPlan base = kern::plan_split(dtype(), L_, k, k, compute_cus_, spare_waves(), 0, 0, cfg_.arith);
      if (base.valid) {
        synchronize();
        v = time_plan(base, 2);
        H2D_HIP(hipEventRecord(ev_int_, s_compute_));
        H2D_HIP(hipEventRecord(ev_bnd_, s_comm_));
        synchronize();
      }
    }
    tr_->allreduce(&v, 1, 1);
    pre_ms_[k] = v > 0 ? (float)v : -1.f;
    if (tune_log()) std::fprintf(stderr, "heat2d sched prescan k=%d ms %.4f\n", k, pre_ms_[k]);
  }
  return pre_ms_[k];
}

// The measured schedule of n steps (schedule.cpp search_schedule): the default
// plans of the deep depths prescanned (1 warm-up + 2 trial cycles each), the
// near-best ones autotuned, the exact DP over the tuned cycle times, walks past
// the tuned range on long runs. Both measurements are max-over-ranks all-reduces
// issued in the same order on every rank (the search is a function of their
// values), so the ranks agree without exchanging the schedule.
ScheduleSearch Solver::choose_schedule(int64_t n) {
  ScheduleSearchOptions o;
  o.near_tol = 0.05;  // prepare_plans keeps 5 % (tiny graph runs) or 3 % of them
  o.near_max = 4;
  ScheduleSearch r = search_schedule(
      n, cfg_.tb, [this](int k) { return (double)prescan_ms(k); }, [this](int k) { return (double)depth_ms(k); }, o);
  if (tune_log()) {
    std::fprintf(stderr, "heat2d sched n=%lld: %zu cycles of %d..%d, tuned cost %.4f ms (prescanned %zu, tuned %zu)\n",
                 (long long)n, r.best.size(), r.best.empty() ? 0 : r.best.back(), r.best.empty() ? 0 : r.best.front(),
                 r.cost, r.prescanned.size(), r.tuned.size());
    for (const auto& c : r.near)
      std::fprintf(stderr, "heat2d sched n=%lld near: %zu cycles of %d..%d, %.4f ms\n", (long long)n, c.second.size(),
                   c.second.back(), c.second.front(), c.first);
  }
  return r;
}

// One timed replay of a graph of sc's TRIAL cycles (each reads the current
// buffer and writes the other one: the solution is untouched), captured like
// capture_schedule's graph: what step(n) would replay, minus the data flow.
// The fastest of reps eager launches of sc's TRIAL cycles (as time_plan, over
// a schedule; the solution is untouched), after one untimed pass.
float Solver::time_trial_eager(const std::vector<int>& sc, int reps) {
  for (int k : sc) (void)split_plan(k);
  synchronize();
  if (!ev_t0_) {
    H2D_HIP(hipEventCreate(&ev_t0_));
    H2D_HIP(hipEventCreate(&ev_t1_));
  }
  H2D_HIP(hipEventRecord(ev_int_, s_compute_));
  H2D_HIP(hipEventRecord(ev_bnd_, s_comm_));
  for (int k : sc) trial_cycle(split_plan(k));  // warm
  float best = 1e30f;
  for (int r = 0; r < std::max(1, reps); ++r) {
    H2D_HIP(hipStreamWaitEvent(s_compute_, ev_bnd_, 0));
    H2D_HIP(hipEventRecord(ev_t0_, s_compute_));
    for (int k : sc) trial_cycle(split_plan(k));
    H2D_HIP(hipStreamWaitEvent(s_compute_, ev_bnd_, 0));
    H2D_HIP(hipEventRecord(ev_t1_, s_compute_));
    H2D_HIP(hipEventSynchronize(ev_t1_));
    float ms = 0.f;
    H2D_HIP(hipEventElapsedTime(&ms, ev_t0_, ev_t1_));
    best = std::min(best, ms);
  }
  H2D_HIP(hipEventRecord(ev_int_, s_compute_));
  H2D_HIP(hipEventRecord(ev_bnd_, s_comm_));
  synchronize();
  return best;
}

float Solver::time_trial_schedule(const std::vector<int>& sc, int reps) {
  for (int k : sc) (void)split_plan(k);
  synchronize();
  const hipEvent_t fork = ev_fork_, join = ev_join_;  // (the solver's own: see runtime.hpp)
  hipEvent_t e0 = nullptr, e1 = nullptr;  // (recorded outside the capture)
  H2D_HIP(hipEventCreate(&e0));
  H2D_HIP(hipEventCreate(&e1));
  hipGraph_t g = nullptr;
  H2D_HIP(hipStreamBeginCapture(s_compute_, hipStreamCaptureModeThreadLocal));
  H2D_HIP(hipEventRecord(fork, s_compute_));
  H2D_HIP(hipStreamWaitEvent(s_comm_, fork, 0));
  H2D_HIP(hipEventRecord(ev_int_, s_compute_));
  H2D_HIP(hipEventRecord(ev_bnd_, s_comm_));
  for (int k : sc) trial_cycle(split_plan(k));
  H2D_HIP(hipEventRecord(join, s_comm_));
  H2D_HIP(hipStreamWaitEvent(s_compute_, join, 0));
  H2D_HIP(hipStreamEndCapture(s_compute_, &g));
  hipGraphExec_t ge = nullptr;
  H2D_HIP(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  H2D_HIP(hipGraphDestroy(g));
  H2D_HIP(hipGraphLaunch(ge, s_compute_));  // warm (clocks, caches)
  float ms = 1e30f;
  for (int i = 0; i < std::max(1, reps); ++i) {  // the fastest of reps replays
    H2D_HIP(hipEventRecord(e0, s_compute_));
    H2D_HIP(hipGraphLaunch(ge, s_compute_));
    H2D_HIP(hipEventRecord(e1, s_compute_));
    H2D_HIP(hipEventSynchronize(e1));
    float t = 0.f;
    H2D_HIP(hipEventElapsedTime(&t, e0, e1));
    ms = std::min(ms, t);
  }
  H2D_HIP(hipGraphExecDestroy(ge));
  for (hipEvent_t e : {e0, e1}) H2D_HIP(hipEventDestroy(e));
  // the events were recorded inside the capture only: re-establish them
  H2D_HIP(hipEventRecord(ev_int_, s_compute_));
  H2D_HIP(hipEventRecord(ev_bnd_, s_comm_));
  H2D_HIP(hipEventRecord(ev_comm_, s_comm_));
  synchronize();
  return ms;
}

bool Solver::schedule_graphs() const {
  return cfg_.use_graph && hip_ && cfg_.overlap && (!tr_->exchanges() || tr_->capturable());
}

// Mean cycle time (us) from which step(n) launches its schedule eagerly
// instead of replaying it as a graph (HEAT2D_GRAPH_MAX_CYCLE_US).
static double graph_max_cycle_us() {
  const char* e = std::getenv("HEAT2D_GRAPH_MAX_CYCLE_US");
  return e ? std::atof(e) : 400.0;
}

// Whether step(n) replays its measured schedule as one captured graph. A
// graph removes the host launches between cycles — what a short-cycle
// schedule needs (4096^2 fp32: ~47 us cycles, the launch gaps a quarter of
// one) — but a long-cycle schedule hides them anyway behind its kernels, and
// there the replay measured slower than the eager launches (interleaved on one
// box, profiles/r4/gf/, r4/gg/): 32768^2 fp64 20 steps (one 4.3 ms cycle) 4735
// vs 4861 Gpts/s, 100 steps 4797 vs 4917; 16384^2 fp32 480 steps (0.59 ms
// cycles) 9129 vs 10579; 8192^2 fp64 (0.28 ms cycles) 3676 replayed vs 3638.
// Decided from the tuned cycle times, max over ranks (depth_ms), so every rank
// decides the same.
bool Solver::replay_schedule(int64_t n) {
  if (!schedule_graphs()) return false;
  if (auto it = sched_replay_.find(n); it != sched_replay_.end()) return it->second;
  const std::vector<int>* s = schedule(n);
  if (!s || s->empty()) return false;
  double est = 0.0;
  for (int k : *s) est += std::max(0.0, (double)depth_ms(k));
  const bool g = est * 1e3 < graph_max_cycle_us() * (double)s->size();
  sched_replay_[n] = g;
  return g;
}

// Capture the whole measured schedule of n steps, from the current buffer
// parity, as one graph: both streams (the comm stream forked off the capture),
// the cycles' event protocol as graph edges. Replayed by step(n) with no
// host launches between cycles (small grids: the ~12 us gaps between the
// cross-stream launches are a quarter of a 4096^2 fp32 cycle).
void Solver::capture_schedule(int64_t n) {
  const std::vector<int>& sc = sched_.at(n);
  for (size_t i = 0; i < sc.size(); ++i)  // plan / autotune (synchronising) before the capture
    (void)split_plan_banded(sc[i], std::max(sc[i], exchange_depth(sc, i, sc[0])));
  synchronize();
  const int saved = cur_, saved_ghost = ghost_, saved_last = last_k_;
  const int64_t saved_steps = steps_, saved_halo = halo_rows_;
  ghost_ = (int)band_;  // replays start after step()'s top-up
  const int saved_lx0 = last_x_[0], saved_lx1 = last_x_[1];
  if (tr_->exchanges()) last_x_[0] = last_x_[1] = (int)band_;  // whatever a replay follows
  int64_t saved_hist[kMaxTB + 1];
  std::copy(hist_, hist_ + kMaxTB + 1, saved_hist);
  first_cycle_ = false;  // captured cycles keep their plans' order, whatever ran before
  const hipEvent_t fork = ev_fork_, join = ev_join_;  // (the solver's own: see runtime.hpp)
  hipGraph_t g = nullptr;
  H2D_HIP(hipStreamBeginCapture(s_compute_, hipStreamCaptureModeThreadLocal));
  H2D_HIP(hipEventRecord(fork, s_compute_));
  H2D_HIP(hipStreamWaitEvent(s_comm_, fork, 0));
  H2D_HIP(hipEventRecord(ev_int_, s_compute_));  // in-capture records replace the external ones
  H2D_HIP(hipEventRecord(ev_bnd_, s_comm_));
  H2D_HIP(hipEventRecord(ev_comm_, s_comm_));
  const bool timing = timing_;
  timing_ = false;
  for (size_t i = 0; i < sc.size(); ++i) {
    cycle_launch(sc[i], exchange_depth(sc, i, sc[0]));
    cycle_finish();
  }
  timing_ = timing;
  H2D_HIP(hipEventRecord(join, s_comm_));
  H2D_HIP(hipStreamWaitEvent(s_compute_, join, 0));
  H2D_HIP(hipStreamEndCapture(s_compute_, &g));
  cur_ = saved;
  steps_ = saved_steps;
  ghost_ = saved_ghost;
  last_k_ = saved_last;
  halo_rows_ = saved_halo;
  last_x_[0] = saved_lx0;
  last_x_[1] = saved_lx1;
  std::copy(saved_hist, saved_hist + kMaxTB + 1, hist_);
  hipGraphExec_t ge = nullptr;
  H2D_HIP(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  H2D_HIP(hipGraphDestroy(g));
  // upload it now (prepare), not in the first launch — the timed step(n):
  // small grid 5568 vs 5548, headline 4777 vs 4760 (medians, interleaved,
  // profiles/r4/gu/)
  H2D_HIP(hipGraphUpload(ge, s_compute_));
  hipGraphExec_t& slot = sched_graph_[{n, cur_}];
  if (slot) H2D_HIP(hipGraphExecDestroy(slot));  // a re-captured schedule replaces its old graph
  slot = ge;
  // the events were recorded inside the capture only: re-establish them
  H2D_HIP(hipEventRecord(ev_int_, s_compute_));
  H2D_HIP(hipEventRecord(ev_bnd_, s_comm_));
  H2D_HIP(hipEventRecord(ev_comm_, s_comm_));
}

void Solver::run_schedule_graph(int64_t n) {
  first_cycle_ = false;
  auto it = sched_graph_.find({n, cur_});
  if (it == sched_graph_.end()) {
    capture_schedule(n);
    it = sched_graph_.find({n, cur_});
  }
  const std::vector<int>& sc = sched_.at(n);
  // the graph starts when the eager work on both streams is done
  H2D_HIP(hipStreamWaitEvent(s_compute_, ev_bnd_, 0));
  H2D_HIP(hipStreamWaitEvent(s_compute_, ev_comm_, 0));
  H2D_HIP(hipGraphLaunch(it->second, s_compute_));
  if (tr_->exchanges()) tr_->graph_launched(s_compute_);
  // eager cycles after the graph order against its end
  H2D_HIP(hipEventRecord(ev_int_, s_compute_));
  H2D_HIP(hipEventRecord(ev_bnd_, s_compute_));
  H2D_HIP(hipEventRecord(ev_comm_, s_compute_));
  H2D_HIP(hipStreamWaitEvent(s_comm_, ev_comm_, 0));
  for (size_t i = 0; i < sc.size(); ++i) {
    hist_[sc[i]] += 1;
    steps_ += sc[i];
    if (tr_->exchanges()) halo_rows_ += exchange_depth(sc, i, sc[0]);
  }
  last_k_ = sc.back();
  ghost_ = sc.front();  // the last captured cycle's exchange depth
  if (tr_->exchanges())  // conservative: the deepest exchange of the replay, on both buffers
    last_x_[0] = last_x_[1] = *std::max_element(sc.begin(), sc.end());
  if (sc.size() % 2) cycle_swap();
}

const std::vector<int>* Solver::schedule(int64_t n) const {
  auto it = sched_.find(n);
  return it == sched_.end() ? nullptr : &it->second;
}

void Solver::prepare(int64_t n) {
  if (n <= 0) return;
  if (hip_ && cfg_.overlap && !cfg_.copy_swap) prepare_plans(n);
  // every rank runs the same cycles with the same exchange depths (RCCL pairs
  // the sends / receives by order: a mismatch is a hang or wrong ghost rows)
  agree(sequence_hash(n), "step(" + std::to_string(n) + ")'s cycle sequence / exchange depths");
  // step(n)'s first cycle reads deeper ghost rows than the last exchange moved
  // (e.g. a shallow warmup before it): top up here, outside the timed step
  const std::vector<int> seq = step_cycles(n);
  if (!seq.empty()) topup(seq.front());
  if (const std::vector<int>* s = schedule(n); s && hip_ && cfg_.overlap && !cfg_.copy_swap) {
    // Leave the GPU in the schedule's steady state, last (after the
    // agreement and the top-up): the search ends on its shallowest
    // (HBM-bound) depths, and a VALU-bound cycle that follows HBM-bound work
    // or an idle gap runs at lower clocks (32768^2 fp64, one depth-20 pass:
    // 6.4 ms after a compute-bound cycle, 6.8 ms after a depth-5 one, 7.5 ms
    // after 0.5 s idle; profiles/depth_schedule.md). Trial cycles of its first
    // depths, state untouched.
    synchronize();
    // (>= 3 cycles, until ~100 ms or 64 cycles: the 8-rank slab's one 0.6 ms
    // cycle ran 4252 Gpts/s after 33 of them (20 ms), 4348 after 64 — means of
    // 4 and 10 interleaved runs, profiles/r5/m/, r5/n/)
    float ms = 0.f;
    for (size_t i = 0; i < 64 && (i < 3 || ms < 100.f); ++i) {
      const int k = (*s)[i % s->size()];
      trial_cycle(split_plan(k));
      ms += tuned_ms_[k] > 0.f ? tuned_ms_[k] : 1.f;  // local estimate: no collective here
    }
    H2D_HIP(hipEventRecord(ev_int_, s_compute_));
    H2D_HIP(hipEventRecord(ev_bnd_, s_comm_));
    synchronize();
  }
}

void Solver::prepare_plans(int64_t n) {
  if (measured_schedules() && !sched_.count(n) && cached_schedule(n)) {
    // plans of the cached schedule's depths (cached too: re-validated, else re-tuned)
    for (int k : sched_.at(n)) (void)split_plan(k);
  }
  if (measured_schedules() && !sched_.count(n)) {
    const ScheduleSearch r = choose_schedule(n);
    std::vector<int> s = r.best;
    // Near ties are timed as step(n) will run them: the summed per-depth
    // estimates mispredict a whole schedule by a few % (4096^2 fp64: depth 10
    // estimated 0.4 % faster, replayed 5 % slower than 12, profiles/r2_s3/
    // sched_small/; 32768^2 fp32 480 steps: 22/23-deep cycles estimated 0.5 %
    // cheaper than 20 x 24, ran 2-2.5 % slower eagerly, profiles/r4/gn/).
    // Graph-replayed schedules: captured graphs of trial cycles (runs under
    // 10 ms — the 4096^2 fp32 grid — widen to 4 within 5 %, the fastest of 5
    // replays each: profiles/r4/c/small_*.json); eager ones of >= 8 cycles:
    // eager trial schedules, best of 2. Single-rank runs estimated under 50 ms
    // (no collective needed to agree; candidates are tuned already).
    double est = 0.0;
    for (int k : s) est += std::max(0.0, (double)depth_ms(k));
    const bool replay = schedule_graphs() && est * 1e3 < graph_max_cycle_us() * (double)s.size();
    if (!s.empty() && !tr_->exchanges() && est < 50.0 && (replay || s.size() >= 8)) {
      const bool tiny = replay && est < 10.0;
      const double tol = tiny ? 0.05 : 0.03;
      std::vector<std::vector<int>> near;
      for (const auto& c : r.near)
        if (c.first <= r.cost * (1.0 + tol) && (int)near.size() < (tiny ? 4 : 3)) near.push_back(c.second);
      if (near.size() > 1) {
        float best = 1e30f;
        for (const auto& c : near) {
          const float ms = replay ? time_trial_schedule(c, tiny ? 5 : 1) : time_trial_eager(c, 2);
          if (tune_log())
            std::fprintf(stderr, "heat2d sched n=%lld %s trial %zu cycles of %d..%d: %.4f ms\n", (long long)n,
                         replay ? "graph" : "eager", c.size(), c.back(), c.front(), ms);
          if (ms < best) {
            best = ms;
            s = c;
          }
        }
      }
    }
    if (!s.empty()) {
      if (plancache::enabled()) plancache::put_schedule(sched_ctx(), n, s);
      sched_[n] = std::move(s);
    }
  }
  if (schedule(n) && replay_schedule(n)) {
    // both buffer parities (a warmup between prepare and step(n) may flip it);
    // a capture only records the launches, so flipping cur_ around it is safe
    for (int p = 0; p < 2; ++p) {
      cur_ ^= p;
      if (!sched_graph_.count({n, cur_})) capture_schedule(n);
      cur_ ^= p;
    }
  }
  if (const std::vector<int>* s = schedule(n)) {
    for (size_t i = 0; i < s->size(); ++i)
      (void)split_plan_banded((*s)[i], std::max((*s)[i], exchange_depth(*s, i, (*s)[0])));
    return;
  }
  // walk step(n)'s loop (graph pairs of depth K, then balanced eager cycles)
  // and plan every depth it will launch. Graph pairs start only at buffer
  // parity 0, so the depths depend on the parity step(n) starts from: walk
  // both, since a warmup between prepare() and step(n) may flip it (4096^2
  // fp32 graph, K = 6 / 14: an unplanned remainder depth autotuned inside the
  // timed run cost 10 ms of 16).
  for (int start = 0; start < 2; ++start) {
    const std::vector<CycleRun> runs = step_runs(n, start);
    for (size_t i = 0; i < runs.size(); ++i) {
      if (runs[i].pairs > 0) {
        ensure_pair_graph();
        continue;
      }
      const int x = tr_->exchanges() ? (i + 1 < runs.size() ? runs[i + 1].k : runs[0].k) : runs[i].k;
      (void)split_plan_banded(runs[i].k, std::max(runs[i].k, x));
    }
  }
}

void Solver::synchronize() {
  if (!hip_) return;
  H2D_HIP(hipSetDevice(cfg_.device));
  if (!tr_->exchanges()) {
    // (spin-polling here instead measured the same: headline 4750-4785 vs
    // 4737-4824, small grid 5489-5579 vs 5526-5562, profiles/r4/w/)
    H2D_HIP(hipStreamSynchronize(s_compute_));
    if (s_comm_ != s_compute_) H2D_HIP(hipStreamSynchronize(s_comm_));
    tr_->check();
    return;
  }
  // Exchanging ranks poll both streams, so that a transport abort (its
  // watchdog, or a failed peer in the same process) ends the wait with an
  // error instead of a hang: spinning on hipStreamQuery for the first 50 ms
  // (the end of a sub-ms timed cycle is seen within a microsecond), then 20 us
  // naps.
  const auto t0 = std::chrono::steady_clock::now();
  for (hipStream_t st : {s_compute_, s_comm_}) {
    hipError_t q;
    int spins = 0;
    bool nap = false;
    while ((q = hipStreamQuery(st)) == hipErrorNotReady) {
      if (tr_->aborted()) tr_->check();
      if (nap) std::this_thread::sleep_for(std::chrono::microseconds(20));
      else if ((++spins & 255) == 0) nap = std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(50);
    }
    H2D_HIP(q);
    if (s_comm_ == s_compute_) break;
  }
  tr_->check();
}

void Solver::step_stats(int64_t n, double out[6]) {
  HEAT2D_REQUIRE(n >= 1, "step_stats needs n >= 1");
  if (hip_) H2D_HIP(hipSetDevice(cfg_.device));
  if (!hip_ || jit_ || cfg_.copy_swap) {
    step(n - 1);
    step(1);
    stats(out, true);
    return;
  }
  // the cycles step(n) would run (the measured schedule, else balanced cycles
  // of the preferred depth), eagerly, the last one with the fused statistics
  std::vector<int> seq;
  if (const std::vector<int>* sc = schedule(n)) {
    seq = *sc;
  } else {
    for (int64_t left = n; left > 0;) {
      const int64_t ncyc = (left + k_pref_ - 1) / k_pref_;
      const int k = (int)(left / ncyc + (left % ncyc ? 1 : 0));
      seq.push_back(k);
      left -= k;
    }
  }
  topup(seq.front());
  for (size_t i = 0; i < seq.size(); ++i) {
    stats_next_ = i + 1 == seq.size();
    cycle_launch(seq[i], exchange_depth(seq, i, seq.front()));
    cycle_finish();
  }
  double loc[6];
  H2D_HIP(hipMemcpyAsync(loc, d_work_ + kern::stats_work_elems(), sizeof(loc), hipMemcpyDeviceToHost, s_compute_));
  synchronize();
  reduce_global(loc, out);
}

void Solver::reduce_global(const double loc[6], double out[6]) {
  double sums[3] = {loc[0], loc[1], loc[4]};
  double maxs[3] = {loc[3], loc[5], -loc[2]};
  tr_->allreduce(sums, 3, 0);
  tr_->allreduce(maxs, 3, 1);
  out[0] = sums[0];
  out[1] = sums[1];
  out[2] = -maxs[2];
  out[3] = maxs[0];
  out[4] = sums[2];
  out[5] = maxs[1];
}

void Solver::stats(double out[6], bool residual) {
  double loc[6];
  // the other buffer holds T_{n-1} only after a depth-1 cycle (or a copy-swap step)
  const bool one_step = cfg_.copy_swap || last_k_ == 1;
  const void* other = residual && one_step ? buf_[cur_ ^ 1] : nullptr;
  if (hip_) {
    synchronize();
    kern::launch_stats(dtype(), buf_[cur_], other, L_, d_work_, d_work_ + kern::stats_work_elems(), s_compute_);
    H2D_HIP(hipMemcpyAsync(loc, d_work_ + kern::stats_work_elems(), sizeof(loc), hipMemcpyDeviceToHost, s_compute_));
    H2D_HIP(hipStreamSynchronize(s_compute_));
  } else {
    cpu::stats(dtype(), buf_[cur_], other, L_, loc);
  }
  reduce_global(loc, out);
  if (residual && !one_step) out[4] = out[5] = std::nan("");
}

void Solver::download(void* host, int64_t ld) { download_region(0, L_.nrows, 0, L_.ncols, host, ld); }

void Solver::download_region(int64_t r0, int64_t r1, int64_t c0, int64_t c1, void* host, int64_t ld) {
  HEAT2D_REQUIRE(r0 >= -L_.halo && r1 <= L_.nrows + L_.halo && r0 <= r1, "row range outside allocation");
  HEAT2D_REQUIRE(c0 >= -L_.cpad && c1 <= L_.col_hi() && c0 <= c1, "column range outside allocation");
  if (r1 == r0 || c1 == c0) return;
  const size_t es = dtype_size(dtype());
  const char* src = static_cast<const char*>(buf_[cur_]) + (size_t)L_.offset(r0, c0) * es;
  const size_t w = (size_t)(c1 - c0) * es;
  if (hip_) {
    synchronize();
    H2D_HIP(hipMemcpy2DAsync(host, (size_t)ld * es, src, (size_t)L_.pitch * es, w, (size_t)(r1 - r0),
                             hipMemcpyDeviceToHost, s_compute_));
    H2D_HIP(hipStreamSynchronize(s_compute_));
  } else {
    for (int64_t i = 0; i < r1 - r0; ++i)
      std::memcpy(static_cast<char*>(host) + (size_t)(i * ld) * es, src + (size_t)(i * L_.pitch) * es, w);
  }
}

void Solver::compare(Solver& other, int64_t r0, int64_t nrows, int64_t other_r0, double out[2]) {
  const SlabLayout& Lo = other.layout();
  HEAT2D_REQUIRE(other.dtype() == dtype() && other.hip_ == hip_, "compared solvers differ in dtype or backend");
  HEAT2D_REQUIRE(Lo.ncols == L_.ncols, "compared solvers differ in width");
  HEAT2D_REQUIRE(nrows >= 0 && r0 >= 0 && r0 + nrows <= L_.nrows && other_r0 >= 0 && other_r0 + nrows <= Lo.nrows,
                 "compared rows outside the owned slabs");
  out[0] = out[1] = 0.0;
  if (nrows == 0) return;
  if (hip_) {
    HEAT2D_REQUIRE(other.cfg_.device == cfg_.device, "compared solvers live on different devices");
    other.synchronize();
    synchronize();
    double* res = d_work_ + kern::stats_work_elems();
    kern::launch_compare(dtype(), buf_[cur_], L_, r0, other.field(), Lo, other_r0, nrows, d_work_, res, s_compute_);
    H2D_HIP(hipMemcpyAsync(out, res, 2 * sizeof(double), hipMemcpyDeviceToHost, s_compute_));
    H2D_HIP(hipStreamSynchronize(s_compute_));
    return;
  }
  const size_t es = dtype_size(dtype());
  for (int64_t i = 0; i < nrows; ++i) {
    const char* pa = static_cast<const char*>(buf_[cur_]) + (size_t)L_.offset(r0 + i, 0) * es;
    const char* pb = static_cast<const char*>(other.field()) + (size_t)Lo.offset(other_r0 + i, 0) * es;
    for (int64_t j = 0; j < L_.ncols; ++j) {
      double x, y;
      if (dtype() == DType::F32) {
        x = reinterpret_cast<const float*>(pa)[j];
        y = reinterpret_cast<const float*>(pb)[j];
      } else {
        x = reinterpret_cast<const double*>(pa)[j];
        y = reinterpret_cast<const double*>(pb)[j];
      }
      const double d = std::fabs(x - y);
      if (d > out[0] || d != d) out[0] = std::isnan(out[0]) ? out[0] : d;
      out[1] += std::memcmp(pa + (size_t)j * es, pb + (size_t)j * es, es) != 0 ? 1.0 : 0.0;
    }
  }
}

void Solver::upload(const void* host, int64_t ld) {
  upload_owned(host, ld);
  exchange_post();
  exchange_now();
  synchronize();
}

void Solver::upload_owned(const void* host, int64_t ld) {
  const size_t es = dtype_size(dtype());
  char* dst = static_cast<char*>(buf_[cur_]) + (size_t)L_.origin() * es;
  if (hip_) {
    synchronize();
    H2D_HIP(hipMemcpy2DAsync(dst, (size_t)L_.pitch * es, host, (size_t)ld * es, (size_t)L_.ncols * es,
                             (size_t)L_.nrows, hipMemcpyHostToDevice, s_compute_));
  } else {
    for (int64_t i = 0; i < L_.nrows; ++i)
      std::memcpy(dst + (size_t)(i * L_.pitch) * es, static_cast<const char*>(host) + (size_t)(i * ld) * es,
                  (size_t)L_.ncols * es);
  }
}

// ------------------------------------------------------------------ loopback

LoopbackGroup::LoopbackGroup(const SolverConfig& cfg, int nranks) {
  HEAT2D_REQUIRE(nranks >= 1, "nranks >= 1");
  // every member owns its streams, events, split plans and autotuner, exactly
  // like one rank of a multi-GPU run; only the transport differs
  auto trs = make_loopback_transports(nranks);
  for (int i = 0; i < nranks; ++i) members_.emplace_back(new Solver(cfg, trs[(size_t)i]));
}

LoopbackGroup::~LoopbackGroup() {
  try {
    synchronize();
  } catch (...) {
  }
  members_.clear();
}

void LoopbackGroup::init(const kern::IcParams& ic, const double* xg, const double* yg) {
  for (auto& m : members_) m->init(ic, xg, yg);
}

// step()'s loop (balanced depths; no graphs: a capture cannot span the
// members' streams) with the two phases of every cycle interleaved across
// members: all launches (each posts its new field and band event), then all
// exchanges — the order a multi-process run gets from RCCL's rendezvous.
void LoopbackGroup::step(int64_t n) {
  if (n <= 0) return;
  const int K = members_[0]->pref_depth();
  std::vector<int> seq;
  for (int64_t left = n; left > 0;) {
    const int64_t ncyc = (left + K - 1) / K;
    const int k = (int)(left / ncyc + (left % ncyc ? 1 : 0));
    seq.push_back(k);
    left -= k;
  }
  // deeper first cycle than the last exchange moved: every member posts its
  // current field, then every member pulls (Solver::topup's two phases)
  if (members_[0]->needs_topup(seq[0])) {
    for (auto& m : members_) m->synchronize();
    for (auto& m : members_) m->exchange_post();
    for (auto& m : members_) m->exchange_now(seq[0]);
    synchronize();
  }
  for (size_t i = 0; i < seq.size(); ++i) {
    const int x = exchange_depth(seq, i, seq[0]);
    for (auto& m : members_) m->cycle_launch(seq[i], x);
    for (auto& m : members_) m->cycle_finish();
  }
}

void LoopbackGroup::upload(const void* host, int64_t ld) {
  const size_t es = dtype_size(members_[0]->dtype());
  for (auto& m : members_) {
    m->synchronize();
    m->upload_owned(static_cast<const char*>(host) + (size_t)(m->layout().row0 * ld) * es, ld);
  }
  for (auto& m : members_) m->exchange_post();
  for (auto& m : members_) m->exchange_now();
  synchronize();
}

void LoopbackGroup::synchronize() {
  for (auto& m : members_) m->synchronize();
}

void LoopbackGroup::download(void* host, int64_t ld) {
  const size_t es = dtype_size(members_[0]->dtype());
  for (auto& m : members_) {
    const SlabLayout& L = m->layout();
    m->download(static_cast<char*>(host) + (size_t)(L.row0 * ld) * es, ld);
  }
}

}  // namespace heat2d
