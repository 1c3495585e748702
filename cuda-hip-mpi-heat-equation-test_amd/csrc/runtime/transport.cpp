// Transports for the slab halo exchange.
//
// The reference does, per step and per rank: pack kernel -> device sync ->
// 2 D2H copies -> 2 blocking MPI_Sendrecv -> 2 H2D copies -> 2 unpack kernels
// (fortran/hip/heat.F90:196-230; CUDA-aware variant fortran/mpi+cuda/heat.F90:169-171).
// Here the halo rows are contiguous in memory, so the RCCL transport sends
// and receives them in place (no pack, no host staging) as ONE grouped
// send/recv on a stream that the solver orders against its kernels with
// events. xGMI is point-to-point: a 1-D slab talks to exactly two peers over
// two direct links.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "heat2d/runtime.hpp"
#include "heat2d/watchdog.hpp"

namespace heat2d {

#define H2D_HIP(expr)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess) fail(__FILE__, __LINE__, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

#define H2D_NCCL(expr)                                                                  \
  do {                                                                                  \
    ncclResult_t r_ = (expr);                                                           \
    if (r_ != ncclSuccess) fail(__FILE__, __LINE__, std::string(#expr) + ": " + ncclGetErrorString(r_)); \
  } while (0)

namespace {

// ------------------------------------------------------------------ self (P=1)
class SelfTransport final : public Transport {
 public:
  int rank() const override { return 0; }
  int size() const override { return 1; }
  void exchange(void*, const SlabLayout&, DType, int64_t, hipStream_t, bool) override {}
  void allreduce(double*, int, int) override {}
  void barrier() override {}
  std::string name() const override { return "self"; }
  bool capturable() const override { return true; }
};

// ------------------------------------------------------------------ RCCL
// Failure detection: every exchange / all-reduce records a completion event;
// a Watchdog thread polls them and ncclCommGetAsyncError. Outstanding
// exchanges with none completing for HEAT2D_COMM_TIMEOUT seconds (default
// 600), or an RCCL async error, abort the communicator (ncclCommAbort: the
// blocked RCCL kernels and host waits return) and the next check() — every
// Solver::synchronize — raises with the rank and the reason.
class RcclTransport final : public Transport {
 public:
  RcclTransport(const void* uid, int rank, int size, int device, bool loop = false)
      : rank_(rank), size_(size), loop_(loop && size == 1) {
    if (device >= 0) H2D_HIP(hipSetDevice(device));
    H2D_HIP(hipGetDevice(&device_));
    ncclUniqueId id;
    std::memcpy(&id, uid, sizeof(id));
    H2D_NCCL(ncclCommInitRank(&comm_, size, id, rank));
    H2D_HIP(hipStreamCreateWithFlags(&aux_, hipStreamNonBlocking));
    H2D_HIP(hipMalloc(&d_scratch_, 64 * sizeof(double)));
    const double timeout = Watchdog::env_timeout(600.0);
    if (timeout > 0 && (size_ > 1 || loop_))
      wd_.reset(new Watchdog(
          timeout, 0.05, [this](std::string* d) { return poll(d); }, [this](const std::string& r) { abort(r); }));
  }
  ~RcclTransport() override {
    wd_.reset();  // stop the watchdog before anything it polls goes away
    if (comm_) ncclCommDestroy(comm_);
    for (auto& p : pend_) (void)hipEventDestroy(p.ev);
    for (auto e : pool_) (void)hipEventDestroy(e);
    if (d_scratch_) (void)hipFree(d_scratch_);
    if (aux_) (void)hipStreamDestroy(aux_);
    (void)hipGetLastError();  // teardown errors must not surface as the next launch's
  }
  int rank() const override { return rank_; }
  int size() const override { return size_; }
  std::string name() const override { return loop_ ? "rccl-loop" : "rccl"; }
  // Not captured into hipGraphs: capturing the grouped ncclSend/ncclRecv of
  // the overlapped cycle segfaults inside step() on the MI355X box (RCCL
  // 2.26.6, 1-rank self-loop, tools/graph_rccl_probe.py, either split order),
  // also with the watchdog's event tracking kept out of the capture (track()
  // skips capturing streams) — the fault is inside RCCL's captured send/recv
  // path. --graph therefore runs eager cycles whenever RCCL exchanges halos
  // (single-rank runs use graphs).
  bool capturable() const override { return false; }
  void graph_launched(hipStream_t stream) override { track(stream, "graph replay"); }
  bool exchanges() const override { return size_ > 1 || loop_; }
  bool aborted() const override { return aborted_.load(); }
  // collectives of an I/O phase wait on peers' host I/O: not tracked (a slow
  // output turn is not a hung fabric); exchanges are never issued inside one
  void io_phase(bool on) override { io_ += on ? 1 : -1; }

  FabricInfo fabric_info() override {
    std::unique_lock<std::timed_mutex> lk(cmu_);
    live();
    int n = 0, r = 0, d = -1;
    H2D_NCCL(ncclCommCount(comm_, &n));
    H2D_NCCL(ncclCommUserRank(comm_, &r));
    H2D_NCCL(ncclCommCuDevice(comm_, &d));
    return {1, n, r, d};
  }

  void check() override {
    if (aborted_) fail_aborted();
    std::unique_lock<std::timed_mutex> lk(cmu_);
    live();  // an abort between the test above and the lock: report it, not a null communicator
    ncclResult_t st = ncclSuccess;
    H2D_NCCL(ncclCommGetAsyncError(comm_, &st));
    if (st != ncclSuccess && st != ncclInProgress)
      fail(__FILE__, __LINE__, std::string("RCCL communicator failed asynchronously: ") + ncclGetErrorString(st) +
                                   " (rank " + std::to_string(rank_) + " of " + std::to_string(size_) + ")");
  }

  void abort(const std::string& reason) override {
    bool expect = false;
    if (!aborted_.compare_exchange_strong(expect, true)) return;
    {
      std::lock_guard<std::mutex> g(pmu_);
      abort_reason_ = reason;
    }
    // the comm lock keeps a host thread from entering RCCL on a freed
    // communicator; if the host thread is itself stuck inside an RCCL call
    // (holding it), abort anyway: that is the hang being broken
    std::unique_lock<std::timed_mutex> lk(cmu_, std::defer_lock);
    (void)lk.try_lock_for(std::chrono::seconds(2));
    if (comm_) {
      (void)ncclCommAbort(comm_);
      comm_ = nullptr;
    }
  }

  void exchange(void* field, const SlabLayout& L, DType dt, int64_t k, hipStream_t stream,
                bool on_device) override {
    HEAT2D_REQUIRE(on_device, "RCCL transport needs device-resident fields");
    if ((size_ == 1 && !loop_) || k <= 0) return;
    const size_t es = dtype_size(dt);
    char* base = static_cast<char*>(field);
    const size_t count = halo_msg_bytes(L, k, es) / es;  // whole padded rows: contiguous, zero-copy
    const ncclDataType_t t = dt == DType::F32 ? ncclFloat32 : ncclFloat64;
    HaloMsg msg[2];
    int nmsg = 0;
    if (loop_) {  // periodic self-exchange (rehearsal): the two messages of an interior rank, both to itself
      nmsg = halo_msgs(1, 3, L, k, msg);
      for (int i = 0; i < nmsg; ++i) msg[i].peer = 0;
      std::swap(msg[0].recv_row, msg[1].recv_row);  // the wrap: row 0 lands above the top, the top below row 0
    } else {
      nmsg = halo_msgs(rank_, size_, L, k, msg);
    }
    {
      std::unique_lock<std::timed_mutex> lk(cmu_);
      live();
      H2D_NCCL(ncclGroupStart());
      for (int i = 0; i < nmsg; ++i) {
        H2D_NCCL(ncclSend(base + halo_row_bytes(L, msg[i].send_row, es), count, t, msg[i].peer, comm_, stream));
        H2D_NCCL(ncclRecv(base + halo_row_bytes(L, msg[i].recv_row, es), count, t, msg[i].peer, comm_, stream));
      }
      H2D_NCCL(ncclGroupEnd());
    }
    track(stream, "halo exchange");
  }

  void allreduce(double* vals, int n, int op) override {
    HEAT2D_REQUIRE(n <= 64, "allreduce too large");
    H2D_HIP(hipSetDevice(device_));
    H2D_HIP(hipMemcpyAsync(d_scratch_, vals, n * sizeof(double), hipMemcpyHostToDevice, aux_));
    const ncclRedOp_t o = op == 0 ? ncclSum : (op == 1 ? ncclMax : ncclMin);
    {
      std::unique_lock<std::timed_mutex> lk(cmu_);
      live();
      H2D_NCCL(ncclAllReduce(d_scratch_, d_scratch_, n, ncclFloat64, o, comm_, aux_));
    }
    track(aux_, "all-reduce");
    H2D_HIP(hipMemcpyAsync(vals, d_scratch_, n * sizeof(double), hipMemcpyDeviceToHost, aux_));
    // poll instead of blocking, so an abort by the watchdog ends the wait
    hipError_t q;
    while ((q = hipStreamQuery(aux_)) == hipErrorNotReady) {
      if (aborted_) check();
      std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    H2D_HIP(q);
    check();
  }
  void barrier() override {
    double v = 0.0;
    allreduce(&v, 1, 0);
  }

 private:
  [[noreturn]] void fail_aborted() {
    std::string why;
    {
      std::lock_guard<std::mutex> g(pmu_);
      why = abort_reason_;
    }
    fail(__FILE__, __LINE__, "RCCL communicator aborted (rank " + std::to_string(rank_) + " of " +
                                 std::to_string(size_) + "): " + why);
  }
  void live() {  // with cmu_ held
    if (aborted_ || !comm_) fail_aborted();
  }
  // record a completion event of the operation just enqueued on `s` (watchdog)
  void track(hipStream_t s, const char* what) {
    if (!wd_ || io_.load() > 0) return;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    H2D_HIP(hipStreamIsCapturing(s, &cs));
    if (cs != hipStreamCaptureStatusNone) return;  // inside a capture: the replay is tracked
    std::lock_guard<std::mutex> g(pmu_);
    if (pend_.size() >= 4096) return;  // the host is far ahead: the oldest ones tell the story
    hipEvent_t e = nullptr;
    if (!pool_.empty()) {
      e = pool_.back();
      pool_.pop_back();
    } else {
      H2D_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    H2D_HIP(hipEventRecord(e, s));
    pend_.push_back(Pend{e, ++nops_, what});
  }
  // watchdog thread: completions since the last poll
  Watchdog::Status poll(std::string* detail) {
    if (aborted_) return Watchdog::Idle;
    static thread_local int dev_set = -1;
    if (dev_set != device_) {
      (void)hipSetDevice(device_);
      dev_set = device_;
    }
    {
      std::unique_lock<std::timed_mutex> lk(cmu_, std::defer_lock);
      if (lk.try_lock_for(std::chrono::milliseconds(10)) && comm_) {
        ncclResult_t st = ncclSuccess;
        if (ncclCommGetAsyncError(comm_, &st) == ncclSuccess && st != ncclSuccess && st != ncclInProgress) {
          *detail = std::string("ncclCommGetAsyncError: ") + ncclGetErrorString(st);
          return Watchdog::Error;
        }
      }
    }
    std::lock_guard<std::mutex> g(pmu_);
    int done = 0;
    while (!pend_.empty()) {
      const hipError_t q = hipEventQuery(pend_.front().ev);
      if (q == hipErrorNotReady) break;
      if (q != hipSuccess) {
        *detail = std::string("hipEventQuery: ") + hipGetErrorString(q);
        return Watchdog::Error;
      }
      pool_.push_back(pend_.front().ev);
      pend_.pop_front();
      ++done;
    }
    if (done) return Watchdog::Progress;
    if (pend_.empty()) return Watchdog::Idle;
    *detail = std::string(pend_.front().what) + " #" + std::to_string(pend_.front().seq) + " of rank " +
              std::to_string(rank_) + " of " + std::to_string(size_) + " still pending";
    return Watchdog::Pending;
  }

  struct Pend {
    hipEvent_t ev;
    int64_t seq;
    const char* what;
  };
  int rank_, size_;
  bool loop_ = false;
  int device_ = 0;
  ncclComm_t comm_ = nullptr;
  hipStream_t aux_ = nullptr;
  double* d_scratch_ = nullptr;
  std::timed_mutex cmu_;  // comm_ vs the watchdog's abort
  std::mutex pmu_;        // pend_ / pool_ / abort_reason_
  std::deque<Pend> pend_;
  std::vector<hipEvent_t> pool_;
  int64_t nops_ = 0;
  std::atomic<bool> aborted_{false};
  std::atomic<int> io_{0};
  std::string abort_reason_;
  std::unique_ptr<Watchdog> wd_;
};

// ------------------------------------------------------------------ callbacks
// Host-side transport driven by function pointers (Python: torch.distributed
// gloo for CPU-only multi-process tests; anything else a user plugs in).
class CallbackTransport final : public Transport {
 public:
  CallbackTransport(const CallbackOps& ops, int rank, int size) : ops_(ops), rank_(rank), size_(size) {}
  ~CallbackTransport() override {
    if (ev_) {
      (void)hipEventSynchronize(ev_);
      (void)hipEventDestroy(ev_);
    }
    if (d_stage_) (void)hipFree(d_stage_);
    if (h_stage_) (void)hipHostFree(h_stage_);
  }
  int rank() const override { return rank_; }
  int size() const override { return size_; }
  std::string name() const override { return "callback"; }

  void exchange(void* field, const SlabLayout& L, DType dt, int64_t k, hipStream_t stream,
                bool on_device) override {
    if (size_ == 1 || k <= 0) return;
    const size_t es = dtype_size(dt);
    const int64_t count = k * L.ncols;
    const size_t bytes = (size_t)(4 * count) * es;
    const bool has_lo = rank_ > 0, has_hi = rank_ < size_ - 1;
    if (on_device) {
      // device -> pinned host staging (the reference's path, kept for generic
      // transports): buffers grow once and are reused; the previous
      // exchange's H2D copies must have drained before the host reuses them
      if (ev_) H2D_HIP(hipEventSynchronize(ev_));
      else H2D_HIP(hipEventCreateWithFlags(&ev_, hipEventDisableTiming));
      if (bytes > cap_) {
        if (d_stage_) H2D_HIP(hipFree(d_stage_));
        if (h_stage_) H2D_HIP(hipHostFree(h_stage_));
        H2D_HIP(hipMalloc(&d_stage_, bytes));
        H2D_HIP(hipHostMalloc(&h_stage_, bytes, hipHostMallocDefault));
        cap_ = bytes;
      }
      char* h = static_cast<char*>(h_stage_);
      char* d = static_cast<char*>(d_stage_);
      const size_t half = (size_t)(2 * count) * es;  // [send_lo | send_hi | recv_lo | recv_hi]
      if (has_lo) kern::launch_pack_rows(dt, field, L, 0, k, d, stream);
      if (has_hi) kern::launch_pack_rows(dt, field, L, L.nrows - k, k, d + count * es, stream);
      H2D_HIP(hipMemcpyAsync(h, d, half, hipMemcpyDeviceToHost, stream));
      H2D_HIP(hipStreamSynchronize(stream));
      int rc = ops_.exchange(ops_.ctx, has_lo ? h : nullptr, has_hi ? h + count * es : nullptr,
                             has_lo ? h + half : nullptr, has_hi ? h + half + count * es : nullptr, count, (int32_t)dt);
      HEAT2D_REQUIRE(rc == 0, "exchange callback failed");
      H2D_HIP(hipMemcpyAsync(d + half, h + half, half, hipMemcpyHostToDevice, stream));
      if (has_lo) kern::launch_unpack_rows(dt, field, L, -k, k, d + half, stream);
      if (has_hi) kern::launch_unpack_rows(dt, field, L, L.nrows, k, d + half + count * es, stream);
      H2D_HIP(hipEventRecord(ev_, stream));  // no host sync: the next exchange waits on it
    } else {
      stage_.resize(bytes);
      char* s_lo = stage_.data();
      char* s_hi = s_lo + count * es;
      char* r_lo = s_hi + count * es;
      char* r_hi = r_lo + count * es;
      if (has_lo) cpu::pack_rows(dt, field, L, 0, k, s_lo);
      if (has_hi) cpu::pack_rows(dt, field, L, L.nrows - k, k, s_hi);
      int rc = ops_.exchange(ops_.ctx, has_lo ? s_lo : nullptr, has_hi ? s_hi : nullptr,
                             has_lo ? r_lo : nullptr, has_hi ? r_hi : nullptr, count, (int32_t)dt);
      HEAT2D_REQUIRE(rc == 0, "exchange callback failed");
      if (has_lo) cpu::unpack_rows(dt, field, L, -k, k, r_lo);
      if (has_hi) cpu::unpack_rows(dt, field, L, L.nrows, k, r_hi);
    }
  }
  void allreduce(double* vals, int n, int op) override {
    if (size_ == 1) return;
    HEAT2D_REQUIRE(ops_.allreduce(ops_.ctx, vals, n, op) == 0, "allreduce callback failed");
  }
  void barrier() override {
    if (size_ == 1) return;
    HEAT2D_REQUIRE(ops_.barrier(ops_.ctx) == 0, "barrier callback failed");
  }

 private:
  CallbackOps ops_;
  int rank_, size_;
  std::vector<char> stage_;      // host fields
  void* d_stage_ = nullptr;      // device fields: [send_lo | send_hi | recv_lo | recv_hi]
  void* h_stage_ = nullptr;      // pinned host mirror of d_stage_
  size_t cap_ = 0;
  hipEvent_t ev_ = nullptr;      // end of the last exchange's H2D copies
};

// ------------------------------------------------------------------ loopback
// P ranks of one process, halos copied on the RECEIVING rank's exchange
// stream (a pull): the messages are halo_msgs' — the ones RCCL moves — and the
// cross-rank ordering RCCL's rendezvous provides is rebuilt from events:
//   * a pull of cycle c waits for the peer's band event of cycle c (its post),
//   * and for the peer's own pulls of cycle c-1 (done[(c-1) & 1]), which read
//     this rank's band rows of the buffer this rank's bands of cycle c+1 will
//     overwrite — those bands sit behind this exchange in stream order (on the
//     comm stream, or, edge-first, behind ev_comm on the compute stream).
// Both hold because LoopbackGroup posts every rank's cycle c before it
// enqueues any rank's exchange of cycle c.
struct LoopbackHub {
  struct Slot {
    void* field = nullptr;  // posted field of the current cycle
    SlabLayout L{};
    hipEvent_t ready = nullptr;  // the poster's band event (not owned)
    hipEvent_t done[2] = {nullptr, nullptr};  // owned: pulls of cycle parity p done
    int64_t posted = 0, pulled = 0;  // cycles posted / exchanged
  };
  explicit LoopbackHub(int n) : slot((size_t)n) {}
  ~LoopbackHub() {
    for (auto& s : slot)
      for (auto& e : s.done)
        if (e) (void)hipEventDestroy(e);
  }
  std::vector<Slot> slot;
};

class LoopbackTransport final : public Transport {
 public:
  LoopbackTransport(std::shared_ptr<LoopbackHub> hub, int rank) : hub_(std::move(hub)), rank_(rank) {}
  int rank() const override { return rank_; }
  int size() const override { return (int)hub_->slot.size(); }
  std::string name() const override { return "loopback"; }
  // the members share one host thread: collectives over them are the group's job
  bool collective() const override { return false; }
  void allreduce(double*, int, int) override {}
  void barrier() override {}

  void post(void* field, const SlabLayout& L, hipEvent_t ready) override {
    auto& me = hub_->slot[(size_t)rank_];
    HEAT2D_REQUIRE(me.posted == me.pulled, "loopback: a cycle was posted twice without an exchange");
    me.field = field;
    me.L = L;
    me.ready = ready;
    ++me.posted;
  }

  void exchange(void* field, const SlabLayout& L, DType dt, int64_t k, hipStream_t stream,
                bool on_device) override {
    if (size() == 1 || k <= 0) return;
    auto& me = hub_->slot[(size_t)rank_];
    HEAT2D_REQUIRE(me.posted == me.pulled + 1 && me.field == field,
                   "loopback: exchange of a field that was not posted this cycle (drive members through LoopbackGroup)");
    const int64_t c = me.pulled;
    const size_t es = dtype_size(dt);
    const size_t bytes = halo_msg_bytes(L, k, es);
    HaloMsg msg[2];
    const int nmsg = halo_msgs(rank_, size(), L, k, msg);
    if (on_device) {
      for (auto& e : me.done)
        if (!e) H2D_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    for (int i = 0; i < nmsg; ++i) {
      const auto& peer = hub_->slot[(size_t)msg[i].peer];
      HEAT2D_REQUIRE(peer.posted == c + 1, "loopback: peer has not posted this cycle");
      HEAT2D_REQUIRE(peer.L.pitch == L.pitch, "loopback: slabs of different pitch");
      // the peer's message toward this rank: its send rows
      HaloMsg pm[2];
      const int np = halo_msgs(msg[i].peer, size(), peer.L, k, pm);
      int64_t send_row = -1;
      for (int j = 0; j < np; ++j)
        if (pm[j].peer == rank_) send_row = pm[j].send_row;
      HEAT2D_REQUIRE(send_row >= 0, "loopback: peer does not send to this rank");
      const char* src = static_cast<const char*>(peer.field) + halo_row_bytes(peer.L, send_row, es);
      char* dst = static_cast<char*>(field) + halo_row_bytes(L, msg[i].recv_row, es);
      if (on_device) {
        H2D_HIP(hipStreamWaitEvent(stream, peer.ready, 0));
        if (c > 0 && peer.done[(c - 1) & 1]) H2D_HIP(hipStreamWaitEvent(stream, peer.done[(c - 1) & 1], 0));
        H2D_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, stream));
      } else {
        std::memcpy(dst, src, bytes);
      }
    }
    if (on_device) H2D_HIP(hipEventRecord(me.done[c & 1], stream));
    ++me.pulled;
  }

 private:
  std::shared_ptr<LoopbackHub> hub_;
  int rank_;
};

// ------------------------------------------------------------------ host threads
// P ranks as host threads of one process with host-memory fields (the CPU
// twin): the native CLI's `--cpu --gpus P`, the reference's `make mpi` CPU
// MPI build (fortran/mpi+cuda/makefile:1-2). An exchange publishes this
// rank's field, meets the others at a barrier, copies its ghost rows straight
// out of the neighbours' fields (halo_msgs, as RCCL), and meets them again
// before anyone overwrites a field. Barriers time out after
// HEAT2D_COMM_TIMEOUT seconds and can be aborted (a failed rank), so a dead
// or failed thread never leaves the others blocked.
struct ThreadHub {
  explicit ThreadHub(int n) : n(n), field((size_t)n), layout((size_t)n), vals((size_t)n * 64) {
    timeout = Watchdog::env_timeout(600.0);
  }
  // io: an I/O-phase barrier (Transport::io_phase) — a peer may be writing
  // its output for long, so no timeout (abort() still wakes it)
  void barrier(int rank, bool io = false) {
    std::unique_lock<std::mutex> lk(mu);
    if (aborted) throw_aborted(rank);
    const int64_t g = gen;
    if (++count == n) {
      count = 0;
      ++gen;
      cv.notify_all();
      return;
    }
    const auto pred = [&] { return gen != g || aborted; };
    if (timeout > 0 && !io) {
      if (!cv.wait_for(lk, std::chrono::duration<double>(timeout), pred)) {
        aborted = true;
        reason = "rank " + std::to_string(rank) + " waited " + std::to_string(timeout) +
                 " s at a barrier (HEAT2D_COMM_TIMEOUT): a peer rank is dead or hung";
        cv.notify_all();
      }
    } else {
      cv.wait(lk, pred);
    }
    if (aborted) throw_aborted(rank);
  }
  void abort(const std::string& why) {
    std::lock_guard<std::mutex> g(mu);
    if (!aborted) reason = why;
    aborted = true;
    cv.notify_all();
  }
  [[noreturn]] void throw_aborted(int rank) {
    fail(__FILE__, __LINE__, "host-thread transport aborted (rank " + std::to_string(rank) + " of " +
                                 std::to_string(n) + "): " + reason);
  }
  const int n;
  double timeout = 0;
  std::mutex mu;
  std::condition_variable cv;
  int64_t gen = 0;
  int count = 0;
  bool aborted = false;
  std::string reason;
  std::vector<char*> field;
  std::vector<SlabLayout> layout;
  std::vector<double> vals;  // allreduce slots, 64 per rank
};

class ThreadTransport final : public Transport {
 public:
  ThreadTransport(std::shared_ptr<ThreadHub> hub, int rank) : hub_(std::move(hub)), rank_(rank) {}
  int rank() const override { return rank_; }
  int size() const override { return hub_->n; }
  std::string name() const override { return "host-threads"; }
  void io_phase(bool on) override { io_ += on ? 1 : -1; }
  void abort(const std::string& reason) override { hub_->abort(reason); }
  bool aborted() const override {
    std::lock_guard<std::mutex> g(hub_->mu);
    return hub_->aborted;
  }
  void check() override {
    std::unique_lock<std::mutex> lk(hub_->mu);
    if (hub_->aborted) hub_->throw_aborted(rank_);
  }

  void exchange(void* field, const SlabLayout& L, DType dt, int64_t k, hipStream_t, bool on_device) override {
    HEAT2D_REQUIRE(!on_device, "the host-thread transport moves host-memory fields (CPU backend)");
    if (size() == 1 || k <= 0) return;
    hub_->field[(size_t)rank_] = static_cast<char*>(field);
    hub_->layout[(size_t)rank_] = L;
    hub_->barrier(rank_);  // every rank's new field is published
    const size_t es = dtype_size(dt);
    HaloMsg msg[2];
    const int nmsg = halo_msgs(rank_, size(), L, k, msg);
    for (int i = 0; i < nmsg; ++i) {
      const int p = msg[i].peer;
      const SlabLayout& PL = hub_->layout[(size_t)p];
      HEAT2D_REQUIRE(PL.pitch == L.pitch, "slabs of different pitch");
      HaloMsg pm[2];
      const int np = halo_msgs(p, size(), PL, k, pm);
      for (int j = 0; j < np; ++j)
        if (pm[j].peer == rank_)
          std::memcpy(static_cast<char*>(field) + halo_row_bytes(L, msg[i].recv_row, es),
                      hub_->field[(size_t)p] + halo_row_bytes(PL, pm[j].send_row, es), halo_msg_bytes(L, k, es));
    }
    hub_->barrier(rank_);  // nobody moves on (and overwrites its field) before all copies are done
  }
  void allreduce(double* vals, int n, int op) override {
    HEAT2D_REQUIRE(n <= 64, "allreduce too large");
    if (size() == 1) return;
    std::copy(vals, vals + n, hub_->vals.begin() + (ptrdiff_t)rank_ * 64);
    hub_->barrier(rank_, io_ > 0);
    for (int j = 0; j < n; ++j) {  // same fixed order on every rank: identical results
      double a = hub_->vals[(size_t)j];
      for (int r = 1; r < size(); ++r) {
        const double b = hub_->vals[(size_t)r * 64 + j];
        a = op == 0 ? a + b : (op == 1 ? std::max(a, b) : std::min(a, b));
      }
      vals[j] = a;
    }
    hub_->barrier(rank_, io_ > 0);
  }
  void barrier() override { hub_->barrier(rank_, io_ > 0); }

 private:
  std::shared_ptr<ThreadHub> hub_;
  int rank_;
  int io_ = 0;
};

// ------------------------------------------------------------------ peer
// P ranks as host threads of one process, each on its own GPU (or sharing one:
// the native CLI's --share-gpu), device fields, NO RCCL: every halo is pulled
// by the receiving rank on its exchange stream with a device-to-device
// hipMemcpyAsync straight out of the neighbour's field (peer access over xGMI
// between GPUs: a copy, not a send/recv kernel competing for wave slots with
// the persistent interior, profiles/thin_slab.md §7-§8). The ordering is the
// loopback transport's event protocol (a pull of cycle c waits for the peer's
// band event of cycle c and for the peer's own pulls of cycle c-1); threads add
// host-side waits so that those events are RECORDED before anyone waits on
// them: a pull of cycle c starts once the peer has posted cycle c and enqueued
// its pulls of cycle c-1. A peer runs at most one cycle ahead (its pull of
// c+1 needs this rank's post of c+1), so its posted fields are kept per cycle
// parity; waiting on a newer record of its band / done events is only
// conservative. Barrier / all-reduce / abort / timeout: ThreadHub.
struct PeerHub : ThreadHub {
  struct Slot {
    void* field[2] = {nullptr, nullptr};  // posted field of cycle c at [c & 1]
    SlabLayout L{};
    hipEvent_t ready = nullptr;  // the poster's band event (not owned)
    hipEvent_t done[2] = {nullptr, nullptr};  // owned: pulls of cycle parity p done
    int device = -1;
    int64_t posted = 0, pulled = 0;
  };
  explicit PeerHub(int n) : ThreadHub(n), slot((size_t)n) {}
  ~PeerHub() {
    for (auto& sl : slot)
      for (auto& e : sl.done)
        if (e) (void)hipEventDestroy(e);
  }
  std::vector<Slot> slot;
  std::mutex peer_mu;  // device pairs with peer access enabled
  std::vector<std::pair<int, int>> peer_on;
};

class PeerTransport final : public Transport {
 public:
  PeerTransport(std::shared_ptr<PeerHub> hub, int rank) : hub_(std::move(hub)), rank_(rank) {}
  int rank() const override { return rank_; }
  int size() const override { return hub_->n; }
  std::string name() const override { return "peer"; }
  void io_phase(bool on) override { io_ += on ? 1 : -1; }
  void abort(const std::string& reason) override { hub_->abort(reason); }
  bool aborted() const override {
    std::lock_guard<std::mutex> g(hub_->mu);
    return hub_->aborted;
  }
  void check() override {
    std::unique_lock<std::mutex> lk(hub_->mu);
    if (hub_->aborted) hub_->throw_aborted(rank_);
  }

  void post(void* field, const SlabLayout& L, hipEvent_t ready) override {
    int dev = 0;
    H2D_HIP(hipGetDevice(&dev));
    std::lock_guard<std::mutex> g(hub_->mu);
    auto& me = hub_->slot[(size_t)rank_];
    HEAT2D_REQUIRE(me.posted == me.pulled, "peer: a cycle was posted twice without an exchange");
    me.field[me.posted & 1] = field;
    me.L = L;
    me.ready = ready;
    me.device = dev;
    ++me.posted;
    hub_->cv.notify_all();
  }

  void exchange(void* field, const SlabLayout& L, DType dt, int64_t k, hipStream_t stream,
                bool on_device) override {
    HEAT2D_REQUIRE(on_device, "the peer transport moves device fields");
    if (size() == 1 || k <= 0) return;
    auto& me = hub_->slot[(size_t)rank_];
    int dev = 0;
    H2D_HIP(hipGetDevice(&dev));
    int64_t c;
    {
      std::lock_guard<std::mutex> g(hub_->mu);
      HEAT2D_REQUIRE(me.posted == me.pulled + 1 && me.field[me.pulled & 1] == field,
                     "peer: exchange of a field that was not posted this cycle");
      c = me.pulled;
    }
    for (auto& e : me.done)
      if (!e) H2D_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    const size_t es = dtype_size(dt);
    const size_t bytes = halo_msg_bytes(L, k, es);
    HaloMsg msg[2];
    const int nmsg = halo_msgs(rank_, size(), L, k, msg);
    for (int i = 0; i < nmsg; ++i) {
      const int p = msg[i].peer;
      PeerHub::Slot peer;
      {  // the peer's post of cycle c and its pulls of cycle c-1 are enqueued
        std::unique_lock<std::mutex> lk(hub_->mu);
        const auto& ps = hub_->slot[(size_t)p];
        const auto pred = [&] { return (ps.posted >= c + 1 && ps.pulled >= c) || hub_->aborted; };
        if (hub_->timeout > 0) {
          if (!hub_->cv.wait_for(lk, std::chrono::duration<double>(hub_->timeout), pred)) {
            hub_->aborted = true;
            hub_->reason = "rank " + std::to_string(rank_) + " waited " + std::to_string(hub_->timeout) +
                           " s for rank " + std::to_string(p) + "'s halo (HEAT2D_COMM_TIMEOUT)";
            hub_->cv.notify_all();
          }
        } else {
          hub_->cv.wait(lk, pred);
        }
        if (hub_->aborted) hub_->throw_aborted(rank_);
        peer = ps;
      }
      HEAT2D_REQUIRE(peer.L.pitch == L.pitch, "peer: slabs of different pitch");
      HaloMsg pm[2];
      const int np = halo_msgs(p, size(), peer.L, k, pm);
      int64_t send_row = -1;
      for (int j = 0; j < np; ++j)
        if (pm[j].peer == rank_) send_row = pm[j].send_row;
      HEAT2D_REQUIRE(send_row >= 0, "peer: neighbour does not send to this rank");
      if (peer.device != dev) enable_peer(dev, peer.device);
      const char* src = static_cast<const char*>(peer.field[c & 1]) + halo_row_bytes(peer.L, send_row, es);
      char* dst = static_cast<char*>(field) + halo_row_bytes(L, msg[i].recv_row, es);
      H2D_HIP(hipStreamWaitEvent(stream, peer.ready, 0));
      if (c > 0) H2D_HIP(hipStreamWaitEvent(stream, peer.done[(c - 1) & 1], 0));
      H2D_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, stream));
    }
    H2D_HIP(hipEventRecord(me.done[c & 1], stream));
    std::lock_guard<std::mutex> g(hub_->mu);
    ++me.pulled;
    hub_->cv.notify_all();
  }

  void allreduce(double* vals, int n, int op) override {
    HEAT2D_REQUIRE(n <= 64, "allreduce too large");
    if (size() == 1) return;
    std::copy(vals, vals + n, hub_->vals.begin() + (ptrdiff_t)rank_ * 64);
    hub_->barrier(rank_, io_ > 0);
    for (int j = 0; j < n; ++j) {  // same fixed order on every rank: identical results
      double a = hub_->vals[(size_t)j];
      for (int r = 1; r < size(); ++r) {
        const double b = hub_->vals[(size_t)r * 64 + j];
        a = op == 0 ? a + b : (op == 1 ? std::max(a, b) : std::min(a, b));
      }
      vals[j] = a;
    }
    hub_->barrier(rank_, io_ > 0);
  }
  void barrier() override { hub_->barrier(rank_, io_ > 0); }

 private:
  int io_ = 0;
  // direct peer reads over xGMI for the copies this device pulls from `peer`
  void enable_peer(int dev, int peer) {
    std::lock_guard<std::mutex> g(hub_->peer_mu);
    for (const auto& pr : hub_->peer_on)
      if (pr.first == dev && pr.second == peer) return;
    int can = 0;
    H2D_HIP(hipDeviceCanAccessPeer(&can, dev, peer));
    if (can) {
      const hipError_t e = hipDeviceEnablePeerAccess(peer, 0);
      if (e == hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
      else H2D_HIP(e);
    }
    hub_->peer_on.emplace_back(dev, peer);
  }
  std::shared_ptr<PeerHub> hub_;
  int rank_;
};

}  // namespace

std::shared_ptr<Transport> make_self_transport() { return std::make_shared<SelfTransport>(); }

std::vector<std::shared_ptr<Transport>> make_peer_transports(int nranks) {
  HEAT2D_REQUIRE(nranks >= 1, "nranks >= 1");
  auto hub = std::make_shared<PeerHub>(nranks);
  std::vector<std::shared_ptr<Transport>> v;
  for (int i = 0; i < nranks; ++i) v.push_back(std::make_shared<PeerTransport>(hub, i));
  return v;
}

std::vector<std::shared_ptr<Transport>> make_thread_transports(int nranks) {
  HEAT2D_REQUIRE(nranks >= 1, "nranks >= 1");
  auto hub = std::make_shared<ThreadHub>(nranks);
  std::vector<std::shared_ptr<Transport>> v;
  for (int i = 0; i < nranks; ++i) v.push_back(std::make_shared<ThreadTransport>(hub, i));
  return v;
}

std::vector<std::shared_ptr<Transport>> make_loopback_transports(int nranks) {
  HEAT2D_REQUIRE(nranks >= 1, "nranks >= 1");
  auto hub = std::make_shared<LoopbackHub>(nranks);
  std::vector<std::shared_ptr<Transport>> v;
  for (int i = 0; i < nranks; ++i) v.push_back(std::make_shared<LoopbackTransport>(hub, i));
  return v;
}

std::shared_ptr<Transport> make_rccl_transport(const void* uid, int rank, int size, int device) {
  return std::make_shared<RcclTransport>(uid, rank, size, device);
}

std::shared_ptr<Transport> make_rccl_loop_transport(int device) {
  ncclUniqueId id;
  H2D_NCCL(ncclGetUniqueId(&id));
  return std::make_shared<RcclTransport>(&id, 0, 1, device, true);
}

void rccl_unique_id(void* out128) {
  ncclUniqueId id;
  H2D_NCCL(ncclGetUniqueId(&id));
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  std::memcpy(out128, &id, sizeof(id));
}

std::shared_ptr<Transport> make_callback_transport(const CallbackOps& ops, int rank, int size) {
  return std::make_shared<CallbackTransport>(ops, rank, size);
}

}  // namespace heat2d
