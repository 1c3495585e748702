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
#include <cstring>
#include <vector>

#include "heat2d/runtime.hpp"

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
  }
  ~RcclTransport() override {
    if (comm_) ncclCommDestroy(comm_);
    if (d_scratch_) (void)hipFree(d_scratch_);
    if (aux_) (void)hipStreamDestroy(aux_);
  }
  int rank() const override { return rank_; }
  int size() const override { return size_; }
  std::string name() const override { return loop_ ? "rccl-loop" : "rccl"; }
  // Not captured into hipGraphs: capturing the grouped ncclSend/ncclRecv of
  // the overlapped cycle segfaulted inside step() on the MI355X box (RCCL
  // 2.26.6, tools/graph_rccl_probe.py, either split order), so --graph runs
  // eager cycles whenever RCCL exchanges halos (single-rank runs still use
  // graphs).
  bool capturable() const override { return false; }
  bool exchanges() const override { return size_ > 1 || loop_; }
  void check() override {
    ncclResult_t st = ncclSuccess;
    H2D_NCCL(ncclCommGetAsyncError(comm_, &st));
    if (st != ncclSuccess && st != ncclInProgress)
      fail(__FILE__, __LINE__, std::string("RCCL communicator failed asynchronously: ") + ncclGetErrorString(st) +
                                   " (rank " + std::to_string(rank_) + " of " + std::to_string(size_) + ")");
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
    H2D_NCCL(ncclGroupStart());
    for (int i = 0; i < nmsg; ++i) {
      H2D_NCCL(ncclSend(base + halo_row_bytes(L, msg[i].send_row, es), count, t, msg[i].peer, comm_, stream));
      H2D_NCCL(ncclRecv(base + halo_row_bytes(L, msg[i].recv_row, es), count, t, msg[i].peer, comm_, stream));
    }
    H2D_NCCL(ncclGroupEnd());
  }

  void allreduce(double* vals, int n, int op) override {
    HEAT2D_REQUIRE(n <= 64, "allreduce too large");
    H2D_HIP(hipSetDevice(device_));
    H2D_HIP(hipMemcpyAsync(d_scratch_, vals, n * sizeof(double), hipMemcpyHostToDevice, aux_));
    const ncclRedOp_t o = op == 0 ? ncclSum : (op == 1 ? ncclMax : ncclMin);
    H2D_NCCL(ncclAllReduce(d_scratch_, d_scratch_, n, ncclFloat64, o, comm_, aux_));
    H2D_HIP(hipMemcpyAsync(vals, d_scratch_, n * sizeof(double), hipMemcpyDeviceToHost, aux_));
    H2D_HIP(hipStreamSynchronize(aux_));
  }
  void barrier() override {
    double v = 0.0;
    allreduce(&v, 1, 0);
  }

 private:
  int rank_, size_;
  bool loop_ = false;
  int device_ = 0;
  ncclComm_t comm_ = nullptr;
  hipStream_t aux_ = nullptr;
  double* d_scratch_ = nullptr;
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

}  // namespace

std::shared_ptr<Transport> make_self_transport() { return std::make_shared<SelfTransport>(); }

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
