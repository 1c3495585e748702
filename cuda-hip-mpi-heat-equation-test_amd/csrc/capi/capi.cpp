// C ABI over the native runtime (see heat2d/capi.h).
#include "heat2d/capi.h"
#include "heat2d/jit.hpp"

#include <hip/hip_runtime.h>

#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>
#include <string>

#include "heat2d/config.hpp"
#include "heat2d/plan_cache.hpp"
#include "heat2d/runtime.hpp"
#include "heat2d/watchdog.hpp"

extern "C" int heat2d_io_write_xyz_impl(const char*, int, const void*, int64_t, int64_t, int64_t,
                                        const double*, const double*, int);
extern "C" int heat2d_io_write_npy_impl(const char*, int, const void*, int64_t, int64_t, int64_t);

using namespace heat2d;

namespace {
thread_local std::string g_err;

template <typename F>
int guarded(F&& f) {
  try {
    f();
    return 0;
  } catch (const std::exception& e) {
    g_err = e.what();
  } catch (...) {
    g_err = "unknown error";
  }
  return 1;
}

SlabLayout to_layout(const heat2d_layout* l) {
  SlabLayout L{};
  static_assert(sizeof(heat2d_layout) == sizeof(SlabLayout), "layout ABI");
  std::memcpy(&L, l, sizeof(L));
  return L;
}
kern::IcParams to_ic(const heat2d_ic* ic) {
  static_assert(sizeof(heat2d_ic) == sizeof(kern::IcParams), "ic ABI");
  kern::IcParams p{};
  std::memcpy(&p, ic, sizeof(p));
  return p;
}
SolverConfig to_cfg(const heat2d_config* c) {
  static_assert(sizeof(heat2d_config) == sizeof(SolverConfig), "config ABI");
  SolverConfig s{};
  std::memcpy(&s, c, sizeof(s));
  return s;
}
hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

struct TransportHandle {
  std::shared_ptr<Transport> t;
};
}  // namespace

extern "C" {

const char* heat2d_last_error(void) { return g_err.c_str(); }

// Native backtrace on a fatal signal (SIGABRT from glibc's heap checks such
// as "free(): invalid pointer", SIGSEGV, SIGBUS, SIGFPE, SIGILL): the frames
// name the library that called free(), which Python's faulthandler (Python
// frames only) cannot. Then the previous handler runs (faulthandler, or the
// default action), so the exit status stays the signal's.
namespace {
struct sigaction g_prev_sig[65];
void crash_handler(int sig, siginfo_t*, void*) {
  static const char head[] = "\nheat2d: fatal signal, native backtrace:\n";
  (void)!::write(2, head, sizeof(head) - 1);
  void* frames[64];
  const int n = ::backtrace(frames, 64);
  ::backtrace_symbols_fd(frames, n, 2);
  ::sigaction(sig, &g_prev_sig[sig], nullptr);
  ::raise(sig);
}
}  // namespace

int heat2d_install_crash_handler(void) {
  return guarded([&] {
    static std::once_flag once;
    std::call_once(once, [] {
      void* warm[2];
      (void)::backtrace(warm, 2);  // load libgcc's unwinder now, not inside the handler
      for (int sig : {SIGABRT, SIGSEGV, SIGBUS, SIGFPE, SIGILL}) {
        struct sigaction sa {};
        sa.sa_sigaction = crash_handler;
        sa.sa_flags = SA_SIGINFO | SA_NODEFER;
        sigemptyset(&sa.sa_mask);
        ::sigaction(sig, &sa, &g_prev_sig[sig]);
      }
    });
  });
}
int heat2d_version(void) { return 100; }
int heat2d_max_tb(void) { return kMaxTB; }

int heat2d_device_count(int* n) {
  return guarded([&] {
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    *n = c;
  });
}

int heat2d_wave_times(uint64_t* out, int64_t max_waves, int64_t* n) {
  return guarded([&] { *n = kern::wave_times(out, max_waves); });
}

int heat2d_device_limits(int device, int64_t* out10) {
  return guarded([&] {
    const hipDeviceAttribute_t attrs[10] = {
        hipDeviceAttributeMaxBlockDimX,  hipDeviceAttributeMaxBlockDimY,   hipDeviceAttributeMaxBlockDimZ,
        hipDeviceAttributeMaxGridDimX,   hipDeviceAttributeMaxGridDimY,    hipDeviceAttributeMaxGridDimZ,
        hipDeviceAttributeTotalConstantMemory, hipDeviceAttributeMaxThreadsPerBlock, hipDeviceAttributeWarpSize,
        hipDeviceAttributeMultiprocessorCount};
    for (int i = 0; i < 10; ++i) {
      int v = 0;
      if (hipDeviceGetAttribute(&v, attrs[i], device) != hipSuccess) fail(__FILE__, __LINE__, "hipDeviceGetAttribute failed");
      out10[i] = v;
    }
  });
}

int heat2d_make_layout(int64_t nrows, int64_t ncols, int64_t halo, int64_t row0, int64_t nrows_global,
                       heat2d_layout* out) {
  return guarded([&] {
    SlabLayout L = make_layout(nrows, ncols, halo, row0, nrows_global);
    std::memcpy(out, &L, sizeof(L));
  });
}

int heat2d_decompose_shifted(int64_t n, int nranks, int rank, int64_t edge_shift, int64_t* row0, int64_t* nrows) {
  return guarded([&] {
    SlabRange r = decompose(n, nranks, rank, edge_shift);
    *row0 = r.row0;
    *nrows = r.nrows;
  });
}

int heat2d_decompose(int64_t n, int nranks, int rank, int64_t* row0, int64_t* nrows) {
  return guarded([&] {
    SlabRange r = decompose(n, nranks, rank);
    *row0 = r.row0;
    *nrows = r.nrows;
  });
}

int heat2d_parse_input(const char* text, double* out7) {
  return guarded([&] {
    InputDat in = parse_input_text(text);
    out7[0] = (double)in.n;
    out7[1] = in.sigma;
    out7[2] = in.nu;
    out7[3] = in.dom_len;
    out7[4] = (double)in.ntime;
    out7[5] = (double)in.soln;
    out7[6] = (double)in.nfields;
  });
}

int heat2d_plan_tb(int dtype, const heat2d_layout* L, int64_t rb, int64_t re, int k, int64_t tile_rows,
                   heat2d_tb_plan* out) {
  return guarded([&] {
    kern::TbPlan p = kern::plan_tb((DType)dtype, to_layout(L), rb, re, k, tile_rows);
    static_assert(sizeof(heat2d_tb_plan) == sizeof(kern::TbPlan), "plan ABI");
    std::memcpy(out, &p, sizeof(p));
  });
}

int heat2d_plan_split(int dtype, const heat2d_layout* L, int k, int64_t band, heat2d_split_plan* out) {
  return guarded([&] {
    kern::SplitPlan p = kern::plan_split((DType)dtype, to_layout(L), k, band);
    static_assert(sizeof(heat2d_split_plan) == sizeof(kern::SplitPlan), "split plan ABI");
    std::memcpy(out, &p, sizeof(p));
  });
}

int heat2d_tb(int dtype, const void* src, void* dst, const heat2d_layout* L, int64_t rb, int64_t re, int k,
              double r, void* stream, int64_t tile_rows, int arith) {
  return guarded([&] {
    kern::launch_tb((DType)dtype, src, dst, to_layout(L), rb, re, k, r, as_stream(stream), tile_rows, 0, arith);
  });
}

int heat2d_init_field(int dtype, void* field, const heat2d_layout* L, const heat2d_ic* ic,
                      const double* xc, const double* yc, void* stream) {
  return guarded([&] { kern::launch_init((DType)dtype, field, to_layout(L), to_ic(ic), xc, yc, as_stream(stream)); });
}

int heat2d_stats(int dtype, const void* field, const void* other, const heat2d_layout* L, double* work,
                 double* out, void* stream) {
  return guarded([&] { kern::launch_stats((DType)dtype, field, other, to_layout(L), work, out, as_stream(stream)); });
}

int64_t heat2d_stats_work_elems(void) { return kern::stats_work_elems(); }

int heat2d_copy(void* dst, const void* src, int64_t bytes, void* stream, int blocks) {
  return guarded([&] { kern::launch_copy(dst, src, bytes, as_stream(stream), blocks); });
}

int heat2d_read(const void* src, int64_t bytes, void* sink, void* stream, int blocks) {
  return guarded([&] { kern::launch_read(src, bytes, static_cast<unsigned*>(sink), as_stream(stream), blocks); });
}

int heat2d_pack_rows(int dtype, const void* field, const heat2d_layout* L, int64_t row, int64_t nrows,
                     void* buf, void* stream) {
  return guarded([&] { kern::launch_pack_rows((DType)dtype, field, to_layout(L), row, nrows, buf, as_stream(stream)); });
}

int heat2d_unpack_rows(int dtype, void* field, const heat2d_layout* L, int64_t row, int64_t nrows,
                       const void* buf, void* stream) {
  return guarded([&] { kern::launch_unpack_rows((DType)dtype, field, to_layout(L), row, nrows, buf, as_stream(stream)); });
}

int heat2d_cpu_tb(int dtype, const void* src, void* dst, const heat2d_layout* L, int64_t rb, int64_t re, int k,
                  double r, int arith) {
  return guarded([&] { cpu::tb((DType)dtype, src, dst, to_layout(L), rb, re, k, r, arith); });
}

int heat2d_cpu_init_field(int dtype, void* field, const heat2d_layout* L, const heat2d_ic* ic, const double* xc,
                          const double* yc) {
  return guarded([&] { cpu::init((DType)dtype, field, to_layout(L), to_ic(ic), xc, yc); });
}

int heat2d_cpu_stats(int dtype, const void* field, const void* other, const heat2d_layout* L, double* out6) {
  return guarded([&] { cpu::stats((DType)dtype, field, other, to_layout(L), out6); });
}

int heat2d_rccl_unique_id(void* out128) {
  return guarded([&] { rccl_unique_id(out128); });
}

int heat2d_transport_self(void** out) {
  return guarded([&] { *out = new TransportHandle{make_self_transport()}; });
}

int heat2d_transport_rccl(const void* uid128, int rank, int size, int device, void** out) {
  return guarded([&] { *out = new TransportHandle{make_rccl_transport(uid128, rank, size, device)}; });
}

int heat2d_transport_rccl_loop(int device, void** out) {
  return guarded([&] { *out = new TransportHandle{make_rccl_loop_transport(device)}; });
}

int heat2d_transport_callback(heat2d_exchange_fn ex, heat2d_allreduce_fn ar, heat2d_barrier_fn br, void* ctx,
                              int rank, int size, void** out) {
  return guarded([&] {
    CallbackOps ops{ctx, ex, ar, br};
    *out = new TransportHandle{make_callback_transport(ops, rank, size)};
  });
}

int heat2d_transport_ipc(heat2d_allgather_fn ag, heat2d_allreduce_fn ar, heat2d_barrier_fn br, void* ctx, int rank,
                         int size, int device, void** out) {
  return guarded([&] {
    IpcOps ops{ctx, ag, ar, br};
    *out = new TransportHandle{make_ipc_transport(ops, rank, size, device)};
  });
}

int heat2d_transport_ipc_loop(int device, void** out) {
  return guarded([&] { *out = new TransportHandle{make_ipc_loop_transport(device)}; });
}

int heat2d_transport_free(void* t) {
  return guarded([&] { delete static_cast<TransportHandle*>(t); });
}

int heat2d_transport_info(void* t, int32_t* out4) {
  return guarded([&] {
    const Transport::FabricInfo f = static_cast<TransportHandle*>(t)->t->fabric_info();
    out4[0] = f.kind;
    out4[1] = f.nranks;
    out4[2] = f.rank;
    out4[3] = f.device;
  });
}

int heat2d_device_pci_bus_id(int device, char* out, int64_t cap) {
  return guarded([&] {
    HEAT2D_REQUIRE(cap >= 16, "PCI bus id buffer too small");
    const hipError_t e = hipDeviceGetPCIBusId(out, (int)cap, device);
    if (e != hipSuccess) fail(__FILE__, __LINE__, std::string("hipDeviceGetPCIBusId: ") + hipGetErrorString(e));
  });
}

int heat2d_solver_create(const heat2d_config* cfg, void* transport, void** out) {
  return guarded([&] {
    std::shared_ptr<Transport> t =
        transport ? static_cast<TransportHandle*>(transport)->t : make_self_transport();
    *out = new Solver(to_cfg(cfg), t);
  });
}

int heat2d_solver_footprint(const heat2d_config* cfg, int rank, int nranks, int64_t* out3) {
  return guarded([&] {
    const Footprint f = solver_footprint(to_cfg(cfg), rank, nranks);
    out3[0] = f.field_bytes;
    out3[1] = f.work_bytes;
    out3[2] = f.total_bytes;
  });
}

int heat2d_plan_max_grid(int dtype, int nranks, int64_t budget_bytes, int64_t* n) {
  return guarded([&] { *n = plan_max_grid(dtype, nranks, budget_bytes); });
}

int heat2d_mem_info(int device, int64_t* free_bytes, int64_t* total_bytes) {
  return guarded([&] {
    if (hipSetDevice(device) != hipSuccess) fail(__FILE__, __LINE__, "hipSetDevice failed");
    size_t f = 0, t = 0;
    if (hipMemGetInfo(&f, &t) != hipSuccess) fail(__FILE__, __LINE__, "hipMemGetInfo failed");
    *free_bytes = (int64_t)f;
    *total_bytes = (int64_t)t;
  });
}

int heat2d_solver_free(void* s) {
  return guarded([&] { delete static_cast<Solver*>(s); });
}

int heat2d_solver_init(void* s, const heat2d_ic* ic, const double* xg, const double* yg) {
  return guarded([&] { static_cast<Solver*>(s)->init(to_ic(ic), xg, yg); });
}

int heat2d_solver_step(void* s, int64_t n) {
  return guarded([&] { static_cast<Solver*>(s)->step(n); });
}

int heat2d_solver_sync(void* s) {
  return guarded([&] { static_cast<Solver*>(s)->synchronize(); });
}

int heat2d_solver_stats(void* s, double* out6, int residual) {
  return guarded([&] { static_cast<Solver*>(s)->stats(out6, residual != 0); });
}

int heat2d_solver_download(void* s, void* host, int64_t ld) {
  return guarded([&] { static_cast<Solver*>(s)->download(host, ld); });
}

int heat2d_solver_compare(void* s, void* other, int64_t r0, int64_t nrows, int64_t other_r0, double* out2) {
  return guarded([&] { static_cast<Solver*>(s)->compare(*static_cast<Solver*>(other), r0, nrows, other_r0, out2); });
}

int heat2d_solver_upload(void* s, const void* host, int64_t ld) {
  return guarded([&] { static_cast<Solver*>(s)->upload(host, ld); });
}

int heat2d_solver_layout(void* s, heat2d_layout* out) {
  return guarded([&] {
    const SlabLayout& L = static_cast<Solver*>(s)->layout();
    std::memcpy(out, &L, sizeof(L));
  });
}

int heat2d_jit_create(int dtype, const heat2d_layout* L, double r, int device, int arith, void** out) {
  return guarded([&] { *out = new JitStencil((DType)dtype, to_layout(L), r, device, arith); });
}

int heat2d_jit_free(void* j) {
  return guarded([&] { delete static_cast<JitStencil*>(j); });
}

int heat2d_jit_step(void* j, const void* src, void* dst, void* stream) {
  return guarded([&] { static_cast<JitStencil*>(j)->step(src, dst, as_stream(stream)); });
}

int heat2d_jit_render(int dtype, const heat2d_layout* L, double r, int arith, char* buf, int64_t cap, int64_t* len) {
  return guarded([&] {
    const std::string s = jit_render((DType)dtype, to_layout(L), r, arith);
    *len = (int64_t)s.size();
    if (buf && cap > 0) {
      const size_t n = std::min<size_t>((size_t)cap - 1, s.size());
      std::memcpy(buf, s.data(), n);
      buf[n] = 0;
    }
  });
}

int heat2d_jit_compile_check(const char* source, const char* arch, int64_t* code_bytes) {
  return guarded([&] { *code_bytes = (int64_t)jit_compile(source, arch).size(); });
}

int heat2d_solver_timing(void* s, int on) {
  return guarded([&] { static_cast<Solver*>(s)->set_timing(on != 0); });
}

int heat2d_solver_phase_times(void* s, double* out5) {
  return guarded([&] { static_cast<Solver*>(s)->phase_times(out5); });
}

int heat2d_solver_prepare(void* s, int64_t n) {
  return guarded([&] { static_cast<Solver*>(s)->prepare(n); });
}

int heat2d_solver_plans_made(void* s, int64_t* out) {
  return guarded([&] { *out = static_cast<Solver*>(s)->plans_made(); });
}

int heat2d_solver_plan(void* s, int k, heat2d_split_plan* out, float* tuned_ms) {
  return guarded([&] {
    Solver& sv = *static_cast<Solver*>(s);
    HEAT2D_REQUIRE(k >= 1 && k <= kMaxTB, "k out of range");
    const kern::SplitPlan& p = sv.plan_for(k);
    std::memcpy(out, &p, sizeof(p));
    if (tuned_ms) *tuned_ms = sv.tuned_ms(k);
  });
}

int heat2d_solver_info(void* s, int32_t* tb, int64_t* band, int64_t* steps, void** field, void** stream) {
  return guarded([&] {
    Solver* so = static_cast<Solver*>(s);
    if (tb) *tb = so->config().tb;
    if (band) *band = so->band();
    if (steps) *steps = so->steps_done();
    if (field) *field = so->field();
    if (stream) *stream = reinterpret_cast<void*>(so->stream());
  });
}

int heat2d_group_create(const heat2d_config* cfg, int nranks, void** out) {
  return guarded([&] { *out = new LoopbackGroup(to_cfg(cfg), nranks); });
}

int heat2d_group_free(void* g) {
  return guarded([&] { delete static_cast<LoopbackGroup*>(g); });
}

int heat2d_group_init(void* g, const heat2d_ic* ic, const double* xg, const double* yg) {
  return guarded([&] { static_cast<LoopbackGroup*>(g)->init(to_ic(ic), xg, yg); });
}

int heat2d_group_step(void* g, int64_t n) {
  return guarded([&] { static_cast<LoopbackGroup*>(g)->step(n); });
}

int heat2d_group_upload(void* g, const void* host, int64_t ld) {
  return guarded([&] { static_cast<LoopbackGroup*>(g)->upload(host, ld); });
}

int heat2d_group_member(void* g, int i, void** solver) {
  return guarded([&] {
    auto* gr = static_cast<LoopbackGroup*>(g);
    HEAT2D_REQUIRE(i >= 0 && i < gr->nranks(), "member index out of range");
    *solver = &gr->member(i);
  });
}

int heat2d_solver_cycle_hist(void* s, int64_t* out, int n, int reset) {
  return guarded([&] {
    HEAT2D_REQUIRE(n >= kMaxTB + 1, "cycle_hist needs kMaxTB + 1 slots");
    static_cast<Solver*>(s)->cycle_hist(out, reset != 0);
  });
}

int heat2d_watchdog_selftest(double timeout_s, int mode, int progress_polls, double wait_s, double* fired_after_s,
                             char* reason, int64_t cap) {
  return guarded([&] {
    // mode 0: progress for `progress_polls` polls, then pending forever (a hang);
    // 1: idle forever (nothing outstanding: must never fire); 2: a fabric error
    std::atomic<int> polls{0};
    std::atomic<bool> fired{false};
    const auto t0 = std::chrono::steady_clock::now();
    double after = -1.0;
    std::mutex mu;
    std::string why;
    {
      Watchdog wd(
          timeout_s, 0.02,
          [&](std::string* d) {
            const int i = polls++;
            if (mode == 1) return Watchdog::Idle;
            if (mode == 2) {
              *d = "injected";
              return Watchdog::Error;
            }
            if (i < progress_polls) return Watchdog::Progress;
            *d = "selftest op pending";
            return Watchdog::Pending;
          },
          [&](const std::string& r) {
            std::lock_guard<std::mutex> g(mu);
            after = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            why = r;
            fired = true;
          });
      while (!fired && std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < wait_s)
        std::this_thread::sleep_for(std::chrono::milliseconds(5));
    }
    *fired_after_s = after;
    if (reason && cap > 0) {
      const size_t n = std::min<size_t>((size_t)cap - 1, why.size());
      std::memcpy(reason, why.data(), n);
      reason[n] = 0;
    }
  });
}

int heat2d_dp_schedule(int64_t n, int kmax, const double* t_ms, int32_t* out, int64_t cap, int64_t* len,
                       double* total) {
  return guarded([&] {
    const std::vector<int> v = dp_schedule(n, kmax, [&](int k) { return k >= 1 && k <= kmax ? t_ms[k] : -1.0; }, total);
    *len = (int64_t)v.size();
    for (int64_t i = 0; i < std::min<int64_t>(cap, *len); ++i) out[i] = v[(size_t)i];
  });
}

int heat2d_near_schedules(int64_t n, int kmax, const double* t_ms, double tol, int m, int32_t* out, int64_t cap,
                          int64_t* lens, double* costs, int32_t* count) {
  return guarded([&] {
    const auto v = near_schedules(n, kmax, [&](int k) { return k >= 1 && k <= kmax ? t_ms[k] : -1.0; }, tol, m);
    *count = (int32_t)v.size();
    int64_t pos = 0;
    for (size_t i = 0; i < v.size(); ++i) {
      lens[i] = (int64_t)v[i].second.size();
      costs[i] = v[i].first;
      for (int d : v[i].second) {
        HEAT2D_REQUIRE(pos < cap, "schedule output buffer too small");
        out[pos++] = d;
      }
    }
  });
}

int heat2d_search_schedule(int64_t n, int kmax, const double* pre_ms, const double* tuned_ms, int32_t* out,
                           int64_t cap, int64_t* len, double* cost, int32_t* prescanned, int32_t* nprescanned,
                           int32_t* tuned, int32_t* ntuned) {
  return guarded([&] {
    const ScheduleSearch r = search_schedule(
        n, kmax, [&](int k) { return pre_ms[k]; }, [&](int k) { return tuned_ms[k]; });
    *len = (int64_t)r.best.size();
    for (int64_t i = 0; i < std::min<int64_t>(cap, *len); ++i) out[i] = r.best[(size_t)i];
    *cost = r.cost;
    *nprescanned = (int32_t)r.prescanned.size();
    for (size_t i = 0; i < r.prescanned.size(); ++i) prescanned[i] = r.prescanned[i];
    *ntuned = (int32_t)r.tuned.size();
    for (size_t i = 0; i < r.tuned.size(); ++i) tuned[i] = r.tuned[i];
  });
}

int heat2d_transport_abort(void* t, const char* reason) {
  return guarded([&] { static_cast<TransportHandle*>(t)->t->abort(reason ? reason : "aborted by the caller"); });
}

int heat2d_solver_pref_depth(void* s, int32_t* out) {
  return guarded([&] { *out = static_cast<Solver*>(s)->pref_depth(); });
}

int heat2d_solver_step_stats(void* s, int64_t n, double* out6) {
  return guarded([&] { static_cast<Solver*>(s)->step_stats(n, out6); });
}

int heat2d_solver_schedule(void* s, int64_t n, int32_t* out, int64_t cap, int64_t* len) {
  return guarded([&] {
    const std::vector<int>* v = static_cast<Solver*>(s)->schedule(n);
    *len = v ? (int64_t)v->size() : -1;
    if (v && out)
      for (int64_t i = 0; i < std::min<int64_t>(cap, (int64_t)v->size()); ++i) out[i] = (*v)[(size_t)i];
  });
}

int heat2d_solver_schedule_replayed(void* s, int64_t n, int32_t* out) {
  return guarded([&] { *out = static_cast<Solver*>(s)->schedule_replayed(n) ? 1 : 0; });
}

int heat2d_solver_step_cycles(void* s, int64_t n, int32_t* out, int64_t cap, int64_t* len) {
  return guarded([&] {
    const std::vector<int> v = static_cast<Solver*>(s)->step_cycles(n);
    *len = (int64_t)v.size();
    if (out)
      for (int64_t i = 0; i < std::min<int64_t>(cap, *len); ++i) out[i] = v[(size_t)i];
  });
}

int heat2d_solver_halo_rows(void* s, int reset, int64_t* out) {
  return guarded([&] { *out = static_cast<Solver*>(s)->halo_rows_exchanged(reset != 0); });
}

int heat2d_solver_ghost_rows(void* s, int32_t* out) {
  return guarded([&] { *out = static_cast<Solver*>(s)->ghost_rows(); });
}

int heat2d_solver_tune_stats(void* s, int64_t* depths, int64_t* candidates) {
  return guarded([&] {
    *depths = static_cast<Solver*>(s)->depths_tuned();
    *candidates = static_cast<Solver*>(s)->tune_trials();
  });
}

int heat2d_solver_plan_cache_hits(void* s, int64_t* out) {
  return guarded([&] { *out = static_cast<Solver*>(s)->plan_cache_hits(); });
}

// The plan cache's own entry points (tests of its on-disk format): reload the
// file named by $HEAT2D_PLAN_CACHE, put / get one plan and one schedule.
int heat2d_plan_cache_reload() {
  return guarded([&] { plancache::reset(); });
}

int heat2d_plan_cache_put(const char* ctx, int k, int64_t band, const heat2d_split_plan* p, float ms) {
  return guarded([&] {
    kern::SplitPlan q;
    std::memcpy(&q, p, sizeof(q));
    plancache::put_plan(ctx, k, band, q, ms);
  });
}

int heat2d_plan_cache_get(const char* ctx, int k, int64_t band, heat2d_split_plan* p, float* ms, int32_t* found) {
  return guarded([&] {
    kern::SplitPlan q{};
    *found = plancache::get_plan(ctx, k, band, &q, ms) ? 1 : 0;
    if (*found) std::memcpy(p, &q, sizeof(q));
  });
}

int heat2d_plan_cache_put_schedule(const char* ctx, int64_t n, const int32_t* depths, int64_t count) {
  return guarded([&] { plancache::put_schedule(ctx, n, std::vector<int>(depths, depths + count)); });
}

int heat2d_plan_cache_get_schedule(const char* ctx, int64_t n, int32_t* depths, int64_t cap, int64_t* count) {
  return guarded([&] {
    std::vector<int> s;
    *count = plancache::get_schedule(ctx, n, &s) ? (int64_t)s.size() : -1;
    for (int64_t i = 0; i < std::min<int64_t>(cap, (int64_t)s.size()); ++i) depths[i] = s[(size_t)i];
  });
}

int heat2d_plan_cache_path(char* buf, int64_t cap) {
  return guarded([&] {
    const std::string p = plancache::enabled() ? plancache::path() : std::string();
    const size_t n = std::min<size_t>((size_t)std::max<int64_t>(cap - 1, 0), p.size());
    if (cap > 0) {
      std::memcpy(buf, p.data(), n);
      buf[n] = 0;
    }
  });
}

int heat2d_solver_plan_origin(void* s, int k, int32_t* out) {
  return guarded([&] { *out = static_cast<Solver*>(s)->plan_origin(k); });
}

int heat2d_autotune_slabs(int64_t n_rows, int64_t n_cols, int nranks, int autotune, int32_t* out) {
  return guarded([&] { *out = autotune_slabs(n_rows, n_cols, nranks, autotune) ? 1 : 0; });
}

int heat2d_group_download(void* g, void* host, int64_t ld) {
  return guarded([&] {
    auto* gr = static_cast<LoopbackGroup*>(g);
    gr->synchronize();
    gr->download(host, ld);
  });
}

int heat2d_write_xyz(const char* path, int dtype, const void* host, int64_t nrows, int64_t ncols, int64_t ld,
                     const double* x, const double* y, int append) {
  return guarded([&] { heat2d_io_write_xyz_impl(path, dtype, host, nrows, ncols, ld, x, y, append); });
}

int heat2d_write_npy(const char* path, int dtype, const void* host, int64_t nrows, int64_t ncols, int64_t ld) {
  return guarded([&] { heat2d_io_write_npy_impl(path, dtype, host, nrows, ncols, ld); });
}

}  // extern "C"
