// heat2d — native command-line driver.
//
// `heat2d [input.dat] [flags]` reproduces the run behaviour of every
// reference program (reads ./input.dat by default, prints the same progress /
// completion / timing lines, writes int.dat / soln.dat / soln%05d.dat):
//   --variant mpi     fortran/hip (6-field input; ghost frame, uniform IC,
//                     per-rank soln%05d.dat, "Average time:")
//   --variant mpicuda fortran/mpi+cuda (as mpi, but "Sum of Temperature:" — here
//                     the real all-reduced sum — and a per-iteration "total time:")
//   --variant serial  fortran/serial (5-field input; boundary-inclusive grid,
//                     hat IC, int.dat + soln.dat, "total time:")
//   --variant cuda    fortran/cuda_cuf + fortran/cuda_kernel (hat on y in [0.5,1.0])
//   --managed         fortran/cuda_kernel/heat_managed.F90 (hipMallocManaged fields)
//   --cpu             native CPU path (replaces the gfortran serial build)
//   --engine jit      run-time specialised hipRTC kernel (python/cuda/cuda.py's JIT)
// Multi-GPU is one host thread per GPU (hipSetDevice(rank), the reference's
// node-local rank -> device binding, fortran/hip/heat.F90:119-125); the halo
// exchange is RCCL send/recv over xGMI, or — `--transport auto` (default) when
// RCCL cannot build its communicators on every rank, or `--transport peer` —
// device copies out of the neighbours' fields (peer access over xGMI).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "heat2d/capi.h"
#include "heat2d/ckpt.hpp"
#include "heat2d/config.hpp"
#include "heat2d/runtime.hpp"

using namespace heat2d;

namespace {

struct Args {
  std::string input = "input.dat";
  std::string variant;  // mpi | serial | cuda (default: by number of input fields)
  std::string ic;       // override IC
  std::string dtype = "fp64";
  std::string output = "ascii";  // ascii | npy | none
  std::string json;
  int gpus = -1;  // -1: 1 if a GPU exists
  bool cpu = false;
  int tb = 0;  // 0: measured best per dtype (solver.cpp)
  bool overlap = true;
  bool copy_swap = false;
  bool managed = false;
  bool graph = false;
  int64_t print_every = 0;
  int64_t check_every = 0;
  int64_t ntime = -1;  // override
  int64_t n = -1;      // override
  bool n_max = false;  // --n max: the largest grid the GPUs' free memory holds (memory-fit planner)
  bool quiet = false;
  bool timers = false;
  std::string engine = "tb";
  // auto | exact | fma | jacobi | fast (SolverConfig::arith). auto: jacobi when
  // r == 1/4 and the IC keeps every value in [m, 2m] (bitwise the reference
  // rounding then, ic_sterbenz_safe), else fma when r is a power of two
  // (bitwise identical too), else exact
  std::string arith = "auto";
  bool time_transfers = false;  // --time-transfers: H2D of the IC and D2H of the result inside the timed region
  std::string checkpoint;       // --checkpoint DIR (utils/checkpoint.py format)
  int64_t checkpoint_every = 0;
  std::string restart;          // --restart DIR (any writer rank count)
  // GPU ranks: auto (RCCL if its communicators build on every rank, else
  // peer) | rccl | peer (device copies between the ranks' fields, no RCCL)
  std::string transport = "auto";
  bool share_gpu = false;          // --share-gpu: every rank on device 0 (peer transport; tests / rehearsals)
  int autotune = -1;               // --autotune auto|on|off (SolverConfig::autotune)
  int edge_shift = 0;              // --edge-shift N: rows each edge slab gives the middle ones (>= 3 ranks)
};

void usage() {
  std::printf(
      "usage: heat2d [input.dat] [--variant mpi|mpicuda|serial|cuda] [--gpus N | --cpu] [--dtype fp64|fp32]\n"
      "              [--tb K] [--no-overlap] [--copy-swap] [--managed] [--graph] [--ic NAME]\n"
      "              [--print-every N] [--check-every N] [--output ascii|npy|none] [--json FILE]\n"
      "              [--n N|max] [--ntime N] [--quiet] [--timers] [--engine tb|jit] [--arith auto|exact|fma|jacobi|fast]\n"
      "              [--time-transfers]\n"
      "              [--checkpoint DIR [--checkpoint-every N]] [--restart DIR]\n"
      "              [--transport auto|rccl|peer] [--share-gpu] [--autotune auto|on|off] [--edge-shift N]\n");
}

Args parse_args(int argc, char** argv) {
  Args a;
  for (int i = 1; i < argc; ++i) {
    std::string s = argv[i];
    auto need = [&](const char* what) -> std::string {
      if (i + 1 >= argc) {
        std::fprintf(stderr, "missing value for %s\n", what);
        std::exit(2);
      }
      return argv[++i];
    };
    if (s == "-h" || s == "--help") { usage(); std::exit(0); }
    else if (s == "--variant") a.variant = need("--variant");
    else if (s == "--ic") a.ic = need("--ic");
    else if (s == "--dtype") a.dtype = need("--dtype");
    else if (s == "--output") a.output = need("--output");
    else if (s == "--json") a.json = need("--json");
    else if (s == "--gpus" || s == "-np") a.gpus = std::atoi(need("--gpus").c_str());
    else if (s == "--cpu") a.cpu = true;
    else if (s == "--tb") a.tb = std::atoi(need("--tb").c_str());
    else if (s == "--no-overlap") a.overlap = false;
    else if (s == "--copy-swap") a.copy_swap = true;
    else if (s == "--managed") a.managed = true;
    else if (s == "--graph") a.graph = true;
    else if (s == "--engine") a.engine = need("--engine");
    else if (s == "--arith") a.arith = need("--arith");
    else if (s == "--time-transfers") a.time_transfers = true;
    else if (s == "--print-every") a.print_every = std::atoll(need("--print-every").c_str());
    else if (s == "--check-every") a.check_every = std::atoll(need("--check-every").c_str());
    else if (s == "--ntime") a.ntime = std::atoll(need("--ntime").c_str());
    else if (s == "--n") {
      const std::string v = need("--n");
      if (v == "max") a.n_max = true;
      else a.n = std::atoll(v.c_str());
    }
    else if (s == "--quiet") a.quiet = true;
    else if (s == "--timers") a.timers = true;
    else if (s == "--checkpoint") a.checkpoint = need("--checkpoint");
    else if (s == "--checkpoint-every") a.checkpoint_every = std::atoll(need("--checkpoint-every").c_str());
    else if (s == "--restart") a.restart = need("--restart");
    else if (s == "--transport") a.transport = need("--transport");
    else if (s == "--share-gpu") a.share_gpu = true;
    else if (s == "--edge-shift") {
      a.edge_shift = std::atoi(need("--edge-shift").c_str());
      if (a.edge_shift < 0) {
        std::fprintf(stderr, "--edge-shift must be >= 0\n");
        std::exit(2);
      }
    }
    else if (s == "--autotune") {
      const std::string v = need("--autotune");
      if (v != "auto" && v != "on" && v != "off") {
        std::fprintf(stderr, "--autotune must be auto, on or off\n");
        std::exit(2);
      }
      a.autotune = v == "on" ? 1 : (v == "off" ? 0 : -1);
    }
    else if (!s.empty() && s[0] != '-') a.input = s;
    else { std::fprintf(stderr, "unknown flag %s\n", s.c_str()); usage(); std::exit(2); }
  }
  return a;
}

struct Shared {
  Args args;
  InputDat in;
  Problem prob;
  int nranks = 1;
  unsigned char uid[128];
  std::vector<double> t_elapsed;
  std::atomic<int> failed{0};
  std::mutex mu;  // err, trs
  std::string err;
  std::vector<std::shared_ptr<Transport>> trs;  // every rank's transport (fail-fast abort)
  std::vector<std::shared_ptr<Transport>> cpu_trs;  // --cpu with P > 1: the host-thread transports
  std::vector<std::shared_ptr<Transport>> peer_trs;  // --transport peer (or auto's fallback) with P > 1
  std::vector<std::shared_ptr<Transport>> rccl_trs;  // --transport auto: the communicators built up front
  std::string transport_used = "self";               // self | rccl | peer | host
  std::string transport_note;                        // why auto fell back (empty: no fallback)
  double final_stats[6] = {0};
  int tb_used = 1;  // largest temporal depth the solver may run (jit / copy-swap force 1)
  int64_t hist[kMaxTB + 1] = {0};  // cycles per depth of the timed loop (rank 0)
  std::vector<std::vector<int64_t>> rank_hist;  // the same, every rank (they must agree)
  std::vector<int64_t> rank_halo_rows;          // halo rows exchanged per side by each rank's timed loop
  bool measured = false;  // a chunk of the timed loop runs a measured cycle schedule (Solver::prepare)
  int64_t start_step = 0;  // > 0 after --restart
  std::string arith_used;  // the arithmetic the run used (auto resolved)
  double t_h2d = 0, t_d2h = 0;  // --time-transfers: rank 0's whole-field copies inside the timed region
};

// Collective checkpoint (every rank its slab, then rank 0 publishes meta.json).
void save_checkpoint(Shared& sh, Solver& s, Transport& tr, int rank, int64_t step) {
  const Args& a = sh.args;
  IoPhase io(tr);  // ranks wait on each other's file writes: not a hung fabric
  // every rank names the same fresh step directory before any rank creates it
  const std::string name = ckpt::step_dir_name(a.checkpoint, step);
  tr.barrier();
  ckpt::write_rank(a.checkpoint, name, rank, s);
  tr.barrier();
  if (rank == 0) {
    ckpt::Meta m;
    m.step = step;
    m.nranks = sh.nranks;
    m.dtype = (int)s.dtype();
    m.n_owned = sh.prob.n_owned;
    m.n_input = sh.in.n;
    m.convention = sh.prob.conv == Convention::Inclusive ? "inclusive" : "ghost";
    m.sigma = sh.in.sigma;
    m.nu = sh.in.nu;
    m.dom_len = sh.in.dom_len;
    m.r = sh.prob.r;
    m.edge_shift = a.edge_shift;
    ckpt::write_meta(a.checkpoint, name, m);
  }
  tr.barrier();
}

std::string json_str(const std::string& v) {
  std::string o = "\"";
  for (char c : v) {
    if (c == '"' || c == '\\') o += '\\';
    if ((unsigned char)c < 0x20) c = ' ';
    o += c;
  }
  return o + "\"";
}

std::string rank_file(int rank) {
  char b[32];
  std::snprintf(b, sizeof(b), "soln%05d.dat", rank);
  return b;
}

void write_inclusive(Solver& s, const Problem& p, const char* path, bool first_rank, bool last_rank, bool append) {
  // full frame-inclusive rows of this slab: x outer, y inner (fortran/serial/heat.f90:77-83)
  const SlabLayout& L = s.layout();
  const int64_t r0 = first_rank ? -1 : 0, r1 = last_rank ? L.nrows + 1 : L.nrows;
  const int64_t w = L.ncols + 2;
  std::vector<char> host((size_t)((r1 - r0) * w) * dtype_size(s.dtype()));
  s.download_region(r0, r1, -1, L.ncols + 1, host.data(), w);
  std::vector<double> xs((size_t)(r1 - r0));
  for (int64_t i = r0; i < r1; ++i) xs[(size_t)(i - r0)] = p.x[(size_t)(L.row0 + i + 1)];
  if (heat2d_write_xyz(path, (int)s.dtype(), host.data(), r1 - r0, w, w, xs.data(), p.x.data(), append ? 1 : 0))
    fail(__FILE__, __LINE__, heat2d_last_error());
}

void run_rank(Shared& sh, int rank) {
  const Args& a = sh.args;
  const int P = sh.nranks;
  const bool root = rank == 0;
  try {
    std::shared_ptr<Transport> tr;
    const int device = a.share_gpu ? 0 : rank;
    if (!a.cpu) {
      if (hipSetDevice(device) != hipSuccess) fail(__FILE__, __LINE__, "hipSetDevice failed");
      if (!a.quiet && (root || P > 1)) std::printf(" MPI rank %12d using GPU %12d\n", rank, device);
    }
    if (P == 1) tr = make_self_transport();
    else if (a.cpu) tr = sh.cpu_trs[(size_t)rank];  // host threads (the reference's `make mpi`)
    else if (!sh.peer_trs.empty()) tr = sh.peer_trs[(size_t)rank];
    else if (!sh.rccl_trs.empty()) tr = sh.rccl_trs[(size_t)rank];
    else tr = make_rccl_transport(sh.uid, rank, P, device);
    {
      std::lock_guard<std::mutex> g(sh.mu);
      sh.trs[(size_t)rank] = tr;
      if (sh.failed) tr->abort("another rank failed first");
    }

    SolverConfig cfg{};
    cfg.n_rows = sh.prob.n_owned;
    cfg.n_cols = sh.prob.n_owned;
    cfg.dtype = a.dtype == "fp32" ? 0 : 1;
    cfg.backend = a.cpu ? 1 : 0;
    cfg.r = sh.prob.r;
    cfg.tb = a.tb;
    cfg.overlap = a.overlap ? 1 : 0;
    cfg.copy_swap = a.copy_swap ? 1 : 0;
    cfg.managed = a.managed ? 1 : 0;
    cfg.device = a.cpu ? -1 : device;
    cfg.use_graph = a.graph ? 1 : 0;
    // split schedule: the fastest launch plan per depth and a measured cycle schedule
    // (auto: slabs of >= 2^24 points — decided from the thinnest slab, the same on every rank)
    cfg.autotune = a.autotune;
    cfg.edge_shift = a.edge_shift;
    if (a.engine != "tb" && a.engine != "jit") fail(__FILE__, __LINE__, "--engine must be tb or jit");
    cfg.engine = a.engine == "jit" ? 1 : 0;  // jit: hipRTC kernel rendered for this slab (python/cuda/cuda.py)
    if (a.arith != "exact" && a.arith != "fma" && a.arith != "jacobi" && a.arith != "fast" && a.arith != "auto")
      fail(__FILE__, __LINE__, "--arith must be auto, exact, fma, jacobi or fast");
    cfg.arith = a.arith == "fast" ? 3 : a.arith == "jacobi" ? 2 : a.arith == "fma" ? 1 : (a.arith == "exact" ? 0 : -1);
    std::string arith_used = a.arith;
    if (cfg.arith < 0) {
      // auto: the r = 1/4 form when it rounds exactly like the reference for
      // the whole run — the IC in [m, 2m] (the reference's: 1 and 2) keeps
      // every sum - 4c exact; a restart's data is not known to be
      if (sh.prob.r == 0.25 && ic_sterbenz_safe(sh.prob.ic) && a.restart.empty() && cfg.engine == 0) {
        cfg.arith = 2;
        arith_used = "jacobi (auto)";
      } else {
        int e = 0;
        const bool pow2 = sh.prob.r > 0 && std::frexp(sh.prob.r, &e) == 0.5;
        arith_used = pow2 ? "fma (auto)" : "exact (auto)";
      }
    }
    if (root) sh.arith_used = arith_used;
    Solver s(cfg, tr);
    s.init(sh.prob.ic, sh.prob.x.data(), sh.prob.x.data());
    const bool inclusive = sh.prob.conv == Convention::Inclusive;
    int64_t start = 0;
    if (!a.restart.empty()) {  // resume (bitwise: FTCS carries no state besides the field)
      const ckpt::Meta m = ckpt::read_meta(a.restart);
      HEAT2D_REQUIRE(m.n_owned == sh.prob.n_owned, "checkpoint grid differs from input.dat's");
      HEAT2D_REQUIRE(m.convention == (inclusive ? "inclusive" : "ghost"), "checkpoint grid convention differs");
      const SlabLayout& L = s.layout();
      std::vector<char> host((size_t)(L.nrows * L.ncols) * dtype_size(s.dtype()));
      {
        IoPhase io(*tr);
        ckpt::read_rows(m, L.row0, L.nrows, L.ncols, (int)s.dtype(), host.data());
        tr->barrier();  // every rank has read its rows: the upload's exchange waits on no file system
      }
      s.upload(host.data(), L.ncols);  // + halo exchange
      start = std::min<int64_t>(m.step, sh.in.ntime);
      if (root) {
        sh.start_step = start;
        if (!a.quiet) std::printf(" restarted from %s at step %lld\n", a.restart.c_str(), (long long)start);
      }
    }
    if (root && !a.quiet) {
      // (fortran/hip prints the decomposition line; fortran/mpi+cuda only nx / ny)
      if (P > 1 || sh.args.variant == "mpi") std::printf(" Automatic MPI decomposition: %12d  x 1\n", P);
      std::printf(" nx: %12lld\n", (long long)s.layout().nrows);
      std::printf(" ny: %12lld\n", (long long)s.layout().ncols);
      std::fflush(stdout);
    }
    if (inclusive && a.output == "ascii" && start == 0) {  // int.dat: the IC (fortran/serial/heat.f90:50-55)
      IoPhase io(*tr);
      for (int turn = 0; turn < P; ++turn) {
        if (turn == rank) write_inclusive(s, sh.prob, "int.dat", rank == 0, rank == P - 1, rank > 0);
        tr->barrier();
      }
    }

    const int64_t ntime = sh.in.ntime;
    // plan / autotune every cycle depth the loop will use before the clock starts
    // time_it lines (fortran/hip/heat.F90:241 prints one per step) do not cut
    // the run into cycles shorter than the preferred depth: chunks of
    // max(print_every, pref_depth) steps, every due line printed after its chunk
    // fault injection for the fail-fast tests: rank HEAT2D_FAIL_RANK throws
    // once it has run HEAT2D_FAIL_STEP steps (tests/test_cli.py)
    const char* fr = std::getenv("HEAT2D_FAIL_RANK");
    const int fail_rank = fr ? std::atoi(fr) : -1;
    const char* fs = std::getenv("HEAT2D_FAIL_STEP");
    const int64_t fail_step = fs ? std::atoll(fs) : 0;
    const int64_t print_chunk = a.print_every > 0 ? std::max<int64_t>(a.print_every, s.pref_depth()) : 0;
    {  // walk the chunking of the loop below and prepare each distinct chunk length
      const bool ckpt_every = !a.checkpoint.empty() && a.checkpoint_every > 0;
      std::vector<int64_t> seen;
      for (int64_t d = start; d < ntime;) {
        int64_t c = ntime - d;
        if (print_chunk > 0) c = std::min(c, print_chunk - (d % print_chunk));
        if (a.check_every > 0) c = std::min(c, a.check_every - (d % a.check_every));
        if (ckpt_every) c = std::min(c, a.checkpoint_every - (d % a.checkpoint_every));
        if (std::find(seen.begin(), seen.end(), c) == seen.end()) {
          seen.push_back(c);
          s.prepare(c);
          if (root && s.schedule(c)) sh.measured = true;
        }
        d += c;
      }
    }
    if (a.timers) s.set_timing(true);
    {
      int64_t h[kMaxTB + 1];
      s.cycle_hist(h, true);  // count the timed loop's cycles only
      (void)s.halo_rows_exchanged(true);
    }
    // --time-transfers: the reference's timed region also moves the whole
    // field host -> device before the loop and back after it
    // (fortran/hip/heat.F90:284-295); the host copy of the IC is taken here,
    // outside it (pinned memory: the copies run at DMA speed)
    void* host_field = nullptr;
    bool host_pinned = false;
    const size_t host_bytes = (size_t)(s.layout().nrows * s.layout().ncols) * dtype_size(s.dtype());
    if (a.time_transfers) {
      if (!a.cpu && hipHostMalloc(&host_field, host_bytes, 0) == hipSuccess) host_pinned = true;
      else host_field = std::malloc(host_bytes);
      HEAT2D_REQUIRE(host_field != nullptr, "host buffer for --time-transfers");
      s.download(host_field, s.layout().ncols);
    }
    tr->barrier();
    s.synchronize();
    const auto t0 = std::chrono::steady_clock::now();
    if (a.time_transfers) {
      s.upload(host_field, s.layout().ncols);  // H2D + the halo exchange of the uploaded field
      if (root) sh.t_h2d = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    }
    int64_t done = start;
    const bool ckpt_periodic = !a.checkpoint.empty() && a.checkpoint_every > 0;
    while (done < ntime) {
      int64_t chunk = ntime - done;
      if (print_chunk > 0) chunk = std::min(chunk, print_chunk - (done % print_chunk));
      if (a.check_every > 0) chunk = std::min(chunk, a.check_every - (done % a.check_every));
      if (ckpt_periodic) chunk = std::min(chunk, a.checkpoint_every - (done % a.checkpoint_every));
      if (fail_rank == rank && done >= fail_step)  // fault injection (HEAT2D_FAIL_RANK / HEAT2D_FAIL_STEP)
        fail(__FILE__, __LINE__, "injected failure at step " + std::to_string(done));
      const bool check = a.check_every > 0 && (done + chunk) % a.check_every == 0;
      double st[6];
      if (check) s.step_stats(chunk, st);  // statistics + one-step residual fused into the last cycle
      else s.step(chunk);
      const int64_t before = done;
      done += chunk;
      if (root && a.print_every > 0)
        for (int64_t t = (before / a.print_every + 1) * a.print_every; t <= done; t += a.print_every)
          std::printf(" time_it: %12lld\n", (long long)t);
      if (check) {
        if (root)
          std::printf(" step %lld: sum=%.17g min=%.6g max=%.6g residual_l2=%.6e residual_max=%.6e\n", (long long)done,
                      st[0], st[2], st[3], std::sqrt(st[4]), st[5]);
        if (!std::isfinite(st[0])) fail(__FILE__, __LINE__, "non-finite temperature at step " + std::to_string(done));
      }
      if (ckpt_periodic && done % a.checkpoint_every == 0 && done < ntime) save_checkpoint(sh, s, *tr, rank, done);
    }
    s.synchronize();
    if (a.time_transfers) {
      const auto td = std::chrono::steady_clock::now();
      s.download(host_field, s.layout().ncols);  // D2H of the result
      if (root) sh.t_d2h = std::chrono::duration<double>(std::chrono::steady_clock::now() - td).count();
    }
    tr->barrier();
    const auto t1 = std::chrono::steady_clock::now();
    if (host_field) {
      if (host_pinned) (void)hipHostFree(host_field);
      else std::free(host_field);
    }
    sh.t_elapsed[(size_t)rank] = std::chrono::duration<double>(t1 - t0).count();
    if (a.timers) {
      double ph[5];
      s.phase_times(ph);
      std::printf(" heat2d: rank %d phases (GPU timeline, summed over %lld cycles): main %.3f ms, edge %.3f ms, "
                  "exchange %.3f ms, cycle %.3f ms\n",
                  rank, (long long)ph[4], ph[0], ph[1], ph[2], ph[3]);
    }

    if (!a.checkpoint.empty()) save_checkpoint(sh, s, *tr, rank, done);  // final state (outside the timed region)

    // outputs (serial rank turns / per-rank files: ranks wait on each other's I/O)
    if (a.output != "none") {
      IoPhase io(*tr);
      if (inclusive) {
        if (a.output == "ascii") {
          for (int turn = 0; turn < P; ++turn) {
            if (turn == rank) write_inclusive(s, sh.prob, "soln.dat", rank == 0, rank == P - 1, rank > 0);
            tr->barrier();
          }
        }
      } else if (sh.in.soln == 1 || a.output == "npy") {
        const SlabLayout& L = s.layout();
        std::vector<char> host((size_t)(L.nrows * L.ncols) * dtype_size(s.dtype()));
        s.download(host.data(), L.ncols);
        if (a.output == "npy") {
          char b[32];
          std::snprintf(b, sizeof(b), "soln%05d.npy", rank);
          if (heat2d_write_npy(b, (int)s.dtype(), host.data(), L.nrows, L.ncols, L.ncols)) fail(__FILE__, __LINE__, heat2d_last_error());
        } else {
          // soln%05d.dat: x(i), y(j), T(i,j) for owned points (fortran/hip/heat.F90:308-319)
          const double* xs = sh.prob.x.data() + 1 + L.row0;
          if (heat2d_write_xyz(rank_file(rank).c_str(), (int)s.dtype(), host.data(), L.nrows, L.ncols, L.ncols, xs,
                               sh.prob.x.data() + 1, 0))
            fail(__FILE__, __LINE__, heat2d_last_error());
        }
      }
      tr->barrier();  // the statistics' all-reduce below then waits on no file system
    }
    double st[6];
    s.stats(st, false);
    if (root) {
      std::memcpy(sh.final_stats, st, sizeof(st));
      sh.tb_used = s.config().tb;
      s.cycle_hist(sh.hist, false);
    }
    {
      int64_t h[kMaxTB + 1];
      s.cycle_hist(h, false);
      std::lock_guard<std::mutex> g(sh.mu);
      sh.rank_hist[(size_t)rank].assign(h, h + kMaxTB + 1);
      sh.rank_halo_rows[(size_t)rank] = s.halo_rows_exchanged(false);
    }
  } catch (const std::exception& e) {
    // fail fast: the first error is reported; every rank's communicator is
    // aborted so that the others, blocked in an exchange or a barrier with
    // this rank, return with an error instead of hanging in join()
    std::lock_guard<std::mutex> g(sh.mu);
    if (!sh.failed) sh.err = "rank " + std::to_string(rank) + ": " + e.what();
    sh.failed = 1;
    for (auto& t : sh.trs)
      if (t) t->abort("rank " + std::to_string(rank) + " failed: " + e.what());
  }
}

// --n max: the memory-fit planner (runtime.hpp plan_max_grid) on the smallest
// free memory of the GPUs the ranks use (hipMemGetInfo; shared by the ranks
// with --share-gpu), minus a reserve for what the solver does not own
// (2 GiB + 1 %: runtime growth, RCCL buffers; utils/memplan.py uses the same).
// The reference's grid is whatever input.dat says, plus a whole-field host
// mirror (fortran/hip/heat.F90:161-176); here nothing mirrors the field.
void plan_n_max(Shared& sh, int ndev, Convention conv) {
  const Args& a = sh.args;
  HEAT2D_REQUIRE(!a.cpu, "--n max plans device memory: it needs a GPU");
  const int P = sh.nranks;
  int64_t free_min = INT64_MAX, total = 0;
  for (int d = 0; d < (a.share_gpu ? 1 : std::min(P, ndev)); ++d) {
    size_t f = 0, t = 0;
    if (hipSetDevice(d) != hipSuccess || hipMemGetInfo(&f, &t) != hipSuccess)
      fail(__FILE__, __LINE__, "hipMemGetInfo failed");
    free_min = std::min<int64_t>(free_min, (int64_t)f);
    total = (int64_t)t;
  }
  if (a.share_gpu) free_min /= P;
  const int64_t reserve = (int64_t(2) << 30) + free_min / 100;
  const int dt = a.dtype == "fp32" ? 0 : 1;
  const int64_t n_owned = plan_max_grid(dt, P, free_min - reserve);
  sh.in.n = conv == Convention::Inclusive ? n_owned + 2 : n_owned;  // input.dat's n
  SolverConfig c{};
  c.n_rows = c.n_cols = n_owned;
  c.dtype = dt;
  const Footprint fp = solver_footprint(c, 0, P);
  if (!a.quiet)
    std::printf(" heat2d: --n max: n = %lld (%d rank%s, %s): %.2f GB per GPU of %.2f GB free (%.1f %%), %.2f GB total\n",
                (long long)sh.in.n, P, P > 1 ? "s" : "", a.dtype.c_str(), fp.total_bytes / 1e9, free_min / 1e9,
                100.0 * fp.total_bytes / free_min, total / 1e9);
}

// --transport auto: build every rank's RCCL communicator up front (one thread
// per rank: ncclCommInitRank is collective) and keep them only if EVERY rank
// got one; otherwise release the ones that did and run on the peer transport
// (device copies out of the neighbours' fields), so a node whose RCCL cannot
// initialise — or ranks sharing a GPU, which RCCL refuses — still runs. The
// reference has one fabric and fails with it (mpirun, fortran/hip/heat.F90:115-125).
// An init that neither returns nor fails within HEAT2D_RCCL_INIT_TIMEOUT
// seconds (default 120) ends the program with an error instead of a hang.
void choose_gpu_transport(Shared& sh) {
  const Args& a = sh.args;
  const int P = sh.nranks;
  std::vector<std::shared_ptr<Transport>> trs((size_t)P);
  std::vector<std::string> errs((size_t)P);
  if (const char* f = std::getenv("HEAT2D_FORCE_RCCL_FAIL"); f && std::atoi(f) != 0) {
    errs[0] = "HEAT2D_FORCE_RCCL_FAIL set (fallback test)";
  } else {
    rccl_unique_id(sh.uid);
    std::mutex mu;
    std::condition_variable cv;
    int finished = 0;
    std::vector<std::thread> th;
    for (int r = 0; r < P; ++r)
      th.emplace_back([&, r] {
        try {
          const int device = a.share_gpu ? 0 : r;
          trs[(size_t)r] = make_rccl_transport(sh.uid, r, P, device);
        } catch (const std::exception& e) {
          errs[(size_t)r] = e.what();
        }
        std::lock_guard<std::mutex> g(mu);
        ++finished;
        cv.notify_all();
      });
    const char* tv = std::getenv("HEAT2D_RCCL_INIT_TIMEOUT");
    const double limit = tv ? std::atof(tv) : 120.0;
    {
      std::unique_lock<std::mutex> lk(mu);
      if (!cv.wait_for(lk, std::chrono::duration<double>(limit), [&] { return finished == P; })) {
        std::fprintf(stderr, "heat2d: RCCL communicator init did not finish within %.0f s on every rank\n", limit);
        std::fflush(stderr);
        std::_Exit(1);  // threads stuck inside RCCL's bootstrap cannot be joined
      }
    }
    for (auto& t : th) t.join();
  }
  std::string why;
  for (int r = 0; r < P; ++r)
    if (!errs[(size_t)r].empty() && why.empty()) why = "rank " + std::to_string(r) + ": " + errs[(size_t)r];
  if (why.empty()) {
    sh.rccl_trs = std::move(trs);
    sh.transport_used = "rccl";
    return;
  }
  for (auto& t : trs)
    if (t) t->abort("RCCL unavailable on another rank: falling back to the peer transport");
  trs.clear();
  sh.peer_trs = make_peer_transports(P);
  sh.transport_used = "peer";
  sh.transport_note = "RCCL unavailable (" + why + ")";
  if (!a.quiet) std::fprintf(stderr, "heat2d: %s: falling back to the peer transport\n", sh.transport_note.c_str());
}

}  // namespace

int main(int argc, char** argv) {
  Shared sh;
  sh.args = parse_args(argc, argv);
  Args& a = sh.args;
  try {
    sh.in = read_input_file(a.input);
    if (a.n > 0) sh.in.n = a.n;
    if (a.ntime >= 0) sh.in.ntime = a.ntime;
    if (a.variant.empty()) a.variant = sh.in.nfields >= 6 ? "mpi" : "serial";
    if (a.variant != "mpi" && a.variant != "mpicuda" && a.variant != "serial" && a.variant != "cuda")
      fail(__FILE__, __LINE__, "--variant must be mpi, mpicuda, serial or cuda");
    const bool ghost = a.variant == "mpi" || a.variant == "mpicuda";
    Convention conv = ghost ? Convention::Ghost : Convention::Inclusive;
    std::string ic = a.ic.empty() ? (ghost ? "uniform" : a.variant == "cuda" ? "hat-cuda" : "hat") : a.ic;
    int ndev = 0;
    if (!a.cpu && hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0;
    if (!a.cpu && ndev == 0) {
      if (!a.quiet) std::fprintf(stderr, "no GPU found: running the CPU path\n");
      a.cpu = true;
    }
    sh.nranks = a.cpu ? std::max(1, a.gpus) : (a.gpus > 0 ? a.gpus : 1);
    if (a.n_max) plan_n_max(sh, ndev, conv);
    sh.prob = make_problem(sh.in, conv, ic);
    if (sh.prob.r > 0.25 + 1e-12 && !a.quiet)
      std::fprintf(stderr, "warning: r = %.6g > 0.25: FTCS is unstable in 2-D\n", sh.prob.r);
    if (a.transport != "auto" && a.transport != "rccl" && a.transport != "peer")
      fail(__FILE__, __LINE__, "--transport must be auto, rccl or peer");
    if (a.share_gpu && a.transport == "rccl")
      fail(__FILE__, __LINE__, "--share-gpu needs --transport peer or auto (RCCL refuses two ranks on one GPU)");
    if (!a.cpu && !a.share_gpu && sh.nranks > ndev) fail(__FILE__, __LINE__, "more GPUs requested than present");
    if (a.cpu && sh.nranks > 1) {
      sh.cpu_trs = make_thread_transports(sh.nranks);
      sh.transport_used = "host";
    } else if (sh.nranks > 1 && a.transport == "peer") {
      sh.peer_trs = make_peer_transports(sh.nranks);
      sh.transport_used = "peer";
    } else if (sh.nranks > 1 && a.transport == "auto") {
      choose_gpu_transport(sh);
    } else if (sh.nranks > 1) {
      rccl_unique_id(sh.uid);
      sh.transport_used = "rccl";
    }
  } catch (const std::exception& e) {
    std::fprintf(stderr, "heat2d: %s\n", e.what());
    return 1;
  }
  sh.t_elapsed.assign((size_t)sh.nranks, 0.0);
  sh.trs.assign((size_t)sh.nranks, nullptr);
  sh.rank_hist.assign((size_t)sh.nranks, std::vector<int64_t>(kMaxTB + 1, 0));
  sh.rank_halo_rows.assign((size_t)sh.nranks, 0);
  std::vector<std::thread> th;
  for (int r = 1; r < sh.nranks; ++r) th.emplace_back(run_rank, std::ref(sh), r);
  run_rank(sh, 0);
  for (auto& t : th) t.join();
  if (sh.failed) {
    std::fprintf(stderr, "heat2d: %s\n", sh.err.c_str());
    return 1;
  }
  double tmax = 0;
  for (double t : sh.t_elapsed) tmax = std::max(tmax, t);
  const int64_t ntime = sh.in.ntime - sh.start_step;  // steps this run executed
  const double pts = (double)sh.prob.n_owned * (double)sh.prob.n_owned;
  const double gpts = ntime > 0 && tmax > 0 ? pts * (double)ntime / tmax / 1e9 : 0.0;
  const int es = a.dtype == "fp32" ? 4 : 8;
  const int K = sh.tb_used;
  // passes (cycles) the timed loop launched, and their depths: the measured
  // schedule / balanced cycles decide them, not K alone
  int64_t passes = 0;
  std::string depths;
  for (int k = 1; k <= kMaxTB; ++k) {
    if (!sh.hist[k]) continue;
    passes += sh.hist[k];
    depths += (depths.empty() ? "" : ", ") + std::string("\"") + std::to_string(k) + "\": " + std::to_string(sh.hist[k]);
  }
  // model bytes/pt/step: one read + one write of the field per HBM pass; copy mode adds the copy
  const double bpp = a.copy_swap ? 4.0 * es
                                 : (passes > 0 && ntime > 0 ? 2.0 * es * (double)passes / (double)ntime : 2.0 * es / K);
  // fortran/mpi+cuda/heat.F90:275 prints gsum, whose reduction is commented
  // out (an uninitialised value); here it is the real all-reduced sum of T
  if (a.variant == "mpicuda") std::printf(" Sum of Temperature: %24.16g\n", sh.final_stats[0]);
  std::printf(" simulation completed!!!!\n");
  if (a.time_transfers && !a.quiet)
    std::printf(" heat2d: timed region includes the whole-field H2D (%.6f s) and D2H (%.6f s)\n", sh.t_h2d, sh.t_d2h);
  if (a.variant == "mpi")
    std::printf(" Average time: %24.16g\n", ntime > 0 ? tmax / (double)ntime : 0.0);
  else if (a.variant == "mpicuda")  // per iteration, fortran/mpi+cuda/heat.F90:292
    std::printf(" total time: %24.16g\n", ntime > 0 ? tmax / (double)ntime : 0.0);
  else
    std::printf(" total time: %24.16g\n", tmax);
  if (!a.quiet && sh.nranks > 1)
    std::printf(" heat2d: halo transport %s%s%s\n", sh.transport_used.c_str(), sh.transport_note.empty() ? "" : ": ",
                sh.transport_note.c_str());
  if (!a.quiet)
    std::printf(" heat2d: n=%lld P=%d %s K<=%d passes=%lld steps=%lld wall=%.6f s  %.3f Gpts/s  %.1f GB/s(model)  "
                "sum(T)=%.17g\n",
                (long long)sh.prob.n_owned, sh.nranks, a.dtype.c_str(), K, (long long)passes, (long long)ntime, tmax,
                gpts, gpts * bpp, sh.final_stats[0]);
  if (!a.json.empty()) {
    // per-rank cycles (identical on every rank by construction: Solver::prepare
    // agrees on the sequence) and halo rows moved per side
    std::string per_rank, halo;
    for (int r = 0; r < sh.nranks; ++r) {
      std::string d;
      for (int k = 1; k <= kMaxTB; ++k)
        if (sh.rank_hist[(size_t)r][(size_t)k])
          d += (d.empty() ? "" : ", ") + std::string("\"") + std::to_string(k) + "\": " +
               std::to_string(sh.rank_hist[(size_t)r][(size_t)k]);
      per_rank += (r ? ", {" : "{") + d + "}";
      halo += (r ? ", " : "") + std::to_string(sh.rank_halo_rows[(size_t)r]);
    }
    FILE* f = std::fopen(a.json.c_str(), "w");
    if (f) {
      std::fprintf(f,
                   "{\"n\": %lld, \"nranks\": %d, \"dtype\": \"%s\", \"tb\": %d, \"cycles\": {%s}, \"steps\": %lld, \"wall_s\": %.9g, "
                   "\"gpts_per_s\": %.9g, \"model_gb_per_s\": %.9g, \"sum\": %.17g, \"min\": %.17g, \"max\": %.17g, "
                   "\"backend\": \"%s\", \"variant\": \"%s\", \"arith\": \"%s\", \"cycles_per_rank\": [%s], "
                   "\"halo_rows_per_rank\": [%s], \"schedule\": \"%s\", \"arith_used\": \"%s\", "
                   "\"time_transfers\": %s, \"h2d_s\": %.9g, \"d2h_s\": %.9g, \"transport\": \"%s\", "
                   "\"transport_fallback\": %s}\n",
                   (long long)sh.prob.n_owned, sh.nranks, a.dtype.c_str(), K, depths.c_str(), (long long)ntime, tmax,
                   gpts, gpts * bpp,
                   sh.final_stats[0], sh.final_stats[2], sh.final_stats[3], a.cpu ? "cpu" : "hip", a.variant.c_str(),
                   a.arith.c_str(), per_rank.c_str(), halo.c_str(), sh.measured ? "measured" : "balanced",
                   sh.arith_used.c_str(), a.time_transfers ? "true" : "false", sh.t_h2d, sh.t_d2h,
                   sh.transport_used.c_str(), sh.transport_note.empty() ? "null" : json_str(sh.transport_note).c_str());
      std::fclose(f);
    }
  }
  return 0;
}
