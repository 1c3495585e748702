#!/usr/bin/env python3
"""Headline benchmark: stencil Gpoints/s (whole node) on the reference's own
benchmark configuration — fortran/hip/input.dat = `32768 0.25 0.05 1.0 25000 0`:
a 32768 x 32768 fp64 grid (ghost-frame convention, T=2 inside, Dirichlet T=1
frame, fortran/hip/heat.F90:274-282), slab-decomposed over N GPUs (strong
scaling: the grid is fixed), RCCL halo exchange over xGMI.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

W untimed warm-up steps, then exactly K FTCS time steps, bracketed by a
barrier + device synchronisation on both sides; the time is the MAX over
ranks. One "step" = one full time step of every grid point (temporal blocking
fuses up to --tb steps per HBM pass; every point is still updated every step).
Rank 0 prints one JSON line. Without torchrun, --gpus N > 1 starts the N rank
processes itself (and fails if fewer than N GPUs are visible).

The JSON reports what the timed region launched: `cycles` (depth -> cycles),
each depth's launch plan, and `hbm_gb_per_s_plan`, the DRAM traffic those
plans move per second (utils/metrics.plan_hbm_bytes: strip halos and priming
rows counted, no cache reuse assumed — an upper bound; rocprof cross-check in
profiles/hbm_model_check.md).

Arithmetic (--arith, default "bench": jacobi when r == 1/4, as here, else the
library's auto). The reference update is c + r*(sum - 4c)
(fortran/hip/heat_kernel.cpp:43). At r = 1/4 its centre weight 1 - 4r is zero
and the step is r * (((S + E) + N) + W) — the same sum, one exact multiply:
the kernels then carry the interior levels scaled by 4^level and spend 3 adds
+ 2 DPP moves per point and level instead of 5 + 2 (tb_impl.hpp, AR 2). On
this benchmark's IC (T = 2 inside, 1 on the frame) every value stays in
[1, 2], so sum - 4c is exact (Sterbenz) and the field is bitwise identical to
--arith exact (GPU-checked: tests/test_jacobi.py::
test_hip_jacobi_equals_exact_on_reference_ic). --arith auto (fma, also bitwise
identical here) and exact remain available. The timed field is checked
bitwise against the run-time compiled r * sum form and against the reference
rounding: bitwise on this IC, within the stated bound on data where sum - 4c
rounds (--ic hotspot, the zero + hot-spot data BASELINE.json names).

Multi-rank runs (--transport auto): RCCL, and the IPC transport only where
RCCL cannot be built on every rank. Transport and solver construction are
bounded (HEAT2D_INIT_TIMEOUT); the JSON proves the decomposition per rank:
what RCCL reports (ncclCommCount / ncclCommUserRank / ncclCommCuDevice), the
PCI bus id of each rank's device, its slab rows and its own timed ms.

vs_baseline: the reference publishes no numbers. We divide by the
derived reference ceiling of BASELINE.md — 50 Gpts/s per MI250X GCD for its
kernel + per-step D2D copy (>= 32 B/pt/step at 1.6 TB/s) — times N ranks.
"""
import argparse
import gc
import json
import math
import os
import sys
import time

_ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, _ROOT)

REF_GPTS_PER_RANK = 50.0  # BASELINE.md derived ceiling, 1 MI250X GCD, fp64


def arith_name(r, arith):
    """The update form the run uses (see --arith)."""
    import math
    if arith == "auto":
        return "fma" if r > 0 and math.frexp(r)[0] == 0.5 else "exact"
    return arith


def _free_port():
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _launch_ranks(n, backend, share_gpu=False):
    """`python bench.py --gpus N` without torchrun: start N rank processes of
    this script (one per GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set,
    rendezvous on 127.0.0.1) and return the exit status. Rank 0 prints the
    JSON line on the inherited stdout. If a rank fails, the others are
    terminated (they would block in RCCL forever) and its status is returned.
    Runs before this process touches the GPU: children are started, never
    exec'd over a GPU-initialised process."""
    import signal
    import subprocess
    if backend == "hip" and not share_gpu:
        import torch  # device_count() does not initialise the GPU on this image
        have = torch.cuda.device_count()
        if have < n:
            print(f"bench.py: --gpus {n} but only {have} GPU(s) visible", file=sys.stderr)
            return 2
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                print(f"bench.py: rank {procs.index(p)} exited with {code}; stopping the others", file=sys.stderr)
                for q in live:
                    q.send_signal(signal.SIGTERM)
        if live:
            try:
                live[0].wait(timeout=0.2)
            except subprocess.TimeoutExpired:
                pass
    return rc


def _claim_stdout():
    """Keep the driver's stdout for the ONE JSON line: RCCL (torch's and ours)
    prints a version banner on stdout from C at communicator init, and C stdio
    buffers flush at exit. Point fd 1 at stderr for the whole run and return a
    private duplicate of the real stdout for the result line."""
    sys.stdout.flush()
    fd = os.dup(1)
    os.dup2(2, 1)
    return fd


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=480)
    ap.add_argument("--warmup", type=int, default=48)
    ap.add_argument("--n", "--grid", dest="n", default="32768",
                    help="grid edge (use --grid under torchrun: its parser takes --n as an abbreviation), or 'max': "
                         "the memory-fit planner's largest grid (utils/memplan.py: free device memory minus a "
                         "reserve; --weak: the largest global grid on N GPUs, else the largest 1-GPU grid)")
    ap.add_argument("--ic", default="uniform", choices=["uniform", "hotspot", "hat"],
                    help="initial data: uniform (default) — the reference benchmark's own IC, T = 2 inside a "
                         "Dirichlet T = 1 frame (fortran/hip/heat.F90:274-282); hotspot — the zero field with a "
                         "unit hot spot BASELINE.json names (utils/config.make_ic); hat — the serial solver's "
                         "T = 2 box in T = 1 (fortran/serial/heat.f90:40-48)")
    ap.add_argument("--sigma", type=float, default=0.25,
                    help="input.dat sigma (= r, the FTCS coefficient); the reference's inputs all use 0.25")
    ap.add_argument("--weak", action="store_true",
                    help="weak scaling: --n is the 1-GPU grid edge; the global square grid grows to n*sqrt(N) so "
                         "every rank keeps ~n^2 points (e.g. --dtype fp32 --n 173056: the full-HBM 240 GB per GPU)")
    ap.add_argument("--dtype", default="fp64", choices=["fp64", "fp32"])
    ap.add_argument("--tb", type=int, default=0,
                    help="largest time-step depth fused per HBM pass (0: every depth the kernels have, 24; "
                         "prepare() picks the cycle schedule of the timed steps by measurement)")
    ap.add_argument("--tile-rows", type=int, default=0)
    ap.add_argument("--arith", default="bench", choices=["bench", "auto", "exact", "fma", "jacobi", "fast"],
                    help="fma: contracted update (one op fewer per point); exact: every op rounded; auto: fma when "
                         "bitwise identical to exact (r a power of two, as here), else exact; jacobi: r == 1/4 "
                         "only, r * (S + E + N + W) (3 adds per point; bitwise == exact on this benchmark's IC); "
                         "fast: any r, levels carried as T / r^level (3 adds + 1 fma per point, within a stated "
                         "error bound of exact); bench (default): jacobi when r == 1/4, else auto")
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--graph", default="auto", choices=["auto", "on", "off"],
                    help="replay the timed schedule from one hipGraph captured in prepare() (auto: single-rank "
                         "runs without an exchange, schedules of cycles under 400 us — longer ones launch eager, "
                         "HEAT2D_GRAPH_MAX_CYCLE_US; on: every schedule; exchanging runs stay eager — a graph launch starts the "
                         "interior ~40 us after the band launch, eager ~12 us: 4096-row IPC slab rehearsal "
                         "3362-3468 with the graph, 3768-3943 eager, profiles/r4/k/)")
    ap.add_argument("--comm-cus", type=int, default=0, help="CUs reserved for bands + RCCL (0: default, -1: none)")
    ap.add_argument("--check", action="store_true", help="print field statistics after the run")
    ap.add_argument("--phase-timers", action="store_true",
                    help="record hipEvent phase timers in the timed region and report them (adds event records)")
    ap.add_argument("--rows", type=int, default=0,
                    help="with --rehearse-comm: rows of the slab (e.g. 4096 = one of 8 ranks of 32768)")
    ap.add_argument("--slab-pos", default="middle", choices=["first", "middle", "last"],
                    help="with --rehearse-comm --rows R: which rank's slab of the grid the rehearsal owns — the "
                         "first / last (the global frame row on one side, rank 0 / N-1) or a middle one")
    ap.add_argument("--edge-shift", default="auto",
                    help="rows each edge slab (rank 0 and the last rank, the global frame rows on one side) gives "
                         "to the middle slabs of a >= 3-rank run: an integer, or auto (default): measured — every "
                         "rank times its own slab alone (1-rank loop-exchange rehearsal: RCCL's, or IPC's where the "
                         "run falls back to it) uniform, then with "
                         "the estimated shift, and the shift is kept if the slowest slab gets faster "
                         "(parallel/select.balance_edges; one rank after another with --share-gpu); measure: "
                         "the same on any backend (the CPU rehearsal of this path). JSON config.decomposition")
    ap.add_argument("--balance-loop", default="auto", choices=["auto", "rccl", "ipc"],
                    help="--edge-shift auto: the loop exchange of the slab rehearsals (auto: RCCL's when the run "
                         "tries RCCL first and ranks own their GPUs, else IPC's)")
    ap.add_argument("--backend", default="hip", choices=["hip", "cpu"],
                    help="cpu: the same harness on the native CPU twin over gloo (CI rehearsal of the "
                         "multi-process path: tests/test_bench_contract.py); not a performance number")
    ap.add_argument("--transport", default="auto", choices=["auto", "best", "rccl", "ipc", "peer", "host"],
                    help="halo exchange between rank processes: rccl (RCCL send/recv over xGMI), ipc (alias peer: "
                         "no RCCL, the neighbours' fields mapped through hipIpc handles, halos pulled by device "
                         "copies ordered by stream-side counters; capturable into hipGraphs), auto (default): RCCL, "
                         "and IPC only where RCCL cannot be built on every rank (a transport that fails to "
                         "initialise on any rank is skipped on every rank), or best: build both, time the real "
                         "timed loop with each (MAX over ranks) and keep the faster; host: halos staged through "
                         "pinned host memory over torch.distributed (gloo), auto's last resort")
    ap.add_argument("--share-gpu", action="store_true",
                    help="every rank on GPU 0: the exact multi-process path on a 1-GPU box (RCCL refuses two ranks "
                         "on one GPU, so auto falls back to ipc); a correctness / overhead rehearsal, not a node "
                         "throughput")
    ap.add_argument("--verify", default="on", choices=["on", "off"],
                    help="after the timed run: a small uneven rough-data problem on the same transport kind and "
                         "rank layout, gathered and compared bitwise with the NumPy golden (JSON 'verified')")
    ap.add_argument("--field-check", default="auto", choices=["auto", "full", "windows", "off"],
                    help="after the timed run (untimed): its field checked against the run-time compiled one-step "
                         "kernel in the reference arithmetic from the same IC (JSON 'timed_field_check'); auto: the "
                         "whole slab when a second copy fits, else row windows at the slab boundaries and middle")
    ap.add_argument("--window-rows", type=int, default=64, help="rows per checked window (--field-check windows)")
    ap.add_argument("--measure-hbm", action="store_true",
                    help="1 rank: after the run, re-run the timed region twice under rocprofv3 --pmc (FETCH_SIZE, "
                         "then WRITE_SIZE; child processes, the same plans and schedule through the plan cache) and "
                         "report the DRAM bytes of its stencil dispatches over this run's timed seconds "
                         "(JSON 'hbm_gb_per_s_measured')")
    ap.add_argument("--hbm-child", default="", help=argparse.SUPPRESS)
    ap.add_argument("--rehearse-comm", action="store_true",
                    help="1 GPU only: run the multi-GPU schedule (bands + RCCL self-exchange beside a CU-masked "
                         "interior) to measure its per-rank cost; not the headline (periodic halo)")
    args = ap.parse_args()
    import faulthandler
    faulthandler.enable()  # Python stacks on a fatal signal (the native library adds its backtrace)
    if args.transport == "peer":
        args.transport = "ipc"
    if args.graph == "on":  # replay every measured schedule, long cycles too
        os.environ.setdefault("HEAT2D_GRAPH_MAX_CYCLE_US", "1e30")
    if args.share_gpu and args.transport == "rccl":
        ap.error("--share-gpu needs --transport ipc or auto (RCCL refuses two ranks on one GPU)")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(_launch_ranks(args.gpus, args.backend, args.share_gpu))
    if args.measure_hbm and os.environ.get("HEAT2D_PLAN_CACHE", "") in ("", "off") and not args.hbm_child:
        # the profiled re-runs take this run's plans from a cache file (their
        # own trials would be timed under counter collection)
        import tempfile
        os.environ["HEAT2D_PLAN_CACHE"] = os.path.join(tempfile.mkdtemp(prefix="heat2d_hbm_"), "plans.txt")
    out_fd = _claim_stdout()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    hip = args.backend == "hip"
    device = 0 if args.share_gpu else local
    if hip:
        torch.cuda.set_device(device)
    if world > 1:
        # Host collectives (barriers, the timing MAX, the transport choice, the
        # RCCL unique id) over gloo: the halo fabric is the native transport's
        # own (an RCCL communicator or IPC mappings), whichever wins. A dead
        # peer fails the run instead of hanging it: the native transports'
        # watchdogs use the same limit.
        from datetime import timedelta
        to = timedelta(seconds=float(os.environ.get("HEAT2D_COMM_TIMEOUT", "600")))
        dist.init_process_group("gloo", timeout=to)

    def reduce(v, op):
        if world == 1:
            return float(v)
        t = torch.tensor([float(v)], dtype=torch.float64)
        dist.all_reduce(t, op=op)
        return float(t.item())

    amin = (lambda v: reduce(v, dist.ReduceOp.MIN))
    amax = (lambda v: reduce(v, dist.ReduceOp.MAX))

    def sync():
        if hip:
            torch.cuda.synchronize()

    def barrier():
        if world > 1:
            dist.barrier()
        sync()

    import heat2d
    from heat2d.models.heat2d import HeatSolver
    from heat2d.parallel import select
    from heat2d.parallel.transport import (IpcLoopTransport, IpcTransport, RcclLoopTransport, RcclTransport,
                                           SelfTransport, TorchDistTransport)

    mem_plan = None
    if args.n == "max":
        # the largest grid the free device memory holds (rank 0's slab is the
        # largest): over `world` ranks for weak scaling, one GPU's for strong
        # scaling (a fixed total problem); min free memory over the ranks
        from heat2d.utils import memplan
        if hip:
            free = memplan.mem_info(device)[0] / (world if args.share_gpu else 1)
        else:
            free = 64 << 20  # CPU rehearsal of the planner: a 64 MiB "device"
        free = int(amin(free))
        mem_plan = memplan.plan_max_grid(args.dtype, world if args.weak else 1, free_bytes=free,
                                         reserve=memplan.reserve_bytes(free) if hip else 0)
        n_glob = mem_plan["n"]
        n_per_gpu = n_glob if not args.weak else int(round(n_glob / math.sqrt(world)))
    else:
        n_per_gpu = int(args.n)
        n_glob = n_per_gpu
        if args.weak:
            n_glob = int(round(n_per_gpu * math.sqrt(world)))
    inp = heat2d.InputDat(n=n_glob, sigma=args.sigma, nu=0.05, dom_len=1.0, ntime=args.steps, soln=0, nfields=6)
    prob = heat2d.make_problem(inp, "ghost", args.ic)
    arith = args.arith if args.arith != "bench" else ("jacobi" if prob.r == 0.25 else "auto")
    rows = args.rows if (args.rows and world == 1) else None
    # a rehearsal of one rank's slab is a MIDDLE slab of the grid (interior
    # boundary bands, as on rank 3 of 8); --rows alone is a standalone rows x n grid
    slab_row0 = None
    if rows and args.rehearse_comm:
        slab_row0 = {"first": 0, "middle": (prob.n_owned - rows) // 2, "last": prob.n_owned - rows}[args.slab_pos]

    def make_transport(kind):
        if kind == "rccl":
            return RcclTransport(rank, world, device)
        if kind == "ipc":
            return IpcTransport(device)
        if kind == "torch-dist":
            return TorchDistTransport()
        if kind == "rccl-loop":
            return RcclLoopTransport(device)
        if kind == "ipc-loop":
            return IpcLoopTransport(device)
        return SelfTransport()

    def uses_graph(kind):
        # auto: graphs for single-rank runs without an exchange (their short
        # cycles are launch-bound: the small grid); "on": also IPC (RCCL's exchange does not capture)
        if not hip or args.graph == "off":
            return False
        return kind == "self" or (args.graph == "on" and kind in ("ipc", "ipc-loop"))

    edge_shift = [0]  # the decomposition's edge shift (balance_edges below)

    def build(kind, tr):
        return HeatSolver(prob, dtype=args.dtype, backend=args.backend, tb=args.tb, overlap=not args.no_overlap,
                          graph=uses_graph(kind), tile_rows=args.tile_rows, transport=tr,
                          device=device if hip else None, rows=rows, comm_cus=args.comm_cus, arith=arith,
                          slab_row0=slab_row0, edge_shift=edge_shift[0])

    own_s = [0.0]  # this rank's own seconds of the last timed run (the JSON's per-rank proof)

    def timed(s):
        # no collector pause inside a sub-ms timed region (and no gc.collect()
        # here: its pause idles the GPU, whose clocks then drop before a 3 ms
        # timed run — 4096^2 fp32: 5008-5153 Gpts/s with it, profiles/r4/l/)
        gc.disable()
        barrier()
        t0 = time.perf_counter()
        s.step(args.steps)
        s.synchronize()
        sync()
        t1 = time.perf_counter()
        barrier()
        gc.enable()
        own_s[0] = t1 - t0
        return amax(t1 - t0)

    live = {}  # kind -> (transport, solver, prepare seconds)
    warm_s = {}  # kind -> warm-up seconds

    init_timeout = float(os.environ.get("HEAT2D_INIT_TIMEOUT", "300"))

    def setup(kind):
        """Transport + solver + warm-up + prepare(steps), each phase collective:
        a failure on any rank raises Skip on every rank. Construction is
        bounded (select.deadline, HEAT2D_INIT_TIMEOUT, default 300 s): a rank
        blocked inside a native init call (RCCL bootstrap, an IPC import) exits
        non-zero and the launcher stops the others — no hang."""
        with select.deadline(init_timeout, f"{kind} transport construction", rank):
            tr, why = select.try_collective(lambda: make_transport(kind), amin,
                                            cleanup=lambda t: (t.abort("another rank failed to initialise"),
                                                               t.close()))
        if why is not None:
            raise select.Skip(why)
        with select.deadline(init_timeout, f"{kind} solver construction (field allocation, peer attach)", rank):
            s, why = select.try_collective(lambda: build(kind, tr), amin, cleanup=lambda x: x.close())
        if why is not None:
            tr.close()
            raise select.Skip(why)
        tw = time.perf_counter()
        s.step(args.warmup)
        s.synchronize()
        warm_s[kind] = time.perf_counter() - tw  # (the warm-up's own depths are planned / autotuned here)
        # plan / autotune every depth the timed run uses, pick its cycle schedule
        # by measurement, and end on non-mutating trial cycles of that schedule
        # (GPU clocks as in a long run) — outside the timed region, after the warmup
        tp = time.perf_counter()
        s.prepare(args.steps)
        live[kind] = (tr, s, time.perf_counter() - tp)
        return s

    def release(kind):
        tr, s, _ = live.pop(kind)
        s.close()
        tr.close()

    from heat2d.ops import _native as N
    balance_report = None
    if args.edge_shift not in ("auto", "measure"):
        edge_shift[0] = int(args.edge_shift)
    elif world >= 3 and (hip or args.edge_shift == "measure") and not args.rehearse_comm:
        # Edge-balanced slabs (profiles/r6/b/: an edge
        # slab's frame-side band runs on the general kernel and ends ~30 us
        # after the interior at N = 8, so rank 0 and the last rank set the
        # MAX). Each rank times its own slab alone — a 1-rank loop exchange
        # of its boundary bands, the bench's own warmup / prepare / timed
        # step — before any transport or field of the real run exists. The
        # loop is the run's own kind of exchange: RCCL's channel kernels share
        # the CUs with the bands (a 1-rank RCCL communicator per GPU), the IPC
        # loop is local device copies; their edge excesses differ 2x
        # (profiles/r6/h/: 41 vs ~80 us at N = 8).
        # (--backend cpu --edge-shift measure: the CI rehearsal of this path,
        # each rank's slab on the CPU twin without an exchange)
        first = select.candidate_transports(args.transport, world, hip)[0]
        loop_kind = "self" if not hip else (("rccl-loop" if first == "rccl" and not args.share_gpu else "ipc-loop")
                                            if args.balance_loop == "auto" else args.balance_loop + "-loop")

        def own_slab_ms(shift):
            r0, nr = N.decompose(prob.n_owned, world, rank, shift)

            def make():
                tr_l = make_transport(loop_kind)
                try:
                    s_l = HeatSolver(prob, dtype=args.dtype, backend=args.backend, tb=args.tb,
                                     overlap=not args.no_overlap, graph=False, tile_rows=args.tile_rows,
                                     transport=tr_l, device=device if hip else None, rows=nr,
                                     comm_cus=args.comm_cus, arith=arith, slab_row0=r0)
                except Exception:
                    tr_l.close()
                    raise
                return s_l, lambda: (s_l.close(), tr_l.close())

            def run():
                return select.time_own_slab(make, args.steps, args.warmup, sync=sync)
            if not args.share_gpu:
                return run()
            # ranks sharing one GPU take turns (their rehearsals would contend)
            v = float("nan")
            for r in range(world):
                if r == rank:
                    try:
                        v = run()
                    except Exception:  # noqa: BLE001 - reported as NaN by balance_edges
                        import traceback
                        traceback.print_exc()
                barrier()
            return v

        def gather_ms(v):
            t = torch.zeros(world, dtype=torch.float64)
            t[rank] = v
            dist.all_reduce(t)
            return t.tolist()

        tb0 = time.perf_counter()
        with select.deadline(init_timeout, "edge-balance rehearsal of the slabs", rank):
            edge_shift[0], balance_report = select.balance_edges(
                own_slab_ms, gather_ms, lambda d: [N.decompose(prob.n_owned, world, r, d)[1] for r in range(world)],
                cap=(prob.n_owned // world) // 4)
        balance_report["loop"] = loop_kind
        balance_report["seconds"] = round(time.perf_counter() - tb0, 2)
        if rank == 0:
            print(f"bench.py: edge balance: shift {edge_shift[0]} rows: {json.dumps(balance_report)}",
                  file=sys.stderr, flush=True)
        barrier()

    cands = select.candidate_transports(args.transport, world, hip)
    choice_report = None
    if cands:
        field_bytes = 2.0 * (prob.n_owned / world + 48) * (prob.n_owned + 128) * (8 if args.dtype == "fp64" else 4)

        def trial(kind):
            s = setup(kind)
            ms = min(timed(s) for _ in range(2)) * 1e3
            if hip and kind != cands[-1]:
                # keep this candidate for the timed run only if another solver fits beside it
                free = torch.cuda.mem_get_info(device)[0] / (world if args.share_gpu else 1)
                if amin(free) < 1.5 * field_bytes:
                    release(kind)
            return ms

        chosen, choice_report = select.choose_transport(cands, trial, amin, amax,
                                                        first_working=args.transport != "best")
        if chosen is None:
            # exit without interpreter teardown: a candidate's native init may
            # still be blocked on a helper thread (the bounded IPC attach)
            print(f"bench.py: no transport works on every rank: {choice_report}", file=sys.stderr, flush=True)
            os._exit(3)
        for k in list(live):
            if k != chosen:
                release(k)
        if chosen not in live:
            setup(chosen)
        else:
            # the trials advanced the field: back to the IC and the same warm-up,
            # so the timed run starts from the state a single-rank run times
            # (plans, schedule and graphs stay; prepare() re-warms the clocks)
            tr_c, s_c, prep = live[chosen]
            s_c.synchronize()
            barrier()
            s_c.init()
            s_c.step(args.warmup)
            s_c.synchronize()
            tp = time.perf_counter()
            s_c.prepare(args.steps)
            live[chosen] = (tr_c, s_c, prep + time.perf_counter() - tp)
        kind = chosen
    else:
        kind = ("torch-dist" if world > 1 else
                (("ipc-loop" if args.transport == "ipc" else "rccl-loop") if (args.rehearse_comm and hip) else "self"))
        setup(kind)
    def hbm_marker():
        """A 16-byte read kernel: brackets the timed region's dispatches in the profile."""
        from heat2d.ops import _native as native
        buf = torch.zeros(64, dtype=torch.uint8, device=f"cuda:{device}")
        sink = torch.zeros(16, dtype=torch.uint8, device=f"cuda:{device}")
        torch.cuda.synchronize()
        native.call("heat2d_read", buf.data_ptr(), 16, sink.data_ptr(), None, 1)
        torch.cuda.synchronize()

    def measure_hbm(elapsed, nrows, ncols):
        """DRAM bytes of the timed region: two child processes re-run this
        bench (same flags, this run's plans and schedule from the plan cache,
        HEAT2D_PLAN_CACHE_TRUST: no re-timing under the profiler) under
        rocprofv3 --pmc, one counter set each (FETCH_SIZE needs 3 of the 4
        TCC counters, WRITE_SIZE 2), the program right after `--`. The
        stencil dispatches between the child's two marker dispatches are its
        timed region; FETCH_SIZE is doubled (gfx950 counts wide streaming
        reads at half: MI355X_MICROARCH.md §HBM, profiles/r4/c/). The rate is
        over THIS run's timed seconds."""
        import csv
        import glob
        import shutil
        import subprocess
        import tempfile
        rocprof = shutil.which("rocprofv3")
        if not rocprof:
            return {"error": "rocprofv3 not found"}
        # the parent's resolved grid (a child planning --grid max itself would see
        # less free memory), everything else as given
        argv, skip = [], False
        for a in sys.argv[1:]:
            if skip:
                skip = False
                continue
            if a in ("--n", "--grid"):
                skip = True
                continue
            if a == "--measure-hbm" or a == "--weak" or a.startswith(("--n=", "--grid=")):
                continue
            argv.append(a)
        argv += ["--grid", str(n_glob)]
        out = {"method": "rocprofv3 --pmc FETCH_SIZE (x2) / WRITE_SIZE over the stencil dispatches of two "
                         "profiled re-runs of the timed region (same plans); rate over this run's timed seconds"}
        tot = {}
        work = tempfile.mkdtemp(prefix="heat2d_hbm_prof_")
        from heat2d.ops import _native as native
        env = dict(os.environ, HEAT2D_PLAN_CACHE=native.plan_cache_path(), HEAT2D_PLAN_CACHE_TRUST="1")
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(work, ctr)
            info = os.path.join(work, ctr + ".json")
            cmd = ["timeout", "-s", "KILL", "300", rocprof, "--pmc", ctr, "--output-format", "csv", "-d", d, "--",
                   sys.executable, os.path.abspath(__file__), *argv, "--hbm-child", info, "--verify", "off",
                   "--field-check", "off"]
            p = subprocess.run(cmd, capture_output=True, text=True, env=env, cwd=work)
            if p.returncode != 0 or not os.path.exists(info):
                # the child's own lines (rocprofv3 logs with a glog prefix: [IWE]yyyymmdd ...)
                own = [ln for ln in p.stderr.splitlines() if not (len(ln) > 9 and ln[0] in "IWE" and ln[1:9].isdigit())]
                with open(os.path.join(work, ctr + ".stderr"), "w") as f:
                    f.write(p.stderr)
                return dict(out, error=f"{ctr} pass failed (rc {p.returncode}); stderr kept in {work}: "
                                       + "\n".join(own[-25:]))
            rows_ = []
            for fcsv in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
                rows_ += list(csv.DictReader(open(fcsv)))
            marks = sorted(int(r["Dispatch_Id"]) for r in rows_ if "read16_kernel" in r["Kernel_Name"])
            if len(marks) < 2:
                return dict(out, error=f"{ctr}: timed-region markers not found in the profile")
            lo, hi = marks[-2], marks[-1]
            sel = [r for r in rows_ if lo < int(r["Dispatch_Id"]) < hi and "tb_kernel" in r["Kernel_Name"]
                   and r["Counter_Name"] == ctr]
            tot[ctr] = sum(float(r["Counter_Value"]) for r in sel) * 1024.0  # KiB
            out[ctr.lower() + "_dispatches"] = len({r["Dispatch_Id"] for r in sel})
            child = json.load(open(info))
            if (child.get("n"), child.get("nrows")) != (n_glob, nrows):
                return dict(out, error=f"{ctr}: the profiled child ran n={child.get('n')} nrows={child.get('nrows')}, "
                                       f"not this run's n={n_glob} nrows={nrows}")
            out["child_cycles"] = child["cycles"]
        shutil.rmtree(work, ignore_errors=True)
        rd, wr = 2.0 * tot["FETCH_SIZE"], tot["WRITE_SIZE"]
        es = 8 if args.dtype == "fp64" else 4
        field = float(nrows) * ncols * es
        out.update({"read_bytes": rd, "write_bytes": wr, "read_over_field_per_cycle":
                    round(rd / field / max(1, sum(out["child_cycles"].values())), 4),
                    "gb_per_s": round((rd + wr) / elapsed / 1e9, 1)})
        return out

    def timed_field_check(s, kind):
        """The timed field itself (IC + warmup + steps, the state the timed run
        left), checked against an independent engine started from the same IC:
        the run-time compiled one-step kernel (hipRTC, ops/jit.py) in the
        reference arithmetic, run for warmup + steps steps on the same rank
        layout through a fresh transport of the same kind, compared on the
        device (max |diff| and differing bit patterns, reduced over ranks).
        When a second copy of the slab does not fit (the full-HBM grids), row
        windows at both slab boundaries and the middle of every slab are
        checked by single-rank reference runs instead (select.field_windows).
        Outside the timed region. Skipped for the self-exchange rehearsals
        (their periodic halo is not the problem's physics)."""
        if kind in ("rccl-loop", "ipc-loop"):
            return {"skipped": "self-exchange rehearsal: not the problem's physics"}
        total = args.warmup + args.steps
        es = 8 if args.dtype == "fp64" else 4
        if hip:
            need = 2.0 * (s.nrows + 2 * s.layout.halo) * s.layout.pitch * es + (256 << 20)
            free = torch.cuda.mem_get_info(device)[0] / (world if args.share_gpu else 1)
            fits = args.field_check == "full" or (args.field_check == "auto" and free >= 1.05 * need)
        else:
            fits = args.field_check != "windows"
        full = amin(1.0 if fits else 0.0) >= 1.0

        def make_ref(full_run, rows=None, slab_row0=None, arith="exact"):
            if full_run:
                vkind = kind
                tr_ref = make_transport(vkind)
                rr, r0 = (s.nrows, slab_row0_run) if rows_run else (None, None)
            else:
                tr_ref = SelfTransport()
                rr, r0 = rows, slab_row0
            try:
                ref = HeatSolver(prob, dtype=args.dtype, backend=args.backend, transport=tr_ref,
                                 device=device if hip else None, rows=rr, slab_row0=r0, arith=arith,
                                 engine="jit" if hip else "tb", tb=1, overlap=False, graph=False, autotune=0,
                                 edge_shift=edge_shift[0] if full_run else 0)
            except Exception:
                tr_ref.close()
                raise
            close = ref.close

            def close_both():
                close()
                tr_ref.close()
            ref.close = close_both
            return ref

        rows_run = rows
        slab_row0_run = slab_row0
        t0 = time.perf_counter()
        out = select.check_timed_field(s, make_ref, total, arith=arith_name(prob.r, arith), r=prob.r,
                                       dtype=args.dtype, t0_absmax=prob.ic.absmax(), full=full, amax=amax,
                                       asum=lambda v: reduce(v, dist.ReduceOp.SUM), window=args.window_rows,
                                       sterbenz=prob.ic.sterbenz_safe())
        out["seconds"] = round(time.perf_counter() - t0, 2)
        if not hip:
            for d in [out] + [v for k, v in out.items() if k.startswith("vs_")]:
                d["engine"] = d["engine"].replace("jit", "cpu")
        return out

    tr, s, prepare_s = live[kind]
    s.cycle_hist(reset=True)
    s.halo_rows_exchanged(reset=True)
    if args.phase_timers:
        s.set_timing(True)
    if args.hbm_child:
        # --measure-hbm's profiled re-run: the timed region between two marker
        # dispatches (read16_kernel), nothing after it
        hbm_marker()
        elapsed = timed(s)
        hbm_marker()
        with open(args.hbm_child, "w") as f:
            json.dump({"elapsed": elapsed, "cycles": {str(k): c for k, c in s.cycle_hist().items()}, "n": n_glob,
                       "nrows": s.nrows}, f)
        s.close()
        tr.close()
        return
    elapsed = timed(s)

    pts = float(prob.n_owned) * float(rows or prob.n_owned)
    gpts = pts * args.steps / elapsed / 1e9
    es = 8 if args.dtype == "fp64" else 4
    info = s.info()
    tb = info["tb"]
    # what the timed region launched: cycles per depth (this rank), each depth's
    # launch plan, and the DRAM traffic those plans move (strip halos W vs U and
    # the 2k priming rows per band counted; no cache reuse assumed)
    hist = s.cycle_hist()
    assert sum(k * c for k, c in hist.items()) == args.steps, hist
    plans, traffic = {}, 0.0
    from heat2d.utils.metrics import plan_hbm_bytes
    from heat2d.ops import _native as N
    for k, c in sorted(hist.items()):
        pl = s.plan(k) if hip else {"k": k, "valid": 0}
        if hip:
            plans[str(k)] = {kk: pl[kk] for kk in ("order", "dynamic", "origin", "ring", "main_bands", "main_waves",
                                                    "edge_items", "tuned_ms")}
        traffic += c * plan_hbm_bytes(pl, es, s.nrows, s.ncols)["total"]
    # halo traffic of the timed region: each exchange moves the NEXT cycle's
    # depth in whole padded rows, one message per neighbour
    nmsg = 2 if (args.rehearse_comm and world == 1) else (rank > 0) + (rank < world - 1)
    halo_bytes = float(s.halo_rows_exchanged()) * s.layout.pitch * es * nmsg
    if world > 1:
        tt = torch.tensor([traffic, halo_bytes], dtype=torch.float64)
        dist.all_reduce(tt)
        traffic, halo_bytes = float(tt[0].item()), float(tt[1].item())
    stats = s.stats() if args.check else None
    phases = s.phase_times() if args.phase_timers else None
    plan_cache = {"hits": s.plan_cache_hits, "path": N.plan_cache_path()} if hip else None
    tune = s.tune_stats if hip else None
    measured = s.schedule(args.steps) is not None
    # a measured schedule of long cycles launches eagerly even with graph=True
    replayed = bool(uses_graph(kind)) and (s.schedule_replayed(args.steps) if measured else True)
    # per-rank proof of the decomposition (what the fabric reports, devices, own timings)
    gather = ((lambda me: (lambda out: (dist.all_gather_object(out, me), out)[1])([None] * world))
              if world > 1 else (lambda me: [me]))
    proof = select.rank_report(gather, rank=rank, device=device if hip else None, transport=tr, rows=s.nrows,
                               row0=s.row0, timed_s=own_s[0], extra={"transport": tr.name})
    field_check = None
    if args.field_check != "off":
        field_check = timed_field_check(s, kind)
    nrows_run, ncols_run = s.nrows, s.ncols
    s.close()
    tr.close()
    live.clear()
    hbm = None
    if args.measure_hbm:
        # (after this run's solver is gone: the profiled children get the whole GPU)
        hbm = (measure_hbm(elapsed, nrows_run, ncols_run) if hip and world == 1
               else {"error": "--measure-hbm profiles single-rank GPU runs"})
    verify = None
    if args.verify == "on":
        # the chosen transport kind and rank layout on a small uneven problem
        # (a rehearsal's self-exchange is not physics: its slab verifies alone)
        vkind = kind if kind not in ("rccl-loop", "ipc-loop") else "self"
        verify = select.verify_decomposition(lambda: make_transport(vkind), rank=rank, world=world,
                                             dtype=args.dtype, arith=arith, backend=args.backend,
                                             device=device if hip else None, graph=uses_graph(vkind), r=prob.r)
    if rank == 0:
        out = {
            "metric": "stencil Gpoints/sec (whole node)",
            "value": round(gpts, 3),
            "unit": "Gpts/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 6),
            "higher_is_better": True,
            "scaling": "weak" if args.weak else "strong",
            "vs_baseline": round(gpts / (REF_GPTS_PER_RANK * world), 3),
            "dtype": args.dtype,
            "data": {"uniform": "synthetic (reference benchmark IC: T=2 interior, Dirichlet T=1 frame)",
                     "hotspot": "synthetic (zero field + unit hot spot on [0.4, 0.6]^2 L, zero Dirichlet frame)",
                     "hat": "synthetic (fortran/serial IC: T=2 on [0.5, 1.5]^2, T=1 elsewhere)"}[args.ic],
            "config": {
                "model": (f"heat2d FTCS 5-point, weak scaling: {n_per_gpu}^2 points per GPU (global {n_glob}^2)"
                          + (" — the memory-fit planner's largest grid" if mem_plan else "") if args.weak
                          else "heat2d FTCS 5-point, fortran/hip/input.dat (32768 0.25 0.05 1.0 25000 0)"
                          if n_glob == 32768 and args.sigma == 0.25 and args.ic == "uniform"
                          else f"heat2d FTCS 5-point, {n_glob}^2 (sigma {args.sigma:g}, nu 0.05, L 1.0, IC {args.ic})"),
                "grid": [rows or prob.n_owned, prob.n_owned],
                "global_batch": 1,
                "seq_len": prob.n_owned,
                "sigma": args.sigma,
                "ic": args.ic,
                "parallelism": f"slab{world}" + (f"-rehearsal-{args.slab_pos}" if args.rehearse_comm and world == 1 else "")
                               + ("-shared-gpu" if args.share_gpu and world > 1 else ""),
                "transport": tr.name,
                "decomposition": ({"edge_shift": edge_shift[0], "rows": [d["rows"] for d in proof["ranks"]],
                                   "balance": balance_report} if world > 1 else None),
                "transport_choice": (dict(choice_report, chosen=kind, requested=args.transport)
                                     if choice_report is not None else None),
                "tb_max": tb,
                "cycles": {str(k): c for k, c in sorted(hist.items())},
                "schedule": "measured" if measured else "balanced",
                "prepare_s": round(prepare_s, 2),
                "warmup_s": round(warm_s.get(kind, 0.0), 2),
                "plan_cache": plan_cache,
                "autotune": tune,
                "arith": arith_name(prob.r, arith) + {"auto": " (auto)", "bench": " (r = 1/4)" if prob.r == 0.25
                                                      else " (auto)"}.get(args.arith, ""),
                "overlap": not args.no_overlap,
                "graph": replayed,
                "launch_plans": plans or None,
                "backend": args.backend,
            },
            "hbm_gb_per_s_plan": round(traffic / elapsed / 1e9, 1),
            "hbm_gb_per_s_measured": (hbm or {}).get("gb_per_s"),
            "hbm_measured": hbm,
            # halo bytes moved by all ranks in the timed region, and per cycle (whole node)
            "halo_bytes": halo_bytes,
            "halo_bytes_per_cycle": round(halo_bytes / max(1, sum(hist.values())), 1),
            "verified": None if verify is None else verify["verified"],
            "verify": verify,
            "timed_field_check": field_check,
            # proof of the decomposition: what the fabric reports per rank
            # (RCCL: ncclCommCount / ncclCommUserRank / ncclCommCuDevice), the
            # devices' PCI bus ids, slab rows and each rank's own timed ms
            "rccl_nranks": proof["fabric_nranks"] if proof["fabric_kind"] == "rccl" else None,
            "fabric": {"kind": proof["fabric_kind"], "nranks": proof["fabric_nranks"]},
            "distinct_devices": proof["distinct_devices"],
            "rank_timed_ms": proof["timed_ms"],
            "per_rank": proof["ranks"],
            "memory_plan": mem_plan,
            "baseline_basis": "BASELINE.md derived ceiling 50 Gpts/s per MI250X GCD x n_gpus",
        }
        if stats:
            out["field_stats"] = stats
        if phases:
            out["phase_ms"] = phases
        os.write(out_fd, (json.dumps(out) + "\n").encode())
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
