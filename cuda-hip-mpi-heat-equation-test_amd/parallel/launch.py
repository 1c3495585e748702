"""Python driver: `python -m heat2d [input.dat] [flags]`, torchrun-aware.

Behaves like the reference programs (reads ./input.dat, prints
"MPI rank r using GPU d", "Automatic MPI decomposition: P x 1", "nx:", "ny:",
optional per-step "time_it:", "simulation completed!!!!", and "Average time:"
or "total time:"; writes int.dat / soln.dat / soln%05d.dat per variant) on the
native engine. One process per GPU:

    python -m heat2d input.dat                                   # 1 GPU (or CPU)
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m heat2d input.dat   # 8 GPUs, RCCL
    torchrun --nproc-per-node 4 -m heat2d input.dat --backend cpu              # 4 CPU ranks, gloo

    torchrun --nproc-per-node 2 -m heat2d input.dat --transport peer --share-gpu  # 2 ranks, 1 GPU, hipIpc

GPU ranks exchange halos over RCCL (--transport auto, the default: RCCL when
its communicator builds on every rank, else the peer transport — hipIpc
mappings of the neighbours' fields — on every rank alike; parallel/select.py).

Extras: --tb K, --dtype, --check-every N (global sum / residual, NaN abort),
--checkpoint DIR --checkpoint-every N, --restart DIR, --json FILE, --output npy.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np


def build_parser():
    ap = argparse.ArgumentParser(prog="python -m heat2d", description=__doc__.split("\n")[0])
    ap.add_argument("input", nargs="?", default="input.dat")
    ap.add_argument("--variant", default=None, help="mpi | mpicuda | serial | cuda | managed | python | pycuda")
    ap.add_argument("--backend", default="auto", choices=["auto", "hip", "cpu"])
    ap.add_argument("--dtype", default="fp64", choices=["fp64", "fp32"])
    ap.add_argument("--ic", default=None)
    ap.add_argument("--tb", type=int, default=0, help="time steps per HBM pass (0: measured best per dtype)")
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--copy-swap", action="store_true")
    ap.add_argument("--managed", action="store_true")
    ap.add_argument("--graph", action="store_true")
    ap.add_argument("--engine", default=None, choices=["tb", "jit"],
                    help="tb: temporal-blocked kernels; jit: hipRTC kernel rendered at run time "
                         "(default: jit for --variant pycuda on a GPU, else tb)")
    ap.add_argument("--arith", default="auto", choices=["auto", "exact", "fma", "jacobi", "fast"],
                    help="exact: reference rounding (bitwise == NumPy golden); fma: contracted update, one op fewer; "
                         "jacobi: r == 1/4 only, r * (S + E + N + W), 3 adds per point")
    ap.add_argument("--edge-shift", default="0",
                    help="rows each edge slab gives to the middle slabs (>= 3 ranks; checkpoints record it): a "
                         "number, auto (GPU ranks: measured before the run — every rank times its own slab on a "
                         "1-rank loop exchange, uniform and shifted, parallel/select.balance_edges, as bench.py "
                         "does) or measure (the same on any backend)")
    ap.add_argument("--n", type=int, default=None)
    ap.add_argument("--ntime", type=int, default=None)
    ap.add_argument("--print-every", type=int, default=0)
    ap.add_argument("--check-every", type=int, default=0)
    ap.add_argument("--output", default="ascii", choices=["ascii", "npy", "none"])
    ap.add_argument("--json", default=None)
    ap.add_argument("--checkpoint", default=None)
    ap.add_argument("--checkpoint-every", type=int, default=0)
    ap.add_argument("--restart", default=None)
    ap.add_argument("--quiet", action="store_true")
    ap.add_argument("--transport", default="auto", choices=["auto", "rccl", "peer", "host"],
                    help="halo exchange between GPU rank processes: rccl (RCCL send/recv), peer (hipIpc "
                         "mappings of the neighbours' fields, stream-ordered by host-shared counters), or auto "
                         "(default): rccl if its communicator and solver build on every rank, else peer on every "
                         "rank, else host; host: halos staged through pinned host memory over torch.distributed "
                         "(gloo); host collectives over gloo")
    ap.add_argument("--share-gpu", action="store_true",
                    help="every rank on GPU 0 (--transport peer or auto): the multi-process path on one GPU")
    return ap


def _dist_setup(backend: str, share_gpu: bool = False):
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if share_gpu else int(os.environ.get("LOCAL_RANK", "0"))
    if backend == "hip":
        torch.cuda.set_device(local)
    if world > 1 and not dist.is_initialized():
        from datetime import timedelta
        to = timedelta(seconds=float(os.environ.get("HEAT2D_COMM_TIMEOUT", "600")))  # dead peer -> error, not hang
        # host collectives over gloo whatever the halo fabric (the RCCL unique
        # id, barriers, the timing MAX, the transport choice)
        dist.init_process_group("gloo", timeout=to)
    return rank, world, local


def _make_solver(kinds, make_transport, make_solver, world):
    """The first transport kind whose transport AND solver build on every rank
    (parallel/select.try_collective: a failure on any rank skips the kind on
    every rank — e.g. RCCL refusing ranks that share a GPU, or a node whose RCCL
    cannot initialise). Returns (transport, solver, kind, {kind: error})."""
    from heat2d.parallel import select

    def amin(v):
        if world == 1:
            return float(v)
        import torch
        import torch.distributed as dist
        t = torch.tensor([float(v)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return float(t.item())

    errors = {}
    for kind in kinds:
        tr, why = select.try_collective(lambda: make_transport(kind), amin,
                                        cleanup=lambda t: (t.abort("another rank failed to initialise"), t.close()))
        if why is None:
            s, why = select.try_collective(lambda: make_solver(tr), amin, cleanup=lambda x: x.close())
            if why is None:
                return tr, s, kind, errors
            tr.close()
        errors[kind] = why
    raise SystemExit(f"heat2d: no halo transport works on every rank: {errors}")


def _measure_edge_shift(prob, a, rank, world, local, backend, first_kind, engine, arith, steps, verbose) -> int:
    """--edge-shift auto / measure: every rank times its own slab alone — a
    1-rank loop exchange of the run's kind (RCCL's, IPC's where the run would
    fall back or ranks share a GPU, none on CPU ranks), one rank after another
    with --share-gpu — and parallel/select.balance_edges keeps the shift only
    if the slowest slab gets faster (bench.py runs the same measurement)."""
    import torch
    import torch.distributed as dist
    from heat2d.models.heat2d import HeatSolver
    from heat2d.ops import _native as N
    from heat2d.parallel import select
    from heat2d.parallel import transport as T
    hip = backend == "hip"
    loop = (T.RcclLoopTransport if first_kind == "rccl" and not a.share_gpu else T.IpcLoopTransport) if hip \
        else T.SelfTransport
    sync = torch.cuda.synchronize if hip else (lambda: None)

    def measure(shift):
        r0, nr = N.decompose(prob.n_owned, world, rank, shift)

        def make():
            tr = loop(local) if hip else loop()
            try:
                s = HeatSolver(prob, dtype=a.dtype, backend=backend, tb=a.tb, overlap=not a.no_overlap,
                               transport=tr, device=local if hip else None, rows=nr, slab_row0=r0, engine=engine,
                               arith=arith)
            except Exception:
                tr.close()
                raise
            return s, lambda: (s.close(), tr.close())

        if not a.share_gpu:
            return select.time_own_slab(make, steps, 0, sync=sync)
        v = float("nan")
        for r in range(world):  # ranks sharing one GPU take turns
            if r == rank:
                try:
                    v = select.time_own_slab(make, steps, 0, sync=sync)
                except Exception:  # noqa: BLE001 - a NaN makes every rank keep 0
                    import traceback
                    traceback.print_exc()
            dist.barrier()
        return v

    def gather(v):
        t = torch.zeros(world, dtype=torch.float64)
        t[rank] = v
        dist.all_reduce(t)
        return t.tolist()

    shift, rep = select.balance_edges(measure, gather,
                                      lambda d: [N.decompose(prob.n_owned, world, r, d)[1] for r in range(world)],
                                      cap=(prob.n_owned // world) // 4)
    if verbose:
        print(f" edge balance: shift {shift} rows (estimate {rep.get('estimate')}, slowest slab "
              f"{max(rep['uniform_ms']):.4f} ms uniform"
              + (f", {max(rep['shifted_ms']):.4f} ms shifted" if rep.get("shifted_ms") else "") + ")", flush=True)
    return shift


def run(argv=None) -> int:
    a = build_parser().parse_args(argv)
    import heat2d
    from heat2d.models import presets
    from heat2d.models.heat2d import HeatSolver, resolve_backend
    from heat2d.parallel import transport as T
    from heat2d.utils import checkpoint, io, metrics
    from heat2d.utils.config import make_problem, read_input

    backend = resolve_backend(a.backend)
    if a.share_gpu and a.transport == "rccl":
        raise SystemExit("--share-gpu needs --transport peer or auto (RCCL refuses two ranks on one GPU)")
    rank, world, local = _dist_setup(backend, a.share_gpu)
    root = rank == 0
    inp = read_input(a.input)
    if a.n:
        inp.n = a.n
    if a.ntime is not None:
        inp.ntime = a.ntime
    var = presets.get(a.variant or presets.default_variant(inp))
    prob = make_problem(inp, var.convention, a.ic or var.ic)
    nsteps = inp.ntime + (1 if var.extra_step else 0)
    if prob.r > 0.25 + 1e-12 and root:
        print(f"warning: r = {prob.r:.6g} > 0.25: FTCS is unstable in 2-D", file=sys.stderr)

    if backend == "hip" and not a.quiet:
        print(f" MPI rank {rank:12d} using GPU {local:12d}", flush=True)
    if var.name == "pycuda" and backend == "hip" and root and not a.quiet:
        # the reference's PyCUDA program queries the device limits and prints
        # MAX_THREADS_PER_BLOCK (python/cuda/cuda.py:16-27)
        from heat2d.ops import _native as N
        lim = N.device_limits(local)
        print(lim["MAX_THREADS_PER_BLOCK"])
        print(" device limits: " + " ".join(f"{k}={v}" for k, v in lim.items()), flush=True)
    engine = a.engine or ("jit" if var.name == "pycuda" and backend == "hip" else "tb")
    arith = a.arith
    if arith == "auto" and prob.r == 0.25 and prob.ic.sterbenz_safe() and not a.restart and engine == "tb":
        arith = "jacobi"  # bitwise the reference rounding on this IC (the CLI's auto does the same)

    def make_transport(kind):
        return {"torch-dist": T.TorchDistTransport, "self": T.SelfTransport,
                "rccl": lambda: T.RcclTransport(rank, world, local), "peer": lambda: T.IpcTransport(local)}[kind]()

    if world == 1:
        kinds = ["self"]
    elif backend != "hip":
        kinds = ["torch-dist"]
    else:
        # auto ends with the host-staged exchange (pinned staging + gloo): the
        # run still completes where neither RCCL nor the IPC mappings attach
        kinds = {"auto": ["rccl", "peer", "torch-dist"], "rccl": ["rccl"], "peer": ["peer"],
                 "host": ["torch-dist"]}[a.transport]

    edge_shift = 0
    if a.edge_shift not in ("auto", "measure"):
        edge_shift = int(a.edge_shift)
    elif world >= 3 and (backend == "hip" or a.edge_shift == "measure") and engine == "tb":
        edge_shift = _measure_edge_shift(prob, a, rank, world, local, backend, kinds[0], engine, arith,
                                         min(nsteps, 48), root and not a.quiet)

    def make_solver(tr):
        return HeatSolver(prob, dtype=a.dtype, backend=backend, tb=a.tb, overlap=not a.no_overlap,
                          copy_swap=a.copy_swap, managed=a.managed or var.managed, graph=a.graph, transport=tr,
                          device=local if backend == "hip" else None, engine=engine, arith=arith,
                          edge_shift=edge_shift)

    tr, s, kind, fallback = _make_solver(kinds, make_transport, make_solver, world)
    if fallback and root and not a.quiet:
        print(f"heat2d: halo transport {kind} ({'; '.join(f'{k} failed: {v}' for k, v in fallback.items())})",
              file=sys.stderr, flush=True)
    if root and not a.quiet:
        if world > 1 or var.outputs == "mpi":
            print(f" Automatic MPI decomposition: {world:12d}  x 1")
        print(f" nx: {s.nrows:12d}")
        print(f" ny: {s.ncols:12d}", flush=True)

    start_step = 0
    if a.restart:
        meta = checkpoint.load(s, a.restart)
        start_step = int(meta["step"])
        if root and not a.quiet:
            print(f" restarted from {a.restart} at step {start_step}")

    x = prob.x
    if var.outputs == "serial" and a.output == "ascii" and start_step == 0:
        _write_inclusive(s, prob, "int.dat", world)

    # time_it lines (fortran/hip/heat.F90:241: one per step) do not cut the run
    # into cycles shorter than the preferred depth: chunks of
    # max(print_every, pref_depth) steps, every due line printed after its chunk
    print_chunk = max(a.print_every, s.pref_depth) if a.print_every > 0 else 0
    # plan / autotune outside the timed region: every chunk length the loop below runs
    rules = [v for v in (print_chunk, a.check_every, a.checkpoint_every) if v > 0]
    d, seen = start_step, set()
    while d < nsteps:
        c = nsteps - d
        for v in rules:
            c = min(c, v - d % v)
        if c not in seen:
            seen.add(c)
            s.prepare(c)
        d += c
    s.cycle_hist(reset=True)  # count the timed loop's cycles only
    _barrier(world)
    s.synchronize()
    t0 = time.perf_counter()
    done = start_step
    while done < nsteps:
        chunk = nsteps - done
        for v in rules:
            chunk = min(chunk, v - done % v)
        check = a.check_every > 0 and (done + chunk) % a.check_every == 0
        st = s.step_stats(chunk) if check else s.step(chunk)  # stats + one-step residual fused into the last cycle
        before, done = done, done + chunk
        if root and a.print_every:
            for t in range((before // a.print_every + 1) * a.print_every, done + 1, a.print_every):
                print(f" time_it: {t:12d}")
        if check:
            if root:
                print(f" step {done}: sum={st['sum']:.17g} min={st['min']:.6g} max={st['max']:.6g} "
                      f"residual_l2={st['residual_l2']:.6e} residual_max={st['residual_max']:.6e}", flush=True)
            if not np.isfinite(st["sum"]):
                raise FloatingPointError(f"non-finite temperature at step {done}")
        if a.checkpoint and a.checkpoint_every and done % a.checkpoint_every == 0 and done < nsteps:
            checkpoint.save(s, a.checkpoint, step=done)
    s.synchronize()
    _barrier(world)
    elapsed = time.perf_counter() - t0
    elapsed = _max_over_ranks(elapsed, world, "cpu")
    ran = nsteps - start_step
    cycles = s.cycle_hist()

    if a.checkpoint:
        checkpoint.save(s, a.checkpoint, step=done)
    if a.output != "none":
        if var.outputs == "serial":
            if a.output == "ascii":
                _write_inclusive(s, prob, "soln.dat", world)
            else:
                full = s.gather()
                if root:
                    io.write_npy("soln.npy", full)
        elif inp.soln == 1 or a.output == "npy":
            local_T = s.download()
            if a.output == "npy":
                io.write_npy(f"soln{rank:05d}.npy", local_T)
            else:
                io.write_xyz(f"soln{rank:05d}.dat", local_T, x[1 + s.row0:1 + s.row0 + s.nrows], x[1:-1])
    st = s.stats()
    if root:
        if var.sum_line:  # fortran/mpi+cuda/heat.F90:275 (there an uninitialised gsum; here the all-reduced sum)
            print(f" Sum of Temperature: {st['sum']:24.16g}")
        print(" simulation completed!!!!")
        per = elapsed / max(ran, 1) if var.per_step else elapsed
        print(f" {var.timing_line} {per:24.16g}")
        rec = metrics.record(prob.n_owned, ran, elapsed, world, a.dtype, s.tb, backend, a.copy_swap,
                             {"variant": var.name, "arith": arith, "sum": st["sum"], "min": st["min"], "max": st["max"],
                              "transport": kind, "transport_fallback": fallback or None},
                             cycles=cycles)
        if not a.quiet:
            print(f" heat2d: n={prob.n_owned} P={world} {a.dtype} K<={s.tb} passes={sum(cycles.values())} "
                  f"steps={ran} wall={elapsed:.6f} s  "
                  f"{rec['gpts_per_s']:.3f} Gpts/s  {rec['model_hbm_gb_per_s']:.1f} GB/s(model)  "
                  f"sum(T)={st['sum']:.17g}", flush=True)
        if a.json:
            metrics.write_json(a.json, rec)
    s.close()
    tr.close()
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    return 0


def _write_inclusive(s, prob, path, world):
    """Frame-inclusive n x n dump (fortran/serial/heat.f90:50-55): rank 0 gathers."""
    from heat2d.utils import io
    full = s.gather()
    if s.rank != 0:
        return
    m = prob.n_owned
    T = np.empty((m + 2, m + 2), dtype=full.dtype)
    T[1:-1, 1:-1] = full
    # frame values: the IC on the frame (kept fixed by the solver)
    from heat2d.models.reference import initial_field
    frame = initial_field(prob, full.dtype)
    T[0, :], T[-1, :], T[:, 0], T[:, -1] = frame[0, :], frame[-1, :], frame[:, 0], frame[:, -1]
    io.write_xyz(path, T, prob.x, prob.x)


def _barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def _max_over_ranks(v, world, backend):
    if world == 1:
        return v
    import torch
    import torch.distributed as dist
    dev = "cuda" if backend == "hip" else "cpu"
    t = torch.tensor([v], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


if __name__ == "__main__":
    sys.exit(run())
