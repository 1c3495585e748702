"""Multi-process runs of the native slab solver: P ranks exchanging halos over
torch.distributed (gloo) through the callback transport. The same native
schedule (bands, exchange depth, remainder cycles) that the RCCL transport
drives on MI355X. Result must be bitwise identical to the single-rank golden.

CPU variants run anywhere; GPU variants put every rank on the one visible GPU
(HIP backend: the overlap path with a comm stream and events is exercised,
the exchange is staged through host memory by the callback transport)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import heat2d
from heat2d.models import reference as R

HERE = os.path.dirname(os.path.abspath(__file__))


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_world(tmp_path, world, args, timeout=240):
    port = free_port()
    env = dict(os.environ, OMP_NUM_THREADS="1", HEAT2D_CPU_THREADS="2", MASTER_ADDR="127.0.0.1")
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker.py"), str(r), str(world), str(port),
                               str(tmp_path), json.dumps(args)], env=env, stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT) for r in range(world)]
    outs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=timeout)
            outs.append(out.decode(errors="replace"))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for p, o in zip(procs, outs):
        assert p.returncode == 0, o[-3000:]
    got = np.load(tmp_path / "result.npy")
    with open(tmp_path / "stats.json") as f:
        meta = json.load(f)
    return got, meta


def golden(args, steps=None):
    inp = heat2d.InputDat(n=args["n"], sigma=0.25, nu=0.05, dom_len=args.get("dom", 1.0), ntime=args["steps"])
    prob = heat2d.make_problem(inp, args.get("conv", "ghost"), args.get("ic", "uniform"))
    dt = np.float64 if args.get("dtype", "fp64") == "fp64" else np.float32
    if args.get("random"):
        sys.path.insert(0, HERE)
        from dist_worker import random_field
        return R.owned(R.ftcs(prob, steps, dtype=dt, T0=random_field(prob, args.get("dtype", "fp64"))))
    return R.owned(R.ftcs(prob, steps, dtype=dt))


def check_stats(st, args):
    """Global statistics + one-step residual reduced over the ranks (step_stats)."""
    T = golden(args).astype(np.float64)
    d = T - golden(args, args["steps"] - 1).astype(np.float64)
    assert np.isclose(st["sum"], T.sum(), rtol=1e-12, atol=0)
    assert st["min"] == T.min() and st["max"] == T.max()
    assert np.isclose(st["residual_l2"], np.sqrt((d * d).sum()), rtol=1e-10)
    assert st["residual_max"] == np.abs(d).max()


@pytest.mark.parametrize("world,tb", [(2, 1), (2, 8), (3, 3), (4, 5)])
def test_gloo_cpu_bitwise(native, tmp_path, world, tb):
    args = {"n": 67, "steps": 23, "tb": tb, "backend": "cpu", "random": True}
    got, meta = run_world(tmp_path, world, args)
    assert np.array_equal(got, golden(args))
    assert meta["info"]["size"] == world
    check_stats(meta["stats"], args)


def test_gloo_cpu_inclusive_fp32(native, tmp_path):
    args = {"n": 50, "steps": 17, "tb": 4, "backend": "cpu", "conv": "inclusive", "ic": "hat", "dom": 2.0,
            "dtype": "fp32"}
    got, _ = run_world(tmp_path, 2, args)
    assert np.array_equal(got, golden(args))


@pytest.mark.gpu
@pytest.mark.parametrize("world,tb,overlap,n,order", [(2, 8, True, 301, None), (3, 4, True, 301, None),
                                                      (2, 6, False, 301, None), (4, 8, True, 301, None),
                                                      (4, 8, True, 60, None), (2, 10, True, 1500, None),
                                                      (2, 10, True, 1500, "edge-first"),
                                                      (3, 8, True, 900, "edge-first")])
def test_gloo_hip_ranks_share_gpu(native, gpu, tmp_path, world, tb, overlap, n, order, monkeypatch):
    """Overlapped schedule (interior on the compute stream, bands + exchange on
    the comm stream; or edge-first) on random data, P processes on the one GPU;
    n=60 at 4 ranks makes every slab thinner than its two bands (the
    all-on-comm-stream branch). The last chunk runs with the fused statistics
    (one general launch, then the exchange), reduced over the ranks."""
    if order:
        monkeypatch.setenv("HEAT2D_SPLIT_ORDER", order)  # run_world copies os.environ
    args = {"n": n, "steps": 37, "tb": tb, "backend": "hip", "overlap": overlap, "random": True}
    got, meta = run_world(tmp_path, world, args)
    assert np.array_equal(got, golden(args))
    check_stats(meta["stats"], args)


@pytest.mark.gpu
@pytest.mark.parametrize("world,tb,n,dtype,graph,order", [(3, 10, 1100, "fp64", False, "lead"),
                                                          (4, 8, 1500, "fp32", False, "edge-first"),
                                                          (3, 10, 1100, "fp64", True, "lead"),
                                                          (3, 10, 1100, "fp64", True, "edge-first"),
                                                          (2, 6, 900, "fp64", True, None)])
def test_ipc_ranks_share_gpu_bitwise(native, gpu, tmp_path, monkeypatch, world, tb, n, dtype, graph, order):
    """Rank PROCESSES on the one GPU exchanging halos through the IPC transport
    (neighbours' fields mapped via hipIpc handles, pulls ordered by stream-side
    counters), optionally replayed from hipGraphs (the IPC exchange captures),
    per split order (lead: every cycle's band launch issued before the
    interior, no wait between them; edge-first; the autotuner's).
    Random data, bitwise the single-rank golden, global statistics reduced."""
    if order:
        monkeypatch.setenv("HEAT2D_SPLIT_ORDER", order)
    args = {"n": n, "steps": 37, "tb": tb, "backend": "hip", "overlap": True, "random": True, "dtype": dtype,
            "transport": "ipc", "graph": graph}
    got, meta = run_world(tmp_path, world, args)
    ref = golden(args)
    assert np.array_equal(got, ref), np.abs(got.astype(np.float64) - ref).max()
    assert meta["info"]["transport"] == "ipc"


@pytest.mark.gpu
def test_ipc_dead_rank_survivor_fails_fast(native, gpu, tmp_path):
    """IPC transport, two rank processes on the one GPU: rank 1 dies
    (os._exit) after its first chunk while rank 0 keeps exchanging. Rank 0's
    arrive kernel must not spin past the comm timeout: its watchdog (or the
    kernel's own wall-clock limit) raises the shared abort word, the wait
    returns, and the process exits non-zero within seconds."""
    import time
    port = free_port()
    args = {"n": 1100, "steps": 40, "tb": 8, "backend": "hip", "transport": "ipc", "die_rank": 1, "die_after": 8}
    env = dict(os.environ, OMP_NUM_THREADS="1", HEAT2D_COMM_TIMEOUT="5", MASTER_ADDR="127.0.0.1")
    t0 = time.time()
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker.py"), str(r), "2", str(port),
                               str(tmp_path), json.dumps(args)], env=env, stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT) for r in range(2)]
    try:
        outs = [p.communicate(timeout=150)[0].decode(errors="replace") for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    elapsed = time.time() - t0
    assert procs[1].returncode == 3, outs[1][-2000:]  # the injected death
    assert procs[0].returncode != 0, outs[0][-2000:]  # the survivor fails instead of hanging
    # (the IPC watchdog's abort normally; a gloo collective may notice the dead peer first)
    assert any(w in outs[0] for w in ("abort", "timed out", "no halo exchange", "onnection", "peer")), outs[0][-2000:]
    assert elapsed < 120, elapsed
