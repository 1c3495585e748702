"""RCCL transport on the GPU box (one GPU => a single-rank communicator; the
multi-rank schedule itself is covered by test_distributed.py): the unique id
is broadcast over a torch.distributed NCCL(=RCCL) group, the native engine
creates its own communicator with it, steps, and all-reduces statistics."""
import os
import socket

import numpy as np
import pytest

import heat2d
from heat2d.models import reference as R

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_rccl_single_rank(native, gpu):
    import torch
    import torch.distributed as dist
    from heat2d.models.heat2d import HeatSolver
    from heat2d.parallel.transport import RcclTransport

    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        tr = RcclTransport(0, 1, 0)
        assert tr.name == "rccl"
        p = heat2d.make_problem(heat2d.InputDat(n=257, sigma=0.25, nu=0.05, dom_len=1.0, ntime=30), "ghost",
                                "uniform")
        s = HeatSolver(p, dtype="fp64", backend="hip", tb=8, transport=tr, device=0)
        s.step(p.ntime)
        got = s.download()
        assert np.array_equal(got, R.owned(R.ftcs(p)))
        st = s.stats()  # RCCL all-reduce path
        assert np.isclose(st["sum"], got.sum(), rtol=1e-12)
        s.close()
        tr.close()
    finally:
        dist.destroy_process_group()


def periodic_golden(p, steps, k, dtype=np.float64):
    """The rehearsal's physics: at the start of every cycle of depth k the two
    x-frame rows receive the periodic neighbours (row n-1 below row 0, row 0
    above row n-1: the self send/recv of the loop transport), and stay fixed
    (frame rows are pinned) through the cycle's k FTCS steps."""
    T = R.initial_field(p, dtype)
    m = p.n_owned
    assert steps % k == 0
    for _ in range(steps // k):
        T[0, :] = T[m, :]
        T[m + 1, :] = T[1, :]
        for _ in range(k):
            T = R.ftcs_step(T, p.r)
    return R.owned(T)


@pytest.mark.parametrize("order,graph", [("auto", False), ("edge-first", False), ("edge-first", True),
                                         ("concurrent", True), ("concurrent", False), ("lead", False),
                                         ("lead", True)])
def test_rccl_loop_rehearsal(native, gpu, order, graph, monkeypatch):
    """The 1-GPU rehearsal of the multi-GPU schedule: bands + RCCL self
    send/recv on the comm stream beside the interior. Checked bitwise on ALL
    rows against the periodic-in-x golden the self exchange implements."""
    from heat2d.models.heat2d import HeatSolver
    from heat2d.parallel.transport import RcclLoopTransport

    if order != "auto":
        monkeypatch.setenv("HEAT2D_SPLIT_ORDER", order)
    tr = RcclLoopTransport(0)
    assert tr.name == "rccl-loop"
    K = 8
    p = heat2d.make_problem(heat2d.InputDat(n=400, sigma=0.25, nu=0.05, dom_len=1.0, ntime=5 * K), "ghost", "sine")
    s = HeatSolver(p, dtype="fp64", backend="hip", tb=K, transport=tr, device=0, graph=graph, autotune=1)
    s.upload(R.owned(R.initial_field(p)))  # includes the first (periodic) exchange
    s.step(p.ntime)
    got = s.download()
    assert s.cycle_hist() == {K: 5}
    if order != "auto":
        assert s.plan(K)["order"] == order
    ref = periodic_golden(p, p.ntime, K)
    assert np.array_equal(got, ref), np.argwhere(got != ref)[:5]
    assert not np.array_equal(got[:5], R.owned(R.ftcs(p))[:5])  # the periodic exchange really moved rows
    s.close()
    tr.close()


def periodic_slab_golden(T, r, steps):
    """A middle slab exchanging with itself (bench.py --rehearse-comm): the
    halo rows above receive its last rows and the rows below its first ones,
    so its rows evolve periodically (period = its row count); the column
    frame stays pinned. T: the slab's rows with both frame columns."""
    for _ in range(steps):
        pad = np.vstack([T[-1:], T, T[:1]])
        T = R.ftcs_step(pad, r)[1:-1]
    return T


@pytest.mark.parametrize("kind", ["rccl", "ipc"])
@pytest.mark.parametrize("order", ["edge-first", "lead", "concurrent", "auto", "edge-first-only"])
def test_middle_slab_rehearsal(native, gpu, monkeypatch, kind, order):
    """The bench's strong-scaling rehearsal geometry: a middle slab (rows
    [200, 360) of a 600^2 grid, interior boundary bands) exchanging both
    bands with itself, per split order (lead: the band launch issued before
    the interior, no wait between them; every order's first cycle runs
    lead-ordered unless HEAT2D_LEAD_FIRST=0), bitwise the periodic-slab golden
    on rough data."""
    from heat2d.models.heat2d import HeatSolver
    from heat2d.parallel.transport import IpcLoopTransport, RcclLoopTransport

    if order == "edge-first-only":  # no lead-ordered first cycle either
        monkeypatch.setenv("HEAT2D_LEAD_FIRST", "0")
        order = "edge-first"
    if order != "auto":
        monkeypatch.setenv("HEAT2D_SPLIT_ORDER", order)
    K, rows, row0 = 8, 160, 200
    p = heat2d.make_problem(heat2d.InputDat(n=600, sigma=0.25, nu=0.05, dom_len=1.0, ntime=5 * K), "ghost", "sine")
    full = R.initial_field(p)
    full[1:-1, 1:-1] = 1.0 + np.random.default_rng(5).random((600, 600))
    slab = full[1 + row0:1 + row0 + rows].copy()
    tr = RcclLoopTransport(0) if kind == "rccl" else IpcLoopTransport(0)
    s = HeatSolver(p, dtype="fp64", backend="hip", tb=K, transport=tr, device=0, rows=rows, slab_row0=row0,
                   graph=kind == "ipc", autotune=1, arith="exact")
    s.upload(slab[:, 1:-1])
    s.step(p.ntime)
    got = s.download()
    assert s.cycle_hist() == {K: 5}
    if order != "auto":
        assert s.plan(K)["order"] == order
    s.close()
    tr.close()
    ref = periodic_slab_golden(slab, p.r, p.ntime)[:, 1:-1]
    assert np.array_equal(got, ref), np.argwhere(got != ref)[:5]
