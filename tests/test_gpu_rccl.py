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


@pytest.mark.parametrize("order,graph", [("auto", False), ("edge-first", False), ("edge-first", True),
                                         ("concurrent", True)])
def test_rccl_loop_rehearsal(native, gpu, order, graph, monkeypatch):
    """The 1-GPU rehearsal of the multi-GPU schedule: bands + RCCL self
    send/recv on the comm stream beside the CU-masked interior. The physics is
    periodic-ish (the frame rows are overwritten), so check what must hold:
    it runs to completion, rows far from the x boundaries match the Dirichlet
    golden exactly (information travels one row per step), and all is finite."""
    from heat2d.models.heat2d import HeatSolver
    from heat2d.parallel.transport import RcclLoopTransport

    if order != "auto":
        monkeypatch.setenv("HEAT2D_SPLIT_ORDER", order)
    tr = RcclLoopTransport(0)
    assert tr.name == "rccl-loop"
    p = heat2d.make_problem(heat2d.InputDat(n=400, sigma=0.25, nu=0.05, dom_len=1.0, ntime=40), "ghost", "sine")
    s = HeatSolver(p, dtype="fp64", backend="hip", tb=8, transport=tr, device=0, graph=graph)
    s.upload(R.owned(R.initial_field(p)))
    s.step(p.ntime)
    got = s.download()
    ref = R.owned(R.ftcs(p))
    assert np.isfinite(got).all()
    assert np.array_equal(got[60:-60], ref[60:-60])
    assert not np.array_equal(got[:5], ref[:5])  # the periodic exchange really moved rows
    s.close()
    tr.close()
