"""Memory-fit planner (utils/memplan.py, csrc/runtime/solver.cpp plan_max_grid /
solver_footprint): the footprint formula is the Solver constructor's own
allocation (fields from its layout; on the GPU, hipMemGetInfo), and the
planned grid is the largest whose largest slab fits the budget."""
import json
import os
import subprocess
import sys

import pytest

import heat2d
from heat2d.ops import _native as N
from heat2d.utils import memplan

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("n,P,dtype", [(100, 1, "fp64"), (1001, 3, "fp32"), (4097, 8, "fp64"), (257, 2, "fp32")])
def test_footprint_is_the_solver_layout(n, P, dtype):
    """field_bytes == 2 fields x the solver's own layout (uneven slabs: every rank)."""
    es = 8 if dtype == "fp64" else 4
    for rank in range(P):
        r0, nr = N.decompose(n, P, rank)
        L = N.make_layout(nr, n, heat2d_max_halo(), r0, n)
        fp = memplan.footprint(n, P, dtype, rank=rank, backend="cpu")
        assert fp["field_bytes"] == 2 * (L.nrows + 2 * L.halo) * L.pitch * es
        assert fp["work_bytes"] == 0 and fp["total_bytes"] == fp["field_bytes"]
        gpu = memplan.footprint(n, P, dtype, rank=rank, backend="hip")
        assert gpu["field_bytes"] == fp["field_bytes"] and 0 < gpu["work_bytes"] < (1 << 20)


def heat2d_max_halo():
    return N.max_tb()


@pytest.mark.parametrize("dtype,P", [("fp32", 1), ("fp64", 1), ("fp32", 8), ("fp64", 3)])
def test_plan_max_grid_is_the_largest_fitting(dtype, P):
    """n fits, n + 1 does not (rank 0's slab is the largest), at MI355X scale."""
    budget = 280 * 10**9
    plan = memplan.plan_max_grid(dtype, P, free_bytes=budget, reserve=0)
    n = plan["n"]
    assert memplan.footprint(n, P, dtype)["total_bytes"] <= budget
    assert memplan.footprint(n + 1, P, dtype)["total_bytes"] > budget
    assert plan["fraction_of_free"] > 0.99
    # fp32 one GPU: two fields of n^2 points ~ 280 GB -> n ~ 187k (~184k^2 per GPU)
    if dtype == "fp32" and P == 1:
        assert 185000 < n < 188000
    # P ranks hold P times the points of one (the ghost bands cost a little)
    if P > 1:
        one = memplan.plan_max_grid(dtype, 1, free_bytes=budget, reserve=0)["n"]
        assert one * P ** 0.5 * 0.99 < n <= one * P ** 0.5


def test_reserve_default():
    free = 287 * 10**9
    plan = memplan.plan_max_grid("fp32", 1, free_bytes=free)
    assert plan["reserve_bytes"] == memplan.reserve_bytes(free)
    assert 0.95 < plan["fraction_of_free"] < 0.99


def test_bench_grid_max_cpu():
    """bench.py --grid max (CPU rehearsal: a 64 MiB budget): the planned grid
    is the one run, reported with its plan; weak mode plans over the ranks."""
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--backend", "cpu", "--grid", "max",
                        "--dtype", "fp32", "--steps", "4", "--warmup", "1", "--tb", "4", "--verify", "off",
                        "--weak", "--gpus", "2"], capture_output=True, text=True, timeout=600, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    d = json.loads(p.stdout.strip().splitlines()[-1])
    mp = d["memory_plan"]
    assert mp["n"] == d["config"]["grid"][1] and mp["nranks"] == 2
    assert memplan.footprint(mp["n"], 2, "fp32")["total_bytes"] <= 64 << 20
    assert memplan.footprint(mp["n"] + 1, 2, "fp32")["total_bytes"] > 64 << 20
    assert d["timed_field_check"]["ok"] is True


def test_cli_n_max_needs_gpu(tmp_path):
    (tmp_path / "input.dat").write_text("64 0.25 0.05 1.0 5 0\n")
    p = subprocess.run([N.CLI_PATH, "--cpu", "--n", "max"], cwd=tmp_path, capture_output=True, text=True, timeout=60)
    assert p.returncode != 0 and "--n max plans device memory" in p.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("n,dtype", [(20000, "fp64"), (30001, "fp32")])
def test_footprint_matches_device_allocation(n, dtype):
    """What a solver allocates on the device (hipMemGetInfo before / after
    building it) is the footprint: the difference between a big and a small
    solver equals the difference of their footprints up to the allocator's
    page rounding (one-time runtime costs — streams, code objects — cancel), and
    the fixed part is far below the planner's reserve."""
    import torch
    from heat2d.models.heat2d import HeatSolver
    torch.cuda.set_device(0)

    def used(m):
        inp = heat2d.InputDat(n=m, sigma=0.25, nu=0.05, dom_len=1.0, ntime=1, soln=0, nfields=6)
        prob = heat2d.make_problem(inp, "ghost", "uniform")
        torch.cuda.synchronize()
        f0 = memplan.mem_info(0)[0]
        s = HeatSolver(prob, dtype=dtype, backend="hip", device=0, init=False, autotune=0)
        f1 = memplan.mem_info(0)[0]
        s.close()
        return f0 - f1

    used(2048)  # one-time runtime allocations of the first solver in the process
    small, big = used(2048), used(n)
    fs, fb = memplan.footprint(2048, 1, dtype)["total_bytes"], memplan.footprint(n, 1, dtype)["total_bytes"]
    assert big >= fb, (big, fb)
    assert abs((big - small) - (fb - fs)) <= (16 << 20), (big, small, fb, fs)
    assert big - fb < memplan.RESERVE_FIXED // 4, (big, fb)


@pytest.mark.gpu
def test_plan_max_grid_on_device():
    """On the box's GPU the planned fp32 grid uses >= 95 % of the free memory."""
    import torch
    torch.cuda.set_device(0)
    plan = memplan.plan_max_grid("fp32", 1, device=0)
    assert plan["fraction_of_free"] >= 0.95 and plan["n"] > 150000, plan
