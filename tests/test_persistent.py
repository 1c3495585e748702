"""Persistent multi-cycle launches (VERDICT r2 task 4): many cycles of one
depth in ONE cooperative dispatch, one co-resident wave per work item, items
synchronised by per-item completion counters (an item of cycle c waits only
for the items whose cycle-(c-1) output it reads, which are also the only
readers of the rows it overwrites) instead of kernel boundaries. Bitwise the
NumPy golden on non-dyadic data, for band and segment items, items shorter
than the temporal depth (dependencies spanning several items), both dtypes,
both buffer parities, and repeated launches (epoch counters)."""
import numpy as np
import pytest

import heat2d
from heat2d.models import reference as R
from heat2d.models.heat2d import HeatSolver

pytestmark = pytest.mark.gpu


def prob(n, steps, ic="sine"):
    return heat2d.make_problem(heat2d.InputDat(n=n, sigma=0.25, nu=0.05, dom_len=1.0, ntime=steps), "ghost", ic)


def run(p, dtype, tb, env, monkeypatch, calls=1, autotune=0):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    npdt = np.float64 if dtype == "fp64" else np.float32
    s = HeatSolver(p, dtype=dtype, backend="hip", tb=tb, device=0, autotune=autotune)
    s.upload(R.owned(R.initial_field(p, npdt)))
    per = p.ntime // calls
    assert per * calls == p.ntime
    s.prepare(per)
    assert s.persistent(per)
    for _ in range(calls):
        s.step(per)
    got = s.download()
    s.close()
    return got, R.owned(R.ftcs(p, dtype=npdt))


@pytest.mark.parametrize("dtype,tb,n,steps", [("fp64", 8, 301, 37), ("fp32", 16, 515, 45), ("fp64", 13, 1100, 40),
                                              ("fp32", 5, 777, 31), ("fp64", 1, 203, 9)])
def test_persistent_bitwise(gpu, native, monkeypatch, dtype, tb, n, steps):
    got, ref = run(prob(n, steps), dtype, tb, {"HEAT2D_PERSIST": "1"}, monkeypatch)
    assert np.array_equal(got, ref), np.abs(got.astype(np.float64) - ref).max()


@pytest.mark.parametrize("items_env", [{"HEAT2D_SEGMENTS": "997"}, {"HEAT2D_SEGMENTS": "61"},
                                       {"HEAT2D_BANDS": "40"}, {"HEAT2D_BANDS": "3"}])
def test_persistent_item_shapes(gpu, native, monkeypatch, items_env):
    """Segment items (crossing strip ends) and band items, including items of
    fewer rows than the depth (600 rows / 40 bands = 15 < 16 ... and segments
    of ~2 rows): a cycle's dependencies then span several items per strip."""
    env = {"HEAT2D_PERSIST": "1", "HEAT2D_SPLIT_ORDER": "single", **items_env}
    got, ref = run(prob(600, 48), "fp32", 16, env, monkeypatch)
    assert np.array_equal(got, ref), np.abs(got.astype(np.float64) - ref).max()


def test_persistent_repeated_calls(gpu, native, monkeypatch):
    """Several step(n) calls: epoch-based counters carry across launches, and an
    odd cycle count per call alternates the starting buffer."""
    got, ref = run(prob(450, 3 * 21), "fp64", 7, {"HEAT2D_PERSIST": "1"}, monkeypatch, calls=3)
    assert np.array_equal(got, ref)


def test_persistent_auto_choice_small_grid(gpu, native, monkeypatch):
    """Auto mode on the 4096^2 fp32 small grid (BASELINE config 2): prepare()
    times persistent launches against the schedule's graph replay and keeps the
    faster; whichever it keeps, the result is bitwise."""
    monkeypatch.delenv("HEAT2D_PERSIST", raising=False)
    p = prob(4096, 64, "uniform")
    s = HeatSolver(p, dtype="fp32", backend="hip", device=0, graph=True)
    s.prepare(64)
    s.step(64)
    got = s.download()
    s.close()
    assert np.array_equal(got, R.owned(R.ftcs(p, dtype=np.float32)))
