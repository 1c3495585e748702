"""CPU path of the native engine (same runtime schedule, CPU twin kernels)
against the NumPy golden model — bitwise — plus analytic and reference-demo
oracles. Runs without a GPU."""
import numpy as np
import pytest

import heat2d
from heat2d.models import reference as R
from heat2d.models.heat2d import HeatSolver, LoopbackGroup
from heat2d.ops import _native as N


def prob(n, steps, conv="ghost", ic="uniform", dom=1.0, sigma=0.25):
    return heat2d.make_problem(heat2d.InputDat(n=n, sigma=sigma, nu=0.05, dom_len=dom, ntime=steps), conv, ic)


@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
@pytest.mark.parametrize("tb", [1, 2, 3, 7, 8, 16])
def test_cpu_matches_golden_bitwise(native, dtype, tb):
    p = prob(97, 41, "inclusive", "hat", dom=2.0)
    npdt = np.float64 if dtype == "fp64" else np.float32
    s = HeatSolver(p, dtype=dtype, backend="cpu", tb=tb)
    s.step(p.ntime)
    got = s.download()
    assert np.array_equal(got, R.owned(R.ftcs(p, dtype=npdt)))
    assert s.steps_done == p.ntime


@pytest.mark.parametrize("conv,ic", [("ghost", "uniform"), ("inclusive", "hat"), ("inclusive", "hat-cuda"),
                                     ("ghost", "hotspot")])
def test_cpu_conventions(native, conv, ic):
    p = prob(64, 30, conv, ic, dom=2.0)
    s = HeatSolver(p, dtype="fp64", backend="cpu", tb=5)
    s.step(13)
    s.step(17)  # split calls == one call
    assert np.array_equal(s.download(), R.owned(R.ftcs(p)))


@pytest.mark.parametrize("P", [1, 2, 3, 4, 7])
@pytest.mark.parametrize("tb", [1, 3, 8])
def test_cpu_loopback_bitwise(native, P, tb):
    p = prob(71, 25, "ghost", "uniform")
    g = LoopbackGroup(p, P, dtype="fp64", backend="cpu", tb=tb)
    g.step(p.ntime)
    assert np.array_equal(g.download(), R.owned(R.ftcs(p)))


@pytest.mark.parametrize("P,shift", [(3, 4), (4, 17), (7, 2), (5, 3)])
def test_cpu_loopback_edge_shift_bitwise(native, P, shift):
    """Edge-balanced slabs (thinner first and last slab): the same field, bitwise."""
    p = prob(71, 25, "ghost", "uniform")
    g = LoopbackGroup(p, P, dtype="fp64", backend="cpu", tb=3, edge_shift=shift)
    assert g.slabs() == [N.decompose(71, P, r, shift) for r in range(P)]
    assert g.slabs()[0][1] < N.decompose(71, P, 0)[1]  # the shift applies
    g.step(p.ntime)
    assert np.array_equal(g.download(), R.owned(R.ftcs(p)))


def test_copy_swap_cpu(native):
    p = prob(50, 9, "inclusive", "hat", dom=2.0)
    s = HeatSolver(p, dtype="fp64", backend="cpu", copy_swap=True)
    s.step(p.ntime)
    assert np.array_equal(s.download(), R.owned(R.ftcs(p)))
    assert s.tb == 1


def test_eigenmode_cpu(native):
    p = prob(65, 100, "inclusive", "sine")
    s = HeatSolver(p, dtype="fp64", backend="cpu", tb=8)
    s.step(p.ntime)
    exact = R.owned(R.eigenmode(p, p.ntime))
    assert np.abs(s.download() - exact).max() < 1e-12
    # decay factor g < 1 for r <= 1/4
    assert 0 < R.eigen_factor(p) < 1


def test_python_demo_parity(native):
    """python/serial/heat.py (31x31, diffuse(10) = 11 steps): same physics, its own
    update formula -> agreement to rounding."""
    demo = R.python_serial_demo()
    # index-slice hat u[7:16, 7:16] = 2 on the 31x31 frame-inclusive grid
    p = prob(31, 11, "inclusive", "hat", dom=2.0)
    p.ic = heat2d.utils.config.IcSpec(kind=heat2d.utils.config.IC_INDEX_BOX, a=2.0, b=1.0, i0=7, i1=16, j0=7,
                                      j1=16)
    p.r = 0.05 * (0.25 * (2 / 30) * (2 / 30) / 0.05) / (2 / 30) ** 2
    s = HeatSolver(p, dtype="fp64", backend="cpu", tb=4)
    s.step(11)
    got = s.download()
    assert np.abs(got - demo[1:-1, 1:-1].T).max() < 1e-13


def test_stats_cpu(native):
    p = prob(40, 6, "ghost", "uniform")
    s = HeatSolver(p, dtype="fp64", backend="cpu", tb=2)
    s.step(6)
    st = s.stats(residual=True)
    T = R.owned(R.ftcs(p))
    assert np.isclose(st["sum"], T.sum(), rtol=1e-13)
    assert st["max"] == T.max() and st["min"] == T.min()
    # the last cycle had depth 2: the other buffer is T_4, not T_5 -> no residual claimed
    assert np.isnan(st["residual_l2"]) and np.isnan(st["residual_max"])
    s.close()


@pytest.mark.parametrize("tb,n", [(1, 6), (2, 7), (8, 19)])
def test_step_stats_cpu(native, tb, n):
    """step_stats: global statistics + the one-step residual T_n - T_{n-1} at any depth."""
    p = prob(40, n, "ghost", "sine")
    s = HeatSolver(p, dtype="fp64", backend="cpu", tb=tb)
    s.upload(R.owned(R.initial_field(p)))
    st = s.step_stats(n)
    T = R.owned(R.ftcs(p))
    d = T - R.owned(R.ftcs(p, n - 1))
    assert np.isclose(st["sum"], T.sum(), rtol=1e-13, atol=1e-12)
    assert st["max"] == T.max() and st["min"] == T.min()
    assert np.isclose(st["residual_l2"], np.sqrt((d * d).sum()), rtol=1e-12)
    assert st["residual_max"] == np.abs(d).max()
    assert np.array_equal(s.download(), T)
    s.close()


def test_upload_download_cpu(native):
    p = prob(33, 3, "ghost", "uniform")
    s = HeatSolver(p, dtype="fp32", backend="cpu", tb=3)
    a = np.random.default_rng(1).random((33, 33)).astype(np.float32)
    s.upload(a)
    assert np.array_equal(s.download(), a)
    # stepping from an uploaded state == golden from the same state
    s.step(3)
    T0 = R.initial_field(p, np.float32)
    T0[1:-1, 1:-1] = a
    ref = T0
    for _ in range(3):
        ref = R.ftcs_step(ref, p.r)
    assert np.array_equal(s.download(), ref[1:-1, 1:-1])


def test_unstable_sigma_blows_up(native):
    """sigma > 1/4 violates the 2-D FTCS limit: the checksum exposes it."""
    p = prob(32, 400, "inclusive", "hat", dom=2.0, sigma=0.3)
    s = HeatSolver(p, dtype="fp64", backend="cpu", tb=8)
    s.step(p.ntime)
    st = s.stats()
    assert not np.isfinite(st["sum"]) or st["max"] > 1e3
