"""Scaled-level arithmetic for any r (``arith="fast"``, the kernels' AR 3,
tb_impl.hpp): levels carried as X_s = T_s / r^s, so one level is
X_{s+1} = fma((1 - 4r)/r, X_s(C), ((S + E) + N) + W) — 3 adds + 1 fma per point
instead of the contracted reference form's 5 ops — unscaled by r^K at the
store. Not the reference rounding, so checked against the exact NumPy golden
(models/reference.py) within the stated bound

    max |T_fast - T_exact| <= 16 * n * u * max|T0|   (models.reference.fast_error_bound)

on rough data (random values, so no rounding happens to be exact), for several
sigmas (r), depths, both dtypes and both plan shapes (split + single launch).
At r = 1/4 it is bitwise the r = 1/4 form ("jacobi"). The CPU twin runs the
unscaled contracted form (arith 1) for it."""
import dataclasses

import numpy as np
import pytest

import heat2d
from heat2d.models import reference as R
from heat2d.models.heat2d import HeatSolver


def prob(n, steps, sigma):
    return heat2d.make_problem(heat2d.InputDat(n=n, sigma=sigma, nu=0.05, dom_len=1.0, ntime=steps), "ghost",
                               "uniform")


def rough(p, npdt, seed=3):
    return np.random.default_rng(seed).random((p.n_owned, p.n_owned)).astype(npdt)


def exact(p, npdt, T0, steps):
    full = R.initial_field(p, npdt)
    full[1:-1, 1:-1] = T0
    return R.owned(R.ftcs(p, steps, dtype=npdt, T0=full, arith="exact"))


def run(p, backend, dtype, tb, arith, T0, steps, **kw):
    s = HeatSolver(p, dtype=dtype, backend=backend, tb=tb, arith=arith, device=0 if backend == "hip" else None, **kw)
    s.upload(T0)
    s.step(steps)
    out = s.download()
    info = s.info()
    s.close()
    return out, info


def test_bound_formula():
    assert R.fast_error_bound(10, np.float64, 2.0) == 16 * 10 * 2.0 ** -53 * 2.0
    assert R.fast_error_bound(3, np.float32, 1.0) == 16 * 3 * 2.0 ** -24


@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
def test_cpu_fast_is_the_contracted_form(native, dtype):
    p = prob(97, 23, 0.2)
    npdt = np.float64 if dtype == "fp64" else np.float32
    T0 = rough(p, npdt)
    a, _ = run(p, "cpu", dtype, 6, "fast", T0, 23)
    b, _ = run(p, "cpu", dtype, 6, "fma", T0, 23)
    assert np.array_equal(a, b)
    d = np.abs(a.astype(np.float64) - exact(p, npdt, T0, 23).astype(np.float64)).max()
    assert d <= R.fast_error_bound(23, npdt, float(T0.max()))


def test_fast_needs_positive_r(native):
    p = prob(64, 4, 0.0)
    with pytest.raises(Exception, match="r > 0"):
        HeatSolver(p, dtype="fp64", backend="cpu", arith="fast")


def test_fast_depth_clamped_to_exponent_range(native):
    """fp32 keeps r^K >= 2^-60: at r = 0.01 at most 9 levels per pass."""
    p = prob(200, 4, 0.01)
    s = HeatSolver(p, dtype="fp32", backend="cpu", tb=20, arith="fast")
    assert s.tb == 9
    s.close()
    s = HeatSolver(p, dtype="fp64", backend="cpu", tb=20, arith="fast")
    assert s.tb == 20
    s.close()


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
@pytest.mark.parametrize("sigma", [0.2, 0.1, 0.2371])
@pytest.mark.parametrize("tb,steps", [(1, 5), (7, 31), (16, 49), (20, 61)])
def test_hip_fast_within_bound(gpu, native, dtype, sigma, tb, steps):
    """Split schedule (autotuned plans, measured schedule: every kernel kind,
    scaled interior + unscaled pinned items) on 1100^2 rough data."""
    if dtype == "fp32" and tb > 20:
        pytest.skip("fp32 depth")
    p = prob(1100, steps, sigma)
    npdt = np.float64 if dtype == "fp64" else np.float32
    T0 = rough(p, npdt) + npdt(0.5)
    got, info = run(p, "hip", dtype, tb, "fast", T0, steps, autotune=1)
    ref = exact(p, npdt, T0, steps)
    d = np.abs(got.astype(np.float64) - ref.astype(np.float64)).max()
    bound = R.fast_error_bound(steps, npdt, float(T0.max()))
    assert d <= bound, (d, bound)
    assert d > 0 or tb == 1, "fast arithmetic is not the reference rounding on rough data"


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,tb,env", [("fp32", 16, {"HEAT2D_SEGMENTS": "30"}), ("fp64", 12, {"HEAT2D_BANDS": "3"}),
                                          ("fp32", 9, {"HEAT2D_TB_RING": "8", "HEAT2D_SEGMENTS": "44"})])
def test_hip_fast_single_launch_within_bound(gpu, native, monkeypatch, dtype, tb, env):
    """Single launches (the small grid's plan: frame-weighted rects, every edge kind in one launch)."""
    monkeypatch.setenv("HEAT2D_SPLIT_ORDER", "single")
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    p = prob(1100, 2 * tb + 3, 0.2)
    npdt = np.float64 if dtype == "fp64" else np.float32
    T0 = rough(p, npdt)
    got, _ = run(p, "hip", dtype, tb, "fast", T0, p.ntime, autotune=0)
    d = np.abs(got.astype(np.float64) - exact(p, npdt, T0, p.ntime).astype(np.float64)).max()
    assert d <= R.fast_error_bound(p.ntime, npdt, float(T0.max())), d


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
def test_hip_fast_at_quarter_is_jacobi(gpu, native, dtype):
    """r = 1/4: b = 0 and r^K is a power of two — the r = 1/4 form, bitwise."""
    p = dataclasses.replace(prob(777, 45, 0.25), r=0.25)  # (r = nu dt / delta^2 is 1/4 only up to rounding)
    npdt = np.float64 if dtype == "fp64" else np.float32
    T0 = rough(p, npdt)
    a, _ = run(p, "hip", dtype, 15, "fast", T0, 45, autotune=1)
    b, _ = run(p, "hip", dtype, 15, "jacobi", T0, 45, autotune=1)
    assert np.array_equal(a, b)


@pytest.mark.gpu
def test_hip_fast_step_stats(gpu, native):
    """The fused-statistics cycle with scaled levels (the residual's level K-1
    is unscaled by r^(K-1)): statistics of the field it stores."""
    p = prob(900, 37, 0.2)
    T0 = rough(p, np.float64)
    s = HeatSolver(p, dtype="fp64", backend="hip", tb=12, arith="fast", device=0)
    s.upload(T0)
    st = s.step_stats(37)
    got = s.download()
    s.close()
    assert np.isclose(st["sum"], got.astype(np.float64).sum(), rtol=1e-12)
    assert st["min"] == got.min() and st["max"] == got.max()
    ref = exact(p, np.float64, T0, 37)
    ref1 = exact(p, np.float64, T0, 36)
    assert np.isclose(st["residual_max"], np.abs(ref - ref1).max(), rtol=1e-6)
