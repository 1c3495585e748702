"""Contracted arithmetic (``arith="fma"``): the reference update
c + r*(sum - 4c) (fortran/hip/heat_kernel.cpp:43) evaluated as
fma(r, sum - 4c, c) — what hipcc's default -ffp-contract=fast makes of the
reference line. Oracles:
  * r a power of two (sigma = 0.25, every shipped input): r*x is exact, so the
    contracted and the fully rounded forms agree bitwise -> the NumPy golden;
  * any r: the CPU twin (std::fma) and the gfx950 kernels agree bitwise, the
    decomposition is bitwise invariant, and the result stays within rounding of
    the NumPy golden (and actually differs from it, i.e. the fma path ran)."""
import numpy as np
import pytest

import heat2d
from heat2d.models import reference as R
from heat2d.models.heat2d import HeatSolver, LoopbackGroup


def prob(n, steps, conv="ghost", ic="uniform", dom=1.0, sigma=0.25):
    return heat2d.make_problem(heat2d.InputDat(n=n, sigma=sigma, nu=0.05, dom_len=dom, ntime=steps), conv, ic)


def random_field(p, npdt, seed=0):
    return np.random.default_rng(seed).random((p.n_owned, p.n_owned)).astype(npdt)


def run(p, backend, dtype, tb, arith, upload=None, **kw):
    s = HeatSolver(p, dtype=dtype, backend=backend, tb=tb, arith=arith, device=0 if backend == "hip" else None, **kw)
    if upload is not None:
        s.upload(upload)
    s.step(p.ntime)
    out = s.download()
    s.close()
    return out


@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
@pytest.mark.parametrize("tb", [1, 5, 12])
def test_cpu_fma_pow2_r_equals_golden(native, dtype, tb):
    p = prob(73, 31, "inclusive", "hat", dom=2.0)
    assert p.r == 0.25
    npdt = np.float64 if dtype == "fp64" else np.float32
    got = run(p, "cpu", dtype, tb, "fma")
    assert np.array_equal(got, R.owned(R.ftcs(p, dtype=npdt)))


@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
def test_cpu_fma_general_r(native, dtype):
    p = prob(61, 40, "ghost", "uniform", sigma=0.2)
    assert p.r != 0.25
    npdt = np.float64 if dtype == "fp64" else np.float32
    T0 = random_field(p, npdt)  # rough data: r*(sum - 4c) is O(c), so its rounding matters
    fma = run(p, "cpu", dtype, 7, "fma", upload=T0)
    exact = run(p, "cpu", dtype, 7, "exact", upload=T0)
    full = R.initial_field(p, npdt)
    full[1:-1, 1:-1] = T0
    ref = R.owned(R.ftcs(p, dtype=npdt, T0=full))
    assert np.array_equal(exact, ref)
    assert not np.array_equal(fma, exact)  # the contracted path really ran
    tol = 1e-13 if dtype == "fp64" else 1e-5
    assert np.abs(fma.astype(np.float64) - ref).max() < tol
    # depth-invariant: K = 1 and K = 7 contracted runs agree bitwise
    assert np.array_equal(run(p, "cpu", dtype, 1, "fma", upload=T0), fma)


@pytest.mark.parametrize("P", [2, 3])
def test_cpu_fma_decomposition_bitwise(native, P):
    p = prob(59, 27, "ghost", "sine", sigma=0.2)
    single = run(p, "cpu", "fp64", 4, "fma")
    g = LoopbackGroup(p, P, dtype="fp64", backend="cpu", tb=4, arith="fma")
    g.step(p.ntime)
    assert np.array_equal(g.download(), single)
    g.close()
    g = LoopbackGroup(p, P, dtype="fp64", backend="cpu", tb=4, arith="exact")
    g.step(p.ntime)
    assert np.array_equal(g.download(), R.owned(R.ftcs(p)))
    g.close()


def test_bad_arith(native):
    with pytest.raises(ValueError):
        HeatSolver(prob(8, 1), backend="cpu", arith="fastest")


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
@pytest.mark.parametrize("tb", [1, 4, 12, 16])
def test_hip_fma_matches_cpu_twin(gpu, native, dtype, tb):
    """Any r: gfx950 kernel (fma form, every edge kind) == CPU twin, bitwise."""
    p = prob(301, 29, "ghost", "uniform", sigma=0.2)
    npdt = np.float64 if dtype == "fp64" else np.float32
    T0 = random_field(p, npdt)
    gpu_out = run(p, "hip", dtype, tb, "fma", upload=T0)
    cpu_out = run(p, "cpu", dtype, tb, "fma", upload=T0)
    assert np.array_equal(gpu_out, cpu_out), np.abs(gpu_out.astype(np.float64) - cpu_out).max()


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,tb,n", [("fp64", 12, 1100), ("fp32", 10, 1100), ("fp64", 16, 1500)])
def test_hip_fma_split_schedule(gpu, native, dtype, tb, n):
    """Split (MAIN + EDGE) schedule and the autotuner in fma mode == CPU twin."""
    p = prob(n, 2 * tb + 3, "ghost", "uniform", sigma=0.2)
    npdt = np.float64 if dtype == "fp64" else np.float32
    T0 = random_field(p, npdt)
    gpu_out = run(p, "hip", dtype, tb, "fma", upload=T0, autotune=1)
    cpu_out = run(p, "cpu", dtype, tb, "fma", upload=T0)
    assert np.array_equal(gpu_out, cpu_out)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
def test_hip_fma_equals_exact_pow2(gpu, native, dtype):
    """The bench configuration's arithmetic claim: r = 0.25 (reference IC, values
    in [1, 2]) -> contracted == fully rounded, bitwise, on the split schedule."""
    p = prob(2048, 60, "ghost", "uniform")
    assert p.r == 0.25
    a = run(p, "hip", dtype, 12, "fma")
    b = run(p, "hip", dtype, 12, "exact")
    assert np.array_equal(a, b)
    npdt = np.float64 if dtype == "fp64" else np.float32
    assert np.array_equal(a, R.owned(R.ftcs(p, dtype=npdt)))


@pytest.mark.gpu
def test_jit_fma(gpu, native):
    """hipRTC engine in fma mode == temporal-blocked fma engine, bitwise."""
    p = prob(257, 9, "ghost", "uniform", sigma=0.2)
    T0 = random_field(p, np.float64)
    a = run(p, "hip", "fp64", 1, "fma", upload=T0, engine="jit")
    b = run(p, "hip", "fp64", 4, "fma", upload=T0)
    assert np.array_equal(a, b)
