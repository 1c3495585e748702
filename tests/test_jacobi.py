"""r = 1/4 arithmetic (``arith="jacobi"``, SolverConfig::arith 2): with
sigma = 0.25 (every shipped input.dat, the reference benchmark) the centre
weight 1 - 4r of the FTCS update is zero and the step is
r * (((S + E) + N) + W) — the reference's own sum with one exact multiply. The
kernels carry the interior levels scaled by 4^level (3 adds + 2 DPP moves per
point) and unscale at the store; pinned kinds use fma(re, sum, ke*C).
Oracles:
  * the NumPy golden of the same expression (models.reference.ftcs(arith=
    "jacobi")) and the CPU twin, bitwise, on rough data where the form really
    differs from the reference rounding (checked: it does);
  * the reference rounding itself, bitwise, where every sum - 4c is exact
    (Sterbenz: the reference IC, values in [1, 2]) — the bench configuration.
GPU cases cover every edge kind, the split schedule + autotuner, the fused
statistics, the hipRTC engine and multi-rank slabs."""
import numpy as np
import pytest

import heat2d
from heat2d.models import reference as R
from heat2d.models.heat2d import HeatSolver, LoopbackGroup


def prob(n, steps, conv="ghost", ic="sine", sigma=0.25, dom=1.0):
    return heat2d.make_problem(heat2d.InputDat(n=n, sigma=sigma, nu=0.05, dom_len=dom, ntime=steps), conv, ic)


def rough(p, npdt, seed=0):
    return np.random.default_rng(seed).random((p.n_owned, p.n_owned)).astype(npdt)


def golden(p, npdt, T0=None, arith="jacobi", steps=None):
    full = None
    if T0 is not None:
        full = R.initial_field(p, npdt)
        full[1:-1, 1:-1] = T0
    return R.owned(R.ftcs(p, steps, dtype=npdt, T0=full, arith=arith))


def run(p, backend, dtype, tb, arith="jacobi", upload=None, steps=None, **kw):
    s = HeatSolver(p, dtype=dtype, backend=backend, tb=tb, arith=arith, device=0 if backend == "hip" else None, **kw)
    if upload is not None:
        s.upload(upload)
    s.step(p.ntime if steps is None else steps)
    out = s.download()
    s.close()
    return out


@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
@pytest.mark.parametrize("tb", [1, 5, 12])
def test_cpu_jacobi_equals_golden(native, dtype, tb):
    p = prob(71, 29)
    assert p.r == 0.25
    npdt = np.float64 if dtype == "fp64" else np.float32
    T0 = rough(p, npdt)
    got = run(p, "cpu", dtype, tb, upload=T0)
    assert np.array_equal(got, golden(p, npdt, T0))
    assert not np.array_equal(got, golden(p, npdt, T0, arith="exact"))  # a different rounding really ran


@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
def test_cpu_jacobi_equals_reference_rounding_on_reference_ic(native, dtype):
    """Reference IC (T = 2 inside, 1 on the frame): every value stays in [1, 2],
    so sum - 4c is exact and the r = 1/4 form rounds like the reference."""
    p = prob(90, 40, "ghost", "uniform")
    npdt = np.float64 if dtype == "fp64" else np.float32
    got = run(p, "cpu", dtype, 6)
    assert np.array_equal(got, R.owned(R.ftcs(p, dtype=npdt)))


@pytest.mark.parametrize("P", [2, 3])
def test_cpu_jacobi_decomposition_bitwise(native, P):
    p = prob(59, 27)
    single = run(p, "cpu", "fp64", 4)
    g = LoopbackGroup(p, P, dtype="fp64", backend="cpu", tb=4, arith="jacobi")
    g.step(p.ntime)
    assert np.array_equal(g.download(), single)
    g.close()


def test_jacobi_needs_quarter_r(native):
    p = prob(40, 3, sigma=0.2)
    assert p.r != 0.25
    with pytest.raises(Exception, match="1/4"):
        HeatSolver(p, backend="cpu", arith="jacobi")
    with pytest.raises(ValueError):
        R.ftcs(p, arith="jacobi")


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,tb", [("fp64", 1), ("fp64", 4), ("fp64", 12), ("fp64", 20), ("fp64", 24),
                                      ("fp32", 1), ("fp32", 7), ("fp32", 16), ("fp32", 18), ("fp32", 20),
                                      ("fp32", 22), ("fp32", 24)])
def test_hip_jacobi_equals_golden(gpu, native, dtype, tb):
    """Every edge kind (frame rows, frame columns, corners, interior) on a small
    odd grid, rough data: the scaled interior and the unscaled pinned kinds
    give the golden bits."""
    p = prob(301, 2 * tb + 3)
    npdt = np.float64 if dtype == "fp64" else np.float32
    T0 = rough(p, npdt)
    got = run(p, "hip", dtype, tb, upload=T0)
    ref = golden(p, npdt, T0)
    assert np.array_equal(got, ref), np.abs(got.astype(np.float64) - ref).max()


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,tb,n", [("fp64", 12, 1100), ("fp32", 10, 1100), ("fp64", 20, 1500),
                                        ("fp32", 16, 1300), ("fp32", 20, 1300), ("fp32", 17, 1500),
                                        ("fp32", 24, 1300), ("fp32", 21, 1500)])
def test_hip_jacobi_split_schedule(gpu, native, dtype, tb, n):
    """Split (MAIN + EDGE) schedule with the autotuner, rough data."""
    p = prob(n, 2 * tb + 3)
    npdt = np.float64 if dtype == "fp64" else np.float32
    T0 = rough(p, npdt)
    got = run(p, "hip", dtype, tb, upload=T0, autotune=1)
    assert np.array_equal(got, golden(p, npdt, T0))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
def test_hip_jacobi_equals_exact_on_reference_ic(gpu, native, dtype):
    """The bench configuration: reference IC, r = 1/4 -> the jacobi kernels give
    the reference rounding's bits (split schedule, measured plans)."""
    p = prob(2048, 60, "ghost", "uniform")
    npdt = np.float64 if dtype == "fp64" else np.float32
    a = run(p, "hip", dtype, 0)
    b = run(p, "hip", dtype, 0, arith="exact")
    assert np.array_equal(a, b)
    assert np.array_equal(a, R.owned(R.ftcs(p, dtype=npdt)))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,tb", [("fp64", 14), ("fp64", 20), ("fp32", 16)])
def test_hip_jacobi_step_stats(gpu, native, dtype, tb):
    """Fused statistics + one-step residual: the scaled level K-1 is unscaled."""
    p = prob(1100, 3 * tb + 2)
    npdt = np.float64 if dtype == "fp64" else np.float32
    s = HeatSolver(p, dtype=dtype, backend="hip", tb=tb, device=0, arith="jacobi")
    s.upload(R.owned(R.initial_field(p, npdt)))
    n1 = p.ntime - tb
    st = s.step_stats(n1)
    T = golden(p, npdt, steps=n1).astype(np.float64)
    d = T - golden(p, npdt, steps=n1 - 1).astype(np.float64)
    assert np.isclose(st["sum"], T.sum(), rtol=1e-12, atol=1e-9)
    assert st["min"] == T.min() and st["max"] == T.max()
    assert np.isclose(st["residual_l2"], np.sqrt((d * d).sum()), rtol=1e-10)
    assert st["residual_max"] == np.abs(d).max()
    s.step(tb)
    assert np.array_equal(s.download(), golden(p, npdt))
    s.close()


@pytest.mark.gpu
def test_hip_jacobi_jit_and_ranks(gpu, native):
    """hipRTC engine and a 3-rank loopback group == the temporal-blocked engine."""
    p = prob(257, 9)
    T0 = rough(p, np.float64)
    a = run(p, "hip", "fp64", 1, upload=T0, engine="jit")
    b = run(p, "hip", "fp64", 4, upload=T0)
    assert np.array_equal(a, b) and np.array_equal(b, golden(p, np.float64, T0))
    p = prob(700, 41)
    g = LoopbackGroup(p, 3, dtype="fp64", backend="hip", tb=13, arith="jacobi")
    g.upload(R.owned(R.initial_field(p)))  # the host IC (device sin() may differ in the last bit)
    g.step(p.ntime)
    assert np.array_equal(g.download(), golden(p, np.float64))
    g.close()


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,tb,env", [("fp32", 16, {"HEAT2D_SEGMENTS": "30"}),
                                          ("fp64", 12, {"HEAT2D_SEGMENTS": "44"}),
                                          ("fp32", 15, {"HEAT2D_BANDS": "4"}),
                                          ("fp64", 20, {"HEAT2D_BANDS": "3"})])
def test_hip_jacobi_single_launch_frame_rects(gpu, native, monkeypatch, dtype, tb, env):
    """Single-launch plan (the small grid's) with frame-weighted rects: the two
    frame-column strips and a short top / bottom band on every interior strip
    (edge kind 1 costs ~1.5x an interior row: stencil_tb.hip weighted_main),
    strip-aligned segments or bands in between — 5 rects, rough data, bitwise."""
    monkeypatch.setenv("HEAT2D_SPLIT_ORDER", "single")
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    p = prob(1100, 2 * tb + 3)
    npdt = np.float64 if dtype == "fp64" else np.float32
    T0 = rough(p, npdt)
    s = HeatSolver(p, dtype=dtype, backend="hip", tb=tb, device=0, autotune=0, arith="jacobi")
    s.upload(T0)
    s.step(p.ntime)
    got = s.download()
    pl = s.plan(tb)
    s.close()
    assert pl["order"] == "single" and len(pl["main_rects"]) == 5, pl
    top, bot = pl["main_rects"][1], pl["main_rects"][3]
    assert top[0] == 0 and top[4] == 1 and bot[1] == p.n_owned and bot[4] == 1, pl
    assert top[1] - top[0] >= tb and bot[1] - bot[0] >= tb
    assert np.array_equal(got, golden(p, npdt, T0))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,ring,arith,tb", [("fp32", 8, "jacobi", 16), ("fp32", 8, "fma", 15), ("fp32", 8, "exact", 3),
                                                ("fp32", 8, "jacobi", 9)])
def test_hip_ring8_single_launch(gpu, native, monkeypatch, dtype, ring, arith, tb):
    """Ring 8 for single launches (fp32 general kernel: 6 level-0 rows in
    flight instead of 4): frame-weighted segments, bitwise."""
    monkeypatch.setenv("HEAT2D_SPLIT_ORDER", "single")
    monkeypatch.setenv("HEAT2D_TB_RING", str(ring))
    monkeypatch.setenv("HEAT2D_SEGMENTS", "30" if dtype == "fp32" else "44")
    p = prob(1100, 2 * tb + 3)
    npdt = np.float64 if dtype == "fp64" else np.float32
    T0 = rough(p, npdt)
    s = HeatSolver(p, dtype=dtype, backend="hip", tb=tb, device=0, autotune=0, arith=arith)
    s.upload(T0)
    s.step(p.ntime)
    got = s.download()
    pl = s.plan(tb)
    s.close()
    assert pl["order"] == "single" and pl["ring"] == ring, pl
    assert np.array_equal(got, golden(p, npdt, T0, arith=arith))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,tb,order,nseg,graph", [("fp64", 12, "single", 400, False), ("fp32", 16, "single", 300, True),
                                                       ("fp64", 20, "concurrent", 500, True),
                                                       ("fp32", 20, "edge-first", 700, False)])
def test_hip_dynamic_queue(gpu, native, monkeypatch, dtype, tb, order, nseg, graph):
    """Dynamic item queue (HEAT2D_DYNAMIC=1: after its first item a wave takes
    the next free one from a device counter, reset by the last wave): many
    more segments than waves would be needed to show balance, but correctness
    needs only > 1 item per wave — forced here with HEAT2D_MAX_WAVES=96;
    several cycles (the reset between launches), graph replays, bitwise."""
    monkeypatch.setenv("HEAT2D_SPLIT_ORDER", order)
    monkeypatch.setenv("HEAT2D_DYNAMIC", "1")
    monkeypatch.setenv("HEAT2D_SEGMENTS", str(nseg))
    monkeypatch.setenv("HEAT2D_MAX_WAVES", "96")
    p = prob(1100, 3 * tb + 5)
    npdt = np.float64 if dtype == "fp64" else np.float32
    T0 = rough(p, npdt)
    s = HeatSolver(p, dtype=dtype, backend="hip", tb=tb, device=0, autotune=0, arith="jacobi", graph=graph)
    s.upload(T0)
    s.step(p.ntime)
    got = s.download()
    pl = s.plan(tb)
    s.close()
    assert pl["dynamic"] == 1 and pl["main_items"] > pl["main_waves"], pl
    assert np.array_equal(got, golden(p, npdt, T0))
