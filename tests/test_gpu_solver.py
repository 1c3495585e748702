"""GPU numerics: the native HIP engine against the NumPy golden (fp64 reference
order, bitwise) on a real MI355X. Every test runs the HIP kernels through
_native/libheat2d.so — there is no fallback path."""
import numpy as np
import pytest

import heat2d
from heat2d.models import reference as R
from heat2d.models.heat2d import HeatSolver, LoopbackGroup

pytestmark = pytest.mark.gpu


def prob(n, steps, conv="ghost", ic="uniform", dom=1.0):
    return heat2d.make_problem(heat2d.InputDat(n=n, sigma=0.25, nu=0.05, dom_len=dom, ntime=steps), conv, ic)


@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
@pytest.mark.parametrize("tb", [1, 2, 3, 5, 8, 13, 16])
def test_hip_matches_golden_bitwise(gpu, native, dtype, tb):
    p = prob(203, 37, "inclusive", "hat", dom=2.0)  # odd size: partial strips / lanes
    npdt = np.float64 if dtype == "fp64" else np.float32
    s = HeatSolver(p, dtype=dtype, backend="hip", tb=tb, device=0)
    s.step(p.ntime)
    got = s.download()
    ref = R.owned(R.ftcs(p, dtype=npdt))
    assert got.dtype == npdt
    assert np.array_equal(got, ref), np.abs(got.astype(np.float64) - ref).max()
    s.close()


@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
@pytest.mark.parametrize("tb", [1, 4, 7, 10, 16])
def test_hip_sine_bitwise(gpu, native, dtype, tb):
    """Non-dyadic data (the sine eigenmode): every rounding step of the update
    is exercised, so an fp32 kernel that silently computes in fp64 (or any
    reassociation) fails here."""
    p = prob(301, 29, "ghost", "sine")
    npdt = np.float64 if dtype == "fp64" else np.float32
    s = HeatSolver(p, dtype=dtype, backend="hip", tb=tb, device=0)
    # host IC (device sin() and NumPy's may differ in the last ulp; the frame is exactly 0)
    s.upload(R.owned(R.initial_field(p, npdt)))
    s.step(p.ntime)
    got = s.download()
    ref = R.owned(R.ftcs(p, dtype=npdt))
    assert np.array_equal(got, ref), np.abs(got.astype(np.float64) - ref).max()
    s.close()


@pytest.mark.parametrize("dtype,tb,n", [("fp64", 10, 1100), ("fp32", 9, 1100), ("fp64", 4, 777),
                                         ("fp32", 16, 1500), ("fp64", 1, 700)])
def test_hip_split_schedule_bitwise(gpu, native, dtype, tb, n):
    """Grids large enough for the MAIN + EDGE split (interior-only kernel on the
    compute stream, bands + frame strips on the comm stream), on non-dyadic
    data, against the golden; and identical to the serial single-launch
    schedule."""
    from heat2d.ops import _native as N
    p = prob(n, 23, "ghost", "sine")
    npdt = np.float64 if dtype == "fp64" else np.float32
    T0 = R.owned(R.initial_field(p, npdt))
    outs = []
    for overlap in (True, False):
        s = HeatSolver(p, dtype=dtype, backend="hip", tb=tb, device=0, overlap=overlap)
        s.upload(T0)
        s.step(p.ntime)
        outs.append(s.download())
        s.close()
    ref = R.owned(R.ftcs(p, dtype=npdt))
    assert np.array_equal(outs[0], ref), np.abs(outs[0].astype(np.float64) - ref).max()
    assert np.array_equal(outs[1], ref)
    sp = N.plan_split(N.F64 if dtype == "fp64" else N.F32, N.make_layout(n, n, halo=16), min(tb, 16), min(tb, 16))
    assert sp.valid == 1 and sp.main_items > 0 and sp.edge_items > 0


@pytest.mark.parametrize("dtype,tb", [("fp64", 12), ("fp32", 10)])
def test_hip_autotune_keeps_state_bitwise(gpu, native, dtype, tb):
    """The split-plan autotuner runs trial cycles on the real buffers and
    writes only the non-current buffer (no swap): the solution must be untouched
    (bitwise vs the golden), and the chosen plan valid."""
    p = prob(1100, 29, "ghost", "sine")
    npdt = np.float64 if dtype == "fp64" else np.float32
    s = HeatSolver(p, dtype=dtype, backend="hip", tb=tb, device=0, autotune=1)
    s.upload(R.owned(R.initial_field(p, npdt)))
    s.prepare(p.ntime)
    pl = s.plan()
    assert pl["valid"] in (1, 2, 3) and pl["tuned_ms"] > 0.0 and pl["ring"] in (4, 6, 8)  # split or single launch (8: fp32 single)
    s.step(p.ntime)
    ref = R.owned(R.ftcs(p, dtype=npdt))
    got = s.download()
    assert np.array_equal(got, ref), np.abs(got.astype(np.float64) - ref).max()
    s.close()


@pytest.mark.parametrize("n", [3, 17, 64, 130, 257, 1000])
def test_hip_sizes(gpu, native, n):
    p = prob(n, 21, "ghost", "uniform")
    s = HeatSolver(p, dtype="fp64", backend="hip", tb=8, device=0)
    s.step(p.ntime)
    assert np.array_equal(s.download(), R.owned(R.ftcs(p)))
    s.close()


# negative: -tile_rows segment work items (TbRect nb < 0); 300 x 300 fp64 at
# depth 6 is 3 strips = 900 strip rows, so -5000 clamps to one-row segments
@pytest.mark.parametrize("tile_rows", [1, 7, 64, 512, -1, -7, -250, -5000])
def test_hip_tile_rows(gpu, native, tile_rows):
    p = prob(300, 19, "inclusive", "hat-cuda", dom=2.0)
    s = HeatSolver(p, dtype="fp64", backend="hip", tb=6, tile_rows=tile_rows, device=0)
    s.step(p.ntime)
    assert np.array_equal(s.download(), R.owned(R.ftcs(p)))
    s.close()


@pytest.mark.parametrize("P", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("tb", [1, 4, 8])
def test_loopback_group_bitwise(gpu, native, P, tb):
    """P slabs on one GPU with device-copy halo exchange == the single-slab run."""
    p = prob(161, 29, "ghost", "uniform")
    g = LoopbackGroup(p, P, dtype="fp64", backend="hip", tb=tb, device=0)
    g.step(p.ntime)
    got = g.download()
    assert np.array_equal(got, R.owned(R.ftcs(p)))
    g.close()


def test_copy_swap_and_managed(gpu, native):
    p = prob(150, 11, "inclusive", "hat", dom=2.0)
    ref = R.owned(R.ftcs(p))
    for kw in (dict(copy_swap=True), dict(managed=True), dict(graph=True, tb=4)):
        s = HeatSolver(p, dtype="fp64", backend="hip", device=0, **kw)
        s.step(p.ntime)
        assert np.array_equal(s.download(), ref), kw
        s.close()


def test_graph_replay_many(gpu, native):
    p = prob(512, 200, "ghost", "uniform")
    s = HeatSolver(p, dtype="fp64", backend="hip", tb=8, graph=True, device=0)
    s.step(123)
    s.step(77)
    assert np.array_equal(s.download(), R.owned(R.ftcs(p)))
    s.close()


@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
def test_graph_split_schedule_bitwise(gpu, native, dtype):
    """hipGraph capture of the two-stream split cycle (fork/join of the comm
    stream, event protocol as graph edges), interleaved with eager cycles
    (remainders, odd buffer parity), on non-dyadic data."""
    p = prob(1100, 200, "ghost", "sine")
    npdt = np.float64 if dtype == "fp64" else np.float32
    s = HeatSolver(p, dtype=dtype, backend="hip", tb=8, graph=True, device=0)
    s.upload(R.owned(R.initial_field(p, npdt)))
    for n in (123, 5, 72):
        s.step(n)
    assert s.steps_done == 200
    got = s.download()
    ref = R.owned(R.ftcs(p, dtype=npdt))
    assert np.array_equal(got, ref), np.abs(got.astype(np.float64) - ref).max()
    s.close()


@pytest.mark.parametrize("dtype,tb,overlap", [("fp64", 1, True), ("fp64", 8, True), ("fp64", 14, True),
                                               ("fp64", 14, False), ("fp64", 20, True), ("fp32", 8, True),
                                               ("fp32", 16, False)])
def test_step_stats_fused(gpu, native, dtype, tb, overlap):
    """Statistics of T_n and the ONE-STEP residual T_n - T_{n-1} fused into the
    last cycle's stencil launch, at any depth, against NumPy; the field itself
    stays bitwise, and the run continues correctly after the stats cycle."""
    p = prob(1100, 3 * tb + 2, "ghost", "sine")
    npdt = np.float64 if dtype == "fp64" else np.float32
    s = HeatSolver(p, dtype=dtype, backend="hip", tb=tb, device=0, overlap=overlap)
    s.upload(R.owned(R.initial_field(p, npdt)))
    n1 = p.ntime - tb
    st = s.step_stats(n1)
    T = R.owned(R.ftcs(p, n1, dtype=npdt)).astype(np.float64)
    d = T - R.owned(R.ftcs(p, n1 - 1, dtype=npdt)).astype(np.float64)
    assert np.isclose(st["sum"], T.sum(), rtol=1e-12, atol=1e-9)
    assert np.isclose(st["sum_sq"], (T * T).sum(), rtol=1e-12)
    assert st["min"] == T.min() and st["max"] == T.max()
    assert np.isclose(st["residual_l2"], np.sqrt((d * d).sum()), rtol=1e-10)
    assert st["residual_max"] == np.abs(d).max()
    s.step(tb)
    got = s.download()
    assert np.array_equal(got, R.owned(R.ftcs(p, dtype=npdt)))
    s.close()


def test_stats_and_residual(gpu, native):
    p = prob(300, 10, "ghost", "uniform")
    s = HeatSolver(p, dtype="fp64", backend="hip", tb=1, device=0)
    s.step(10)
    st = s.stats(residual=True)
    T = R.ftcs(p)
    T9 = R.ftcs(p, 9)
    assert np.isclose(st["sum"], R.owned(T).sum(), rtol=1e-13)
    assert st["min"] == R.owned(T).min() and st["max"] == R.owned(T).max()
    d = R.owned(T) - R.owned(T9)
    assert np.isclose(st["residual_l2"], np.sqrt((d * d).sum()), rtol=1e-10)
    s.close()


def test_eigenmode_gpu(gpu, native):
    p = prob(129, 200, "inclusive", "sine")
    s = HeatSolver(p, dtype="fp64", backend="hip", tb=8, device=0)
    s.step(p.ntime)
    exact = R.owned(R.eigenmode(p, p.ntime))
    assert np.abs(s.download() - exact).max() < 1e-12
    s.close()


def test_upload_roundtrip(gpu, native):
    p = prob(100, 5, "ghost", "uniform")
    s = HeatSolver(p, dtype="fp64", backend="hip", tb=4, device=0)
    a = np.random.default_rng(0).random((100, 100))
    s.upload(a)
    assert np.array_equal(s.download(), a)
    s.close()


def test_phase_timers(gpu, native):
    """hipEvent phase timers: split cycles report main/edge time, serial cycles
    compute/exchange; counts match the number of cycles; reading resets."""
    p = prob(1100, 40, "ghost", "uniform")
    s = HeatSolver(p, dtype="fp64", backend="hip", tb=8, device=0)
    s.set_timing(True)
    s.step(40)
    ph = s.phase_times()
    assert ph["cycles"] == 5 and ph["main_ms"] > 0 and ph["edge_ms"] > 0 and ph["cycle_ms"] >= ph["main_ms"]
    assert s.phase_times()["cycles"] == 0
    s.close()
    s = HeatSolver(p, dtype="fp64", backend="hip", tb=8, device=0, overlap=False)
    s.set_timing(True)
    s.step(20)
    ph = s.phase_times()
    assert ph["cycles"] == 3 and ph["main_ms"] > 0 and ph["edge_ms"] == 0
    s.close()


@pytest.mark.parametrize("order", ["edge-first", "concurrent"])
@pytest.mark.parametrize("P,tb,dtype,n", [(2, 8, "fp64", 1100), (4, 12, "fp64", 1100), (3, 16, "fp32", 1300),
                                          (5, 14, "fp64", 900)])
def test_split_orders_with_exchange_bitwise(gpu, native, order, P, tb, dtype, n, monkeypatch):
    """The overlapped multi-rank schedule with REAL halo exchanges on one GPU:
    P member solvers, each with its own compute / comm streams and autotuned
    split plans, exchange band rows through the loopback transport (RCCL's
    messages, copied device-to-device, ordered by events). Both split orders —
    edge-first (bands, then interior, exchange beside the interior) and
    concurrent (interior beside bands + exchange) — on non-dyadic data must be
    bitwise equal to the golden on ALL rows, and every member must really have
    run the requested order."""
    monkeypatch.setenv("HEAT2D_SPLIT_ORDER", order)
    steps = 3 * tb + 5  # full cycles and a balanced remainder
    p = prob(n, steps, "ghost", "sine")
    npdt = np.float64 if dtype == "fp64" else np.float32
    g = LoopbackGroup(p, P, dtype=dtype, backend="hip", tb=tb, device=0, autotune=1)
    g.upload(R.owned(R.initial_field(p, npdt)))
    g.step(p.ntime)
    got = g.download()
    want = 3 if order == "edge-first" else 1
    for i in range(P):
        hist = g.cycle_hist(i)
        assert sum(k * c for k, c in hist.items()) == steps
        for k in hist:
            pl = g.plan(i, k)
            assert pl["valid"] == want and pl["tuned_ms"] > 0, (i, k, pl)
    g.close()
    ref = R.owned(R.ftcs(p, dtype=npdt))
    assert np.array_equal(got, ref), np.argwhere(got != ref)[:5]


@pytest.mark.parametrize("order,nb", [("edge-first", 3), ("concurrent", 2), ("edge-first", 40)])
@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
def test_edge_band_plans_bitwise(gpu, native, order, nb, dtype, monkeypatch):
    """Boundary-band rects cut into nb row bands each (kern::with_edge_bands,
    HEAT2D_EDGE_BANDS; 40 > band rows: one-row items), split orders with real
    loopback exchanges: bitwise the golden."""
    monkeypatch.setenv("HEAT2D_SPLIT_ORDER", order)
    monkeypatch.setenv("HEAT2D_EDGE_BANDS", str(nb))
    tb = 12 if dtype == "fp64" else 16
    p = prob(1100, 2 * tb + 3, "ghost", "sine")
    npdt = np.float64 if dtype == "fp64" else np.float32
    g = LoopbackGroup(p, 3, dtype=dtype, backend="hip", tb=tb, device=0, autotune=0)
    g.upload(R.owned(R.initial_field(p, npdt)))
    g.step(p.ntime)
    got = g.download()
    plans = [g.plan(i, tb) for i in range(3)]
    g.close()
    for pl in plans:
        assert all(e[4] == min(nb, e[1] - e[0]) for e in pl["edge_rects"]), pl
    assert np.array_equal(got, R.owned(R.ftcs(p, dtype=npdt)))


@pytest.mark.parametrize("order,nseg", [("edge-first", 37), ("concurrent", 1000), ("single", 5), ("single", 4097),
                                        ("concurrent", -3), ("single", -40)])
@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
def test_segment_plans_bitwise(gpu, native, order, nseg, dtype, monkeypatch):
    """Interior / single launches cut into segment work items (HEAT2D_SEGMENTS,
    TbRect nb < 0 — runs of the strip-major row sequence crossing strip ends)
    or forced row-band counts (HEAT2D_BANDS, nseg < 0 here) are bitwise equal
    to the golden: split orders with real loopback exchanges, and the single
    launch of an unsplit grid."""
    monkeypatch.setenv("HEAT2D_SPLIT_ORDER", order)
    monkeypatch.setenv("HEAT2D_SEGMENTS" if nseg > 0 else "HEAT2D_BANDS", str(abs(nseg)))
    tb = 12 if dtype == "fp64" else 16
    p = prob(1100, 2 * tb + 3, "ghost", "sine")
    npdt = np.float64 if dtype == "fp64" else np.float32
    if order == "single":
        s = HeatSolver(p, dtype=dtype, backend="hip", tb=tb, device=0, autotune=0)
        s.upload(R.owned(R.initial_field(p, npdt)))
        s.step(p.ntime)
        got = s.download()
        pl = s.plan(tb)
        s.close()
        plans = [pl]
    else:
        g = LoopbackGroup(p, 3, dtype=dtype, backend="hip", tb=tb, device=0, autotune=0)
        g.upload(R.owned(R.initial_field(p, npdt)))
        g.step(p.ntime)
        got = g.download()
        plans = [g.plan(i, tb) for i in range(3)]
        g.close()
    for pl in plans:
        if nseg > 0:
            assert pl["main_bands"] == -pl["main_items"] and 0 < pl["main_items"] <= nseg, pl
        else:
            assert 0 < pl["main_bands"] <= -nseg, pl
        assert pl["valid"] == {"edge-first": 3, "concurrent": 1, "single": 2}[order], pl
    ref = R.owned(R.ftcs(p, dtype=npdt))
    assert np.array_equal(got, ref), np.argwhere(got != ref)[:5]


@pytest.mark.parametrize("P", [2, 3])
def test_loopback_serial_schedule_bitwise(gpu, native, P):
    """overlap=False: one launch per cycle on the compute stream, exchange
    behind it on the same stream (the two-phase post / pull protocol still
    orders the ranks)."""
    p = prob(600, 41, "ghost", "sine")
    g = LoopbackGroup(p, P, dtype="fp64", backend="hip", tb=9, device=0, overlap=False)
    g.upload(R.owned(R.initial_field(p)))
    g.step(p.ntime)
    got = g.download()
    g.close()
    assert np.array_equal(got, R.owned(R.ftcs(p)))


@pytest.mark.parametrize("n,tb,graph", [(1000, 16, True), (1000, 16, False), (100, 12, False), (50, 12, True),
                                        (13, 12, False), (480, 12, False)])
def test_prepare_covers_every_depth(gpu, native, n, tb, graph):
    """prepare(n) plans every cycle depth step(n) launches (graph pairs, then
    balanced eager cycles), so no plan — and no autotuning — happens inside a
    timed step(n)."""
    p = prob(300, n, "ghost", "uniform")
    s = HeatSolver(p, dtype="fp32", backend="hip", tb=tb, device=0, graph=graph)
    s.prepare(n)
    before = s.plans_made
    s.step(n)
    s.synchronize()
    assert s.plans_made == before
    assert np.array_equal(s.download(), R.owned(R.ftcs(p, dtype=np.float32)))
    s.close()


@pytest.mark.parametrize("tb", [6, 14])
def test_prepare_covers_warmup_parity(gpu, native, tb):
    """bench order: prepare(n), an untimed warmup that leaves the buffer parity
    at 1, then step(n). Graph pairs start only at parity 0, so step(n) launches
    other remainder depths than a walk from parity 0 would plan."""
    n, warm = 1000, 64
    p = prob(300, warm + n, "ghost", "uniform")
    s = HeatSolver(p, dtype="fp32", backend="hip", tb=tb, device=0, graph=True)
    s.prepare(n)
    s.step(warm)
    s.synchronize()
    before = s.plans_made
    s.step(n)
    s.synchronize()
    assert s.plans_made == before
    assert np.array_equal(s.download(), R.owned(R.ftcs(p, dtype=np.float32)))
    s.close()


@pytest.mark.parametrize("dtype,n,steps", [("fp64", 1100, 20), ("fp32", 1100, 37), ("fp64", 700, 45)])
def test_measured_schedule(gpu, native, dtype, n, steps):
    """prepare(n) on an autotuned slab picks step(n)'s cycle schedule from
    measured cycle times (the exact DP over the tuned depths, up to max_tb: 24
    for both dtypes — any mix of depths, e.g. 12 + 12 + 12 + 9); step(n) runs
    exactly that schedule, plans nothing new, and stays bitwise equal to the
    golden."""
    from collections import Counter
    p = prob(n, steps, "ghost", "sine")
    npdt = np.float64 if dtype == "fp64" else np.float32
    s = HeatSolver(p, dtype=dtype, backend="hip", device=0, autotune=1)
    assert s.tb == 24
    s.upload(R.owned(R.initial_field(p, npdt)))
    s.prepare(steps)
    sched = s.schedule(steps)
    assert sched and sum(sched) == steps and max(sched) <= s.tb and sched == sorted(sched, reverse=True)
    before = s.plans_made
    s.cycle_hist(reset=True)
    s.step(steps)
    s.synchronize()
    assert s.plans_made == before
    assert s.cycle_hist() == dict(Counter(sched))
    got = s.download()
    ref = R.owned(R.ftcs(p, dtype=npdt))
    assert np.array_equal(got, ref), np.abs(got.astype(np.float64) - ref).max()
    s.close()


@pytest.mark.parametrize("k", [17, 20, 24])
def test_deep_fp64_bitwise(gpu, native, k):
    """fp64 depths 17..24 (one-pass short runs): both kernels (split + single) bitwise."""
    p = prob(1100, 2 * k + 3, "ghost", "sine")
    for overlap in (True, False):
        s = HeatSolver(p, dtype="fp64", backend="hip", tb=k, device=0, overlap=overlap)
        s.upload(R.owned(R.initial_field(p)))
        s.step(p.ntime)
        got = s.download()
        s.close()
        assert np.array_equal(got, R.owned(R.ftcs(p))), (k, overlap)


@pytest.mark.parametrize("dtype,n,steps,warm,eager", [("fp32", 1100, 61, 0, False), ("fp32", 1100, 61, 3, False),
                                                      ("fp64", 900, 45, 5, False), ("fp32", 1100, 61, 3, True)])
def test_measured_schedule_graph(gpu, native, monkeypatch, dtype, n, steps, warm, eager):
    """graph=True + a measured schedule: prepare(n) captures the whole schedule
    (both streams, both buffer parities) as one hipGraph; step(n) replays it
    with nothing planned or captured inside; bitwise, also after a warmup
    that flips the parity, and when replayed twice. These short cycles replay;
    with the eager threshold at 0 us (every schedule "long") the same steps
    launch eagerly, still bitwise."""
    if eager:
        monkeypatch.setenv("HEAT2D_GRAPH_MAX_CYCLE_US", "0")
    p = prob(n, warm + 2 * steps, "ghost", "sine")
    npdt = np.float64 if dtype == "fp64" else np.float32
    s = HeatSolver(p, dtype=dtype, backend="hip", device=0, autotune=1, graph=True)
    s.upload(R.owned(R.initial_field(p, npdt)))
    s.step(warm)
    s.prepare(steps)
    assert s.schedule(steps)
    assert s.schedule_replayed(steps) == (not eager)
    before = s.plans_made
    s.cycle_hist(reset=True)
    s.step(steps)
    s.step(steps)
    s.synchronize()
    assert s.plans_made == before and s.steps_done == warm + 2 * steps
    assert sum(k * c for k, c in s.cycle_hist().items()) == 2 * steps
    got = s.download()
    ref = R.owned(R.ftcs(p, dtype=npdt))
    assert np.array_equal(got, ref), np.abs(got.astype(np.float64) - ref).max()
    s.close()
