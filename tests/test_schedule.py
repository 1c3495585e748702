"""The measured-schedule search (Solver::prepare -> cycle_schedule), on CPU with
synthetic cycle-time curves: it must find the cheapest cut of n steps into
cycles of at most kmax steps among balanced splits, which for the convex t(k)
the hardware shows (flat while a pass is HBM-bound, then linear in k) is the
global optimum — checked against brute force over all compositions."""
import ctypes as C

import pytest

from heat2d.ops import _native as N


def schedule(n, kmax, t):
    tm = (C.c_double * (kmax + 1))(*([0.0] + [t(k) for k in range(1, kmax + 1)]))
    out = (C.c_int32 * max(1, n))()
    ln = C.c_int64()
    N.call("heat2d_cycle_schedule", n, kmax, tm, out, n, C.byref(ln))
    return [int(v) for v in out[:ln.value]]


def brute(n, kmax, t):
    """Cheapest cut of n steps into cycles of <= kmax steps, over ALL compositions (DP)."""
    best = [0.0] + [float("inf")] * n
    for m in range(1, n + 1):
        best[m] = min(t(k) + best[m - k] for k in range(1, min(kmax, m) + 1))
    return best[n]


def mi355x_fp64(k):  # measured shape at 32768^2 fp64 (profiles/depth_schedule.md): ms per cycle
    return max(3.61, 0.30 * k - 0.05) + 0.02


CURVES = {
    "measured-fp64": mi355x_fp64,
    "hbm-flat-then-linear": lambda k: max(1.0, 0.12 * k),
    "pure-linear": lambda k: 0.2 * k + 0.05,
    "launch-bound": lambda k: 0.05 + 0.004 * k,
}


@pytest.mark.parametrize("curve", sorted(CURVES))
@pytest.mark.parametrize("n,kmax", [(20, 24), (480, 24), (37, 16), (7, 24), (1, 24), (100, 14), (25000, 24)])
def test_schedule_optimal(native, curve, n, kmax):
    t = CURVES[curve]
    s = schedule(n, kmax, t)
    assert sum(s) == n and max(s) <= kmax and max(s) - min(s) <= 1
    cost = sum(t(k) for k in s)
    if n <= 30000:
        assert cost <= brute(n, kmax, t) * (1 + 1e-9)


def test_schedule_examples(native):
    assert schedule(20, 24, mi355x_fp64) == [20]  # one pass beats 2 x 10 (profiles/depth_schedule.md)
    assert schedule(20, 14, mi355x_fp64) == [10, 10]
    s = schedule(480, 24, mi355x_fp64)
    assert set(s) <= {13, 14, 15, 16} and sum(s) == 480


def test_schedule_missing_depth(native):
    """A depth without a tuned time (t < 0, e.g. a slab too thin to split) aborts the search."""
    assert schedule(20, 24, lambda k: -1.0 if k == 20 else 1.0) == []


def schedules_near(n, kmax, t, tol, m):
    tm = (C.c_double * (kmax + 1))(*([0.0] + [t(k) for k in range(1, kmax + 1)]))
    out = (C.c_int32 * (m * n))()
    lens = (C.c_int64 * m)()
    cnt = C.c_int32()
    N.call("heat2d_cycle_schedule_near", n, kmax, tm, tol, m, out, m * n, lens, C.byref(cnt))
    res, pos = [], 0
    for i in range(cnt.value):
        res.append([int(v) for v in out[pos:pos + lens[i]]])
        pos += lens[i]
    return res


@pytest.mark.parametrize("curve", sorted(CURVES))
@pytest.mark.parametrize("n,kmax", [(20, 24), (1000, 16), (1000, 24), (480, 24), (37, 5)])
def test_schedule_near_candidates(native, curve, n, kmax):
    """prepare()'s graph-timed choice among near-tied schedules starts from
    cycle_schedule_near: the best estimate first (= cycle_schedule), then other
    balanced cycle counts within tol of it, at most m."""
    t = CURVES[curve]
    cost = lambda s: sum(t(k) for k in s)
    near = schedules_near(n, kmax, t, 0.03, 3)
    assert 1 <= len(near) <= 3
    assert near[0] == schedule(n, kmax, t)
    for s in near:
        assert sum(s) == n and max(s) <= kmax and max(s) - min(s) <= 1
        assert cost(s) <= cost(near[0]) * 1.03 + 1e-12
    assert len({min(s) for s in near}) == len(near)  # one candidate per base depth
    assert schedules_near(n, kmax, t, 0.0, 3)[0] == near[0]


def shallower(n, kmax, t, best, lo):
    tm = (C.c_double * (kmax + 1))(*([0.0] + [t(k) for k in range(1, kmax + 1)]))
    b = (C.c_int32 * len(best))(*best)
    out = (C.c_int32 * max(1, n))()
    ln = C.c_int64()
    N.call("heat2d_cycle_schedule_shallower", n, kmax, tm, b, len(best), sum(t(k) for k in best), lo, out, n,
           C.byref(ln))
    return [int(v) for v in out[:ln.value]]


def cliff16(k):
    """16384^2 fp64 tuned cycle ms (profiles/r4/gh, r4/gi): an occupancy cliff
    makes depth 16 far cheaper per step than 17..20."""
    return {15: 0.905, 16: 0.940, 17: 1.136, 18: 1.170, 19: 1.237, 20: 1.310}.get(k, 1.5 + 0.05 * k)


def test_schedule_shallower_finds_cliff(native):
    """The prescan's candidates (bases 17..20 or 18..24, the best 26 x 18/19)
    missed depth 16: walking shallower on tuned times finds 30 x 16 (28.2 ms)
    and stops after two bases in a row that do not beat it (15, 14). From base
    18 the first step (17: 27 cycles, 31.4 ms) is no cheaper, the next is."""
    best = [19] * 12 + [18] * 14  # 26 cycles of 18/19 (the candidates' best)
    assert shallower(480, 24, cliff16, best, lo=17) == [16] * 30
    assert shallower(480, 24, cliff16, best, lo=18) == [16] * 30
    # a cost that only rises toward shallow depths keeps the candidates' choice
    assert shallower(480, 24, lambda k: 1.0 + 0.01 * k, best, lo=18) == best


def test_schedule_shallower_short_runs_untouched(native):
    """Runs of few cycles (the headline's 20 steps) never pay for tuning more depths."""
    assert shallower(20, 24, cliff16, [20], lo=10) == [20]
    assert shallower(64, 24, lambda k: 0.1 * k, [22, 21, 21], lo=21) == [22, 21, 21]


@pytest.mark.parametrize("curve", sorted(CURVES))
def test_schedule_shallower_never_worse(native, curve):
    t = CURVES[curve]
    best = schedule(480, 24, t)
    got = shallower(480, 24, t, best, lo=min(best))
    assert sum(got) == 480 and sum(t(k) for k in got) <= sum(t(k) for k in best) * (1 + 1e-12)


def deeper(n, kmax, t, best, hi):
    tm = (C.c_double * (kmax + 1))(*([0.0] + [t(k) for k in range(1, kmax + 1)]))
    b = (C.c_int32 * len(best))(*best)
    out = (C.c_int32 * max(1, n))()
    ln = C.c_int64()
    N.call("heat2d_cycle_schedule_deeper", n, kmax, tm, b, len(best), sum(t(k) for k in best), hi, out, n,
           C.byref(ln))
    return [int(v) for v in out[:ln.value]]


def hbm_bound(k):
    """fp32 32768^2-like: a pass costs about the same at any depth (HBM-bound),
    so the deepest cut is cheapest."""
    return 2.0 + 0.01 * k


def test_schedule_deeper_walks_to_kmax(native):
    """Candidates that stopped at base 20 (25 cycles of 19/20) walk up to 20 x 24."""
    best = [20] * 5 + [19] * 20
    assert deeper(480, 24, hbm_bound, best, hi=19) == [24] * 20
    assert deeper(480, 22, hbm_bound, best, hi=19)[0] <= 22  # never past kmax
    # a per-step cost that rises with depth (VALU-bound) keeps the candidates' choice
    assert deeper(480, 24, lambda k: 0.3 * k + 0.01 * k * k, best, hi=19) == best


def test_schedule_deeper_short_runs_untouched(native):
    assert deeper(20, 24, hbm_bound, [10, 10], hi=10) == [10, 10]  # 1 cycle < 8: no extra tuning
    assert deeper(64, 24, hbm_bound, [16] * 4, hi=16) == [16] * 4


@pytest.mark.parametrize("curve", sorted(CURVES))
def test_schedule_deeper_never_worse(native, curve):
    t = CURVES[curve]
    best = [16] * 30
    got = deeper(480, 24, t, best, hi=16)
    assert sum(got) == 480 and max(got) <= 24 and sum(t(k) for k in got) <= sum(t(k) for k in best) * (1 + 1e-12)
