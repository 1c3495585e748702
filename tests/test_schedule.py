"""The measured-schedule search of Solver::prepare (csrc/runtime/schedule.cpp),
on CPU with synthetic cycle-time curves:

* dp_schedule — the exact least-cost cut of n steps into cycles of at most
  kmax steps (checked against brute force over all compositions, and against
  every balanced split);
* near_schedules — one balanced candidate per base depth within a tolerance;
* search_schedule — prescan (default plans) -> tune the near-best depths ->
  DP over tuned costs -> walks past the tuned range on long runs, with the
  measurements as callbacks: the known cases of the hardware (the 16384^2 fp64
  occupancy cliff at depth 16, the HBM-bound fp32 grid that wants kmax, the
  one-pass headline) and what it measures on the way.
"""
import ctypes as C

import pytest

from heat2d.ops import _native as N


def _costs(kmax, t):
    return (C.c_double * (kmax + 1))(*([0.0] + [float(t(k)) for k in range(1, kmax + 1)]))


def dp(n, kmax, t):
    out = (C.c_int32 * max(1, n))()
    ln, tot = C.c_int64(), C.c_double()
    N.call("heat2d_dp_schedule", n, kmax, _costs(kmax, t), out, n, C.byref(ln), C.byref(tot))
    return [int(v) for v in out[:ln.value]], tot.value


def near(n, kmax, t, tol, m):
    out = (C.c_int32 * (m * n + 1))()
    lens = (C.c_int64 * (m + 1))()
    costs = (C.c_double * (m + 1))()
    cnt = C.c_int32()
    N.call("heat2d_near_schedules", n, kmax, _costs(kmax, t), tol, m, out, m * n, lens, costs, C.byref(cnt))
    res, pos = [], 0
    for i in range(cnt.value):
        res.append((costs[i], [int(v) for v in out[pos:pos + lens[i]]]))
        pos += lens[i]
    return res


def search(n, kmax, pre, tuned):
    out = (C.c_int32 * max(1, n))()
    ln, cost = C.c_int64(), C.c_double()
    ps, ts = (C.c_int32 * (kmax + 1))(), (C.c_int32 * (kmax + 1))()
    nps, nts = C.c_int32(), C.c_int32()
    N.call("heat2d_search_schedule", n, kmax, _costs(kmax, pre), _costs(kmax, tuned), out, n, C.byref(ln),
           C.byref(cost), ps, C.byref(nps), ts, C.byref(nts))
    return ([int(v) for v in out[:ln.value]], cost.value, [int(v) for v in ps[:nps.value]],
            [int(v) for v in ts[:nts.value]])


def brute(n, kmax, t):
    """Cheapest cut of n steps into cycles of <= kmax steps over ALL compositions."""
    best = [0.0] + [float("inf")] * n
    for m in range(1, n + 1):
        best[m] = min(t(k) + best[m - k] for k in range(1, min(kmax, m) + 1))
    return best[n]


def mi355x_fp64(k):  # measured shape at 32768^2 fp64 (profiles/depth_schedule.md): ms per cycle
    return max(3.61, 0.30 * k - 0.05) + 0.02


def cliff16(k):
    """16384^2 fp64 TUNED cycle ms (profiles/r4/gh, r4/gi): an occupancy cliff
    makes depth 16 far cheaper per step than 17..20."""
    return {15: 0.905, 16: 0.940, 17: 1.136, 18: 1.170, 19: 1.237, 20: 1.310}.get(k, 1.5 + 0.05 * k)


def cliff16_default(k):
    """... and its DEFAULT plans (what the prescan sees): depth 16's default
    plan is no better than its neighbours', so the prescan ranks 17..20 first."""
    return {14: 1.40, 15: 1.42, 16: 1.38, 17: 1.25, 18: 1.29, 19: 1.36, 20: 1.47}.get(k, 2.0 + 0.05 * k)


def hbm_bound(k):
    """fp32 32768^2-like: a pass costs about the same at any depth (HBM-bound)."""
    return 2.0 + 0.01 * k


CURVES = {
    "measured-fp64": mi355x_fp64,
    "hbm-flat-then-linear": lambda k: max(1.0, 0.12 * k),
    "pure-linear": lambda k: 0.2 * k + 0.05,
    "launch-bound": lambda k: 0.05 + 0.004 * k,
    "cliff16": cliff16,
    "hbm-bound": hbm_bound,
    "bumpy": lambda k: 1.0 + 0.07 * k + (0.3 if k % 3 == 0 else 0.0),
}


@pytest.mark.parametrize("curve", sorted(CURVES))
@pytest.mark.parametrize("n,kmax", [(20, 24), (480, 24), (37, 16), (7, 24), (1, 24), (100, 14), (1000, 20)])
def test_dp_is_optimal(native, curve, n, kmax):
    t = CURVES[curve]
    s, tot = dp(n, kmax, t)
    assert sum(s) == n and max(s) <= kmax and s == sorted(s, reverse=True)
    assert tot == pytest.approx(sum(t(k) for k in s), rel=1e-12)
    assert tot <= brute(n, kmax, t) * (1 + 1e-12)
    # never worse than any balanced split
    for c in range(-(-n // kmax), n + 1):
        b, rem = n // c, n % c
        assert tot <= (c - rem) * t(b) + rem * (t(b + 1) if rem else 0) + 1e-9


def test_dp_large_n_and_unusable_depths(native):
    s, tot = dp(25000, 24, mi355x_fp64)  # the reference's literal 25000-step run
    assert sum(s) == 25000 and tot > 0
    # depths with a negative cost are never used; an unreachable n gives nothing
    s, _ = dp(40, 24, lambda k: 1.0 if k in (8, 12) else -1.0)
    assert sum(s) == 40 and set(s) <= {8, 12}
    assert dp(7, 24, lambda k: 1.0 if k in (4,) else -1.0) == ([], -1.0)


@pytest.mark.parametrize("curve", ["measured-fp64", "cliff16", "bumpy", "pure-linear", "hbm-bound"])
@pytest.mark.parametrize("n", [20011, 31000])
def test_dp_long_runs_stay_exact(native, curve, n):
    """Above K * K * k* steps the DP takes the surplus as cycles of the
    cheapest depth per step (some optimal schedule does) and solves only the
    rest exactly: the same least cost as the full DP."""
    t = CURVES[curve]
    s, tot = dp(n, 24, t)
    assert sum(s) == n and s == sorted(s, reverse=True)
    assert tot == pytest.approx(brute(n, 24, t), rel=1e-12)


def test_dp_ten_million_steps_is_cheap(native):
    import time
    t0 = time.perf_counter()
    s, tot = dp(10_000_000, 24, cliff16)
    assert time.perf_counter() - t0 < 2.0
    assert sum(s) == 10_000_000 and s.count(16) > 600_000 and tot > 0


def test_dp_ties_fewer_cycles_deeper_first(native):
    s, _ = dp(20, 24, lambda k: 1.0)  # every cycle costs the same: one cycle
    assert s == [20]
    s, _ = dp(30, 16, lambda k: 1.0 + 0.0 * k)
    assert s == [16, 14]


def test_dp_mixes_depths_around_a_cliff(native):
    """Balanced splits miss what the exact DP sees: 500 steps with the cheap
    depth 16 and an expensive 17+ -> mostly 16s plus a 20 where 500 % 16 != 0."""
    s, tot = dp(500, 24, cliff16)
    assert sum(s) == 500 and s.count(16) >= 28
    assert tot <= brute(500, 24, cliff16) * (1 + 1e-12)


def test_near_candidates(native):
    cand = near(480, 24, mi355x_fp64, 0.05, 4)
    assert 1 <= len(cand) <= 4
    costs = [c for c, _ in cand]
    assert costs == sorted(costs) and costs[-1] <= costs[0] * 1.05
    bases = [min(s) for _, s in cand]
    assert len(set(bases)) == len(bases)  # one per base depth
    for c, s in cand:
        assert sum(s) == 480 and max(s) - min(s) <= 1 and c == pytest.approx(sum(mi355x_fp64(k) for k in s))


def test_search_headline_one_pass(native):
    """20 steps (the driver's headline): one depth-20 pass, only a handful of
    depths prescanned and one or two tuned (prepare() stays ~2 s)."""
    s, cost, pre, tun = search(20, 24, mi355x_fp64, lambda k: 0.97 * mi355x_fp64(k))
    assert s == [20]
    assert pre[0] == 20 and len(pre) <= 12
    assert 20 in tun and len(tun) <= 3


def test_search_finds_the_cliff(native):
    """16384^2 fp64 480 steps: the prescan (default plans) ranks 17..20, their
    tuned costs are tuned, and the downward walk from the lowest tuned depth
    finds 16 (30 x 16, 28.2 ms) — round 4's 19/20 schedule ran 4055 Gpts/s,
    30 x 16 4550 (profiles/r4/gh, r4/gi)."""
    s, cost, pre, tun = search(480, 24, cliff16_default, cliff16)
    assert s == [16] * 30 and cost == pytest.approx(30 * 0.94)
    assert 16 in tun and 17 in tun
    assert len(tun) <= 9


def test_search_fills_gaps_next_to_the_best(native):
    """The prescan of profiles/r5/g (16384^2 fp64, 480 steps) put depth 16's
    default plan behind 15's and 14's: the tuned depths became 12..15 and
    18..20, the walks (below 12, above 20) never reach 16, and the DP took
    32 x 15 (29.9 ms, 4314 Gpts/s). The neighbours of the best's depths are
    tuned too: 16 joins and wins (30 x 16)."""
    pre = {24: 1.7821, 23: 1.6835, 22: 1.8589, 21: 1.7732, 20: 1.4719, 19: 1.3863, 18: 1.3331, 17: 1.2580,
           16: 1.3059, 15: 1.2669, 14: 1.0108, 13: 1.2365}
    tuned = {20: 1.3236, 19: 1.2327, 18: 1.1801, 17: 1.136, 16: 0.940, 15: 0.9351, 14: 1.0108, 13: 0.9987,
             12: 0.8982, 11: 0.85, 10: 0.80}
    s, cost, _, tun = search(480, 24, lambda k: pre.get(k, 2.0 + 0.05 * k), lambda k: tuned.get(k, 1.5))
    assert s == [16] * 30 and cost == pytest.approx(28.2)
    assert 16 in tun and 17 in tun and len(tun) <= 11


def test_search_prescans_until_n_is_reachable(native):
    """A flat cycle cost stops the prescan at depth 19 (per step 25 % worse
    than depth 24's), and no schedule of exactly 25 steps uses only depths
    19..24: the prescan goes on until one exists (round 5: 8 ranks of 525
    rows, 25-step chunks, ran the balanced fallback)."""
    s, cost, pre, tun = search(25, 24, lambda k: 1.0, lambda k: 1.0)
    assert sum(s) == 25 and len(s) == 2 and cost == pytest.approx(2.0)
    assert min(pre) <= 12 and len(pre) <= 13


def test_search_walks_past_near_misses(native):
    """profiles/r5/i (priming skip in the fp64 interior, 16384^2, 480 steps):
    the prescan ranked depths 20..24 first and depth 20 won the DP; the walk
    down met 19 and 18, each a little worse per step than 20 — two misses, so
    it stopped and 24 x 20 ran (4336 Gpts/s) instead of 30 x 16 (4797). Depths
    within walk_tol (8 %) per step of the best are not misses: the walk goes on
    through 17 to 16."""
    pre = {24: 1.45, 23: 1.40, 22: 1.36, 21: 1.30, 20: 1.25, 19: 1.30, 18: 1.28, 17: 1.26, 16: 1.40, 15: 1.30}
    tuned = {24: 1.508, 23: 1.480, 22: 1.5015, 21: 1.33, 20: 1.2296, 19: 1.19, 18: 1.15, 17: 1.1158, 16: 0.8977,
             15: 0.9246, 14: 0.9662, 13: 0.9605}
    s, cost, _, tun = search(480, 24, lambda k: pre.get(k, 2.0 + 0.05 * k), lambda k: tuned.get(k, 1.5))
    assert s == [16] * 30 and cost == pytest.approx(30 * 0.8977)
    assert 16 in tun and len(tun) <= 12


def test_search_walks_up_when_the_deepest_wins(native):
    """HBM-bound fp32: the deepest tuned depth wins, so the walk goes up to kmax."""
    s, cost, pre, tun = search(480, 24, lambda k: 1.05 * hbm_bound(k), hbm_bound)
    assert s == [24] * 20


def test_search_short_runs_do_not_walk(native):
    s, cost, pre, tun = search(40, 24, cliff16_default, cliff16)
    assert sum(s) == 40
    assert all(40 // k >= 1 for k in tun) and len(tun) <= 5


@pytest.mark.parametrize("curve", sorted(CURVES))
@pytest.mark.parametrize("n", [20, 64, 480, 1000])
def test_search_matches_dp_over_what_it_tuned(native, curve, n):
    """Whatever it measured, the result is the exact optimum over the tuned
    costs (and no worse than the DP over the default plans it prescanned)."""
    t = CURVES[curve]
    s, cost, pre, tun = search(n, 24, lambda k: 1.1 * t(k), t)
    assert sum(s) == n and set(s) <= set(tun)
    best_over_tuned, _ = dp(n, 24, lambda k: t(k) if k in tun else -1.0)
    assert cost == pytest.approx(sum(t(k) for k in best_over_tuned), rel=1e-12)
    assert len(set(pre)) == len(pre) and len(set(tun)) == len(tun)  # each measured once
