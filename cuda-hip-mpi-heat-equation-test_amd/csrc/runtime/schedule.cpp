// Cycle schedules: how n time steps are cut into HBM passes (cycles of depth
// k <= kmax, temporal blocking), from measured per-depth cycle times.
//
// The reference has no such choice — one full-field pass per step
// (fortran/hip/heat.F90:240-250). Here a cycle of depth k costs t(k): flat while
// the pass is HBM-bound, then rising with k once it is VALU-bound, with steps
// at occupancy boundaries (the fp64 general kernel drops from 2 to 1 wave per
// SIMD at K = 17, the chained march starts at 17, profiles/r4/gk/) — so no
// smooth model of t(k) picks the depths; measurements do:
//
//   1. prescan  — the DEFAULT plan of depths kmax, kmax-1, ... (a few trial
//                 cycles each), until the per-step cost is `stop_ratio` worse
//                 than the best seen;
//   2. tune     — every depth of the near-best prescan schedules (one per base
//                 depth, within prescan_tol, at most prescan_bases of them);
//   3. DP       — the exact schedule of n steps minimising the sum of the best
//                 known cycle times (tuned, else prescan); a depth it picks that
//                 is not tuned yet is tuned and the DP re-run, until its choice
//                 is all tuned;
//   4. walks    — runs of >= walk_min_cycles cycles also tune the depths below
//                 the lowest tuned one (and above the highest, when the best
//                 uses it), one at a time, until walk_patience in a row do not
//                 lower the DP cost and cost more than walk_tol per step above
//                 the best (a default plan far worse than its tuned
//                 plan hides such a depth from the prescan: 16384^2 fp64 480
//                 steps, depth 16 tuned 0.94 ms vs 17..20 at 1.14-1.31);
//   5. near     — the tuned-cost schedules within near_tol of the best (one per
//                 base depth) for the caller to time as step(n) would run them.
//
// Pure functions of the two measuring callbacks, so the search is unit-tested
// on CPU with synthetic cost curves (tests/test_schedule.py); the solver passes
// collective (max-over-ranks) measurements, so every rank searches alike.
#include <algorithm>
#include <cmath>
#include <limits>

#include "heat2d/runtime.hpp"

namespace heat2d {

namespace {

// The exact DP over m steps: best[m'] for every m' <= m (costs c[1..K], < 0 = unusable).
std::vector<int> dp_exact(int64_t n, int K, const std::vector<double>& c, double* total) {
  const double inf = std::numeric_limits<double>::infinity();
  // best[m]: least cost of exactly m steps; cyc[m]: its cycle count; take[m]: its first (deepest) depth
  std::vector<double> best((size_t)n + 1, inf);
  std::vector<int64_t> cyc((size_t)n + 1, 0);
  std::vector<int> take((size_t)n + 1, 0);
  best[0] = 0.0;
  for (int64_t m = 1; m <= n; ++m) {
    for (int k = 1; k <= std::min<int64_t>(K, m); ++k) {
      const double ck = c[(size_t)k];
      const double prev = best[(size_t)(m - k)];
      if (ck < 0 || prev == inf) continue;
      const double v = prev + ck;
      const double cur = best[(size_t)m];
      // ties (1e-12 relative): fewer cycles, then the deeper cycle first
      const bool tie = cur < inf && std::fabs(v - cur) <= 1e-12 * std::max(v, cur);
      if ((!tie && v < cur) ||
          (tie && (cyc[(size_t)(m - k)] + 1 < cyc[(size_t)m] ||
                   (cyc[(size_t)(m - k)] + 1 == cyc[(size_t)m] && k > take[(size_t)m])))) {
        best[(size_t)m] = v;
        cyc[(size_t)m] = cyc[(size_t)(m - k)] + 1;
        take[(size_t)m] = k;
      }
    }
  }
  if (total) *total = best[(size_t)n] == inf ? -1.0 : best[(size_t)n];
  if (best[(size_t)n] == inf) return {};
  std::vector<int> s;
  for (int64_t m = n; m > 0; m -= take[(size_t)m]) s.push_back(take[(size_t)m]);
  return s;
}

}  // namespace

std::vector<int> dp_schedule(int64_t n, int kmax, const std::function<double(int)>& cost, double* total) {
  HEAT2D_REQUIRE(n >= 1 && kmax >= 1, "dp_schedule needs n >= 1, kmax >= 1");
  const int K = (int)std::min<int64_t>(kmax, n);
  std::vector<double> c((size_t)K + 1, -1.0);
  for (int k = 1; k <= K; ++k) c[(size_t)k] = cost(k);
  // Long runs (the CLI prepares ntime = 25 000 steps; 10^7 would be 200 MB and
  // 2.4e8 inner steps per call, and the search calls the DP dozens of times):
  // with k* the cheapest depth per step, some optimal schedule repeats every
  // other depth fewer than k* times (k* cycles of depth k cost at least k
  // cycles of depth k*, same steps), so its other cycles sum to under
  // K * K * k* steps. The steps above that bound are k* cycles in some optimal
  // schedule: they are taken as such and only the rest goes through the DP —
  // the same least cost, in O(K^3 k*) time and memory whatever n.
  int ks = 0;
  for (int k = 1; k <= K; ++k) {
    if (c[(size_t)k] < 0) continue;
    const double per = c[(size_t)k] / k;
    const double bper = ks ? c[(size_t)ks] / ks : 0.0;
    if (ks == 0 || per < bper * (1.0 - 1e-12) || (per <= bper * (1.0 + 1e-12) && k > ks)) ks = k;
  }
  const int64_t cap = (int64_t)K * K * std::max(ks, 1);
  std::vector<int> s;
  if (ks > 0 && n > cap) {
    const int64_t j = (n - cap + ks - 1) / ks;
    double rest = 0.0;
    s = dp_exact(n - j * ks, K, c, &rest);
    if (!s.empty() || n - j * ks == 0) {
      s.insert(s.end(), (size_t)j, ks);
      if (total) *total = rest + (double)j * c[(size_t)ks];
    } else {
      s = dp_exact(n, K, c, total);  // (no schedule of the rest over the known depths: the whole DP)
    }
  } else {
    s = dp_exact(n, K, c, total);
  }
  std::sort(s.begin(), s.end(), std::greater<int>());
  return s;
}

std::vector<std::pair<double, std::vector<int>>> near_schedules(int64_t n, int kmax, const std::function<double(int)>& cost,
                                                                 double tol, int m) {
  HEAT2D_REQUIRE(n >= 1 && kmax >= 1, "near_schedules needs n >= 1, kmax >= 1");
  const int K = (int)std::min<int64_t>(kmax, n);
  std::vector<double> c((size_t)K + 2, -1.0);
  for (int k = 1; k <= K; ++k) c[(size_t)k] = cost(k);
  // one candidate per base depth b: the balanced schedule (depths b and b + 1)
  // of the cycle count with the least cost among those whose base is b
  std::vector<std::pair<double, std::vector<int>>> out;
  for (int b = K; b >= 1; --b) {
    double bc = -1.0;
    int64_t bn = 0;
    for (int64_t cy = n / (b + 1) + 1; cy <= n / b; ++cy) {  // n / cy == b
      const int64_t rem = n % cy;
      if (c[(size_t)b] < 0 || (rem && (b + 1 > K || c[(size_t)b + 1] < 0))) continue;
      const double v = (double)(cy - rem) * c[(size_t)b] + (double)rem * (rem ? c[(size_t)b + 1] : 0.0);
      if (bc < 0 || v < bc) {
        bc = v;
        bn = cy;
      }
    }
    if (bn == 0) continue;
    std::vector<int> s;
    for (int64_t i = 0; i < bn; ++i) s.push_back(i < n % bn ? b + 1 : b);
    out.emplace_back(bc, std::move(s));
  }
  std::stable_sort(out.begin(), out.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
  if (out.empty()) return out;
  const double lim = out.front().first * (1.0 + tol);
  size_t keep = 0;
  while (keep < out.size() && (int)keep < m && out[keep].first <= lim) ++keep;
  out.resize(keep);
  return out;
}

ScheduleSearch search_schedule(int64_t n, int kmax, const std::function<double(int)>& prescan,
                               const std::function<double(int)>& tune, const ScheduleSearchOptions& o) {
  HEAT2D_REQUIRE(n >= 1 && kmax >= 1, "search_schedule needs n >= 1, kmax >= 1");
  const int K = (int)std::min<int64_t>(kmax, n);
  ScheduleSearch r;
  std::vector<double> P((size_t)K + 1, std::nan("")), T((size_t)K + 1, std::nan(""));
  auto pre = [&](int k) {
    if (std::isnan(P[(size_t)k])) {
      P[(size_t)k] = prescan(k);
      r.prescanned.push_back(k);
    }
    return P[(size_t)k];
  };
  auto tun = [&](int k) {
    if (std::isnan(T[(size_t)k])) {
      T[(size_t)k] = tune(k);
      r.tuned.push_back(k);
    }
    return T[(size_t)k];
  };
  auto tuned = [&](int k) { return k >= 1 && k <= K && !std::isnan(T[(size_t)k]); };
  // best known cost: tuned, else prescanned, else unusable
  auto est = [&](int k) {
    if (tuned(k)) return T[(size_t)k];
    return std::isnan(P[(size_t)k]) ? -1.0 : P[(size_t)k];
  };

  // 1. prescan, deepest first, until the per-step cost is stop_ratio worse than the best seen
  double best_step = std::numeric_limits<double>::infinity();
  for (int k = K; k >= 1; --k) {
    const double v = pre(k);
    if (v <= 0) continue;
    best_step = std::min(best_step, v / k);
    if (v / k > o.stop_ratio * best_step) break;
  }
  // ... and on, until some schedule of exactly n steps exists over the known
  // depths (n = 25 with only 19..24 prescanned has none: 8 thin slabs of
  // 525 rows, profiles/r5/k/)
  for (int k = K; k >= 1; --k) {
    double c = -1.0;
    if (!dp_schedule(n, K, est, &c).empty()) break;
    (void)pre(k);
  }
  // 2. tune the depths of the near-best prescan schedules
  for (const auto& c : near_schedules(n, K, [&](int k) { return est(k); }, o.prescan_tol, o.prescan_bases))
    for (int k : c.second) (void)tun(k);
  // 3. + 4. DP over the best known costs; tune what it picks; walks
  // (one depth at a time — the one the DP uses most, then the deeper — and the
  // DP re-run: a tuned depth often makes another pick unnecessary)
  auto settle = [&] {
    for (;;) {
      r.best = dp_schedule(n, K, est, &r.cost);
      int pick = 0;
      int64_t uses = 0;
      for (int k : r.best) {
        if (tuned(k)) continue;
        const int64_t u = std::count(r.best.begin(), r.best.end(), k);
        if (u > uses || (u == uses && k > pick)) {
          uses = u;
          pick = k;
        }
      }
      if (pick == 0) return;
      (void)tun(pick);
    }
  };
  settle();
  if (!r.best.empty() && (int64_t)r.best.size() >= o.walk_min_cycles) {
    auto walk = [&](int from, int dir) {
      int misses = 0;
      for (int k = from + dir; k >= 1 && k <= K && misses < o.walk_patience; k += dir) {
        if (n / k < o.walk_min_cycles) break;  // a base needing fewer cycles: not a long run's depth
        if (tuned(k)) continue;
        const double before = r.cost;
        const double v = tun(k);
        settle();
        // a depth within walk_tol of the best per step does not count as a
        // miss: the walk goes on past near misses to a cliff's far side
        const bool near_best = v > 0 && r.cost > 0 && v / k <= (1.0 + o.walk_tol) * r.cost / (double)n;
        misses = (r.cost >= 0 && r.cost < before * (1.0 - 1e-9)) ? 0 : (near_best ? misses : misses + 1);
      }
    };
    int lo = K, hi = 1;
    for (int k = 1; k <= K; ++k)
      if (tuned(k)) {
        lo = std::min(lo, k);
        hi = std::max(hi, k);
      }
    walk(lo, -1);
    // upward only when the best already runs the deepest tuned depth (each
    // deeper fp64 32768^2 depth costs ~2.5 s of tuning, profiles/r4/gn/)
    if (std::find(r.best.begin(), r.best.end(), hi) != r.best.end()) walk(hi, +1);
    // neighbours: the untuned depths next to the ones the best runs, until all
    // are tuned — the walks leave gaps INSIDE the tuned range (16384^2 fp64:
    // tuned 12..15 and 18..20 around the cliff, 16 never, so 32 x 15 at 29.9 ms
    // instead of 30 x 16 at 28.2, profiles/r5/g/)
    for (bool more = true; more;) {
      more = false;
      std::vector<int> uses(r.best);
      std::sort(uses.begin(), uses.end());
      uses.erase(std::unique(uses.begin(), uses.end()), uses.end());
      for (int k : uses)
        for (int nk : {k - 1, k + 1})
          if (!more && nk >= 1 && nk <= K && !tuned(nk) && n / nk >= o.walk_min_cycles) {
            (void)tun(nk);
            settle();
            more = true;
          }
    }
  }
  // 5. near ties among tuned depths (the caller times them as they would run)
  r.near = near_schedules(n, K, [&](int k) { return tuned(k) ? T[(size_t)k] : -1.0; }, o.near_tol, o.near_max);
  bool have = false;
  for (const auto& c : r.near) have = have || c.second == r.best;
  if (!r.best.empty() && !have) r.near.insert(r.near.begin(), {r.cost, r.best});
  return r;
}

}  // namespace heat2d
