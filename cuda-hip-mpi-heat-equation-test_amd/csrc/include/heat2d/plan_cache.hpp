// Persistent cache of autotuned launch plans and measured cycle schedules.
//
// Solver::prepare() tunes every depth a run uses (autotune_split: ~30 timed
// trial cycles per depth) and searches the cycle schedule from those
// measurements: 6 s of a 10 s 20-step bench at 32768^2 fp64, 54 s at the
// 240 GB grid, redone by every process of every run. The cache keeps the
// winners on disk, keyed by everything the measurement depended on — GPU
// architecture and CU count, dtype, arithmetic, the slab's rows / columns /
// pitch / position in the domain, the depth and band, the compute stream's CU
// budget, the exchange kind, the transport name, a hash of
// the plan-shaping HEAT2D_* environment knobs, and the build (a hash of the
// kernel and runtime sources, HEAT2D_BUILD_ID; a build without one, "dev",
// disables the cache) — and a hit is checked semantically (a plan kind this
// run may not use is refused) and re-validated by ONE short re-time of the
// cached plan (a drift of more than 10 % re-tunes).
//
// File: $HEAT2D_PLAN_CACHE (path; "off" disables), default
// $XDG_CACHE_HOME/heat2d/plans-v4.txt or ~/.cache/heat2d/plans-v4.txt. One
// "key<TAB>value" line per entry, appended (O_APPEND: concurrent rank
// processes add whole lines); the last line of a key wins.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "heat2d/kernels.hpp"

namespace heat2d {
namespace plancache {

bool enabled();
std::string path();
// Build identity compiled into the library (hash of the sources).
const char* build_id();

bool get_plan(const std::string& ctx, int k, int64_t band, kern::SplitPlan* plan, float* ms);
void put_plan(const std::string& ctx, int k, int64_t band, const kern::SplitPlan& plan, float ms);
bool get_schedule(const std::string& ctx, int64_t n, std::vector<int>* sched);
void put_schedule(const std::string& ctx, int64_t n, const std::vector<int>& sched);
// Forget the in-memory copy (tests switch $HEAT2D_PLAN_CACHE between runs).
void reset();

}  // namespace plancache
}  // namespace heat2d
