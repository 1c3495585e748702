# Round 4, run GJ: per-depth tuned cycles of fp64 16384^2 / 32768^2 for depths
# 14..24 (tools/cycle_probe.py, autotuned plan, hipEvent phase timers:
# interior vs boundary-band launch) — where the per-level cost jumps from
# depth 16 to 17 (16384^2: 58.8 -> 66.8 us per level, runs GH / GI).
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off CP_AUTOTUNE=1 CP_TIMERS=1
O=gpurun_out/r4gj
mkdir -p $O
for n in 16384 32768; do
  for k in 14 15 16 17 18 20 21 24; do
    timeout -k 10 120 python -u tools/cycle_probe.py fp64 $n $k 6 >> $O/probe.jsonl 2>> $O/probe.err || exit 1
  done
done
