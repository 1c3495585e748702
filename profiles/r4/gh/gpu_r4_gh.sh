# Round 4, run GH: why the eager 16384^2 fp64 480-step run picks 19/20-deep
# cycles (4055-4105 Gpts/s) when 30 x depth 16 ran 4594: schedule-search log
# (prescan default-plan times, candidates, tuned costs), eager, 2 runs each.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off HEAT2D_TUNE_LOG=1
O=gpurun_out/r4gh
mkdir -p $O
for i in 1 2; do
  timeout -k 10 240 python -u bench.py --grid 16384 --steps 480 --warmup 20 > $O/f64_16k_$i.json 2> $O/f64_16k_$i.err || exit 1
done
timeout -k 10 240 python -u bench.py --grid 8192 --steps 480 --warmup 20 > $O/f64_8k.json 2> $O/f64_8k.err || exit 1
timeout -k 10 240 python -u bench.py --steps 480 --warmup 20 > $O/f64_32k.json 2> $O/f64_32k.err || exit 1
python tools/summarize_json.py $O/*.json
grep -h "heat2d sched" $O/*.err > $O/sched_log.txt
