# Round 4, run L: small grid (4096^2 fp32, 1000 steps; BASELINE config 2) with
# the widened near-tie schedule scan: bench.py x3 without the plan cache, then
# bench/configs.py (graph row) with a fresh cache and 3 cached reruns.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r4l
mkdir -p $O
for i in 1 2 3; do
  HEAT2D_PLAN_CACHE=off timeout -k 10 200 python -u bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 100 > $O/small_$i.json 2> $O/small_$i.err || exit 1
done
export HEAT2D_PLAN_CACHE=$GRAFT_REPO_ROOT/$O/plancache
for i in 0 1 2 3; do
  timeout -k 10 200 python -u bench/configs.py --only gpu-4096-fp32-graph gpu-4096-fp32 > $O/cfg_$i.jsonl 2> $O/cfg_$i.err || exit 1
done
python tools/summarize_json.py $O/small_*.json
cat $O/cfg_*.jsonl | python -c "import sys,json; [print(d['config'], d['gpts'], d['cycles'], d['prepare_s'], {k: v['origin'] for k, v in d['launch_plans'].items()}) for d in map(json.loads, sys.stdin)]"
