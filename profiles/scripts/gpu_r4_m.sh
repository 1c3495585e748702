# Round 4, run M: small grid after dropping gc.collect() before the timed
# region; comm-stream priority A/B; headline.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
O=gpurun_out/r4m
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 100 > $O/small_$i.json 2> $O/small_$i.err || exit 1
  HEAT2D_COMM_PRIORITY=0 timeout -k 10 200 python -u bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 100 > $O/small_np_$i.json 2> $O/small_np_$i.err || exit 1
done
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench20_$i.json 2> $O/bench20_$i.err || exit 1
done
python tools/summarize_json.py $O/*.json
