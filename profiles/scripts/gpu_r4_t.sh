# Round 4, run T: same-box A/B of the fp32 depths 21..24 (default: max depth
# 24) against the old limit (--tb 20) on the HBM-bound fp32 grids.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
O=gpurun_out/r4t
mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --dtype fp32 --grid 173056 --steps 64 --warmup 16 > $O/max_new_$i.json 2> $O/max_new_$i.err || exit 1
  timeout -k 10 300 python -u bench.py --dtype fp32 --grid 173056 --steps 64 --warmup 16 --tb 20 > $O/max_tb20_$i.json 2> $O/max_tb20_$i.err || exit 1
  timeout -k 10 300 python -u bench.py --dtype fp32 --steps 480 --warmup 20 > $O/b32_new_$i.json 2> $O/b32_new_$i.err || exit 1
  timeout -k 10 300 python -u bench.py --dtype fp32 --steps 480 --warmup 20 --tb 20 > $O/b32_tb20_$i.json 2> $O/b32_tb20_$i.err || exit 1
done
python tools/summarize_json.py $O/*.json
