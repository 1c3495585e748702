# Round 4, run Q: every BASELINE.json configuration on the final tree
# (bench/configs.py: CPU 256^2, 4096^2 fp32 with / without graph, 16384^2 fp64,
# 32768^2 fp64 / fp32, the 240 GB fp32 grid, sigma = 0.2 fast / exact), then
# the per-rank slabs of BASELINE configs 4 and 5 rehearsed on one GPU
# (32768^2 fp32 strong-scaled to 8 ranks, 480 steps; the 8-rank weak-scaled
# 240 GB-per-GPU fp32 grid, 64 steps).
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
O=gpurun_out/r4q
mkdir -p $O
timeout -k 10 900 python -u bench/configs.py > $O/configs.jsonl 2> $O/configs.err || exit 1
cat $O/configs.jsonl | python -c "import sys,json; [print(d['config'], d['gpts'], d.get('cycles'), d.get('prepare_s'), d.get('hbm_gb_per_s_plan')) for d in map(json.loads, sys.stdin)]"
timeout -k 10 300 python -u bench.py --dtype fp32 --rehearse-comm --rows 4096 --steps 480 --warmup 20 > $O/reh32_480.json 2> $O/reh32_480.err || exit 1
timeout -k 10 600 python -u bench.py --dtype fp32 --rehearse-comm --n 489477 --rows 61185 --steps 64 --warmup 16 > $O/weak8_slab.json 2> $O/weak8_slab.err || exit 1
python tools/summarize_json.py $O/reh32_480.json $O/weak8_slab.json
