# Round 4, run V: the 8-rank weak-scaled 240 GB-per-GPU fp32 slab (BASELINE
# config 5, one rank rehearsed with the RCCL self-exchange) with the fp32
# depths 21..24, against --tb 20 on the same box.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
O=gpurun_out/r4v
mkdir -p $O
timeout -k 10 600 python -u bench.py --dtype fp32 --rehearse-comm --n 489477 --rows 61185 --steps 64 --warmup 16 > $O/weak8_slab.json 2> $O/weak8_slab.err || exit 1
timeout -k 10 600 python -u bench.py --dtype fp32 --rehearse-comm --n 489477 --rows 61185 --steps 64 --warmup 16 --tb 20 > $O/weak8_slab_tb20.json 2> $O/weak8_slab_tb20.err || exit 1
python tools/summarize_json.py $O/*.json
