# Round 4, run W: spin-polling synchronisation for single-rank runs
# (HEAT2D_SYNC_SPIN=0: hipStreamSynchronize, the old path), interleaved A/B on
# the headline and the small grid; then the weak-scaling slab with fp32 depths.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
O=gpurun_out/r4w
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b20_spin_$i.json 2> $O/b20_spin_$i.err || exit 1
  HEAT2D_SYNC_SPIN=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b20_block_$i.json 2> $O/b20_block_$i.err || exit 1
done
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 100 > $O/small_spin_$i.json 2> $O/small_spin_$i.err || exit 1
  HEAT2D_SYNC_SPIN=0 timeout -k 10 200 python -u bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 100 > $O/small_block_$i.json 2> $O/small_block_$i.err || exit 1
done
python tools/summarize_json.py $O/*.json
timeout -k 10 600 python -u bench.py --dtype fp32 --rehearse-comm --n 489477 --rows 61185 --steps 64 --warmup 16 > $O/weak8_slab.json 2> $O/weak8_slab.err || exit 1
timeout -k 10 600 python -u bench.py --dtype fp32 --rehearse-comm --n 489477 --rows 61185 --steps 64 --warmup 16 --tb 20 > $O/weak8_slab_tb20.json 2> $O/weak8_slab_tb20.err || exit 1
python tools/summarize_json.py $O/weak8*.json
