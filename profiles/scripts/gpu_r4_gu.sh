# Round 4, run GU: hipGraphUpload of the measured-schedule graph at capture
# (prepare) vs its first (timed) launch uploading it (HEAT2D_GRAPH_UPLOAD=0),
# interleaved, small grid and headline.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
O=gpurun_out/r4gu
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 100 > $O/small_up_$i.json 2> $O/small_up_$i.err || exit 1
  HEAT2D_GRAPH_UPLOAD=0 timeout -k 10 200 python -u bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 100 > $O/small_noup_$i.json 2> $O/small_noup_$i.err || exit 1
done
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b20_up_$i.json 2> $O/b20_up_$i.err || exit 1
  HEAT2D_GRAPH_UPLOAD=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b20_noup_$i.json 2> $O/b20_noup_$i.err || exit 1
done
python tools/summarize_json.py $O/*.json
