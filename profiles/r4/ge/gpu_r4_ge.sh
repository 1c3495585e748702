# Round 4, run GE: the headline's one-cycle timed step replayed from a graph
# (default for single-rank runs) vs launched eager (--graph off), interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
O=gpurun_out/r4ge
mkdir -p $O
for i in 1 2 3 4; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b20_graph_$i.json 2> $O/b20_graph_$i.err || exit 1
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --graph off > $O/b20_eager_$i.json 2> $O/b20_eager_$i.err || exit 1
done
python tools/summarize_json.py $O/*.json
