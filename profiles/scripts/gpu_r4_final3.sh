# Round 4, final tree (last: synchronize backoff): GPU suite, smoke, headline,
# the small grid x3 (its schedule search now sees fp32 depths up to 24), the
# 240 GB grid.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r4final3
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log || exit 1
export HEAT2D_PLAN_CACHE=off
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || exit 1
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 100 > $O/small_$i.json 2> $O/small_$i.err || exit 1
done
timeout -k 10 400 python -u bench.py --dtype fp32 --grid 173056 --steps 64 --warmup 16 > $O/max.json 2> $O/max.err || exit 1
python tools/summarize_json.py $O/*.json
