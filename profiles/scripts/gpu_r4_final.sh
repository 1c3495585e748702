# Round 4, final tree: the round-end driver's tiers — GPU suite, smoke, the
# 1-GPU headline — plus the small grid and the slab rehearsal once more.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r4final
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log || exit 1
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || exit 1
export HEAT2D_PLAN_CACHE=off
timeout -k 10 200 python -u bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 100 > $O/small.json 2> $O/small.err || exit 1
timeout -k 10 200 python -u bench.py --rehearse-comm --rows 4096 --steps 20 --warmup 5 > $O/reh64.json 2> $O/reh64.err || exit 1
python tools/summarize_json.py $O/*.json
