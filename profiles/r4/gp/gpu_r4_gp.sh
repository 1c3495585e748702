# Round 4, run GP: shallower walk with patience 2 + eager near-tie scan:
# 16384^2 fp64 (the cliff at depth 16) x2, 32768^2 fp64 / fp32 480 steps
# (prepare cost), small grid, headline; schedule GPU tests first.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off HEAT2D_TUNE_LOG=1
O=gpurun_out/r4gp
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_solver.py -m gpu -x -q -k "schedule" --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > $O/$name.json 2> $O/$name.err
}
run f64_16k_1 --grid 16384 --steps 480 --warmup 20 || exit 1
run f64_16k_2 --grid 16384 --steps 480 --warmup 20 || exit 1
run f64_32k_480 --steps 480 --warmup 20 || exit 1
run f32_32k_480 --dtype fp32 --steps 480 --warmup 20 || exit 1
run small --grid 4096 --dtype fp32 --steps 1000 --warmup 100 || exit 1
run b20 --steps 20 --warmup 5 || exit 1
python tools/summarize_json.py $O/*.json
grep -h "heat2d sched n=480 \(candidate\|walk\|eager\)" $O/*.err > $O/sched_log.txt || true
