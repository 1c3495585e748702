# Round 4, last tree (schedule walk patience, eager near-tie scan): whole GPU suite, smoke, headline x2, 32768^2 fp64 / fp32
# 480 steps (prepare time with the gated deeper walk), small grid.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r4final6
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log || exit 1
export HEAT2D_PLAN_CACHE=off
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > $O/$name.json 2> $O/$name.err
}
run bench20_1 --steps 20 --warmup 5 || exit 1
run bench20_2 --steps 20 --warmup 5 || exit 1
run f64_32k_480 --steps 480 --warmup 20 || exit 1
run f32_32k_480 --dtype fp32 --steps 480 --warmup 20 || exit 1
run small --grid 4096 --dtype fp32 --steps 1000 --warmup 100 || exit 1
python tools/summarize_json.py $O/*.json
