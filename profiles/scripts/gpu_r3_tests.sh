set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/r3_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1 && tail -1 gpurun_out/r3_smoke.log &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench20.json 2> gpurun_out/r3_bench20.err && cat gpurun_out/r3_bench20.json
