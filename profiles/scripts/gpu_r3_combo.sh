set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_r3_persist.sh || exit $?
timeout -k 10 120 python -u -m pytest tests/test_runner.py -m gpu -x -q --timeout 100 --timeout-method thread > gpurun_out/r3_pycuda.log 2>&1; echo "pycuda test rc=$?"; tail -2 gpurun_out/r3_pycuda.log
bash tools/gpu_r3_thin.sh
