#!/bin/bash
# r6 session 3, V10: the runner and bench-contract GPU tiers after the test
# helper move (tests/diag.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r6v10
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
timeout -k 10 900 python3 -u -m pytest tests/test_runner.py tests/test_bench_contract.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc $(tail -1 $O/gpu_tests.log)"; exit $rc
