#!/bin/bash
# r5 run F: the whole GPU suite + smoke on the current tree (regression check
# after the schedule-search rewrite, the knob pruning and the new features).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5f
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/gpu_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 $O/smoke.log
