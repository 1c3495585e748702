#!/bin/bash
# r6 session 3, V9 (final tree, second box): the GPU suite again, the no-flag
# bench (480 steps), and every BASELINE.json configuration on one GPU
# (bench/configs.py, the full-HBM grid included).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r6v9
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc $(tail -1 $O/gpu_tests.log)"; fatal $rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py > $O/noflag.json 2> $O/noflag.err
rc=$?; echo "noflag rc=$rc $(head -c 120 $O/noflag.json | tail -c 50)"; fatal $rc
timeout -k 10 900 python3 bench/configs.py > $O/configs.jsonl 2> $O/configs.err
rc=$?; echo "configs rc=$rc $(wc -l < $O/configs.jsonl) lines"; fatal $rc
echo done
