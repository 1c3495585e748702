#!/bin/bash
# r6 session 3, V4: the host-staged transport on GPU ranks: the runner test
# (3 rank processes on one GPU, bitwise) and bench.py --transport host beside
# IPC at 8192^2 (3 ranks sharing the GPU), both with their field checks.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r6v4
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
timeout -k 10 300 python3 -u -m pytest tests/test_runner.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/runner_gpu.log 2>&1
rc=$?; echo "runner gpu tests rc=$rc $(tail -1 $O/runner_gpu.log)"; fatal $rc; [ $rc -eq 0 ] || exit $rc
for t in host ipc; do
  timeout -k 10 400 python3 bench.py --gpus 3 --share-gpu --transport $t --grid 8192 --steps 20 --warmup 5 > $O/b3_$t.json 2> $O/b3_$t.err
  rc=$?; echo "bench 3 ranks $t rc=$rc $(head -c 120 $O/b3_$t.json | tail -c 50)"; fatal $rc
done
echo done
