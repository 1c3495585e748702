#!/bin/bash
# r6 IPC run 3: fields of [2^31, 2^32) bytes allocated as 2^32 + 16 MiB by the
# IPC transport. The bench-contract and IPC GPU tests (incl. the new 23170^2
# two-rank test), then the configurations that stalled before: 4 and 3 rank
# processes at 32768^2 (the 20-step headline on one GPU, timed field checked),
# 2 at 26000^2, 4 at 36000^2.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ipc3
mkdir -p $O
export HEAT2D_PLAN_CACHE=off HEAT2D_IPC_ATTACH_LOG=1 PYTHONUNBUFFERED=1
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
timeout -k 10 900 python3 -u -m pytest tests/test_bench_contract.py tests/test_distributed.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $O/tests.log)"; fatal $rc; [ $rc -eq 0 ] || exit $rc
export HEAT2D_IPC_ATTACH_TIMEOUT=20
for cfg in "4 32768" "3 32768" "2 26000" "4 36000"; do
  set -- $cfg
  timeout -k 10 400 python3 $R/bench.py --gpus $1 --share-gpu --steps 20 --warmup 5 --grid $2 > $O/share$1_$2.json 2> $O/share$1_$2.err
  rc=$?
  echo "share N=$1 grid $2 rc=$rc $(grep -h 'heat2d ipc' $O/share$1_$2.err | head -2 | tr '\n' ' ') $(head -c 80 $O/share$1_$2.json | tail -c 30)"
  fatal $rc
done
echo done
