#!/bin/bash
# r5 run AC: the --share-gpu N = 4 stall at 32768^2 (hipIpcOpenMemHandle of a
# neighbour's 2 GB field, profiles/r5/x/) with the fields opened without
# hipIpcMemLazyEnablePeerAccess when the peer is on the same device.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5ac
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
run() {
  tag=$1; shift
  timeout -k 10 300 python3 bench.py "$@" > $O/$tag.json 2> $O/$tag.err &
  pid=$!
  while kill -0 $pid 2>/dev/null; do sleep 30; echo "alive $(date +%s) err_lines=$(wc -l < $O/$tag.err)"; done
  wait $pid; rc=$?; echo "$tag rc=$rc $(head -c 150 $O/$tag.json | tail -c 80)"
  [ $rc = 0 ] || exit $rc
}
run share4 --gpus 4 --share-gpu --steps 20 --warmup 5
run share8 --gpus 8 --share-gpu --steps 20 --warmup 5
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -k "ipc or share or multi or runner or cli" > $O/tests.log 2>&1; echo "tests rc=$?"; tail -2 $O/tests.log
echo done
