#!/bin/bash
# r6 session 3, V1: the rebuilt tree (fresh container, same sources): GPU suite,
# smoke and the driver's headline twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r6v1
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
timeout -k 10 60 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc $(tail -1 $O/smoke.log)"; fatal $rc; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $O/h20_$i.json 2> $O/h20_$i.err
  rc=$?; echo "h20_$i rc=$rc $(head -c 200 $O/h20_$i.json | tail -c 120)"; fatal $rc
done
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc $(tail -1 $O/gpu_tests.log)"; fatal $rc
echo done
