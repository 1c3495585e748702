#!/bin/bash
# r6 session 3, V8 (final tree, persistent capture events): the GPU suite with the host-transport runner test,
# smoke, the headline three times, the small grid; no profiler run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6v8
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc $(tail -1 $O/gpu_tests.log)"; fatal $rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc $(tail -1 $O/smoke.log)"; fatal $rc
for i in 1 2 3; do
  timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $O/h20_$i.json 2> $O/h20_$i.err
  rc=$?; echo "h20_$i rc=$rc $(head -c 120 $O/h20_$i.json | tail -c 50)"; fatal $rc
done
timeout -k 10 300 python3 bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 64 > $O/small.json 2> $O/small.err
rc=$?; echo "small rc=$rc $(head -c 120 $O/small.json | tail -c 50)"; fatal $rc
echo done
