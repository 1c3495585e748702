#!/bin/bash
# r6 FINAL 1 (the round's final tree): the GPU suite, smoke, then the driver's
# headline command (32768^2 fp64, 20 steps) three times interleaved with the
# BASELINE.json hot-spot data twice, and one --measure-hbm run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6final1
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
b() { tag=$1; shift; timeout -k 10 400 python3 bench.py "$@" > $O/$tag.json 2> $O/$tag.err; rc=$?; echo "$tag rc=$rc $(head -c 130 $O/$tag.json | tail -c 60)"; fatal $rc; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc $(tail -1 $O/gpu_tests.log)"; fatal $rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc $(tail -1 $O/smoke.log)"; fatal $rc
b h20_1 --steps 20 --warmup 5
b hot20_1 --steps 20 --warmup 5 --ic hotspot
b h20_2 --steps 20 --warmup 5
b hot20_2 --steps 20 --warmup 5 --ic hotspot
b h20_3 --steps 20 --warmup 5
b h20_hbm --steps 20 --warmup 5 --measure-hbm
echo done
