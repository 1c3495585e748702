#!/bin/bash
# r5 FINAL 3: the final tree's GPU suite and smoke (after the test fix that
# followed final1), and the headline / 8-rank slab once more on this box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5final3
mkdir -p $O
export PYTHONUNBUFFERED=1
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/gpu_tests.log; fatal $rc
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc $(tail -1 $O/smoke.log)"; fatal $rc
export HEAT2D_PLAN_CACHE=off
b() { tag=$1; shift; timeout -k 10 300 python3 bench.py "$@" > $O/$tag.json 2> $O/$tag.err; rc=$?; echo "$tag rc=$rc $(head -c 130 $O/$tag.json | tail -c 60)"; fatal $rc; }
b bench_default
b bench20_1 --steps 20 --warmup 5
b slab8_rccl --rehearse-comm --rows 4096 --steps 20 --warmup 5 --transport rccl
b bench20_2 --steps 20 --warmup 5
echo done
