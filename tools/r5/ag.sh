#!/bin/bash
# r5 run AG: edge ranks' first cycle with the bands apart (far band led on the interior kernel, frame-side band behind the exchange) — probe, bench, the whole GPU suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5ag
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
f() { tag=$1; shift; timeout -k 10 150 python3 tools/first_step.py --timers 1 --reps 8 "$@" --json $O/$tag.json > $O/$tag.log 2> $O/$tag.err; rc=$?; echo "$tag rc=$rc"; fatal $rc; }
b() { tag=$1; shift; timeout -k 10 300 python3 bench.py "$@" > $O/$tag.json 2> $O/$tag.err; rc=$?; echo "$tag rc=$rc $(head -c 150 $O/$tag.json | tail -c 70)"; fatal $rc; }
f middle --transport rccl
f first --transport rccl --row0 0
f last --transport rccl --row0 28672
b slab_rccl_1 --rehearse-comm --rows 4096 --steps 20 --warmup 5 --transport rccl
b whole_1 --steps 20 --warmup 5
b slab_rccl_2 --rehearse-comm --rows 4096 --steps 20 --warmup 5 --transport rccl
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/gpu_tests.log; fatal $rc
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$? $(tail -1 $O/smoke.log)"
echo done
