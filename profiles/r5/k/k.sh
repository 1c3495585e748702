#!/bin/bash
# r5 run K: the priming skip in every interior kernel (fp64 too) — the GPU
# suite (bitwise), then the bench rows it changes and the 8-rank slab rehearsal.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5k
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off PYTHONFAULTHANDLER=1 MALLOC_CHECK_=3
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/gpu_tests.log; fatal $rc; [ $rc = 0 ] || exit $rc
b() { tag=$1; shift; HEAT2D_TUNE_LOG=1 timeout -k 10 300 python3 bench.py "$@" > $O/$tag.json 2> $O/$tag.err; rc=$?; echo "$tag rc=$rc $(head -c 130 $O/$tag.json | tail -c 60)"; fatal $rc; }
for i in 1 2 3; do
  b h20_$i --steps 20 --warmup 5
  b slab_$i --rehearse-comm --rows 4096 --steps 20 --warmup 5 --transport rccl
done
b slab_ipc --rehearse-comm --rows 4096 --steps 20 --warmup 5 --transport ipc
b f16k --grid 16384 --steps 480 --warmup 48
b f32k480 --steps 480 --warmup 48
echo done
