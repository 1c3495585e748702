#!/bin/bash
# r5 run S: is the first step()'s extra host time (~50-65 us outside the C++
# step body, run R) the CPU leaving its idle state after prepare()'s long
# final synchronize? A busy-wait of the host right before the first rep.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5s
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
f() { tag=$1; shift; timeout -k 10 150 python3 tools/first_step.py --timers 0 "$@" --json $O/$tag.json > $O/$tag.log 2> $O/$tag.err; rc=$?; echo "$tag rc=$rc"; fatal $rc; }
for i in 1 2; do
  f slab_spin0_$i --transport rccl
  f slab_spin2_$i --transport rccl --spin-ms 2
  f slab_spin20_$i --transport rccl --spin-ms 20
  f whole_spin0_$i --transport self --rows 32768
  f whole_spin20_$i --transport self --rows 32768 --spin-ms 20
done
echo done
