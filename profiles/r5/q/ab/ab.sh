#!/bin/bash
# r5 run AB: does launching a few tiny kernels (and synchronising) right before
# the first step() after prepare() remove its slow first launch (profiles/r5/q/)?
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5ab
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
f() { tag=$1; shift; timeout -k 10 150 python3 tools/first_step.py --timers 0 "$@" --json $O/$tag.json > $O/$tag.log 2> $O/$tag.err; rc=$?; echo "$tag rc=$rc"; fatal $rc; }
for i in 1 2; do
  f slab_pre0_$i --transport rccl
  f slab_pre4_$i --transport rccl --pre-launch 4
  f slab_pre64_$i --transport rccl --pre-launch 64
  f whole_pre0_$i --transport self --rows 32768
  f whole_pre4_$i --transport self --rows 32768 --pre-launch 4
done
echo done
