#!/bin/bash
# r5 run AD: the 8-GPU run's edge ranks — the first slab (global frame row on
# one side) against a middle one, same one-cycle step (tools/first_step.py,
# RCCL loop exchange of both bands: timing only).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5ad
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
f() { tag=$1; shift; timeout -k 10 150 python3 tools/first_step.py --timers 1 --reps 8 "$@" --json $O/$tag.json > $O/$tag.log 2> $O/$tag.err; rc=$?; echo "$tag rc=$rc"; fatal $rc; }
for i in 1 2; do
  f middle_$i --transport rccl
  f first_$i --transport rccl --row0 0
  f last_$i --transport rccl --row0 28672
done
echo done
