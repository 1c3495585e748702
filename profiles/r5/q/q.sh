#!/bin/bash
# r5 run Q: where the first step() after prepare() loses its 17-56 us
# (tools/first_step.py: wall, enqueue and GPU span per rep), slab and whole grid,
# with and without an idle pause before it.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5q
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
f() { tag=$1; shift; timeout -k 10 150 python3 tools/first_step.py "$@" --json $O/$tag.json > $O/$tag.log 2>&1; rc=$?; echo "$tag rc=$rc"; fatal $rc; }
f slab_t1 --transport rccl
f slab_t0 --transport rccl --timers 0
f slab_idle50 --transport rccl --idle-ms 50
f slab_self --transport self
f whole_t1 --transport self --rows 32768
f whole_t0 --transport self --rows 32768 --timers 0
f slab_t1b --transport rccl
echo done
