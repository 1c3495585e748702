#!/bin/bash
# r5 run U: prepare() closing on a lead-ordered trial cycle (the comm stream
# warm for step()'s first band launch): first step vs the following ones, and
# the bench's 8-rank slab rehearsal (final2: 4336.1 RCCL / 4373.0 IPC).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5u
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
f() { tag=$1; shift; timeout -k 10 150 python3 tools/first_step.py --timers 0 "$@" --json $O/$tag.json > $O/$tag.log 2> $O/$tag.err; rc=$?; echo "$tag rc=$rc"; fatal $rc; }
b() { tag=$1; shift; timeout -k 10 300 python3 bench.py "$@" > $O/$tag.json 2> $O/$tag.err; rc=$?; echo "$tag rc=$rc $(head -c 130 $O/$tag.json | tail -c 60)"; fatal $rc; }
f first_1 --transport rccl
f first_2 --transport rccl
f first_ipc --transport ipc
for i in 1 2 3; do
  b slab_rccl_$i --rehearse-comm --rows 4096 --steps 20 --warmup 5 --transport rccl
  b slab_ipc_$i --rehearse-comm --rows 4096 --steps 20 --warmup 5 --transport ipc
done
b whole_1 --steps 20 --warmup 5
b slab4_rccl --rehearse-comm --rows 8192 --steps 20 --warmup 5 --transport rccl
b slab2_rccl --rehearse-comm --rows 16384 --steps 20 --warmup 5 --transport rccl
b whole_2 --steps 20 --warmup 5
echo done
