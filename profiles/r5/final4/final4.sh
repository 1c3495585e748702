#!/bin/bash
# r5 FINAL 4: VERDICT r4 item 1's measurement on the final tree, as specified:
# median of 3 interleaved runs of the 4096-row middle-slab rehearsal (RCCL and
# IPC loops) against the whole grid, fp64 20 steps; fp32 480 steps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5final4
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
b() { tag=$1; shift; timeout -k 10 300 python3 bench.py "$@" > $O/$tag.json 2> $O/$tag.err; rc=$?; echo "$tag rc=$rc $(head -c 150 $O/$tag.json | tail -c 70)"; fatal $rc; }
for i in 1 2 3; do
  b whole_$i --steps 20 --warmup 5
  b slab_rccl_$i --rehearse-comm --rows 4096 --steps 20 --warmup 5 --transport rccl
  b slab_ipc_$i --rehearse-comm --rows 4096 --steps 20 --warmup 5 --transport ipc
done
for i in 1 2 3; do
  b f32_whole_$i --dtype fp32 --steps 480 --warmup 48
  b f32_slab_$i --dtype fp32 --rehearse-comm --rows 4096 --steps 480 --warmup 48 --transport rccl
done
echo done
