#!/bin/bash
# r5 run H: VERDICT r4 item 1 as specified — whole grid vs the 4096-row
# middle-slab rehearsal (RCCL and IPC loops), fp64 20 steps and fp32 480
# steps, three interleaved runs each; the measured-HBM headline; 16384^2 fp64
# 480 steps after the schedule-search neighbour fix.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5h
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
b() { tag=$1; shift; timeout -k 10 300 python3 bench.py "$@" > $O/$tag.json 2> $O/$tag.err; rc=$?; echo "$tag rc=$rc $(head -c 150 $O/$tag.json)"; fatal $rc; }
for i in 1 2 3; do
  b f64_whole_$i --steps 20 --warmup 5
  b f64_rccl_$i --rehearse-comm --rows 4096 --steps 20 --warmup 5 --transport rccl
  b f64_ipc_$i --rehearse-comm --rows 4096 --steps 20 --warmup 5 --transport ipc
done
for i in 1 2 3; do
  b f32_whole_$i --dtype fp32 --steps 480 --warmup 48
  b f32_rccl_$i --dtype fp32 --rehearse-comm --rows 4096 --steps 480 --warmup 48 --transport rccl
done
b f32_ipc_1 --dtype fp32 --rehearse-comm --rows 4096 --steps 480 --warmup 48 --transport ipc
HEAT2D_TUNE_LOG=1 b f64_16k --grid 16384 --steps 480 --warmup 48
b hbm --steps 20 --warmup 5 --measure-hbm
echo done
