#!/bin/bash
# r5 FINAL 2 (the round's final tree): the BASELINE configs at 480 / 1000
# steps, the full-HBM grid from the memory-fit planner and its 8-rank weak
# slab, the strong-scaling slab rehearsals at N = 2 / 4 / 8 (RCCL and IPC
# loops) beside two whole-grid runs, the fp32 8-rank slab, and the small grid's
# kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5final2
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
b() { tag=$1; shift; timeout -k 10 400 python3 bench.py "$@" > $O/$tag.json 2> $O/$tag.err; rc=$?; echo "$tag rc=$rc $(head -c 130 $O/$tag.json | tail -c 60)"; fatal $rc; }
b whole_1 --steps 20 --warmup 5
for n in 2 4 8; do
  rows=$((32768 / n))
  b slab${n}_rccl --rehearse-comm --rows $rows --steps 20 --warmup 5 --transport rccl
  b slab${n}_ipc --rehearse-comm --rows $rows --steps 20 --warmup 5 --transport ipc
done
b whole_2 --steps 20 --warmup 5
b f64_32k_480 --steps 480 --warmup 48
b f64_16k_480 --grid 16384 --steps 480 --warmup 48
b f32_32k_480 --dtype fp32 --steps 480 --warmup 48
b f32_slab8_480 --dtype fp32 --rehearse-comm --rows 4096 --steps 480 --warmup 48 --transport rccl
for i in 1 2 3; do b small_$i --grid 4096 --dtype fp32 --steps 1000 --warmup 64; done
mkdir -p $O/trace_small && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_small -o small -- python3 bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 64 --verify off --field-check off > $O/trace_small/bench.json 2> $O/trace_small/bench.err
rc=$?; echo "trace rc=$rc"; fatal $rc
b weak_max_fp32 --weak --dtype fp32 --grid max --steps 64 --warmup 8
N8=$(timeout -k 10 120 python3 -c "import heat2d; from heat2d.utils import memplan; print(memplan.plan_max_grid('fp32', 8, device=0)['n'])") && echo "N8=$N8" > $O/n8.txt
rc=$?; fatal $rc
b weak_max_fp32_slab8 --rehearse-comm --grid $N8 --rows $((N8 / 8)) --dtype fp32 --steps 64 --warmup 8
echo done
