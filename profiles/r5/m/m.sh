#!/bin/bash
# r5 run M: the first step() after prepare() — how much steady-state warm-up
# prepare() should end on (HEAT2D_WARM_MS / HEAT2D_WARM_MIN, experiment knobs):
# the 8-rank slab rehearsal and the headline, interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5m
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
b() { tag=$1; shift; timeout -k 10 300 python3 bench.py --field-check off --verify off "$@" > $O/$tag.json 2> $O/$tag.err; rc=$?; echo "$tag rc=$rc $(head -c 130 $O/$tag.json | tail -c 60)"; fatal $rc; }
for i in 1 2; do
  HEAT2D_WARM_MS=20 b slab_w20_$i --rehearse-comm --rows 4096 --steps 20 --warmup 5 --transport rccl
  HEAT2D_WARM_MS=2 HEAT2D_WARM_MIN=3 b slab_w2_$i --rehearse-comm --rows 4096 --steps 20 --warmup 5 --transport rccl
  HEAT2D_WARM_MS=0 HEAT2D_WARM_MIN=1 b slab_w1c_$i --rehearse-comm --rows 4096 --steps 20 --warmup 5 --transport rccl
  HEAT2D_WARM_MS=0 HEAT2D_WARM_MIN=0 b slab_w0_$i --rehearse-comm --rows 4096 --steps 20 --warmup 5 --transport rccl
  HEAT2D_WARM_MS=60 HEAT2D_WARM_MIN=3 b slab_w60_$i --rehearse-comm --rows 4096 --steps 20 --warmup 5 --transport rccl
done
for i in 1 2; do
  HEAT2D_WARM_MS=20 b h20_w20_$i --steps 20 --warmup 5
  HEAT2D_WARM_MS=0 HEAT2D_WARM_MIN=1 b h20_w1c_$i --steps 20 --warmup 5
done
echo done
