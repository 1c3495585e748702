#!/bin/bash
# r5 run AA: the 8-rank slab's 20 steps cut shallower (bench --tb caps the
# depth; each depth then tuned): is one depth-20 pass still best on the slab?
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5aa
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
b() { tag=$1; shift; timeout -k 10 300 python3 bench.py --field-check off --verify off "$@" > $O/$tag.json 2> $O/$tag.err; rc=$?; echo "$tag rc=$rc $(head -c 150 $O/$tag.json | tail -c 70)"; fatal $rc; }
for i in 1 2; do
  b slab_tb24_$i --rehearse-comm --rows 4096 --steps 20 --warmup 5 --transport rccl
  b slab_tb10_$i --rehearse-comm --rows 4096 --steps 20 --warmup 5 --transport rccl --tb 10
  b slab_tb12_$i --rehearse-comm --rows 4096 --steps 20 --warmup 5 --transport rccl --tb 12
  b slab_tb14_$i --rehearse-comm --rows 4096 --steps 20 --warmup 5 --transport rccl --tb 14
done
echo done
