#!/bin/bash
# r5 run AH: real multi-process runs through the new edge-rank first cycle
# (every rank of N = 2 is an edge rank): bench.py --share-gpu, IPC after RCCL
# refuses, the timed field checked bitwise over the ranks.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5ah
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
b() { tag=$1; shift; timeout -k 10 170 python3 bench.py "$@" > $O/$tag.json 2> $O/$tag.err; rc=$?; echo "$tag rc=$rc $(head -c 150 $O/$tag.json | tail -c 70)"; fatal $rc; }
b share2 --gpus 2 --share-gpu --steps 20 --warmup 5
b share4_8192 --gpus 4 --share-gpu --grid 8192 --steps 20 --warmup 5
b share3_fp32 --gpus 3 --share-gpu --grid 8192 --dtype fp32 --steps 40 --warmup 5
echo done
