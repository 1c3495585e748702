#!/bin/bash
# r5 run V: the fp32 8-rank slab (4096 x 32768, 480 steps) — tuner log of every
# depth it measures, against the whole 32768^2 fp32 grid's.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5v
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off HEAT2D_TUNE_LOG=1
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
b() { tag=$1; shift; timeout -k 10 300 python3 bench.py --field-check off --verify off "$@" > $O/$tag.json 2> $O/$tag.err; rc=$?; echo "$tag rc=$rc $(head -c 130 $O/$tag.json | tail -c 60)"; fatal $rc; }
b slab32 --dtype fp32 --rehearse-comm --rows 4096 --steps 480 --warmup 48 --transport rccl
b whole32 --dtype fp32 --steps 480 --warmup 48
echo done
