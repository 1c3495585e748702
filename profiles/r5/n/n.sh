#!/bin/bash
# r5 run N: prepare()'s closing warm-up length (HEAT2D_WARM_MS, experiment
# knob; run M: 60 ms beat 20 on the 8-rank slab) — where it saturates, and
# that no other row loses.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5n
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off HEAT2D_WARM_MIN=3
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
b() { tag=$1; shift; timeout -k 10 300 python3 bench.py --field-check off --verify off "$@" > $O/$tag.json 2> $O/$tag.err; rc=$?; echo "$tag rc=$rc $(head -c 130 $O/$tag.json | tail -c 60)"; fatal $rc; }
for i in 1 2; do
  for w in 20 60 100 200 400; do
    HEAT2D_WARM_MS=$w b slab_w${w}_$i --rehearse-comm --rows 4096 --steps 20 --warmup 5 --transport rccl
  done
done
for i in 1 2; do
  for w in 20 100 200; do
    HEAT2D_WARM_MS=$w b h20_w${w}_$i --steps 20 --warmup 5
    HEAT2D_WARM_MS=$w b f32_4k_w${w}_$i --grid 4096 --dtype fp32 --steps 1000 --warmup 64
  done
done
for w in 20 200; do
  HEAT2D_WARM_MS=$w b slab32_w${w} --dtype fp32 --rehearse-comm --rows 4096 --steps 480 --warmup 48 --transport rccl
  HEAT2D_WARM_MS=$w b f16k_w${w} --grid 16384 --steps 480 --warmup 48
done
echo done
