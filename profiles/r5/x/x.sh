#!/bin/bash
# r5 run X: the driver's multi-rank bench path end to end on one GPU — N rank
# processes sharing the card (bench.py starts them itself), the default
# transport choice (RCCL refuses ranks on one GPU -> IPC), the timed-field
# check over the ranks and the decomposition self-check, N = 2 / 4 / 8.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5x
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
b() { tag=$1; shift; timeout -k 10 600 python3 bench.py "$@" > $O/$tag.json 2> $O/$tag.err; rc=$?; echo "$tag rc=$rc $(head -c 150 $O/$tag.json | tail -c 80)"; fatal $rc; }
b share2 --gpus 2 --share-gpu --steps 20 --warmup 5
b share4 --gpus 4 --share-gpu --steps 20 --warmup 5
b share8 --gpus 8 --share-gpu --steps 20 --warmup 5
echo done
