#!/bin/bash
# r5 run G: the guided interior candidate (kern::with_guided_main) — the
# 8-rank slab one-cycle probe (as run D) with the tuner's log, then the bench
# rows it can change (the autotuner picks it only where it times faster).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5g
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
HEAT2D_TUNE_LOG=1 timeout -k 10 150 python3 tools/probe_host.py --transport rccl --reps 15 --json $O/auto.json > $O/auto.log 2>&1; fatal $?
HEAT2D_TUNE_LOG=1 timeout -k 10 150 python3 tools/probe_host.py --transport rccl --reps 15 --json $O/auto2.json > $O/auto2.log 2>&1; fatal $?
HEAT2D_TUNE_LOG=1 timeout -k 10 150 python3 tools/probe_host.py --transport self --rows 4096 --reps 15 --json $O/self_slab.json > $O/self_slab.log 2>&1; fatal $?
b() { tag=$1; shift; HEAT2D_TUNE_LOG=1 timeout -k 10 240 python3 bench.py "$@" > $O/$tag.json 2> $O/$tag.err; rc=$?; echo "$tag rc=$rc $(head -c 160 $O/$tag.json)"; fatal $rc; }
b h20 --steps 20 --warmup 5
b f32_4k --grid 4096 --dtype fp32 --steps 1000 --warmup 64
b f64_16k --grid 16384 --steps 480 --warmup 48
b f32_32k --dtype fp32 --steps 480 --warmup 48
timeout -k 10 400 python3 -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -k "split or plan or tb or dynamic or bench" > $O/tests.log 2>&1; echo "tests rc=$?"; tail -2 $O/tests.log
echo done
