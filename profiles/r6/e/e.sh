#!/bin/bash
# r6 run E: continued items (kVarCont interior kernels, kPlanContinue) — the
# new GPU tests (bitwise against the golden, forced plans, graphs), then
# interleaved A/B against HEAT2D_CONTINUE=0 (no continued-item candidates) on
# the configurations whose interior kernels have the twin: the fp32 8-rank
# slab (480 steps), 16384^2 fp64 and 32768^2 fp32 (480 steps); the fp64
# headline (depth 20: no twin) as the control.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6e
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_solver.py -k "continued" -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $O/tests.log)"; [ $rc -eq 0 ] || exit $rc
b() { tag=$1; shift; timeout -k 10 300 python3 $R/bench.py "$@" > $O/$tag.json 2> $O/$tag.err; rc=$?; echo "$tag rc=$rc $(head -c 150 $O/$tag.json | tail -c 70)"; fatal $rc; }
for i in 1 2; do
  for v in off on; do
    if [ $v = off ]; then export HEAT2D_CONTINUE=0; else unset HEAT2D_CONTINUE; fi
    b f32slab_${v}_$i --dtype fp32 --rehearse-comm --rows 4096 --steps 480 --warmup 48 --transport rccl
    b f64_16k_${v}_$i --grid 16384 --steps 480 --warmup 48
    b f32_32k_${v}_$i --dtype fp32 --steps 480 --warmup 48
    b h20_${v}_$i --steps 20 --warmup 5
  done
done
unset HEAT2D_CONTINUE
echo done
