#!/bin/bash
# r5 run T: when does C++ step() start after Python's t0 (same monotonic
# clock): the first step() after prepare() against the following ones.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5t
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
for i in 1 2; do
  HEAT2D_STEP_TRACE=1 timeout -k 10 150 python3 tools/first_step.py --transport rccl --timers 0 --json $O/slab_$i.json > $O/slab_$i.log 2> $O/slab_$i.err; echo "slab rc=$?"
done
HEAT2D_STEP_TRACE=1 timeout -k 10 150 python3 tools/first_step.py --transport self --rows 32768 --timers 0 --json $O/whole.json > $O/whole.log 2> $O/whole.err; echo "whole rc=$?"
echo done
