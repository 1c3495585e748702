#!/bin/bash
# r5 run R: host time inside the first step() calls after prepare()
# (HEAT2D_STEP_TRACE, a temporary trace: us since step() entry at each mark).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5r
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
HEAT2D_STEP_TRACE=1 timeout -k 10 150 python3 tools/first_step.py --transport rccl --timers 0 --json $O/slab.json > $O/slab.log 2> $O/slab.err; echo "slab rc=$?"
HEAT2D_STEP_TRACE=1 timeout -k 10 150 python3 tools/first_step.py --transport self --rows 32768 --timers 0 --json $O/whole.json > $O/whole.log 2> $O/whole.err; echo "whole rc=$?"
head -c 2000 $O/slab.err | tail -c 1200
echo done
