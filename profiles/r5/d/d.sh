#!/bin/bash
# r5 run D: the 8-rank strong-scaling slab (4096 x 32768 fp64, one depth-20
# cycle): forced interior plans (row bands / segments, dynamic queue, ring)
# against the autotuned one, median of 15 one-cycle regions each (probe_host).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5d
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
p() {  # tag env...
  tag=$1; shift
  env "$@" timeout -k 10 150 python3 tools/probe_host.py --transport rccl --reps 15 --json $O/$tag.json > $O/$tag.log 2>&1
}
p auto && p auto2 && \
p b4 HEAT2D_BANDS=4 HEAT2D_DYNAMIC=1 && p b6 HEAT2D_BANDS=6 HEAT2D_DYNAMIC=1 && p b7 HEAT2D_BANDS=7 HEAT2D_DYNAMIC=1 && \
p b8 HEAT2D_BANDS=8 HEAT2D_DYNAMIC=1 && p b10 HEAT2D_BANDS=10 HEAT2D_DYNAMIC=1 && p b12 HEAT2D_BANDS=12 HEAT2D_DYNAMIC=1 && \
p b16 HEAT2D_BANDS=16 HEAT2D_DYNAMIC=1 && p b8s HEAT2D_BANDS=8 HEAT2D_DYNAMIC=0 && p b5s HEAT2D_BANDS=5 HEAT2D_DYNAMIC=0 && \
p s2040 HEAT2D_SEGMENTS=2040 && p s3060 HEAT2D_SEGMENTS=3060 HEAT2D_DYNAMIC=1 && p s4080 HEAT2D_SEGMENTS=4080 HEAT2D_DYNAMIC=1 && \
p s6120 HEAT2D_SEGMENTS=6120 HEAT2D_DYNAMIC=1 && p b8r6 HEAT2D_BANDS=8 HEAT2D_DYNAMIC=1 HEAT2D_TB_RING=6 && \
p b8con HEAT2D_BANDS=8 HEAT2D_DYNAMIC=1 HEAT2D_SPLIT_ORDER=concurrent HEAT2D_LEAD_FIRST=0 && \
timeout -k 10 150 python3 tools/probe_host.py --transport self --rows 4096 --reps 15 --json $O/self_slab.json > $O/self_slab.log 2>&1
echo done rc=$?
