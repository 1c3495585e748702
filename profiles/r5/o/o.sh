#!/bin/bash
# r5 run O: the 8-rank slab after the fp64 priming skip — phase breakdown
# (probe_host, RCCL loop and the same middle slab without exchange, the whole
# grid) and the forced interior plans again (run D was before the skip).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5o
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
p() {  # tag transport [rows] [NAME=VALUE...]
  tag=$1; tr=$2; shift 2
  rows=4096; case $1 in [0-9]*) rows=$1; shift;; esac
  env "$@" timeout -k 10 150 python3 tools/probe_host.py --transport $tr --rows $rows --reps 15 --json $O/$tag.json > $O/$tag.log 2>&1
  rc=$?; echo "$tag rc=$rc"; fatal $rc
}
p auto rccl
p self_slab self 4096
p whole self 32768
p b6 rccl HEAT2D_BANDS=6 HEAT2D_DYNAMIC=1
p b10 rccl HEAT2D_BANDS=10 HEAT2D_DYNAMIC=1
p b12 rccl HEAT2D_BANDS=12 HEAT2D_DYNAMIC=1
p b16 rccl HEAT2D_BANDS=16 HEAT2D_DYNAMIC=1
p b24 rccl HEAT2D_BANDS=24 HEAT2D_DYNAMIC=1
p s2040 rccl HEAT2D_SEGMENTS=2040
p s3060 rccl HEAT2D_SEGMENTS=3060 HEAT2D_DYNAMIC=1
p s4080 rccl HEAT2D_SEGMENTS=4080 HEAT2D_DYNAMIC=1
p b8r4 rccl HEAT2D_BANDS=8 HEAT2D_DYNAMIC=1 HEAT2D_TB_RING=4
echo done
