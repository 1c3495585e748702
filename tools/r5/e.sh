#!/bin/bash
# r5 run E: A/B of the round-4 final tree (build_ab/r4: its bench.py, package and
# library) against this tree, ABBA-interleaved per configuration on one box:
# the schedule search rewrite (schedule.cpp) and the knob pruning must not lose.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5e
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
run() {  # tag tree args...
  tag=$1; tree=$2; shift 2
  if [ $tree = old ]; then
    timeout -k 10 240 python3 build_ab/r4/bench.py --verify off "$@" > $O/$tag.json 2> $O/$tag.err
  else
    timeout -k 10 240 python3 bench.py --verify off --field-check off "$@" > $O/$tag.json 2> $O/$tag.err
  fi
  rc=$?; echo "$tag rc=$rc $(head -c 120 $O/$tag.json)"; fatal $rc
}
cfg() {  # name args...
  name=$1; shift
  run ${name}_old1 old "$@"; run ${name}_new1 new "$@"; run ${name}_new2 new "$@"; run ${name}_old2 old "$@"
}
cfg h20 --steps 20 --warmup 5
cfg f64_16k --grid 16384 --steps 480 --warmup 48
cfg f64_32k --steps 480 --warmup 48
cfg f32_32k --dtype fp32 --steps 480 --warmup 48
cfg f32_4k --grid 4096 --dtype fp32 --steps 1000 --warmup 64
cfg fast20 --sigma 0.2 --arith fast --steps 20 --warmup 5
echo done
