#!/bin/bash
# r5 run J: (1) per-depth tuned costs with and without the fp64 interior
# priming skip (build_ab/ps) on 16384^2 and 32768^2 fp64 480 steps (tuner log);
# (2) the warm exchange at the end of prepare(): first step() after prepare
# (probe_host first_us) and the slab rehearsal bench, with / without it.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5j
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
run() {  # tag lib args...
  tag=$1; lib=$2; shift 2
  if [ $lib = ps ]; then
    HEAT2D_TUNE_LOG=1 HEAT2D_LIB=$PWD/build_ab/ps/libheat2d.so timeout -k 10 300 python3 bench.py --field-check off "$@" > $O/$tag.json 2> $O/$tag.err
  else
    HEAT2D_TUNE_LOG=1 timeout -k 10 300 python3 bench.py --field-check off "$@" > $O/$tag.json 2> $O/$tag.err
  fi
  rc=$?; echo "$tag rc=$rc $(head -c 130 $O/$tag.json | tail -c 60)"; fatal $rc
}
run f16k_base base --grid 16384 --steps 480 --warmup 48
run f16k_ps ps --grid 16384 --steps 480 --warmup 48
run f32k_base base --steps 480 --warmup 48
run f32k_ps ps --steps 480 --warmup 48
p() { tag=$1; shift; env "$@" timeout -k 10 150 python3 tools/probe_host.py --transport rccl --reps 15 --json $O/$tag.json > $O/$tag.log 2>&1; rc=$?; echo "$tag rc=$rc"; fatal $rc; }
p probe_warm
p probe_nowarm HEAT2D_NO_WARM_X=1
for i in 1 2; do
  run slab_warm_$i base --rehearse-comm --rows 4096 --steps 20 --warmup 5 --transport rccl
  HEAT2D_NO_WARM_X=1 run slab_nowarm_$i base --rehearse-comm --rows 4096 --steps 20 --warmup 5 --transport rccl
done
echo done
