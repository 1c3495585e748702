#!/bin/bash
# r5 run I: A/B of the priming skip in the fp64 interior kernel
# (build_ab/ps: -DHEAT2D_PS_ALL=1) against this tree's library, ABBA on one box:
# the headline whole grid, the 8-rank middle slab (RCCL loop), 16384^2 fp64.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5i
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
run() {  # tag lib args...
  tag=$1; lib=$2; shift 2
  if [ $lib = ps ]; then
    HEAT2D_LIB=$PWD/build_ab/ps/libheat2d.so timeout -k 10 300 python3 bench.py --field-check off "$@" > $O/$tag.json 2> $O/$tag.err
  else
    timeout -k 10 300 python3 bench.py --field-check off "$@" > $O/$tag.json 2> $O/$tag.err
  fi
  rc=$?; echo "$tag rc=$rc $(head -c 130 $O/$tag.json | tail -c 60)"; fatal $rc
}
abba() { name=$1; shift; run ${name}_base1 base "$@"; run ${name}_ps1 ps "$@"; run ${name}_ps2 ps "$@"; run ${name}_base2 base "$@"; }
abba h20 --steps 20 --warmup 5
abba slab --rehearse-comm --rows 4096 --steps 20 --warmup 5 --transport rccl
abba slab_b --rehearse-comm --rows 4096 --steps 20 --warmup 5 --transport rccl
run f16k_base base --grid 16384 --steps 480 --warmup 48
run f16k_ps ps --grid 16384 --steps 480 --warmup 48
HEAT2D_LIB=$PWD/build_ab/ps/libheat2d.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_solver.py -q -x --timeout 120 --timeout-method thread > $O/ps_tests.log 2>&1; echo "ps tests rc=$?"; tail -1 $O/ps_tests.log
echo done
