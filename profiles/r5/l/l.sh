#!/bin/bash
# r5 run L: A/B of the priming skip in the GENERAL kernels too (build_ab/psg,
# -DHEAT2D_PS_GEN=1) against this tree, ABBA on one box; then the variant's
# bitwise GPU tests (frame-row edge kinds march through the skipped levels).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5l
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
run() {  # tag lib args...
  tag=$1; lib=$2; shift 2
  if [ $lib = psg ]; then
    HEAT2D_LIB=$PWD/build_ab/psg/libheat2d.so timeout -k 10 300 python3 bench.py --field-check off "$@" > $O/$tag.json 2> $O/$tag.err
  else
    timeout -k 10 300 python3 bench.py --field-check off "$@" > $O/$tag.json 2> $O/$tag.err
  fi
  rc=$?; echo "$tag rc=$rc $(head -c 130 $O/$tag.json | tail -c 60)"; fatal $rc
}
abba() { name=$1; shift; run ${name}_base1 base "$@"; run ${name}_psg1 psg "$@"; run ${name}_psg2 psg "$@"; run ${name}_base2 base "$@"; }
abba f32_4k --grid 4096 --dtype fp32 --steps 1000 --warmup 64
abba f64_4k --grid 4096 --steps 1000 --warmup 64
abba h20 --steps 20 --warmup 5
abba f64_16k --grid 16384 --steps 480 --warmup 48
abba fast20 --sigma 0.2 --arith fast --steps 20 --warmup 5
HEAT2D_LIB=$PWD/build_ab/psg/libheat2d.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_solver.py tests/test_jacobi.py tests/test_arith.py tests/test_arith_fast.py -m gpu -q -x --timeout 120 --timeout-method thread > $O/psg_tests.log 2>&1; echo "psg tests rc=$?"; tail -2 $O/psg_tests.log
echo done
