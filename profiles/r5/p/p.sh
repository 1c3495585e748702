#!/bin/bash
# r5 run P: wave priority by items done (build_ab/prio,
# -DHEAT2D_PRIO=1: s_setprio 3 for a wave's first interior item, 2 for its second, ...: a
# wave ahead of its SIMD partner yields to it) against this tree, ABBA on one box:
# the 8-rank slab (probe and bench), the headline, 16384^2 fp64, fp32 slab.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5p
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
L=$PWD/build_ab/prio/libheat2d.so
run() {  # tag lib args...
  tag=$1; lib=$2; shift 2
  if [ $lib = prio ]; then
    HEAT2D_LIB=$L timeout -k 10 300 python3 bench.py --field-check off --verify off "$@" > $O/$tag.json 2> $O/$tag.err
  else
    timeout -k 10 300 python3 bench.py --field-check off --verify off "$@" > $O/$tag.json 2> $O/$tag.err
  fi
  rc=$?; echo "$tag rc=$rc $(head -c 130 $O/$tag.json | tail -c 60)"; fatal $rc
}
abba() { name=$1; shift; run ${name}_base1 base "$@"; run ${name}_prio1 prio "$@"; run ${name}_prio2 prio "$@"; run ${name}_base2 base "$@"; }
timeout -k 10 150 python3 tools/probe_host.py --transport rccl --reps 15 --json $O/probe_base.json > $O/probe_base.log 2>&1; fatal $?
HEAT2D_LIB=$L timeout -k 10 150 python3 tools/probe_host.py --transport rccl --reps 15 --json $O/probe_prio.json > $O/probe_prio.log 2>&1; fatal $?
HEAT2D_LIB=$L HEAT2D_SEGMENTS=2040 timeout -k 10 150 python3 tools/probe_host.py --transport rccl --reps 15 --json $O/probe_prio_s2040.json > $O/probe_prio_s2040.log 2>&1; fatal $?
HEAT2D_LIB=$L timeout -k 10 150 python3 tools/probe_host.py --transport self --rows 32768 --reps 5 --json $O/probe_prio_whole.json > $O/probe_prio_whole.log 2>&1; fatal $?
abba slab --rehearse-comm --rows 4096 --steps 20 --warmup 5 --transport rccl
abba h20 --steps 20 --warmup 5
abba f16k --grid 16384 --steps 480 --warmup 48
abba slab32 --dtype fp32 --rehearse-comm --rows 4096 --steps 480 --warmup 48 --transport rccl
HEAT2D_LIB=$L timeout -k 10 400 python3 -u -m pytest tests/test_gpu_solver.py tests/test_jacobi.py -m gpu -q -x --timeout 120 --timeout-method thread > $O/prio_tests.log 2>&1; echo "prio tests rc=$?"; tail -1 $O/prio_tests.log
echo done
