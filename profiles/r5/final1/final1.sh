#!/bin/bash
# r5 FINAL 1 (the round's final tree): GPU suite, smoke, headline x3, the
# headline with measured HBM traffic and its kernel trace, the reference's
# literal 25000-step CLI run, sigma = 0.2 (fast / exact).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5final1
mkdir -p $O
export PYTHONUNBUFFERED=1
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/gpu_tests.log; fatal $rc
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc $(tail -1 $O/smoke.log)"; fatal $rc
export HEAT2D_PLAN_CACHE=off
b() { tag=$1; shift; timeout -k 10 400 python3 bench.py "$@" > $O/$tag.json 2> $O/$tag.err; rc=$?; echo "$tag rc=$rc $(head -c 130 $O/$tag.json | tail -c 60)"; fatal $rc; }
for i in 1 2 3; do b bench20_$i --steps 20 --warmup 5; done
b bench20_hbm --steps 20 --warmup 5 --measure-hbm
b s02_fast --sigma 0.2 --arith fast --steps 20 --warmup 5
b s02_exact --sigma 0.2 --steps 20 --warmup 5
BIN=$GRAFT_REPO_ROOT/cuda-hip-mpi-heat-equation-test_amd/_native/heat2d
mkdir -p $O/ref && (cd $O/ref && printf "32768 0.25 0.05 1.0 25000 0\n" > input.dat && \
  timeout -k 10 300 $BIN input.dat --output none --json auto.json > auto.txt 2>&1 && tail -3 auto.txt && \
  timeout -k 10 300 $BIN input.dat --output none --time-transfers --json auto_tt.json > auto_tt.txt 2>&1 && tail -3 auto_tt.txt)
rc=$?; echo "cli rc=$rc"; fatal $rc
mkdir -p $O/trace && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o headline -- python3 bench.py --steps 20 --warmup 5 --verify off --field-check off > $O/trace/bench.json 2> $O/trace/bench.err
rc=$?; echo "trace rc=$rc"; fatal $rc
echo done
