#!/bin/bash
# r6 FINAL 5: the reference's literal run on the final tree (native CLI,
# fortran/hip/input.dat = 32768 0.25 0.05 1.0 25000 0, no output files), and
# the no-flag bench.py (480 steps) twice more (box-to-box spread of that row).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6final5
mkdir -p $O/lit
export HEAT2D_PLAN_CACHE=off PYTHONUNBUFFERED=1
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
printf "32768 0.25 0.05 1.0 25000 0\n" > $O/lit/input.dat
(cd $O/lit && timeout -k 10 300 $R/cuda-hip-mpi-heat-equation-test_amd/_native/heat2d --gpus 1 --output none --json m.json > out.txt 2>&1)
rc=$?; echo "literal rc=$rc $(tail -3 $O/lit/out.txt | tr '\n' ' ')"; fatal $rc
for i in 1 2; do
  timeout -k 10 400 python3 $R/bench.py > $O/noflag_$i.json 2> $O/noflag_$i.err
  rc=$?; echo "noflag_$i rc=$rc $(head -c 80 $O/noflag_$i.json | tail -c 30)"; fatal $rc
done
echo done
