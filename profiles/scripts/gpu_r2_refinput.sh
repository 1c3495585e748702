#!/bin/bash
# The reference's own benchmark input (fortran/hip/input.dat: 32768 0.25 0.05 1.0 25000 0), full run, native CLI.
set -o pipefail
O=$PWD/gpurun_out/refinput
mkdir -p $O/run
cd $O/run
echo "32768 0.25 0.05 1.0 25000 0" > input.dat
timeout -k 10 300 $GRAFT_REPO_ROOT/cuda-hip-mpi-heat-equation-test_amd/_native/heat2d --print-every 5000 --check-every 5000 --json ../run.json > ../stdout.txt 2>&1 || { tail -20 ../stdout.txt; exit 1; }
grep -v "^time_it" ../stdout.txt | tail -25
