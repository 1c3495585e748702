#!/bin/bash
# 4096^2 fp32, 1000 steps: one rank (eager / graph) vs P rank threads sharing the GPU (peer transport).
set -o pipefail
O=$PWD/gpurun_out/smallsplit
mkdir -p $O/run
cd $O/run
CLI=$GRAFT_REPO_ROOT/cuda-hip-mpi-heat-equation-test_amd/_native/heat2d
echo "4096 0.25 0.05 1.0 1000 0" > input.dat
run() { timeout -k 10 120 $CLI --dtype fp32 --output none --quiet --json ../r.json "$@" > ../o.txt 2>&1 || { tail ../o.txt; exit 1; }
  python -c "import json;d=json.load(open('../r.json'));print('$*', round(d['gpts_per_s']), d['cycles'])"; }
run --gpus 1
run --gpus 1 --graph
for P in 2 3 4 8; do run --gpus $P --transport peer --share-gpu; done
