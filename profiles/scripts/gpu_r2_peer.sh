#!/bin/bash
# Native CLI: 1 rank vs 8 rank threads sharing the GPU through the peer transport (same 32768^2 work).
set -o pipefail
O=$PWD/gpurun_out/peer
mkdir -p $O/run
cd $O/run
CLI=$GRAFT_REPO_ROOT/cuda-hip-mpi-heat-equation-test_amd/_native/heat2d
for dt in fp64 fp32; do
  echo "32768 0.25 0.05 1.0 480 0" > input.dat
  timeout -k 10 300 $CLI --dtype $dt --output none --json ../r1.json > ../o1.txt 2>&1 || { tail ../o1.txt; exit 1; }
  timeout -k 10 300 $CLI --dtype $dt --gpus 8 --transport peer --share-gpu --output none --json ../r8.json > ../o8.txt 2>&1 || { tail ../o8.txt; exit 1; }
  python -c "
import json
a=json.load(open('../r1.json')); b=json.load(open('../r8.json'))
print('$dt', '1 rank', round(a['gpts_per_s']), a['cycles'], '| 8 ranks sharing (peer)', round(b['gpts_per_s']), b['cycles'], '| ratio', round(b['gpts_per_s']/a['gpts_per_s'],3), '| sums equal', a['sum']==b['sum'])"
done
