#!/bin/bash
# fp64 default depth: K=12 vs K=14 on the full grid and on the 2/4/8-rank slabs (rehearsal)
set -o pipefail
mkdir -p gpurun_out/k14
for i in 1 2; do for K in 12 14; do
  timeout -k 10 200 python bench.py --tb $K > gpurun_out/k14/full_k${K}_$i.json 2>/dev/null || exit 1
  for R in 16384 8192 4096; do
    timeout -k 10 200 python bench.py --tb $K --rehearse-comm --rows $R --steps 240 --warmup 48 > gpurun_out/k14/r${R}_k${K}_$i.json 2>/dev/null || exit 1
  done
done; done
echo done
