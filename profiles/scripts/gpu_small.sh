#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/small
for K in 2 4 6 8 10 12 16; do
  timeout -k 10 120 python bench.py --n 4096 --dtype fp32 --tb $K --steps 960 --warmup 96 > gpurun_out/small/k$K.json 2>/dev/null || exit 1
done
for K in 4 8 12; do
  timeout -k 10 120 python bench.py --n 16384 --tb $K --steps 480 --warmup 48 > gpurun_out/small/f64_16k_k$K.json 2>/dev/null || exit 1
done
echo ok
