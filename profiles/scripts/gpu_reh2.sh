#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/reh2
for dt in fp64 fp32; do for R in 16384 8192 4096; do
  timeout -k 10 200 python bench.py --dtype $dt --rehearse-comm --rows $R --steps 240 --warmup 48 > gpurun_out/reh2/${dt}_$R.json 2>/dev/null || exit 1
done; done
for K in 12 14; do timeout -k 10 200 python bench.py --dtype fp32 --tb $K > gpurun_out/reh2/f32_k$K.json 2>/dev/null || exit 1; done
echo done
