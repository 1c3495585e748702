#!/bin/bash
# thin slabs (1 of 8 ranks): depth sweep with the rehearsal exchange, and no-exchange reference
set -o pipefail
mkdir -p gpurun_out/thin
export PYTHONUNBUFFERED=1
for K in 10 12 14 16; do
  timeout -k 10 200 python bench.py --dtype fp32 --tb $K --rehearse-comm --rows 4096 --steps 480 --warmup 48 > gpurun_out/thin/f32_reh_k$K.json 2>/dev/null || exit 1
done
timeout -k 10 200 python bench.py --dtype fp32 --rows 4096 --steps 480 --warmup 48 > gpurun_out/thin/f32_noex_k16.json 2>/dev/null || exit 1
for K in 8 10 11 12; do
  timeout -k 10 200 python bench.py --tb $K --rehearse-comm --rows 4096 --steps 480 --warmup 48 > gpurun_out/thin/f64_reh_k$K.json 2>/dev/null || exit 1
done
timeout -k 10 200 python bench.py --rows 4096 --steps 480 --warmup 48 > gpurun_out/thin/f64_noex_k12.json 2>/dev/null || exit 1
echo done
