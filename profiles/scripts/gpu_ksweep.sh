#!/bin/bash
# fp64 depth sweep on the headline config (two-pass autotuner), two rounds interleaved
set -o pipefail
mkdir -p gpurun_out/ks
for i in 1 2; do for K in 10 12 13 14 15 16; do
  timeout -k 10 200 python bench.py --tb $K --steps 480 > gpurun_out/ks/k${K}_$i.json 2>/dev/null || exit 1
done; done
echo done
