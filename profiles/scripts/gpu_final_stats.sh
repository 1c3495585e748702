#!/bin/bash
# final numbers: 5 headline runs (driver defaults), 3 runs of the 8-rank slab rehearsal, fp32 headline x2
set -o pipefail
mkdir -p gpurun_out/fin
for i in 1 2 3 4 5; do timeout -k 10 200 python bench.py > gpurun_out/fin/h_$i.json 2>/dev/null || exit 1; done
for i in 1 2; do timeout -k 10 200 python bench.py --dtype fp32 > gpurun_out/fin/h32_$i.json 2>/dev/null || exit 1; done
for i in 1 2 3; do timeout -k 10 200 python bench.py --rehearse-comm --rows 4096 --steps 240 --warmup 48 > gpurun_out/fin/r_$i.json 2>/dev/null || exit 1; done
echo done
