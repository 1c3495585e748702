#!/bin/bash
# RCCL spare wave slots beside the interior (HEAT2D_SPARE_WAVES) x split order, 8-rank slabs
set -o pipefail
mkdir -p gpurun_out/sp2
for dt in fp32 fp64; do for sp in 8 32 64; do for o in auto edge-first; do
  if [ $o = auto ]; then unset HEAT2D_SPLIT_ORDER; else export HEAT2D_SPLIT_ORDER=$o; fi
  HEAT2D_SPARE_WAVES=$sp timeout -k 10 200 python bench.py --dtype $dt --rehearse-comm --rows 4096 --steps 240 --warmup 48 --phase-timers > gpurun_out/sp2/${dt}_s${sp}_$o.json 2>/dev/null || exit 1
done; done; done
echo done
