#!/bin/bash
# XCD-contiguous wave numbering (HEAT2D_XCD_REMAP=1) on Infinity-Cache-resident grids, interleaved A/B.
set -o pipefail
O=gpurun_out/remap_small
mkdir -p $O
export PYTHONUNBUFFERED=1
show() { python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];print(sys.argv[1].split('/')[-1], d['value'], d['ms_per_step'], c['cycles'], {k:(v['order'],v['ring'],v['main_bands'],v['main_waves'],round(v['tuned_ms'],4)) for k,v in (c['launch_plans'] or {}).items()})" $1; }
for i in 1 2; do
  for x in 0 1; do
    HEAT2D_XCD_REMAP=$x timeout -k 10 300 python bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 10 > $O/s4096_${x}_$i.json || exit 1; show $O/s4096_${x}_$i.json
    HEAT2D_XCD_REMAP=$x timeout -k 10 300 python bench.py --grid 4096 --dtype fp64 --steps 1000 --warmup 10 > $O/d4096_${x}_$i.json || exit 1; show $O/d4096_${x}_$i.json
    HEAT2D_XCD_REMAP=$x timeout -k 10 300 python bench.py --grid 8192 --dtype fp32 --steps 1000 --warmup 10 > $O/s8192_${x}_$i.json || exit 1; show $O/s8192_${x}_$i.json
  done
done
