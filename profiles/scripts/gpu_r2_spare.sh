#!/bin/bash
# Thin-slab rehearsal vs the wave slots reserved beside the interior (HEAT2D_SPARE_WAVES).
set -o pipefail
O=gpurun_out/spare
mkdir -p $O
show() { python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];print(sys.argv[2], d['value'], c['cycles'], {k:(v['order'],v['main_bands'],v['main_waves'],v['edge_items']) for k,v in (c['launch_plans'] or {}).items()})" $1 "$2"; }
for sp in 8 160 460; do
  for dt in fp32 fp64; do
    HEAT2D_SPARE_WAVES=$sp timeout -k 10 300 python bench.py --dtype $dt --rehearse-comm --rows 4096 --steps 480 --warmup 16 > $O/r.json || exit 1; show $O/r.json "spare=$sp $dt"
  done
done
HEAT2D_SPARE_WAVES=160 timeout -k 10 300 python bench.py --dtype fp32 --rehearse-comm --rows 8192 --steps 480 --warmup 16 > $O/r.json || exit 1; show $O/r.json "spare=160 fp32 8192"
HEAT2D_SPARE_WAVES=160 timeout -k 10 300 python bench.py --rehearse-comm --rows 8192 --steps 480 --warmup 16 > $O/r.json || exit 1; show $O/r.json "spare=160 fp64 8192"
