#!/bin/bash
# Boundary-band kernel A/B (HEAT2D_EDGE_KERNEL=0/1): fixed split plans and autotuned slab rehearsals.
set -o pipefail
O=gpurun_out/edgeab
mkdir -p $O
for e in 0 1; do
  for cfg in "fp64 32768 14 4 1 0" "fp32 4096 12 40 1 0" "fp32 32768 16 4 1 0" "fp64 8192 14 20 1 0"; do
    HEAT2D_SPLIT_ORDER=concurrent HEAT2D_EDGE_KERNEL=$e timeout -k 10 120 python tools/cycle_probe.py $cfg > $O/p.json || exit 1
    python -c "import json;d=json.load(open('$O/p.json'));print('edge=$e', '$cfg', round(d['gpts'],1), 'Gpts/s', round(d['ms']/d['cycles']*1e3,2),'us/cycle', d['plan'].get('order'), d['plan'].get('main_waves'), d['plan'].get('edge_waves'))"
  done
  for dt in fp32 fp64; do
    HEAT2D_EDGE_KERNEL=$e timeout -k 10 300 python bench.py --dtype $dt --rehearse-comm --rows 4096 --steps 480 --warmup 16 > $O/r.json || exit 1
    python -c "import json;d=json.load(open('$O/r.json'));c=d['config'];print('edge=$e rehearsal $dt', d['value'], c['cycles'], {k:(v['order'],v['main_bands'],v['main_waves']) for k,v in c['launch_plans'].items()})"
  done
done
