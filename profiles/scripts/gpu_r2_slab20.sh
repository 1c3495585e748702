#!/bin/bash
# 4096-row fp64 slab (1 of 8 ranks, strong scaling), K = 20, edge-first with RCCL self-exchange: forced interior plans.
set -o pipefail
O=gpurun_out/slab20
mkdir -p $O
run() { HEAT2D_SPLIT_ORDER=edge-first CP_ROWS=4096 CP_LOOP=1 timeout -k 10 120 python tools/cycle_probe.py fp64 32768 20 12 > $O/p.json || exit 1
  python -c "import json;d=[json.loads(l) for l in open('$O/p.json') if l.startswith('{')][-1];p=d['plan'];print('$1', round(d['gpts']), round(d['ms']/d['cycles']*1e3,1),'us/cycle', p['order'], p['ring'], p['main_bands'], p['main_items'], p['main_waves'])"; }
for b in 4 5 6 8 11 16; do HEAT2D_BANDS=$b run "bands=$b" || exit 1; done
unset HEAT2D_BANDS
for sgm in 1865 2040 3730 4080; do HEAT2D_SEGMENTS=$sgm run "segs=$sgm" || exit 1; done
unset HEAT2D_SEGMENTS
HEAT2D_TB_RING=6 HEAT2D_BANDS=8 run "ring6 bands=8" || exit 1
HEAT2D_TB_RING=6 HEAT2D_SEGMENTS=2040 run "ring6 segs=2040" || exit 1
