#!/bin/bash
# Forced segment counts on a 4096-row slab (single launch, no exchange) vs the band plan.
set -o pipefail
p() { python -c "
import sys,json
for l in sys.stdin:
    if '\"gpts\"' not in l: continue
    d=json.loads(l[l.index('{'):]); pl=d['plan']; print(sys.argv[1], d['dtype'], d['k'], round(d['gpts']), round(d['ms']/d['cycles']*1e3,1), 'us/cycle', pl.get('order'), pl.get('ring'), pl.get('main_bands'), pl.get('main_waves'))" "$1"; }
for seg in 0 1020 1024 2040 2048 3072 4096; do
  if [ $seg = 0 ]; then unset HEAT2D_SEGMENTS; else export HEAT2D_SEGMENTS=$seg; fi
  HEAT2D_SPLIT_ORDER=single CP_ROWS=4096 timeout -k 10 120 python tools/cycle_probe.py fp32 32768 16 30 1 | p "seg=$seg" || exit 1
done
for seg in 0 3072 6144; do
  if [ $seg = 0 ]; then unset HEAT2D_SEGMENTS; else export HEAT2D_SEGMENTS=$seg; fi
  HEAT2D_SPLIT_ORDER=single CP_ROWS=4096 timeout -k 10 120 python tools/cycle_probe.py fp64 32768 14 30 1 | p "seg=$seg" || exit 1
done
