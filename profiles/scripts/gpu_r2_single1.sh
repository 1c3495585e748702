#!/bin/bash
# One-cycle schedules on strong-scaling slabs: autotuned no-exchange plan (may pick single) vs the exchanging edge-first plan.
set -o pipefail
O=gpurun_out/single1
mkdir -p $O
p() { python -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[2]) if l.startswith('{')][-1]; pl=d['plan']
print(sys.argv[1], round(d['gpts']), round(d['ms']/d['cycles']*1e3,1), 'us/cycle', pl['order'], pl['ring'], pl['main_bands'], round(pl['tuned_ms'],3))" "$1" $O/p.json; }
for rows in 4096 8192; do
  CP_ROWS=$rows CP_AUTOTUNE=1 timeout -k 10 120 python tools/cycle_probe.py fp64 32768 20 6 > $O/p.json || exit 1; p "rows=$rows noexch"
  HEAT2D_SPLIT_ORDER=single CP_ROWS=$rows CP_AUTOTUNE=1 timeout -k 10 120 python tools/cycle_probe.py fp64 32768 20 6 > $O/p.json || exit 1; p "rows=$rows single"
  CP_ROWS=$rows CP_LOOP=1 CP_AUTOTUNE=1 timeout -k 10 120 python tools/cycle_probe.py fp64 32768 20 6 > $O/p.json || exit 1; p "rows=$rows loop"
done
