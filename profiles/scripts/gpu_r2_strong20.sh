#!/bin/bash
# The driver's command (20 steps, 5 warmup) on the per-rank slabs of strong scaling (N = 2/4/8), RCCL self-exchange.
set -o pipefail
O=gpurun_out/strong20
mkdir -p $O
show() { python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];print(sys.argv[2], d['value'], d['ms_per_step'], 'prep', round(c.get('prepare_s',0),1), c['cycles'], {k:(v['order'],v['ring'],v['main_bands'],v['main_waves'],round(v['tuned_ms'],3)) for k,v in (c['launch_plans'] or {}).items()})" $1 "$2"; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/r1.json || exit 1; show $O/r1.json "N=1 whole"
for rows in 16384 8192 4096; do
  timeout -k 10 300 python bench.py --rehearse-comm --rows $rows --steps 20 --warmup 5 > $O/r$rows.json || exit 1; show $O/r$rows.json "rows=$rows"
  timeout -k 10 300 python bench.py --rehearse-comm --rows $rows --steps 20 --warmup 5 --phase-timers > $O/t$rows.json || exit 1; python -c "import json;d=json.load(open('$O/t$rows.json'));print('  phases', d['config'].get('phases'))"
done
