#!/bin/bash
# Measured-schedule choice on the cache-resident 4096^2 grids: autotuned schedule (--tb 0) vs depth caps, interleaved.
set -o pipefail
O=gpurun_out/sched_small
mkdir -p $O
export PYTHONUNBUFFERED=1
show() { python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];print(sys.argv[1].split('/')[-1], d['value'], d['ms_per_step'], c['cycles'], {k:round(v['tuned_ms']/int(k)*1e3,3) for k,v in (c['launch_plans'] or {}).items()})" $1; }
for i in 1 2; do
  for tb in 0 12 14; do
    timeout -k 10 300 python bench.py --grid 4096 --dtype fp64 --steps 1000 --warmup 10 --tb $tb > $O/d_${tb}_$i.json || exit 1; show $O/d_${tb}_$i.json
  done
done
for i in 1 2; do
  for tb in 0 13; do
    timeout -k 10 300 python bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 10 --tb $tb > $O/s_${tb}_$i.json || exit 1; show $O/s_${tb}_$i.json
  done
done
