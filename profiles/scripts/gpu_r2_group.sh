#!/bin/bash
# Group march (fp64 interior kernel over 4-strip super-strips sharing edge columns through LDS): bitwise suite,
# fixed-plan probes group vs plain (HEAT2D_GROUP=1|0), interleaved driver-command benches (autotuner with / without
# group candidates), 480-step bench.
set -o pipefail
O=gpurun_out/group
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_solver.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
show() { python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];print(sys.argv[1].split('/')[-1], d['value'], d['ms_per_step'], c['cycles'], d['hbm_gb_per_s_plan'], {k:(v['order'],v.get('group'),v['ring'],v['main_bands'],v['main_waves'],round(v['tuned_ms'],3)) for k,v in (c['launch_plans'] or {}).items()})" $1; }
probe() { python -c "import json;d=json.load(open('$1'));p=d['plan'];print('$2', round(d['gpts'],1), round(d['ms']/d['cycles'],3), 'ms/cycle', p['order'], p.get('group'), p['main_items'], p['main_waves'], p['ring'])"; }
for k in 20 16 14; do
  for g in 0 1; do
    HEAT2D_GROUP=$g timeout -k 10 120 python tools/cycle_probe.py fp64 32768 $k 3 > $O/p_${g}_$k.json || exit 1; probe $O/p_${g}_$k.json "probe group=$g K=$k"
  done
done
for i in 1 2; do
  for g in 0 auto; do
    if [ $g = 0 ]; then export HEAT2D_GROUP=0; else unset HEAT2D_GROUP; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/b20_${g}_$i.json || exit 1; show $O/b20_${g}_$i.json
  done
done
unset HEAT2D_GROUP
timeout -k 10 300 python bench.py --steps 480 --warmup 16 > $O/b480.json || exit 1; show $O/b480.json
