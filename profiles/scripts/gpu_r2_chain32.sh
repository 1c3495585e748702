#!/bin/bash
# fp32 chained march (chains of 4 / 8 levels, builds in exp/) vs one chain, at 1 wave/SIMD segment plans.
set -o pipefail
O=gpurun_out/chain32
mkdir -p $O
for v in base c4 c8; do
  if [ $v = base ]; then unset HEAT2D_LIB; else export HEAT2D_LIB=$PWD/exp/$v/libheat2d.so; fi
  for ring in 4 6; do
    HEAT2D_SPLIT_ORDER=single HEAT2D_SEGMENTS=1007 HEAT2D_TB_RING=$ring timeout -k 10 120 python tools/cycle_probe.py fp32 4096 16 40 1 1 > $O/p.json || exit 1
    python -c "import json;d=json.load(open('$O/p.json'));print('$v ring$ring probe', round(d['gpts']), round(d['ms']/d['cycles']*1e3,1),'us/cycle')"
  done
  timeout -k 10 300 python bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 50 > $O/b.json || exit 1
  python -c "import json;d=json.load(open('$O/b.json'));c=d['config'];print('$v bench4096', d['value'], c['cycles'], {k:(v['order'],v['ring'],v['main_bands'],v['main_waves']) for k,v in c['launch_plans'].items()})"
done
for v in base c4; do
  if [ $v = base ]; then unset HEAT2D_LIB; else export HEAT2D_LIB=$PWD/exp/$v/libheat2d.so; fi
  timeout -k 10 300 python bench.py --dtype fp32 --steps 480 --warmup 16 > $O/b.json || exit 1
  python -c "import json;d=json.load(open('$O/b.json'));c=d['config'];print('$v bench32768', d['value'], c['cycles'], {k:(v['order'],v['ring'],v['main_bands'],v['main_waves']) for k,v in c['launch_plans'].items()})"
done
