#!/bin/bash
# fp64 across-lane moves on the LDS crossbar (ds_bpermute) vs DPP moves: bitwise suite per build, interleaved
# driver-command benches, fixed-plan K = 20 / 16 probes. Builds: tools/build_ab_f64.sh xl1|xl2 (HEAT2D_XLANE_F64=1|2).
set -o pipefail
O=gpurun_out/xlane
mkdir -p $O
export PYTHONUNBUFFERED=1
L1=build_ab/xl1/libheat2d.so; L2=build_ab/xl2/libheat2d.so
for l in $L1 $L2; do
  HEAT2D_LIB=$l timeout -k 10 300 python -u -m pytest tests/test_gpu_solver.py -x -q --timeout 120 --timeout-method thread > $O/pytest_$(basename $(dirname $l)).log 2>&1 || { tail -30 $O/pytest_$(basename $(dirname $l)).log; exit 1; }
  tail -1 $O/pytest_$(basename $(dirname $l)).log
done
show() { python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];print(sys.argv[1].split('/')[-1], d['value'], d['ms_per_step'], c['cycles'], {k:(v['order'],v['ring'],v['main_bands'],v['main_waves'],round(v['tuned_ms'],3)) for k,v in (c['launch_plans'] or {}).items()})" $1; }
probe() { python -c "import json;d=json.load(open('$1'));print('$2', round(d['gpts'],1), round(d['ms']/d['cycles'],3), 'ms/cycle', d['plan']['order'], d['plan']['main_items'], d['plan']['ring'])"; }
for i in 1 2; do
  for l in default $L1 $L2; do
    t=$(basename $(dirname $l)); [ $l = default ] && t=dpp
    if [ $l = default ]; then unset HEAT2D_LIB; else export HEAT2D_LIB=$l; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/b20_${t}_$i.json || exit 1; show $O/b20_${t}_$i.json
  done
done
for l in default $L1 $L2; do
  t=$(basename $(dirname $l)); [ $l = default ] && t=dpp
  if [ $l = default ]; then unset HEAT2D_LIB; else export HEAT2D_LIB=$l; fi
  for k in 20 16; do
    timeout -k 10 120 python tools/cycle_probe.py fp64 32768 $k 3 > $O/p_${t}_$k.json || exit 1; probe $O/p_${t}_$k.json "probe $t K=$k"
  done
  timeout -k 10 300 python bench.py --steps 480 --warmup 16 > $O/b480_${t}.json || exit 1; show $O/b480_${t}.json
done
