#!/bin/bash
# Priming-skip general kernel (kVarPrime) for fp32 single launches: bitwise tests, fixed-plan probes, A/B of the
# autotuned small-grid bench (HEAT2D_PRIME=0 keeps the variant out of the autotuner), big-grid fp32 check.
set -o pipefail
O=gpurun_out/prime2
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_solver.py -x -q -k "prime or segment" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
show() { python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];print(sys.argv[1].split('/')[-1], d['value'], d['ms_per_step'], c['cycles'], c.get('graph'), {k:(v['order'],v.get('prime'),v['ring'],v['main_bands'],v['main_waves'],round(v['tuned_ms'],4)) for k,v in (c['launch_plans'] or {}).items()})" $1; }
probe() { python -c "import json;d=json.load(open('$1'));print('$2', round(d['gpts'],1), round(d['ms']/d['cycles']*1e3,2), 'us/cycle', d['plan']['main_items'], d['plan']['ring'])"; }
for pr in 0 1; do
  for k in 16 12; do
    HEAT2D_SPLIT_ORDER=single HEAT2D_PRIME=$pr timeout -k 10 120 python tools/cycle_probe.py fp32 4096 $k 40 1 1 > $O/p_${pr}_$k.json || exit 1
    probe $O/p_${pr}_$k.json "probe prime=$pr K=$k"
  done
done
for i in 1 2; do
  for pr in 0 1; do
    if [ $pr = 0 ]; then export HEAT2D_PRIME=0; else unset HEAT2D_PRIME; fi
    timeout -k 10 300 python bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 10 > $O/s4096_${pr}_$i.json || exit 1; show $O/s4096_${pr}_$i.json
  done
done
unset HEAT2D_PRIME
timeout -k 10 300 python bench.py --dtype fp32 --steps 480 --warmup 16 > $O/b32k_fp32.json || exit 1; show $O/b32k_fp32.json
timeout -k 10 300 python bench.py --grid 8192 --dtype fp32 --steps 1000 --warmup 10 > $O/s8192.json || exit 1; show $O/s8192.json
