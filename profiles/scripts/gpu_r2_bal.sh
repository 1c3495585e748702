#!/bin/bash
# SIMD-balanced band chooser: fixed-plan probes, then the benches and slab rehearsals.
set -o pipefail
O=gpurun_out/bal
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_solver.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in "fp32 4096 16 40 1 0" "fp32 4096 12 40 1 0" "fp32 4096 16 40 1 1" "fp32 32768 16 4 1 0" "fp64 32768 14 4 1 0"; do
  timeout -k 10 120 python tools/cycle_probe.py $cfg > $O/p.json || exit 1
  python -c "import json;d=json.load(open('$O/p.json'));print('$cfg', round(d['gpts'],1), 'Gpts/s', round(d['ms']/d['cycles']*1e3,2),'us/cycle', d['plan'].get('order'), d['plan'].get('main_bands'), d['plan'].get('main_waves'))"
done
show() { python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];print(sys.argv[1].split('/')[-1], d['value'], d['ms_per_step'], c['cycles'], {k:(v['order'],v['main_bands'],v['main_waves'],v['edge_items']) for k,v in (c['launch_plans'] or {}).items()})" $1; }
timeout -k 10 300 python bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 10 > $O/s4096.json || exit 1; show $O/s4096.json
timeout -k 10 300 python bench.py --dtype fp32 --steps 480 --warmup 5 > $O/f32.json || exit 1; show $O/f32.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/b20.json || exit 1; show $O/b20.json
timeout -k 10 300 python bench.py --steps 480 --warmup 5 > $O/b480.json || exit 1; show $O/b480.json
timeout -k 10 300 python bench.py --dtype fp32 --rehearse-comm --rows 4096 --steps 480 --warmup 16 > $O/r32.json || exit 1; show $O/r32.json
