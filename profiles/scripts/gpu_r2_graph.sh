#!/bin/bash
# graph default off + pair graph built in prepare(): suite subset, small grid eager vs graph, headline benches.
set -o pipefail
O=gpurun_out/graph
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_solver.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
show() { python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];print(sys.argv[1].split('/')[-1], d['value'], d['ms_per_step'], c['cycles'], c.get('graph'), {k:(v['order'],v['main_bands'],v['main_waves'],v['edge_items']) for k,v in (c['launch_plans'] or {}).items()})" $1; }
for g in off on; do
  timeout -k 10 300 python bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 10 --graph $g > $O/s4096_$g.json || exit 1; show $O/s4096_$g.json
done
for i in 1 2; do timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/b20_$i.json || exit 1; show $O/b20_$i.json; done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --graph on > $O/b20_g.json || exit 1; show $O/b20_g.json
timeout -k 10 300 python bench.py --steps 480 --warmup 5 > $O/b480.json || exit 1; show $O/b480.json
for g in 0 1; do timeout -k 10 120 python tools/cycle_probe.py fp32 4096 16 40 1 $g > $O/p.json || exit 1; python -c "import json;d=json.load(open('$O/p.json'));print('probe graph=$g', round(d['gpts'],1), round(d['ms']/d['cycles']*1e3,2), 'us/cycle')"; done
