#!/bin/bash
# After the boundary-band kernel: GPU suite, small grid, headline benches, 8-rank slab rehearsals.
set -o pipefail
O=gpurun_out/edge
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
show() { python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];print(sys.argv[1].split('/')[-1], d['value'], d['ms_per_step'], c['cycles'], {k:(v['order'],v['main_bands'],v['main_waves'],v['edge_items']) for k,v in (c['launch_plans'] or {}).items()})" $1; }
timeout -k 10 300 python bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 10 > $O/s4096.json || exit 1; show $O/s4096.json
timeout -k 10 300 python bench.py --dtype fp32 --steps 480 --warmup 5 > $O/f32.json || exit 1; show $O/f32.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/b20.json || exit 1; show $O/b20.json
timeout -k 10 300 python bench.py --steps 480 --warmup 5 > $O/b480.json || exit 1; show $O/b480.json
timeout -k 10 300 python bench.py --dtype fp32 --rehearse-comm --rows 4096 --steps 480 --warmup 16 > $O/r32.json || exit 1; show $O/r32.json
timeout -k 10 300 python bench.py --rehearse-comm --rows 4096 --steps 480 --warmup 16 > $O/r64.json || exit 1; show $O/r64.json
