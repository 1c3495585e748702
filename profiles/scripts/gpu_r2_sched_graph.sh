#!/bin/bash
# prepare(n) times near-tied schedules as captured graphs of trial cycles: GPU suite, small-grid benches, headline.
set -o pipefail
O=gpurun_out/${SG_OUT:-sched_graph}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputests.log 2>&1 || { tail -30 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
show() { python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];print(sys.argv[1].split('/')[-1], d['value'], d['ms_per_step'], c['cycles'], c['prepare_s'])" $1; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --grid 4096 --dtype fp64 --steps 1000 --warmup 10 > $O/d4096_$i.json || exit 1; show $O/d4096_$i.json
  timeout -k 10 300 python bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 10 > $O/s4096_$i.json || exit 1; show $O/s4096_$i.json
done
timeout -k 10 300 python bench.py --grid 8192 --dtype fp64 --steps 1000 --warmup 10 > $O/d8192.json || exit 1; show $O/d8192.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/b20.json || exit 1; show $O/b20.json
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
