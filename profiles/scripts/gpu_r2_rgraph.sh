#!/bin/bash
# Full GPU suite; then RCCL graph-capture probes (1-rank loop) and rehearsals with --graph on; 8-rank weak shape.
set -o pipefail
O=gpurun_out/rgraph
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/suite.log 2>&1 || { tail -40 $O/suite.log; exit 1; }
tail -2 $O/suite.log
show() { python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];print(sys.argv[2], d['value'], c['cycles'], c.get('graph'), {k:(v['order'],v['main_bands'],v['main_waves']) for k,v in (c['launch_plans'] or {}).items()})" $1 "$2"; }
timeout -k 10 300 python bench.py --rehearse-comm --rows 11585 --n 92682 --steps 100 --warmup 10 > $O/r.json || exit 1; show $O/r.json "fp64 weak-8 slab 11585x92682"
for o in concurrent edge-first; do
  HEAT2D_RCCL_GRAPH=1 timeout -k 10 120 python tools/graph_rccl_probe.py $o || exit 1
done
for dt in fp32 fp64; do
  timeout -k 10 300 python bench.py --dtype $dt --rehearse-comm --rows 4096 --steps 480 --warmup 16 > $O/r.json || exit 1; show $O/r.json "$dt 4096 eager"
  HEAT2D_RCCL_GRAPH=1 timeout -k 10 300 python bench.py --dtype $dt --rehearse-comm --rows 4096 --steps 480 --warmup 16 --graph on > $O/r.json || exit 1; show $O/r.json "$dt 4096 graph"
done
