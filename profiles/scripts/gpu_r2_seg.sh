#!/bin/bash
# Segment work items: bitwise tests, then thin-slab rehearsals + whole-grid benches.
set -o pipefail
O=gpurun_out/seg
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_solver.py tests/test_ops.py -m gpu \
  -k "segment or tile_rows or split_orders or guard or loopback_group" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
show() { python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];print(sys.argv[2], d['value'], c['cycles'], {k:(v['order'],v['ring'],v['main_bands'],v['main_waves'],v['edge_items']) for k,v in (c['launch_plans'] or {}).items()})" $1 "$2"; }
for dt in fp32 fp64; do
  for rows in 4096 8192; do
    timeout -k 10 300 python bench.py --dtype $dt --rehearse-comm --rows $rows --steps 480 --warmup 16 > $O/r.json || exit 1; show $O/r.json "$dt rows=$rows"
  done
done
timeout -k 10 300 python bench.py --dtype fp32 --steps 480 --warmup 16 > $O/r.json || exit 1; show $O/r.json "fp32 whole"
timeout -k 10 300 python bench.py --steps 480 --warmup 16 > $O/r.json || exit 1; show $O/r.json "fp64 whole-480"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/r.json || exit 1; show $O/r.json "fp64 whole-20"
timeout -k 10 300 python bench.py --dtype fp32 --n 4096 --steps 1000 --warmup 50 > $O/r.json || exit 1; show $O/r.json "fp32 4096^2"
