#!/bin/bash
# Per-rank cost of the multi-GPU schedule (RCCL self-exchange rehearsal) at 2/4/8-rank slab shapes, both dtypes.
set -o pipefail
O=gpurun_out/thin
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_rccl.py tests/test_distributed.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
show() { python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];print(sys.argv[1].split('/')[-1], d['value'], c['grid'], c['cycles'], {k:(v['order'],v['main_bands'],v['main_waves'],v['edge_items']) for k,v in (c['launch_plans'] or {}).items()})" $1; }
for dt in fp32 fp64; do
  for rows in 4096 8192 16384; do
    timeout -k 10 300 python bench.py --dtype $dt --rehearse-comm --rows $rows --steps 480 --warmup 16 > $O/r_${dt}_$rows.json || exit 1; show $O/r_${dt}_$rows.json
  done
done
timeout -k 10 300 python bench.py --dtype fp32 --steps 480 --warmup 5 > $O/whole32.json || exit 1; show $O/whole32.json
timeout -k 10 300 python bench.py --steps 480 --warmup 5 > $O/whole64.json || exit 1; show $O/whole64.json
