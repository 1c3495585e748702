#!/bin/bash
# fp64 strong-scaling slabs with the RCCL self-exchange: autotuned order vs forced concurrent / edge-first.
set -o pipefail
O=gpurun_out/order
mkdir -p $O
show() { python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];print(sys.argv[2], d['value'], c['cycles'], {k:(v['order'],v['main_bands']) for k,v in c['launch_plans'].items()})" $1 "$2"; }
for rows in 4096 8192; do
  for st in "480 16" "20 5"; do
    set -- $st
    for o in auto concurrent edge-first; do
      if [ $o = auto ]; then unset HEAT2D_SPLIT_ORDER; else export HEAT2D_SPLIT_ORDER=$o; fi
      timeout -k 10 300 python bench.py --rehearse-comm --rows $rows --steps $1 --warmup $2 > $O/b.json || exit 1; show $O/b.json "rows=$rows steps=$1 order=$o"
    done
  done
done
