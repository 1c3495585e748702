#!/bin/bash
# RCCL channel cap (NCCL_MAX_NCHANNELS) x wave slots left free (HEAT2D_SPARE_WAVES) on strong-scaling slabs, driver command.
set -o pipefail
O=gpurun_out/nch
mkdir -p $O
show() { python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];print(sys.argv[2], d['value'], {k:(v['order'],v['main_bands'],v['main_waves'],round(v['tuned_ms'],3)) for k,v in c['launch_plans'].items()})" $1 "$2"; }
for rows in 4096 8192; do
  for nch in def 1 2 4; do
    for sp in 8 32; do
      if [ $nch = def ]; then unset NCCL_MAX_NCHANNELS; else export NCCL_MAX_NCHANNELS=$nch; fi
      HEAT2D_SPARE_WAVES=$sp timeout -k 10 300 python bench.py --rehearse-comm --rows $rows --steps 20 --warmup 5 > $O/b.json || exit 1; show $O/b.json "rows=$rows nch=$nch spare=$sp"
    done
  done
done
