#!/bin/bash
# Multi-cycle regimes (480 steps) under spare 8 vs 32 and the RCCL channel cap, interleaved.
set -o pipefail
O=gpurun_out/nch2
mkdir -p $O
show() { python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];print(sys.argv[2], d['value'], {k:(v['order'],v['main_bands'],v['main_waves']) for k,v in c['launch_plans'].items()})" $1 "$2"; }
for rep in 1 2; do
  for cfg in "def 8" "4 32" "def 32"; do
    set -- $cfg
    if [ $1 = def ]; then unset NCCL_MAX_NCHANNELS; else export NCCL_MAX_NCHANNELS=$1; fi
    HEAT2D_SPARE_WAVES=$2 timeout -k 10 300 python bench.py --dtype fp32 --rehearse-comm --rows 4096 --steps 480 --warmup 16 > $O/b.json || exit 1; show $O/b.json "fp32-4096-480 nch=$1 spare=$2"
    HEAT2D_SPARE_WAVES=$2 timeout -k 10 300 python bench.py --rehearse-comm --rows 4096 --steps 480 --warmup 16 > $O/b.json || exit 1; show $O/b.json "fp64-4096-480 nch=$1 spare=$2"
    HEAT2D_SPARE_WAVES=$2 timeout -k 10 300 python bench.py --rehearse-comm --rows 4096 --steps 20 --warmup 5 > $O/b.json || exit 1; show $O/b.json "fp64-4096-20 nch=$1 spare=$2"
  done
done
