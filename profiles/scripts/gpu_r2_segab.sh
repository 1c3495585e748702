#!/bin/bash
# Segment candidates in the autotuner on/off (HEAT2D_TUNE_SEGMENTS), interleaved, whole-grid benches.
set -o pipefail
O=gpurun_out/segab
mkdir -p $O
show() { python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];print(sys.argv[2], d['value'], c['cycles'], {k:(v['order'],v['ring'],v['main_bands'],v['main_waves']) for k,v in c['launch_plans'].items()})" $1 "$2"; }
for rep in 1 2; do
  for seg in 1 0; do
    HEAT2D_TUNE_SEGMENTS=$seg timeout -k 10 300 python bench.py --dtype fp32 --steps 480 --warmup 16 > $O/b.json || exit 1; show $O/b.json "seg=$seg fp32-480"
    HEAT2D_TUNE_SEGMENTS=$seg timeout -k 10 300 python bench.py --steps 480 --warmup 16 > $O/b.json || exit 1; show $O/b.json "seg=$seg fp64-480"
    HEAT2D_TUNE_SEGMENTS=$seg timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/b.json || exit 1; show $O/b.json "seg=$seg fp64-20"
  done
done
