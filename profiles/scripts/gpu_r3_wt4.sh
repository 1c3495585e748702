# Where the headline interior launch's slow waves are (by XCD / SIMD slot / launch order).
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off HEAT2D_WAVE_TIMES=1 CP_ARITH=jacobi HEAT2D_SPLIT_ORDER=edge-first HEAT2D_TB_RING=6
O=gpurun_out/wt4
mkdir -p $O
HEAT2D_SEGMENTS=2048 timeout -k 10 120 python tools/wave_times.py fp64 32768 20 1 > $O/b20_seg2048.json || exit 1
HEAT2D_SEGMENTS=2048 HEAT2D_XCD_REMAP=1 timeout -k 10 120 python tools/wave_times.py fp64 32768 20 1 > $O/b20_seg2048_xcd.json || exit 1
HEAT2D_SEGMENTS=4096 timeout -k 10 120 python tools/wave_times.py fp64 32768 20 1 > $O/b20_seg4096.json || exit 1
for f in $O/*.json; do python -c "
import json; d=json.load(open('$f')); print('$f', d['waves'], d['span_us'], d['dur_mean_us'], d['end_p50_p90_p99_max_us'], 'xcd', d['dur_by_xcd'], 'slot', d['dur_by_slot'], 'order', d['dur_by_order_eighth'])"; done
