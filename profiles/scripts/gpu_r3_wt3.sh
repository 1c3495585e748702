# Per-wave timeline of the headline's interior launch (edge-first order: the interior is the last launch).
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off HEAT2D_WAVE_TIMES=1 CP_ARITH=jacobi HEAT2D_SPLIT_ORDER=edge-first HEAT2D_TB_RING=6
O=gpurun_out/wt3
mkdir -p $O
HEAT2D_SEGMENTS=2048 timeout -k 10 120 python tools/wave_times.py fp64 32768 20 1 > $O/b20_seg2048.json || exit 1
HEAT2D_SEGMENTS=1865 timeout -k 10 120 python tools/wave_times.py fp64 32768 20 1 > $O/b20_seg1865.json || exit 1
HEAT2D_BANDS=16 HEAT2D_TB_RING=4 timeout -k 10 120 python tools/wave_times.py fp64 32768 20 1 > $O/b20_b16_r4.json || exit 1
for f in $O/*.json; do python -c "
import json; d=json.load(open('$f')); print('$f', d['waves'], d['span_us'], d['dur_mean_us'], d['dur_max_us'], d['end_p50_p90_p99_max_us'], [(r['rect'][:4], r['waves'], r['dur_mean_us'], r['dur_max_us']) for r in d['per_rect']])"; done
