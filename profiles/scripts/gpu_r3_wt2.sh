# Frame-row weight re-check from per-wave timelines (fp32 W_ROW 1.3 / 1.5; fp64 aligned segments).
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off HEAT2D_WAVE_TIMES=1 CP_ARITH=jacobi HEAT2D_SPLIT_ORDER=single HEAT2D_TB_RING=6
O=gpurun_out/wt2
mkdir -p $O
for w in 1.2 1.3; do
  HEAT2D_W_ROW=$w HEAT2D_SEGMENTS=1007 timeout -k 10 60 python tools/wave_times.py fp32 4096 16 4 > $O/s4096_k16_wr$w.json || exit 1
done
for w in 1.2 1.4; do
  HEAT2D_W_ROW=$w HEAT2D_SEGMENTS=1000 timeout -k 10 60 python tools/wave_times.py fp64 4096 12 4 > $O/d4096_k12_wr$w.json || exit 1
done
HEAT2D_BANDS=46 timeout -k 10 60 python tools/wave_times.py fp64 4096 12 4 > $O/d4096_k12_b46.json || exit 1
for f in $O/*.json; do python -c "
import json; d=json.load(open('$f')); print('$f', d['span_us'], d['dur_mean_us'], [(r['rect'][:2]+r['rect'][2:4], r['dur_mean_us'], r['dur_max_us']) for r in d['per_rect']])"; done
unset HEAT2D_WAVE_TIMES HEAT2D_SPLIT_ORDER HEAT2D_TB_RING CP_ARITH
for w in 1.3 1.5; do
  HEAT2D_W_ROW=$w timeout -k 10 200 python -u bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 100 > $O/s4096b_wr$w.out 2> $O/s4096b_wr$w.err || exit 1
done
for f in $O/*.out; do python -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['config']['cycles'], json.dumps(d['config']['launch_plans'])[:300])"; done
