# Dynamic item queue: numerics first, then the headline interior timeline static vs dynamic.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/dyn
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_jacobi.py -m gpu -x -q --timeout 120 --timeout-method thread -k "dynamic or single_launch or ring8" > $O/tests_dyn.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests_dyn.log; [ $rc -eq 0 ] || exit $rc
export HEAT2D_PLAN_CACHE=off
( export HEAT2D_WAVE_TIMES=1 CP_ARITH=jacobi HEAT2D_SPLIT_ORDER=edge-first HEAT2D_TB_RING=6
  HEAT2D_SEGMENTS=2048 timeout -k 10 120 python tools/wave_times.py fp64 32768 20 1 > $O/wt_seg2048.json || exit 1
  HEAT2D_SEGMENTS=8192 HEAT2D_DYNAMIC=1 timeout -k 10 120 python tools/wave_times.py fp64 32768 20 1 > $O/wt_seg8192_dyn.json || exit 1
) || exit 1
for f in $O/wt*.json; do python -c "
import json; d=json.load(open('$f')); print('$f', d['waves'], d['span_us'], d['dur_mean_us'], d['end_p50_p90_p99_max_us'], 'xcd', d['dur_by_xcd'], 'slot', d['dur_by_slot'], 'order', d['dur_by_order_eighth'])"; done
HEAT2D_DYNAMIC=2 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/b20_dyncand.json 2> $O/b20_dyncand.err || exit 1
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/b20.json 2> $O/b20.err || exit 1
for f in $O/b20*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['config']['prepare_s'], json.dumps(d['config']['launch_plans'])[:300])"; done
