# fp32 ring 10 / fp64 ring 8 single launches: numerics, timelines, benches.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/ring10
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_jacobi.py -m gpu -x -q --timeout 120 --timeout-method thread -k "ring8" > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
export HEAT2D_PLAN_CACHE=off CP_ARITH=jacobi HEAT2D_SPLIT_ORDER=single
for r in 8 10; do
  HEAT2D_SEGMENTS=1007 HEAT2D_WAVE_TIMES=1 HEAT2D_TB_RING=$r timeout -k 10 60 python tools/wave_times.py fp32 4096 16 4 > $O/wt_k16_r$r.json || exit 1
  HEAT2D_SEGMENTS=1007 HEAT2D_TB_RING=$r timeout -k 10 60 python tools/cycle_probe.py fp32 4096 16 40 1 1 > $O/s4096_k16_r$r.json || exit 1
done
for r in 6 8; do
  HEAT2D_SEGMENTS=1000 HEAT2D_WAVE_TIMES=1 HEAT2D_TB_RING=$r timeout -k 10 60 python tools/wave_times.py fp64 4096 12 4 > $O/wt_d_k12_r$r.json || exit 1
done
for f in $O/s4096*.json; do python -c "import json;d=json.load(open('$f'));print('$f', round(d['gpts']), round(d['ms']/d['cycles']*1e3,1),'us/cycle')"; done
for f in $O/wt*.json; do python -c "
import json; d=json.load(open('$f')); print('$f', d['span_us'], d['dur_mean_us'], [(r['rect'][:4], r['dur_mean_us'], r['dur_max_us']) for r in d['per_rect']])"; done
unset HEAT2D_PLAN_CACHE HEAT2D_SPLIT_ORDER CP_ARITH
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 100 > $O/s4096b_$i.json 2> $O/s4096b_$i.err || exit 1
done
timeout -k 10 200 python -u bench.py --grid 4096 --dtype fp64 --steps 1000 --warmup 100 > $O/d4096b.json 2> $O/d4096b.err || exit 1
for f in $O/*b*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['config']['cycles'], json.dumps(d['config']['launch_plans'])[:300])"; done
