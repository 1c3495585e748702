# Ring 8 for the fp32 single launch (small grid): numerics, fixed-plan cycles, timeline, benches.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/ring8
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_jacobi.py -m gpu -x -q --timeout 120 --timeout-method thread -k "ring8 or single_launch" > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
export HEAT2D_PLAN_CACHE=off CP_ARITH=jacobi HEAT2D_SPLIT_ORDER=single HEAT2D_SEGMENTS=1007
for r in 6 8; do
  for k in 15 16; do
    HEAT2D_TB_RING=$r timeout -k 10 60 python tools/cycle_probe.py fp32 4096 $k 40 1 1 > $O/s4096_k${k}_r$r.json || exit 1
  done
  HEAT2D_WAVE_TIMES=1 HEAT2D_TB_RING=$r timeout -k 10 60 python tools/wave_times.py fp32 4096 16 4 > $O/wt_k16_r$r.json || exit 1
done
for f in $O/s4096*.json; do python -c "import json;d=json.load(open('$f'));print('$f', round(d['gpts']), round(d['ms']/d['cycles']*1e3,1),'us/cycle')"; done
for f in $O/wt*.json; do python -c "import json;d=json.load(open('$f'));print('$f', d['span_us'], d['dur_mean_us'])"; done
unset HEAT2D_PLAN_CACHE HEAT2D_SPLIT_ORDER HEAT2D_SEGMENTS CP_ARITH
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 100 > $O/s4096b_$i.json 2> $O/s4096b_$i.err || exit 1
done
for f in $O/s4096b*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['config']['cycles'], json.dumps(d['config']['launch_plans'])[:300])"; done
