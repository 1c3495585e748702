# Persistent launch over frame-weighted rects + frame-weight sweep + small-grid benches.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/persist4
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_persistent.py tests/test_jacobi.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
export HEAT2D_PLAN_CACHE=off
for wr in 1.5 1.7; do
  for wc in 1.4 1.6 1.75; do
    HEAT2D_W_ROW=$wr HEAT2D_W_COL=$wc CP_ARITH=jacobi HEAT2D_SPLIT_ORDER=single HEAT2D_SEGMENTS=1007 HEAT2D_TB_RING=6 timeout -k 10 60 python tools/cycle_probe.py fp32 4096 16 40 1 1 > $O/s4096_k16_r${wr}_c${wc}.json || exit 1
  done
done
for f in $O/*.json; do python -c "import json;d=json.load(open('$f'));print('$f', round(d['gpts']), round(d['ms']/d['cycles']*1e3,1),'us/cycle', d['plan']['main_items'])"; done
for p in 0 1; do
  HEAT2D_PERSIST=$p timeout -k 10 200 python -u bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 100 > $O/s4096b_p$p.out 2> $O/s4096b_p$p.err || exit 1
  HEAT2D_PERSIST=$p timeout -k 10 200 python -u bench.py --grid 4096 --dtype fp64 --steps 1000 --warmup 100 > $O/d4096b_p$p.out 2> $O/d4096b_p$p.err || exit 1
  HEAT2D_PERSIST=$p timeout -k 10 200 python -u bench.py --grid 8192 --dtype fp32 --steps 1000 --warmup 100 > $O/s8192b_p$p.out 2> $O/s8192b_p$p.err || exit 1
done
timeout -k 10 200 python -u bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 100 > $O/s4096b_auto.out 2> $O/s4096b_auto.err || exit 1
for f in $O/*.out; do python -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['config']['cycles'], d['config']['prepare_s'], json.dumps(d['config']['launch_plans'])[:300])"; done
