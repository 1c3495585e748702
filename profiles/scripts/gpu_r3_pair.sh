# Wave-pair kernel: numerics, fixed-plan cycle times (single vs pair), small-grid benches.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/pair
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_jacobi.py -m gpu -x -q --timeout 120 --timeout-method thread -k pair > $O/tests_pair.log 2>&1
rc=$?; echo "pair tests rc=$rc"; tail -3 $O/tests_pair.log; [ $rc -eq 0 ] || exit $rc
export HEAT2D_PLAN_CACHE=off
for k in 14 15 16; do
  for pr in 0 1; do
    for ring in 4 6; do
      HEAT2D_PAIR=$pr CP_ARITH=jacobi HEAT2D_SPLIT_ORDER=single HEAT2D_SEGMENTS=1007 HEAT2D_TB_RING=$ring timeout -k 10 60 python tools/cycle_probe.py fp32 4096 $k 40 1 1 > $O/s4096_k${k}_p${pr}_r${ring}.json || exit 1
    done
  done
done
HEAT2D_PAIR=1 CP_ARITH=jacobi HEAT2D_SPLIT_ORDER=single HEAT2D_SEGMENTS=2014 HEAT2D_TB_RING=6 timeout -k 10 60 python tools/cycle_probe.py fp32 4096 16 40 1 1 > $O/s4096_k16_p1_r6_seg2014.json || exit 1
for f in $O/*.json; do python -c "import json;d=json.load(open('$f'));print('$f', round(d['gpts']), round(d['ms']/d['cycles']*1e3,1),'us/cycle', d['plan']['main_items'], d['plan']['main_waves'])"; done
unset HEAT2D_PLAN_CACHE
timeout -k 10 200 python -u bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 100 > $O/s4096b.out 2> $O/s4096b.err || exit 1
HEAT2D_PAIR=0 timeout -k 10 200 python -u bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 100 > $O/s4096b_nopair.out 2> $O/s4096b_nopair.err || exit 1
timeout -k 10 200 python -u bench.py --grid 8192 --dtype fp32 --steps 1000 --warmup 100 > $O/s8192b.out 2> $O/s8192b.err || exit 1
for f in $O/*.out; do python -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['config']['cycles'], json.dumps(d['config']['launch_plans'])[:400])"; done
timeout -k 10 600 python -u -m pytest tests/test_jacobi.py tests/test_persistent.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
