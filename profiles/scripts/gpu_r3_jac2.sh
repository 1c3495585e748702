# r = 1/4 kernels after the kind-1 fix: numerics, fixed-plan cycle times, benches.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/jac2
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_jacobi.py tests/test_arith.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
export HEAT2D_PLAN_CACHE=off
for a in fma jacobi; do
  CP_ARITH=$a HEAT2D_SPLIT_ORDER=single HEAT2D_SEGMENTS=1007 HEAT2D_TB_RING=6 timeout -k 10 120 python tools/cycle_probe.py fp32 4096 15 40 1 1 > $O/s4096_$a.json || exit 1
  CP_ARITH=$a HEAT2D_SPLIT_ORDER=single timeout -k 10 120 python tools/cycle_probe.py fp32 32768 16 4 1 0 > $O/f32_$a.json || exit 1
  CP_ARITH=$a HEAT2D_SPLIT_ORDER=single HEAT2D_TB_RING=6 timeout -k 10 120 python tools/cycle_probe.py fp64 32768 20 3 1 0 > $O/b20s_$a.json || exit 1
done
for f in $O/*.json; do python -c "import json;d=json.load(open('$f'));print('$f', round(d['gpts']), round(d['ms']/d['cycles']*1e3,1),'us/cycle')"; done
unset HEAT2D_PLAN_CACHE
for a in auto jacobi; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --arith $a > $O/b20_$a.out 2> $O/b20_$a.err || exit 1
  timeout -k 10 200 python -u bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 100 --arith $a > $O/s4096b_$a.out 2> $O/s4096b_$a.err || exit 1
  timeout -k 10 300 python -u bench.py --dtype fp32 --steps 480 --warmup 20 --arith $a > $O/f32b_$a.out 2> $O/f32b_$a.err || exit 1
done
for f in $O/*.out; do python -c "import json; d=json.load(open('$f')); print('$f', d['value'], json.dumps(d['config']['launch_plans']))"; done
