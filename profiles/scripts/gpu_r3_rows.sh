# Frame-row weighted single-launch plans (stencil_tb.hip weighted_main): numerics,
# fixed-plan cycle times (single launch, segments), and the small-grid / headline benches.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/rows
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_jacobi.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
export HEAT2D_PLAN_CACHE=off
for w in 1.0 1.3 1.5 1.7; do
  HEAT2D_W_ROW=$w CP_ARITH=jacobi HEAT2D_SPLIT_ORDER=single HEAT2D_SEGMENTS=1007 HEAT2D_TB_RING=6 timeout -k 10 120 python tools/cycle_probe.py fp32 4096 15 40 1 1 > $O/s4096_w$w.json || exit 1
done
CP_ARITH=fma HEAT2D_SPLIT_ORDER=single HEAT2D_SEGMENTS=1007 HEAT2D_TB_RING=6 timeout -k 10 120 python tools/cycle_probe.py fp32 4096 15 40 1 1 > $O/s4096_fma.json || exit 1
for w in 1.0 1.4; do
  HEAT2D_W_ROW=$w CP_ARITH=jacobi HEAT2D_SPLIT_ORDER=single HEAT2D_TB_RING=6 timeout -k 10 120 python tools/cycle_probe.py fp64 32768 20 3 1 0 > $O/b20s_w$w.json || exit 1
done
for f in $O/*.json; do python -c "import json;d=json.load(open('$f'));print('$f', round(d['gpts']), round(d['ms']/d['cycles']*1e3,1),'us/cycle', d['plan']['main_items'])"; done
unset HEAT2D_PLAN_CACHE
timeout -k 10 200 python -u bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 100 > $O/s4096b.out 2> $O/s4096b.err || exit 1
HEAT2D_SPLIT_ORDER=single timeout -k 10 200 python -u bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 100 > $O/s4096b_single.out 2> $O/s4096b_single.err || exit 1
timeout -k 10 200 python -u bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 100 --arith auto > $O/s4096b_fma.out 2> $O/s4096b_fma.err || exit 1
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/b20.out 2> $O/b20.err || exit 1
for f in $O/*.out; do python -c "import json; d=json.load(open('$f')); print('$f', d['value'], json.dumps(d['config']['launch_plans']))"; done
