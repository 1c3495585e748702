# Frame weights sweep (HEAT2D_W_ROW / HEAT2D_W_COL) on the 1007-segment single
# launch, depths 14-16, then the small-grid bench with strip-aligned segment
# candidates in the autotuner.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/rows2
mkdir -p $O
export HEAT2D_PLAN_CACHE=off
for k in 14 15 16; do
  for wr in 1.7 2.0; do
    for wc in 1.75 2.0 2.3; do
      HEAT2D_W_ROW=$wr HEAT2D_W_COL=$wc CP_ARITH=jacobi HEAT2D_SPLIT_ORDER=single HEAT2D_SEGMENTS=1007 HEAT2D_TB_RING=6 timeout -k 10 60 python tools/cycle_probe.py fp32 4096 $k 40 1 1 > $O/s4096_k${k}_r${wr}_c${wc}.json || exit 1
    done
  done
done
for f in $O/*.json; do python -c "import json;d=json.load(open('$f'));print('$f', round(d['gpts']), round(d['ms']/d['cycles']*1e3,1),'us/cycle', d['plan']['main_items'])"; done
unset HEAT2D_PLAN_CACHE
timeout -k 10 200 python -u bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 100 > $O/s4096b.out 2> $O/s4096b.err || exit 1
HEAT2D_W_ROW=2.0 HEAT2D_W_COL=2.0 timeout -k 10 200 python -u bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 100 > $O/s4096b_w2.out 2> $O/s4096b_w2.err || exit 1
timeout -k 10 200 python -u bench.py --grid 4096 --dtype fp64 --steps 1000 --warmup 100 > $O/d4096b.out 2> $O/d4096b.err || exit 1
timeout -k 10 200 python -u bench.py --grid 4096 --dtype fp64 --steps 1000 --warmup 100 --arith auto > $O/d4096b_fma.out 2> $O/d4096b_fma.err || exit 1
for f in $O/*.out; do python -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['config']['cycles'], json.dumps(d['config']['launch_plans']))"; done
