# Frame-column weight sweep (fp32 4096^2, K = 16, 1007 segments), then the
# thin-slab rehearsals (one rank of 8 at 32768^2) against the whole grid, r = 1/4.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/sweep5
mkdir -p $O
export HEAT2D_PLAN_CACHE=off
for wc in 1.0 1.15 1.3 1.4 1.5 1.4b; do
  HEAT2D_W_ROW=1.5 HEAT2D_W_COL=${wc%b} CP_ARITH=jacobi HEAT2D_SPLIT_ORDER=single HEAT2D_SEGMENTS=1007 HEAT2D_TB_RING=6 timeout -k 10 60 python tools/cycle_probe.py fp32 4096 16 40 1 1 > $O/s4096_k16_c${wc}.json || exit 1
done
for f in $O/*.json; do python -c "import json;d=json.load(open('$f'));print('$f', round(d['gpts']), round(d['ms']/d['cycles']*1e3,1),'us/cycle', d['plan']['main_items'])"; done
unset HEAT2D_PLAN_CACHE
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/whole64_20.out 2> $O/whole64_20.err || exit 1
timeout -k 10 200 python -u bench.py --rehearse-comm --rows 4096 --steps 20 --warmup 5 > $O/reh64_20_rccl.out 2> $O/reh64_20_rccl.err || exit 1
timeout -k 10 200 python -u bench.py --rehearse-comm --rows 4096 --steps 20 --warmup 5 --transport peer > $O/reh64_20_ipc.out 2> $O/reh64_20_ipc.err || exit 1
timeout -k 10 300 python -u bench.py --dtype fp32 --steps 480 --warmup 20 > $O/whole32_480.out 2> $O/whole32_480.err || exit 1
timeout -k 10 200 python -u bench.py --dtype fp32 --rehearse-comm --rows 4096 --steps 480 --warmup 20 > $O/reh32_480_rccl.out 2> $O/reh32_480_rccl.err || exit 1
timeout -k 10 200 python -u bench.py --dtype fp32 --rehearse-comm --rows 4096 --steps 480 --warmup 20 --transport peer > $O/reh32_480_ipc.out 2> $O/reh32_480_ipc.err || exit 1
for f in $O/*.out; do python -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['config']['cycles'], d['config']['transport'], json.dumps(d['config']['launch_plans'])[:200])"; done
