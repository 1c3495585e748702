# Round 4, run Y: achieved DRAM traffic (rocprofv3 FETCH_SIZE / WRITE_SIZE) of
# the fp32 32768^2 pass at depth 20 (20 bands, the old limit's plan) and depth
# 24 (64 bands, this round's), the autotuner's plans of run T.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
O=gpurun_out/r4y
mkdir -p $O
P=$GRAFT_REPO_ROOT/$O
cd /tmp && export TMPDIR=/tmp
run() {  # tag k bands
  tag=$1; k=$2; b=$3
  env CP_ARITH=jacobi HEAT2D_BANDS=$b HEAT2D_TB_RING=4 HEAT2D_DYNAMIC=1 timeout -k 10 120 python3 $GRAFT_REPO_ROOT/tools/cycle_probe.py fp32 32768 $k 3 1 0 > $P/$tag.json || return 1
  for ctr in FETCH_SIZE WRITE_SIZE; do
    env CP_ARITH=jacobi HEAT2D_BANDS=$b HEAT2D_TB_RING=4 HEAT2D_DYNAMIC=1 timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $P/${tag}_$ctr -- python3 $GRAFT_REPO_ROOT/tools/cycle_probe.py fp32 32768 $k 3 1 0 > /dev/null || return 1
  done
}
run k20 20 20 || exit 1
run k24 24 64 || exit 1
cd $GRAFT_REPO_ROOT
for t in k20 k24; do
  python tools/prof_summary.py hbm $P/${t}_FETCH_SIZE $P/${t}_WRITE_SIZE $P/$t.json > $P/${t}_hbm.json && cat $P/${t}_hbm.json
  python -c "import json; d=json.load(open('$P/$t.json')); print('$t', round(d['ms']/d['cycles'],3), 'ms/cycle', round(d['gpts']), 'Gpts/s')"
done
