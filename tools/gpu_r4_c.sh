# Round 4 profiles: kernel trace + stats of the headline bench, and achieved
# DRAM traffic (rocprofv3 FETCH_SIZE / WRITE_SIZE, one counter per pass) of the
# headline pass (32768^2 fp64 K = 20, r = 1/4 kernels) and of the sigma = 0.2
# fast-arith pass, against the plan model.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
O=$GRAFT_REPO_ROOT/gpurun_out/r4c
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --verify off > $O/trace_bench.json 2> $O/trace.err || exit 1
run() {  # tag dtype n k cycles env...
  tag=$1; shift; dt=$1; n=$2; k=$3; c=$4; shift 4
  env "$@" timeout -k 10 120 python3 $GRAFT_REPO_ROOT/tools/cycle_probe.py $dt $n $k $c 1 0 > $O/$tag.json || return 1
  for ctr in FETCH_SIZE WRITE_SIZE; do
    env "$@" timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $O/${tag}_$ctr -- python3 $GRAFT_REPO_ROOT/tools/cycle_probe.py $dt $n $k $c 1 0 > /dev/null || return 1
  done
}
run b20 fp64 32768 20 2 CP_ARITH=jacobi HEAT2D_BANDS=8 HEAT2D_TB_RING=6 HEAT2D_DYNAMIC=1 || exit 1
run fast20 fp64 32768 20 2 CP_ARITH=fast CP_SIGMA=0.2 HEAT2D_BANDS=8 HEAT2D_TB_RING=6 HEAT2D_DYNAMIC=1 || exit 1
cd $GRAFT_REPO_ROOT
for t in b20 fast20; do
  python tools/prof_summary.py hbm $O/${t}_FETCH_SIZE $O/${t}_WRITE_SIZE $O/$t.json > $O/${t}_hbm.json && echo $t && cat $O/${t}_hbm.json
  python -c "import json; d=json.load(open('$O/$t.json')); print('$t', round(d['ms']/d['cycles'],3), 'ms/cycle', round(d['gpts']), 'Gpts/s')"
done
python tools/prof_summary.py trace $O/trace > $O/trace_summary.txt; head -30 $O/trace_summary.txt
