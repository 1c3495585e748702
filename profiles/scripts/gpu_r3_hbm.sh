# Achieved DRAM traffic of the final kernels (rocprofv3 FETCH_SIZE / WRITE_SIZE, one counter per pass):
# the headline pass (32768^2 fp64 K = 20) and the fp32 depth-20 pass, against the plan model.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off CP_ARITH=jacobi
O=$GRAFT_REPO_ROOT/gpurun_out/hbm
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() {  # tag dtype n k cycles env...
  tag=$1; shift; dt=$1; n=$2; k=$3; c=$4; shift 4
  env "$@" timeout -k 10 120 python3 $GRAFT_REPO_ROOT/tools/cycle_probe.py $dt $n $k $c 1 0 > $O/$tag.json || return 1
  for ctr in FETCH_SIZE WRITE_SIZE; do
    env "$@" timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $O/${tag}_$ctr -- python3 $GRAFT_REPO_ROOT/tools/cycle_probe.py $dt $n $k $c 1 0 > /dev/null || return 1
  done
}
run b20 fp64 32768 20 2 HEAT2D_SEGMENTS=2048 HEAT2D_TB_RING=6 || exit 1
run f32k20 fp32 32768 20 3 HEAT2D_BANDS=40 HEAT2D_TB_RING=4 || exit 1
run f64k16 fp64 32768 16 3 HEAT2D_SEGMENTS=3072 HEAT2D_TB_RING=6 || exit 1
cd $GRAFT_REPO_ROOT
for t in b20 f32k20 f64k16; do
  python tools/prof_summary.py hbm $O/${t}_FETCH_SIZE $O/${t}_WRITE_SIZE $O/$t.json > $O/${t}_hbm.json && echo $t && cat $O/${t}_hbm.json
  python -c "import json; d=json.load(open('$O/$t.json')); print('$t', round(d['ms']/d['cycles'],3), 'ms/cycle', round(d['gpts']), 'Gpts/s')"
done
