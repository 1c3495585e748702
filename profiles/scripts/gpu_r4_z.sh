# Round 4, run Z: SQ counters of this round's headline pass (32768^2 fp64,
# depth 20, r = 1/4 form, 8 row bands on the dynamic queue, ring 6) and of the
# sigma = 0.2 fast pass: VALU utilisation, wait fractions (one rocprofv3 pass
# per counter group).
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
O=gpurun_out/r4z
mkdir -p $O
P=$GRAFT_REPO_ROOT/$O
cd /tmp && export TMPDIR=/tmp
for cfg in "jac jacobi 0.25" "fast fast 0.2"; do
  set -- $cfg
  tag=$1; ar=$2; sg=$3
  env CP_ARITH=$ar CP_SIGMA=$sg HEAT2D_BANDS=8 HEAT2D_TB_RING=6 HEAT2D_DYNAMIC=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $P/${tag}_a -- python3 $GRAFT_REPO_ROOT/tools/cycle_probe.py fp64 32768 20 2 1 0 > $P/${tag}_a.json || exit 1
  env CP_ARITH=$ar CP_SIGMA=$sg HEAT2D_BANDS=8 HEAT2D_TB_RING=6 HEAT2D_DYNAMIC=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM --kernel-trace --output-format csv -d $P/${tag}_b -- python3 $GRAFT_REPO_ROOT/tools/cycle_probe.py fp64 32768 20 2 1 0 > $P/${tag}_b.json || exit 1
done
cd $GRAFT_REPO_ROOT
for t in jac_a jac_b fast_a fast_b; do python tools/prof_summary.py sq $P/$t > $P/${t}_sq.json && echo $t && cat $P/${t}_sq.json; done
