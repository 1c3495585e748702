# SQ wait counters of the headline pass (32768^2 fp64 K = 20, split plan, r = 1/4).
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off CP_ARITH=jacobi HEAT2D_TB_RING=6 HEAT2D_SEGMENTS=2048
O=gpurun_out/hlprof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/a -- python3 $GRAFT_REPO_ROOT/tools/cycle_probe.py fp64 32768 20 2 1 0 > $GRAFT_REPO_ROOT/$O/a.json || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/b -- python3 $GRAFT_REPO_ROOT/tools/cycle_probe.py fp64 32768 20 2 1 0 > $GRAFT_REPO_ROOT/$O/b.json || exit 1
cd $GRAFT_REPO_ROOT
for d in a b; do python tools/prof_summary.py sq $O/$d > $O/sq_$d.json; python -c "
import json; d=json.load(open('$O/sq_$d.json')); print('$d', {k: v for k, v in d.items() if k != 'SQ_totals'}, {k: round(v) for k, v in d['SQ_totals'].items()})"; done
