# SQ counters of the 4096^2 fp32 K = 16 single launch: one wave per item vs the wave pair.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off CP_ARITH=jacobi HEAT2D_SPLIT_ORDER=single HEAT2D_SEGMENTS=1007 HEAT2D_TB_RING=6
O=gpurun_out/pairprof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for pr in 0 1; do
  HEAT2D_PAIR=$pr timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/a_p$pr -- python3 $GRAFT_REPO_ROOT/tools/cycle_probe.py fp32 4096 16 10 1 0 > /dev/null || exit 1
  HEAT2D_PAIR=$pr timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/b_p$pr -- python3 $GRAFT_REPO_ROOT/tools/cycle_probe.py fp32 4096 16 10 1 0 > /dev/null || exit 1
done
cd $GRAFT_REPO_ROOT
for d in $O/*_p*; do echo "== $d"; python tools/prof_summary.py sq $d; done
