# fma vs r = 1/4 (jacobi) kernels with fixed plans: cycle times + SQ counters.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
O=gpurun_out/jacprof
mkdir -p $O
for a in fma jacobi; do
  CP_ARITH=$a HEAT2D_SPLIT_ORDER=single HEAT2D_SEGMENTS=1007 HEAT2D_TB_RING=6 timeout -k 10 120 python tools/cycle_probe.py fp32 4096 15 40 1 1 > $O/s4096_$a.json || exit 1
  CP_ARITH=$a HEAT2D_SPLIT_ORDER=single HEAT2D_TB_RING=6 timeout -k 10 120 python tools/cycle_probe.py fp64 32768 20 3 1 0 > $O/b20_$a.json || exit 1
  CP_ARITH=$a HEAT2D_SPLIT_ORDER=single timeout -k 10 120 python tools/cycle_probe.py fp32 32768 16 4 1 0 > $O/f32_$a.json || exit 1
done
for f in $O/*.json; do python -c "import json;d=json.load(open('$f'));print('$f', round(d['gpts']), round(d['ms']/d['cycles']*1e3,1),'us/cycle')"; done
cd /tmp && export TMPDIR=/tmp
for a in fma jacobi; do
  CP_ARITH=$a HEAT2D_SPLIT_ORDER=single HEAT2D_SEGMENTS=1007 HEAT2D_TB_RING=6 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/sq_s4096_$a -- python3 $GRAFT_REPO_ROOT/tools/cycle_probe.py fp32 4096 15 10 1 0 > /dev/null || exit 1
  CP_ARITH=$a HEAT2D_SPLIT_ORDER=single HEAT2D_TB_RING=6 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/sq_b20_$a -- python3 $GRAFT_REPO_ROOT/tools/cycle_probe.py fp64 32768 20 2 1 0 > /dev/null || exit 1
done
cd $GRAFT_REPO_ROOT
for d in $O/sq_*; do echo "== $d"; python tools/prof_summary.py sq $d | tail -6; done
