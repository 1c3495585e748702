# fma vs jacobi: which item kinds are slow? kernel traces of split plans (MAIN:
# kinds 0/2, EDGE: bands, kinds 1/3) at 4096^2 and 32768^2 fp32.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
O=gpurun_out/jacprof2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for a in fma jacobi; do
  CP_ARITH=$a HEAT2D_SPLIT_ORDER=concurrent timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/t4096_$a -- python3 $GRAFT_REPO_ROOT/tools/cycle_probe.py fp32 4096 15 20 1 0 > $GRAFT_REPO_ROOT/$O/t4096_$a.json || exit 1
  CP_ARITH=$a HEAT2D_SPLIT_ORDER=concurrent timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/t32k_$a -- python3 $GRAFT_REPO_ROOT/tools/cycle_probe.py fp32 32768 16 3 1 0 > $GRAFT_REPO_ROOT/$O/t32k_$a.json || exit 1
  CP_ARITH=$a HEAT2D_SPLIT_ORDER=single timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/s32k_$a -- python3 $GRAFT_REPO_ROOT/tools/cycle_probe.py fp32 32768 16 3 1 0 > $GRAFT_REPO_ROOT/$O/s32k_$a.json || exit 1
done
cd $GRAFT_REPO_ROOT
for d in $O/t4096_* $O/t32k_* $O/s32k_*; do [ -d $d ] || continue; echo "== $d"; python tools/prof_summary.py trace $d | python -c "
import json,sys
for r in json.load(sys.stdin)[-6:]: print('  ', r)"; done
