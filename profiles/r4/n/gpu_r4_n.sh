# Round 4, run N: per-wave timeline of the headline interior launch (32768^2
# fp64, depth 20, the autotuner's usual plan: ring 6, 8 bands, dynamic queue)
# and of the static-item variant (edge-first order: the interior is the last launch).
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off HEAT2D_WAVE_TIMES=1 CP_ARITH=jacobi HEAT2D_SPLIT_ORDER=edge-first
O=gpurun_out/r4n
mkdir -p $O
HEAT2D_BANDS=8 HEAT2D_TB_RING=6 HEAT2D_DYNAMIC=1 timeout -k 10 120 python -u tools/wave_times.py fp64 32768 20 2 > $O/wt_dyn.json || exit 1
HEAT2D_BANDS=8 HEAT2D_TB_RING=6 HEAT2D_DYNAMIC=0 timeout -k 10 120 python -u tools/wave_times.py fp64 32768 20 2 > $O/wt_static.json || exit 1
HEAT2D_BANDS=11 HEAT2D_TB_RING=6 HEAT2D_DYNAMIC=1 timeout -k 10 120 python -u tools/wave_times.py fp64 32768 20 2 > $O/wt_dyn11.json || exit 1
cat $O/*.json
