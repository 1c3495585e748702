# Per-wave timelines (HEAT2D_WAVE_TIMES) of the small-grid single launch and the headline pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off HEAT2D_WAVE_TIMES=1
O=gpurun_out/wt
mkdir -p $O
CP_ARITH=jacobi HEAT2D_SPLIT_ORDER=single HEAT2D_SEGMENTS=1007 HEAT2D_TB_RING=6 timeout -k 10 60 python tools/wave_times.py fp32 4096 16 4 > $O/s4096_k16.json || exit 1
CP_ARITH=jacobi HEAT2D_SPLIT_ORDER=single HEAT2D_SEGMENTS=1007 HEAT2D_TB_RING=6 timeout -k 10 60 python tools/wave_times.py fp32 4096 15 4 > $O/s4096_k15.json || exit 1
CP_ARITH=jacobi HEAT2D_SPLIT_ORDER=single HEAT2D_SEGMENTS=2014 HEAT2D_TB_RING=6 timeout -k 10 60 python tools/wave_times.py fp32 4096 16 4 > $O/s4096_k16_2014.json || exit 1
CP_ARITH=jacobi HEAT2D_SPLIT_ORDER=single HEAT2D_BANDS=48 HEAT2D_TB_RING=6 timeout -k 10 60 python tools/wave_times.py fp32 4096 16 4 > $O/s4096_k16_b48.json || exit 1
CP_ARITH=jacobi HEAT2D_SPLIT_ORDER=single HEAT2D_SEGMENTS=1007 HEAT2D_TB_RING=6 timeout -k 10 60 python tools/wave_times.py fp64 4096 12 4 > $O/d4096_k12.json || exit 1
for f in $O/*.json; do cat $f; echo; done
