set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off HEAT2D_WAVE_TIMES=1
O=gpurun_out/r4f; mkdir -p $O
for cfg in "edge-first 1" "fused 1" "fused 0"; do
  set -- $cfg
  HEAT2D_SPLIT_ORDER=$1 HEAT2D_FUSED_BALANCE=$2 HEAT2D_BANDS=8 HEAT2D_TB_RING=6 timeout -k 10 120 python -u tools/wave_times_slab.py fp64 32768 4096 20 3 | tee $O/wt_$1_$2.json || exit 1
done
