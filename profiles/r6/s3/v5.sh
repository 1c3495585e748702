#!/bin/bash
# r6 session 3, V5: the driver's N = 8 command shape on one GPU: bench.py --gpus 8
# --share-gpu at the headline grid (32768^2 fp64, 20 steps): 8 rank processes,
# RCCL refused -> IPC, the edge-balance rehearsal rank by rank, the timed field
# checked over all ranks.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r6v5
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
timeout -k 10 900 python3 bench.py --gpus 8 --share-gpu --steps 20 --warmup 5 > $O/b8_share.json 2> $O/b8_share.err
rc=$?; echo "bench 8 ranks share-gpu rc=$rc $(head -c 120 $O/b8_share.json | tail -c 50)"
exit $rc
