# Round 4, run P: the driver's multi-GPU command shape on the 1-GPU box —
# torchrun with N rank processes sharing the GPU (--share-gpu): transport
# selection (RCCL refuses, IPC), fallback, verification and the JSON line, at
# N = 2 and 8 (throughput meaningless: the ranks time-share one GPU).
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
O=gpurun_out/r4p
mkdir -p $O
for n in 2 8; do
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 29$((500 + n)) bench.py --gpus $n --steps 20 --warmup 5 --share-gpu > $O/share$n.json 2> $O/share$n.err || { echo "n=$n failed"; tail -30 $O/share$n.err; exit 1; }
  cat $O/share$n.json
done
