# Round 4, run J: host-side timeline (HIP API + kernels) of the timed single
# cycle of the middle-slab rehearsal, RCCL (eager) and IPC (graph), lead order.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
O=gpurun_out/r4j
mkdir -p $O
P=$GRAFT_REPO_ROOT/$O
cd /tmp && export TMPDIR=/tmp
for t in rccl ipc; do
  HEAT2D_SPLIT_ORDER=lead timeout -s KILL 200 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $P/tr_$t -o run -- python3 $GRAFT_REPO_ROOT/bench.py --rehearse-comm --transport $t --rows 4096 --steps 20 --warmup 5 --verify off > $P/tr_$t.json 2> $P/tr_$t.err || exit 1
done
echo done
