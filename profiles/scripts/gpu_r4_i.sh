# Round 4, run I: high-priority comm stream (bands + exchange dispatched first
# when both streams become ready together) — slab rehearsals per order,
# headline A/B (HEAT2D_COMM_PRIORITY=0), kernel trace of an IPC lead rehearsal.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
O=gpurun_out/r4i
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_rccl.py tests/test_distributed.py tests/test_gpu_solver.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
reh() {  # tag transport dtype steps env...
  tag=$1; t=$2; dt=$3; st=$4; shift 4
  env "$@" timeout -k 10 200 python -u bench.py --dtype $dt --rehearse-comm --transport $t --rows 4096 --steps $st --warmup 5 > $O/$tag.json 2> $O/$tag.err
}
for i in 1 2; do
  reh r64_rccl_auto_$i rccl fp64 20 || exit 1
  reh r64_rccl_lead_$i rccl fp64 20 HEAT2D_SPLIT_ORDER=lead || exit 1
  reh r64_rccl_lead_np_$i rccl fp64 20 HEAT2D_SPLIT_ORDER=lead HEAT2D_COMM_PRIORITY=0 || exit 1
  reh r64_ipc_lead_$i ipc fp64 20 HEAT2D_SPLIT_ORDER=lead || exit 1
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench20_$i.json 2> $O/bench20_$i.err || exit 1
  HEAT2D_COMM_PRIORITY=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench20_np_$i.json 2> $O/bench20_np_$i.err || exit 1
done
reh r32_rccl_auto rccl fp32 480 || exit 1
reh r32_rccl_np rccl fp32 480 HEAT2D_COMM_PRIORITY=0 || exit 1
reh r32_ipc_auto ipc fp32 480 || exit 1
timeout -k 10 300 python -u bench.py --steps 480 --warmup 20 --dtype fp32 > $O/b32_480.json 2> $O/b32_480.err || exit 1
python tools/summarize_json.py $O/*.json
P=$GRAFT_REPO_ROOT/$O
cd /tmp && export TMPDIR=/tmp
HEAT2D_SPLIT_ORDER=lead timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $P/tr -o run -- python3 $GRAFT_REPO_ROOT/bench.py --rehearse-comm --transport ipc --rows 4096 --steps 20 --warmup 5 --verify off > $P/tr.json 2> $P/tr.err || exit 1
cd $GRAFT_REPO_ROOT
python tools/trace_tail.py $P/tr/run_kernel_trace.csv 14
