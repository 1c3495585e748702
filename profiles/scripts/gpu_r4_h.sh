# Round 4, run H: the lead order (band launch issued before the interior, no
# wait between them) on the middle-slab rehearsals: focused GPU tests, the
# autotuner's choice vs forced orders, kernel trace of a forced-lead rehearsal.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
O=gpurun_out/r4h
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_rccl.py tests/test_distributed.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
reh() {  # tag transport dtype steps env...
  tag=$1; t=$2; dt=$3; st=$4; shift 4
  env "$@" timeout -k 10 200 python -u bench.py --dtype $dt --rehearse-comm --transport $t --rows 4096 --steps $st --warmup 5 > $O/$tag.json 2> $O/$tag.err
}
for i in 1 2; do
  reh r64_rccl_auto_$i rccl fp64 20 HEAT2D_TUNE_LOG=1 || exit 1
  reh r64_rccl_lead_$i rccl fp64 20 HEAT2D_SPLIT_ORDER=lead || exit 1
  reh r64_rccl_ef_$i rccl fp64 20 HEAT2D_LEAD=0 || exit 1
  reh r64_ipc_auto_$i ipc fp64 20 || exit 1
  reh r64_ipc_lead_$i ipc fp64 20 HEAT2D_SPLIT_ORDER=lead || exit 1
done
reh r32_rccl_auto rccl fp32 480 || exit 1
reh r32_rccl_lead rccl fp32 480 HEAT2D_SPLIT_ORDER=lead || exit 1
reh r32_ipc_auto ipc fp32 480 || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || exit 1
python tools/summarize_json.py $O/*.json
P=$GRAFT_REPO_ROOT/$O
cd /tmp && export TMPDIR=/tmp
HEAT2D_SPLIT_ORDER=lead timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $P/tr -o run -- python3 $GRAFT_REPO_ROOT/bench.py --rehearse-comm --transport rccl --rows 4096 --steps 20 --warmup 5 --verify off > $P/tr.json 2> $P/tr.err || exit 1
cd $GRAFT_REPO_ROOT
python tools/trace_tail.py $P/tr/run_kernel_trace.csv 8
