# Round 4, run K: the first cycle of every step() in the lead order
# (HEAT2D_LEAD_FIRST=0: off) — GPU tests, interleaved slab rehearsals A/B,
# IPC with and without graphs, headline.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
O=gpurun_out/r4k
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_rccl.py tests/test_distributed.py tests/test_gpu_solver.py tests/test_jacobi.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
reh() {  # tag transport dtype steps extra-args env...
  tag=$1; t=$2; dt=$3; st=$4; xa=$5; shift 5
  env "$@" timeout -k 10 200 python -u bench.py --dtype $dt --rehearse-comm --transport $t --rows 4096 --steps $st --warmup 5 $xa > $O/$tag.json 2> $O/$tag.err
}
for i in 1 2 3; do
  reh r64_rccl_$i rccl fp64 20 "" || exit 1
  reh r64_rccl_off_$i rccl fp64 20 "" HEAT2D_LEAD_FIRST=0 || exit 1
done
for i in 1 2; do
  reh r64_ipc_$i ipc fp64 20 "" || exit 1
  reh r64_ipc_eager_$i ipc fp64 20 "--graph off" || exit 1
  reh r64_ipc_off_$i ipc fp64 20 "" HEAT2D_LEAD_FIRST=0 || exit 1
done
reh r32_rccl rccl fp32 480 "" || exit 1
reh r32_rccl_off rccl fp32 480 "" HEAT2D_LEAD_FIRST=0 || exit 1
reh r32_ipc ipc fp32 480 "" || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || exit 1
python tools/summarize_json.py $O/*.json
