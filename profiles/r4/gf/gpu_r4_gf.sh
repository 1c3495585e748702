# Round 4, run GF: per-step-count graph / eager decision (long-cycle measured
# schedules launch eagerly). Graph-path GPU tests, then interleaved A/B of the
# default (auto: eager for the headline's one 4.3 ms cycle) vs --graph on
# (the previous behaviour: replay every schedule): headline x3, fp32 32768^2
# 480 steps x2, small grid x2 (stays replayed).
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r4gf
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_solver.py tests/test_bench_contract.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
export HEAT2D_PLAN_CACHE=off
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b20_auto_$i.json 2> $O/b20_auto_$i.err || exit 1
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --graph on > $O/b20_on_$i.json 2> $O/b20_on_$i.err || exit 1
done
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --dtype fp32 --steps 480 --warmup 20 > $O/b32_auto_$i.json 2> $O/b32_auto_$i.err || exit 1
  timeout -k 10 300 python -u bench.py --dtype fp32 --steps 480 --warmup 20 --graph on > $O/b32_on_$i.json 2> $O/b32_on_$i.err || exit 1
done
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 100 > $O/small_$i.json 2> $O/small_$i.err || exit 1
done
python tools/summarize_json.py $O/*.json
