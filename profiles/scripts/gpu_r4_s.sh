# Round 4, run S: fp32 temporal depths 21..24 (the packed interior kernel keeps
# 2 waves/SIMD to K = 24): bitwise GPU tests at the new depths, then the
# HBM-bound fp32 configurations (32768^2 480 steps, the 240 GB grid, the
# 8-rank slab rehearsal) with the schedule search free to take them.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
O=gpurun_out/r4s
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_jacobi.py tests/test_arith_fast.py tests/test_gpu_solver.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench/configs.py --only gpu-32768-fp32 gpu-max-fp32 > $O/configs.jsonl 2> $O/configs.err || exit 1
cat $O/configs.jsonl | python -c "import sys,json; [print(d['config'], d['gpts'], d.get('cycles'), d.get('prepare_s'), d.get('hbm_gb_per_s_plan')) for d in map(json.loads, sys.stdin)]"
timeout -k 10 300 python -u bench.py --dtype fp32 --steps 480 --warmup 20 > $O/b32_480.json 2> $O/b32_480.err || exit 1
timeout -k 10 300 python -u bench.py --dtype fp32 --rehearse-comm --rows 4096 --steps 480 --warmup 20 > $O/reh32_480.json 2> $O/reh32_480.err || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || exit 1
python tools/summarize_json.py $O/*.json
