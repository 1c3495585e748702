# fp32 depths 17..20 (HBM-bound big fp32 grids): numerics, then big-grid benches K <= 16 vs K <= 20.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/f32deep
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_jacobi.py tests/test_gpu_solver.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
export HEAT2D_PLAN_CACHE=off
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --dtype fp32 --steps 480 --warmup 20 > $O/f32_480_k20_$i.json 2> $O/f32_480_k20_$i.err || exit 1
  timeout -k 10 300 python -u bench.py --dtype fp32 --steps 480 --warmup 20 --tb 16 > $O/f32_480_k16_$i.json 2> $O/f32_480_k16_$i.err || exit 1
done
timeout -k 10 300 python -u bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 100 > $O/s4096.json 2> $O/s4096.err || exit 1
timeout -k 10 600 python -u bench/configs.py --only gpu-max-fp32 > $O/max_fp32.jsonl 2> $O/max_fp32.err || exit 1
for f in $O/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['config']['cycles'], d['config']['prepare_s'], json.dumps(d['config']['launch_plans'])[:250])"; done
cat $O/max_fp32.jsonl | cut -c1-400
