# r = 1/4 arithmetic (arith jacobi): GPU numerics, then A/B benches against the
# default (fma, bitwise the reference rounding here).
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/jac
timeout -k 10 500 python -u -m pytest tests/test_jacobi.py tests/test_arith.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/jac/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/jac/tests.log; [ $rc -eq 0 ] || exit $rc
for a in auto jacobi; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --arith $a > gpurun_out/jac/b20_$a.json 2> gpurun_out/jac/b20_$a.err || exit 1
done
for a in auto jacobi; do
  timeout -k 10 200 python -u bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 100 --arith $a > gpurun_out/jac/s4096_$a.json 2> gpurun_out/jac/s4096_$a.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/jac/s4096_$a.json')); print('$a s4096', d['value'], d['config']['cycles'])"
done
for a in auto jacobi; do
  timeout -k 10 300 python -u bench.py --dtype fp32 --steps 480 --warmup 20 --arith $a > gpurun_out/jac/f32_480_$a.json 2> gpurun_out/jac/f32_480_$a.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/jac/f32_480_$a.json')); print('$a f32_480', d['value'], d['config']['cycles'])"
  timeout -k 10 300 python -u bench.py --dtype fp64 --steps 480 --warmup 20 --arith $a > gpurun_out/jac/f64_480_$a.json 2> gpurun_out/jac/f64_480_$a.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/jac/f64_480_$a.json')); print('$a f64_480', d['value'], d['config']['cycles'])"
done
