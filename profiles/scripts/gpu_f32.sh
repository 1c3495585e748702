#!/bin/bash
# packed-fp32 march: fp32 bitwise tests, then fp32 benches (32768^2 K=10/12/14, 4096^2 graph config)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_solver.py tests/test_ops.py tests/test_arith.py -k "fp32 or float32 or f32" > gpurun_out/pytest_f32.log 2>&1 || { tail -40 gpurun_out/pytest_f32.log; exit 1; }
tail -3 gpurun_out/pytest_f32.log
for K in 10 12 14 16; do
  timeout -k 10 200 python bench.py --dtype fp32 --tb $K > gpurun_out/f32_k$K.json 2>gpurun_out/f32_k$K.err || { cat gpurun_out/f32_k$K.err; exit 1; }
  cat gpurun_out/f32_k$K.json
done
timeout -k 10 200 python bench.py > gpurun_out/f64_default.json 2>/dev/null || exit 1
cat gpurun_out/f64_default.json
