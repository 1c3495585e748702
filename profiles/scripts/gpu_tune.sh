#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/tune
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_solver.py > gpurun_out/tune/pytest.log 2>&1 || { tail -30 gpurun_out/tune/pytest.log; exit 1; }
tail -1 gpurun_out/tune/pytest.log
timeout -k 10 200 python bench.py > gpurun_out/tune/f64.json || exit 1
timeout -k 10 200 python bench.py --dtype fp32 > gpurun_out/tune/f32.json || exit 1
timeout -k 10 600 python bench/configs.py --only gpu-max gpu-4096 gpu-16384 > gpurun_out/tune/configs.jsonl || exit 1
cat gpurun_out/tune/configs.jsonl | cut -c1-300
