#!/bin/bash
# Round-2 baseline on a fresh box: GPU tests, smoke, driver-style bench (20 steps) and the 480-step default.
set -o pipefail
mkdir -p gpurun_out/r2base
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2base/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r2base/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r2base/pytest_gpu.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r2base/b20.json || exit 1
cat gpurun_out/r2base/b20.json
timeout -k 10 200 python bench.py > gpurun_out/r2base/b480.json || exit 1
cat gpurun_out/r2base/b480.json
