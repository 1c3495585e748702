#!/bin/bash
# Full GPU check: pytest -m gpu, smoke, headline bench, all BASELINE configs.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 200 python bench.py > gpurun_out/bench_fp64.json || exit 1
cat gpurun_out/bench_fp64.json
timeout -k 10 200 python bench.py --dtype fp32 > gpurun_out/bench_fp32.json || exit 1
cat gpurun_out/bench_fp32.json
timeout -k 10 600 python bench/configs.py > gpurun_out/configs.jsonl || exit 1
cat gpurun_out/configs.jsonl
