#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/tune2
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_solver.py > gpurun_out/tune2/pytest.log 2>&1 || { tail -30 gpurun_out/tune2/pytest.log; exit 1; }
tail -1 gpurun_out/tune2/pytest.log
for i in 1 2 3; do timeout -k 10 200 python bench.py > gpurun_out/tune2/f64_$i.json 2>/dev/null || exit 1; done
for i in 1 2; do timeout -k 10 200 python bench.py --dtype fp32 > gpurun_out/tune2/f32_$i.json 2>/dev/null || exit 1; done
for i in 1 2; do timeout -k 10 200 python bench.py --rehearse-comm --rows 4096 --steps 240 --warmup 48 > gpurun_out/tune2/reh_$i.json 2>/dev/null || exit 1; done
echo done
