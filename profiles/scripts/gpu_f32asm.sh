#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/f32asm
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_solver.py tests/test_ops.py tests/test_arith.py > gpurun_out/f32asm/pytest.log 2>&1 || { tail -30 gpurun_out/f32asm/pytest.log; exit 1; }
tail -1 gpurun_out/f32asm/pytest.log
for i in 1 2; do timeout -k 10 200 python bench.py --dtype fp32 > gpurun_out/f32asm/f32_$i.json 2>/dev/null || exit 1; done
timeout -k 10 200 python bench.py --dtype fp32 --n 4096 --steps 960 --warmup 96 > gpurun_out/f32asm/f32_4096.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --dtype fp32 --rehearse-comm --rows 4096 --steps 240 --warmup 48 > gpurun_out/f32asm/reh.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --weak --dtype fp32 --n 173056 --steps 64 --warmup 16 > gpurun_out/f32asm/weak.json 2>/dev/null || exit 1
echo done
