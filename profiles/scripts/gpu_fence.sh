#!/bin/bash
# A/B: packed fp32 across-lane adds as fenced C++ (compiler-combined DPP, default lib) vs hand asm (ab lib)
set -o pipefail
mkdir -p gpurun_out/fence
export PYTHONUNBUFFERED=1
ASM=$GRAFT_REPO_ROOT/cuda-hip-mpi-heat-equation-test_amd/_native/ab/libheat2d_asm.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_solver.py tests/test_ops.py tests/test_arith.py > gpurun_out/fence/pytest.log 2>&1 || { tail -30 gpurun_out/fence/pytest.log; exit 1; }
tail -1 gpurun_out/fence/pytest.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --dtype fp32 > gpurun_out/fence/fence_$i.json 2>/dev/null || exit 1
  HEAT2D_LIB=$ASM timeout -k 10 200 python bench.py --dtype fp32 > gpurun_out/fence/asm_$i.json 2>/dev/null || exit 1
done
timeout -k 10 200 python bench.py --dtype fp32 --rehearse-comm --rows 4096 --steps 240 --warmup 48 > gpurun_out/fence/reh_fence.json 2>/dev/null || exit 1
HEAT2D_LIB=$ASM timeout -k 10 200 python bench.py --dtype fp32 --rehearse-comm --rows 4096 --steps 240 --warmup 48 > gpurun_out/fence/reh_asm.json 2>/dev/null || exit 1
echo done
