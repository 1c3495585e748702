#!/bin/bash
# A/B: fp64 neighbour shifts by DPP (default lib) vs ds_bpermute (ab/libheat2d_bp.so)
set -o pipefail
mkdir -p gpurun_out/bp
export PYTHONUNBUFFERED=1
BP=$GRAFT_REPO_ROOT/cuda-hip-mpi-heat-equation-test_amd/_native/ab/libheat2d_bp.so
HEAT2D_LIB=$BP timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_solver.py -k fp64 > gpurun_out/bp/pytest.log 2>&1 || { tail -30 gpurun_out/bp/pytest.log; exit 1; }
tail -1 gpurun_out/bp/pytest.log
for K in 12 14 16; do
  timeout -k 10 200 python bench.py --tb $K > gpurun_out/bp/dpp_k$K.json 2>/dev/null || exit 1
  HEAT2D_LIB=$BP timeout -k 10 200 python bench.py --tb $K > gpurun_out/bp/bp_k$K.json 2>/dev/null || exit 1
done
echo done
