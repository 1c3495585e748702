#!/bin/bash
# A/B of the XCD-aware wave numbering (HEAT2D_XCD_REMAP), plus FETCH_SIZE for both
set -o pipefail
mkdir -p gpurun_out/xcd
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_solver.py > gpurun_out/xcd/pytest.log 2>&1 || { tail -30 gpurun_out/xcd/pytest.log; exit 1; }
tail -1 gpurun_out/xcd/pytest.log
for i in 1 2; do for x in 0 1; do
  HEAT2D_XCD_REMAP=$x timeout -k 10 200 python bench.py > gpurun_out/xcd/f64_x${x}_$i.json 2>/dev/null || exit 1
  HEAT2D_XCD_REMAP=$x timeout -k 10 200 python bench.py --dtype fp32 > gpurun_out/xcd/f32_x${x}_$i.json 2>/dev/null || exit 1
done; done
for x in 0 1; do
  HEAT2D_XCD_REMAP=$x timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/xcd/fetch$x -o run --output-format csv -- python3 bench.py --n 16384 --steps 120 --warmup 24 > gpurun_out/xcd/fetch$x.log 2>&1 || { tail -20 gpurun_out/xcd/fetch$x.log; exit 1; }
done
echo done
