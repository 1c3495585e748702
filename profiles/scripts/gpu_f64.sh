#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/f64
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_solver.py -k "fp64" > gpurun_out/f64/pytest.log 2>&1 || { tail -30 gpurun_out/f64/pytest.log; exit 1; }
tail -1 gpurun_out/f64/pytest.log
for i in 1 2; do
timeout -k 10 200 python bench.py > gpurun_out/f64/auto_$i.json || exit 1
HEAT2D_TB_RING=4 timeout -k 10 200 python bench.py > gpurun_out/f64/r4_$i.json || exit 1
done
timeout -k 10 200 python bench.py --rehearse-comm --rows 4096 --steps 240 --warmup 48 > gpurun_out/f64/reh4096.json || exit 1
cat gpurun_out/f64/*.json | cut -c1-200
