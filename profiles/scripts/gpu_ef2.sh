#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/ef2
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/ef2/pytest.log 2>&1 || { tail -30 gpurun_out/ef2/pytest.log; exit 1; }
tail -1 gpurun_out/ef2/pytest.log
for R in 16384 8192 4096; do for dt in fp64 fp32; do
  timeout -k 10 200 python bench.py --dtype $dt --rehearse-comm --rows $R --steps 240 --warmup 48 > gpurun_out/ef2/${dt}_$R.json 2>/dev/null || exit 1
done; done
timeout -k 10 200 python bench.py > gpurun_out/ef2/bench.json 2>/dev/null || exit 1
echo done
