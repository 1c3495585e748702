#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/bal
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/bal/pytest.log 2>&1 || { tail -30 gpurun_out/bal/pytest.log; exit 1; }
tail -1 gpurun_out/bal/pytest.log
for S in 100 50 480; do
  timeout -k 10 200 python bench.py --steps $S --warmup 10 > gpurun_out/bal/f64_s$S.json 2>/dev/null || exit 1
done
echo done
