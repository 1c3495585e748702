#!/bin/bash
# edge-first split ordering (valid = 3): correctness with real exchanges, then the 2/4/8-rank slab rehearsals
set -o pipefail
mkdir -p gpurun_out/ef
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_solver.py tests/test_gpu_rccl.py tests/test_distributed.py -m gpu > gpurun_out/ef/pytest.log 2>&1 || { tail -30 gpurun_out/ef/pytest.log; exit 1; }
tail -1 gpurun_out/ef/pytest.log
for R in 16384 8192 4096; do for o in auto edge-first concurrent; do
  if [ $o = auto ]; then unset HEAT2D_SPLIT_ORDER; else export HEAT2D_SPLIT_ORDER=$o; fi
  timeout -k 10 200 python bench.py --rehearse-comm --rows $R --steps 240 --warmup 48 --phase-timers > gpurun_out/ef/f64_${R}_$o.json 2>/dev/null || exit 1
done; done
unset HEAT2D_SPLIT_ORDER
for o in auto edge-first; do
  if [ $o = auto ]; then unset HEAT2D_SPLIT_ORDER; else export HEAT2D_SPLIT_ORDER=$o; fi
  timeout -k 10 200 python bench.py --dtype fp32 --rehearse-comm --rows 4096 --steps 240 --warmup 48 --phase-timers > gpurun_out/ef/f32_4096_$o.json 2>/dev/null || exit 1
done
echo done
