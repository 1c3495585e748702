#!/bin/bash
# Loopback / RCCL-loop GPU tests, then the fp64 depth sweep K = 12..24 at 32768^2:
# one pass (steps = K) and steady state (steps = 8K).
set -o pipefail
mkdir -p gpurun_out/deep
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_solver.py tests/test_gpu_rccl.py -x -q --timeout 120 --timeout-method thread > gpurun_out/deep/pytest.log 2>&1 || { tail -40 gpurun_out/deep/pytest.log; exit 1; }
tail -2 gpurun_out/deep/pytest.log
for k in 12 14 16 18 20 22 24; do
  timeout -k 10 200 python bench.py --tb $k --steps $k --warmup $k > gpurun_out/deep/one_$k.json || exit 1
  timeout -k 10 200 python bench.py --tb $k --steps $((8*k)) --warmup $k > gpurun_out/deep/st_$k.json || exit 1
  python - $k <<'PY'
import json,sys
k=sys.argv[1]
for f in ("one","st"):
    d=json.load(open(f"gpurun_out/deep/{f}_{k}.json"))
    pl=d["config"]["launch_plans"]
    print(f, k, d["value"], d["ms_per_step"], d["config"]["cycles"], {kk:(v["order"],v["ring"],v["main_bands"],round(v["tuned_ms"],3)) for kk,v in pl.items()})
PY
done
