#!/bin/bash
# r5 run B: new GPU tests (field check, memory plan, transport fallback, measure-hbm),
# headline with measured HBM, full-HBM weak grid (memory-fit planner) + its 8-rank slab rehearsal
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5b
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
timeout -k 10 900 python3 -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_memory_plan.py tests/test_bench_contract.py tests/test_cli.py tests/test_runner.py \
  -k "memory or footprint or plan_max or field_check or measure_hbm or falls_back or auto_transport" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; fatal $rc
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 --measure-hbm > $O/bench20_hbm.json 2> $O/bench20_hbm.err
rc=$?; echo "bench20_hbm rc=$rc"; fatal $rc
timeout -k 10 600 python3 bench.py --weak --dtype fp32 --grid max --steps 64 --warmup 8 > $O/weak_max_fp32.json 2> $O/weak_max_fp32.err
rc=$?; echo "weak_max rc=$rc"; fatal $rc
N8=$(timeout -k 10 120 python3 -c "import heat2d; from heat2d.utils import memplan; print(memplan.plan_max_grid('fp32', 8, device=0)['n'])") && \
echo "N8=$N8" > $O/n8.txt && \
timeout -k 10 600 python3 bench.py --rehearse-comm --grid $N8 --rows $((N8 / 8)) --dtype fp32 --steps 64 --warmup 8 > $O/weak_max_fp32_slab8.json 2> $O/weak_max_fp32_slab8.err
echo done rc=$?
