#!/bin/bash
# r6 session 3, V2: the host abort (free(): invalid pointer in ~Solver, seen in
# test_bench_plan_cache_second_run's first run): the same bench run with a fresh
# plan cache, full stderr kept; stops at the first failing run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r6v2
mkdir -p $O
export PYTHONUNBUFFERED=1 OMP_NUM_THREADS=1
for i in 1 2 3 4 5 6; do
  export HEAT2D_PLAN_CACHE=/tmp/plans_v2_$i.txt
  timeout -k 10 300 python3 bench.py --gpus 1 --grid 8192 --steps 20 --warmup 5 > $O/run_$i.json 2> $O/run_$i.err
  rc=$?; echo "run $i rc=$rc $(head -c 120 $O/run_$i.json)"
  [ $rc -eq 0 ] || { echo "stopping at the first failure"; exit $rc; }
  rm -f $O/run_$i.err
done
echo done
