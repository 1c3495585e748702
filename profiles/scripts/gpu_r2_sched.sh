#!/bin/bash
# Full GPU suite, then the driver's bench command and the long default with measured schedules.
set -o pipefail
mkdir -p gpurun_out/sched
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/sched/pytest.log 2>&1 || { tail -40 gpurun_out/sched/pytest.log; exit 1; }
tail -2 gpurun_out/sched/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
for st in 20 480; do
  timeout -k 10 300 python bench.py --steps $st --warmup 5 > gpurun_out/sched/b$st.json || exit 1
  cat gpurun_out/sched/b$st.json
done
