#!/bin/bash
# Full GPU suite + smoke + driver bench command.
set -o pipefail
O=gpurun_out/full
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/suite.log 2>&1 || { tail -40 $O/suite.log; exit 1; }
tail -2 $O/suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 || exit 1
