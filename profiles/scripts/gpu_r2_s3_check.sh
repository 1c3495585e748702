#!/bin/bash
# Re-entry check of the rebuilt tree: GPU suite, smoke, driver bench command.
set -o pipefail
O=gpurun_out/s3check
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputests.log 2>&1 || { tail -30 $O/gputests.log; exit 1; }
tail -3 $O/gputests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { cat $O/bench20.err; exit 1; }
cat $O/bench20.json
