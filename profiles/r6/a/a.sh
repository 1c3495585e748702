#!/bin/bash
# r6 run A: the GPU suite on the round-6 tree (transport policy, bounded IPC
# attach, per-rank proof fields, hot-spot bench, crash backtraces), smoke, the
# headline on the reference IC and on BASELINE.json's zero + hot-spot data
# (interleaved, 2 each), then the 4-rank shared-GPU 32768^2 run that stalled in
# round 5 (now: bitwise or IPC skipped within its attach limit).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6a
mkdir -p $O
export HEAT2D_PLAN_CACHE=off PYTHONFAULTHANDLER=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/h20_1.json 2> $O/h20_1.err &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --ic hotspot > $O/hot20_1.json 2> $O/hot20_1.err &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/h20_2.json 2> $O/h20_2.err &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --ic hotspot > $O/hot20_2.json 2> $O/hot20_2.err &&
{ HEAT2D_INIT_TIMEOUT=240 timeout -k 10 480 python bench.py --gpus 4 --share-gpu --steps 20 --warmup 5 \
    > $O/share4_32k.json 2> $O/share4_32k.err; echo "share4_32k rc=$?" > $O/share4_rc.txt; }
