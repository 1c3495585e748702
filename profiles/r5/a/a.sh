#!/bin/bash
# r5 run A: host overhead of the one-cycle slab region (probe_host), API timeline, baseline bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5a
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err && \
timeout -k 10 200 python3 tools/probe_host.py --transport rccl --json $O/probe_rccl.json > $O/probe_rccl.log 2>&1 && \
timeout -k 10 200 python3 tools/probe_host.py --transport ipc --json $O/probe_ipc.json > $O/probe_ipc.log 2>&1 && \
timeout -k 10 200 python3 tools/probe_host.py --transport self --rows 32768 --json $O/probe_self.json > $O/probe_self.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/trace -- python3 $GRAFT_REPO_ROOT/tools/probe_host.py --transport rccl --reps 3 > $GRAFT_REPO_ROOT/$O/trace.log 2>&1
echo done rc=$?
