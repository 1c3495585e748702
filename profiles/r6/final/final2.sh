#!/bin/bash
# r6 FINAL 2 (the round's final tree): the BASELINE configs at 480 / 1000
# steps (the no-flag bench.py is the 32768^2 480-step row), general r
# (sigma 0.2: fast and exact), the small grid three times plus its kernel
# trace, the fp32 8-rank slab, and the full-HBM fp32 grid.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6final2
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
b() { tag=$1; shift; timeout -k 10 400 python3 bench.py "$@" > $O/$tag.json 2> $O/$tag.err; rc=$?; echo "$tag rc=$rc $(head -c 130 $O/$tag.json | tail -c 60)"; fatal $rc; }
b noflag
b f64_16k_480 --grid 16384 --steps 480 --warmup 48
b f32_32k_480 --dtype fp32 --steps 480 --warmup 48
b s02_fast --steps 20 --warmup 5 --sigma 0.2 --arith fast
b s02_exact --steps 20 --warmup 5 --sigma 0.2 --arith exact
for i in 1 2 3; do b small_$i --grid 4096 --dtype fp32 --steps 1000 --warmup 64; done
cd /tmp && export TMPDIR=/tmp
mkdir -p $GRAFT_REPO_ROOT/$O/trace_small && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/trace_small -o small -- python3 $GRAFT_REPO_ROOT/bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 64 --verify off --field-check off > $GRAFT_REPO_ROOT/$O/trace_small/bench.json 2> $GRAFT_REPO_ROOT/$O/trace_small/bench.err
rc=$?; echo "trace rc=$rc"; fatal $rc
db=$(find $GRAFT_REPO_ROOT/$O/trace_small -name "*.db" | head -1)
[ -n "$db" ] && timeout -k 10 120 python3 $GRAFT_REPO_ROOT/tools/trace_stats.py $db --top 8 --last tb_kernel 70 > $GRAFT_REPO_ROOT/$O/small_kernel_trace.txt 2>&1
cd "$GRAFT_REPO_ROOT"
b f32_slab8_480 --dtype fp32 --rehearse-comm --rows 4096 --steps 480 --warmup 48 --transport rccl
b weak_max_fp32 --weak --dtype fp32 --grid max --steps 64 --warmup 8
echo done
