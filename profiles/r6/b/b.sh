#!/bin/bash
# r6 run B: VERDICT r5 item 2's measurement — one rank's slab of the
# strong-scaling run at N = 2 / 4 / 8 (16384 / 8192 / 4096 rows of 32768^2
# fp64, 20 steps, RCCL loop exchange), first / middle / last slab, medians of
# 3 interleaved with the whole grid, one kernel trace per slab.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6b
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
b() { tag=$1; shift; timeout -k 10 300 python3 $R/bench.py "$@" > $O/$tag.json 2> $O/$tag.err; rc=$?; echo "$tag rc=$rc $(head -c 150 $O/$tag.json | tail -c 70)"; fatal $rc; }

# (1) slabs, medians of 3
for i in 1 2 3; do
  b whole_$i --steps 20 --warmup 5 --field-check off
  for rows in 16384 8192 4096; do
    for pos in first middle last; do
      b slab${rows}_${pos}_$i --rehearse-comm --rows $rows --slab-pos $pos --steps 20 --warmup 5 --transport rccl
    done
  done
done
# one kernel trace per slab (and the whole grid)
cd /tmp && export TMPDIR=/tmp
tr() { tag=$1; shift; mkdir -p $O/tr_$tag
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr_$tag -o $tag -- python3 $R/bench.py "$@" > $O/tr_$tag/bench.json 2> $O/tr_$tag/bench.err
  rc=$?; echo "trace $tag rc=$rc"; fatal $rc
  db=$(find $O/tr_$tag -name "*.db" | head -1)
  [ -n "$db" ] && python3 $R/tools/trace_stats.py $db --top 8 --last tb_kernel 6 > $O/trace_$tag.txt 2>&1
  rm -rf $O/tr_$tag/*/ $db
}
tr whole --steps 20 --warmup 5 --field-check off --verify off
for rows in 16384 8192 4096; do
  for pos in first middle last; do
    tr slab${rows}_$pos --rehearse-comm --rows $rows --slab-pos $pos --steps 20 --warmup 5 --transport rccl --verify off
  done
done
cd "$GRAFT_REPO_ROOT"

echo done
