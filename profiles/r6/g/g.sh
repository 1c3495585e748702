#!/bin/bash
# r6 run G: the frame-row band kernel (kVarFrame) with the frame-column corners on a side stream — the GPU suite on the new
# tree, then the edge slabs of the strong-scaling run (N = 8 / 4) and the whole
# grid, interleaved A/B against HEAT2D_FRAME_KERNEL=0 (frame bands on the
# general kernel, round-5 behaviour); the whole grid also with its first cycle
# lead-ordered (HEAT2D_LEAD_SOLO=1); kernel traces of the new edge slab.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $O/gpu_tests.log)"; [ $rc -eq 0 ] || exit $rc
b() { tag=$1; shift; timeout -k 10 300 python3 $R/bench.py "$@" > $O/$tag.json 2> $O/$tag.err; rc=$?; echo "$tag rc=$rc $(head -c 150 $O/$tag.json | tail -c 70)"; fatal $rc; }
for i in 1 2 3; do
  for v in gen frame; do
    if [ $v = gen ]; then export HEAT2D_FRAME_KERNEL=0; else unset HEAT2D_FRAME_KERNEL; fi
    b s8first_${v}_$i --rehearse-comm --rows 4096 --slab-pos first --steps 20 --warmup 5 --transport rccl
    b s8last_${v}_$i --rehearse-comm --rows 4096 --slab-pos last --steps 20 --warmup 5 --transport rccl
    b s4first_${v}_$i --rehearse-comm --rows 8192 --slab-pos first --steps 20 --warmup 5 --transport rccl
    b whole_${v}_$i --steps 20 --warmup 5
  done
  unset HEAT2D_FRAME_KERNEL
  HEAT2D_LEAD_SOLO=1 b whole_leadsolo_$i --steps 20 --warmup 5
  b s8mid_$i --rehearse-comm --rows 4096 --slab-pos middle --steps 20 --warmup 5 --transport rccl
done
cd /tmp && export TMPDIR=/tmp
tr() { tag=$1; shift; mkdir -p $O/tr_$tag
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr_$tag -o $tag -- python3 $R/bench.py "$@" > $O/tr_$tag/bench.json 2> $O/tr_$tag/bench.err
  rc=$?; echo "trace $tag rc=$rc"; fatal $rc
  db=$(find $O/tr_$tag -name "*.db" | head -1)
  [ -n "$db" ] && python3 $R/tools/trace_stats.py $db --top 8 --last tb_kernel 8 > $O/trace_$tag.txt 2>&1
  rm -rf $O/tr_$tag/*/ $db
}
tr s8first --rehearse-comm --rows 4096 --slab-pos first --steps 20 --warmup 5 --transport rccl --verify off
tr whole --steps 20 --warmup 5 --field-check off --verify off
HEAT2D_LEAD_SOLO=1 tr whole_leadsolo --steps 20 --warmup 5 --field-check off --verify off
cd "$GRAFT_REPO_ROOT"
echo done
