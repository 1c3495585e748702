#!/bin/bash
# r5 run W: the counters of run C again on the final kernels (the fp64 priming skip):
# the headline pass (32768^2 fp64 K = 20), the 8-rank slab and 16384^2 K = 16.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r5w
mkdir -p $O
export PYTHONUNBUFFERED=1
export HEAT2D_PLAN_CACHE=$O/plans.txt
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
SQA="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"
SQB="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM"
probe() {  # tag dtype n k cycles
  tag=$1; shift
  timeout -k 10 180 python3 $GRAFT_REPO_ROOT/tools/depth_probe.py "$@" > $O/$tag.json 2> $O/$tag.err || return 1
  timeout -k 10 180 python3 $GRAFT_REPO_ROOT/tools/depth_probe.py "$@" > $O/${tag}_t2.json 2>> $O/$tag.err || return 1
  i=0
  for ctrs in "$SQA" "$SQB" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    HEAT2D_PLAN_CACHE_TRUST=1 timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d $O/${tag}_p$i -- python3 $GRAFT_REPO_ROOT/tools/depth_probe.py "$@" > /dev/null 2>> $O/$tag.err || return 1
  done
  # L2 hit / miss in a pass of their own (names not used on this pool before: a failure only loses them)
  grep -q "TCC_HIT_sum" $O/avail.txt && grep -q "TCC_MISS_sum" $O/avail.txt && [ ! -s $O/failures.txt ] && \
  HEAT2D_PLAN_CACHE_TRUST=1 timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $O/${tag}_p5 -- python3 $GRAFT_REPO_ROOT/tools/depth_probe.py "$@" > /dev/null 2>> $O/$tag.err || echo "$tag: TCC pass failed" >> $O/failures.txt
  P5=""; [ -d $O/${tag}_p5 ] && P5=$O/${tag}_p5
  python3 $GRAFT_REPO_ROOT/tools/counters.py $O/${tag}_p1 $O/${tag}_p2 $O/${tag}_p3 $O/${tag}_p4 $P5 > $O/${tag}_ctr.json || return 1
  rm -rf $O/${tag}_p1 $O/${tag}_p2 $O/${tag}_p3 $O/${tag}_p4 $O/${tag}_p5
}
probe f64_32k_k20 fp64 32768 20 3 && probe f64_slab_k20 fp64 32768 20 6 --rows 4096 && probe f64_16k_k16 fp64 16384 16 8
echo done rc=$?
