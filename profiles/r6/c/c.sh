#!/bin/bash
# r6 run C: VERDICT r5 item 7 — sigma = 0.2 (r != 1/4) rates and VALU
# counters per arithmetic form; item 1 — where the shared-GPU IPC attach
# stalls (process count vs field size), each open logged.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6c
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
b() { tag=$1; shift; timeout -k 10 300 python3 $R/bench.py "$@" > $O/$tag.json 2> $O/$tag.err; rc=$?; echo "$tag rc=$rc $(head -c 150 $O/$tag.json | tail -c 70)"; fatal $rc; }

# (1) sigma = 0.2: rates (2 each) and VALU counters per arithmetic form
for i in 1 2; do
  b s02_fast_$i --sigma 0.2 --arith fast --steps 20 --warmup 5
  b s02_fma_$i --sigma 0.2 --arith fma --steps 20 --warmup 5
  b s02_exact_$i --sigma 0.2 --arith exact --steps 20 --warmup 5
done
cd /tmp
SQ="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"
for a in jacobi:0.25 fast:0.2 fma:0.2 exact:0.2; do
  ar=${a%%:*}; sg=${a##*:}
  export HEAT2D_PLAN_CACHE=$O/plans_$ar.txt
  timeout -k 10 180 python3 $R/tools/depth_probe.py fp64 32768 20 3 --arith $ar --sigma $sg > $O/ctr_$ar.json 2> $O/ctr_$ar.err
  rc=$?; echo "probe $ar rc=$rc"; fatal $rc
  HEAT2D_PLAN_CACHE_TRUST=1 timeout -s KILL 120 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d $O/ctr_${ar}_p -- python3 $R/tools/depth_probe.py fp64 32768 20 3 --arith $ar --sigma $sg > /dev/null 2>> $O/ctr_$ar.err
  rc=$?; echo "pmc $ar rc=$rc"; fatal $rc
  python3 $R/tools/counters.py $O/ctr_${ar}_p > $O/ctr_${ar}_counters.json; rm -rf $O/ctr_${ar}_p
done
export HEAT2D_PLAN_CACHE=off
cd "$GRAFT_REPO_ROOT"

# (2) where the shared-GPU IPC attach stalls (round 5: N = 4 at 32768^2 stalls,
# also with the opens serialised; N = 2 at 32768^2 and N = 4 at 8192^2 pass):
# N = 3 at 32768^2, N = 4 at 16384^2 / 24576^2, each open logged and bounded
export HEAT2D_IPC_ATTACH_LOG=1 HEAT2D_IPC_ATTACH_TIMEOUT=30 HEAT2D_INIT_TIMEOUT=120
for cfg in 3:32768 4:16384 4:24576; do
  g=${cfg%%:*}; n=${cfg##*:}
  timeout -k 10 300 python3 $R/bench.py --gpus $g --share-gpu --grid $n --steps 20 --warmup 5 \
    > $O/share${g}_$n.json 2> $O/share${g}_$n.err
  rc=$?; echo "share$g $n rc=$rc $(grep -c 'opened after' $O/share${g}_$n.err) opened, $(grep -c 'NOT opened' $O/share${g}_$n.err) not"
  case $rc in 0|3) ;; *) fatal $rc; exit $rc;; esac
done
echo done
