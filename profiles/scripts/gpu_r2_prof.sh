#!/bin/bash
# HBM-model cross-check (FETCH_SIZE / WRITE_SIZE per dispatch) and small-grid counters.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/prof
mkdir -p $O
for cfg in "fp64 32768 14" "fp64 32768 20" "fp32 32768 16"; do
  set -- $cfg
  tag=$1_$2_$3
  timeout -k 10 120 python tools/cycle_probe.py $1 $2 $3 4 > $O/probe_$tag.json || exit 1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch_$tag -- python tools/cycle_probe.py $1 $2 $3 4 > /dev/null || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write_$tag -- python tools/cycle_probe.py $1 $2 $3 4 > /dev/null || exit 1
done
# small grid: timeline + SQ counters
timeout -k 10 120 python tools/cycle_probe.py fp32 4096 16 20 > $O/probe_small.json || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/small_trace -- python tools/cycle_probe.py fp32 4096 16 20 > /dev/null || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace --output-format csv -d $O/small_sq -- python tools/cycle_probe.py fp32 4096 16 20 > /dev/null || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace --output-format csv -d $O/big_sq -- python tools/cycle_probe.py fp32 32768 16 4 > /dev/null || exit 1
cat $O/probe_*.json
