#!/bin/bash
# rocprof roofline evidence for BASELINE config "16384x16384 fp64 single MI355X": kernel trace + FETCH_SIZE + WRITE_SIZE (separate passes)
set -o pipefail
mkdir -p gpurun_out/roof
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python3 bench.py --n 16384 --steps 240 --warmup 24"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/roof/trace -o run --output-format csv -- $B > gpurun_out/roof/trace.log 2>&1 || { tail -20 gpurun_out/roof/trace.log; exit 1; }
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/roof/fetch -o run --output-format csv -- $B > gpurun_out/roof/fetch.log 2>&1 || { tail -20 gpurun_out/roof/fetch.log; exit 1; }
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/roof/write -o run --output-format csv -- $B > gpurun_out/roof/write.log 2>&1 || { tail -20 gpurun_out/roof/write.log; exit 1; }
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES -d gpurun_out/roof/sq -o run --output-format csv -- $B > gpurun_out/roof/sq.log 2>&1 || { tail -20 gpurun_out/roof/sq.log; exit 1; }
grep -h '^{' gpurun_out/roof/*.log | cut -c1-200
