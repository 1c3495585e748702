#!/bin/bash
# Multi-GPU schedule rehearsal (1-rank RCCL self-exchange) per slab shape + kernel traces / counters
set -o pipefail
mkdir -p gpurun_out/reh
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for dt in fp64 fp32; do
  for R in 4096 8192 16384; do
    timeout -k 10 200 python bench.py --dtype $dt --rehearse-comm --rows $R --steps 240 --warmup 48 > gpurun_out/reh/reh_${dt}_$R.json 2>gpurun_out/reh/reh_${dt}_$R.err || { cat gpurun_out/reh/reh_${dt}_$R.err; exit 1; }
    cat gpurun_out/reh/reh_${dt}_$R.json
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/reh/prof_reh64 -o run -- python3 bench.py --rehearse-comm --rows 4096 --steps 120 --warmup 24 > gpurun_out/reh/prof_reh64.log 2>&1 || { tail -20 gpurun_out/reh/prof_reh64.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/reh/prof_f32 -o run -- python3 bench.py --dtype fp32 --steps 160 --warmup 32 > gpurun_out/reh/prof_f32.log 2>&1 || { tail -20 gpurun_out/reh/prof_f32.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d gpurun_out/reh/pmc_f32 -o run -- python3 bench.py --dtype fp32 --steps 32 --warmup 16 > gpurun_out/reh/pmc_f32.log 2>&1 || { tail -20 gpurun_out/reh/pmc_f32.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/reh/pmc_f32_fetch -o run -- python3 bench.py --dtype fp32 --steps 32 --warmup 16 > gpurun_out/reh/pmc_f32_fetch.log 2>&1 || { tail -20 gpurun_out/reh/pmc_f32_fetch.log; exit 1; }
ls -R gpurun_out/reh | head -40
