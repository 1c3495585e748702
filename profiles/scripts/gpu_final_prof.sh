#!/bin/bash
# final kernel traces of the headline configs + phase timers of the multi-GPU schedule rehearsal
set -o pipefail
mkdir -p gpurun_out/final
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/final/f64 -o run --output-format csv -- python3 bench.py --steps 240 --warmup 24 > gpurun_out/final/f64.log 2>&1 || { tail -20 gpurun_out/final/f64.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/final/f32 -o run --output-format csv -- python3 bench.py --dtype fp32 --steps 240 --warmup 32 > gpurun_out/final/f32.log 2>&1 || { tail -20 gpurun_out/final/f32.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/final/reh -o run --output-format csv -- python3 bench.py --rehearse-comm --rows 4096 --steps 240 --warmup 48 > gpurun_out/final/reh.log 2>&1 || { tail -20 gpurun_out/final/reh.log; exit 1; }
timeout -k 10 200 python bench.py --rehearse-comm --rows 4096 --steps 240 --warmup 48 --phase-timers > gpurun_out/final/reh_phases.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --dtype fp32 --rehearse-comm --rows 4096 --steps 240 --warmup 48 --phase-timers > gpurun_out/final/reh32_phases.json 2>/dev/null || exit 1
grep -h '^{' gpurun_out/final/*.log gpurun_out/final/*.json | cut -c1-160
