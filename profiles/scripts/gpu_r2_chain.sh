#!/bin/bash
# Chained-march A/B: bitwise tests on the default (chain 4) build, then fixed-plan cycle times for
# single-chain (c0), chain 4 (default) and chain 8 builds.
set -o pipefail
O=gpurun_out/chain
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_solver.py -x -q --timeout 200 --timeout-method thread -k "golden_bitwise or sine_bitwise or split_schedule or deep or tile_rows or sizes or step_stats" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
P=cuda-hip-mpi-heat-equation-test_amd
for cfg in "fp32 4096 16 40" "fp32 4096 8 40" "fp32 32768 16 4" "fp64 32768 14 4" "fp64 32768 20 3" "fp64 8192 14 20"; do
  for v in c0 c4 c8; do
    lib=$P/_native_$v/libheat2d.so; [ $v = c4 ] && lib=$P/_native/libheat2d.so
    HEAT2D_LIB=$lib timeout -k 10 120 python tools/cycle_probe.py $cfg > $O/p.json || exit 1
    python -c "import json;d=json.load(open('$O/p.json'));print('$v', '$cfg', round(d['gpts'],1), 'Gpts/s', round(d['ms']/d['cycles'],4),'ms/cycle', d['plan'].get('order'), d['plan'].get('main_waves'))"
  done
done
