#!/bin/bash
# Full GPU suite (fused stats, loopback, schedules), then time_it parity cost on the CLI.
set -o pipefail
mkdir -p gpurun_out/stats
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/stats/pytest.log 2>&1 || { tail -60 gpurun_out/stats/pytest.log; exit 1; }
tail -2 gpurun_out/stats/pytest.log
cd gpurun_out/stats && printf '32768 0.25 0.05 1.0 280 0\n' > input.dat
CLI=../../cuda-hip-mpi-heat-equation-test_amd/_native/heat2d
timeout -k 10 300 $CLI --json plain.json --output none > plain.out || exit 1
timeout -k 10 300 $CLI --json printed.json --output none --print-every 1 > printed.out || exit 1
timeout -k 10 300 $CLI --json checked.json --output none --check-every 70 > checked.out || exit 1
grep -c time_it printed.out; grep "step " checked.out
python -c "
import json
for f in ('plain','printed','checked'):
    d=json.load(open(f+'.json')); print(f, round(d['wall_s']*1e3,2), 'ms', round(d['gpts_per_s'],1), 'Gpts/s')
"
