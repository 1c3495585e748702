#!/bin/bash
# fp32 4096-row slab + RCCL self-exchange: phase timers and kernel trace of the autotuned plan.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/thin2
mkdir -p $O
export CP_ROWS=4096 CP_LOOP=1 CP_AUTOTUNE=1
CP_TIMERS=1 timeout -k 10 120 python tools/cycle_probe.py fp32 32768 16 20 > $O/p.json || exit 1
python -c "import json;d=json.load(open('$O/p.json'));print(round(d['gpts'],1), round(d['ms']/d['cycles']*1e3,1),'us/cycle', d['plan']['order'], d['plan']['main_bands'], d['plan']['main_waves'], d['plan']['edge_items'], d['phases'])"
CP_SPLIT= timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $O/tr -- python tools/cycle_probe.py fp32 32768 16 20 > /dev/null || exit 1
HEAT2D_SPLIT_ORDER=edge-first CP_TIMERS=1 timeout -k 10 120 python tools/cycle_probe.py fp32 32768 16 20 > $O/pe.json || exit 1
python -c "import json;d=json.load(open('$O/pe.json'));print('edge-first', round(d['gpts'],1), round(d['ms']/d['cycles']*1e3,1),'us/cycle', d['plan']['order'], d['plan']['main_bands'], d['plan']['main_waves'], d['phases'])"
