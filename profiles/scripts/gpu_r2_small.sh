#!/bin/bash
# 4096^2 fp32 K=16, single launch over 1007 segments (the autotuner's plan): kernel trace + SQ/GRBM counters.
set -o pipefail
O=gpurun_out/small2
mkdir -p $O
export HEAT2D_SPLIT_ORDER=single HEAT2D_SEGMENTS=1007 HEAT2D_TB_RING=6
timeout -k 10 120 python tools/cycle_probe.py fp32 4096 16 40 1 0 > $O/eager.json || exit 1
timeout -k 10 120 python tools/cycle_probe.py fp32 4096 16 40 1 1 > $O/graph.json || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $O/trace -- python tools/cycle_probe.py fp32 4096 16 40 1 1 > /dev/null || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $O/sq -- python tools/cycle_probe.py fp32 4096 16 10 1 0 > /dev/null || exit 1
python tools/prof_summary.py trace $O/trace > $O/trace.txt || exit 1
python tools/prof_summary.py sq $O/sq > $O/sq.txt || exit 1
for f in $O/eager.json $O/graph.json; do python -c "import json;d=json.load(open('$f'));print('$f', round(d['gpts']), round(d['ms']/d['cycles']*1e3,1),'us/cycle')"; done
tail -8 $O/trace.txt; cat $O/sq.txt | head -40
