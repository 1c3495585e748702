#!/bin/bash
# 4096^2 fp32 K=12: kernel traces of the split (concurrent) and single-launch plans, eager and graph.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/trace
mkdir -p $O
for order in concurrent single; do
  for g in 0 1; do
    HEAT2D_SPLIT_ORDER=$order timeout -k 10 120 python tools/cycle_probe.py fp32 4096 12 40 1 $g > $O/p_${order}_$g.json || exit 1
    python -c "import json;d=json.load(open('$O/p_${order}_$g.json'));print('$order graph=$g', round(d['gpts'],1), 'Gpts/s', round(d['ms']/d['cycles']*1e3,2),'us/cycle', d['plan'].get('order'), d['plan'].get('main_waves'))"
  done
  HEAT2D_SPLIT_ORDER=$order timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $O/t_$order -- python tools/cycle_probe.py fp32 4096 12 40 1 0 > /dev/null || exit 1
done
