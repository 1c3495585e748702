#!/bin/bash
# fp32 K = 16, single general launch per cycle: whole 32768^2 grid vs a 4096-row slab. SQ/GRBM counters + trace.
set -o pipefail
O=gpurun_out/slabsq
mkdir -p $O
export HEAT2D_SPLIT_ORDER=single
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $O/whole -- python tools/cycle_probe.py fp32 32768 16 4 > $O/whole.json || exit 1
CP_ROWS=4096 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $O/slab -- python tools/cycle_probe.py fp32 32768 16 24 > $O/slab.json || exit 1
for t in whole slab; do
  python tools/prof_summary.py sq $O/$t > $O/$t.sq || exit 1
  python - "$t" <<'PY'
import json, sys
t = sys.argv[1]
d = json.load(open(f"gpurun_out/slabsq/{t}.sq"))
S = d["SQ_totals"]
w = S["SQ_WAVES"]
print(t, "dispatches", d.get("dispatches"), "mean_us", d.get("mean_us"), "clock_GHz/8", round(d.get("clock_GHz", 0) / 8, 3),
      "wave_life_us", round(S["SQ_WAVE_CYCLES"] * 4 / w / (d.get("clock_GHz", 8) / 8) / 1e3, 1),
      "valu_per_wave", round(S["SQ_INSTS_VALU"] / w), "wait_inst", d["wait_inst_any/wave_cycles"], "wait_any", d["wait_any/wave_cycles"])
PY
done
