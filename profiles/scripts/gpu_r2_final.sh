#!/bin/bash
# Final-state evidence for the headline: kernel trace + stats of the driver command, SQ/GRBM counters of the K = 20 pass.
set -o pipefail
O=gpurun_out/final2
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace20 -- python3 bench.py --steps 20 --warmup 5 > $O/bench20.json || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace480 -- python3 bench.py --steps 480 --warmup 16 > $O/bench480.json || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $O/sq20 -- python tools/cycle_probe.py fp64 32768 20 3 > $O/probe20.json || exit 1
python tools/prof_summary.py sq $O/sq20 > $O/sq20.txt || exit 1
python - <<'PY'
import csv, glob, json
O = "gpurun_out/final2"
for tag in ("trace20", "trace480"):
    ks = []
    for f in glob.glob(f"{O}/{tag}/**/*kernel_trace.csv", recursive=True):
        ks += [r for r in csv.DictReader(open(f))]
    ks.sort(key=lambda r: int(r["Start_Timestamp"]))
    tb = [r for r in ks if "tb_kernel" in r["Kernel_Name"]]
    # the timed region = the last cycles of the run: print the last few tb launches
    print(tag, "tb_kernel dispatches", len(tb))
    for r in tb[-4:]:
        name = r["Kernel_Name"].split("tb_kernel<")[1].split(">")[0]
        print("  ", name, round((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, 1), "us grid", r["Grid_Size_X"])
for tag in ("bench20", "bench480"):
    d = json.load(open(f"{O}/{tag}.json"))
    print(tag, d["value"], d["ms_per_step"], d["config"]["cycles"])
PY
cat $O/sq20.txt
