"""Summaries of the rocprofv3 CSVs written by tools/gpurun/gpu_r2_prof.sh:
  * hbm: per-cycle DRAM bytes of the timed tb_kernel dispatches
    (FETCH_SIZE x 2 — gfx950 counts wide streaming reads at half,
    MI355X_MICROARCH.md §HBM — + WRITE_SIZE) vs the plan model
    (utils/metrics.plan_hbm_bytes);
  * sq: SQ counter ratios per tb_kernel dispatch;
  * trace: per-kernel durations and gaps of a kernel trace.
python tools/prof_summary.py hbm|sq|trace DIR [probe.json]"""
import csv
import glob
import json
import sys
from collections import defaultdict


def rows(d, suffix):
    out = []
    for f in glob.glob(f"{d}/**/*_{suffix}.csv", recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


def tb_counter(d, name):
    """{dispatch: value} of the tb_kernel dispatches, dispatch order."""
    v = {}
    for r in rows(d, "counter_collection"):
        if "tb_kernel" in r["Kernel_Name"] and r["Counter_Name"] == name:
            v[int(r["Dispatch_Id"])] = float(r["Counter_Value"])
    return dict(sorted(v.items()))


def hbm(tag_dir_fetch, tag_dir_write, probe):
    p = json.load(open(probe))
    f = tb_counter(tag_dir_fetch, "FETCH_SIZE")
    w = tb_counter(tag_dir_write, "WRITE_SIZE")
    launches = 2 if p["plan"].get("valid") in (1, 3) else 1
    cyc = p["cycles"]
    # the last `cycles` cycles' dispatches (the warm cycle precedes them)
    fv = list(f.values())[-cyc * launches:]
    wv = list(w.values())[-cyc * launches:]
    read = 2 * sum(fv) * 1024 / cyc
    write = sum(wv) * 1024 / cyc
    m = p["model_bytes_per_cycle"]
    es = 8 if p["dtype"] == "fp64" else 4
    field = p["n"] * p["n"] * es
    return {"cfg": f"{p['dtype']} {p['n']}^2 K={p['k']} ({p['plan'].get('order')})",
            "measured_read_GB": round(read / 1e9, 3), "model_read_GB": round(m["read"] / 1e9, 3),
            "measured_write_GB": round(write / 1e9, 3), "model_write_GB": round(m["write"] / 1e9, 3),
            "read_over_field": round(read / field, 3), "model_read_over_field": round(m["read"] / field, 3),
            "model_over_measured_total": round(m["total"] / (read + write), 3)}


def sq(d):
    acc = defaultdict(float)
    n = 0
    for r in rows(d, "counter_collection"):
        if "tb_kernel" in r["Kernel_Name"]:
            acc[r["Counter_Name"]] += float(r["Counter_Value"])
            n += 1
    wc = acc["SQ_WAVE_CYCLES"] or 1
    # dispatches / mean duration of the same run's tb_kernel dispatches (kernel
    # trace beside the counters): GRBM_GUI_ACTIVE per dispatch / duration = clock
    ks = [r for r in rows(d, "kernel_trace") if "tb_kernel" in r["Kernel_Name"]]
    dur = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in ks]
    extra = {}
    if dur and acc.get("GRBM_GUI_ACTIVE"):
        extra = {"dispatches": len(dur), "mean_us": round(sum(dur) / len(dur) / 1e3, 2),
                 "clock_GHz": round(acc["GRBM_GUI_ACTIVE"] / sum(dur), 3)}
    return {**extra, "SQ_totals": {k: v for k, v in sorted(acc.items())},
            "wait_any/wave_cycles": round(acc["SQ_WAIT_ANY"] / wc, 3),
            "wait_inst_any/wave_cycles": round(acc["SQ_WAIT_INST_ANY"] / wc, 3),
            "active_inst_any/wave_cycles": round(acc["SQ_ACTIVE_INST_ANY"] / wc, 3),
            "active_valu/busy_cycles_per_simd": round(acc["SQ_ACTIVE_INST_VALU"] / max(1, acc["SQ_BUSY_CYCLES"]), 3)}


def trace(d):
    ks = sorted(rows(d, "kernel_trace"), key=lambda r: int(r["Start_Timestamp"]))
    ks = [r for r in ks if "tb_kernel" in r["Kernel_Name"]]
    out = []
    prev_end = None
    for r in ks[-12:]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].split("tb_kernel<")[1].split(">")[0]
        out.append({"kernel": name, "us": round((e - s) / 1e3, 2), "grid": r["Grid_Size_X"],
                    "gap_us": None if prev_end is None else round((s - prev_end) / 1e3, 2)})
        prev_end = max(prev_end or 0, e)
    return out


if __name__ == "__main__":
    mode = sys.argv[1]
    if mode == "hbm":
        print(json.dumps(hbm(sys.argv[2], sys.argv[3], sys.argv[4])))
    elif mode == "sq":
        print(json.dumps(sq(sys.argv[2]), indent=1))
    else:
        for t in trace(sys.argv[2]):
            print(t)
