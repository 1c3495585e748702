#!/usr/bin/env python3
"""Counter totals of the dispatches between the last two marker dispatches
(read16_kernel) of a rocprofv3 --pmc run (tools/depth_probe.py, bench.py
--measure-hbm): per counter the sum over the stencil (tb_kernel) dispatches,
their count, and the kernel resources from the kernel trace when present.

    python tools/counters.py DIR [DIR ...]   -> one JSON object (merged passes)
"""
import csv
import glob
import json
import os
import sys


def window(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    marks = sorted({int(r["Dispatch_Id"]) for r in rows if "read16_kernel" in r["Kernel_Name"]})
    if len(marks) < 2:
        raise SystemExit(f"{d}: no marker pair")
    lo, hi = marks[-2], marks[-1]
    sel = [r for r in rows if lo < int(r["Dispatch_Id"]) < hi and "tb_kernel" in r["Kernel_Name"]]
    tot = {}
    for r in sel:
        tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    info = {"dispatches": len({r["Dispatch_Id"] for r in sel})}
    kt = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        kt += list(csv.DictReader(open(f)))
    if kt:
        kern = sorted({(r["Kernel_Name"].split("tb_kernel<")[1].split(">")[0], r["VGPR_Count"],
                        r.get("Accum_VGPR_Count", ""), r["Grid_Size_X"])
                       for r in kt if "tb_kernel" in r["Kernel_Name"]})
        info["kernels"] = [{"template": t, "vgpr": v, "agpr": a, "grid_threads": g} for t, v, a, g in kern][-4:]
    return tot, info


if __name__ == "__main__":
    out, meta = {}, {}
    for d in sys.argv[1:]:
        t, info = window(d)
        out.update(t)
        meta[os.path.basename(d.rstrip("/"))] = info
    print(json.dumps({"counters": out, "passes": meta}))
