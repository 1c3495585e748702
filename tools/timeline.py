"""Kernel timeline from a rocprofv3 kernel_trace.csv: which kernels ran
concurrently, per-cycle spans, gaps on the compute stream.

usage: python tools/timeline.py KERNEL_TRACE_CSV [--last N]
"""
import argparse
import csv


def short(name):
    name = name.replace("heat2d::kern::", "").replace("tbimpl::", "")
    if "tb_kernel" in name:
        return "tb" + name[name.index("<"):name.index(">") + 1] if "<" in name else "tb"
    if "nccl" in name.lower() or "rccl" in name.lower():
        return "rccl:" + name.split("(")[0][-40:]
    return name.split("(")[0][-50:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--last", type=int, default=24)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                  int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0)) for r in rows))
    ev = ev[-a.last:]
    t0 = ev[0][0]
    for s, e, n, g in ev:
        print(f"{(s - t0) / 1e3:10.1f} {(e - t0) / 1e3:10.1f} {(e - s) / 1e3:8.1f} us  grid={g:<8d} {n}")
    span = (ev[-1][1] - t0) / 1e3
    busy = {}
    for s, e, n, g in ev:
        busy[n] = busy.get(n, 0) + (e - s) / 1e3
    print(f"span {span:.1f} us over {len(ev)} kernels")
    for n, b in sorted(busy.items(), key=lambda x: -x[1]):
        print(f"  {b:10.1f} us  {n}")


if __name__ == "__main__":
    main()
