"""Summarise rocprofv3 CSV output (kernel stats / counter collection) as markdown."""
import csv
import sys
from collections import defaultdict


def short(name, n=90):
    name = name.replace("heat2d::kern::", "").replace("(anonymous namespace)::", "").replace("tbimpl::", "")
    return name if len(name) <= n else name[:n] + "..."


def stats(path):
    rows = list(csv.DictReader(open(path)))
    out = ["| kernel | calls | avg us | total ms | % |", "|---|---|---|---|---|"]
    for r in rows:
        out.append(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.1f} | "
                   f"{float(r['TotalDurationNs'])/1e6:.2f} | {float(r['Percentage']):.1f} |")
    return "\n".join(out)


def counters(path):
    rows = list(csv.DictReader(open(path)))
    agg = defaultdict(list)
    for r in rows:
        agg[(short(r["Kernel_Name"], 60), r["Counter_Name"])].append(float(r["Counter_Value"]))
    out = ["| kernel | counter | dispatches | mean value |", "|---|---|---|---|"]
    for (k, c), v in sorted(agg.items()):
        out.append(f"| `{k}` | {c} | {len(v)} | {sum(v)/len(v):.4g} |")
    return "\n".join(out)


if __name__ == "__main__":
    kind, path = sys.argv[1], sys.argv[2]
    print(stats(path) if kind == "stats" else counters(path))
