"""Summaries of a `rocprofv3 --kernel-trace` database (ROCm 7 writes SQLite
`*_results.db` by default): per-kernel totals (the `--stats` table) and the
dispatch timeline around a named kernel, as text for `profiles/`.

    python tools/trace_stats.py DB [--top 12] [--last tb_kernel 8] [--before jit]

--last NAME N: the last N dispatches whose name contains NAME (start offset,
duration, gap to the previous one, grid), optionally only those before the
first dispatch whose name contains --before (e.g. the timed step before the
bench's field check starts its run-time compiled kernels)."""
import argparse
import re
import sqlite3


def short(name: str) -> str:
    name = re.sub(r"\(.*\)$", "", name)
    name = name.replace("heat2d::kern::tbimpl::", "").replace("heat2d::kern::", "").replace("void ", "")
    return name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=12)
    ap.add_argument("--last", nargs=2, metavar=("NAME", "N"))
    ap.add_argument("--before", default="")
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    cur = con.cursor()
    rows = cur.execute("select name, total_calls, total_duration, average, percentage from top_kernels").fetchall()
    print(f"{'kernel':<64} {'calls':>6} {'total ms':>10} {'avg us':>9} {'%':>6}")
    for name, calls, tot, avg, pct in rows[:a.top]:
        print(f"{short(name)[:64]:<64} {calls:>6} {tot / 1e3:>10.3f} {avg:>9.2f} {pct:>6.2f}")
    if a.last:
        pat, n = a.last[0], int(a.last[1])
        ks = cur.execute("select name, start, end, grid_x, workgroup_x from kernels order by start").fetchall()
        if a.before:
            first = next((i for i, k in enumerate(ks) if a.before in k[0]), len(ks))
            ks = ks[:first]
        sel = [k for k in ks if pat in k[0]][-n:]
        if sel:
            t0 = sel[0][1]
            print(f"\nlast {len(sel)} dispatches matching '{pat}'" + (f" before the first '{a.before}'" if a.before else ""))
            print(f"{'kernel':<56} {'start us':>10} {'dur us':>10} {'gap us':>9} {'waves':>7}")
            prev_end = None
            for name, s, e, gx, wx in sel:
                gap = "" if prev_end is None else f"{(s - prev_end) / 1e3:9.2f}"
                print(f"{short(name)[:56]:<56} {(s - t0) / 1e3:>10.2f} {(e - s) / 1e3:>10.2f} {gap:>9} {gx // 64:>7}")
                prev_end = e


if __name__ == "__main__":
    main()
