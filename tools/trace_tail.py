"""Timeline of the last N kernel dispatches of a rocprofv3 kernel trace
(run_kernel_trace.csv): start / end relative to the first of them (us),
duration, grid, queue. Usage: trace_tail.py CSV [N]"""
import csv
import sys


def main():
    path = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    tail = rows[-n:]
    t0 = int(tail[0]["Start_Timestamp"])
    for r in tail:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        name = r["Kernel_Name"]
        if "<" in name:
            name = name[name.index("<"):][:40]
        print(f"{s / 1e3:9.1f} {e / 1e3:9.1f} {(e - s) / 1e3:8.1f}  q{r['Queue_Id']:>3} grid {int(r['Grid_Size_X']):>7}  {name[:60]}")


if __name__ == "__main__":
    main()
