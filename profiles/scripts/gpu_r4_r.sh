# Round 4, run R: kernel trace of the small grid's graph-replayed timed run
# (4096^2 fp32, 1000 steps): per-kernel time and the gaps between launches.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
O=gpurun_out/r4r
mkdir -p $O
P=$GRAFT_REPO_ROOT/$O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $P/tr -o run -- python3 $GRAFT_REPO_ROOT/bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 100 --verify off > $P/small.json 2> $P/small.err || exit 1
cd $GRAFT_REPO_ROOT
python tools/trace_tail.py $P/tr/run_kernel_trace.csv 70 > $O/tail.txt
python - <<'PY'
import csv
rows = sorted(csv.DictReader(open("gpurun_out/r4r/tr/run_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
t = rows[-63:]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in t]
g = [(int(t[i + 1]["Start_Timestamp"]) - int(t[i]["End_Timestamp"])) / 1e3 for i in range(len(t) - 1)]
span = (int(t[-1]["End_Timestamp"]) - int(t[0]["Start_Timestamp"])) / 1e3
print("last 63 kernels: span %.1f us, kernel sum %.1f, gaps sum %.1f, gap mean %.2f min %.2f max %.2f" % (span, sum(d), sum(g), sum(g) / len(g), min(g), max(g)))
PY
cat $O/small.json | python tools/summarize_json.py /dev/stdin || true
