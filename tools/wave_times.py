"""Per-wave timeline of one stencil launch (diagnostics): which work items end
last, and how long the dispatch ramp and the drain are.

    HEAT2D_WAVE_TIMES=1 python tools/wave_times.py DTYPE N K [CYCLES]

Runs CYCLES eager cycles of depth K on an N x N grid with the plan the env
selects (HEAT2D_SPLIT_ORDER / HEAT2D_SEGMENTS / HEAT2D_TB_RING / CP_ARITH, as
tools/cycle_probe.py), then reads the per-wave {start, end} wall-clock stamps
of the LAST launch (kern::wave_times; 100 MHz) and prints one JSON line: the
launch span, the start spread (ramp), and per-rect duration statistics (rects
of a frame-weighted plan: frame-column strips, frame-row bands, interior)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import heat2d  # noqa: E402
from heat2d.models.heat2d import HeatSolver  # noqa: E402
from heat2d.ops import _native as N  # noqa: E402

assert os.environ.get("HEAT2D_WAVE_TIMES") == "1", "set HEAT2D_WAVE_TIMES=1"
dtype, n, k = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
cycles = int(sys.argv[4]) if len(sys.argv) > 4 else 4
torch.cuda.set_device(0)
inp = heat2d.InputDat(n=n, sigma=0.25, nu=0.05, dom_len=1.0, ntime=k * cycles, soln=0, nfields=6)
prob = heat2d.make_problem(inp, "ghost", "uniform")
s = HeatSolver(prob, dtype=dtype, backend="hip", tb=k, device=0, autotune=0, graph=False,
               arith=os.environ.get("CP_ARITH", "auto"))
s.step(k * cycles)
s.synchronize()
w = N.wave_times().astype(np.int64)
pl = s.plan(k)
s.close()
t0 = w[:, 0].min()
start, end = (w[:, 0] - t0) / 100.0, (w[:, 1] - t0) / 100.0  # us
dur = end - start
rects = pl["main_rects"] or [pl["main_rect"]]
bounds, acc = [], 0
for r in rects:
    items = r[4] * (r[3] - r[2]) if r[4] > 0 else -r[4]
    bounds.append((acc, acc + items, r))
    acc += items
per = []
for lo, hi, r in bounds:
    sel = (w[:, 2] >= lo) & (w[:, 2] < hi)
    if sel.any():
        d = dur[sel]
        per.append({"rect": r, "waves": int(sel.sum()), "dur_mean_us": round(float(d.mean()), 2),
                    "dur_max_us": round(float(d.max()), 2), "dur_min_us": round(float(d.min()), 2),
                    "end_max_us": round(float(end[sel].max()), 2)})
# by XCD (blocks are dealt round-robin over the 8 XCDs: block = wave // 4) and
# by the wave's slot in its block (its SIMD)
wid = w[:, 2]
xcd = {int(x): round(float(dur[(wid // 4) % 8 == x].mean()), 2) for x in range(8) if ((wid // 4) % 8 == x).any()}
slot = {int(x): round(float(dur[wid % 4 == x].mean()), 2) for x in range(4)}
# waves in eighths of the launch order (item order: strip-major segments / band-major bands)
n8 = max(1, len(w) // 8)
order = [round(float(dur[(wid >= i * n8) & (wid < (i + 1) * n8)].mean()), 2) for i in range(8)]
q = np.percentile(end, [50, 90, 99, 100])
print(json.dumps({"dtype": dtype, "n": n, "k": k, "waves": int(len(w)), "plan": {kk: pl[kk] for kk in ("order", "dynamic", "ring", "main_bands", "main_items")},
                  "span_us": round(float(end.max()), 2), "start_spread_us": round(float(start.max()), 2),
                  "start_p90_us": round(float(np.percentile(start, 90)), 2),
                  "dur_mean_us": round(float(dur.mean()), 2), "dur_max_us": round(float(dur.max()), 2),
                  "end_p50_p90_p99_max_us": [round(float(x), 2) for x in q], "dur_by_xcd": xcd,
                  "dur_by_slot": slot, "dur_by_order_eighth": order, "per_rect": per}))
