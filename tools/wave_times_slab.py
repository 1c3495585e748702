"""Per-wave timeline of the interior launch of a middle-slab rehearsal cycle
(diagnostics): the bench's strong-scaling slab (rows ROWS of an N x N grid,
middle rank, RCCL self-exchange), CYCLES eager cycles of depth K with the plan
the env selects (HEAT2D_SPLIT_ORDER=edge-first puts the interior last /
HEAT2D_BANDS / HEAT2D_TB_RING), then the per-wave {start, end} stamps of the
LAST stencil launch (kern::wave_times, 100 MHz):

    HEAT2D_WAVE_TIMES=1 python tools/wave_times_slab.py DTYPE N ROWS K [CYCLES]

One JSON line: span, dispatch ramp, end-time and duration percentiles, and
the mean duration of the waves with two static items vs one (grid stride).
(Round 4 also timed the removed fused cycle with it: profiles/r4/lead/.)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import heat2d  # noqa: E402
from heat2d.models.heat2d import HeatSolver  # noqa: E402
from heat2d.ops import _native as N  # noqa: E402
from heat2d.parallel.transport import RcclLoopTransport  # noqa: E402

assert os.environ.get("HEAT2D_WAVE_TIMES") == "1", "set HEAT2D_WAVE_TIMES=1"
dtype, n, rows, k = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
cycles = int(sys.argv[5]) if len(sys.argv) > 5 else 4
torch.cuda.set_device(0)
inp = heat2d.InputDat(n=n, sigma=0.25, nu=0.05, dom_len=1.0, ntime=k * cycles, soln=0, nfields=6)
prob = heat2d.make_problem(inp, "ghost", "uniform")
tr = RcclLoopTransport(0)
s = HeatSolver(prob, dtype=dtype, backend="hip", tb=k, device=0, autotune=1, graph=False, transport=tr,
               rows=rows, slab_row0=(n - rows) // 2, arith="jacobi" if prob.r == 0.25 else "auto")
s.step(k)  # autotune (its trial launches record wave times too: discarded by the timed cycles below)
s.step(k * cycles)
s.synchronize()
w = N.wave_times().astype(np.int64)
pl = s.plan(k)
s.close()
tr.close()
t0 = w[:, 0].min()
start, end = (w[:, 0] - t0) / 100.0, (w[:, 1] - t0) / 100.0  # us
wid = w[:, 2]
items = int(pl["main_items"])
two = wid < max(0, items - len(w))  # static grid stride: these waves take a second item


def pct(x):
    return [round(float(v), 1) for v in np.percentile(x, [0, 50, 90, 100])] if len(x) else None


dur = end - start
print(json.dumps({"dtype": dtype, "rows": rows, "n": n, "k": k, "waves": int(len(w)),
                  "plan": {kk: pl.get(kk) for kk in ("order", "dynamic", "ring", "main_bands", "main_items",
                                                     "main_waves", "main_rects")},
                  "span_us": round(float(end.max()), 1), "start_p50_p90_max_us": pct(start)[1:],
                  "end_min_p50_p90_max_us": pct(end), "dur_min_p50_p90_max_us": pct(dur),
                  "dur_two_item_waves_mean": round(float(dur[two].mean()), 1) if two.any() else None,
                  "dur_one_item_waves_mean": round(float(dur[~two].mean()), 1) if (~two).any() else None}))
