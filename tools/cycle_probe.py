"""Fixed-plan cycle runner for profiling (rocprofv3 counters / kernel trace):
no autotuning (so the profile holds only the timed cycles), `cycles` cycles
of depth k on an n x n grid. Prints the plan and the plan-derived DRAM bytes
per cycle (utils/metrics.plan_hbm_bytes) as one JSON line.

    python tools/cycle_probe.py DTYPE N K CYCLES [overlap=1] [graph=0]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import heat2d  # noqa: E402
from heat2d.models.heat2d import HeatSolver  # noqa: E402
from heat2d.utils.metrics import plan_hbm_bytes  # noqa: E402

dtype, n, k, cycles = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
overlap = bool(int(sys.argv[5])) if len(sys.argv) > 5 else True
graph = bool(int(sys.argv[6])) if len(sys.argv) > 6 else False
torch.cuda.set_device(0)
inp = heat2d.InputDat(n=n, sigma=0.25, nu=0.05, dom_len=1.0, ntime=k * cycles, soln=0, nfields=6)
prob = heat2d.make_problem(inp, "ghost", "uniform")
s = HeatSolver(prob, dtype=dtype, backend="hip", tb=k, device=0, autotune=0, overlap=overlap, graph=graph)
s.prepare(k * cycles)
s.step(k)  # warm
s.synchronize()
t0 = time.perf_counter()
s.step(k * cycles)
s.synchronize()
dt = time.perf_counter() - t0
es = 8 if dtype == "fp64" else 4
pl = s.plan(k) if overlap else {"k": k, "valid": 0}
print(json.dumps({"dtype": dtype, "n": n, "k": k, "cycles": cycles, "ms": dt * 1e3,
                  "gpts": n * n * k * cycles / dt / 1e9, "plan": pl,
                  "model_bytes_per_cycle": plan_hbm_bytes(pl, es, n, n)}), flush=True)
s.close()
