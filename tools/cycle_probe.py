"""Fixed-plan cycle runner for profiling (rocprofv3 counters / kernel trace):
no autotuning (so the profile holds only the timed cycles), `cycles` cycles
of depth k on an n x n grid. Prints the plan and the plan-derived DRAM bytes
per cycle (utils/metrics.plan_hbm_bytes) as one JSON line.

    python tools/cycle_probe.py DTYPE N K CYCLES [overlap=1] [graph=0]

Env: CP_ROWS=R solves the first R rows only (one rank's slab shape); CP_LOOP=1
exchanges the slab's band rows with itself over a 1-rank RCCL communicator
(the multi-GPU schedule rehearsal of bench.py --rehearse-comm); CP_AUTOTUNE=1
autotunes the plan first (its trial cycles appear in a profile before the
timed ones); CP_TIMERS=1 prints the hipEvent phase times of the timed cycles;
CP_ARITH=exact|fma|jacobi|fast picks the update form (default auto); CP_SIGMA=s
the FTCS coefficient (default 0.25).
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
inp = heat2d.InputDat(n=n, sigma=float(os.environ.get("CP_SIGMA", "0.25")), nu=0.05, dom_len=1.0, ntime=k * cycles, soln=0, nfields=6)
prob = heat2d.make_problem(inp, "ghost", "uniform")
rows = int(os.environ.get("CP_ROWS", "0")) or None
tr = None
if os.environ.get("CP_LOOP") == "1":
    from heat2d.parallel.transport import RcclLoopTransport
    tr = RcclLoopTransport(0)
s = HeatSolver(prob, dtype=dtype, backend="hip", tb=k, device=0, autotune=int(os.environ.get("CP_AUTOTUNE", "0")),
               overlap=overlap, graph=graph, rows=rows, transport=tr, arith=os.environ.get("CP_ARITH", "auto"))
s.prepare(k * cycles)
s.step(k)  # warm
s.synchronize()
if os.environ.get("CP_TIMERS") == "1":
    s.set_timing(True)
t0 = time.perf_counter()
s.step(k * cycles)
s.synchronize()
dt = time.perf_counter() - t0
phases = s.phase_times() if os.environ.get("CP_TIMERS") == "1" else None
n_rows = rows or n
es = 8 if dtype == "fp64" else 4
pl = s.plan(k) if overlap else {"k": k, "valid": 0}
print(json.dumps({"dtype": dtype, "n": n, "rows": n_rows, "k": k, "cycles": cycles, "ms": dt * 1e3,
                  "gpts": n_rows * n * k * cycles / dt / 1e9, "plan": pl, "phases": phases,
                  "model_bytes_per_cycle": plan_hbm_bytes(pl, es, n_rows, n)}), flush=True)
s.close()
