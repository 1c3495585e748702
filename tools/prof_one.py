"""Run one temporal-block configuration for a few cycles (for rocprofv3 counter runs).
usage: prof_one.py DTYPE TB [N] [STEPS]; variant via HEAT2D_TB_NV / HEAT2D_TB_SKEW."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import heat2d  # noqa: E402
from heat2d.models.heat2d import HeatSolver  # noqa: E402

dt, tb = sys.argv[1], int(sys.argv[2])
n = int(sys.argv[3]) if len(sys.argv) > 3 else 32768
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 4 * tb
torch.cuda.set_device(0)
p = heat2d.make_problem(heat2d.InputDat(n=n, sigma=0.25, nu=0.05, dom_len=1.0, ntime=steps, nfields=6), "ghost", "uniform")
s = HeatSolver(p, dtype=dt, backend="hip", tb=tb, device=0)
s.step(steps)
s.synchronize()
print("done", s.info()["tb"], flush=True)
