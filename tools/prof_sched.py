"""Run a few cycles of one schedule for rocprofv3 timelines.
usage: prof_sched.py DTYPE TB N STEPS OVERLAP(0|1)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import heat2d  # noqa: E402
from heat2d.models.heat2d import HeatSolver  # noqa: E402

dt, tb, n, steps, ovl = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), bool(int(sys.argv[5]))
torch.cuda.set_device(0)
p = heat2d.make_problem(heat2d.InputDat(n=n, sigma=0.25, nu=0.05, dom_len=1.0, ntime=steps, nfields=6), "ghost",
                        "uniform")
s = HeatSolver(p, dtype=dt, backend="hip", tb=tb, device=0, overlap=ovl)
s.step(steps)
s.synchronize()
print("done", s.info()["tb"], flush=True)
