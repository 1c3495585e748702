"""Isolated-cycle timing probe: prepare(n), then time step(n) repeatedly after
different warmups (what the driver's short bench sees), with hipEvent phase
timers. python tools/sched_probe.py [n_steps] [grid]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import heat2d  # noqa: E402
from heat2d.models.heat2d import HeatSolver  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
grid = int(sys.argv[2]) if len(sys.argv) > 2 else 32768
torch.cuda.set_device(0)
inp = heat2d.InputDat(n=grid, sigma=0.25, nu=0.05, dom_len=1.0, ntime=n, soln=0, nfields=6)
prob = heat2d.make_problem(inp, "ghost", "uniform")
s = HeatSolver(prob, dtype="fp64", backend="hip", device=0)
t = time.perf_counter()
s.prepare(n)
print("prepare_s", round(time.perf_counter() - t, 2), "schedule", s.schedule(n), flush=True)
pts = prob.n_owned ** 2


def timed(tag, warm):
    if warm:
        s.step(warm)
    s.synchronize()
    s.set_timing(True)
    t0 = time.perf_counter()
    s.step(n)
    s.synchronize()
    dt = time.perf_counter() - t0
    ph = s.phase_times()
    s.set_timing(False)
    print(json.dumps({"tag": tag, "warm": warm, "ms": round(dt * 1e3, 3), "gpts": round(pts * n / dt / 1e9, 1),
                      "phase": {k: round(v, 3) for k, v in ph.items()}}), flush=True)


for w in (5, 5, 20, 20, 0, 0, 14, 40):
    timed("w", w)
for i in range(3):
    time.sleep(0.5)
    timed("idle0.5s", 0)
s.close()
