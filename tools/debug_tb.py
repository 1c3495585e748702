"""Debug helper: compare the HIP solver to the NumPy golden and report where it differs."""
import sys
import numpy as np
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import heat2d
from heat2d.models import reference as R
from heat2d.models.heat2d import HeatSolver

for dt in ("fp64", "fp32"):
    for tb in (1, 2, 4, 8):
        for n in (600, 1000):
            p = heat2d.make_problem(heat2d.InputDat(n=n, sigma=0.25, nu=0.05, dom_len=1.0, ntime=tb * 2), "ghost", "uniform")
            s = HeatSolver(p, dtype=dt, backend="hip", tb=tb, device=0)
            s.step(p.ntime)
            got = s.download()
            ref = R.owned(R.ftcs(p, dtype=np.float64 if dt == "fp64" else np.float32))
            bad = np.argwhere(got != ref)
            msg = "ok" if len(bad) == 0 else f"{len(bad)} bad; rows {bad[:,0].min()}..{bad[:,0].max()} cols {np.unique(bad[:,1])[:20]}"
            print(dt, "tb", tb, "n", n, msg, flush=True)
            s.close()
