"""Probe: hipGraph capture of the overlapped cycle with the 1-rank RCCL loop transport.
python tools/graph_rccl_probe.py ORDER (concurrent | edge-first)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["HEAT2D_SPLIT_ORDER"] = sys.argv[1]
import numpy as np  # noqa: E402
import heat2d  # noqa: E402
from heat2d.models import reference as R  # noqa: E402
from heat2d.models.heat2d import HeatSolver  # noqa: E402
from heat2d.parallel.transport import RcclLoopTransport  # noqa: E402

tr = RcclLoopTransport(0)
p = heat2d.make_problem(heat2d.InputDat(n=400, sigma=0.25, nu=0.05, dom_len=1.0, ntime=40), "ghost", "sine")
s = HeatSolver(p, dtype="fp64", backend="hip", tb=8, transport=tr, device=0, graph=True)
print("plan", s.plan(), flush=True)
s.upload(R.owned(R.initial_field(p)))
s.step(p.ntime)
got = s.download()
ref = R.owned(R.ftcs(p))
print(sys.argv[1], "finite", np.isfinite(got).all(), "interior==golden", np.array_equal(got[60:-60], ref[60:-60]), flush=True)
