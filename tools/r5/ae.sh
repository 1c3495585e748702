#!/bin/bash
# r5 run AE: the split plans of the first (frame-side) slab and a middle slab.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5ae
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off HEAT2D_TUNE_LOG=1
timeout -k 10 200 python3 - > $O/plans.txt 2> $O/plans.err <<'PY'
import torch, heat2d, json
from heat2d.models.heat2d import HeatSolver
from heat2d.parallel.transport import RcclLoopTransport
torch.cuda.set_device(0)
inp = heat2d.InputDat(n=32768, sigma=0.25, nu=0.05, dom_len=1.0, ntime=20, soln=0, nfields=6)
prob = heat2d.make_problem(inp, "ghost", "uniform")
for row0 in (14336, 0):
    tr = RcclLoopTransport(0)
    s = HeatSolver(prob, dtype="fp64", backend="hip", transport=tr, device=0, rows=4096, slab_row0=row0, arith="jacobi", graph=False)
    s.step(5); s.synchronize(); s.prepare(20)
    print(row0, json.dumps(s.plan(20)), flush=True)
    s.close(); tr.close()
PY
echo "rc=$?"; cat $O/plans.txt
grep -E "tune k=20 cycles=12" $O/plans.err | head -12
