#!/usr/bin/env python3
"""Per-depth cycle cost on the autotuned plan (why 16384^2
fp64 runs ~10 % slower per level at K >= 17 than at K = 16).

    python tools/depth_probe.py DTYPE N K [CYCLES] [--arith jacobi]

Autotunes depth K (split_plan: the plan the schedules use), then times CYCLES
back-to-back eager depth-K cycles (hipEvent-free wall clock around them, after
one warm cycle) and prints one JSON line: ms per cycle, us per level, the plan.
The timed cycles are bracketed by two marker dispatches (read16_kernel), so a
profiled re-run (rocprofv3 --pmc ..., with HEAT2D_PLAN_CACHE pointing at the
first run's cache and HEAT2D_PLAN_CACHE_TRUST=1: the same plan, no re-timing)
can be cut to exactly those dispatches: tools/counters.py.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dtype")
    ap.add_argument("n", type=int)
    ap.add_argument("k", type=int)
    ap.add_argument("cycles", type=int, nargs="?", default=6)
    ap.add_argument("--arith", default="jacobi")
    ap.add_argument("--rows", type=int, default=0)
    ap.add_argument("--sigma", type=float, default=0.25)
    args = ap.parse_args()
    import torch
    import heat2d
    from heat2d.models.heat2d import HeatSolver
    from heat2d.ops import _native as N

    torch.cuda.set_device(0)
    inp = heat2d.InputDat(n=args.n, sigma=args.sigma, nu=0.05, dom_len=1.0, ntime=args.k, soln=0, nfields=6)
    prob = heat2d.make_problem(inp, "ghost", "uniform")
    s = HeatSolver(prob, dtype=args.dtype, backend="hip", tb=args.k, device=0, autotune=1, arith=args.arith,
                   rows=args.rows or None)
    plan = s.plan(args.k)  # autotuned (or taken from the plan cache)

    def marker():
        buf = torch.zeros(64, dtype=torch.uint8, device="cuda:0")
        sink = torch.zeros(16, dtype=torch.uint8, device="cuda:0")
        torch.cuda.synchronize()
        N.call("heat2d_read", buf.data_ptr(), 16, sink.data_ptr(), None, 1)
        torch.cuda.synchronize()

    s.step(args.k)  # warm
    s.synchronize()
    marker()
    t0 = time.perf_counter()
    for _ in range(args.cycles):
        s.step(args.k)
    s.synchronize()
    dt = time.perf_counter() - t0
    marker()
    rows = args.rows or args.n
    ms = dt * 1e3 / args.cycles
    print(json.dumps({"dtype": args.dtype, "n": args.n, "rows": rows, "k": args.k, "cycles": args.cycles,
                      "arith": args.arith, "sigma": args.sigma,
                      "ms_per_cycle": round(ms, 4), "us_per_level": round(ms * 1e3 / args.k, 2),
                      "gpts": round(rows * args.n * args.k / (ms * 1e-3) / 1e9, 1),
                      "launches_per_cycle": 2 if plan["order"] in ("concurrent", "edge-first", "lead") else 1,
                      "plan": {k: plan[k] for k in ("order", "ring", "dynamic", "main_bands", "main_items",
                                                    "main_waves", "edge_items", "tuned_ms", "origin")}}),
          flush=True)
    s.close()


if __name__ == "__main__":
    main()
