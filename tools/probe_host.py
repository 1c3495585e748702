#!/usr/bin/env python3
"""Host overhead of a one-cycle timed region.

The 8-GPU strong-scaling bench times ONE depth-20 cycle per rank (a 4096-row
middle slab of 32768^2 fp64). This probe builds that slab on one GPU
(rehearsal transports: RCCL / IPC self-exchange), then times reps of

    torch.cuda.synchronize(); t0; step(20); <sync variant>; t1

for several sync variants, and the GPU span of the same cycle from the
solver's phase timers (hipEvents), so wall - span = the host's share.

    python tools/probe_host.py [--transport rccl|ipc] [--reps 15] [--json out.json]
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--transport", default="rccl", choices=["rccl", "ipc", "self"])
    ap.add_argument("--rows", type=int, default=4096)
    ap.add_argument("--n", type=int, default=32768)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--dtype", default="fp64")
    ap.add_argument("--json", default="")
    args = ap.parse_args()
    import torch
    import heat2d
    from heat2d.models.heat2d import HeatSolver
    from heat2d.parallel.transport import IpcLoopTransport, RcclLoopTransport, SelfTransport

    torch.cuda.set_device(0)
    inp = heat2d.InputDat(n=args.n, sigma=0.25, nu=0.05, dom_len=1.0, ntime=args.steps, soln=0, nfields=6)
    prob = heat2d.make_problem(inp, "ghost", "uniform")
    tr = {"rccl": lambda: RcclLoopTransport(0), "ipc": lambda: IpcLoopTransport(0), "self": SelfTransport}[args.transport]()
    rows = args.rows if args.rows < args.n else None
    s = HeatSolver(prob, dtype=args.dtype, backend="hip", transport=tr, device=0, rows=rows,
                   slab_row0=(args.n - rows) // 2 if rows else None, arith="jacobi", graph=False)
    s.step(5)
    s.synchronize()
    s.prepare(args.steps)
    out = {"transport": args.transport, "rows": args.rows, "steps": args.steps, "cycles": s.step_cycles(args.steps),
           "plan": {k: v for k, v in s.plan(s.step_cycles(args.steps)[0]).items() if k in ("order", "ring", "main_bands", "main_waves", "tuned_ms")}}

    def rep(variant):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s.step(args.steps)
        t_enq = time.perf_counter()
        if variant == "native+torch":
            s.synchronize()
            torch.cuda.synchronize()
        elif variant == "torch":
            torch.cuda.synchronize()
        elif variant == "native":
            s.synchronize()
        t1 = time.perf_counter()
        return (t1 - t0) * 1e6, (t_enq - t0) * 1e6

    for variant in ("native+torch", "torch", "native", "native+torch"):
        walls, enq = [], []
        for _ in range(args.reps):
            w, e = rep(variant)
            walls.append(w)
            enq.append(e)
        out.setdefault("wall_us", {})[variant] = {"median": statistics.median(walls), "min": min(walls),
                                                  "max": max(walls)}
        out.setdefault("enqueue_us", {})[variant] = statistics.median(enq)
        out.setdefault("first_us", walls[0])  # the first step() after prepare()
    s.set_timing(True)
    spans = []
    for _ in range(args.reps):
        torch.cuda.synchronize()
        s.step(args.steps)
        s.synchronize()
        spans.append(s.phase_times())
    s.set_timing(False)
    out["gpu_cycle_us_median"] = statistics.median(p["cycle_ms"] * 1e3 for p in spans)
    out["gpu_main_us_median"] = statistics.median(p["main_ms"] * 1e3 for p in spans)
    out["gpu_edge_us_median"] = statistics.median(p["edge_ms"] * 1e3 for p in spans)
    out["gpu_exchange_us_median"] = statistics.median(p["exchange_ms"] * 1e3 for p in spans)
    s.close()
    tr.close()
    line = json.dumps(out)
    print(line)
    if args.json:
        with open(args.json, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
