#!/usr/bin/env python3
"""The first step() after prepare() against the ones after it.

bench.py times ONE step(n) right after warm-up + prepare(); tools/probe_host.py
showed that first step 17-56 us slower than the median of back-to-back ones
(profiles/r5/o/). This probe separates host from GPU: per rep, the wall time
(sync; t0; step; sync; t1), the time step() took to return (enqueue) and the
GPU span of the cycle from the solver's phase timers (hipEvents), for
`--reps` steps right after prepare(), optionally after an idle pause.

    python tools/first_step.py [--transport rccl|self] [--rows 4096] [--idle-ms 0] [--spin-ms 0] [--json out.json]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--transport", default="rccl", choices=["rccl", "ipc", "self"])
    ap.add_argument("--rows", type=int, default=4096)
    ap.add_argument("--n", type=int, default=32768)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--row0", type=int, default=-1, help="the slab's first global row (default: the middle slab)")
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--idle-ms", type=float, default=0.0, help="sleep between prepare() and the first rep")
    ap.add_argument("--timers", type=int, default=1, help="phase timers on (GPU spans) or off (wall only)")
    ap.add_argument("--spin-ms", type=float, default=0.0,
                    help="busy-wait the host this long right before the first rep (CPU out of its idle state)")
    ap.add_argument("--pre-launch", type=int, default=0,
                    help="launch N tiny torch kernels (and synchronise) right before the first rep")
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
    s = HeatSolver(prob, dtype="fp64", backend="hip", transport=tr, device=0, rows=rows,
                   slab_row0=(args.row0 if args.row0 >= 0 else (args.n - rows) // 2) if rows else None,
                   arith="jacobi", graph=False)
    s.step(5)
    s.synchronize()
    s.prepare(args.steps)
    if args.timers:
        s.set_timing(True)
    if args.idle_ms > 0:
        time.sleep(args.idle_ms / 1e3)
    reps = []
    for i in range(args.reps):
        torch.cuda.synchronize()
        if i == 0 and args.pre_launch > 0:
            x = torch.zeros(16, device="cuda:0")
            for _ in range(args.pre_launch):
                x.add_(1.0)
            torch.cuda.synchronize()
        if i == 0 and args.spin_ms > 0:
            te = time.perf_counter() + args.spin_ms / 1e3
            while time.perf_counter() < te:
                pass
        t0 = time.perf_counter()
        s.step(args.steps)
        te = time.perf_counter()
        s.synchronize()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        r = {"wall_us": (t1 - t0) * 1e6, "enqueue_us": (te - t0) * 1e6}
        if args.timers:
            p = s.phase_times()
            r.update(gpu_cycle_us=p["cycle_ms"] * 1e3, gpu_main_us=p["main_ms"] * 1e3)
        reps.append(r)
    s.close()
    tr.close()
    out = {"transport": args.transport, "rows": args.rows, "idle_ms": args.idle_ms, "spin_ms": args.spin_ms,
           "timers": args.timers, "hsa_enable_interrupt": os.environ.get("HSA_ENABLE_INTERRUPT"), "reps": reps}
    line = json.dumps(out)
    print(line)
    if args.json:
        with open(args.json, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
