#!/usr/bin/env python3
"""Single-GPU tuning sweep of the temporal-blocked stencil: Gpts/s per
(dtype, temporal depth K, tile rows) at a given grid, all in ONE process
(interleaved rounds, median of R repeats — cross-process variance is larger
than most deltas we care about).

    python bench/sweep.py --n 32768 --dtype fp64 fp32 --tb 1 2 4 6 8 10 12 16 --steps 96
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
    ap.add_argument("--n", type=int, default=32768)
    ap.add_argument("--dtype", nargs="+", default=["fp64"])
    ap.add_argument("--tb", type=int, nargs="+", default=[1, 2, 4, 6, 8, 10, 12, 16])
    ap.add_argument("--tile-rows", type=int, nargs="+", default=[0])
    ap.add_argument("--steps", type=int, default=96)
    ap.add_argument("--repeats", type=int, default=3)
    ap.add_argument("--copy-swap", action="store_true", help="also time the reference-parity copy schedule")
    ap.add_argument("--variants", nargs="+", default=["default"],
                    help="kernel variants r<4|6>[s] (HEAT2D_TB_RING; s = serial schedule: one general launch per "
                         "cycle instead of the MAIN + EDGE split), or default")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    import torch
    import heat2d
    from heat2d.models.heat2d import HeatSolver

    torch.cuda.set_device(0)
    inp = heat2d.InputDat(n=args.n, sigma=0.25, nu=0.05, dom_len=1.0, ntime=args.steps, nfields=6)
    prob = heat2d.make_problem(inp, "ghost", "uniform")
    pts = float(prob.n_owned) ** 2
    results = []
    configs = [(dt, tb, tr, False, v) for v in args.variants for dt in args.dtype for tb in args.tb
               for tr in args.tile_rows]
    if args.copy_swap:
        configs += [(dt, 1, 0, True, "default") for dt in args.dtype]
    for dt, tb, tr, cs, var in configs:
        os.environ.pop("HEAT2D_TB_RING", None)
        serial = var.endswith("s")
        if var.startswith("r"):  # r<4|6>[s]
            os.environ["HEAT2D_TB_RING"] = var[1]
        s = HeatSolver(prob, dtype=dt, backend="hip", tb=tb, tile_rows=tr, copy_swap=cs, device=0,
                       overlap=not serial)
        s.step(2 * tb)
        s.synchronize()
        times = []
        for _ in range(args.repeats):
            t0 = time.perf_counter()
            s.step(args.steps)
            s.synchronize()
            times.append(time.perf_counter() - t0)
        med = statistics.median(times)
        es = 8 if dt == "fp64" else 4
        k = s.tb
        from heat2d.ops import _native as N
        plan = N.plan_tb(s.dtype, s.layout, 0, s.nrows, k)
        rec = {"variant": var, "vec": plan.vec, "ring": plan.prefetch, "bpc": plan.blocks_per_cu,
               "nwaves": plan.nwaves, "dtype": dt, "tb": k, "tile_rows": tr, "copy_swap": cs, "n": args.n, "steps": args.steps,
               "gpts": pts * args.steps / med / 1e9, "gpts_best": pts * args.steps / min(times) / 1e9}
        rec["model_gbps"] = rec["gpts"] * ((4.0 * es) if cs else (2.0 * es / k))
        results.append(rec)
        print(json.dumps(rec), flush=True)
        s.close()
        torch.cuda.empty_cache()
    if args.out:
        with open(args.out, "w") as f:
            json.dump(results, f, indent=1)


if __name__ == "__main__":
    main()
