#!/usr/bin/env python3
"""The BASELINE.json configuration list, measured on one MI355X (plus the CPU
serial case). Prints one JSON line per configuration.

    python bench/configs.py [--only NAME ...] [--max-gb GB]

  cpu-256-fp64      256x256 fp64, native CPU path (python/serial + fortran/serial scale)
  gpu-4096-fp32     4096x4096 fp32, 1000 steps (fields live in the 256 MiB Infinity Cache)
  gpu-16384-fp64    16384x16384 fp64 (HBM-bound regime)
  gpu-32768-fp64    32768x32768 fp64 — the reference's benchmark input (fortran/hip/input.dat)
  gpu-32768-fp32    32768x32768 fp32 (the 8-GPU config of BASELINE.json, here on 1 GPU)
  gpu-max-fp32      the largest fp32 grid the free device memory holds (utils/memplan.py, the
                    memory-fit planner; --max-gb GB: two fields of at most GB instead)
  gpu-32768-fp64-s0.2  the reference input with sigma = 0.2 (r != 1/4): the scaled-level
                       "fast" arithmetic (any r) and the exact reference rounding, 20 steps
"""
import argparse
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(name, n, dtype, steps, warmup, backend, tb, graph=False, arith="bench", sigma=0.25):
    import heat2d
    from heat2d.models.heat2d import HeatSolver
    from heat2d.utils.metrics import plan_hbm_bytes
    inp = heat2d.InputDat(n=n, sigma=sigma, nu=0.05, dom_len=1.0, ntime=steps, nfields=6)
    prob = heat2d.make_problem(inp, "ghost", "uniform")
    # bench: the r = 1/4 form when r == 1/4 (every config here), as bench.py
    ar = ("jacobi" if prob.r == 0.25 else "auto") if arith == "bench" else arith
    t_init = time.perf_counter()
    s = HeatSolver(prob, dtype=dtype, backend=backend, tb=tb, graph=graph, device=0 if backend == "hip" else None,
                   arith=ar)
    s.synchronize()
    t_init = time.perf_counter() - t_init
    # as bench.py: warm-up, then plan / autotune / pick the cycle schedule of the
    # timed run by measurement, outside the timed region
    tw = time.perf_counter()
    s.step(warmup)
    s.synchronize()
    warm_s = time.perf_counter() - tw  # (the warm-up's own depths are planned / autotuned here)
    tp = time.perf_counter()
    s.prepare(steps)
    prepare_s = time.perf_counter() - tp
    s.cycle_hist(reset=True)
    t0 = time.perf_counter()
    s.step(steps)
    s.synchronize()
    dt = time.perf_counter() - t0
    st = s.stats()
    es = 8 if dtype == "fp64" else 4
    gpts = float(n) * n * steps / dt / 1e9
    hist = s.cycle_hist()
    rec = {"config": name, "n": n, "dtype": dtype, "backend": backend, "arith": ar, "sigma": sigma, "tb_max": s.tb,
           "graph": graph,
           "steps": steps, "s": round(dt, 6), "ms_per_step": round(dt / steps * 1e3, 5), "gpts": round(gpts, 2),
           "cycles": {str(k): c for k, c in sorted(hist.items())}, "field_gb": round(s.layout.elems() * es / 1e9, 2),
           "init_s": round(t_init, 3), "prepare_s": round(prepare_s, 2), "warmup_s": round(warm_s, 2), "finite": bool(math.isfinite(st["sum"]))}
    if backend == "hip":
        rec["autotune"] = s.tune_stats
    if backend == "hip":
        plans, traffic = {}, 0.0
        for k, c in sorted(hist.items()):
            pl = s.plan(k)
            plans[str(k)] = {kk: pl[kk] for kk in ("order", "dynamic", "origin", "ring", "main_bands", "main_waves", "tuned_ms")}
            traffic += c * plan_hbm_bytes(pl, es, n, n)["total"]
        rec["launch_plans"] = plans
        rec["hbm_gb_per_s_plan"] = round(traffic / dt / 1e9, 1)
    s.close()
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="*", default=None)
    ap.add_argument("--max-gb", type=float, default=0.0,
                    help="gpu-max-fp32: two fields of at most this many GB (default 0: the memory-fit planner)")
    ap.add_argument("--arith", default="bench", choices=["bench", "auto", "exact", "fma", "jacobi", "fast"],
                    help="update form (bench.py --arith): bench = jacobi where r == 1/4")
    a = ap.parse_args()
    import torch
    have_gpu = torch.cuda.is_available()
    if have_gpu:
        torch.cuda.set_device(0)
    es32 = 4
    if a.max_gb > 0:
        nmax = int(math.sqrt(a.max_gb * 1e9 / (2 * es32))) // 1024 * 1024
    elif have_gpu:
        from heat2d.utils import memplan
        nmax = memplan.plan_max_grid("fp32", 1, device=0)["n"]
    else:
        nmax = 0
    plan = [
        # tb 0: depths up to the dtype's maximum, chosen per run by measurement
        ("cpu-256-fp64", 256, "fp64", 200, 8, "cpu", 8, False),
        ("gpu-4096-fp32", 4096, "fp32", 1000, 64, "hip", 0, False),
        ("gpu-4096-fp32-graph", 4096, "fp32", 1000, 64, "hip", 0, True),
        ("gpu-16384-fp64", 16384, "fp64", 480, 48, "hip", 0, False),
        ("gpu-32768-fp64", 32768, "fp64", 480, 48, "hip", 0, False),
        ("gpu-32768-fp32", 32768, "fp32", 480, 48, "hip", 0, False),
        ("gpu-max-fp32", nmax, "fp32", 64, 16, "hip", 0, False),
        # sigma 0.2 (any r): the scaled-level arithmetic against the reference rounding
        ("gpu-32768-fp64-s0.2-fast", 32768, "fp64", 20, 5, "hip", 0, True, "fast", 0.2),
        ("gpu-32768-fp64-s0.2-exact", 32768, "fp64", 20, 5, "hip", 0, True, "exact", 0.2),
    ]
    for entry in plan:
        name, n, dt, steps, warm, be, tb, graph = entry[:8]
        arith, sigma = (entry[8], entry[9]) if len(entry) > 8 else (a.arith, 0.25)
        if a.only and not any(name.startswith(o) for o in a.only):
            continue
        if be == "hip" and not have_gpu:
            continue
        print(json.dumps(run(name, n, dt, steps, warm, be, tb, graph, arith, sigma)), flush=True)
        if have_gpu:
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
