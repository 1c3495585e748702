#!/usr/bin/env python3
"""Depth sweep of the small (Infinity-Cache resident) grid: one JSON line per
(K, graph) point, using bench/configs.py's timed run.

    python bench/sweep_small.py [--n 4096] [--dtype fp32] [--tb 8 10 12 14 16] [--steps 1000]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from configs import run  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "fp64"])
    ap.add_argument("--tb", type=int, nargs="*", default=[8, 10, 12, 14, 16])
    ap.add_argument("--steps", type=int, default=1000)
    a = ap.parse_args()
    for tb in a.tb:
        for graph in (False, True):
            rec = run(f"sweep-{a.n}-{a.dtype}", a.n, a.dtype, a.steps, 64, "hip", tb, graph)
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
