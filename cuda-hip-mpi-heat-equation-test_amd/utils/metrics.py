"""Run metrics: the reference prints only seconds (per iteration for the MPI
programs, fortran/hip/heat.F90:323; whole-run CPU time for the others,
fortran/serial/heat.f90:71-74). We report those strings for parity plus
Gpoints/s and the model HBM traffic, as a JSON record."""
from __future__ import annotations

import json
import time
from typing import Optional


def model_bytes_per_point_step(dtype_bytes: int, tb: int, copy_swap: bool = False) -> float:
    """One HBM read + one write of the field per pass of `tb` fused steps; the
    reference-parity copy schedule adds the full-field copy (read + write)."""
    return 4.0 * dtype_bytes if copy_swap else 2.0 * dtype_bytes / max(1, tb)


def strip_geometry(dtype_bytes: int, k: int) -> tuple:
    """(W, U): columns a wave loads / stores per strip of the temporal-blocked
    kernel at depth k (tb_impl.hpp TbShape: 16 B per lane, halo of whole lanes)."""
    v = 16 // dtype_bytes
    ka = (k + v - 1) // v * v
    w = 64 * v
    return w, w - 2 * ka


def work_pieces(rows: int, nstrips: int, nb: int) -> int:
    """Marches (each with its own 2k priming rows) of one rect of the
    temporal-blocked kernel: nb > 0 row bands -> nb per strip; nb < 0 -> -nb
    equal segments of the strip-major row sequence, cut again at strip ends
    (tb_impl.hpp tb_range / tb_piece)."""
    if nb > 0:
        return nb * nstrips
    total, nseg = rows * nstrips, -nb
    cuts = {j * total // nseg for j in range(nseg + 1)} | {s * rows for s in range(nstrips + 1)}
    return len(cuts) - 1


def plan_hbm_bytes(plan: dict, dtype_bytes: int, nrows: int, ncols: int) -> dict:
    """DRAM traffic of ONE cycle of a split plan, from its geometry alone: every
    march (a row band or a segment piece of one strip) loads its rows plus 2k priming
    rows at the strip's full width W (the k-column halos on both sides
    included) and stores its useful U columns once. This counts no cache reuse
    between neighbouring strips / bands (rocprof measured 1.13-1.19x the field
    read per pass vs this model's W/U, profiles/hbm_model_check.md), so it is
    an upper bound on the reads."""
    k = int(plan["k"])
    w, u = strip_geometry(dtype_bytes, k)
    rects = [plan["main_rect"]] + list(plan.get("edge_rects", [])) if plan.get("valid", 0) else []
    if not rects:  # unsplit launch over the whole slab (one band per strip)
        nstrips = (ncols + u - 1) // u
        rects = [[0, nrows, 0, nstrips, 1]]
    rd = 0.0
    for r0, r1, s0, s1, nb in rects:
        if r1 <= r0 or s1 <= s0:
            continue
        rd += float((r1 - r0) * (s1 - s0) + 2 * k * work_pieces(r1 - r0, s1 - s0, nb)) * w * dtype_bytes
    wr = float(nrows) * ncols * dtype_bytes
    return {"read": rd, "write": wr, "total": rd + wr}


def record(n_owned: int, steps: int, seconds: float, nranks: int, dtype: str, tb: int, backend: str,
           copy_swap: bool = False, extra: Optional[dict] = None, cycles: Optional[dict] = None) -> dict:
    """Run record. cycles: {depth: count} the timed loop launched (Solver.cycle_hist);
    with it the model counts one read + one write per pass actually run
    instead of assuming depth tb throughout."""
    es = 8 if dtype == "fp64" else 4
    pts = float(n_owned) * float(n_owned)
    gpts = pts * steps / seconds / 1e9 if seconds > 0 and steps > 0 else 0.0
    passes = sum(cycles.values()) if cycles else 0
    if passes and steps and not copy_swap:
        bpp = 2.0 * es * passes / steps
    else:
        bpp = model_bytes_per_point_step(es, tb, copy_swap)
    r = {
        "n": n_owned, "steps": steps, "wall_s": seconds, "nranks": nranks, "dtype": dtype, "tb": tb,
        "cycles": {str(k): v for k, v in sorted((cycles or {}).items())},
        "backend": backend, "gpts_per_s": gpts,
        "model_hbm_gb_per_s": gpts * bpp,
        "s_per_iteration": seconds / steps if steps else 0.0,
        "time": time.time(),
    }
    r.update(extra or {})
    return r


def write_json(path: str, rec: dict) -> None:
    with open(path, "w") as f:
        json.dump(rec, f, indent=1)
