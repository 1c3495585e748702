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


def record(n_owned: int, steps: int, seconds: float, nranks: int, dtype: str, tb: int, backend: str,
           copy_swap: bool = False, extra: Optional[dict] = None) -> dict:
    es = 8 if dtype == "fp64" else 4
    pts = float(n_owned) * float(n_owned)
    gpts = pts * steps / seconds / 1e9 if seconds > 0 and steps > 0 else 0.0
    r = {
        "n": n_owned, "steps": steps, "wall_s": seconds, "nranks": nranks, "dtype": dtype, "tb": tb,
        "backend": backend, "gpts_per_s": gpts,
        "model_hbm_gb_per_s": gpts * model_bytes_per_point_step(es, tb, copy_swap),
        "s_per_iteration": seconds / steps if steps else 0.0,
        "time": time.time(),
    }
    r.update(extra or {})
    return r


def write_json(path: str, rec: dict) -> None:
    with open(path, "w") as f:
        json.dump(rec, f, indent=1)
