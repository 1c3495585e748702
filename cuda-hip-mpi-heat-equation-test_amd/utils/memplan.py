"""Memory-fit planner: the largest grid a run can hold in device memory.

The reference sizes nothing — its grid is input.dat's n, allocated as two
device fields plus a whole-field host mirror (fortran/hip/heat.F90:161-176),
so its largest run is whatever the user guessed. Here the IC is generated on
the device and nothing mirrors the field on the host, so a rank's footprint is
its solver's two pitched fields with their ghost bands plus a few KiB of
workspaces — solver_footprint() in csrc/runtime/solver.cpp, the very formula
the Solver constructor allocates by (tests/test_memory_plan.py). The planner
finds the largest n x n grid whose largest slab fits the free device memory
(hipMemGetInfo) minus a reserve for what the solver does not own: the HIP
runtime's growth, the transport's buffers (RCCL channels), hipRTC modules of
the field check and graph workspaces.

    heat2d.utils.memplan.plan_max_grid("fp32", nranks=1)   # ~186k^2 on one MI355X
    bench.py --weak --dtype fp32 --grid max                 # full-HBM weak scaling
    heat2d input.dat --n max                                # the native CLI
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

from ..ops import _native as N

DTYPES = {"fp32": 0, "float32": 0, "fp64": 1, "float64": 1}

# not owned by the solver: runtime growth, RCCL's channel buffers, modules
RESERVE_FIXED = 2 << 30
RESERVE_FRACTION = 0.01


def reserve_bytes(free_bytes: int) -> int:
    """Device memory left unplanned for what the solver does not allocate."""
    return int(RESERVE_FIXED + RESERVE_FRACTION * free_bytes)


def mem_info(device: int = 0) -> tuple:
    """(free, total) device bytes (hipMemGetInfo)."""
    f, t = C.c_int64(), C.c_int64()
    N.call("heat2d_mem_info", int(device), C.byref(f), C.byref(t))
    return f.value, t.value


def footprint(n: int, nranks: int = 1, dtype: str = "fp32", rank: int = 0, backend: str = "hip") -> dict:
    """Device bytes of one rank's solver for an n x n grid on nranks ranks:
    {"field_bytes", "work_bytes", "total_bytes"} (the constructor's allocations)."""
    cfg = N.Config()
    cfg.n_rows = cfg.n_cols = int(n)
    cfg.dtype = DTYPES[dtype]
    cfg.backend = N.BACKEND_HIP if backend == "hip" else N.BACKEND_CPU
    out = (C.c_int64 * 3)()
    N.call("heat2d_solver_footprint", C.byref(cfg), int(rank), int(nranks), out)
    return {"field_bytes": out[0], "work_bytes": out[1], "total_bytes": out[2]}


def plan_max_grid(dtype: str = "fp32", nranks: int = 1, free_bytes: Optional[int] = None, device: int = 0,
                  reserve: Optional[int] = None) -> dict:
    """The largest n x n grid of ``dtype`` whose largest slab on ``nranks``
    ranks fits ``free_bytes`` (default: this device's hipMemGetInfo free
    memory) minus ``reserve`` (default: reserve_bytes(free)). Returns {"n",
    "free_bytes", "reserve_bytes", "footprint_bytes" (rank 0's solver),
    "fraction_of_free"}."""
    free = mem_info(device)[0] if free_bytes is None else int(free_bytes)
    res = reserve_bytes(free) if reserve is None else int(reserve)
    n = C.c_int64()
    N.call("heat2d_plan_max_grid", DTYPES[dtype], int(nranks), int(free - res), C.byref(n))
    fp = footprint(n.value, nranks, dtype)["total_bytes"]
    return {"n": int(n.value), "nranks": int(nranks), "dtype": dtype, "free_bytes": free, "reserve_bytes": res,
            "footprint_bytes": fp, "fraction_of_free": fp / free if free > 0 else 0.0}
