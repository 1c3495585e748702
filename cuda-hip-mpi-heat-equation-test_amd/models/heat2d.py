"""The heat-equation model: a distributed 2-D FTCS slab solver on the native engine.

One :class:`HeatSolver` per rank (process or host thread). It owns a native
``heat2d::Solver`` (csrc/runtime/solver.cpp) holding this rank's slab of the
global grid in two pitched device (or host) fields, and a transport for the
halo exchange. Everything in the time loop runs natively; Python only issues
``step(n)``.

Parity map (reference -> here):
  * fortran/hip/heat.F90 setup()/heat_eqn()/swap()  -> HeatSolver(problem, backend="hip")
  * fortran/mpi+cuda/heat.F90 (CUDA-aware / staged)  -> RCCL transport (device-direct)
  * fortran/cuda_kernel/heat_managed.F90             -> managed=True
  * fortran/serial/heat.f90                          -> backend="cpu"
  * per-step D2D ``Td_old = Td`` (heat.F90:243)      -> copy_swap=True (parity mode)
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np

from ..ops import _native as N
from ..parallel import transport as T
from ..utils.config import Problem

DTYPES = {"fp32": N.F32, "float32": N.F32, "fp64": N.F64, "float64": N.F64}
NP_DTYPES = {N.F32: np.float32, N.F64: np.float64}


def resolve_backend(backend: str) -> str:
    if backend == "auto":
        try:
            import torch
            return "hip" if torch.cuda.is_available() else "cpu"
        except Exception:  # pragma: no cover
            return "cpu"
    if backend not in ("hip", "cpu"):
        raise ValueError("backend must be hip|cpu|auto")
    return backend


PLAN_ORIGINS = {-1: "none", 0: "planned", 1: "tuned", 2: "cache"}


def _plan(h, k: int) -> dict:
    p, ms, org = N.SplitPlan(), C.c_float(), C.c_int32()
    N.call("heat2d_solver_plan", h, int(k), C.byref(p), C.byref(ms))
    N.call("heat2d_solver_plan_origin", h, int(k), C.byref(org))
    return {"k": p.k, "ring": p.ring, "valid": p.valid,
            "order": ("lead" if p.valid == 1 and p.flags & 4 else
                      {1: "concurrent", 2: "single", 3: "edge-first"}.get(p.valid, "serial")),
            "dynamic": int((p.flags >> 1) & 1), "origin": PLAN_ORIGINS.get(org.value, "?"),
            "main_bands": p.main.nb, "main_items": p.main_items, "main_waves": p.main_waves,
            "edge_items": p.edge_items, "edge_waves": p.edge_waves, "tuned_ms": ms.value,
            "main_rect": [p.main.r0, p.main.r1, p.main.s0, p.main.s1, p.main.nb],
            "edge_rects": [[e.r0, e.r1, e.s0, e.s1, e.nb] for e in list(p.edge)[:p.nedge]],
            # the rects launched instead of main_rect: frame-weighted (arith 2)
            "main_rects": [[e.r0, e.r1, e.s0, e.s1, e.nb] for e in list(p.rects)[:p.nrects]]}


def _cycle_hist(h, reset: bool) -> dict:
    n = N.max_tb() + 1
    out = (C.c_int64 * n)()
    N.call("heat2d_solver_cycle_hist", h, out, n, int(bool(reset)))
    return {k: int(out[k]) for k in range(n) if out[k]}


class HeatSolver:
    """Distributed FTCS solver for one rank.

    Args:
        problem: resolved :class:`~utils.config.Problem`.
        dtype: "fp64" (reference precision) or "fp32".
        backend: "hip", "cpu" or "auto".
        tb: largest temporal-block depth K (time steps fused per HBM pass; fp64
            1..24, fp32 1..20). 0: all depths up to that limit for the measured
            schedules of prepare() (autotuned slabs), balanced cycles of the
            steady-state best (fp64 14 / fp32 16) otherwise; 8 on the CPU twin.
        overlap: boundary/interior split with the halo exchange on a comm stream.
        copy_swap: reference-parity schedule (full field copy every step, K=1).
        managed: allocate fields with hipMallocManaged.
        graph: replay step pairs from a captured hipGraph (single-rank / serial schedule).
        transport: a :class:`parallel.transport.Transport`; default picks self / RCCL / gloo.
        device: HIP device ordinal (default: torch's current device).
        comm_cus: room for the bands + RCCL beside the interior kernel when
            overlapping: >0 CUs masked off the compute stream; 0 (default): the
            interior planned for all wave slots but 8 spare ones, no mask; -1 none.
        engine: "tb" — the temporal-blocked gfx950 kernels; "jit" — a kernel
            rendered for this slab and r and compiled at run time with hipRTC
            (one step per launch; the reference's PyCUDA program, ops/jit.py).
        autotune: overlapped (split) schedule: time candidate (ring, band count)
            launch plans on the first cycle of each depth and keep the fastest
            (-1: only for slabs of >= 2**24 points, 0: off, 1: on).
        rows: solve only the first ``rows`` x-rows of the grid (a rectangular
            rows x n domain, e.g. one rank's slab shape for a 1-GPU rehearsal).
        slab_row0: with ``rows``: own rows [slab_row0, slab_row0 + rows) of the
            WHOLE grid instead — a middle rank's slab (its boundary bands are
            interior bands, as on rank 3 of 8) for 1-GPU rehearsals.
        arith: "exact" — every operation of the reference update rounded as
            written (-ffp-contract=off; bitwise equal to the NumPy golden);
            "fma" — the update contracted to fma(r, sum - 4c, c), what hipcc's
            default contraction makes of fortran/hip/heat_kernel.cpp:43: one op
            fewer per point; identical to "exact" when r is a power of two
            (sigma = 0.25), bitwise equal to the CPU twin for any r;
            "jacobi" — r == 1/4 only: the centre weight 1 - 4r is zero and the
            update is r * (((S + E) + N) + W) (3 adds per interior point and
            level in the kernels instead of 5); bitwise equal to the CPU twin
            and to models.reference.ftcs(arith="jacobi"), and to "exact"
            wherever sum - 4c is exact (e.g. the reference IC, values in [1, 2]).
        edge_shift: rows each edge slab (rank 0 and the last rank: the global
            frame rows on one side) gives to the middle slabs of a >= 3-rank
            decomposition (common.hpp decompose): an edge slab's cycle costs
            more per row, and a step lasts as long as the slowest rank;
            bench.py measures the excess and picks the shift. Same on every rank.
    """

    def __init__(self, problem: Problem, *, dtype: str = "fp64", backend: str = "auto", tb: int = 0,
                 overlap: bool = True, copy_swap: bool = False, managed: bool = False, graph: bool = False,
                 tile_rows: int = 0, halo: int = 0, transport: Optional[T.Transport] = None,
                 device: Optional[int] = None, init: bool = True, rows: Optional[int] = None,
                 comm_cus: int = 0, autotune: int = -1, engine: str = "tb", arith: str = "auto",
                 slab_row0: Optional[int] = None, edge_shift: int = 0):
        self.problem = problem
        self.edge_shift = int(edge_shift)
        self.backend = resolve_backend(backend)
        self.dtype = DTYPES[dtype]
        self.np_dtype = NP_DTYPES[self.dtype]
        if self.backend == "hip" and device is None:
            import torch
            device = torch.cuda.current_device()
        self.device = -1 if self.backend == "cpu" else int(device)
        self.transport = transport or T.default_transport(self.backend, None if self.device < 0 else self.device)
        cfg = N.Config()
        if rows is not None and not 1 <= rows <= problem.n_owned:
            raise ValueError(f"rows must be in [1, {problem.n_owned}]")
        cfg.n_rows = problem.n_owned if rows is None else int(rows)  # rows < n: the first rows x n of the grid
        if slab_row0 is not None:  # 1-rank rehearsal of the middle slab rows [slab_row0, slab_row0 + rows)
            if rows is None or not 0 <= slab_row0 <= problem.n_owned - rows:
                raise ValueError("slab_row0 needs rows and must keep the slab inside the grid")
            cfg.slab_row0 = int(slab_row0)
            cfg.slab_rows_global = problem.n_owned
        cfg.n_cols = problem.n_owned
        cfg.dtype = self.dtype
        cfg.backend = N.BACKEND_HIP if self.backend == "hip" else N.BACKEND_CPU
        cfg.r = problem.r
        cfg.tb = tb
        cfg.overlap = int(overlap)
        cfg.copy_swap = int(copy_swap)
        cfg.managed = int(managed)
        cfg.device = self.device
        cfg.use_graph = int(graph)
        cfg.tile_rows = tile_rows
        cfg.halo = halo
        cfg.comm_cus = comm_cus
        cfg.autotune = autotune
        cfg.edge_shift = self.edge_shift
        if engine not in ("tb", "jit"):
            raise ValueError("engine must be 'tb' (temporal-blocked kernels) or 'jit' (hipRTC, one step per launch)")
        cfg.engine = 1 if engine == "jit" else 0
        if arith not in N.ARITH:
            raise ValueError(f"arith must be one of {sorted(N.ARITH)}")
        cfg.arith = N.ARITH[arith]
        self.arith = arith
        self._cfg = cfg
        h = C.c_void_p()
        N.call("heat2d_solver_create", C.byref(cfg), self.transport.handle, C.byref(h))
        self._h = h
        self.layout = N.Layout()
        N.call("heat2d_solver_layout", self._h, C.byref(self.layout))
        if init:
            self.init()

    # ------------------------------------------------------------------ info
    @property
    def rank(self) -> int:
        return self.transport.rank

    @property
    def size(self) -> int:
        return self.transport.size

    @property
    def row0(self) -> int:
        return int(self.layout.row0)

    @property
    def nrows(self) -> int:
        return int(self.layout.nrows)

    @property
    def ncols(self) -> int:
        return int(self.layout.ncols)

    def info(self) -> dict:
        tb, band, steps = C.c_int32(), C.c_int64(), C.c_int64()
        field, stream = C.c_void_p(), C.c_void_p()
        N.call("heat2d_solver_info", self._h, C.byref(tb), C.byref(band), C.byref(steps), C.byref(field),
               C.byref(stream))
        return {"tb": tb.value, "band": band.value, "steps": steps.value, "field": field.value,
                "stream": stream.value, "backend": self.backend, "transport": self.transport.name,
                "rank": self.rank, "size": self.size, "layout": self.layout.as_dict()}

    def set_timing(self, on: bool = True) -> None:
        """Record hipEvent phase timers for every cycle from now on (HIP backend)."""
        N.call("heat2d_solver_timing", self._h, int(bool(on)))

    def phase_times(self) -> dict:
        """Sum of the phase timers since the last call (synchronises, then resets):
        main / edge / exchange / cycle milliseconds and the number of cycles."""
        out = (C.c_double * 5)()
        N.call("heat2d_solver_phase_times", self._h, out)
        return {"main_ms": out[0], "edge_ms": out[1], "exchange_ms": out[2], "cycle_ms": out[3],
                "cycles": int(out[4])}

    def prepare(self, n: int) -> None:
        """Plan / autotune every cycle depth a ``step(n)`` will use (call before timing it)."""
        N.call("heat2d_solver_prepare", self._h, int(n))

    def plan(self, k: Optional[int] = None) -> dict:
        """The split plan (MAIN / EDGE launches) used for depth k (default: tb)."""
        return _plan(self._h, self.tb if k is None else k)

    def schedule(self, n: int):
        """Depths of the measured cycle schedule prepare(n) chose for step(n), or None
        (balanced cycles of the preferred depth)."""
        ln = C.c_int64()
        N.call("heat2d_solver_schedule", self._h, int(n), None, 0, C.byref(ln))
        if ln.value < 0:
            return None
        out = (C.c_int32 * max(1, ln.value))()
        N.call("heat2d_solver_schedule", self._h, int(n), out, ln.value, C.byref(ln))
        return [int(v) for v in out[:ln.value]]

    def schedule_replayed(self, n: int) -> bool:
        """Whether step(n) replays its measured schedule as one captured hipGraph
        (graph=True and short cycles; long-cycle schedules launch eagerly)."""
        out = C.c_int32()
        N.call("heat2d_solver_schedule_replayed", self._h, int(n), C.byref(out))
        return bool(out.value)

    def cycle_hist(self, reset: bool = False) -> dict:
        """{depth: cycles} that step() launched since the last reset (graph replays count 2 each)."""
        return _cycle_hist(self._h, reset)

    def step_cycles(self, n: int) -> list:
        """The cycle depths step(n) will run from the current state, in order."""
        ln = C.c_int64()
        N.call("heat2d_solver_step_cycles", self._h, int(n), None, 0, C.byref(ln))
        out = (C.c_int32 * max(1, ln.value))()
        N.call("heat2d_solver_step_cycles", self._h, int(n), out, ln.value, C.byref(ln))
        return [int(v) for v in out[:ln.value]]

    def halo_rows_exchanged(self, reset: bool = False) -> int:
        """Halo rows this rank exchanged per side since the last reset (each
        cycle moves the rows the NEXT cycle reads: its depth, not the maximum)."""
        v = C.c_int64()
        N.call("heat2d_solver_halo_rows", self._h, int(bool(reset)), C.byref(v))
        return v.value

    @property
    def plan_cache_hits(self) -> int:
        """Plans / schedules taken from the persistent plan cache (re-validated by one re-time)."""
        v = C.c_int64()
        N.call("heat2d_solver_plan_cache_hits", self._h, C.byref(v))
        return v.value

    @property
    def tune_stats(self) -> dict:
        """{"depths": depths autotuned in this process, "candidates": plans screened for them}."""
        d, c = C.c_int64(), C.c_int64()
        N.call("heat2d_solver_tune_stats", self._h, C.byref(d), C.byref(c))
        return {"depths": d.value, "candidates": c.value}

    @property
    def ghost_rows(self) -> int:
        """Valid ghost rows of the current field (the last exchange's depth)."""
        v = C.c_int32()
        N.call("heat2d_solver_ghost_rows", self._h, C.byref(v))
        return v.value

    @property
    def plans_made(self) -> int:
        """Split plans made so far (each the first use of a depth; autotuned on
        big slabs). After prepare(n), step(n) must not add any."""
        v = C.c_int64()
        N.call("heat2d_solver_plans_made", self._h, C.byref(v))
        return v.value

    @property
    def tb(self) -> int:
        """Largest temporal depth this solver may run (the halo / band depth)."""
        return self.info()["tb"]

    @property
    def pref_depth(self) -> int:
        """Depth of the balanced cycles when no measured schedule applies."""
        v = C.c_int32()
        N.call("heat2d_solver_pref_depth", self._h, C.byref(v))
        return v.value

    @property
    def steps_done(self) -> int:
        return self.info()["steps"]

    # ------------------------------------------------------------------ ops
    def init(self) -> None:
        x = np.ascontiguousarray(self.problem.x, dtype=np.float64)
        ic = self.problem.ic.to_native()
        N.call("heat2d_solver_init", self._h, C.byref(ic), x.ctypes.data_as(C.c_void_p),
               x.ctypes.data_as(C.c_void_p))

    def step(self, n: int = 1) -> None:
        """Advance n time steps (asynchronous on the GPU)."""
        N.call("heat2d_solver_step", self._h, int(n))

    def step_stats(self, n: int) -> dict:
        """step(n), returning the global statistics of the new field and its
        one-step residual T_n - T_{n-1}, fused into the last cycle's stencil
        launch on the HIP engine (no extra pass over the field)."""
        out = (C.c_double * 6)()
        N.call("heat2d_solver_step_stats", self._h, int(n), out)
        s = list(out)
        return {"sum": s[0], "sum_sq": s[1], "min": s[2], "max": s[3], "residual_l2": float(np.sqrt(s[4])),
                "residual_max": s[5]}

    def run(self, ntime: Optional[int] = None) -> None:
        self.step(self.problem.ntime if ntime is None else ntime)

    def synchronize(self) -> None:
        N.call("heat2d_solver_sync", self._h)

    def stats(self, residual: bool = False) -> dict:
        """Global (all-rank) statistics of the current field (a separate pass).
        residual=True: the one-step residual, available only right after a
        depth-1 cycle (else NaN) — step_stats(n) gives it at any depth."""
        out = (C.c_double * 6)()
        N.call("heat2d_solver_stats", self._h, out, int(residual))
        s = list(out)
        d = {"sum": s[0], "sum_sq": s[1], "min": s[2], "max": s[3]}
        if residual:  # NaN unless the last cycle had depth 1 (see step_stats)
            d["residual_l2"] = float(np.sqrt(s[4]))
            d["residual_max"] = s[5]
        return d

    def download(self) -> np.ndarray:
        """This rank's owned rows (nrows x ncols) as a host array."""
        out = np.empty((self.nrows, self.ncols), dtype=self.np_dtype)
        N.call("heat2d_solver_download", self._h, out.ctypes.data_as(C.c_void_p), self.ncols)
        return out

    def upload(self, arr: np.ndarray) -> None:
        """Set this rank's owned rows (collective: followed by a halo exchange)."""
        a = np.ascontiguousarray(arr, dtype=self.np_dtype)
        if a.shape != (self.nrows, self.ncols):
            raise ValueError(f"expected {(self.nrows, self.ncols)}, got {a.shape}")
        N.call("heat2d_solver_upload", self._h, a.ctypes.data_as(C.c_void_p), self.ncols)

    def compare(self, other: "HeatSolver", r0: int = 0, nrows: Optional[int] = None, other_r0: Optional[int] = None
                ) -> dict:
        """This rank's current field, local rows [r0, r0 + nrows), against
        ``other``'s current field, local rows [other_r0, other_r0 + nrows)
        (default: the same rows), on the device (same GPU, dtype and width):
        {"max_abs_diff": max |a - b| (NaN if either holds one), "mismatches":
        elements whose bit patterns differ}. Local to this rank."""
        n = self.nrows - r0 if nrows is None else int(nrows)
        out = (C.c_double * 2)()
        N.call("heat2d_solver_compare", self._h, other._h, int(r0), n, int(r0 if other_r0 is None else other_r0), out)
        return {"max_abs_diff": float(out[0]), "mismatches": int(out[1])}

    def gather(self) -> Optional[np.ndarray]:
        """Whole owned grid on rank 0 (None elsewhere). Uses torch.distributed when size > 1."""
        local = self.download()
        if self.size == 1:
            return local
        import torch
        import torch.distributed as dist
        parts = [None] * self.size if self.rank == 0 else None
        dist.gather_object(local, parts, dst=0)
        return np.concatenate(parts, axis=0) if self.rank == 0 else None

    def close(self) -> None:
        if getattr(self, "_h", None):
            N.call("heat2d_solver_free", self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class LoopbackGroup:
    """P slabs of one domain on a single device (or host), exchanging halos
    through the native loopback transport.

    Every member is a full native solver with its own compute / comm streams,
    split plans and autotuner — one rank of a multi-GPU run — and the halo
    messages are the ones the RCCL transport sends (whole padded rows, shared
    ``halo_msgs`` plan), copied device-to-device and ordered by events. So the
    overlapped multi-rank schedule (both split orders, balanced depths) runs
    with real exchanges on one GPU; results must be bitwise identical to P = 1.
    """

    def __init__(self, problem: Problem, nranks: int, *, dtype: str = "fp64", backend: str = "auto",
                 tb: int = 0, tile_rows: int = 0, device: Optional[int] = None, arith: str = "auto",
                 overlap: bool = True, autotune: int = -1, comm_cus: int = 0, edge_shift: int = 0):
        self.problem = problem
        self.backend = resolve_backend(backend)
        self.dtype = DTYPES[dtype]
        if self.backend == "hip" and device is None:
            import torch
            device = torch.cuda.current_device()
        cfg = N.Config()
        cfg.n_rows = problem.n_owned
        cfg.n_cols = problem.n_owned
        cfg.dtype = self.dtype
        cfg.backend = N.BACKEND_HIP if self.backend == "hip" else N.BACKEND_CPU
        cfg.r = problem.r
        cfg.tb = tb
        cfg.overlap = int(overlap)
        cfg.autotune = autotune
        cfg.comm_cus = comm_cus
        cfg.device = -1 if device is None else int(device)
        cfg.tile_rows = tile_rows
        cfg.arith = N.ARITH[arith]
        cfg.edge_shift = int(edge_shift)
        self.nranks = nranks
        h = C.c_void_p()
        N.call("heat2d_group_create", C.byref(cfg), nranks, C.byref(h))
        self._h = h
        x = np.ascontiguousarray(problem.x, dtype=np.float64)
        ic = problem.ic.to_native()
        N.call("heat2d_group_init", self._h, C.byref(ic), x.ctypes.data_as(C.c_void_p),
               x.ctypes.data_as(C.c_void_p))

    def step(self, n: int) -> None:
        N.call("heat2d_group_step", self._h, int(n))

    def upload(self, arr: np.ndarray) -> None:
        """Whole owned grid -> the members' slabs, then a loopback halo exchange."""
        m = self.problem.n_owned
        a = np.ascontiguousarray(arr, dtype=NP_DTYPES[self.dtype])
        if a.shape != (m, m):
            raise ValueError(f"expected {(m, m)}, got {a.shape}")
        N.call("heat2d_group_upload", self._h, a.ctypes.data_as(C.c_void_p), m)

    def download(self) -> np.ndarray:
        m = self.problem.n_owned
        out = np.empty((m, m), dtype=NP_DTYPES[self.dtype])
        N.call("heat2d_group_download", self._h, out.ctypes.data_as(C.c_void_p), m)
        return out

    def _member(self, i: int):
        h = C.c_void_p()
        N.call("heat2d_group_member", self._h, int(i), C.byref(h))
        return h

    def slabs(self) -> list:
        """(row0, nrows) of every member's slab."""
        out = []
        for i in range(self.nranks):
            L = N.Layout()
            N.call("heat2d_solver_layout", self._member(i), C.byref(L))
            out.append((int(L.row0), int(L.nrows)))
        return out

    def plan(self, i: int, k: int) -> dict:
        """Member i's split plan for depth k (as HeatSolver.plan)."""
        return _plan(self._member(i), k)

    def cycle_hist(self, i: int, reset: bool = False) -> dict:
        return _cycle_hist(self._member(i), reset)

    def close(self) -> None:
        if getattr(self, "_h", None):
            N.call("heat2d_group_free", self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass
