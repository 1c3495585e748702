"""NumPy golden models (the test oracle; no native code).

* :func:`initial_field` / :func:`ftcs` — the frame-inclusive FTCS solver in the
  reference's exact arithmetic order ``c + r*((((S + E) + N) + W) - 4c)``
  (fortran/hip/heat_kernel.cpp:43, fortran/serial/heat.f90:66). The native
  engine (any K, any P, CPU or GPU) must match it **bitwise**.
* :func:`python_serial_demo` — python/serial/heat.py as written (31x31, index-slice
  hat, ``diffuse(10)`` = 11 steps, its own update formula).
* :func:`eigenmode` — closed form of FTCS on a zero-Dirichlet sine mode:
  ``T_m = g^m T_0``, ``g = 1 - 4r(sin^2(k pi d/2L) + sin^2(l pi d/2L))``.
"""
from __future__ import annotations

import numpy as np

from ..utils.config import (IC_BOX, IC_CONST, IC_INDEX_BOX, IC_SINE, IC_UNIFORM, IcSpec, Problem)


def initial_field(problem: Problem, dtype=np.float64) -> np.ndarray:
    """Frame-inclusive (m+2)x(m+2) initial field (row = x index, column = y index)."""
    x = problem.x
    m = problem.n_owned
    ic: IcSpec = problem.ic
    X = x[:, None]
    Y = x[None, :]
    frame = np.zeros((m + 2, m + 2), dtype=bool)
    frame[0, :] = frame[-1, :] = frame[:, 0] = frame[:, -1] = True
    if ic.kind == IC_UNIFORM:
        T = np.where(frame, ic.b, ic.a)
    elif ic.kind == IC_BOX:
        inside = (X <= ic.x1) & (X >= ic.x0) & (Y <= ic.y1) & (Y >= ic.y0)
        T = np.where(inside, ic.a, ic.b)
    elif ic.kind == IC_INDEX_BOX:
        gi = np.arange(m + 2)[:, None]
        gj = np.arange(m + 2)[None, :]
        inside = (gi >= ic.i0) & (gi < ic.i1) & (gj >= ic.j0) & (gj < ic.j1)
        T = np.where(inside, ic.a, ic.b)
    elif ic.kind == IC_SINE:
        T = ic.a * np.sin(ic.kx * np.pi * (X - ic.x0) / (ic.x1 - ic.x0)) * \
            np.sin(ic.ky * np.pi * (Y - ic.y0) / (ic.y1 - ic.y0))
        T = np.where(frame, 0.0, T)
    elif ic.kind == IC_CONST:
        T = np.full((m + 2, m + 2), ic.a)
    else:
        raise ValueError(ic.kind)
    return np.ascontiguousarray(T, dtype=np.float64).astype(dtype)


def ftcs_step(T: np.ndarray, r, arith: str = "exact") -> np.ndarray:
    """One FTCS step of a frame-inclusive field (frame kept fixed).
    arith "jacobi" (r == 1/4 only): r * sum, the zero centre weight folded
    away — the engine's arith 2."""
    r = T.dtype.type(r)
    four = T.dtype.type(4)
    c = T[1:-1, 1:-1]
    south = T[2:, 1:-1]   # x+1
    east = T[1:-1, 2:]    # y+1
    north = T[:-2, 1:-1]  # x-1
    west = T[1:-1, :-2]   # y-1
    out = T.copy()
    if arith == "jacobi":
        if r != 0.25:
            raise ValueError("arith 'jacobi' needs r == 1/4")
        out[1:-1, 1:-1] = r * (((south + east) + north) + west)
    else:
        out[1:-1, 1:-1] = c + r * ((((south + east) + north) + west) - four * c)
    return out


def ftcs(problem: Problem, nsteps: int | None = None, dtype=np.float64, T0: np.ndarray | None = None,
         arith: str = "exact") -> np.ndarray:
    """Run FTCS; returns the frame-inclusive field."""
    T = initial_field(problem, dtype) if T0 is None else T0.astype(dtype)
    n = problem.ntime if nsteps is None else nsteps
    for _ in range(n):
        T = ftcs_step(T, problem.r, arith)
    return T


def fast_error_bound(nsteps: int, dtype, tmax: float) -> float:
    """Stated bound of the scaled-level arithmetic ("fast", the kernels' AR 3)
    against the reference rounding ("exact") after ``nsteps`` steps from a
    field with max |T0| = tmax, for r <= 1/4:

        max |T_fast - T_exact| <= 16 * nsteps * u * tmax,   u = eps / 2.

    Per step the reference form rounds ~6 times on values <= tmax (the sum,
    sum - 4c, r * (...), c + ...) and the scaled form ~5 times (sum, fma, and
    the rounded coefficient b = (1 - 4r) / r), plus 2 per pass for r^K and the
    unscaling multiply; FTCS with r <= 1/4 is non-expansive in the max norm, so
    per-step errors add up at most linearly (16 > 6 + 5 + 2 covers both)."""
    u = float(np.finfo(dtype).eps) / 2.0
    return 16.0 * nsteps * u * tmax


def owned(T: np.ndarray) -> np.ndarray:
    return T[1:-1, 1:-1]


def python_serial_demo(nx: int = 31, nt: int = 10, nu: float = 0.05, sigma: float = 0.25) -> np.ndarray:
    """python/serial/heat.py:8-58 verbatim semantics (without the plots)."""
    ny = nx
    dx = 2 / (nx - 1)
    dy = 2 / (ny - 1)
    dt = sigma * dx * dy / nu
    u = np.ones((ny, nx))
    u[int(.5 / dy):int(1 / dy + 1), int(.5 / dx):int(1 / dx + 1)] = 2
    for _ in range(nt + 1):
        un = u.copy()
        u[1:-1, 1:-1] = (un[1:-1, 1:-1] + nu * dt / dx ** 2 * (un[1:-1, 2:] - 2 * un[1:-1, 1:-1] + un[1:-1, 0:-2])
                         + nu * dt / dy ** 2 * (un[2:, 1:-1] - 2 * un[1:-1, 1:-1] + un[0:-2, 1:-1]))
        u[0, :] = 1
        u[-1, :] = 1
        u[:, 0] = 1
        u[:, -1] = 1
    return u


def eigen_factor(problem: Problem, kx: float = 1.0, ky: float = 1.0) -> float:
    """Per-step amplification g of the sine mode on the boundary-inclusive grid."""
    L = problem.x[-1] - problem.x[0]
    d = problem.delta
    return 1.0 - 4.0 * problem.r * (np.sin(kx * np.pi * d / (2 * L)) ** 2 + np.sin(ky * np.pi * d / (2 * L)) ** 2)


def eigenmode(problem: Problem, nsteps: int) -> np.ndarray:
    """Closed-form FTCS solution for the `sine` IC (frame-inclusive)."""
    T0 = initial_field(problem, np.float64)
    return T0 * eigen_factor(problem, problem.ic.kx, problem.ic.ky) ** nsteps
