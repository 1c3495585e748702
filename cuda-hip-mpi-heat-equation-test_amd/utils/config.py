"""``input.dat`` parsing and problem set-up.

The reference reads ``n, sigma, nu, dom_len, ntime [, soln]`` with a Fortran
list-directed ``read(11,*)`` from ``./input.dat`` (fortran/serial/heat.f90:11-13,
fortran/hip/heat.F90:136-140; fields documented in README.md:7). This module
accepts the same files (blank/comma separated, newlines, ``1.0d0`` exponents,
``r*c`` repeats, ``/`` terminator) and resolves them, per grid convention,
into the exact solver parameters the reference computes:

    delta = dom_len/real(n-1); dt = (sigma*delta**2)/nu; r = (nu*dt)/delta**2
    (fortran/hip/heat.F90:178-182)

so ``r`` equals ``sigma`` only up to rounding, exactly as in the reference.
The C++ twin is ``csrc/runtime/config.cpp``.
"""
from __future__ import annotations

import dataclasses
import os
import re
from typing import Optional

import numpy as np

# IC kinds (must match kern::IcKind)
IC_UNIFORM, IC_BOX, IC_INDEX_BOX, IC_SINE, IC_CONST = 0, 1, 2, 3, 4


@dataclasses.dataclass
class InputDat:
    n: int
    sigma: float
    nu: float
    dom_len: float
    ntime: int
    soln: int = 0
    nfields: int = 5

    def to_text(self) -> str:
        base = f"{self.n} {self.sigma!r} {self.nu!r} {self.dom_len!r} {self.ntime}"
        return base + (f" {self.soln}" if self.nfields >= 6 else "") + "\n"


def _tokens(text: str) -> list[str]:
    text = text.split("/", 1)[0]
    out: list[str] = []
    for tok in re.split(r"[\s,;]+", text):
        if not tok:
            continue
        m = re.fullmatch(r"(\d+)\*(.+)", tok)
        if m:
            out.extend([m.group(2)] * int(m.group(1)))
        else:
            out.append(tok)
    return out


def _real(tok: str) -> float:
    return float(re.sub(r"[dDqQ]", "e", tok))


def parse_input_text(text: str) -> InputDat:
    tok = _tokens(text)
    if len(tok) < 5:
        raise ValueError("input.dat needs at least 5 fields: n sigma nu dom_len ntime [soln]")
    inp = InputDat(n=int(tok[0]), sigma=_real(tok[1]), nu=_real(tok[2]), dom_len=_real(tok[3]),
                   ntime=int(tok[4]))
    if len(tok) >= 6:
        inp.soln = int(tok[5])
        inp.nfields = 6
    if inp.n < 3:
        raise ValueError("grid size must be >= 3")
    if inp.nu <= 0 or inp.dom_len <= 0:
        raise ValueError("nu and dom_len must be positive")
    if inp.ntime < 0:
        raise ValueError("ntime must be >= 0")
    return inp


def read_input(path: str = "input.dat") -> InputDat:
    with open(path) as f:
        return parse_input_text(f.read())


def write_input(path: str, inp: InputDat) -> None:
    with open(path, "w") as f:
        f.write(inp.to_text())


def coefficients(n: int, sigma: float, nu: float, dom_len: float) -> tuple[float, float, float]:
    """(delta, dt, r) in the reference's floating-point order."""
    delta = dom_len / float(n - 1)
    dt = (sigma * (delta * delta)) / nu
    r = (nu * dt) / (delta * delta)
    return delta, dt, r


@dataclasses.dataclass
class IcSpec:
    """Mirror of kern::IcParams."""
    kind: int = IC_UNIFORM
    a: float = 2.0
    b: float = 1.0
    x0: float = 0.0
    x1: float = 0.0
    y0: float = 0.0
    y1: float = 0.0
    i0: int = 0
    i1: int = 0
    j0: int = 0
    j1: int = 0
    kx: float = 1.0
    ky: float = 1.0
    pad: float = 1.0

    def sterbenz_safe(self) -> bool:
        """Every value this IC puts in the field lies in [m, 2m], m > 0 (the
        C++ twin: config.hpp ic_sterbenz_safe). FTCS at r <= 1/4 keeps the
        field in that range, so every sum - 4c is exact and the r = 1/4 form
        ("jacobi") rounds bitwise like the reference update."""
        if self.kind in (IC_UNIFORM, IC_BOX, IC_INDEX_BOX):
            vals = (self.a, self.b, self.pad)
        elif self.kind == IC_CONST:
            vals = (self.a, self.pad)
        else:
            return False
        return min(vals) > 0 and max(vals) <= 2 * min(vals)

    def absmax(self) -> float:
        """max |T| this IC puts in the field (frame included): the scale of the
        stated error bounds (models/reference.fast_error_bound). FTCS at
        r <= 1/4 never exceeds it."""
        if self.kind == IC_SINE:
            return abs(self.a)
        if self.kind == IC_CONST:
            return max(abs(self.a), abs(self.pad))
        return max(abs(self.a), abs(self.b), abs(self.pad))

    def to_native(self):
        from ..ops import _native as N
        p = N.IcParams()
        for f in dataclasses.fields(self):
            setattr(p, f.name, getattr(self, f.name))
        return p


def make_ic(name: str, dom_len: float = 2.0, coords: Optional[np.ndarray] = None) -> IcSpec:
    """Initial/boundary conditions of the reference variants (+ synthetic ones)."""
    if name in ("uniform", "mpi"):  # fortran/hip/heat.F90:274-282: T=2 inside, Dirichlet frame T=1
        return IcSpec(kind=IC_UNIFORM, a=2.0, b=1.0)
    if name in ("hat", "serial"):  # fortran/serial/heat.f90:40-48
        return IcSpec(kind=IC_BOX, a=2.0, b=1.0, x0=0.5, x1=1.5, y0=0.5, y1=1.5)
    if name in ("hat-cuda", "cuda"):  # fortran/cuda_kernel/heat.F90:97-105, fortran/cuda_cuf/heat.F90:84-92
        return IcSpec(kind=IC_BOX, a=2.0, b=1.0, x0=0.5, x1=1.5, y0=0.5, y1=1.0)
    if name == "hotspot":  # synthetic benchmark data: zero field + unit hot spot
        L = dom_len
        return IcSpec(kind=IC_BOX, a=1.0, b=0.0, x0=0.4 * L, x1=0.6 * L, y0=0.4 * L, y1=0.6 * L, pad=0.0)
    if name in ("python-hat", "pycuda-hat", "const-1"):
        # python/serial/heat.py:25 : u[int(.5/dy):int(1/dy+1), int(.5/dx):int(1/dx+1)] = 2 (frame-inclusive
        # indices); python/cuda/cuda.py:53 slices [int(1.5/dy):int(1/dy+1)], an EMPTY range -> all ones.
        n = len(coords) if coords is not None else 31
        d = dom_len / (n - 1)
        lo = int((1.5 if name != "python-hat" else 0.5) / d)
        hi = int(1 / d + 1)
        return IcSpec(kind=IC_INDEX_BOX, a=2.0, b=1.0, i0=lo, i1=hi, j0=lo, j1=hi)
    if name == "sine":  # analytic FTCS eigenmode (zero Dirichlet)
        lo = float(coords[0]) if coords is not None else 0.0
        hi = float(coords[-1]) if coords is not None else dom_len
        return IcSpec(kind=IC_SINE, a=1.0, x0=lo, x1=hi, y0=lo, y1=hi, kx=1.0, ky=1.0, pad=0.0)
    raise ValueError(f"unknown IC '{name}' (uniform|hat|hat-cuda|hotspot|sine|python-hat|pycuda-hat)")


GHOST, INCLUSIVE = "ghost", "inclusive"


@dataclasses.dataclass
class Problem:
    """A fully resolved run: grid, coefficients, coordinates and IC."""
    convention: str
    n_input: int          # n as written in input.dat
    n_owned: int          # owned (updated) points per axis
    sigma: float
    nu: float
    dom_len: float
    ntime: int
    delta: float
    dt: float
    r: float
    x: np.ndarray         # n_owned + 2 frame-inclusive coordinates (x and y share them)
    ic: IcSpec
    soln: int = 0

    @property
    def points(self) -> int:
        return self.n_owned * self.n_owned


def coordinates(n: int, dom_len: float, delta: float, convention: str) -> np.ndarray:
    if convention == GHOST:
        # xg(i) = (i-1)*delta, i = 0..n+1 (fortran/hip/heat.F90:184-186)
        return np.arange(-1, n + 1, dtype=np.float64) * delta
    # boundary-inclusive: x(1)=0, x(n)=L, interior by cumulative sums (fortran/serial/heat.f90:28-36)
    x = np.empty(n, dtype=np.float64)
    x[0] = 0.0
    acc = 0.0
    for i in range(1, n - 1):
        acc = acc + delta
        x[i] = acc
    x[n - 1] = dom_len
    return x


def make_problem(inp: InputDat, convention: str = GHOST, ic: str = "uniform") -> Problem:
    delta, dt, r = coefficients(inp.n, inp.sigma, inp.nu, inp.dom_len)
    x = coordinates(inp.n, inp.dom_len, delta, convention)
    n_owned = inp.n if convention == GHOST else inp.n - 2
    spec = make_ic(ic, inp.dom_len, x)
    return Problem(convention=convention, n_input=inp.n, n_owned=n_owned, sigma=inp.sigma, nu=inp.nu,
                   dom_len=inp.dom_len, ntime=inp.ntime, delta=delta, dt=dt, r=r, x=x, ic=spec, soln=inp.soln)


def default_input_path() -> str:
    return os.path.join(os.getcwd(), "input.dat")
