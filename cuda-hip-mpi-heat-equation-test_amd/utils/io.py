"""Output files.

* ``x y T`` ASCII triples, x outer / y inner, one point per line — the
  reference's ``int.dat`` / ``soln.dat`` (fortran/serial/heat.f90:50-55,77-83)
  and per-rank ``soln%05d.dat`` (fortran/hip/heat.F90:308-319). Written by the
  native multi-threaded formatter (17 significant digits: exact round trip).
* ``.npy`` binary dumps for large grids.
* readers + the per-rank merge the reference leaves to the user (its
  ``fortran/mpi+cuda/out.py:7`` reads ``soln.dat`` while the solver writes
  ``soln%05d.dat``; ranks own contiguous x-slabs, so rank order == global order).
"""
from __future__ import annotations

import ctypes as C
import glob
import os
from typing import Optional

import numpy as np

from ..ops import _native as N


def write_xyz(path: str, T: np.ndarray, x: np.ndarray, y: np.ndarray, append: bool = False) -> None:
    """T: (len(x), len(y)) array; writes len(x)*len(y) lines."""
    T = np.ascontiguousarray(T)
    dt = N.F64 if T.dtype == np.float64 else N.F32
    if T.dtype not in (np.float64, np.float32):
        T = T.astype(np.float64)
        dt = N.F64
    x = np.ascontiguousarray(x, np.float64)
    y = np.ascontiguousarray(y, np.float64)
    if T.shape != (len(x), len(y)):
        raise ValueError(f"T shape {T.shape} != ({len(x)}, {len(y)})")
    N.call("heat2d_write_xyz", path.encode(), dt, T.ctypes.data_as(C.c_void_p), T.shape[0], T.shape[1],
           T.shape[1], x.ctypes.data_as(C.c_void_p), y.ctypes.data_as(C.c_void_p), int(append))


def write_npy(path: str, T: np.ndarray) -> None:
    np.save(path, np.ascontiguousarray(T), allow_pickle=False)


def read_xyz(path: str) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Parse a triples file (any whitespace, lines with exactly 3 fields — the rule
    of fortran/serial/out.py:17-26); returns x (nx,), y (ny,), T (nx, ny)."""
    rows = []
    with open(path) as f:
        for line in f:
            parts = line.split()
            if len(parts) == 3:
                rows.append([float(p.replace("D", "E").replace("d", "e")) for p in parts])
    a = np.asarray(rows, dtype=np.float64)
    if a.size == 0:
        raise ValueError(f"{path}: no x y T triples")
    xs = a[:, 0]
    # x is the outer index: the first run of equal x values gives ny
    ny = int(np.argmax(xs != xs[0])) if np.any(xs != xs[0]) else len(xs)
    nx = len(xs) // ny
    if nx * ny != len(xs):
        raise ValueError(f"{path}: {len(xs)} points do not form a grid")
    T = a[:, 2].reshape(nx, ny)
    return a[::ny, 0].copy(), a[:ny, 1].copy(), T


def rank_files(directory: str = ".", stem: str = "soln") -> list[str]:
    return sorted(glob.glob(os.path.join(directory, f"{stem}[0-9][0-9][0-9][0-9][0-9].dat")))


def merge_rank_files(directory: str = ".", out: Optional[str] = "soln.dat", stem: str = "soln") -> str:
    """Concatenate soln%05d.dat in rank order into one global file (== `cat soln0*.dat`)."""
    files = rank_files(directory, stem)
    if not files:
        raise FileNotFoundError(f"no {stem}%05d.dat files in {directory}")
    dst = os.path.join(directory, out)
    with open(dst, "wb") as fo:
        for fn in files:
            with open(fn, "rb") as fi:
                while True:
                    b = fi.read(1 << 24)
                    if not b:
                        break
                    fo.write(b)
    return dst
