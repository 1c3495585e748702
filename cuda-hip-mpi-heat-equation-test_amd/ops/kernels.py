"""Raw kernel ops on PyTorch tensors (device or host), backed by the native engine.

A field is a flat 1-D tensor of ``layout.elems()`` elements laid out as
``csrc/include/heat2d/common.hpp`` describes (row-major, ``halo`` ghost rows
above/below, ``cpad`` padding columns on the left, 256-B aligned pitch). These
ops run on torch's current HIP stream, so they compose with torch code and with
stream capture. CUDA(HIP) tensors dispatch to the gfx950 kernels, CPU tensors to
the CPU twins — the results are bitwise identical.

Reference kernels replaced: ``heat_eqn`` (fortran/hip/heat_kernel.cpp:31-61) ->
:func:`tb_step`; ``swap_send`` / ``swap_recv1`` / ``swap_recv2`` (:63-150) ->
:func:`pack_rows` / :func:`unpack_rows`; the commented-out checksum
(fortran/hip/heat.F90:297-306) -> :func:`stats`.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np
import torch

from . import _native as N

TORCH_DTYPES = {N.F32: torch.float32, N.F64: torch.float64}


def dtype_code(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return N.F32
    if t.dtype == torch.float64:
        return N.F64
    raise TypeError(f"unsupported dtype {t.dtype} (fp32 / fp64)")


def _stream(t: torch.Tensor):
    return C.c_void_p(torch.cuda.current_stream(t.device).cuda_stream) if t.is_cuda else None


def _check_field(t: torch.Tensor, layout: N.Layout) -> None:
    if t.dim() != 1 or not t.is_contiguous():
        raise ValueError("field must be a contiguous 1-D tensor")
    if t.numel() != layout.elems():
        raise ValueError(f"field has {t.numel()} elements, layout needs {layout.elems()}")


def make_layout(nrows: int, ncols: int, halo: int = 16, row0: int = 0,
                nrows_global: Optional[int] = None) -> N.Layout:
    return N.make_layout(nrows, ncols, halo, row0, nrows if nrows_global is None else nrows_global)


def empty_field(layout: N.Layout, dtype=torch.float64, device="cuda") -> torch.Tensor:
    return torch.empty(layout.elems(), dtype=dtype, device=device)


def view2d(field: torch.Tensor, layout: N.Layout) -> torch.Tensor:
    """(rows_alloc, pitch) view of a field (ghost rows / pad columns included)."""
    return field.view(layout.rows_alloc(), layout.pitch)


def owned(field: torch.Tensor, layout: N.Layout) -> torch.Tensor:
    """(nrows, ncols) view of the owned region."""
    v = view2d(field, layout)
    return v[layout.halo:layout.halo + layout.nrows, layout.cpad:layout.cpad + layout.ncols]


def init_field(field: torch.Tensor, layout: N.Layout, ic, xcoord: np.ndarray,
               ycoord: Optional[np.ndarray] = None) -> None:
    """Fill the whole allocation from an IC (utils.config.IcSpec). ``xcoord`` holds
    nrows_global+2 frame-inclusive x coordinates, ``ycoord`` ncols+2 (default: xcoord)."""
    _check_field(field, layout)
    ycoord = xcoord if ycoord is None else ycoord
    p = ic.to_native() if hasattr(ic, "to_native") else ic
    if field.is_cuda:
        xd = torch.as_tensor(np.ascontiguousarray(xcoord, np.float64), device=field.device)
        yd = torch.as_tensor(np.ascontiguousarray(ycoord, np.float64), device=field.device)
        N.call("heat2d_init_field", dtype_code(field), C.c_void_p(field.data_ptr()), C.byref(layout), C.byref(p),
               C.c_void_p(xd.data_ptr()), C.c_void_p(yd.data_ptr()), _stream(field))
        torch.cuda.current_stream(field.device).synchronize()  # keep xd/yd alive until done
    else:
        xh = np.ascontiguousarray(xcoord, np.float64)
        yh = np.ascontiguousarray(ycoord, np.float64)
        N.call("heat2d_cpu_init_field", dtype_code(field), C.c_void_p(field.data_ptr()), C.byref(layout),
               C.byref(p), xh.ctypes.data_as(C.c_void_p), yh.ctypes.data_as(C.c_void_p))


def tb_step(src: torch.Tensor, dst: torch.Tensor, layout: N.Layout, k: int, r: float,
            rows: Optional[tuple[int, int]] = None, tile_rows: int = 0, arith: str = "exact") -> None:
    """dst[rows] = k FTCS steps of src (temporal-blocked kernel). The k ghost rows
    around ``rows`` must be valid in ``src``; Dirichlet rows/cols are kept.
    ``arith``: "exact" (reference rounding), "fma" (contracted update) or
    "jacobi" (r == 1/4: r * sum)."""
    _check_field(src, layout)
    _check_field(dst, layout)
    if src.dtype != dst.dtype or src.device != dst.device:
        raise ValueError("src/dst dtype/device mismatch")
    if src.data_ptr() == dst.data_ptr():
        raise ValueError("tb_step is out-of-place (ping-pong fields)")
    rb, re = (0, layout.nrows) if rows is None else rows
    ar = N.arith_code(arith, r)
    if src.is_cuda:
        N.call("heat2d_tb", dtype_code(src), C.c_void_p(src.data_ptr()), C.c_void_p(dst.data_ptr()),
               C.byref(layout), rb, re, k, r, _stream(src), tile_rows, ar)
    else:
        N.call("heat2d_cpu_tb", dtype_code(src), C.c_void_p(src.data_ptr()), C.c_void_p(dst.data_ptr()),
               C.byref(layout), rb, re, k, r, ar)


def stats(field: torch.Tensor, layout: N.Layout, other: Optional[torch.Tensor] = None) -> dict:
    """sum, sum of squares, min, max (+ L2 / max-abs difference vs `other`) of the owned region."""
    _check_field(field, layout)
    optr = C.c_void_p(other.data_ptr()) if other is not None else None
    if field.is_cuda:
        work = torch.empty(int(N.lib().heat2d_stats_work_elems()) + 8, dtype=torch.float64, device=field.device)
        out = work[-8:]
        N.call("heat2d_stats", dtype_code(field), C.c_void_p(field.data_ptr()), optr, C.byref(layout),
               C.c_void_p(work.data_ptr()), C.c_void_p(out.data_ptr()), _stream(field))
        v = out[:6].cpu().tolist()
    else:
        o = (C.c_double * 6)()
        N.call("heat2d_cpu_stats", dtype_code(field), C.c_void_p(field.data_ptr()), optr, C.byref(layout), o)
        v = list(o)
    d = {"sum": v[0], "sum_sq": v[1], "min": v[2], "max": v[3]}
    if other is not None:
        d["diff_l2"] = float(np.sqrt(v[4]))
        d["diff_max"] = v[5]
    return d


def pack_rows(field: torch.Tensor, layout: N.Layout, row: int, nrows: int,
              out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Copy owned columns of rows [row, row+nrows) into a contiguous (nrows*ncols) buffer."""
    _check_field(field, layout)
    if out is None:
        out = torch.empty(nrows * layout.ncols, dtype=field.dtype, device=field.device)
    if field.is_cuda:
        N.call("heat2d_pack_rows", dtype_code(field), C.c_void_p(field.data_ptr()), C.byref(layout), row, nrows,
               C.c_void_p(out.data_ptr()), _stream(field))
    else:
        out.view(nrows, layout.ncols).copy_(view2d(field, layout)[layout.halo + row:layout.halo + row + nrows,
                                                                   layout.cpad:layout.cpad + layout.ncols])
    return out


def unpack_rows(field: torch.Tensor, layout: N.Layout, row: int, nrows: int, buf: torch.Tensor) -> None:
    _check_field(field, layout)
    if field.is_cuda:
        N.call("heat2d_unpack_rows", dtype_code(field), C.c_void_p(field.data_ptr()), C.byref(layout), row, nrows,
               C.c_void_p(buf.data_ptr()), _stream(field))
    else:
        view2d(field, layout)[layout.halo + row:layout.halo + row + nrows,
                              layout.cpad:layout.cpad + layout.ncols].copy_(buf.view(nrows, layout.ncols))


def copy_(dst: torch.Tensor, src: torch.Tensor) -> None:
    """Vectorised 16-B streaming device copy (the copy-swap parity op)."""
    nbytes = src.numel() * src.element_size()
    if not (src.is_cuda and dst.is_cuda) or nbytes % 16:
        dst.copy_(src)
        return
    N.call("heat2d_copy", C.c_void_p(dst.data_ptr()), C.c_void_p(src.data_ptr()), nbytes, _stream(src), 0)
