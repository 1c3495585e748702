"""Run-time specialised FTCS kernels (hipRTC) — the capability of the
reference's PyCUDA program (python/cuda/cuda.py:58-89: a Jinja2-rendered CUDA-C
kernel with the grid sizes and r baked in, compiled by SourceModule at run
time). :func:`render` gives the HIP source for a slab layout and r;
:class:`JitStencil` compiles it for the running GPU (hipRTC, cached per source)
and steps torch tensors laid out per ``ops.kernels`` on torch's current stream.
Bitwise identical to the temporal-blocked engine (same summation order, same
``arith``: reference rounding, or the contracted fma form). Native code: ``csrc/runtime/jit.cpp``.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _native as N
from .kernels import _check_field, _stream, dtype_code


def render(dtype: int, layout: N.Layout, r: float, arith: str = "exact") -> str:
    """HIP source of one FTCS step specialised for ``layout`` and ``r``."""
    n = C.c_int64()
    ar = N.arith_code(arith, r)
    N.call("heat2d_jit_render", dtype, C.byref(layout), float(r), ar, None, 0, C.byref(n))
    buf = C.create_string_buffer(n.value + 1)
    N.call("heat2d_jit_render", dtype, C.byref(layout), float(r), ar, buf, n.value + 1, C.byref(n))
    return buf.value.decode()


def compile_check(source: str, arch: str = "gfx950") -> int:
    """Compile HIP source with hipRTC for ``arch`` (no GPU needed); returns the code-object size."""
    nbytes = C.c_int64()
    N.call("heat2d_jit_compile_check", source.encode(), arch.encode(), C.byref(nbytes))
    return nbytes.value


class JitStencil:
    """One FTCS step per call, compiled at run time for this layout, dtype and r."""

    def __init__(self, dtype: torch.dtype, layout: N.Layout, r: float, device: int | None = None,
                 arith: str = "exact"):
        self.layout = layout
        self.dtype = dtype
        self.r = float(r)
        code = N.F32 if dtype == torch.float32 else N.F64
        dev = torch.cuda.current_device() if device is None else device
        h = C.c_void_p()
        N.call("heat2d_jit_create", code, C.byref(layout), self.r, dev, N.arith_code(arith, self.r), C.byref(h))
        self._h = h
        self.source = render(code, layout, self.r, arith)

    def step(self, src: torch.Tensor, dst: torch.Tensor) -> None:
        """dst(owned rows) = one FTCS step of src (both CUDA tensors of layout.elems() elements)."""
        for t in (src, dst):
            _check_field(t, self.layout)
            if not t.is_cuda or t.dtype != self.dtype:
                raise ValueError("JitStencil steps device tensors of its own dtype")
        dtype_code(src)
        N.call("heat2d_jit_step", self._h, C.c_void_p(src.data_ptr()), C.c_void_p(dst.data_ptr()), _stream(src))

    def close(self) -> None:
        if getattr(self, "_h", None):
            N.call("heat2d_jit_free", self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass
