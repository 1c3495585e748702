"""ctypes binding of the native engine ``_native/libheat2d.so`` (C ABI:
``csrc/include/heat2d/capi.h``).

The library carries the gfx950 HIP kernels, the CPU twin kernels, the slab
solver runtime and the RCCL / callback transports. It is built in-tree
(``make -C csrc``, or :func:`build`) so that it travels with the repository
snapshot to the GPU box. Loading it is mandatory for every compute path: there
is no silent Python fallback — :func:`lib` raises if the library is missing.

``import torch`` happens before the library is loaded so that the HIP runtime
and RCCL already mapped by PyTorch (same SONAMEs: libamdhip64.so.7,
librccl.so.1) are the ones the engine binds to.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import threading

_PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE_DIR = os.path.join(_PKG_DIR, "_native")
CSRC_DIR = os.path.join(_PKG_DIR, "csrc")
# HEAT2D_LIB: load an alternative build (kernel A/B experiments, bench/ab.py)
LIB_PATH = os.environ.get("HEAT2D_LIB") or os.path.join(NATIVE_DIR, "libheat2d.so")
CLI_PATH = os.path.join(NATIVE_DIR, "heat2d")

F32, F64 = 0, 1
# SolverConfig::arith: reference rounding (bitwise == NumPy golden) | contracted fma(r, sum - 4c, c) |
# jacobi: r == 1/4 only, r * sum (the zero centre weight folded away)
ARITH = {"exact": 0, "fma": 1, "jacobi": 2, "fast": 3, "auto": -1}


def arith_code(arith: str, r: float) -> int:
    """0 / 1 for the raw kernels; "auto" = fma iff r is an exact power of two
    (then the contracted form is bitwise identical to the reference rounding)."""
    import math
    if arith == "auto":
        return 1 if r > 0 and math.frexp(r)[0] == 0.5 else 0
    if arith == "jacobi" and r != 0.25:
        raise ValueError("arith 'jacobi' needs r == 1/4 exactly (sigma = 0.25)")
    return ARITH[arith]
BACKEND_HIP, BACKEND_CPU = 0, 1


class Layout(C.Structure):
    _fields_ = [(n, C.c_int64) for n in ("nrows", "ncols", "halo", "cpad", "pitch", "row0", "nrows_global")]

    def rows_alloc(self) -> int:
        return self.nrows + 2 * self.halo

    def elems(self) -> int:
        return self.rows_alloc() * self.pitch

    def offset(self, i: int, j: int) -> int:
        return (i + self.halo) * self.pitch + (j + self.cpad)

    def as_dict(self) -> dict:
        return {n: getattr(self, n) for n, _ in self._fields_}


class IcParams(C.Structure):
    _fields_ = [
        ("kind", C.c_int32),
        ("a", C.c_double), ("b", C.c_double),
        ("x0", C.c_double), ("x1", C.c_double), ("y0", C.c_double), ("y1", C.c_double),
        ("i0", C.c_int64), ("i1", C.c_int64), ("j0", C.c_int64), ("j1", C.c_int64),
        ("kx", C.c_double), ("ky", C.c_double),
        ("pad", C.c_double),
    ]


class Config(C.Structure):
    _fields_ = [
        ("n_rows", C.c_int64), ("n_cols", C.c_int64),
        ("dtype", C.c_int32), ("backend", C.c_int32),
        ("r", C.c_double),
        ("tb", C.c_int32), ("overlap", C.c_int32), ("copy_swap", C.c_int32), ("managed", C.c_int32),
        ("device", C.c_int32), ("use_graph", C.c_int32),
        ("tile_rows", C.c_int64), ("halo", C.c_int64),
        ("comm_cus", C.c_int32), ("autotune", C.c_int32),
        ("engine", C.c_int32), ("arith", C.c_int32),
        ("edge_shift", C.c_int32), ("slab_row0", C.c_int64), ("slab_rows_global", C.c_int64),
    ]


class Rect(C.Structure):
    _fields_ = [(n, C.c_int64) for n in ("r0", "r1", "s0", "s1", "nb")]


class SplitPlan(C.Structure):
    _fields_ = [
        ("k", C.c_int32), ("ring", C.c_int32), ("valid", C.c_int32), ("nedge", C.c_int32),
        ("main", Rect), ("edge", Rect * 4),
        ("main_waves", C.c_int64), ("edge_waves", C.c_int64), ("main_items", C.c_int64), ("edge_items", C.c_int64),
        ("nrects", C.c_int32), ("flags", C.c_int32), ("rects", Rect * 6),
    ]


class TbPlan(C.Structure):
    _fields_ = [
        ("k", C.c_int32), ("vec", C.c_int32), ("strip_w", C.c_int32), ("useful_w", C.c_int32),
        ("tile_rows", C.c_int64), ("nstrips", C.c_int64), ("ntiles", C.c_int64),
        ("nwaves", C.c_int64), ("nblocks", C.c_int64),
        ("skew", C.c_int32), ("blocks_per_cu", C.c_int32), ("prefetch", C.c_int32), ("main", C.c_int32),
    ]


EXCHANGE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                          C.c_int64, C.c_int32)
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_double), C.c_int32, C.c_int32)
BARRIER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p)
ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64)

_P = C.c_void_p
_I64 = C.c_int64
_LP = C.POINTER(Layout)
_SIGS = {
    "heat2d_last_error": (C.c_char_p, []),
    "heat2d_version": (C.c_int, []),
    "heat2d_max_tb": (C.c_int, []),
    "heat2d_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "heat2d_device_limits": (C.c_int, [C.c_int, C.POINTER(C.c_int64)]),
    "heat2d_wave_times": (C.c_int, [C.POINTER(C.c_uint64), C.c_int64, C.POINTER(C.c_int64)]),
    "heat2d_make_layout": (C.c_int, [_I64, _I64, _I64, _I64, _I64, _LP]),
    "heat2d_parse_input": (C.c_int, [C.c_char_p, C.POINTER(C.c_double)]),
    "heat2d_decompose": (C.c_int, [_I64, C.c_int, C.c_int, C.POINTER(_I64), C.POINTER(_I64)]),
    "heat2d_decompose_shifted": (C.c_int, [_I64, C.c_int, C.c_int, _I64, C.POINTER(_I64), C.POINTER(_I64)]),
    "heat2d_plan_tb": (C.c_int, [C.c_int, _LP, _I64, _I64, C.c_int, _I64, C.POINTER(TbPlan)]),
    "heat2d_plan_split": (C.c_int, [C.c_int, _LP, C.c_int, _I64, C.POINTER(SplitPlan)]),
    "heat2d_solver_prepare": (C.c_int, [_P, _I64]),
    "heat2d_solver_timing": (C.c_int, [_P, C.c_int]),
    "heat2d_jit_create": (C.c_int, [C.c_int, _LP, C.c_double, C.c_int, C.c_int, C.POINTER(_P)]),
    "heat2d_jit_free": (C.c_int, [_P]),
    "heat2d_jit_step": (C.c_int, [_P, _P, _P, _P]),
    "heat2d_jit_render": (C.c_int, [C.c_int, _LP, C.c_double, C.c_int, C.c_char_p, _I64, C.POINTER(_I64)]),
    "heat2d_jit_compile_check": (C.c_int, [C.c_char_p, C.c_char_p, C.POINTER(_I64)]),
    "heat2d_solver_phase_times": (C.c_int, [_P, C.POINTER(C.c_double)]),
    "heat2d_solver_plan": (C.c_int, [_P, C.c_int, C.POINTER(SplitPlan), C.POINTER(C.c_float)]),
    "heat2d_solver_plans_made": (C.c_int, [_P, C.POINTER(C.c_int64)]),
    "heat2d_tb": (C.c_int, [C.c_int, _P, _P, _LP, _I64, _I64, C.c_int, C.c_double, _P, _I64, C.c_int]),
    "heat2d_init_field": (C.c_int, [C.c_int, _P, _LP, C.POINTER(IcParams), _P, _P, _P]),
    "heat2d_stats": (C.c_int, [C.c_int, _P, _P, _LP, _P, _P, _P]),
    "heat2d_stats_work_elems": (_I64, []),
    "heat2d_copy": (C.c_int, [_P, _P, _I64, _P, C.c_int]),
    "heat2d_read": (C.c_int, [_P, _I64, _P, _P, C.c_int]),
    "heat2d_pack_rows": (C.c_int, [C.c_int, _P, _LP, _I64, _I64, _P, _P]),
    "heat2d_unpack_rows": (C.c_int, [C.c_int, _P, _LP, _I64, _I64, _P, _P]),
    "heat2d_cpu_tb": (C.c_int, [C.c_int, _P, _P, _LP, _I64, _I64, C.c_int, C.c_double, C.c_int]),
    "heat2d_cpu_init_field": (C.c_int, [C.c_int, _P, _LP, C.POINTER(IcParams), _P, _P]),
    "heat2d_cpu_stats": (C.c_int, [C.c_int, _P, _P, _LP, _P]),
    "heat2d_rccl_unique_id": (C.c_int, [_P]),
    "heat2d_transport_self": (C.c_int, [C.POINTER(_P)]),
    "heat2d_transport_rccl": (C.c_int, [_P, C.c_int, C.c_int, C.c_int, C.POINTER(_P)]),
    "heat2d_transport_rccl_loop": (C.c_int, [C.c_int, C.POINTER(_P)]),
    "heat2d_transport_callback": (C.c_int, [EXCHANGE_FN, ALLREDUCE_FN, BARRIER_FN, _P, C.c_int, C.c_int,
                                            C.POINTER(_P)]),
    "heat2d_transport_free": (C.c_int, [_P]),
    "heat2d_transport_info": (C.c_int, [_P, C.POINTER(C.c_int32)]),
    "heat2d_device_pci_bus_id": (C.c_int, [C.c_int, C.c_char_p, _I64]),
    "heat2d_install_crash_handler": (C.c_int, []),
    "heat2d_transport_ipc_loop": (C.c_int, [C.c_int, C.POINTER(_P)]),
    "heat2d_transport_ipc": (C.c_int, [ALLGATHER_FN, ALLREDUCE_FN, BARRIER_FN, _P, C.c_int, C.c_int, C.c_int,
                                       C.POINTER(_P)]),
    "heat2d_solver_create": (C.c_int, [C.POINTER(Config), _P, C.POINTER(_P)]),
    "heat2d_solver_free": (C.c_int, [_P]),
    "heat2d_solver_init": (C.c_int, [_P, C.POINTER(IcParams), _P, _P]),
    "heat2d_solver_step": (C.c_int, [_P, _I64]),
    "heat2d_solver_sync": (C.c_int, [_P]),
    "heat2d_solver_stats": (C.c_int, [_P, _P, C.c_int]),
    "heat2d_solver_download": (C.c_int, [_P, _P, _I64]),
    "heat2d_solver_compare": (C.c_int, [_P, _P, _I64, _I64, _I64, _P]),
    "heat2d_solver_footprint": (C.c_int, [C.POINTER(Config), C.c_int, C.c_int, C.POINTER(_I64)]),
    "heat2d_plan_max_grid": (C.c_int, [C.c_int, C.c_int, _I64, C.POINTER(_I64)]),
    "heat2d_mem_info": (C.c_int, [C.c_int, C.POINTER(_I64), C.POINTER(_I64)]),
    "heat2d_solver_upload": (C.c_int, [_P, _P, _I64]),
    "heat2d_solver_layout": (C.c_int, [_P, _LP]),
    "heat2d_solver_info": (C.c_int, [_P, C.POINTER(C.c_int32), C.POINTER(_I64), C.POINTER(_I64),
                                     C.POINTER(_P), C.POINTER(_P)]),
    "heat2d_group_create": (C.c_int, [C.POINTER(Config), C.c_int, C.POINTER(_P)]),
    "heat2d_group_free": (C.c_int, [_P]),
    "heat2d_group_init": (C.c_int, [_P, C.POINTER(IcParams), _P, _P]),
    "heat2d_group_step": (C.c_int, [_P, _I64]),
    "heat2d_group_download": (C.c_int, [_P, _P, _I64]),
    "heat2d_group_upload": (C.c_int, [_P, _P, _I64]),
    "heat2d_group_member": (C.c_int, [_P, C.c_int, C.POINTER(_P)]),
    "heat2d_solver_cycle_hist": (C.c_int, [_P, C.POINTER(C.c_int64), C.c_int, C.c_int]),
    "heat2d_transport_abort": (C.c_int, [_P, C.c_char_p]),
    "heat2d_watchdog_selftest": (C.c_int, [C.c_double, C.c_int, C.c_int, C.c_double, C.POINTER(C.c_double),
                                           C.c_char_p, _I64]),
    "heat2d_solver_pref_depth": (C.c_int, [_P, C.POINTER(C.c_int32)]),
    "heat2d_solver_step_stats": (C.c_int, [_P, _I64, C.POINTER(C.c_double)]),
    "heat2d_dp_schedule": (C.c_int, [_I64, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_int32), _I64,
                                     C.POINTER(_I64), C.POINTER(C.c_double)]),
    "heat2d_near_schedules": (C.c_int, [_I64, C.c_int, C.POINTER(C.c_double), C.c_double, C.c_int,
                                        C.POINTER(C.c_int32), _I64, C.POINTER(_I64), C.POINTER(C.c_double),
                                        C.POINTER(C.c_int32)]),
    "heat2d_search_schedule": (C.c_int, [_I64, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double),
                                         C.POINTER(C.c_int32), _I64, C.POINTER(_I64), C.POINTER(C.c_double),
                                         C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                         C.POINTER(C.c_int32)]),
    "heat2d_solver_schedule": (C.c_int, [_P, _I64, C.POINTER(C.c_int32), _I64, C.POINTER(C.c_int64)]),
    "heat2d_solver_schedule_replayed": (C.c_int, [_P, _I64, C.POINTER(C.c_int32)]),
    "heat2d_write_xyz": (C.c_int, [C.c_char_p, C.c_int, _P, _I64, _I64, _I64, _P, _P, C.c_int]),
    "heat2d_write_npy": (C.c_int, [C.c_char_p, C.c_int, _P, _I64, _I64, _I64]),
    "heat2d_solver_step_cycles": (C.c_int, [_P, _I64, C.POINTER(C.c_int32), _I64, C.POINTER(C.c_int64)]),
    "heat2d_solver_halo_rows": (C.c_int, [_P, C.c_int, C.POINTER(C.c_int64)]),
    "heat2d_solver_ghost_rows": (C.c_int, [_P, C.POINTER(C.c_int32)]),
    "heat2d_autotune_slabs": (C.c_int, [_I64, _I64, C.c_int, C.c_int, C.POINTER(C.c_int32)]),
    "heat2d_solver_plan_cache_hits": (C.c_int, [_P, C.POINTER(C.c_int64)]),
    "heat2d_solver_tune_stats": (C.c_int, [_P, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    "heat2d_plan_cache_path": (C.c_int, [C.c_char_p, _I64]),
    "heat2d_plan_cache_reload": (C.c_int, []),
    "heat2d_plan_cache_put": (C.c_int, [C.c_char_p, C.c_int, _I64, C.c_void_p, C.c_float]),
    "heat2d_plan_cache_get": (C.c_int, [C.c_char_p, C.c_int, _I64, C.c_void_p, C.POINTER(C.c_float),
                                        C.POINTER(C.c_int32)]),
    "heat2d_plan_cache_put_schedule": (C.c_int, [C.c_char_p, _I64, C.POINTER(C.c_int32), _I64]),
    "heat2d_plan_cache_get_schedule": (C.c_int, [C.c_char_p, _I64, C.POINTER(C.c_int32), _I64,
                                                 C.POINTER(C.c_int64)]),
    "heat2d_solver_plan_origin": (C.c_int, [_P, C.c_int, C.POINTER(C.c_int32)]),
}

_lib = None
_lock = threading.Lock()


class NativeError(RuntimeError):
    """An error reported by the native engine."""


def build(jobs: int = 8, quiet: bool = True) -> None:
    """Compile the engine in-tree for gfx950 (hipcc cross-compiles without a GPU)."""
    cmd = ["make", "-C", CSRC_DIR, f"-j{jobs}"]
    out = subprocess.run(cmd, capture_output=True, text=True)
    if out.returncode != 0:
        raise NativeError(f"native build failed:\n{out.stdout[-4000:]}\n{out.stderr[-4000:]}")
    if not quiet:
        print(out.stdout)


def available() -> bool:
    return os.path.exists(LIB_PATH)


def lib():
    """Load (once) and return the native library. Raises if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        import torch  # noqa: F401  (map torch's HIP runtime / RCCL first: shared SONAMEs)
        if not os.path.exists(LIB_PATH):
            raise NativeError(
                f"native engine not built: {LIB_PATH} missing. Run `make -C {CSRC_DIR}` "
                "or `python -c 'import __graft_entry__ as g; g.build()'`.")
        L = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if os.environ.get("HEAT2D_CRASH_BACKTRACE", "1") != "0":
            # a native backtrace on SIGABRT / SIGSEGV / ... (then the previous
            # handler, e.g. Python's faulthandler): names the library that
            # called free() on a glibc heap-check abort
            L.heat2d_install_crash_handler()
        _lib = L
        return _lib


def check(rc: int) -> None:
    if rc != 0:
        raise NativeError(lib().heat2d_last_error().decode(errors="replace"))


def call(name: str, *args):
    """Call a native function returning an int status; raise NativeError on failure."""
    check(getattr(lib(), name)(*args))


def make_layout(nrows: int, ncols: int, halo: int, row0: int = 0, nrows_global: int | None = None) -> Layout:
    out = Layout()
    call("heat2d_make_layout", nrows, ncols, halo, row0, nrows if nrows_global is None else nrows_global,
         C.byref(out))
    return out


def decompose(n: int, nranks: int, rank: int, edge_shift: int = 0) -> tuple[int, int]:
    """(row0, nrows) of `rank`'s slab (common.hpp decompose; edge_shift: rows
    each edge slab gives the middle ones)."""
    r0, nr = C.c_int64(), C.c_int64()
    if edge_shift:
        call("heat2d_decompose_shifted", n, nranks, rank, int(edge_shift), C.byref(r0), C.byref(nr))
    else:
        call("heat2d_decompose", n, nranks, rank, C.byref(r0), C.byref(nr))
    return r0.value, nr.value


def parse_input_native(text: str) -> dict:
    """Parse input.dat text with the C++ parser (csrc/runtime/config.cpp)."""
    out = (C.c_double * 7)()
    call("heat2d_parse_input", text.encode(), out)
    v = list(out)
    return {"n": int(v[0]), "sigma": v[1], "nu": v[2], "dom_len": v[3], "ntime": int(v[4]), "soln": int(v[5]),
            "nfields": int(v[6])}


def plan_tb(dtype: int, layout: Layout, rb: int, re: int, k: int, tile_rows: int = 0) -> TbPlan:
    out = TbPlan()
    call("heat2d_plan_tb", dtype, C.byref(layout), rb, re, k, tile_rows, C.byref(out))
    return out


def plan_split(dtype: int, layout: Layout, k: int, band: int) -> SplitPlan:
    """The MAIN + EDGE launch split of one overlapped cycle (csrc/kernels/stencil_tb.hip)."""
    out = SplitPlan()
    call("heat2d_plan_split", dtype, C.byref(layout), k, band, C.byref(out))
    return out


def autotune_slabs(n_rows: int, n_cols: int, nranks: int, autotune: int = -1) -> bool:
    """Whether a decomposition's slabs are autotuned and run measured schedules
    (decided from the global problem: identical on every rank)."""
    out = C.c_int32()
    call("heat2d_autotune_slabs", n_rows, n_cols, nranks, autotune, C.byref(out))
    return bool(out.value)


def plan_cache_path() -> str:
    """The persistent plan cache file ("" when disabled: HEAT2D_PLAN_CACHE=off)."""
    buf = C.create_string_buffer(4096)
    call("heat2d_plan_cache_path", buf, 4096)
    return buf.value.decode()


def max_tb() -> int:
    return int(lib().heat2d_max_tb())


def device_count() -> int:
    n = C.c_int(0)
    call("heat2d_device_count", C.byref(n))
    return n.value


LIMIT_NAMES = ("MAX_BLOCK_DIM_X", "MAX_BLOCK_DIM_Y", "MAX_BLOCK_DIM_Z", "MAX_GRID_DIM_X", "MAX_GRID_DIM_Y",
               "MAX_GRID_DIM_Z", "TOTAL_CONSTANT_MEMORY", "MAX_THREADS_PER_BLOCK", "WARP_SIZE", "MULTIPROCESSOR_COUNT")


def wave_times(max_waves: int = 1 << 16):
    """Per-wave [start, end, wave, 0] wall-clock ticks (100 MHz on MI355X) of
    the last stencil launch, when the process runs with HEAT2D_WAVE_TIMES=1
    (diagnostics; eager launches). numpy array of shape (n, 4)."""
    import numpy as np
    buf = (C.c_uint64 * (4 * max_waves))()
    n = C.c_int64()
    call("heat2d_wave_times", buf, int(max_waves), C.byref(n))
    return np.frombuffer(buf, dtype=np.uint64, count=4 * n.value).reshape(-1, 4).copy()


def device_limits(device: int = 0) -> dict:
    """The device attributes python/cuda/cuda.py:16-27 queries (plus wave size and CU count)."""
    out = (C.c_int64 * 10)()
    call("heat2d_device_limits", int(device), out)
    return dict(zip(LIMIT_NAMES, (int(v) for v in out)))


def rccl_unique_id() -> bytes:
    buf = (C.c_ubyte * 128)()
    call("heat2d_rccl_unique_id", buf)
    return bytes(buf)


FABRIC_KINDS = {0: "host", 1: "rccl", 2: "ipc"}


def transport_info(handle) -> dict:
    """What the fabric reports for this rank: kind, nranks, rank, device
    (RCCL: ncclCommCount / ncclCommUserRank / ncclCommCuDevice)."""
    out = (C.c_int32 * 4)()
    call("heat2d_transport_info", handle, out)
    return {"kind": FABRIC_KINDS.get(int(out[0]), str(out[0])), "nranks": int(out[1]), "rank": int(out[2]),
            "device": int(out[3])}


def pci_bus_id(device: int) -> str:
    """hipDeviceGetPCIBusId of a device ordinal."""
    buf = C.create_string_buffer(64)
    call("heat2d_device_pci_bus_id", int(device), buf, 64)
    return buf.value.decode()


def loaded_path() -> str:
    return LIB_PATH
