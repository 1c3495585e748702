"""heat2d — MI355X-native 2-D heat-equation framework.

Same capabilities as cssrikanth/CUDA-HIP-MPI-Heat-equation-test (input.dat
driven explicit FTCS solver: serial, single-GPU, managed-memory and
multi-GPU slab-decomposed variants, int.dat/soln.dat outputs, plotting),
re-designed for AMD Instinct MI355X (gfx950): hand-written temporal-blocked
HIP stencil kernels, a native C++ slab runtime, RCCL halo exchange over xGMI.

Layout:
  ops/       native engine binding (ctypes) + raw kernel ops on torch tensors
  models/    the heat model (HeatSolver), reference-variant presets, NumPy golden
  parallel/  decomposition, transports (RCCL / torch.distributed / callbacks), launcher
  utils/     input.dat config, I/O, plotting, metrics, checkpoint/restart
  csrc/      C++/HIP sources (kernels, runtime, CPU twins, C ABI, native CLI)
"""
__version__ = "0.1.0"

from .utils.config import InputDat, Problem, make_problem, parse_input_text, read_input  # noqa: F401


def __getattr__(name):
    # lazy: importing the models pulls in the native library / torch
    if name in ("HeatSolver", "LoopbackGroup"):
        from .models import heat2d as _m
        return getattr(_m, name)
    if name in ("plan_max_grid", "footprint"):  # the memory-fit planner (utils/memplan.py)
        from .utils import memplan as _p
        return getattr(_p, name)
    raise AttributeError(name)
