"""Presets reproducing each program of the reference gallery.

Every preset fixes the grid convention, the initial condition, the step-count
rule and the outputs / stdout strings of one reference program; all of them run
on the same native engine (any backend, any number of ranks).
"""
from __future__ import annotations

import dataclasses
from typing import Optional

from ..utils.config import GHOST, INCLUSIVE, InputDat


@dataclasses.dataclass(frozen=True)
class Variant:
    name: str
    reference: str          # reference program(s)
    convention: str         # GHOST (n owned + ghost frame) or INCLUSIVE (n incl. boundary)
    ic: str                 # IC name (utils.config.make_ic)
    outputs: str            # "serial": int.dat + soln.dat; "mpi": soln%05d.dat if soln == 1
    timing_line: str        # "total time:" or "Average time:"
    managed: bool = False
    per_step: bool = False    # the timing line is seconds per iteration (V7 / V8), not the whole run
    sum_line: bool = False    # "Sum of Temperature:" before the completion line (V7)
    extra_step: bool = False  # python variants run nt+1 steps (python/serial/heat.py:48)
    default_input: Optional[InputDat] = None
    notes: str = ""


VARIANTS = {
    "mpi": Variant("mpi", "fortran/hip/heat.F90 + heat_kernel.cpp (V8)",
                   GHOST, "uniform", "mpi", "Average time:", per_step=True,
                   default_input=InputDat(32768, 0.25, 0.05, 1.0, 25000, 0, 6),
                   notes="slab decomposition along x, Dirichlet T=1 ghost frame, T=2 inside; soln%05d.dat per rank"),
    "mpicuda": Variant("mpicuda", "fortran/mpi+cuda/heat.F90 (V7)", GHOST, "uniform", "mpi", "total time:",
                       per_step=True, sum_line=True, default_input=InputDat(100, 0.25, 0.05, 2.0, 10, 1, 6),
                       notes="as mpi; prints \"Sum of Temperature:\" (the reference's gsum is uninitialised, its "
                             "reduction commented out, heat.F90:266-275; here the all-reduced sum) and a "
                             "per-iteration \"total time:\" (heat.F90:292)"),
    "serial": Variant("serial", "fortran/serial/heat.f90 (V3)", INCLUSIVE, "hat", "serial", "total time:",
                      default_input=InputDat(1024, 0.25, 0.05, 2.0, 30, 0, 5),
                      notes="n points incl. boundary, hat T=2 on [0.5,1.5]^2, int.dat + soln.dat"),
    "cuda": Variant("cuda", "fortran/cuda_kernel/heat.F90 (V5), fortran/cuda_cuf/heat.F90 (V4)", INCLUSIVE,
                    "hat-cuda", "serial", "total time:",
                    default_input=InputDat(100, 0.25, 0.05, 2.0, 1000, 0, 5),
                    notes="as serial but the hat covers y in [0.5,1.0]"),
    "managed": Variant("managed", "fortran/cuda_kernel/heat_managed.F90 (V6)", INCLUSIVE, "hat-cuda", "serial",
                       "total time:", managed=True, default_input=InputDat(100, 0.25, 0.05, 2.0, 1000, 0, 5),
                       notes="fields in managed (unified) memory; the reference's host/device race is absent"),
    "python": Variant("python", "python/serial/heat.py (V1)", INCLUSIVE, "python-hat", "serial", "total time:",
                      extra_step=True, default_input=InputDat(31, 0.25, 0.05, 2.0, 10, 0, 5),
                      notes="31x31, index-slice hat u[7:16,7:16]=2, diffuse(10) = 11 steps"),
    "pycuda": Variant("pycuda", "python/cuda/cuda.py (V2)", INCLUSIVE, "pycuda-hat", "serial", "total time:",
                      extra_step=True, default_input=InputDat(4096, 0.25, 0.05, 2.0, 10000, 0, 5),
                      notes="4096^2, nt+1 = 10001 steps; its hot-spot slice is empty, so T stays 1 everywhere"),
}


def get(name: str) -> Variant:
    try:
        return VARIANTS[name]
    except KeyError:
        raise ValueError(f"unknown variant '{name}' ({', '.join(VARIANTS)})") from None


def default_variant(inp: InputDat) -> str:
    """The reference's own choice: 6-field inputs belong to the MPI programs."""
    return "mpi" if inp.nfields >= 6 else "serial"
