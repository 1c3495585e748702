"""Import alias for the framework package.

The package lives in ``cuda-hip-mpi-heat-equation-test_amd/`` (a directory name
that is not a valid Python identifier). Importing ``heat2d`` from the repository
root loads that directory as the package ``heat2d`` and replaces this module in
``sys.modules``, so ``import heat2d.models`` etc. work as usual.
"""
import importlib.util
import os
import sys

_PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cuda-hip-mpi-heat-equation-test_amd")
_spec = importlib.util.spec_from_file_location("heat2d", os.path.join(_PKG_DIR, "__init__.py"),
                                               submodule_search_locations=[_PKG_DIR])
_mod = importlib.util.module_from_spec(_spec)
sys.modules["heat2d"] = _mod
_spec.loader.exec_module(_mod)

if __name__ == "__main__":  # `python -m heat2d [input.dat] [flags]` (torchrun -m heat2d ...)
    from heat2d.parallel.launch import run

    sys.exit(run())
