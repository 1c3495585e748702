import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import heat2d  # noqa: E402,F401  (registers the package alias)


def pytest_configure(config):
    # No test reads or extends the user's plan cache (~/.cache/heat2d): a hit
    # would skip the autotuner and schedule search the tests exercise, and
    # plans tuned under one test's HEAT2D_* knobs would leak into the next.
    # The dedicated cache tests point HEAT2D_PLAN_CACHE at their own file.
    os.environ["HEAT2D_PLAN_CACHE"] = "off"
    config.addinivalue_line("markers", "gpu: needs an AMD Instinct GPU (MI355X / gfx950)")
    config.addinivalue_line("markers", "multigpu: needs >= 2 visible GPUs (skipped otherwise)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def native():
    from heat2d.ops import _native as N
    if not N.available():
        N.build()
    return N.lib()


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test collected on a machine without a GPU (run with -m 'not gpu')")
    torch.cuda.set_device(0)
    return 0
