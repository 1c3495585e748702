"""Failure detection on the communication path (no GPU needed):

* the watchdog mechanism itself (csrc/runtime/watchdog.cpp, the one the RCCL
  transport runs): a hang — outstanding work with no completion — fires after
  the timeout and not before; an idle fabric never fires; an async fabric
  error fires at once;
* a dead rank: in a 2-process gloo run one rank exits abruptly mid-run; the
  survivor must exit non-zero promptly instead of blocking forever (the
  reference's MPI_Sendrecv would, fortran/hip/heat.F90:212-213)."""
import ctypes as C
import json
import os
import subprocess
import sys
import time

import pytest

from heat2d.ops import _native as N

HERE = os.path.dirname(os.path.abspath(__file__))


def selftest(timeout, mode, progress_polls=0, wait=3.0):
    after = C.c_double()
    buf = C.create_string_buffer(512)
    N.call("heat2d_watchdog_selftest", timeout, mode, progress_polls, wait, C.byref(after), buf, 512)
    return after.value, buf.value.decode()


def test_watchdog_fires_on_hang(native):
    after, why = selftest(0.4, 0, progress_polls=10)  # ~0.2 s of progress, then stuck
    assert 0.55 <= after <= 2.0, after
    assert "no halo exchange completed" in why and "selftest op pending" in why


def test_watchdog_quiet_when_idle(native):
    after, why = selftest(0.2, 1, wait=1.0)
    assert after == -1.0 and why == ""


def test_watchdog_fires_on_fabric_error(native):
    after, why = selftest(100.0, 2)
    assert 0 <= after < 0.5 and "communication error: injected" in why


def test_dead_rank_survivor_fails_fast(native, tmp_path):
    """Rank 1 dies (os._exit) after its first chunk; rank 0, still exchanging
    halos with it, must exit non-zero within seconds."""
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    args = {"n": 80, "steps": 40, "tb": 4, "backend": "cpu", "die_rank": 1, "die_after": 8}
    env = dict(os.environ, OMP_NUM_THREADS="1", HEAT2D_CPU_THREADS="1", HEAT2D_COMM_TIMEOUT="20")
    t0 = time.time()
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker.py"), str(r), "2", str(port),
                               str(tmp_path), json.dumps(args)], env=env, stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT) for r in range(2)]
    try:
        outs = [p.communicate(timeout=120)[0].decode(errors="replace") for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    elapsed = time.time() - t0
    assert procs[1].returncode == 3, outs[1][-2000:]  # the injected death
    assert procs[0].returncode != 0, outs[0][-2000:]  # the survivor fails instead of finishing or hanging
    assert elapsed < 90, elapsed
