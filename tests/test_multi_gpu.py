"""Multi-GPU tier: runs only where >= 2 GPUs are visible (an 8-GPU MI355X node),
skipped cleanly on the 1-GPU pool. The reference's defining run is P ranks on
P devices (fortran/hip/heat.F90:115-158 bootstrap + cart topology, :196-230 the
per-step swap); here every cross-device path is checked BITWISE against the
NumPy golden on uneven slabs:

* the native CLI, one host thread per GPU, with RCCL send/recv and with the
  peer transport (device copies over xGMI with peer access);
* bench.py's rank processes with RCCL, IPC (hipIpc handles opened on another
  device, host-shared counters polled by two GPUs) and --transport auto,
  whose field statistics must equal the 1-GPU run's and whose own
  self-verification must pass.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import heat2d
from heat2d.models import reference as R
from heat2d.ops import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def ngpus():
    try:
        import torch
        return torch.cuda.device_count()  # does not initialise the GPU on this image
    except Exception:  # pragma: no cover
        return 0


pytestmark = [pytest.mark.gpu, pytest.mark.multigpu,
              pytest.mark.skipif(ngpus() < 2, reason="needs >= 2 visible GPUs (multi-GPU node)")]
SIZES = [p for p in (2, 4, 8) if p <= max(ngpus(), 2)]


def run_cli(cwd, *args, timeout=600):
    out = subprocess.run([N.CLI_PATH, *args], cwd=cwd, capture_output=True, text=True, timeout=timeout)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    return out.stdout


@pytest.mark.parametrize("transport", ["rccl", "peer"])
@pytest.mark.parametrize("P", SIZES)
@pytest.mark.parametrize("extra", [[], ["--autotune", "on", "--dtype", "fp32"]])
def test_cli_multi_gpu_bitwise(tmp_path, transport, P, extra):
    """P GPUs, uneven slabs (2051 = P * q + rem), 57 steps of balanced cycles
    (or, with --autotune on, autotuned split plans and a measured schedule),
    every rank on its own device: the slabs put together are the golden."""
    (tmp_path / "input.dat").write_text("2051 0.25 0.05 1.0 57 0\n")
    out = run_cli(tmp_path, "--gpus", str(P), "--transport", transport, "--output", "npy", *extra)
    for r in range(P):
        assert f"using GPU {r:12d}" in out
    prob = heat2d.make_problem(heat2d.read_input(str(tmp_path / "input.dat")), "ghost", "uniform")
    npdt = np.float32 if "fp32" in extra else np.float64
    got = np.concatenate([np.load(tmp_path / f"soln{r:05d}.npy") for r in range(P)])
    assert np.array_equal(got, R.owned(R.ftcs(prob, dtype=npdt)))


@pytest.mark.parametrize("force_fail", [False, True])
def test_cli_multi_gpu_auto_transport(tmp_path, force_fail):
    """--transport auto (the CLI default) on P distinct GPUs: RCCL when its
    communicators build on every rank; with HEAT2D_FORCE_RCCL_FAIL=1 (a node
    whose RCCL cannot initialise) every rank falls back to the peer transport.
    Both bitwise the golden."""
    P = SIZES[-1]
    (tmp_path / "input.dat").write_text("2051 0.25 0.05 1.0 57 0\n")
    env = dict(os.environ)
    if force_fail:
        env["HEAT2D_FORCE_RCCL_FAIL"] = "1"
    p = subprocess.run([N.CLI_PATH, "--gpus", str(P), "--output", "npy", "--json", "m.json"], cwd=tmp_path,
                       capture_output=True, text=True, timeout=600, env=env)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    d = json.loads((tmp_path / "m.json").read_text())
    assert d["transport"] == ("peer" if force_fail else "rccl"), d
    assert (d["transport_fallback"] is not None) == force_fail
    prob = heat2d.make_problem(heat2d.read_input(str(tmp_path / "input.dat")), "ghost", "uniform")
    got = np.concatenate([np.load(tmp_path / f"soln{r:05d}.npy") for r in range(P)])
    assert np.array_equal(got, R.owned(R.ftcs(prob)))


def run_bench(*args, timeout=900):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=timeout, env=env)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


@pytest.fixture(scope="module")
def one_gpu_stats():
    return run_bench("--gpus", "1", "--grid", "8192", "--steps", "40", "--warmup", "5", "--check")["field_stats"]


@pytest.mark.parametrize("transport", ["rccl", "ipc", "auto", "best"])
@pytest.mark.parametrize("P", SIZES)
def test_bench_multi_gpu_matches_one_gpu(one_gpu_stats, transport, P):
    d = run_bench("--gpus", str(P), "--grid", "8192", "--steps", "40", "--warmup", "5", "--check", "--transport",
                  transport)
    ch = d["config"]["transport_choice"]
    assert ch["requested"] == transport and d["config"]["transport"] == ch["chosen"]
    if transport in ("rccl", "ipc"):
        assert ch["chosen"] == transport
    elif transport == "auto":  # RCCL works on a node: IPC (its fallback) is never built
        assert ch["chosen"] == "rccl" and "skipped" in ch["ipc"], ch
    else:
        assert "ms" in ch["rccl"] and "ms" in ch["ipc"], ch
    # the decomposition proves itself: what the fabric reports on every rank
    assert d["fabric"]["nranks"] == P and d["distinct_devices"] == P, d["per_rank"]
    assert [r["rank"] for r in d["per_rank"]] == list(range(P))
    assert sum(r["rows"] for r in d["per_rank"]) == 8192
    if d["config"]["transport"] == "rccl":
        assert d["rccl_nranks"] == P
        assert sorted(r["fabric"]["device"] for r in d["per_rank"]) == list(range(P))
    assert d["verified"] is True, d["verify"]
    fc = d["timed_field_check"]
    assert fc["ok"] is True and fc["mode"] == "full" and fc["mismatches"] == 0, fc
    b = d["field_stats"]
    assert one_gpu_stats["min"] == b["min"] and one_gpu_stats["max"] == b["max"]
    assert b["sum"] == pytest.approx(one_gpu_stats["sum"], rel=1e-12, abs=0)
    assert d["halo_bytes"] > 0 and d["n_gpus"] == P
