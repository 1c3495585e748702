"""The native `heat2d` executable: reference run behaviour (input.dat in the
working directory, stdout lines, int.dat / soln.dat / soln%05d.dat outputs)
for the serial, cuda and mpi variants; values round-trip exactly (17
significant digits) and match the NumPy golden bitwise."""
import os
import subprocess

import numpy as np
import pytest

import heat2d
from heat2d.models import reference as R
from heat2d.ops import _native as N


def run_cli(cwd, *args, timeout=300):
    out = subprocess.run([N.CLI_PATH, *args], cwd=cwd, capture_output=True, text=True, timeout=timeout)
    assert out.returncode == 0, out.stdout + out.stderr
    return out.stdout


def read_xyz(path):
    a = np.loadtxt(path)
    assert a.ndim == 2 and a.shape[1] == 3
    return a


@pytest.fixture(scope="module")
def cli(native):
    if not os.path.exists(N.CLI_PATH):
        N.build()
    return N.CLI_PATH


@pytest.mark.parametrize("variant,ic", [("serial", "hat"), ("cuda", "hat-cuda")])
def test_cli_serial_variants_cpu(cli, tmp_path, variant, ic):
    (tmp_path / "input.dat").write_text("40 0.25 0.05 2.0 25\n")
    out = run_cli(tmp_path, "--cpu", "--variant", variant)
    assert "simulation completed!!!!" in out and "total time:" in out
    inp = heat2d.read_input(str(tmp_path / "input.dat"))
    prob = heat2d.make_problem(inp, "inclusive", ic)
    T0 = R.initial_field(prob)
    T = R.ftcs(prob)
    a0 = read_xyz(tmp_path / "int.dat")
    a = read_xyz(tmp_path / "soln.dat")
    assert a.shape == (40 * 40, 3)
    assert np.array_equal(a0[:, 2], T0.ravel())
    assert np.array_equal(a[:, 2], T.ravel())
    # coordinates: x outer, y inner (fortran/serial/heat.f90:77-83)
    assert np.array_equal(a[:, 0].reshape(40, 40)[:, 0], prob.x)
    assert np.array_equal(a[:, 1].reshape(40, 40)[0, :], prob.x)


def test_cli_mpi_variant_cpu(cli, tmp_path):
    (tmp_path / "input.dat").write_text("64 0.25 0.05 1.0 17 1\n")
    out = run_cli(tmp_path, "--cpu")
    assert "Automatic MPI decomposition:" in out and "Average time:" in out
    a = read_xyz(tmp_path / "soln00000.dat")
    prob = heat2d.make_problem(heat2d.read_input(str(tmp_path / "input.dat")), "ghost", "uniform")
    assert np.array_equal(a[:, 2], R.owned(R.ftcs(prob)).ravel())
    assert np.array_equal(np.unique(a[:, 0]), prob.x[1:-1])


def test_cli_flags_and_json(cli, tmp_path):
    (tmp_path / "input.dat").write_text("32768 0.25 0.05 1.0 25000 0\n")  # the reference benchmark file
    out = run_cli(tmp_path, "--cpu", "--n", "48", "--ntime", "9", "--tb", "4", "--dtype", "fp32", "--json", "r.json",
                  "--check-every", "3", "--print-every", "3")
    assert "time_it:" in out and "residual_l2" in out
    import json
    r = json.loads((tmp_path / "r.json").read_text())
    assert r["n"] == 48 and r["steps"] == 9 and r["dtype"] == "fp32" and r["backend"] == "cpu"
    # the cycles the timed loop launched, per depth: they add up to the steps run
    assert sum(int(k) * c for k, c in r["cycles"].items()) == 9 and max(map(int, r["cycles"])) <= 4
    assert "passes=" in out


@pytest.mark.parametrize("dev", [pytest.param(["--cpu"], id="cpu"),
                                 pytest.param(["--gpus", "1"], id="gpu", marks=pytest.mark.gpu)])
def test_cli_time_transfers(cli, tmp_path, dev):
    """--time-transfers: the whole-field H2D of the IC and D2H of the result
    inside the timed region, as fortran/hip/heat.F90:284-295 times them. The
    field round-trips unchanged (bitwise the golden), the JSON reports both
    copy times, and they are part of the elapsed time."""
    import json
    (tmp_path / "input.dat").write_text("300 0.25 0.05 1.0 37 0\n")
    prob = heat2d.make_problem(heat2d.read_input(str(tmp_path / "input.dat")), "ghost", "uniform")
    ref = R.owned(R.ftcs(prob))
    out = run_cli(tmp_path, *dev, "--tb", "8", "--time-transfers", "--json", "t.json", "--output", "npy")
    assert "Average time:" in out
    r = json.loads((tmp_path / "t.json").read_text())
    assert r["time_transfers"] is True and r["h2d_s"] > 0 and r["d2h_s"] > 0
    assert r["wall_s"] >= r["h2d_s"] + r["d2h_s"]
    assert np.array_equal(np.load(tmp_path / "soln00000.npy"), ref)
    run_cli(tmp_path, *dev, "--tb", "8", "--json", "n.json", "--output", "npy")
    n = json.loads((tmp_path / "n.json").read_text())
    assert n["time_transfers"] is False and n["h2d_s"] == 0 and n["d2h_s"] == 0
    assert np.array_equal(np.load(tmp_path / "soln00000.npy"), ref)


def test_cli_time_it_every_step_keeps_deep_cycles(cli, tmp_path):
    """--print-every 1: one time_it line per step, in order (the reference,
    fortran/hip/heat.F90:241), without cutting the run into depth-1 cycles:
    lines are printed after each cycle of pref_depth steps; the result stays
    bitwise; --check-every prints the fused one-step residual."""
    (tmp_path / "input.dat").write_text("64 0.25 0.05 1.0 29 0\n")
    out = run_cli(tmp_path, "--cpu", "--tb", "8", "--print-every", "1", "--check-every", "16", "--output", "npy")
    steps = [int(l.split()[1]) for l in out.splitlines() if l.strip().startswith("time_it:")]
    assert steps == list(range(1, 30))
    checks = [l for l in out.splitlines() if l.strip().startswith("step 16:")]
    assert len(checks) == 1 and "residual_l2=" in checks[0] and "residual_max=" in checks[0]
    prob = heat2d.make_problem(heat2d.read_input(str(tmp_path / "input.dat")), "ghost", "uniform")
    T16, T15 = R.owned(R.ftcs(prob, 16)), R.owned(R.ftcs(prob, 15))
    rl2 = float(checks[0].split("residual_l2=")[1].split()[0])
    assert np.isclose(rl2, np.sqrt(((T16 - T15) ** 2).sum()), rtol=1e-6)
    assert np.array_equal(np.load(tmp_path / "soln00000.npy"), R.owned(R.ftcs(prob)))


@pytest.mark.parametrize("P", [2, 3])
def test_cli_cpu_multirank(cli, tmp_path, P):
    """`heat2d --cpu --gpus P`: P host-thread ranks of the CPU twin exchanging
    halos through the host-thread transport (the reference's `make mpi` CPU
    MPI build): per-rank soln%05d.dat, bitwise the golden, and the global sum
    all-reduced over the ranks."""
    (tmp_path / "input.dat").write_text("67 0.25 0.05 1.0 23 1\n")
    out = run_cli(tmp_path, "--cpu", "--gpus", str(P), "--tb", "4", "--check-every", "23")
    assert f"Automatic MPI decomposition: {P:12d}  x 1" in out
    prob = heat2d.make_problem(heat2d.read_input(str(tmp_path / "input.dat")), "ghost", "uniform")
    T = R.owned(R.ftcs(prob))
    parts = [read_xyz(tmp_path / f"soln{r:05d}.dat")[:, 2] for r in range(P)]
    assert np.array_equal(np.concatenate(parts), T.ravel())
    line = [l for l in out.splitlines() if l.strip().startswith("step 23:")][0]
    assert np.isclose(float(line.split("sum=")[1].split()[0]), T.sum(), rtol=1e-13)


def test_cli_failing_rank_fails_fast(cli, tmp_path):
    """One rank fails mid-run (fault injection): the others, blocked exchanging
    with it, are aborted and the process exits non-zero at once naming the
    failed rank — no hang in join()."""
    import time
    (tmp_path / "input.dat").write_text("64 0.25 0.05 1.0 400 0\n")
    env = dict(os.environ, HEAT2D_FAIL_RANK="1", HEAT2D_FAIL_STEP="8", HEAT2D_COMM_TIMEOUT="60")
    t0 = time.time()
    p = subprocess.run([N.CLI_PATH, "--cpu", "--gpus", "3", "--tb", "4", "--print-every", "4"], cwd=tmp_path,
                       capture_output=True, text=True, timeout=120, env=env)
    assert p.returncode != 0
    assert "rank 1" in p.stderr and "injected failure" in p.stderr, p.stderr
    assert time.time() - t0 < 30


def test_cli_bad_input(cli, tmp_path):
    (tmp_path / "input.dat").write_text("10 0.25\n")
    out = subprocess.run([N.CLI_PATH, "--cpu"], cwd=tmp_path, capture_output=True, text=True)
    assert out.returncode != 0 and "at least 5 fields" in out.stderr


@pytest.mark.gpu
def test_cli_gpu_mpi_variant(cli, gpu, tmp_path):
    (tmp_path / "input.dat").write_text("300 0.25 0.05 1.0 40 1\n")
    out = run_cli(tmp_path, "--gpus", "1", "--tb", "8")
    assert "MPI rank" in out and "using GPU" in out
    a = read_xyz(tmp_path / "soln00000.dat")
    prob = heat2d.make_problem(heat2d.read_input(str(tmp_path / "input.dat")), "ghost", "uniform")
    assert np.array_equal(a[:, 2], R.owned(R.ftcs(prob)).ravel())


@pytest.mark.gpu
@pytest.mark.parametrize("extra", [[], ["--copy-swap"], ["--managed"], ["--graph"]])
def test_cli_gpu_serial_variant(cli, gpu, tmp_path, extra):
    (tmp_path / "input.dat").write_text("100 0.25 0.05 2.0 60\n")
    run_cli(tmp_path, "--variant", "serial", *extra)
    prob = heat2d.make_problem(heat2d.read_input(str(tmp_path / "input.dat")), "inclusive", "hat")
    a = read_xyz(tmp_path / "soln.dat")
    assert np.array_equal(a[:, 2], R.ftcs(prob).ravel())


@pytest.mark.gpu
@pytest.mark.parametrize("extra", [[], ["--no-overlap"], ["--tb", "5"], ["--check-every", "10"], ["--dtype", "fp32"]])
def test_cli_peer_transport_bitwise(cli, gpu, tmp_path, extra):
    """P ranks as threads of the native CLI with the peer transport (no RCCL:
    halos pulled by device copies out of the neighbours' fields, ordered by
    events and host-side waits), all on one GPU (--share-gpu): the rank slabs
    put together are bitwise the golden — split schedule (1100^2 slabs are
    split into interior + bands), serial schedule, other depths, fused
    statistics, fp32."""
    (tmp_path / "input.dat").write_text("1100 0.25 0.05 1.0 31 0\n")
    out = run_cli(tmp_path, "--gpus", "3", "--transport", "peer", "--share-gpu", "--output", "npy", *extra)
    assert out.count("using GPU            0") == 3
    prob = heat2d.make_problem(heat2d.read_input(str(tmp_path / "input.dat")), "ghost", "uniform")
    npdt = np.float32 if "fp32" in extra else np.float64
    got = np.concatenate([np.load(tmp_path / f"soln{r:05d}.npy") for r in range(3)])
    assert np.array_equal(got, R.owned(R.ftcs(prob, dtype=npdt)))


@pytest.mark.gpu
def test_cli_peer_transport_eight_ranks(cli, gpu, tmp_path):
    """8 rank threads on one GPU (525-row slabs: below the 2^24-point autotune
    threshold, so balanced cycles; the forced-autotune run with prepare()'s
    collective measured schedule is tests/test_collective.py): many cycles of
    real host concurrency through the peer transport's waits, bitwise the golden."""
    (tmp_path / "input.dat").write_text("4200 0.25 0.05 1.0 75 0\n")
    run_cli(tmp_path, "--gpus", "8", "--transport", "peer", "--share-gpu", "--output", "npy", "--quiet",
            "--print-every", "25", "--check-every", "25")
    prob = heat2d.make_problem(heat2d.read_input(str(tmp_path / "input.dat")), "ghost", "uniform")
    got = np.concatenate([np.load(tmp_path / f"soln{r:05d}.npy") for r in range(8)])
    assert np.array_equal(got, R.owned(R.ftcs(prob)))


@pytest.mark.gpu
def test_cli_peer_transport_fails_fast(cli, gpu, tmp_path):
    """Peer transport: one rank fails mid-run (fault injection); the others,
    blocked in the transport's host-side waits for its halo, are woken by the
    abort and the process exits non-zero naming the failed rank, well inside
    the comm timeout."""
    import time
    (tmp_path / "input.dat").write_text("600 0.25 0.05 1.0 400 0\n")
    env = dict(os.environ, HEAT2D_FAIL_RANK="1", HEAT2D_FAIL_STEP="16", HEAT2D_COMM_TIMEOUT="60")
    t0 = time.time()
    p = subprocess.run([N.CLI_PATH, "--gpus", "3", "--transport", "peer", "--share-gpu", "--tb", "8",
                        "--print-every", "8", "--output", "none"], cwd=tmp_path, capture_output=True, text=True,
                       timeout=120, env=env)
    assert p.returncode != 0
    assert "rank 1" in p.stderr and "injected failure" in p.stderr, p.stderr
    assert time.time() - t0 < 40


def test_cli_share_gpu_needs_peer(cli, tmp_path):
    (tmp_path / "input.dat").write_text("64 0.25 0.05 1.0 5 0\n")
    p = subprocess.run([N.CLI_PATH, "--gpus", "2", "--share-gpu", "--transport", "rccl"], cwd=tmp_path,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and "--share-gpu needs --transport peer or auto" in p.stderr


def test_cli_mpicuda_variant_cpu(cli, tmp_path):
    """--variant mpicuda (fortran/mpi+cuda, V7): its stdout lines — nx / ny,
    "Sum of Temperature:" (there an uninitialised gsum, heat.F90:266-275; here
    the all-reduced sum of the field), "simulation completed!!!!" and a
    per-iteration "total time:" (heat.F90:292) — on 3 host-thread ranks."""
    (tmp_path / "input.dat").write_text("100 0.25 0.05 2.0 10 1\n")
    out = run_cli(tmp_path, "--cpu", "--variant", "mpicuda", "--gpus", "3", "--json", "m.json")
    lines = out.splitlines()
    i_sum = next(i for i, l in enumerate(lines) if "Sum of Temperature:" in l)
    i_done = next(i for i, l in enumerate(lines) if "simulation completed!!!!" in l)
    i_time = next(i for i, l in enumerate(lines) if l.strip().startswith("total time:"))
    assert i_sum < i_done < i_time and "Average time:" not in out
    prob = heat2d.make_problem(heat2d.read_input(str(tmp_path / "input.dat")), "ghost", "uniform")
    ref = float(np.sum(R.owned(R.ftcs(prob))))
    assert float(lines[i_sum].split(":")[1]) == pytest.approx(ref, rel=1e-15)
    import json
    d = json.loads((tmp_path / "m.json").read_text())
    per_step = float(lines[i_time].split(":")[1])
    assert per_step == pytest.approx(d["wall_s"] / 10, rel=1e-6)
    assert d["transport"] == "host" and d["transport_fallback"] is None
    got = np.concatenate([read_xyz(tmp_path / f"soln{r:05d}.dat")[:, 2] for r in range(3)])
    assert np.array_equal(got, R.owned(R.ftcs(prob)).ravel())


@pytest.mark.gpu
def test_cli_auto_transport_falls_back_to_peer(cli, gpu, tmp_path):
    """--transport auto (the default) with ranks sharing one GPU: RCCL refuses
    to build the communicators, every rank falls back to the peer transport
    (reported on stderr and in the JSON), and the run is bitwise the golden."""
    (tmp_path / "input.dat").write_text("1100 0.25 0.05 1.0 31 0\n")
    p = subprocess.run([N.CLI_PATH, "--gpus", "3", "--share-gpu", "--output", "npy", "--json", "m.json"],
                       cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "falling back to the peer transport" in p.stderr
    import json
    d = json.loads((tmp_path / "m.json").read_text())
    assert d["transport"] == "peer" and "RCCL unavailable" in d["transport_fallback"], d
    prob = heat2d.make_problem(heat2d.read_input(str(tmp_path / "input.dat")), "ghost", "uniform")
    got = np.concatenate([np.load(tmp_path / f"soln{r:05d}.npy") for r in range(3)])
    assert np.array_equal(got, R.owned(R.ftcs(prob)))


@pytest.mark.gpu
def test_cli_gpu_checkpoint_restart(cli, gpu, tmp_path):
    """GPU run checkpointed mid-way (HIP fields -> rank .npy), resumed on the GPU
    and, separately, on the CPU twin: both finish bitwise equal to the golden."""
    (tmp_path / "input.dat").write_text("300 0.25 0.05 1.0 40 1\n")
    run_cli(tmp_path, "--gpus", "1", "--ntime", "17", "--checkpoint", "ck", "--output", "none", "--quiet")
    prob = heat2d.make_problem(heat2d.read_input(str(tmp_path / "input.dat")), "ghost", "uniform")
    ref = R.owned(R.ftcs(prob)).ravel()
    for dev in (["--gpus", "1"], ["--cpu"]):
        run_cli(tmp_path, *dev, "--restart", "ck", "--quiet")
        assert np.array_equal(read_xyz(tmp_path / "soln00000.dat")[:, 2], ref), dev


def test_cmake_configures(tmp_path):
    """The CMake build (alternative to csrc/Makefile) configures for gfx950."""
    import shutil
    import subprocess
    if shutil.which("cmake") is None:
        pytest.skip("cmake not installed")
    src = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cuda-hip-mpi-heat-equation-test_amd", "csrc")
    r = subprocess.run(["cmake", "-S", src, "-B", str(tmp_path / "b")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "gfx950" in open(tmp_path / "b" / "CMakeCache.txt").read()
