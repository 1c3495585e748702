"""Python driver (`python -m heat2d`), torchrun multi-rank (gloo, CPU), I/O
helpers, plotting and checkpoint/restart across different rank counts."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
from diag import failure_text

import heat2d
from heat2d.models import reference as R
from heat2d.ops import _native as N
from heat2d.utils import io

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def py(cwd, *args, nproc=1, timeout=300):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1", HEAT2D_CPU_THREADS="2")
    if nproc == 1:
        cmd = [sys.executable, "-m", "heat2d", *args]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", str(nproc), "--master-addr",
               "127.0.0.1", "--master-port", str(port()), "-m", "heat2d", *args]
    out = subprocess.run(cmd, cwd=cwd, env=env, capture_output=True, text=True, timeout=timeout)
    assert out.returncode == 0, out.stdout[-3000:] + failure_text(out.stderr)
    return out.stdout


def test_python_driver_serial(native, tmp_path):
    (tmp_path / "input.dat").write_text("36 0.25 0.05 2.0 21\n")
    out = py(tmp_path, "--backend", "cpu", "--json", "m.json")
    assert "simulation completed!!!!" in out and "total time:" in out
    prob = heat2d.make_problem(heat2d.read_input(str(tmp_path / "input.dat")), "inclusive", "hat")
    x, y, T = io.read_xyz(str(tmp_path / "soln.dat"))
    assert np.array_equal(T, R.ftcs(prob))
    assert np.array_equal(x, prob.x) and np.array_equal(y, prob.x)
    _, _, T0 = io.read_xyz(str(tmp_path / "int.dat"))
    assert np.array_equal(T0, R.initial_field(prob))
    m = json.loads((tmp_path / "m.json").read_text())
    assert m["steps"] == 21 and m["variant"] == "serial"


def test_python_variant_demo(native, tmp_path):
    """python/serial/heat.py: 31x31, diffuse(10) = 11 steps, index-slice hat."""
    (tmp_path / "input.dat").write_text("31 0.25 0.05 2.0 10\n")
    py(tmp_path, "--backend", "cpu", "--variant", "python")
    _, _, T = io.read_xyz(str(tmp_path / "soln.dat"))
    demo = R.python_serial_demo()
    assert np.abs(T - demo.T).max() < 1e-13


def test_torchrun_gloo_mpi_variant_and_merge(native, tmp_path):
    (tmp_path / "input.dat").write_text("48 0.25 0.05 1.0 19 1\n")
    out = py(tmp_path, "--backend", "cpu", "--tb", "4", nproc=3)
    assert "Automatic MPI decomposition:            3  x 1" in out and "Average time:" in out
    merged = io.merge_rank_files(str(tmp_path))
    x, y, T = io.read_xyz(merged)
    prob = heat2d.make_problem(heat2d.read_input(str(tmp_path / "input.dat")), "ghost", "uniform")
    assert np.array_equal(T, R.owned(R.ftcs(prob)))
    assert np.array_equal(x, prob.x[1:-1])


def ck_meta(ck):
    """meta.json of the newest complete checkpoint (DIR/latest -> DIR/step-N/)."""
    name = (ck / "latest").read_text().strip()
    return json.loads((ck / name / "meta.json").read_text())


@pytest.mark.parametrize("p_write,p_read", [(2, 1), (1, 3), (3, 2)])
def test_checkpoint_restart_changes_rank_count(native, tmp_path, p_write, p_read):
    (tmp_path / "input.dat").write_text("50 0.25 0.05 1.0 30 1\n")
    # run 12 steps with a checkpoint, then resume to 30 steps on a different rank count
    py(tmp_path, "--backend", "cpu", "--ntime", "12", "--checkpoint", "ck", "--output", "none", nproc=p_write)
    meta = ck_meta(tmp_path / "ck")
    assert meta["step"] == 12 and meta["nranks"] == p_write
    for f in tmp_path.glob("soln*.dat"):
        f.unlink()
    py(tmp_path, "--backend", "cpu", "--restart", "ck", nproc=p_read)
    T = np.concatenate([io.read_xyz(f)[2] for f in io.rank_files(str(tmp_path))], axis=0)
    prob = heat2d.make_problem(heat2d.read_input(str(tmp_path / "input.dat")), "ghost", "uniform")
    assert np.array_equal(T, R.owned(R.ftcs(prob)))


def test_checkpoint_edge_shifted_writer(native, tmp_path):
    """A checkpoint of edge-balanced slabs (--edge-shift) records the shift, and
    a reader with another rank count (and no shift) cuts its rows right."""
    (tmp_path / "input.dat").write_text("60 0.25 0.05 1.0 30 1\n")
    py(tmp_path, "--backend", "cpu", "--ntime", "12", "--checkpoint", "ck", "--output", "none", "--edge-shift", "3",
       nproc=3)
    meta = ck_meta(tmp_path / "ck")
    assert meta["edge_shift"] == 3 and meta["nranks"] == 3
    name = (tmp_path / "ck" / "latest").read_text().strip()
    rows = sorted(np.load(f, allow_pickle=False).shape[0] for f in (tmp_path / "ck" / name).glob("*.npy"))
    assert rows == [17, 17, 26]
    py(tmp_path, "--backend", "cpu", "--restart", "ck", nproc=2)
    T = np.concatenate([io.read_xyz(f)[2] for f in io.rank_files(str(tmp_path))], axis=0)
    prob = heat2d.make_problem(heat2d.read_input(str(tmp_path / "input.dat")), "ghost", "uniform")
    assert np.array_equal(T, R.owned(R.ftcs(prob)))


def test_plot_out(native, tmp_path):
    pytest.importorskip("matplotlib")
    (tmp_path / "input.dat").write_text("30 0.25 0.05 2.0 5\n")
    py(tmp_path, "--backend", "cpu")
    from heat2d.utils import plot
    fig = plot.plot(str(tmp_path / "soln.dat"), save=str(tmp_path / "sol.png"))
    assert (tmp_path / "sol.png").stat().st_size > 1000
    plot.plot(str(tmp_path / "int.dat"), save=str(tmp_path / "int.png"), heatmap=True)
    assert (tmp_path / "int.png").exists()
    del fig


def test_io_roundtrip_and_npy(native, tmp_path):
    rng = np.random.default_rng(3)
    T = rng.random((7, 5))
    x = np.linspace(0, 1, 7)
    y = np.linspace(-1e-3, 2e5, 5)
    io.write_xyz(str(tmp_path / "a.dat"), T, x, y)
    x2, y2, T2 = io.read_xyz(str(tmp_path / "a.dat"))
    assert np.array_equal(T, T2) and np.array_equal(x, x2) and np.array_equal(y, y2)
    io.write_npy(str(tmp_path / "a.npy"), T.astype(np.float32))
    assert np.array_equal(np.load(tmp_path / "a.npy", allow_pickle=False), T.astype(np.float32))


@pytest.mark.parametrize("writer,reader", [("cli", "cli"), ("py", "cli"), ("cli", "py")])
def test_checkpoint_native_cli_interop(native, tmp_path, writer, reader):
    """The native CLI's --checkpoint / --restart use the Python driver's format
    (csrc/runtime/checkpoint.cpp): each driver resumes the other's checkpoints,
    bitwise, on another rank count, and periodic checkpoints carry the step."""
    (tmp_path / "input.dat").write_text("50 0.25 0.05 1.0 30 1\n")
    cli = [N.CLI_PATH, "--cpu", "--quiet"]
    if writer == "cli":
        subprocess.run([*cli, "--ntime", "12", "--checkpoint", "ck", "--checkpoint-every", "5", "--output", "none"],
                       cwd=tmp_path, check=True, capture_output=True)
    else:
        py(tmp_path, "--backend", "cpu", "--ntime", "12", "--checkpoint", "ck", "--output", "none", nproc=2)
    meta = ck_meta(tmp_path / "ck")
    assert meta["step"] == 12 and meta["format"] == "heat2d-checkpoint-v2"
    if reader == "cli":
        out = subprocess.run([*cli, "--restart", "ck"], cwd=tmp_path, check=True, capture_output=True, text=True)
        assert out.returncode == 0
        T = io.read_xyz(str(tmp_path / "soln00000.dat"))[2]
    else:
        py(tmp_path, "--backend", "cpu", "--restart", "ck", nproc=3)
        T = np.concatenate([io.read_xyz(f)[2] for f in io.rank_files(str(tmp_path))], axis=0)
    prob = heat2d.make_problem(heat2d.read_input(str(tmp_path / "input.dat")), "ghost", "uniform")
    assert np.array_equal(T, R.owned(R.ftcs(prob)))


def test_torchrun_edge_shift_measured(native, tmp_path):
    """`python -m heat2d --edge-shift measure` on 4 gloo ranks: every rank
    rehearses its own slab (CPU twin), the shift is decided alike on every
    rank, and whatever it is the merged field is bitwise the golden one."""
    (tmp_path / "input.dat").write_text("200 0.25 0.05 1.0 30 1\n")
    out = py(tmp_path, "--backend", "cpu", "--tb", "4", "--edge-shift", "measure", nproc=4)
    assert " edge balance: shift " in out, out[-2000:]
    T = np.concatenate([io.read_xyz(f)[2] for f in io.rank_files(str(tmp_path))], axis=0)
    prob = heat2d.make_problem(heat2d.read_input(str(tmp_path / "input.dat")), "ghost", "uniform")
    assert np.array_equal(T, R.owned(R.ftcs(prob)))


@pytest.mark.parametrize("writer", ["cli", "py"])
def test_checkpoint_edge_shift_cli_interop(native, tmp_path, writer):
    """Edge-shifted writers (CLI host-thread ranks or Python gloo ranks, 3 ranks,
    --edge-shift 4): meta.json records the shift; the other driver resumes
    with another rank count and a different shift, bitwise."""
    (tmp_path / "input.dat").write_text("60 0.25 0.05 1.0 30 1\n")
    cli = [N.CLI_PATH, "--cpu", "--quiet"]
    if writer == "cli":
        subprocess.run([*cli, "--gpus", "3", "--edge-shift", "4", "--ntime", "12", "--checkpoint", "ck", "--output",
                        "none"], cwd=tmp_path, check=True, capture_output=True)
    else:
        py(tmp_path, "--backend", "cpu", "--ntime", "12", "--checkpoint", "ck", "--output", "none", "--edge-shift",
           "4", nproc=3)
    meta = ck_meta(tmp_path / "ck")
    assert meta["step"] == 12 and meta["edge_shift"] == 4 and meta["nranks"] == 3
    name = (tmp_path / "ck" / "latest").read_text().strip()
    assert sorted(np.load(f, allow_pickle=False).shape[0] for f in (tmp_path / "ck" / name).glob("*.npy")) == \
        [16, 16, 28]
    if writer == "cli":
        py(tmp_path, "--backend", "cpu", "--restart", "ck", "--edge-shift", "2", nproc=4)
        T = np.concatenate([io.read_xyz(f)[2] for f in io.rank_files(str(tmp_path))], axis=0)
    else:
        subprocess.run([*cli, "--gpus", "4", "--edge-shift", "3", "--restart", "ck", "--output", "npy"],
                       cwd=tmp_path, check=True, capture_output=True)
        T = np.concatenate([np.load(tmp_path / f"soln{r:05d}.npy") for r in range(4)], axis=0)
    prob = heat2d.make_problem(heat2d.read_input(str(tmp_path / "input.dat")), "ghost", "uniform")
    assert np.array_equal(T, R.owned(R.ftcs(prob)))


def test_checkpoint_native_rejects_mismatch(native, tmp_path):
    (tmp_path / "input.dat").write_text("40 0.25 0.05 1.0 10 0\n")
    subprocess.run([N.CLI_PATH, "--cpu", "--quiet", "--checkpoint", "ck"], cwd=tmp_path, check=True,
                   capture_output=True)
    (tmp_path / "input.dat").write_text("41 0.25 0.05 1.0 10 0\n")
    p = subprocess.run([N.CLI_PATH, "--cpu", "--quiet", "--restart", "ck"], cwd=tmp_path, capture_output=True,
                       text=True)
    assert p.returncode != 0 and "checkpoint grid differs" in p.stderr
    (tmp_path / "input.dat").write_text("40 0.25 0.05 1.0 10 0\n")
    p = subprocess.run([N.CLI_PATH, "--cpu", "--quiet", "--dtype", "fp32", "--restart", "ck"], cwd=tmp_path,
                       capture_output=True, text=True)
    assert p.returncode != 0 and "dtype" in p.stderr


def test_checkpoint_torn_write_resumes_last_complete(native, tmp_path):
    """Periodic checkpoints go to per-step directories behind an atomic
    `latest` pointer: a crash while writing step 15 (a partial rank file, no
    meta.json, `latest` not moved) resumes bitwise from step 10; only the two
    newest complete steps are kept."""
    (tmp_path / "input.dat").write_text("50 0.25 0.05 1.0 30 1\n")
    cli = [N.CLI_PATH, "--cpu", "--quiet", "--gpus", "2", "--tb", "3"]
    subprocess.run([*cli, "--ntime", "12", "--checkpoint", "ck", "--checkpoint-every", "5", "--output", "none"],
                   cwd=tmp_path, check=True, capture_output=True)
    ck = tmp_path / "ck"
    assert sorted(d.name for d in ck.iterdir() if d.name.startswith("step-")) == [
        "step-000000000010", "step-000000000012"]
    (ck / "latest").write_text("step-000000000010\n")  # as if step 12's publish had not happened
    torn = ck / "step-000000000012"
    (torn / "meta.json").unlink()
    with open(torn / "rank00000.npy", "r+b") as f:
        f.truncate(100)
    subprocess.run([*cli, "--restart", "ck"], cwd=tmp_path, check=True, capture_output=True)
    T = np.concatenate([io.read_xyz(f)[2] for f in io.rank_files(str(tmp_path))], axis=0)
    prob = heat2d.make_problem(heat2d.read_input(str(tmp_path / "input.dat")), "ghost", "uniform")
    assert np.array_equal(T, R.owned(R.ftcs(prob)))


def test_checkpoint_python_load_checks(native, tmp_path):
    """Python loader: a dtype mismatch raises (no silent cast); the v1 flat
    layout of round-1 checkpoints still loads."""
    from heat2d.models.heat2d import HeatSolver
    from heat2d.utils import checkpoint
    p = heat2d.make_problem(heat2d.InputDat(n=40, sigma=0.25, nu=0.05, dom_len=1.0, ntime=7), "ghost", "uniform")
    s = HeatSolver(p, dtype="fp64", backend="cpu", tb=2)
    s.step(7)
    checkpoint.save(s, str(tmp_path / "ck"))
    s32 = HeatSolver(p, dtype="fp32", backend="cpu", tb=2)
    with pytest.raises(ValueError, match="dtype"):
        checkpoint.load(s32, str(tmp_path / "ck"))
    # v1: flat directory
    v1 = tmp_path / "v1"
    v1.mkdir()
    m = ck_meta(tmp_path / "ck")
    m["format"] = "heat2d-checkpoint-v1"
    (v1 / "meta.json").write_text(json.dumps(m))
    np.save(v1 / "rank00000.npy", s.download(), allow_pickle=False)
    s2 = HeatSolver(p, dtype="fp64", backend="cpu", tb=2)
    assert checkpoint.load(s2, str(v1))["step"] == 7
    assert np.array_equal(s2.download(), R.owned(R.ftcs(p)))


@pytest.mark.gpu
def test_pycuda_variant_prints_device_limits(native, gpu, tmp_path):
    """--variant pycuda (python/cuda/cuda.py): the device limits the reference
    queries (:16-27) are printed, MAX_THREADS_PER_BLOCK on its own line, and the
    run goes through the hipRTC-specialised kernel (the reference's JIT)."""
    (tmp_path / "input.dat").write_text("64 0.25 0.05 2.0 10\n")
    out = py(tmp_path, "--backend", "hip", "--variant", "pycuda", "--output", "none")
    lim = N.device_limits(0)
    lines = [l.strip() for l in out.splitlines()]
    assert str(lim["MAX_THREADS_PER_BLOCK"]) in lines
    assert lim["MAX_THREADS_PER_BLOCK"] >= 256 and lim["WARP_SIZE"] == 64 and lim["MAX_BLOCK_DIM_X"] >= 256
    assert any(l.startswith("device limits:") and "MAX_GRID_DIM_X=" in l for l in lines)


@pytest.mark.parametrize("writer", ["native", "python"])
def test_checkpoint_resave_same_step_never_overwrites(native, tmp_path, writer):
    """A step saved again (a restart at its final step, a re-run into the same
    directory) goes to a fresh generation directory: the files `latest` points
    at are never rewritten in place, and the new save resumes bitwise."""
    from heat2d.models.heat2d import HeatSolver
    from heat2d.utils import checkpoint
    (tmp_path / "input.dat").write_text("44 0.25 0.05 1.0 9 1\n")
    ck = tmp_path / "ck"
    prob = heat2d.make_problem(heat2d.read_input(str(tmp_path / "input.dat")), "ghost", "uniform")
    for _ in range(4):
        if writer == "native":
            subprocess.run([N.CLI_PATH, "--cpu", "--quiet", "--tb", "3", "--checkpoint", "ck", "--output", "none"],
                           cwd=tmp_path, check=True, capture_output=True)
        else:
            s = HeatSolver(prob, dtype="fp64", backend="cpu", tb=3)
            s.step(9)
            checkpoint.save(s, str(ck))
            s.close()
    # generations are zero-padded and never reuse a pruned name: name order is
    # write order, and pruning keeps the two newest
    names = sorted(d.name for d in ck.iterdir() if d.name.startswith("step-"))
    assert names == ["step-000000000009-000002", "step-000000000009-000003"]
    assert (ck / "latest").read_text().strip() == "step-000000000009-000003"
    assert checkpoint.load_meta(str(ck))["step"] == 9
    s = HeatSolver(prob, dtype="fp64", backend="cpu", tb=3)
    checkpoint.load(s, str(ck))
    assert np.array_equal(s.download(), R.owned(R.ftcs(prob)))


def test_share_gpu_needs_peer_transport(native, tmp_path):
    (tmp_path / "input.dat").write_text("20 0.25 0.05 1.0 3 0\n")
    env = dict(os.environ, PYTHONPATH=ROOT)
    out = subprocess.run([sys.executable, "-m", "heat2d", "--backend", "cpu", "--share-gpu", "--transport", "rccl"],
                         cwd=tmp_path, env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode != 0 and "--share-gpu needs --transport peer or auto" in out.stderr


def test_torchrun_mpicuda_variant_cpu(native, tmp_path):
    """--variant mpicuda (fortran/mpi+cuda, V7) on 2 gloo ranks: "Sum of
    Temperature:" with the all-reduced sum, then the completion line and a
    per-iteration "total time:"; per-rank soln%05d.dat files."""
    (tmp_path / "input.dat").write_text("60 0.25 0.05 2.0 9 1\n")
    out = py(tmp_path, "--backend", "cpu", "--variant", "mpicuda", "--json", "m.json", nproc=2)
    lines = [l.strip() for l in out.splitlines()]
    i_sum = next(i for i, l in enumerate(lines) if l.startswith("Sum of Temperature:"))
    i_done = lines.index("simulation completed!!!!")
    i_time = next(i for i, l in enumerate(lines) if l.startswith("total time:"))
    assert i_sum < i_done < i_time
    prob = heat2d.make_problem(heat2d.read_input(str(tmp_path / "input.dat")), "ghost", "uniform")
    ref = R.owned(R.ftcs(prob))
    assert float(lines[i_sum].split(":")[1]) == pytest.approx(float(ref.sum()), rel=1e-15)
    T = np.concatenate([io.read_xyz(f)[2] for f in io.rank_files(str(tmp_path))], axis=0)
    assert np.array_equal(T, ref)


@pytest.mark.gpu
def test_torchrun_auto_transport_falls_back_share_gpu(native, gpu, tmp_path):
    """`python -m heat2d --share-gpu` with the default --transport auto under
    torchrun: RCCL refuses two ranks on one GPU on every rank, every rank takes
    the peer (hipIpc) transport, and the result is bitwise the golden."""
    (tmp_path / "input.dat").write_text("300 0.25 0.05 1.0 23 1\n")
    out = py(tmp_path, "--backend", "hip", "--share-gpu", "--arith", "exact", "--json", "m.json", nproc=2)
    d = json.loads((tmp_path / "m.json").read_text())
    assert d["transport"] == "peer" and "rccl" in d["transport_fallback"], d
    T = np.concatenate([io.read_xyz(f)[2] for f in io.rank_files(str(tmp_path))], axis=0)
    prob = heat2d.make_problem(heat2d.read_input(str(tmp_path / "input.dat")), "ghost", "uniform")
    assert np.array_equal(T, R.owned(R.ftcs(prob)))


@pytest.mark.gpu
def test_torchrun_host_transport_share_gpu(native, gpu, tmp_path):
    """`python -m heat2d --transport host` under torchrun: GPU ranks whose halos
    go device -> pinned host -> gloo send/recv -> device (the reference's
    host-staged MPI swap, fortran/hip/heat.F90:196-230; auto's last resort
    after RCCL and IPC), uneven slabs — bitwise == the NumPy golden."""
    (tmp_path / "input.dat").write_text("301 0.25 0.05 1.0 29 1\n")
    py(tmp_path, "--backend", "hip", "--transport", "host", "--share-gpu", "--arith", "exact", "--json", "m.json",
       nproc=3)
    d = json.loads((tmp_path / "m.json").read_text())
    assert d["transport"] == "torch-dist", d
    T = np.concatenate([io.read_xyz(f)[2] for f in io.rank_files(str(tmp_path))], axis=0)
    prob = heat2d.make_problem(heat2d.read_input(str(tmp_path / "input.dat")), "ghost", "uniform")
    assert np.array_equal(T, R.owned(R.ftcs(prob)))


@pytest.mark.gpu
def test_torchrun_peer_transport_share_gpu_checkpoint(native, gpu, tmp_path):
    """`python -m heat2d --transport peer --share-gpu` under torchrun: rank
    processes on one GPU, halos over hipIpc mappings; a 3-rank run checkpoints
    at step 12 and a 2-rank run resumes it — bitwise == the NumPy golden."""
    (tmp_path / "input.dat").write_text("200 0.25 0.05 1.0 37 1\n")
    flags = ("--backend", "hip", "--transport", "peer", "--share-gpu", "--arith", "exact")
    py(tmp_path, *flags, "--ntime", "12", "--checkpoint", "ck", "--output", "none", nproc=3)
    assert ck_meta(tmp_path / "ck")["nranks"] == 3
    out = py(tmp_path, *flags, "--restart", "ck", nproc=2)
    assert "Automatic MPI decomposition:            2  x 1" in out
    T = np.concatenate([io.read_xyz(f)[2] for f in io.rank_files(str(tmp_path))], axis=0)
    prob = heat2d.make_problem(heat2d.read_input(str(tmp_path / "input.dat")), "ghost", "uniform")
    assert np.array_equal(T, R.owned(R.ftcs(prob)))


@pytest.mark.parametrize("writer", ["python", "native"])
def test_checkpoint_legacy_generation_names(native, tmp_path, writer):
    """Saves are ordered by (step, generation) parsed from the names, legacy
    unpadded -N generations included: a new save of step 9 after a legacy
    step-...9-7 becomes -000008 (never a lexically-earlier name), and pruning
    keeps the two newest by that order."""
    from heat2d.models.heat2d import HeatSolver
    from heat2d.utils import checkpoint
    (tmp_path / "input.dat").write_text("44 0.25 0.05 1.0 9 1\n")
    ck = tmp_path / "ck"
    prob = heat2d.make_problem(heat2d.read_input(str(tmp_path / "input.dat")), "ghost", "uniform")

    def save():
        if writer == "native":
            subprocess.run([N.CLI_PATH, "--cpu", "--quiet", "--tb", "3", "--checkpoint", "ck", "--output", "none"],
                           cwd=tmp_path, check=True, capture_output=True)
        else:
            s = HeatSolver(prob, dtype="fp64", backend="cpu", tb=3)
            s.step(9)
            checkpoint.save(s, str(ck))
            s.close()

    save()
    save()  # step-...9 and step-...9-000001
    os.rename(ck / "step-000000000009-000001", ck / "step-000000000009-7")  # a legacy generation name
    (ck / "latest").write_text("step-000000000009-7\n")
    assert checkpoint.fresh_step_dir(str(ck), 9).endswith("step-000000000009-000008")
    save()
    names = sorted((d.name for d in ck.iterdir() if d.name.startswith("step-")), key=checkpoint.step_key)
    assert names == ["step-000000000009-7", "step-000000000009-000008"]
    assert (ck / "latest").read_text().strip() == "step-000000000009-000008"
    s = HeatSolver(prob, dtype="fp64", backend="cpu", tb=3)
    checkpoint.load(s, str(ck))
    assert np.array_equal(s.download(), R.owned(R.ftcs(prob)))


@pytest.mark.gpu
def test_torchrun_edge_shift_auto_share_gpu(native, gpu, tmp_path):
    """`python -m heat2d --edge-shift auto --share-gpu` under torchrun: 3 GPU
    rank processes take turns timing their own slabs (1-rank IPC loop), agree
    on the shift, run over the peer (hipIpc) transport — bitwise the golden."""
    (tmp_path / "input.dat").write_text("1200 0.25 0.05 1.0 40 1\n")
    out = py(tmp_path, "--backend", "hip", "--share-gpu", "--arith", "exact", "--edge-shift", "auto", nproc=3,
             timeout=600)
    assert " edge balance: shift " in out, out[-2000:]
    T = np.concatenate([io.read_xyz(f)[2] for f in io.rank_files(str(tmp_path))], axis=0)
    prob = heat2d.make_problem(heat2d.read_input(str(tmp_path / "input.dat")), "ghost", "uniform")
    assert np.array_equal(T, R.owned(R.ftcs(prob)))
