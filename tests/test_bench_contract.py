"""The bench.py driver contract, rehearsed on CPU: the multi-process path the
driver launches with torchrun on 2/4/8 GPUs (init, transport, prepare,
barrier-bracketed timed region, MAX over ranks, rank 0 prints ONE JSON line on
stdout — RCCL's version banners are kept off it) runs here with --backend cpu
(gloo + the native CPU twin) and must produce exactly that line."""
import json
import os
import subprocess
import sys

import pytest
from diag import failure_text

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def run_bench(nproc, *args, port):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", str(nproc), "--backend", "cpu", *args]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
    assert p.returncode == 0, failure_text(p.stderr)
    lines = [l for l in p.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("nproc,dtype", [(2, "fp64"), (3, "fp32")])
def test_bench_json_line_multi_rank(nproc, dtype):
    d = run_bench(nproc, "--grid", "100", "--steps", "24", "--warmup", "4", "--dtype", dtype, "--tb", "4",
                  port=29560 + nproc)
    assert KEYS <= set(d)
    assert d["n_gpus"] == nproc and d["steps"] == 24 and d["warmup"] == 4 and d["dtype"] == dtype
    assert d["value"] > 0 and d["ms_per_step"] > 0 and d["higher_is_better"] is True
    assert d["scaling"] == "strong" and d["config"]["parallelism"] == f"slab{nproc}"
    assert d["config"]["grid"] == [100, 100]
    # the self-check after the timed run: an uneven rough-data problem over the
    # same ranks and transport kind, gathered and compared bitwise to the golden
    assert d["verified"] is True and d["verify"]["n"] == 256 * nproc + 5 and d["verify"]["max_abs_diff"] == 0.0
    # the timed field itself, against the one-step reference run from the same IC
    fc = d["timed_field_check"]
    assert fc["ok"] is True and fc["mode"] == "full" and fc["mismatches"] == 0 and fc["max_abs_diff"] == 0.0, fc
    assert fc["rows_checked"] == 100 and fc["steps"] == 28
    # per-rank proof of the decomposition (gathered over the ranks)
    assert d["fabric"] == {"kind": "host", "nranks": nproc} and d["rccl_nranks"] is None
    pr = d["per_rank"]
    assert [r["rank"] for r in pr] == list(range(nproc)) and sum(r["rows"] for r in pr) == 100
    assert all(r["fabric"]["rank"] == r["rank"] and r["transport"] == "torch-dist" for r in pr)
    assert d["rank_timed_ms"]["max"] == pytest.approx(d["ms_per_step"] * 24, rel=1e-3)
    assert d["rank_timed_ms"]["min"] <= d["rank_timed_ms"]["max"]


def test_bench_multi_rank_times_the_same_state_as_one_rank():
    """The transport trials run the timed loop before the timed run; the field
    then goes back to the IC and the warm-up, so the timed run ends on the same
    state a single-rank run does (field statistics equal)."""
    args = ["--grid", "100", "--steps", "24", "--warmup", "4", "--tb", "4", "--check"]
    two = run_bench(2, *args, port=29566)
    one = run_plain("--backend", "cpu", "--gpus", "1", *args)
    assert two["config"]["transport_choice"]["chosen"] == "torch-dist"
    a, b = one["field_stats"], two["field_stats"]
    assert a["min"] == b["min"] and a["max"] == b["max"] and b["sum"] == pytest.approx(a["sum"], rel=1e-12, abs=0)


def test_bench_weak_mode():
    d = run_bench(2, "--grid", "64", "--weak", "--steps", "8", "--warmup", "2", "--tb", "4", port=29570)
    assert d["scaling"] == "weak" and d["config"]["grid"] == [91, 91]  # round(64 * sqrt(2))


def test_bench_single_process_cpu():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--backend", "cpu", "--grid", "80", "--steps",
                        "8", "--warmup", "2", "--tb", "4", "--check"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.strip()]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["field_stats"]["max"] <= 2.0


def test_bench_launches_ranks_itself():
    """`python bench.py --gpus N` without torchrun starts N rank processes
    (never silently one): the driver's N-GPU command works either way."""
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--backend", "cpu", "--gpus", "4", "--grid",
                        "100", "--steps", "8", "--warmup", "2", "--tb", "4"], capture_output=True, text=True,
                       timeout=600, env=env)
    assert p.returncode == 0, failure_text(p.stderr)
    lines = [l for l in p.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 4 and d["config"]["parallelism"] == "slab4"
    # the timed region's cycles are reported, and they add up to the timed steps
    assert sum(int(k) * c for k, c in d["config"]["cycles"].items()) == 8


def test_bench_refuses_missing_gpus():
    """More GPUs requested than visible: a non-zero exit, not a 1-GPU number."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "64", "--steps", "4"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode != 0 and p.stdout.strip() == ""
    assert "GPU(s) visible" in p.stderr


def run_plain(*args, timeout=600):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=timeout, env=env)
    assert p.returncode == 0, failure_text(p.stderr)
    lines = [l for l in p.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def test_bench_share_gpu_refuses_forced_rccl():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--share-gpu", "--transport",
                        "rccl"], capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode != 0 and "--share-gpu needs --transport ipc or auto" in p.stderr


def test_bench_reports_halo_traffic_cpu():
    """Halo bytes of the timed region: each exchange moves the next cycle's depth (whole padded rows)."""
    d = run_plain("--backend", "cpu", "--gpus", "2", "--grid", "100", "--steps", "16", "--warmup", "4", "--tb", "4")
    cyc = sum(d["config"]["cycles"].values())
    assert d["halo_bytes"] > 0 and d["halo_bytes_per_cycle"] == pytest.approx(d["halo_bytes"] / cyc, rel=1e-3)
    # 4 cycles of depth 4, two messages (one per rank), 4 rows of a 192-element (pitch) fp64 row each
    assert d["halo_bytes"] == 4 * 2 * 4 * 192 * 8


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,steps,graph", [("fp64", 40, "on"), ("fp32", 37, "auto")])
def test_bench_ipc_transport_share_gpu_matches_one_rank(dtype, steps, graph):
    """`bench.py --gpus 4 --share-gpu --transport peer`: four rank PROCESSES on the
    one GPU, fields mapped through hipIpc handles, halos pulled by device copies
    ordered by stream-side counters (no RCCL), cycles replayed from hipGraphs
    (--graph on) or eager (auto) — the exact multi-process bench path on a
    1-GPU box. The field statistics
    equal the 1-rank run's exactly (sum, min, max; the sum is all-reduced, so
    compared to 1e-12)."""
    common = ["--grid", "8192", "--steps", str(steps), "--warmup", "5", "--check", "--dtype", dtype]
    one = run_plain("--gpus", "1", *common)
    four = run_plain("--gpus", "4", "--share-gpu", "--transport", "peer", "--graph", graph, *common)
    assert four["config"]["transport"] == "ipc" and four["config"]["graph"] is (graph == "on")
    assert four["config"]["parallelism"] == "slab4-shared-gpu"
    a, b = one["field_stats"], four["field_stats"]
    assert a["min"] == b["min"] and a["max"] == b["max"]
    assert b["sum"] == pytest.approx(a["sum"], rel=1e-12, abs=0)
    assert four["halo_bytes"] > 0


@pytest.mark.gpu
def test_bench_auto_transport_falls_back_to_ipc_share_gpu():
    """`bench.py --gpus 4 --share-gpu` with the default --transport auto: RCCL
    refuses four ranks on one GPU, every rank skips it alike and the run
    proceeds on the IPC transport (the fallback a node whose RCCL cannot
    initialise takes), then verifies the decomposition bitwise."""
    common = ["--grid", "8192", "--steps", "20", "--warmup", "5", "--check"]
    four = run_plain("--gpus", "4", "--share-gpu", *common)
    ch = four["config"]["transport_choice"]
    assert four["config"]["transport"] == "ipc" and ch["chosen"] == "ipc" and ch["requested"] == "auto", ch
    assert "error" in ch["rccl"] and ch["ipc"]["ms"] > 0, ch
    assert four["verified"] is True and four["verify"]["max_abs_diff"] == 0.0, four["verify"]
    # the timed field itself: 4 rank slabs vs the one-step JIT engine on the same layout and transport
    fc = four["timed_field_check"]
    assert fc["ok"] is True and fc["mode"] == "full" and fc["engine"] in ("jit-exact", "jit-jacobi"), fc
    assert fc["mismatches"] == 0 and fc["max_abs_diff"] == 0.0 and fc["rows_checked"] == 8192 and fc["steps"] == 25
    if fc["engine"] == "jit-jacobi":  # the r = 1/4 form is bitwise the reference rounding on this IC, too
        assert fc["vs_exact"]["ok"] is True and fc["vs_exact"]["mismatches"] == 0, fc
    assert four["fabric"] == {"kind": "ipc", "nranks": 4} and len(four["per_rank"]) == 4
    assert four["distinct_devices"] == 1  # --share-gpu: every rank on the one GPU
    # the edge-balance rehearsal ran (one rank after another on the shared GPU)
    # and the run used the shift it kept
    dec = four["config"]["decomposition"]
    bal = dec["balance"]
    assert len(bal["uniform_ms"]) == 4 and min(bal["uniform_ms"]) > 0 and "error" not in bal, bal
    assert bal["uniform_rows"] == [2048] * 4 and dec["rows"] == [r["rows"] for r in four["per_rank"]]
    assert dec["rows"][0] == 2048 - dec["edge_shift"] and sum(dec["rows"]) == 8192
    assert (dec["edge_shift"] > 0) == bool(bal.get("kept")), bal
    one = run_plain("--gpus", "1", *common)
    assert one["timed_field_check"]["ok"] is True and one["timed_field_check"]["mismatches"] == 0
    assert one["verified"] is True and one["config"]["transport_choice"] is None
    a, b = one["field_stats"], four["field_stats"]
    assert a["min"] == b["min"] and a["max"] == b["max"]
    assert b["sum"] == pytest.approx(a["sum"], rel=1e-12, abs=0)


@pytest.mark.gpu
@pytest.mark.parametrize("transport", ["rccl", "ipc"])
def test_bench_rehearsal_then_verification(transport):
    """A 1-GPU rehearsal of one rank's exchanging cycle (periodic self-exchange
    over a 1-rank RCCL communicator / the IPC loop transport), then the
    verification problem on a fresh solver: the loop transports' teardown
    leaves no HIP error behind for the next launch."""
    d = run_plain("--rehearse-comm", "--transport", transport, "--grid", "4096", "--rows", "1024", "--steps", "20",
                  "--warmup", "5")
    assert d["config"]["transport"] == f"{transport}-loop" and d["verified"] is True, d
    assert d["halo_bytes"] > 0
    # what the fabric reports (RCCL: ncclCommCount / ncclCommCuDevice of the 1-rank communicator)
    assert d["fabric"] == {"kind": transport, "nranks": 1}, d["fabric"]
    assert d["per_rank"][0]["fabric"]["device"] == 0 and d["per_rank"][0]["pci_bus_id"].count(":") == 2
    assert d["rccl_nranks"] == (1 if transport == "rccl" else None)


@pytest.mark.gpu
@pytest.mark.parametrize("transport", ["ipc", "auto"])
def test_bench_ipc_attach_is_bounded(transport):
    """An IPC attach that never returns (HEAT2D_IPC_ATTACH_STALL: rank 1's
    hipIpcOpenMemHandle hangs, as 4 ranks sharing a GPU at 32768^2 once did,
    profiles/r6/ipc/) fails the attach after HEAT2D_IPC_ATTACH_TIMEOUT seconds
    on EVERY rank. Forced IPC: the run ends promptly with "no transport
    works", not a hang. auto (RCCL refused too: ranks sharing a GPU): the run
    goes on over its last resort, the host-staged torch.distributed exchange,
    and its decomposition still verifies bitwise."""
    import time
    env = dict(os.environ, HEAT2D_IPC_ATTACH_STALL="1", HEAT2D_IPC_ATTACH_TIMEOUT="5", OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    t0 = time.time()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--share-gpu", "--grid", "2048",
                        "--steps", "4", "--warmup", "1", "--transport", transport, "--edge-shift", "0"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert "did not return within" in p.stderr, p.stderr[-3000:]
    assert time.time() - t0 < 240
    if transport == "ipc":
        assert p.returncode != 0 and p.stdout.strip() == "", p.stdout
        assert "no transport works on every rank" in p.stderr, p.stderr[-3000:]
        return
    assert p.returncode == 0, failure_text(p.stderr)
    d = json.loads(p.stdout.strip().splitlines()[-1])
    ch = d["config"]["transport_choice"]
    assert d["config"]["transport"] == "torch-dist" and ch["chosen"] == "torch-dist", ch
    assert "error" in ch["rccl"] and "error" in ch["ipc"] and ch["torch-dist"]["ms"] > 0, ch
    assert d["verified"] is True and d["timed_field_check"]["ok"] is True, (d["verify"], d["timed_field_check"])


@pytest.mark.gpu
def test_bench_ipc_field_in_the_stalling_size_window():
    """Two rank processes on one GPU at 23170^2 fp64: each field buffer is
    2.17 GB, inside [2^31, 2^32) bytes, where the runtime's IPC import never
    returned (profiles/r6/ipc/: every such size stalled, at 2, 3 and 4 ranks).
    The IPC transport allocates such fields as 2^32 + 16 MiB, and the attach,
    the timed run and its field check go through (bitwise)."""
    env = dict(os.environ, HEAT2D_IPC_ATTACH_TIMEOUT="20", HEAT2D_IPC_ATTACH_LOG="1", OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--share-gpu", "--transport",
                        "ipc", "--grid", "23170", "--steps", "4", "--warmup", "1", "--verify", "off"],
                       capture_output=True, text=True, timeout=280, env=env)
    assert p.returncode == 0, failure_text(p.stderr)
    d = json.loads(p.stdout.strip().splitlines()[-1])
    assert d["config"]["transport"] == "ipc" and "NOT opened" not in p.stderr
    fc = d["timed_field_check"]
    assert fc["ok"] is True and fc["mismatches"] == 0, fc


@pytest.mark.gpu
def test_bench_plan_cache_second_run(tmp_path):
    """Persistent plan cache: the second identical bench run takes its split
    plans and measured schedule from the cache (each re-validated by one short
    re-time) — prepare() under a second, the same throughput."""
    env_cache = str(tmp_path / "plans.txt")
    old = os.environ.get("HEAT2D_PLAN_CACHE")
    os.environ["HEAT2D_PLAN_CACHE"] = env_cache
    try:
        args = ["--gpus", "1", "--grid", "8192", "--steps", "20", "--warmup", "5"]
        first = run_plain(*args)
        second = run_plain(*args)
    finally:
        os.environ["HEAT2D_PLAN_CACHE"] = old if old is not None else "off"
    assert first["config"]["plan_cache"]["path"] == env_cache and os.path.getsize(env_cache) > 0
    assert first["config"]["plan_cache"]["hits"] == 0 and second["config"]["plan_cache"]["hits"] >= 2
    assert second["config"]["prepare_s"] < 1.0, second["config"]
    assert second["config"]["cycles"] == first["config"]["cycles"]
    # one ~0.5 ms timed cycle per run: a cold first process (clocks) can be
    # 10 % off the second; the cache must not make it slower
    assert second["value"] >= 0.9 * first["value"], (first["value"], second["value"])


@pytest.mark.gpu
def test_bench_plan_cache_respects_knobs(tmp_path):
    """A run with a plan-shaping knob neither reuses plans tuned without it
    nor the other way round: HEAT2D_DYNAMIC=1 (queue forced) fills the cache,
    a HEAT2D_DYNAMIC=0 run on the same cache file then tunes afresh and runs
    the static plan (round 3 replayed the cached dynamic plan instead)."""
    env_cache = str(tmp_path / "plans.txt")
    saved = {k: os.environ.get(k) for k in ("HEAT2D_PLAN_CACHE", "HEAT2D_DYNAMIC")}
    os.environ["HEAT2D_PLAN_CACHE"] = env_cache
    try:
        args = ["--gpus", "1", "--grid", "8192", "--steps", "20", "--warmup", "5", "--verify", "off"]
        os.environ["HEAT2D_DYNAMIC"] = "1"
        dyn = run_plain(*args)
        os.environ["HEAT2D_DYNAMIC"] = "0"
        static = run_plain(*args)
        static2 = run_plain(*args)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    pd = dyn["config"]["launch_plans"]
    ps = static["config"]["launch_plans"]
    assert any(p["dynamic"] == 1 for p in pd.values()), pd
    assert all(p["dynamic"] == 0 and p["origin"] != "cache" for p in ps.values()), ps
    assert static["config"]["plan_cache"]["hits"] == 0
    # the static run's own plans are cached under its key (a hit is re-timed:
    # a drifted one is re-tuned, so hits, not every plan's origin, are checked)
    assert static2["config"]["plan_cache"]["hits"] >= 1
    assert all(p["dynamic"] == 0 for p in static2["config"]["launch_plans"].values())


@pytest.mark.parametrize("nproc", [1, 2])
def test_bench_timed_field_check_windows_cpu(nproc):
    """--field-check windows (what a grid too big for a second copy gets): row
    windows at both slab boundaries and the middle of every slab, each run by a
    single-rank reference solver with steps + 1 rows of margin, bitwise."""
    args = ["--backend", "cpu", "--gpus", str(nproc), "--grid", "150", "--steps", "12", "--warmup", "3", "--tb", "4",
            "--field-check", "windows", "--window-rows", "16", "--verify", "off"]
    d = run_plain(*args)
    fc = d["timed_field_check"]
    assert fc["mode"] == "windows" and fc["ok"] is True and fc["mismatches"] == 0, fc
    assert fc["rows_checked"] == nproc * 3 * 16 and fc["steps"] == 15


@pytest.mark.parametrize("field_check", ["full", "windows"])
def test_bench_edge_shift_cpu(field_check):
    """--edge-shift D: the first and last slab give D rows (clamped to a quarter
    of a slab) to the middle ones; the timed field is checked against a
    reference on the same shifted layout (full) or by row windows, and the
    JSON reports the rows."""
    d = run_plain("--backend", "cpu", "--gpus", "4", "--grid", "100", "--steps", "12", "--warmup", "3", "--tb", "4",
                  "--edge-shift", "5", "--field-check", field_check)
    dec = d["config"]["decomposition"]
    assert dec["edge_shift"] == 5 and dec["rows"] == [20, 30, 30, 20] and dec["balance"] is None
    assert [r["rows"] for r in d["per_rank"]] == [20, 30, 30, 20]
    fc = d["timed_field_check"]
    assert fc["ok"] is True and fc["mode"] == field_check and fc["mismatches"] == 0, fc
    assert d["verified"] is True


def test_bench_edge_shift_measured_cpu():
    """--edge-shift measure on gloo ranks: the path a >= 3-GPU node run takes by
    default (every rank rehearses its own slab, the shifts are gathered and
    decided alike on every rank, the real run is built on the kept shift),
    with the CPU twin's timings; whatever it decides, the run is bitwise."""
    d = run_bench(4, "--grid", "400", "--steps", "12", "--warmup", "3", "--tb", "4", "--edge-shift", "measure",
                  port=29574)
    dec = d["config"]["decomposition"]
    bal = dec["balance"]
    assert bal["loop"] == "self" and len(bal["uniform_ms"]) == 4 and min(bal["uniform_ms"]) > 0, bal
    assert "error" not in bal and bal["uniform_rows"] == [100] * 4
    assert dec["rows"] == [r["rows"] for r in d["per_rank"]] and sum(dec["rows"]) == 400
    assert dec["rows"][0] == 100 - dec["edge_shift"] and dec["edge_shift"] <= 25
    assert (dec["edge_shift"] > 0) == bool(bal.get("kept")), bal
    fc = d["timed_field_check"]
    assert fc["ok"] is True and fc["mismatches"] == 0 and d["verified"] is True, fc


@pytest.mark.parametrize("ic", ["hotspot", "uniform"])
def test_bench_hotspot_jacobi_check_cpu(ic):
    """--ic hotspot (the zero + hot-spot data BASELINE.json names) with the
    r = 1/4 form: the timed field is checked bitwise against the one-step
    r * sum form and against the reference rounding — bitwise on the
    Sterbenz-safe reference IC, within the stated bound on the hot spot
    (values in [0, 1]: sum - 4c can round)."""
    d = run_plain("--backend", "cpu", "--gpus", "2", "--grid", "257", "--steps", "40", "--warmup", "3", "--tb", "6",
                  "--ic", ic, "--verify", "off")
    assert d["config"]["arith"] == "jacobi (r = 1/4)" and d["config"]["ic"] == ic
    fc = d["timed_field_check"]
    assert fc["ok"] is True and fc["engine"] == "cpu-jacobi" and fc["mismatches"] == 0, fc
    ve = fc["vs_exact"]
    assert ve["ok"] is True and ve["engine"] == "cpu-exact", ve
    assert ("bound" in ve) == (ic == "hotspot") and ve["max_abs_diff"] <= ve.get("bound", 0.0)
    assert ("hot spot" in d["data"]) == (ic == "hotspot")


def test_bench_timed_field_check_sigma_fast_cpu():
    """A non-reference arithmetic is checked within its stated bound (fast form,
    sigma 0.2); the contracted form at that sigma is checked bitwise against the
    contracted one-step reference."""
    fast = run_plain("--backend", "cpu", "--grid", "96", "--steps", "10", "--warmup", "2", "--tb", "5", "--sigma", "0.2",
                     "--arith", "fast", "--verify", "off")
    fc = fast["timed_field_check"]
    assert fc["ok"] is True and "bound" in fc and fc["max_abs_diff"] <= fc["bound"], fc
    fma = run_plain("--backend", "cpu", "--grid", "96", "--steps", "10", "--warmup", "2", "--tb", "5", "--sigma", "0.2",
                    "--arith", "fma")
    assert fma["timed_field_check"]["ok"] is True and fma["timed_field_check"]["mismatches"] == 0
    assert fma["verified"] is True and "bound" in fma["verify"], fma["verify"]


@pytest.mark.gpu
def test_bench_timed_field_check_windows_gpu():
    """The full-HBM grids' check (row windows at the slab boundaries and middle,
    single-rank JIT reference runs) on a 4-rank shared-GPU run, and the fast
    arithmetic within its bound."""
    d = run_plain("--gpus", "4", "--share-gpu", "--grid", "4099", "--steps", "23", "--warmup", "3",
                  "--field-check", "windows", "--verify", "off")
    fc = d["timed_field_check"]
    assert fc["mode"] == "windows" and fc["ok"] is True and fc["mismatches"] == 0, fc
    assert fc["rows_checked"] == 4 * 3 * 64
    f = run_plain("--grid", "4096", "--steps", "20", "--warmup", "3", "--sigma", "0.2", "--arith", "fast",
                  "--verify", "off")
    fc = f["timed_field_check"]
    assert fc["ok"] is True and fc["max_abs_diff"] <= fc["bound"] and fc["mode"] == "full", fc


@pytest.mark.gpu
def test_bench_measure_hbm():
    """--measure-hbm: the timed region's stencil dispatches re-run under
    rocprofv3 --pmc (two child processes, the same plans): DRAM bytes close to
    one read + one write of the field per pass, reported beside the plan model."""
    d = run_plain("--grid", "8192", "--steps", "20", "--warmup", "5", "--measure-hbm", "--verify", "off",
                  "--field-check", "off", timeout=900)
    h = d["hbm_measured"]
    assert "error" not in h, h
    assert h["child_cycles"] == d["config"]["cycles"]
    assert 0.9 < h["read_over_field_per_cycle"] < 2.0, h
    field = 8192 * 8192 * 8
    passes = sum(d["config"]["cycles"].values())
    assert 0.95 * field * passes < h["write_bytes"] < 1.2 * field * passes, h
    assert d["hbm_gb_per_s_measured"] == h["gb_per_s"] > 0
