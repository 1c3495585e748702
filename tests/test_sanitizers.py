"""Host sanitizers: the native CLI's host code (runtime, CPU twin kernels,
input.dat parser, I/O, checkpoint-free CLI paths) built with
AddressSanitizer + UndefinedBehaviorSanitizer (`make -C csrc asan`, run by
__graft_entry__.build()) and driven through its CPU path on every reference
program variant, both dtypes, several temporal depths, the output writers and a
set of malformed input.dat files. GPU ASan / xnack+ code objects are not
available on the MI355X pool, so device code is covered by the NaN guard-band
tests (tests/test_ops.py) instead. SURVEY.md §5 (race detection / sanitizers)."""
import os
import subprocess

import numpy as np
import pytest

from heat2d.ops import _native as N

ASAN_CLI = os.path.join(os.path.dirname(N.CLI_PATH), "asan", "heat2d")

pytestmark = pytest.mark.skipif(not os.path.exists(ASAN_CLI), reason="sanitizer build missing (make -C csrc asan)")

ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=99",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=98")


def run(tmp_path, text, *args):
    (tmp_path / "input.dat").write_text(text)
    p = subprocess.run([ASAN_CLI, *args], cwd=tmp_path, env=ENV, capture_output=True, text=True, timeout=300)
    bad = [w for w in ("AddressSanitizer", "LeakSanitizer", "runtime error:") if w in p.stderr + p.stdout]
    assert not bad, p.stderr[-3000:]
    assert p.returncode not in (98, 99), p.stderr[-3000:]
    return p


@pytest.mark.parametrize("args", [
    ["--cpu", "--dtype", "fp64", "--tb", "1"],
    ["--cpu", "--dtype", "fp64", "--tb", "7", "--arith", "fma"],
    ["--cpu", "--dtype", "fp32", "--tb", "16"],
    ["--cpu", "--variant", "serial"],
    ["--cpu", "--variant", "cuda", "--output", "npy"],
    ["--cpu", "--copy-swap"],
    ["--cpu", "--check-every", "3", "--print-every", "4", "--json", "run.json", "--timers"],
    ["--cpu", "--checkpoint", "ck", "--checkpoint-every", "5"],
    ["--cpu", "--gpus", "3", "--tb", "4", "--check-every", "6"],  # host-thread ranks: exchange + all-reduce
])
def test_cli_cpu_paths_clean(tmp_path, args):
    p = run(tmp_path, "67 0.25 0.05 2.0 23 1\n", *args)
    assert p.returncode == 0, p.stderr[-2000:]
    assert "simulation completed" in p.stdout


def test_checkpoint_restart_clean(tmp_path):
    """Native checkpoint writer + meta.json / .npy parsers under ASan/UBSan,
    including a truncated rank file (clean error, no memory error)."""
    run(tmp_path, "33 0.25 0.05 1.0 9 1\n", "--cpu", "--quiet", "--checkpoint", "ck")
    p = run(tmp_path, "33 0.25 0.05 1.0 20 1\n", "--cpu", "--quiet", "--restart", "ck")
    assert p.returncode == 0, p.stderr[-2000:]
    f = tmp_path / "ck" / (tmp_path / "ck" / "latest").read_text().strip() / "rank00000.npy"
    f.write_bytes(f.read_bytes()[:200])
    p = run(tmp_path, "33 0.25 0.05 1.0 20 1\n", "--cpu", "--quiet", "--restart", "ck")
    assert p.returncode != 0 and "truncated" in p.stderr


def test_outputs_match_uninstrumented(tmp_path):
    """The instrumented build computes the same field as the regular CLI."""
    a, b = tmp_path / "a", tmp_path / "b"
    a.mkdir()
    b.mkdir()
    run(a, "50 0.25 0.05 1.0 17 1\n", "--cpu", "--output", "npy", "--quiet")
    (b / "input.dat").write_text("50 0.25 0.05 1.0 17 1\n")
    subprocess.run([N.CLI_PATH, "--cpu", "--output", "npy", "--quiet"], cwd=b, check=True, capture_output=True)
    fa = sorted(f for f in os.listdir(a) if f.endswith(".npy"))
    assert fa and fa == sorted(f for f in os.listdir(b) if f.endswith(".npy"))
    for f in fa:
        assert np.array_equal(np.load(a / f), np.load(b / f))


@pytest.mark.parametrize("text", ["", "64", "64 0.25 0.05", "abc def", "64 0.25 0.05 1.0 -3",
                                  "0 0.25 0.05 1.0 5", "64,0.25,0.05,1.0d0,5,0\n", "64 0.25 0.05 1.0 5 0 extra junk",
                                  "9" * 40 + " 0.25 0.05 1.0 5", "64 1e999 0.05 1.0 5"])
def test_malformed_input_dat(tmp_path, text):
    """Parser edge cases: a clean error (or a clean run), never a memory error."""
    run(tmp_path, text, "--cpu", "--quiet")


def test_unstable_run_writes_non_finite(tmp_path):
    """sigma far above the 1/4 stability limit: the field overflows to inf/NaN
    and the ASCII writers must still format it (they dereferenced a missing
    exponent before the UBSan build caught it)."""
    p = run(tmp_path, "16 40.0 0.05 1.0 400 1\n", "--cpu", "--quiet")
    assert p.returncode == 0, p.stderr[-2000:]
    txt = (tmp_path / "soln00000.dat").read_text()
    assert "Infinity" in txt or "NaN" in txt


@pytest.mark.parametrize("how", ["abort", "free"])
def test_fatal_signal_prints_native_backtrace(how):
    """A glibc heap-check abort ("free(): invalid pointer") or any fatal
    signal in a process that loaded the engine prints the native frames (which
    library called free()) and then Python's faulthandler stacks; the exit
    status stays the signal's. The round-5 abort left neither."""
    import sys
    body = ("import os, faulthandler; faulthandler.enable()\n"
            "from heat2d.ops import _native as N; N.lib()\n")
    if how == "abort":
        body += "os.abort()\n"
    else:  # free() of a pointer malloc never returned: glibc aborts
        body += ("import ctypes; libc = ctypes.CDLL('libc.so.6'); buf = ctypes.create_string_buffer(64)\n"
                 "libc.free(ctypes.cast(ctypes.addressof(buf) + 16, ctypes.c_void_p))\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "-c", body], capture_output=True, text=True, timeout=120, cwd=root)
    assert p.returncode == -6, (p.returncode, p.stderr[-2000:])
    assert "heat2d: fatal signal, native backtrace:" in p.stderr, p.stderr[-2000:]
    assert "Fatal Python error: Aborted" in p.stderr  # the previous handler (faulthandler) ran after ours
    if how == "free":
        assert "free()" in p.stderr and "libc.so.6" in p.stderr


ASAN_DIR = os.path.dirname(ASAN_CLI)


@pytest.mark.skipif(not os.path.exists(os.path.join(ASAN_DIR, "python")), reason="make -C csrc asan-python missing")
def test_bench_multi_rank_cpu_under_asan(tmp_path):
    """the multi-process `bench.py --backend cpu --check`
    path (3 gloo ranks started by bench.py itself, transport trials, timed run,
    field check, verification, checkpoint-free teardown) with every rank under
    host AddressSanitizer: an interpreter with ASan's runtime linked first,
    PYTHONMALLOC=malloc (every Python allocation through ASan's allocator) and
    the instrumented engine (HEAT2D_LIB). No report, a clean exit and the one
    JSON line. (The GPU path cannot run under this runtime: its HSA
    interceptors refuse the first device-pool allocation, profiles/r6/d/.)"""
    import json
    import sys  # noqa: F401
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:exitcode=99", PYTHONMALLOC="malloc",
               HEAT2D_LIB=os.path.join(ASAN_DIR, "libheat2d.so"), OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([os.path.join(ASAN_DIR, "python"), os.path.join(root, "bench.py"), "--backend", "cpu",
                        "--gpus", "3", "--grid", "100", "--steps", "24", "--warmup", "4", "--tb", "4", "--check",
                        "--edge-shift", "4"], cwd=tmp_path, env=env, capture_output=True, text=True, timeout=600)
    assert "AddressSanitizer" not in p.stderr, p.stderr[-4000:]
    assert p.returncode == 0, p.stderr[-3000:]
    d = json.loads(p.stdout.strip().splitlines()[-1])
    assert d["n_gpus"] == 3 and d["verified"] is True and d["timed_field_check"]["ok"] is True
    assert d["config"]["decomposition"]["rows"] == [30, 41, 29]  # 34 / 33 / 33, 4 rows from each edge
