"""Collective transport selection (parallel/select.py) and the bench's
self-verification, on CPU: the logic bench.py runs on a multi-GPU node before
its timed region (try RCCL and IPC, skip whatever fails on any rank, keep the
faster by the MAX over ranks, then check a small decomposition bitwise).

Pure-function cases use single-rank collectives; the multi-rank cases run gloo
ranks (tests/select_worker.py), where a failure on ONE rank must make every
rank skip the candidate alike."""
import json
import os
import socket
import subprocess
import sys

import pytest

from heat2d.parallel import select

HERE = os.path.dirname(os.path.abspath(__file__))
ident = (lambda v: v)  # noqa: E731  (a 1-rank all-reduce)


def test_edge_shift_estimate():
    # N = 8 slabs of 32768^2 (profiles/r6/b/): edges 668 / 663 us, middles 624 us on 4096 rows
    ms = [0.668] + [0.624] * 6 + [0.663]
    rows = [4096] * 8
    d = select.edge_shift_estimate(ms, rows, cap=1024)
    a = 0.624 / 4096
    assert d == round((0.668 - 0.624) / a * 6 / 8) and 200 < d < 300
    # after the shift the edges and the middles meet (the linear model)
    assert abs((0.668 - a * d) - (0.624 + a * 2 * d / 6)) < a
    assert select.edge_shift_estimate(ms, rows, cap=100) == 100  # clamped
    assert select.edge_shift_estimate([1.0, 1.0, 1.0], [10, 10, 10], cap=5) == 0  # balanced already
    assert select.edge_shift_estimate([0.9, 1.0, 0.9], [10, 10, 10], cap=5) == 0  # edges faster: never negative
    assert select.edge_shift_estimate([2.0, 1.0], [10, 10], cap=5) == 0  # 2 ranks: both are edges


def _slab_model(P, n, a=1e-3, excess=0.0504):
    """Rank r's ms on its slab of decompose(n, P, r, shift): a per row, edges + excess."""
    from heat2d.ops import _native as N
    state = {}

    def rows_of(shift):
        return [N.decompose(n, P, r, shift)[1] for r in range(P)]

    def measure(shift):
        state["shift"] = shift
        return 0.0  # (every rank's value comes from gather below)

    def gather(_v):
        rows = rows_of(state["shift"])
        return [a * rows[r] + (excess if r in (0, P - 1) else 0.0) for r in range(P)]
    return measure, gather, rows_of


def test_balance_edges_keeps_a_faster_shift():
    measure, gather, rows_of = _slab_model(8, 32768)
    d, rep = select.balance_edges(measure, gather, rows_of, cap=1024)
    assert d == rep["estimate"] == 38 and rep["kept"] is True  # 50.4 rows of excess x 6 / 8
    assert max(rep["shifted_ms"]) < max(rep["uniform_ms"]) and rep["shifted_rows"][0] == 4096 - d


def test_balance_edges_repeats_outvote_one_slow_rehearsal():
    """One slow shifted rehearsal on one rank: with one timing per layout it
    decides (shift rejected); alternating two per layout, each rank's fastest
    counts and the shift is kept."""
    for reps, kept in ((1, False), (2, True)):
        measure, gather, rows_of = _slab_model(8, 32768)
        seen = []

        def measure_n(shift):
            seen.append(shift)
            return measure(shift)

        def gather_n(v):
            ms = gather(v)
            if len(seen) == 2:  # the first shifted round: rank 3 hiccups
                ms[3] += 0.5
            return ms
        d, rep = select.balance_edges(measure_n, gather_n, rows_of, cap=1024, reps=reps)
        assert rep["kept"] is kept and (d > 0) is kept and rep["reps"] == reps
        assert seen == ([0, 38] if reps == 1 else [0, 38, 0, 38])


def test_balance_edges_rejects_a_slower_shift_and_failures():
    measure, gather, rows_of = _slab_model(4, 1000)
    d, rep = select.balance_edges(measure, gather, rows_of, cap=200)
    assert d == rep["estimate"] > 0  # (the model's shift helps)

    calls = []

    def measure_n(shift):
        calls.append(shift)
        return measure(shift)

    def gather_n(v):
        ms = gather(v)
        return ms if len(calls) == 1 else [x + 1.0 for x in ms]  # round 2 measured slower
    d, rep = select.balance_edges(measure_n, gather_n, rows_of, cap=200)
    assert d == 0 and rep["kept"] is False and rep["estimate"] > 0

    def broken(shift):
        raise RuntimeError("rehearsal failed")
    d, rep = select.balance_edges(broken, lambda v: [v] * 4, rows_of, cap=200)
    assert d == 0 and "failed" in rep["error"]


def test_choose_fastest():
    chosen, rep = select.choose_transport(["rccl", "ipc"], lambda k: {"rccl": 2.0, "ipc": 1.5}[k], ident, ident)
    assert chosen == "ipc" and rep == {"rccl": {"ms": 2.0}, "ipc": {"ms": 1.5}}


def test_choose_skips_failing_candidate():
    def trial(kind):
        if kind == "rccl":
            raise RuntimeError("ncclCommInitRank failed")
        return 3.0
    chosen, rep = select.choose_transport(["rccl", "ipc"], trial, ident, ident)
    assert chosen == "ipc" and "ncclCommInitRank failed" in rep["rccl"]["error"] and rep["ipc"] == {"ms": 3.0}


def test_choose_none_when_all_fail():
    def trial(kind):
        raise select.Skip("no fabric")
    chosen, rep = select.choose_transport(["rccl", "ipc"], trial, ident, ident)
    assert chosen is None and set(rep) == {"rccl", "ipc"}


def test_try_collective_cleans_up_on_remote_failure():
    """Local success but a failure elsewhere (the MIN all-reduce says 0):
    the local object is cleaned up and the caller sees the failure."""
    cleaned = []
    obj, why = select.try_collective(lambda: "comm", lambda v: 0.0, cleanup=cleaned.append)
    assert obj is None and why == "failed on another rank" and cleaned == ["comm"]


def test_choose_first_working_never_builds_the_fallback():
    """"auto": RCCL works on every rank, so IPC (its fallback) is never tried."""
    tried = []

    def trial(kind):
        tried.append(kind)
        return 2.0
    chosen, rep = select.choose_transport(["rccl", "ipc"], trial, ident, ident, first_working=True)
    assert chosen == "rccl" and tried == ["rccl"] and "skipped" in rep["ipc"] and rep["rccl"] == {"ms": 2.0}


def test_choose_first_working_falls_back():
    def trial(kind):
        if kind == "rccl":
            raise RuntimeError("invalid usage (two ranks on one GPU)")
        return 3.0
    chosen, rep = select.choose_transport(["rccl", "ipc"], trial, ident, ident, first_working=True)
    assert chosen == "ipc" and "error" in rep["rccl"] and rep["ipc"] == {"ms": 3.0}


def test_choose_auto_reaches_the_host_transport():
    """auto's whole chain on a node where neither RCCL nor the IPC mappings
    attach: both fail on every rank alike and the host-staged exchange runs."""
    tried = []

    def trial(kind):
        tried.append(kind)
        if kind != "torch-dist":
            raise RuntimeError(f"{kind} cannot attach")
        return 9.0
    cands = select.candidate_transports("auto", 8, True)
    chosen, rep = select.choose_transport(cands, trial, ident, ident, first_working=True)
    assert chosen == "torch-dist" and tried == ["rccl", "ipc", "torch-dist"]
    assert "cannot attach" in rep["rccl"]["error"] and "cannot attach" in rep["ipc"]["error"]
    assert rep["torch-dist"] == {"ms": 9.0}


def test_deadline_fires_on_a_stuck_phase():
    import time
    fired = []
    with select.deadline(0.2, "RCCL transport construction", rank=3, on_expire=fired.append):
        time.sleep(0.6)
    assert len(fired) == 1 and "rank 3: RCCL transport construction did not finish within 0.2 s" in fired[0]
    fired.clear()
    with select.deadline(5.0, "quick phase", on_expire=fired.append):
        pass
    time.sleep(0.05)
    assert fired == []
    with select.deadline(0, "unbounded", on_expire=fired.append):
        pass
    assert fired == []


def test_deadline_exits_the_process():
    """Without a test hook the stuck process exits with status 124 and every
    thread's stack on stderr (the launcher then stops the other ranks)."""
    code = ("import time; from heat2d.parallel import select\n"
            "with select.deadline(0.3, 'IPC solver construction', rank=1):\n    time.sleep(30)\n")
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60,
                       cwd=os.path.dirname(HERE))
    assert p.returncode == select.EXIT_DEADLINE, p.stderr
    assert "rank 1: IPC solver construction did not finish" in p.stderr and "time.sleep" not in p.stdout
    assert "Thread" in p.stderr  # faulthandler's dump of every thread


def test_rank_report_summarises_the_ranks():
    from heat2d.parallel.transport import SelfTransport
    tr = SelfTransport()
    try:
        rows = [(0, 50), (50, 50)]
        mine = []

        def gather(me):  # two ranks: this one and a fabricated peer on another device
            other = dict(me, rank=1, row0=rows[1][0], rows=rows[1][1], timed_ms=2.5, device=1,
                         fabric=dict(me["fabric"], rank=1))
            mine.append(me)
            return [other, me]
        rep = select.rank_report(gather, rank=0, device=None, transport=tr, rows=50, row0=0, timed_s=0.002)
    finally:
        tr.close()
    assert [r["rank"] for r in rep["ranks"]] == [0, 1] and rep["timed_ms"] == {"min": 2.0, "max": 2.5}
    assert rep["fabric_kind"] == "host" and rep["fabric_nranks"] == 1 and rep["distinct_devices"] == 2
    assert mine[0]["fabric"] == {"kind": "host", "nranks": 1, "rank": 0, "device": -1}


@pytest.mark.parametrize("arith,sterbenz,expect", [
    ("exact", True, [("exact", True)]), ("fma", False, [("fma", True)]), ("fast", True, [("exact", False)]),
    ("jacobi", True, [("jacobi", True), ("exact", True)]), ("jacobi", False, [("jacobi", True), ("exact", False)])])
def test_reference_checks(arith, sterbenz, expect):
    """The r = 1/4 form is checked bitwise against its own one-step form and
    against the reference rounding: bitwise only on Sterbenz-safe data."""
    assert select.reference_checks(arith, 0.25, sterbenz) == expect


@pytest.mark.parametrize("requested,world,hip,expect", [("auto", 8, True, ["rccl", "ipc", "torch-dist"]),
                                                        ("best", 8, True, ["rccl", "ipc"]),
                                                        ("host", 2, True, ["torch-dist"]),
                                                        ("peer", 2, True, ["ipc"]),
                                                        ("rccl", 2, True, ["rccl"]), ("auto", 1, True, []),
                                                        ("auto", 4, False, ["torch-dist"])])
def test_candidates(requested, world, hip, expect):
    assert select.candidate_transports(requested, world, hip) == expect


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_ranks(tmp_path, world, scenario, timeout=240):
    port = free_port()
    env = dict(os.environ, OMP_NUM_THREADS="1", HEAT2D_CPU_THREADS="2")
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "select_worker.py"), str(r), str(world), str(port),
                               str(tmp_path), scenario], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
             for r in range(world)]
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=timeout)[0].decode(errors="replace"))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for p, o in zip(procs, outs):
        assert p.returncode == 0, o[-3000:]
    res = []
    for r in range(world):
        with open(tmp_path / f"rank{r}.json") as f:
            res.append(json.load(f))
    return res


def test_gloo_failure_on_one_rank_falls_back_everywhere(tmp_path):
    res = run_ranks(tmp_path, 3, "fail_rccl_on_1")
    for r in res:
        assert r["chosen"] == "ipc", r
        assert "duplicate GPU" in r["report"]["rccl"]["error"] or r["report"]["rccl"]["error"] == "failed on another rank"
        assert r["report"]["ipc"] == {"ms": 2.0}
    # ranks that did build an RCCL object released it
    assert res[0]["built"] == ["rccl", "cleanup-rccl", "ipc"] and res[1]["built"] == ["ipc"]


def test_gloo_choice_uses_the_slowest_rank(tmp_path):
    """rccl is faster on rank 0 but slow on rank 1: MAX over ranks decides."""
    res = run_ranks(tmp_path, 2, "slow_rank")
    assert all(r["chosen"] == "ipc" and r["report"] == {"rccl": {"ms": 5.0}, "ipc": {"ms": 3.0}} for r in res), res


def test_gloo_verify_decomposition_bitwise(tmp_path):
    res = run_ranks(tmp_path, 3, "verify")
    for r in res:
        assert r["verify"] == {"verified": True, "n": 113, "steps": 29, "max_abs_diff": 0.0}, r
