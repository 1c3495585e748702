"""Collective transport selection and a bitwise self-check of a decomposition.

The reference has exactly one way to move halos: host-staged MPI_Sendrecv
(fortran/hip/heat.F90:196-230) over whatever MPI the job was linked with.
Here a multi-GPU run can exchange halos through RCCL send/recv or through the
IPC transport (hipIpc mappings of the neighbours' fields, device copies
ordered by stream-side counters), and which one is faster depends on the node
(xGMI topology, RCCL's channel kernels sharing the CUs with the interior
launch, whether the exchange can be graph-captured: IPC's can, RCCL's cannot).
So the first run on a node decides by measurement, collectively:

* :func:`collective_ok` — a step that may fail on some ranks (e.g. RCCL
  refusing two ranks on one GPU) succeeds only if it succeeded on every rank;
  every rank then takes the same branch.
* :func:`choose_transport` — try each candidate (build + time the real timed
  loop), MAX over ranks per candidate, keep the fastest; a candidate that
  fails anywhere is skipped on every rank (the fallback).
* :func:`balance_edges` — the edge slabs' rows for >= 3 ranks: each rank
  times its own slab, and rows move from the two edge slabs (whose frame-side
  band costs extra) to the middle ones when that lowers the slowest slab.
* :func:`verify_decomposition` — a small uneven, rough-data problem run with
  the chosen transport and rank layout through the same engine paths
  (autotuned split plans, measured schedule, graphs where the transport
  captures), gathered to rank 0 and compared bitwise with the NumPy golden
  model (models/reference.py).

The selection logic takes its collectives as callables, so it is tested on CPU
with plain functions and with gloo ranks (tests/test_select.py).
"""
from __future__ import annotations

import contextlib
import traceback
from typing import Callable, Dict, List, Optional, Sequence, Tuple


class Skip(Exception):
    """A candidate failed a collective phase on some rank: raised on EVERY
    rank (after the phase's agreement), so all of them skip it alike."""


def collective_ok(local_ok: bool, allreduce_min: Callable[[float], float]) -> bool:
    """True iff ``local_ok`` holds on every rank (one MIN all-reduce)."""
    return allreduce_min(1.0 if local_ok else 0.0) >= 1.0


def try_collective(fn: Callable[[], object], allreduce_min: Callable[[float], float],
                   cleanup: Optional[Callable[[object], None]] = None) -> Tuple[Optional[object], Optional[str]]:
    """Run ``fn`` on every rank; if it raised on ANY rank, undo it where it
    succeeded (``cleanup``) and return (None, reason) everywhere, else
    (result, None). Exceptions are caught, never propagated: the caller picks
    the next candidate on every rank alike."""
    obj, why = None, None
    try:
        obj = fn()
    except Skip as e:  # a nested phase already agreed (and reported) that it failed
        why = str(e)
    except Exception as e:  # noqa: BLE001 - any failure of a candidate is a fallback, reported
        why = f"{type(e).__name__}: {e}".strip()
        traceback.print_exc()
    if collective_ok(why is None, allreduce_min):
        return obj, None
    if obj is not None and cleanup is not None:
        try:
            cleanup(obj)
        except Exception:  # noqa: BLE001
            traceback.print_exc()
    return None, why or "failed on another rank"


def choose_transport(candidates: Sequence[str], trial: Callable[[str], float],
                     allreduce_min: Callable[[float], float],
                     allreduce_max: Callable[[float], float],
                     first_working: bool = False) -> Tuple[Optional[str], Dict[str, dict]]:
    """Try the candidate transports in order with ``trial(kind) -> ms`` (it
    builds the transport and the solver and times the real loop; raising =
    unusable), reduce each time with MAX over ranks, and return (kind, report).
    ``first_working``: stop at the first candidate that works on every rank
    (the later ones are fallbacks, never built — bench.py's default "auto":
    RCCL, and IPC only where RCCL cannot be built); else time them all and
    keep the fastest ("best"). The report holds {"ms": max-over-ranks ms},
    {"error": reason} or {"skipped": why} per kind, identical on every rank (a
    failure anywhere skips the kind everywhere). None if no candidate works."""
    report: Dict[str, dict] = {}
    best, best_ms = None, float("inf")
    for kind in candidates:
        if first_working and best is not None:
            report[kind] = {"skipped": f"{best} works on every rank ({kind} is its fallback)"}
            continue
        ms, why = try_collective(lambda: trial(kind), allreduce_min)
        if why is not None:
            report[kind] = {"error": why}
            continue
        ms = allreduce_max(float(ms))
        report[kind] = {"ms": round(ms, 4)}
        if ms < best_ms:
            best, best_ms = kind, ms
    return best, report


def candidate_transports(requested: str, world: int, hip: bool) -> List[str]:
    """Transports a run may use, in order: one forced kind, or both GPU
    transports for "auto" / "best" (RCCL first: the reference's own model of
    an MPI-style fabric; IPC second — with "auto" only as the fallback where
    RCCL cannot be built, so a node run whose RCCL works never builds the IPC
    mappings; "best" times both). "auto" ends with the host-staged
    torch.distributed exchange (pinned staging + gloo send/recv, the
    reference's own MPI path): slow, but a node where neither RCCL nor the IPC
    mappings attach still runs and reports. Single-rank runs have nothing to
    choose; CPU ranks have one transport (torch.distributed host callbacks),
    run through the same trial."""
    if world <= 1:
        return []
    if not hip:
        return ["torch-dist"]
    if requested == "auto":
        return ["rccl", "ipc", "torch-dist"]
    if requested == "best":
        return ["rccl", "ipc"]
    if requested == "host":
        return ["torch-dist"]
    return ["ipc" if requested in ("ipc", "peer") else "rccl"]


EXIT_DEADLINE = 124


@contextlib.contextmanager
def deadline(seconds: float, what: str, rank: int = 0, on_expire: Optional[Callable[[str], None]] = None):
    """Bound a phase that may block inside a native call no other timeout
    covers (transport construction: RCCL bootstrap, hipIpcOpenMemHandle;
    solver construction with its collective attach). If the phase has not
    finished after ``seconds``, every thread's Python stack goes to stderr and
    the process exits with status 124 (``on_expire(message)`` instead, for
    tests): the launcher (bench.py's own, or torchrun) then stops the other
    ranks, so a stuck rank ends the run in bounded time instead of hanging it.
    Exiting is the only safe end: the blocked thread may hold HIP runtime
    locks, and a GPU-initialised process is never re-exec'd. ``seconds`` <= 0:
    unbounded."""
    if not seconds or seconds <= 0:
        yield
        return
    import faulthandler
    import os
    import sys
    import threading
    done = threading.Event()

    def watch():
        if done.wait(seconds):
            return
        msg = f"rank {rank}: {what} did not finish within {seconds:g} s (HEAT2D_INIT_TIMEOUT); exiting"
        if on_expire is not None:
            on_expire(msg)
            return
        sys.stderr.write(f"heat2d: {msg}\n")
        sys.stderr.flush()
        faulthandler.dump_traceback(all_threads=True)
        os._exit(EXIT_DEADLINE)

    t = threading.Thread(target=watch, name="heat2d-deadline", daemon=True)
    t.start()
    try:
        yield
    finally:
        done.set()


def rank_report(gather: Callable[[dict], List[dict]], *, rank: int, device: Optional[int], transport,
                rows: int, row0: int, timed_s: float, extra: Optional[dict] = None) -> dict:
    """Per-rank proof of a multi-rank run, gathered to every rank: what the
    fabric itself reports (RCCL: ncclCommCount / ncclCommUserRank /
    ncclCommCuDevice), the rank's device ordinal and PCI bus id, host, slab
    rows and its own timed seconds. Summarised as {"ranks": [...],
    "fabric_nranks": n or None (ranks disagree), "distinct_devices": k,
    "timed_ms": {"min", "max"}} — the reference prints "MPI rank r using GPU
    d" and "Automatic MPI decomposition: P x 1" (fortran/hip/heat.F90:125,145)."""
    import socket
    from ..ops import _native as N
    me = {"rank": int(rank), "host": socket.gethostname(), "device": device, "rows": int(rows), "row0": int(row0),
          "timed_ms": round(float(timed_s) * 1e3, 4)}
    try:
        me["fabric"] = N.transport_info(transport.handle)
    except Exception as e:  # noqa: BLE001 - reported, never fatal after the timed run
        me["fabric"] = {"error": str(e)}
    if device is not None and device >= 0:
        try:
            me["pci_bus_id"] = N.pci_bus_id(device)
        except Exception as e:  # noqa: BLE001
            me["pci_bus_id"] = f"error: {e}"
    if extra:
        me.update(extra)
    ranks = sorted(gather(me), key=lambda d: d["rank"])
    nr = {d["fabric"].get("nranks") for d in ranks}
    devs = {(d["host"], d.get("pci_bus_id") or d.get("device")) for d in ranks}
    ms = [d["timed_ms"] for d in ranks]
    return {"ranks": ranks, "fabric_nranks": nr.pop() if len(nr) == 1 else None,
            "fabric_kind": ranks[0]["fabric"].get("kind"),
            "distinct_devices": len(devs), "timed_ms": {"min": min(ms), "max": max(ms)}}


def edge_shift_estimate(slab_ms: Sequence[float], rows: Sequence[int], cap: int) -> int:
    """Rows each edge slab should give to the middle slabs (decompose()'s
    ``edge_shift``) so the first and last rank finish with the middle ones.

    ``slab_ms[r]`` is rank r's own cycle time on ``rows[r]`` rows. A middle
    slab costs a = (sum of middle ms) / (sum of middle rows) per row; an edge
    slab's excess over that rate is E = ms - a * rows (its frame-side band:
    profiles/r6/b/). Moving d rows from each edge slab to the P - 2 middle
    ones saves a * d on the edges and costs a * 2d / (P - 2) in the middle,
    so they meet at d = E / a * (P - 2) / P (rounded, clamped to [0, cap]).
    The larger of the two edges' excesses sets d. 0 below 3 ranks."""
    P = len(slab_ms)
    if P < 3 or len(rows) != P:
        return 0
    mid = range(1, P - 1)
    mid_rows = sum(rows[i] for i in mid)
    a = sum(slab_ms[i] for i in mid) / mid_rows if mid_rows > 0 else 0.0
    if not a > 0:
        return 0
    excess = max(slab_ms[0] - a * rows[0], slab_ms[-1] - a * rows[-1])
    d = int(round(excess / a * (P - 2) / P))
    return max(0, min(d, int(cap)))


def time_own_slab(make: Callable[[], Tuple[object, Callable[[], None]]], steps: int, warmup: int,
                  sync: Callable[[], None] = lambda: None, reps: int = 5) -> float:
    """ms of one ``step(steps)`` of a rehearsal solver: ``make()`` returns
    (solver, cleanup) — this rank's slab on a 1-rank loop exchange (or none) —
    then ``warmup`` steps, ``prepare(steps)``, one untimed ``step(steps)``
    (clocks as in a timed loop) and the fastest of ``reps`` timed ones. The
    per-rank measurement :func:`balance_edges` gathers."""
    import time
    s, cleanup = make()
    try:
        if warmup > 0:
            s.step(warmup)
        s.synchronize()
        s.prepare(steps)
        s.step(steps)
        best = float("inf")
        for _ in range(max(1, reps)):
            sync()
            t0 = time.perf_counter()
            s.step(steps)
            s.synchronize()
            sync()
            best = min(best, time.perf_counter() - t0)
        return best * 1e3
    finally:
        cleanup()


def balance_edges(measure: Callable[[int], float], gather: Callable[[float], List[float]],
                  rows_of: Callable[[int], List[int]], cap: int, reps: int = 2) -> Tuple[int, dict]:
    """The edge-balanced decomposition of a >= 3-rank run, by measurement.

    ``measure(shift)`` times THIS rank's own slab of the decomposition with
    that edge shift (bench.py: a 1-rank loop-exchange rehearsal of the slab,
    the driver's timing) and returns ms; ``gather(v)`` returns every rank's v
    in rank order; ``rows_of(shift)`` the rows of every rank. The uniform
    slabs are timed first and d estimated from them
    (:func:`edge_shift_estimate`); then shifted and uniform slabs alternate
    until each layout has ``reps`` timings, and every rank keeps its fastest
    per layout (one slow rehearsal on one rank would otherwise decide). d is
    kept only if the shifted layout's slowest slab beats the uniform one's (a
    node run reports the MAX over ranks). A failure on any rank (measure
    raising, a non-finite time) keeps 0 on every rank. Collective: every rank
    calls it with the same ``cap`` and ``reps``. Returns (shift, report),
    identical on every rank."""
    import math

    def timed(shift: int) -> List[float]:
        try:
            v = float(measure(shift))
        except Exception:  # noqa: BLE001 - reported below through the gathered NaN
            traceback.print_exc()
            v = float("nan")
        return [float(x) for x in gather(v)]

    def ok(ms: List[float]) -> bool:
        return all(math.isfinite(x) and x > 0 for x in ms)

    ms0 = timed(0)
    report: Dict[str, object] = {"uniform_rows": rows_of(0), "uniform_ms": [round(x, 4) for x in ms0]}
    if not ok(ms0):
        report["error"] = "a rank's uniform slab rehearsal failed"
        return 0, report
    d = edge_shift_estimate(ms0, rows_of(0), cap)
    report["estimate"] = d
    if d == 0:
        return 0, report
    report["shifted_rows"] = rows_of(d)
    ms1 = None
    for rep in range(max(1, reps)):
        t1 = timed(d)
        if not ok(t1):
            report["error"] = "a rank's shifted slab rehearsal failed"
            return 0, report
        ms1 = t1 if ms1 is None else [min(a, b) for a, b in zip(ms1, t1)]
        if rep + 1 < reps:
            t0 = timed(0)
            if not ok(t0):
                report["error"] = "a rank's uniform slab rehearsal failed"
                return 0, report
            ms0 = [min(a, b) for a, b in zip(ms0, t0)]
    report["uniform_ms"] = [round(x, 4) for x in ms0]
    report["shifted_ms"] = [round(x, 4) for x in ms1]
    report["reps"] = max(1, reps)
    keep = max(ms1) < max(ms0)
    report["kept"] = keep
    return (d if keep else 0), report


def _pow2(r: float) -> bool:
    import math
    return r > 0 and math.frexp(r)[0] == 0.5


def reference_checks(arith: str, r: float, sterbenz: bool) -> List[Tuple[str, bool]]:
    """The independent reference runs a timed field of ``arith`` is checked
    against, as (run-time compiled one-step form, bitwise?) pairs; the first
    one is the field check's verdict, the others are reported beside it.

    * exact / fma: their own one-step forms, bitwise (any r, any data);
    * jacobi (r = 1/4): the JIT's own r * sum form, bitwise (scaling by
      powers of 4 is exact, so the temporal-blocked scaled levels round like
      one step per launch), plus the reference rounding ``exact``: bitwise
      where sum - 4c is exact (``sterbenz``: the reference IC, values in
      [1, 2]), else within the stated bound (models/reference.fast_error_bound)
      — on the hot-spot data BASELINE.json names (values in [0, 1]) the two
      forms round differently and only the bound holds;
    * fast (scaled levels, any r): the reference rounding, within the bound."""
    if arith == "fma":
        return [("fma", True)]
    if arith == "fast":
        return [("exact", False)]
    if arith == "jacobi":
        return [("jacobi", True), ("exact", bool(sterbenz))]
    return [("exact", True)]


def reference_arith(arith: str, r: float, sterbenz: bool = True) -> Tuple[str, bool]:
    """(arithmetic of the primary independent reference run, bitwise?)."""
    return reference_checks(arith, r, sterbenz)[0]


def field_windows(nrows: int, steps: int, row0: int, n_global: int, window: int = 64) -> List[Tuple[int, int, int, int]]:
    """Row windows of a slab checked when a second copy of the whole slab does
    not fit (the full-HBM grids): its first rows, its last rows and its middle
    rows — slab boundaries are where a decomposition or band error shows.
    Each entry (local r0, rows, ref global row0, ref rows): the reference run
    covers the window plus ``steps + 1`` rows on each side (clipped to the
    grid), because its own edge rows are stale ghost rows — an error entering
    there moves at most one row per step, so the window itself is exact."""
    m = max(1, min(window, nrows))
    starts = sorted({0, max(0, nrows - m), max(0, (nrows - m) // 2)})
    out = []
    for a in starts:
        g0 = row0 + a
        lo = max(0, g0 - steps - 1)
        hi = min(n_global, g0 + m + steps + 1)
        out.append((a, m, lo, hi - lo))
    return out


def check_timed_field(timed, make_ref: Callable[..., object], steps: int, *, arith: str, r: float, dtype: str,
                      t0_absmax: float, full: bool, amax: Callable[[float], float],
                      asum: Callable[[float], float], window: int = 64, sterbenz: bool = True) -> dict:
    """Check the field a timed run produced against independent engines.

    ``timed`` holds IC + ``steps`` steps. ``make_ref(full, rows=None,
    slab_row0=None, arith=...)`` builds a reference solver from the same IC:
    full=True — the same rank layout and transport kind as the timed run
    (collective); full=False — a single-rank solver owning global rows
    [slab_row0, slab_row0 + rows) (see field_windows). Each reference runs
    ``steps`` steps one step per launch and the fields are compared on the
    device (HeatSolver.compare); results are reduced over ranks (``amax`` /
    ``asum``, the same on every rank). The references are
    :func:`reference_checks` of ``arith``: the first decides "ok", the others
    are reported under "vs_<arith>" with their own verdict (``t0_absmax``:
    max |T| of the IC, for the error bounds; ``sterbenz``: the IC keeps every
    sum - 4c exact)."""
    import numpy as np
    npdt = np.float64 if dtype == "fp64" else np.float32

    def one(ref_arith: str, bitwise: bool) -> dict:
        diff, mism, rows = 0.0, 0.0, 0
        if full:
            ref = make_ref(True, arith=ref_arith)
            try:
                ref.step(steps)
                ref.synchronize()
                res = timed.compare(ref)
            finally:
                ref.close()
            diff, mism, rows = res["max_abs_diff"], float(res["mismatches"]), timed.nrows
        else:
            for a, m, g0, nr in field_windows(timed.nrows, steps, timed.row0, timed.problem.n_owned, window):
                ref = make_ref(False, rows=nr, slab_row0=g0, arith=ref_arith)
                try:
                    ref.step(steps)
                    ref.synchronize()
                    res = timed.compare(ref, r0=a, nrows=m, other_r0=timed.row0 + a - g0)
                finally:
                    ref.close()
                d = res["max_abs_diff"]
                diff = d if (d != d or diff != diff) else max(diff, d)
                mism += float(res["mismatches"])
                rows += m
        nan = diff != diff
        diff = amax(float("inf") if nan else diff)
        mism = asum(mism)
        rows = int(asum(float(rows)))
        out = {"mode": "full" if full else "windows", "engine": "jit-" + ref_arith, "steps": int(steps),
               "rows_checked": rows, "max_abs_diff": diff, "mismatches": int(mism)}
        if bitwise:
            out["ok"] = bool(mism == 0 and diff == 0.0)
        else:
            from ..models import reference as R
            bound = R.fast_error_bound(steps, npdt, t0_absmax)
            out["bound"] = bound
            out["ok"] = bool(diff <= bound)
        return out

    checks = reference_checks(arith, r, sterbenz)
    out = one(*checks[0])
    for ref_arith, bitwise in checks[1:]:
        out["vs_" + ref_arith] = one(ref_arith, bitwise)
    return out


def verify_decomposition(make_transport: Callable[[], object], *, rank: int, world: int, dtype: str, arith: str,
                         backend: str = "hip", device: Optional[int] = None, n: Optional[int] = None,
                         steps: int = 57, graph: bool = False, seed: int = 1234, r: float = 0.25) -> dict:
    """Run a small problem with a fresh transport of the chosen kind on every
    rank — n x n (default 256 * world + 5: uneven slabs), rough random data
    (sum - 4c is not exact, so the arithmetic is really checked), ``steps``
    steps through the autotuned split plans and measured schedule — gather it
    to rank 0 and compare it BITWISE with the NumPy golden model of the same
    arithmetic, with the run's FTCS coefficient ``r`` (the same update bits as
    the run: r = nu dt / delta^2 is sigma only up to rounding, which differs
    with n). Returns {"verified": bool, "n": n, "steps": steps,
    "max_abs_diff": float} (the verdict is broadcast: the same on every rank)."""
    import numpy as np
    import torch
    import torch.distributed as dist

    import heat2d
    from ..models import reference as R
    from ..models.heat2d import HeatSolver

    n = int(n or 256 * world + 5)
    npdt = np.float64 if dtype == "fp64" else np.float32
    import dataclasses
    prob = heat2d.make_problem(heat2d.InputDat(n=n, sigma=0.25, nu=0.05, dom_len=1.0, ntime=steps, soln=0, nfields=6),
                               "ghost", "uniform")
    prob = dataclasses.replace(prob, r=float(r))
    # values over two decades: sum - 4c then rounds (data within a factor of 2
    # would make it exact by Sterbenz, and exact / r = 1/4 / fma forms agree)
    T0 = (np.random.default_rng(seed).random((n, n)) * 10.0 + 0.01).astype(npdt)
    tr = make_transport()
    s = None
    try:
        s = HeatSolver(prob, dtype=dtype, backend=backend, transport=tr, device=device, autotune=1, graph=graph,
                       arith=arith)
        s.upload(T0[s.row0:s.row0 + s.nrows])
        s.prepare(steps)
        s.step(steps)
        s.synchronize()
        got = s.gather()
    finally:
        if s is not None:
            s.close()
        tr.close()
    # "fast" (scaled levels) is not the reference rounding, nor is the
    # contracted form at an r that is not a power of two (one rounding fewer):
    # checked against the exact golden within the stated bound
    # (models/reference.fast_error_bound); every other form bitwise
    bounded = arith == "fast" or (arith == "fma" and not _pow2(float(r)))
    bound = R.fast_error_bound(steps, npdt, float(np.max(np.abs(T0)))) if bounded else 0.0
    verdict = torch.zeros(2, dtype=torch.float64)
    if rank == 0:
        full = R.initial_field(prob, npdt)
        full[1:-1, 1:-1] = T0
        ref = R.owned(R.ftcs(prob, steps, dtype=npdt, T0=full, arith="jacobi" if arith == "jacobi" else "exact"))
        diff = float(np.max(np.abs(got.astype(np.float64) - ref.astype(np.float64))))
        ok = diff <= bound if bounded else np.array_equal(got, ref)
        verdict[0] = 1.0 if ok else 0.0
        verdict[1] = diff
    if world > 1:
        dist.broadcast(verdict, src=0)
    out = {"verified": bool(verdict[0].item() == 1.0), "n": n, "steps": steps,
           "max_abs_diff": float(verdict[1].item())}
    if bounded:
        out["bound"] = bound
    return out
