"""The persistent plan cache's on-disk format (csrc/runtime/plan_cache.cpp), on
CPU: a plan with every field set (lead order + dynamic queue flags, weighted
rects) and a schedule round-trip through the file; a later line of the same
key wins; entries of a plan kind no build can launch (fused cycles, unknown
flags) and torn lines are refused, not loaded. The GPU side — keys, semantic
refusal, re-validation — is covered by tests/test_bench_contract.py."""
import ctypes as C

import pytest

from heat2d.ops import _native as N

CTX = b"gfx950|cu256|fp64|ar2|4096x32768|p32896|h24|pos0|ccu0|sp8|x1|tr=rccl|env0123456789abcdef"


@pytest.fixture
def cache(native, tmp_path, monkeypatch):
    path = tmp_path / "plans.txt"
    monkeypatch.setenv("HEAT2D_PLAN_CACHE", str(path))
    N.call("heat2d_plan_cache_reload")
    if N.plan_cache_path() != str(path):
        pytest.skip("plan cache disabled in this build (no source hash)")
    yield path
    monkeypatch.setenv("HEAT2D_PLAN_CACHE", "off")
    N.call("heat2d_plan_cache_reload")


def rect(r0, r1, s0, s1, nb):
    return N.Rect(r0, r1, s0, s1, nb)


def sample_plan(k=20):
    p = N.SplitPlan()
    p.k, p.ring, p.valid, p.nedge = k, 6, 1, 2
    p.main = rect(20, 4076, 0, 373, 8)
    p.edge[0], p.edge[1] = rect(0, 20, 0, 373, 2), rect(4076, 4096, 0, 373, 2)
    p.main_waves, p.edge_waves, p.main_items, p.edge_items = 2040, 1492, 2996, 1492
    p.nrects, p.flags = 3, 2 | 4  # dynamic queue + lead order
    p.rects[0], p.rects[1], p.rects[2] = rect(20, 4076, 0, 1, 14), rect(20, 4076, 1, 372, 8), rect(20, 4076, 372, 373, 14)
    return p


def get(k, band):
    p, ms, found = N.SplitPlan(), C.c_float(), C.c_int32()
    N.call("heat2d_plan_cache_get", CTX, k, band, C.byref(p), C.byref(ms), C.byref(found))
    return (p, ms.value) if found.value else (None, None)


def fields(p):
    return {name: (list(map(tuple, ((r.r0, r.r1, r.s0, r.s1, r.nb) for r in getattr(p, name))))
                   if name in ("edge", "rects") else
                   ((p.main.r0, p.main.r1, p.main.s0, p.main.s1, p.main.nb) if name == "main" else getattr(p, name)))
            for name, _ in N.SplitPlan._fields_}


def test_plan_round_trip(cache):
    p = sample_plan()
    N.call("heat2d_plan_cache_put", CTX, 20, 20, C.byref(p), C.c_float(0.6418))
    N.call("heat2d_plan_cache_reload")  # from the file, not the in-memory map
    q, ms = get(20, 20)
    assert q is not None and abs(ms - 0.6418) < 1e-6
    assert fields(q) == fields(p)
    assert get(20, 21) == (None, None) and get(19, 20) == (None, None)
    assert cache.read_text().startswith("plan|")


def test_last_line_wins(cache):
    p = sample_plan()
    N.call("heat2d_plan_cache_put", CTX, 20, 20, C.byref(p), C.c_float(0.70))
    p.ring, p.flags = 4, 0
    N.call("heat2d_plan_cache_put", CTX, 20, 20, C.byref(p), C.c_float(0.65))
    N.call("heat2d_plan_cache_reload")
    q, ms = get(20, 20)
    assert q.ring == 4 and q.flags == 0 and abs(ms - 0.65) < 1e-6
    assert len(cache.read_text().splitlines()) == 2  # appended, not rewritten


@pytest.mark.parametrize("mutate", ["fused", "flags", "torn"])
def test_unloadable_entries_refused(cache, mutate):
    p = sample_plan()
    N.call("heat2d_plan_cache_put", CTX, 20, 20, C.byref(p), C.c_float(0.6))
    line = cache.read_text().splitlines()[0]
    key, val = line.split("\t")
    v = val.split()
    if mutate == "fused":  # round 3's fused-cycle plans (valid = 4) are no longer launchable
        v[2] = "4"
    elif mutate == "flags":
        v[-1] = "64"
    else:
        v = v[: len(v) // 2]
    cache.write_text(key + "\t" + " ".join(v) + "\n")
    N.call("heat2d_plan_cache_reload")
    assert get(20, 20) == (None, None)


def test_schedule_round_trip(cache):
    sched = (C.c_int32 * 25)(*([19] * 20 + [20] * 5))
    N.call("heat2d_plan_cache_put_schedule", CTX, 480, sched, 25)
    N.call("heat2d_plan_cache_reload")
    out, cnt = (C.c_int32 * 64)(), C.c_int64()
    N.call("heat2d_plan_cache_get_schedule", CTX, 480, out, 64, C.byref(cnt))
    assert cnt.value == 25 and list(out[:25]) == [19] * 20 + [20] * 5
    N.call("heat2d_plan_cache_get_schedule", CTX, 20, out, 64, C.byref(cnt))
    assert cnt.value == -1
