"""Multi-rank decisions are collective (VERDICT r2 task 1) and halo exchanges
move the depth the next cycle reads (task 2).

* Autotune / measured-schedule eligibility is a function of the global
  problem (the thinnest slab), so uneven slabs that straddle the 2^24-point
  threshold cannot split the ranks into some that all-reduce inside prepare()
  and some that do not (reference: every rank derives the same decomposition
  and loop, fortran/hip/heat.F90:142-158).
* prepare(n) all-reduces a hash of the cycle sequence and exchange depths and
  fails on EVERY rank, naming each rank's value, when they differ.
* Each cycle's exchange moves x = the next cycle's depth rows (the rows the
  next cycle reads; reference: the exchange moves exactly what the next step
  needs, fortran/hip/heat.F90:196-230), the last one the call's first depth;
  a deeper first cycle tops up once. Results stay bitwise.
"""
import json
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_distributed import golden, run_world  # noqa: E402

from heat2d.ops import _native as N  # noqa: E402


def test_autotune_eligibility_is_global(native):
    # 5793^2 on 2 ranks: slabs of 2897 and 2896 rows straddle 2^24 points
    # (2897 * 5793 = 16 782 321 >= 2^24 > 2896 * 5793 = 16 776 528). The
    # decision follows the thinnest slab, so both ranks skip autotuning.
    assert 2897 * 5793 >= 2 ** 24 > 2896 * 5793
    assert not N.autotune_slabs(5793, 5793, 2)
    assert N.autotune_slabs(5800, 5800, 2)  # 2900 * 5800 >= 2^24 on both slabs
    assert N.autotune_slabs(5793, 5793, 1)
    assert not N.autotune_slabs(1 << 16, 1 << 16, 1, 0) and N.autotune_slabs(8, 8, 3, 1)  # explicit off / on
    # every rank count: the answer depends on (n, P) only, never on a rank's own slab
    for n in (4097, 5793, 5800, 8191):
        for P in (2, 3, 4, 8):
            assert N.autotune_slabs(n, n, P) == ((n // P) * n >= 2 ** 24)


def expected_halo_rows(seqs, ghost0):
    """Rows one rank exchanges per side over consecutive step() calls: each
    cycle's exchange moves the next cycle's depth (the call's first depth after
    its last cycle), plus a top-up when a call starts deeper than the ghost rows."""
    total, ghost = 0, ghost0
    for seq in seqs:
        if seq[0] > ghost:
            total += seq[0]
        for i in range(len(seq)):
            x = seq[i + 1] if i + 1 < len(seq) else seq[0]
            total += x
            ghost = x
    return total


@pytest.mark.parametrize("world,tb,steps", [(2, 8, 23), (3, 6, 40), (2, 8, 20)])
def test_exchange_depth_follows_next_cycle_cpu(native, tmp_path, world, tb, steps):
    """gloo ranks of the CPU twin: step(steps//3) then step(rest) — the
    second call starts deeper than the first call's last exchange (a top-up) —
    bitwise the golden, and the halo rows moved are the next-cycle depths."""
    args = {"n": 61, "steps": steps, "tb": tb, "backend": "cpu", "random": True, "prepare": True,
            "plain_step": True}
    got, meta = run_world(tmp_path, world, args)
    assert np.array_equal(got, golden(args))
    seqs = meta["seqs"]
    first = steps // 3
    assert sum(seqs[0]) == first and sum(seqs[1]) == steps - first
    assert max(seqs[0] + seqs[1]) <= tb
    # after the upload's band-deep exchange: tb ghost rows; prepare(first) does not top up
    assert meta["halo_rows"] == expected_halo_rows(seqs, tb)
    assert meta["ghost_after"] == seqs[1][0]
    # fewer rows than exchanging the full band after every cycle
    assert meta["halo_rows"] <= tb * (len(seqs[0]) + len(seqs[1]) + 1)


def test_ranks_disagreeing_fail_loudly(native, tmp_path):
    """Two ranks configured with different temporal depths (so different cycle
    sequences and exchange depths): prepare() fails on BOTH ranks, naming each
    rank's value, instead of mismatching exchanges (a hang or wrong ghost rows)."""
    args = {"n": 61, "steps": 24, "tb": 8, "tb_rank": {"1": 5}, "backend": "cpu", "prepare": True}
    import subprocess  # noqa: F401
    with pytest.raises(FileNotFoundError):
        run_world(tmp_path, 2, args)  # no result.npy: both ranks stopped in prepare()
    for r in range(2):
        msg = (tmp_path / f"err{r}.txt").read_text()
        assert "ranks disagree" in msg and "rank 0:" in msg and "rank 1:" in msg, msg
        assert f"this is rank {r}" in msg


def _cli_json(tmp_path, n, ranks, steps, *extra):
    from test_cli import run_cli
    (tmp_path / "input.dat").write_text(f"{n} 0.25 0.05 1.0 {steps} 0\n")
    run_cli(tmp_path, "--gpus", str(ranks), "--transport", "peer", "--share-gpu", "--output", "npy", "--quiet",
            "--json", "r.json", *extra, timeout=600)
    return json.loads((tmp_path / "r.json").read_text())


def _golden_cli(tmp_path, ranks):
    import heat2d
    from heat2d.models import reference as R
    prob = heat2d.make_problem(heat2d.read_input(str(tmp_path / "input.dat")), "ghost", "uniform")
    got = np.concatenate([np.load(tmp_path / f"soln{r:05d}.npy") for r in range(ranks)])
    return got, R.owned(R.ftcs(prob))


@pytest.mark.gpu
@pytest.mark.parametrize("n", [5793, 5800])
def test_cli_two_ranks_straddling_autotune_threshold(native, gpu, tmp_path, n):
    """2 rank threads on one GPU (peer transport): 5793^2 puts the 2^24-point
    autotune threshold between the two slabs (the round-2 divergence: one rank
    all-reducing inside prepare(), the other not); 5800^2 autotunes both and
    runs prepare()'s collective measured schedule. Bitwise the golden, the same
    cycles on every rank, halos of the next cycle's depth."""
    r = _cli_json(tmp_path, n, 2, 40, "--check-every", "40")
    got, ref = _golden_cli(tmp_path, 2)
    assert np.array_equal(got, ref)
    assert r["cycles_per_rank"][0] == r["cycles_per_rank"][1], r
    assert sum(int(k) * c for k, c in r["cycles_per_rank"][0].items()) == 40
    assert r["halo_rows_per_rank"][0] == r["halo_rows_per_rank"][1] > 0
    # 5800^2: both slabs autotuned, prepare()'s collective measured schedule; 5793^2: neither
    assert r["schedule"] == ("measured" if n == 5800 else "balanced"), r


@pytest.mark.gpu
def test_cli_eight_ranks_measured_schedule(native, gpu, tmp_path):
    """8 rank threads on one GPU with autotuning forced on (each 525-row slab is
    far below 2^24 points, so `auto` would not tune): every rank autotunes its
    split plans and prepare()'s measured schedule all-reduces the per-depth
    cycle times across the 8 ranks; chunks of 25 steps with fused statistics.
    Bitwise the golden, identical cycles on every rank."""
    r = _cli_json(tmp_path, 4200, 8, 75, "--print-every", "25", "--check-every", "25", "--autotune", "on")
    got, ref = _golden_cli(tmp_path, 8)
    assert np.array_equal(got, ref)
    assert all(c == r["cycles_per_rank"][0] for c in r["cycles_per_rank"]), r["cycles_per_rank"]
    assert r["schedule"] == "measured"
    assert len(set(r["halo_rows_per_rank"][1:-1])) == 1
