"""input.dat parsing (Python and C++ parsers agree), coefficients in the
reference's floating-point order, grid coordinates per convention, and the
slab decomposition (uneven remainder, no dropped rows)."""
import glob
import os

import numpy as np
import pytest

import heat2d
from heat2d.ops import _native as N
from heat2d.utils import config as cfg

REF = "/root/reference"

CASES = [
    ("32768 0.25 0.05 1.0 25000 0", (32768, 0.25, 0.05, 1.0, 25000, 0, 6)),
    ("1024 0.25 0.05 2.0 30", (1024, 0.25, 0.05, 2.0, 30, 0, 5)),
    ("100,0.25,0.05,2.0,10,1", (100, 0.25, 0.05, 2.0, 10, 1, 6)),
    ("100 0.25d0 5.0D-2 2.0 10 1\n", (100, 0.25, 0.05, 2.0, 10, 1, 6)),
    ("  64\n 0.25\n 0.05\n 1.0\n 7 / trailing comment", (64, 0.25, 0.05, 1.0, 7, 0, 5)),
    ("50 2*0.25 1.0 3", (50, 0.25, 0.25, 1.0, 3, 0, 5)),
]


@pytest.mark.parametrize("text,want", CASES)
def test_parse_python(text, want):
    inp = cfg.parse_input_text(text)
    assert (inp.n, inp.sigma, inp.nu, inp.dom_len, inp.ntime, inp.soln, inp.nfields) == want


@pytest.mark.parametrize("text,want", CASES)
def test_parse_cpp_matches_python(native, text, want):
    d = N.parse_input_native(text)
    assert (d["n"], d["sigma"], d["nu"], d["dom_len"], d["ntime"], d["soln"], d["nfields"]) == want


@pytest.mark.parametrize("bad", ["10 0.25", "2 0.25 0.05 1.0 3", "10 0.25 -1 1.0 3", "x 0.25 0.05 1.0 3"])
def test_parse_errors(native, bad):
    with pytest.raises(ValueError):
        cfg.parse_input_text(bad)
    with pytest.raises(N.NativeError):
        N.parse_input_native(bad)


def test_reference_input_files_parse(native):
    files = sorted(glob.glob(os.path.join(REF, "**", "input*.dat"), recursive=True))
    if not files:
        pytest.skip("reference tree not mounted")
    for f in files:
        text = open(f).read()
        a = cfg.parse_input_text(text)
        b = N.parse_input_native(text)
        assert a.n == b["n"] and a.ntime == b["ntime"] and a.nfields == b["nfields"], f


def test_coefficients_reference_order():
    delta, dt, r = cfg.coefficients(100, 0.25, 0.05, 2.0)
    assert delta == 2.0 / 99.0
    assert dt == (0.25 * (delta * delta)) / 0.05
    assert r == (0.05 * dt) / (delta * delta)
    assert abs(r - 0.25) < 1e-15  # r == sigma up to rounding (nu and L cancel)


def test_coordinates():
    d = 2.0 / 9
    g = cfg.coordinates(10, 2.0, d, cfg.GHOST)
    assert len(g) == 12 and g[0] == -d and g[1] == 0.0 and g[-1] == 10 * d
    inc = cfg.coordinates(10, 2.0, d, cfg.INCLUSIVE)
    assert len(inc) == 10 and inc[0] == 0.0 and inc[-1] == 2.0
    acc = 0.0
    for i in range(1, 9):
        acc += d
        assert inc[i] == acc  # cumulative, as fortran/serial/heat.f90:34


@pytest.mark.parametrize("n,P", [(32768, 8), (100, 3), (7, 7), (1000, 6), (17, 4)])
def test_decompose_uneven(native, n, P):
    rows = [N.decompose(n, P, r) for r in range(P)]
    assert sum(nr for _, nr in rows) == n  # the reference drops n mod P (fortran/hip/heat.F90:147)
    assert rows[0][0] == 0
    for (a0, an), (b0, _) in zip(rows, rows[1:]):
        assert b0 == a0 + an
    sizes = [nr for _, nr in rows]
    assert max(sizes) - min(sizes) <= 1


@pytest.mark.parametrize("n,P,shift", [(32768, 8, 235), (32768, 4, 215), (100, 3, 5), (1003, 7, 40), (100, 4, 99),
                                       (64, 2, 10), (17, 5, 3)])
def test_decompose_edge_shift(native, n, P, shift):
    """decompose(n, P, r, edge_shift): the two edge slabs give e = min(shift,
    (n // P) // 4) rows each to the P - 2 middle ones (the first 2e mod (P - 2)
    of them one more); contiguous, all n rows; below 3 ranks uniform."""
    rows = [N.decompose(n, P, r, shift) for r in range(P)]
    uni = [N.decompose(n, P, r)[1] for r in range(P)]
    assert sum(nr for _, nr in rows) == n and rows[0][0] == 0
    for (a0, an), (b0, _) in zip(rows, rows[1:]):
        assert b0 == a0 + an
    e = min(shift, (n // P) // 4) if P >= 3 else 0
    sizes = [nr for _, nr in rows]
    assert sizes[0] == uni[0] - e and sizes[-1] == uni[-1] - e
    mid = [s - u for s, u in zip(sizes[1:-1], uni[1:-1])]
    assert sum(mid) == 2 * e and (not mid or max(mid) - min(mid) <= 1)
    assert N.decompose(n, P, 0, 0) == N.decompose(n, P, 0)


def test_problem_conventions():
    inp = cfg.parse_input_text("100 0.25 0.05 2.0 10")
    g = heat2d.make_problem(inp, "ghost", "uniform")
    i = heat2d.make_problem(inp, "inclusive", "hat")
    assert g.n_owned == 100 and len(g.x) == 102
    assert i.n_owned == 98 and len(i.x) == 100
    py = cfg.make_ic("python-hat", 2.0, np.zeros(31))
    assert (py.i0, py.i1) == (7, 16)
    pc = cfg.make_ic("pycuda-hat", 2.0, np.zeros(4096))
    assert pc.i0 >= pc.i1  # python/cuda/cuda.py:53 slices an empty range
