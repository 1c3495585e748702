"""Raw kernel ops on torch tensors: layout views, init, temporal-blocked step,
stats, pack/unpack — and NaN guard bands: every element the kernel must not
write is pre-filled with NaN and checked afterwards (catches the out-of-bounds
class of bugs the reference's CUDA kernels have)."""
import numpy as np
import pytest
import torch

import heat2d
from heat2d.models import reference as R
from heat2d.ops import kernels as K


def problem(n, steps=0, conv="ghost", ic="uniform"):
    return heat2d.make_problem(heat2d.InputDat(n=n, sigma=0.25, nu=0.05, dom_len=2.0, ntime=steps), conv, ic)


def golden_rows(p, k, dtype):
    return R.owned(R.ftcs(p, k, dtype=dtype))


def run_guard(device, dtype, n, k, rows, row0=0, nrows=None, tile_rows=0):
    """A slab [row0, row0+nrows) of an n x n problem: step rows `rows` by k, check
    against the golden and that nothing outside rows x owned-cols was written."""
    tdt = torch.float64 if dtype == np.float64 else torch.float32
    p = problem(n, 0, "inclusive", "hat")
    m = p.n_owned
    nrows = m if nrows is None else nrows
    L = K.make_layout(nrows, m, halo=16, row0=row0, nrows_global=m)
    src = K.empty_field(L, tdt, device)
    K.init_field(src, L, p.ic, p.x)
    dst = torch.full_like(src, float("nan"))
    K.tb_step(src, dst, L, k, p.r, rows=rows, tile_rows=tile_rows)
    if device == "cuda":
        torch.cuda.synchronize()
    ref = golden_rows(p, k, dtype)[row0:row0 + nrows]
    got = K.owned(dst, L).cpu().numpy()
    rb, re = rows
    assert np.array_equal(got[rb:re], ref[rb:re])
    v = K.view2d(dst, L).cpu().numpy().copy()
    sv = K.view2d(src, L).cpu().numpy()
    v[L.halo + rb:L.halo + re, L.cpad:L.cpad + L.ncols] = np.nan
    # The only writes allowed outside the output rectangle: the HIP kernel's
    # last 16-B vector of a row may cover the right Dirichlet column / pad of
    # the SAME output rows, written back with src's (pinned) values.
    rr, cc = np.nonzero(~np.isnan(v))
    assert ((rr >= L.halo + rb) & (rr < L.halo + re)).all(), "kernel wrote outside its output rows"
    assert (cc >= L.cpad + L.ncols).all(), "kernel wrote left of / inside the owned columns"
    assert (cc < L.cpad + L.ncols + 8).all(), "kernel wrote beyond one vector of right pad"
    assert np.array_equal(v[rr, cc], sv[rr, cc]), "frame / pad write changed a value"


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("k", [1, 4, 9])
def test_guard_cpu(native, dtype, k):
    run_guard("cpu", dtype, 70, k, (0, 68))
    run_guard("cpu", dtype, 70, k, (10, 30), row0=20, nrows=30)


def test_layout_views(native):
    L = K.make_layout(10, 13, halo=4)
    f = torch.arange(L.elems(), dtype=torch.float64)
    assert K.view2d(f, L).shape == (L.rows_alloc(), L.pitch)
    assert K.owned(f, L).shape == (10, 13)
    assert L.pitch % 64 == 0 and L.cpad >= 16
    assert K.owned(f, L)[0, 0].item() == L.offset(0, 0)


def test_pack_unpack_cpu(native):
    L = K.make_layout(12, 9, halo=4)
    f = torch.randn(L.elems(), dtype=torch.float64)
    buf = K.pack_rows(f, L, 2, 3)
    assert torch.equal(buf.view(3, 9), K.owned(f, L)[2:5])
    g = torch.zeros_like(f)
    K.unpack_rows(g, L, -2, 3, buf)
    assert torch.equal(K.view2d(g, L)[2:5, L.cpad:L.cpad + 9], buf.view(3, 9))


def test_stats_cpu(native):
    p = problem(30)
    L = K.make_layout(30, 30, halo=4)
    f = K.empty_field(L, torch.float64, "cpu")
    K.init_field(f, L, p.ic, p.x)
    st = K.stats(f, L)
    assert st["sum"] == 2.0 * 900 and st["min"] == 2.0 and st["max"] == 2.0


def test_work_pieces():
    """Marches per rect: bands -> nb per strip; segments -> cut again at strip ends."""
    from heat2d.utils.metrics import work_pieces
    assert work_pieces(100, 3, 4) == 12
    assert work_pieces(100, 3, -1) == 3        # one segment over all strips
    assert work_pieces(100, 3, -3) == 3        # aligned with the strips
    assert work_pieces(100, 3, -2) == 4        # the middle strip cut once
    assert work_pieces(100, 3, -300) == 300    # one-row segments
    assert work_pieces(4096, 147, -1020) == 1020 + 146 - sum(
        1 for s in range(1, 147) if (s * 4096 * 1020) % (4096 * 147) == 0)


def test_plan_segments(native):
    from heat2d.ops import _native as N
    L = K.make_layout(4096, 32768, halo=16)
    pl = N.plan_tb(N.F32, L, 0, 4096, 16, -1000)
    assert pl.ntiles == -1000 and pl.nwaves == 1000
    pl = N.plan_tb(N.F32, L, 0, 10, 16, -10 ** 9)      # clamped to one strip row each
    assert pl.ntiles == -10 * pl.nstrips


def test_plan_fills_chip(native):
    from heat2d.ops import _native as N
    L = K.make_layout(32768, 32768, halo=16)
    pl = N.plan_tb(N.F64, L, 0, 32768, 8)
    assert pl.useful_w == pl.strip_w - 2 * 8
    assert pl.nstrips * pl.useful_w >= 32768
    assert pl.nwaves >= 1 and pl.ntiles >= 1


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("k,tile_rows", [(1, 0), (3, 0), (8, 0), (8, 5), (13, 0), (16, 0), (8, -3), (16, -77)])
def test_guard_gpu(native, gpu, dtype, k, tile_rows):
    run_guard("cuda", dtype, 203, k, (0, 201), tile_rows=tile_rows)
    run_guard("cuda", dtype, 203, k, (17, 61), row0=40, nrows=100, tile_rows=tile_rows)


@pytest.mark.gpu
def test_ops_gpu_matches_cpu(native, gpu):
    p = problem(150, 0, "ghost", "hotspot")
    L = K.make_layout(150, 150, halo=16)
    outs = []
    for dev in ("cpu", "cuda"):
        a = K.empty_field(L, torch.float64, dev)
        b = torch.zeros_like(a)
        K.init_field(a, L, p.ic, p.x)
        K.init_field(b, L, p.ic, p.x)
        for _ in range(5):
            K.tb_step(a, b, L, 7, p.r)
            a, b = b, a
        outs.append(K.owned(a, L).cpu())
    assert torch.equal(outs[0], outs[1])
    st = K.stats(outs[0].contiguous().view(-1), K.make_layout(150, 150, halo=0)) if False else None  # noqa
    buf = K.pack_rows(a, L, 0, 4)
    assert torch.equal(buf.view(4, 150).cpu(), K.owned(a, L)[:4].cpu())
    c = torch.empty_like(a)
    K.copy_(c, a)
    assert torch.equal(c, a)
