"""ISA-level regression checks of the built gfx950 code objects (CPU only: the
code objects are read out of _native/libheat2d.so, no GPU needed).

* no temporal-blocked kernel spills to scratch;
* the interior kernels (priming skip) keep their occupancy: fp64 >= 3
  waves/SIMD to K = 12, 2 to K = 24 (ring 4 or 6), the packed fp32 one 3
  waves/SIMD to K = 11;
* the packed fp32 march stays compact (the element-wise one needed 209 VGPRs at
  K = 10 and AGPRs from K = 12, profiles/packed_fp32.md)."""
import os
import shutil
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import isa_report  # noqa: E402

from heat2d.ops import _native as N  # noqa: E402

pytestmark = pytest.mark.skipif(not (N.available() and os.path.exists(isa_report.READELF)),
                                reason="native library or llvm-readelf missing")


@pytest.fixture(scope="module")
def tb():
    ks = {}
    for k in isa_report.kernels(N.LIB_PATH):
        p = isa_report.tb_params(k["name"])
        if p:
            ks[p] = k
    # main/gen x 4 arith x (ring 4: fp32 K 1..24 + fp64 K 1..24; ring 6: fp32
    # K 1..16 + fp64 K 1..24), the fp32 general ring-8 kernels of single
    # launches (4 arith x K 1..16), plus the fused-statistics variants
    # (general, ring 4, 4 arith)
    assert sum(len(p) == 6 for p in ks) == 8 * (24 + 24) + 8 * (16 + 24) + 4 * 16, len(ks)
    assert sum(len(p) == 7 and p[6] == "stats" for p in ks) == 4 * (24 + 24), len(ks)
    assert len(ks) == 8 * (24 + 24) + 8 * (16 + 24) + 4 * 16 + 4 * (24 + 24), len(ks)
    return ks


def test_no_scratch(tb):
    spill = {p: k["scratch"] for p, k in tb.items() if k["scratch"]}
    assert not spill, spill


def test_occupancy_floors(tb):
    # fp64 interior kernels with the priming skip: >= 3 waves/SIMD up to K = 12
    for k in range(1, 13):
        for ar in (0, 1, 2, 3):
            assert tb[("fp64", 1, k, 4, True, ar)]["waves_per_simd"] >= 3, (k, ar)
    for k in range(1, 12):  # the packed fp32 interior kernel keeps >= 3 waves/SIMD up to K = 11
        for ar in (0, 1, 2, 3):
            assert tb[("fp32", 1, k, 4, True, ar)]["waves_per_simd"] >= 3, k


def test_deep_fp64_interior_two_waves(tb):
    """fp64 K = 17..24 exist for one-pass short runs, fp32 K = 17..24 for the
    HBM-bound big fp32 grids: the interior (MAIN) kernel
    must keep 2 waves/SIMD there, fp64 with ring 4 or ring 6 (the general one
    may drop to 1; with the priming skip fp64 K = 18..20 fit 2 waves with ring
    6 only, K = 22..24 with ring 4 only)."""
    for k in range(17, 25):
        for ar in (0, 1, 2, 3):
            assert max(tb[("fp64", 1, k, ring, True, ar)]["waves_per_simd"] for ring in (4, 6)) >= 2, (k, ar)
    assert not any(p[0] == "fp32" and p[2] > 24 for p in tb)
    for k in range(17, 25):  # fp32 K = 17..24: the interior kernel keeps 2 waves/SIMD at ring 4 (floor)
        for ar in (0, 1, 2, 3):
            assert tb[("fp32", 1, k, 4, True, ar)]["waves_per_simd"] >= 2, (k, ar)


def test_packed_fp32_compact(tb):
    assert tb[("fp32", 1, 10, 4, True, 1)]["vgpr"] <= 160
    assert all(tb[("fp32", 1, k, 4, True, 1)]["agpr"] == 0 for k in range(1, 17))
