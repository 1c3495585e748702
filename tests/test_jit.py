"""Run-time specialised kernel (hipRTC) — the reference's PyCUDA/Jinja2 JIT
program (python/cuda/cuda.py:58-89) re-done natively (csrc/runtime/jit.cpp).

CPU: the rendered source bakes the slab geometry and r (exactly, as a hex
float) and compiles for gfx950 with hipRTC (no GPU needed).
GPU: the JIT engine is bitwise identical to the NumPy golden and to the
temporal-blocked engine, on one rank and across ranks."""
import numpy as np
import pytest

import heat2d
from heat2d.models import reference as R
from heat2d.ops import _native as N
from heat2d.ops import jit


def test_render_bakes_constants(native):
    L = N.make_layout(100, 77, halo=4)
    src = jit.render(N.F64, L, 0.25)
    assert "#define NROWS 100L" in src and "#define NCOLS 77L" in src
    assert f"#define PITCH {L.pitch}L" in src and f"#define ORIGIN {L.offset(0, 0)}L" in src
    assert "#define R (0x1p-2)" in src and "typedef double real;" in src
    s32 = jit.render(N.F32, L, 0.1)
    assert "typedef float real;" in s32 and "#define R (0x1.99999ap-4f)" in s32  # float(0.1) exactly


@pytest.mark.parametrize("dt", [N.F32, N.F64])
def test_render_compiles_for_gfx950(native, dt):
    L = N.make_layout(1000, 513, halo=16)
    assert jit.compile_check(jit.render(dt, L, 0.2), "gfx950") > 1000


def test_compile_error_is_reported(native):
    with pytest.raises(RuntimeError, match="hiprtcCompileProgram"):
        jit.compile_check("this is not HIP", "gfx950")


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
def test_jit_engine_bitwise(gpu, native, dtype):
    from heat2d.models.heat2d import HeatSolver
    p = heat2d.make_problem(heat2d.InputDat(n=333, sigma=0.25, nu=0.05, dom_len=1.0, ntime=41), "ghost", "sine")
    npdt = np.float64 if dtype == "fp64" else np.float32
    T0 = R.owned(R.initial_field(p, npdt))
    outs = []
    for engine in ("jit", "tb"):
        s = HeatSolver(p, dtype=dtype, backend="hip", tb=8, device=0, engine=engine)
        s.upload(T0)
        s.step(p.ntime)
        outs.append(s.download())
        if engine == "jit":
            assert s.tb == 1
        s.close()
    ref = R.owned(R.ftcs(p, dtype=npdt))
    assert np.array_equal(outs[0], ref), np.abs(outs[0].astype(np.float64) - ref).max()
    assert np.array_equal(outs[0], outs[1])


@pytest.mark.gpu
def test_jit_op_on_tensors(gpu, native):
    import torch
    from heat2d.ops import kernels as K
    p = heat2d.make_problem(heat2d.InputDat(n=150, sigma=0.25, nu=0.05, dom_len=2.0, ntime=0), "inclusive", "hat")
    L = K.make_layout(p.n_owned, p.n_owned, halo=16)
    a = K.empty_field(L, torch.float64, "cuda")
    K.init_field(a, L, p.ic, p.x)
    b = a.clone()
    c = a.clone()
    st = jit.JitStencil(torch.float64, L, p.r)
    assert "#define NROWS" in st.source
    st.step(a, b)
    K.tb_step(a, c, L, 1, p.r)
    torch.cuda.synchronize()
    assert torch.equal(K.owned(b, L), K.owned(c, L))
    st.close()
