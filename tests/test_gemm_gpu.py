"""MFMA GEMM core (ocf_gemm) vs a torch fp32 reference of the same op, every layout / dtype."""
import numpy as np
import pytest
import torch

from omnidirectional_collaborative_filtering_amd import _lib
from omnidirectional_collaborative_filtering_amd.engine import cur_stream

TD = {_lib.DT_F32: torch.float32, _lib.DT_F16: torch.float16, _lib.DT_BF16: torch.bfloat16}
TOL = {_lib.DT_F32: 2e-5, _lib.DT_F16: 2e-3, _lib.DT_BF16: 2e-2}


def run_gemm(cd, a_col, b_col, b_dt, M, N, K, epi, splits=1, seed=0):
    g = torch.Generator().manual_seed(seed)
    A = torch.randn(*(K, M) if a_col else (M, K), generator=g)
    Bm = torch.randn(*(K, N) if b_col else (N, K), generator=g)
    Ad = A.to(TD[cd]).cuda()
    Bd = Bm.to(TD[b_dt]).cuda()
    A32 = Ad.float().cpu()
    B32 = Bd.to(TD[cd]).float().cpu()          # staged to the compute dtype in LDS
    Am = A32.t() if a_col else A32
    Bmm = B32 if b_col else B32.t()
    ref = Am.double() @ Bmm.double()
    out = torch.zeros(splits, M, N, device="cuda")
    a = _lib.OcfGemmArgs()
    a.compute_dtype = cd
    a.A, a.a_dtype, a.a_col, a.lda = Ad.data_ptr(), cd, a_col, Ad.stride(0)
    a.B, a.b_dtype, a.b_col, a.ldb = Bd.data_ptr(), b_dt, b_col, Bd.stride(0)
    a.M, a.N, a.K, a.splits, a.epi = M, N, K, splits, epi
    a.out, a.ld_out, a.split_stride = out.data_ptr(), N, M * N
    a.opt.gscale = 1.0
    _lib.call("ocf_gemm", a, cur_stream())
    torch.cuda.synchronize()
    got = out.sum(0).double().cpu()
    scale = (Am.abs().double() @ Bmm.abs().double()).clamp_min(1.0)
    return ((got - ref).abs() / scale).max().item()


CASES = [
    # a_col, b_col, b dtype (None = compute dtype), epilogue
    (0, 1, "f32", _lib.EPI_SLAB),
    (0, 0, "f32", _lib.EPI_SLAB),
    (1, 1, None, _lib.EPI_GRAD),
]


@pytest.mark.gpu
@pytest.mark.parametrize("cd", [_lib.DT_F32, _lib.DT_F16, _lib.DT_BF16])
@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("shape", [(128, 128, 64), (256, 384, 320), (128, 256, 1024)])
def test_gemm_layouts(gpu, cd, case, shape):
    a_col, b_col, bdt, epi = case
    M, N, K = shape
    if cd == _lib.DT_F32 and K % 32:
        pytest.skip("K")
    b_dt = _lib.DT_F32 if bdt == "f32" else cd
    err = run_gemm(cd, a_col, b_col, b_dt, M, N, K, epi)
    assert err < TOL[cd], err


@pytest.mark.gpu
@pytest.mark.parametrize("cd", [_lib.DT_F32, _lib.DT_F16])
def test_gemm_splitk(gpu, cd):
    err = run_gemm(cd, 0, 1, _lib.DT_F32, 256, 128, 2048, _lib.EPI_SLAB, splits=7)
    assert err < TOL[cd], err
    err = run_gemm(cd, 0, 0, _lib.DT_F32, 128, 256, 1024, _lib.EPI_SLAB, splits=3)
    assert err < TOL[cd], err
