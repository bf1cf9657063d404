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


def _blocked(t):
    """64x64-blocked copy of a [R][C] 16-bit array (ocf.h b_blocked layout)."""
    R, C = t.shape
    return t.view(R // 64, 64, C // 64, 64).permute(0, 2, 1, 3).contiguous()


def _slab_gemm(cd, a_col, b_col, Ad, Bd, M, N, K, splits, blocked):
    out = torch.zeros(splits, M, N, device="cuda")
    a = _lib.OcfGemmArgs()
    a.compute_dtype = cd
    a.A, a.a_dtype, a.a_col, a.lda = Ad.data_ptr(), cd, a_col, Ad.stride(0)
    a.B, a.b_dtype, a.b_col, a.ldb = Bd.data_ptr(), cd, b_col, (N if b_col else K)
    a.b_blocked = int(blocked)
    a.M, a.N, a.K, a.splits, a.epi = M, N, K, splits, _lib.EPI_SLAB
    a.out, a.ld_out, a.split_stride = out.data_ptr(), N, M * N
    _lib.call("ocf_gemm", a, cur_stream())
    torch.cuda.synchronize()
    return out.sum(0)


@pytest.mark.gpu
@pytest.mark.parametrize("cd", [_lib.DT_F16, _lib.DT_BF16])
@pytest.mark.parametrize("b_col", [0, 1])
def test_blocked_weight_operand_is_bit_identical(gpu, cd, b_col):
    """The 64x64-blocked B layout (the weight shadows) gives exactly the row-major product."""
    M, N, K, splits = 256, 384, 1024, 3
    g = torch.Generator().manual_seed(3)
    A = torch.randn(M, K, generator=g).to(TD[cd]).cuda()
    Bm = torch.randn(*(K, N) if b_col else (N, K), generator=g).to(TD[cd]).cuda()
    ref = _slab_gemm(cd, 0, b_col, A, Bm, M, N, K, splits, False)
    got = _slab_gemm(cd, 0, b_col, A, _blocked(Bm), M, N, K, splits, True)
    assert torch.equal(got, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("blocked", [0, 1])
def test_optimizer_writes_rounded_shadow(gpu, blocked):
    """EPI_OPTIM's shadow is the updated fp32 weights rounded to f16, in the requested layout."""
    M, N, K = 256, 384, 256     # W [M][N], K = batch
    g = torch.Generator().manual_seed(4)
    A = torch.randn(K, M, generator=g).half().cuda()      # delta^T as [K][M]
    Bm = torch.randn(K, N, generator=g).half().cuda()     # activations [K][N]
    P = (torch.randn(M, N, generator=g) * 0.05).cuda()
    S1 = torch.zeros(M, N, device="cuda")
    Sh = torch.zeros(M, N, device="cuda", dtype=torch.float16)
    a = _lib.OcfGemmArgs()
    a.compute_dtype = _lib.DT_F16
    a.A, a.a_dtype, a.a_col, a.lda = A.data_ptr(), _lib.DT_F16, 1, M
    a.B, a.b_dtype, a.b_col, a.ldb = Bm.data_ptr(), _lib.DT_F16, 1, N
    a.M, a.N, a.K, a.splits, a.epi = M, N, K, 1, _lib.EPI_OPTIM
    a.p, a.s1, a.ld_out = P.data_ptr(), S1.data_ptr(), N
    a.opt = _lib.OcfOptParams(_lib.OPT_ADAGRAD, 0.01, 1e-8, 0, 0, 0, 1e-3)
    a.p_shadow, a.shadow_blocked = Sh.data_ptr(), blocked
    _lib.call("ocf_gemm", a, cur_stream())
    torch.cuda.synchronize()
    want = P.half()
    assert torch.equal(Sh, _blocked(want).view(M, N) if blocked else want)
