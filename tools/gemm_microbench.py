"""Microbenchmark of ocf_gemm layout variants at the ML-20M shapes (diagnostic tool, GPU)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from omnidirectional_collaborative_filtering_amd import _lib  # noqa: E402
from omnidirectional_collaborative_filtering_amd.engine import cur_stream  # noqa: E402

Bp, Np, Hp = 256, 138752, 512
F16, F32 = _lib.DT_F16, _lib.DT_F32


def gemm(A, a_col, lda, Bm, b_dt, b_col, ldb, M, N, K, epi, splits=1, **kw):
    g = _lib.OcfGemmArgs()
    g.compute_dtype = F16
    g.A, g.a_dtype, g.a_col, g.lda = A.data_ptr(), F16, a_col, lda
    g.B, g.b_dtype, g.b_col, g.ldb = Bm.data_ptr(), b_dt, b_col, ldb
    g.M, g.N, g.K, g.splits, g.epi = M, N, K, splits, epi
    for k, v in kw.items():
        setattr(g, k, v.data_ptr() if torch.is_tensor(v) else v)
    _lib.call("ocf_gemm", g, cur_stream())


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


def main():
    torch.manual_seed(0)
    X = torch.randn(Bp, Np, device="cuda").half()          # [B][N]
    XT = X.t().contiguous()                                 # [N][B]
    W = torch.randn(Np, Hp, device="cuda") * 0.01           # [N][H] fp32
    dh = torch.randn(Bp, Hp, device="cuda").half()
    S = 64
    slabs = torch.zeros(S * Bp * Hp, device="cuda")
    P = torch.zeros(Np, Hp, device="cuda")
    A1 = torch.zeros(Np, Hp, device="cuda")
    res = {}
    op = _lib.OcfOptParams(_lib.OPT_ADAGRAD, 0.005, 1e-8, 0, 0, 0, 1e-7)
    res["enc_slab_A[B][N]"] = timeit(lambda: gemm(X, 0, Np, W, F32, 1, Hp, Bp, Hp, Np, _lib.EPI_SLAB, S, out=slabs,
                                                  ld_out=Hp, split_stride=Bp * Hp))
    res["enc_slab_A[N][B]"] = timeit(lambda: gemm(XT, 1, Bp, W, F32, 1, Hp, Bp, Hp, Np, _lib.EPI_SLAB, S, out=slabs,
                                                  ld_out=Hp, split_stride=Bp * Hp))
    for s in (16, 32, 128):
        res["enc_slab_A[N][B]_S%d" % s] = timeit(lambda: gemm(XT, 1, Bp, W, F32, 1, Hp, Bp, Hp, Np, _lib.EPI_SLAB, s,
                                                              out=slabs, ld_out=Hp, split_stride=Bp * Hp))
    res["optim_A[B][N]"] = timeit(lambda: gemm(X, 1, Np, dh, F16, 1, Hp, Np, Hp, Bp, _lib.EPI_OPTIM, p=P, s1=A1,
                                               ld_out=Hp, opt=op))
    res["optim_A[N][B]"] = timeit(lambda: gemm(XT, 0, Bp, dh, F16, 1, Hp, Np, Hp, Bp, _lib.EPI_OPTIM, p=P, s1=A1,
                                               ld_out=Hp, opt=op))
    copy_src = torch.empty(Np * Hp * 2, device="cuda")
    copy_dst = torch.empty_like(copy_src)
    res["torch_copy_568MB"] = timeit(lambda: copy_dst.copy_(copy_src))
    print(json.dumps({k: round(v, 1) for k, v in res.items()}))


if __name__ == "__main__":
    main()
