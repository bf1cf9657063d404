"""Diagnostic: decoder-forward GEMM (h[B][H] x W_out[N][H]^T) under different epilogues at the
ML-20M shape, to separate operand streaming from epilogue cost (GPU)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from omnidirectional_collaborative_filtering_amd import _lib  # noqa: E402
from tools.gemm_microbench import gemm, timeit  # noqa: E402

Bp, Np, Hp = 256, 138496, 512
F16, F32 = _lib.DT_F16, _lib.DT_F32


def main():
    torch.manual_seed(0)
    h = torch.randn(Bp, Hp, device="cuda").half()
    W = torch.randn(Np, Hp, device="cuda") * 0.01
    Wh = W.half()
    b = torch.zeros(Np, device="cuda")
    nt = Np // 128
    bk_ptr = torch.zeros(nt + 1, device="cuda", dtype=torch.int32)
    dummy_i = torch.zeros(16, device="cuda", dtype=torch.int32)
    dummy_f = torch.zeros(16, device="cuda")
    stats = torch.zeros(nt * 2 * 4, device="cuda")
    rsse = torch.zeros(nt * Bp, device="cuda")
    d_out = torch.zeros(Bp, Np, device="cuda").half()
    dbp = torch.zeros(2, Np, device="cuda")
    out = torch.zeros(Bp, Np, device="cuda")
    res = {}
    op = _lib.OcfOptParams(0, 0, 0, 0, 0, 0, 1e-7)

    def mse(dout, db, Wm=W, dt=F32, order=1):
        gemm(h, 0, Hp, Wm, dt, 0, Hp, Bp, Np, Hp, _lib.EPI_MASKED_MSE, 1, order=order, bias=b, bk_ptr=bk_ptr,
             bk_rc=dummy_i, bk_t=dummy_f, bk_m=dummy_f, h_out=dout, h_dtype=F16, ld_out=Np, db_part=db, ld_db=Np,
             opt=op, stats_part=stats, row_sse_part=rsse, m_real=Bp)
    res["mse_full"] = timeit(lambda: mse(d_out, dbp))
    res["mse_full_Wf16"] = timeit(lambda: mse(d_out, dbp, Wh, F16))
    res["mse_full_Wf16_order0"] = timeit(lambda: mse(d_out, dbp, Wh, F16, 0))
    res["slab_order1"] = timeit(lambda: gemm(h, 0, Hp, W, F32, 0, Hp, Bp, Np, Hp, _lib.EPI_SLAB, 1, order=1,
                                             out=d_out, ld_out=0, split_stride=0))
    res["slab_order1_Wf16"] = timeit(lambda: gemm(h, 0, Hp, Wh, F16, 0, Hp, Bp, Np, Hp, _lib.EPI_SLAB, 1, order=1,
                                                  out=d_out, ld_out=0, split_stride=0))
    # encoder shape: x[B][N] (f16) x W1[N][H] -> split-K slabs
    X = torch.randn(Bp, Np, device="cuda").half()
    S = 64
    slabs = torch.zeros(S * Bp * Hp, device="cuda")
    for o in (0, 1):
        res["enc_W32_order%d" % o] = timeit(lambda: gemm(X, 0, Np, W, F32, 1, Hp, Bp, Hp, Np, _lib.EPI_SLAB, S,
                                                         order=o, out=slabs, ld_out=Hp, split_stride=Bp * Hp))
        res["enc_W16_order%d" % o] = timeit(lambda: gemm(X, 0, Np, Wh, F16, 1, Hp, Bp, Hp, Np, _lib.EPI_SLAB, S,
                                                         order=o, out=slabs, ld_out=Hp, split_stride=Bp * Hp))
    res["mse_no_db"] = timeit(lambda: mse(d_out, None))
    res["mse_no_dout_no_db"] = timeit(lambda: mse(None, None))
    res["predict_f32out"] = timeit(lambda: gemm(h, 0, Hp, W, F32, 0, Hp, Bp, Np, Hp, _lib.EPI_PREDICT, 1, bias=b,
                                                out=out, ld_out=Np, m_real=Bp, n_real=Np))
    res["slab_order0"] = timeit(lambda: gemm(h, 0, Hp, W, F32, 0, Hp, Bp, Np, Hp, _lib.EPI_SLAB, 1,
                                             out=d_out, ld_out=0, split_stride=0))
    res["torch_read_W"] = timeit(lambda: W.sum())
    res["torch_copy_W"] = timeit(lambda: W.clone())
    print(json.dumps({"lib": os.path.basename(_lib.LIB_PATH), **{k: round(v, 1) for k, v in res.items()}}))


if __name__ == "__main__":
    main()
