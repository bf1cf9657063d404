"""Diagnostic: the masked-MSE decoder GEMM as it runs inside the ML-20M step -- row-segment targets of
256 synthetic item rows (~750 ratings each) and, optionally, a cold Infinity Cache (a 1 GiB stream is
copied before every launch).  Times only the GEMM with HIP events (GPU)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from omnidirectional_collaborative_filtering_amd import _lib  # noqa: E402
from omnidirectional_collaborative_filtering_amd.dataset import RatingsCSR, synthetic_ratings  # noqa: E402
from tools.gemm_microbench import gemm  # noqa: E402

Bp, N, Hp = 256, 138493, 512
Np = 138496


def blocked(t):
    R, C = t.shape
    return t.view(R // 64, 64, C // 64, 64).permute(0, 2, 1, 3).contiguous()


def main():
    torch.manual_seed(0)
    r, c, v = synthetic_ratings(Bp, N, Bp * 750, half_stars=True, seed=1)
    rp = np.zeros(Bp + 1, np.int64)
    np.cumsum(np.bincount(r, minlength=Bp), out=rp[1:])
    csr = RatingsCSR(rp, c.astype(np.int32), v.astype(np.float32), list(range(Bp)))
    col_s, val_s, lidx_s, tptr = csr.tile_index(N)
    d = "cuda"
    T = {k: torch.as_tensor(x, device=d) for k, x in
         dict(col=col_s, val=val_s, lidx=lidx_s, tptr=tptr, rp=rp, rows=np.arange(Bp, dtype=np.int32),
              lboff=rp.copy(), flag=np.ones(len(col_s), np.uint8)).items()}
    h = (torch.randn(Bp, Hp, device=d) * 0.5).half()
    W = (torch.randn(Np, Hp, device=d) * 0.01).half()
    Wb = blocked(W)
    b = torch.zeros(Np, device=d)
    nt = Np // 128
    stats = torch.zeros(nt * 2 * 4, device=d)
    rsse = torch.zeros(nt * Bp, device=d)
    d_out = torch.zeros(Bp, Np, device=d).half()
    dbp = torch.zeros(2, Np, device=d)
    junk_a = torch.empty(256 << 20, device=d)
    junk_b = torch.empty_like(junk_a)
    op = _lib.OcfOptParams(0, 0, 0, 0, 0, 0, 1e-7)

    def mse(Wm, blk, targets=True, null=False):
        if null:
            return gemm(h, 0, Hp, Wm, _lib.DT_F16, 0, Hp, Bp, Np, Hp, _lib.EPI_SLAB, 1, order=1, out=dbp, ld_out=0,
                        split_stride=0, b_blocked=blk)
        seg = dict(t_rows=T["rows"], t_rp=T["rp"], t_tptr=T["tptr"], t_col=T["col"], t_val=T["val"], t_lidx=T["lidx"],
                   t_flag=T["flag"], t_lboff=T["lboff"], t_ntiles=tptr.shape[1] - 1, t_aux=-1.0)
        if not targets:
            seg["t_tptr"] = torch.zeros_like(T["tptr"])
        gemm(h, 0, Hp, Wm, _lib.DT_F16, 0, Hp, Bp, Np, Hp, _lib.EPI_MASKED_MSE, 1, order=1, bias=b, h_out=d_out,
             h_dtype=_lib.DT_F16, ld_out=Np, db_part=dbp, ld_db=Np, opt=op, stats_part=stats, row_sse_part=rsse,
             m_real=Bp, b_blocked=blk, **seg)

    def timed(fn, cold, n=10):
        ts = []
        for i in range(n + 2):
            if cold:
                junk_b.copy_(junk_a)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            fn()
            e.record()
            torch.cuda.synchronize()
            if i >= 2:
                ts.append(s.elapsed_time(e) * 1e3)
        return round(float(np.median(ts)), 1)

    res = {}
    for cold in (0, 1):
        res["mse_rowmajor_cold%d" % cold] = timed(lambda: mse(W, 0), cold)
        res["mse_blocked_cold%d" % cold] = timed(lambda: mse(Wb, 1), cold)
        res["mse_blocked_notargets_cold%d" % cold] = timed(lambda: mse(Wb, 1, targets=False), cold)
        res["null_blocked_cold%d" % cold] = timed(lambda: mse(Wb, 1, null=True), cold)
    print(json.dumps({"lib": os.path.basename(_lib.LIB_PATH), **res}))


if __name__ == "__main__":
    main()
