"""Diagnostic: the row-gather encoder / decoder kernels at the ML-20M batch shape (256 item rows,
~750 entries each, N = 138,493, H = 512, f16 weights) with variants of the decoder outputs (GPU)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from omnidirectional_collaborative_filtering_amd import _lib  # noqa: E402
from omnidirectional_collaborative_filtering_amd.data_reader import BatchGenerator  # noqa: E402
from omnidirectional_collaborative_filtering_amd.dataset import synthetic_ratings  # noqa: E402
from omnidirectional_collaborative_filtering_amd.engine import cur_stream  # noqa: E402

Bp, N, Hp, Np = 256, 138493, 512, 138496


def main():
    r, c, v = synthetic_ratings(Bp, N, Bp * 750, half_stars=True, seed=1)
    lens = np.bincount(r, minlength=Bp)
    rp = np.zeros(Bp + 1, np.int64)
    np.cumsum(lens, out=rp[1:])
    d = "cuda"
    rows = np.arange(Bp).reshape(1, Bp)
    ch = BatchGenerator._chunk_tables(lens, rows, d)
    T = {k: torch.as_tensor(x, device=d) for k, x in dict(col=c.astype(np.int32), val=v.astype(np.float32), rp=rp,
                                                         rows=np.arange(Bp, dtype=np.int32), lboff=rp.copy(),
                                                         flag=np.ones(len(c), np.uint8)).items()}
    xval = T["val"].clone()
    W = (torch.randn(Np, Hp, device=d) * 0.01).half()
    h = (torch.randn(Bp, Hp, device=d) * 0.5).half()
    bias = torch.zeros(Np, device=d)
    nch = int(ch["cbase"][1])
    part = torch.zeros(nch * Hp, device=d)
    cst = torch.zeros(nch * 4, device=d)
    delta = torch.zeros(len(c), device=d)
    d_out = torch.zeros(Bp, Np, device=d).half()

    def args():
        g = _lib.OcfGatherArgs()
        g.rows, g.rp, g.col, g.val, g.lboff = (T[k].data_ptr() for k in ("rows", "rp", "col", "val", "lboff"))
        g.ch_row, g.ch_j0, g.ch_j1 = (ch[k].data_ptr() for k in ("ch_row", "ch_j0", "ch_j1"))
        g.n_chunks = nch
        g.W, g.w_dtype, g.ldw, g.H, g.part = W.data_ptr(), _lib.DT_F16, Hp, Hp, part.data_ptr()
        return g

    def enc():
        g = args()
        g.xval = xval.data_ptr()
        _lib.call("ocf_gather_encoder", g, cur_stream())

    def dec(with_delta, with_dout):
        g = args()
        g.flag, g.h, g.h_dtype, g.bias, g.aux = T["flag"].data_ptr(), h.data_ptr(), _lib.DT_F16, bias.data_ptr(), -1.0
        g.chunk_stats = cst.data_ptr()
        if with_delta:
            g.delta_e = delta.data_ptr()
        if with_dout:
            g.d_out, g.d_dtype, g.ld_d = d_out.data_ptr(), _lib.DT_F16, Np
        _lib.call("ocf_gather_decoder", g, cur_stream())

    def timed(fn, n=20):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(n):
            fn()
        e.record()
        torch.cuda.synchronize()
        return round(s.elapsed_time(e) / n * 1e3, 1)

    res = {"entries": int(len(c)), "chunks": nch,
           "enc": timed(enc), "dec_plain": timed(lambda: dec(False, False)),
           "dec_delta": timed(lambda: dec(True, False)), "dec_delta_dout": timed(lambda: dec(True, True)),
           "memset_dout": timed(lambda: d_out.zero_())}
    print(json.dumps({"lib": os.path.basename(_lib.LIB_PATH), **res}))


if __name__ == "__main__":
    main()
