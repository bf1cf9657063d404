"""Diagnostic: null-epilogue GEMM time vs K and M at N = 138,496 (f16 weights stored [N][K]), to split
per-tile fixed cost from per-K-step cost (GPU)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from omnidirectional_collaborative_filtering_amd import _lib  # noqa: E402
from tools.gemm_microbench import gemm, timeit  # noqa: E402

Np = 138496
F16 = _lib.DT_F16


def main():
    res = {}
    out = torch.zeros(Np, device="cuda")
    for M in (128, 256, 512):
        for K in (256, 512, 1024, 2048):
            h = torch.randn(M, K, device="cuda").half()
            W = (torch.randn(Np, K, device="cuda") * 0.01).half()
            us = timeit(lambda: gemm(h, 0, K, W, F16, 0, K, M, Np, K, _lib.EPI_SLAB, 1, order=1, out=out, ld_out=0,
                                     split_stride=0))
            res["M%d_K%d" % (M, K)] = round(us, 1)
            res["M%d_K%d_TBs" % (M, K)] = round(Np * K * 2 / us / 1e6, 2)
            del h, W
    print(json.dumps({"lib": os.path.basename(_lib.LIB_PATH), **res}))


if __name__ == "__main__":
    main()
