"""Diagnostic: one null-epilogue GEMM shape, repeated (for PMC collection)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from omnidirectional_collaborative_filtering_amd import _lib  # noqa: E402
from tools.gemm_microbench import gemm  # noqa: E402

M, K, Np = int(sys.argv[1]), int(sys.argv[2]), 138496
h = torch.randn(M, K, device="cuda").half()
W = (torch.randn(Np, K, device="cuda") * 0.01).half()
out = torch.zeros(Np, device="cuda")
for _ in range(5):
    gemm(h, 0, K, W, _lib.DT_F16, 0, K, M, Np, K, _lib.EPI_SLAB, 1, order=1, out=out, ld_out=0, split_stride=0)
torch.cuda.synchronize()
