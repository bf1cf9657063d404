"""Diagnostic (GPU, run under rocprofv3 --kernel-trace): idle gap before the persistent dW kernel.
Alternates a small kernel with (a) the role-split optimizer kernel, (b) the generic OPTIM tile kernel,
at a small dW shape, so the trace shows the dispatch gap each one pays after its predecessor."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from omnidirectional_collaborative_filtering_amd import _lib  # noqa: E402
from omnidirectional_collaborative_filtering_amd.engine import cur_stream  # noqa: E402
from tools.gemm_microbench import gemm  # noqa: E402


def main():
    Bp, Np, Hp = 256, 128 * 256, 512
    F16 = _lib.DT_F16
    X = torch.randn(Bp, Np, device="cuda").half()
    dh = torch.randn(Bp, Hp, device="cuda").half()
    P = torch.zeros(Np, Hp, device="cuda")
    A1 = torch.zeros(Np, Hp, device="cuda")
    z = torch.zeros(1 << 16, device="cuda")
    ada = _lib.OcfOptParams(_lib.OPT_ADAGRAD, 0.005, 1e-8, 0, 0, 0, 1e-7)
    prev = _lib.I32(0)
    for ws in (1, 0, 1, 0):
        _lib.call("ocf_set_tuning", b"optim_ws", ws, prev)
        for _ in range(10):
            z.add_(1.0)
            gemm(X, 1, Np, dh, F16, 1, Hp, Np, Hp, Bp, _lib.EPI_OPTIM, p=P, s1=A1, ld_out=Hp, opt=ada)
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
