"""Diagnostic: where the time of the fused weight-gradient + Adagrad GEMM goes (GPU).

ML-20M dW shapes (M = N users, N = H hidden, K = B batch rows).  Times the fused kernel at K = 256 and at
K = 64 (one K-step: nearly pure epilogue stream), the standalone elementwise optimizer (ocf_opt_step,
reads a materialised gradient) and a plain copy, each with the HBM rate of its algorithmic bytes.
OCF_LIB_PATH selects a variant build of libocf.so (e.g. -DOCF_KLOOP_EXP=1, -DOCF_OPT_U=8)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from omnidirectional_collaborative_filtering_amd import _lib  # noqa: E402
from omnidirectional_collaborative_filtering_amd.engine import cur_stream  # noqa: E402
from tools.gemm_microbench import gemm, timeit  # noqa: E402

F16 = _lib.DT_F16


def main(Bp=256, Np=138496, Hp=512):
    torch.manual_seed(0)
    X = (torch.randn(Bp, Np, device="cuda") * (torch.rand(Bp, Np, device="cuda") < 0.05)).half()
    dh = torch.randn(Bp, Hp, device="cuda").half()
    P = torch.randn(Np, Hp, device="cuda") * 0.01
    A1 = torch.rand(Np, Hp, device="cuda")
    G = torch.randn(Np, Hp, device="cuda") * 1e-3
    C = torch.empty_like(P)
    Sh = torch.zeros(Np * Hp, device="cuda", dtype=torch.float16)
    ada = _lib.OcfOptParams(_lib.OPT_ADAGRAD, 0.005, 1e-8, 0, 0, 0, 1e-7)
    n = Np * Hp
    res = {}

    def fused(K):
        return lambda: gemm(X, 1, Np, dh, F16, 1, Hp, Np, Hp, K, _lib.EPI_OPTIM, p=P, s1=A1, ld_out=Hp, opt=ada,
                            p_shadow=Sh, shadow_blocked=1)
    for K in (256, 64):
        us = timeit(fused(K))
        res["fused_K%d_us" % K] = round(us, 1)
        res["fused_K%d_TBs" % K] = round(n * 18 / us / 1e6, 3)
    us = timeit(lambda: _lib.call("ocf_opt_step", P.data_ptr(), G.data_ptr(), A1.data_ptr(), None, n, ada,
                                  cur_stream()))
    res["elem_opt_us"] = round(us, 1)
    res["elem_opt_TBs"] = round(n * 20 / us / 1e6, 3)
    us = timeit(lambda: C.copy_(P))
    res["copy_us"] = round(us, 1)
    res["copy_TBs"] = round(n * 8 / us / 1e6, 3)
    print(json.dumps({"lib": os.path.basename(_lib.LIB_PATH), "shape": [Np, Hp], **res}), flush=True)


if __name__ == "__main__":
    import sys as _s
    if len(_s.argv) > 2:
        main(Np=int(_s.argv[1]), Hp=int(_s.argv[2]))
    else:
        main()
