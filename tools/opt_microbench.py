"""Diagnostic: fused weight-gradient + optimizer GEMM (EPI_OPTIM) at the ML-20M dW shapes (GPU).
OCF_LIB_PATH selects a variant build of libocf.so."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from omnidirectional_collaborative_filtering_amd import _lib  # noqa: E402
from tools.gemm_microbench import gemm, timeit  # noqa: E402

Bp, Np, Hp = 256, 138496, 512
F16 = _lib.DT_F16


def main():
    torch.manual_seed(0)
    X = torch.randn(Bp, Np, device="cuda").half()     # d_out / xin [B][N]
    dh = torch.randn(Bp, Hp, device="cuda").half()    # h / dh [B][H]
    P = torch.randn(Np, Hp, device="cuda") * 0.01
    A1 = torch.rand(Np, Hp, device="cuda")
    A2 = torch.rand(Np, Hp, device="cuda")
    Sh = torch.zeros(Np, Hp, device="cuda").half()
    res = {}
    ada = _lib.OcfOptParams(_lib.OPT_ADAGRAD, 0.005, 1e-8, 0, 0, 0, 1e-7)
    adam = _lib.OcfOptParams(_lib.OPT_ADAM, 0.001, 1e-8, 0.9, 0.999, 0, 1e-7)
    res["adagrad"] = timeit(lambda: gemm(X, 1, Np, dh, F16, 1, Hp, Np, Hp, Bp, _lib.EPI_OPTIM, p=P, s1=A1,
                                         ld_out=Hp, opt=ada))
    res["adagrad_shadow"] = timeit(lambda: gemm(X, 1, Np, dh, F16, 1, Hp, Np, Hp, Bp, _lib.EPI_OPTIM, p=P, s1=A1,
                                                ld_out=Hp, opt=ada, p_shadow=Sh))
    res["adam_shadow"] = timeit(lambda: gemm(X, 1, Np, dh, F16, 1, Hp, Np, Hp, Bp, _lib.EPI_OPTIM, p=P, s1=A1, s2=A2,
                                             ld_out=Hp, opt=adam, p_shadow=Sh))
    Z = torch.zeros(Np, Hp, device="cuda")
    Z1 = torch.zeros(Np, Hp, device="cuda")
    res["adagrad_zero_state"] = timeit(lambda: gemm(X, 1, Np, dh, F16, 1, Hp, Np, Hp, Bp, _lib.EPI_OPTIM, p=Z, s1=Z1,
                                                    ld_out=Hp, opt=ada))
    res["torch_copy_P"] = timeit(lambda: A2.copy_(P))
    print(json.dumps({"lib": os.path.basename(_lib.LIB_PATH), **{k: round(v, 1) for k, v in res.items()}}))


if __name__ == "__main__":
    main()
