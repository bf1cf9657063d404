"""Diagnostic: max-abs weight / bias differences of the GPU training steps vs the fp64 oracle for
several configurations, and (16-bit modes) the worst error / Adagrad-envelope ratio -- the
statistics the parity tests' tolerances (tests/parity.py) are checked against.

    python tools/parity_probe.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from parity import FP32_ABS, run_parity  # noqa: E402

CASES = [
    dict(compute_dtype="float32", opt_name="adagrad", layers=1, act="sigmoid", dropout=0.2),
    dict(compute_dtype="float32", opt_name="adam", layers=2, act="tanh", dropout=0.2, H=96),
    dict(compute_dtype="float16", opt_name="adagrad", layers=1, act="sigmoid", dropout=0.2, envelope=True),
    dict(compute_dtype="float16", opt_name="adagrad", layers=1, act="sigmoid", dropout=0.2, gather=False,
         envelope=True),
    dict(compute_dtype="bfloat16", opt_name="adagrad", layers=1, act="sigmoid", dropout=0.2, envelope=True),
]


def main():
    for c in CASES:
        res = run_parity(**c)
        row = dict(case=c, loss_rel=abs(res.loss_g - res.loss_o) / abs(res.loss_o),
                   rmse_abs=abs(res.rmse_g - res.rmse_o), max_err=dict(res.max_param_err()))
        if res.env is not None:
            ratios = []
            for g, o, e in zip(res.w, res.ora.params(), res.env):
                err = np.abs(g - o)
                ratios.append(float((err / (FP32_ABS + e)).max()))
                row.setdefault("tight_frac", []).append(float((e < 1e-4).mean()))
            row["env_ratio"] = ratios
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
