"""Training-step parity: GPU engine (fit_generator fast path) vs the NumPy restatement of the
Keras 2.0.4 arithmetic (oracle/model_oracle.py), identical inputs and initial weights; the harness
and the stated tolerances are in tests/parity.py.

Bar (north_star): masked-RMSE within 1e-5 in the exact-fp32 mode; per-step loss within 1e-5
relative; every weight within 1e-5 (max-abs).  f16 / bf16 MFMA modes: loss / RMSE within 2e-3 /
1e-2 relative and every weight inside its Adagrad rounding envelope.  Dropout (p = 0.2, the
benchmarked configuration, train.py:40) is checked by feeding the device's Philox masks to the
oracle after every step."""
import pytest

from parity import assert_fp32, assert_low_precision, run_parity


@pytest.mark.gpu
@pytest.mark.parametrize("opt_name", ["adagrad", "rmsprop", "adam"])
def test_fp32_parity_one_hidden(gpu, opt_name):
    assert_fp32(run_parity("float32", opt_name, 1, "sigmoid"))


@pytest.mark.gpu
def test_fp32_parity_two_hidden_tanh_causal(gpu):
    assert_fp32(run_parity("float32", "rmsprop", 2, "tanh", aux_type="causal", causal=True, H=96))


@pytest.mark.gpu
@pytest.mark.parametrize("gather,sparse_dw", [(False, None), (True, False), (True, True)])
def test_fp32_parity_operand_paths(gpu, gather, sparse_dw):
    """The three first/last-layer operand paths of the generator step -- dense MFMA GEMMs
    (gather off), row gathers with dense weight-gradient operands (the feature-parallel global
    batch), row gathers with sparse-A weight gradients (short K) -- each meet the fp32 bar."""
    assert_fp32(run_parity("float32", "adagrad", 1, "sigmoid", gather=gather, sparse_dw=sparse_dw))


# ---- dropout on (the benchmarked configuration: train.py:40,52; model.py:72-73) -------------------
@pytest.mark.gpu
@pytest.mark.parametrize("gather,sparse_dw", [(False, None), (True, False), (True, True)])
def test_fp32_dropout_parity(gpu, gather, sparse_dw):
    """forward mask / keep scaling and the backward mask / keep * sigma' product -- in the fused
    decoder gather (gather=True) and in the dense split-K reductions (gather=False) -- against the
    oracle fed the device's masks"""
    res = run_parity("float32", "adagrad", 1, "sigmoid", dropout=0.2, gather=gather, sparse_dw=sparse_dw)
    assert_fp32(res)
    keep_frac = sum(float(m[0].mean()) for m in res.masks) / len(res.masks)
    assert 0.75 < keep_frac < 0.85, keep_frac            # Bernoulli(0.8) draws


@pytest.mark.gpu
@pytest.mark.parametrize("opt_name", ["rmsprop", "adam"])
def test_fp32_dropout_two_hidden(gpu, opt_name):
    """two hidden layers: the hidden->hidden GEMM epilogues (EPI_BIAS_ACT / EPI_GRAD_ACT) apply and
    differentiate their own layer's mask"""
    assert_fp32(run_parity("float32", opt_name, 2, "tanh", dropout=0.2, H=96))


@pytest.mark.gpu
@pytest.mark.parametrize("cd,tol", [("float16", 2e-3), ("bfloat16", 1e-2)])
@pytest.mark.parametrize("gather", [True, False])
def test_low_precision_dropout(gpu, cd, tol, gather):
    """the benchmarked arithmetic (16-bit MFMA operands, fp32 accumulation and master weights,
    dropout 0.2, Adagrad, row skipping on the gather path)"""
    res = run_parity(cd, "adagrad", 1, "sigmoid", dropout=0.2, gather=gather, envelope=True)
    assert_low_precision(res, tol)


@pytest.mark.gpu
@pytest.mark.parametrize("gather", [True, False])
def test_fp32_l2_regulariser(gpu, gather):
    """l2_weight_regulatization (model.py:66,82 W_regularizer=l2): the update sees g + 2 l2 W and the
    logged loss carries l2 * sum(W^2) of every kernel (Keras' total loss), both against the oracle;
    row skipping is off (a zero-gradient row still decays under l2)"""
    res = run_parity("float32", "adagrad", 1, "sigmoid", l2=1e-3, gather=gather)
    assert not res.om.engine._rtag_live
    assert_fp32(res)


