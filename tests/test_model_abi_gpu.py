"""GPU: the model-level C ABI (ocf_ctx_create / ocf_forward / ocf_masked_mse / ocf_backward + ocf_opt_step,
driven by model_abi.ModelABI over ctypes) against the NumPy oracle of model.py / train.py on the reference's
dense batches (data_reader.py:354-361 arrays from the golden-pinned batch restatement).  Dropout masks are
read back through ocf_forward's masks_out and fed to the oracle.  Tolerances (tests/parity.py): exact fp32
1e-5 on the loss (relative), the per-row sums and every weight (max-abs); f16 operands inside the Adagrad
rounding envelope."""
import numpy as np
import pytest
import torch

from tests import parity

pytestmark = pytest.mark.gpu


def _run(dtype, opt_name, hidden, act, dropout, causal, steps=3, B=128, seed=3, max_batch=None):
    from omnidirectional_collaborative_filtering_amd.model_abi import ModelABI
    data = parity.dataset()
    N = data.num_cols
    k = 2 if causal else 1
    ora = parity.OmniOracle([k * N] + hidden + [N], activation=act, dropout=dropout or None).init(seed)
    m = ModelABI(N, hidden, max_batch or B, k_blocks=k, activation=act, dropout=dropout, compute_dtype=dtype, seed=11,
                 optimizer=parity.our_opt(opt_name))
    m.set_weights([x.astype(np.float32) for x in ora.params()])
    assert all(np.array_equal(a, b.astype(np.float32)) for a, b in zip(m.get_weights(), ora.params()))
    opt = parity.oracle_opt(opt_name)
    u = parity.UNIT_ROUNDOFF[dtype]
    env = [np.zeros_like(p) for p in ora.params()]
    rmax = [np.zeros_like(p) for p in ora.params()]
    rng = np.random.RandomState(seed)
    dev = torch.device("cuda")
    for step in range(steps):
        rows = rng.choice(data.train.n_rows, B, replace=False)
        m_in, m_out, x, t, m_miss = parity.dense(data.train, rows, N, -1.0)
        xs = [x, m_miss] if causal else [x]
        ins = [torch.as_tensor(a, dtype=torch.float32, device=dev).contiguous() for a in xs]
        mo = torch.as_tensor(m_out, dtype=torch.float32, device=dev).contiguous()
        tt = torch.as_tensor(t, dtype=torch.float32, device=dev).contiguous()
        masks = [torch.zeros(B, h, dtype=torch.uint8, device=dev) for h in hidden] if dropout else None
        stats = m.train_on_batch(ins, mo, tt, masks_out=masks).cpu().numpy()
        dm = [mk.cpu().numpy().astype(np.float64) for mk in masks] if dropout else None
        xin = np.concatenate(xs, 1)
        loss, y, gW, gb = ora.loss_and_grads(xin, m_out, t, drop_masks=dm)
        e = y - t
        assert abs(stats[3] - loss) <= 1e-5 * abs(loss) + (0 if dtype == "float32" else 2e-3 * abs(loss))
        if dtype == "float32":
            np.testing.assert_allclose(stats[4:4 + B], (e * e).sum(1), rtol=1e-5, atol=1e-6)
            np.testing.assert_allclose(stats[4 + B:4 + 2 * B], np.abs(e).sum(1), rtol=1e-5, atol=1e-6)
            np.testing.assert_array_equal(stats[4 + 2 * B:], np.count_nonzero(t + y, axis=1))
        grads = [g for pair in zip(gW, gb) for g in pair]
        if dtype != "float32":
            GW, Gb = ora.grad_magnitudes(xin, m_out, t, drop_masks=dm, u=u)
            for j, (g, G) in enumerate(zip(grads, [z for pair in zip(GW, Gb) for z in pair])):
                rmax[j] = np.maximum(rmax[j], parity.CHAIN_ROUNDINGS * u * G / np.maximum(np.abs(g), 1e-30))
                env[j] += opt.lr * np.minimum(2.0, 3.0 * rmax[j])
        ora.set_flat(opt.step(ora.params(), grads))
    torch.cuda.synchronize()
    for j, (wg, wo) in enumerate(zip(m.get_weights(), ora.params())):
        err = np.abs(wg.astype(np.float64) - wo)
        if dtype == "float32":
            assert err.max() <= parity.FP32_ABS, (j, err.max())
        else:
            assert np.all(err <= env[j] + 1e-6), (j, float((err - env[j]).max()))
    return m


@pytest.mark.parametrize("opt_name,hidden,act,dropout,causal", [
    ("adagrad", [100], "sigmoid", 0.2, False),          # train.py's I-AutoRec
    ("rmsprop", [64, 48], "tanh", 0.2, True),           # train_jester.py-like: 2 layers, causal concat
    ("adam", [130], "relu", 0.0, False),                # padded hidden width (130 -> 256), no dropout
])
def test_model_abi_fp32_vs_oracle(opt_name, hidden, act, dropout, causal):
    _run("float32", opt_name, hidden, act, dropout, causal)


def test_model_abi_batch_below_max():
    """B = 100 rows in a context sized for 256 (padded rows of the activations must not leak into any gradient)"""
    _run("float32", "adagrad", [100, 60], "tanh", 0.2, False, B=100, max_batch=256)


@pytest.mark.parametrize("dtype", ["float16", "bfloat16"])
def test_model_abi_16bit_envelope(dtype):
    _run(dtype, "adagrad", [100], "sigmoid", 0.2, False)


def test_model_abi_eval_forward_and_errors():
    from omnidirectional_collaborative_filtering_amd import _lib
    from omnidirectional_collaborative_filtering_amd.model_abi import ModelABI
    data = parity.dataset()
    N = data.num_cols
    ora = parity.OmniOracle([N, 50, N], activation="sigmoid").init(1)
    m = ModelABI(N, [50], 64, dropout=0.2, optimizer=parity.our_opt("adagrad"))
    m.set_weights([x.astype(np.float32) for x in ora.params()])
    rows = np.arange(40)
    _, m_out, x, t, _ = parity.dense(data.train, rows, N, -1.0)
    dev = torch.device("cuda")
    pred = m.forward([torch.as_tensor(x, dtype=torch.float32, device=dev)],
                     torch.as_tensor(m_out, dtype=torch.float32, device=dev), 40, False)
    y, _ = ora.forward(x, m_out)            # no dropout outside training
    assert np.abs(pred.cpu().numpy() - y).max() <= 1e-5
    # backward with another batch size than the forward's is refused; B above max_batch too
    with pytest.raises(_lib.OcfError):
        m.backward(torch.zeros(39, N, device=dev), 39)
    with pytest.raises(_lib.OcfError):
        m.forward([torch.zeros(65, N, device=dev)], None, 65, False)
