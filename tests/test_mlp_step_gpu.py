"""GPU: the fused small-model step (ocf.h ocf_mlp_step: the whole Model.fit step of a small dense model in
one persistent launch) against the oracle replaying Keras 2.0.4's fit loop (train_jester.py:78-79: the
NumPy shuffle of the training rows, ceil(n / B) batches with the trailing partial one, size-weighted epoch
loss, val_loss over every held-out row).  Layer counts 1 / 2 / 3, sigmoid / tanh / relu, Adagrad / RMSprop /
Adam, k = 1 / 2 / 3 input blocks, exact fp32 (1e-5 on the epoch loss, val_loss and every weight) and the
16-bit operand modes (loss within 1e-2, every weight inside the per-element rounding envelope).  The
layer-wise dense path (Engine.fused_mlp = False) is run on the same data as a second witness."""
import numpy as np
import pytest

from parity import CHAIN_ROUNDINGS, UNIT_ROUNDOFF


def _data(n, N, k, seed=3):
    rng = np.random.RandomState(seed)
    obs = (rng.rand(n, N) < 0.5).astype(np.float32)
    vals = np.round(rng.uniform(-5, 5, (n, N)), 2).astype(np.float32) * obs
    drop = (rng.rand(n, N) < 0.5).astype(np.float32)
    x = [vals * drop] + [obs * drop, obs][: k - 1]
    return x, obs * (1 - drop), vals * (1 - drop)


def _opt(name):
    from omnidirectional_collaborative_filtering_amd import optimizers as O
    from oracle.model_oracle import AdagradOracle, AdamOracle, RMSpropOracle
    return {"adagrad": (lambda: O.Adagrad(lr=0.01, epsilon=1e-8), lambda: AdagradOracle(lr=0.01, epsilon=1e-8)),
            "rmsprop": (lambda: O.RMSprop(lr=0.001), lambda: RMSpropOracle(lr=0.001)),
            "adam": (lambda: O.Adam(lr=0.001), lambda: AdamOracle(lr=0.001))}[name]


def _fit(layers, H, act, opt, cd, k, n, N, B, fused, vs=0.1, epochs=1, wgs=0):
    from omnidirectional_collaborative_filtering_amd.model import omni_model
    x, om_, t = _data(n, N, k)
    m = omni_model(layers, H, N, B, dense_activation=act, use_causal_info=k >= 2, use_both_masks=k == 3,
                   compute_dtype=cd, seed=5)
    m.engine.fused_mlp = fused
    m.engine.mlp_wgs = wgs
    model = m.model
    model.compile(_opt(opt)[0](), "mean_squared_error")
    w0 = model.get_weights()
    np.random.seed(42)
    ins = x[:2] + [om_] + x[2:]               # model.py:89-97's input order: data, mask, output mask, second mask
    h = model.fit(ins, t, batch_size=B, validation_split=vs, epochs=epochs, shuffle=True)
    ran = m.engine._mlp_args is not None
    return h.history, w0, model.get_weights(), ran, (x, om_, t)


def _oracle(layers, H, act, opt, k, n, N, B, w0, data, u, vs=0.1):
    from oracle.model_oracle import OmniOracle
    x, om_, t = data
    ora = OmniOracle([k * N] + [H] * layers + [N], activation=act).set_params(w0[0::2], w0[1::2])
    o = _opt(opt)[1]()
    split = int(n * (1 - vs))
    np.random.seed(42)
    idx = np.arange(split)
    np.random.shuffle(idx)
    losses, sizes = [], []
    env = [np.zeros_like(p) for p in ora.params()]
    rmax = [np.zeros_like(p) for p in ora.params()]
    # the largest single update in units of lr (Adagrad 1, RMSprop 1 / sqrt(1 - rho), Adam ~ sqrt(10) x lr_t)
    step_max = {"adagrad": 1.0, "rmsprop": 1.0 / np.sqrt(0.1), "adam": 3.2}[opt]
    for s in range(-(-split // B)):
        sel = idx[s * B:(s + 1) * B]
        xin = np.concatenate([a[sel] for a in x], 1)
        loss, _, gW, gb = ora.loss_and_grads(xin, om_[sel], t[sel])
        grads = [g for pair in zip(gW, gb) for g in pair]
        GW, Gb = ora.grad_magnitudes(xin, om_[sel], t[sel], u=u)
        for j, (g, G) in enumerate(zip(grads, [z for pair in zip(GW, Gb) for z in pair])):
            rmax[j] = np.maximum(rmax[j], CHAIN_ROUNDINGS * u * G / np.maximum(np.abs(g), 1e-30))
            env[j] += o.lr * step_max * np.minimum(2.0, 3.0 * rmax[j])
        losses.append(loss)
        sizes.append(len(sel))
        ora.set_flat(o.step(ora.params(), grads))
    sse = 0.0
    for s0 in range(split, n, B):
        sel = np.arange(s0, min(n, s0 + B))
        y, _ = ora.forward(np.concatenate([a[sel] for a in x], 1), om_[sel])
        sse += float(((y - t[sel]) ** 2).sum())
    return float(np.dot(losses, sizes) / np.sum(sizes)), sse / ((n - split) * N), ora.params(), env


CASES = [(2, 256, "tanh", "rmsprop", "float32", 2), (1, 200, "sigmoid", "adagrad", "float32", 1),
         (3, 96, "relu", "adam", "float32", 3), (2, 256, "tanh", "rmsprop", "bfloat16", 2),
         (1, 200, "sigmoid", "adagrad", "float16", 1)]


@pytest.mark.gpu
@pytest.mark.parametrize("layers,H,act,opt,cd,k", CASES)
def test_fused_step_vs_oracle(gpu, layers, H, act, opt, cd, k):
    n, N, B = 700, 100, 128                   # 630 training rows: 4 batches of 128 + Keras' trailing 118
    hist, w0, w, ran, data = _fit(layers, H, act, opt, cd, k, n, N, B, fused=True)
    assert ran, "the fused small-model step (ocf_mlp_step) did not run"
    u = UNIT_ROUNDOFF[cd]
    loss_o, val_o, p, env = _oracle(layers, H, act, opt, k, n, N, B, w0, data, u)
    tol = 1e-5 if cd == "float32" else 1e-2
    assert abs(hist["loss"][0] - loss_o) <= tol * loss_o, (hist["loss"][0], loss_o)
    assert abs(hist["val_loss"][0] - val_o) <= tol * val_o, (hist["val_loss"][0], val_o)
    for i, (g, o, e) in enumerate(zip(w, p, env)):
        err = np.abs(g - o)
        assert (err <= 1e-5 + e).all(), (i, float(err.max()), int((err > 1e-5 + e).sum()))


@pytest.mark.gpu
def test_fused_step_matches_layerwise_path(gpu):
    """the fused step and the layer-wise dense path (split-K GEMMs, masked-MSE epilogue, fused optimizer
    epilogues) agree in exact fp32 on the same Model.fit epoch"""
    a = _fit(2, 256, "tanh", "rmsprop", "float32", 2, 700, 100, 128, fused=True)
    b = _fit(2, 256, "tanh", "rmsprop", "float32", 2, 700, 100, 128, fused=False)
    assert a[3] and not b[3]
    assert abs(a[0]["loss"][0] - b[0]["loss"][0]) <= 1e-5 * b[0]["loss"][0]
    assert abs(a[0]["val_loss"][0] - b[0]["val_loss"][0]) <= 1e-5 * b[0]["val_loss"][0]
    for x, y in zip(a[2], b[2]):
        assert np.abs(x - y).max() <= 2e-5, float(np.abs(x - y).max())


@pytest.mark.gpu
@pytest.mark.parametrize("wgs", [5, 128])
def test_fused_step_grid_sizes_match_layerwise(gpu, wgs):
    """the phases' hand-offs (write-through stores, L1-bypassing loads, the arrival counter) on a grid of 5
    workgroups (each walks many tiles) and of 128 (most idle in some phases): three epochs of 24 steps with
    Adam, 3 hidden layers, k = 3 equal the layer-wise path's in exact fp32 (a stale hand-off would not)"""
    args = (3, 160, "sigmoid", "adam", "float32", 3, 3000, 100, 112)
    a = _fit(*args, fused=True, epochs=3, wgs=wgs)
    b = _fit(*args, fused=False, epochs=3)
    assert a[3] and not b[3]
    for e in range(3):
        assert abs(a[0]["loss"][e] - b[0]["loss"][e]) <= 1e-5 * b[0]["loss"][e], e
        assert abs(a[0]["val_loss"][e] - b[0]["val_loss"][e]) <= 1e-5 * b[0]["val_loss"][e], e
    for x, y in zip(a[2], b[2]):
        assert np.abs(x - y).max() <= 5e-5, float(np.abs(x - y).max())


@pytest.mark.gpu
def test_mlp_barrier_gives_up_safely(gpu):
    """A grid barrier that gives up (injected: workgroup 0 never arrives at the first barrier, ocf_set_tuning
    "mlp_max_polls" < 0) poisons the barrier: every workgroup leaves without writing, so the step's weights,
    biases, slots and shadows are untouched; the next library call reports OCF_ASYNC_MLP_BARRIER once, the
    barrier words are zero again, and the next step runs normally on them"""
    import ctypes
    import torch
    from omnidirectional_collaborative_filtering_amd import _lib
    from omnidirectional_collaborative_filtering_amd.model import omni_model
    x, om_, t = _data(300, 100, 2)
    m = omni_model(2, 128, 100, 128, dense_activation="tanh", use_causal_info=True, compute_dtype="bfloat16", seed=5)
    eng = m.engine
    model = m.model
    model.compile(_opt("rmsprop")[0](), "mean_squared_error")
    model.fit(x[:2] + [om_], t, batch_size=128, epochs=1, shuffle=False)
    assert eng._mlp_args is not None, "the fused small-model step (ocf_mlp_step) did not run"
    torch.cuda.synchronize()

    def state():
        return [a.clone() for a in eng.W + eng.b + [s for sw, sb in eng.slots for s in sw + sb if s is not None]
                + [w for w in eng.Wsh if w is not None]]
    s0 = state()
    lib = _lib.load()
    prev = ctypes.c_int32()
    _lib.call("ocf_set_tuning", b"mlp_max_polls", -1, ctypes.byref(prev))
    try:
        eng._mlp_step()
        torch.cuda.synchronize()
        # (before any other library call: every entry point reports a pending error)
        assert lib.ocf_check_async() != 0 and b"ocf_mlp_step" in lib.ocf_last_error()
        assert lib.ocf_check_async() == 0          # reported once
    finally:
        lib.ocf_set_tuning(b"mlp_max_polls", prev.value, None)
    for a, b in zip(s0, state()):
        assert torch.equal(a, b)
    assert int(eng._mlp_bar.abs().sum()) == 0
    eng._mlp_step()                                # the same barrier words work again
    torch.cuda.synchronize()
    _lib.call("ocf_check_async")                   # (raises if that step's barriers gave up)
    assert not torch.equal(s0[0], eng.W[0]) and int(eng._mlp_bar.abs().sum()) == 0
