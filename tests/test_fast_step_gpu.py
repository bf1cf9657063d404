"""GPU: fit_generator through the one-call step (Engine.fast_train_step -> ocf_train_step_rows) is
bit-identical to the general path (four library calls per step) -- weights, optimizer slots, the 16-bit
shadows and the logged history -- over two epochs with dropout, the reference's reciprocal split (NumPy's
MT19937 draws on the device) and Adagrad / Adam; and the one-call step really ran."""
import numpy as np
import pytest

from parity import dataset


def _run(fast, cd, opt, sparsity):
    import torch
    from omnidirectional_collaborative_filtering_amd import optimizers as O
    from omnidirectional_collaborative_filtering_amd.data_reader import data_reader
    from omnidirectional_collaborative_filtering_amd.model import omni_model
    data = dataset(rows=900, cols=700, nnz=40000)
    np.random.seed(21)
    rd = data_reader(data.num_cols, data.train.n_rows, dataset=data, eval_mode="fixed_split", rng="numpy")
    om = omni_model(1, 500, data.num_cols, 128, dense_activation="sigmoid", use_causal_info=False,
                    dropout_probability=0.2, compute_dtype=cd, seed=3)
    m = om.model
    m.compile(O.Adagrad(lr=0.005, epsilon=1e-8) if opt == "adagrad" else O.Adam(lr=0.001), "mean_squared_error",
              metrics=["mae", "accurate_RMSE"])
    eng = om.engine
    eng.fast_steps = fast
    hist = []
    issued = 0
    for ep in range(2):
        gen = rd.data_gen(128, sparsity, "train", True, None, -1,
                          pass_through_input_training=sparsity == [1.0, 1.0])
        steps = gen.num_batches - 1
        n0 = eng.step_count
        h = m.fit_generator(gen, steps, epochs=1, verbose=0)
        hist.append(h.history)
        issued += eng.step_count - n0
    torch.cuda.synchronize()
    st = [t.cpu().numpy().copy() for sw, sb in eng.slots for t in sw + sb if t is not None]
    sh = [t.float().cpu().numpy() for t in eng.Wsh if t is not None]
    ready = eng._plan is not None and eng._plan.get("ready")
    return hist, m.get_weights(), st, sh, ready, issued


@pytest.mark.gpu
@pytest.mark.parametrize("cd,opt,sparsity", [("float16", "adagrad", [1.0, 1.0]), ("float32", "adagrad", [0.3, 0.7]),
                                             ("bfloat16", "adam", [0.5, 0.9])])
def test_fast_step_bit_identical(gpu, cd, opt, sparsity):
    h_f, w_f, s_f, sh_f, ready, n = _run(True, cd, opt, sparsity)
    h_g, w_g, s_g, sh_g, ready_g, n_g = _run(False, cd, opt, sparsity)
    assert ready and not ready_g and n == n_g > 0
    assert h_f == h_g and all(np.isfinite(v).all() and v[0] > 0 for h in h_f for v in h.values())
    for a, b in zip(w_f + s_f + sh_f, w_g + s_g + sh_g):
        assert np.array_equal(a, b), float(np.abs(a - b).max())
