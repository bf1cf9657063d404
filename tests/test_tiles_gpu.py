"""GPU: the encoder over column tiles on the matrix cores (ocf_encoder_tiles, engine.enc_tiles) -- the first Dense
layer's X W1 (model.py:64-71) for batches whose weight rows carry many entries.

* the pre-activation X W1 it produces (via ocf_rows_reduce BIAS_ACT, bias 0) against an fp64 product of the
  batch's dense X (the reference's scatter, oracle/batch_oracle.py; duplicates last-write-wins) and the 16-bit
  weight shadow, and against the row-gather encoder: within 1e-5 of the terms' absolute sum (fp32
  accumulation in a different order), with padding rows and duplicate ratings;
* training through it against the oracle (tests/parity.py: f16 / bf16 envelope and quantile bars)."""
import numpy as np
import pytest
import torch

from tests.parity import assert_low_precision, run_parity, with_duplicates


def _model_and_batch(cd, rows, cols, nnz, B, tiles, dup, seed=3):
    from omnidirectional_collaborative_filtering_amd.data_reader import data_reader
    from omnidirectional_collaborative_filtering_amd.dataset import split_ratings, synthetic_ratings
    from omnidirectional_collaborative_filtering_amd.model import omni_model
    from omnidirectional_collaborative_filtering_amd.optimizers import Adagrad
    if dup:
        data = with_duplicates(rows, cols, nnz, seed=seed)
    else:
        r, c, v = synthetic_ratings(rows, cols, nnz, half_stars=True, seed=seed)
        data = split_ratings(r, c, v, rows, cols, rng=np.random.RandomState(seed))
    np.random.seed(seed)
    rd = data_reader(cols, rows, dataset=data, eval_mode="fixed_split")
    # (linear: the stored activation a = the pre-activation itself)
    om = omni_model(1, 500, cols, B, dense_activation="linear", use_causal_info=False, compute_dtype=cd, seed=9)
    om.engine.enc_tiles = tiles
    om.engine.fuse_enc_epilogue = False      # (the gather encoder's epilogue in its own launch: forward() alone)
    m = om.model
    m.compile(Adagrad(lr=0.005, epsilon=1e-8), "mean_squared_error")
    gen = rd.data_gen(B, [1.0, 1.0], "train", True, None, -1, pass_through_input_training=True)
    return data, om, gen


@pytest.mark.gpu
@pytest.mark.parametrize("cd,rows,cols,nnz,B,dup", [
    ("float16", 1500, 20000, 600000, 256, False),   # ~2 entries per live column, 157 tiles
    ("bfloat16", 1500, 9000, 400000, 100, True),    # padding rows (B = 100 of a 256-row group), duplicates
    ("float16", 3000, 16384, 600000, 512, False),   # two row groups (the XCD-shared W tiles)
    ("float16", 3000, 16384, 2000000, 256, False),  # buckets over 1,024 words (~4 entries per row per tile)
    ("float16", 3000, 16384, 2000000, 512, False),  # both
])
@pytest.mark.parametrize("pack", [1, 0])
def test_encoder_tiles_preactivation(gpu, cd, rows, cols, nnz, B, dup, pack):
    from omnidirectional_collaborative_filtering_amd import _lib
    from oracle.batch_oracle import scatter_rows_numpy
    prev = _lib.ctypes.c_int32()
    _lib.call("ocf_set_tuning", b"enc_tiles_pack", pack, _lib.ctypes.byref(prev))
    try:
        _preactivation(cd, rows, cols, nnz, B, dup, scatter_rows_numpy)
    finally:
        _lib.call("ocf_set_tuning", b"enc_tiles_pack", prev.value, None)


def _preactivation(cd, rows, cols, nnz, B, dup, scatter_rows_numpy):
    out = {}
    for tiles in (True, False):
        data, om, gen = _model_and_batch(cd, rows, cols, nnz, B, tiles, dup)
        e = om.engine
        gen._start()
        bi = 1
        om.model._load(None, gen, bi)
        e.forward(training=False)
        torch.cuda.synchronize()
        assert e._enc_tiles_used == tiles
        out[tiles] = e.a[0][:B, :500].double().cpu().numpy()
        if tiles:
            rws = gen.rows_host[bi]
            _, _, x, _, _ = scatter_rows_numpy(data.train.row_ptr, data.train.col, data.train.val, rws, cols, aux=-1.0)
            dt = torch.float16 if cd == "float16" else torch.bfloat16
            xq = torch.as_tensor(x).to(dt).double().numpy()           # the MFMA operand rounding of X
            W = e.Wsh[0][:cols, :500].double().cpu().numpy()
            ref = xq @ W
            scale = np.abs(xq) @ np.abs(W)
        del om, e, gen
    err_t = np.abs(out[True] - ref)
    bad = np.argwhere(err_t > 1e-5 * scale + 1e-6)
    assert len(bad) == 0, (len(bad), bad[:8].tolist(), float((err_t / (scale + 1e-30)).max()))
    err_g = np.abs(out[False] - ref)
    assert (err_g <= 1e-5 * scale + 1e-6).all()
    assert np.abs(out[True] - out[False]).max() <= 2e-5 * scale.max()


@pytest.mark.gpu
@pytest.mark.parametrize("cd", ["float16", "bfloat16"])
def test_encoder_tiles_train_parity(gpu, cd):
    """three Adagrad steps with dropout 0.2 through the tile encoder against the oracle (the envelope of
    tests/parity.py); the path really ran"""
    from omnidirectional_collaborative_filtering_amd.dataset import split_ratings, synthetic_ratings
    rows, cols, nnz = 1500, 20000, 600000
    r, c, v = synthetic_ratings(rows, cols, nnz, half_stars=True, seed=7)
    data = split_ratings(r, c, v, rows, cols, rng=np.random.RandomState(7))
    used = []

    def hook(om):
        om.engine.enc_tiles = True
        used.append(om.engine)
    res = run_parity(cd, "adagrad", 1, "sigmoid", steps=3, B=256, H=500, dropout=0.2, data=data, envelope=True,
                     sparse_oracle=True, eval_batches=2, model_hook=hook)
    assert used and used[0].enc_tiles_count == 3
    assert_low_precision(res, 2e-3 if cd == "float16" else 1e-2)
