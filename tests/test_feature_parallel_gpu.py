"""GPU, 2 ranks sharing cuda:0 over gloo: feature-parallel training (column-sharded W1 / W_out,
two [B,H] all-reduces per step) equals single-engine training on the full model -- with the
reciprocal input/output split (s < 1, NumPy RNG via full-row positions), the causal/dropout mask
concat (k = 2 input blocks) and dropout (same Philox stream on every rank).  With k = 1 the rank steps
after the first two run as four ocf_rank_step phase calls (Engine._fast_rank_step)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

ROWS, COLS, NNZ, B, H, STEPS = 900, 333, 18000, 128, 100, 6


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dataset():
    from omnidirectional_collaborative_filtering_amd.dataset import split_ratings, synthetic_ratings
    r, c, v = synthetic_ratings(ROWS, COLS, NNZ, half_stars=True, seed=5)
    return split_ratings(r, c, v, ROWS, COLS, rng=np.random.RandomState(5))


def _train(data, shard=None, comm=None, causal=True):
    from omnidirectional_collaborative_filtering_amd.data_reader import data_reader
    from omnidirectional_collaborative_filtering_amd.model import omni_model
    from omnidirectional_collaborative_filtering_amd.optimizers import Adagrad
    np.random.seed(77)
    rd = data_reader(data.num_cols, ROWS, dataset=data, eval_mode="fixed_split")
    om = omni_model(1, H, data.num_cols, B, dense_activation="sigmoid", use_causal_info=causal,
                    dropout_probability=0.2, compute_dtype="float32", seed=11, shard=shard, comm=comm)
    m = om.model
    m.compile(Adagrad(lr=0.005, epsilon=1e-8), "mean_squared_error", metrics=["accurate_MSE"])
    aux = "dropout" if causal else None
    gen = rd.data_gen(B, [0.5, 0.9], "train", True, aux, -1, pass_through_input_training=False)
    h = m.fit_generator(gen, STEPS, verbose=0)
    np.random.seed(99)
    tg = rd.data_gen(B, None, "test", True, aux, -1, return_target_count=True)
    sse, cnt = m.evaluate_sse(tg, rd.test_set_size // B)
    pl = om.engine._rplan
    one_call = bool(pl is not None and pl.get("ready"))    # the rank steps ran as ocf_rank_step phases
    return h.history["loss"][0], h.history["accurate_MSE"][0], float(np.sqrt(sse / cnt)), m.get_weights(), one_call


def _worker(rank, world, port, q, causal):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    import torch
    import torch.distributed as dist
    from omnidirectional_collaborative_filtering_amd.parallel import feature_shard_range, make_comm
    dist.init_process_group("gloo", init_method="env://")
    torch.cuda.set_device(0)
    data = _dataset()
    c0, c1 = feature_shard_range(data.num_cols, rank, world)
    out = _train(data.column_shard(c0, c1), shard=(c0, c1, data.num_cols), comm=make_comm(world), causal=causal)
    q.put((rank, c0, c1) + out)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("causal", [True, False])
def test_feature_parallel_equals_single_engine(gpu, causal):
    """causal=True: k = 2 input blocks (dense GEMM path); causal=False: k = 1 (row-gather path)"""
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, causal)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=600) for _ in range(world)], key=lambda z: z[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    data = _dataset()
    loss, amse, rmse, w, _ = _train(data, causal=causal)
    N = data.num_cols
    for rank, c0, c1, l_r, a_r, rmse_r, w_r, one_call in res:
        # the row-gather layout (k = 1) takes the one-call-per-phase rank step after two recorded steps
        assert one_call == (not causal)
        assert abs(l_r - loss) <= 1e-5 * loss, (l_r, loss)
        assert abs(a_r - amse) <= 1e-5 * amse
        assert abs(rmse_r - rmse) <= 1e-5, (rmse_r, rmse)
        rows = np.concatenate([np.arange(c0, c1), N + np.arange(c0, c1)]) if causal else np.arange(c0, c1)
        pairs = [(w_r[0], w[0][rows]), (w_r[1], w[1]), (w_r[2], w[2][:, c0:c1]), (w_r[3], w[3][c0:c1])]
        for got, want in pairs:
            assert got.shape == want.shape
            assert np.abs(got - want).max() <= 1e-5, float(np.abs(got - want).max())
