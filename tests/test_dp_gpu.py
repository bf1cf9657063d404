"""GPU, 2 ranks sharing cuda:0 over gloo: row data parallelism (parallel.DataParallel, the
north_star's user-batch DP) equals ONE training step per global 2B-row batch -- the oracle replays
the concatenated batches of both ranks with the device dropout masks read back from each rank
(each rank draws its own Philox stream: the rank is mixed into the stream id) -- for the sharded
mode (reduce-scatter, 1/G optimizer, all-gather; fp32 or bf16 gradients) and the all-reduce mode,
on the row-gather path (k = 1) and the dense GEMM path (causal concat, k = 2).  The replicas must
stay bit-identical.  Tolerances: fp32 1e-5 (loss relative, every weight max-abs); bf16 gradients:
every weight inside its Adagrad envelope for gradients rounded to 8 bits (tests/parity.py)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from parity import CHAIN_ROUNDINGS, FP32_ABS, dataset, dense

B, H, STEPS, WORLD = 128, 64, 2, 2     # 700 train rows: 5 batches of 128, 2 per global step


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, mode, gdt, causal, cd):
    try:
        _work(rank, world, port, q, mode, gdt, causal, cd)
    except BaseException:                  # surface the failure in the parent instead of a hang
        import traceback
        q.put(("error", rank, traceback.format_exc()))
        q.close()
        q.join_thread()                    # flush the message before the hard exit
        os._exit(1)


def _log(rank, msg):
    if os.environ.get("OCF_TEST_DEBUG"):
        d = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "dbg_dp_rank%d.log" % rank), "a") as f:
            f.write(msg + "\n")


def _work(rank, world, port, q, mode, gdt, causal, cd):
    _log(rank, "start %s %s %s" % (mode, gdt, causal))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    import torch
    import torch.distributed as dist
    from omnidirectional_collaborative_filtering_amd.data_reader import data_reader
    from omnidirectional_collaborative_filtering_amd.model import omni_model
    from omnidirectional_collaborative_filtering_amd.optimizers import Adagrad
    dist.init_process_group("gloo", init_method="env://")
    _log(rank, "pg up")
    torch.cuda.set_device(0)
    data = dataset()
    np.random.seed(77)
    rd = data_reader(data.num_cols, data.train.n_rows, dataset=data, eval_mode="fixed_split")
    # different seeds per rank: the broadcast must make rank 0's weights everyone's
    om = omni_model(1, H, data.num_cols, B, dense_activation="sigmoid", use_causal_info=causal,
                    dropout_probability=0.2, compute_dtype=cd, seed=11 + rank)
    m = om.model
    m.compile(Adagrad(lr=0.005, epsilon=1e-8), "mean_squared_error")
    _log(rank, "model built")
    m.enable_data_parallel(rank, world, mode=mode, grad_dtype=gdt)
    _log(rank, "dp enabled")
    w0 = m.get_weights()
    aux = "causal" if causal else None
    gen = rd.data_gen(B, [1.0, 1.0], "train", True, aux, -1, pass_through_input_training=True)
    masks, losses = [], []
    for st in range(STEPS):
        _log(rank, "step %d" % st)
        h = m.fit_generator(gen, world, epochs=1, verbose=0)
        losses.append(h.history["loss"][0])
        masks.append(om.engine.mask[0][:B, :H].cpu().numpy().astype(np.float64))
    w = m.get_weights()                    # (ZeRO-1: gathers the fp32 masters first, on every rank)
    e = om.engine
    sh = [(t.cpu().numpy(), e.W[i].to(t.dtype).cpu().numpy()) for i, t in enumerate(e.Wsh) if t is not None]
    zero = sorted(m.dp.zero_layers) if m.dp is not None else []
    q.put((rank, w0, w, masks, losses, gen.rows_host[: STEPS * world], sh, zero))
    dist.barrier()
    dist.destroy_process_group()


def _run(mode, gdt, causal, cd="float32"):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, WORLD, port, q, mode, gdt, causal, cd)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = []
    while len(res) < WORLD:
        r = q.get(timeout=240)
        if r[0] == "error":
            for p in procs:
                p.kill()
            raise AssertionError("rank %d failed:\n%s" % (r[1], r[2]))
        res.append(r)
    res.sort(key=lambda z: z[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return res


def _oracle(res, causal, u=None, all_params=False):
    from oracle.model_oracle import AdagradOracle, OmniOracle
    data = dataset()
    N = data.num_cols
    w0 = res[0][1]
    k = 2 if causal else 1
    ora = OmniOracle([k * N, H, N], activation="sigmoid", dropout=0.2).set_params(w0[0::2], w0[1::2])
    opt = AdagradOracle(lr=0.005)
    rows = res[0][5]
    losses, env, rmax = [], None, None
    for s in range(STEPS):
        xs, ms, ts = [], [], []
        for r in range(WORLD):
            _, mo, x, t, mm = dense(data.train, rows[s * WORLD + r], N, -1.0)
            xs.append(np.concatenate([x, mm], 1) if causal else x)
            ms.append(mo)
            ts.append(t)
        x, mo, t = np.concatenate(xs), np.concatenate(ms), np.concatenate(ts)
        drop = [np.concatenate([res[r][3][s] for r in range(WORLD)])]
        loss, _, gW, gb = ora.loss_and_grads(x, mo, t, drop_masks=drop)
        grads = [g for pair in zip(gW, gb) for g in pair]
        if u is not None:
            GW, Gb = ora.grad_magnitudes(x, mo, t, drop_masks=drop, u=u)
            if env is None:
                env = [np.zeros_like(g) for g in grads]
                rmax = [np.zeros_like(g) for g in grads]
            for j, (g, G) in enumerate(zip(grads, [z for pair in zip(GW, Gb) for z in pair])):
                if j % 2 == 0 or all_params:   # bf16 gradients: weights only (biases stay fp32)
                    rmax[j] = np.maximum(rmax[j], CHAIN_ROUNDINGS * u * G / np.maximum(np.abs(g), 1e-30))
                env[j] += opt.lr * np.minimum(2.0, 3.0 * rmax[j])
        losses.append(loss)
        ora.set_flat(opt.step(ora.params(), grads))
    return losses, ora.params(), env


@pytest.mark.gpu
@pytest.mark.parametrize("mode,causal", [("sharded", False), ("sharded", True), ("allreduce", False)])
def test_dp_equals_global_batch_step(gpu, mode, causal):
    res = _run(mode, "float32", causal)
    for a, b in zip(res[0][2], res[1][2]):
        np.testing.assert_array_equal(a, b)            # replicas identical
    for a, b in zip(res[0][1], res[1][1]):
        np.testing.assert_array_equal(a, b)            # started from rank 0's weights on both
    assert not np.array_equal(res[0][3][0], res[1][3][0]), "ranks must draw different dropout masks"
    losses, want, _ = _oracle(res, causal)
    for lg, lo in zip(res[0][4], losses):
        assert abs(lg - lo) <= FP32_ABS * lo, (lg, lo)
    for j, (g, o) in enumerate(zip(res[0][2], want)):
        assert np.abs(g - o).max() <= FP32_ABS, (j, float(np.abs(g - o).max()))


@pytest.mark.gpu
def test_dp_bf16_gradients(gpu):
    res = _run("sharded", "bfloat16", False)
    for a, b in zip(res[0][2], res[1][2]):
        np.testing.assert_array_equal(a, b)
    losses, want, env = _oracle(res, False, u=2.0 ** -8)
    for lg, lo in zip(res[0][4], losses):
        assert abs(lg - lo) <= 1e-3 * lo, (lg, lo)
    for j, (g, o, e) in enumerate(zip(res[0][2], want, env)):
        err = np.abs(g - o)
        assert (err <= FP32_ABS + e).all(), (j, float(err.max()), int((err > FP32_ABS + e).sum()))


@pytest.mark.gpu
@pytest.mark.parametrize("gdt", ["float32", "bfloat16"])
def test_dp_f16_zero1_shadows(gpu, gdt):
    """f16 compute, sharded mode with ZeRO-1 (the first / last layers' fp32 masters and slots stay sharded;
    ocf_opt_step_ex writes the f16 shadow shard and only the shadows are all-gathered): the replicas' shadows
    are bit-identical, every shadow element is the RNE f16 rounding of its gathered fp32 master (what the
    per-step refresh produced), and the weights stay inside the oracle's f16 envelope"""
    res = _run("sharded", gdt, False, cd="float16")
    assert res[0][7] == [0, 1] and res[1][7] == [0, 1], "ZeRO-1 layers"
    for (sa, ma), (sb, mb) in zip(res[0][6], res[1][6]):
        np.testing.assert_array_equal(sa, sb)             # replicas' shadows identical
        np.testing.assert_array_equal(sa, ma)             # shadow == rounded master (rank 0)
        np.testing.assert_array_equal(sb, mb)
    for a, b in zip(res[0][2], res[1][2]):
        np.testing.assert_array_equal(a, b)
    losses, want, env = _oracle(res, False, u=2.0 ** -8 if gdt == "bfloat16" else 2.0 ** -11, all_params=True)
    for lg, lo in zip(res[0][4], losses):
        assert abs(lg - lo) <= 2e-3 * lo, (lg, lo)
    for j, (g, o, e) in enumerate(zip(res[0][2], want, env)):
        err = np.abs(g - o)
        assert (err <= FP32_ABS + e).all(), (j, float(err.max()), int((err > FP32_ABS + e).sum()))
