"""CPU, world_size 2 over gloo: the data-parallel step's algebra.  Each rank computes the (oracle)
gradient of its own B-row batch; parallel.grad_sync all-reduces ONE flat bucket; averaging gives
exactly the gradient of the concatenated 2B-row batch (Keras' MSE is a mean over rows), which is
what makes G-GPU data parallel training equal to one step on the global batch."""
import os
import socket
import types

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle.model_oracle import OmniOracle


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(seed=0, B=8, N=13, H=5):
    rng = np.random.RandomState(seed)
    x = rng.rand(2 * B, N) * (rng.rand(2 * B, N) < 0.4)
    m = -1.0 * (x != 0)
    t = x.copy()
    ora = OmniOracle([N, H, N], activation="sigmoid").init(3)
    ora.W = [w.astype(np.float64) for w in ora.W]
    return ora, x, m, t, B


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from omnidirectional_collaborative_filtering_amd.parallel import GradBucket, grad_sync, init_from_env, shard_batches
    r, w, _ = init_from_env(backend="gloo")
    ora, x, m, t, B = _data()
    sl = slice(rank * B, (rank + 1) * B)
    _, _, gW, gb = ora.loss_and_grads(x[sl], m[sl], t[sl])
    eng = types.SimpleNamespace(W=[torch.zeros(*wt.shape, dtype=torch.float64) for wt in ora.W],
                                b=[torch.zeros(*bt.shape, dtype=torch.float64) for bt in ora.b],
                                dev=torch.device("cpu"))
    bucket = GradBucket(eng, dtype=torch.float64)
    for v, g in zip(bucket.views, [g for pair in zip(gW, gb) for g in pair]):
        v.copy_(torch.as_tensor(g))
    grad_sync(bucket, w)
    avg = (bucket.flat / w).numpy()
    q.put((rank, avg, shard_batches(10, r, w)))
    dist.destroy_process_group()


def test_dp_average_equals_global_batch_gradient():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda z: z[0])
    ora, x, m, t, B = _data()
    _, _, gW, gb = ora.loss_and_grads(x, m, t)
    ref = np.concatenate([g.reshape(-1) for pair in zip(gW, gb) for g in pair])
    for _, avg, _ in res:
        np.testing.assert_allclose(avg, ref, rtol=1e-12, atol=1e-15)
    s0, s1 = res[0][2], res[1][2]
    assert set(s0).isdisjoint(s1) and sorted(s0 + s1) == list(range(10))


def _sharded_worker(rank, world, port, q, gdt):
    """ShardedSync on CPU tensors: each rank's oracle gradient of its own B rows -> reduce-scatter ->
    this rank's 1/G of a Keras Adagrad step (scale 1/G) -> all-gather.  Every rank must end with the
    parameters of ONE Adagrad step on the concatenated batch's gradient."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from omnidirectional_collaborative_filtering_amd.parallel import ShardedSync, init_from_env
    init_from_env(backend="gloo")
    ora, x, m, t, B = _data(N=16, H=8)
    sl = slice(rank * B, (rank + 1) * B)
    _, _, gW, gb = ora.loss_and_grads(x[sl], m[sl], t[sl])
    dt = {"float32": torch.float32, "bfloat16": torch.bfloat16}[gdt]
    params = [torch.as_tensor(p, dtype=torch.float32).clone() for p in ora.params()]
    grads = [torch.as_tensor(g).to(dt) for g in [g for pair in zip(gW, gb) for g in pair]]
    acc = [torch.zeros_like(p) for p in params]
    sync = ShardedSync(params, grads, rank, world)
    for j in range(len(params)):
        sync.start(j)

    def update(j, lo, hi, g):            # Keras Adagrad, lr 0.005, on the shard, gradient / world
        g = g / world
        a = acc[j].view(-1)[lo:hi]
        a += g * g
        params[j].view(-1)[lo:hi] -= 0.005 * g / (a.sqrt() + 1e-8)
    sync.finish(update)
    sync.gather_tensors(acc)
    q.put((rank, [p.numpy() for p in params], [a.numpy() for a in acc]))
    dist.destroy_process_group()


@pytest.mark.parametrize("gdt", ["float32", "bfloat16"])
def test_sharded_update_equals_one_global_step(gdt):
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_sharded_worker, args=(r, world, port, q, gdt)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda z: z[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ora, x, m, t, B = _data(N=16, H=8)
    _, _, gW, gb = ora.loss_and_grads(x, m, t)
    grads = [g for pair in zip(gW, gb) for g in pair]
    want = []
    for p, g in zip(ora.params(), grads):
        g32 = np.asarray(g, np.float32)
        a = g32 * g32
        want.append((np.asarray(p, np.float32) - 0.005 * g32 / (np.sqrt(a) + 1e-8), a))
    # fp32: the sum of two fp32 halves vs the fp64 global gradient (one rounding); bf16: the halves
    # rounded to 8 bits first -- Adagrad's first step is lr * sign(g) except where |g| ~ rounding
    tol = 2e-6 if gdt == "float32" else 2 * 0.005
    for _, ps, accs in res:
        for (wp, wa), gp, ga in zip(want, ps, accs):
            assert np.abs(gp - wp).max() <= tol
            if gdt == "float32":
                np.testing.assert_allclose(ga, wa, rtol=1e-5, atol=1e-12)
    for a, b in zip(res[0][1], res[1][1]):               # replicas identical
        np.testing.assert_array_equal(a, b)
