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
