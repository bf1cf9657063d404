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
        g = g.float() / world
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


def test_sharded_rccl_branch_ordering(monkeypatch):
    """The data-parallel step's RCCL branch (async reduce-scatter / in-place all-gather), which the gloo
    tests never take (they stage collectives through host copies), driven in one process with a stubbed
    torch.distributed that records the call order: every layer's reduce-scatter starts only after that
    layer's gradients are written (Engine.grad_hook), each shard's update runs only after its reduce-scatter
    was waited on, the all-gather sends this rank's slice of the gathered tensor into that tensor
    (in place), ZeRO-1 gathers the 16-bit shadows of the first / last layer (the update writes the shadow
    shard) and the fp32 tensors otherwise, and every gather is waited on before the step returns."""
    from omnidirectional_collaborative_filtering_amd import _lib
    from omnidirectional_collaborative_filtering_amd import parallel as P
    world, rank = 2, 1
    log = []

    class Work:
        def __init__(self, tag):
            self.tag = tag

        def wait(self):
            log.append(("wait",) + self.tag)

    def name_of(t):
        for k, v in tensors.items():
            if t.data_ptr() == v.data_ptr() and t.numel() == v.numel():
                return k
        return None

    def reduce_scatter_tensor(out, inp, op=None, group=None, async_op=False):
        assert async_op, "the RCCL branch must be asynchronous"
        n = out.numel()
        out.copy_((inp[rank * n:(rank + 1) * n].float() * world).to(out.dtype))
        log.append(("rs", name_of(inp)))
        return Work(("rs", name_of(inp)))

    def all_gather_into_tensor(out, inp, group=None, async_op=False):
        assert async_op
        assert inp.data_ptr() == out.data_ptr() + rank * inp.numel() * inp.element_size(), "in place: flat[lo:hi]"
        assert inp.numel() * world == out.numel()
        log.append(("ag", name_of(out)))
        return Work(("ag", name_of(out)))

    monkeypatch.setattr(P.dist, "is_initialized", lambda: True)
    monkeypatch.setattr(P.dist, "get_backend", lambda group=None: "nccl")
    monkeypatch.setattr(P.dist, "broadcast", lambda t, src, group=None: None)
    monkeypatch.setattr(P.dist, "reduce_scatter_tensor", reduce_scatter_tensor)
    monkeypatch.setattr(P.dist, "all_gather_into_tensor", all_gather_into_tensor)
    monkeypatch.setattr(P.torch.cuda, "current_stream", lambda: types.SimpleNamespace(cuda_stream=0))

    def fake_call(name, *args):
        assert name == "ocf_opt_step_ex", name
        a = args[0]
        log.append(("update", a.p, a.g, a.shadow, a.n))
        return 0
    monkeypatch.setattr(_lib, "call", fake_call)

    dims = [(256, 128), (128, 256)]          # W0 [in][out], W1 stored transposed [N][H]

    class Opt:
        iterations = 0

        def step_params(self, scale, l2):
            return _lib.OcfOptParams(1, 0.005, 1e-8, 0, 0, l2, scale)

    class FakeEngine:
        def __init__(self):
            self.W = [torch.zeros(*d) for d in dims]
            self.b = [torch.zeros(128), torch.zeros(256)]
            self.Wsh = [torch.zeros(*d, dtype=torch.float16) for d in dims]
            self.l2, self.shadow_blocked, self.dev, self.cdt = 0.0, False, torch.device("cpu"), _lib.DT_F16
            self.slots = [([torch.zeros_like(w), None], [torch.zeros_like(b), None]) for w, b in zip(self.W, self.b)]
            self.opt, self.trainable, self.grad_hook, self.master_sync = Opt(), [True, True], None, None

        def _refresh_shadows(self):
            log.append(("refresh_all",))

        def _refresh_shadow(self, i):
            log.append(("refresh", i))

        def train_step(self, grads_out):
            for i in (1, 0):                  # output layer first, as Engine._backward_gather
                grads_out[2 * i].fill_(1.0)
                grads_out[2 * i + 1].fill_(1.0)
                log.append(("grad", i))
                if self.grad_hook:
                    self.grad_hook(i)

    e = FakeEngine()
    dp = P.DataParallel(e, rank, world, mode="sharded", grad_dtype="bfloat16")
    assert dp.zero_layers == {0, 1} and e.master_sync is not None
    tensors = {"W0": e.W[0], "b0": e.b[0], "W1": e.W[1], "b1": e.b[1], "sh0": e.Wsh[0], "sh1": e.Wsh[1],
               "gW0": dp.views[0], "gb0": dp.views[1], "gW1": dp.views[2], "gb1": dp.views[3]}
    log.clear()
    dp.step()
    ev = [x[:2] for x in log]
    for i in (0, 1):
        assert ev.index(("grad", i)) < ev.index(("rs", "gW%d" % i)) and ev.index(("grad", i)) < ev.index(("rs", "gb%d" % i))
    ups = [k for k, x in enumerate(log) if x[0] == "update"]
    rs_waits = [k for k, x in enumerate(log) if x[:2] == ("wait", "rs")]
    assert len(ups) == 4 and len(rs_waits) == 4
    for u, w in zip(ups, rs_waits):
        assert w < u, "update before its reduce-scatter completed"
    # ZeRO-1: the weights' updates carry their shadow shard; the biases' do not
    lo = rank * e.W[0].numel() // world
    w_up = [x for x in log if x[0] == "update" and x[3]]
    assert sorted(x[3] for x in w_up) == sorted(e.Wsh[i].view(-1)[lo:].data_ptr() for i in (0, 1))
    gathered = [x[1] for x in log if x[0] == "ag"]
    assert sorted(gathered) == ["b0", "b1", "sh0", "sh1"], gathered
    for g in gathered:                                    # each gather after its update, waited before the end
        assert ev.index(("wait", "ag")) > ev.index(("ag", g))
    assert sum(1 for x in log if x[:2] == ("wait", "ag")) == 4
    assert ("refresh_all",) not in log, "ZeRO-1: no full shadow refresh"
    assert dp._masters_stale


def test_sharded_falls_back_when_shards_do_not_divide(monkeypatch):
    from omnidirectional_collaborative_filtering_amd import parallel as P
    monkeypatch.setattr(P.dist, "is_initialized", lambda: True)
    monkeypatch.setattr(P.dist, "get_backend", lambda group=None: "nccl")
    monkeypatch.setattr(P.dist, "broadcast", lambda t, src, group=None: None)
    e = types.SimpleNamespace(W=[torch.zeros(256, 128)], b=[torch.zeros(128)], Wsh=[None], l2=0.0,
                              shadow_blocked=False, dev=torch.device("cpu"), _refresh_shadows=lambda: None)
    with pytest.warns(UserWarning, match="allreduce"):
        dp = P.DataParallel(e, 0, 3, mode="sharded")
    assert dp.mode == "allreduce" and dp.sync is None
