"""GPU, ONE rank over RCCL (torch.distributed backend 'nccl'): the collective branches the multi-GPU
layouts take on RCCL -- the asynchronous reduce_scatter_tensor started from the engine's grad_hook,
the in-place all_gather_into_tensor of the ZeRO-1 shadow shards, the gather of the fp32 masters, the
feature layout's asynchronous all_reduce (make_comm.start) overlapped with the output layer's update
-- run on RCCL and give bit-identical results to the same layouts over gloo's host-staged branches
(with one rank both collectives are the identity, so any difference is an ordering / stream /
layout bug of the RCCL branch).  Every test in the other files stages its collectives through gloo;
RCCL between GPUs runs only in the driver's multi-GPU jobs (a box here has one GPU and RCCL refuses
two ranks on one device)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from parity import dataset

B, H, STEPS = 128, 64, 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _comm(dist, group):
    def comm(t):
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)

    def start(t):
        return dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group, async_op=True)
    comm.start = start
    return comm


def _train(group, layout, cd):
    import torch.distributed as dist
    from omnidirectional_collaborative_filtering_amd.data_reader import data_reader
    from omnidirectional_collaborative_filtering_amd.model import omni_model
    from omnidirectional_collaborative_filtering_amd.optimizers import Adagrad
    from omnidirectional_collaborative_filtering_amd.parallel import DataParallel
    data = dataset()
    np.random.seed(77)
    rd = data_reader(data.num_cols, data.train.n_rows, dataset=data, eval_mode="fixed_split")
    kw = {}
    if layout == "feature":
        kw = dict(shard=(0, data.num_cols, data.num_cols), comm=_comm(dist, group))
    om = omni_model(1, H, data.num_cols, B, dense_activation="sigmoid", use_causal_info=False, dropout_probability=0.2,
                    compute_dtype=cd, seed=11, **kw)
    m = om.model
    m.compile(Adagrad(lr=0.005, epsilon=1e-8), "mean_squared_error")
    if layout.startswith("dp"):
        m.rank, m.world = 0, 1
        m.dp = DataParallel(om.engine, 0, 1, mode="sharded", group=group,
                            grad_dtype="bfloat16" if layout == "dp_bf16" else "float32")
    gen = rd.data_gen(B, [0.5, 0.9], "train", True, None, -1, pass_through_input_training=False)
    h = m.fit_generator(gen, STEPS, verbose=0)
    w = m.get_weights()
    sh = [t.detach().cpu().float().numpy() for t in om.engine.Wsh if t is not None]
    return h.history["loss"][0], w, sh


def _worker(port, q, layout, cd):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                          LOCAL_RANK="0")
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", init_method="env://", device_id=torch.device("cuda", 0))
        gloo = dist.new_group(backend="gloo")
        assert dist.get_backend() == "nccl" and dist.get_backend(gloo) == "gloo"
        out_rccl = _train(None, layout, cd)
        out_gloo = _train(gloo, layout, cd)
        torch.cuda.synchronize()
        q.put(("ok", out_rccl, out_gloo))
        dist.destroy_process_group()
    except BaseException:
        import traceback
        q.put(("error", traceback.format_exc()))
        q.close()
        q.join_thread()
        os._exit(1)


@pytest.mark.gpu
@pytest.mark.parametrize("layout,cd", [("dp", "float32"), ("dp", "float16"), ("dp_bf16", "bfloat16"),
                                       ("feature", "float32"), ("feature", "float16")])
def test_rccl_branches_match_staged(gpu, layout, cd):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), q, layout, cd))
    p.start()
    res = q.get(timeout=300)
    p.join(timeout=120)
    assert res[0] == "ok", res[1]
    assert p.exitcode == 0
    (l_r, w_r, s_r), (l_g, w_g, s_g) = res[1], res[2]
    assert np.isfinite(l_r) and l_r == l_g, (l_r, l_g)
    assert len(w_r) == len(w_g) and len(s_r) == len(s_g)
    for a, b in zip(w_r + s_r, w_g + s_g):
        assert a.shape == b.shape and np.array_equal(a, b), float(np.abs(a - b).max())
