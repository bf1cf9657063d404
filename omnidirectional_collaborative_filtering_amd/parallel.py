"""Row (user/item-batch) data parallelism over torch.distributed (backend 'nccl' = RCCL on ROCm).

One process per GPU.  Rank r takes batches r, r+G, r+2G, ... of the shared epoch permutation, so
G ranks process a global batch of G*B rows per step.  Keras' MSE is a mean over B*N, hence the
gradient of the concatenated G*B-row batch is the AVERAGE of the G local gradients -- exactly
what ``grad_sync`` computes (one flat fp32 bucket, one all-reduce), after which every rank
applies the same elementwise optimizer (``Engine.apply_grads``) and the replicas stay identical.
With G = 1 nothing here runs: the optimizer is fused into the weight-gradient GEMM epilogues.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def init_from_env(backend=None):
    """torchrun / torch.distributed.run environment -> (rank, world, local_rank)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # OCF_REHEARSAL=1: rehearse an N-rank run on ONE GPU (all ranks on device 0, gloo transport);
    # correctness only, timings meaningless
    if os.environ.get("OCF_REHEARSAL") == "1":
        backend, local = "gloo", 0
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend, init_method="env://")
    return rank, world, local


class GradBucket:
    """All parameter gradients of an Engine as views into ONE flat fp32 buffer (one collective)."""

    def __init__(self, engine, dtype=torch.float32):
        sizes = []
        for w, b in zip(engine.W, engine.b):
            sizes += [w.numel(), b.numel()]
        self.flat = torch.zeros(sum(sizes), device=engine.dev, dtype=dtype)
        self.views = []
        off = 0
        shapes = []
        for w, b in zip(engine.W, engine.b):
            shapes += [w.shape, b.shape]
        for n, shp in zip(sizes, shapes):
            self.views.append(self.flat[off: off + n].view(shp))
            off += n


def grad_sync(bucket, world):
    if world > 1:
        dist.all_reduce(bucket.flat, op=dist.ReduceOp.SUM)


def dp_train_step(engine, bucket, world):
    """forward + backward (raw grads) -> all-reduce -> averaged optimizer step."""
    if world == 1:
        engine.train_step()
        return
    engine.train_step(grads_out=bucket.views)
    grad_sync(bucket, world)
    engine.apply_grads(bucket.views, scale=1.0 / world)


def shard_batches(num_batches, rank, world):
    """batch indices of this rank within an epoch (rank-strided)."""
    return list(range(rank, num_batches - (num_batches % world), world))


# ---------------------------------------------------------------------------------------------
# Feature (column) parallelism -- SURVEY.md 8(e) "N-sharding".
#
# Rank g owns output/input columns [c0_g, c1_g) (users, in I-AutoRec): its rows of W1 and W_out,
# their optimizer state, and the matching column shard of the rating CSR.  Every rank processes the
# SAME global batch.  Per step the ranks exchange two [B, H] fp32 tensors: the partial encoder
# pre-activation X[:, shard] W1[shard] (summed -> identical hidden activations everywhere) and the
# partial backward delta  delta_out[:, shard] W_out[shard] (summed -> identical dh).  Weight
# gradients never cross the fabric; the hidden layers are recomputed identically on every rank.
# The result is one optimizer step on the global batch, exactly as on a single device (up to the
# order of the fp32 sums).

def feature_shard_range(N, rank, world, tile=128):
    per = -(-N // world)
    per = -(-per // tile) * tile
    c0 = min(N, rank * per)
    c1 = min(N, c0 + per)
    if c1 <= c0:
        raise ValueError("N=%d too small for %d feature shards of %d columns" % (N, world, per))
    return c0, c1


def make_comm(world):
    """sum-all-reduce of a device tensor over the process group (RCCL for 'nccl'), or None."""
    if world <= 1:
        return None

    def comm(t):
        dist.all_reduce(t, op=dist.ReduceOp.SUM)

    def start(t):
        """asynchronous form: returns the work handle; wait() orders the caller's stream after it"""
        return dist.all_reduce(t, op=dist.ReduceOp.SUM, async_op=True)
    comm.start = start
    return comm
