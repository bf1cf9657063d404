"""Multi-GPU layouts over torch.distributed (backend 'nccl' = RCCL on ROCm), one process per GPU.

Row data parallelism (``DataParallel``): rank r takes batches r, r+G, r+2G, ... of the shared epoch
permutation, so G ranks process a global batch of G*B rows per step.  Keras' MSE is a mean over B*N,
hence the gradient of the concatenated G*B-row batch is the AVERAGE of the G local gradients; after
the exchange every rank holds the same parameters.  With G = 1 nothing here runs: the optimizer is
fused into the weight-gradient kernels.  Feature (column) parallelism: see the second half.
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
    """forward + backward (raw grads) -> all-reduce -> averaged optimizer step (mode 'allreduce')."""
    if world == 1:
        engine.train_step()
        return
    engine.train_step(grads_out=bucket.views)
    grad_sync(bucket, world)
    engine.apply_grads(bucket.views, scale=1.0 / world)


def _staged(backend, t):
    """gloo moves CUDA tensors through host copies for all_reduce only; the tensor collectives below
    get explicit host staging there (rehearsals on one GPU), device tensors directly over RCCL"""
    return backend == "gloo" and t.is_cuda


class ShardedSync:
    """Reduce-scatter / sharded update / all-gather of a list of parameter tensors (SURVEY 8(e)'s
    data-parallel mitigations): for tensor j, rank r owns elements [r n/G, (r+1) n/G) of its flat view.
      start(j)         : reduce-scatter of grads[j] (sum; fp32 or bf16) into this rank's shard buffer,
                         asynchronous -- issued as soon as the engine has written that gradient, so the
                         output layer's exchange overlaps the input layer's weight-gradient kernel;
      finish(update)   : for every started tensor in order: wait, update(j, lo, hi, g_shard) (the
                         optimizer on this rank's 1/G of the parameters and slots; g_shard in the
                         gradient's dtype), then an asynchronous in-place all-gather of gather[j]'s
                         updated shard into the full gather[j] (default: the fp32 parameter; the 16-bit
                         weight shadow under ZeRO-1, DataParallel); waits for all.
    Traffic per step: (G-1)/G of the gradient bytes (bf16: half) + (G-1)/G of the gathered bytes (fp32
    parameters, or 16-bit shadows: half), with the HBM-bound optimizer pass cut to 1/G per rank."""

    def __init__(self, params, grads, rank, world, group=None, gather=None):
        self.params, self.grads = params, grads
        self.gather = list(gather) if gather is not None else list(params)
        self.rank, self.world, self.group = rank, world, group
        self.backend = dist.get_backend(group) if dist.is_initialized() else "gloo"
        for p, g, t in zip(params, grads, self.gather):
            if not shardable(p.numel(), world):
                raise ValueError("tensor of %d elements does not split into %d 16-B aligned shards" % (p.numel(), world))
            if g.numel() != p.numel() or t.numel() != p.numel():
                raise ValueError("gradient / gathered / parameter size mismatch")
        self.shard = [torch.empty(g.numel() // world, dtype=g.dtype, device=g.device) for g in grads]
        self._started = []

    def bounds(self, j):
        n = self.params[j].numel() // self.world
        return self.rank * n, (self.rank + 1) * n

    def start(self, j):
        g = self.grads[j].view(-1)
        out = self.shard[j]
        if _staged(self.backend, g):
            gh, oh = g.cpu(), torch.empty(out.numel(), dtype=out.dtype)
            dist.reduce_scatter_tensor(oh, gh, op=dist.ReduceOp.SUM, group=self.group)
            out.copy_(oh)
            work = None
        else:
            work = dist.reduce_scatter_tensor(out, g, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        self._started.append((j, work))

    def finish(self, update):
        gathers = []
        for j, work in self._started:
            if work is not None:
                work.wait()
            lo, hi = self.bounds(j)
            update(j, lo, hi, self.shard[j])
            flat = self.gather[j].view(-1)
            mine = flat[lo:hi]
            if _staged(self.backend, flat):
                fh = torch.empty(flat.numel(), dtype=flat.dtype)
                dist.all_gather_into_tensor(fh, mine.cpu(), group=self.group)
                flat.copy_(fh)
            else:
                gathers.append(dist.all_gather_into_tensor(flat, mine, group=self.group, async_op=True))
        for w in gathers:
            w.wait()
        self._started = []

    def gather_tensors(self, tensors):
        """all-gather every rank's shard of same-shaped companions of the parameters (optimizer slots
        before a checkpoint; the fp32 masters under ZeRO-1)"""
        for j, t in enumerate(tensors):
            if t is None:
                continue
            flat = t.view(-1)
            lo, hi = self.bounds(j)
            if _staged(self.backend, flat):
                fh = torch.empty(flat.numel(), dtype=flat.dtype)
                dist.all_gather_into_tensor(fh, flat[lo:hi].cpu(), group=self.group)
                flat.copy_(fh)
            else:
                dist.all_gather_into_tensor(flat, flat[lo:hi].clone(), group=self.group)


def shardable(n, world):
    """n elements split into `world` equal shards of a multiple of 4 elements (16-B aligned)"""
    return n % world == 0 and (n // world) % 4 == 0


class DataParallel:
    """Row (user/item-batch) data parallelism of one Engine replica per rank -- the north_star's
    "user-batch data parallelism with RCCL gradient all-reduce", with SURVEY 8(e)'s mitigations.

    mode 'sharded' (default): the engine writes raw per-layer gradients (EPI_GRAD; bf16 with
      grad_dtype='bfloat16'); each layer's reduce-scatter starts as soon as that layer's gradient is
      written (the output layer's overlaps the input layer's weight-gradient kernel); every rank updates
      its 1/G of every parameter tensor and its slots (ocf_opt_step_ex, reading the shard in its own
      dtype).  ZeRO-1 for the weights the kernels read through a 16-bit row-major shadow (first and last
      layer in f16 / bf16 compute, l2 = 0): the update also writes the shadow shard and only the shadow is
      all-gathered -- half the bytes, no per-step shadow refresh; the fp32 masters stay sharded (each rank
      current on its 1/G) until get_weights / save / predict gathers them (gather_masters).  Every other
      tensor: the fp32 parameter shard is all-gathered.
    mode 'allreduce': one flat fp32 bucket, one all-reduce, the full optimizer on every rank.
    A tensor that does not split into G 16-B aligned shards (e.g. G = 3, 5, 6) makes 'sharded' fall back
    to 'allreduce' (with a warning).  Both start from rank 0's weights (broadcast here), and the engine
    mixes the rank into the Philox stream of its dropout masks so the G local batches draw independent
    masks like one global batch."""

    def __init__(self, engine, rank, world, mode="sharded", grad_dtype="float32", group=None, zero=True):
        if mode not in ("sharded", "allreduce"):
            raise ValueError("mode must be 'sharded' or 'allreduce'")
        if grad_dtype not in ("float32", "bfloat16"):
            raise ValueError("grad_dtype must be float32 or bfloat16")
        if grad_dtype == "bfloat16" and mode != "sharded":
            raise ValueError("bf16 gradients need mode='sharded'")
        self.engine, self.rank, self.world, self.group = engine, int(rank), int(world), group
        params = [t for w, b in zip(engine.W, engine.b) for t in (w, b)]
        if mode == "sharded" and not all(shardable(p.numel(), self.world) for p in params):
            import warnings
            warnings.warn("DataParallel: parameters do not split into %d aligned shards; using mode='allreduce'"
                          % self.world)
            mode, grad_dtype = "allreduce", "float32"
        self.mode, self.grad_dtype = mode, grad_dtype
        engine.dp_rank, engine.dp_world = self.rank, self.world
        self.broadcast_params()
        # ZeRO-1 layers: weights read only through a row-major 16-bit shadow
        self.zero_layers = set()
        if mode == "sharded" and zero and not engine.l2 and not engine.shadow_blocked:
            self.zero_layers = {i for i, sh in enumerate(engine.Wsh) if sh is not None}
        self._masters_stale = False
        if mode == "allreduce":
            self.bucket = GradBucket(engine)
            self.views = self.bucket.views
            self.sync = None
        else:
            gdt = torch.bfloat16 if grad_dtype == "bfloat16" else torch.float32
            self.views = []
            for w, b in zip(engine.W, engine.b):
                self.views += [torch.zeros(w.shape, device=engine.dev, dtype=gdt),
                               torch.zeros(b.shape, device=engine.dev, dtype=torch.float32)]
            gather = [engine.Wsh[j // 2] if (j % 2 == 0 and j // 2 in self.zero_layers) else p
                      for j, p in enumerate(params)]
            self.sync = ShardedSync(params, self.views, self.rank, self.world, group, gather=gather)
        engine.master_sync = self.gather_masters if self.zero_layers else None

    def broadcast_params(self):
        e = self.engine
        if self.world > 1:
            for t in [x for w, b in zip(e.W, e.b) for x in (w, b)]:
                if _staged(dist.get_backend(self.group), t):
                    h = t.cpu()
                    dist.broadcast(h, 0, group=self.group)
                    t.copy_(h)
                else:
                    dist.broadcast(t, 0, group=self.group)
        e._refresh_shadows()

    def gather_masters(self):
        """ZeRO-1: every rank's fp32 master shards -> full fp32 weights (before reading them)"""
        if not self._masters_stale:
            return
        e = self.engine
        self.sync.gather_tensors([e.W[j // 2] if (j % 2 == 0 and j // 2 in self.zero_layers) else None
                                  for j in range(2 * len(e.W))])
        self._masters_stale = False

    def step(self):
        e = self.engine
        if self.mode == "allreduce":
            e.train_step(grads_out=self.views)
            grad_sync(self.bucket, self.world)
            e.apply_grads(self.views, scale=1.0 / self.world)
            return
        from . import _lib
        sync = self.sync
        e.grad_hook = lambda i: (sync.start(2 * i), sync.start(2 * i + 1))
        try:
            e.train_step(grads_out=self.views)
        finally:
            e.grad_hook = None
        scale = 1.0 / self.world
        opw = e.opt.step_params(scale, e.l2)     # l2 regularises kernels only
        opb = e.opt.step_params(scale, 0.0)
        stream = torch.cuda.current_stream().cuda_stream

        def update(j, lo, hi, g):
            i = j // 2
            if not e.trainable[i]:
                return
            p = e.W[i] if j % 2 == 0 else e.b[i]
            sw, sb = e.slots[i]
            s = sw if j % 2 == 0 else sb
            f = lambda t: None if t is None else t.view(-1)[lo:hi].data_ptr()
            a = _lib.OcfOptStepArgs()
            a.p, a.g, a.s1, a.s2, a.n = f(p), g.data_ptr(), f(s[0]), f(s[1]), hi - lo
            a.g_dtype = _lib.DT_BF16 if g.dtype == torch.bfloat16 else _lib.DT_F32
            a.opt = opw if j % 2 == 0 else opb
            if j % 2 == 0 and i in self.zero_layers:
                a.shadow, a.shadow_dtype = f(e.Wsh[i]), e.cdt
            _lib.call("ocf_opt_step_ex", a, stream)
        sync.finish(update)
        if self.zero_layers:
            self._masters_stale = True
            # shadows of the other layers (none in the ZeRO-1 layouts; kept for completeness)
            for i, sh in enumerate(e.Wsh):
                if sh is not None and i not in self.zero_layers:
                    e._refresh_shadow(i)
        else:
            e._refresh_shadows()
        e.opt.iterations += 1

    def gather_slots(self):
        """every rank's optimizer-slot shards -> full slots on every rank (sharded mode; before save)"""
        if self.sync is None:
            return
        e = self.engine
        for k in range(2):
            ts = [t for sw, sb in e.slots for t in (sw[k], sb[k])]
            if any(t is not None for t in ts):
                self.sync.gather_tensors(ts)


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
