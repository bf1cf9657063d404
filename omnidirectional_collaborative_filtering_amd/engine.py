"""GPU engine: parameters, workspaces and the per-step kernel sequence of the autoencoder.

Replaces what Keras/TF do for model.py:43-99 + train.py:49-51,131-133 (graph build, MatMul,
BiasAdd, activation, Dropout, Mul, MSE, gradients, optimizer Assign ops) with calls into
libocf.so.  Tensors are PyTorch-ROCm device tensors (memory + streams only); every byte of
arithmetic runs in the hand-written HIP kernels.

Padded HBM layout (DESIGN.md "Data layout"):
  * batch rows       B  -> Bp = roundup(B, 128)
  * output width     N  -> Np = roundup(N, 128); layer-0 input = k blocks of Np (concat order of
                            model.py:47-56: data | observed mask | second mask)
  * hidden widths    H  -> Hp = roundup(H, 128)
  * W_i  fp32 [in_p][out_p] (Keras (in, out) layout) for the encoder and hidden layers; the
    decoder W_L is stored transposed, [Np][H_p] (one row per output user), so that every weight
    stream of the step (encoder/decoder forward, decoder backward, both fused optimizers) reads
    whole 2-KB rows instead of 512-B column pieces 555 KB apart; b_i fp32 [out_p].  Pads are zero
    and stay zero (their gradients are exactly zero; the optimizers map g = 0, state = 0 to no change)
Per step the loss gradient is carried unscaled (err * mask) in the compute dtype and the
constant 2/(B*N) of Keras' MSE is folded into the weight/bias-gradient epilogues (gscale), which
keeps f16 operands far from underflow.
"""
from __future__ import annotations

import ctypes
import math

import numpy as np
import torch

from . import _lib
from ._lib import OcfGemmArgs, OcfScatterArgs

# while Engine._recorded_step runs: every library call of the step as (name, args) -- the template of the
# one-call step (Engine.fast_train_step)
_recorder = None


def call(name, *args):
    if _recorder is not None:
        _recorder.append((name, args))
    return _lib.call(name, *args)

TILE = 128
# the decoder gather re-reduces a row's encoder chunk partials in every one of that row's chunks
# (O(chunks^2) per row): past this many chunks in a batch row, a separate ocf_rows_reduce runs instead
# (skewed ML-20M-shaped batch, rows up to ~170 chunks: fused 128 us vs 135 us for the two gathers;
# a Netflix-sized row of 900 chunks would re-read 1.6 GB of partials)
FUSE_MAX_CHUNKS = 256
# ... and past this many chunks per batch row on average: every decoder chunk re-reads all of its row's encoder
# partials (O(chunks^2) per row).  Netflix (~22 chunks per row): 2.029 -> 1.997 ms/step with the separate launch
# (profiles/r05_cfg/nf_base.jsonl); ML-20M (~3): the fused form
FUSE_MEAN_CHUNKS = 8
# the encoder as an MFMA contraction over 128-column tiles of W1 (ocf_encoder_tiles) instead of row gathers, when
# a weight row carries this many batch entries on average (the gathers read a W1 row per entry, the tiles read each
# tile once per 256 batch rows) on a weight of at least ENC_TILES_MIN_TILES tiles, 16-bit compute.  Measured in
# round 6 (tools/probes/enc_tiles_probe.py, profiles/r06_tiles/): pre-pass + tile kernel vs the gather encoder
# Netflix 211 vs 207 us, the 8-way Netflix rank 196 vs 165, the 8-way ML-20M rank 88 vs 28 -- it does not win
# anywhere yet, so the automatic choice never takes it (engine.enc_tiles = True forces it)
ENC_TILES_MIN_ENTRIES = float("inf")
ENC_TILES_MIN_TILES = 64
ENC_TILES_WGS = 256           # workgroups to aim for (one per CU): splits = WGS / (row groups x hidden slices)
DTYPES = {"float32": (_lib.DT_F32, torch.float32), "float16": (_lib.DT_F16, torch.float16),
          "bfloat16": (_lib.DT_BF16, torch.bfloat16)}
DTYPE_ALIASES = {"f32": "float32", "fp32": "float32", "f16": "float16", "fp16": "float16", "half": "float16",
                 "bf16": "bfloat16"}


def ru(x, m):
    return ((int(x) + m - 1) // m) * m


def ptr(t):
    return None if t is None else t.data_ptr()


def cur_stream():
    """the current HIP stream of the current device, as a raw pointer for the C ABI (the torch._C getters:
    torch.cuda.current_stream() costs ~8 us of Python per call, ~9 calls per training step)"""
    return torch._C._cuda_getCurrentRawStream(torch._C._cuda_getDevice())


def _counter_reset(engine):
    """a hook for _lib.enc_wait_hooks that clears the engine's hand-off counters (weakly bound: a dead engine's
    hook removes itself)"""
    import weakref
    ref = weakref.ref(engine)

    def hook():
        e = ref()
        if e is None:
            if hook in _lib.enc_wait_hooks:
                _lib.enc_wait_hooks.remove(hook)
            return
        torch.cuda.synchronize(e.dev)
        e.enc_arrive.zero_()
        e.row_arrive.zero_()
        torch.cuda.synchronize(e.dev)
    hook.ref = ref
    _lib.enc_wait_hooks[:] = [h for h in _lib.enc_wait_hooks if getattr(h, "ref", lambda: 1)() is not None]
    return hook


def glorot_uniform(rng, fan_in, fan_out):
    lim = math.sqrt(6.0 / (fan_in + fan_out))
    return rng.uniform(-lim, lim, size=(fan_in, fan_out)).astype(np.float32)


class Engine:
    def __init__(self, N, hidden, batch_size, k_blocks=1, activation="tanh", dropout=None, l2=None,
                 compute_dtype="float32", device=None, seed=None, shard=None, comm=None):
        """shard = (c0, c1, N_total): this engine holds output columns [c0, c1) of an N_total-wide
        model (feature parallelism, parallel.py); comm(tensor) sums a device tensor over the ranks."""
        if not torch.cuda.is_available():
            raise RuntimeError("omnidirectional_collaborative_filtering_amd needs a ROCm GPU (MI355X); none visible")
        _lib.load()
        cd = DTYPE_ALIASES.get(compute_dtype, compute_dtype)
        if cd not in DTYPES:
            raise ValueError("compute_dtype must be float32, float16 or bfloat16")
        self.cdtype = cd
        self.cdt, self.tdt = DTYPES[cd]
        self.dev = torch.device(device if device is not None else "cuda")
        self.N = int(N)
        self.shard = shard
        self.N_total = int(shard[2]) if shard else self.N
        self.comm = comm
        self.Np = ru(N, TILE)
        self.k = int(k_blocks)
        self.H = [int(h) for h in hidden]
        self.Hp = [ru(h, TILE) for h in self.H]
        self.B = int(batch_size)
        self.Bp = ru(self.B, TILE)
        self.rows_real = None         # real rows of a zero-padded dense batch (load_dense), None = B
        # dense batches gathered by row (Model.fit): packing deferred to the layer-wise path; small models take
        # the fused one-launch step (ocf_mlp_step) instead
        self._pending_pack = self._mlp_batch = self._mlp_args = None
        self.fused_mlp = True
        self.mlp_trace = None
        self.mlp_wgs = 0                        # ocf_mlp_step's grid (0: the library's choice)
        self.step_paths = {"one_call": 0, "general": 0}   # fast_train_step's choices (diagnostics)
        self.act = _lib.ACT[activation]
        self.activation = activation
        self.dropout = dropout
        self.keep = 1.0 - float(dropout) if dropout else 1.0
        self.l2 = float(l2) if l2 else 0.0
        self.seed = int(seed if seed is not None else np.random.randint(0, 2 ** 31 - 1))
        self.real_dims = [self.k * self.N] + self.H + [self.N]
        self.pad_dims = [self.k * self.Np] + self.Hp + [self.Np]
        self.n_tiles = self.Np // TILE
        self.step_count = 0
        # one-call training steps (fast_train_step): template + per-batch rewrite, invalidated by any
        # reallocation of a buffer the step reads (_bufgen)
        self.fast_steps = True
        self._plan = None
        self._bufgen = 0
        # row data parallelism (parallel.DataParallel): the rank is mixed into the dropout stream so the
        # G local batches draw independent masks, like one global batch; grad_hook(i) is called once
        # layer i's raw gradients are written (grads_out steps), so its exchange can start right away
        self.dp_rank, self.dp_world = 0, 1
        self.grad_hook = None
        # data parallelism with ZeRO-1 masters (parallel.DataParallel): gathers the fp32 weights before
        # anything reads them outside the step (get_weights, predict, the l2 penalty)
        self.master_sync = None
        self.opt = None
        self.slots = []
        self._alloc_params()
        self._alloc_workspace()
        self.init_weights(np.random.RandomState(self.seed))

    # ---------------------------------------------------------------- parameters
    def _alloc_params(self):
        f = dict(device=self.dev, dtype=torch.float32)
        self.W = [torch.zeros(i, o, **f) for i, o in zip(self.pad_dims[:-2], self.pad_dims[1:-1])]
        self.W.append(torch.zeros(self.pad_dims[-1], self.pad_dims[-2], **f))     # decoder, transposed
        self.b = [torch.zeros(o, **f) for o in self.pad_dims[1:]]
        # Keras layer.trainable per dense layer (model.py:107-170): a frozen layer still propagates
        # deltas to the layers below it, but its kernel and bias receive no update and no slot state
        self.trainable = [True] * len(self.W)
        # half-width shadows of the two N-sized weights (f16/bf16 compute): the MFMA operand would be
        # rounded to the compute dtype while staging anyway, so streaming a copy rounded once by the
        # optimizer epilogue gives bit-identical products at half the bytes
        self.Wsh = [None] * len(self.W)
        # shadows stored 64x64-blocked: a GEMM K-step reads two contiguous 8 KB blocks instead of 64-128
        # strided row pieces (tools/probes/hbm_pattern.hip: 5.0 vs 3.7-4.0 TB/s from HBM).  Models that
        # take the row-gather path (one 1-block input layer, H <= 512) read the shadows by whole rows
        # instead (one contiguous 1 KB row per entry): row-major there (ML-20M step 0.512 -> 0.506 ms)
        self.shadow_blocked = not (self.k == 1 and self.Hp[0] <= 512 and self.Hp[-1] <= 512)
        if self.cdt != _lib.DT_F32:
            for i in sorted({0, len(self.W) - 1}):
                self.Wsh[i] = torch.zeros(self.W[i].shape, device=self.dev, dtype=self.tdt)

    def _refresh_shadows(self):
        for i in range(len(self.W)):
            self._refresh_shadow(i)

    def _refresh_shadow(self, i):
        w, sh = self.W[i], self.Wsh[i]
        if sh is not None:
            if self.shadow_blocked:     # 64x64 blocks, 8 KB contiguous each (ocf.h b_blocked)
                R, C = w.shape
                sh.view(R // 64, C // 64, 64, 64).copy_(w.view(R // 64, 64, C // 64, 64).permute(0, 2, 1, 3))
            else:
                sh.copy_(w)

    def _wblk(self, i):
        return int(self.Wsh[i] is not None and self.shadow_blocked)

    def _wop(self, i):
        """(tensor, dtype code) of weight i as a GEMM operand: the shadow when there is one."""
        if self.Wsh[i] is not None:
            return self.Wsh[i], self.cdt
        return self.W[i], _lib.DT_F32

    def _keras_view(self, i):
        """W_i as a padded (in, out) view (the decoder is stored transposed)."""
        return self.W[i].t() if i == len(self.W) - 1 else self.W[i]

    def _row_map(self, layer):
        """padded row index of each real input row of layer `layer`."""
        if layer == 0:
            blk = np.arange(self.k * self.N) // self.N
            return blk * self.Np + np.arange(self.k * self.N) % self.N
        return np.arange(self.real_dims[layer])

    def init_weights(self, rng):
        """Keras glorot_uniform kernels, zero biases (fan in/out of the real, unpadded layer).  A
        column shard takes its slice of the global initialisation, so G sharded engines start from
        exactly the single-engine weights."""
        if self.shard:
            c0, c1, NT = self.shard
            dims = [self.k * NT] + self.H + [NT]
            ws = [glorot_uniform(rng, i, o) for i, o in zip(dims[:-1], dims[1:])]
            rows0 = np.concatenate([np.arange(b * NT + c0, b * NT + c1) for b in range(self.k)])
            ws[0] = ws[0][rows0]
            ws[-1] = ws[-1][:, c0:c1]
        else:
            ws = [glorot_uniform(rng, i, o) for i, o in zip(self.real_dims[:-1], self.real_dims[1:])]
        self.set_weights([x for w in ws for x in (w, np.zeros(w.shape[1], np.float32))])

    def get_weights(self):
        """Keras-layout numpy list [W0, b0, W1, b1, ...] (padding stripped)."""
        if self.master_sync is not None:
            self.master_sync()
        out = []
        for i, b in enumerate(self.b):
            rows = torch.as_tensor(self._row_map(i), device=self.dev)
            w = self._keras_view(i)
            out.append(w.index_select(0, rows)[:, : self.real_dims[i + 1]].cpu().numpy())
            out.append(b[: self.real_dims[i + 1]].cpu().numpy())
        return out

    def set_weights(self, weights):
        for i in range(len(self.W)):
            w = torch.as_tensor(np.asarray(weights[2 * i], np.float32), device=self.dev)
            bb = torch.as_tensor(np.asarray(weights[2 * i + 1], np.float32), device=self.dev)
            if tuple(w.shape) != (self.real_dims[i], self.real_dims[i + 1]):
                raise ValueError("weight %d has shape %s, expected %s" % (i, tuple(w.shape),
                                                                         (self.real_dims[i], self.real_dims[i + 1])))
            self.W[i].zero_()
            rows = torch.as_tensor(self._row_map(i), device=self.dev)
            kv = self._keras_view(i)
            full = torch.zeros(kv.shape, device=self.dev, dtype=torch.float32)
            full[:, : self.real_dims[i + 1]].index_copy_(0, rows, w)
            kv.copy_(full)
            self.b[i].zero_()
            self.b[i][: self.real_dims[i + 1]] = bb
        self._refresh_shadows()

    def set_optimizer(self, opt):
        self.opt = opt
        self._bufgen += 1
        self.slots = []
        for w, b in zip(self.W, self.b):
            sw = [torch.zeros_like(w) for _ in range(opt.n_slots)] + [None] * (2 - opt.n_slots)
            sb = [torch.zeros_like(b) for _ in range(opt.n_slots)] + [None] * (2 - opt.n_slots)
            self.slots.append((sw, sb))

    # ---------------------------------------------------------------- workspace
    def _alloc_workspace(self):
        d = self.dev
        Bp = self.Bp
        self.xin = torch.zeros(Bp, self.pad_dims[0], device=d, dtype=self.tdt)
        self.a = [torch.zeros(Bp, h, device=d, dtype=torch.float32) for h in self.Hp]
        self.h = [torch.zeros(Bp, h, device=d, dtype=self.tdt) for h in self.Hp]
        self.dh = [torch.zeros(Bp, h, device=d, dtype=self.tdt) for h in self.Hp]
        self.mask = [torch.zeros(Bp, h, device=d, dtype=torch.uint8) for h in self.Hp] if self.keep < 1 else \
            [None] * len(self.Hp)
        self.d_out = torch.zeros(Bp, self.Np, device=d, dtype=self.tdt)
        self.db_out_part = torch.zeros(Bp // TILE, self.Np, device=d, dtype=torch.float32)
        # bias-gradient partials: Bp/4 rows from the split-K reduction, Bp/128 from GRAD_ACT tiles
        self.db_h = [torch.zeros(Bp // 4, h, device=d, dtype=torch.float32) for h in self.Hp]
        self.splits0 = self._pick_splits(self.pad_dims[0], self.Hp[0])
        self.splitsL = self._pick_splits(self.Np, self.Hp[-1])
        # hidden -> hidden layers (forward: h[i-1] W[i]; backward: dh[i] W[i]^T): a batch of 128 rows and
        # 256 hidden units is 2 output tiles, i.e. 2 workgroups for the whole GEMM (Jester: 74 / 47 us
        # in fp32).  With few tiles the K-loop is split into one K-step per workgroup (EPI_SLAB) and the
        # layer epilogue runs in the split-K reduction (ocf_splitk_bias_act / ocf_splitk_grad_act)
        self.splits_fwd = [1] + [self._pick_splits_hidden(self.Hp[i - 1], self.Hp[i]) for i in range(1, len(self.H))]
        self.splits_bwd = [1] + [self._pick_splits_hidden(self.Hp[i], self.Hp[i - 1]) for i in range(1, len(self.H))]
        smax = max([self.splits0 * self.Hp[0], self.splitsL * self.Hp[-1]] +
                   [self.splits_fwd[i] * self.Hp[i] for i in range(1, len(self.H))] +
                   [self.splits_bwd[i] * self.Hp[i - 1] for i in range(1, len(self.H))])
        self.slabs = torch.zeros(smax * Bp, device=d, dtype=torch.float32)
        self.tile_cnt = torch.zeros(self.n_tiles, device=d, dtype=torch.int32)
        self.bk_ptr = torch.zeros(self.n_tiles + 1, device=d, dtype=torch.int32)
        self.bk_cur = torch.zeros(self.n_tiles, device=d, dtype=torch.int32)
        self.bk_cap = 0
        self._grow_buckets(1 << 16)
        self.tflag = torch.zeros(1 << 16, device=d, dtype=torch.uint8)   # live-target flag per batch entry
        # xin (dense path) is cleared by the scatter's memset unless already clean
        self._xin_clean = True
        self.tseg = None            # row-segment target descriptor of the loaded batch (None: buckets)
        # row-gather (sparse batch) path: chunk tables of the loaded batch (None: dense GEMM path)
        self.gt = None
        self.sparse_ok = self.k == 1 and self.Hp[0] <= 512 and self.Hp[-1] <= 512
        self.use_sparse = True
        # dW_out / dW_in operand A: the batch entries (sparse A, ocf.h a_sparse; no dense [B][N] arrays,
        # no memsets: row lists for the row-stream kernel, or LDS-filled tiles for the MFMA kernels) or
        # the dense d_out / xin.  With the MFMA kernels the sparse fill pays a chain of dependent index
        # loads per K-step and lost beyond K = 512 (8-way feature-parallel rank step 0.46 vs 0.375 ms);
        # the row-stream kernel has no K-loop and wins up to K = 4,096, the row lists' limit (ML-20M at
        # B = 4,096: 2.14 vs 3.31 ms/step with the dense-operand MFMA GEMMs); it takes first / last layers
        # of up to 512 hidden units
        rows_ok = max(self.Hp[0], self.Hp[-1]) <= 512
        self.sparse_dw = Bp <= (4096 if rows_ok else 2048 if self.cdt != _lib.DT_F32 else 512)
        # ... and as row lists (per weight row: the batch's entries in that column) for the row-stream kernel
        # (ocf_rows_dw.h): one wave per live weight row streams whole parameter / slot rows and forms the
        # row's gradient from its entries, no MFMA over the mostly-zero batch operand.  ML-20M step 0.50 ->
        # 0.44 ms against the role-split MFMA kernel on per-batch tile buckets (that sparse path is gone: the
        # row lists serve every sparse first / last layer of up to 512 hidden units, fp32 and 16-bit).

        self.tb = None
        # one hidden layer, one GPU: the decoder gather applies the hidden layer's epilogue to the encoder's
        # chunk partials (no separate row-reduce launch between the two gathers)
        self.fuse_enc_epilogue = True
        self._enc_fused = None
        # row skipping (ocf.h OcfGemmArgs row_tag): the scatter tags the columns holding a live input /
        # live target with the step's tag (cycling 1..255, no clearing); with Adagrad and l2 = 0 the
        # role-split dW kernels skip the parameter / slot / shadow traffic of the untagged rows, whose
        # update is the identity (zero gradient).  Bit-identical to the full update.
        self.row_skip = True        # (epoch row lists: records only for batches of < 2 entries per weight row
        #                             on average; "always": records whatever the density)
        self.rtag = [torch.zeros(self.Np, device=d, dtype=torch.uint8) for _ in range(2)]   # inputs, targets
        # per 128-row tile: the live rows (ocf.h OCF_LIVE_REC), built by ocf_sparse_tiles from the tags
        self.live_rec = [torch.zeros(self.Np // TILE * _lib.LIVE_REC, device=d, dtype=torch.uint8) for _ in range(2)]
        self._rtag_val = 0
        self._rtag_live = False
        self._stats_pending = None
        self._gbuf = {}
        HpL = self.Hp[-1]
        self.db_rows = torch.zeros(Bp, HpL, device=d, dtype=torch.float32)      # hidden-bias grad rows
        self.dh_raw = torch.zeros(Bp, HpL, device=d, dtype=torch.float32)       # decoder RAW reduce target
        self.stats_rows = torch.zeros(Bp, 4, device=d, dtype=torch.float32)
        self.row_sse_rows = torch.zeros(Bp, device=d, dtype=torch.float32)
        self.db_out_col = torch.zeros(1, self.Np, device=d, dtype=torch.float32)
        gm = Bp // TILE
        self.stats_part = torch.zeros(self.n_tiles * gm * 4, device=d, dtype=torch.float32)
        self.row_sse_part = torch.zeros(self.n_tiles * Bp, device=d, dtype=torch.float32)
        self.stats_cap = 0
        self.stats_hist = None
        self._grow_stats(64)
        self.n_stats = 0
        self.dense_in = None
        self.timers = None          # {phase: [(start_event, end_event), ...]} when profiling
        self.timer_only = None
        # side stream for the small kernels that do not feed the next GEMM (stats, bias updates, the
        # delta split-K reduction): they overlap the weight-gradient GEMMs instead of adding kernel
        # boundaries to the main chain.  Joined at the end of every step.
        self.side = torch.cuda.Stream(device=d) if d.type == "cuda" else None
        self._side_busy = False
        # generator batches: the row lists come from the generator's per-epoch build (BatchGenerator.
        # prepare_row_lists) instead of the per-step ocf_row_lists launches
        # (False: per-step ocf_scatter_batch + ocf_row_lists, for a batch source without an epoch plan;
        # bit-identical, tests/test_rows_dw_gpu.py, and oracle-checked, tests/test_semantics_gpu.py)
        self.epoch_row_lists = True
        self.epoch_scatter = True   # ... and their scatter outputs
        # fused single-GPU step: the decoder's δh row reduction as jobs of the dW_out launch
        self.fold_reduce = True
        self._reduce_job = None
        # ... or done in the decoder launch itself by the last chunk of each batch row (OcfGatherArgs jr /
        # row_arrive: a per-row arrival counter the launch leaves at zero): None = on small weights, where
        # ocf_gemm_pair's dual-row form then runs both updates without waiting for it; True / False forced
        self.reduce_in_decoder = None
        self._dec_reduced = False
        self.row_arrive = torch.zeros(Bp, device=d, dtype=torch.int32)
        # the encoder and the decoder as one launch (ocf_gather_encdec) where the decoder does the hidden epilogue and
        # the row reduction on the encoder's own chunk table; per-row encoder arrival counters.  None: on large
        # weights (ML-20M 0.3882 -> 0.3855 ms/step; ML-1M 0.0778 -> 0.0788, ML-100K 0.0490 -> 0.0487: the encoder
        # chunks run at the decoder's 163 VGPRs there; profiles/r05_cfg/encdec*.jsonl)
        self.fuse_enc_dec = None
        self.enc_arrive = torch.zeros(Bp, device=d, dtype=torch.int32)
        # the encoder over column tiles on the matrix cores (ocf_encoder_tiles): None = where weight rows carry
        # many entries (ENC_TILES_MIN_ENTRIES), True / False forced
        self.enc_tiles = None
        self._enc_tiles_used = False
        self.enc_tiles_count = 0      # (diagnostics: ocf_encoder_tiles launches)
        # a decoder chunk that gives up (OCF_ASYNC_ENC_WAIT) leaves both counters at zero itself; an encoder chunk
        # arriving after that give-up would not, so the counters are cleared when the error is reported
        _lib.enc_wait_hooks.append(_counter_reset(self))
        # ... and dW_out + dW_in as one launch (ocf_gemm_pair: a device word the launches count up, never
        # cleared, and its host-side running count)
        self.pair_dw = True
        self.pair_sync = torch.zeros(1, device=d, dtype=torch.int64)
        self.pair_state = _lib.OcfPairSync(ptr(self.pair_sync), 0)
        self._fused_step = False
        self._live_ptrs = None
        if self.comm is not None:   # feature parallel: reduced pre-activations, summed over ranks
            self.hpre = torch.zeros(Bp, self.Hp[0], device=d, dtype=torch.float32)
            self.dhpre = torch.zeros(Bp, self.Hp[-1], device=d, dtype=torch.float32)
            self.zero_bias = torch.zeros(max(self.Hp), device=d, dtype=torch.float32)

    # ---------------------------------------------------------------- phase timing (bench.py)
    def enable_timers(self, on=True, only=None):
        """HIP-event timing of phases (every phase, or the names in `only`).  The previous timers' events go
        back to a pool (creating an event costs HIP calls: none is created in bench.py's timed region)."""
        pool = self.__dict__.setdefault("_ev_pool", [])
        for v in (self.timers or {}).values():
            for a, b in v:
                pool += (a, b)
        self.timers = {} if on else None
        self.timer_only = set(only) if only else None

    def _timing_event(self):
        pool = self.__dict__.get("_ev_pool")
        if pool:
            return pool.pop()
        # (hipEventDisableSystemFence: a torch.cuda.Event record idled the stream ~5.7 us for its system-scope
        # cache write-back / invalidate and left the timed launch a cold L2)
        return _lib.TimingEvent()

    class _Phase:
        def __init__(self, eng, name):
            self.eng, self.name = eng, name

        def __enter__(self):
            e = self.eng
            self.prev, e._active_phase = e.__dict__.get("_active_phase"), self
            self.on = e.timers is not None and (e.timer_only is None or self.name in e.timer_only)
            if self.on:
                self.s = e._timing_event()
                self.s.record()
            return self

        def __exit__(self, *exc):
            self.eng._active_phase = self.prev
            if self.on:
                e = self.eng._timing_event()
                e.record()
                self.eng.timers.setdefault(self.name, []).append((self.s, e))
            return False

        def restart(self):
            """the phase's interval starts here (work issued since its start belongs to another phase)"""
            if self.on:
                self.s.record()

        def drop(self):
            """nothing of this phase was issued: no interval is recorded"""
            if self.on:
                self.on = False
                self.eng.__dict__.setdefault("_ev_pool", []).append(self.s)

    def phase(self, name):
        return Engine._Phase(self, name)

    # ---------------------------------------------------------------- side stream
    # one reusable event per direction: a stream wait takes the event's latest record at the time of the wait
    # call, so re-recording it for the next fork / join is safe (creating an event per fork cost ~15 us of
    # host time, twice per feature-parallel step)
    def _sync_event(self, name):
        ev = getattr(self, name, None)
        if ev is None:
            ev = torch.cuda.Event()          # timing disabled (the default): a plain sync event
            setattr(self, name, ev)
        return ev

    def _fork(self):
        """side stream waits for everything issued so far on the current stream"""
        ev = self._sync_event("_ev_fork")
        ev.record()
        self.side.wait_event(ev)
        self._side_busy = True

    def _join(self):
        """current stream waits for the side stream"""
        if self._side_busy:
            ev = self._sync_event("_ev_join")
            ev.record(self.side)
            torch.cuda.current_stream().wait_event(ev)
            self._side_busy = False

    def phase_times_ms(self, skip=0):
        """mean / total milliseconds per phase (call after synchronize), dropping the first `skip`
        launches of each phase."""
        out = {}
        for k, v in (self.timers or {}).items():
            ts = [a.elapsed_time(b) for a, b in v[skip:]] or [a.elapsed_time(b) for a, b in v]
            out[k] = {"mean_ms": float(np.mean(ts)), "total_ms": float(np.sum(ts)), "n": len(ts)}
        return out

    def _pick_splits_hidden(self, K, N):
        """split-K factor of a hidden -> hidden GEMM [Bp][K] x [K][N]: 1 (fused epilogue) when it has 16+
        output tiles, else one K-step per workgroup (up to 64 workgroups)"""
        bk = 32 if self.cdt == _lib.DT_F32 else 64
        tiles = (self.Bp // TILE) * (N // TILE)
        if tiles >= 16:
            return 1
        ks = K // bk
        s = max(1, min(ks, 64 // tiles))
        while ks % s:
            s -= 1
        return s

    def _pick_splits(self, K, Hp):
        bk = 32 if self.cdt == _lib.DT_F32 else 64
        ksteps = K // bk
        tiles = (self.Bp // TILE) * (Hp // TILE)
        if ksteps < 64 and tiles < 16:
            # a short K-loop over few tiles (Jester's 200-wide input): one or two K-steps per workgroup
            return self._pick_splits_hidden(K, Hp)
        s = max(1, min(ksteps // 8, max(1, 512 // tiles)))
        return s

    def _buf(self, name, n, dtype=torch.float32):
        """grow-only device scratch, with 1/4 headroom: per-batch sizes (entries, chunks) vary by a few
        percent, and every new maximum cost a zero-fill kernel inside the step"""
        t = self._gbuf.get(name)
        if t is None or t.numel() < n:
            t = torch.zeros(max(n + n // 4, 1 << 12), device=self.dev, dtype=dtype)
            self._gbuf[name] = t
            self._bufgen += 1          # the one-call step's template holds the old pointers
        return t

    def _grow_buckets(self, n):
        if n <= self.bk_cap:
            return
        cap = max(n, 2 * self.bk_cap)
        self.bk_rc = torch.zeros(cap, device=self.dev, dtype=torch.int32)
        self.bk_t = torch.zeros(cap, device=self.dev, dtype=torch.float32)
        self.bk_m = torch.zeros(cap, device=self.dev, dtype=torch.float32)
        self.bk_cap = cap

    def _grow_stats(self, n):
        if n <= self.stats_cap:
            return
        # at least STATS_MIN_ROWS: every growth re-records the one-call step's template (two general steps),
        # and a doubling from a handful of rows did that three times in the first 40 steps
        cap = max(n, 2 * self.stats_cap, self.STATS_MIN_ROWS)
        new = torch.zeros(cap, 4 + self.Bp, device=self.dev, dtype=torch.float32)
        # l2 penalty per step: [cap][2] = (column-sharded kernels, replicated kernels)
        pen = torch.zeros(cap, 2, device=self.dev, dtype=torch.float32)
        if self.stats_hist is not None and self.n_stats:
            new[: self.n_stats] = self.stats_hist[: self.n_stats]
            pen[: self.n_stats] = self.pen_hist[: self.n_stats]
        self.stats_hist = new
        self.pen_hist = pen
        self.stats_cap = cap

    STATS_MIN_ROWS = 1024

    def _l2_penalty(self):
        """Keras adds l2 * sum(W^2) of every kernel with a W_regularizer (all of them,
        /root/reference/model.py:66,82) to the logged loss, at the weights the batch starts from.
        Under feature parallelism the first and last kernels are column shards (summed over the
        ranks in take_stats), the hidden ones replicas (counted once)."""
        self._grow_stats(self.n_stats + 1)
        ws = self._buf("sumsq_ws", 1024)
        for i, w in enumerate(self.W):
            sharded = self.comm is not None and i in (0, len(self.W) - 1)
            dst = self.pen_hist[self.n_stats, 0 if sharded else 1:]
            call("ocf_sumsq", ptr(w), w.numel(), self.l2, ptr(ws), ptr(dst), cur_stream())

    # ---------------------------------------------------------------- batch assembly
    def scatter_args(self):
        """K1 arguments onto this engine's layer-0 input; target bucketing is added by load_dense's
        path only (generator batches use the row-segment mode, see load_batch)."""
        a = OcfScatterArgs()
        a.B = self.B
        a.B_pad = self.Bp
        a.N = self.N
        a.xin = ptr(self.xin)
        a.xin_dtype = self.cdt
        a.xin_ld = self.pad_dims[0]
        a.xin_block = self.Np
        a.tile_cnt = ptr(self.tile_cnt)
        a.bk_ptr = ptr(self.bk_ptr)
        a.bk_cur = ptr(self.bk_cur)
        a.bk_rc = ptr(self.bk_rc)
        a.bk_t = ptr(self.bk_t)
        a.bk_m = ptr(self.bk_m)
        a.n_tiles = self.n_tiles
        a.s0 = a.s1 = 1.0
        return a

    def load_batch(self, a, targets, gather=None):
        """K1 scatter for a batch described by OcfScatterArgs (pointers filled by the caller).

        ``targets`` (BatchGenerator.targets) names the target CSR's tile index: the scatter marks
        each target entry live/dead in self.tflag and the masked-MSE epilogue reads every batch
        row's segment per column tile directly -- no bucketing pass, no atomics."""
        if targets["t_ntiles"] != self.n_tiles:
            raise ValueError("target tile index has %d tiles, engine %d" % (targets["t_ntiles"], self.n_tiles))
        self.rows_real = None
        self._pending_pack = self._mlp_batch = None     # the scatter writes this batch's layer-0 input
        if targets["E"] > self.tflag.numel():
            self.tflag = torch.zeros(max(targets["E"], 2 * self.tflag.numel()), device=self.dev, dtype=torch.uint8)
        a.tile_cnt = a.bk_ptr = a.bk_cur = a.bk_rc = a.bk_t = a.bk_m = None
        a.tflag1 = ptr(self.tflag) if targets["flag"] == 1 else None
        a.tflag2 = ptr(self.tflag) if targets["flag"] == 2 else None
        seg = {k: v for k, v in targets.items() if k.startswith("t_")}
        seg["t_flag"] = self.tflag
        self.tseg = seg
        self.gt = None
        self._enc_fused = None
        a.tb_cnt, a.tb_nk = None, 0
        a.col_cnt = a.ecb = None
        lists = False
        epoch_lists = None
        epoch_entries = None
        a.rtag_in = a.rtag_out = None
        self._rtag_live = False
        self._live_ptrs = None
        if gather is not None and self.sparse_ok and self.use_sparse:
            xval = self._buf("xval", int(a.E1))
            a.xval1 = ptr(xval)
            if self.sparse_dw and targets["flag"] == 1:   # train split: inputs = targets
                rl = gather.get("row_lists") if self.epoch_row_lists else None
                if rl is not None:
                    # the epoch's row lists and live records, built once per epoch by the generator
                    # (ocf_epoch_row_lists): no per-step counting, keys or tags
                    t = rl(self.Np)
                    epoch_lists = dict(sp_rowptr=t["row_ptr"], sp_rowent=t["row_ent"], sp_nent=int(a.E1))
                    # live-row records only where rows go without entries: with >= 2 entries per weight row
                    # on average (ML-1M, ML-100K, feature-parallel global batches) nearly every row is live
                    # and the records' two dependent loads would only lengthen each wave's index chain
                    self._live_ptrs = (t["live"], t["live"]) if (
                        self.row_skip == "always" or (self.row_skip and not gather.get("rows_dense"))) else None
                    # ... and the batch's scatter outputs (ocf_epoch_scatter): no per-step scatter
                    if self.epoch_scatter:
                        epoch_entries = dict(xval=t["xval"], flag=t["tflag"])
                else:
                    # per-column counts and entry keys from the scatter -> row lists (ocf_row_lists)
                    a.col_cnt = ptr(self._buf("col_cnt", self.Np, torch.int32))
                    a.ecb = ptr(self._buf("ecb", int(a.E1), torch.int32))
                    lists = True
                if self.row_skip and epoch_lists is None:
                    self._rtag_val = self._rtag_val % 255 + 1
                    a.rtag_in, a.rtag_out, a.rtag = ptr(self.rtag[0]), ptr(self.rtag[1]), self._rtag_val
                    self._rtag_live = True
                    self._live_ptrs = (ptr(self.live_rec[0]), ptr(self.live_rec[1]))
                elif self._live_ptrs is not None:
                    self._rtag_live = True
            if self.sparse_dw:
                a.xin = None          # no dense layer-0 input: encoder and dW_in read the entries
            self.gt = dict(gather, xval=xval, aux=float(targets["t_aux"]), E=int(targets["E"]))
            if epoch_entries is not None:
                self.gt.update(epoch_entries)
        with self.phase("scatter"):
            if epoch_entries is None:
                a.xin_clean = int(self._xin_clean)
                call("ocf_scatter_batch", a, cur_stream())
            if epoch_lists is not None:
                self.tb = epoch_lists
            else:
                self.tb = self._row_lists(int(a.E1)) if lists else None
        self._xin_clean = False

    def _row_lists(self, E):
        """the batch's entries grouped by weight row (ocf_row_lists, from the scatter's per-column counts)
        for the row-stream weight-gradient kernel; shared by dW_out (deltas) and dW_in (inputs)"""
        a = _lib.OcfRowListArgs()
        a.ecb, a.E = ptr(self._buf("ecb", E, torch.int32)), E
        a.col_cnt, a.cursor = ptr(self._buf("col_cnt", self.Np, torch.int32)), ptr(self._buf("rl_cur", 3 * self.Np + 256, torch.int32))
        a.n_cols = self.Np
        rptr = self._buf("tb_rowptr", self.Np + 1, torch.int32)
        rent = self._buf("tb_rowent", 2 * max(E, 1), torch.int32)
        a.row_ptr, a.row_ent = ptr(rptr), ptr(rent)
        if self._rtag_live:
            a.rtag_in, a.rtag_out, a.rtag = ptr(self.rtag[0]), ptr(self.rtag[1]), self._rtag_val
            a.live_in, a.live_out = ptr(self.live_rec[0]), ptr(self.live_rec[1])
        call("ocf_row_lists", a, cur_stream())
        return dict(sp_rowptr=rptr, sp_rowent=rent, sp_nent=E)

    def load_dense(self, inputs, out_mask, targets, rows=None, rows_real=None):
        """API path: dense arrays in the model.py input order.  rows (device int64 [B]): the batch is rows
        `rows` of device-resident fp32 [n][ld] arrays (Model.fit uploads its arrays once), gathered by the
        packing and target kernels -- no per-step copy and no host synchronisation; otherwise [B, N]
        host or device arrays are staged into one device buffer first.  rows_real: the batch's real row
        count when its last rows are all-zero padding (Keras' trailing partial batch): the MSE's 2/(b N)."""
        B, N = self.B, self.N
        if rows_real is not None and not (1 <= int(rows_real) <= B):
            raise ValueError("load_dense: rows_real must be in [1, %d]" % B)
        self.rows_real = None if rows_real is None or int(rows_real) == B else int(rows_real)
        s = cur_stream()
        if rows is not None:
            srcs = list(inputs) + [out_mask, targets]
            ld = srcs[0].stride(0)
            for t in srcs:
                if not (torch.is_tensor(t) and t.is_cuda and t.dtype == torch.float32 and t.dim() == 2
                        and t.shape[1] == N and t.stride(0) == ld and t.stride(1) == 1):
                    raise ValueError("load_dense(rows=...): device fp32 [n, %d] arrays with one row stride" % N)
            if rows.numel() != B or rows.dtype != torch.int64 or not rows.is_cuda:
                raise ValueError("load_dense(rows=...): rows must be %d device int64 indices" % B)
            p = [ptr(t) for t in inputs] + [None] * (3 - len(inputs))
            # packed into xin when a layer-wise path needs it (forward); the fused small-model step
            # (ocf_mlp_step) gathers the rows itself
            self._pending_pack = (p, ld, ptr(rows))
            T, M, rp = targets, out_mask, ptr(rows)
            self._mlp_batch = (p, ld, ptr(rows), ptr(out_mask), ptr(targets))
        else:
            if self.dense_in is None:
                self.dense_in = torch.zeros(5, self.B, self.Np, device=self.dev, dtype=torch.float32)
            buf = self.dense_in
            buf.zero_()
            srcs = list(inputs) + [out_mask, targets]
            for i, src in enumerate(srcs):
                t = torch.as_tensor(np.asarray(src) if not torch.is_tensor(src) else src)
                if tuple(t.shape) != (B, N):
                    raise ValueError("input %d has shape %s, expected (%d, %d)" % (i, tuple(t.shape), B, N))
                slot = i if i < len(inputs) else (3 if src is out_mask else 4)
                buf[slot, :, :N] = t.to(self.dev, torch.float32)
            p0 = ptr(buf[0])
            p1 = ptr(buf[1]) if len(inputs) > 1 else None
            p2 = ptr(buf[2]) if len(inputs) > 2 else None
            call("ocf_pack_input", p0, p1, p2, self.Np, B, N, ptr(self.xin), self.cdt, self.pad_dims[0], self.Np,
                 self.Bp, None, s)
            T, M, rp, ld = buf[4], buf[3], None, self.Np
            self._pending_pack = self._mlp_batch = None
        self._xin_clean = False      # xin written densely
        self.tb = None
        self.gt = None                 # dense batch: the GEMM path, never a previous batch's gather tables
        self._enc_fused = None
        # the masked-MSE epilogue reads the dense targets / output masks directly (no bucket pass); keep
        # the arrays alive while the step is queued
        self.tseg = dict(dn_t=ptr(T), dn_m=ptr(M), ld_dn=ld, dn_rows=rp, n_real=N)
        self._dense_keep = (T, M, rows)

    def _pack_pending(self):
        """ocf_pack_input for a row-gathered dense batch whose packing load_dense deferred"""
        pp = self._pending_pack
        if pp is not None:
            p, ld, rp = pp
            call("ocf_pack_input", p[0], p[1], p[2], ld, self.B, self.N, ptr(self.xin), self.cdt, self.pad_dims[0],
                 self.Np, self.Bp, rp, cur_stream())
            self._pending_pack = None

    # ---------------------------------------------------------------- fused small-model step
    # A small dense model (train_jester.py: 0.14 M parameters, batch 128) on a row-gathered dense batch
    # (Model.fit) takes ONE persistent launch for the whole step (ocf.h ocf_mlp_step) instead of the
    # layer-wise path's ~14 latency-bound launches.  No l2, every layer trainable, one GPU.  (Generator batches
    # of the small I-AutoRec models through it, on the dense data_gen arrays, were exact but slower than the
    # row gathers -- ML-100K 0.089 vs 0.051 ms, ML-1M 0.39 vs 0.079 -- and were removed in round 5.)
    MLP_MAX_PARAMS = 4 << 20

    def _mlp_static_ok(self):
        return (self.fused_mlp and self.comm is None and self.dp_world == 1
                and not self.l2 and all(self.trainable) and self.grad_hook is None and self.master_sync is None
                and self.Bp <= 512 and self.opt is not None and self.opt.kind != _lib.OPT_SGD
                and sum(w.numel() for w in self.W) <= self.MLP_MAX_PARAMS)

    def _mlp_ok(self):
        return self._mlp_batch is not None and self._pending_pack is not None and self._mlp_static_ok()

    def _mlp_step(self):
        a = self._mlp_args
        if a is None:
            a = _lib.OcfMlpStepArgs()
            L = len(self.H)
            a.n_hidden, a.Bp, a.N, a.Np, a.k_blocks = L, self.Bp, self.N, self.Np, self.k
            for i, h in enumerate(self.H):
                a.hidden[i], a.hidden_p[i] = h, self.Hp[i]
            for i in range(L + 1):
                sw, sb = self.slots[i]
                a.W[i], a.b[i] = ptr(self.W[i]), ptr(self.b[i])
                a.sW1[i], a.sW2[i], a.sb1[i], a.sb2[i] = ptr(sw[0]), ptr(sw[1]), ptr(sb[0]), ptr(sb[1])
                a.shadow[i] = ptr(self.Wsh[i])
            a.shadow_blocked = int(self.shadow_blocked)
            a.act, a.compute_dtype = self.act, self.cdt
            a.keep = self.keep                     # (dropout scratch is part of the workspace)
            n = _lib.load().ocf_mlp_step_workspace(a)
            if n < 0:
                raise _lib.OcfError("ocf_mlp_step_workspace: " + _lib.load().ocf_last_error().decode())
            self._mlp_work = torch.empty(max(int(n), 1), dtype=torch.uint8, device=self.dev)
            self._mlp_bar = torch.zeros(2, dtype=torch.int32, device=self.dev)
            a.work, a.work_bytes, a.barrier = ptr(self._mlp_work), int(n), ptr(self._mlp_bar)
            self._mlp_args = a
        p, ld, rp, om, tg = self._mlp_batch
        a.B = self.rows_real or self.B
        a.x[0], a.x[1], a.x[2] = p[0], p[1], p[2]
        a.ld_x, a.rows, a.out_mask, a.targets, a.ld_t = ld, rp, om, tg, ld
        a.keep, a.seed = self.keep, self.seed
        a.stream = (self.step_count * self.dp_world + self.dp_rank) * 16     # forward()'s dropout stream
        if self.keep < 1.0:
            for i in range(len(self.H)):
                a.mask[i] = ptr(self.mask[i])
        o = self.opt.step_params(2.0 / ((self.rows_real or self.B) * self.N_total), 0.0)
        a.opt = o
        a.trace = ptr(self.mlp_trace)          # (diagnostics: tools/mlp_trace.py)
        a.wgs = self.mlp_wgs
        self._grow_stats(self.n_stats + 1)
        a.stats = self._stats_row(self.n_stats)
        with self.phase("mlp_step"):
            call("ocf_mlp_step", a, cur_stream())
        self._pending_pack = None
        self._xin_clean = False
        self.n_stats += 1
        self.opt.iterations += 1
        self.step_count += 1

    # ---------------------------------------------------------------- GEMM helper
    def _gemm(self, A, a_col, lda, Bm, b_dtype, b_col, ldb, M, N, K, epi, **kw):
        g = OcfGemmArgs()
        g.compute_dtype = self.cdt
        g.A = ptr(A)
        g.a_dtype = self.cdt
        g.a_col = a_col
        g.lda = lda
        g.B = ptr(Bm)
        g.b_dtype = b_dtype
        g.b_col = b_col
        g.ldb = ldb
        g.M, g.N, g.K = M, N, K
        g.splits = kw.pop("splits", 1)
        g.order = kw.pop("order", 0)
        g.epi = epi
        g.keep = 1.0
        issue = kw.pop("_issue", True)
        T = torch.Tensor
        for k, v in kw.items():
            setattr(g, k, v.data_ptr() if isinstance(v, T) else v)
        if not issue:
            return g
        call("ocf_gemm", g, cur_stream())

    # ---------------------------------------------------------------- forward
    def forward(self, training):
        """Encoder stack; leaves h[-1] (compute dtype) for the output layer."""
        self._pack_pending()
        s = cur_stream()
        Bp, L = self.Bp, len(self.H)
        keep = self.keep if training else 1.0
        stream_id = ((self.step_count * self.dp_world + self.dp_rank) * 16) if training else 0
        # layer 0: split-K over the (k x Np)-wide input
        Hp0 = self.Hp[0]
        sstride = Bp * Hp0
        if self.gt is not None:
            self._forward_gather(keep, stream_id)
        else:
            with self.phase("enc_gemm"):
                self._gemm(self.xin, 0, self.pad_dims[0], *self._wop(0), 1, Hp0, Bp, Hp0, self.pad_dims[0],
                           _lib.EPI_SLAB, splits=self.splits0, out=self.slabs, ld_out=Hp0, split_stride=sstride,
                           b_blocked=self._wblk(0))
        src, nsplit = self.slabs, self.splits0
        if self.gt is not None and self.comm is None:
            pass                      # fused bias/activation/dropout already applied by the row reduce
        elif self.gt is not None:
            with self.phase("allreduce_fwd"):
                self.comm(self.hpre)
            call("ocf_splitk_bias_act", ptr(self.hpre), 1, sstride, Bp, Hp0, Hp0, ptr(self.b[0]), self.act,
                 keep, self.seed, stream_id, None, ptr(self.mask[0]) if keep < 1 else None, ptr(self.a[0]),
                 ptr(self.h[0]), self.cdt, self.B, self.H[0], s)
        elif self.comm is not None:
            # partial pre-activation over this rank's columns -> sum over ranks -> activation
            call("ocf_splitk_bias_act", ptr(self.slabs), self.splits0, sstride, Bp, Hp0, Hp0, ptr(self.zero_bias),
                 _lib.ACT["linear"], 1.0, 0, 0, None, None, ptr(self.hpre), None, self.cdt, Bp, Hp0, s)
            with self.phase("allreduce_fwd"):
                self.comm(self.hpre)
            src, nsplit = self.hpre, 1
        if self.gt is None:
            call("ocf_splitk_bias_act", ptr(src), nsplit, sstride, Bp, Hp0, Hp0, ptr(self.b[0]), self.act,
                 keep, self.seed, stream_id, None, ptr(self.mask[0]) if keep < 1 else None, ptr(self.a[0]),
                 ptr(self.h[0]), self.cdt, self.B, self.H[0], s)
        for i in range(1, L):
            sp = self.splits_fwd[i]
            if sp > 1:
                st = Bp * self.Hp[i]
                self._gemm(self.h[i - 1], 0, self.Hp[i - 1], self.W[i], _lib.DT_F32, 1, self.Hp[i], Bp, self.Hp[i],
                           self.Hp[i - 1], _lib.EPI_SLAB, splits=sp, out=self.slabs, ld_out=self.Hp[i], split_stride=st)
                call("ocf_splitk_bias_act", ptr(self.slabs), sp, st, Bp, self.Hp[i], self.Hp[i], ptr(self.b[i]), self.act,
                     keep, self.seed, stream_id + i, None, ptr(self.mask[i]) if keep < 1 else None, ptr(self.a[i]),
                     ptr(self.h[i]), self.cdt, self.B, self.H[i], s)
                continue
            self._gemm(self.h[i - 1], 0, self.Hp[i - 1], self.W[i], _lib.DT_F32, 1, self.Hp[i], Bp, self.Hp[i],
                       self.Hp[i - 1], _lib.EPI_BIAS_ACT, bias=self.b[i], act=self.act, keep=keep, seed=self.seed,
                       stream=stream_id + i, mask_out=self.mask[i] if keep < 1 else None, a_out=self.a[i],
                       h_out=self.h[i], h_dtype=self.cdt, ld_out=self.Hp[i], m_real=self.B, n_real=self.H[i])

    # ---------------------------------------------------------------- row-gather (sparse batch) path
    def _gather_args(self, tab, layer, part, n_cols):
        g = _lib.OcfGatherArgs()
        for k in ("rows", "rp", "col", "val", "lboff", "ch_row", "ch_j0", "ch_j1", "n_chunks"):
            setattr(g, k, tab[k])
        Wt, wdt = self._wop(layer)
        g.W, g.w_dtype, g.ldw, g.w_blocked = ptr(Wt), wdt, Wt.shape[1], self._wblk(layer)
        g.H = n_cols
        g.part = ptr(part)
        return g

    def _reduce_args(self, tab, part, H, mode):
        r = _lib.OcfRowsReduceArgs()
        r.part, r.row_cptr, r.B, r.Bp, r.H, r.mode = ptr(part), tab["row_cptr"], self.B, self.Bp, H, mode
        return r

    def _enc_tiles_ok(self):
        """the encoder over column tiles (ocf_encoder_tiles) for this batch"""
        Wt, wdt = self._wop(0)
        # (train batches: the target view the kernel reads is then the input CSR's own, inputs = targets)
        if (self.k != 1 or wdt == _lib.DT_F32 or self._wblk(0) or self.tseg is None or "t_tptr" not in self.tseg
                or "row_lists" not in self.gt):
            return False
        if self.enc_tiles is not None:
            return bool(self.enc_tiles)
        return self.n_tiles >= ENC_TILES_MIN_TILES and self.gt["E"] >= ENC_TILES_MIN_ENTRIES * self.Np

    def _enc_splits(self, Hp0):
        n_rg, n_hs = -(-self.Bp // 256), Hp0 // 128
        S = max(1, min(self.n_tiles, round(ENC_TILES_WGS / (n_rg * n_hs))))
        if S > 8:                                           # whole groups of 8 splits (one per XCD)
            S = min(self.n_tiles, -(-S // 8) * 8)
        return S

    def _encoder_tiles(self, part_name, Hp0, xv):
        """ocf_encoder_tiles -> split-K partials [Bp][S][Hp0] and their row table (row_cptr[b] = b S)"""
        S = self._enc_splits(Hp0)
        part = self._buf(part_name, self.Bp * S * Hp0)
        t = self.tseg
        a = _lib.OcfEncTileArgs()
        a.rows, a.rp, a.tptr, a.tcol, a.tlidx, a.lboff = (t["t_rows"], t["t_rp"], ptr(t["t_tptr"]), ptr(t["t_col"]),
                                                          ptr(t["t_lidx"]), t["t_lboff"])
        a.xval = xv
        Wt, wdt = self._wop(0)
        a.W, a.ldw, a.w_dtype = ptr(Wt), Wt.shape[1], wdt
        a.B, a.Bp, a.n_tiles, a.H, a.splits, a.part = self.B, self.Bp, self.n_tiles, Hp0, S, ptr(part)
        a.nnz, a.n_entries = t["t_col"].numel(), max(int(self.gt["E"]), 1)
        a.max_row_len = max(int(t.get("t_maxlen", 0)), 1)
        nb = int(_lib.load().ocf_encoder_tiles_workspace(ctypes.byref(a)))
        if nb < 0:
            raise _lib.OcfError("ocf_encoder_tiles_workspace: bad arguments")
        w = self._buf("enc_tiles_work", -(-nb // 4), torch.int32)
        a.work, a.work_bytes = ptr(w), w.numel() * 4
        call("ocf_encoder_tiles", a, cur_stream())
        cp = self._gbuf.get("tile_cptr_%d" % S)
        if cp is None:
            cp = self._gbuf["tile_cptr_%d" % S] = torch.arange(0, (self.Bp + 1) * S, S, device=self.dev,
                                                                dtype=torch.int32)
        self._enc_tiles_used = True
        self.enc_tiles_count += 1
        return part, ptr(cp)

    def _forward_gather(self, keep, stream_id):
        """layer 0 as a row gather over the batch's live input entries + fused bias/act/dropout"""
        tab = self.gt["enc"]
        Hp0 = self.Hp[0]
        self._enc_tiles_used = False
        if self._enc_tiles_ok():
            with self.phase("enc_gemm"):
                xv = self.gt["xval"]
                part, cptr = self._encoder_tiles("part_enc", Hp0, xv if isinstance(xv, int) else ptr(xv))
                r = self._reduce_args(dict(tab, row_cptr=cptr), part, Hp0,
                                      _lib.REDUCE_RAW if self.comm is not None else _lib.REDUCE_BIAS_ACT)
                if self.comm is not None:        # partial over this rank's columns -> all-reduce
                    r.out = ptr(self.hpre)
                else:
                    r.bias, r.act, r.keep, r.seed, r.stream = ptr(self.b[0]), self.act, keep, self.seed, stream_id
                    r.mask_out = ptr(self.mask[0]) if keep < 1 else None
                    r.a_out, r.h_out, r.h_dtype, r.n_real = ptr(self.a[0]), ptr(self.h[0]), self.cdt, self.H[0]
                call("ocf_rows_reduce", r, cur_stream())
            return
        part = self._buf("part_enc", tab["n_chunks"] * Hp0)
        with self.phase("enc_gemm") as ph:
            g = self._gather_args(tab, 0, part, Hp0)
            xv = self.gt["xval"]
            g.xval = xv if isinstance(xv, int) else ptr(xv)
            if (self.comm is None and len(self.H) == 1 and self.fuse_enc_epilogue
                    and (self._rowres() or (tab.get("max_chunks", 0) <= FUSE_MAX_CHUNKS
                                            and tab["n_chunks"] <= FUSE_MEAN_CHUNKS * self.B))):
                # the decoder gather applies bias / activation / dropout to these partials itself; the encoder's
                # launch is deferred to the decoder's (one fused launch when the decoder can take it)
                self._enc_fused = dict(enc_part=ptr(part), enc_cptr=tab["row_cptr"], keep=keep, stream=stream_id,
                                       args=g, tab=tab)
                ph.drop()                        # (timed where it is launched: _output_gather)
                return
            call("ocf_gather_encoder", g, cur_stream())
            if self.comm is not None:            # partial over this rank's columns -> all-reduce
                r = self._reduce_args(tab, part, Hp0, _lib.REDUCE_RAW)
                r.out = ptr(self.hpre)
            else:
                r = self._reduce_args(tab, part, Hp0, _lib.REDUCE_BIAS_ACT)
                r.bias, r.act, r.keep, r.seed, r.stream = ptr(self.b[0]), self.act, keep, self.seed, stream_id
                r.mask_out = ptr(self.mask[0]) if keep < 1 else None
                r.a_out, r.h_out, r.h_dtype, r.n_real = ptr(self.a[0]), ptr(self.h[0]), self.cdt, self.H[0]
            call("ocf_rows_reduce", r, cur_stream())

    def _output_gather(self, with_grad, gscale):
        """decoder at the live targets: y, loss/metric sums, delta, and delta x W_out rows -> the last
        hidden layer's delta (through its activation and dropout) in the same pass"""
        L = len(self.H)
        HpL = self.Hp[L - 1]
        tab = self.gt["dec"]
        part = self._buf("part_dec", tab["n_chunks"] * HpL)
        cst = self._buf("chunk_stats", tab["n_chunks"] * 4)
        g = self._gather_args(tab, L, part, HpL)
        g.flag = self.gt.get("flag") or ptr(self.tflag)
        g.h, g.h_dtype, g.bias, g.aux = ptr(self.h[L - 1]), self.cdt, ptr(self.b[L]), self.gt["aux"]
        g.chunk_stats = ptr(cst)
        ef, self._enc_fused = self._enc_fused, None
        if ef is not None:
            g.enc_part, g.enc_cptr, g.keep, g.stream = ef["enc_part"], ef["enc_cptr"], ef["keep"], ef["stream"]
            g.bias_h, g.act, g.seed = ptr(self.b[0]), self.act, self.seed
            g.a_out, g.mask_out = ptr(self.a[0]), ptr(self.mask[0]) if ef["keep"] < 1 else None
            g.m_real, g.n_real = self.B, self.H[0]
        if with_grad and self.sparse_dw:
            g.delta_e = ptr(self._buf("delta_e", self.gt["E"]))
        elif with_grad:               # dense delta for the output-layer weight-gradient GEMM
            self.d_out.zero_()
            g.d_out, g.d_dtype, g.ld_d = ptr(self.d_out), self.cdt, self.Np
        if with_grad and self.comm is None:
            r = self._reduce_args(tab, part, HpL, _lib.REDUCE_GRAD_ACT)
            r.a_in = ptr(self.a[L - 1])
            r.mask_in = ptr(self.mask[L - 1]) if self.keep < 1 else None
            r.act, r.keep, r.h_out, r.h_dtype, r.n_real = self.act, self.keep, ptr(self.dh[L - 1]), self.cdt, self.H[L - 1]
            r.db_part, r.gscale = ptr(self.db_rows), gscale
        else:
            r = self._reduce_args(tab, part, HpL, _lib.REDUCE_RAW)
            r.out = ptr(self.dhpre if (with_grad and self.comm is not None) else self.dh_raw)
        r.chunk_stats, r.stats_part, r.row_sse = ptr(cst), ptr(self.stats_rows), ptr(self.row_sse_rows)
        self._reduce_job = None
        self._dec_reduced = False
        fold = (with_grad and self.comm is None and self._fused_step and self.fold_reduce and self._folds()
                and self.trainable[0])
        in_dec = self.reduce_in_decoder
        if in_dec is None:
            # one input block: ocf_gemm_pair's dual-row launch (ocf_rows_impl.h; both layers' rows share the row
            # lists), which needs the reduction done; large weights with k >= 2 inputs: the pair launch, whose
            # consumers then wait for nothing (ML-20M pair launch 311.6 -> 303.8 us, dual-row 299.8 us:
            # profiles/r05_dual_large/); small weights with k >= 2: two launches with the reduction riding in
            # the first (the measured round-4 form)
            in_dec = self.k == 1 or self.Np // TILE * 48 >= 8192
        if fold and in_dec and tab["n_chunks"] > 0:
            g.jr, g.row_arrive = ctypes.addressof(r), ptr(self.row_arrive)
            self._last_jr = r             # (kept alive: the recorded step's decoder arguments point at it)
            self._dec_reduced = True
        if ef is not None:
            ea, et = ef["args"], ef["tab"]
            # (the row-resident form runs on any weight size: ML-1M bf16 0.0711 -> 0.0587 ms/step, ML-1M U 0.0549 ->
            # 0.0441, same box, profiles/r06_rowres/; the chunked form only pays on large weights)
            fuse = self.fuse_enc_dec if self.fuse_enc_dec is not None else (
                self.Np // TILE * 48 >= 8192 or self._rowres())
            if (fuse and g.jr and et["ch_row"] == tab["ch_row"] and et["n_chunks"] == tab["n_chunks"]
                    and et["lboff"] == tab["lboff"]):
                # (one launch: the caller's dec_gemm_mse phase times both, enc_gemm records nothing)
                call("ocf_gather_encdec", ea, g, ptr(self.enc_arrive), cur_stream())
                return self._after_decoder(g, fold, r)
            dec_phase = self.__dict__.get("_active_phase")
            with self.phase("enc_gemm"):
                call("ocf_gather_encoder", ea, cur_stream())
            if dec_phase is not None:
                dec_phase.restart()
        call("ocf_gather_decoder", g, cur_stream())
        return self._after_decoder(g, fold, r)

    def _after_decoder(self, g, fold, r):
        if g.jr:
            pass                          # done by the decoder's last chunk of each row
        elif fold:
            self._reduce_job = r          # rides in the dW_out launch (OcfGemmArgs jr), see _backward_gather
            self._last_jr = r             # (kept alive: the recorded step's dW_out arguments point at it)
        else:
            call("ocf_rows_reduce", r, cur_stream())

    def output_loss(self, with_grad):
        """Decoder (dense GEMM with the fused masked-MSE epilogue, or the row gather for sparse
        batches); stats -> stats_hist[n_stats]."""
        L = len(self.H)
        gscale = 2.0 / ((self.rows_real or self.B) * self.N_total)
        with self.phase("dec_gemm_mse"):
            if self.gt is not None:
                self._output_gather(with_grad, gscale)
                sp, n_sp, rs, n_rs = self.stats_rows, self.Bp, self.row_sse_rows, 1
            else:
                self._gemm_mse(L, gscale, with_grad)
                sp, n_sp, rs, n_rs = self.stats_part, self.n_tiles * (self.Bp // TILE), self.row_sse_part, self.n_tiles
        self._grow_stats(self.n_stats + 1)
        dst = self.stats_hist[self.n_stats]
        if with_grad and self._folds():
            # finalized by the output-layer weight-gradient launch (OcfGemmArgs js_*)
            self._stats_pending = (sp, n_sp, rs, n_rs, self.Bp, dst)
        elif self.side is not None:
            self._fork()
            with torch.cuda.stream(self.side):
                call("ocf_stats_finalize", ptr(sp), n_sp, ptr(rs), n_rs, self.Bp, ptr(dst), cur_stream())
        else:
            call("ocf_stats_finalize", ptr(sp), n_sp, ptr(rs), n_rs, self.Bp, ptr(dst), cur_stream())
        self.n_stats += 1

    def _folds(self):
        """single-GPU row-gather step with the fused optimizer: the stats finalisation and both
        bias updates ride in the output-layer dW launch instead of side-stream kernels"""
        return (self.gt is not None and self.comm is None and len(self.H) == 1
                and self.sparse_dw and self.tb is not None and self.trainable[1])

    def _flush_stats(self):
        if self._stats_pending is not None:
            call("ocf_stats_finalize", *[ptr(x) if torch.is_tensor(x) else x for x in self._stats_pending],
                 cur_stream())
            self._stats_pending = None

    def _gemm_mse(self, L, gscale, with_grad):
        tg = self.tseg if self.tseg is not None else dict(bk_ptr=self.bk_ptr, bk_rc=self.bk_rc, bk_t=self.bk_t,
                                                          bk_m=self.bk_m)
        self._gemm(self.h[L - 1], 0, self.Hp[L - 1], *self._wop(L), 0, self.Hp[L - 1], self.Bp, self.Np,
                   self.Hp[L - 1], _lib.EPI_MASKED_MSE, order=1, bias=self.b[L], m_real=self.B, **tg,
                   b_blocked=self._wblk(L),
                   h_out=self.d_out if with_grad else None, h_dtype=self.cdt, ld_out=self.Np,
                   db_part=self.db_out_part if with_grad else None, ld_db=self.Np,
                   opt=_lib.OcfOptParams(0, 0, 0, 0, 0, 0, gscale),
                   stats_part=self.stats_part, row_sse_part=self.row_sse_part)

    def predict_dense(self, out_mask, out):
        """PREDICT epilogue: out[B][N] = out_mask * (h W + b)."""
        if self.master_sync is not None:
            self.master_sync()
        L = len(self.H)
        self._gemm(self.h[L - 1], 0, self.Hp[L - 1], self.W[L], _lib.DT_F32, 0, self.Hp[L - 1], self.Bp, self.Np,
                   self.Hp[L - 1], _lib.EPI_PREDICT, bias=self.b[L], pmask=out_mask,
                   ld_pmask=out_mask.stride(0) if out_mask is not None else 0, out=out, ld_out=out.stride(0),
                   m_real=self.B, n_real=self.N)

    # ---------------------------------------------------------------- backward + update
    def backward_update(self, grads_out=None):
        """Backward pass; with grads_out=None the optimizer is fused into the weight-gradient GEMMs
        (single GPU).  Otherwise raw gradients are written to grads_out (list matching params) and
        the caller all-reduces and calls apply_grads()."""
        s = cur_stream()
        L, Bp = len(self.H), self.Bp
        gscale = 2.0 / ((self.rows_real or self.B) * self.N_total)
        fused = grads_out is None
        op = self.opt.step_params(1.0, self.l2) if fused else None
        self._bias_op = self.opt.step_params(1.0, 0.0) if fused else None   # l2 regularises kernels only
        if self.gt is not None:
            return self._backward_gather(grads_out, op, gscale)
        # delta of the last hidden layer: split-K over Np
        HpL = self.Hp[L - 1]
        sstride = Bp * HpL
        with self.phase("dec_bwd_gemm"):
            self._gemm(self.d_out, 0, self.Np, *self._wop(L), 1, HpL, Bp, HpL, self.Np, _lib.EPI_SLAB,
                       splits=self.splitsL, out=self.slabs, ld_out=HpL, split_stride=sstride,
                       b_blocked=self._wblk(L))
        db_last = self.db_h[L - 1]
        src, nsplit = self.slabs, self.splitsL
        if fused and L == 1 and self.comm is None and self.side is not None:
            # side stream: delta reduction + both bias updates, overlapping the output-layer GEMM
            self._fork()
            with torch.cuda.stream(self.side):
                call("ocf_splitk_grad_act", ptr(src), nsplit, sstride, Bp, HpL, HpL, ptr(self.a[0]),
                     ptr(self.mask[0]), self.keep, self.act, ptr(self.dh[0]), self.cdt, ptr(db_last[0]), gscale,
                     self.B, self.H[0], cur_stream())
                self._bias_update(1, self.db_out_part, Bp // TILE, self.Np, self.Np, grads_out, op)
                self._bias_update(0, db_last, Bp // 4, self.Hp[0], self.Hp[0], grads_out, op)
            with self.phase("dW_out"):
                self._weight_update(1, self.d_out, self.Np, self.h[0], HpL, self.Np, HpL, gscale, grads_out, op)
            self._join()
            with self.phase("dW_in"):
                self._weight_update(0, self.xin, self.pad_dims[0], self.dh[0], self.Hp[0], self.pad_dims[0],
                                    self.Hp[0], gscale, grads_out, op)
            self.opt.iterations += 1
            return
        if self.comm is not None:
            call("ocf_splitk_bias_act", ptr(self.slabs), self.splitsL, sstride, Bp, HpL, HpL, ptr(self.zero_bias),
                 _lib.ACT["linear"], 1.0, 0, 0, None, None, ptr(self.dhpre), None, self.cdt, Bp, HpL, s)
            with self.phase("allreduce_bwd"):
                self.comm(self.dhpre)
            src, nsplit = self.dhpre, 1
        call("ocf_splitk_grad_act", ptr(src), nsplit, sstride, Bp, HpL, HpL, ptr(self.a[L - 1]),
             ptr(self.mask[L - 1]), self.keep, self.act, ptr(self.dh[L - 1]), self.cdt, ptr(db_last[0]), gscale,
             self.B, self.H[L - 1], s)
        # output layer bias + weights
        self._bias_update(L, self.db_out_part, Bp // TILE, self.Np, self.Np, grads_out, op)
        with self.phase("dW_out"):
            self._weight_update(L, self.d_out, self.Np, self.h[L - 1], HpL, self.Np, HpL, gscale, grads_out, op)
        self._grad_ready(L, grads_out)
        parts_last = Bp // 4
        for i in range(L - 1, 0, -1):
            # delta of hidden layer i-1 through W_i (before W_i changes)
            parts_next = self._hidden_delta(i, gscale)
            self._bias_update(i, self.db_h[i], parts_last, self.Hp[i], self.Hp[i], grads_out, op)
            self._weight_update(i, self.h[i - 1], self.Hp[i - 1], self.dh[i], self.Hp[i], self.Hp[i - 1],
                                self.Hp[i], gscale, grads_out, op)
            self._grad_ready(i, grads_out)
            parts_last = parts_next
        self._bias_update(0, self.db_h[0], parts_last, self.Hp[0], self.Hp[0], grads_out, op)
        with self.phase("dW_in"):
            self._weight_update(0, self.xin, self.pad_dims[0], self.dh[0], self.Hp[0], self.pad_dims[0],
                                self.Hp[0], gscale, grads_out, op)
        self._grad_ready(0, grads_out)
        if fused:
            self.opt.iterations += 1

    def _weight_update_sparse(self, i, vals, Bm, ldb, N, gscale, grads_out, op, colsum=None, jobs=None, issue=True):
        """EPI_OPTIM / EPI_GRAD for a first/last layer whose A operand (the batch entries: deltas or
        inputs, [B][N] transposed) is built in LDS from the target CSR's column-sorted view"""
        if grads_out is None and not self.trainable[i]:
            return
        M, K = self.Np, self.Bp
        if self.sparse_dw:
            t = self.tseg
            sp = dict(a_sparse=1, sp_rows=t["t_rows"], sp_rp=t["t_rp"], sp_tptr=t["t_tptr"], sp_col=t["t_col"],
                      sp_lidx=t["t_lidx"], sp_lboff=t["t_lboff"], sp_vals=vals, sp_ntiles=t["t_ntiles"],
                      sp_krows=self.B, sp_colsum=colsum, **(self.tb or {}))
            A = Bm                    # not read (sparse A); any valid pointer
        else:                         # dense operand: the decoder's delta or the scattered layer-0 input
            sp = dict(sp_colsum=colsum)
            A = self.d_out if i == len(self.W) - 1 else self.xin
        if grads_out is None:
            sw, _ = self.slots[i]
            o = _lib.OcfOptParams(op.kind, op.lr, op.eps, op.rho, op.beta2, op.l2, gscale)
            if self._rtag_live and self.sparse_dw and op.kind == _lib.OPT_ADAGRAD and op.l2 == 0:
                sp.update(row_live=self._live_ptrs[0 if i == 0 else 1])
            return self._gemm(A, 1, M, Bm, self.cdt, 1, ldb, M, N, K, _lib.EPI_OPTIM, p=self.W[i], s1=sw[0],
                              s2=sw[1], ld_out=N, opt=o, p_shadow=self.Wsh[i], shadow_blocked=self._wblk(i), **sp,
                              **(jobs or {}), _issue=issue)
        else:
            self._gemm(A, 1, M, Bm, self.cdt, 1, ldb, M, N, K, _lib.EPI_GRAD, out=grads_out[2 * i], ld_out=N,
                       opt=_lib.OcfOptParams(0, 0, 0, 0, 0, 0, gscale), h_dtype=self._grad_dt(grads_out[2 * i]),
                       **sp)

    def _backward_gather(self, grads_out, op, gscale):
        """backward after the row-gather decoder: the last hidden delta already exists (single GPU) or
        its partial sum does (feature parallel: all-reduce, then activation/dropout)"""
        s = cur_stream()
        L, Bp = len(self.H), self.Bp
        HpL = self.Hp[L - 1]
        fused = grads_out is None
        delta = self._buf("delta_e", self.gt["E"]) if self.sparse_dw else None
        xval = self.gt["xval"]
        out_done = False
        if self.comm is not None:
            start = getattr(self.comm, "start", None)
            if start is not None:
                # the output layer's update needs only the deltas and h, not the summed dh: it runs
                # while the all-reduce of the dh partials is in flight on the collective's stream
                work = start(self.dhpre)
                if self.side is not None:
                    # ... on the side stream, so the input layer's update (main stream, after the
                    # all-reduce) fills the CUs the output layer's last tiles leave idle
                    self._fork()
                    with torch.cuda.stream(self.side):
                        with self.phase("dW_out"):
                            self._weight_update_sparse(L, delta, self.h[L - 1], HpL, HpL, gscale, grads_out, op,
                                                       self.db_out_col)
                        self._bias_update(L, self.db_out_col, 1, self.Np, self.Np, grads_out, op)
                else:
                    with self.phase("dW_out"):
                        self._weight_update_sparse(L, delta, self.h[L - 1], HpL, HpL, gscale, grads_out, op,
                                                   self.db_out_col)
                    self._bias_update(L, self.db_out_col, 1, self.Np, self.Np, grads_out, op)
                out_done = True
                with self.phase("allreduce_bwd"):
                    work.wait()
            else:
                with self.phase("allreduce_bwd"):
                    self.comm(self.dhpre)
            call("ocf_splitk_grad_act", ptr(self.dhpre), 1, Bp * HpL, Bp, HpL, HpL, ptr(self.a[L - 1]),
                 ptr(self.mask[L - 1]), self.keep, self.act, ptr(self.dh[L - 1]), self.cdt, ptr(self.db_h[L - 1][0]),
                 gscale, self.B, self.H[L - 1], s)
            db_last, parts_last = self.db_h[L - 1], Bp // 4
        else:
            db_last, parts_last = self.db_rows, Bp
        if fused and self._folds():
            # dW_out also: output-bias gradient (column sums of the deltas) and its update, and -- when the
            # decoder's row reduction rides here too (jr: it writes δh, the hidden-bias rows and the stats
            # rows, which dW_out does not read) -- nothing else; the hidden-bias update from the δh rows
            # and the step's stats then ride in dW_in, after it.  Without jr all of them ride in dW_out.
            jobs_out, jobs_in = {}, {}
            if self.trainable[1]:
                sb = self.slots[1][1]
                jobs_out.update(cb_p=self.b[1], cb_s1=sb[0], cb_s2=sb[1], cb_op=self._bias_op)
            late = jobs_out
            if self._reduce_job is not None:
                jobs_out.update(jr=ctypes.addressof(self._reduce_job))
                late = jobs_in
            elif self._dec_reduced:         # (the decoder reduced: the same job layout, nothing to wait for)
                late = jobs_in
            if self.trainable[0]:
                sb = self.slots[0][1]
                late.update(jb_part=db_last, jb_parts=parts_last, jb_ld=HpL, jb_n=HpL, jb_p=self.b[0], jb_s1=sb[0],
                            jb_s2=sb[1], jb_op=self._bias_op)
            if self._stats_pending is not None:
                sp, n_sp, rs, n_rs, M, dst = self._stats_pending
                late.update(js_sp=sp, js_nparts=n_sp, js_rs=rs, js_ntiles=n_rs, js_M=M, js_out=dst)
                self._stats_pending = None
            if self.pair_dw:
                # both updates as one launch (ocf_gemm_pair): dW_in's workgroups wait in the kernel for the
                # row reduction riding in dW_out's, instead of a kernel boundary
                g_out = self._weight_update_sparse(1, delta, self.h[0], HpL, HpL, gscale, grads_out, op,
                                                   self.db_out_col, jobs=jobs_out, issue=False)
                g_in = self._weight_update_sparse(0, xval, self.dh[0], self.Hp[0], self.Hp[0], gscale, grads_out,
                                                  op, jobs=jobs_in, issue=False)
                with self.phase("dW_pair"):
                    call("ocf_gemm_pair", g_out, g_in, ctypes.addressof(self.pair_state), cur_stream())
            else:
                with self.phase("dW_out"):
                    self._weight_update_sparse(1, delta, self.h[0], HpL, HpL, gscale, grads_out, op,
                                               self.db_out_col, jobs=jobs_out)
                with self.phase("dW_in"):
                    self._weight_update_sparse(0, xval, self.dh[0], self.Hp[0], self.Hp[0], gscale, grads_out, op,
                                               jobs=jobs_in)
            self._reduce_job = None
            self.opt.iterations += 1
            return
        self._flush_stats()
        if fused and L == 1 and self.comm is None and self.side is not None:
            self._fork()
            with torch.cuda.stream(self.side):
                self._bias_update(0, db_last, parts_last, HpL, HpL, grads_out, op)
            with self.phase("dW_out"):        # also the output-bias gradient (column sums of the deltas)
                self._weight_update_sparse(1, delta, self.h[0], HpL, HpL, gscale, grads_out, op, self.db_out_col)
            self._fork()
            with torch.cuda.stream(self.side):
                self._bias_update(1, self.db_out_col, 1, self.Np, self.Np, grads_out, op)
            with self.phase("dW_in"):
                self._weight_update_sparse(0, xval, self.dh[0], self.Hp[0], self.Hp[0], gscale, grads_out, op)
            self.opt.iterations += 1
            return
        if not out_done:
            with self.phase("dW_out"):
                self._weight_update_sparse(L, delta, self.h[L - 1], HpL, HpL, gscale, grads_out, op,
                                           self.db_out_col)
            self._bias_update(L, self.db_out_col, 1, self.Np, self.Np, grads_out, op)
        self._grad_ready(L, grads_out)
        for i in range(L - 1, 0, -1):
            parts_next = self._hidden_delta(i, gscale)
            self._bias_update(i, db_last, parts_last, self.Hp[i], self.Hp[i], grads_out, op)
            self._weight_update(i, self.h[i - 1], self.Hp[i - 1], self.dh[i], self.Hp[i], self.Hp[i - 1],
                                self.Hp[i], gscale, grads_out, op)
            self._grad_ready(i, grads_out)
            db_last, parts_last = self.db_h[i - 1], parts_next
        jobs_in = None
        if fused and L == 1 and self.comm is not None and self.trainable[0]:
            # feature parallelism: the hidden-bias update from the δh partial rows rides in the input layer's
            # launch as a job (the same sums) instead of a kernel ahead of it on the critical path (8-way rank:
            # 512 partial rows, 40 us as a separate launch)
            sb = self.slots[0][1]
            jobs_in = dict(jb_part=db_last, jb_parts=parts_last, jb_ld=HpL, jb_n=HpL, jb_p=self.b[0], jb_s1=sb[0],
                           jb_s2=sb[1], jb_op=self._bias_op)
        else:
            self._bias_update(0, db_last, parts_last, self.Hp[0], self.Hp[0], grads_out, op)
        with self.phase("dW_in"):
            self._weight_update_sparse(0, xval, self.dh[0], self.Hp[0], self.Hp[0], gscale, grads_out, op,
                                       jobs=jobs_in)
        self._grad_ready(0, grads_out)
        if fused:
            self.opt.iterations += 1

    def _hidden_delta(self, i, gscale):
        """dh[i-1] = (dh[i] W_i^T) * act'(a[i-1]) * dropout, and the hidden bias' gradient partials db_h[i-1];
        returns how many partial rows db_h[i-1] holds (fused GRAD_ACT epilogue: one per 128-row tile;
        split-K reduction: one per 4 rows)"""
        Bp = self.Bp
        sp = self.splits_bwd[i]
        if sp > 1:
            st = Bp * self.Hp[i - 1]
            self._gemm(self.dh[i], 0, self.Hp[i], self.W[i], _lib.DT_F32, 0, self.Hp[i], Bp, self.Hp[i - 1], self.Hp[i],
                       _lib.EPI_SLAB, splits=sp, out=self.slabs, ld_out=self.Hp[i - 1], split_stride=st)
            call("ocf_splitk_grad_act", ptr(self.slabs), sp, st, Bp, self.Hp[i - 1], self.Hp[i - 1], ptr(self.a[i - 1]),
                 ptr(self.mask[i - 1]), self.keep, self.act, ptr(self.dh[i - 1]), self.cdt, ptr(self.db_h[i - 1][0]),
                 gscale, self.B, self.H[i - 1], cur_stream())
            return Bp // 4
        self._gemm(self.dh[i], 0, self.Hp[i], self.W[i], _lib.DT_F32, 0, self.Hp[i], Bp, self.Hp[i - 1],
                   self.Hp[i], _lib.EPI_GRAD_ACT, a_in=self.a[i - 1], mask_in=self.mask[i - 1], keep=self.keep,
                   act=self.act, h_out=self.dh[i - 1], h_dtype=self.cdt, ld_out=self.Hp[i - 1],
                   db_part=self.db_h[i - 1], opt=_lib.OcfOptParams(0, 0, 0, 0, 0, 0, gscale),
                   m_real=self.B, n_real=self.H[i - 1])
        return Bp // TILE

    def _bias_update(self, i, part, parts, ld, n, grads_out, op):
        if grads_out is None and not self.trainable[i]:
            return
        s = cur_stream()
        sw, sb = self.slots[i] if self.slots else ([None, None], [None, None])
        if grads_out is None:
            call("ocf_bias_opt_from_partials", ptr(self.b[i]), ptr(part), parts, ld, n, ptr(sb[0]), ptr(sb[1]),
                 None, self._bias_op, s)
        else:
            call("ocf_bias_opt_from_partials", ptr(self.b[i]), ptr(part), parts, ld, n, None, None,
                 ptr(grads_out[2 * i + 1]), _lib.OcfOptParams(), s)

    def _weight_update(self, i, A, lda, Bm, ldb, M, N, gscale, grads_out, op):
        if grads_out is None and not self.trainable[i]:
            return
        K = self.Bp
        if grads_out is None:
            sw, _ = self.slots[i]
            o = _lib.OcfOptParams(op.kind, op.lr, op.eps, op.rho, op.beta2, op.l2, gscale)
            self._gemm(A, 1, lda, Bm, self.cdt, 1, ldb, M, N, K, _lib.EPI_OPTIM, p=self.W[i], s1=sw[0], s2=sw[1],
                       ld_out=N, opt=o, p_shadow=self.Wsh[i], shadow_blocked=self._wblk(i))
        else:
            self._gemm(A, 1, lda, Bm, self.cdt, 1, ldb, M, N, K, _lib.EPI_GRAD, out=grads_out[2 * i], ld_out=N,
                       opt=_lib.OcfOptParams(0, 0, 0, 0, 0, 0, gscale), h_dtype=self._grad_dt(grads_out[2 * i]))

    @staticmethod
    def _grad_dt(g):
        if g.dtype == torch.bfloat16:
            return _lib.DT_BF16
        if g.dtype != torch.float32:
            raise ValueError("weight gradients are written in fp32 or bf16")
        return _lib.DT_F32

    def _grad_ready(self, i, grads_out):
        if grads_out is not None and self.grad_hook is not None:
            self.grad_hook(i)

    def apply_grads(self, grads, scale=1.0):
        """Elementwise optimizer over all parameters (after a data-parallel all-reduce)."""
        s = cur_stream()
        op = self.opt.step_params(scale, self.l2)
        for i in range(len(self.W)):
            if not self.trainable[i]:
                continue
            sw, sb = self.slots[i]
            call("ocf_opt_step", ptr(self.W[i]), ptr(grads[2 * i]), ptr(sw[0]), ptr(sw[1]), self.W[i].numel(), op, s)
            ob = self.opt.step_params(scale, 0.0)
            call("ocf_opt_step", ptr(self.b[i]), ptr(grads[2 * i + 1]), ptr(sb[0]), ptr(sb[1]), self.b[i].numel(), ob, s)
        self._refresh_shadows()
        self.opt.iterations += 1

    def grad_buffers(self):
        out = []
        for w, b in zip(self.W, self.b):
            out += [torch.zeros_like(w), torch.zeros_like(b)]
        return out

    # ---------------------------------------------------------------- steps
    def train_step(self, grads_out=None):
        if grads_out is None and self._mlp_ok():
            return self._mlp_step()
        self._fused_step = grads_out is None
        if self.l2:
            self._l2_penalty()
        self.forward(training=True)
        self.output_loss(with_grad=True)
        self.backward_update(grads_out)
        self._join()
        self.step_count += 1

    # ---------------------------------------------------------------- one-call training step
    # A step of the default single-GPU path (one hidden layer, generator batch, epoch row lists, the folded
    # jobs) is four library calls whose argument blocks differ from step to step only in the batch's table
    # pointers / sizes, the dropout stream, the stats slot and the optimizer constants.  Building the blocks
    # in Python costs ~0.07 ms per step -- as long as the whole GPU step of ML-100K / ML-1M.  So the blocks
    # of one recorded step become a template (ocf.h OcfRowStepArgs) and later steps rewrite only those
    # fields and issue ocf_train_step_rows.  The template is checked before use: a second recorded step
    # must equal the template rewritten for that step, byte for byte (any field that varies and is not
    # rewritten fails the check and the engine stays on the general path).
    _STEP_CALLS = (("ocf_gather_encoder", "ocf_gather_decoder", "ocf_gemm_pair"),
                   ("ocf_gather_encoder", "ocf_gather_decoder", "ocf_gemm", "ocf_gemm"),
                   ("ocf_gather_encdec", "ocf_gemm_pair"), ("ocf_gather_encdec", "ocf_gemm", "ocf_gemm"))
    # generator step fields (BatchGenerator.step_fields): rows, lboff, ch_row, ch_j0, ch_j1, n_chunks,
    # row_cptr, max_chunks, entries, row_ptr, row_ent, live, xval, tflag -> template fields
    _F_ROWS, _F_LBOFF, _F_CHR, _F_J0, _F_J1, _F_NCH, _F_CPTR, _F_MAXCH, _F_E, _F_RPTR, _F_RENT, _F_LIVE, \
        _F_XVAL, _F_TFLAG = range(14)
    _GATHER_FIELDS = (("rows", 0), ("lboff", 1), ("ch_row", 2), ("ch_j0", 3), ("ch_j1", 4), ("n_chunks", 5))
    _DW_FIELDS = (("sp_rows", 0), ("sp_lboff", 1), ("sp_nent", 8), ("sp_rowptr", 9), ("sp_rowent", 10))

    def _fast_key(self, gen):
        """identity of everything the template holds besides the per-step fields, or None when the step
        takes the general path"""
        tok = getattr(gen, "_step_token", None)
        if tok is None:
            from .data_reader import BatchGenerator
            if not (isinstance(gen, BatchGenerator) and gen.split == "train"):
                return None
            Engine._gen_tokens += 1
            tok = gen._step_token = Engine._gen_tokens
        key = (tok, self._bufgen, id(self.opt), self.opt.lr, self.opt.decay, getattr(self.opt, "epsilon", 0.0),
               self.row_skip, self.shadow_blocked, self.keep,
               self.seed, self.act, self.comm, self.dp_world, self.use_sparse, self.sparse_dw, self.epoch_row_lists,
               self.epoch_scatter, self.fold_reduce, self.fuse_enc_epilogue, self.l2,
               tuple(self.trainable), self.grad_hook, self.master_sync, self.pair_dw, self.fuse_enc_dec)
        pl = self._plan
        if pl is not None and pl["key"] == key:
            return key
        if not (self.comm is None and self.dp_world == 1 and len(self.H) == 1 and self.sparse_ok and self.use_sparse
                and self.sparse_dw and self.epoch_row_lists and self.epoch_scatter and
                self.fold_reduce and self.fuse_enc_epilogue and not self.l2 and all(self.trainable) and
                self.grad_hook is None and self.master_sync is None):
            return None
        return key

    _gen_tokens = 0

    def _count_general(self, pl, key):
        """diagnostics: why a step took the recorded general path"""
        self.step_paths["general"] += 1
        why = ("no template" if pl is None else "unverified" if not pl.get("ready") else
               "key" if pl["key"] != key else "capacity")
        self.step_paths[why] = self.step_paths.get(why, 0) + 1
        if why == "key" and self.step_paths.get("key_diff") is None:
            self.step_paths["key_diff"] = [i for i, (x, y) in enumerate(zip(pl["key"], key)) if x != y]

    def fast_train_step(self, gen, bi):
        """Model._train_one's step on generator batch bi through ocf_train_step_rows; False when this step
        must take the general path (then nothing was done)."""
        self.rows_real = None         # a generator batch: always B rows
        if not self.fast_steps or (self.timers is not None and self.timer_only is None):
            return False
        if self.comm is not None:
            return self._fast_rank_step(gen, bi)
        key = self._fast_key(gen)
        if key is None:
            return False
        pl = self._plan
        if pl is not None and pl.get("ready") and pl["key"] == key:
            f = gen.step_fields(bi, self.Np)
            if f is not None and self._fits(pl, f):
                self._issue(pl, f)
                self.step_paths["one_call"] += 1
                return True
        self._count_general(pl, key)
        # the general path, recorded
        self._grow_stats(self.n_stats + 1)
        per = self._per_step()
        calls = self._recorded_step(gen, bi)
        key = self._fast_key(gen)              # (buffers may have grown during the step)
        f = gen.step_fields(bi, self.Np)
        if key is None or f is None or tuple(n for n, _ in calls) not in self._STEP_CALLS:
            self._plan = None
            return True
        if pl is not None and pl["key"] == key and not pl.get("ready") and pl.get("bad", 0) < 2:
            # second recorded step: the template rewritten for it must reproduce it exactly
            st = _lib.OcfRowStepArgs.from_buffer_copy(pl["st"])
            cand = dict(pl, st=st)
            self._bind(cand)
            self._rewrite(cand, f, per)
            if self._same(cand, calls):
                cand["ready"] = True
                self._plan = cand
            else:                              # start over from this step (at most twice)
                self._plan = self._template(key, calls, f)
                self._plan["bad"] = pl.get("bad", 0) + 1
            return True
        if pl is not None and pl.get("bad", 0) >= 2 and pl["key"] == key:
            return True                        # this template does not verify: stay on the general path
        self._plan = self._template(key, calls, f)
        return True

    def _recorded_step(self, gen, bi):
        global _recorder
        a = gen.scatter_args(bi, engine_args=self.scatter_args())
        self.load_batch(a, gen.targets(bi, self.N), gather=gen.gather_tables(bi))
        _recorder = []
        try:
            self.train_step()
            return list(_recorder)
        finally:
            _recorder = None

    def _per_step(self):
        """the fields of a step that change with the step itself: Philox stream of the dropout mask
        (forward), stats slot, optimizer constants (Keras decay / Adam bias correction)"""
        row = self.stats_hist.data_ptr() + self.n_stats * self.stats_hist.stride(0) * 4
        stream = (self.step_count * self.dp_world + self.dp_rank) * 16
        if self.opt.kind != _lib.OPT_ADAM and not self.opt.decay and self._plan is not None \
                and self._plan.get("ready"):
            return stream, row, None, None     # constant optimizer scalars: the template's stand
        gscale = 2.0 / ((self.rows_real or self.B) * self.N_total)
        op = self.opt.step_params(1.0, self.l2)
        o = _lib.OcfOptParams(op.kind, op.lr, op.eps, op.rho, op.beta2, op.l2, gscale)
        return stream, row, o, self.opt.step_params(1.0, 0.0)

    def _template(self, key, calls, f):
        st = _lib.OcfRowStepArgs()
        enc, dec, g_out, g_in, sync, arrive = self._step_blocks(calls)
        st.enc_arrive = arrive
        ctypes.memmove(ctypes.addressof(st.enc), ctypes.addressof(enc), ctypes.sizeof(enc))
        ctypes.memmove(ctypes.addressof(st.dec), ctypes.addressof(dec), ctypes.sizeof(dec))
        ctypes.memmove(ctypes.addressof(st.dw_out), ctypes.addressof(g_out), ctypes.sizeof(g_out))
        ctypes.memmove(ctypes.addressof(st.dw_in), ctypes.addressof(g_in), ctypes.sizeof(g_in))
        if g_out.jr:
            ctypes.memmove(ctypes.addressof(st.jr), g_out.jr, ctypes.sizeof(st.jr))
            st.jr_on = 1
        elif dec.jr:
            ctypes.memmove(ctypes.addressof(st.jr), dec.jr, ctypes.sizeof(st.jr))
            st.jr_on = 2
        st.dw_out.jr = None
        st.dec.jr = None
        st.pair_sync = sync
        pl = dict(key=key, st=st, cap_enc=self._gbuf["part_enc"].numel() // self.Hp[0],
                  cap_dec=min(self._gbuf["part_dec"].numel() // self.Hp[-1], self._gbuf["chunk_stats"].numel() // 4),
                  cap_e=self._gbuf["delta_e"].numel())
        self._bind(pl)
        return pl

    @staticmethod
    def _step_blocks(calls):
        """(encoder, decoder, dW_out, dW_in argument blocks, pair sync pointer or None, encoder counter or None) of
        a recorded step"""
        arrive = None
        if calls[0][0] == "ocf_gather_encdec":
            enc, dec, arrive, _ = calls[0][1]
            calls = [("ocf_gather_encoder", (enc,)), ("ocf_gather_decoder", (dec,))] + list(calls[1:])
        if len(calls) == 3:
            (g_out, g_in, sync, _) = calls[2][1]
            return calls[0][1][0], calls[1][1][0], g_out, g_in, sync, arrive
        return calls[0][1][0], calls[1][1][0], calls[2][1][0], calls[3][1][0], None, arrive

    def _bind(self, pl):
        st = pl["st"]
        sets = []
        for obj in (st.enc, st.dec):
            sets += [(obj, n, i) for n, i in self._GATHER_FIELDS]
        for obj in (st.dw_out, st.dw_in):
            sets += [(obj, n, i) for n, i in self._DW_FIELDS]
            sets.append((obj, "row_live", self._F_LIVE))
        sets += [(st.enc, "xval", self._F_XVAL), (st.dec, "flag", self._F_TFLAG), (st.dec, "enc_cptr", self._F_CPTR),
                 (st.dw_in, "sp_vals", self._F_XVAL)]
        if st.jr_on:
            sets.append((st.jr, "row_cptr", self._F_CPTR))
        pl["sets"] = sets
        pl["live"] = bool(st.dw_out.row_live)
        # the same writes as two NumPy scatters into the template's bytes (~35 setattr calls cost ~10 us of host
        # time per step; the first step of a row-list window waits for it on an idle GPU)
        base = ctypes.addressof(st)
        o8, i8, o4, i4 = [], [], [], []
        for obj, name, i in sets:
            fd = getattr(type(obj), name)
            off = ctypes.addressof(obj) - base + fd.offset
            if dict(type(obj)._fields_)[name] in (ctypes.c_float, ctypes.c_double):
                raise AssertionError("step template field %s: integer fields only" % name)
            if fd.size == 8 and off % 8 == 0:
                o8.append(off // 8), i8.append(i)
            elif fd.size == 4 and off % 4 == 0:
                o4.append(off // 4), i4.append(i)
            else:
                raise AssertionError("step template field %s: size %d at offset %d" % (name, fd.size, off))
        raw = (ctypes.c_char * ctypes.sizeof(st)).from_buffer(st)
        pl["w8"] = (np.frombuffer(raw, dtype=np.int64, count=ctypes.sizeof(st) // 8), np.array(o8), np.array(i8))
        pl["w4"] = (np.frombuffer(raw, dtype=np.int32), np.array(o4), np.array(i4))

    def _fits(self, pl, f):
        # (every template fuses the encoder's epilogue into the decoder: _forward_gather's gates apply to it too)
        return (f[self._F_NCH] <= pl["cap_enc"] and f[self._F_NCH] <= pl["cap_dec"] and f[self._F_E] <= pl["cap_e"]
                and (self._rowres() or (f[self._F_MAXCH] <= FUSE_MAX_CHUNKS
                                        and f[self._F_NCH] <= FUSE_MEAN_CHUNKS * self.B))
                and self.n_stats < self.stats_cap)

    def _rowres(self):
        """ocf_gather_encdec takes its row-resident form (the library's "encdec_rowres" switch, read when the
        engine is built; fp32 at H % 256 == 0, 16-bit at H != 384): one workgroup per batch row, no chunk partials re-read, so the encoder's
        epilogue rides in the decoder launch whatever the chunks per row"""
        rr = self.__dict__.get("_rowres_on")
        if rr is None:
            prev = ctypes.c_int32(0)
            _lib.call("ocf_set_tuning", b"encdec_rowres", -1, ctypes.byref(prev))
            rr = self._rowres_on = bool(prev.value) and (self.Hp[-1] % 256 == 0 if self.cdt == _lib.DT_F32
                                                          else self.Hp[-1] != 384)
        return rr

    def _rewrite(self, pl, f, per):
        v = np.array(f, dtype=np.int64)
        w, o, i = pl["w8"]
        w[o] = v[i]
        w, o, i = pl["w4"]
        w[o] = v[i]
        st = pl["st"]
        if not pl["live"]:
            st.dw_out.row_live = st.dw_in.row_live = None
        st.dec.stream, st.dw_in.js_out = per[0], per[1]
        if per[2] is not None:
            st.dw_out.opt = st.dw_in.opt = per[2]
            st.dw_out.cb_op = st.dw_in.jb_op = per[3]

    def _same(self, pl, calls):
        st = pl["st"]
        enc, dec, g_out, g_in, sync, arrive = self._step_blocks(calls)
        if (sync or None) != (st.pair_sync or None) or (arrive or None) != (st.enc_arrive or None):
            return False
        b = lambda x: ctypes.string_at(ctypes.addressof(x), ctypes.sizeof(x))
        o = type(g_out).from_buffer_copy(g_out)
        d = type(dec).from_buffer_copy(dec)
        on, src = (1, g_out.jr) if g_out.jr else ((2, dec.jr) if dec.jr else (0, None))
        jr_ok = on == st.jr_on and (not on or ctypes.string_at(src, ctypes.sizeof(st.jr)) == b(st.jr))
        o.jr = d.jr = None
        return jr_ok and b(enc) == b(st.enc) and b(d) == b(st.dec) and b(o) == b(st.dw_out) and b(g_in) == b(st.dw_in)

    # phase -> (event slot before, after) in OcfRowStepArgs.ev; dW_pair with ocf_gemm_pair
    _EV_SLOTS = {"enc_gemm": (0, 1), "dec_gemm_mse": (2, 3), "dW_out": (4, 5), "dW_in": (6, 7), "dW_pair": (4, 7)}

    def _issue(self, pl, f):
        self._rewrite(pl, f, self._per_step())
        st = pl["st"]
        timed = []
        if self.timers is not None:            # bench.py's per-kernel HIP events, recorded by the library
            names = ("enc_gemm", "dec_gemm_mse") + (("dW_pair",) if st.pair_sync else ("dW_out", "dW_in"))
            for name in names:
                if self.timer_only is None or name in self.timer_only:
                    a, b = self._timing_event(), self._timing_event()     # (recorded by the library)
                    i0, i1 = self._EV_SLOTS[name]
                    st.ev[i0], st.ev[i1] = a.cuda_event, b.cuda_event
                    timed.append((i0, i1, name, a, b))
        call("ocf_train_step_rows", st, cur_stream())
        for i0, i1, name, a, b in timed:
            self.timers.setdefault(name, []).append((a, b))
            st.ev[i0] = st.ev[i1] = None
        # the general path's bookkeeping (load_batch + train_step)
        self._fused_step = True
        self._xin_clean = False
        # what the general path leaves behind for the loaded batch (callers inspect the path taken)
        self.gt = dict(xval=f[self._F_XVAL], flag=f[self._F_TFLAG], E=f[self._F_E], one_call=True)
        self.tb = dict(sp_rowptr=f[self._F_RPTR], sp_rowent=f[self._F_RENT], sp_nent=f[self._F_E])
        self._rtag_live = pl["live"]
        self.tseg = None
        self._enc_fused = self._reduce_job = self._stats_pending = None
        self.n_stats += 1
        self.opt.iterations += 1
        self.step_count += 1

    # ---------------------------------------------------------------- one call per phase: feature parallel
    # A feature-parallel rank step (comm set) is ten library calls in three groups around its two all-reduces
    # (pre-activations after the encoder, hidden-delta partials after the decoder).  Built in Python they cost
    # ~0.19 ms of host time per step -- about the rank's whole GPU step at G = 8 -- so, as for the single-GPU
    # step, a recorded step becomes a template (ocf.h OcfRankStepArgs) whose per-step fields (the batch's
    # table pointers, the dropout stream, the stats slot) are rewritten, and the step is issued as four
    # ocf_rank_step calls with the collectives between them.  The template is used only after a second
    # recorded step equals it rewritten for that step, byte for byte.
    _RANK_CALLS = ("ocf_gather_encoder", "ocf_rows_reduce", "ocf_splitk_bias_act", "ocf_gather_decoder",
                   "ocf_rows_reduce", "ocf_stats_finalize", "ocf_gemm", "ocf_bias_opt_from_partials",
                   "ocf_splitk_grad_act", "ocf_gemm")
    _RANK_EV = {"enc_gemm": (0, 1), "dec_gemm_mse": (2, 3), "dW_out": (4, 5), "dW_in": (6, 7)}
    _rplan = None

    def _rank_key(self, gen):
        tok = getattr(gen, "_step_token", None)
        if tok is None:
            from .data_reader import BatchGenerator
            if not (isinstance(gen, BatchGenerator) and gen.split == "train"):
                return None
            Engine._gen_tokens += 1
            tok = gen._step_token = Engine._gen_tokens
        if not (self.comm is not None and getattr(self.comm, "start", None) is not None and self.dp_world == 1
                and len(self.H) == 1 and self.sparse_ok and self.use_sparse and self.sparse_dw
                and self.epoch_row_lists and self.epoch_scatter and not self.l2
                and all(self.trainable) and self.grad_hook is None and self.master_sync is None
                and self.opt.kind != _lib.OPT_ADAM and not self.opt.decay):
            return None
        return (tok, self._bufgen, id(self.opt), self.opt.lr, getattr(self.opt, "epsilon", 0.0), self.row_skip,
                self.shadow_blocked, self.keep, self.seed, self.act, id(self.comm),
                self.side is not None)

    def _fast_rank_step(self, gen, bi):
        key = self._rank_key(gen)
        if key is None:
            return False
        pl = self._rplan
        if pl is not None and pl.get("ready") and pl["key"] == key:
            f = gen.step_fields(bi, self.Np)
            if f is not None and self._rank_fits(pl, f):
                self._rank_issue(pl, f)
                self.step_paths["one_call"] += 1
                return True
        self._count_general(pl, key)
        self._grow_stats(self.n_stats + 1)
        calls = self._recorded_step(gen, bi)
        key = self._rank_key(gen)
        f = gen.step_fields(bi, self.Np)
        if key is None or f is None or tuple(n for n, _ in calls) != self._RANK_CALLS:
            self._rplan = None
            return True
        cand = self._rank_template(key, calls)
        if pl is not None and pl["key"] == key and not pl.get("ready") and pl.get("bad", 0) < 2:
            # second recorded step: the first one's template rewritten for it must reproduce it exactly
            st = _lib.OcfRankStepArgs.from_buffer_copy(pl["st"])
            self._rank_rewrite(st, f, self._rank_stream(self.step_count - 1), self._stats_row(self.n_stats - 1),
                               pl["live"])
            b = lambda x: ctypes.string_at(ctypes.addressof(x), ctypes.sizeof(x))
            if b(st) == b(cand["st"]):
                pl["ready"] = True
            else:
                cand["bad"] = pl.get("bad", 0) + 1
                self._rplan = cand
            return True
        if pl is not None and pl.get("bad", 0) >= 2 and pl["key"] == key:
            return True
        self._rplan = cand
        return True

    def _rank_stream(self, step):
        return (step * self.dp_world + self.dp_rank) * 16          # forward()'s Philox stream of the dropout

    def _stats_row(self, n):
        return self.stats_hist.data_ptr() + n * self.stats_hist.stride(0) * 4

    @staticmethod
    def _as_block(cls, args):
        """a positional call's arguments (without the stream) as its ocf.h argument block"""
        blk = cls()
        for (name, _), v in zip(cls._fields_, args):
            setattr(blk, name, v)
        return blk

    def _rank_template(self, key, calls):
        st = _lib.OcfRankStepArgs()
        a = [c[1] for c in calls]
        copy = lambda dst, src: ctypes.memmove(ctypes.addressof(dst), ctypes.addressof(src), ctypes.sizeof(src))
        copy(st.enc, a[0][0])
        copy(st.enc_sum, a[1][0])
        st.hidden = self._as_block(_lib.OcfBiasActArgs, a[2][:-1])
        copy(st.dec, a[3][0])
        copy(st.dec_sum, a[4][0])
        st.stats = self._as_block(_lib.OcfStatsArgs, a[5][:-1])
        copy(st.dw_out, a[6][0])
        st.out_bias = self._as_block(_lib.OcfBiasOptArgs, a[7][:-1])
        st.hidden_grad = self._as_block(_lib.OcfGradActArgs, a[8][:-1])
        copy(st.dw_in, a[9][0])
        if self.side is not None:
            evs = getattr(self, "_rank_evs", None)
            if evs is None:                        # one set per engine (templates compare byte for byte)
                evs = []
                for _ in range(3):
                    e = torch.cuda.Event()
                    e.record()                     # (creates the event; the library records it again)
                    evs.append(e)
                self._rank_evs = evs
            st.side = self.side.cuda_stream
            st.fork[0], st.fork[1], st.join = (e.cuda_event for e in evs)
        return dict(key=key, st=st, live=bool(st.dw_out.row_live),
                    cap_enc=self._gbuf["part_enc"].numel() // self.Hp[0],
                    cap_dec=min(self._gbuf["part_dec"].numel() // self.Hp[-1], self._gbuf["chunk_stats"].numel() // 4),
                    cap_e=self._gbuf["delta_e"].numel())

    def _rank_fits(self, pl, f):
        return (f[self._F_NCH] <= pl["cap_enc"] and f[self._F_NCH] <= pl["cap_dec"] and f[self._F_E] <= pl["cap_e"]
                and self.n_stats < self.stats_cap)

    def _rank_rewrite(self, st, f, stream_id, stats_row, live):
        for obj in (st.enc, st.dec):
            for n, i in self._GATHER_FIELDS:
                setattr(obj, n, f[i])
        st.enc.xval, st.dec.flag = f[self._F_XVAL], f[self._F_TFLAG]
        st.enc_sum.row_cptr = st.dec_sum.row_cptr = f[self._F_CPTR]
        for obj in (st.dw_out, st.dw_in):
            for n, i in self._DW_FIELDS:
                setattr(obj, n, f[i])
            obj.row_live = f[self._F_LIVE] if live else None
        st.dw_in.sp_vals = f[self._F_XVAL]
        st.hidden.stream = stream_id
        st.stats.out = stats_row

    def _rank_issue(self, pl, f):
        st = pl["st"]
        self._rank_rewrite(st, f, self._rank_stream(self.step_count), self._stats_row(self.n_stats), pl["live"])
        timed = []
        if self.timers is not None:            # bench.py's per-kernel HIP events, recorded by the library
            for name, (i0, i1) in self._RANK_EV.items():
                if self.timer_only is None or name in self.timer_only:
                    a, b = self._timing_event(), self._timing_event()     # (recorded by the library)
                    st.ev[i0], st.ev[i1] = a.cuda_event, b.cuda_event
                    timed.append((i0, i1, name, a, b))
        s = cur_stream()
        call("ocf_rank_step", st, 0, s)
        self.comm(self.hpre)                   # the pre-activation partials, summed over the ranks
        call("ocf_rank_step", st, 1, s)
        work = self.comm.start(self.dhpre)     # the hidden-delta partials: in flight during phase 2
        call("ocf_rank_step", st, 2, s)
        work.wait()
        call("ocf_rank_step", st, 3, s)
        for i0, i1, name, a, b in timed:
            self.timers.setdefault(name, []).append((a, b))
            st.ev[i0] = st.ev[i1] = None
        # the general path's bookkeeping
        self._fused_step = True
        self._xin_clean = False
        self.gt = dict(xval=f[self._F_XVAL], flag=f[self._F_TFLAG], E=f[self._F_E], one_call=True)
        self.tb = dict(sp_rowptr=f[self._F_RPTR], sp_rowent=f[self._F_RENT], sp_nent=f[self._F_E])
        self._rtag_live = pl["live"]
        self.tseg = None
        self._enc_fused = self._reduce_job = self._stats_pending = None
        self._side_busy = False
        self.n_stats += 1
        self.opt.iterations += 1
        self.step_count += 1

    def eval_step(self):
        if self.l2:
            self._l2_penalty()     # Keras' test loss includes the regularisers too
        self.forward(training=False)
        self.output_loss(with_grad=False)
        self._join()

    def take_stats(self):
        """host copy of the per-step stats recorded since the last call: [steps, 4 + Bp]."""
        self._flush_stats()
        st = self.stats_hist[: self.n_stats]
        pen = self.pen_hist[: self.n_stats]
        if self.comm is not None and self.n_stats:
            st = st.clone()
            self.comm(st)          # SSE / SAE / counts / row SSE are sums over the column shards
            sh = pen[:, 0].clone()
            self.comm(sh)
            pen = torch.stack([sh, pen[:, 1]], 1)
        out = st.cpu().numpy().astype(np.float64)
        # a kernel fault recorded without stopping (a pair-launch wait or a fused-step barrier that gave up) in
        # the steps just read back surfaces here, at every epoch end, not only at the next library call
        _lib.call("ocf_check_async")
        # column 3 (0 from the loss epilogues) carries the step's l2 penalty
        out[:, 3] = pen.double().sum(1).cpu().numpy()
        self.pen_hist[: self.n_stats].zero_()
        self.n_stats = 0
        return out
