"""Drop-in for the reference's ``data_reader`` (data_reader.py:11-419).

Same constructor and ``data_gen`` signature; batches come out of the GPU scatter kernel (K1,
``ocf_scatter_batch``) instead of a Python double loop over dicts.  Differences that are
deliberate:

* arrays are float32 CUDA tensors of shape [B, num_items] (the reference yields float64 NumPy
  arrays that Keras immediately casts to float32);
* the dataset is uploaded to HBM once as row-CSR (dataset.py); a batch never leaves the GPU;
* the NumPy global RNG is consumed exactly as the reference consumes it (same permutation,
  same ``uniform`` / ``choice`` draws -> bit-identical reciprocal masks): the permutation by NumPy,
  the epoch's uniform / choice draws by ocf_recip_keep on the GPU from NumPy's own MT19937 state
  (jump-ahead segments, bit-identical; the state is handed back).  The draws of a whole
  training epoch are taken when the generator is first pulled: Keras 2.0.4's GeneratorEnqueuer
  drains the generator ahead of ``fit_generator`` (queue of 10 > the one batch train.py leaves
  unused), so every train draw precedes the validation permutation in the reference as well.
  ``rng="device"`` instead draws reciprocal masks with Philox on the GPU (same distribution,
  no host work) and skips the NumPy draws; with data_sparsity [1, 1] (train.py:28) both modes
  give identical masks.
"""
from __future__ import annotations

import ctypes
import os
import time

import numpy as np
import torch

from . import _lib
from .dataset import FixedSplit, load_reference_json
from .engine import TILE, cur_stream, ptr, ru
from .parallel import shard_batches

AUX_FEED = {None: 0, "dropout": 1, "both": 1, "causal": 2, "zeros": 3}
# entries per row-gather work unit (ocf_gather_*): a group of 32 lanes walks its chunk's entries 4 at a time,
# so a chunk's latency grows with its length; batches of fewer entries than GATHER_BIG use short chunks
# (more workgroups, each a few dependent steps), large batches the long ones (fewer partial sums)
GATHER_CHUNK = 256
GATHER_CHUNK_SMALL = 64
GATHER_CHUNK_MID = 96
GATHER_CHUNK_MID_MIN_CHUNKS = 512
GATHER_BIG = 100_000
ROWLIST_MAX_BATCHES = 4096      # batches per ocf_epoch_row_lists build (the library takes up to 65,535)
ROWLIST_MAX_ENTRIES = 4096      # entries per column list of one batch (ocf_epoch_row_lists' LDS sort)
ROWLIST_RG_WORK = 160           # (batches x row groups) per row-list build: at least this many, row groups <= 8
ROWS_DENSE_MAX_COLS = 170 * 128  # the row-stream kernel's small regime (ocf_gemm.hip rows_small_waves: 170 tiles)


_RNG_STREAMS = {}


def _h2d(x, dev):
    """Upload a host array without draining the current stream: a pageable copy makes torch synchronise
    the stream (every queued training step), so the epoch's tables go through pinned memory (the caching
    host allocator keeps the pinned block until the copy on the current stream is done)."""
    t = torch.as_tensor(np.ascontiguousarray(x))
    if torch.device(dev).type != "cuda":
        return t.to(dev)
    return t.pin_memory().to(dev, non_blocking=True)


def _rng_stream(dev):
    """one stream per device for ocf_recip_keep (created on first use)"""
    key = torch.device(dev).index if torch.device(dev).index is not None else torch.cuda.current_device()
    if key not in _RNG_STREAMS:
        _RNG_STREAMS[key] = torch.cuda.Stream(device=key)
    return _RNG_STREAMS[key]


class _DeviceCSR:
    def __init__(self, csr, dev):
        self.host = csr
        self.rp = torch.as_tensor(csr.row_ptr, device=dev)
        self.col = torch.as_tensor(csr.col, device=dev)
        self.val = torch.as_tensor(csr.val, device=dev)
        self.dup = None if csr.dup is None else torch.as_tensor(csr.dup, device=dev)
        self.pos = None if csr.pos is None else torch.as_tensor(csr.pos, device=dev)
        self.lens = csr.row_lengths()          # entries held here (a column shard holds fewer)
        self.rng_lens = csr.rng_lengths()      # entries of the full rows (RNG draws, batch offsets)
        self.dev = dev
        self._tiles = {}

    def tiles(self, n_cols):
        """Column-sorted copy + per-row tile pointers (dataset.RatingsCSR.tile_index) on the device,
        built once per CSR: the masked-MSE epilogue reads each batch row's targets of its column
        tile from here (row-segment mode)."""
        if n_cols not in self._tiles:
            col_s, val_s, lidx_s, tptr = self.host.tile_index(n_cols)
            d = self.dev
            self._tiles[n_cols] = dict(t_col=torch.as_tensor(col_s, device=d), t_val=torch.as_tensor(val_s, device=d),
                                       t_lidx=torch.as_tensor(lidx_s, device=d), t_tptr=torch.as_tensor(tptr, device=d),
                                       t_ntiles=tptr.shape[1] - 1,
                                       t_maxlen=int(self.lens.max()) if len(self.lens) else 0)
        return self._tiles[n_cols]


class data_reader(object):
    """``data_reader(num_items, num_users, filepath, nonsequentialusers, use_json, eval_mode,
    useTimestamps, reverse_user_item_data)`` (data_reader.py:12).  ``dataset=`` accepts a prebuilt
    ``FixedSplit`` (or a path to its .npz) instead of the JSON files; ``rng`` selects the
    reciprocal-mask RNG ('numpy' exact, or 'device')."""

    def __init__(self, num_items, num_users, filepath=None, nonsequentialusers=False, use_json=True,
                 eval_mode="ablation", useTimestamps=False, reverse_user_item_data=False, dataset=None,
                 rng="numpy", device=None):
        if useTimestamps:
            raise NotImplementedError("useTimestamps: broken in the reference (data_reader.py:358-359 feeds the "
                                      "whole dict); not supported")
        if eval_mode != "fixed_split":
            raise NotImplementedError("eval_mode='ablation' (split_for_validation) is out of scope; use fixed_split")
        self.num_items = int(num_items)
        self.num_users = int(num_users)
        self.filepath = filepath
        self.nonsequentialusers = nonsequentialusers
        self.eval_mode = eval_mode
        self.useTimestamps = False
        self.rng = rng
        if dataset is None:
            dataset = load_reference_json(filepath, reverse_user_item_data, use_json)
        elif isinstance(dataset, str):
            dataset = FixedSplit.load(dataset)
        self.data = dataset
        if dataset.num_cols != self.num_items:
            raise ValueError("num_items=%d but the data has %d columns" % (self.num_items, dataset.num_cols))
        self.items_to_densevec = {c: i for i, c in enumerate(dataset.col_ids)}
        self.densevec_to_items = {i: c for i, c in enumerate(dataset.col_ids)}
        # data_reader.py:73-80
        self.train_set = list(dataset.train.keys)
        self.val_set = list(dataset.valid_tgt.keys)
        self.test_set = list(dataset.test_tgt.keys)
        self.train_set_size = len(self.train_set)
        self.val_set_size = len(self.val_set)
        self.test_set_size = len(self.test_set)
        self.device = torch.device(device if device is not None else "cuda")
        self._dev = None
        print("Finished loading data")

    def _on_device(self):
        if self._dev is None:
            d = self.device
            self._dev = {k: _DeviceCSR(getattr(self.data, k), d)
                         for k in ("train", "valid_in", "valid_tgt", "test_in", "test_tgt")}
        return self._dev

    def split_for_validation(self, val_split, seed=None):
        raise NotImplementedError("ablation eval mode is out of scope")

    def data_gen(self, batch_size, data_sparsity, train_val_test="train", shuffle=True,
                 auxilliary_mask_type="dropout", aux_var_value=-1, return_target_count=False,
                 sparse_representation=False, pass_through_input_training=False):
        """data_reader.py:314-419 -- returns a generator object (also usable by Model's fast path)."""
        if sparse_representation:
            raise NotImplementedError("sparse_representation needs a patched Keras backend in the reference "
                                      "(train.py:53); dense only")
        if auxilliary_mask_type not in AUX_FEED:
            raise ValueError("Auxilliary mask type %r doesn't exist" % (auxilliary_mask_type,))
        return BatchGenerator(self, int(batch_size), data_sparsity, train_val_test, shuffle, auxilliary_mask_type,
                              float(aux_var_value), return_target_count, bool(pass_through_input_training))


class BatchGenerator(object):
    """Lazy like the reference generator: nothing is drawn before the first pull."""

    def __init__(self, reader, B, sparsity, split, shuffle, aux_type, aux, return_count, pass_through):
        self.r = reader
        self.B = B
        self.sparsity = sparsity
        self.split = split
        self.shuffle = shuffle
        self.aux_type = aux_type
        self.aux = aux
        self.return_count = return_count
        self.pass_through = pass_through
        self.keys = {"train": reader.train_set, "valid": reader.val_set, "test": reader.test_set}[split]
        self.n = len(self.keys)
        self.num_batches = self.n // B                                   # data_reader.py:329
        self.i = 0
        self.started = False
        self.dp_shard = None          # (rank, world) under data parallelism (Model._train_one)
        self.seed = int(np.random.randint(0, 2 ** 31 - 1)) if reader.rng == "device" else 0

    # ------------------------------------------------------------ epoch plan
    def plan(self, row_lengths1, row_lengths2=None):
        """Host half of the epoch plan (no GPU): the NumPy permutation of the row set
        (data_reader.py:326-327), batch rows, batch-local entry offsets, target counts."""
        order = np.random.permutation(self.n) if self.shuffle else np.arange(self.n)   # :326-327
        nb, B = self.num_batches, self.B
        rows = order[: nb * B].reshape(nb, B).astype(np.int64)
        lens1 = row_lengths1[rows]                       # [nb, B]
        boff = np.zeros((nb, B + 1), dtype=np.int64)
        np.cumsum(lens1, axis=1, out=boff[:, 1:])
        tcount = row_lengths2[rows].sum(axis=1) if row_lengths2 is not None else None
        return rows, boff, tcount

    def _draw_keep(self, boff):
        """The epoch's reciprocal-split draws (data_reader.py:120 uniform per batch, :130 choice per row)
        on the device from NumPy's own global MT19937 state, bit-identical, the state handed back to
        NumPy afterwards (ocf_recip_keep).  Returns the keep flags (None when data_sparsity is [1, 1]: every
        rating is an input, but the stream still advances exactly as the reference's draws advance it)."""
        nb, B = self.num_batches, self.B
        E = int(boff[:, -1].sum()) if nb else 0
        s0, s1 = float(self.sparsity[0]), float(self.sparsity[1])
        st = np.random.get_state()
        if st[0] != "MT19937":
            raise ValueError("the reference's draws need NumPy's legacy MT19937 global state")
        dev = self.r.device
        a = _lib.OcfRecipKeepArgs()
        key = np.ascontiguousarray(st[1], dtype=np.uint32)
        ctypes.memmove(a.key, key.ctypes.data, 624 * 4)
        a.pos, a.nb, a.B, a.n_entries = int(st[2]), nb, B, E
        a.s0, a.s1 = s0, s1
        keep = None
        nbytes = _lib.load().ocf_recip_keep_workspace(nb, B, E, a.pos)
        if nbytes < 0:
            raise _lib.OcfError("ocf_recip_keep_workspace: " + _lib.load().ocf_last_error().decode())
        # its own stream, with its own copies of the batch offsets (uploaded on it, pinned): the call
        # synchronises that stream to hand the state back -- and the keep flags / workspace are complete when
        # it returns --, while the main stream's queued steps are not waited for
        with torch.cuda.stream(_rng_stream(dev)):
            ws = torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=dev)
            a.workspace, a.workspace_bytes = ptr(ws), int(nbytes)
            if not (s0 >= 1.0 and s1 >= 1.0) and E:
                keep = torch.empty(E, dtype=torch.uint8, device=dev)
                boff_r = _h2d(boff, dev)
                ebase = _h2d(np.concatenate([[0], np.cumsum(boff[:, -1])]).astype(np.int64), dev)
                a.keep, a.boff, a.ebase = ptr(keep), ptr(boff_r), ptr(ebase)
            _lib.call("ocf_recip_keep", a, cur_stream())
        if keep is not None and keep.is_cuda:   # allocated on the RNG stream, read on the main stream from here on
            keep.record_stream(torch.cuda.current_stream(dev))
        np.random.set_state((st[0], np.frombuffer(a.key, dtype=np.uint32).copy(), int(a.pos), st[3], st[4]))
        return keep

    def _start(self):
        self.started = True
        r = self.r
        dev = r._on_device()
        if self.split == "train":
            self.src1, self.src2 = dev["train"], None
        elif self.split == "valid":
            self.src1, self.src2 = dev["valid_in"], dev["valid_tgt"]
        else:
            self.src1, self.src2 = dev["test_in"], dev["test_tgt"]
        rows, boff, self.tcount = self.plan(self.src1.rng_lens, None if self.src2 is None else self.src2.rng_lens)
        nb = self.num_batches
        self.rows_host = rows
        self.nnz_full = boff[:, -1].copy()
        self.nnz1 = self.src1.lens[rows].sum(axis=1) if nb else np.zeros(0, np.int64)   # entries held here
        self.rows_dev = _h2d(rows.astype(np.int32), r.device)
        self.boff_dev = _h2d(boff, r.device)
        keep = self._draw_keep(boff) if (self.split == "train" and r.rng == "numpy") else None
        # batch-local offsets of the entries held by this CSR (one scatter thread per entry)
        self.lboff1_dev = _h2d(self._local_offsets(self.src1.lens, rows), r.device)
        if self.src2 is not None:
            self.tlocal = self.src2.lens[rows].sum(axis=1) if nb else np.zeros(0, np.int64)
            self.lboff2_dev = _h2d(self._local_offsets(self.src2.lens, rows), r.device)
        # row-gather chunk tables (inputs from source 1; targets from source 1 in training, else source 2)
        self.chunks1 = self._chunk_tables(self.src1.lens, rows, r.device)
        self.chunks2 = self.chunks1 if self.src2 is None else self._chunk_tables(self.src2.lens, rows, r.device)
        self.keep_dev = None
        self.keep_off = None
        self._ep_tabs = None           # per-epoch device tables of the row-list builds (_epoch_tables)
        self._ep_fields = None         # per-epoch constant step fields (step_fields)
        if keep is not None:
            self.keep_dev = keep
            self.keep_off = np.concatenate([[0], np.cumsum(self.nnz_full)])
        self.max_targets = int(max(self.nnz1.max() if nb else 0,
                                   self.tlocal.max() if (self.src2 is not None and nb) else 0))

    @staticmethod
    def _chunk_tables(lens, rows, dev, chunk=None):
        """Every batch's rows cut into chunks of <= `chunk` entries (of equal length within a row): (batch
        row, first, end local entry) per chunk, [nb][B+1] first chunk of each row (relative to the batch),
        per-batch chunk base.  chunk: GATHER_CHUNK, or GATHER_CHUNK_SMALL for batches of few entries."""
        nb, B = rows.shape
        L = lens[rows].astype(np.int64).reshape(-1)                  # [nb*B]
        if chunk is None:
            per_batch = L.sum() / max(nb, 1)
            chunk = GATHER_CHUNK if per_batch >= GATHER_BIG else GATHER_CHUNK_SMALL
            # mid-size batches (ML-1M I: ~55 K entries) keep >= 512 chunks at 96 entries -- fewer redundant hidden
            # epilogues in the decoder: ML-1M 0.093 -> 0.089 ms/step; ML-1M U (~34 K) and ML-100K (~12 K) stay
            # at 64, where 96 was neutral / 5 % slower (tools/exp_chunk_small.sh, profiles/r03c_chunk_small/;
            # same-box A/B of the rule: tools/exp_chunk_ab.sh, 0.0931 -> 0.0898 ms, profiles/r03c_chunk_mid/)
            if chunk == GATHER_CHUNK_SMALL and per_batch >= GATHER_CHUNK_MID_MIN_CHUNKS * GATHER_CHUNK_MID:
                chunk = GATHER_CHUNK_MID
        nc = (L + chunk - 1) // chunk
        row_cptr = np.zeros((nb, B + 1), dtype=np.int32)
        np.cumsum(nc.reshape(nb, B), axis=1, out=row_cptr[:, 1:])
        cbase = np.zeros(nb + 1, dtype=np.int64)
        np.cumsum(row_cptr[:, -1], out=cbase[1:])
        tot = int(cbase[-1])
        rep = np.repeat(np.arange(nb * B, dtype=np.int64), nc)
        first = np.repeat(np.cumsum(nc) - nc, nc)
        k = np.arange(tot, dtype=np.int64) - first
        ncr = nc[rep]
        Lr = L[rep]
        j0 = k * Lr // ncr                 # equal-length chunks within a row
        j1 = (k + 1) * Lr // ncr
        t = lambda x: _h2d(np.ascontiguousarray(x, dtype=np.int32), dev)
        max_chunks = nc.reshape(nb, B).max(axis=1) if nb else np.zeros(0, np.int64)
        return dict(ch_row=t(rep % B), ch_j0=t(j0), ch_j1=t(j1), row_cptr=t(row_cptr), cbase=cbase,
                    max_chunks=max_chunks)

    def gather_tables(self, bi):
        """pointer sets for the row-gather kernels of batch bi: 'enc' (source-1 inputs) and 'dec'
        (the target CSR)"""
        B = self.B
        out = {}
        for key, src, ch, lb in (("enc", self.src1, self.chunks1, self.lboff1_dev),
                                 ("dec", self.src1 if self.src2 is None else self.src2, self.chunks2,
                                  self.lboff1_dev if self.src2 is None else self.lboff2_dev)):
            c0 = int(ch["cbase"][bi])
            out[key] = dict(rows=self.rows_dev.data_ptr() + 4 * bi * B, rp=ptr(src.rp), col=ptr(src.col),
                            val=ptr(src.val), lboff=lb.data_ptr() + 8 * bi * (B + 1),
                            ch_row=ch["ch_row"].data_ptr() + 4 * c0, ch_j0=ch["ch_j0"].data_ptr() + 4 * c0,
                            ch_j1=ch["ch_j1"].data_ptr() + 4 * c0, n_chunks=int(ch["cbase"][bi + 1]) - c0,
                            row_cptr=ch["row_cptr"].data_ptr() + 4 * bi * (B + 1),
                            max_chunks=int(ch["max_chunks"][bi]))
        if self.split == "train":      # train batches: inputs = targets -> the weight-gradient row lists
            out["row_lists"] = lambda n_cols, bi=bi: self.row_lists(bi, n_cols)
            # >= 2 entries per weight row on average: (nearly) every row is live, and on a weight of few row
            # tiles (the row-stream kernel's small regime: about one row per wave) the live-row records' two
            # dependent loads would only lengthen every wave's index chain -> the engine passes no records
            N = self.r.num_items
            out["rows_dense"] = bool(self.num_batches and self.nnz1.mean() >= 2 * N and N <= ROWS_DENSE_MAX_COLS)
        return out

    def prepare_row_lists(self, n_cols, batches=None):
        """The row lists (per weight row: the batch entries in that column, in batch-row order) and
        live-row records of the given epoch batches (default: every batch of the epoch), built on the
        device by one ocf_epoch_row_lists launch sequence instead of per step.  n_cols = the engine's
        padded column count."""
        t0 = time.perf_counter()
        if not self.started:
            self._start()
        if self.split != "train":
            raise ValueError("row lists are built for train batches (inputs = targets)")
        nb = self.num_batches
        if batches is None:
            # under data parallelism a rank only trains on its own batches (parallel.shard_batches)
            batches = shard_batches(nb, *self.dp_shard) if self.dp_shard else np.arange(nb)
        if isinstance(batches, (list, tuple, range)):
            sel = np.array(sorted(set(batches)), dtype=np.int64)     # (np.unique costs ~10-25 us on 20 ints)
        else:
            sel = np.asarray(batches, dtype=np.int64)
            if sel.size > 1 and not bool((sel[1:] > sel[:-1]).all()):
                sel = np.unique(sel)
        if len(sel) and (sel[0] < 0 or sel[-1] >= nb):
            raise ValueError("batch index out of range")
        # one build holds at most ROWLIST_MAX_BATCHES batches and ~1 GiB of row pointers (the library's
        # limit is 65,535); row_lists() builds the next window when it reaches a batch outside this one
        cap = int(min(ROWLIST_MAX_BATCHES, max(1, (1 << 28) // (n_cols + 1))))
        if len(sel) > cap:
            sel = sel[:cap]
        if self.src1.dup is not None and len(sel):
            self._check_list_lengths(sel)
        dev = self.rows_dev.device
        ep = self._epoch_tables(dev)
        n = len(sel)
        if n and int(sel[-1]) - int(sel[0]) + 1 == n:
            # consecutive batches (an epoch, the bench's timed window): sel / ebase point into the epoch's device
            # tables, ebase0 rebases the entry offsets -- nothing to upload (a staged copy cost 65-116 us of
            # host time on an idle GPU at the start of a timed window)
            b0 = int(sel[0])
            e0 = int(ep["ebase"][b0])
            ebase = ep["ebase"][b0:b0 + n + 1] - e0
            p_sel, p_ebase = ep["sel_dev"].data_ptr() + 4 * b0, ep["ebase_dev"].data_ptr() + 8 * b0
        else:
            e0 = 0
            ebase = np.zeros(n + 1, dtype=np.int64)
            np.cumsum(self.nnz1[sel], out=ebase[1:])
            p_ebase, p_sel = self._stage([ebase, sel.astype(np.int32)], dev)
        E = int(ebase[-1])
        # row groups per batch for the count / fill walks: a build of few batches (the bench's timed window, the
        # tail of an epoch) would leave most CUs idle with one workgroup per (batch, column block)
        n_rg = int(min(8, max(1, -(-ROWLIST_RG_WORK // max(n, 1)))))
        # grow-only device tables (an epoch rebuild reuses them: no allocation on the step path)
        need = (("cnt", n_rg * n * n_cols // 2 + n * (n_cols // 4096 + 1) + 1 + 2 * (E // 1025 + 1), torch.int32),
                ("row_ptr", n * (n_cols + 1), torch.int32), ("row_ent", 2 * max(E, 1), torch.int32),
                ("live", max(n * (n_cols // 128) * _lib.LIVE_REC, 1), torch.uint8),
                ("xval", max(E, 1), torch.float32), ("tflag", max(E, 1), torch.uint8))
        bufs = getattr(self, "_rl_bufs", None)
        if bufs is None:
            bufs = self._rl_bufs = {}
        for k, m, dt in need:
            b = bufs.get(k)
            if b is None or b[1] < m:
                t = torch.empty(m, dtype=dt, device=dev)
                bufs[k] = (t, m, t.data_ptr())
        t1 = time.perf_counter()
        a = _lib.OcfEpochRowListArgs()
        a.n_sel, a.B, a.n_cols, a.n_rg, a.ebase0 = n, self.B, n_cols, n_rg, e0
        a.max_list = self.B if self.src1.dup is None else 0       # (duplicate ratings: a list may exceed B)
        a.entries = E
        a.rows, a.rp, a.col, a.lboff = ep["args_const"]
        a.sel, a.ebase = p_sel, p_ebase
        a.cnt, a.row_ptr, a.row_ent, a.live = bufs["cnt"][2], bufs["row_ptr"][2], bufs["row_ent"][2], bufs["live"][2]
        _lib.call("ocf_epoch_row_lists", a, cur_stream())
        t2 = time.perf_counter()
        # ... and the batches' per-entry scatter outputs (live input value, live-target flag): the per-step
        # ocf_scatter_batch has nothing left to do for them
        if n:
            es = _lib.OcfEpochScatterArgs()
            es.keep_off = ep["keep_off"]
            es.n_sel, es.sel, es.ebase, es.ebase0 = n, p_sel, p_ebase, e0
            es.max_e = int(self.nnz1[sel].max())
            es.stream_mul = 2
            es.xval, es.tflag = bufs["xval"][2], bufs["tflag"][2]
            _lib.call("ocf_epoch_scatter", ep["scatter_base"], es, cur_stream())
        self._rl = dict(row_ptr=bufs["row_ptr"][0], row_ent=bufs["row_ent"][0], live=bufs["live"][0],
                        xval=bufs["xval"][0], tflag=bufs["tflag"][0], n_cols=n_cols,
                        slot=dict(zip(sel.tolist(), range(n))), ebase_host=ebase, fields={})
        t3 = time.perf_counter()
        # host time of the build's parts (us; bench.py reports them: the prelude of a timed window)
        self.rl_host_us = dict(plan=(t1 - t0) * 1e6, lists=(t2 - t1) * 1e6, scatter=(t3 - t2) * 1e6)

    def _epoch_tables(self, dev):
        """per epoch plan, on the first row-list build: sel = 0 .. nb - 1 and ebase = the batches' cumulative
        entry counts on the device (a build of consecutive batches points into them), the keep-flag offsets, the
        epoch scatter's base arguments and the constant pointers of the row-list build"""
        ep = getattr(self, "_ep_tabs", None)
        if ep is None:
            nb = self.num_batches
            ebase = np.zeros(nb + 1, dtype=np.int64)
            np.cumsum(self.nnz1, out=ebase[1:])
            ep = dict(ebase=ebase, ebase_dev=_h2d(ebase, dev), sel_dev=_h2d(np.arange(max(nb, 1), dtype=np.int32), dev),
                      scatter_base=self.scatter_args(0) if nb else _lib.OcfScatterArgs(),
                      args_const=(ptr(self.rows_dev), ptr(self.src1.rp), ptr(self.src1.col), ptr(self.lboff1_dev)))
            ep["keep_off_dev"] = None if self.keep_dev is None else \
                _h2d(np.ascontiguousarray(self.keep_off, dtype=np.int64), dev)
            ep["keep_off"] = None if ep["keep_off_dev"] is None else ep["keep_off_dev"].data_ptr()
            self._ep_tabs = ep
        return ep

    def _stage(self, parts, dev):
        """host arrays to the device in ONE copy through a persistent pinned staging buffer (8-byte aligned
        parts); returns the parts' device addresses.  A row-list build inside the bench's timed region starts on
        an idle GPU, so its host prelude counts: per-array pin_memory() + copy cost ~0.1-0.2 ms there.  The
        device buffer is reused by the next build: its copy is ordered on the stream after this build's kernels;
        the pinned one is rewritten only after this copy's event."""
        sizes = [(a.nbytes + 7) // 8 * 8 for a in parts]
        tot = max(sum(sizes), 8)
        if torch.device(dev).type != "cuda":
            flat = np.zeros(tot, dtype=np.uint8)
        st = getattr(self, "_stage_bufs", None)
        if torch.device(dev).type == "cuda":
            if st is None or st[0].numel() < tot:
                st = [torch.empty(2 * tot, dtype=torch.uint8, pin_memory=True),
                      torch.empty(2 * tot, dtype=torch.uint8, device=dev), None]
                self._stage_bufs = st
            if st[2] is not None:
                st[2].synchronize()
            flat = st[0].numpy()
        off, addr = 0, []
        for a, sz in zip(parts, sizes):
            flat[off:off + a.nbytes] = np.ascontiguousarray(a).view(np.uint8).ravel()
            addr.append(off)
            off += sz
        if torch.device(dev).type != "cuda":
            self._stage_bufs = [None, torch.as_tensor(flat), None]
            return [self._stage_bufs[1].data_ptr() + o for o in addr]
        st[1][:tot].copy_(st[0][:tot], non_blocking=True)
        st[2] = torch.cuda.Event()
        st[2].record()
        return [st[1].data_ptr() + o for o in addr]

    def _check_list_lengths(self, sel):
        """duplicate (row, col) ratings: a column can hold more entries than batch rows; the row-list build
        sorts a list of up to 4,096 entries (ocf_epoch_row_lists) -- refuse longer ones loudly"""
        csr = self.src1.host
        for bi in sel:
            idx = np.concatenate([np.arange(csr.row_ptr[r], csr.row_ptr[r + 1]) for r in self.rows_host[bi]])
            if len(idx) and np.bincount(csr.col[idx]).max() > ROWLIST_MAX_ENTRIES:
                raise ValueError("batch %d: a column holds more than %d entries (duplicate ratings); the row-list "
                                 "build takes at most %d per column -- use a smaller batch_size"
                                 % (bi, ROWLIST_MAX_ENTRIES, ROWLIST_MAX_ENTRIES))

    def row_lists(self, bi, n_cols):
        """device pointers of batch bi's row lists (sp_rowptr / sp_rowent of the row-stream weight-gradient
        kernel) and live records; the epoch's (or this rank's) are built on first use, in windows of at most
        ROWLIST_MAX_BATCHES batches"""
        rl = getattr(self, "_rl", None)
        if rl is None or rl["n_cols"] != n_cols or bi not in rl["slot"]:
            want = shard_batches(self.num_batches, *self.dp_shard) if self.dp_shard else range(self.num_batches)
            self.prepare_row_lists(n_cols, [b for b in want if b >= bi] or [bi])
            rl = self._rl
        s = rl["slot"][bi]
        e0 = int(rl["ebase_host"][s])
        return dict(row_ptr=rl["row_ptr"].data_ptr() + 4 * s * (n_cols + 1),
                    row_ent=rl["row_ent"].data_ptr() + 8 * e0,
                    live=rl["live"].data_ptr() + s * (n_cols // 128) * _lib.LIVE_REC,
                    xval=rl["xval"].data_ptr() + 4 * e0, tflag=rl["tflag"].data_ptr() + e0)

    def step_fields(self, bi, n_cols):
        """batch bi's table pointers and sizes for the one-call training step (Engine.fast_train_step):
        (rows, lboff, ch_row, ch_j0, ch_j1, n_chunks, row_cptr, max_chunks, entries, row_ptr, row_ent, live,
        xval, tflag) -- the values gather_tables / targets / row_lists give -- or None when batch bi's row
        lists are not built (row_lists builds them on the general path).  The batch-constant part is computed
        once per epoch plan, the window's part once per batch and window."""
        rl = getattr(self, "_rl", None)
        if self.split != "train" or rl is None or rl["n_cols"] != n_cols:
            return None
        s = rl["slot"].get(bi)
        if s is None:
            return None
        f = rl["fields"].get(bi)
        if f is None:
            ep = self._ep_fields
            if ep is None:
                # the epoch's batch-constant fields, once per epoch plan (tuples per batch)
                B, ch = self.B, self.chunks1
                sel = np.arange(self.num_batches, dtype=np.int64)
                c0 = ch["cbase"][:-1]
                cols = [self.rows_dev.data_ptr() + 4 * sel * B, self.lboff1_dev.data_ptr() + 8 * sel * (B + 1),
                        ch["ch_row"].data_ptr() + 4 * c0, ch["ch_j0"].data_ptr() + 4 * c0,
                        ch["ch_j1"].data_ptr() + 4 * c0, ch["cbase"][1:] - c0,
                        ch["row_cptr"].data_ptr() + 4 * sel * (B + 1), ch["max_chunks"], self.nnz1]
                ep = self._ep_fields = list(zip(*[np.asarray(c, dtype=np.int64).tolist() for c in cols]))
            # ... and the row-list window's
            e0 = int(rl["ebase_host"][s])
            f = rl["fields"][bi] = ep[bi] + (
                rl["row_ptr"].data_ptr() + 4 * s * (n_cols + 1), rl["row_ent"].data_ptr() + 8 * e0,
                rl["live"].data_ptr() + s * (n_cols // 128) * _lib.LIVE_REC, rl["xval"].data_ptr() + 4 * e0,
                rl["tflag"].data_ptr() + e0)
        return f

    @staticmethod
    def _local_offsets(lens, rows):
        off = np.zeros((rows.shape[0], rows.shape[1] + 1), dtype=np.int64)
        np.cumsum(lens[rows], axis=1, out=off[:, 1:])
        return off

    def scatter_args(self, bi, engine_args=None, dense=None, B_pad=None):
        """OcfScatterArgs for batch bi (onto an engine's xin/buckets and/or dense outputs)."""
        a = engine_args if engine_args is not None else _lib.OcfScatterArgs()
        B = self.B
        s1 = self.src1
        a.rp1, a.col1, a.val1, a.dup1 = ptr(s1.rp), ptr(s1.col), ptr(s1.val), ptr(s1.dup)
        a.pos1 = ptr(s1.pos)
        a.rows1 = self.rows_dev.data_ptr() + 4 * bi * B
        a.boff1 = self.boff_dev.data_ptr() + 8 * bi * (B + 1)
        a.lboff1 = self.lboff1_dev.data_ptr() + 8 * bi * (B + 1)
        a.E1 = int(self.nnz1[bi])
        a.keep1 = None if self.keep_dev is None else self.keep_dev.data_ptr() + int(self.keep_off[bi])
        if self.split == "train":
            a.mode = 0
            a.pass_through = int(self.pass_through)
            if self.r.rng == "device":
                a.s0, a.s1 = float(self.sparsity[0]), float(self.sparsity[1])
                a.seed, a.stream = self.seed, 2 * (bi + 1)
            else:
                a.s0 = a.s1 = 1.0
        else:
            a.mode = 1
            s2 = self.src2
            a.rp2, a.col2, a.val2, a.dup2 = ptr(s2.rp), ptr(s2.col), ptr(s2.val), ptr(s2.dup)
            a.rows2 = a.rows1
            a.lboff2 = self.lboff2_dev.data_ptr() + 8 * bi * (B + 1)
            a.E2 = int(self.tlocal[bi])
        a.B = B
        a.aux = self.aux
        a.feed = AUX_FEED[self.aux_type]
        a.both = int(self.aux_type == "both")
        if dense is not None:
            a.X, a.Min, a.Mout, a.T, a.Mmiss = [ptr(t) for t in dense]
            a.ld = dense[0].stride(0)
            a.B_pad = B_pad if B_pad is not None else B
        return a

    # ------------------------------------------------------------ fast path (Model.fit_generator)
    def next_batch_index(self):
        if not self.started:
            self._start()
        if self.i >= self.num_batches:
            return None
        bi = self.i
        self.i += 1
        return bi

    def targets(self, bi, n_cols):
        """Where batch bi's target entries live, for the masked-MSE epilogue's row-segment mode:
        the target CSR's tile index, the batch rows, their local entry offsets, the entry count and
        which scatter flag array (1 = train entries, 2 = eval target entries) marks live targets."""
        B = self.B
        train = self.split == "train"
        src = self.src1 if train else self.src2
        lb = self.lboff1_dev if train else self.lboff2_dev
        t = dict(src.tiles(n_cols))
        t.update(t_rows=self.rows_dev.data_ptr() + 4 * bi * B, t_rp=ptr(src.rp),
                 t_lboff=lb.data_ptr() + 8 * bi * (B + 1), t_aux=self.aux,
                 E=int(self.nnz1[bi] if train else self.tlocal[bi]), flag=1 if train else 2)
        return t

    def target_count(self, bi):
        """target_count of batch bi (data_reader.py:268): list entries of the target rows (full rows;
        under feature parallelism every rank reports the global count)"""
        return int(self.tcount[bi]) if self.tcount is not None else None

    # ------------------------------------------------------------ reference-compatible iteration
    def __iter__(self):
        return self

    def __next__(self):
        bi = self.next_batch_index()
        if bi is None:
            return None                                                                 # :418-419
        B, N = self.B, self.r.num_items
        ld = ru(N, 4)
        buf = torch.empty(5, B, ld, device=self.r.device, dtype=torch.float32)
        X, Min, Mout, T, Mmiss = buf[0], buf[1], buf[2], buf[3], buf[4]
        a = self.scatter_args(bi, dense=(X, Min, Mout, T, Mmiss))
        _lib.call("ocf_scatter_batch", a, cur_stream())
        v = lambda t: t[:, :N]
        x, m_in, m_out, t, m_miss = v(X), v(Min), v(Mout), v(T), v(Mmiss)
        if self.aux_type is None:
            inputs = [x, m_out]
        else:
            feed = {"causal": m_miss, "dropout": m_in, "both": m_in,
                    "zeros": torch.zeros_like(m_in)}[self.aux_type]
            inputs = [x, feed, m_out]
            if self.aux_type == "both":
                inputs.append(m_miss)
        if self.split != "train" and self.return_count:
            return inputs, t, self.target_count(bi)
        return inputs, t

    next = __next__   # py2-style gen.next() as used at train.py:233
