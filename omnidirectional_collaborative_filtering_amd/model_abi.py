"""The model-level C ABI (include/ocf.h "Model ABI": ocf_ctx_create / ocf_forward / ocf_masked_mse /
ocf_backward + ocf_opt_step) driven over ctypes -- the binding a caller with its own training loop writes
(INTEGRATION.md shows the same for the reference's side).  One train step is the reference's
Keras train_on_batch (/root/reference/train.py:157 -> model.py:64-86, train.py:49-51) as five library calls:

    forward(inputs, out_mask) -> masked_mse(pred, targets, out_mask) -> backward(grad) -> opt_step per param

Parameters, optimizer slots and gradients are fp32 device tensors in the padded Keras layout
(ocf_model_dims), owned here; the library's context owns only the per-batch activations.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import call


def ptr(t):
    return None if t is None else t.data_ptr()


class ModelABI:
    def __init__(self, N, hidden, max_batch, k_blocks=1, activation="sigmoid", dropout=0.0,
                 compute_dtype="float32", seed=0, optimizer=None, device="cuda"):
        if not torch.cuda.is_available():
            raise RuntimeError("ModelABI needs a ROCm GPU (MI355X)")
        _lib.load()
        self.N, self.k, self.H, self.B_max = int(N), int(k_blocks), [int(h) for h in hidden], int(max_batch)
        self.dev = torch.device(device)
        d = _lib.OcfModelDesc()
        d.n_hidden, d.N, d.k_blocks = len(self.H), self.N, self.k
        for i, h in enumerate(self.H):
            d.hidden[i] = h
        d.act = _lib.ACT[activation]
        d.dropout = float(dropout or 0.0)
        d.compute_dtype = {"float32": _lib.DT_F32, "float16": _lib.DT_F16, "bfloat16": _lib.DT_BF16}[compute_dtype]
        d.max_batch, d.seed = self.B_max, int(seed)
        n = len(self.H) + 1
        rows, cols = (ctypes.c_int64 * n)(), (ctypes.c_int64 * n)()
        call("ocf_model_dims", d, rows, cols)
        self.shapes = [(rows[i], cols[i]) for i in range(n)]
        f = dict(device=self.dev, dtype=torch.float32)
        self.W = [torch.zeros(r, c, **f) for r, c in self.shapes]
        self.b = [torch.zeros(c, **f) for _, c in self.shapes]
        self.gW = [torch.zeros_like(w) for w in self.W]
        self.gb = [torch.zeros_like(b) for b in self.b]
        for i in range(n):
            d.W[i], d.b[i] = ptr(self.W[i]), ptr(self.b[i])
        self.desc = d
        self.ctx = ctypes.c_void_p()
        call("ocf_ctx_create", d, ctypes.byref(self.ctx))
        self.real = [self.k * self.N] + self.H + [self.N]
        self.Np = self.shapes[-1][1]
        self.step = 0
        self._bufs = {}
        self.opt = None
        if optimizer is not None:
            self.set_optimizer(optimizer)

    def __del__(self):
        ctx = getattr(self, "ctx", None)
        if ctx:
            try:
                _lib.load().ocf_ctx_destroy(ctx)
            except Exception:          # interpreter shutdown: the module globals may already be gone
                pass
            self.ctx = None

    # Keras-layout weights in / out (padding stripped; layer 0's block j at rows j * Np ...)
    def _rows0(self):
        blk = np.arange(self.k * self.N) // self.N
        return blk * self.Np + np.arange(self.k * self.N) % self.N

    def set_weights(self, weights):
        for i in range(len(self.W)):
            w = torch.as_tensor(np.asarray(weights[2 * i], np.float32))
            rows = self._rows0() if i == 0 else np.arange(self.real[i])
            full = torch.zeros(self.shapes[i])
            full[torch.as_tensor(rows), : self.real[i + 1]] = w
            self.W[i].copy_(full)
            self.b[i].zero_()
            self.b[i][: self.real[i + 1]] = torch.as_tensor(np.asarray(weights[2 * i + 1], np.float32))

    def get_weights(self):
        out = []
        for i in range(len(self.W)):
            rows = self._rows0() if i == 0 else np.arange(self.real[i])
            out.append(self.W[i].cpu().numpy()[rows, : self.real[i + 1]])
            out.append(self.b[i].cpu().numpy()[: self.real[i + 1]])
        return out

    def set_optimizer(self, opt):
        self.opt = opt
        self.slots = [[torch.zeros_like(p) for _ in range(opt.n_slots)] + [None] * (2 - opt.n_slots)
                      for p in self.W + self.b]

    def _out(self, name, *shape):
        """a reused output buffer: the calls write every element they own (ocf.h: pred / out_grad for b < B,
        n < N, all 4 + 3 B stats), so nothing is zero-filled per call"""
        t = self._bufs.get(name)
        if t is None or tuple(t.shape) != shape:
            t = self._bufs[name] = torch.empty(*shape, device=self.dev, dtype=torch.float32)
        return t

    # the five calls
    def forward(self, inputs, out_mask, B, training, masks_out=None):
        """ocf_forward into the reused buffer self.pred (overwritten by the next call: clone to keep it)"""
        s = torch.cuda.current_stream().cuda_stream
        self.pred = self._out("pred", B, self.N)
        ins = (ctypes.c_void_p * self.k)(*[ptr(x) for x in inputs])
        mo = None
        if masks_out is not None:
            mo = (ctypes.c_void_p * len(self.H))(*[ptr(m) for m in masks_out])
        call("ocf_forward", self.ctx, ins, inputs[0].stride(0), B, int(training), self.step,
             ptr(out_mask), out_mask.stride(0) if out_mask is not None else 0, ptr(self.pred), self.N, mo, s)
        return self.pred

    def masked_mse(self, pred, targets, out_mask, B):
        """ocf_masked_mse into the reused buffers self.grad / self.stats (overwritten by the next call)"""
        s = torch.cuda.current_stream().cuda_stream
        # ocf_masked_mse takes one row stride for pred / targets / mask: [B][N] contiguous (data_gen's arrays are
        # views with a padded stride)
        targets = targets if targets.stride(0) == self.N else targets.contiguous()
        out_mask = out_mask if out_mask is None or out_mask.stride(0) == self.N else out_mask.contiguous()
        self.grad = self._out("grad", B, self.N)
        self.stats = self._out("stats", 4 + 3 * B)
        call("ocf_masked_mse", ptr(pred), ptr(targets), ptr(out_mask), self.N, B, self.N, ptr(self.grad), self.N,
             ptr(self.stats), s)
        return self.grad, self.stats

    def backward(self, grad, B):
        s = torch.cuda.current_stream().cuda_stream
        n = len(self.W)
        gw = (ctypes.c_void_p * n)(*[ptr(g) for g in self.gW])
        gb = (ctypes.c_void_p * n)(*[ptr(g) for g in self.gb])
        call("ocf_backward", self.ctx, ptr(grad), grad.stride(0), B, 2.0 / (B * self.N), gw, gb, s)

    def opt_step(self):
        s = torch.cuda.current_stream().cuda_stream
        op = self.opt.step_params(1.0, 0.0)
        for p, g, sl in zip(self.W + self.b, self.gW + self.gb, self.slots):
            call("ocf_opt_step", ptr(p), ptr(g), ptr(sl[0]), ptr(sl[1]), p.numel(), op, s)
        self.opt.iterations += 1

    def train_on_batch(self, inputs, out_mask, targets, masks_out=None):
        """train.py:157's per-batch step; returns this step's device stats (ocf_masked_mse layout) as a fresh
        tensor (4 + 3 B floats), so a caller may keep per-step stats on the device and read them later.
        forward / masked_mse return the model's reused output buffers instead (pred, grad, stats: the next
        call overwrites them)."""
        B = targets.shape[0]
        pred = self.forward(inputs, out_mask, B, True, masks_out)
        grad, stats = self.masked_mse(pred, targets, out_mask, B)
        self.backward(grad, B)
        self.opt_step()
        self.step += 1
        return stats.clone()
