"""Drop-in for the reference's ``omni_model`` (model.py:33-99) and the Keras ``Model`` subset that
train.py / train_jester.py use: compile, fit_generator, evaluate_generator, predict, fit,
train_on_batch, test_on_batch, save, metrics_names, get_weights / set_weights.

Graph (model.py:43-99):  x = concat([data, observed_mask?, second_mask?]);
L x [Dense(H, act) -> Dropout(p, noise_shape=[B, H])] ; y = output_mask * Dense(N, linear)(x)
Loss: Keras 'mean_squared_error' (train.py:49).  Everything runs through engine.Engine on the GPU.
"""
from __future__ import annotations

import time

import numpy as np
import torch

from . import metrics as M
from . import optimizers
from .data_reader import BatchGenerator
from .engine import Engine


class History(object):
    def __init__(self):
        self.history = {}
        self.epoch = []


class EarlyStopping(object):
    """keras.callbacks.EarlyStopping(monitor, min_delta, patience, mode='auto') as train_jester.py:65 uses it."""

    def __init__(self, monitor="val_loss", min_delta=0, patience=0, verbose=0, mode="auto"):
        self.monitor, self.min_delta, self.patience = monitor, min_delta, patience
        self.best = np.inf
        self.wait = 0
        self.stop = False

    def on_epoch_end(self, logs):
        v = logs.get(self.monitor)
        if v is None:
            return
        if v < self.best - self.min_delta:
            self.best, self.wait = v, 0
        else:
            self.wait += 1
            if self.wait > self.patience:
                self.stop = True


class Model(object):
    def __init__(self, engine, use_causal_info, use_both_masks, rating_range=1.0):
        self.engine = engine
        self.use_causal_info = use_causal_info
        self.use_both_masks = use_both_masks
        self.optimizer = None
        self.metric_names = []
        self.rating_range = float(rating_range)
        self.stop_training = False
        self.rank, self.world, self.dp = 0, 1, None
        # feature parallelism (engine built with shard / comm): (rank, world) for per-shard checkpoints
        self.fp = None

    def enable_data_parallel(self, rank, world, mode="sharded", grad_dtype="float32"):
        """Row data parallelism (parallel.DataParallel): call on every rank after torch.distributed is
        initialised and the model is compiled; rank 0's weights are broadcast."""
        from .parallel import DataParallel
        if self.engine.comm is not None:
            raise ValueError("data parallelism over a feature-parallel (column-sharded) engine is not supported")
        self.rank, self.world = int(rank), int(world)
        self.dp = DataParallel(self.engine, rank, world, mode=mode, grad_dtype=grad_dtype) if world > 1 else None

    def enable_feature_parallel(self, rank, world):
        """record the column-shard layout (the engine was built with shard=/comm=) for checkpoints"""
        self.fp = (int(rank), int(world))

    def _train_one(self, gen):
        """One optimizer step; under data parallelism rank r takes the r-th of the next `world` batches."""
        if self.world > 1 and isinstance(gen, BatchGenerator):
            gen.dp_shard = (self.rank, self.world)
            idx = [gen.next_batch_index() for _ in range(self.world)]
            if idx[-1] is None:
                raise StopIteration("generator exhausted")
            self._check_gen(gen)
            self._load(None, gen, idx[self.rank])
        elif self.dp is None and isinstance(gen, BatchGenerator):
            self._check_gen(gen)
            bi = gen.next_batch_index()
            if bi is None:
                raise StopIteration("generator exhausted (data_reader.py:418 yields None)")
            # the whole step in one library call when the engine's template applies (Engine.fast_train_step)
            if not self.engine.fast_train_step(gen, bi):
                self._load(None, gen, bi)
                self.engine.train_step()
            return
        else:
            self._pull(gen)
        if self.dp is not None:
            self.dp.step()
        else:
            self.engine.train_step()

    # ------------------------------------------------------------------ compile
    def compile(self, optimizer, loss="mean_squared_error", metrics=None, rating_range=None):
        if loss not in ("mean_squared_error", "mse"):
            raise NotImplementedError("only the masked 'mean_squared_error' loss of train.py:49 is implemented")
        self.optimizer = optimizers.get(optimizer)
        self.engine.set_optimizer(self.optimizer)
        self.metric_names = [M.metric_name(m) for m in (metrics or [])]
        if rating_range is not None:
            self.rating_range = float(rating_range)

    @property
    def metrics_names(self):
        return ["loss"] + list(self.metric_names)

    def _logs_from_stats(self, st, rows=None):
        """st: [steps, 4 + Bp] device stats -> epoch-mean logs.  rows: the row count of every step's batch
        (None: all full) -- Keras weights each batch's values by its size (BaseLogger for the training
        logs, _test_loop for evaluation), which matters only for Model.fit's trailing partial batch."""
        e = self.engine
        B = e.B
        rows = [B] * len(st) if rows is None else list(rows)
        assert len(rows) == len(st)
        out = {k: [] for k in self.metrics_names}
        for row, b in zip(st, rows):
            sse, sae, cnt = row[0], row[1], row[2]
            # Keras' total loss = MSE + the kernels' l2 penalty (row[3], 0 without l2); metrics have none
            out["loss"].append(sse / (b * e.N_total) + row[3])
            for name in self.metric_names:
                out[name].append(M.from_stats(name, sse, sae, cnt, row[4:], B, e.N_total, self.rating_range, rows=b))
        w = np.asarray(rows, np.float64)
        return {k: float(np.dot(v, w) / w.sum()) if v else float("nan") for k, v in out.items()}

    # ------------------------------------------------------------------ batch plumbing
    def _split_inputs(self, x):
        """model.py:89-97 input order -> (layer-0 blocks, output mask)."""
        x = list(x)
        if self.use_causal_info:
            blocks = [x[0], x[1]]
            out_mask = x[2]
            rest = x[3:]
        else:
            blocks = [x[0]]
            out_mask = x[1]
            rest = x[2:]
        if self.use_both_masks:
            blocks.append(rest[0])
        return blocks, out_mask

    def _load(self, item, gen=None, bi=None):
        e = self.engine
        if gen is not None:
            args = gen.scatter_args(bi, engine_args=e.scatter_args())
            e.load_batch(args, gen.targets(bi, e.N), gather=gen.gather_tables(bi))
            return gen.target_count(bi)
        x, y = item[0], item[1]
        blocks, out_mask = self._split_inputs(x)
        e.load_dense(blocks, out_mask, y)
        return item[2] if len(item) > 2 else None

    def _pull(self, gen):
        if isinstance(gen, BatchGenerator):
            self._check_gen(gen)
            bi = gen.next_batch_index()
            if bi is None:
                raise StopIteration("generator exhausted (data_reader.py:418 yields None)")
            return self._load(None, gen, bi)
        item = next(gen)
        if item is None:
            raise StopIteration("generator yielded None")
        return self._load(item)

    def _check_gen(self, gen):
        e = self.engine
        if gen.B != e.B:
            raise ValueError("generator batch_size %d != model batch_size %d (Dropout noise_shape, model.py:73)"
                             % (gen.B, e.B))
        want_k = 1 + int(self.use_causal_info) + int(self.use_both_masks)
        have_k = 1 + int(gen.aux_type is not None) + int(gen.aux_type == "both")
        if want_k != have_k:
            raise ValueError("auxilliary_mask_type=%r does not match the model inputs" % (gen.aux_type,))

    # ------------------------------------------------------------------ training
    def train_on_batch(self, x, y):
        self._load((x, y))
        self.engine.train_step()
        return self._finish(self.engine.take_stats())

    def test_on_batch(self, x, y):
        self._load((x, y))
        self.engine.eval_step()
        return self._finish(self.engine.take_stats())

    def _finish(self, st):
        logs = self._logs_from_stats(st)
        vals = [logs[k] for k in self.metrics_names]
        return vals[0] if len(vals) == 1 else vals

    def fit_generator(self, generator, steps_per_epoch, epochs=1, verbose=1, callbacks=None, validation_data=None,
                      validation_steps=None, initial_epoch=0, **kw):
        hist = History()
        callbacks = callbacks or []
        steps = int(steps_per_epoch)
        for epoch in range(initial_epoch, epochs):
            t0 = time.time()
            for _ in range(steps // self.world if self.world > 1 else steps):
                self._train_one(generator)
            logs = self._logs_from_stats(self.engine.take_stats())
            if self.world > 1:
                logs = self._mean_over_ranks(logs)
            if validation_data is not None:
                vals = self.evaluate_generator(validation_data, validation_steps)
                vals = vals if isinstance(vals, list) else [vals]
                for k, v in zip(self.metrics_names, vals):
                    logs["val_" + k] = v
            for k, v in logs.items():
                hist.history.setdefault(k, []).append(v)
            hist.epoch.append(epoch)
            if verbose:
                print("Epoch %d - %.1fs - " % (epoch + 1, time.time() - t0) +
                      " - ".join("%s: %.4f" % kv for kv in logs.items()))
            for cb in callbacks:
                cb.on_epoch_end(logs)
                self.stop_training |= getattr(cb, "stop", False)
            if self.stop_training:
                break
        return hist

    def _mean_over_ranks(self, logs):
        import torch.distributed as dist
        keys = sorted(logs)
        t = torch.tensor([logs[k] for k in keys], dtype=torch.float64, device=self.engine.dev)
        dist.all_reduce(t)
        return {k: float(v) / self.world for k, v in zip(keys, t.tolist())}

    def evaluate_generator(self, generator, steps, **kw):
        steps = int(steps)
        self.engine.take_stats()
        for _ in range(steps):
            self._pull(generator)
            self.engine.eval_step()
        return self._finish(self.engine.take_stats())

    def evaluate_sse(self, generator, steps):
        """Fused form of train.py:225-255: (sum of squared errors, sum of target_count)."""
        self.engine.take_stats()
        count = 0
        for _ in range(int(steps)):
            c = self._pull(generator)
            self.engine.eval_step()
            count += int(c) if c is not None else 0
        st = self.engine.take_stats()
        return float(st[:, 0].sum()), count

    def predict(self, x, batch_size=None, verbose=0):
        """Returns y = output_mask * (h W_out + b_out) as a float32 CUDA tensor [B, N].

        Collective under data parallelism with ZeRO-1 (enable_data_parallel(mode="sharded")): the output
        layer reads the fp32 masters, which each rank holds only 1/G of, so every rank must call predict
        together (the masters are all-gathered first); a rank-0-only predict would wait forever."""
        e = self.engine
        blocks, out_mask = self._split_inputs(x)
        dummy_t = torch.zeros(e.B, e.N, device=e.dev)
        e.load_dense(blocks, out_mask, dummy_t)
        e.forward(training=False)
        out = torch.empty(e.B, e.N, device=e.dev, dtype=torch.float32)
        om = out_mask if torch.is_tensor(out_mask) else torch.as_tensor(np.asarray(out_mask, np.float32))
        om = om.to(e.dev, torch.float32).contiguous()
        e.predict_dense(om, out)
        return out

    def fit(self, x, y, batch_size=None, epochs=1, verbose=1, callbacks=None, validation_split=0.0, shuffle=True,
            **kw):
        """Keras 2.0.4 Model.fit on dense arrays (train_jester.py:78-79): the last validation_split fraction
        held out (split_at = int(n (1 - validation_split))), np.random.shuffle of the training indices each
        epoch, ceil(n / batch_size) batches -- the last one partial --, epoch logs weighted by batch size
        (BaseLogger) and the validation logs by sample over every held-out row (_test_loop).  With a Dropout
        layer the reference fixes noise_shape = [batch_size, H] (model.py:73), so a partial batch cannot run
        there: with dropout only full TRAINING batches are taken.  Evaluation runs the layer through
        in_train_phase (its noise never applies at test time), so the validation logs always cover every
        held-out row, the trailing partial batch included."""
        e = self.engine
        bs = int(batch_size or e.B)
        if bs != e.B:
            raise ValueError("batch_size must equal the model batch_size (Dropout noise_shape, model.py:73)")
        partial = e.keep >= 1.0
        # the arrays go to the device once, plus one all-zero row that pads a partial batch (its input, output
        # mask and target are zero, so it adds nothing to the loss, the statistics or any gradient; the
        # gradient scale uses the real row count); every batch is then gathered there by row index (no per-step
        # host copies, no synchronisation between steps)
        dev = e.dev

        def on_dev(a):
            t = a if torch.is_tensor(a) else torch.as_tensor(np.ascontiguousarray(a, dtype=np.float32))
            out = torch.zeros(t.shape[0] + 1, t.shape[1], device=dev, dtype=torch.float32)
            out[:-1] = t.to(dev, torch.float32)
            return out
        xd = [on_dev(a) for a in x]
        yd = on_dev(y)
        n = xd[0].shape[0] - 1
        split_at = int(n * (1.0 - validation_split)) if validation_split else n
        hist = History()
        callbacks = callbacks or []

        def batches(m, allow_partial):
            full, rest = divmod(m, bs)
            return [(s * bs, bs) for s in range(full)] + ([(full * bs, rest)] if rest and allow_partial else [])

        def rows_of(ix, b):
            if b == bs:
                return ix
            return torch.cat([ix, torch.full((bs - b,), n, dtype=torch.int64, device=dev)])
        val_rows = torch.arange(split_at, n, dtype=torch.int64, device=dev)
        for epoch in range(epochs):
            idx = np.arange(split_at)
            if shuffle:
                np.random.shuffle(idx)
            idx_d = torch.as_tensor(idx, dtype=torch.int64).to(dev)
            tb = batches(split_at, partial)
            for s0, b in tb:
                self._load_rows(xd, yd, rows_of(idx_d[s0:s0 + b], b), b)
                e.train_step()
            logs = self._logs_from_stats(e.take_stats(), [b for _, b in tb])
            vb = batches(n - split_at, True)
            if vb:
                for s0, b in vb:
                    self._load_rows(xd, yd, rows_of(val_rows[s0:s0 + b], b), b)
                    e.eval_step()
                vl = self._logs_from_stats(e.take_stats(), [b for _, b in vb])
                for k, v in vl.items():
                    logs["val_" + k] = v
            for k, v in logs.items():
                hist.history.setdefault(k, []).append(v)
            hist.epoch.append(epoch)
            for cb in callbacks:
                cb.on_epoch_end(logs)
                self.stop_training |= getattr(cb, "stop", False)
            if self.stop_training:
                break
        return hist

    def _load_rows(self, xd, yd, rows, real=None):
        """batch = rows `rows` of the device-resident arrays of Model.fit (the first `real` of them real)"""
        blocks, out_mask = self._split_inputs(xd)
        self.engine.load_dense(blocks, out_mask, yd, rows=rows, rows_real=real)

    # ------------------------------------------------------------------ weights / checkpoints
    def get_weights(self):
        """Keras-layout weights.  Collective under data parallelism with ZeRO-1 (the sharded fp32 masters
        are all-gathered first): call it on every rank, as predict and save."""
        return self.engine.get_weights()

    def set_weights(self, weights):
        self.engine.set_weights(weights)

    def shard_path(self, path):
        """feature parallelism: every rank checkpoints its own column shard"""
        if self.fp is None:
            return path
        return "%s.shard%dof%d" % (path, self.fp[0], self.fp[1])

    def save(self, path):
        """Weights (Keras layout) + optimizer state in a safetensors file (replaces the h5 of train.py:169).
        Collective under data parallelism (the sharded optimizer slots are gathered first; rank 0 writes)
        and under feature parallelism (every rank writes its shard, Model.shard_path)."""
        from safetensors.numpy import save_file
        e = self.engine
        if self.dp is not None:
            self.dp.gather_slots()
            if e.master_sync is not None:       # ZeRO-1 masters: a collective, so on every rank
                e.master_sync()
            if self.rank != 0:
                return
        path = self.shard_path(path)
        tensors = {}
        for i, w in enumerate(e.get_weights()):
            tensors["param/%d" % i] = np.ascontiguousarray(w)
        if self.optimizer is not None and e.slots:
            for i, (sw, sb) in enumerate(e.slots):
                for j, t in enumerate(sw):
                    if t is not None:
                        tensors["opt/W%d/%d" % (i, j)] = t.cpu().numpy()
                for j, t in enumerate(sb):
                    if t is not None:
                        tensors["opt/b%d/%d" % (i, j)] = t.cpu().numpy()
            tensors["opt/iterations"] = np.array([self.optimizer.iterations], np.int64)
        save_file(tensors, path)

    def load(self, path, with_optimizer=True):
        from safetensors.numpy import load_file
        t = load_file(self.shard_path(path))
        n = len([k for k in t if k.startswith("param/")])
        self.set_weights([t["param/%d" % i] for i in range(n)])
        e = self.engine
        if with_optimizer and self.optimizer is not None and "opt/iterations" in t:
            for i, (sw, sb) in enumerate(e.slots):
                for j, s in enumerate(sw):
                    if s is not None:
                        s.copy_(torch.as_tensor(t["opt/W%d/%d" % (i, j)]))
                for j, s in enumerate(sb):
                    if s is not None:
                        s.copy_(torch.as_tensor(t["opt/b%d/%d" % (i, j)]))
            self.optimizer.iterations = int(t["opt/iterations"][0])


class _Donor(object):
    """weights of a saved model (Model.save safetensors) in the Keras order, for the transfer helpers"""

    def __init__(self, weights):
        self.weights = weights

    def get_weights(self):
        return self.weights


def load_donor(path):
    """the donor model of train.py:136-145 (keras.models.load_model there; a Model.save file here)"""
    from safetensors.numpy import load_file
    t = load_file(path)
    return _Donor([t["param/%d" % i] for i in range(len([k for k in t if k.startswith("param/")]))])


class omni_model(object):
    """model.py:34-35 signature; extra keyword ``compute_dtype`` ('float32' = exact-fp32 MFMA, the
    parity mode; 'float16' / 'bfloat16' MFMA with fp32 accumulation) and ``seed``."""

    def __init__(self, numlayers, num_hidden_units, input_shape, batch_size, dense_activation="tanh",
                 use_causal_info=True, use_timestamps=False, use_both_masks=False, l2_weight_regulatization=None,
                 sparse_representation=False, dropout_probability=None, use_sparse_masking_layer=False,
                 compute_dtype="float32", seed=None, device=None, rating_range=1.0, shard=None, comm=None):
        if use_timestamps:
            raise NotImplementedError("use_timestamps: broken in the reference; not supported")
        if sparse_representation:
            raise NotImplementedError("sparse_representation: needs a patched Keras in the reference; dense only")
        if use_sparse_masking_layer:
            raise NotImplementedError("Dynamic_Masking_Layer is broken in the reference (model.py:186)")
        self.numlayers = numlayers
        self.num_hidden_units = num_hidden_units
        self.input_shape = input_shape
        self.batch_size = batch_size
        k = 1 + int(bool(use_causal_info)) + int(bool(use_both_masks))
        self.engine = Engine(input_shape, [num_hidden_units] * numlayers, batch_size, k_blocks=k,
                             activation=dense_activation, dropout=dropout_probability, l2=l2_weight_regulatization,
                             compute_dtype=compute_dtype, device=device, seed=seed, shard=shard, comm=comm)
        self.model = Model(self.engine, bool(use_causal_info), bool(use_both_masks), rating_range)

    def save_weights(self, filename):
        self.model.save(filename)

    def load_weights(self, weights):
        self.model.set_weights(weights)

    # ---- transfer / denoising-autoencoder helpers (model.py:107-170) ------------------------
    # Every dense layer of the omni model has an input or output width equal to the hidden width, so
    # the reference's layer filter selects all of them, in order: hidden layers, then the output
    # layer.  ``trainable`` takes effect immediately (Keras needs a recompile, model.py:135).
    @staticmethod
    def _dense_weights(donor):
        eng = donor.engine if hasattr(donor, "engine") else donor
        w = eng.get_weights()
        return [[w[2 * i], w[2 * i + 1]] for i in range(len(w) // 2)]

    def _set_layer(self, i, wb):
        w = self.model.get_weights()
        w[2 * i], w[2 * i + 1] = wb
        self.model.set_weights(w)

    def replace_dense_layer_weights(self, donor_model, layers_to_replace, make_layers_trainable=False):
        """model.py:107-125: copy the selected dense layers from the donor; set their trainable flag."""
        donor = self._dense_weights(donor_model)
        if layers_to_replace == "all":
            layers_to_replace = [True] * len(donor)
        for i in range(len(self.engine.W)):
            if i < len(layers_to_replace) and layers_to_replace[i]:
                self._set_layer(i, donor[i])
                self.engine.trainable[i] = bool(make_layers_trainable)
                print("Loaded weights for dense layer ", i)

    def manually_load_all_weights(self, donor_model):
        """model.py:127-132: every layer's weights from the donor (same architecture)."""
        eng = donor_model.engine if hasattr(donor_model, "engine") else donor_model
        self.model.set_weights(eng.get_weights())

    def make_trainable(self):
        """model.py:134-138: layers whose OUTPUT width is the hidden width become trainable (the
        output layer keeps its flag -- the reference's filter)."""
        for i in range(len(self.engine.W) - 1):
            self.engine.trainable[i] = True

    def load_and_fix_for_denoising_autoencoders(self, donor_model):
        """model.py:140-170: the outer floor(D/2) donor layers on each side are copied into this
        model's first / last layers and frozen; the middle layers stay trainable."""
        donor = self._dense_weights(donor_model)
        print("Number of weight layers to donate", len(donor))
        k = len(donor) // 2
        n_new = len(self.engine.W)
        for i in range(n_new):
            if i < k:
                self._set_layer(i, donor[i])
                self.engine.trainable[i] = False
                print("Loaded and fixed weights for dense layer ", i, " from donor dense layer ", i)
            elif i >= n_new - k:
                src = len(donor) - (n_new - i)
                self._set_layer(i, donor[src])
                self.engine.trainable[i] = False
                print("Loaded and fixed weights for dense layer ", i, " from donor dense layer ", src)
