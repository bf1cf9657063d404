"""Headline benchmark: ML-20M-shaped I-AutoRec training steps on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

One step = one pass of the hot path over one batch resident in HBM: the epoch's batch
preparation for the timed batches, the row-gather encoder, the row-gather decoder with the hidden layer's
epilogue and the fused masked MSE, and both weight updates (row-stream dW + Adagrad, one launch) -- at N>1
each rank runs its column shard of the same step with two [B*G, H] all-reduces (feature layout, default)
or the data-parallel step (--parallel dp).  Configuration = train.py's
(sigmoid, dropout 0.2, Adagrad lr 0.005, pass-through training, data_sparsity [1,1]) at
BASELINE.json configs[2]: ML-20M I-AutoRec (26,744 item rows x 138,493 users), 500 hidden units,
batch 256, fp16 MFMA with fp32 accumulation.  Data: synthetic, ML-20M density, seeded.

Prints ONE JSON line (rank 0).  value = ratings/s summed over ranks = sum of input ratings
processed / max-over-ranks wall time of the K timed steps.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "ratings/sec + masked-RMSE, ML-20M I-AutoRec at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
MFMA_F16_PEAK_TFS = 2500.0     # dense f16/bf16 MFMA (spec)
OPT_STATE_BYTES = {"adagrad": 16, "rmsprop": 16, "adam": 24, "sgd": 8}
TIMER_EVERY = 4                # timed steps per dominant-kernel event sample
TIMER_EVERY_SHORT = 10         # ... when the dominant kernel is short (< 0.1 ms): a sample's two event records idle
                               # the stream ~11 us, ~6 % of an ML-100K step at every 4th step


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="ml20m")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--skew", type=float, default=0.0,
                    help="synthetic item / user popularity ~ rank^-skew (0: uniform; 0.5: ML-20M-like heavy "
                         "tail with duplicates removed, so somewhat fewer ratings)")
    ap.add_argument("--hidden", type=int, default=500)
    ap.add_argument("--dtype", default="float16")
    ap.add_argument("--optimizer", default="adagrad")
    ap.add_argument("--dropout", type=float, default=0.2)
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--cpu-steps", type=int, default=2)
    ap.add_argument("--fp32-steps", type=int, default=10,
                    help="N=1, 16-bit runs: also time this many steps of the exact-fp32 parity mode "
                         "(compute_dtype float32; reported as fp32_parity_mode, not the headline)")
    ap.add_argument("--phase-timers", type=int, default=1)
    ap.add_argument("--epoch", type=int, default=1,
                    help="N=1: also time one whole training epoch through fit_generator (train.py:157: floor(n/B)-1 "
                         "steps, the epoch plan and the reference RNG's draws included; reported as full_epoch)")
    ap.add_argument("--rmse", type=int, default=1)
    ap.add_argument("--configs", type=int, default=1,
                    help="N=1, default workload: also run the other BASELINE configs as short child benches "
                         "(ml100k, ml1m, ml1m_u, jester, netflix) and report them in the line's 'configs' object")
    ap.add_argument("--emulate-shards", type=int, default=0,
                    help="diagnostic: run rank 0 of a G-way feature-parallel job alone (collectives skipped, "
                         "numerics of a partial model); not a bench line")
    ap.add_argument("--emulate-comm", type=int, default=1,
                    help="with --emulate-shards: run the rank's collective code path with no-op collectives")
    ap.add_argument("--enc-tiles", type=int, default=-1,
                    help="the encoder over column tiles on the matrix cores (ocf_encoder_tiles; 1), the row gathers (0), "
                         "or the engine's choice by entries per weight row (-1)")
    ap.add_argument("--parallel", default="feature", choices=["feature", "dp"],
                    help="N>1: feature (column-sharded W1/W_out, 2 x [B,H] all-reduces per step) or dp "
                         "(replicated weights, gradient exchange)")
    ap.add_argument("--dp-mode", default="sharded", choices=["sharded", "allreduce"],
                    help="dp: reduce-scatter + sharded optimizer + all-gather, or one all-reduce + full optimizer")
    ap.add_argument("--dp-grad-dtype", default="float32", choices=["float32", "bfloat16"],
                    help="dp sharded: gradient dtype of the reduce-scatter")
    return ap.parse_args()


class _NoComm:
    """--emulate-shards with --emulate-comm: the feature-parallel rank step with its collectives replaced by
    no-ops (same kernels, streams and ordering as a real rank; the all-reduce time itself is missing)"""

    class _Work:
        def wait(self):
            pass

    def __call__(self, t):
        pass

    def start(self, t):
        return self._Work()


def compute_label(eng, dtype, dom):
    """what the step's arithmetic runs on (config.compute)"""
    dt = {"float16": "f16", "bfloat16": "bf16", "float32": "fp32"}[dtype]
    if dom == "mlp_step":
        return "%s operands, %s MFMA, fp32 accumulate (one ocf_mlp_step launch)" % (dt, dt)
    if eng.use_sparse and eng.sparse_ok and eng.sparse_dw:
        return ("%s operands, fp32 VALU accumulate (row gathers for the encoder / decoder, row-stream weight "
                "updates)" % dt)
    return "%s operands, %s MFMA, fp32 accumulate (dense GEMMs)" % (dt, dt)


def optim(name, lr):
    from omnidirectional_collaborative_filtering_amd import optimizers as O
    return {"adagrad": lambda: O.Adagrad(lr=lr, epsilon=1e-8), "rmsprop": lambda: O.RMSprop(lr=lr),
            "adam": lambda: O.Adam(lr=lr), "sgd": lambda: O.SGD(lr=lr)}[name]()


# BASELINE.json configs by workload name: (index, dataset shape label)
CONFIGS = {"ml100k": (0, "ML-100K", "1,682 x 943"), "ml1m": (1, "ML-1M", "3,706 x 6,040"),
           "ml1m_u": (1, "ML-1M (U orientation: 256 users x 3,706 items)", "6,040 x 3,706"),
           "ml20m": (2, "ML-20M", "26,744 x 138,493"), "netflix": (3, "Netflix", "17,770 x 480,189")}
REF_ASM_MS_PER_128 = {"ml20m": 233.9, "ml1m": 41.7}   # the reference's own assembler, 1 core


def cpu_baseline(data, rows_batches, N, H, w0, lr, n_steps, config):
    """The oracle restatement on the host cores (bounded sample): the reference's batch assembler
    restated with its own data structures (ReaderOracle: dict of rows -> [[column id string, rating]],
    column ids through the id dict, per-rating scalar stores into float64 zeros; data_reader.py:95-200,
    one core) + a NumPy fp32 dense model step (Keras math, Adagrad; BLAS threads)."""
    from threadpoolctl import threadpool_info
    from oracle.batch_oracle import ReaderOracle
    from oracle.model_oracle import AdagradOracle, OmniOracle
    tr = data.train
    t_asm = t_mod = 0.0
    nnz = 0
    ora = OmniOracle([N, H, N], activation="sigmoid", dtype=np.float32).set_params(w0[0::2], w0[1::2])
    opt = AdagradOracle(lr=lr)
    # the sampled rows in the reference's JSON-dict form (only these rows: the full dict of 20M
    # ratings would be minutes of host setup for a bounded sample)
    rows_all = np.unique(np.concatenate([np.asarray(r) for r in rows_batches[:n_steps]]))
    rdict = {str(r): [[str(int(c)), float(v)] for c, v in zip(tr.col[tr.row_ptr[r]:tr.row_ptr[r + 1]],
                                                               tr.val[tr.row_ptr[r]:tr.row_ptr[r + 1]])]
             for r in rows_all}
    ro = ReaderOracle([str(c) for c in range(N)], rdict)
    for rows in rows_batches[:n_steps]:
        keys = [str(r) for r in rows]
        t0 = time.perf_counter()
        m_in, m_out, x, t, m_miss = ro.train_batch(keys, len(keys), 0, (1.0, 1.0), -1.0, True)
        t1 = time.perf_counter()
        loss, _, gW, gb = ora.loss_and_grads(x, m_out, t)
        ora.set_flat(opt.step(ora.params(), [g for pair in zip(gW, gb) for g in pair]))
        t2 = time.perf_counter()
        t_asm += t1 - t0
        t_mod += t2 - t1
        nnz += int(tr.row_lengths()[rows].sum())
    threads = max([d.get("num_threads", 1) for d in threadpool_info()] + [1])
    B = len(rows_batches[0])
    out = {"value": nnz / (t_asm + t_mod), "unit": "ratings/s", "cores": int(threads), "kind": "port",
           "sample": "%d %s-shaped train steps (B=%d): the reference's dict-of-lists assembler restated, %.2fs/step "
                     "on 1 core + NumPy fp32 dense model step (Adagrad) %.2fs/step on %d BLAS threads"
                     % (n_steps, CONFIGS[config][1], B, t_asm / n_steps, t_mod / n_steps, threads),
           "assembler_ms_per_128_rows": round(t_asm / n_steps * 1e3 * 128 / B, 1)}
    if config in REF_ASM_MS_PER_128:
        out["assembler_cross_check"] = ("the reference's own assembler measured %.1f ms per 128-row batch in the "
                                        "survey container (BASELINE.md)" % REF_ASM_MS_PER_128[config])
    return out


def same_batch_one_gpu(args, data_full, n_rows, Bg, dev, steps=10, warmup=3):
    """The reference point for a weak-scaling feature-parallel line: the SAME global batch (B x G rows) on ONE
    GPU with the whole model -- measured in this run, on rank 0 before the timed region (the other ranks wait
    in their first collective)."""
    from omnidirectional_collaborative_filtering_amd.data_reader import data_reader
    from omnidirectional_collaborative_filtering_amd.model import omni_model
    st = np.random.get_state()
    np.random.seed(4321)
    rd = data_reader(data_full.num_cols, n_rows, dataset=data_full, eval_mode="fixed_split", rng="numpy", device=dev)
    om = omni_model(1, args.hidden, data_full.num_cols, Bg, dense_activation="sigmoid", use_causal_info=False,
                    dropout_probability=args.dropout or None, compute_dtype=args.dtype, seed=7, device=dev)
    m = om.model
    m.compile(optim(args.optimizer, 0.005 if args.optimizer == "adagrad" else 0.001), "mean_squared_error")
    gen = rd.data_gen(Bg, [1.0, 1.0], "train", True, None, -1, pass_through_input_training=True)
    gen._start()
    nb = gen.num_batches
    eng = om.engine
    gen.prepare_row_lists(eng.Np, [i % nb for i in range(warmup + steps)])

    def step(i):
        bi = i % nb
        if not eng.fast_train_step(gen, bi):
            m._load(None, gen, bi)
            eng.train_step()
        return int(gen.nnz1[bi])
    for i in range(warmup):
        step(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    nnz = sum(step(warmup + i) for i in range(steps))
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    eng.take_stats()
    np.random.set_state(st)
    out = {"global_batch": Bg, "ms_per_step": round(dt / steps * 1e3, 4), "ratings_per_s": round(nnz / dt, 1),
           "steps": steps, "source": "measured in this run: rank 0, one GPU, the whole model, before the timed region"}
    del om, m, eng, gen, rd
    torch.cuda.empty_cache()
    return out


PARITY_STEPS = 3


def _gloo():
    import torch.distributed as dist
    return dist.get_backend() == "gloo"


def _bcast(t):
    """broadcast from rank 0 (host-staged over gloo: rehearsals with every rank on one GPU)"""
    import torch.distributed as dist
    if _gloo():
        h = t.cpu()
        dist.broadcast(h, 0)
        t.copy_(h)
    else:
        dist.broadcast(t, 0)


def _all_gather(t, world):
    import torch.distributed as dist
    if _gloo():
        out = [torch.zeros_like(t, device="cpu") for _ in range(world)]
        dist.all_gather(out, t.cpu())
        return out
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return out


def _delta_stats(got, want, unit):
    """max-abs, 99th and 99.9th percentile of |got - want| (device tensors), in units of `unit`"""
    d = (got.float() - want.float()).abs().view(-1)
    n = d.numel()
    if n == 0:
        return [0.0, 0.0, 0.0, 0]
    top = torch.topk(d, min(n, n // 100 + 1)).values
    return [float(top[0]) / unit, float(top[min(len(top) - 1, n // 100)]) / unit,
            float(top[min(len(top) - 1, n // 1000)]) / unit, n]


def n_rank_parity(args, m, eng, step, data_full, n_rows, Bg, shard, dev, rank, world, batches, gen):
    """The N-rank run checks itself (feature layout): the first PARITY_STEPS steps of this job against the SAME
    steps of a one-GPU model of the whole network built on rank 0 (the same seed, hence the same initial weights,
    the same global batches of B x G rows, the same dropout stream).  Reported: the per-step loss difference and
    the max-abs / 99th / 99.9th percentile weight difference after those steps, in the units and against the bars
    of tests/parity.py -- fp32: 1e-5 absolute; f16 / bf16: loss 2e-3 / 1e-2 relative and weights within 2, 0.02,
    0.15 of lr x steps (max, p99, p99.9; the per-element Adagrad envelope).  Runs before the warm-up, outside the
    timed region (the steps it takes are steps of the job: the warm-up and timed steps continue from them)."""
    from omnidirectional_collaborative_filtering_amd.data_reader import data_reader
    from omnidirectional_collaborative_filtering_amd.model import omni_model
    k = PARITY_STEPS
    lr = 0.005 if args.optimizer == "adagrad" else 0.001
    N = data_full.num_cols
    H = args.hidden
    ref = None
    info = torch.zeros(2, dtype=torch.float64, device=dev)    # [batches match, reference ran]
    if rank == 0:
        st = np.random.get_state()
        np.random.seed(1234)                  # the job's generator seed: the same permutation, the same batches
        rd_r = data_reader(N, n_rows, dataset=data_full, eval_mode="fixed_split", rng="numpy", device=dev)
        om_r = omni_model(1, H, N, Bg, dense_activation="sigmoid", use_causal_info=False,
                          dropout_probability=args.dropout or None, compute_dtype=args.dtype, seed=7, device=dev)
        m_r = om_r.model
        m_r.compile(optim(args.optimizer, lr), "mean_squared_error")
        gen_r = rd_r.data_gen(Bg, [1.0, 1.0], "train", True, None, -1, pass_through_input_training=True)
        gen_r._start()
        np.random.set_state(st)
        same = all(np.array_equal(np.asarray(gen_r.rows_host[batches[i % len(batches)]]),
                                  np.asarray(gen.rows_host[batches[i % len(batches)]])) for i in range(k))
        e_r = om_r.engine
        for i in range(k):
            bi = batches[i % len(batches)]
            if not e_r.fast_train_step(gen_r, bi):
                m_r._load(None, gen_r, bi)
                e_r.train_step()
        sse_r = e_r.take_stats()[:, 0]
        torch.cuda.synchronize()
        ref = [e_r.W[0].clone(), e_r.W[1].clone(), e_r.b[0].clone(), e_r.b[1].clone()]
        del om_r, m_r, e_r, gen_r, rd_r
        torch.cuda.empty_cache()
        info[0], info[1] = float(same), 1.0
    for i in range(k):
        step(i)
    sse = eng.take_stats()[:, 0]              # (summed over the column shards)
    torch.cuda.synchronize()
    c0, c1, _ = shard
    Np_full = -(-N // 128) * 128
    Hp = eng.Hp[0]
    if rank != 0:
        ref = [torch.empty(Np_full, Hp, device=dev), torch.empty(Np_full, Hp, device=dev),
               torch.empty(Hp, device=dev), torch.empty(Np_full, device=dev)]
    for t in ref + [info]:
        _bcast(t)
    fp32 = args.dtype == "float32"
    unit = 1.0 if fp32 else lr * k
    n = c1 - c0
    rows = [_delta_stats(eng.W[0][:n, :H], ref[0][c0:c1, :H], unit),
            _delta_stats(eng.W[1][:n, :H], ref[1][c0:c1, :H], unit),
            _delta_stats(eng.b[0][:H], ref[2][:H], unit),
            _delta_stats(eng.b[1][:n], ref[3][c0:c1], unit)]
    mine = torch.tensor([x for r in rows for x in r[:3]], dtype=torch.float64, device=dev)
    allr = _all_gather(mine, world)
    del ref
    torch.cuda.empty_cache()
    if rank != 0:
        return None
    a = torch.stack([x.cpu() for x in allr]).numpy().reshape(world, 4, 3).max(0)     # worst rank per tensor and statistic
    rel = [abs(float(x) - float(y)) / max(abs(float(y)), 1e-30) for x, y in zip(sse, sse_r)]
    worst = a.max(0)
    bars = ([1e-5, 1e-5, 1e-5] if fp32 else [2.0, 0.02, 0.15])
    loss_bar = 1e-5 if fp32 else (2e-3 if args.dtype == "float16" else 1e-2)
    ok = bool(info[0].item() == 1.0 and max(rel) <= loss_bar and all(w <= b for w, b in zip(worst, bars)))
    return {"ok": ok, "steps": k, "batches_match": bool(info[0].item() == 1.0),
            "loss_rel_diff_per_step": [float("%.3g" % r) for r in rel], "loss_bar": loss_bar,
            "weights": {name: {"max": float("%.4g" % v[0]), "p99": float("%.4g" % v[1]), "p999": float("%.4g" % v[2])}
                        for name, v in zip(("W1", "W_out", "b1", "b_out"), a)},
            "weight_units": "absolute" if fp32 else "lr x steps (%g)" % unit,
            "weight_bars": {"max": bars[0], "p99": bars[1], "p999": bars[2]},
            "against": "one GPU, the whole model, the same seed and global batches (rank 0, before the warm-up)"}


def replica_consistency(eng, dev, world):
    """DP layout: after the warm-up every rank must hold the same weights (16-bit shadows, biases): per-tensor
    float64 sums and abs-sums, all-gathered, equal on every rank"""
    ts = [sh if sh is not None else w for w, sh in zip(eng.W, eng.Wsh)] + list(eng.b)
    v = torch.tensor([x for t in ts for x in (float(t.double().sum()), float(t.double().abs().sum()))],
                     dtype=torch.float64, device=dev)
    allv = [x.cpu() for x in _all_gather(v, world)]
    same = all(torch.equal(allv[0], x) for x in allv[1:])
    return {"replicas_identical": bool(same), "tensors": len(ts),
            "note": "data-parallel replicas after the warm-up (sums and abs-sums of every shadow and bias)"}


def fp32_mode(args, data, rd, n_rows, dev, steps):
    """ms/step of the exact-fp32 parity mode (compute_dtype float32, v_mfma_f32_32x32x2_f32; the mode the
    1e-5 parity bar is tested in) on the same workload, N=1"""
    from omnidirectional_collaborative_filtering_amd.model import omni_model
    om = omni_model(1, args.hidden, data.num_cols, args.batch, dense_activation="sigmoid", use_causal_info=False,
                    dropout_probability=args.dropout or None, compute_dtype="float32", seed=7, device=dev)
    m = om.model
    m.compile(optim(args.optimizer, 0.005 if args.optimizer == "adagrad" else 0.001), "mean_squared_error")
    gen = rd.data_gen(args.batch, [1.0, 1.0], "train", True, None, -1, pass_through_input_training=True)
    gen._start()
    nb = gen.num_batches
    for i in range(3):
        m._load(None, gen, i % nb)
        om.engine.train_step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        m._load(None, gen, (3 + i) % nb)
        om.engine.train_step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    om.engine.take_stats()
    return {"ms_per_step": round(ms, 4), "steps": steps, "compute": "float32 throughout (fp32 weight rows in the gathers, fp32 row-stream dW)"}


def full_epoch(args, m, rd, B):
    """one train.py epoch, wall clock: fresh generator (permutation, batch tables, the NumPy-stream draws
    of data_reader.py:120,130 on the device, row lists, scatter outputs) + fit_generator over
    floor(n/B) - 1 steps (train.py:157) + the epoch-end stats read-back.  Also the epoch plan alone with
    a reciprocal split (data_sparsity [0.3, 0.7]: the keep flags of every rating drawn)."""
    out = {}
    for name, sp in (("train_py", [1.0, 1.0]), ("recip_0.3_0.7", [0.3, 0.7])):
        np.random.seed(4321)
        gen = rd.data_gen(B, sp, "train", True, None, -1, pass_through_input_training=sp[0] >= 1.0)
        steps = gen.num_batches - 1
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if name == "train_py":
            m.fit_generator(gen, steps, epochs=1, verbose=0)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            nnz = int(gen.nnz1[:steps].sum())
            out[name] = {"batches": steps, "ms_per_batch": round(dt / steps * 1e3, 4),
                         "ratings_per_s": round(nnz / dt, 1), "wall_s": round(dt, 4)}
        else:
            gen._start()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            gen.prepare_row_lists(m.engine.Np)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            out[name] = {"plan_ms": round((t1 - t0) * 1e3, 3), "row_lists_and_scatter_ms": round((t2 - t1) * 1e3, 3),
                         "batches": gen.num_batches, "entries": int(gen.nnz_full.sum())}
    out["rng"] = "numpy (NumPy's global MT19937 stream; the epoch's draws by ocf_recip_keep on the device)"
    return out


def jester_arrays(n=73_421, N=100, seed=1):
    """train_jester.py:34-75 on synthetic data of the Jester shape (the CSV is not in the image): ratings
    uniform in [-10, 10] (2 decimals) with 99 = missing at Jester's ~56 % density, the observed mask, and
    the reciprocal 0.5 input / output split drawn once with np.random.choice (:69-74)"""
    rng = np.random.RandomState(seed)
    data = np.where(rng.rand(n, N) < 0.56, np.round(rng.uniform(-10, 10, (n, N)), 2), 99.0)
    observed = (data != 99).astype(np.float64)
    np.random.seed(seed)
    drop = np.random.choice([0, 1], size=data.shape, p=[0.5, 0.5])
    in_m, out_m = drop * observed, (1 - drop) * observed
    return (data * in_m).astype(np.float32), observed.astype(np.float32), out_m.astype(np.float32), \
        (data * out_m).astype(np.float32)


def jester_main(args):
    """BASELINE configs[4]: the Jester omnidirectional denoising AE with train_jester.py's parameters --
    100 jokes, causal concat of the observed mask (input 200), 2 x 256 tanh hidden layers, linear output,
    RMSprop (Keras defaults), batch 128, Model.fit on dense arrays with validation_split 0.1 (:44-79).  A step
    is one Model.fit batch (the dense MFMA path: split-K encoder, hidden-layer GEMM, masked-MSE decoder,
    backward GEMMs with fused RMSprop); ratings/s counts the observed ratings of the batches."""
    from omnidirectional_collaborative_filtering_amd.model import omni_model
    rank, world, local = 0, 1, 0
    if args.gpus != 1:
        raise SystemExit("--config jester: one GPU per process (replicas only; see DESIGN.md)")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    t0 = time.time()
    inputs, observed, out_m, targets = jester_arrays()
    n, N = inputs.shape
    B, H = 128, 256
    om = omni_model(2, H, N, B, dense_activation="tanh", use_causal_info=True, compute_dtype=args.dtype, seed=3,
                    rating_range=20, device=dev)
    m = om.model
    m.compile("rmsprop", "mean_squared_error", metrics=["mae", "accurate_MAE", "nMAE"])
    w0 = m.get_weights()
    e = om.engine
    split_at = int(n * 0.9)
    np.random.seed(42)
    idx = np.arange(split_at)
    np.random.shuffle(idx)                     # Model.fit's shuffle of the training part
    x = [inputs, observed, out_m]
    n_batches = split_at // B
    obs_per = [int(observed[idx[s * B:(s + 1) * B]].sum()) for s in range(n_batches)]
    setup_s = time.time() - t0

    # Model.fit's data path: the arrays resident on the device, each batch gathered by row index
    xd = [torch.as_tensor(a).to(dev) for a in x]
    yd = torch.as_tensor(targets).to(dev)
    idx_d = torch.as_tensor(idx, dtype=torch.int64).to(dev)

    def step(i):
        s = i % n_batches
        m._load_rows(xd, yd, idx_d[s * B:(s + 1) * B])
        e.train_step()
        return obs_per[s]

    e.enable_timers(bool(args.phase_timers))
    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    phases = e.phase_times_ms(skip=1 if args.warmup > 1 else 0)
    cand = {k: v for k, v in phases.items()
            if k in ("dW_in", "dW_out", "dW_pair", "enc_gemm", "dec_gemm_mse", "dec_bwd_gemm", "mlp_step")}
    dom = max(cand, key=lambda k: cand[k]["mean_ms"]) if cand else None
    # the dominant kernel's duration inside the timed region.  The one-launch step (ocf_mlp_step): workgroup 0's
    # constant-rate clock at the kernel's start and end, written by the kernel itself into one row per step (no
    # event records on the stream: at ~45 us per launch an event pair's own ~5-10 us would make the sampled
    # kernel look longer than the step); other kernels: HIP events every TIMER_EVERY_SHORT-th step
    trace = dom == "mlp_step"
    tr_rows = torch.zeros(args.steps, 24, dtype=torch.int64, device=dev) if trace else None
    e.enable_timers(dom is not None and not trace, only=[dom] if dom else None)
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    nnz = 0
    for i in range(args.steps):
        if trace:
            e.mlp_trace = tr_rows[i]
        elif dom:
            e.timer_only = {dom} if i % TIMER_EVERY_SHORT == 0 else {"-"}
        nnz += step(args.warmup + i)
    t_issued = time.perf_counter()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    if trace:
        e.mlp_trace = None
        t = tr_rows.cpu().numpy().astype(np.float64)
        dur = [(r[r > 0].max() - r[0]) / 100.0 for r in t if (r > 0).sum() >= 2]      # 100 MHz clock -> us
        dom_timed = {"mean_ms": float(np.mean(dur)) * 1e-3, "n": len(dur),
                     "source": "the kernel's own clock (workgroup 0, start to end), every timed step"} if dur else None
    else:
        dom_timed = e.phase_times_ms().get(dom) if dom else None
    e.enable_timers(False)
    e.take_stats()
    ms = elapsed / args.steps * 1e3
    # algorithmic work per step: dims 200 -> 256 -> 256 -> 100, no input gradient
    dims = [2 * N, H, H, N]
    P = sum(a * b + b for a, b in zip(dims[:-1], dims[1:]))
    flops = sum(6.0 * B * a * b for a, b in zip(dims[:-1], dims[1:])) - 2.0 * B * dims[0] * dims[1]
    w_b = 4 if args.dtype == "float32" else 2
    step_bytes = P * (16 + 4) + w_b * (sum(a * b for a, b in zip(dims[:-1], dims[1:])) * 2) + 5 * B * N * 4
    if dom is not None and not dom_timed:
        dom = None
    line = {
        "metric": METRIC, "value": round(nnz / elapsed, 1), "unit": "ratings/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": {"float16": "f16", "bfloat16": "bf16", "float32": "f32"}[args.dtype],
        "data": "synthetic Jester-shaped dense matrix (73,421 users x 100 jokes, ~56 % observed, ratings in "
                "[-10, 10], 99 = missing, reciprocal 0.5 split drawn once); random-init weights",
        "config": {"workload": "Jester omnidirectional denoising AE train step, Model.fit (BASELINE configs[4], "
                               "train_jester.py:44-79)", "rows": n, "N": N, "hidden": [H, H], "input": 2 * N,
                   "batch_per_gpu": B, "global_batch": B, "optimizer": "rmsprop", "activation": "tanh",
                   "compute": compute_label(e, args.dtype, "mlp_step" if e.fused_mlp else None),
                   "parallelism": "dp1"},
        "roofline": None,
        "step_roofline": {"alg_bytes": int(step_bytes), "alg_flops": int(flops),
                          "hbm_bound_ms": round(step_bytes / (HBM_PEAK_GBS * 1e9) * 1e3, 5),
                          "mfma_bound_ms": round(flops / (MFMA_F16_PEAK_TFS * 1e12) * 1e3, 5),
                          "frac_of_binding_roof": round(max(step_bytes / (HBM_PEAK_GBS * 1e9),
                                                            flops / (MFMA_F16_PEAK_TFS * 1e12)) / (ms * 1e-3), 4)},
        "phases_ms": {k: round(v["mean_ms"], 4) for k, v in phases.items()},
        "phases_from": "warm-up steps 2..%d, every phase bracketed by HIP events" % args.warmup,
        "host_issue_ms_per_step": round((t_issued - t_start) / args.steps * 1e3, 4),
        "setup_s": round(setup_s, 1),
    }
    if dom == "mlp_step":
        # the whole step in one launch (ocf_mlp_step): against the step's own bytes and flops (the binding one)
        kms = dom_timed["mean_ms"]
        hb, mf = step_bytes / (kms * 1e-3) / 1e9, flops / (kms * 1e-3) / 1e12
        by_bytes = hb / HBM_PEAK_GBS >= mf / MFMA_F16_PEAK_TFS
        line["roofline"] = {"bound": "hbm" if by_bytes else "mfma", "achieved": round(hb if by_bytes else mf, 2),
                            "peak": HBM_PEAK_GBS if by_bytes else MFMA_F16_PEAK_TFS,
                            "unit": "GB/s" if by_bytes else "TFLOP/s",
                            "frac": round(hb / HBM_PEAK_GBS if by_bytes else mf / MFMA_F16_PEAK_TFS, 5), "traffic": None,
                            "kernel": dom, "kernel_mean_us": round(kms * 1e3, 2), "kernel_samples": dom_timed["n"],
                            "kernel_time_source": dom_timed.get("source", "HIP events"),
                            "alg_bytes_per_launch": int(step_bytes),
                            "alg_flops_per_launch": int(flops),
                            "note": "the whole step of a 0.14 M-parameter model in one persistent launch (ocf_mlp_step): "
                                    "latency-bound (phases separated by grid barriers); reported, not a target"}
    elif dom is not None:
        # the dominant launch against its own algorithmic bytes (tiny model: latency-bound, reported as is)
        Pd = {"dW_in": dims[0] * dims[1], "dW_out": dims[2] * dims[3], "enc_gemm": dims[0] * dims[1],
              "dec_gemm_mse": dims[2] * dims[3], "dec_bwd_gemm": dims[2] * dims[3]}[dom]
        alg = Pd * (16 if dom.startswith("dW") else w_b) + 2 * B * max(dims) * w_b
        kms = dom_timed["mean_ms"]
        line["roofline"] = {"bound": "hbm", "achieved": round(alg / (kms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                            "unit": "GB/s", "frac": round(alg / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5), "traffic": None,
                            "kernel": dom, "kernel_mean_us": round(kms * 1e3, 2), "alg_bytes_per_launch": int(alg),
                            "note": "a 0.14 M-parameter model: every launch is latency-bound; the fraction is "
                                    "reported, not a target"}
    if args.cpu_baseline:
        from threadpoolctl import threadpool_info
        from oracle.model_oracle import OmniOracle, RMSpropOracle
        ora = OmniOracle(dims, activation="tanh", dtype=np.float32).set_params(w0[0::2], w0[1::2])
        opt = RMSpropOracle(lr=0.001)
        ks = max(args.cpu_steps, 20)
        t1 = time.perf_counter()
        nn = 0
        for s in range(ks):
            sel = idx[s * B:(s + 1) * B]
            xin = np.concatenate([inputs[sel], observed[sel]], 1)
            _, _, gW, gb = ora.loss_and_grads(xin, out_m[sel], targets[sel])
            ora.set_flat(opt.step(ora.params(), [g for pair in zip(gW, gb) for g in pair]))
            nn += obs_per[s]
        dt = time.perf_counter() - t1
        threads = max([d.get("num_threads", 1) for d in threadpool_info()] + [1])
        line["cpu_baseline"] = {"value": round(nn / dt, 1), "unit": "ratings/s", "cores": int(threads), "kind": "port",
                                "sample": "%d Model.fit steps of the same workload: NumPy fp32 dense model step "
                                          "(RMSprop) on %d BLAS threads, %.2f ms/step" % (ks, threads, dt / ks * 1e3)}
    print(json.dumps(line), flush=True)


# the other BASELINE configs, run as child processes after the headline (bench args, timeout s)
SIDE_CONFIGS = [
    ("ml100k", ["--config", "ml100k", "--dtype", "float32"], 240),
    ("ml1m", ["--config", "ml1m", "--dtype", "bfloat16"], 240),
    ("ml1m_u", ["--config", "ml1m_u", "--dtype", "bfloat16"], 240),
    ("jester", ["--config", "jester", "--dtype", "bfloat16"], 240),
    ("train_py_ml1m_h512_b128", ["--config", "ml1m", "--dtype", "float32", "--hidden", "512", "--batch", "128"], 240),
    ("netflix", ["--config", "netflix"], 420),
]


def side_configs():
    """short in-run lines of the other BASELINE configs (each a child bench.py: own process, own GPU memory;
    CPU baseline, test RMSE, fp32 mode and full epoch off), reduced to ms/step, ratings/s and the roofline
    fractions.  A config that fails is reported with its error, never retried."""
    import subprocess
    out = {}
    for name, extra, tmo in SIDE_CONFIGS:
        cmd = [sys.executable, os.path.abspath(__file__), "--cpu-baseline", "0", "--rmse", "0", "--fp32-steps", "0",
               "--epoch", "0", "--configs", "0", "--warmup", "5"] + (["--steps", "20"] if "--steps" not in extra else []) \
            + extra
        t0 = time.time()
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=tmo)
            lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
            if r.returncode != 0 or not lines:
                out[name] = {"error": "rc %d: %s" % (r.returncode, (r.stderr or r.stdout)[-300:])}
                continue
            d = json.loads(lines[-1])
        except subprocess.TimeoutExpired:
            out[name] = {"error": "timeout after %d s" % tmo}
            continue
        roof, sr = d.get("roofline") or {}, d.get("step_roofline") or {}
        out[name] = {"workload": d["config"]["workload"], "dtype": d["dtype"], "hidden": d["config"].get("hidden"),
                     "batch": d["config"].get("batch_per_gpu"), "ms_per_step": d["ms_per_step"],
                     "ratings_per_s": d["value"], "steps": d["steps"], "kernel": roof.get("kernel"),
                     "kernel_mean_us": roof.get("kernel_mean_us"), "frac": roof.get("frac"),
                     "step_roofline_frac": sr.get("frac_of_binding_roof"), "wall_s": round(time.time() - t0, 1)}
    return out


def main():
    args = parse()
    if os.environ.get("OCF_TUNING"):
        # experiment hook for tools/ab.py: "key=value,key=value" passed to ocf_set_tuning before any launch
        from omnidirectional_collaborative_filtering_amd import _lib
        for kv in os.environ["OCF_TUNING"].split(","):
            k, _, v = kv.partition("=")
            _lib.call("ocf_set_tuning", k.strip().encode(), int(v), None)
    if args.config == "jester":
        return jester_main(args)
    from omnidirectional_collaborative_filtering_amd.parallel import (DataParallel, feature_shard_range,
                                                                      init_from_env, make_comm, shard_batches)
    rank, world, local = init_from_env()
    if world != args.gpus:
        raise SystemExit("--gpus %d but WORLD_SIZE %d" % (args.gpus, world))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    from omnidirectional_collaborative_filtering_amd.data_reader import data_reader
    from omnidirectional_collaborative_filtering_amd.dataset import synthetic_fixed_split
    from omnidirectional_collaborative_filtering_amd.model import omni_model

    t0 = time.time()
    data_full = synthetic_fixed_split(args.config, seed=0, skew=args.skew)
    N = data_full.num_cols
    n_rows = data_full.train.n_rows
    fp = world > 1 and args.parallel == "feature"
    B, H = args.batch, args.hidden
    if args.emulate_shards > 1:
        G = args.emulate_shards
        c0, c1 = feature_shard_range(N, 0, G)
        data = data_full.column_shard(c0, c1)
        Bg, shard, comm = B * G, (c0, c1, N), _NoComm() if args.emulate_comm else None
        fp = True
    elif fp:
        # weak scaling: 256 rows per GPU -> global batch 256*G, each rank owns N/G users
        c0, c1 = feature_shard_range(N, rank, world)
        data = data_full.column_shard(c0, c1)
        Bg, shard, comm = B * world, (c0, c1, N), make_comm(world)
    else:
        data, Bg, shard, comm = data_full, B, None, None
    np.random.seed(1234)
    # rng="numpy": the reference's own RNG stream (NumPy's MT19937 state, epoch draws on the device)
    rd = data_reader(data.num_cols, n_rows, dataset=data, eval_mode="fixed_split", rng="numpy", device=dev)
    om = omni_model(1, H, data.num_cols, Bg, dense_activation="sigmoid", use_causal_info=False,
                    dropout_probability=args.dropout or None, compute_dtype=args.dtype, seed=7, device=dev,
                    shard=shard, comm=comm)
    m = om.model
    lr = 0.005 if args.optimizer == "adagrad" else 0.001
    m.compile(optim(args.optimizer, lr), "mean_squared_error", metrics=["mae", "accurate_MSE", "accurate_RMSE"])
    w0 = m.get_weights() if (rank == 0 and world == 1 and args.cpu_baseline) else None
    eng = om.engine
    if args.enc_tiles >= 0:
        eng.enc_tiles = bool(args.enc_tiles)
    gen = rd.data_gen(Bg, [1.0, 1.0], "train", True, None, -1, pass_through_input_training=True)
    gen._start()
    batches = list(range(gen.num_batches)) if (fp or world == 1) else shard_batches(gen.num_batches, rank, world)
    dpo = DataParallel(eng, rank, world, mode=args.dp_mode, grad_dtype=args.dp_grad_dtype) \
        if (world > 1 and not fp) else None
    nnz_of = gen.nnz1
    same_batch = None
    if fp and world > 1 and rank == 0 and not args.emulate_shards:
        same_batch = same_batch_one_gpu(args, data_full, n_rows, B * world, dev)
    setup_s = time.time() - t0

    def step(i):
        bi = batches[i % len(batches)]
        if dpo is None and eng.fast_train_step(gen, bi):    # Model._train_one's one-call step
            return int(nnz_of[bi])
        m._load(None, gen, bi)
        if dpo is not None:
            dpo.step()
        else:
            eng.train_step()
        return int(nnz_of[bi])

    # N > 1: this run's first steps against one GPU (feature layout), before the warm-up
    parity = None
    if fp and world > 1 and not args.emulate_shards:
        parity = n_rank_parity(args, m, eng, step, data_full, n_rows, Bg, shard, dev, rank, world, batches, gen)

    # warm-up (untimed): every phase bracketed by HIP events -> per-phase breakdown and the dominant
    # kernel.  The timed region then brackets only that kernel, so the timers cost ~2 events/step.
    # the first W - 2 warm-up steps with every phase timed (the general path), the last two with only the dominant
    # kernel's timers: the one-call step records and verifies its template there, not in the timed region
    w_all = max(1, args.warmup - 2) if args.warmup >= 3 else args.warmup
    eng.enable_timers(bool(args.phase_timers))
    for i in range(w_all):
        step(i)
    torch.cuda.synchronize()
    phases = eng.phase_times_ms(skip=1 if w_all > 1 else 0)
    cand = {k: v for k, v in phases.items()
            if k in ("dW_in", "dW_out", "dW_pair", "enc_gemm", "dec_gemm_mse", "dec_bwd_gemm", "mlp_step")}
    dom = max(cand, key=lambda k: cand[k]["total_ms"]) if cand else None
    eng.enable_timers(dom is not None, only=[dom] if dom else None)
    for i in range(w_all, args.warmup):
        eng.timer_only = {"-"}
        step(i)
    if world > 1:
        torch.distributed.barrier()
    eng.enable_timers(dom is not None, only=[dom] if dom else None)
    fused_step = dom == "mlp_step"          # a small model: dense arrays + ocf_mlp_step, no row lists
    epoch_lists = eng.epoch_row_lists and eng.sparse_dw and eng.use_sparse and not fused_step
    torch.cuda.synchronize()
    paths0 = dict(eng.step_paths)
    t_start = time.perf_counter()
    nnz = 0
    if epoch_lists:
        # the timed batches' row lists, built inside the timed region (one launch sequence, as at the
        # start of every training epoch)
        gen.prepare_row_lists(eng.Np, [batches[(args.warmup + i) % len(batches)] for i in range(args.steps)])
    t_lists = time.perf_counter()
    # the dominant kernel's HIP events on every TIMER_EVERY-th timed step (TIMER_EVERY_SHORT-th for a kernel under
    # 0.1 ms): each event record idles the stream ~4.7 us even without its system-scope fence (rocprof trace,
    # profiles/r06_events/), so sampling keeps the timing overhead small while still averaging over the whole timed
    # region (every 4th vs every 10th step at ML-20M: 0.3821 vs 0.3820 ms, same box)
    sampled = {dom} if dom else None
    every = TIMER_EVERY if (not dom or phases[dom]["mean_ms"] >= 0.1) else TIMER_EVERY_SHORT
    t_first = None
    # (the samples end each group of `every` steps: the first step of the window, issued while the GPU waits on
    # the host, takes no timer bookkeeping)
    first_sample = min(every, args.steps) - 1
    for i in range(args.steps):
        if dom:
            eng.timer_only = sampled if i % every == first_sample else {"-"}
        nnz += step(args.warmup + i)
        if t_first is None:
            t_first = time.perf_counter()
    t_issued = time.perf_counter()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t_start
    host_ms = (t_issued - t_start) / args.steps * 1e3    # host time to issue one step (diagnostic)
    step_paths = {k: (v - paths0.get(k, 0) if isinstance(v, int) else v)          # one-call vs recorded general
                  for k, v in eng.step_paths.items()}                            # steps (and why)
    dom_timed = eng.phase_times_ms().get(dom) if dom else None
    eng.timers = None
    if dpo is not None:
        parity = replica_consistency(eng, dev, world)
    row_skip_used = eng._rtag_live          # (the eval batches below reset it)
    tot = torch.tensor([elapsed, float(nnz)], device=dev, dtype=torch.float64)
    if world > 1:
        tmax = tot[:1].clone()
        torch.distributed.all_reduce(tmax, op=torch.distributed.ReduceOp.MAX)
        nsum = tot[1:].clone()
        torch.distributed.all_reduce(nsum, op=torch.distributed.ReduceOp.SUM)
        elapsed, nnz = float(tmax.item()), float(nsum.item())
    eng.take_stats()

    # masked RMSE on the test split (train.py:225-255, fused form)
    rmse = None
    if args.rmse:
        tgen = rd.data_gen(Bg, None, "test", True, None, -1, return_target_count=True)
        sse, cnt = m.evaluate_sse(tgen, rd.test_set_size // Bg)
        rmse = float(np.sqrt(sse / cnt)) if cnt else None

    if rank != 0:
        if world > 1:
            torch.distributed.destroy_process_group()
        return

    # roofline of the dominant kernel: fused weight-gradient GEMM + optimizer update (per rank)
    Nl = data.num_cols
    P = Nl * H
    # row skipping: only the weight rows of columns holding a batch entry carry optimizer traffic
    # (pass-through training with data_sparsity [1,1]: every entry is a live input and a live target,
    # so both weight matrices have the batch's distinct columns as live rows)
    live = 1.0
    if row_skip_used and args.optimizer == "adagrad":
        tr = data.train
        fr = []
        for i in range(args.steps):
            rows = np.asarray(gen.rows_host[batches[(args.warmup + i) % len(batches)]])
            rows = rows[rows >= 0]
            cols = np.concatenate([tr.col[tr.row_ptr[r]:tr.row_ptr[r + 1]] for r in rows])
            fr.append(len(np.unique(cols)) / Nl)
        live = float(np.mean(fr))
    opt_b = OPT_STATE_BYTES[args.optimizer]
    # weight operands: the compute-dtype shadow (2 B) written by the optimizer epilogue, fp32 in fp32 mode
    w_b = 4 if args.dtype == "float32" else 2
    sh_b = 0 if args.dtype == "float32" else 2
    # batch operand of the weight-gradient GEMMs: dense [B][N] (2 B per element) or, on the sparse
    # path, the batch's entries (4-B value + 4-B packed index each)
    sparse_a = bool(eng.use_sparse and eng.sparse_ok and eng.sparse_dw)
    a_bytes = (8.0 * nnz / args.steps / max(world, 1)) if sparse_a else Bg * Nl * 2
    alg = {
        # bytes per launch, algorithmic (real, unpadded sizes of this rank): optimizer state r/w (+ shadow
        # write) + streamed operands
        "dW_in": P * live * (opt_b + sh_b) + a_bytes + Bg * H * 2,
        "dW_out": P * live * (opt_b + sh_b) + a_bytes + Bg * H * 2,
        # both updates in one launch (ocf_gemm_pair)
        "dW_pair": 2 * (P * live * (opt_b + sh_b) + a_bytes + Bg * H * 2),
        "enc_gemm": P * w_b + Bg * Nl * 2,
        "dec_gemm_mse": P * w_b + Bg * H * 2 + Bg * Nl * 2,
        "dec_bwd_gemm": P * w_b + Bg * Nl * 2,
    }
    if sparse_a and eng.use_sparse:
        # the row gathers (encoder / decoder / both in one launch, ocf_gather_encdec): a weight row per entry
        # (H real elements in the compute dtype) + the entry's index / value / flag / delta bytes; the decoder also
        # writes the batch's a / mask / h / hidden-delta rows.  The one launch is timed as dec_gemm_mse (no
        # enc_gemm phase then)
        ent = nnz / args.steps / max(world, 1)
        g_enc = ent * (H * w_b + 8)
        g_dec = ent * (H * w_b + 13) + Bg * H * (4 + 1 + 2 * w_b)
        alg["enc_gemm"] = g_enc
        alg["dec_gemm_mse"] = g_dec + (g_enc if "enc_gemm" not in phases else 0)
    # the fused small-model step: the whole step in one launch, against its dense-update bytes and its flops
    # (forward, output layer, input-delta-free backward: 3 GEMMs of 2 B N H each way + the hidden delta)
    alg["mlp_step"] = P * 2 * (opt_b + 4 + sh_b) + Bg * Nl * 4 * 3
    roof = None
    if dom is not None and dom_timed:
        if world > 1 and not fp and dom in ("dW_in", "dW_out"):
            # gradient store instead of the fused update
            alg[dom] = P * (2 if args.dp_grad_dtype == "bfloat16" else 4) + a_bytes + B * H * 2
        ms = dom_timed["mean_ms"]
        ach = alg[dom] / (ms * 1e-3) / 1e9
        roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None, "kernel": dom,
                "kernel_mean_us": round(ms * 1e3, 1), "kernel_samples": dom_timed["n"],
                "alg_bytes_per_launch": int(alg[dom]), "live_row_frac": round(live, 4)}
        if dom == "mlp_step":
            fl = 10.0 * Bg * Nl * H
            tf = fl / (ms * 1e-3) / 1e12
            if tf / MFMA_F16_PEAK_TFS > ach / HBM_PEAK_GBS:
                roof.update(bound="mfma", achieved=round(tf, 2), peak=MFMA_F16_PEAK_TFS, unit="TFLOP/s",
                            frac=round(tf / MFMA_F16_PEAK_TFS, 4))
            roof["alg_flops_per_launch"] = int(fl)
            roof["note"] = ("the whole step in one persistent launch (ocf_mlp_step): dense GEMMs on the batch's "
                            "data_gen arrays, fused masked MSE, optimizer updates")
        # HBM bytes per launch from the latest round's PMC passes (tools/pmc_traffic.py output)
        # the latest round's PMC summary that measured this kernel (r03_, r03b_, r03c_ ... sort in round order)
        # (measured on the default workloads: ML-20M -> r*_pmc_traffic.json, Netflix -> r*_netflix_pmc_traffic.json;
        # B = 256, f16, one GPU)
        others = [c for c in CONFIGS if c != args.config]
        pmcs = [f for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]*_pmc_traffic.json")))
                if not any("_%s_" % c in os.path.basename(f) for c in others)
                and (args.config == "ml20m" or "_%s_" % args.config in os.path.basename(f))
                and dom in json.load(open(f))]
        if pmcs and world == 1 and args.config in ("ml20m", "netflix") and args.batch == 256 and \
                args.dtype == "float16" and args.hidden == 500 and not args.emulate_shards:
            with open(pmcs[-1]) as f:
                tr = json.load(f).get(dom)
            if tr:
                roof["traffic"] = tr["hbm_bytes"]
                roof["traffic_source"] = os.path.relpath(pmcs[-1], ROOT)
    ms_step = elapsed / args.steps * 1e3
    step_flops = 10.0 * Bg * Nl * H
    # SURVEY §8(d) step bytes; with row skipping the optimizer term covers the live rows only
    step_bytes_dense = P * 2 * (opt_b + 4) + 2 * (3 * Nl * H) + 8 * (nnz / args.steps / max(world, 1))
    step_bytes = step_bytes_dense - P * 2 * (opt_b + 4) * (1.0 - live)
    line = {
        "metric": METRIC, "value": round(nnz / elapsed, 1), "unit": "ratings/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": {"float16": "f16", "bfloat16": "bf16",
                                                          "float32": "f32"}[args.dtype],
        "data": "synthetic %s-shaped fixed split (%s, %.1fM ratings, seed 0, %s); random-init weights"
                % (CONFIGS[args.config][1], CONFIGS[args.config][2],
                   (data_full.train.nnz + data_full.valid_tgt.nnz + data_full.test_tgt.nnz) / 1e6,
                   "popularity ~ rank^-%g" % args.skew if args.skew > 0 else "uniform popularity"),
        "config": {"workload": "%s %s train step (BASELINE configs[%d])" % (args.config, "U-AutoRec" if args.config.endswith("_u")
                                                                            else "I-AutoRec", CONFIGS[args.config][0]),
                   "rows": n_rows, "N": N,
                   "hidden": H, "batch_per_gpu": B, "global_batch": Bg if fp else B * world,
                   "optimizer": args.optimizer, "activation": "sigmoid", "dropout": args.dropout,
                   "compute": compute_label(eng, args.dtype, dom),
                   "parallelism": ("feature%d" % world) if fp else ("dp%d" % world)},
        "masked_rmse": rmse,
        "roofline": roof,
        "step_roofline": {"alg_bytes": int(step_bytes), "alg_bytes_dense_update": int(step_bytes_dense),
                          "live_row_frac": round(live, 4), "alg_flops": int(step_flops),
                          "hbm_bound_ms": round(step_bytes / (HBM_PEAK_GBS * 1e9) * 1e3, 4),
                          "mfma_bound_ms": round(step_flops / (MFMA_F16_PEAK_TFS * 1e12) * 1e3, 4),
                          "frac_of_binding_roof": round(max(step_bytes / (HBM_PEAK_GBS * 1e9),
                                                            step_flops / (MFMA_F16_PEAK_TFS * 1e12))
                                                        / (ms_step * 1e-3), 4)},
        "phases_ms": {k: round(v["mean_ms"], 4) for k, v in phases.items()},
        "phases_from": "warm-up steps 2..%d, every phase bracketed by HIP events (timed region: only %s, "
                       "every %d-th step)" % (w_all, dom, every),
        "setup_s": round(setup_s, 1),
        "host_issue_ms_per_step": round(host_ms, 4),
        # host time inside the timed region before the GPU has work: the row-list build's prelude (staging,
        # launches) and the first step's issue (the window's step table); later steps are issued behind the GPU
        "window_host_us": {"row_lists": round((t_lists - t_start) * 1e6, 1),
                           "first_step": round(((t_first or t_lists) - t_lists) * 1e6, 1),
                           "row_list_parts": {k: round(v, 1) for k, v in getattr(gen, "rl_host_us", {}).items()}
                           if epoch_lists else None},
        "timed_step_paths": step_paths,
        "row_lists": ("per epoch: ocf_epoch_row_lists for the %d timed batches inside the timed region"
                      % len(set(batches[(args.warmup + i) % len(batches)] for i in range(args.steps))))
                     if epoch_lists else "per step (ocf_row_lists)" if eng.sparse_dw else "n/a",
    }
    # this rank's device memory (weights, slots, shadows, epoch tables, scratch): the per-rank footprint of a layout
    line["rank_memory"] = {"peak_allocated_gb": round(torch.cuda.max_memory_allocated(dev) / 1e9, 3),
                           "reserved_gb": round(torch.cuda.memory_reserved(dev) / 1e9, 3)}
    if dpo is not None:
        sync = getattr(dpo, "sync", None)
        line["dp_layout"] = {"mode": args.dp_mode, "grad_dtype": args.dp_grad_dtype,
                             "zero1_shards": [[int(p.numel()), int(p.numel()) // world] for p in sync.params]
                             if sync is not None else None,
                             "grad_bytes_per_step": int(sum(g.numel() * g.element_size() for g in dpo.views))}
    if parity is not None:
        line["n_rank_parity"] = parity
    if same_batch is not None:
        # weak scaling grows the global batch with the ranks; the same global batch on ONE GPU is the reference
        # point for the speed-up, not the B = 256 line
        line["same_global_batch_1gpu"] = same_batch
    if world == 1 and args.fp32_steps > 0 and args.dtype != "float32" and not args.emulate_shards:
        line["fp32_parity_mode"] = fp32_mode(args, data, rd, n_rows, dev, args.fp32_steps)
    if world == 1 and args.epoch and not args.emulate_shards:
        line["full_epoch"] = full_epoch(args, m, rd, Bg)
    if world == 1 and args.cpu_baseline:
        rows_b = [gen.rows_host[bi] for bi in batches[: args.cpu_steps]]
        try:
            line["cpu_baseline"] = cpu_baseline(data, rows_b, N, H, w0, lr, args.cpu_steps, args.config)
        except Exception as e:  # the baseline is reported, never the measured value
            line["cpu_baseline"] = {"error": repr(e)}
    if world == 1 and args.configs and args.config == "ml20m" and not args.emulate_shards:
        del om, m, eng, gen, rd
        torch.cuda.empty_cache()
        line["configs"] = side_configs()
    print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
