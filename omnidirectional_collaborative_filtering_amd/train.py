"""Training driver with the reference train.py parameter surface (train.py:19-59).

    python -m omnidirectional_collaborative_filtering_amd.train --dataset ml1m --metadata datasets_metadata.json
    python -m omnidirectional_collaborative_filtering_amd.train --synthetic ml1m --max_epochs 5
    torchrun --nproc-per-node 8 -m omnidirectional_collaborative_filtering_amd.train --synthetic ml20m \
        [--parallel feature|dp] [--dp_mode sharded|allreduce] [--dp_grad_dtype float32|bfloat16]

Multi-GPU (no counterpart in the reference, which runs on one CPU; train.py:125-129):
  --parallel feature (default): every rank holds a column shard of the first and last layers and
      processes every batch; the collectives are two [B, H] all-reduces per step, so training is the
      single-GPU computation (batch_size = the global batch).  Checkpoints are per-rank shard files.
  --parallel dp: row data parallelism, rank r takes the r-th of every `world` consecutive batches
      (batch_size = the per-GPU batch, global batch = world x batch_size); gradients exchanged by
      reduce-scatter / sharded optimizer / all-gather (--dp_mode sharded) or one all-reduce.
The seed is chosen on rank 0 and broadcast, so every rank draws the same permutations and weights.

Flow (train.py:61-256): metadata -> I/U orientation swap (:71-76) -> data_reader -> omni_model ->
compile(Adagrad(lr, 1e-8), 'mean_squared_error', metrics) -> epoch loop of fit_generator with
steps = floor(n/B) - 1 (:157-158) and validation -> early stopping on val_accurate_MSE with
patience (:160-177, first epoch never saves, :164-165) -> best checkpoint (safetensors instead of
h5) -> test: evaluate_generator + the manual masked RMSE of compute_full_RMSE (:225-255, fused:
SSE and target counts come from the loss epilogue).
"""
from __future__ import annotations

import argparse
import datetime
import json
import os

import numpy as np

DEFAULTS = dict(
    dataset="ml1m", useTimestamps=False, reverse_user_item_data=True, max_epochs=500,
    train_sparsity=[1.0, 1.0], test_sparsities=[0.0, 0.1, 0.4, 0.5, 0.6, 0.9], batch_size=128, patience=0,
    shuffle_data_every_epoch=True, val_split=[0.8, 0.1, 0.1], useJSON=True, early_stopping_metric="val_accurate_MSE",
    eval_mode="fixed_split", l2_weight_regulatization=None, pass_through_input_training=True, dropout_probability=0.2,
    numlayers=1, num_hidden_units=512, use_causal_info=False, auxilliary_mask_type=None, aux_var_value=-1,
    model_save_path="models/", model_loss="mean_squared_error", learning_rate=0.005, optimizer="adagrad",
    activation_type="sigmoid", use_sparse_representation=False, use_experimental_sparse_masking_layer=False,
    load_weights_from=None, perform_finetuning=False, compute_dtype="float32", metadata="./datasets_metadata.json",
    synthetic=None, seed=None, rng="numpy", parallel="feature", dp_mode="sharded", dp_grad_dtype="float32",
)


def shard_donor_weights(weights, c0, c1, n_total, k=1):
    """Keras-order weights [W0, b0, ..., W_L, b_L] of a full model -> the feature-parallel shard owning
    columns [c0, c1): W0's rows of those columns in each of the k input blocks, W_L's and b_L's columns;
    the hidden layers whole"""
    w = list(weights)
    rows = np.concatenate([np.arange(b * n_total + c0, b * n_total + c1) for b in range(k)])
    if w[0].shape[0] != k * n_total or w[-2].shape[1] != n_total:
        raise ValueError("donor shapes %s / %s do not match a %d-column model" % (w[0].shape, w[-2].shape, n_total))
    w[0] = w[0][rows]
    w[-2] = w[-2][:, c0:c1]
    w[-1] = w[-1][c0:c1]
    return w


class EarlyStopper(object):
    """The reference's early-stopping bookkeeping (train.py:147-177), separated from the training loop:
    the first epoch only sets the baseline and never saves (:164-165); an improvement saves and
    becomes the best epoch (:166-169); otherwise the run stops once i - best_epoch > patience (:171-177)."""

    def __init__(self, patience):
        self.patience = patience
        self.min_loss = None
        self.best_epoch = 0
        self.val_history = []

    def update(self, i, val_loss_list):
        """epoch i's validation history -> 'save', 'stop' or 'continue'"""
        val_loss = val_loss_list[-1]
        self.val_history.extend(val_loss_list)
        if self.min_loss is None:
            self.min_loss = val_loss
        elif self.min_loss > val_loss:
            self.min_loss, self.best_epoch = val_loss, i
            return "save"
        elif i - self.best_epoch > self.patience:
            return "stop"
        return "continue"

    def best_checkpoint(self, path_of_epoch, exists=os.path.exists):
        """train.py:181-199: the best epoch's checkpoint, or None -> test the most recent model"""
        fn = path_of_epoch(self.best_epoch + 1)
        return fn if exists(fn) else None


def _agree_on_seed(seed, world):
    """rank 0's seed (drawn if None) on every rank: same permutations, reciprocal masks and weights"""
    if seed is None:
        seed = int(np.random.randint(0, 2 ** 31 - 1))
    if world > 1:
        import torch.distributed as dist
        box = [seed]
        dist.broadcast_object_list(box, src=0)
        seed = int(box[0])
    return seed


def run(cfg):
    from . import optimizers as O
    from .data_reader import data_reader
    from .dataset import synthetic_fixed_split
    from .model import omni_model
    from .parallel import init_from_env
    from .parallel import feature_shard_range, make_comm
    rank, world, local = init_from_env()
    import torch
    torch.cuda.set_device(local)
    seed = cfg["seed"]
    if world > 1:
        seed = _agree_on_seed(seed, world)
    if seed is not None:
        np.random.seed(seed)
    fp = world > 1 and cfg["parallel"] == "feature"
    if world > 1 and cfg["parallel"] not in ("feature", "dp"):
        raise ValueError("--parallel must be feature or dp")
    # dataset parameters (train.py:62-76)
    if cfg["synthetic"]:
        data = synthetic_fixed_split(cfg["synthetic"], seed=0)
        num_items, num_users, rating_range = data.num_cols, data.train.n_rows, 4.5
        data_path = None
    else:
        with open(cfg["metadata"]) as f:
            meta = json.load(f)[cfg["dataset"]]
        data_path, num_items, num_users = meta["data_path"], meta["num_items"], meta["num_users"]
        rating_range = meta["rating_range"]
        data = None
        if cfg["reverse_user_item_data"]:
            num_items, num_users = num_users, num_items
    name = "stackedDenoising_WITHfinetuning_%s_%dbs_%dlay_%dhu_%slr_%sregul_%s_%s" % (
        cfg["train_sparsity"], cfg["batch_size"], cfg["numlayers"], cfg["num_hidden_units"], cfg["learning_rate"],
        cfg["l2_weight_regulatization"], cfg["auxilliary_mask_type"], cfg["activation_type"])
    if cfg["reverse_user_item_data"]:
        name += "_itemUserReverse"
    name += "_" + (cfg["synthetic"] or cfg["dataset"]) + "_" + datetime.datetime.now().strftime("%I_%M%p_%B_%d_%Y")
    shard = comm = None
    if fp:
        from .dataset import load_reference_json
        if data is None:
            data = load_reference_json(data_path, cfg["reverse_user_item_data"], cfg["useJSON"])
        c0, c1 = feature_shard_range(num_items, rank, world)
        data = data.column_shard(c0, c1)
        shard, comm = (c0, c1, num_items), make_comm(world)
    reader = data_reader(data.num_cols if fp else num_items, num_users, data_path, use_json=cfg["useJSON"],
                         eval_mode=cfg["eval_mode"], reverse_user_item_data=cfg["reverse_user_item_data"], dataset=data,
                         rng=cfg["rng"])
    B = cfg["batch_size"]
    om = omni_model(cfg["numlayers"], cfg["num_hidden_units"], reader.num_items, B,
                    dense_activation=cfg["activation_type"], use_causal_info=cfg["use_causal_info"],
                    use_both_masks=cfg["auxilliary_mask_type"] == "both",
                    l2_weight_regulatization=cfg["l2_weight_regulatization"],
                    dropout_probability=cfg["dropout_probability"], compute_dtype=cfg["compute_dtype"],
                    seed=seed, rating_range=rating_range, shard=shard, comm=comm)
    m = om.model
    opt = {"adagrad": lambda: O.Adagrad(lr=cfg["learning_rate"], epsilon=1e-08, decay=0.0),
           "rmsprop": lambda: O.RMSprop(lr=cfg["learning_rate"]),
           "adam": lambda: O.Adam(lr=cfg["learning_rate"])}[cfg["optimizer"]]()
    m.compile(opt, cfg["model_loss"], metrics=["mae", "accurate_MAE", "nMAE", "accurate_RMSE", "accurate_MSE"])
    if fp:
        m.enable_feature_parallel(rank, world)
    elif world > 1:
        m.enable_data_parallel(rank, world, mode=cfg["dp_mode"], grad_dtype=cfg["dp_grad_dtype"])
    if cfg["load_weights_from"]:
        # train.py:136-145: a donor checkpoint (safetensors from Model.save) -> every layer
        # (perform_finetuning) or the frozen outer layers of load_and_fix_for_denoising_autoencoders
        from .model import load_donor
        if rank == 0:
            print("Loading weights from ", cfg["load_weights_from"])
        full = os.path.join(cfg["model_save_path"], cfg["load_weights_from"])
        if fp and not os.path.exists(m.shard_path(full)):
            # a donor saved by an ordinary single-device run (the reference's case): this rank's columns of
            # the first and last layers
            donor = load_donor(full)
            donor.weights = shard_donor_weights(donor.weights, shard[0], shard[1], shard[2],
                                                1 + int(cfg["use_causal_info"]) + int(cfg["auxilliary_mask_type"] == "both"))
        else:
            donor = load_donor(m.shard_path(full))
        if cfg["perform_finetuning"]:
            if rank == 0:
                print("Fine tuning")
            om.manually_load_all_weights(donor)
        else:
            om.load_and_fix_for_denoising_autoencoders(donor)
        if m.dp is not None:
            m.dp.broadcast_params()
    os.makedirs(cfg["model_save_path"], exist_ok=True)
    stopper = EarlyStopper(cfg["patience"])
    path_of_epoch = lambda e: os.path.join(cfg["model_save_path"], name + "_epoch_%d_bestValidScore.safetensors" % e)
    aux, auxv = cfg["auxilliary_mask_type"], cfg["aux_var_value"]
    i = 0
    for i in range(cfg["max_epochs"]):
        if rank == 0:
            print("Starting epoch ", i + 1)
        tg = reader.data_gen(B, cfg["train_sparsity"], "train", cfg["shuffle_data_every_epoch"], aux, auxv,
                             pass_through_input_training=cfg["pass_through_input_training"])
        vg = reader.data_gen(B, cfg["train_sparsity"], "valid", cfg["shuffle_data_every_epoch"], aux, auxv)
        hist = m.fit_generator(tg, np.floor(reader.train_set_size / B) - 1, validation_data=vg,
                               validation_steps=np.floor(reader.val_set_size / B) - 1, verbose=int(rank == 0))
        action = stopper.update(i, hist.history[cfg["early_stopping_metric"]])
        if action == "save":
            m.save(path_of_epoch(i + 1))      # collective under dp / feature parallelism
        elif action == "stop":
            if rank == 0:
                print("Stopping early at epoch ", i + 1)
                print("Best epoch was ", stopper.best_epoch + 1)
                print("Val history: ", stopper.val_history)
            break
    best_epoch = stopper.best_epoch
    if world > 1:
        import torch.distributed as dist
        dist.barrier()                         # rank 0's checkpoint is complete before anyone reads it
    best_fn = stopper.best_checkpoint(lambda e: m.shard_path(path_of_epoch(e)))
    if best_fn is not None:
        m.load(path_of_epoch(best_epoch + 1), with_optimizer=False)
    elif rank == 0:
        print("FAILED TO LOAD BEST MODEL. TESTING WITH MOST RECENT MODEL.")
    test_gen = reader.data_gen(B, None, "test", cfg["shuffle_data_every_epoch"], aux, auxv)
    test_results = m.evaluate_generator(test_gen, np.floor(reader.test_set_size / B) - 1)
    test_results = test_results if isinstance(test_results, list) else [test_results]
    out = {"test_" + k: v for k, v in zip(m.metrics_names, test_results)}
    manual = reader.data_gen(B, None, "test", cfg["shuffle_data_every_epoch"], aux, auxv, return_target_count=True)
    sse, count = m.evaluate_sse(manual, int(np.floor(reader.test_set_size / B)))
    out["manual_test_RMSE"] = float(np.sqrt(sse / count)) if count else float("nan")
    out["best_epoch"] = best_epoch + 1
    out["epochs_run"] = i + 1
    out["val_history"] = list(stopper.val_history)
    out["tested_checkpoint"] = best_fn
    out["manual_test_rows"] = manual.rows_host[: int(np.floor(reader.test_set_size / B))]
    if rank == 0:
        print("Test results with fixed split")
        for k, v in out.items():
            if k != "manual_test_rows":
                print(k, " : ", v)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    for k, v in DEFAULTS.items():
        if isinstance(v, bool):
            ap.add_argument("--" + k, type=lambda s: s.lower() in ("1", "true", "yes"), default=v)
        elif isinstance(v, list):
            ap.add_argument("--" + k, type=json.loads, default=v)
        elif v is None:
            ap.add_argument("--" + k, type=lambda s: None if s in ("None", "none") else _num(s), default=None)
        else:
            ap.add_argument("--" + k, type=type(v), default=v)
    cfg = vars(ap.parse_args(argv))
    return run(cfg)


def _num(s):
    for t in (int, float):
        try:
            return t(s)
        except ValueError:
            pass
    return s


if __name__ == "__main__":
    main()
