"""Training driver with the reference train.py parameter surface (train.py:19-59).

    python -m omnidirectional_collaborative_filtering_amd.train --dataset ml1m --metadata datasets_metadata.json
    python -m omnidirectional_collaborative_filtering_amd.train --synthetic ml1m --max_epochs 5
    torchrun --nproc-per-node 8 -m omnidirectional_collaborative_filtering_amd.train --synthetic ml20m

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
    load_weights_from=None, compute_dtype="float32", metadata="./datasets_metadata.json", synthetic=None, seed=None,
    rng="numpy",
)


def run(cfg):
    from . import optimizers as O
    from .data_reader import data_reader
    from .dataset import synthetic_fixed_split
    from .model import omni_model
    from .parallel import init_from_env
    rank, world, local = init_from_env()
    import torch
    torch.cuda.set_device(local)
    if cfg["seed"] is not None:
        np.random.seed(cfg["seed"])
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
    reader = data_reader(num_items, num_users, data_path, use_json=cfg["useJSON"], eval_mode=cfg["eval_mode"],
                         reverse_user_item_data=cfg["reverse_user_item_data"], dataset=data, rng=cfg["rng"])
    B = cfg["batch_size"]
    om = omni_model(cfg["numlayers"], cfg["num_hidden_units"], num_items, B, dense_activation=cfg["activation_type"],
                    use_causal_info=cfg["use_causal_info"], use_both_masks=cfg["auxilliary_mask_type"] == "both",
                    l2_weight_regulatization=cfg["l2_weight_regulatization"],
                    dropout_probability=cfg["dropout_probability"], compute_dtype=cfg["compute_dtype"],
                    seed=cfg["seed"], rating_range=rating_range)
    m = om.model
    opt = {"adagrad": lambda: O.Adagrad(lr=cfg["learning_rate"], epsilon=1e-08, decay=0.0),
           "rmsprop": lambda: O.RMSprop(lr=cfg["learning_rate"]),
           "adam": lambda: O.Adam(lr=cfg["learning_rate"])}[cfg["optimizer"]]()
    m.compile(opt, cfg["model_loss"], metrics=["mae", "accurate_MAE", "nMAE", "accurate_RMSE", "accurate_MSE"])
    if world > 1:
        m.enable_data_parallel(rank, world)
    if cfg["load_weights_from"]:
        m.load(cfg["load_weights_from"], with_optimizer=False)
    os.makedirs(cfg["model_save_path"], exist_ok=True)
    min_loss, best_epoch, val_history = None, 0, []
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
        vl = hist.history[cfg["early_stopping_metric"]]
        val_loss = vl[-1]
        val_history.extend(vl)
        if min_loss is None:
            min_loss = val_loss
        elif min_loss > val_loss:
            min_loss, best_epoch = val_loss, i
            if rank == 0:
                m.save(os.path.join(cfg["model_save_path"], name + "_epoch_%d_bestValidScore.safetensors" % (i + 1)))
        elif i - best_epoch > cfg["patience"]:
            if rank == 0:
                print("Stopping early at epoch ", i + 1)
                print("Best epoch was ", best_epoch + 1)
                print("Val history: ", val_history)
            break
    best_fn = os.path.join(cfg["model_save_path"], name + "_epoch_%d_bestValidScore.safetensors" % (best_epoch + 1))
    if os.path.exists(best_fn):
        m.load(best_fn, with_optimizer=False)
    else:
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
    if rank == 0:
        print("Test results with fixed split")
        for k, v in out.items():
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
