"""Generate the golden batch fixtures by running the REFERENCE batch assembler.

Run in the build container only (needs /root/reference):   python tests/golden/make_golden.py

What it does
  1. Writes a small fixed-split dataset in the reference's JSON layout
     (ratingsByItem_dicts_{train,valid,test}.json + unique_users_list.json, I-AutoRec orientation,
     split semantics of TrainValidTestSplit.py:74-103) under tests/golden/toy/.
  2. Imports /root/reference/data_reader.py with two shims: a stub
     ``tensorflow`` module (data_reader.py:7 imports SparseTensor but never uses it) and
     dict_keys -> list for the set orders (data_reader.py:78-80 are py2 lists).
  3. Runs the reference ``data_gen`` for a matrix of configurations under fixed seeds, consuming
     generators in the order train.py does (train epoch, then valid, then test, then a second
     train epoch -- so RNG carry-over between generators is pinned too), and stores every
     yielded array as data in tests/golden/batches.npz.
  4. Cross-checks oracle/batch_oracle.py against the same outputs.

Only inputs/outputs (data) are committed; no reference source travels.
"""
from __future__ import annotations

import json
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
TOY = os.path.join(HERE, "toy")
TOY_U = os.path.join(HERE, "toy_u")     # the same ratings in the U-AutoRec orientation

B = 8

# (name, split-config) for train generators
TRAIN_CONFIGS = [
    # name,          sparsity,     pass_through, aux_type,  aux_value
    ("default",      [1.0, 1.0],   True,  None,      -1),
    ("recip_drop",   [0.3, 0.7],   False, "dropout", -1),
    ("recip_both",   [0.3, 0.7],   True,  "both",     1),
    ("half_causal",  [0.5, 0.5],   False, "causal",  -1),
    ("low_zeros",    [0.0, 0.2],   True,  "zeros",    1),
]


def make_toy_dataset(path, n_rows=43, n_cols=29, density=0.35, seed=11):
    """Rating-level 80/10/10 split (TrainValidTestSplit.py:74-103), I-orientation, JSON layout."""
    rng = np.random.RandomState(seed)
    ratings = []
    for r in range(n_rows):
        for c in range(n_cols):
            if rng.random_sample() < density:
                ratings.append((r, c, float(rng.randint(1, 11)) / 2.0))
    # edge cases: a duplicated (row, col) with a different value (last-write-wins),
    # and a rating of exactly 0.0 (Jester-style, must still set the masks)
    ratings.append((ratings[3][0], ratings[3][1], 4.5))
    ratings.append((5, 7, 0.0))
    n = len(ratings)
    perm = rng.permutation(n)
    ntr, nva = int(n * 0.8), int(n * 0.1)
    tr, va, te = perm[:ntr], perm[ntr:ntr + nva], perm[ntr + nva:]
    row_key = lambda r: str(1000 + 3 * r)          # raw item ids as JSON string keys
    col_key = lambda c: str(500 + 7 * c)           # raw user ids, as in unique_users_list

    def build(idx):
        d = {}
        for i in idx:
            r, c, v = ratings[i]
            d.setdefault(row_key(r), []).append([col_key(c), v])
        return d

    train = build(tr)
    valid_t = build(va)
    test_t = build(te)
    test_in = build(np.concatenate([tr, va]))
    valid_in = {k: train.get(k) for k in valid_t}          # None -> zero input row
    test_inp = {k: test_in.get(k) for k in test_t}
    os.makedirs(path, exist_ok=True)
    uniq = [col_key(c) for c in rng.permutation(n_cols)]    # column order != raw-id order
    files = {
        "ratingsByItem_dicts_train": train,
        "ratingsByItem_dicts_valid": [valid_in, valid_t],
        "ratingsByItem_dicts_test": [test_inp, test_t],
        "unique_users_list": uniq,
        "unique_items_list": sorted({row_key(r) for r, _, _ in ratings}),
    }
    for k, v in files.items():
        with open(os.path.join(path, k + ".json"), "w") as f:
            json.dump(v, f)
    meta = {"num_items": len(files["unique_items_list"]), "num_users": n_cols,
            "rating_range": 4.5, "nonsequentialusers": True}
    with open(os.path.join(path, "metadata.json"), "w") as f:
        json.dump(meta, f)
    # U orientation (reverse_user_item_data=False, data_reader.py:20-23,46-49): rows = users,
    # columns = items in unique_items_list order (permuted: column order != raw-id order)
    rng_u = np.random.RandomState(seed + 1)

    def build_u(idx):
        d = {}
        for i in idx:
            r, c, v = ratings[i]
            d.setdefault(col_key(c), []).append([row_key(r), v])
        return d
    train_u, valid_u, test_u = build_u(tr), build_u(va), build_u(te)
    test_in_u = build_u(np.concatenate([tr, va]))
    items = sorted({row_key(r) for r, _, _ in ratings})
    files_u = {
        "ratingsByUser_dicts_train": train_u,
        "ratingsByUser_dicts_valid": [{k: train_u.get(k) for k in valid_u}, valid_u],
        "ratingsByUser_dicts_test": [{k: test_in_u.get(k) for k in test_u}, test_u],
        "unique_items_list": [items[i] for i in rng_u.permutation(len(items))],
        "unique_users_list": sorted({col_key(c) for _, c, _ in ratings}),
    }
    os.makedirs(TOY_U, exist_ok=True)
    for k, v in files_u.items():
        with open(os.path.join(TOY_U, k + ".json"), "w") as f:
            json.dump(v, f)
    meta_u = {"num_items": len(items), "num_users": len(files_u["unique_users_list"]), "rating_range": 4.5,
              "nonsequentialusers": True}
    with open(os.path.join(TOY_U, "metadata.json"), "w") as f:
        json.dump(meta_u, f)
    return meta, meta_u


def import_reference():
    tf = types.ModuleType("tensorflow")
    tf.SparseTensor = object
    sys.modules.setdefault("tensorflow", tf)
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import data_reader as ref_dr  # noqa: E402  (reference module, build container only)
    return ref_dr


def ref_reader(ref_dr, meta, u=False):
    if u:      # U orientation: train.py passes num_items / num_users unswapped (train.py:71-76)
        rd = ref_dr.data_reader(meta["num_items"], meta["num_users"], TOY_U + "/", nonsequentialusers=True,
                                use_json=True, eval_mode="fixed_split", useTimestamps=False,
                                reverse_user_item_data=False)
    else:      # train.py:71-76 swaps num_items/num_users for I-AutoRec
        rd = ref_dr.data_reader(meta["num_users"], meta["num_items"], TOY + "/", nonsequentialusers=True,
                                use_json=True, eval_mode="fixed_split", useTimestamps=False,
                                reverse_user_item_data=True)
    rd.train_set = list(rd.train_set)
    rd.val_set = list(rd.val_set)
    rd.test_set = list(rd.test_set)
    return rd


def drain(gen, n, with_count=False):
    out = []
    for _ in range(n):
        item = next(gen)
        out.append(item)
    assert next(gen) is None
    return out


def run_configs(ref_dr, meta, u):
    from oracle.batch_oracle import ReaderOracle
    store = {}
    for ci, (name, sp, pt, aux_type, auxv) in enumerate(TRAIN_CONFIGS):
        for impl in ("ref", "oracle"):
            np.random.seed(1234 + ci)
            rd = ref_reader(ref_dr, meta, u) if impl == "ref" else \
                ReaderOracle.from_dir(TOY_U if u else TOY, reverse_user_item_data=not u)
            ntr = rd.train_set_size if impl == "ref" else len(rd.train_keys)
            nva = rd.val_set_size if impl == "ref" else len(rd.valid_keys)
            nte = rd.test_set_size if impl == "ref" else len(rd.test_keys)
            seq = []
            if impl == "ref":
                g = lambda split, **kw: rd.data_gen(B, sp, train_val_test=split, shuffle=True,
                                                   auxilliary_mask_type=aux_type, aux_var_value=auxv, **kw)
            else:
                g = lambda split, **kw: rd.data_gen(B, sp, split=split, shuffle=True, aux_type=aux_type,
                                                   aux=auxv, **{("pass_through" if k == "pass_through_input_training" else k): v for k, v in kw.items()})
            seq.append(("train1", drain(g("train", pass_through_input_training=pt), ntr // B)))
            seq.append(("valid", drain(g("valid", return_target_count=True), nva // B)))
            seq.append(("test", drain(g("test", return_target_count=True), nte // B)))
            seq.append(("train2", drain(g("train", pass_through_input_training=pt), ntr // B)))
            if impl == "ref":
                ref_seq = seq
            else:
                ora_seq = seq
        # compare + store
        for (tag, rb), (_, ob) in zip(ref_seq, ora_seq):
            assert len(rb) == len(ob)
            for bi, (ri, oi) in enumerate(zip(rb, ob)):
                rin, oin = ri[0], oi[0]
                assert len(rin) == len(oin), (name, tag, bi)
                for k, (a, b) in enumerate(zip(rin, oin)):
                    assert np.array_equal(a, b), (name, tag, bi, k)
                    store["%s/%s/%d/in%d" % (name, tag, bi, k)] = np.asarray(a)
                assert np.array_equal(ri[1], oi[1]), (name, tag, bi, "targets")
                store["%s/%s/%d/targets" % (name, tag, bi)] = np.asarray(ri[1])
                if len(ri) == 3:
                    assert ri[2] == oi[2]
                    store["%s/%s/%d/count" % (name, tag, bi)] = np.asarray(ri[2])
        print("%s config %-12s ok (%d train batches)" % ("U" if u else "I", name, ntr // B))
    return store


def main():
    meta, meta_u = make_toy_dataset(TOY)
    ref_dr = import_reference()
    sys.path.insert(0, REPO)
    np.savez_compressed(os.path.join(HERE, "batches.npz"), **run_configs(ref_dr, meta, False))
    store_u = run_configs(ref_dr, meta_u, True)
    np.savez_compressed(os.path.join(HERE, "batches_u.npz"), **store_u)
    store = store_u
    cfg = {"B": B, "train_configs": TRAIN_CONFIGS, "seed_base": 1234,
           "sequence": ["train1", "valid", "test", "train2"], "meta": meta,
           "u": {"dir": "toy_u", "npz": "batches_u.npz", "meta": meta_u, "reverse_user_item_data": False},
           "generator": "reference data_reader.py via tests/golden/make_golden.py"}
    with open(os.path.join(HERE, "batches_config.json"), "w") as f:
        json.dump(cfg, f, indent=1)
    print("wrote", len(store), "arrays")


if __name__ == "__main__":
    main()
