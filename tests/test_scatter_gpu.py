"""K1 scatter (ocf_scatter_batch via data_reader.data_gen) vs the golden batches that the REFERENCE
data_reader.py produced (tests/golden/make_golden.py): bit-exact masks, ratings, target counts and
RNG carry-over across generators."""
import json
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _cfg():
    with open(os.path.join(GOLD, "batches_config.json")) as f:
        return json.load(f)


def _drain(gen, n):
    out = [next(gen) for _ in range(n)]
    assert next(gen) is None
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("ci", range(5))
def test_scatter_matches_reference_golden(gpu, ci):
    from omnidirectional_collaborative_filtering_amd.data_reader import data_reader
    cfg = _cfg()
    gold = np.load(os.path.join(GOLD, "batches.npz"))
    name, sp, pt, aux_type, auxv = cfg["train_configs"][ci]
    B = cfg["B"]
    meta = cfg["meta"]
    np.random.seed(cfg["seed_base"] + ci)
    rd = data_reader(meta["num_users"], meta["num_items"], os.path.join(GOLD, "toy"), nonsequentialusers=True,
                     use_json=True, eval_mode="fixed_split", reverse_user_item_data=True)
    seq = [
        ("train1", rd.data_gen(B, sp, "train", True, aux_type, auxv, pass_through_input_training=pt),
         rd.train_set_size),
        ("valid", rd.data_gen(B, sp, "valid", True, aux_type, auxv, return_target_count=True), rd.val_set_size),
        ("test", rd.data_gen(B, sp, "test", True, aux_type, auxv, return_target_count=True), rd.test_set_size),
        ("train2", rd.data_gen(B, sp, "train", True, aux_type, auxv, pass_through_input_training=pt),
         rd.train_set_size),
    ]
    checked = 0
    for tag, gen, n in seq:
        for bi, item in enumerate(_drain(gen, n // B)):
            ins = item[0]
            k = 0
            while "%s/%s/%d/in%d" % (name, tag, bi, k) in gold:
                want = gold["%s/%s/%d/in%d" % (name, tag, bi, k)].astype(np.float32)
                got = ins[k].cpu().numpy()
                np.testing.assert_array_equal(got, want, err_msg="%s %s batch %d input %d" % (name, tag, bi, k))
                k += 1
            assert k == len(ins)
            np.testing.assert_array_equal(item[1].cpu().numpy(),
                                          gold["%s/%s/%d/targets" % (name, tag, bi)].astype(np.float32))
            ck = "%s/%s/%d/count" % (name, tag, bi)
            if ck in gold:
                assert item[2] == int(gold[ck])
            checked += 1
    assert checked > 10


@pytest.mark.gpu
@pytest.mark.parametrize("ci", range(5))
def test_sparse_clear_keeps_layer0_input_exact(gpu, ci):
    """Generator batches reuse one layer-0 input buffer: each load clears only the previous batch's
    entries (ocf_scatter_clear) instead of a dense memset.  After a sequence of train and eval
    batches the buffer must equal the dense batch arrays exactly (no stale entries)."""
    import torch
    from omnidirectional_collaborative_filtering_amd.data_reader import data_reader
    from omnidirectional_collaborative_filtering_amd.model import omni_model
    cfg = _cfg()
    name, sp, pt, aux_type, auxv = cfg["train_configs"][ci]
    B = cfg["B"]
    meta = cfg["meta"]
    np.random.seed(cfg["seed_base"] + ci)
    rd = data_reader(meta["num_users"], meta["num_items"], os.path.join(GOLD, "toy"), nonsequentialusers=True,
                     use_json=True, eval_mode="fixed_split", reverse_user_item_data=True)
    N = rd.num_items
    causal = aux_type is not None
    both = aux_type == "both"
    om = omni_model(1, 8, N, B, use_causal_info=causal, use_both_masks=both, compute_dtype="float32", seed=1)
    e = om.engine
    e.sparse_clear = True
    gens = [rd.data_gen(B, sp, "train", True, aux_type, auxv, pass_through_input_training=pt),
            rd.data_gen(B, sp, "valid", True, aux_type, auxv, return_target_count=True),
            rd.data_gen(B, sp, "train", True, aux_type, auxv, pass_through_input_training=pt)]
    loads = 0
    for gen in gens:
        while True:
            item = next(gen)
            if item is None:
                break
            bi = gen.i - 1
            e.load_batch(gen.scatter_args(bi, engine_args=e.scatter_args()), gen.targets(bi, e.N), owner=gen)
            loads += 1
            torch.cuda.synchronize()
            ins = item[0]
            blocks = [ins[0]] + ([ins[1]] if causal else []) + ([ins[3]] if both else [])
            for k, want in enumerate(blocks):
                got = e.xin[:B, k * e.Np: k * e.Np + N].cpu().numpy()
                np.testing.assert_array_equal(got, want.cpu().numpy(), err_msg="%s load %d block %d" % (name, loads, k))
            rest = e.xin.clone()
            for k in range(len(blocks)):
                rest[:B, k * e.Np: k * e.Np + N] = 0
            assert not torch.any(rest != 0), "%s load %d: entries outside the batch" % (name, loads)
    assert loads >= 3
