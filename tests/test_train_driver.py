"""CPU: the epoch driver's early-stopping bookkeeping (train.py:147-199) on scripted validation
histories: the first epoch only sets the baseline and never saves, an improvement saves and becomes
the best epoch, the run stops once i - best_epoch > patience, and the best checkpoint (or, if none
was written, the most recent model) is what gets tested."""
from omnidirectional_collaborative_filtering_amd.train import EarlyStopper, _agree_on_seed


def _drive(vals, patience):
    st = EarlyStopper(patience)
    log = []
    for i, v in enumerate(vals):
        a = st.update(i, [v])
        log.append(a)
        if a == "stop":
            break
    return st, log


def test_first_epoch_never_saves():
    st, log = _drive([1.0, 2.0, 3.0], patience=5)
    assert log == ["continue", "continue", "continue"]
    assert st.best_epoch == 0
    # no checkpoint was written: train.py:195-198 falls back to the most recent model
    assert st.best_checkpoint(lambda e: "ckpt_%d" % e, exists=lambda fn: False) is None


def test_improvement_saves_and_moves_best_epoch():
    st, log = _drive([1.0, 0.9, 0.95, 0.8], patience=5)
    assert log == ["continue", "save", "continue", "save"]
    assert st.best_epoch == 3 and st.min_loss == 0.8
    written = {"ckpt_4"}
    assert st.best_checkpoint(lambda e: "ckpt_%d" % e, exists=written.__contains__) == "ckpt_4"


def test_patience_zero_stops_on_first_non_improvement_after_best():
    # train.py:31 patience = 0: i - best_epoch > 0 -> stop at the first epoch after the best that does
    # not improve; epoch 0 is the baseline (best_epoch stays 0), so epoch 1 without improvement stops
    st, log = _drive([1.0, 1.1, 0.5], patience=0)
    assert log == ["continue", "stop"]
    st, log = _drive([1.0, 0.9, 0.95, 0.7], patience=0)
    assert log == ["continue", "save", "stop"]
    assert st.best_epoch == 1 and st.val_history == [1.0, 0.9, 0.95]


def test_patience_counts_epochs_since_best():
    st, log = _drive([1.0, 0.9, 1.0, 1.0, 1.0, 0.1], patience=2)
    assert log == ["continue", "save", "continue", "continue", "stop"]


def test_equal_value_is_not_an_improvement():
    st, log = _drive([1.0, 0.5, 0.5], patience=1)
    assert log == ["continue", "save", "continue"]
    assert st.best_epoch == 1


def test_seed_agreement_single_process():
    assert _agree_on_seed(17, 1) == 17
    s = _agree_on_seed(None, 1)
    assert isinstance(s, int) and 0 <= s < 2 ** 31


def test_shard_donor_weights_slices_like_the_engine():
    """a single-device donor (the reference's load_weights_from case) sliced for feature-parallel rank
    columns [c0, c1): the same rows / columns Engine.init_weights gives a column shard"""
    import numpy as np
    from omnidirectional_collaborative_filtering_amd.train import shard_donor_weights
    rng = np.random.RandomState(0)
    NT, H, k, c0, c1 = 300, 7, 2, 128, 256
    w = [rng.rand(k * NT, H), rng.rand(H), rng.rand(H, H), rng.rand(H), rng.rand(H, NT), rng.rand(NT)]
    s = shard_donor_weights(w, c0, c1, NT, k)
    rows = np.concatenate([np.arange(b * NT + c0, b * NT + c1) for b in range(k)])
    np.testing.assert_array_equal(s[0], w[0][rows])
    np.testing.assert_array_equal(s[1], w[1])
    np.testing.assert_array_equal(s[2], w[2])
    np.testing.assert_array_equal(s[4], w[4][:, c0:c1])
    np.testing.assert_array_equal(s[5], w[5][c0:c1])
