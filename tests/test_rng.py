"""CPU: the MT19937 jump-ahead machinery behind ocf_recip_keep (csrc/ocf_rng.hip) is bit-identical to
NumPy's legacy global RandomState -- the stream the reference's reciprocal split draws from
(data_reader.py:120,130) and its row permutation (:326-327).  These run the library's host twin of the
device algorithm (same characteristic polynomial, same x^(624 * 2^k) jump table, same segment plan and
doubling tree of jumps, same double conversion); the device kernels are checked against NumPy in
tests/test_rng_gpu.py."""
import ctypes

import numpy as np
import pytest

from omnidirectional_collaborative_filtering_amd import _lib


def _state():
    st = np.random.get_state()
    return np.ascontiguousarray(st[1], dtype=np.uint32).copy(), int(st[2])


def _host_sample(key, pos, n):
    k = np.ascontiguousarray(key, dtype=np.uint32).copy()
    p = ctypes.c_int32(pos)
    out = np.empty(n, np.float64)
    _lib.call("ocf_mt_host_random_sample", k.ctypes.data, ctypes.addressof(p), n, out.ctypes.data)
    return out, k, p.value


@pytest.mark.parametrize("n_blocks", [0, 1, 2, 3, 255, 256, 257, 1000, 12345])
def test_jump_matches_numpy(n_blocks):
    """a block-aligned state (pos = 624, right after seeding) jumped by n_blocks * 624 words equals the
    state NumPy holds after drawing that many words (random_sample: 2 words per double)"""
    np.random.seed(1000 + n_blocks)
    key, pos = _state()
    assert pos == 624
    out = np.empty(624, np.uint32)
    _lib.call("ocf_mt_host_jump", key.ctypes.data, n_blocks, out.ctypes.data)
    np.random.random_sample(n_blocks * 312)
    want, wpos = _state()
    assert wpos == 624
    np.testing.assert_array_equal(out, want)


@pytest.mark.parametrize("pre,n", [(0, 1), (7, 311), (5, 312), (1, 20_000_000 // 2), (311, 5_000_001), (3, 79_872)])
def test_random_sample_bit_identical(pre, n):
    """n doubles from a state with pos = 2 * pre (mid-block): every double bit-identical, the end state
    (key and pos) equal, and NumPy continues identically after set_state (the next permutation).
    (1, 10^7): >= 10^7 draws across 126 jump-started segments."""
    np.random.seed(77 + pre)
    np.random.random_sample(pre)
    key, pos = _state()
    got, k2, p2 = _host_sample(key, pos, n)
    want = np.random.random_sample(n)
    assert got.tobytes() == want.tobytes()
    wk, wp = _state()
    assert p2 == wp
    np.testing.assert_array_equal(k2, wk)
    perm_ref = np.random.permutation(26744)
    st = np.random.get_state()
    np.random.set_state((st[0], k2, p2, st[3], st[4]))
    np.testing.assert_array_equal(np.random.permutation(26744), perm_ref)


def test_uniform_and_choice_restatement():
    """the two reference calls in terms of random_sample (what ocf_recip_keep computes per batch)"""
    B, lens = 16, np.array([0, 3, 7, 1, 12, 0, 5, 9, 2, 2, 4, 8, 1, 6, 3, 10])
    for s0, s1 in ([0.3, 0.7], [0.5, 0.5], [0.0, 0.2], [1.0, 1.0], [0.123456, 0.9999]):
        np.random.seed(5)
        s = np.random.uniform(low=s0, high=s1, size=B)
        ref = [np.random.choice([0, 1], size=int(n), p=[1 - s[j], s[j]]) for j, n in enumerate(lens)]
        np.random.seed(5)
        u = np.random.random_sample(B + int(lens.sum()))
        s_r = s0 + (s1 - s0) * u[:B]
        assert s_r.tobytes() == s.tobytes()
        cut = (1.0 - s_r) / ((1.0 - s_r) + s_r)
        keep = u[B:] >= np.repeat(cut, lens)
        np.testing.assert_array_equal(keep, np.concatenate(ref).astype(bool))
