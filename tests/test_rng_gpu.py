"""ocf_recip_keep on the device vs NumPy's legacy global RandomState (the reference's reciprocal-split
draws, data_reader.py:120,130, and everything NumPy draws after them): the raw uniform stream and the
end state bit-identical over >= 10^7 draws, the keep flags of an ML-20M-sized epoch bit-identical, and
the state-only path (data_sparsity [1, 1]) leaves NumPy exactly where the reference's draws leave it.
The golden batch tests (test_scatter_gpu.py, test_semantics_gpu.py) run the same path through
data_reader."""
import ctypes
import time

import numpy as np
import pytest


def _args(nb, B, boff, ebase, E, s0, s1, keep, doubles, dev):
    import torch

    from omnidirectional_collaborative_filtering_amd import _lib
    from omnidirectional_collaborative_filtering_amd.engine import ptr
    st = np.random.get_state()
    a = _lib.OcfRecipKeepArgs()
    key = np.ascontiguousarray(st[1], dtype=np.uint32)
    ctypes.memmove(a.key, key.ctypes.data, 624 * 4)
    a.pos, a.nb, a.B, a.n_entries, a.s0, a.s1 = int(st[2]), nb, B, E, s0, s1
    a.boff, a.ebase, a.keep = ptr(boff), ptr(ebase), ptr(keep)
    a.doubles = doubles.ctypes.data if doubles is not None else None
    n = _lib.load().ocf_recip_keep_workspace(nb, B, E, a.pos)
    assert n > 0
    ws = torch.empty(n, dtype=torch.uint8, device=dev)
    a.workspace, a.workspace_bytes = ptr(ws), n
    return a, st, ws


def _run(a):
    from omnidirectional_collaborative_filtering_amd import _lib
    from omnidirectional_collaborative_filtering_amd.engine import cur_stream
    _lib.call("ocf_recip_keep", a, cur_stream())
    return np.frombuffer(a.key, dtype=np.uint32).copy(), int(a.pos)


def _epoch(nb, B, mean_len, seed):
    g = np.random.default_rng(seed)
    lens = g.poisson(mean_len, size=(nb, B)).astype(np.int64)
    boff = np.zeros((nb, B + 1), np.int64)
    np.cumsum(lens, axis=1, out=boff[:, 1:])
    ebase = np.concatenate([[0], np.cumsum(boff[:, -1])]).astype(np.int64)
    return lens, boff, ebase


@pytest.mark.gpu
@pytest.mark.parametrize("pre", [0, 1, 311])
def test_uniform_stream_and_end_state(gpu, pre):
    """nb * B + entries doubles (>= 10^7) from a state with pos = 2 * pre, and the permutation after"""
    import torch
    lens, boff, ebase = _epoch(40, 256, 1000.0, pre)
    E = int(ebase[-1])
    n = 40 * 256 + E
    assert n >= 10_000_000
    np.random.seed(5 + pre)
    np.random.random_sample(pre)
    out = np.empty(n, np.float64)
    a, st, ws = _args(40, 256, None, None, E, 0.3, 0.7, None, out, gpu)
    k2, p2 = _run(a)
    np.random.set_state(st)
    want = np.random.random_sample(n)
    assert out.tobytes() == want.tobytes()
    wst = np.random.get_state()
    assert p2 == int(wst[2])
    np.testing.assert_array_equal(k2, wst[1])
    perm = np.random.permutation(26744)
    np.random.set_state((wst[0], k2, p2, wst[3], wst[4]))
    np.testing.assert_array_equal(np.random.permutation(26744), perm)
    del ws
    torch.cuda.synchronize()


@pytest.mark.gpu
@pytest.mark.parametrize("sp", [(0.3, 0.7), (0.5, 0.5), (0.0, 0.2), (0.123456, 0.9999)])
def test_keep_flags_ml20m_epoch(gpu, sp):
    """an ML-20M-sized epoch (104 batches of 256 item rows, ~600 ratings per row): keep flags equal the
    reference's choice([0, 1], p=[1-s, s]) draws (restated on random_sample, pinned in tests/test_rng.py)"""
    import torch
    nb, B = 104, 256
    lens, boff, ebase = _epoch(nb, B, 600.0, 9)
    E = int(ebase[-1])
    np.random.seed(1234)
    np.random.permutation(26744)              # the plan's permutation comes first (data_reader.py:326-327)
    boff_d = torch.as_tensor(boff, device=gpu)
    ebase_d = torch.as_tensor(ebase, device=gpu)
    keep = torch.empty(E, dtype=torch.uint8, device=gpu)
    a, st, ws = _args(nb, B, boff_d, ebase_d, E, sp[0], sp[1], keep, None, gpu)
    t0 = time.perf_counter()
    k2, p2 = _run(a)
    dt = time.perf_counter() - t0
    np.random.set_state(st)
    want = []
    for bi in range(nb):
        s = np.random.uniform(low=sp[0], high=sp[1], size=B)                  # data_reader.py:120
        u = np.random.random_sample(int(boff[bi, -1]))                        # :130, row after row
        want.append(u >= np.repeat((1.0 - s) / ((1.0 - s) + s), lens[bi]))
    want = np.concatenate(want)
    got = keep.cpu().numpy().astype(bool)
    assert np.array_equal(got, want), int((got != want).sum())
    wst = np.random.get_state()
    assert p2 == int(wst[2])
    np.testing.assert_array_equal(k2, wst[1])
    print("ML-20M-sized epoch (%d entries): %.2f ms" % (E, dt * 1e3))


@pytest.mark.gpu
@pytest.mark.parametrize("nb,B,mean_len", [(104, 256, 600.0), (3, 8, 2.0), (0, 256, 10.0), (1, 128, 0.1)])
def test_state_only_path(gpu, nb, B, mean_len):
    """keep = null (data_sparsity [1, 1]): no flags, but NumPy's state afterwards is the reference's"""
    lens, boff, ebase = _epoch(nb, B, mean_len, 3)
    E = int(ebase[-1])
    np.random.seed(99)
    np.random.random_sample(17)
    a, st, ws = _args(nb, B, None, None, E, 1.0, 1.0, None, None, gpu)
    k2, p2 = _run(a)
    np.random.set_state(st)
    for bi in range(nb):
        np.random.uniform(low=1.0, high=1.0, size=B)
        for n in lens[bi]:
            np.random.choice([0, 1], size=int(n), p=[0.0, 1.0])
    wst = np.random.get_state()
    assert p2 == int(wst[2])
    np.testing.assert_array_equal(k2, wst[1])


@pytest.mark.gpu
def test_tiny_epoch_flags_ready_when_the_call_returns(gpu):
    """every draw inside the caller's current 624-word block (no end-state copy to wait for): the call still
    synchronises its stream, so flags written on a side stream (data_reader's RNG stream) are complete when it
    returns -- read here on the main stream with no torch.cuda.synchronize in between"""
    import torch
    nb, B = 2, 8
    lens, boff, ebase = _epoch(nb, B, 3.0, 4)
    E = int(ebase[-1])
    np.random.seed(7)
    np.random.random_sample(3)
    pos = int(np.random.get_state()[2])
    assert 2 * (nb * B + E) <= 624 - pos, "the tiny epoch must fit in the current block"
    side = torch.cuda.Stream(device=gpu)
    with torch.cuda.stream(side):
        boff_d = torch.as_tensor(boff, device=gpu)
        ebase_d = torch.as_tensor(ebase, device=gpu)
        keep = torch.full((E,), 7, dtype=torch.uint8, device=gpu)
        a, st, ws = _args(nb, B, boff_d, ebase_d, E, 0.3, 0.7, keep, None, gpu)
        k2, p2 = _run(a)
    got = keep.cpu().numpy()                 # main stream: no wait on `side` besides the call's own
    np.random.set_state(st)
    want = []
    for bi in range(nb):
        s = np.random.uniform(low=0.3, high=0.7, size=B)
        u = np.random.random_sample(int(boff[bi, -1]))
        want.append(u >= np.repeat((1.0 - s) / ((1.0 - s) + s), lens[bi]))
    assert np.array_equal(got.astype(bool), np.concatenate(want)) and set(np.unique(got)) <= {0, 1}
    assert p2 == int(np.random.get_state()[2])
