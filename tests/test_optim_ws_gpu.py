"""The persistent role-split optimizer kernel (ocf_optim_ws.h; the dense-operand EPI_OPTIM path: 16-bit
dense batches, K <= 512) is bit-identical to the generic tile kernel + EpiOptim epilogue: every optimizer,
shadows, the in-kernel output-bias column sums, K from one K-step to many (odd and even), fewer tiles than
workgroups; its oracle parity is tests/test_train_gpu.py::test_low_precision_dropout[False-*].  Also the
tile buckets / row lists of ocf_sparse_tiles (the row-stream kernel tests build their lists with it)."""
import numpy as np
import pytest
import torch

from omnidirectional_collaborative_filtering_amd import _lib
from omnidirectional_collaborative_filtering_amd.engine import cur_stream

OPTS = {
    "adagrad": lambda gs: _lib.OcfOptParams(_lib.OPT_ADAGRAD, 0.01, 1e-8, 0, 0, 0, gs),
    "rmsprop": lambda gs: _lib.OcfOptParams(_lib.OPT_RMSPROP, 0.001, 1e-8, 0.9, 0, 0, gs),
    "adam": lambda gs: _lib.OcfOptParams(_lib.OPT_ADAM, 0.001, 1e-8, 0.9, 0.999, 0, gs),
    "adagrad_l2": lambda gs: _lib.OcfOptParams(_lib.OPT_ADAGRAD, 0.01, 1e-8, 0, 0, 1e-3, gs),
}


def _tune(key, value):
    prev = _lib.I32(0)
    _lib.call("ocf_set_tuning", key, int(value), prev)
    return prev.value


def set_ws(on):
    """route EPI_OPTIM to the role-split kernel (at every K, so all shapes here exercise it) or to
    the generic kernel; returns the previous setting for set_ws(prev)"""
    if isinstance(on, tuple):
        _tune(b"optim_ws_max_k", on[1])
        return (_tune(b"optim_ws", on[0]), None)
    return (_tune(b"optim_ws", on), _tune(b"optim_ws_max_k", 1 << 30))


def _sparse_batch(M, K, krows, seed, col_frac=None):
    """a CSR over M columns, a batch of `krows` of its rows (some batch slots empty) and per-entry
    values in list order; returns the descriptor tensors and the dense [K][M] equivalent"""
    from omnidirectional_collaborative_filtering_amd.dataset import RatingsCSR
    rng = np.random.RandomState(seed)
    R = 3 * krows + 5
    lens = rng.randint(0, max(2, M // 4), size=R)
    lens[rng.rand(R) < 0.1] = 0
    rp = np.zeros(R + 1, np.int64)
    np.cumsum(lens, out=rp[1:])
    if col_frac is None:
        col = np.concatenate([rng.choice(M, size=n, replace=False) for n in lens]).astype(np.int32)
    else:                                           # columns from a random subset only
        cand = np.setdiff1d(np.arange(M), np.arange(128, 256)) if M >= 384 else np.arange(M)   # tile 1 empty
        pool = np.sort(rng.choice(cand, size=int(len(cand) * col_frac), replace=False))
        lens = np.minimum(lens, len(pool))
        rp[1:] = np.cumsum(lens)
        col = np.concatenate([rng.choice(pool, size=n, replace=False) for n in lens]).astype(np.int32)
    csr = RatingsCSR(rp, col, np.ones(len(col), np.float32))
    col_s, _, lidx_s, tptr = csr.tile_index(M)
    rows = rng.choice(R, size=krows, replace=False).astype(np.int32)
    rows[rng.rand(krows) < 0.1] = -1
    blens = np.where(rows >= 0, lens[np.maximum(rows, 0)], 0)
    lboff = np.zeros(krows + 1, np.int64)
    np.cumsum(blens, out=lboff[1:])
    vals = rng.randn(max(1, int(lboff[-1]))).astype(np.float32)
    vals[rng.rand(len(vals)) < 0.2] = 0.0           # live-entry flags zero some entries
    dense = np.zeros((K, M), np.float32)
    for b, r in enumerate(rows):
        if r < 0:
            continue
        for j in range(lens[r]):
            dense[b, col[rp[r] + j]] = vals[lboff[b] + j]
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    d = dict(sp_rows=dev(rows), sp_rp=dev(rp), sp_tptr=dev(tptr), sp_col=dev(col_s), sp_lidx=dev(lidx_s),
             sp_lboff=dev(lboff), sp_vals=dev(vals), sp_ntiles=tptr.shape[1] - 1, sp_krows=krows)
    return d, dense


def _buckets(sp, M, K, extra=None):
    """ocf_sparse_tiles on a sparse descriptor: (bptr, ent) device tensors"""
    gm, nk = M // 128, K // 64
    cap = max(1, int(sp["sp_lboff"][-1].item()) + 4 * M)
    cnt = torch.zeros(gm * nk, dtype=torch.int32, device="cuda")
    bptr = torch.zeros(gm * nk + 1, dtype=torch.int32, device="cuda")
    ent = torch.full((cap, 2), -9, dtype=torch.int32, device="cuda")
    a = _lib.OcfTileBucketArgs()
    a.rows, a.rp, a.tptr = sp["sp_rows"].data_ptr(), sp["sp_rp"].data_ptr(), sp["sp_tptr"].data_ptr()
    a.col, a.lidx, a.lboff = sp["sp_col"].data_ptr(), sp["sp_lidx"].data_ptr(), sp["sp_lboff"].data_ptr()
    a.krows, a.ntiles, a.gm, a.nk = sp["sp_krows"], sp["sp_ntiles"], gm, nk
    a.cnt, a.bptr, a.ent, a.cap = cnt.data_ptr(), bptr.data_ptr(), ent.data_ptr(), cap
    for k, v in (extra or {}).items():
        setattr(a, k, v.data_ptr() if torch.is_tensor(v) else v)
    _lib.call("ocf_sparse_tiles", a, cur_stream())
    torch.cuda.synchronize()
    return bptr, ent


def _run(cd, M, N, K, opt, A, Bm, state, sparse=None, shadow_blocked=None, colsum=False, extra=None):
    P, S1, S2 = (t.clone() for t in state)
    sdt = torch.float16 if cd == _lib.DT_F16 else torch.bfloat16
    # shadow starts as the rounded copy of P (row-major layout), as the engine keeps it
    Sh = (P.to(sdt) if shadow_blocked == 0 else torch.zeros(M, N, device="cuda", dtype=sdt)) \
        if shadow_blocked is not None else None
    cs = torch.full((M,), -7.0, device="cuda") if colsum else None
    a = _lib.OcfGemmArgs()
    a.compute_dtype = cd
    a.A, a.a_dtype, a.a_col, a.lda = A.data_ptr(), cd, 1, M
    a.B, a.b_dtype, a.b_col, a.ldb = Bm.data_ptr(), cd, 1, N
    a.M, a.N, a.K, a.splits, a.epi = M, N, K, 1, _lib.EPI_OPTIM
    a.p, a.ld_out = P.data_ptr(), N
    a.s1 = S1.data_ptr()
    a.s2 = S2.data_ptr() if opt.kind == _lib.OPT_ADAM else None
    a.opt = opt
    if Sh is not None:
        a.p_shadow, a.shadow_blocked = Sh.data_ptr(), shadow_blocked
    if cs is not None:
        a.sp_colsum = cs.data_ptr()
    if sparse is not None:
        a.a_sparse = 1
        for k, v in sparse.items():
            setattr(a, k, v.data_ptr() if torch.is_tensor(v) else v)
    for k, v in (extra or {}).items():
        setattr(a, k, v.data_ptr() if torch.is_tensor(v) else v)
    _lib.call("ocf_gemm", a, cur_stream())
    torch.cuda.synchronize()
    return [P, S1, S2] + ([Sh] if Sh is not None else []) + ([cs] if cs is not None else [])


def _both(cd, M, N, K, opt, A, Bm, state, **kw):
    prev = set_ws(0)
    try:
        ref = _run(cd, M, N, K, opt, A, Bm, state, **kw)
        set_ws(1)
        got = _run(cd, M, N, K, opt, A, Bm, state, **kw)
    finally:
        set_ws(prev)
    return ref, got


def _operands(cd, M, N, K, seed):
    g = torch.Generator().manual_seed(seed)
    td = torch.float16 if cd == _lib.DT_F16 else torch.bfloat16
    A = torch.randn(K, M, generator=g).to(td).cuda()
    Bm = torch.randn(K, N, generator=g).to(td).cuda()
    P = (torch.randn(M, N, generator=g) * 0.05).cuda()
    S1 = torch.rand(M, N, generator=g).cuda()
    S2 = torch.rand(M, N, generator=g).cuda()
    return A, Bm, (P, S1, S2)


@pytest.mark.gpu
@pytest.mark.parametrize("cd", [_lib.DT_F16, _lib.DT_BF16])
@pytest.mark.parametrize("shape", [(128, 128, 64), (384, 256, 192), (1152, 512, 256), (640, 384, 2048)])
@pytest.mark.parametrize("opt", ["adagrad", "adam", "rmsprop", "adagrad_l2"])
def test_ws_dense_bit_identical(gpu, cd, shape, opt):
    M, N, K = shape
    A, Bm, state = _operands(cd, M, N, K, seed=M + K)
    ref, got = _both(cd, M, N, K, OPTS[opt](1e-3), A, Bm, state, shadow_blocked=1, colsum=True)
    for r, x in zip(ref, got):
        assert torch.equal(r, x)
    assert not torch.equal(ref[0], state[0])      # the update happened


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(256, 128, 64, 40), (1280, 512, 256, 256), (512, 256, 320, 300)])
def test_sparse_tiles_buckets(gpu, shape):
    """ocf_sparse_tiles against a NumPy restatement: bucket (t, kt) = rows of K-step kt in order,
    each row's entries of column tile t in column order, as (value index, k | m_local << 8)."""
    M, N, K, krows = shape
    sp, _ = _sparse_batch(M, K, krows, seed=K)
    bptr, ent = _buckets(sp, M, K)
    h = {k: (v.cpu().numpy() if torch.is_tensor(v) else v) for k, v in sp.items()}
    gm, nk = M // 128, K // 64
    want = []
    ptr = [0]
    for t in range(gm):
        for kt in range(nk):
            for b in range(kt * 64, min(krows, kt * 64 + 64)):
                r = h["sp_rows"][b]
                if r < 0:
                    continue
                e0 = h["sp_rp"][r] + h["sp_tptr"][r, t]
                e1 = h["sp_rp"][r] + h["sp_tptr"][r, t + 1]
                for e in range(e0, e1):
                    want.append((h["sp_lboff"][b] + h["sp_lidx"][e], (b - kt * 64) | ((h["sp_col"][e] - 128 * t) << 8)))
            ptr.append(len(want))
    np.testing.assert_array_equal(bptr.cpu().numpy(), np.array(ptr, np.int32))
    got = ent[: len(want)].cpu().numpy()
    np.testing.assert_array_equal(got, np.array(want, np.int32).reshape(-1, 2))


@pytest.mark.gpu
def test_ws_matches_torch_reference(gpu):
    """Adagrad on the f16 product against a float64 torch reference of the same op."""
    M, N, K = 768, 256, 256
    cd = _lib.DT_F16
    A, Bm, state = _operands(cd, M, N, K, seed=9)
    gs = 1e-3
    prev = set_ws(1)
    try:
        P, S1, _, cs = _run(cd, M, N, K, OPTS["adagrad"](gs), A, Bm, state, colsum=True)
    finally:
        set_ws(prev)
    G = (A.double().t() @ Bm.double()) * gs
    a = state[1].double() + G * G
    p = state[0].double() - 0.01 * G / (a.sqrt() + 1e-8)
    assert torch.allclose(S1.double(), a, rtol=1e-5, atol=1e-6)
    assert torch.allclose(P.double(), p, rtol=1e-5, atol=1e-6)
    assert torch.allclose(cs.double(), A.double().sum(0) * gs, rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("opt", ["adagrad", "adam"])
def test_folded_jobs_match_separate_kernels(gpu, opt):
    """cb_* / jb_* / js_* jobs folded into the persistent launch equal the separate launches the
    generic path makes (ocf_bias_opt_from_partials, ocf_stats_finalize), bit for bit."""
    M, N, K = 1152, 512, 256
    cd = _lib.DT_F16
    A, Bm, state = _operands(cd, M, N, K, seed=21)
    g = torch.Generator().manual_seed(22)
    H, parts, rows, nt = 500, 256, 256, 3
    part = torch.randn(parts, 512, generator=g).cuda() * 1e-2
    sp_stats = torch.rand(parts, 4, generator=g).cuda()
    rs = torch.rand(nt, rows, generator=g).cuda()
    bias0 = [torch.randn(M, generator=g).cuda(), torch.rand(M, generator=g).cuda(), torch.rand(M, generator=g).cuda()]
    hb0 = [torch.randn(512, generator=g).cuda(), torch.rand(512, generator=g).cuda(), torch.rand(512, generator=g).cuda()]
    bop = OPTS[opt](1.0)

    def run(ws):
        cb = [t.clone() for t in bias0]
        hb = [t.clone() for t in hb0]
        out = torch.zeros(4 + rows, device="cuda")
        P, S1, S2 = (t.clone() for t in state)
        cs = torch.zeros(M, device="cuda")
        a = _lib.OcfGemmArgs()
        a.compute_dtype = cd
        a.A, a.a_dtype, a.a_col, a.lda = A.data_ptr(), cd, 1, M
        a.B, a.b_dtype, a.b_col, a.ldb = Bm.data_ptr(), cd, 1, N
        a.M, a.N, a.K, a.splits, a.epi = M, N, K, 1, _lib.EPI_OPTIM
        a.p, a.s1, a.ld_out = P.data_ptr(), S1.data_ptr(), N
        a.s2 = S2.data_ptr() if opt == "adam" else None
        a.opt = OPTS[opt](1e-3)
        a.sp_colsum = cs.data_ptr()
        a.cb_p, a.cb_s1 = cb[0].data_ptr(), cb[1].data_ptr()
        a.cb_s2 = cb[2].data_ptr() if opt == "adam" else None
        a.cb_op = bop
        a.jb_part, a.jb_parts, a.jb_ld, a.jb_n = part.data_ptr(), parts, 512, H
        a.jb_p, a.jb_s1 = hb[0].data_ptr(), hb[1].data_ptr()
        a.jb_s2 = hb[2].data_ptr() if opt == "adam" else None
        a.jb_op = bop
        a.js_sp, a.js_nparts, a.js_rs, a.js_ntiles, a.js_M, a.js_out = (sp_stats.data_ptr(), parts, rs.data_ptr(), nt,
                                                                          rows, out.data_ptr())
        prev = set_ws(ws)
        try:
            _lib.call("ocf_gemm", a, cur_stream())
            torch.cuda.synchronize()
        finally:
            set_ws(prev)
        return [P, S1, S2, cs, out] + cb + hb

    ref, got = run(0), run(1)
    for i, (r, x) in enumerate(zip(ref, got)):
        assert torch.equal(r, x), i
    assert not torch.equal(ref[5], bias0[0]) and not torch.equal(ref[8], hb0[0])


def live_records(live):
    """NumPy restatement of ocf.h OCF_LIVE_REC for a boolean live-row vector (len a multiple of 128)"""
    gm = len(live) // 128
    rec = np.zeros((gm, _lib.LIVE_REC), np.uint8)
    for t in range(gm):
        rows = np.nonzero(live[128 * t: 128 * t + 128])[0]
        rec[t, :4] = np.frombuffer(np.int32(len(rows)).tobytes(), np.uint8)
        for k, r in enumerate(rows):
            rec[t, 16 + (k % 8) * 16 + k // 8] = r
    return rec.reshape(-1)


def _rec_valid(rec):
    """(L per tile, the bytes of ranks < L) of a record array"""
    rec = rec.reshape(-1, _lib.LIVE_REC)
    L = rec[:, :4].copy().view(np.int32)[:, 0]
    out = []
    for t, n in enumerate(L):
        out.append([rec[t, 16 + (k % 8) * 16 + k // 8] for k in range(n)])
    return L, out


@pytest.mark.gpu
@pytest.mark.parametrize("opt", ["rmsprop", "adam", "adagrad_l2"])
def test_ws_live_rows_rejected_unless_identity(gpu, opt):
    """live-row records are only valid where a zero gradient is an identity update (Adagrad, l2 = 0)"""
    M, N, K = 256, 128, 64
    A, Bm, state = _operands(_lib.DT_F16, M, N, K, seed=3)
    rec = torch.from_numpy(live_records(np.ones(M, bool))).cuda()
    with pytest.raises(_lib.OcfError, match="row_live"):
        _run(_lib.DT_F16, M, N, K, OPTS[opt](1e-3), A, Bm, state, shadow_blocked=0, extra=dict(row_live=rec))


@pytest.mark.gpu
@pytest.mark.parametrize("cd", ["float16", "bfloat16"])
def test_engine_row_skip_bit_identical(gpu, cd):
    """Generator training steps with and without row skipping (Engine.row_skip): identical weights,
    Adagrad slots and weight shadows after several steps on a wide, sparse dataset where most
    columns of a batch hold no rating."""
    from omnidirectional_collaborative_filtering_amd import optimizers as O
    from omnidirectional_collaborative_filtering_amd.data_reader import data_reader
    from omnidirectional_collaborative_filtering_amd.dataset import split_ratings, synthetic_ratings
    from omnidirectional_collaborative_filtering_amd.model import omni_model
    rows, cols, nnz, B = 900, 4000, 30000, 128
    r, c, v = synthetic_ratings(rows, cols, nnz, half_stars=True, seed=3)
    data = split_ratings(r, c, v, rows, cols, rng=np.random.RandomState(3))
    out = []
    for skip in (False, True):
        np.random.seed(5)
        rd = data_reader(cols, rows, dataset=data, eval_mode="fixed_split")
        om = om_ = omni_model(1, 200, cols, B, dense_activation="sigmoid", use_causal_info=False,
                              compute_dtype=cd, seed=4)
        eng = om.engine
        eng.row_skip = "always" if skip else False
        m = om.model
        m.compile(O.Adagrad(lr=0.01, epsilon=1e-8), "mean_squared_error", metrics=["mae"])
        gen = rd.data_gen(B, [1.0, 1.0], "train", True, None, -1, pass_through_input_training=True)
        m.fit_generator(gen, 5, epochs=1, verbose=0)
        assert eng._rtag_live == skip
        torch.cuda.synchronize()
        out.append([t.clone() for t in eng.W] + [t.clone() for t in eng.b] +
                   [s for sw, sb in eng.slots for s in sw + sb if s is not None] + [t.clone() for t in eng.Wsh])
        del om_
    for a, b in zip(*out):
        assert torch.equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("cd", ["float32", "float16"])
def test_engine_fused_encoder_epilogue_bit_identical(gpu, chunked_encdec, cd):
    """The hidden layer's bias / sigmoid / dropout applied inside the decoder gather (Engine.fuse_enc_epilogue)
    against the separate row-reduce launch: identical losses, weights, slots, shadows and test SSE."""
    from omnidirectional_collaborative_filtering_amd import optimizers as O
    from omnidirectional_collaborative_filtering_amd.data_reader import data_reader
    from omnidirectional_collaborative_filtering_amd.dataset import split_ratings, synthetic_ratings
    from omnidirectional_collaborative_filtering_amd.model import omni_model
    rows, cols, nnz, B = 900, 4000, 60000, 128
    r, c, v = synthetic_ratings(rows, cols, nnz, half_stars=True, seed=8)
    data = split_ratings(r, c, v, rows, cols, rng=np.random.RandomState(8))
    out = []
    for fuse in (False, True):
        np.random.seed(6)
        rd = data_reader(cols, rows, dataset=data, eval_mode="fixed_split")
        om = om_ = omni_model(1, 200, cols, B, dense_activation="sigmoid", use_causal_info=False,
                              dropout_probability=0.2, compute_dtype=cd, seed=4)
        eng = om.engine
        eng.fuse_enc_epilogue = fuse
        m = om.model
        m.compile(O.Adagrad(lr=0.01, epsilon=1e-8), "mean_squared_error", metrics=["mae"])
        gen = rd.data_gen(B, [1.0, 1.0], "train", True, None, -1, pass_through_input_training=True)
        loss = m.fit_generator(gen, 5, epochs=1, verbose=0).history["loss"][0]
        np.random.seed(9)
        tg = rd.data_gen(B, None, "test", True, None, -1, return_target_count=True)
        sse, cnt = m.evaluate_sse(tg, rd.test_set_size // B)
        torch.cuda.synchronize()
        out.append(([loss, sse, cnt], [t.clone() for t in eng.W] + [t.clone() for t in eng.b] +
                    [s for sw, sb in eng.slots for s in sw + sb if s is not None] +
                    [t.clone() for t in eng.Wsh if t is not None]))
        del om_
    assert out[0][0] == out[1][0]
    for a, b in zip(out[0][1], out[1][1]):
        assert torch.equal(a, b)
