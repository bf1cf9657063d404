"""Row-list weight-gradient kernel (ocf_rows_dw.h, OcfGemmArgs sp_rowptr / sp_rowent): the row lists
built by ocf_sparse_tiles against a NumPy restatement, the fused update against a plain PyTorch fp32
reference (g = A^T B from the same entries, Keras' optimizer formulas), rows without entries skipped
only where that is the identity (Adagrad, l2 = 0), the output-bias column sums and their update."""
import ctypes

import numpy as np
import pytest
import torch

from omnidirectional_collaborative_filtering_amd import _lib
from omnidirectional_collaborative_filtering_amd.engine import cur_stream
from tests.test_optim_ws_gpu import OPTS, _buckets, _sparse_batch


def _row_lists(sp, M, K):
    rptr = torch.full((M + 1,), -5, dtype=torch.int32, device="cuda")
    cap = max(1, int(sp["sp_lboff"][-1].item()) + 4 * M)
    rent = torch.full((cap, 2), -9, dtype=torch.int32, device="cuda")
    bptr, ent = _buckets(sp, M, K, extra=dict(row_ptr=rptr, row_ent=rent))
    return bptr, ent, rptr, rent


def _dense_entries(sp, M):
    """per column m: [(value index, k)] in k order (NumPy restatement of the row lists)"""
    h = {k: (v.cpu().numpy() if torch.is_tensor(v) else v) for k, v in sp.items()}
    cols = [[] for _ in range(M)]
    for b in range(h["sp_krows"]):
        r = h["sp_rows"][b]
        if r < 0:
            continue
        for e in range(h["sp_rp"][r], h["sp_rp"][r + 1]):
            cols[h["sp_col"][e]].append((h["sp_lboff"][b] + h["sp_lidx"][e], b))
    return cols


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(256, 64, 40), (1280, 256, 256), (512, 320, 300), (640, 2048, 900)])
def test_row_lists_match_numpy(gpu, shape):
    M, K, krows = shape
    sp, _ = _sparse_batch(M, K, krows, seed=K + 3)
    _, _, rptr, rent = _row_lists(sp, M, K)
    cols = _dense_entries(sp, M)
    want_ptr = np.concatenate([[0], np.cumsum([len(c) for c in cols])])
    got_ptr = rptr.cpu().numpy().astype(np.int64)
    np.testing.assert_array_equal(got_ptr - got_ptr[0], want_ptr)
    ent = rent.cpu().numpy()
    for m in range(M):
        got = [tuple(x) for x in ent[got_ptr[m]:got_ptr[m + 1]]]
        assert got == cols[m], m


def _run_rows(cd, M, N, K, opt, Bm, state, sp, rows=True, colsum=False, jobs=None):
    P, S1, S2 = (t.clone() for t in state)
    sdt = {_lib.DT_F16: torch.float16, _lib.DT_BF16: torch.bfloat16}.get(cd)
    Sh = P.to(sdt) if sdt is not None else None
    cs = torch.full((M,), -7.0, device="cuda") if colsum else None
    a = _lib.OcfGemmArgs()
    a.compute_dtype = cd
    a.A, a.a_dtype, a.a_col, a.lda = Bm.data_ptr(), cd, 1, M
    a.B, a.b_dtype, a.b_col, a.ldb = Bm.data_ptr(), cd, 1, N
    a.M, a.N, a.K, a.splits, a.epi = M, N, K, 1, _lib.EPI_OPTIM
    a.p, a.ld_out, a.s1 = P.data_ptr(), N, S1.data_ptr()
    a.s2 = S2.data_ptr() if opt.kind == _lib.OPT_ADAM else None
    a.opt = opt
    if Sh is not None:
        a.p_shadow, a.shadow_blocked = Sh.data_ptr(), 0
    if cs is not None:
        a.sp_colsum = cs.data_ptr()
    a.a_sparse = 1
    for k, v in sp.items():
        if not rows and k in ("sp_rowptr", "sp_rowent"):
            continue
        setattr(a, k, v.data_ptr() if torch.is_tensor(v) else v)
    for k, v in (jobs or {}).items():
        setattr(a, k, v.data_ptr() if torch.is_tensor(v) else v)
    _lib.call("ocf_gemm", a, cur_stream())
    torch.cuda.synchronize()
    return P, S1, S2, Sh, cs


def _torch_update(opt, g, p, s1, s2):
    g = g.double()
    p, s1, s2 = p.double(), s1.double(), s2.double()
    if opt.l2:
        g = g + 2.0 * opt.l2 * p
    if opt.kind == _lib.OPT_ADAGRAD:
        s1 = s1 + g * g
        p = p - opt.lr * g / (s1.sqrt() + opt.eps)
    elif opt.kind == _lib.OPT_RMSPROP:
        s1 = opt.rho * s1 + (1 - opt.rho) * g * g
        p = p - opt.lr * g / (s1.sqrt() + opt.eps)
    else:
        s1 = opt.rho * s1 + (1 - opt.rho) * g
        s2 = opt.beta2 * s2 + (1 - opt.beta2) * g * g
        p = p - opt.lr * s1 / (s2.sqrt() + opt.eps)
    return p.float(), s1.float(), s2.float()


@pytest.mark.gpu
@pytest.mark.parametrize("cd", [_lib.DT_F16, _lib.DT_BF16, _lib.DT_F32])
@pytest.mark.parametrize("opt_name", ["adagrad", "rmsprop", "adam", "adagrad_l2"])
@pytest.mark.parametrize("shape", [(1280, 512, 256, 256), (768, 256, 2048, 900), (384, 128, 64, 40)])
def test_rows_kernel_vs_torch(gpu, cd, opt_name, shape):
    M, N, K, krows = shape
    sp, dense = _sparse_batch(M, K, krows, seed=M + K, col_frac=0.6)
    bptr, ent, rptr, rent = _row_lists(sp, M, K)
    spr = dict(sp, sp_bptr=bptr, sp_ent=ent, sp_rowptr=rptr, sp_rowent=rent)
    g = torch.Generator().manual_seed(K)
    td = {_lib.DT_F16: torch.float16, _lib.DT_BF16: torch.bfloat16, _lib.DT_F32: torch.float32}[cd]
    Bm = torch.randn(K, N, generator=g).to(td).cuda()
    state = ((torch.randn(M, N, generator=g) * 0.05).cuda(), torch.rand(M, N, generator=g).cuda(),
             torch.rand(M, N, generator=g).cuda())
    gscale = 3e-3
    opt = OPTS[opt_name](gscale)
    P, S1, S2, Sh, cs = _run_rows(cd, M, N, K, opt, Bm, state, spr, colsum=True)
    # reference: the same entries (fp32 values, B as stored) in fp64
    A = torch.from_numpy(dense).double().cuda()
    grad = (A.t() @ Bm.double()) * gscale
    rp, r1, r2 = _torch_update(opt, grad, *state)
    torch.testing.assert_close(P, rp, rtol=1e-5, atol=2e-6)
    torch.testing.assert_close(S1, r1, rtol=1e-5, atol=2e-6)
    if opt.kind == _lib.OPT_ADAM:
        torch.testing.assert_close(S2, r2, rtol=1e-5, atol=2e-6)
    if Sh is not None:
        assert torch.equal(Sh, P.to(Sh.dtype))        # shadow = the updated weights, rounded once
    torch.testing.assert_close(cs.double(), A.sum(0) * gscale, rtol=1e-5, atol=1e-7)
    empty = torch.from_numpy(~(dense != 0).any(0)).cuda()
    if opt_name == "adagrad":                          # identity on rows without entries: untouched
        assert torch.equal(P[empty], state[0][empty]) and torch.equal(S1[empty], state[1][empty])
    elif opt_name == "rmsprop":                        # a decays even with g = 0: every row updated
        assert not torch.equal(S1[empty], state[1][empty])


@pytest.mark.gpu
def test_rows_kernel_matches_mfma_kernels_and_bias_job(gpu):
    """same update as the role-split MFMA kernel up to the operand rounding (f16 A values there), and
    the folded output-bias update (cb_*) equals ocf_bias_opt_from_partials on the column sums"""
    M, N, K, krows = 1280, 512, 256, 256
    cd = _lib.DT_F16
    sp, dense = _sparse_batch(M, K, krows, seed=11, col_frac=0.6)
    bptr, ent, rptr, rent = _row_lists(sp, M, K)
    spr = dict(sp, sp_bptr=bptr, sp_ent=ent, sp_rowptr=rptr, sp_rowent=rent)
    g = torch.Generator().manual_seed(1)
    Bm = torch.randn(K, N, generator=g).half().cuda()
    state = ((torch.randn(M, N, generator=g) * 0.05).cuda(), torch.rand(M, N, generator=g).cuda(),
             torch.rand(M, N, generator=g).cuda())
    opt = OPTS["adagrad"](2e-3)
    bias = torch.randn(M, generator=g).cuda()
    bacc = torch.rand(M, generator=g).cuda()
    b1, a1 = bias.clone(), bacc.clone()
    rows = _run_rows(cd, M, N, K, opt, Bm, state, spr, colsum=True,
                     jobs=dict(cb_p=b1, cb_s1=a1, cb_op=OPTS["adagrad"](1.0)))
    ws = _run_rows(cd, M, N, K, opt, Bm, state, spr, rows=False, colsum=True)
    torch.testing.assert_close(rows[0], ws[0], rtol=0, atol=2e-5)
    b2, a2 = bias.clone(), bacc.clone()
    o = OPTS["adagrad"](1.0)
    _lib.call("ocf_bias_opt_from_partials", b2.data_ptr(), rows[4].data_ptr(), 1, M, M, a2.data_ptr(), None, None, o,
              cur_stream())
    torch.cuda.synchronize()
    assert torch.equal(b1, b2) and torch.equal(a1, a2)


@pytest.mark.gpu
def _skewed_entries(rng, ncols, B):
    """unique (batch row, column) pairs, column popularity ~ rank^-1 (lists from 1 to all B rows), in
    flat (batch row, column) order"""
    k = np.minimum(B, (B * 1.3 / np.arange(1, ncols + 1)).astype(np.int64) + 1)
    c = np.repeat(rng.permutation(ncols), k)
    b = np.concatenate([rng.choice(B, int(x), replace=False) for x in k])
    o = np.lexsort((c, b))
    return b[o], c[o]


@pytest.mark.gpu
@pytest.mark.parametrize("ncols,E,B", [(256, 3000, 256), (6144, 69000, 256), (1024, 40000, 2048),
                                       (138496, 191000, 256), (2048, 0, 4096), (1024, 0, 1000)])
def test_ocf_row_lists_match_numpy(gpu, ncols, E, B):
    """ocf_row_lists (the row lists from the scatter's per-column counts and keys): per column, the
    batch entries in entry order (= batch-row order), row_ptr the exclusive scan of the counts, the
    counts left zeroed and the cursor scratch left zeroed; the live records as ocf_sparse_tiles'.
    E = 0: skewed columns (lists up to every batch row: the long-list LDS sort, twice to check its
    queue is reset)"""
    rng = np.random.RandomState(ncols + E)
    if E:
        b = np.sort(rng.randint(0, B, E))                   # entries in batch-row order (flat order)
        c = rng.randint(0, ncols, E)
    else:
        b, c = _skewed_entries(rng, ncols, B)
        E = len(b)
        assert np.bincount(c).max() == B
    ecb = torch.as_tensor((c | (b << 19)).astype(np.int32), device="cuda")
    cnt = torch.as_tensor(np.bincount(c, minlength=ncols).astype(np.int32), device="cuda")
    cur = torch.zeros(3 * ncols + 256, dtype=torch.int32, device="cuda")
    rptr = torch.full((ncols + 1,), -3, dtype=torch.int32, device="cuda")
    rent = torch.full((E, 2), -9, dtype=torch.int32, device="cuda")
    tag = 7
    tags = np.zeros(ncols, np.uint8)
    tags[np.unique(c)] = tag
    tags_d = torch.as_tensor(tags, device="cuda")
    rec = torch.zeros(ncols // 128 * _lib.LIVE_REC, dtype=torch.uint8, device="cuda")
    a = _lib.OcfRowListArgs()
    a.ecb, a.E, a.col_cnt, a.cursor, a.n_cols = ecb.data_ptr(), E, cnt.data_ptr(), cur.data_ptr(), ncols
    a.row_ptr, a.row_ent = rptr.data_ptr(), rent.data_ptr()
    a.rtag_in, a.rtag_out, a.rtag, a.live_in, a.live_out = tags_d.data_ptr(), tags_d.data_ptr(), tag, rec.data_ptr(), None
    for rep in range(2):
        if rep:
            cnt.copy_(torch.as_tensor(np.bincount(c, minlength=ncols).astype(np.int32)))
            rent.fill_(-9)
        _lib.call("ocf_row_lists", a, cur_stream())
    torch.cuda.synchronize()
    want_ptr = np.concatenate([[0], np.cumsum(np.bincount(c, minlength=ncols))])
    np.testing.assert_array_equal(rptr.cpu().numpy(), want_ptr)
    ent = rent.cpu().numpy()
    order = np.argsort(c, kind="stable")                   # per column, entry order
    np.testing.assert_array_equal(ent[:, 0], order)
    np.testing.assert_array_equal(ent[:, 1], b[order])
    assert not cnt.any() and not cur[:ncols].any()
    r = rec.cpu().numpy().reshape(-1, _lib.LIVE_REC)
    for t in range(ncols // 128):
        live = np.nonzero(tags[t * 128:(t + 1) * 128] == tag)[0]
        L = int(r[t, :4].view(np.int32)[0])
        assert L == len(live)
        got = [r[t, 16 + (k % 8) * 16 + k // 8] for k in range(L)]
        np.testing.assert_array_equal(got, live)


def _gen_for(rows, cols, nnz, B, skew, seed, sparsity=(1.0, 1.0), pass_through=True, rng="numpy"):
    from omnidirectional_collaborative_filtering_amd.data_reader import data_reader
    from omnidirectional_collaborative_filtering_amd.dataset import split_ratings, synthetic_ratings
    r, c, v = synthetic_ratings(rows, cols, nnz, half_stars=True, seed=seed, skew=skew)
    data = split_ratings(r, c, v, rows, cols, rng=np.random.RandomState(seed))
    np.random.seed(seed)
    rd = data_reader(cols, rows, dataset=data, eval_mode="fixed_split", rng=rng)
    return rd, rd.data_gen(B, list(sparsity), "train", True, None, -1, pass_through_input_training=pass_through)


@pytest.mark.gpu
@pytest.mark.parametrize("rows,cols,nnz,B,skew,sel", [
    (900, 4000, 30000, 128, 0.0, None),          # every batch of the epoch, short lists
    (900, 4000, 30000, 128, 0.0, [2, 3, 4]),     # consecutive batches past 0: windows of the epoch tables (ebase0)
    (1682, 943, 100000, 256, 0.5, None),         # ML-100K-like: ~16 per list, sorted across lanes (16 / 32 / 64)
    (3000, 1024, 400000, 512, 1.0, [1, 0, 3]),   # a subset, out of order; lists up to ~500 (LDS bitonic)
    (5000, 1024, 1500000, 2048, 1.0, None),      # lists over 1,024 entries (long-list queue)
    # wider than one 4,096-column scan block (the two-pass block scan, the row-group prefix across blocks): the
    # whole epoch (7 batches) and a window of three, eight row groups per batch, skewed
    (2000, 20000, 240000, 256, 0.5, None),
    (2000, 20000, 240000, 256, 1.0, [1, 2, 3]),
])
def test_epoch_row_lists_match_numpy(gpu, rows, cols, nnz, B, skew, sel):
    """ocf_epoch_row_lists (BatchGenerator.prepare_row_lists): per selected batch and column, the batch's
    entries in entry (= batch-row) order, row_ptr the exclusive scan of the column counts, the live
    records = the columns holding an entry; a second build into the same tables agrees"""
    rd, gen = _gen_for(rows, cols, nnz, B, skew, seed=rows + B)
    gen._start()
    Np = (cols + 127) // 128 * 128
    for rep in range(2):
        gen.prepare_row_lists(Np, sel)
        torch.cuda.synchronize()
        rl = gen._rl
        csr = gen.src1.host
        longest = 0
        for bi in (sel if sel is not None else range(gen.num_batches)):
            s = rl["slot"][bi]
            rws = gen.rows_host[bi]
            lens = np.diff(csr.row_ptr)[rws]
            lb = np.concatenate([[0], np.cumsum(lens)])
            e = np.arange(lb[-1])
            b = np.repeat(np.arange(B), lens)
            c = csr.col[np.concatenate([np.arange(csr.row_ptr[r], csr.row_ptr[r + 1]) for r in rws])]
            cnt = np.bincount(c, minlength=Np)
            longest = max(longest, cnt.max())
            rp = rl["row_ptr"][s * (Np + 1):(s + 1) * (Np + 1)].cpu().numpy()
            np.testing.assert_array_equal(rp, np.concatenate([[0], np.cumsum(cnt)]))
            e0 = int(rl["ebase_host"][s])
            ent = rl["row_ent"].view(-1, 2)[e0:e0 + len(e)].cpu().numpy()
            o = np.argsort(c, kind="stable")
            np.testing.assert_array_equal(ent[:, 0], e[o])
            np.testing.assert_array_equal(ent[:, 1], b[o])
            rec = rl["live"].view(-1, Np // 128, _lib.LIVE_REC)[s].cpu().numpy()
            for t in range(Np // 128):
                live = np.nonzero(cnt[t * 128:(t + 1) * 128])[0]
                L = int(rec[t, :4].view(np.int32)[0])
                assert L == len(live)
                np.testing.assert_array_equal([rec[t, 16 + (k % 8) * 16 + k // 8] for k in range(L)], live)
    if B == 2048:
        assert longest > 1024
    elif B == 512:
        assert longest > 32


@pytest.mark.gpu
@pytest.mark.parametrize("cd,sparsity,pt,shape", [
    ("float16", (1.0, 1.0), True, (900, 4000, 40000, 128, 0.5)),
    ("bfloat16", (0.5, 0.9), False, (900, 4000, 40000, 128, 0.5)),
    ("float32", (1.0, 1.0), True, (900, 4000, 40000, 128, 0.5)),
    # popular columns in most of 2,048 batch rows: lists sorted by the LDS bitonic and the long-list queue
    ("float16", (1.0, 1.0), True, (5000, 1024, 1500000, 2048, 1.0)),
])
def test_engine_epoch_lists_bit_identical(gpu, cd, sparsity, pt, shape):
    """Generator training with the epoch row lists (and their structural live records) against the per-step
    ocf_row_lists (and the scatter's row tags): identical weights, slots and shadows -- also under input
    corruption, where the epoch records add columns whose every input was dropped (an identity update),
    and with lists longer than 1,024 entries."""
    from omnidirectional_collaborative_filtering_amd import optimizers as O
    from omnidirectional_collaborative_filtering_amd.model import omni_model
    rows, cols, nnz, B, skew = shape
    out = []
    for epoch in (False, True):
        rd, gen = _gen_for(rows, cols, nnz, B, skew, seed=11, sparsity=sparsity, pass_through=pt)
        om = om_ = omni_model(1, 200, cols, B, dense_activation="sigmoid", use_causal_info=False,
                              dropout_probability=0.2, compute_dtype=cd, seed=4)
        eng = om.engine
        eng.epoch_row_lists = epoch
        eng.row_skip = "always"         # (the epoch records even for dense batches: the superset rows)
        m = om.model
        m.compile(O.Adagrad(lr=0.01, epsilon=1e-8), "mean_squared_error", metrics=["mae"])
        loss = m.fit_generator(gen, min(5, gen.num_batches), epochs=1, verbose=0).history["loss"][0]
        assert eng._rtag_live and (getattr(gen, "_rl", None) is not None) == epoch
        torch.cuda.synchronize()
        out.append(([loss], [t.clone() for t in eng.W] + [t.clone() for t in eng.b] +
                    [s for sw, sb in eng.slots for s in sw + sb if s is not None] +
                    [t.clone() for t in eng.Wsh if t is not None]))
        del om_
    assert out[0][0] == out[1][0]
    for a, b in zip(out[0][1], out[1][1]):
        assert torch.equal(a, b)


@pytest.mark.gpu
def test_rows_job_only_workgroups_stay_in_bounds(gpu):
    """A small weight (M = 128: 8 row workgroups) with more folded jobs than those hold (the step's stats
    over 512 rows: 513 jobs -> 129 workgroups): the workgroups past the last tile run only their jobs --
    no live record read past the table (here the next table's valid record), no colsum zeroing past M,
    no parameter row past M."""
    M, N, K, krows = 128, 128, 256, 200
    sp, _ = _sparse_batch(M, K, krows, seed=21)
    _, _, rptr, rent = _row_lists(sp, M, K)
    rng = np.random.RandomState(3)
    state = [torch.as_tensor(rng.uniform(-0.1, 0.1, (M + 256) * N).astype(np.float32), device="cuda"),
             torch.as_tensor(rng.uniform(0.1, 1.0, (M + 256) * N).astype(np.float32), device="cuda"),
             torch.zeros((M + 256) * N, device="cuda")]
    Bm = torch.as_tensor(rng.uniform(-1, 1, (K, N)), device="cuda").to(torch.float16)
    # two tiles of records: ours, then a neighbour's with every row live
    rec = torch.zeros(2 * _lib.LIVE_REC, dtype=torch.uint8, device="cuda")
    live = torch.nonzero(rptr[1:M + 1] > rptr[:M]).flatten().cpu().numpy()
    r = np.zeros((2, _lib.LIVE_REC), np.uint8)
    for t, rows in ((0, live), (1, np.arange(128))):
        r[t, :4] = np.array([len(rows)], np.int32).view(np.uint8)
        for k, m in enumerate(rows):
            r[t, 16 + (k % 8) * 16 + k // 8] = m
    rec.copy_(torch.as_tensor(r.reshape(-1)))
    js_M = 512
    cs_guard = torch.full((M + 1024,), -7.0, device="cuda")
    jobs = dict(js_sp=torch.zeros(8 * 4, device="cuda"), js_nparts=8, js_rs=torch.zeros(2 * js_M, device="cuda"),
                js_ntiles=2, js_M=js_M, js_out=torch.zeros(4 + js_M, device="cuda"))
    spr = dict(sp, sp_rowptr=rptr, sp_rowent=rent)
    spr["row_live"] = rec
    P0 = [t.clone() for t in state]
    a = _lib.OcfGemmArgs()
    cd = _lib.DT_F16
    a.compute_dtype = cd
    a.A, a.a_dtype, a.a_col, a.lda = Bm.data_ptr(), cd, 1, M
    a.B, a.b_dtype, a.b_col, a.ldb = Bm.data_ptr(), cd, 1, N
    a.M, a.N, a.K, a.splits, a.epi = M, N, K, 1, _lib.EPI_OPTIM
    a.p, a.ld_out, a.s1 = state[0].data_ptr(), N, state[1].data_ptr()
    a.opt = OPTS["adagrad"](1.0)
    a.sp_colsum = cs_guard.data_ptr()
    a.a_sparse = 1
    for k, v in list(spr.items()) + list(jobs.items()):
        setattr(a, k, v.data_ptr() if torch.is_tensor(v) else v)
    _lib.call("ocf_gemm", a, cur_stream())
    torch.cuda.synchronize()
    assert torch.equal(cs_guard[M:], torch.full((1024,), -7.0, device="cuda"))
    assert torch.equal(state[0][M * N:], P0[0][M * N:]) and torch.equal(state[1][M * N:], P0[1][M * N:])
    assert not torch.equal(state[0][:M * N], P0[0][:M * N])


@pytest.mark.gpu
@pytest.mark.parametrize("cd,B", [("float16", 128), ("float32", 128), ("bfloat16", 100)])
def test_engine_fold_reduce_bit_identical(gpu, chunked_encdec, cd, B):
    """The decoder's δh row reduction as jobs of the dW_out launch (Engine.fold_reduce; the hidden-bias and
    stats jobs then ride in dW_in), or in the decoder launch by each row's last chunk (reduce_in_decoder:
    write-through partials and a per-row arrival counter; B = 100 leaves 28 padding rows for its zero-row
    pass), against its own ocf_rows_reduce launch: identical losses, weights, slots, shadows and per-step
    stats; the arrival counters are back at zero after every launch."""
    from omnidirectional_collaborative_filtering_amd import optimizers as O
    from omnidirectional_collaborative_filtering_amd.model import omni_model
    out = []
    for fold, in_dec in ((False, False), (True, False), (True, True)):
        rd, gen = _gen_for(900, 4000, 60000, B, 0.5, seed=8)
        om = om_ = omni_model(1, 200, 4000, B, dense_activation="sigmoid", use_causal_info=False,
                              dropout_probability=0.2, compute_dtype=cd, seed=4)
        eng = om.engine
        eng.fold_reduce = fold
        eng.reduce_in_decoder = in_dec
        m = om.model
        m.compile(O.Adagrad(lr=0.01, epsilon=1e-8), "mean_squared_error", metrics=["mae"])
        h = m.fit_generator(gen, 5, epochs=1, verbose=0).history
        torch.cuda.synchronize()
        assert eng._dec_reduced == in_dec and int(eng.row_arrive.abs().sum()) == 0
        out.append(([h[k][0] for k in sorted(h)], [t.clone() for t in eng.W] + [t.clone() for t in eng.b] +
                    [s for sw, sb in eng.slots for s in sw + sb if s is not None] +
                    [t.clone() for t in eng.Wsh if t is not None]))
        del om_
    for o in out[1:]:
        assert out[0][0] == o[0]
        for a, b in zip(out[0][1], o[1]):
            assert torch.equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("rng", ["numpy", "device"])
@pytest.mark.parametrize("sparsity,pt", [((1.0, 1.0), True), ((0.5, 0.9), False), ((0.3, 0.6), True)])
@pytest.mark.parametrize("sel", [[3, 0, 5], [2, 3, 4]])
def test_epoch_scatter_matches_per_batch(gpu, rng, sparsity, pt, sel):
    """ocf_epoch_scatter (every batch of the plan in one launch, BatchGenerator.prepare_row_lists) writes the
    same per-entry live input values and live-target flags as ocf_scatter_batch batch by batch (reciprocal
    split from the host NumPy draws or the device Philox stream of each batch, pass-through or not); a
    selection out of order (staged sel / ebase) and a window of consecutive batches (the epoch's tables, ebase0)"""
    rd, gen = _gen_for(900, 4000, 40000, 128, 0.5, seed=17, sparsity=sparsity, pass_through=pt, rng=rng)
    gen._start()
    gen.prepare_row_lists(4096, sel)
    torch.cuda.synchronize()
    rl = gen._rl
    for bi in sel:
        E = int(gen.nnz1[bi])
        xv = torch.full((E,), -3.0, device="cuda")
        tf = torch.full((E,), 7, dtype=torch.uint8, device="cuda")
        a = gen.scatter_args(bi)
        a.xval1, a.tflag1, a.B_pad = xv.data_ptr(), tf.data_ptr(), gen.B
        _lib.call("ocf_scatter_batch", a, cur_stream())
        torch.cuda.synchronize()
        e0 = int(rl["ebase_host"][rl["slot"][bi]])
        assert torch.equal(rl["xval"][e0:e0 + E], xv)
        assert torch.equal(rl["tflag"][e0:e0 + E], tf)
        if sparsity[0] < 1:
            assert 0 < int((xv == 0).sum()) < E            # the split dropped some inputs and kept others


@pytest.mark.gpu
@pytest.mark.parametrize("opt", ["adagrad", "rmsprop", "adam"])
@pytest.mark.parametrize("cd,shape", [
    ("float16", (900, 4000, 40000, 128, 0.5)),        # ~1.4 entries per weight row
    ("bfloat16", (3706, 6040, 1000209, 256, 0.0)),    # ML-1M I-AutoRec: ~11 per row
    ("float32", (3706, 6040, 1000209, 256, 0.0)),
    ("float16", (5000, 1024, 1500000, 2048, 1.0)),    # rows over 64 and over 1,024 entries
])
def test_rows_long_variant_bit_identical(gpu, cd, shape, opt):
    """The row-stream kernel's LONG variant (a row's entries loaded as one vector, the B rows of 8 entries in
    flight together; chosen by the library at >= 4 entries per weight row, ocf_set_tuning "rows_long")
    against the scalar-chain variant: identical losses, weights, slots and shadows (same per-element
    summation order), for every optimizer and compute dtype, short and long lists"""
    from omnidirectional_collaborative_filtering_amd import optimizers as O
    from omnidirectional_collaborative_filtering_amd.model import omni_model
    rows, cols, nnz, B, skew = shape
    mk = {"adagrad": lambda: O.Adagrad(lr=0.01, epsilon=1e-8), "rmsprop": lambda: O.RMSprop(lr=0.001),
          "adam": lambda: O.Adam(lr=0.001)}[opt]
    out = []
    prev = ctypes.c_int(0)
    try:
        for long_on in (0, 1):
            _lib.call("ocf_set_tuning", b"rows_long", long_on, ctypes.byref(prev))
            rd, gen = _gen_for(rows, cols, nnz, B, skew, seed=13)
            om = om_ = omni_model(1, 500 if cd != "float32" else 200, cols, B, dense_activation="sigmoid",
                                  use_causal_info=False, dropout_probability=0.2, compute_dtype=cd, seed=4)
            eng = om.engine
            m = om.model
            m.compile(mk(), "mean_squared_error", metrics=["mae"])
            h = m.fit_generator(gen, min(4, gen.num_batches), epochs=1, verbose=0).history
            assert eng.tb is not None and "sp_rowptr" in eng.tb
            torch.cuda.synchronize()
            out.append(([h[k][0] for k in sorted(h)], [t.clone() for t in eng.W] + [t.clone() for t in eng.b] +
                        [s for sw, sb in eng.slots for s in sw + sb if s is not None] +
                        [t.clone() for t in eng.Wsh if t is not None]))
            del om_
    finally:
        _lib.call("ocf_set_tuning", b"rows_long", -1, None)
    assert out[0][0] == out[1][0]
    for a, b in zip(out[0][1], out[1][1]):
        assert torch.equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("opt", ["adagrad", "rmsprop", "adam"])
@pytest.mark.parametrize("cd,shape,skip", [
    ("float16", (900, 4000, 40000, 128, 0.5), "always"),   # ~1.4 entries per weight row, live records
    ("bfloat16", (3706, 6040, 1000209, 256, 0.0), True),    # ML-1M I-AutoRec: ~11 per row
    ("float32", (1682, 943, 100000, 256, 0.0), True),       # ML-100K I-AutoRec: ~16 per row
    ("float16", (5000, 1024, 1500000, 2048, 1.0), True),    # rows over 64 and over 1,024 entries
])
def test_rows_dual_bit_identical(gpu, cd, shape, skip, opt):
    """ocf_gemm_pair's dual-row form on small weights (one chain per column for both layers' rows, the row
    reduction riding in its first workgroups; ocf_set_tuning "rows_dual") against the two row-stream
    launches: identical losses, weights, slots and shadows for every optimizer and compute dtype, and the
    dual launch really ran (one per step)"""
    from omnidirectional_collaborative_filtering_amd import optimizers as O
    from omnidirectional_collaborative_filtering_amd.model import omni_model
    rows, cols, nnz, B, skew = shape
    mk = {"adagrad": lambda: O.Adagrad(lr=0.01, epsilon=1e-8), "rmsprop": lambda: O.RMSprop(lr=0.001),
          "adam": lambda: O.Adam(lr=0.001)}[opt]
    out = []
    prev = ctypes.c_int(0)
    n = 0
    try:
        for dual in (0, 1):
            _lib.call("ocf_set_tuning", b"rows_dual", dual, ctypes.byref(prev))
            _lib.call("ocf_set_tuning", b"rows_dual_count", 0, None)
            rd, gen = _gen_for(rows, cols, nnz, B, skew, seed=13)
            om = om_ = omni_model(1, 500 if cd != "float32" else 200, cols, B, dense_activation="sigmoid",
                                  use_causal_info=False, dropout_probability=0.2, compute_dtype=cd, seed=4)
            eng = om.engine
            eng.row_skip = skip
            m = om.model
            m.compile(mk(), "mean_squared_error", metrics=["mae"])
            n = min(4, gen.num_batches)
            h = m.fit_generator(gen, n, epochs=1, verbose=0).history
            torch.cuda.synchronize()
            cnt = ctypes.c_int(-1)
            _lib.call("ocf_set_tuning", b"rows_dual_count", 0, ctypes.byref(cnt))
            assert cnt.value == (n if dual else 0), (dual, cnt.value)
            out.append(([h[k][0] for k in sorted(h)], [t.clone() for t in eng.W] + [t.clone() for t in eng.b] +
                        [s for sw, sb in eng.slots for s in sw + sb if s is not None] +
                        [t.clone() for t in eng.Wsh if t is not None]))
            del om_
    finally:
        _lib.call("ocf_set_tuning", b"rows_dual", 1, None)
    assert out[0][0] == out[1][0]
    for a, b in zip(out[0][1], out[1][1]):
        assert torch.equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("cd,opt,skip,H", [("float16", "adagrad", True, 500), ("bfloat16", "adam", False, 500),
                                           ("float32", "rmsprop", False, 200), ("float16", "adagrad", True, 512)])
def test_rows_dual_large_bit_identical(gpu, chunked_encdec, cd, opt, skip, H):
    """The dual-row form on LARGE weights (235 row tiles: above the small-weight gate; ocf_set_tuning
    "rows_dual_large", the row reduction in the decoder) against the pair launch and against two launches:
    identical losses, weights, slots and shadows, and the dual launch really ran once per step"""
    from omnidirectional_collaborative_filtering_amd import optimizers as O
    from omnidirectional_collaborative_filtering_amd.model import omni_model
    mk = {"adagrad": lambda: O.Adagrad(lr=0.01, epsilon=1e-8), "rmsprop": lambda: O.RMSprop(lr=0.001),
          "adam": lambda: O.Adam(lr=0.001)}[opt]
    out = []
    try:
        for large, in_dec in ((0, False), (0, True), (1, True)):
            _lib.call("ocf_set_tuning", b"rows_dual_large", large, None)
            _lib.call("ocf_set_tuning", b"rows_dual_count", 0, None)
            rd, gen = _gen_for(2000, 30000, 300000, 256, 0.5, seed=21)
            om = om_ = omni_model(1, H, 30000, 256, dense_activation="sigmoid",
                                  use_causal_info=False, dropout_probability=0.2, compute_dtype=cd, seed=4)
            eng = om.engine
            eng.row_skip = skip
            eng.reduce_in_decoder = in_dec
            m = om.model
            m.compile(mk(), "mean_squared_error", metrics=["mae"])
            n = min(4, gen.num_batches)
            h = m.fit_generator(gen, n, epochs=1, verbose=0).history
            torch.cuda.synchronize()
            cnt = ctypes.c_int(-1)
            _lib.call("ocf_set_tuning", b"rows_dual_count", 0, ctypes.byref(cnt))
            assert cnt.value == (n if large else 0), (large, cnt.value)
            assert eng._dec_reduced == in_dec
            out.append(([h[k][0] for k in sorted(h)], [t.clone() for t in eng.W] + [t.clone() for t in eng.b] +
                        [s for sw, sb in eng.slots for s in sw + sb if s is not None] +
                        [t.clone() for t in eng.Wsh if t is not None]))
            del om_
    finally:
        _lib.call("ocf_set_tuning", b"rows_dual_large", 1, None)
    for o in out[1:]:
        assert out[0][0] == o[0]
        for a, b in zip(out[0][1], o[1]):
            assert torch.equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("cd,shape,B", [("float16", (2000, 30000, 300000, 0.5), 256),   # large weights: dual-row
                                        ("bfloat16", (3706, 6040, 1000209, 0.0), 256),  # ML-1M: rows of 3+ chunks
                                        ("float32", (1682, 943, 100000, 0.0), 100)])    # padding rows
def test_encdec_launch_bit_identical(gpu, cd, shape, B):
    """the encoder and the decoder as ONE launch (ocf_gather_encdec: a decoder chunk starts when its row's
    encoder chunks have counted themselves) against the two launches: identical losses, weights, slots,
    shadows and history over a few steps; the per-row counters are back at zero after every launch"""
    from omnidirectional_collaborative_filtering_amd import optimizers as O
    from omnidirectional_collaborative_filtering_amd.model import omni_model
    rows, cols, nnz, skew = shape
    out = []
    prev = _rowres(0)                      # (the chunked form: the row-resident one sums in another order)
    for fused in (False, True):
        rd, gen = _gen_for(rows, cols, nnz, B, skew, seed=5)
        om = om_ = omni_model(1, 500 if cd != "float32" else 200, cols, B, dense_activation="sigmoid",
                              use_causal_info=False, dropout_probability=0.2, compute_dtype=cd, seed=4)
        eng = om.engine
        eng.fuse_enc_dec = fused
        m = om.model
        m.compile(O.Adagrad(lr=0.01, epsilon=1e-8), "mean_squared_error", metrics=["mae"])
        h = m.fit_generator(gen, min(5, gen.num_batches), epochs=1, verbose=0).history
        torch.cuda.synchronize()
        assert int(eng.enc_arrive.abs().sum()) == 0 and int(eng.row_arrive.abs().sum()) == 0
        out.append(([h[k][0] for k in sorted(h)], [t.clone() for t in eng.W] + [t.clone() for t in eng.b] +
                    [s for sw, sb in eng.slots for s in sw + sb if s is not None] +
                    [t.clone() for t in eng.Wsh if t is not None]))
        del om_
    _rowres(prev)
    assert out[0][0] == out[1][0]
    for a, b in zip(out[0][1], out[1][1]):
        assert torch.equal(a, b)


@pytest.mark.gpu
def test_encdec_gives_up_safely(gpu):
    """A decoder chunk of the fused encoder -> decoder launch that gives up waiting (injected on batch row 0:
    ocf_set_tuning "encdec_max_polls" < 0) still counts itself, so both per-row counters are back at zero after
    the launch; it closes the hand-off gate, so the dual-row update that follows writes no weight, bias, slot or
    shadow; the error is reported once; and the next step equals a twin model's step on the same batch from the
    same state (exact: Adagrad, no dropout)"""
    from omnidirectional_collaborative_filtering_amd import optimizers as O
    from omnidirectional_collaborative_filtering_amd.model import omni_model
    lib = _lib.load()
    prev_rr = _rowres(0)                   # (the chunked form's hand-off: the row-resident form has no wait)
    try:
        _gives_up_safely(lib, O, omni_model)
    finally:
        _rowres(prev_rr)


def _gives_up_safely(lib, O, omni_model):
    def build():
        rd, gen = _gen_for(2000, 30000, 300000, 256, 0.5, seed=21)
        om = omni_model(1, 500, 30000, 256, dense_activation="sigmoid", use_causal_info=False,
                        dropout_probability=None, compute_dtype="float16", seed=4)
        om.model.compile(O.Adagrad(lr=0.01, epsilon=1e-8), "mean_squared_error", metrics=["mae"])
        om.model.fit_generator(gen, 3, epochs=1, verbose=0)
        return om, gen

    def state(eng):
        return [t.clone() for t in eng.W + eng.b + [s for sw, sb in eng.slots for s in sw + sb if s is not None]
                + [w for w in eng.Wsh if w is not None]]

    a, ga = build()
    ea = a.engine
    torch.cuda.synchronize()
    s0 = state(ea)
    prev = ctypes.c_int32()
    _lib.call("ocf_set_tuning", b"encdec_max_polls", -1, ctypes.byref(prev))
    try:
        lib.ocf_set_tuning(b"rows_dual_count", 0, None)
        a.model._train_one(ga)
        torch.cuda.synchronize()
        assert ea.step_paths["one_call"] > 0
        # the counters, before any other library call (no host-side reset has run)
        assert int(ea.enc_arrive.abs().sum()) == 0 and int(ea.row_arrive.abs().sum()) == 0
        for x, y in zip(s0, state(ea)):
            assert torch.equal(x, y)
        # (every entry point reports a pending error first, so this is the first library call after the step)
        assert lib.ocf_check_async() != 0 and b"ocf_gather_encdec" in lib.ocf_last_error()
        assert lib.ocf_check_async() == 0          # reported once
        cnt = ctypes.c_int(-1)
        _lib.call("ocf_set_tuning", b"rows_dual_count", 0, ctypes.byref(cnt))
        assert cnt.value == 1, "the dual-row launch (which found the gate closed) did not run"
    finally:
        lib.ocf_set_tuning(b"encdec_max_polls", prev.value, None)
    # the next step: against a twin that trained the same 3 batches and skips the one the failed step took
    b, gb = build()
    assert gb.next_batch_index() is not None
    a.model._train_one(ga)
    b.model._train_one(gb)
    torch.cuda.synchronize()
    _lib.call("ocf_check_async")                   # (raises if that step gave up)
    sa, sb = state(ea), state(b.engine)
    assert not torch.equal(sa[0], s0[0])
    for x, y in zip(sa, sb):
        assert torch.equal(x, y)
    assert int(ea.enc_arrive.abs().sum()) == 0 and int(ea.row_arrive.abs().sum()) == 0


def _rowres(on):
    prev = _lib.ctypes.c_int32()
    _lib.call("ocf_set_tuning", b"encdec_rowres", int(on), _lib.ctypes.byref(prev))
    return prev.value


@pytest.mark.gpu
@pytest.mark.parametrize("cd,shape,B", [("float16", (2000, 30000, 300000, 0.5), 256),   # large weights, skewed rows
                                        ("bfloat16", (3706, 6040, 1000209, 0.0), 256),  # ML-1M: rows of 3+ chunks
                                        ("float16", (2000, 30000, 300000, 0.0), 100)])   # padding rows
def test_encdec_rowres_matches_chunked(gpu, cd, shape, B):
    """ocf_gather_encdec's row-resident form (one 1,024-thread workgroup per batch row; "encdec_rowres") against
    the chunked form on the same first step from the same state.  Only the order of the fp32 sums differs, so:
    the activations within 1e-5; h (rounded to the compute dtype) equal but for rare one-ulp flips; the hidden
    delta within two ulps of its dtype plus 1e-3 (f16) / 1e-2 (bf16) of its scale (a flipped h element moves
    every delta of its row a little); the loss within 1e-5 relative; padding rows zero"""
    from omnidirectional_collaborative_filtering_amd import optimizers as O
    from omnidirectional_collaborative_filtering_amd.model import omni_model
    rows, cols, nnz, skew = shape
    out = []
    prev = _rowres(0)
    try:
        for rr in (0, 1):
            _rowres(rr)
            rd, gen = _gen_for(rows, cols, nnz, B, skew, seed=5)
            om = omni_model(1, 500, cols, B, dense_activation="sigmoid", use_causal_info=False,
                            dropout_probability=0.2, compute_dtype=cd, seed=4)
            eng = om.engine
            eng.fuse_enc_dec = True
            m = om.model
            m.compile(O.Adagrad(lr=0.01, epsilon=1e-8), "mean_squared_error", metrics=["mae"])
            h = m.fit_generator(gen, 1, epochs=1, verbose=0).history
            torch.cuda.synchronize()
            out.append((h["loss"][0], eng.a[0][:, :500].clone(), eng.h[0][:, :500].float().clone(),
                        eng.dh[0][:, :500].float().clone()))
            del om, eng, m
    finally:
        _rowres(prev)
    (l0, a0, h0, d0), (l1, a1, h1, d1) = out
    assert abs(l1 - l0) <= 1e-5 * abs(l0)
    assert float((a1[:B] - a0[:B]).abs().max()) <= 1e-5
    flips = (h1[:B] != h0[:B]).float().mean().item()
    assert flips <= 2e-3, flips
    ulp = 2.0 ** -10 if cd == "float16" else 2.0 ** -7
    tol = 2 * ulp * d0.abs() + (1e-3 if cd == "float16" else 1e-2) * float(d0.abs().max())
    bad = ((d1 - d0).abs() > tol)[:B]
    assert int(bad.sum()) == 0, (int(bad.sum()), float((d1 - d0).abs().max()))
    if B < d1.shape[0]:
        assert float(d1[B:].abs().max()) == 0.0


@pytest.mark.gpu
@pytest.mark.parametrize("cd", ["float16", "bfloat16"])
def test_encdec_rowres_train_parity(gpu, cd):
    """training through the row-resident launch against the oracle (tests/parity.py envelope and quantile bars):
    three Adagrad steps with dropout 0.2 at a large-weight width"""
    from omnidirectional_collaborative_filtering_amd.dataset import split_ratings, synthetic_ratings
    from tests.parity import assert_low_precision, run_parity
    rows, cols, nnz = 1500, 30000, 600000
    r, c, v = synthetic_ratings(rows, cols, nnz, half_stars=True, seed=7)
    data = split_ratings(r, c, v, rows, cols, rng=np.random.RandomState(7))
    prev = _rowres(1)
    try:
        res = run_parity(cd, "adagrad", 1, "sigmoid", steps=3, B=256, H=500, dropout=0.2, data=data, envelope=True,
                         sparse_oracle=True, eval_batches=2,
                         model_hook=lambda om: setattr(om.engine, "fuse_enc_dec", True))
    finally:
        _rowres(prev)
    assert_low_precision(res, 2e-3 if cd == "float16" else 1e-2)
