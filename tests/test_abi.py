"""CPU: libocf.so loads, exports every function include/ocf.h declares, and the ctypes mirrors of the
ABI structs have exactly the C layout (sizes and offsets from gcc on the same header).  No compute
calls (no GPU here)."""
import ctypes
import os
import re
import subprocess
import tempfile

import pytest

from omnidirectional_collaborative_filtering_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "ocf.h")


def declared_functions():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|const char\*)\s+(ocf_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_expected_entry_points():
    fns = declared_functions()
    for must in ("ocf_scatter_batch", "ocf_gemm", "ocf_opt_step", "ocf_splitk_bias_act", "ocf_splitk_grad_act",
                 "ocf_stats_finalize", "ocf_last_error", "ocf_version"):
        assert must in fns
    assert set(fns) == set(_lib.SIGNATURES), set(fns) ^ set(_lib.SIGNATURES)


def test_library_exports_every_symbol():
    lib = _lib.load()
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert lib.ocf_version() >= 1
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    for name in declared_functions():
        assert re.search(r"\bT %s\b" % name, out), name


STRUCTS = {
    "OcfOptParams": (_lib.OcfOptParams, ["kind", "lr", "gscale"]),
    "OcfScatterArgs": (_lib.OcfScatterArgs, ["keep1", "s0", "seed", "mode", "rows2", "aux", "ld", "xin_dtype",
                                             "feed", "tile_cnt", "n_tiles", "pos1", "lboff2", "E2", "tflag2", "xin_clean",
                                             "xval1", "tb_cnt", "tb_nk", "rtag_in", "rtag_out", "rtag", "col_cnt", "ecb"]),
    "OcfGatherArgs": (_lib.OcfGatherArgs, ["rows", "n_chunks", "ldw", "w_blocked", "H", "part", "aux", "delta_e",
                                           "ld_d", "enc_part", "enc_cptr", "bias_h", "act", "keep", "seed",
                                           "stream", "a_out", "mask_out", "m_real", "n_real", "zero_word"]),
    "OcfRowsReduceArgs": (_lib.OcfRowsReduceArgs, ["mode", "out", "keep", "seed", "stream", "n_real", "gscale",
                                                   "row_sse"]),
    "OcfGemmArgs": (_lib.OcfGemmArgs, ["a_col", "lda", "ldb", "epi", "split_stride", "keep", "seed", "h_dtype",
                                       "ld_db", "n_real", "opt", "ld_pmask", "row_sse_part", "t_rows", "t_lboff", "t_ntiles",
                                       "t_aux", "p_shadow", "b_nt", "shadow_blocked", "a_sparse",
                                       "sp_lboff", "sp_krows", "sp_colsum", "sp_bptr", "sp_ent", "cb_op", "jb_part",
                                       "jb_ld", "jb_op", "js_sp", "js_M", "row_live", "sp_rowptr",
                                       "sp_rowent", "jr", "sp_nent", "dn_t", "ld_dn", "dn_rows"]),
    "OcfPairSync": (_lib.OcfPairSync, ["word", "count"]),
    "OcfEncTileArgs": (_lib.OcfEncTileArgs, ["rows", "xval", "ldw", "w_dtype", "B", "splits", "part", "nnz",
                                             "n_entries", "work", "work_bytes", "max_row_len"]),
    "OcfMlpStepArgs": (_lib.OcfMlpStepArgs, ["n_hidden", "Bp", "k_blocks", "hidden", "hidden_p", "x", "ld_x", "rows",
                                             "targets", "ld_t", "W", "b", "sW2", "sb2", "shadow", "shadow_blocked",
                                             "act", "compute_dtype", "opt", "stats", "work", "work_bytes", "barrier",
                                             "wgs", "trace", "keep", "seed", "stream", "mask"]),
    "OcfBiasActArgs": (_lib.OcfBiasActArgs, ["slabs", "splits", "split_stride", "M", "N", "ld", "bias", "act", "keep",
                                             "seed", "stream", "mask_in", "mask_out", "a_out", "h_out", "h_dtype",
                                             "m_real", "n_real"]),
    "OcfGradActArgs": (_lib.OcfGradActArgs, ["slabs", "splits", "split_stride", "M", "N", "ld", "a_in", "mask", "keep",
                                             "act", "d_out", "d_dtype", "db", "gscale", "m_real", "n_real"]),
    "OcfStatsArgs": (_lib.OcfStatsArgs, ["stats_part", "n_parts", "row_sse_part", "n_tiles", "M", "out"]),
    "OcfBiasOptArgs": (_lib.OcfBiasOptArgs, ["b", "db_part", "parts", "ld", "n", "s1", "s2", "g_out", "opt"]),
    "OcfRankStepArgs": (_lib.OcfRankStepArgs, ["enc", "enc_sum", "hidden", "dec", "dec_sum", "stats", "dw_out",
                                               "out_bias", "hidden_grad", "dw_in", "side", "fork", "join", "ev"]),
    "OcfRowStepArgs": (_lib.OcfRowStepArgs, ["enc", "dec", "dw_out", "dw_in", "jr", "jr_on", "ev", "pair_sync"]),
    "OcfTileBucketArgs": (_lib.OcfTileBucketArgs, ["rows", "lboff", "krows", "nk", "cnt", "ent", "cap", "counted",
                                                       "cnt_clear", "rtag_in", "rtag", "live_in", "live_out",
                                                       "row_ptr", "row_ent"]),
    "OcfRowListArgs": (_lib.OcfRowListArgs, ["ecb", "E", "col_cnt", "cursor", "n_cols", "row_ptr", "row_ent", "rtag_in",
                                             "rtag_out", "rtag", "live_in", "live_out"]),
    "OcfEpochRowListArgs": (_lib.OcfEpochRowListArgs, ["n_sel", "B", "n_cols", "rows", "rp", "col", "lboff", "sel",
                                                       "ebase", "cnt", "row_ptr", "row_ent", "live", "n_rg",
                                                       "ebase0", "max_list", "entries"]),
    "OcfEpochScatterArgs": (_lib.OcfEpochScatterArgs, ["n_sel", "sel", "ebase", "max_e", "keep_off", "stream_mul",
                                                       "xval", "tflag", "ebase0"]),
    "OcfModelDesc": (_lib.OcfModelDesc, ["n_hidden", "N", "k_blocks", "hidden", "act", "dropout", "compute_dtype",
                                         "max_batch", "seed", "W", "b"]),
    "OcfOptStepArgs": (_lib.OcfOptStepArgs, ["p", "g", "g_dtype", "s1", "s2", "n", "opt", "shadow", "shadow_dtype"]),
    "OcfRecipKeepArgs": (_lib.OcfRecipKeepArgs, ["key", "pos", "nb", "B", "n_entries", "boff", "ebase", "s0", "s1",
                                                 "keep", "doubles", "workspace", "workspace_bytes"]),
}


def test_struct_layout_matches_c():
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "%s"' % HDR, "int main(void) {"]
    for s, (_, fields) in STRUCTS.items():
        lines.append('printf("%s size %%zu\\n", sizeof(%s));' % (s, s))
        for f in fields:
            lines.append('printf("%s %s %%zu\\n", offsetof(%s, %s));' % (s, f, s, f))
    lines.append("return 0; }")
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "layout.c")
        with open(c, "w") as fh:
            fh.write("\n".join(lines))
        exe = os.path.join(d, "layout")
        subprocess.run(["gcc", "-std=c99", "-o", exe, c], check=True)
        out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout
    got = {}
    for line in out.splitlines():
        s, f, v = line.split()
        got[(s, f)] = int(v)
    for s, (cls, fields) in STRUCTS.items():
        assert ctypes.sizeof(cls) == got[(s, "size")], s
        for f in fields:
            assert getattr(cls, f).offset == got[(s, f)], (s, f)


def test_errors_are_reported_not_silent():
    """A bad call fails loudly with a message (no compute happens: argument validation only)."""
    a = _lib.OcfGemmArgs()
    a.M, a.N, a.K = 100, 128, 64       # M not a multiple of 128
    a.A = a.B = 1
    with pytest.raises(_lib.OcfError, match="multiples of 128"):
        _lib.call("ocf_gemm", a, None)


def test_model_abi_is_plain_c(tmp_path):
    """the model ABI compiles and links from C (gcc, no C++ / HIP headers): what a cgo / JNI / N-API binding
    or a C training loop includes"""
    src = tmp_path / "drive.c"
    src.write_text(r'''
#include "ocf.h"
int drive(float** W, float** b, float** gW, float** gb, const float* x, const float* mo, const float* t,
          float* pred, float* grad, float* stats, float* slots[][2], int64_t* sizes, void* stream) {
  OcfModelDesc d = {0};
  d.n_hidden = 1; d.N = 333; d.k_blocks = 1; d.hidden[0] = 100; d.act = OCF_ACTV_SIGMOID; d.dropout = 0.2f;
  d.compute_dtype = OCF_DT_F16; d.max_batch = 128; d.seed = 1;
  for (int i = 0; i < 2; ++i) { d.W[i] = W[i]; d.b[i] = b[i]; }
  OcfCtx* ctx = 0;
  if (ocf_ctx_create(&d, &ctx)) return 1;
  const float* in[1] = {x};
  OcfOptParams op = {OCF_OPTK_ADAGRAD, 0.005f, 1e-8f, 0.f, 0.f, 0.f, 1.f};
  int rc = ocf_forward(ctx, in, 333, 128, 1, 0, mo, 333, pred, 333, 0, stream)
        || ocf_masked_mse(pred, t, mo, 333, 128, 333, grad, 333, stats, stream)
        || ocf_backward(ctx, grad, 333, 128, 2.f / (128 * 333), gW, gb, stream);
  for (int i = 0; i < 2 && !rc; ++i)
    rc = ocf_opt_step(W[i], gW[i], slots[2 * i][0], 0, sizes[2 * i], &op, stream)
      || ocf_opt_step(b[i], gb[i], slots[2 * i + 1][0], 0, sizes[2 * i + 1], &op, stream);
  ocf_ctx_destroy(ctx);
  return rc;
}
int main(void) { return 0; }
''')
    exe = tmp_path / "drive"
    r = subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), str(src),
                        "-o", str(exe), _lib.LIB_PATH, "-Wl,--unresolved-symbols=ignore-in-shared-libs"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_model_dims_and_descriptor_checks():
    """ocf_model_dims (host-only): the padded Keras-layout shapes, and the descriptor checks the model ABI
    applies before touching the device"""
    d = _lib.OcfModelDesc()
    d.n_hidden, d.N, d.k_blocks = 2, 333, 2
    d.hidden[0], d.hidden[1] = 100, 130
    d.act, d.dropout, d.compute_dtype, d.max_batch = 1, 0.2, 1, 128
    rows, cols = (ctypes.c_int64 * 3)(), (ctypes.c_int64 * 3)()
    _lib.call("ocf_model_dims", d, rows, cols)
    assert list(rows) == [2 * 384, 128, 256] and list(cols) == [128, 256, 384]
    for field, bad in (("n_hidden", 0), ("n_hidden", 9), ("k_blocks", 4), ("dropout", 1.0), ("compute_dtype", 7),
                       ("max_batch", 0), ("act", 9)):
        e = _lib.OcfModelDesc.from_buffer_copy(d)
        setattr(e, field, bad)
        with pytest.raises(_lib.OcfError):
            _lib.call("ocf_model_dims", e, rows, cols)
    # a context needs every parameter pointer
    ctx = ctypes.c_void_p()
    with pytest.raises(_lib.OcfError, match="null parameter"):
        _lib.call("ocf_ctx_create", d, ctypes.byref(ctx))
