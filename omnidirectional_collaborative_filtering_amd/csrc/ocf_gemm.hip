// ocf_gemm: dispatch of the MFMA GEMM template to the layout / dtype / epilogue combinations the
// autoencoder step uses ("GEMM inventory").
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "ocf_epilogues.h"
#include "ocf_internal.h"
#include "ocf_optim_ws.h"
#include "ocf_rows.h"

using namespace ocf;

namespace {

template <typename CT, bool ACOL, bool BCOL, typename BGT, class Epi, bool SPA = false>
void launch(const OcfGemmArgs& g, const typename Epi::Params& ep, hipStream_t s) {
  using Cfg = GemmCfg<CT, ACOL, BCOL, CT, BGT>;
  constexpr int LDS = std::max(Cfg::OPER_LDS, Epi::LDS_NEED);
  static_assert(LDS <= 160 * 1024, "LDS budget");
  GemmShape sh;
  sh.A = g.A; sh.B = g.B; sh.lda = g.lda; sh.ldb = g.ldb;
  sh.M = g.M; sh.N = g.N; sh.K = g.K; sh.order = g.order;
  sh.a_nt = g.a_nt != 0; sh.b_nt = g.b_nt != 0;
  sh.b_blk = g.b_blocked != 0;
  if (sh.b_blk)
    OCF_CHECK(sizeof(BGT) == 2 && g.ldb % 64 == 0, "ocf_gemm: blocked B needs a 16-bit compute-dtype B and ldb % 64 == 0");
  const int splits = std::max(1, g.splits);
  const int ksteps = g.K / Cfg::BK;
  const int per = (ksteps + splits - 1) / splits;
  sh.kchunk = per * Cfg::BK;
  const int ntile = (g.M / GT_BM) * (g.N / GT_BN);
  sh.sp_colsum = nullptr;
  if constexpr (ACOL) {          // column sums of A (output-bias gradient), dense or sparse A
    sh.sp_colsum = g.sp_colsum;
    sh.colsum_scale = g.opt.gscale;
  }
  if constexpr (SPA) {
    sh.sp_rows = g.sp_rows; sh.sp_rp = g.sp_rp; sh.sp_tptr = g.sp_tptr; sh.sp_col = g.sp_col;
    sh.sp_lidx = g.sp_lidx; sh.sp_lboff = g.sp_lboff; sh.sp_vals = g.sp_vals;
    sh.sp_ntiles = g.sp_ntiles; sh.sp_krows = g.sp_krows;
  }
  hipLaunchKernelGGL((gemm_kernel<CT, ACOL, BCOL, CT, BGT, Epi, LDS, SPA>), dim3(ntile, splits), dim3(GT_THREADS), 0, s,
                     sh, ep);
  OCF_HIP(hipGetLastError());
}

// tuning switches (ocf_set_tuning; no environment variables).
// The role split pays off while the MFMA role's K-loop fits under the stream of a tile: at K = 256
// (ML-20M, one GPU) 238-251 us vs 290-316 us for the generic kernel; at K = 2,048 (8-way feature
// parallel global batch) the K-loop dominates and the generic kernel's two workgroups per CU win
// (dW 132 / 111 us vs 175 / 137 us).
int g_optim_ws = 1;      // role-split kernel for dense-A EPI_OPTIM (ocf_set_tuning "optim_ws")
int g_optim_ws_max_k = 512;   // K = 512 (2-way feature parallel): 0.453 vs 0.509 ms/step on the generic kernel; K = 1,024: 0.42 vs 0.38
bool optim_ws_on() { return g_optim_ws != 0; }


// the folded jobs as separate launches (generic kernel path): before / after the GEMM
void jobs_before(const OcfGemmArgs& g, hipStream_t s) {
  if (g.jr) OCF_CHECK(ocf_rows_reduce(g.jr, s) == 0, ocf_last_error());
  if (g.jb_part)
    OCF_CHECK(ocf_bias_opt_from_partials(g.jb_p, g.jb_part, g.jb_parts, g.jb_ld, g.jb_n, g.jb_s1, g.jb_s2, nullptr,
                                         &g.jb_op, s) == 0, ocf_last_error());
  if (g.js_sp)
    OCF_CHECK(ocf_stats_finalize(g.js_sp, g.js_nparts, g.js_rs, g.js_ntiles, g.js_M, g.js_out, s) == 0,
              ocf_last_error());
}
void jobs_after(const OcfGemmArgs& g, hipStream_t s) {
  if (g.cb_p)
    OCF_CHECK(ocf_bias_opt_from_partials(g.cb_p, g.sp_colsum, 1, g.M, g.M, g.cb_s1, g.cb_s2, nullptr, &g.cb_op, s) == 0,
              ocf_last_error());
}

// EPI_OPTIM on [K][M] x [K][N] operands (the dW GEMMs) through the persistent role-split kernel
template <typename CT, bool SPA>
void launch_ws(const OcfGemmArgs& g, const EpiOptim::Params& ep, hipStream_t s) {
  OCF_CHECK(g.s1 != nullptr, "ocf_gemm OPTIM: optimizer slot s1 required");
  GemmShape sh{};
  sh.A = g.A; sh.B = g.B; sh.lda = g.lda; sh.ldb = g.ldb;
  sh.M = g.M; sh.N = g.N; sh.K = g.K; sh.kchunk = g.K;
  sh.b_blk = g.b_blocked != 0;
  sh.sp_colsum = g.sp_colsum;
  sh.colsum_scale = g.opt.gscale;
  if constexpr (SPA) {
    sh.sp_rows = g.sp_rows; sh.sp_rp = g.sp_rp; sh.sp_tptr = g.sp_tptr; sh.sp_col = g.sp_col;
    sh.sp_lidx = g.sp_lidx; sh.sp_lboff = g.sp_lboff; sh.sp_vals = g.sp_vals;
    sh.sp_ntiles = g.sp_ntiles; sh.sp_krows = g.sp_krows;
    sh.sp_bptr = g.sp_bptr; sh.sp_ent = reinterpret_cast<const int2*>(g.sp_ent);
  }
  const int T = (g.M / GT_BM) * (g.N / GT_BN);
  const int cus = (cu_count() + 7) / 8 * 8;
  const int G = std::min(cus, (T + 7) / 8 * 8);   // one workgroup per CU (LDS), multiple of 8 (XCDs)
  const WsJobs jb = ws_jobs(g);
  switch (g.opt.kind) {
    case OCF_OPT_ADAGRAD:
      hipLaunchKernelGGL((optim_ws_kernel<CT, SPA, OCF_OPT_ADAGRAD>), dim3(G), dim3(WS_THREADS), 0, s, sh, ep, jb);
      break;
    case OCF_OPT_RMSPROP:
      hipLaunchKernelGGL((optim_ws_kernel<CT, SPA, OCF_OPT_RMSPROP>), dim3(G), dim3(WS_THREADS), 0, s, sh, ep, jb);
      break;
    default:
      OCF_CHECK(g.opt.kind == OCF_OPT_ADAM && g.s2, "optim_ws: Adagrad, RMSprop or Adam (with both slots)");
      hipLaunchKernelGGL((optim_ws_kernel<CT, SPA, OCF_OPT_ADAM>), dim3(G), dim3(WS_THREADS), 0, s, sh, ep, jb);
  }
  OCF_HIP(hipGetLastError());
}

BiasActParams bias_act_params(const OcfGemmArgs& g) {
  BiasActParams p;
  p.bias = g.bias; p.act = g.act; p.keep = g.keep; p.seed = g.seed; p.stream = g.stream;
  p.mask_in = g.mask_in; p.mask_out = g.mask_out; p.a_out = g.a_out; p.h_out = g.h_out; p.h_dtype = g.h_dtype;
  p.ld = g.ld_out; p.m_real = g.m_real; p.n_real = g.n_real;
  return p;
}

// WGT = element type the weight operand B is stored in: fp32 master weights (converted while
// staging) or a compute-dtype shadow copy of them (SLAB / MASKED_MSE, half the bytes)
template <typename CT, bool ACOL, bool BCOL, typename WGT>
void dispatch_epi(const OcfGemmArgs& g, hipStream_t s) {
  constexpr bool A_ROW = !ACOL;
  constexpr bool FP32_W = std::is_same<WGT, float>::value;
  constexpr bool ALL = FP32_W || std::is_same<CT, float>::value;   // every weight epilogue instantiated
  switch (g.epi) {
    case OCF_EPI_SLAB: {
      EpiSlab::Params p{g.out, g.ld_out, g.split_stride};
      launch<CT, ACOL, BCOL, WGT, EpiSlab>(g, p, s);
      return;
    }
    case OCF_EPI_BIAS_ACT:
      if constexpr (ALL && A_ROW && BCOL) {
        launch<CT, ACOL, BCOL, WGT, EpiBiasAct>(g, bias_act_params(g), s);
        return;
      }
      break;
    case OCF_EPI_PREDICT:
      if constexpr (ALL && A_ROW) {
        EpiPredict::Params p{g.bias, g.pmask, g.ld_pmask, g.out, g.ld_out, g.m_real, g.n_real};
        launch<CT, ACOL, BCOL, WGT, EpiPredict>(g, p, s);
        return;
      }
      break;
    case OCF_EPI_MASKED_MSE:
      if constexpr (A_ROW) {
        EpiMaskedMSE::Params p;
        p.bias = g.bias; p.bk_ptr = g.bk_ptr; p.bk_rc = g.bk_rc; p.bk_t = g.bk_t; p.bk_m = g.bk_m;
        p.d_out = g.h_out; p.d_dtype = g.h_dtype; p.ld_d = g.ld_out; p.db_part = g.db_part; p.ld_db = g.ld_db;
        p.gscale = g.opt.gscale; p.stats_part = g.stats_part; p.row_sse_part = g.row_sse_part;
        p.t_rows = g.t_rows; p.t_rp = g.t_rp; p.t_tptr = g.t_tptr; p.t_col = g.t_col; p.t_val = g.t_val;
        p.t_lidx = g.t_lidx; p.t_flag = g.t_flag; p.t_lboff = g.t_lboff; p.t_ntiles = g.t_ntiles; p.t_aux = g.t_aux;
        p.m_real = g.m_real;
        p.dn_t = g.dn_t; p.dn_m = g.dn_m; p.ld_dn = g.ld_dn; p.dn_rows = g.dn_rows; p.n_real = g.n_real;
        OCF_CHECK(!g.dn_t || (g.dn_m && g.ld_dn >= g.n_real && g.n_real <= g.N),
                  "ocf_gemm MASKED_MSE: dense targets need dn_m, ld_dn >= n_real, n_real <= N");
        OCF_CHECK(g.stats_part, "ocf_gemm MASKED_MSE: stats_part required");
        OCF_CHECK(!g.db_part || g.h_out, "ocf_gemm MASKED_MSE: db_part needs the delta output (h_out)");
        OCF_CHECK((int64_t)g.M * g.ld_out * 4 < (int64_t(1) << 31), "ocf_gemm MASKED_MSE: delta block over 2 GiB");
        OCF_CHECK(g.dn_t || g.bk_ptr || (g.t_rows && g.t_rp && g.t_tptr && g.t_col && g.t_val && g.t_lidx && g.t_flag &&
                               g.t_lboff && g.t_ntiles * GT_BN >= g.N),
                  "ocf_gemm MASKED_MSE: bucket or row-segment targets required");
        launch<CT, ACOL, BCOL, WGT, EpiMaskedMSE>(g, p, s);
        return;
      }
      break;
    case OCF_EPI_GRAD_ACT:
      if constexpr (ALL && A_ROW && !BCOL) {
        GradActParams p;
        p.a = g.a_in; p.mask = g.mask_in; p.keep = g.keep; p.act = g.act; p.d_out = g.h_out; p.d_dtype = g.h_dtype;
        p.ld = g.ld_out; p.db_part = g.db_part; p.gscale = g.opt.gscale; p.m_real = g.m_real; p.n_real = g.n_real;
        OCF_CHECK(g.a_in && g.h_out, "ocf_gemm GRAD_ACT: a_in / h_out required");
        launch<CT, ACOL, BCOL, WGT, EpiGradAct>(g, p, s);
        return;
      }
      break;
    case OCF_EPI_OPTIM:
      if constexpr (!FP32_W || std::is_same<CT, float>::value) if constexpr (BCOL) {
        EpiOptim::Params p{g.p, g.s1, g.s2, g.ld_out, g.opt, g.p_shadow, g.compute_dtype, g.shadow_blocked != 0};
        OCF_CHECK(g.p != nullptr, "ocf_gemm OPTIM: p required");
        OCF_CHECK((int64_t)g.M * g.ld_out * 4 < (int64_t(1) << 31), "ocf_gemm OPTIM: parameter block over 2 GiB");
        OCF_CHECK(!g.p_shadow || g.compute_dtype != OCF_F32, "ocf_gemm OPTIM: shadow weights need f16/bf16 compute");
        OCF_CHECK(!g.shadow_blocked || g.ld_out % 64 == 0, "ocf_gemm OPTIM: blocked shadow needs ld_out % 64 == 0");
        OCF_CHECK(!g.row_live || (g.opt.kind == OCF_OPT_ADAGRAD && g.opt.l2 == 0.f),
                  "ocf_gemm OPTIM: row_live records need Adagrad with l2 == 0 (zero gradient = identity update)");
        p.row_live = g.row_live;   // used by the role-split kernel; the generic kernel updates every row
        if constexpr (ACOL) {
          // row lists of a sparse batch operand: one wave per weight row, no MFMA over the zeros
          if (g.a_sparse && g.sp_rowptr && g.sp_rowent && g.sp_vals && g_optim_rows && launch_rows<CT>(g, p, s)) return;
          if constexpr (sizeof(CT) == 2) {
            // role-split kernel for a dense A (16-bit, slots present -- SGD stays generic --, row-major B);
            // a sparse A goes to the row-stream kernel above or, without row lists, the generic kernel
            const bool ws_kind = g.opt.kind == OCF_OPT_ADAGRAD || g.opt.kind == OCF_OPT_RMSPROP ||
                                 (g.opt.kind == OCF_OPT_ADAM && g.s2);
            if (optim_ws_on() && g.K <= g_optim_ws_max_k && ws_kind && g.s1 && !g.b_blocked && !g.a_sparse) {
              launch_ws<CT, false>(g, p, s);
              return;
            }
          }
          jobs_before(g, s);
          if (g.a_sparse) launch<CT, ACOL, BCOL, CT, EpiOptim, true>(g, p, s);
          else launch<CT, ACOL, BCOL, CT, EpiOptim>(g, p, s);
          jobs_after(g, s);
          return;
        }
        launch<CT, ACOL, BCOL, CT, EpiOptim>(g, p, s);
        return;
      }
      break;
    case OCF_EPI_GRAD:
      if constexpr (!FP32_W || std::is_same<CT, float>::value) if constexpr (BCOL) {
        OCF_CHECK(g.h_dtype == OCF_F32 || g.h_dtype == OCF_BF16, "ocf_gemm GRAD: fp32 or bf16 gradient output");
        EpiGradStore::Params p{g.out, g.ld_out, g.opt.gscale, g.h_dtype == OCF_BF16 ? 1 : 0};
        if constexpr (ACOL) {
          if (g.a_sparse) {
            launch<CT, ACOL, BCOL, CT, EpiGradStore, true>(g, p, s);
            return;
          }
        }
        launch<CT, ACOL, BCOL, CT, EpiGradStore>(g, p, s);
        return;
      }
      break;
    default:
      break;
  }
  throw std::runtime_error("ocf_gemm: epilogue " + std::to_string(g.epi) + " not instantiated for layout a_col=" +
                           std::to_string(ACOL) + " b_col=" + std::to_string(BCOL) + " b_dtype=" +
                           std::to_string(g.b_dtype));
}

template <typename CT, bool ACOL, bool BCOL>
void dispatch_layout(const OcfGemmArgs& g, hipStream_t s) {
  // weight epilogues: B = fp32 master weights or their compute-dtype shadow; OPTIM/GRAD: B is an
  // activation in the compute dtype
  const bool weight_b = g.epi == OCF_EPI_SLAB || g.epi == OCF_EPI_BIAS_ACT || g.epi == OCF_EPI_PREDICT ||
                        g.epi == OCF_EPI_MASKED_MSE || g.epi == OCF_EPI_GRAD_ACT;
  if (weight_b && g.b_dtype == OCF_F32) return dispatch_epi<CT, ACOL, BCOL, float>(g, s);
  OCF_CHECK(g.b_dtype == g.compute_dtype, weight_b ? "ocf_gemm: weight B must be fp32 or the compute dtype"
                                                   : "ocf_gemm: OPTIM/GRAD take B in the compute dtype");
  dispatch_epi<CT, ACOL, BCOL, CT>(g, s);
}


template <typename CT>
void dispatch(const OcfGemmArgs& g, hipStream_t s) {
  if (!g.a_col && g.b_col) dispatch_layout<CT, false, true>(g, s);
  else if (!g.a_col && !g.b_col) dispatch_layout<CT, false, false>(g, s);
  else if (g.a_col && g.b_col) dispatch_layout<CT, true, true>(g, s);
  else throw std::runtime_error("ocf_gemm: layout A[K][M] x B[N][K] not instantiated");
}

}  // namespace

extern "C" int ocf_set_tuning(const char* key, int value, int* previous) {
  OCF_TRY_BEGIN
  const std::string k = key ? key : "";
  if (k == "optim_rows") {
    if (previous) *previous = g_optim_rows;
    g_optim_rows = value ? 1 : 0;
  } else if (k == "rows_long") {
    if (previous) *previous = g_rows_long;
    g_rows_long = value < 0 ? -1 : (value ? 1 : 0);
  } else if (k == "rows_dual") {          // ocf_gemm_pair on small weights: dual-row launch (1) or two (0)
    if (previous) *previous = g_rows_dual;
    g_rows_dual = value ? 1 : 0;
  } else if (k == "rows_dual_parts") {    // dual-row launch parts per tile: 0 by size, 16 or 32
    if (previous) *previous = g_rows_dual_parts;
    OCF_CHECK(value >= 0 && value <= 64, "ocf_set_tuning: rows_dual_parts 0 (by size) or 1..64");
    g_rows_dual_parts = value;
  } else if (k == "rows_dual_pf") {       // dual-row launch: next row issued ahead (-1 by parts, 0, 1)
    if (previous) *previous = g_rows_dual_pf;
    g_rows_dual_pf = value < 0 ? -1 : value ? 1 : 0;
  } else if (k == "rows_dual_large") {    // the dual-row launch on large weights too (1) or the pair launch (0)
    if (previous) *previous = g_rows_dual_large;
    g_rows_dual_large = value ? 1 : 0;
  } else if (k == "rows_dual_count") {    // read (previous) and reset the dual-row launch count
    if (previous) *previous = g_rows_dual_count;
    g_rows_dual_count = 0;
  } else if (k == "rows_small_waves") {
    if (previous) *previous = g_rows_small_waves;
    g_rows_small_waves = value;
  } else if (k == "optim_ws") {
    if (previous) *previous = optim_ws_on() ? 1 : 0;
    g_optim_ws = value ? 1 : 0;
  } else if (k == "pair_wait_polls") {    // ocf_gemm_pair's bounded hand-off wait (tests shorten it)
    if (previous) *previous = g_pair_wait_polls;
    OCF_CHECK(value > 0, "ocf_set_tuning: pair_wait_polls > 0");
    g_pair_wait_polls = value;
  } else if (k == "encdec_max_polls") {   // ocf_gather_encdec's bounded wait (tests: < 0 injects a give-up)
    if (previous) *previous = g_encdec_max_polls;
    OCF_CHECK(value != 0, "ocf_set_tuning: encdec_max_polls != 0");
    g_encdec_max_polls = value;
  } else if (k == "encdec_rowres") {      // ocf_gather_encdec: one workgroup per batch row (< 0: only report)
    if (previous) *previous = g_encdec_rowres;
    if (value >= 0) g_encdec_rowres = value ? 1 : 0;
  } else if (k == "mlp_max_polls") {      // ocf_mlp_step's bounded barrier wait (tests: < 0 injects a give-up)
    if (previous) *previous = g_mlp_max_polls;
    OCF_CHECK(value != 0, "ocf_set_tuning: mlp_max_polls != 0");
    g_mlp_max_polls = value;
  } else if (k == "enc_tiles_pack") {     // ocf_encoder_tiles: packed pre-pass (1) or per-row entry chain (0)
    if (previous) *previous = g_enc_tiles_pack;
    g_enc_tiles_pack = value ? 1 : 0;
  } else if (k == "optim_ws_max_k") {
    if (previous) *previous = g_optim_ws_max_k;
    g_optim_ws_max_k = value;
  } else {
    throw std::runtime_error("ocf_set_tuning: unknown key '" + k + "'");
  }
  OCF_TRY_END
}

namespace {
void check_gemm(const OcfGemmArgs& g) {
  OCF_CHECK((g.A || g.a_sparse) && g.B, "ocf_gemm: null operand");
  OCF_CHECK(g.M > 0 && g.N > 0 && g.K > 0, "ocf_gemm: empty shape");
  OCF_CHECK(g.M % GT_BM == 0 && g.N % GT_BN == 0, "ocf_gemm: M and N must be multiples of 128");
  const int bk = g.compute_dtype == OCF_F32 ? 32 : 64;
  OCF_CHECK(g.K % bk == 0, "ocf_gemm: K must be a multiple of 64 (f16/bf16) or 32 (f32)");
  OCF_CHECK(g.a_dtype == g.compute_dtype, "ocf_gemm: A must be in the compute dtype");
  OCF_CHECK(g.lda % 8 == 0 && g.ldb % 8 == 0, "ocf_gemm: leading dimensions must be multiples of 8");
  OCF_CHECK(g.splits >= 1, "ocf_gemm: splits >= 1");
  OCF_CHECK(g.splits == 1 || g.epi == OCF_EPI_SLAB, "ocf_gemm: split-K only with the SLAB epilogue");
  if (g.a_sparse) {
    OCF_CHECK(g.a_col && (g.epi == OCF_EPI_OPTIM || g.epi == OCF_EPI_GRAD),
              "ocf_gemm: sparse A only for OPTIM / GRAD with a_col = 1");
    OCF_CHECK(g.sp_rows && g.sp_rp && g.sp_tptr && g.sp_col && g.sp_lidx && g.sp_lboff && g.sp_vals &&
                  g.sp_ntiles * GT_BM >= g.M && g.sp_krows <= g.K,
              "ocf_gemm: sparse A descriptor incomplete");
  }
  OCF_CHECK(!(g.cb_p || g.jb_part || g.js_sp) || (g.epi == OCF_EPI_OPTIM && g.a_col),
            "ocf_gemm: folded jobs only with OPTIM on [K][M] A");
  OCF_CHECK(!g.cb_p || g.sp_colsum, "ocf_gemm: cb_p needs sp_colsum");
  OCF_CHECK(!g.jb_part || g.jb_p, "ocf_gemm: jb_part needs jb_p");
  OCF_CHECK(!g.js_sp || g.js_out, "ocf_gemm: js_sp needs js_out");
}

}  // namespace

extern "C" int ocf_gemm(const OcfGemmArgs* args, void* stream) {
  OCF_TRY_BEGIN
  const OcfGemmArgs& g = *args;
  check_gemm(g);
  hipStream_t s = (hipStream_t)stream;
  switch (g.compute_dtype) {
    case OCF_F16: dispatch<_Float16>(g, s); break;
    case OCF_BF16: dispatch<__bf16>(g, s); break;
    case OCF_F32: dispatch<float>(g, s); break;
    default: throw std::runtime_error("ocf_gemm: bad compute dtype");
  }
  OCF_TRY_END
}

extern "C" int ocf_gemm_pair(const OcfGemmArgs* a, const OcfGemmArgs* b, OcfPairSync* sync, void* stream) {
  OCF_TRY_BEGIN
  OCF_CHECK(a && b, "ocf_gemm_pair: null arguments");
  OCF_CHECK(!sync || sync->word, "ocf_gemm_pair: OcfPairSync without a device word");
  check_gemm(*a);
  check_gemm(*b);
  hipStream_t s = (hipStream_t)stream;
  bool done = false;
  if (sync && a->compute_dtype == b->compute_dtype) {
    switch (a->compute_dtype) {
      case OCF_F16: done = launch_rows_pair<_Float16>(*a, *b, *sync, s); break;
      case OCF_BF16: done = launch_rows_pair<__bf16>(*a, *b, *sync, s); break;
      case OCF_F32: done = launch_rows_pair<float>(*a, *b, *sync, s); break;
      default: break;
    }
  }
  if (!done) {
    OCF_CHECK(ocf_gemm(a, stream) == 0, ocf_last_error());
    OCF_CHECK(ocf_gemm(b, stream) == 0, ocf_last_error());
  }
  OCF_TRY_END
}

// one training step of the row-gather path in one call (ocf.h): the four launches of
// engine.Engine.train_step's folded single-GPU sequence, each through its own entry point (same checks)
extern "C" int ocf_train_step_rows(const OcfRowStepArgs* a, void* stream) {
  OCF_TRY_BEGIN
  OCF_CHECK(a != nullptr, "ocf_train_step_rows: null arguments");
  hipStream_t s = (hipStream_t)stream;
  auto ev = [&](int k) {
    if (a->ev[k]) OCF_HIP(hipEventRecord((hipEvent_t)a->ev[k], s));
  };
  OcfGatherArgs d = a->dec;
  d.jr = a->jr_on == 2 ? &a->jr : nullptr;      // the row reduction in the decoder (d.row_arrive) ...
  ev(0);
  if (!a->enc_arrive) OCF_CHECK(ocf_gather_encoder(&a->enc, stream) == 0, ocf_last_error());
  ev(1);
  ev(2);
  if (a->enc_arrive)                            // the encoder and the decoder as one launch
    OCF_CHECK(ocf_gather_encdec(&a->enc, &d, a->enc_arrive, stream) == 0, ocf_last_error());
  else
    OCF_CHECK(ocf_gather_decoder(&d, stream) == 0, ocf_last_error());
  ev(3);
  OcfGemmArgs o = a->dw_out;
  o.jr = a->jr_on == 1 ? &a->jr : nullptr;      // ... or as jobs of the dW_out launch
  if (a->pair_sync) {          // both updates in one launch (ocf_gemm_pair): events 4 / 7 bracket it
    ev(4);
    OCF_CHECK(ocf_gemm_pair(&o, &a->dw_in, a->pair_sync, stream) == 0, ocf_last_error());
    ev(7);
  } else {
    ev(4);
    OCF_CHECK(ocf_gemm(&o, stream) == 0, ocf_last_error());
    ev(5);
    ev(6);
    OCF_CHECK(ocf_gemm(&a->dw_in, stream) == 0, ocf_last_error());
    ev(7);
  }
  OCF_TRY_END
}
