// Row-stream weight-gradient launches (ocf_rows_dw.h): the single launch and the pair launch of
// ocf_gemm_pair, in their own translation unit (ocf_gemm.hip calls them through ocf_rows.h).
#include <algorithm>

#include "ocf_internal.h"
#include "ocf_rows.h"
#include "ocf_rows_impl.h"

namespace ocf {

// tuning switches (ocf_set_tuning in ocf_gemm.hip)
int g_optim_rows = 1;   // row-list dW kernel when the caller passes row lists (ocf_set_tuning "optim_rows")
int g_rows_long = -1;   // row-stream LONG variant: -1 by entries per row, 0 never, 1 always ("rows_long")
int g_rows_small_waves = 8192;   // row-stream kernel: 32 parts per tile below this many waves at 12 ("rows_small_waves")
int g_rows_dual = 1;   // ocf_gemm_pair on small weights: the dual-row launch ("rows_dual"; 0: two launches)
int g_rows_dual_parts = 0;   // dual-row launch: workgroups per 128-row tile (0: by size, else 1..64, "rows_dual_parts")
int g_rows_dual_pf = -1;   // dual-row launch: next row's chain issued ahead (-1: below 32 parts, 0 / 1: "rows_dual_pf")
int g_rows_dual_large = 1;   // the dual-row launch on large weights too ("rows_dual_large"; 0: the pair launch there)
int g_rows_dual_count = 0;   // dual-row launches since the last read ("rows_dual_count": tests see which form ran)
int g_pair_wait_polls = 1 << 22;   // ocf_gemm_pair's bounded wait (ocf_set_tuning "pair_wait_polls"): seconds


int cu_count() {
  static int n[64] = {0};
  int dev = 0;
  OCF_HIP(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64) dev = 0;
  if (!n[dev]) OCF_HIP(hipDeviceGetAttribute(&n[dev], hipDeviceAttributeMultiprocessorCount, dev));
  return n[dev];
}

WsJobs ws_jobs(const OcfGemmArgs& g) {
  WsJobs j{};
  j.cb_p = g.cb_p; j.cb_s1 = g.cb_s1; j.cb_s2 = g.cb_s2; j.cb_op = g.cb_op;
  j.jb_part = g.jb_part; j.jb_parts = g.jb_parts; j.jb_n = g.jb_n; j.jb_ld = g.jb_ld; j.jb_p = g.jb_p;
  j.jb_s1 = g.jb_s1; j.jb_s2 = g.jb_s2; j.jb_op = g.jb_op;
  j.js_sp = g.js_sp; j.js_rs = g.js_rs; j.js_out = g.js_out; j.js_nparts = g.js_nparts; j.js_ntiles = g.js_ntiles;
  j.js_M = g.js_M;
  if (g.jr) {
    OCF_CHECK(g.jr->mode == OCF_REDUCE_GRAD_ACT && g.jr->part && g.jr->row_cptr && g.jr->h_out && g.jr->a_in &&
                  g.jr->H <= 512,
              "ocf_gemm: the folded row reduction (jr) takes OCF_REDUCE_GRAD_ACT with part, row_cptr, h_out, a_in, "
              "H <= 512");
    j.jr = *g.jr;
    j.jr_on = 1;
  }
  return j;
}


// EPI_OPTIM over a sparse batch operand given as row lists: the row-stream kernel (ocf_rows_dw.h),
// one wave per weight row.  Takes 16-bit or fp32 compute, Adagrad / RMSprop / Adam with their slots, N a
// multiple of 128 up to 512 and a row-major shadow; anything else returns false (the tile kernels).
bool rows_setup(const OcfGemmArgs& g, const EpiOptim::Params& ep, RowsLaunch& L) {
  // a lane's B elements are one 4-, 8- or 16-B load (16-bit or fp32 compute)
  const bool kind_ok = g.opt.kind == OCF_OPT_ADAGRAD || g.opt.kind == OCF_OPT_RMSPROP ||
                       (g.opt.kind == OCF_OPT_ADAM && g.s2);
  if (!(kind_ok && g.s1 && g.N % 128 == 0 && g.N <= 512 && g.ldb >= g.N && g.ld_out == g.N && g.M % 128 == 0))
    return false;
  if (ep.shadow && ep.shadow_blocked) return false;
  RowsDwArgs& ra = L.ra;
  ra = RowsDwArgs{};
  ra.p = g.p; ra.s1 = g.s1; ra.s2 = g.s2; ra.ld = g.ld_out; ra.M = g.M; ra.N = g.N;
  ra.B = g.B; ra.ldb = g.ldb;
  ra.rowptr = g.sp_rowptr; ra.rowent = reinterpret_cast<const int2*>(g.sp_rowent); ra.vals = g.sp_vals;
  ra.live = g.row_live;
  ra.op = g.opt;
  ra.shadow = ep.shadow;
  ra.colsum = g.sp_colsum; ra.colsum_scale = g.opt.gscale;
  L.jb = ws_jobs(g);
  // workgroups per 128-row tile (each a twelfth of the tile's live rows): with the 75-VGPR pipeline
  // (6 waves per SIMD) 12 parts measured best, ML-20M step 0.4243-0.4269 ms against 6 / 8 / 16 / 24 / 32
  // parts 0.439-0.441 / 0.4332-0.4364 / 0.437 / 0.430 / 0.446
  // A weight of few rows (ML-1M: 48 tiles; ML-100K: 8; an 8-way feature rank's 136) leaves the chip
  // mostly idle at 12 parts, each wave walking ~3 rows through the 5-stage pipeline's fill: there a wave
  // takes ~one row (32 parts).  Measured (ms/step, 12 -> 32 parts): ML-1M bf16 0.1225 -> 0.1064, ML-100K
  // fp32 0.0875 -> 0.0794, 8-way emulated rank step 0.2308 -> 0.2178 (ML-20M, 1,082 tiles: 12 parts)
  L.small = g.M / 128 * 12 * 4 < g_rows_small_waves;
  L.parts = L.small ? 32 : 12;
  L.grid = (L.jb.count() + 3) / 4 + g.M / 128 * L.parts;   // job-only workgroups, then the rows
  // many entries per weight row (>= 4 on average): the LONG variant (entries as a vector, B rows of a
  // group of entries in flight together)
  L.lng = g_rows_long < 0 ? g.sp_nent >= 4LL * g.M : g_rows_long != 0;
  L.N = g.N;
  L.kind = g.opt.kind;
  return true;
}

// both weight updates of a step in one row-stream launch (ocf_gemm_pair), when both take the row-stream
// kernel with the same instance
EpiOptim::Params optim_params(const OcfGemmArgs& g) {
  EpiOptim::Params p{g.p, g.s1, g.s2, g.ld_out, g.opt, g.p_shadow, g.compute_dtype, g.shadow_blocked != 0};
  p.row_live = g.row_live;
  return p;
}
bool rows_pair_ok(const OcfGemmArgs& g) {
  return g.epi == OCF_EPI_OPTIM && g.a_col && g.b_col && g.a_sparse && g.sp_rowptr && g.sp_rowent && g.sp_vals &&
         g.p && g.b_dtype == g.compute_dtype && (int64_t)g.M * g.ld_out * 4 < (int64_t(1) << 31) &&
         (!g.p_shadow || g.compute_dtype != OCF_F32) && (!g.row_live || (g.opt.kind == OCF_OPT_ADAGRAD && g.opt.l2 == 0.f));
}

}  // namespace ocf
