// ocf_rank_step (ocf.h): a feature-parallel rank step as one library call per phase between the host's
// collectives.  Every member goes through its own entry point (the same checks as the single calls).
#include "ocf_internal.h"

namespace {
void record(void* ev, hipStream_t s) {
  if (ev) OCF_HIP(hipEventRecord((hipEvent_t)ev, s));
}
// `to` runs after everything issued on `from` so far
void order(void* ev, hipStream_t from, hipStream_t to) {
  OCF_CHECK(ev != nullptr, "ocf_rank_step: side stream without its events");
  OCF_HIP(hipEventRecord((hipEvent_t)ev, from));
  OCF_HIP(hipStreamWaitEvent(to, (hipEvent_t)ev, 0));
}
}  // namespace

extern "C" int ocf_rank_step(const OcfRankStepArgs* a, int phase, void* stream) {
  OCF_TRY_BEGIN
  OCF_CHECK(a != nullptr && phase >= 0 && phase <= 3, "ocf_rank_step: arguments / phase 0..3");
  hipStream_t s = (hipStream_t)stream, side = (hipStream_t)a->side;
  auto ok = [](int rc) { OCF_CHECK(rc == 0, ocf_last_error()); };
  switch (phase) {
    case 0:
      record(a->ev[0], s);
      if (!ocf::rank_rowres_enc(a->enc, a->enc_sum, s)) {     // (the row-resident form: one launch)
        ok(ocf_gather_encoder(&a->enc, stream));
        ok(ocf_rows_reduce(&a->enc_sum, stream));
      }
      record(a->ev[1], s);
      break;
    case 1: {
      record(a->ev[2], s);
      const OcfBiasActArgs& h = a->hidden;
      if (!ocf::rank_rowres_dec(h, a->dec, a->dec_sum, s)) {  // (the row-resident form: one launch)
        ok(ocf_splitk_bias_act(h.slabs, h.splits, h.split_stride, h.M, h.N, h.ld, h.bias, h.act, h.keep, h.seed,
                               h.stream, h.mask_in, h.mask_out, h.a_out, h.h_out, h.h_dtype, h.m_real, h.n_real,
                               stream));
        ok(ocf_gather_decoder(&a->dec, stream));
        ok(ocf_rows_reduce(&a->dec_sum, stream));
      }
      record(a->ev[3], s);
      const OcfStatsArgs& st = a->stats;
      if (side) order(a->fork[0], s, side);
      ok(ocf_stats_finalize(st.stats_part, st.n_parts, st.row_sse_part, st.n_tiles, st.M, st.out,
                            side ? (void*)side : stream));
      break;
    }
    case 2: {
      hipStream_t t = side ? side : s;
      if (side) order(a->fork[1], s, side);
      record(a->ev[4], t);
      ok(ocf_gemm(&a->dw_out, (void*)t));
      const OcfBiasOptArgs& b = a->out_bias;
      if (b.b) ok(ocf_bias_opt_from_partials(b.b, b.db_part, b.parts, b.ld, b.n, b.s1, b.s2, b.g_out, &b.opt, (void*)t));
      record(a->ev[5], t);
      break;
    }
    default: {
      record(a->ev[6], s);
      const OcfGradActArgs& g = a->hidden_grad;
      ok(ocf_splitk_grad_act(g.slabs, g.splits, g.split_stride, g.M, g.N, g.ld, g.a_in, g.mask, g.keep, g.act, g.d_out,
                             g.d_dtype, g.db, g.gscale, g.m_real, g.n_real, stream));
      ok(ocf_gemm(&a->dw_in, stream));
      record(a->ev[7], s);
      if (side) order(a->join, side, s);
    }
  }
  OCF_TRY_END
}
