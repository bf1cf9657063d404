// The row-stream launch templates (ocf_rows.hip's host logic + ocf_rows_dw.h's kernels), instantiated once
// per compute dtype in ocf_rows_f16.hip / ocf_rows_bf16.hip / ocf_rows_f32.hip (the kernel instances take
// minutes to compile: one translation unit per dtype builds them in parallel).
#pragma once
#include <cmath>

#include "ocf_internal.h"
#include "ocf_rows.h"
#include "ocf_rows_dw.h"

namespace ocf {

struct RowsLaunch {
  RowsDwArgs ra;
  WsJobs jb;
  int grid, parts, N;
  bool lng, small;
  int kind;
};

bool rows_setup(const OcfGemmArgs& g, const EpiOptim::Params& ep, RowsLaunch& L);
EpiOptim::Params optim_params(const OcfGemmArgs& g);
bool rows_pair_ok(const OcfGemmArgs& g);

// the kernel instance for (optimizer, N, parts, LONG): f(kernel template tag) launches it
template <typename CT, typename F>
void rows_dispatch(const RowsLaunch& L, F&& f) {
  auto go = [&](auto kind_tag, auto cw_tag, auto nch_tag) {
    constexpr int KIND = decltype(kind_tag)::value, CW = decltype(cw_tag)::value;
    constexpr int NCH = decltype(nch_tag)::value;
    if (L.lng && L.small) f.template go<CT, KIND, CW, NCH, 32, true>();
    else if (L.lng) f.template go<CT, KIND, CW, NCH, 12, true>();
    else if (L.small) f.template go<CT, KIND, CW, NCH, 32, false>();
    else f.template go<CT, KIND, CW, NCH, 12, false>();
  };
  using std::integral_constant;
  auto by_n = [&](auto k) {
    switch (L.N) {
      case 128: go(k, integral_constant<int, 2>{}, integral_constant<int, 1>{}); break;
      case 256: go(k, integral_constant<int, 4>{}, integral_constant<int, 1>{}); break;
      case 384: go(k, integral_constant<int, 2>{}, integral_constant<int, 3>{}); break;
      default: go(k, integral_constant<int, 4>{}, integral_constant<int, 2>{});
    }
  };
  switch (L.kind) {
    case OCF_OPT_ADAGRAD: by_n(integral_constant<int, OCF_OPT_ADAGRAD>{}); break;
    case OCF_OPT_RMSPROP: by_n(integral_constant<int, OCF_OPT_RMSPROP>{}); break;
    default: by_n(integral_constant<int, OCF_OPT_ADAM>{});
  }
}

struct RowsOne {
  const RowsLaunch& L;
  hipStream_t s;
  template <typename CT, int KIND, int CW, int NCH, int PARTS, bool LONG> void go() {
    hipLaunchKernelGGL((optim_rowpipe_kernel<CT, KIND, CW, NCH, PARTS, LONG>), dim3(L.grid), dim3(RS_THREADS), 0, s,
                       L.ra, L.jb);
  }
};
struct RowsPair {
  const RowsLaunch& A;
  const RowsLaunch& B;
  RsPair ps;
  hipStream_t s;
  template <typename CT, int KIND, int CW, int NCH, int PARTS, bool LONG> void go() {
    hipLaunchKernelGGL((optim_rowpipe_pair_kernel<CT, KIND, CW, NCH, PARTS, LONG>), dim3(A.grid + B.grid),
                       dim3(RS_THREADS), 0, s, A.ra, A.jb, B.ra, B.jb, ps);
  }
};

struct RowsDual {
  const RowsLaunch& A;
  const RowsLaunch& B;
  RsPair ps;
  int grid;
  hipStream_t s;
  // one instance per (optimizer, width, prefetch) whatever the single kernel's PARTS / LONG: the parts are a
  // launch argument (ps.parts)
  template <typename CT, int KIND, int CW, int NCH, int PARTS, bool LONG> void go() {
    // (the prefetch pays at ~2 rows per wave: ML-1M's 16 parts; at one row per wave it only costs registers)
    if (g_rows_dual_pf > 0 || (g_rows_dual_pf < 0 && ps.parts <= 16))
      hipLaunchKernelGGL((optim_rowdual_kernel<CT, KIND, CW, NCH, true>), dim3(grid), dim3(RS_THREADS), 0, s, A.ra,
                         A.jb, B.ra, B.jb, ps);
    else
      hipLaunchKernelGGL((optim_rowdual_kernel<CT, KIND, CW, NCH, false>), dim3(grid), dim3(RS_THREADS), 0, s, A.ra,
                         A.jb, B.ra, B.jb, ps);
  }
};

// the dual-row launch (ocf_rows_dw.h optim_rowdual_kernel): both updates of a small weight pair walk the
// shared row lists once.  Needs the same lists, live records and row geometry on both sides, the row
// reduction (if any) as the output side's only job and none on the input side.
inline bool rows_dual_ok(const OcfGemmArgs& a, const OcfGemmArgs& b, const RowsLaunch& A, const RowsLaunch& B) {
  return a.sp_rowptr == b.sp_rowptr && a.sp_rowent == b.sp_rowent && a.row_live == b.row_live && !b.sp_colsum &&
         A.ra.M == B.ra.M && A.ra.ld == B.ra.ld && A.N == B.N && !B.jb.jr_on &&
         !(A.jb.jr_on && (A.jb.jb_part || A.jb.js_sp));
}

template <typename CT>
bool launch_rows(const OcfGemmArgs& g, const EpiOptim::Params& ep, hipStream_t s) {
  RowsLaunch L;
  if (!rows_setup(g, ep, L)) return false;
  rows_dispatch<CT>(L, RowsOne{L, s});
  OCF_HIP(hipGetLastError());
  return true;
}

template <typename CT>
bool launch_rows_pair(const OcfGemmArgs& a, const OcfGemmArgs& b, OcfPairSync& sync, hipStream_t s) {
  if (!g_optim_rows || !rows_pair_ok(a) || !rows_pair_ok(b)) return false;
  RowsLaunch A, B;
  if (!rows_setup(a, optim_params(a), A) || !rows_setup(b, optim_params(b), B)) return false;
  if (A.kind != B.kind || A.N != B.N || A.parts != B.parts || A.lng != B.lng || A.small != B.small) return false;
  // small weights (about one row per wave): the pair form's in-kernel wait (the producers' L2 write-back, the
  // consumers' polling) cost more than the boundary it replaces (ML-1M 36.9 vs 36.8 us, ML-100K 25.8 vs 21.7;
  // ML-20M 303 vs 307: tools/step_parts_probe.py) -- there the dual-row launch walks each row's chain once for
  // both layers instead (g_rows_dual, "rows_dual"), or two launches
  const bool dual = (A.small || g_rows_dual_large) && g_rows_dual && rows_dual_ok(a, b, A, B);
  if (A.small && !dual) return false;
  RsPair ps{};
  ps.word = reinterpret_cast<unsigned long long*>(sync.word);
  ps.n_a = A.grid;
  ps.n_prod = A.jb.jr_on ? (A.jb.jr.Bp + 3) / 4 : 0;   // the job-only workgroups holding the row reduction
  ps.want = (unsigned long long)sync.count + (unsigned long long)ps.n_prod;
  ps.err = async_error_word();
  ps.max_polls = g_pair_wait_polls;
  ps.gate = encdec_gate_word();          // (nullptr until the first ocf_gather_encdec)
  ps.gate_gen = encdec_generation();
  if (dual) {
    ps.n_a = 0;
    const int nprod = (A.jb.count() + 3) / 4;
    ps.n_prod = A.jb.jr_on ? nprod : 0;
    ps.want = (unsigned long long)sync.count + (unsigned long long)ps.n_prod;
    // parts per 128-row tile.  Small weights: 32 (about one row per wave) while the waves fit the chip's slots
    // at the dual kernel's ~110-125 VGPRs (4 waves per SIMD: 4,096), else 16 (ML-1M's 48 tiles: 3,072 waves of
    // ~2 rows instead of 6,144 in 1.5 rounds).  Large weights: about one live row per wave too -- the expected
    // live rows per tile (128 (1 - exp(-entries / rows)) with live records, else 128) / 4 -- but never a multiple
    // of 4: measured at ML-20M (pair launch, HIP events, same box, profiles/r05_dual_large/): parts 8 / 12 / 16 /
    // 20 / 24 311 / 298 / 312 / 298 / 296 us, 13-15 294, 17-19 288-291, 21-23 278-282, 25-27 281-283, 30 / 34
    // 287 / 289 (and the pair launch 311.6).  g_rows_dual_parts forces a count ("rows_dual_parts").
    int parts = A.small ? (A.ra.M / 128 * 32 * 4 > 4096 ? 16 : 32) : 0;
    if (!A.small) {
      const double live = A.ra.live ? 1.0 - std::exp(-(double)a.sp_nent / (double)A.ra.M) : 1.0;
      parts = std::min(63, std::max(5, (int)(128.0 * live / 4.0)));
      if (parts % 4 == 0) --parts;
    }
    if (g_rows_dual_parts) parts = g_rows_dual_parts;
    ps.parts = parts;
    const int grid = nprod + (B.jb.count() + 3) / 4 + A.ra.M / 128 * parts;
    rows_dispatch<CT>(A, RowsDual{A, B, ps, grid, s});
    ++g_rows_dual_count;
  } else {
    rows_dispatch<CT>(A, RowsPair{A, B, ps, s});
  }
  OCF_HIP(hipGetLastError());
  sync.count = ps.want;
  return true;
}

#define OCF_ROWS_INSTANTIATE(CT)                                                                           \
  template bool launch_rows<CT>(const OcfGemmArgs&, const EpiOptim::Params&, hipStream_t);                  \
  template bool launch_rows_pair<CT>(const OcfGemmArgs&, const OcfGemmArgs&, OcfPairSync&, hipStream_t);

}  // namespace ocf
