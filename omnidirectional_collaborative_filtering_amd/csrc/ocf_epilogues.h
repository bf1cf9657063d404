// Fused GEMM epilogues.  Each epilogue receives the 2x2 block of 32x32 fp32 accumulators of one
// wave (C layout of v_mfma_f32_32x32x*: col = lane&31, row = (reg&3) + 8*(reg>>2) + 4*(lane>>5)).
#pragma once
#include "ocf_gemm.h"

namespace ocf {

struct NoPre {};
// two K-steps of operand loads in flight (gemm_kernel DEEP), per epilogue family.  Off by default:
// measured neutral on the ML-20M shapes (the K-loop is issue-bound, not latency-bound) and it costs
// occupancy where the epilogue is register-heavy.
#define OCF_NO_PROLOGUE                                                                            \
  using Pre = NoPre;                                                                             \
  template <class P>                                                                             \
  __device__ static Pre prologue(const P&, int, int, int, int, int, const GemmShape&) { return {}; }

template <class F>
__device__ __forceinline__ void for_each_acc(ocf_f16v (&acc)[2][2], const TileCtx& c, F&& f) {
#pragma unroll
  for (int bi = 0; bi < 2; ++bi)
#pragma unroll
    for (int bj = 0; bj < 2; ++bj)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        int m = c.m0 + c.wm + acc_row(bi, r, c.lane);
        int n = c.n0 + c.wn + acc_col(bj, c.lane);
        f(m, n, acc[bi][bj][r]);
      }
}

// ---- optimizer update (Keras 2.0.4 get_updates, float32 op order) ---------------------
// KIND fixed at compile time where a kernel is specialised per optimizer (optim_ws_kernel: a
// quarter of the code of the runtime switch below, which matters for the instruction cache)
template <int KIND>
__device__ __forceinline__ void opt_update_k(const OcfOptParams& o, float g, float& p, float& s1, float& s2) {
  if (o.l2 != 0.f) g = g + 2.0f * o.l2 * p;
  if constexpr (KIND == OCF_OPT_ADAGRAD) {        // a += g^2 ; p -= lr*g/(sqrt(a)+eps)
    float a = s1 + g * g;
    s1 = a;
    p = p - (o.lr * g) / (sqrtf(a) + o.eps);
  } else if constexpr (KIND == OCF_OPT_RMSPROP) { // a = rho*a + (1-rho)*g^2
    float a = o.rho * s1 + (1.0f - o.rho) * (g * g);
    s1 = a;
    p = p - (o.lr * g) / (sqrtf(a) + o.eps);
  } else if constexpr (KIND == OCF_OPT_ADAM) {    // m,v EMAs; p -= lr_t*m/(sqrt(v)+eps)
    float m = o.rho * s1 + (1.0f - o.rho) * g;
    float v = o.beta2 * s2 + (1.0f - o.beta2) * (g * g);
    s1 = m;
    s2 = v;
    p = p - (o.lr * m) / (sqrtf(v) + o.eps);
  } else {
    (void)s1; (void)s2;
    p = p - o.lr * g;
  }
}
__device__ __forceinline__ void opt_update(const OcfOptParams& o, float g, float& p, float& s1, float& s2) {
  switch (o.kind) {
    case OCF_OPT_ADAGRAD: opt_update_k<OCF_OPT_ADAGRAD>(o, g, p, s1, s2); break;
    case OCF_OPT_RMSPROP: opt_update_k<OCF_OPT_RMSPROP>(o, g, p, s1, s2); break;
    case OCF_OPT_ADAM: opt_update_k<OCF_OPT_ADAM>(o, g, p, s1, s2); break;
    default: opt_update_k<0>(o, g, p, s1, s2);
  }
}

// ---- split-K partial slab: out[split][m][n] --------------------------------------------
struct EpiSlab {
  OCF_NO_PROLOGUE
  static constexpr int LDS_NEED = 0;
  struct Params {
    float* out;
    int64_t ld;
    int64_t split_stride;
  };
  __device__ static void apply(const Params& p, ocf_f16v (&acc)[2][2], const TileCtx& c, const GemmShape&, const Pre&) {
    float* o = p.out + (int64_t)c.split * p.split_stride;
    for_each_acc(acc, c, [&](int m, int n, float v) { o[(int64_t)m * p.ld + n] = v; });
  }
};

// ---- bias + activation + dropout (hidden layers) ----------------------------------------
struct BiasActParams {
  const float* bias;
  int act;
  float keep;              // 1 - dropout rate (1 = no dropout)
  uint64_t seed, stream;   // device RNG for dropout (Philox)
  const uint8_t* mask_in;  // injected dropout mask (nullable)
  uint8_t* mask_out;       // dropout mask record for backward (nullable)
  float* a_out;            // pre-dropout activation fp32 (nullable)
  void* h_out;             // post-dropout activation in compute dtype (nullable)
  int h_dtype;
  int64_t ld;
  int m_real, n_real;
};

// a = act(v + bias), h = dropout(a); stores a / mask / h where the pointers are set; returns h
// (a_o / mk_o, nullable: the activation and the mask value, for a caller that reuses them)
__device__ __forceinline__ float bias_act_value(const BiasActParams& p, int m, int n, float v, float* a_o = nullptr,
                                                uint8_t* mk_o = nullptr) {
  int64_t idx = (int64_t)m * p.ld + n;
  bool live = m < p.m_real && n < p.n_real;
  float a = live ? act_apply(p.act, v + p.bias[n]) : 0.f;
  float h = a;
  if (a_o) *a_o = a;
  if (p.keep < 1.f) {
    uint8_t mk;
    if (p.mask_in) mk = p.mask_in[idx];
    else mk = (uint8_t)floorf(p.keep + philox_uniform(p.seed, p.stream, (uint64_t)idx));
    h = (a / p.keep) * (float)mk;
    if (p.mask_out) p.mask_out[idx] = mk;
    if (mk_o) *mk_o = mk;
  }
  if (p.a_out) p.a_out[idx] = a;
  if (p.h_out) {
    if (p.h_dtype == OCF_F32) reinterpret_cast<float*>(p.h_out)[idx] = h;
    else if (p.h_dtype == OCF_F16) reinterpret_cast<_Float16*>(p.h_out)[idx] = (_Float16)h;
    else reinterpret_cast<__bf16*>(p.h_out)[idx] = (__bf16)h;
  }
  return h;
}
__device__ __forceinline__ void bias_act_store(const BiasActParams& p, int m, int n, float v) {
  (void)bias_act_value(p, m, n, v);
}

struct EpiBiasAct {
  OCF_NO_PROLOGUE
  static constexpr int LDS_NEED = 0;
  using Params = BiasActParams;
  __device__ static void apply(const Params& p, ocf_f16v (&acc)[2][2], const TileCtx& c, const GemmShape&, const Pre&) {
    for_each_acc(acc, c, [&](int m, int n, float v) { bias_act_store(p, m, n, v); });
  }
};

// ---- backward through activation + dropout, with per-m-tile bias-grad column partials ----
struct GradActParams {
  const float* a;          // forward activation (pre-dropout) of this layer, fp32
  const uint8_t* mask;     // dropout mask (nullable)
  float keep;
  int act;
  void* d_out;             // delta in compute dtype (unscaled by gscale)
  int d_dtype;
  int64_t ld;
  float* db_part;          // [M/128][ld] column partial sums (nullable), already * gscale
  float gscale;
  int m_real, n_real;
};

__device__ __forceinline__ float grad_act_value(const GradActParams& p, int m, int n, float v) {
  int64_t idx = (int64_t)m * p.ld + n;
  if (!(m < p.m_real && n < p.n_real)) return 0.f;
  float d = v;
  if (p.keep < 1.f && p.mask) d = d * ((float)p.mask[idx] / p.keep);
  return d * act_grad(p.act, p.a[idx]);
}

__device__ __forceinline__ float load_ct(const void* in, int dtype, int64_t idx) {
  if (dtype == OCF_F32) return reinterpret_cast<const float*>(in)[idx];
  if (dtype == OCF_F16) return (float)reinterpret_cast<const _Float16*>(in)[idx];
  return (float)reinterpret_cast<const __bf16*>(in)[idx];
}

__device__ __forceinline__ void store_ct(void* out, int dtype, int64_t idx, float v) {
  if (dtype == OCF_F32) reinterpret_cast<float*>(out)[idx] = v;
  else if (dtype == OCF_F16) reinterpret_cast<_Float16*>(out)[idx] = (_Float16)v;
  else reinterpret_cast<__bf16*>(out)[idx] = (__bf16)v;
}

struct EpiGradAct {
  OCF_NO_PROLOGUE
  static constexpr int LDS_NEED = 2 * GT_BN * 4;
  using Params = GradActParams;
  __device__ static void apply(const Params& p, ocf_f16v (&acc)[2][2], const TileCtx& c, const GemmShape&, const Pre&) {
    float colsum[2] = {0.f, 0.f};
#pragma unroll
    for (int bi = 0; bi < 2; ++bi)
#pragma unroll
      for (int bj = 0; bj < 2; ++bj)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          int m = c.m0 + c.wm + acc_row(bi, r, c.lane);
          int n = c.n0 + c.wn + acc_col(bj, c.lane);
          float d = grad_act_value(p, m, n, acc[bi][bj][r]);
          store_ct(p.d_out, p.d_dtype, (int64_t)m * p.ld + n, d);
          colsum[bj] += d;
        }
    if (!p.db_part) return;
    // combine lane halves (rows 4..7 of each 8) then the two waves sharing wn, fixed order
#pragma unroll
    for (int bj = 0; bj < 2; ++bj) colsum[bj] += __shfl_xor(colsum[bj], 32);
    float* s = reinterpret_cast<float*>(c.lds);
    __syncthreads();
    if (c.lane < 32) {
#pragma unroll
      for (int bj = 0; bj < 2; ++bj) s[(c.wm / 64) * GT_BN + c.wn + 32 * bj + c.lane] = colsum[bj];
    }
    __syncthreads();
    if (c.tid < GT_BN) {
      float v = s[c.tid] + s[GT_BN + c.tid];
      p.db_part[(int64_t)c.tile_m * p.ld + c.n0 + c.tid] = v * p.gscale;
    }
  }
};

// ---- raw gradient store (data-parallel path: all-reduce before the optimizer) ------------
struct EpiGradStore {
  OCF_NO_PROLOGUE
  static constexpr int LDS_NEED = 0;
  struct Params {
    float* g;
    int64_t ld;
    float gscale;
    int bf16;   // 1: the gradient in bf16 (data parallel: half the bytes of the reduce-scatter)
  };
  __device__ static void apply(const Params& p, ocf_f16v (&acc)[2][2], const TileCtx& c, const GemmShape&, const Pre&) {
    if (p.bf16) {
      __bf16* g = reinterpret_cast<__bf16*>(p.g);
      for_each_acc(acc, c, [&](int m, int n, float v) { g[(int64_t)m * p.ld + n] = (__bf16)(v * p.gscale); });
    } else {
      for_each_acc(acc, c, [&](int m, int n, float v) { p.g[(int64_t)m * p.ld + n] = v * p.gscale; });
    }
  }
};

// ---- fused optimizer: the weight-gradient tile never reaches HBM ------------------------
// The 128x128 fp32 gradient tile is staged in LDS (operand buffers are free by now), then each
// thread streams 16 float4 chunks of the parameter / optimizer-state rows (512 contiguous bytes
// per tile row, 4 chunks = 8-12 16-B loads in flight per lane), applies the Keras update and
// writes them back.  This is the HBM-bound part of the step (16 B/param for Adagrad).
#ifndef OCF_OPT_U
#define OCF_OPT_U 4
#endif
// cache policy of the optimizer's parameter / slot streams (0 plain, 2 nt, 16 sc1).  nt on both
// keeps the fp32 master weights and slots (4 x P bytes, read and written once per step) from
// displacing the compute-dtype shadow in the 256 MiB Infinity Cache, so the next step's encoder
// reads the freshly written shadow on-die: measured -4..5 % per ML-20M step.
#ifndef OCF_OPT_ST_POL
#define OCF_OPT_ST_POL 2
#endif
#ifndef OCF_OPT_LD_POL
#define OCF_OPT_LD_POL 2
#endif
struct EpiOptim {
  static constexpr int YS = GT_BN + 4;
  static constexpr int LDS_NEED = GT_BM * YS * 4;
  static constexpr int CH = GT_BM * (GT_BN / 4) / GT_THREADS;   // 16 chunks of 4 per thread
  static constexpr int U = OCF_OPT_U;                            // chunks in flight per thread
  struct Params {
    float* p;
    float* s1;
    float* s2;
    int64_t ld;
    OcfOptParams op;
    void* shadow;      // compute-dtype copy of the updated weights (nullable)
    int shadow_dtype;
    bool shadow_blocked;  // shadow in the 64x64-blocked layout (else the layout of p)
    // (optim_ws_kernel only) live-row records (ocf.h OcfGemmArgs row_live, OCF_LIVE_REC): rows not
    // listed have a zero gradient and an identity update (Adagrad, l2 = 0); their traffic is skipped
    const uint8_t* row_live = nullptr;
  };
  struct Pre {};
  __device__ static int64_t chunk_off(const Params& p, int m0, int n0, int tid, int g, int u, int& ml, int& c4) {
    const int ch = tid + (g + u) * GT_THREADS;
    ml = ch >> 5;
    c4 = (ch & 31) * 4;
    return (int64_t)(m0 + ml) * p.ld + n0 + c4;
  }
  __device__ static void load_group(const Params& p, int m0, int n0, int tid, int g, float4 (&pv)[U], float4 (&av)[U],
                                    float4 (&bv)[U]) {
    const __amdgpu_buffer_rsrc_t rp = wt_rsrc(p.p), r1 = wt_rsrc(p.s1), r2 = wt_rsrc(p.s2);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      int ml, c4;
      const int64_t off = chunk_off(p, m0, n0, tid, g, u, ml, c4);
      pv[u] = ld_pol16<OCF_OPT_LD_POL>(rp, p.p, (uint32_t)(off * 4));
      av[u] = p.s1 ? ld_pol16<OCF_OPT_LD_POL>(r1, p.s1, (uint32_t)(off * 4)) : make_float4(0.f, 0.f, 0.f, 0.f);
      bv[u] = p.s2 ? ld_pol16<OCF_OPT_LD_POL>(r2, p.s2, (uint32_t)(off * 4)) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  __device__ static Pre prologue(const Params&, int, int, int, int, int, const GemmShape&) { return Pre{}; }
  __device__ static void store_shadow(const Params& p, int row, int col, const float4& v) {
    const int64_t off = p.shadow_blocked
                            ? (((int64_t)(row >> 6) * (p.ld >> 6) + (col >> 6)) << 12) + (row & 63) * 64 + (col & 63)
                            : (int64_t)row * p.ld + col;
    uint2 u;
    if (p.shadow_dtype == OCF_F16) {
      _Float16 h[4] = {(_Float16)v.x, (_Float16)v.y, (_Float16)v.z, (_Float16)v.w};
      __builtin_memcpy(&u, h, 8);
    } else {
      __bf16 h[4] = {(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
      __builtin_memcpy(&u, h, 8);
    }
    *reinterpret_cast<uint2*>(reinterpret_cast<char*>(p.shadow) + off * 2) = u;
  }
  __device__ static void apply(const Params& p, ocf_f16v (&acc)[2][2], const TileCtx& c, const GemmShape&,
                               const Pre&) {
    float* Y = reinterpret_cast<float*>(c.lds);
#pragma unroll
    for (int bi = 0; bi < 2; ++bi)
#pragma unroll
      for (int bj = 0; bj < 2; ++bj)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          Y[(c.wm + acc_row(bi, r, c.lane)) * YS + c.wn + acc_col(bj, c.lane)] = acc[bi][bj][r];
    __syncthreads();
    const OcfOptParams o = p.op;
    const __amdgpu_buffer_rsrc_t rp = wt_rsrc(p.p), r1 = wt_rsrc(p.s1), r2 = wt_rsrc(p.s2);
#pragma unroll 1
    for (int g = 0; g < CH; g += U) {
      float4 pv[U], av[U], bv[U], gv[U];
      int64_t off[U];
      int rw[U], cl[U];
      load_group(p, c.m0, c.n0, c.tid, g, pv, av, bv);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        int ml, c4;
        off[u] = chunk_off(p, c.m0, c.n0, c.tid, g, u, ml, c4);
        rw[u] = c.m0 + ml;
        cl[u] = c.n0 + c4;
        gv[u] = *reinterpret_cast<const float4*>(Y + ml * YS + c4);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        opt_update(o, gv[u].x * o.gscale, pv[u].x, av[u].x, bv[u].x);
        opt_update(o, gv[u].y * o.gscale, pv[u].y, av[u].y, bv[u].y);
        opt_update(o, gv[u].z * o.gscale, pv[u].z, av[u].z, bv[u].z);
        opt_update(o, gv[u].w * o.gscale, pv[u].w, av[u].w, bv[u].w);
        st_pol16<OCF_OPT_ST_POL>(rp, p.p, (uint32_t)(off[u] * 4), pv[u]);
        if (p.shadow) store_shadow(p, rw[u], cl[u], pv[u]);
        if (p.s1) st_pol16<OCF_OPT_ST_POL>(r1, p.s1, (uint32_t)(off[u] * 4), av[u]);
        if (p.s2) st_pol16<OCF_OPT_ST_POL>(r2, p.s2, (uint32_t)(off[u] * 4), bv[u]);
      }
    }
  }
};

// ---- predict: y = mask * (acc + b) (model.py:82-86) -------------------------------------
struct EpiPredict {
  OCF_NO_PROLOGUE
  static constexpr int LDS_NEED = 0;
  struct Params {
    const float* bias;
    const float* mask;   // dense [M][ld_mask] output mask (nullable = no mask)
    int64_t ld_mask;
    float* out;
    int64_t ld_out;
    int m_real, n_real;
  };
  __device__ static void apply(const Params& p, ocf_f16v (&acc)[2][2], const TileCtx& c, const GemmShape&, const Pre&) {
    for_each_acc(acc, c, [&](int m, int n, float v) {
      if (m < p.m_real && n < p.n_real) {
        float y = v + p.bias[n];
        if (p.mask) y = p.mask[(int64_t)m * p.ld_mask + n] * y;
        p.out[(int64_t)m * p.ld_out + n] = y;
      }
    });
  }
};

// ---- masked MSE on the decoder output (train.py:49, model.py:86) ------------------------
// Target entries of the batch are bucketed by 128-column tile (built by the scatter kernels).
// Per tile: y = acc + b is staged to LDS; each target entry (row, col, t, m) gives
//   err = m*y - t            (Keras MSE residual of prediction = mask * y_full)
//   d   = err * m            (dL/dy_full up to the constant 2/(B*N), folded in later)
// The dense d tile (zero where no target) is written in the compute dtype for the backward
// GEMMs, its column sums give the output-bias gradient, and SSE / SAE / count_nonzero(T+yhat)
// / per-row SSE feed the loss and the train.py metrics.
struct EpiMaskedMSE {
  static constexpr int YS = GT_BN + 4;   // LDS row stride (floats) of the staged tile
  static constexpr int NPRE = 2;         // bucket entries per thread loaded in the prologue
  static constexpr int LDS_NEED = GT_BM * YS * 4 + GT_BM * 4 * 4 + GT_BM * 4 + 4 * GT_BN * 4 + 3 * 4 * 4;
  struct Params {
    const float* bias;        // output bias [N]
    // bucket target mode (bk_ptr != nullptr): entries bucketed by 128-column tile
    const int* bk_ptr;        // [n_tiles+1]
    const int* bk_rc;         // (row << 7) | (col & 127)
    const float* bk_t;        // target value
    const float* bk_m;        // output-mask value
    // row-segment target mode: each batch row's entries of this column tile, from the target
    // CSR's column-sorted view; a thread owns a row (deterministic sums, no atomics)
    const int32_t* t_rows;
    const int64_t* t_rp;
    const int32_t* t_tptr;
    const int32_t* t_col;
    const float* t_val;
    const int32_t* t_lidx;
    const uint8_t* t_flag;
    const int64_t* t_lboff;
    int t_ntiles;
    float t_aux;
    // dense target mode (dn_t != nullptr): targets / output masks as dense fp32 arrays, batch row b at row
    // dn_rows[b] (or b) of [*][ld_dn]; an entry wherever t != 0 or m != 0 (Model.fit / train_on_batch)
    const float* dn_t;
    const float* dn_m;
    int64_t ld_dn;
    const int64_t* dn_rows;
    int n_real;
    void* d_out;              // dense delta [M][ld_d] compute dtype (nullable: eval)
    int d_dtype;
    int64_t ld_d;
    float* db_part;           // [M/128][ld_db] column sums * gscale (nullable)
    int64_t ld_db;
    float gscale;
    float* stats_part;        // [n_tiles * gm][4]: sse, sae, nnz(T+yhat), unused
    float* row_sse_part;      // [n_tiles][M] (nullable)
    int m_real;
  };
  struct Pre {
    int b0, b1;               // bucket mode: bucket range
    int rc[NPRE];             // bucket mode: prefetched entries; segment mode: column | -1
    float t[NPRE], m[NPRE];
    int64_t s_lo, s_hi, lb;   // segment mode: this thread's half of its row's segment
  };
  // segment mode: thread tid owns half (tid >> 7) of row (tid & 127)'s entries in this column tile
  __device__ static int seg_col(const Params& p, int64_t e, int64_t lb) {
    return p.t_flag[lb + p.t_lidx[e]] ? (p.t_col[e] & (GT_BN - 1)) : -1;
  }
  __device__ static Pre prologue(const Params& p, int, int tile_n, int m0, int, int tid, const GemmShape&) {
    Pre q;
    q.b0 = q.b1 = 0;
    q.s_lo = q.s_hi = q.lb = 0;
#pragma unroll
    for (int k = 0; k < NPRE; ++k) { q.rc[k] = -1; q.t[k] = 0.f; q.m[k] = 0.f; }
    if (p.dn_t) return q;
    if (p.bk_ptr) {
      q.b0 = p.bk_ptr[tile_n];
      q.b1 = p.bk_ptr[tile_n + 1];
#pragma unroll
      for (int k = 0; k < NPRE; ++k) {
        int e = q.b0 + tid + k * GT_THREADS;
        bool ok = e < q.b1;
        q.rc[k] = ok ? p.bk_rc[e] : -1;
        q.t[k] = ok ? p.bk_t[e] : 0.f;
        q.m[k] = ok ? p.bk_m[e] : 0.f;
      }
      return q;
    }
    const int b = m0 + (tid & (GT_BM - 1));
    if (b >= p.m_real) return q;
    const int r = p.t_rows[b];
    if (r < 0) return q;
    const int64_t base = p.t_rp[r];
    const int32_t* tp = p.t_tptr + (int64_t)r * (p.t_ntiles + 1) + tile_n;
    const int64_t lo = base + tp[0], hi = base + tp[1];
    const int64_t mid = lo + ((hi - lo + 1) >> 1);
    q.s_lo = (tid < GT_BM) ? lo : mid;
    q.s_hi = (tid < GT_BM) ? mid : hi;
    q.lb = p.t_lboff[b];
#pragma unroll
    for (int k = 0; k < NPRE; ++k) {
      const int64_t e = q.s_lo + k;
      if (e < q.s_hi) { q.rc[k] = seg_col(p, e, q.lb); q.t[k] = p.t_val[e]; }
    }
    q.s_lo += NPRE;
    return q;
  }
  __device__ static void entry(float* Y, uint32_t* bits, float* rsse, int m0, int rc, float t, float m, float& sse,
                               float& sae, float& cnt) {
    int row = rc >> 7, nl = rc & 127;
    int ml = row - m0;
    if (rc < 0 || ml < 0 || ml >= GT_BM) return;
    float yhat = m * Y[ml * YS + nl];
    float err = yhat - t;
    Y[ml * YS + nl] = err * m;
    atomicOr(&bits[ml * 4 + (nl >> 5)], 1u << (nl & 31));
    sse += err * err;
    sae += fabsf(err);
    cnt += (t + yhat != 0.f) ? 1.f : 0.f;
    atomicAdd(&rsse[ml], err * err);
  }
  __device__ static void apply(const Params& p, ocf_f16v (&acc)[2][2], const TileCtx& c, const GemmShape& sh,
                               const Pre& q) {
    float* Y = reinterpret_cast<float*>(c.lds);
    uint32_t* bits = reinterpret_cast<uint32_t*>(c.lds + GT_BM * YS * 4);
    float* rsse = reinterpret_cast<float*>(c.lds + GT_BM * YS * 4 + GT_BM * 16);
    float* colp = rsse + GT_BM;          // [4 waves][GT_BN]
    float* red = colp + 4 * GT_BN;       // [3][4]
    // 1. stage y = acc + b
#pragma unroll
    for (int bj = 0; bj < 2; ++bj) {
      const float bias = p.bias[c.n0 + c.wn + acc_col(bj, c.lane)];
#pragma unroll
      for (int bi = 0; bi < 2; ++bi)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          Y[(c.wm + acc_row(bi, r, c.lane)) * YS + c.wn + acc_col(bj, c.lane)] = acc[bi][bj][r] + bias;
    }
    for (int i = c.tid; i < GT_BM * 4; i += GT_THREADS) bits[i] = 0u;
    if (c.tid < GT_BM) rsse[c.tid] = 0.f;
    __syncthreads();
    // 2. this tile's target entries
    float sse = 0.f, sae = 0.f, cnt = 0.f;
    if (p.dn_t) {
      // dense targets: thread tid owns row tid % 128 of the tile and its half (tid / 128) of the columns, so
      // its row-SSE share, the row's mask bits and every sum are its own (no atomics but the final
      // two-addend row SSE, order-independent); 16 T / M loads in flight at a time
      const int ml = c.tid & (GT_BM - 1), c0 = (c.tid >> 7) * (GT_BN / 2);
      const int b = c.m0 + ml;
      float rs = 0.f;
      uint32_t w0 = 0u, w1 = 0u;
      if (b < p.m_real) {
        const int64_t ro = (p.dn_rows ? p.dn_rows[b] : (int64_t)b) * p.ld_dn + c.n0 + c0;
        const int nmax = p.n_real - (c.n0 + c0);
        constexpr int U = 16;
        for (int j0 = 0; j0 < GT_BN / 2; j0 += U) {
          float t[U], m[U];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const bool ok = j0 + u < nmax;
            t[u] = ok ? p.dn_t[ro + j0 + u] : 0.f;
            m[u] = ok ? p.dn_m[ro + j0 + u] : 0.f;
          }
#pragma unroll
          for (int u = 0; u < U; ++u) {
            if (t[u] == 0.f && m[u] == 0.f) continue;
            const int nl = c0 + j0 + u;
            const float yhat = m[u] * Y[ml * YS + nl];
            const float err = yhat - t[u];
            Y[ml * YS + nl] = err * m[u];
            if (j0 + u < 32) w0 |= 1u << (j0 + u);
            else w1 |= 1u << (j0 + u - 32);
            rs += err * err;
            sae += fabsf(err);
            cnt += (t[u] + yhat != 0.f) ? 1.f : 0.f;
          }
        }
      }
      bits[ml * 4 + (c0 >> 5)] = w0;
      bits[ml * 4 + (c0 >> 5) + 1] = w1;
      sse = rs;
      atomicAdd(&rsse[ml], rs);   // exactly two addends onto 0: order-independent
    } else if (p.bk_ptr) {
#pragma unroll
      for (int k = 0; k < NPRE; ++k) entry(Y, bits, rsse, c.m0, q.rc[k], q.t[k], q.m[k], sse, sae, cnt);
      for (int e = q.b0 + c.tid + NPRE * GT_THREADS; e < q.b1; e += GT_THREADS)
        entry(Y, bits, rsse, c.m0, p.bk_rc[e], p.bk_t[e], p.bk_m[e], sse, sae, cnt);
    } else {
      // segment mode: live targets of this row half, at most one per (row, column)
      const int ml = c.tid & (GT_BM - 1);
      const float m = p.t_aux;
      float rs = 0.f;
      auto one = [&](int nl, float t) {
        if (nl < 0) return;
        const float yhat = m * Y[ml * YS + nl];
        const float err = yhat - t;
        Y[ml * YS + nl] = err * m;
        atomicOr(&bits[ml * 4 + (nl >> 5)], 1u << (nl & 31));
        rs += err * err;
        sae += fabsf(err);
        cnt += (t + yhat != 0.f) ? 1.f : 0.f;
      };
#pragma unroll
      for (int k = 0; k < NPRE; ++k) one(q.rc[k], q.t[k]);
      for (int64_t e = q.s_lo; e < q.s_hi; e += 4) {
        int nl[4];
        float t[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const bool ok = e + k < q.s_hi;
          nl[k] = ok ? seg_col(p, e + k, q.lb) : -1;
          t[k] = ok ? p.t_val[e + k] : 0.f;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) one(nl[k], t[k]);
      }
      sse = rs;
      atomicAdd(&rsse[ml], rs);   // exactly two addends onto 0: order-independent
    }
    __syncthreads();
    // 3. dense delta tile (zeros where no target) -> compute dtype, 8 columns per chunk.  A thread
    //    keeps one 8-column group (tid % 16) over rows tid/16 + 16k, so it also accumulates the
    //    output-bias gradient partial of those 8 columns; lanes 16 apart then 4 waves combine
    //    in a fixed order.
    if (p.d_out) {
      float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      const int c8 = (c.tid & 15) * 8;
      const __amdgpu_buffer_rsrc_t rd = wt_rsrc(p.d_out);
#pragma unroll 2
      for (int ml = c.tid >> 4; ml < GT_BM; ml += GT_THREADS / 16) {
        uint32_t w = bits[ml * 4 + (c8 >> 5)] >> (c8 & 31);
        const float4 y0 = *reinterpret_cast<const float4*>(Y + ml * YS + c8);
        const float4 y1 = *reinterpret_cast<const float4*>(Y + ml * YS + c8 + 4);
        float v[8] = {y0.x, y0.y, y0.z, y0.w, y1.x, y1.y, y1.z, y1.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          v[j] = ((w >> j) & 1u) ? v[j] : 0.f;
          cs[j] += v[j];
        }
        int64_t off = (int64_t)(c.m0 + ml) * p.ld_d + c.n0 + c8;
        if (p.d_dtype == OCF_F32) {
          st_pol16<0>(rd, p.d_out, (uint32_t)(off * 4), make_float4(v[0], v[1], v[2], v[3]));
          st_pol16<0>(rd, p.d_out, (uint32_t)(off * 4 + 16), make_float4(v[4], v[5], v[6], v[7]));
        } else if (p.d_dtype == OCF_F16) {
          _Float16 h[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) h[j] = (_Float16)v[j];
          uint4 u; __builtin_memcpy(&u, h, 16);
          st_pol16<0>(rd, p.d_out, (uint32_t)(off * 2), u);
        } else {
          __bf16 h[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) h[j] = (__bf16)v[j];
          uint4 u; __builtin_memcpy(&u, h, 16);
          st_pol16<0>(rd, p.d_out, (uint32_t)(off * 2), u);
        }
      }
      if (p.db_part) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          cs[j] += __shfl_xor(cs[j], 16);
          cs[j] += __shfl_xor(cs[j], 32);
        }
        if (c.lane < 16) {
          const int wave = c.tid >> 6;
#pragma unroll
          for (int j = 0; j < 8; ++j) colp[wave * GT_BN + c8 + j] = cs[j];
        }
      }
    }
    // 5. loss / metric partials: wave butterflies, then 4 wave partials in fixed order
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      sse += __shfl_xor(sse, off);
      sae += __shfl_xor(sae, off);
      cnt += __shfl_xor(cnt, off);
    }
    const int wave = c.tid >> 6;
    if (c.lane == 0) { red[wave] = sse; red[4 + wave] = sae; red[8 + wave] = cnt; }
    __syncthreads();
    if (p.d_out && p.db_part && c.tid < GT_BN)
      p.db_part[(int64_t)c.tile_m * p.ld_db + c.n0 + c.tid] =
          ((colp[c.tid] + colp[GT_BN + c.tid]) + (colp[2 * GT_BN + c.tid] + colp[3 * GT_BN + c.tid])) * p.gscale;
    const int gm = sh.M / GT_BM;
    if (c.tid == 0) {
      float* sp = p.stats_part + ((int64_t)c.tile_n * gm + c.tile_m) * 4;
      sp[0] = (red[0] + red[1]) + (red[2] + red[3]);
      sp[1] = (red[4] + red[5]) + (red[6] + red[7]);
      sp[2] = (red[8] + red[9]) + (red[10] + red[11]);
      sp[3] = 0.f;
    }
    if (p.row_sse_part && c.tid < GT_BM)
      p.row_sse_part[(int64_t)c.tile_n * sh.M + c.m0 + c.tid] = rsse[c.tid];
  }
};

}  // namespace ocf
