// Persistent, role-split weight-gradient + optimizer kernel (EPI_OPTIM, 16-bit compute) for gfx950.
//
// The fused dW GEMM of gemm_kernel spends ~15 % of its time in the K-loop (MFMA + operand staging),
// during which its workgroup streams nothing; at two workgroups per CU the optimizer stream of the
// other one cannot cover it (measured: K = 256 -> 289 us, K = 64 -> 244 us at ML-20M dW shapes).
// Here one 512-thread workgroup per CU walks a static list of 128x128 tiles with two roles:
//   waves 0-3 (MFMA role): each wave owns a 64x64 quarter of the tile and stages its own operand
//             halves (A[k][m0+wm..+64), B[k][n0+wn..+64)) in private LDS images, so the K-loop
//             needs no barrier (a wave's LDS ops execute in order: the next K-step is written after
//             the current one's fragments were read).  A is dense ([K][M], buffer loads one K-step
//             ahead) or sparse, filled from the batch entries bucketed by (column tile, K-step)
//             (ocf_sparse_tiles), bucket entries two K-steps and values one K-step ahead;
//   waves 4-7 (stream role): the optimizer update of the previous tile from the fp32 gradient tile
//             Y in LDS -- parameter / slot chunks double-buffered in registers and prefetched across
//             tile boundaries, so HBM traffic does not stop while the MFMA role runs a K-loop.
// The roles meet twice per tile (LDS-scoped barriers; global loads and stores stay in flight):
//   A: the MFMA role has tile i's product, the stream role is done reading Y (tile i-1);
//   B: Y holds tile i.
// (A first version shared double-buffered operand images between the MFMA waves and so needed a
// workgroup barrier per K-step; every barrier realigned the stream waves: 357 us vs 296 us.)
// Results are bit-identical to gemm_kernel + EpiOptim: the same MFMA sequence per 32x32 block (k in
// order), the same update arithmetic, the bias column sums in the same k order.
#pragma once
#include "ocf_epilogues.h"

namespace ocf {

constexpr int WS_THREADS = 512;
#ifndef OCF_WS_U
#define OCF_WS_U 4
#endif
#ifndef OCF_WS_LOOP
#define OCF_WS_LOOP 1   // stream groups of a tile: 1 run-time loop over the live groups; 0 all (dead slots OOB), 2 unrolled + skip (both measured 1-3 % slower)
#endif
constexpr int WS_YS = GT_BN;                              // Y row stride (floats), unpadded
constexpr int WS_HALF = 64;                               // rows of a wave's operand half
// chunks per group and groups per tile (16 float4 chunks per stream thread per tile)
template <int KIND> struct WsCfg {
  static constexpr int NS = KIND == OCF_OPT_ADAM ? 2 : 1;   // optimizer slot streams
  static constexpr int U = OCF_WS_U;
  static constexpr int NG = GT_BM * (GT_BN / 4) / GT_THREADS / U;
  static_assert(NG % 2 == 0, "groups alternate between two register sets");
};

__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// one wave's [64 k][64 r] operand half of a K-step: 64 lanes x 8 chunks of 8 elements (16 B)
template <typename CT> struct WaveStager {
  using I = Img<CT, WS_HALF, true>;
  uint4 v[8];
  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t rs, int64_t ld, uint32_t soff, int lane) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int c = lane + 64 * i, k = c >> 3, rc = (c & 7) * 8;
      const uint32_t o = (uint32_t)(((int64_t)k * ld + rc) * 2);
      auto w = __builtin_amdgcn_raw_buffer_load_b128(rs, o, soff, 0);
      __builtin_memcpy(&v[i], &w, 16);
    }
  }
  __device__ __forceinline__ void store(char* img, int lane) const {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int c = lane + 64 * i, k = c >> 3, rc = (c & 7) * 8;
      *reinterpret_cast<uint4*>(img + k * I::STRIDE + rc * 2) = v[i];
    }
  }
};

template <int KIND> struct WsSet {
  static constexpr int U = WsCfg<KIND>::U;
  float4 p[U], a[U], b[WsCfg<KIND>::NS == 2 ? U : 1];
};

// Live rows (EpiOptim::Params row_live, ocf.h OCF_LIVE_REC): a stream thread's chunk slot j of a
// tile is the live row of rank r0 + 8 j (r0 = stid / 32, columns (stid % 32) * 4 .. + 3), so the
// live rows are streamed densely: group g (slots gU .. gU+U-1) exists iff 32 g < L for U = 4.  Slots
// past L get an out-of-range buffer offset (the load returns zeros without touching memory, the
// stores are dropped).  Without records every row is live and slot j is row r0 + 8 j.
constexpr uint32_t WS_OOB = 0x80000000u;   // >= num_records (0x7FFFFFFF) of wt_rsrc
struct WsRows {
  int L;      // live rows of the tile (wave-uniform)
  uint4 r;    // this thread's 16 row slots (tile-local row indices, one byte each)
};

template <int KIND> struct WsStream {
  static constexpr int U = WsCfg<KIND>::U;
  static constexpr int NS = WsCfg<KIND>::NS;
  static constexpr int SLOTS = GT_BM * (GT_BN / 4) / GT_THREADS;   // 16 chunk slots per thread per tile
  EpiOptim::Params ep;
  __amdgpu_buffer_rsrc_t rp, r1, r2;
  const float* Y;
  int stid;

  __device__ __forceinline__ WsRows rows_load(int m0) const {
    WsRows q;
    q.r = make_uint4(0, 0, 0, 0);
    if (!ep.row_live) {
      q.L = GT_BM;
      return q;
    }
    const uint8_t* rec = ep.row_live + (int64_t)(m0 / GT_BM) * OCF_LIVE_REC;
    q.L = *reinterpret_cast<const int*>(rec);
    q.r = *reinterpret_cast<const uint4*>(rec + 16 + (stid >> 5) * 16);
    return q;
  }
  // groups of a tile (wave-uniform)
  __device__ __forceinline__ int groups(const WsRows& q) const {
    const int L = __builtin_amdgcn_readfirstlane(q.L);
    const int ng = (L * (GT_BN / 4) + GT_THREADS * U - 1) / (GT_THREADS * U);
    return ng < 1 ? 1 : ng;
  }
  // chunk slot j: tile row ml, column c4; false = dead slot
  __device__ __forceinline__ bool slot(const WsRows& q, int j, int& ml, int& c4) const {
    const int k = (stid >> 5) + (GT_THREADS / 32) * j;
    c4 = (stid & 31) * 4;
    if (!ep.row_live) {
      ml = k;
      return true;
    }
    // word j / 4 of the slots by masks (a select chain on a run-time index becomes a stack array)
    const uint32_t w = (uint32_t)(j >> 2);
    const uint32_t word = (q.r.x & (0u - (uint32_t)(w == 0))) | (q.r.y & (0u - (uint32_t)(w == 1))) |
                          (q.r.z & (0u - (uint32_t)(w == 2))) | (q.r.w & (0u - (uint32_t)(w == 3)));
    const bool lv = k < q.L;
    ml = lv ? (int)((word >> (8 * (j & 3))) & 0xff) : 0;
    return lv;
  }
  __device__ __forceinline__ void load(int m0, int n0, int g, WsSet<KIND>& s, const WsRows& q) const {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      int ml, c4;
      const bool lv = slot(q, g * U + u, ml, c4);
      const uint32_t o = (uint32_t)(((int64_t)(m0 + ml) * ep.ld + n0 + c4) * 4) | (lv ? 0u : WS_OOB);
      s.p[u] = ld_pol16<OCF_OPT_LD_POL>(rp, ep.p, o);
      s.a[u] = ld_pol16<OCF_OPT_LD_POL>(r1, ep.s1, o);
      if constexpr (NS == 2) s.b[u] = ld_pol16<OCF_OPT_LD_POL>(r2, ep.s2, o);
    }
    __builtin_amdgcn_sched_barrier(0);   // keep the prefetch above the consumer of the other set
  }
  __device__ __forceinline__ void apply(int m0, int n0, int g, WsSet<KIND>& s, const WsRows& q) const {
    const OcfOptParams o = ep.op;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      int ml, c4;
      const bool lv = slot(q, g * U + u, ml, c4);
      const int64_t of = (int64_t)(m0 + ml) * ep.ld + n0 + c4;
      const float4 gv = *reinterpret_cast<const float4*>(Y + ml * WS_YS + c4);
      float4 pv = s.p[u];
      float4 av = s.a[u];
      float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
      if constexpr (NS == 2) bv = s.b[u];
      opt_update_k<KIND>(o, gv.x * o.gscale, pv.x, av.x, bv.x);
      opt_update_k<KIND>(o, gv.y * o.gscale, pv.y, av.y, bv.y);
      opt_update_k<KIND>(o, gv.z * o.gscale, pv.z, av.z, bv.z);
      opt_update_k<KIND>(o, gv.w * o.gscale, pv.w, av.w, bv.w);
      const uint32_t ob = (uint32_t)(of * 4) | (lv ? 0u : WS_OOB);
      st_pol16<OCF_OPT_ST_POL>(rp, ep.p, ob, pv);
      if (ep.shadow && lv) EpiOptim::store_shadow(ep, m0 + ml, n0 + c4, pv);
      st_pol16<OCF_OPT_ST_POL>(r1, ep.s1, ob, av);
      if constexpr (NS == 2) st_pol16<OCF_OPT_ST_POL>(r2, ep.s2, ob, bv);
    }
  }
};

// static persistent schedule: workgroup b runs on XCD b % 8; XCD x owns the contiguous tile range
// [x*T/8, (x+1)*T/8) and its G/8 workgroups take every (G/8)-th tile of it, so the gn tiles of one
// 128-row panel of A run together on one XCD's L2
struct WsSched {
  int first, stride, count;
  __device__ __forceinline__ WsSched(int T) {
    const int G = gridDim.x, x = blockIdx.x & 7, slot = blockIdx.x >> 3, nx = G >> 3;
    const int lo = (int)((int64_t)x * T / 8), hi = (int)((int64_t)(x + 1) * T / 8);
    first = lo + slot;
    stride = nx;
    count = first < hi ? (hi - first + nx - 1) / nx : 0;
  }
  __device__ __forceinline__ int tile(int i) const { return first + i * stride; }
};

// tile t -> origin: panel m = t / gn; its gn column tiles are rotated by m / 8, so a workgroup
// (which takes every (G/8)-th tile, G/8 a multiple of gn) cycles through the column tiles instead of
// always drawing the same one -- the n0 == 0 tiles carry the output-bias column sums and would
// otherwise all land on a quarter of the workgroups
__device__ __forceinline__ void ws_tile_origin(int t, int gn, int& m0, int& n0) {
  const int m = t / gn;
  m0 = m * GT_BM;
#ifndef OCF_WS_ROTATE
#define OCF_WS_ROTATE 1
#endif
  n0 = ((t % gn + (OCF_WS_ROTATE ? (m >> 3) : 0)) % gn) * GT_BN;
}

// small jobs of the step folded into the launch (ocf.h OcfGemmArgs cb_* / jb_* / js_*), done by the
// stream role while it waits for the first tile and by the colsum waves.  Each reproduces the
// arithmetic and summation order of the kernel it replaces (bias_opt_partials_kernel,
// stats_finalize_kernel) exactly.
struct WsJobs {
  float* cb_p; float* cb_s1; float* cb_s2; OcfOptParams cb_op;
  const float* jb_part; int jb_parts, jb_n; int64_t jb_ld; float* jb_p; float* jb_s1; float* jb_s2;
  OcfOptParams jb_op;
  const float* js_sp; const float* js_rs; float* js_out; int js_nparts, js_ntiles, js_M;
  OcfRowsReduceArgs jr; int jr_on;   // folded ocf_rows_reduce (GRAD_ACT): one job per batch row

  __host__ __device__ __forceinline__ int count() const {
    int n = jr_on ? jr.Bp : 0;
    n += jb_part ? (jb_n + 15) / 16 : 0;
    if (js_sp) n += 1 + (js_rs ? js_M : 0);
    return n;
  }
  // bias_opt_partials_kernel's four partial groups (k = grp mod 4), 16 columns per job: lane 16 q + c sums
  // group q of column c in row order (16 loads in flight: 4 rounds over 256 partial rows instead of 16 with
  // one lane per column), then lane c adds the four as the kernel does, (p0 + p1) + (p2 + p3)
  template <int KIND>
  __device__ __forceinline__ void bias_block(int blk, int lane) const {
    const int q = lane >> 4, i = blk * 16 + (lane & 15);
    const bool ok = i < jb_n;
    constexpr int NB = 16;
    float p = 0.f;
    for (int k0 = q; k0 < jb_parts; k0 += 4 * NB) {
      float x[NB];
#pragma unroll
      for (int j = 0; j < NB; ++j) x[j] = ok && k0 + 4 * j < jb_parts ? jb_part[(int64_t)(k0 + 4 * j) * jb_ld + i] : 0.f;
#pragma unroll
      for (int j = 0; j < NB; ++j)
        if (k0 + 4 * j < jb_parts) p += x[j];
    }
    const float p1 = __shfl_down(p, 16, 64), p2 = __shfl_down(p, 32, 64), p3 = __shfl_down(p, 48, 64);
    if (q != 0 || !ok) return;
    const float g = (p + p1) + (p2 + p3);
    float w = jb_p[i], a = jb_s1 ? jb_s1[i] : 0.f, b = jb_s2 ? jb_s2[i] : 0.f;
    opt_update_k<KIND>(jb_op, g, w, a, b);
    jb_p[i] = w;
    if (jb_s1) jb_s1[i] = a;
    if (jb_s2) jb_s2[i] = b;
  }
  // stats_finalize_kernel block 0 (256 threads, stride-256 partials, LDS tree) by one wave: lane l
  // plays threads l, l+64, l+128, l+192
  __device__ __forceinline__ void stats_totals(int lane) const {
    float r[3][4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float a = 0.f, b = 0.f, c = 0.f;
      for (int i = lane + 64 * q; i < js_nparts; i += 256) {
        a += js_sp[(int64_t)i * 4 + 0];
        b += js_sp[(int64_t)i * 4 + 1];
        c += js_sp[(int64_t)i * 4 + 2];
      }
      r[0][q] = a; r[1][q] = b; r[2][q] = c;
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      float v0 = r[k][0] + r[k][2], v1 = r[k][1] + r[k][3];   // s = 128
      float v = v0 + v1;                                       // s = 64
      for (int s = 32; s > 0; s >>= 1) {
        const float o = __shfl_down(v, s, 64);
        if (lane < s) v += o;
      }
      r[k][0] = v;
    }
    if (lane == 0) {
      js_out[0] = r[0][0]; js_out[1] = r[1][0]; js_out[2] = r[2][0]; js_out[3] = 0.f;
    }
  }
  // stats_finalize_kernel row-SSE wave (row m)
  __device__ __forceinline__ void stats_row(int m, int lane) const {
    float r = 0.f;
    for (int t = lane; t < js_ntiles; t += 64) r += js_rs[(int64_t)t * js_M + m];
    for (int off = 32; off > 0; off >>= 1) r += __shfl_xor(r, off);
    if (lane == 0) js_out[4 + m] = r;
  }
  // rows_reduce_kernel (OCF_REDUCE_GRAD_ACT) for batch row b by one wave: lane l plays the threads
  // x = l, l + 64, ... of the 256-thread workgroup (the same sums, in the same chunk order)
  __device__ __forceinline__ void reduce_row(int b, int lane) const {
    const bool real = b < jr.B;
    const int c0 = real ? jr.row_cptr[b] : 0, c1 = real ? jr.row_cptr[b + 1] : 0;
    GradActParams p;
    p.a = jr.a_in; p.mask = jr.mask_in; p.keep = jr.keep; p.act = jr.act; p.d_out = jr.h_out; p.d_dtype = jr.h_dtype;
    p.ld = jr.H; p.db_part = nullptr; p.gscale = jr.gscale; p.m_real = jr.B; p.n_real = jr.n_real;
    // H <= 512: the lane's (up to) 8 columns summed over the row's chunks in chunk order, the partial
    // loads of 4 chunks x 8 columns in flight together (the per-column loop waited once per chunk)
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = 0.f;
    const int nx = (jr.H - lane + 63) / 64;
    for (int c = c0; c < c1; c += 4) {
      float x4[4][8];
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int i = 0; i < 8; ++i)
          x4[k][i] = (c + k < c1 && i < nx) ? jr.part[(int64_t)(c + k) * jr.H + lane + 64 * i] : 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (c + k < c1)
#pragma unroll
          for (int i = 0; i < 8; ++i) v[i] += x4[k][i];
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (i >= nx) break;
      const int x = lane + 64 * i;
      const float d = grad_act_value(p, b, x, v[i]);
      store_ct(jr.h_out, jr.h_dtype, (int64_t)b * jr.H + x, d);
      if (jr.db_part) jr.db_part[(int64_t)b * jr.H + x] = d * jr.gscale;
    }
    if (jr.chunk_stats && lane < 4) {
      float v = 0.f;
      if (lane < 3)
        for (int c = c0; c < c1; ++c) v += jr.chunk_stats[(int64_t)c * 4 + lane];
      jr.stats_part[(int64_t)b * 4 + lane] = v;
      if (lane == 0 && jr.row_sse) jr.row_sse[b] = v;
    }
  }
  template <int KIND>
  __device__ __forceinline__ void run(int j, int lane) const {
    if (jr_on) {
      if (j < jr.Bp) {
        reduce_row(j, lane);
        return;
      }
      j -= jr.Bp;
    }
    const int nbj = jb_part ? (jb_n + 15) / 16 : 0;
    if (j < nbj) bias_block<KIND>(j, lane);
    else if (j == nbj) stats_totals(lane);
    else stats_row(j - nbj - 1, lane);
  }
  // output-layer bias from its column sum (bias_opt_partials_kernel with one partial); the bias and
  // its slots are loaded when the tile starts (colsum_pre) so the update does not stall the MFMA
  // role at the tile hand-off
  struct BiasPre {
    float w, a, b;
  };
  __device__ __forceinline__ BiasPre colsum_pre(int m) const {
    return BiasPre{cb_p[m], cb_s1 ? cb_s1[m] : 0.f, cb_s2 ? cb_s2[m] : 0.f};
  }
  template <int KIND>
  __device__ __forceinline__ void colsum_bias(int m, float v, BiasPre q) const {
    const float g = (v + 0.f) + (0.f + 0.f);
    float w = q.w, a = q.a, b = q.b;
    opt_update_k<KIND>(cb_op, g, w, a, b);
    cb_p[m] = w;
    if (cb_s1) cb_s1[m] = a;
    if (cb_s2) cb_s2[m] = b;
  }
};

// prefetch state of one sparse-A bucket: its range and the first 64 entries (one per lane).
// entry = (value index, k | m_local << 8); lanes past the bucket hold y = -1
struct WsBucket {
  int lo, n;
  int2 e;
};

template <typename CT, bool SPA, int KIND>
__global__ void __launch_bounds__(WS_THREADS)
optim_ws_kernel(GemmShape sh, EpiOptim::Params ep, WsJobs jobs) {
  constexpr int BK = KInfo<CT>::BK;
  static_assert(BK == 64 && sizeof(CT) == 2, "16-bit compute");
  using I = Img<CT, WS_HALF, true>;
  constexpr int WAVE_LDS = 2 * I::BYTES;                  // A half + B half
  constexpr int YOFF = 4 * WAVE_LDS;
  __shared__ __attribute__((aligned(16))) char lds[YOFF + GT_BM * WS_YS * 4];

  const int gn = sh.N / GT_BN;
  const WsSched sc(sh.M / GT_BM * gn);
  const int nk = sh.K / BK;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform role
  if (sc.count == 0) {         // no tile here (tiny GEMM): the stream waves still take their jobs
    if (wave >= 4) {
      const int nj = jobs.count(), sw = (gridDim.x - 1 - blockIdx.x) * 4 + (wave - 4);
      for (int j = sw; j < nj; j += gridDim.x * 4) jobs.run<KIND>(j, tid & 63);
    }
    return;
  }
  float* Y = reinterpret_cast<float*>(lds + YOFF);

  if (wave < 4) {
    // ------------------------------------------------------------------ MFMA role
    const int lane = tid & 63;
    const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
    char* imgA = lds + wave * WAVE_LDS;
    char* imgB = imgA + I::BYTES;
    const CT* Ag = reinterpret_cast<const CT*>(sh.A);
    const CT* Bg = reinterpret_cast<const CT*>(sh.B);
    WaveStager<CT> sa, sb;
    const uint32_t sta = (uint32_t)((int64_t)BK * sh.lda * 2), stb = (uint32_t)((int64_t)BK * sh.ldb * 2);
    const int total = sc.count * nk;                      // K-steps over all of this WG's tiles
    auto tile_of = [&](int q, int& m0, int& n0) {
      const int t = sc.tile(q / nk);
      ws_tile_origin(t, gn, m0, n0);
    };
    // sparse A: bucket of step q = (column tile m0/128, K-step q % nk)
    auto bucket_issue = [&](int q, WsBucket& bk) {
      int m0, n0;
      tile_of(q, m0, n0);
      const int bi = (m0 / GT_BM) * nk + q % nk;
      bk.lo = sh.sp_bptr[bi];
      bk.n = sh.sp_bptr[bi + 1] - bk.lo;
      bk.e = lane < bk.n ? sh.sp_ent[bk.lo + lane] : make_int2(0, -1);
    };
    auto val_of = [&](const WsBucket& bk) { return bk.e.y >= 0 ? sh.sp_vals[bk.e.x] : 0.f; };
    // The A half is zeroed once; afterwards each fill first clears only the previous K-step's entries
    // (one 2-B store per lane instead of 8 KB of zeros per wave and K-step), unless that bucket
    // overflowed 64 entries (rare: then the whole half is zeroed again)
    auto zero_a = [&]() {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int c = lane + 64 * i;
        *reinterpret_cast<uint4*>(imgA + (c >> 3) * I::STRIDE + (c & 7) * 16) = make_uint4(0, 0, 0, 0);
      }
    };
    int2 e_prev = make_int2(0, -1);
    int n_prev = 0;
    auto fill = [&](const WsBucket& bk, float v0) {
      auto at = [&](int2 e, int& k, int& m) {
        k = e.y & 255;
        m = (e.y >> 8) - wm;
        return e.y >= 0 && (unsigned)m < 64u;
      };
      if (__builtin_amdgcn_readfirstlane(n_prev) > 64) {
        zero_a();
      } else {
        int k, m;
        if (at(e_prev, k, m)) *reinterpret_cast<CT*>(imgA + k * I::STRIDE + m * 2) = CvtT<CT>::to(0.f);
      }
      auto put = [&](int2 e, float v) {
        int k, m;
        if (at(e, k, m) && v != 0.f) *reinterpret_cast<CT*>(imgA + k * I::STRIDE + m * 2) = CvtT<CT>::to(v);
      };
      put(bk.e, v0);
      for (int j = 64 + lane; j < bk.n; j += 64) {        // buckets beyond 64 entries (rare)
        const int2 e = sh.sp_ent[bk.lo + j];
        put(e, sh.sp_vals[e.x]);
      }
      e_prev = bk.e;
      n_prev = bk.n;
    };
    auto issue = [&](int q) {                              // operand loads of step q into registers
      int m0, n0;
      tile_of(q, m0, n0);
      const int kt = q % nk;
      if constexpr (!SPA) sa.load(tile_rsrc(Ag + m0 + wm), sh.lda, kt * sta, lane);
      sb.load(tile_rsrc(Bg + n0 + wn), sh.ldb, kt * stb, lane);
    };
    // colsum (output-bias gradient): the wn == 0 waves sum their 64 A columns over k, in order
    float csum = 0.f;
    auto sum_a = [&]() { csum += colsum_kstep<CT, BK>(imgA, I::STRIDE, lane); };

    // prologue: step 0 staged; sparse: entries of step 1 and B of step 1 in flight
    auto issue_b = [&](int q, WaveStager<CT>& st) {
      int m0, n0;
      tile_of(q, m0, n0);
      st.load(tile_rsrc(Bg + n0 + wn), sh.ldb, (q % nk) * stb, lane);
    };
    // sparse A pipeline: bucket entries three K-steps ahead, their values two ahead (each load of the
    // index -> value chain has a whole K-step of slack)
    WsBucket b_next{}, b_next2{}, b_next3{};
    float v_next = 0.f;
    if constexpr (SPA) {
      issue_b(0, sb);
      WsBucket b0;
      bucket_issue(0, b0);
      if (total > 1) bucket_issue(1, b_next);
      if (total > 2) bucket_issue(2, b_next2);
      const float v0 = val_of(b0);
      if (total > 1) v_next = val_of(b_next);
      zero_a();
      fill(b0, v0);
    } else {
      issue(0);
      sa.store(imgA, lane);
    }
    sb.store(imgB, lane);

    ocf_f16v acc[2][2];
    WsJobs::BiasPre bpre{0.f, 0.f, 0.f};
    // K-step q: operands of step q+1 in flight during its MFMAs (measured: a second B stage for long
    // K loops gains nothing and costs 32 VGPRs)
    auto body = [&](int q) {
      const int kt = q % nk;
      int m0, n0;
      tile_of(q, m0, n0);
      const bool colsum = sh.sp_colsum && n0 == 0 && wn == 0;
      if (kt == 0) {
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
        csum = 0.f;
        if (colsum && jobs.cb_p) bpre = jobs.colsum_pre(m0 + wm + lane);
      }
      if (colsum) sum_a();
      const bool more = q + 1 < total;
      float v_next2 = 0.f;
      if constexpr (SPA) {
        if (q + 3 < total) bucket_issue(q + 3, b_next3);
        if (q + 2 < total) v_next2 = val_of(b_next2);
        if (more) issue_b(q + 1, sb);
      } else {
        if (more) issue(q + 1);
      }
      mfma_kstep<CT, true, true, WS_HALF, WS_HALF>(imgA, imgB, 0, 0, lane, acc);
      if (more) {
        if constexpr (SPA) {
          fill(b_next, v_next);
          b_next = b_next2;
          b_next2 = b_next3;
          v_next = v_next2;
          sb.store(imgB, lane);
        } else {
          sa.store(imgA, lane);
          sb.store(imgB, lane);
        }
      }
      if (kt == nk - 1) {
        if (colsum) {
          const float v = csum * sh.colsum_scale;
          sh.sp_colsum[m0 + wm + lane] = v;
          if (jobs.cb_p) jobs.colsum_bias<KIND>(m0 + wm + lane, v, bpre);
        }
        lds_barrier();   // A: product of this tile ready; the stream role is done with Y
#pragma unroll
        for (int bi = 0; bi < 2; ++bi)
#pragma unroll
          for (int bj = 0; bj < 2; ++bj)
#pragma unroll
            for (int r = 0; r < 16; ++r)
              Y[(wm + acc_row(bi, r, lane)) * WS_YS + wn + acc_col(bj, lane)] = acc[bi][bj][r];
        lds_barrier();   // B: Y holds this tile
      }
    };
    for (int q = 0; q < total; ++q) body(q);
  } else {
    // ------------------------------------------------------------------ stream role
    const WsStream<KIND> st{ep, wt_rsrc(ep.p), wt_rsrc(ep.s1), wt_rsrc(ep.s2), Y, tid - 256};
    WsSet<KIND> s0, s1;
    auto origin = [&](int i, int& m0, int& n0) {
      const int t = sc.tile(i);
      ws_tile_origin(t, gn, m0, n0);
    };
    // one tile from Y: groups alternate register sets; the last group prefetches group 0 of the
    // next tile into set 0
    // live-row records: of the tile being streamed (qc) and of the next one, loaded at the top of
    // run_tile and first used when its first group is prefetched
    WsRows qc;
    auto run_tile = [&](int i) {
      int m0, n0, pm0 = 0, pn0 = 0;
      origin(i, m0, n0);
      const bool pre = i + 1 < sc.count;
      if (pre) origin(i + 1, pm0, pn0);
      const WsRows qn = pre ? st.rows_load(pm0) : qc;
      const int ng = st.groups(qc);
      if constexpr (OCF_WS_LOOP == 1) {     // run-time loop over the live groups
        for (int g = 0; g < ng; g += 2) {
          const bool two = g + 1 < ng;
          if (two) st.load(m0, n0, g + 1, s1, qc);
          st.apply(m0, n0, g, s0, qc);
          if (g + 2 < ng) st.load(m0, n0, g + 2, s0, qc);
          else if (pre) st.load(pm0, pn0, 0, s0, qn);
          if (two) st.apply(m0, n0, g + 1, s1, qc);
        }
      } else {                             // unrolled; 2: wave-uniform skip of dead groups, 0: none
        constexpr int NG = WsCfg<KIND>::NG;
        const int ne = OCF_WS_LOOP == 2 ? ng : NG;
#pragma unroll
        for (int g = 0; g < NG; g += 2) {
          if (g < ne) {
            const bool two = g + 1 < ne;
            if (two) st.load(m0, n0, g + 1, s1, qc);
            st.apply(m0, n0, g, s0, qc);
            if (g + 2 < ne) st.load(m0, n0, g + 2, s0, qc);
            else if (pre) st.load(pm0, pn0, 0, s0, qn);
            if (two) st.apply(m0, n0, g + 1, s1, qc);
          }
        }
      }
      qc = qn;
    };
    {
      int m0, n0;
      origin(0, m0, n0);
      qc = st.rows_load(m0);
      st.load(m0, n0, 0, s0, qc);
    }
    {  // folded small jobs, one per stream wave, while the MFMA role runs the first K-loop; taken
       // from the last workgroups first (the last slots of each XCD range hold one tile less)
      const int nj = jobs.count(), sw = (gridDim.x - 1 - blockIdx.x) * 4 + (wave - 4);
      for (int j = sw; j < nj; j += gridDim.x * 4) jobs.run<KIND>(j, tid & 63);
    }
    // tile i-1 streams while the MFMA role runs the K-loop of tile i; one call site keeps the
    // (large, unrolled) stream code once in the instruction cache
    for (int i = 0; i <= sc.count; ++i) {
      if (i > 0) run_tile(i - 1);
      if (i < sc.count) {
        lds_barrier();         // A (tile i)
        lds_barrier();         // B (tile i)
      }
    }
  }
}

}  // namespace ocf
