// Row-stream weight-gradient + optimizer kernel (EPI_OPTIM over a sparse batch operand), gfx950.
//
// The weight gradient of a first/last layer on a sparse batch is dW[m][:] = sum over the batch entries
// (v, k) of column m of v * B[k][:] (B = the hidden activations h or deltas dh, [K][N] in the compute
// dtype; v = the live input (dW_in) or the output delta (dW_out), in fp32: one rounding fewer than the
// MFMA form, which stages v in the compute dtype).  At ML-20M a batch holds 0.5 % of the [K][M]
// operand and a live weight row has about two entries: its gradient is two 1-KB row reads from L2,
// and the launch's real cost is the optimizer stream over the parameter / slot rows (Adagrad: 16 B
// per element + the 2-B shadow).  The role-split MFMA kernel (ocf_optim_ws.h) streams that in 128 x
// 128 tiles, i.e. 512-B row pieces 2 KB apart, beside a K-loop over 99.5 % zeros.
//
// This kernel is shaped after the stream instead: one wave per weight row, whole rows, rows in order.
// Lane l owns the CW-float chunks l + 64 j (j < NCH, N = 64 CW NCH), so each wave instruction reads or
// writes 64 CW * 4 contiguous bytes (tools/probes/opt_stream.hip, the parameter stream alone: whole
// 2-KB rows with nt loads and stores 6.05 TB/s with 67 % of the rows live, 128-column tile pieces
// 5.31 TB/s).  A row's entry list is wave-uniform: entries and values are scalar loads and each
// entry's B piece is one coalesced wave load.  Rows come from the live-row records (ocf.h
// OCF_LIVE_REC, compacted per 128-row tile; Adagrad with l2 == 0: a row without entries has the
// identity update) or, without records, every row.  Per element the sum over the entries runs in
// entry (batch-row) order in fp32.  Measured (ML-20M step, dW_in launch, HIP events): 199 us for the
// role-split MFMA kernel; 194 us one row batch per wave without pipelining (the chain record -> row
// pointer -> entry -> value, B row ran after the HBM loads); 150-155 us pipelined as below.
#pragma once
#include "ocf_epilogues.h"
#include "ocf_optim_ws.h"

namespace ocf {

constexpr int RS_THREADS = 256;
constexpr int RS_E0 = 2;   // entries per row loaded with the row's first loads (E0 = 1 / 3: equal / 3 % slower)
constexpr int RS_ET = 4;   // entries loaded together beyond those (rows of long batches)
#ifndef OCF_RS_ETL
#define OCF_RS_ETL 4
#endif
constexpr int RS_ETL = OCF_RS_ETL;  // LONG variant: B rows of this many entries in flight per group
// OCF_RS_GLDS 1: the next row's parameter / slot loads through LDS-DMA (global_load_lds_dwordx4 into the wave's
// LDS slot, read back by the update) instead of into registers.  The stream-only probe gained 2.5 % with it
// (tools/probes/opt_glds.hip); in the kernel the ML-20M pair launch moved 305.4 -> 304.0 us but the step and
// ML-1M did not (profiles/r04_glds/), the kernel's VGPRs rose 75 -> 80: off, kept for the record.
#ifndef OCF_RS_GLDS
#define OCF_RS_GLDS 0
#endif

struct RowsDwArgs {
  float* p; float* s1; float* s2;
  int64_t ld;                 // parameter row stride (floats) = N
  int M, N;
  const void* B; int64_t ldb; // [K][ldb] compute dtype
  const int32_t* rowptr; const int2* rowent; const float* vals;
  const uint8_t* live;        // live-row records per 128-row tile, or null (every row)
  OcfOptParams op;
  void* shadow;               // row-major compute-dtype copy of p, or null
  float* colsum; float colsum_scale;
};

// CW consecutive B-operand elements of type CT as one load (4, 8 or 16 bytes)
template <int BYTES> struct RsBits;
template <> struct RsBits<4> { using T = uint32_t; };
template <> struct RsBits<8> { using T = uint2; };
template <> struct RsBits<16> { using T = uint4; };
template <typename CT, int CW> using RsH = typename RsBits<CW * (int)sizeof(CT)>::T;

template <int CW> struct RsVec;
template <> struct RsVec<4> {
  using F = float4;
  static __device__ __forceinline__ F ld(__amdgpu_buffer_rsrc_t r, const float* base, uint32_t o) {
    return ld_pol16<OCF_OPT_LD_POL>(r, base, o);
  }
  static __device__ __forceinline__ void st(__amdgpu_buffer_rsrc_t r, float* base, uint32_t o, const F& v) {
    st_pol16<OCF_OPT_ST_POL>(r, base, o, v);
  }
  static __device__ __forceinline__ F zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }
};
template <> struct RsVec<2> {
  using F = float2;
  static __device__ __forceinline__ F ld(__amdgpu_buffer_rsrc_t r, const float* base, uint32_t o) {
    typedef unsigned int u2 __attribute__((ext_vector_type(2)));
    const u2 u = __builtin_amdgcn_raw_buffer_load_b64(r, o, 0, OCF_OPT_LD_POL);
    F f;
    __builtin_memcpy(&f, &u, 8);
    (void)base;
    return f;
  }
  static __device__ __forceinline__ void st(__amdgpu_buffer_rsrc_t r, float* base, uint32_t o, const F& v) {
    typedef unsigned int u2 __attribute__((ext_vector_type(2)));
    u2 u;
    __builtin_memcpy(&u, &v, 8);
    __builtin_amdgcn_raw_buffer_store_b64(u, r, o, 0, OCF_OPT_ST_POL);
    (void)base;
  }
  static __device__ __forceinline__ F zero() { return make_float2(0.f, 0.f); }
};

// A workgroup takes one of PARTS equal parts of a tile's live rows and each wave walks its
// rows (ranks kb + wave + 4 i) one per iteration, with the index chain run ahead of the data:
//   A (row i+4): record byte -> row m;     B (row i+3): row pointers;
//   C (row i+2): the first RS_E0 entries;  D (row i+1): p / slot loads (HBM), entry values, B pieces;
//   E (row i):   gradient, update, stores.
// Scalar loads return out of order (a use waits for every outstanding one), so each stage consumes
// only what the previous iteration loaded and the consumers are issued first: the one scalar wait per
// iteration covers loads a whole iteration old.  Against the p / slot loads one stage earlier (B):
// 75 vs 113 VGPRs (6 vs 4 waves per SIMD), dW_in 144.5 vs 157.5 us.
// PARTS = 12 (about 7 rows per wave at ML-20M; ocf_gemm.hip launch_rows has the sweep).
template <typename CT, int CW, int NCH, int E0, bool ADAM, bool LONG> struct RpRow {
  using F = typename RsVec<CW>::F;
  using H = RsH<CT, CW>;
  int m, lo, n;
  bool lv;
  int2 e[LONG ? 1 : E0];
  float v[LONG ? 1 : E0];
  int2 ev;                // LONG: the row's first 64 entries, lane i = entry i
  float vv;               // LONG: their values
  H h[E0][NCH];
  F p[NCH], a[NCH], b[ADAM ? NCH : 1];
  WsJobs::BiasPre bias;   // output-layer bias and its slots (colsum rows with a folded bias update)
};

// LONG (rows with many entries: feature-parallel global batches, dense datasets): stage C loads the row's
// entries as one vector (lane i = entry i, up to 64 at a time), stage D their values as one gather, and
// stage E walks them in groups of RS_ETL whose B rows are all in flight at once -- the entry indices come
// from the vector by readlane, so a group waits for its B rows only, not for an entry -> value -> B chain.
// The row pipeline of one wave over the ranks k0 + stride i (i < nr) of a weight matrix's live rows;
// row_of(k) maps a rank to its weight row (called with increasing ranks, valid ones only).
template <typename CT, int KIND, int CW, int NCH, bool LONG, typename RowOf>
__device__ __forceinline__ void rowpipe_ranks(const RowsDwArgs& ra, const WsJobs& jobs, const int k0, const int stride,
                                              const int nr, RowOf&& row_of) {
  using V = RsVec<CW>;
  using F = typename V::F;
  using H = RsH<CT, CW>;
  constexpr bool ADAM = KIND == OCF_OPT_ADAM;
  constexpr int E0 = RS_E0;
  using Row = RpRow<CT, CW, NCH, E0, ADAM, LONG>;
  const int lane = threadIdx.x & 63;
  if (nr == 0) return;
  const __amdgpu_buffer_rsrc_t rp = wt_rsrc(ra.p), r1 = wt_rsrc(ra.s1), r2 = wt_rsrc(ra.s2);
  const CT* Bg = reinterpret_cast<const CT*>(ra.B);
  // LDS-DMA staging (16-B lanes only): the wave's slot holds one row's p | a (| b), NCH KB each
  constexpr bool GL = OCF_RS_GLDS && CW == 4;
  constexpr int SLOT = NCH * 64 * CW;                     // floats per array of a row
  __shared__ __attribute__((aligned(16))) float gl_slot[GL ? RS_THREADS / 64 : 1][GL ? (ADAM ? 3 : 2) * SLOT : 1];
  float* slot = gl_slot[GL ? (threadIdx.x >> 6) : 0];
  auto col = [&](int j) { return (lane + 64 * j) * CW; };
  auto off = [&](int m, int j) { return (uint32_t)(((int64_t)m * ra.ld + col(j)) * 4); };   // < 2 GiB: host check
  auto bpiece = [&](int k, int j) { return *reinterpret_cast<const H*>(Bg + (int64_t)k * ra.ldb + col(j)); };
  auto stA = [&](Row& r, int i) {
    r.lv = i < nr;
    r.m = r.lv ? __builtin_amdgcn_readfirstlane(row_of(k0 + stride * i)) : 0;
  };
  auto ld_pa = [&](Row& r) {
    if constexpr (GL) {
      // the slot's previous row was read back by stE before this (its ds_reads have returned)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int j = 0; j < NCH; ++j) {
        const int64_t e = (int64_t)r.m * ra.ld + col(j);
        __builtin_amdgcn_global_load_lds(ra.p + e, slot + j * 64 * CW, 16, 0, OCF_OPT_LD_POL);
        __builtin_amdgcn_global_load_lds(ra.s1 + e, slot + SLOT + j * 64 * CW, 16, 0, OCF_OPT_LD_POL);
        if constexpr (ADAM) __builtin_amdgcn_global_load_lds(ra.s2 + e, slot + 2 * SLOT + j * 64 * CW, 16, 0, OCF_OPT_LD_POL);
      }
    } else {
#pragma unroll
      for (int j = 0; j < NCH; ++j) {
        const uint32_t o = off(r.m, j);
        r.p[j] = V::ld(rp, ra.p, o);
        r.a[j] = V::ld(r1, ra.s1, o);
        if constexpr (ADAM) r.b[j] = V::ld(r2, ra.s2, o);
      }
    }
  };
  auto stB = [&](Row& r) {
    if (!r.lv) return;
    r.lo = __builtin_amdgcn_readfirstlane(ra.rowptr[r.m]);
    r.n = __builtin_amdgcn_readfirstlane(ra.rowptr[r.m + 1]) - r.lo;
  };
  auto rdl = [&](int x, int i) { return __builtin_amdgcn_readlane(x, i); };
  auto stC = [&](Row& r) {
    if (!r.lv) return;
    if constexpr (LONG) {
      r.ev = lane < r.n ? ra.rowent[r.lo + lane] : make_int2(0, 0);
    } else {
#pragma unroll
      for (int e = 0; e < E0; ++e) r.e[e] = e < r.n ? ra.rowent[r.lo + e] : make_int2(0, 0);
    }
    if (ra.colsum && jobs.cb_p) r.bias = jobs.colsum_pre(r.m);
  };
  auto stD = [&](Row& r) {
    if (!r.lv) return;
    ld_pa(r);
    if constexpr (LONG) {
      r.vv = lane < r.n ? ra.vals[r.ev.x] : 0.f;
#pragma unroll
      for (int e = 0; e < E0; ++e)
        if (e < r.n) {
          const int k = rdl(r.ev.y, e);
#pragma unroll
          for (int j = 0; j < NCH; ++j) r.h[e][j] = bpiece(k, j);
        }
    } else {
#pragma unroll
      for (int e = 0; e < E0; ++e) {
        r.v[e] = 0.f;
        if (e < r.n) {
          r.v[e] = ra.vals[r.e[e].x];
#pragma unroll
          for (int j = 0; j < NCH; ++j) r.h[e][j] = bpiece(r.e[e].y, j);
        }
      }
    }
  };
  const OcfOptParams o = ra.op;
  auto acc = [&](F& g, float v, H h) {
    CT x[CW];
    __builtin_memcpy(x, &h, sizeof(h));
    float* gf = reinterpret_cast<float*>(&g);
#pragma unroll
    for (int i = 0; i < CW; ++i) gf[i] += v * CvtT<CT>::from(x[i]);
  };
  auto stE = [&](Row& r) {
    if (!r.lv) return;
    if constexpr (GL) {
      // this row's LDS-DMA loads (issued by the previous stD, with its B pieces) have landed
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int j = 0; j < NCH; ++j) {
        r.p[j] = *reinterpret_cast<const F*>(slot + j * 64 * CW + lane * CW);
        r.a[j] = *reinterpret_cast<const F*>(slot + SLOT + j * 64 * CW + lane * CW);
        if constexpr (ADAM) r.b[j] = *reinterpret_cast<const F*>(slot + 2 * SLOT + j * 64 * CW + lane * CW);
      }
    }
    F g[NCH];
#pragma unroll
    for (int j = 0; j < NCH; ++j) g[j] = V::zero();
    float cs = 0.f;
    if constexpr (LONG) {
#pragma unroll
      for (int e = 0; e < E0; ++e)
        if (e < r.n) {
          const float v = __int_as_float(rdl(__float_as_int(r.vv), e));
#pragma unroll
          for (int j = 0; j < NCH; ++j) acc(g[j], v, r.h[e][j]);
          cs += v;
        }
      // the rest in groups of RS_ETL, 64 entries per vector (the first 64 from stage C / D)
      int2 ev = r.ev;
      float vv = r.vv;
      for (int e0 = E0; e0 < r.n; e0 += RS_ETL) {
        if ((e0 & 63) < RS_ETL && e0 >= 64) {     // crossed into the next 64: reload (rows over 64 entries)
          const int c0 = e0 & ~63;
          ev = c0 + lane < r.n ? ra.rowent[r.lo + c0 + lane] : make_int2(0, 0);
          vv = c0 + lane < r.n ? ra.vals[ev.x] : 0.f;
        }
        H hx[RS_ETL][NCH];
#pragma unroll
        for (int e = 0; e < RS_ETL; ++e) {
          const int i = e0 + e;
          if (i < r.n && (i & ~63) == (e0 & ~63)) {
            const int k = rdl(ev.y, i & 63);
#pragma unroll
            for (int j = 0; j < NCH; ++j) hx[e][j] = bpiece(k, j);
          }
        }
#pragma unroll
        for (int e = 0; e < RS_ETL; ++e) {
          const int i = e0 + e;
          if (i < r.n && (i & ~63) == (e0 & ~63)) {
            const float v = __int_as_float(rdl(__float_as_int(vv), i & 63));
#pragma unroll
            for (int j = 0; j < NCH; ++j) acc(g[j], v, hx[e][j]);
            cs += v;
          }
        }
        // a group straddling a 64-entry boundary: continue from the boundary
        if (((e0 + RS_ETL) & ~63) != (e0 & ~63) && ((e0 + RS_ETL) & 63) != 0) e0 = ((e0 + RS_ETL) & ~63) - RS_ETL;
      }
    } else {
#pragma unroll
    for (int e = 0; e < E0; ++e)
      if (e < r.n) {
#pragma unroll
        for (int j = 0; j < NCH; ++j) acc(g[j], r.v[e], r.h[e][j]);
        cs += r.v[e];
      }
    for (int e0 = E0; e0 < r.n; e0 += RS_ET) {            // rows with more entries: RS_ET at a time
      int2 x[RS_ET];
      float v[RS_ET];
      H hx[RS_ET][NCH];
#pragma unroll
      for (int e = 0; e < RS_ET; ++e) x[e] = e0 + e < r.n ? ra.rowent[r.lo + e0 + e] : make_int2(0, 0);
#pragma unroll
      for (int e = 0; e < RS_ET; ++e) {
        v[e] = 0.f;
        if (e0 + e < r.n) {
          v[e] = ra.vals[x[e].x];
#pragma unroll
          for (int j = 0; j < NCH; ++j) hx[e][j] = bpiece(x[e].y, j);
        }
      }
#pragma unroll
      for (int e = 0; e < RS_ET; ++e)
        if (e0 + e < r.n) {
#pragma unroll
          for (int j = 0; j < NCH; ++j) acc(g[j], v[e], hx[e][j]);
          cs += v[e];
        }
    }
    }
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      F p = r.p[j], a = r.a[j], b = V::zero();
      if constexpr (ADAM) b = r.b[j];
      float* pf = reinterpret_cast<float*>(&p);
      float* af = reinterpret_cast<float*>(&a);
      float* bf = reinterpret_cast<float*>(&b);
      const float* gf = reinterpret_cast<const float*>(&g[j]);
#pragma unroll
      for (int i = 0; i < CW; ++i) opt_update_k<KIND>(o, gf[i] * o.gscale, pf[i], af[i], bf[i]);
      const uint32_t ob = off(r.m, j);
      V::st(rp, ra.p, ob, p);
      V::st(r1, ra.s1, ob, a);
      if constexpr (ADAM) V::st(r2, ra.s2, ob, b);
      if (ra.shadow) {
        CT hh[CW];
#pragma unroll
        for (int i = 0; i < CW; ++i) hh[i] = CvtT<CT>::to(pf[i]);
        H w;
        __builtin_memcpy(&w, hh, sizeof(w));
        *reinterpret_cast<H*>(reinterpret_cast<char*>(ra.shadow) + ((int64_t)r.m * ra.ld + col(j)) * sizeof(CT)) = w;
      }
    }
    if (ra.colsum && lane == 0) {   // output-bias gradient (column sum of the entries) and its update
      const float v = cs * ra.colsum_scale;
      ra.colsum[r.m] = v;
      if (jobs.cb_p) jobs.colsum_bias<KIND>(r.m, v, r.bias);
    }
  };
  // every stage consumes only what the previous iteration loaded, and the consumers come first: the
  // one scalar wait per iteration (at E's first use) covers loads a whole iteration old
  Row r0, r1s, r2s, r3s;
  stA(r0, 0);
  stA(r1s, 1);
  stA(r2s, 2);
  stA(r3s, 3);
  stB(r0);
  stB(r1s);
  stB(r2s);
  stC(r0);
  stC(r1s);
  stD(r0);
  for (int i = 0; i < nr; ++i) {
    stE(r0);
    stD(r1s);
    stC(r2s);
    stB(r3s);
    Row r4;
    stA(r4, i + 4);
    r0 = r1s;
    r1s = r2s;
    r2s = r3s;
    r3s = r4;
  }
}

// the workgroup body of one weight matrix's launch: workgroup wbx of [job-only workgroups][row workgroups],
// the row workgroups PARTS per 128-row tile (a part of the tile's live rows each)
template <typename CT, int KIND, int CW, int NCH, int PARTS, bool LONG>
__device__ __forceinline__ void rowpipe_body(const RowsDwArgs& ra, const WsJobs& jobs, const int wbx) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // folded small jobs (the decoder's row reduction, hidden-bias update, the step's stats): one per wave of
  // the FIRST workgroups, which take no rows -- the row workgroups start at once on the other CUs instead
  // of behind a job (a job is a chain of dependent loads: 10-20 us; ML-1M's dW launches were ~25 us of
  // which the jobs' were the floor)
  const int njwg = (jobs.count() + 3) / 4;
  if (wbx < njwg) {
    const int j = wbx * 4 + wave;
    if (j < jobs.count()) jobs.run<KIND>(j, lane);
    return;
  }
  const int wb = wbx - njwg;
  const int t = wb / PARTS, part = wb % PARTS;
  if (t >= ra.M / 128) return;
  const int m0 = t * 128;
  const uint8_t* rec = ra.live ? ra.live + (int64_t)t * OCF_LIVE_REC : nullptr;
  const int L = rec ? *reinterpret_cast<const int*>(rec) : (ra.M - m0 < 128 ? ra.M - m0 : 128);
  auto row_of = [&](int k) { return m0 + (rec ? (int)rec[16 + (k & 7) * 16 + (k >> 3)] : k); };
  if (ra.colsum && rec && part == 0) {      // rows without entries: zero output-bias gradient
    __shared__ uint8_t live_fl[128];
    if (tid < 128) live_fl[tid] = 0;
    __syncthreads();
    if (tid < L) live_fl[row_of(tid) - m0] = 1;
    __syncthreads();
    if (tid < 128 && !live_fl[tid]) ra.colsum[m0 + tid] = 0.f;
  }
  // this part's ranks [kb, ke), this wave's: kb + wave + 4 i, i < nr
  const int kb = part * L / PARTS, ke = (part + 1) * L / PARTS;
  const int nr = __builtin_amdgcn_readfirstlane(ke - kb - wave > 0 ? (ke - kb - wave + 3) / 4 : 0);
  rowpipe_ranks<CT, KIND, CW, NCH, LONG>(ra, jobs, kb + wave, 4, nr, row_of);
}

template <typename CT, int KIND, int CW, int NCH, int PARTS, bool LONG>
__global__ void __launch_bounds__(RS_THREADS) optim_rowpipe_kernel(RowsDwArgs ra, WsJobs jobs) {
  rowpipe_body<CT, KIND, CW, NCH, PARTS, LONG>(ra, jobs, blockIdx.x);
}

// Both weight-gradient launches of a one-hidden-layer step in ONE launch (ocf_gemm_pair): workgroups
// [0, n_a) are the output layer's (its job-only workgroups first, then its rows), the rest the input
// layer's.  The input layer's operand B (the hidden delta) and its jobs' inputs (bias-gradient rows,
// stats rows) are written by the output layer's folded row reduction -- the first n_prod job-only
// workgroups.  Those publish with an agent-scope release (their XCD's L2 written back) and count in
// *word; every input-layer workgroup waits for *word >= want (= the count before this launch + n_prod)
// before it starts.  The word only grows -- no launch resets it, so no caller has to clear it between
// launches (ocf.h OcfPairSync: the host keeps the running count).  Deadlock-free: workgroups are
// dispatched in index order, so every producer is resident or done before a consumer can wait, and
// producers wait on nothing.  The wait is bounded: a workgroup that gives up (a word someone else wrote,
// a count that does not match it) records OCF_ASYNC_PAIR_WAIT in the library's error word and skips
// its rows instead of updating them from a stale delta; the next library call reports it.  The two
// layers' rows then stream back to back without a kernel boundary, and on small weights (about one row
// per wave, each a chain of dependent loads) their latency chains overlap.
struct RsPair {
  unsigned long long* word;   // completed producer workgroups, over all launches on this word
  unsigned long long want;    // the count this launch's consumers wait for
  uint32_t* err;              // the library's asynchronous error word (host-coherent)
  int n_a, n_prod, max_polls;
  int parts;                  // dual-row launch: workgroups per 128-row tile
  const uint32_t* gate;       // the encoder -> decoder hand-off's gate word (nullptr: none), closed when it holds
  uint32_t gate_gen;          // ... this generation: a decoder chunk of the step's encdec launch gave up
};

// The hand-off gate (ocf_internal.h encdec_gate_word): true when the fused encoder -> decoder launch this update
// follows gave up on a row -- its hidden delta and statistics are not valid, so nothing may be written from them.
// One plain load per workgroup (the word was written by an earlier kernel; the kernel start made it visible),
// issued at entry and consumed before the first write.
__device__ __forceinline__ bool gate_closed(const RsPair& ps) {
  if (!ps.gate) return false;
  return __builtin_amdgcn_readfirstlane(*reinterpret_cast<const volatile uint32_t*>(ps.gate)) == ps.gate_gen;
}

// The wait: one plain load first (L2-cached: once a consumer of this XCD has seen the count complete, the
// later ones find it there), then relaxed agent-scope loads until the count is complete.  Measured and
// rejected: an agent-scope acquire per consumer (it invalidates the XCD's L2) and a consumer count for a
// self-reset (thousands of atomics on one word): the ML-20M pair launch took 1.0-1.3 ms instead of 0.31.
// No invalidation is needed: the data the wait guards (the row reduction's outputs) is read in this kernel
// only after the wait and the kernel start invalidated every L1 / L2 line from before it, so a consumer's
// caches hold no stale copy -- its reads miss to memory, which the producers' release (L2 write-back) has
// updated, or hit lines a producer on the same XCD wrote.  Returns true when the producers' count is
// complete, false (error word set) when the bounded wait gave up.
__device__ __forceinline__ bool pair_wait(const RsPair& ps) {
  __shared__ int ok_sh;
  if (threadIdx.x == 0) {
    bool ok = *reinterpret_cast<volatile unsigned long long*>(ps.word) >= ps.want;
    for (int it = 0; !ok && it < ps.max_polls; ++it) {
      ok = __hip_atomic_load(ps.word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= ps.want;
      if (!ok) __builtin_amdgcn_s_sleep(2);
    }
    if (!ok) __hip_atomic_store(ps.err, (uint32_t)OCF_ASYNC_PAIR_WAIT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    ok_sh = ok ? 1 : 0;
  }
  __syncthreads();
  const bool ok = ok_sh != 0;
  if (ok) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  return ok;
}

template <typename CT, int KIND, int CW, int NCH, int PARTS, bool LONG>
__global__ void __launch_bounds__(RS_THREADS) optim_rowpipe_pair_kernel(RowsDwArgs ra, WsJobs ja, RowsDwArgs rb,
                                                                        WsJobs jb, RsPair ps) {
  const int bx = blockIdx.x;
  const bool closed = gate_closed(ps);
  if (bx < ps.n_a) {
    if (!closed) rowpipe_body<CT, KIND, CW, NCH, PARTS, LONG>(ra, ja, bx);
    if (bx < ps.n_prod) {
      // every wave waits for its stores to reach the L2, then ONE release (one L2 write-back per workgroup:
      // a release per wave made the wait cost ~15 us) publishes them with the count
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
      if (threadIdx.x == 0) __hip_atomic_fetch_add(ps.word, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  if (closed || !pair_wait(ps)) return;
  rowpipe_body<CT, KIND, CW, NCH, PARTS, LONG>(rb, jb, bx - ps.n_a);
}

// ---- the dual-row launch (ocf_gemm_pair on small weights): both layers' updates row by row in ONE chain.
// On the generator's train batches the two weight matrices' rows are the same columns with the same entry
// lists (the row lists are shared: dW_out[m] = sum of delta_e h[k], dW_in[m] = sum of x_e dh[k] over the
// entries (e, k) of column m), so a wave walks column m's index chain (row pointer -> entries -> values)
// once and streams both rows' parameters, slots and B rows.  At about one weight row per wave (ML-1M:
// 6,040 rows, ML-100K: 943) the two separate launches were each one such chain (18-22 us); here the chain
// is paid once.  The decoder's row reduction (the dh rows, the hidden-bias partial rows, the stats rows)
// is either done by the decoder launch (OcfGatherArgs jr: the engine's choice on small weights; nothing
// here waits) or rides in the first workgroups as in the pair kernel and publishes through the same
// monotonic counter; then the hidden-bias / stats jobs that read its outputs take the next workgroups and
// wait for it, and every row workgroup waits for it once, after its first row's index chain and parameter
// loads are in flight (they need no dh) and before its first dh row load (measured: slower than the two
// launches, ML-1M 49.5 vs 42.5 us -- the wait puts the reduction back on every row's path).  The per-element sums run in entry order as in
// rowpipe_ranks (the same fp32 results: the bit-identity tests compare both launches).
#ifndef OCF_RD_ETL
#define OCF_RD_ETL 2
#endif
constexpr int RD_ETL = OCF_RD_ETL;   // dual-row launch: entries per group (both layers' B rows in flight)
#ifndef OCF_RD_LATE_IN
#define OCF_RD_LATE_IN 1
#endif
// 1: the input layer's parameter / slot loads issued after the entry groups (fewer VGPRs: the waves of a
// small weight fit the chip in one round), 0: with the output layer's at the row's start
constexpr int RD_LATE_IN = OCF_RD_LATE_IN;
template <typename CT, int KIND, int CW, int NCH>
struct RdRow {
  using F = typename RsVec<CW>::F;
  int m, lo, n;
  int2 ev;                // the row's first 64 entries (lane i = entry i)
  float vo, vi;           // their output deltas / input values
  F po[NCH], ao[NCH], bo[KIND == OCF_OPT_ADAM ? NCH : 1];
  F pi[NCH], ai[NCH], bi[KIND == OCF_OPT_ADAM ? NCH : 1];
  WsJobs::BiasPre bias;
};

template <typename CT, int KIND, int CW, int NCH, bool PF>
__global__ void __launch_bounds__(RS_THREADS) optim_rowdual_kernel(RowsDwArgs ro, WsJobs jo, RowsDwArgs ri, WsJobs ji,
                                                                   RsPair ps) {
  using V = RsVec<CW>;
  using F = typename V::F;
  using H = RsH<CT, CW>;
  constexpr bool ADAM = KIND == OCF_OPT_ADAM;
  using Row = RdRow<CT, KIND, CW, NCH>;
  const int bx = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool closed = gate_closed(ps);   // (consumed before this workgroup's first write)
  // producers: the output side's jobs (the row reduction), published with the pair kernel's release
  const int nprod = (jo.count() + 3) / 4;
  if (bx < nprod) {
    const int j = bx * 4 + wave;
    if (j < jo.count() && !closed) jo.run<KIND>(j, lane);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (tid == 0 && ps.n_prod) __hip_atomic_fetch_add(ps.word, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  // consumers of the reduction's outputs: the hidden-bias update and the stats jobs
  const int ncons = (ji.count() + 3) / 4;
  if (bx < nprod + ncons) {
    if (closed || (ps.n_prod && !pair_wait(ps))) return;
    const int j = (bx - nprod) * 4 + wave;
    if (j < ji.count()) ji.run<KIND>(j, lane);
    return;
  }
  // (workgroups go to the 8 XCDs round robin, so consecutive parts of a tile run on different XCDs; giving
  // each XCD a contiguous range of tiles instead measured slower: 305-313 vs 291-298 us at ML-20M)
  const int wb = bx - nprod - ncons;
  const int PARTS = ps.parts;
  const int t = wb / PARTS, part = wb % PARTS;
  if (t >= ro.M / 128) return;          // (uniform per workgroup: no wait reached)
  const int m0 = t * 128;
  const uint8_t* rec = ro.live ? ro.live + (int64_t)t * OCF_LIVE_REC : nullptr;
  const int L = rec ? *reinterpret_cast<const int*>(rec) : (ro.M - m0 < 128 ? ro.M - m0 : 128);
  auto row_of = [&](int k) { return m0 + (rec ? (int)rec[16 + (k & 7) * 16 + (k >> 3)] : k); };
  if (ro.colsum && rec && part == 0) {      // rows without entries: zero output-bias gradient
    __shared__ uint8_t live_fl[128];
    if (tid < 128) live_fl[tid] = 0;
    __syncthreads();
    if (tid < L) live_fl[row_of(tid) - m0] = 1;
    __syncthreads();
    if (tid < 128 && !live_fl[tid]) ro.colsum[m0 + tid] = 0.f;
  }
  const int kb = part * L / PARTS, ke = (part + 1) * L / PARTS;
  const int nr = __builtin_amdgcn_readfirstlane(ke - kb - wave > 0 ? (ke - kb - wave + 3) / 4 : 0);
  const __amdgpu_buffer_rsrc_t rpo = wt_rsrc(ro.p), r1o = wt_rsrc(ro.s1), r2o = wt_rsrc(ro.s2);
  const __amdgpu_buffer_rsrc_t rpi = wt_rsrc(ri.p), r1i = wt_rsrc(ri.s1), r2i = wt_rsrc(ri.s2);
  const CT* Bo = reinterpret_cast<const CT*>(ro.B);
  const CT* Bi = reinterpret_cast<const CT*>(ri.B);
  auto col = [&](int j) { return (lane + 64 * j) * CW; };
  auto off = [&](int m, int j) { return (uint32_t)(((int64_t)m * ro.ld + col(j)) * 4); };
  auto piece = [&](const CT* Bg, int64_t ldb, int k, int j) {
    return *reinterpret_cast<const H*>(Bg + (int64_t)k * ldb + col(j));
  };
  auto rdl = [&](int x, int i) { return __builtin_amdgcn_readlane(x, i); };
  // the row's index chain and parameter loads (nothing here reads the reduction's outputs)
  auto ld_in = [&](Row& r) {
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      const uint32_t o = off(r.m, j);
      r.pi[j] = V::ld(rpi, ri.p, o);
      r.ai[j] = V::ld(r1i, ri.s1, o);
      if constexpr (ADAM) r.bi[j] = V::ld(r2i, ri.s2, o);
    }
  };
  auto ld_out = [&](Row& r) {
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      const uint32_t o = off(r.m, j);
      r.po[j] = V::ld(rpo, ro.p, o);
      r.ao[j] = V::ld(r1o, ro.s1, o);
      if constexpr (ADAM) r.bo[j] = V::ld(r2o, ro.s2, o);
    }
  };
  auto start = [&](Row& r, int i) {
    r.m = __builtin_amdgcn_readfirstlane(row_of(kb + wave + 4 * i));
    if constexpr (RD_LATE_IN < 2)
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      const uint32_t o = off(r.m, j);
      r.po[j] = V::ld(rpo, ro.p, o);
      r.ao[j] = V::ld(r1o, ro.s1, o);
      if constexpr (ADAM) r.bo[j] = V::ld(r2o, ro.s2, o);
    }
    if constexpr (RD_LATE_IN < 1) ld_in(r);
    r.lo = __builtin_amdgcn_readfirstlane(ro.rowptr[r.m]);
    r.n = __builtin_amdgcn_readfirstlane(ro.rowptr[r.m + 1]) - r.lo;
    r.ev = lane < r.n ? ro.rowent[r.lo + lane] : make_int2(0, 0);
    r.vo = lane < r.n ? ro.vals[r.ev.x] : 0.f;
    r.vi = lane < r.n ? ri.vals[r.ev.x] : 0.f;
    if (ro.colsum && jo.cb_p) r.bias = jo.colsum_pre(r.m);
  };
  auto acc = [&](F& g, float v, H h) {
    CT x[CW];
    __builtin_memcpy(x, &h, sizeof(h));
    float* gf = reinterpret_cast<float*>(&g);
#pragma unroll
    for (int i = 0; i < CW; ++i) gf[i] += v * CvtT<CT>::from(x[i]);
  };
  auto update = [&](const RowsDwArgs& ra, __amdgpu_buffer_rsrc_t rp, __amdgpu_buffer_rsrc_t r1,
                    __amdgpu_buffer_rsrc_t r2, int m, F (&p)[NCH], F (&a)[NCH], F* b, const F (&g)[NCH]) {
    const OcfOptParams o = ra.op;
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      F pj = p[j], aj = a[j], bj = V::zero();
      if constexpr (ADAM) bj = b[j];
      float* pf = reinterpret_cast<float*>(&pj);
      float* af = reinterpret_cast<float*>(&aj);
      float* bf = reinterpret_cast<float*>(&bj);
      const float* gf = reinterpret_cast<const float*>(&g[j]);
#pragma unroll
      for (int i = 0; i < CW; ++i) opt_update_k<KIND>(o, gf[i] * o.gscale, pf[i], af[i], bf[i]);
      const uint32_t ob = off(m, j);
      V::st(rp, ra.p, ob, pj);
      V::st(r1, ra.s1, ob, aj);
      if constexpr (ADAM) V::st(r2, ra.s2, ob, bj);
      if (ra.shadow) {
        CT hh[CW];
#pragma unroll
        for (int i = 0; i < CW; ++i) hh[i] = CvtT<CT>::to(pf[i]);
        H w;
        __builtin_memcpy(&w, hh, sizeof(w));
        *reinterpret_cast<H*>(reinterpret_cast<char*>(ra.shadow) + ((int64_t)m * ra.ld + col(j)) * sizeof(CT)) = w;
      }
    }
  };
  Row r;
  if (nr > 0) start(r, 0);
  if (ps.n_prod && !pair_wait(ps)) return;   // every wave of the workgroup, once (none: the decoder reduced)
  if (closed) return;                        // (the hand-off gave up: no parameter, slot or shadow write)
  // PF (parts < 32: waves of two or more rows): the next row's chain and parameter loads are issued before
  // this row's entry groups (ML-1M at 16 parts: register room, 3 waves per SIMD still hold every wave)
  Row rn;
  for (int i = 0; i < nr; ++i) {
    if constexpr (PF)
      if (i + 1 < nr) start(rn, i + 1);
    F go[NCH], gi[NCH];
#pragma unroll
    for (int j = 0; j < NCH; ++j) go[j] = gi[j] = V::zero();
    float cs = 0.f;
    int2 ev = r.ev;
    float vo = r.vo, vi = r.vi;
    // entries in groups of RD_ETL, every B row of a group (both layers) in flight together
    for (int e0 = 0; e0 < r.n; e0 += RD_ETL) {
      if ((e0 & 63) < RD_ETL && e0 >= 64) {     // crossed into the next 64 entries (rows over 64 entries)
        const int c0 = e0 & ~63;
        ev = c0 + lane < r.n ? ro.rowent[r.lo + c0 + lane] : make_int2(0, 0);
        vo = c0 + lane < r.n ? ro.vals[ev.x] : 0.f;
        vi = c0 + lane < r.n ? ri.vals[ev.x] : 0.f;
      }
      H ho[RD_ETL][NCH], hi[RD_ETL][NCH];
#pragma unroll
      for (int e = 0; e < RD_ETL; ++e) {
        const int q = e0 + e;
        if (q < r.n && (q & ~63) == (e0 & ~63)) {
          const int k = rdl(ev.y, q & 63);
#pragma unroll
          for (int j = 0; j < NCH; ++j) {
            ho[e][j] = piece(Bo, ro.ldb, k, j);
            hi[e][j] = piece(Bi, ri.ldb, k, j);
          }
        }
      }
#pragma unroll
      for (int e = 0; e < RD_ETL; ++e) {
        const int q = e0 + e;
        if (q < r.n && (q & ~63) == (e0 & ~63)) {
          const float a = __int_as_float(rdl(__float_as_int(vo), q & 63));
          const float b = __int_as_float(rdl(__float_as_int(vi), q & 63));
#pragma unroll
          for (int j = 0; j < NCH; ++j) {
            acc(go[j], a, ho[e][j]);
            acc(gi[j], b, hi[e][j]);
          }
          cs += a;
        }
      }
      // a group straddling a 64-entry boundary: continue from the boundary
      if (((e0 + RD_ETL) & ~63) != (e0 & ~63) && ((e0 + RD_ETL) & 63) != 0) e0 = ((e0 + RD_ETL) & ~63) - RD_ETL;
    }
    if constexpr (RD_LATE_IN == 3) {      // one layer's state at a time
      asm volatile("" ::: "memory");
      ld_out(r);
      update(ro, rpo, r1o, r2o, r.m, r.po, r.ao, r.bo, go);
      asm volatile("" ::: "memory");
      ld_in(r);
      update(ri, rpi, r1i, r2i, r.m, r.pi, r.ai, r.bi, gi);
    } else {
    if constexpr (RD_LATE_IN >= 1) {
      asm volatile("" ::: "memory");      // (keeps the compiler from hoisting these loads above the groups)
      if constexpr (RD_LATE_IN >= 2) ld_out(r);
      ld_in(r);
    }
    update(ro, rpo, r1o, r2o, r.m, r.po, r.ao, r.bo, go);
    update(ri, rpi, r1i, r2i, r.m, r.pi, r.ai, r.bi, gi);
    }
    if (ro.colsum && lane == 0) {
      const float v = cs * ro.colsum_scale;
      ro.colsum[r.m] = v;
      if (jo.cb_p) jo.colsum_bias<KIND>(r.m, v, r.bias);
    }
    if constexpr (PF) {
      r = rn;
    } else {
      if (i + 1 < nr) start(r, i + 1);
    }
  }
}

}  // namespace ocf
