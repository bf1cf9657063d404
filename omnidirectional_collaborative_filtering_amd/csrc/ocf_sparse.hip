// Row-gather forms of the weight-streaming products for sparse batches (model.py:64-86 on the
// batch's rating entries instead of the dense [B][N] arrays).
//
//   encoder   hpre[b, :]  = sum over live input entries (b, n, x) of x * W1[n, :]
//   decoder   y = h[b, :] . W_out[n, :] + b_out[n] at every live target (b, n, t);
//             err = m*y - t, delta = err*m, loss/metric sums, and
//             dhpre[b, :] += delta * W_out[n, :]  (the same W_out row, still in registers)
//
// The masked output of model.py:84-86 is m (aux) at target positions and 0 elsewhere, so y off the
// targets never reaches the loss or a gradient: the dense decoder GEMM and the dense delta are
// replaced by these per-entry products, exactly (fp32 accumulation).  Each W row is read once per
// entry (1 KB at H = 512, f16 shadow), about the bytes of the dense product, without its MFMA-issue
// bound at B = 256.
//
// Work unit: a chunk of <= 256 consecutive entries of one batch row (host-built chunk tables, so a
// row with 60k ratings spreads over many workgroups).  A workgroup = 16 groups of 16 lanes; a group
// owns one entry at a time and each lane holds PPL 16-byte pieces of the row (pieces l, l+16, ...:
// every load instruction of a group reads 256 contiguous bytes).  Chunk partials are reduced in a
// fixed order per row by ocf_rows_reduce, which also applies the layer epilogue.
#include <algorithm>
#include <cstdlib>

#include "ocf_epilogues.h"
#include "ocf_internal.h"

namespace ocf {

#ifndef OCF_RG_THREADS
#define OCF_RG_THREADS 256
#endif
constexpr int RG_THREADS = OCF_RG_THREADS;   // threads per row-gather workgroup (one chunk of <= 256 entries)
constexpr int RG_MAX_H = 512;
#ifndef OCF_RG_U
#define OCF_RG_U 4
#endif
constexpr int RG_U = OCF_RG_U;   // entries per group in flight
#ifndef OCF_RG_UE
#define OCF_RG_UE 4
#endif
// ... in the encoder chunks of the fused encoder -> decoder launch: that kernel's register allocation is the
// decoder's (133 VGPRs at f16), so the encoder part can keep more entries in flight at no occupancy cost
constexpr int RG_UE = OCF_RG_UE;
#ifndef OCF_RG_UD
#define OCF_RG_UD 4
#endif
constexpr int RG_UD = OCF_RG_UD;  // ... in the decoder

template <typename WT> struct EPc { static constexpr int v = 16 / (int)sizeof(WT); };

// piece p (16 bytes) of row n of a weight array: row-major [rows][ldw] or 64x64-blocked (16-bit)
template <typename WT>
__device__ __forceinline__ void load_piece(const WT* W, int64_t ldw, int blocked, int n, int p,
                                           float (&out)[EPc<WT>::v]) {
  constexpr int E = EPc<WT>::v;
  const char* base;
  if (blocked) {
    const int h = p * 8;
    base = reinterpret_cast<const char*>(W) + ((((int64_t)(n >> 6) * (ldw >> 6)) + (h >> 6)) << 13) + (n & 63) * 128 +
           (h & 63) * 2;
  } else {
    base = reinterpret_cast<const char*>(W + (int64_t)n * ldw) + p * 16;
  }
  const uint4 u = *reinterpret_cast<const uint4*>(base);
  if constexpr (sizeof(WT) == 4) {
    __builtin_memcpy(out, &u, 16);
  } else {
    WT e[E];
    __builtin_memcpy(e, &u, 16);
#pragma unroll
    for (int k = 0; k < E; ++k) out[k] = (float)e[k];
  }
}

// raw 16-byte piece (kept packed in registers until used: half the VGPRs for 16-bit weights)
template <typename WT>
__device__ __forceinline__ uint4 load_piece_raw(const WT* W, int64_t ldw, int blocked, int n, int p) {
  const char* base;
  if (blocked) {
    const int h = p * 8;
    base = reinterpret_cast<const char*>(W) + ((((int64_t)(n >> 6) * (ldw >> 6)) + (h >> 6)) << 13) + (n & 63) * 128 +
           (h & 63) * 2;
  } else {
    base = reinterpret_cast<const char*>(W + (int64_t)n * ldw) + p * 16;
  }
  return *reinterpret_cast<const uint4*>(base);
}
template <typename WT>
__device__ __forceinline__ void unpack_piece(const uint4& u, float (&out)[EPc<WT>::v]) {
  if constexpr (sizeof(WT) == 4) {
    __builtin_memcpy(out, &u, 16);
  } else {
    WT e[EPc<WT>::v];
    __builtin_memcpy(e, &u, 16);
#pragma unroll
    for (int k = 0; k < EPc<WT>::v; ++k) out[k] = (float)e[k];
  }
}

// the same pieces of a compute-dtype activation row h[b] (row-major, ld = H)
template <typename HT, int E>
__device__ __forceinline__ void load_act_piece(const void* h, int64_t ld, int b, int p, float (&out)[E]) {
  const HT* row = reinterpret_cast<const HT*>(h) + (int64_t)b * ld + p * E;
#pragma unroll
  for (int k = 0; k < E; ++k) out[k] = (float)row[k];
}

// fixed-order reduction of the groups' per-lane vectors into part[chunk][H]
// sc1 (write-through / L1-bypassing) buffer accesses of values another workgroup of the same launch reads
// (MI355X_MICROARCH.md, inter-workgroup visibility: the hand-off table's first row)
constexpr int RG_SC1 = 16;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rg_rsrc(const float* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, 0x7FFFFFFF, 0x00020000);
}
__device__ __forceinline__ void st_sc1(float* base, int64_t e, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rg_rsrc(base), (uint32_t)(e * 4), 0, RG_SC1);
}
__device__ __forceinline__ float ld_sc1(const float* base, int64_t e) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rg_rsrc(base), (uint32_t)(e * 4), 0, RG_SC1));
}

constexpr int RG_XPT = (RG_MAX_H + RG_THREADS - 1) / RG_THREADS;   // columns per thread in the row loops

template <int G, int V, int E, int PPL>
__device__ __forceinline__ void reduce_groups(const float (&acc)[V], float* red, float* part, int c, int H, int grp,
                                              int l, bool wt = false, bool keep_only = false,
                                              float* own = nullptr) {
  constexpr int NG = RG_THREADS / G;
#pragma unroll
  for (int i = 0; i < PPL; ++i)
#pragma unroll
    for (int k = 0; k < E; ++k) red[grp * H + (l + G * i) * E + k] = acc[i * E + k];
  __syncthreads();
  for (int x = threadIdx.x, i = 0; x < H; x += RG_THREADS, ++i) {
    float s0 = 0.f, s1 = 0.f;
#pragma unroll
    for (int g = 0; g < NG; g += 2) {
      s0 += red[g * H + x];
      if (g + 1 < NG) s1 += red[(g + 1) * H + x];
    }
    if (own) own[i] = s0 + s1;            // (this thread's columns x = tid + RG_THREADS i)
    if (keep_only) continue;
    if (wt) st_sc1(part, (int64_t)c * H + x, s0 + s1);
    else part[(int64_t)c * H + x] = s0 + s1;
  }
}

// The decoder's folded row reduction (OcfGatherArgs jr / row_arrive): after its partial and stats stores
// (write-through) have landed, each chunk workgroup counts itself in row_arrive[b]; the one that completes
// the count sums the row's chunk partials in chunk order (sc1 loads) and applies rows_reduce_kernel's
// OCF_REDUCE_GRAD_ACT arithmetic (grad_act_value) and its stats rows.  a / mk: the row's activation and
// dropout mask from this workgroup's own hidden epilogue (stash), else read from jr.a_in / jr.mask_in
// (written by an earlier launch).
// solo: the row's only chunk is this workgroup's -- no stores to hand off, no counter: its own column sums
// (own) and stats total (own_st, threads 0..2) are the row's, added to 0 as the chunk loop would.
__device__ __forceinline__ void dec_row_tail(const OcfGatherArgs& a, const OcfRowsReduceArgs& r, int b,
                                             const float* a_sh, const uint8_t* mk_sh, bool stash, bool solo,
                                             const float* own, float own_st, uint32_t* enc_arrive) {
  __shared__ int last_sh;
  // (fused encoder -> decoder launch) every decoder chunk of the row has passed its wait once the row's last one
  // gets here: the encoder counter goes back to zero for the next launch
  if (enc_arrive && threadIdx.x == 0 && solo)
    __hip_atomic_store(&enc_arrive[b], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (!solo) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // this wave's write-through stores have landed
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint32_t nch = (uint32_t)(r.row_cptr[b + 1] - r.row_cptr[b]);
      const uint32_t old = __hip_atomic_fetch_add(&a.row_arrive[b], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const bool last = old + 1 == nch;
      if (last) __hip_atomic_store(&a.row_arrive[b], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (last && enc_arrive) __hip_atomic_store(&enc_arrive[b], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last_sh = last ? 1 : 0;
    }
    __syncthreads();
    if (!last_sh) return;
  }
  const int c0 = r.row_cptr[b], c1 = solo ? c0 : r.row_cptr[b + 1];
  const int64_t rb = (int64_t)b * r.H;
  float sq[4];                                  // the first 4 chunks' stats, loaded with the partials
#pragma unroll
  for (int k = 0; k < 4; ++k)
    sq[k] = threadIdx.x < 3 && c0 + k < c1 ? ld_sc1(r.chunk_stats, (int64_t)(c0 + k) * 4 + threadIdx.x) : 0.f;
  for (int x = threadIdx.x, i = 0; x < r.H; x += RG_THREADS, ++i) {
    float v = 0.f;
    if (solo) v += own[i];
    for (int c = c0; c < c1; c += 4) {          // 4 chunks' loads in flight, added in chunk order
      float q[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) q[k] = c + k < c1 ? ld_sc1(r.part, (int64_t)(c + k) * r.H + x) : 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (c + k < c1) v += q[k];
    }
    float d = 0.f;
    if (b < r.B && x < r.n_real) {              // grad_act_value
      const float av = stash ? a_sh[x] : r.a_in[rb + x];
      d = v;
      if (r.keep < 1.f && r.mask_in) d = d * ((float)(stash ? mk_sh[x] : r.mask_in[rb + x]) / r.keep);
      d = d * act_grad(r.act, av);
    }
    store_ct(r.h_out, r.h_dtype, rb + x, d);
    if (r.db_part) r.db_part[rb + x] = d * r.gscale;
  }
  if (threadIdx.x < 4) {
    float v = 0.f;
    if (threadIdx.x < 3) {
      if (solo) v += own_st;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (c0 + k < c1) v += sq[k];
      for (int c = c0 + 4; c < c1; ++c) v += ld_sc1(r.chunk_stats, (int64_t)c * 4 + threadIdx.x);
    }
    r.stats_part[(int64_t)b * 4 + threadIdx.x] = v;
    if (threadIdx.x == 0 && r.row_sse) r.row_sse[b] = v;
  }
}

// rows no chunk arrives at (padding rows b >= B, rows without targets): the reduction's outputs for an
// empty row (zero delta, bias-gradient row and stats), by one thread per row (rare)
__device__ __forceinline__ void dec_zero_rows(const OcfRowsReduceArgs& r) {
  for (int b = threadIdx.x; b < r.Bp; b += RG_THREADS) {
    if (b < r.B && r.row_cptr[b + 1] > r.row_cptr[b]) continue;
    const int64_t rb = (int64_t)b * r.H;
    for (int x = 0; x < r.H; ++x) {
      store_ct(r.h_out, r.h_dtype, rb + x, 0.f);
      if (r.db_part) r.db_part[rb + x] = 0.f;
    }
    for (int k = 0; k < 4; ++k) r.stats_part[(int64_t)b * 4 + k] = 0.f;
    if (r.row_sse) r.row_sse[b] = 0.f;
  }
}

// A group of G lanes owns one entry at a time (RG_U entries in flight); lane l holds pieces
// l, l+G, ... (PPL of them) of the weight row, so a group's load instruction reads G*16
// contiguous bytes.
// chunk c of the encoder.  wt (the fused encoder -> decoder launch, gather_encdec_kernel): the partial is stored
// write-through and the chunk counts itself in enc_arrive[b] once its stores have landed
template <typename WT, int G, int PPL, int RG_U = ocf::RG_U>
__device__ __forceinline__ void encoder_chunk(const OcfGatherArgs& a, const int c, float* red, uint32_t* enc_arrive) {
  constexpr int E = EPc<WT>::v;
  constexpr int V = PPL * E;
  constexpr int NG = RG_THREADS / G;
  const int b = a.ch_row[c], j0 = a.ch_j0[c], j1 = a.ch_j1[c];
  const int grp = threadIdx.x / G, l = threadIdx.x % G;
  const int r = a.rows[b];
  const int64_t s = r >= 0 ? a.rp[r] : 0;
  const int64_t lb = a.lboff[b];
  const WT* W = reinterpret_cast<const WT*>(a.W);
  float acc[V];
#pragma unroll
  for (int k = 0; k < V; ++k) acc[k] = 0.f;
  // entry indices one iteration ahead of the weight-row loads that depend on them
  float x[RG_U];
  int n[RG_U];
  auto idx = [&](int j) {
#pragma unroll
    for (int u = 0; u < RG_U; ++u) {
      const int ju = j + u * NG;
      const bool ok = ju < j1;
      x[u] = ok ? a.xval[lb + ju] : 0.f;
      n[u] = ok ? a.col[s + ju] : 0;
    }
  };
  idx(j0 + grp);
  for (int j = j0 + grp; j < j1; j += NG * RG_U) {
    uint4 w[RG_U][PPL];
    float xc[RG_U];
#pragma unroll
    for (int u = 0; u < RG_U; ++u) {
      xc[u] = x[u];
#pragma unroll
      for (int i = 0; i < PPL; ++i)
        w[u][i] = x[u] != 0.f ? load_piece_raw<WT>(W, a.ldw, a.w_blocked, n[u], l + G * i) : make_uint4(0, 0, 0, 0);
    }
    idx(j + NG * RG_U);
#pragma unroll
    for (int u = 0; u < RG_U; ++u)
#pragma unroll
      for (int i = 0; i < PPL; ++i) {
        float f[E];
        unpack_piece<WT>(w[u][i], f);
#pragma unroll
        for (int k = 0; k < E; ++k) acc[i * E + k] += xc[u] * f[k];
      }
  }
  reduce_groups<G, V, E, PPL>(acc, red, a.part, c, a.H, grp, l, enc_arrive != nullptr);
  if (enc_arrive) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // this wave's write-through stores have landed
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(&enc_arrive[b], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <typename WT, int G, int PPL>
__global__ void __launch_bounds__(RG_THREADS) gather_encoder_kernel(OcfGatherArgs a) {
  __shared__ float red[(RG_THREADS / G) * RG_MAX_H];
  encoder_chunk<WT, G, PPL>(a, blockIdx.x, red, nullptr);
}

// The fused encoder -> decoder launch's hand-off (gather_encdec_kernel): enc_arrive = per-row arrival counters of
// the encoder chunks; err = the library's asynchronous error word; gate / gen = the hand-off's gate word and this
// launch's generation (ocf_internal.h encdec_gate_word); max_polls < 0 = fault injection (tests): row 0's decoder
// chunks give up after their wait has completed.  enc_arrive == nullptr: not the fused launch.
struct EncDecSync {
  uint32_t* enc_arrive; uint32_t* err; uint32_t* gate; uint32_t gen; int max_polls;
};

// A decoder chunk that gave up waiting for its row's encoder chunks still counts itself in row_arrive[b], so the
// row's last chunk (this one or another) finds the count complete and returns both counters to zero; it stores
// nothing else.  The row's hidden delta is then not valid (a partial is missing): the weight-update launch that
// follows reads the gate word this launch closed and writes nothing.
__device__ __forceinline__ void dec_row_abandon(const OcfGatherArgs& a, const OcfRowsReduceArgs& r, int b,
                                                uint32_t* enc_arrive) {
  if (threadIdx.x != 0) return;
  const uint32_t nch = (uint32_t)(r.row_cptr[b + 1] - r.row_cptr[b]);
  const uint32_t old = nch == 1 ? 0u : __hip_atomic_fetch_add(&a.row_arrive[b], 1u, __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_AGENT);
  if (old + 1 == nch) {
    if (nch > 1) __hip_atomic_store(&a.row_arrive[b], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&enc_arrive[b], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// chunk c of the decoder.  enc_arrive (the fused encoder -> decoder launch): before its hidden epilogue the chunk
// waits until every encoder chunk of its row has counted itself (bounded: OCF_ASYNC_ENC_WAIT, then the chunk
// stores nothing) and reads their write-through partials with L1-bypassing loads.  Deadlock-free: the encoder
// chunks are the launch's first workgroups and workgroups dispatch in index order, so a waiting decoder chunk's
// producers are resident or done.
template <typename WT, typename HT, int G, int PPL>
__device__ __forceinline__ void decoder_chunk(const OcfGatherArgs& a, const OcfRowsReduceArgs& jr, const int c,
                                              const bool first_wg, float* red, const EncDecSync& sy) {
  constexpr int E = EPc<WT>::v;
  constexpr int V = PPL * E;
  constexpr int NG = RG_THREADS / G;
  __shared__ float st[NG][3];
  const int b = a.ch_row[c], j0 = a.ch_j0[c], j1 = a.ch_j1[c];
  const int grp = threadIdx.x / G, l = threadIdx.x % G;
  const int r = a.rows[b];
  const int64_t s = r >= 0 ? a.rp[r] : 0;
  const int64_t lb = a.lboff[b];
  const WT* W = reinterpret_cast<const WT*>(a.W);
  const float m = a.aux;
  uint32_t* const enc_arrive = sy.enc_arrive;
  if (a.zero_word && first_wg && threadIdx.x == 0)
    __hip_atomic_store(a.zero_word, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const bool fold = a.row_arrive != nullptr;
  if (fold && first_wg) dec_zero_rows(jr);
  __shared__ float a_sh[RG_MAX_H];             // (fold) the row's activation / dropout mask from the epilogue
  __shared__ uint8_t mk_sh[RG_MAX_H];
  float hv[V];
  // entry indices one iteration ahead; the bias of each entry's column loads with its weight row.  The
  // first indices load before the hidden layer's epilogue below: that chain (partials -> activation ->
  // LDS) and this one (flag / column / target) overlap instead of running back to back
  bool live[RG_UD];
  int n[RG_UD];
  float t[RG_UD];
  auto idx = [&](int j) {
#pragma unroll
    for (int u = 0; u < RG_UD; ++u) {
      const int ju = j + u * NG;
      const bool ok = ju < j1;
      live[u] = ok && a.flag[lb + ju];
      n[u] = ok ? a.col[s + ju] : 0;
      t[u] = ok ? a.val[s + ju] : 0.f;
    }
  };
  idx(j0 + grp);
  if (a.enc_part) {
    // the hidden layer's epilogue from the encoder partials (rows_reduce_kernel BIAS_ACT arithmetic); the
    // row's first chunk stores a / h / mask for the backward pass
    // once per workgroup, coalesced over the row, staged through LDS for the groups
    BiasActParams p;
    const bool first = j0 == 0;
    p.bias = a.bias_h; p.act = a.act; p.keep = a.keep; p.seed = a.seed; p.stream = a.stream; p.mask_in = nullptr;
    p.mask_out = first ? a.mask_out : nullptr; p.a_out = first ? a.a_out : nullptr;
    p.h_out = first ? const_cast<void*>(a.h) : nullptr; p.h_dtype = a.h_dtype; p.ld = a.H;
    p.m_real = a.m_real; p.n_real = a.n_real;
    const int e0 = a.enc_cptr[b], e1 = a.enc_cptr[b + 1];
    if (enc_arrive) {                 // the fused launch: this row's encoder chunks done (see above)
      __shared__ int ok_sh;
      if (threadIdx.x == 0) {
        const uint32_t want = (uint32_t)(e1 - e0);
        const int polls = sy.max_polls < 0 ? (1 << 22) : sy.max_polls;
        bool ok = __hip_atomic_load(&enc_arrive[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= want;
        for (int it = 0; !ok && it < polls; ++it) {
          __builtin_amdgcn_s_sleep(1);
          ok = __hip_atomic_load(&enc_arrive[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= want;
        }
        if (sy.max_polls < 0 && b == 0) ok = false;   // fault injection (every encoder chunk of the row is in)
        if (!ok) {
          __hip_atomic_store(sy.gate, sy.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(sy.err, (uint32_t)OCF_ASYNC_ENC_WAIT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        ok_sh = ok ? 1 : 0;
      }
      __syncthreads();
      if (!ok_sh) return dec_row_abandon(a, jr, b, enc_arrive);
    }
    for (int x = threadIdx.x; x < a.H; x += RG_THREADS) {
      // the chunk partials of 4 chunks in flight together, added in chunk order (the same sums)
      float v = 0.f;
      for (int c = e0; c < e1; c += 4) {
        float q[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
          q[k] = c + k < e1 ? (enc_arrive ? ld_sc1(a.enc_part, (int64_t)(c + k) * a.H + x)
                                          : a.enc_part[(int64_t)(c + k) * a.H + x]) : 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (c + k < e1) v += q[k];
      }
      red[x] = (float)CvtT<HT>::to(bias_act_value(p, b, x, v, fold ? &a_sh[x] : nullptr, fold ? &mk_sh[x] : nullptr));
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < PPL; ++i)
#pragma unroll
      for (int k = 0; k < E; ++k) hv[i * E + k] = red[(l + G * i) * E + k];
    __syncthreads();   // red is reused by the group reduction at the end
  } else {
#pragma unroll
    for (int i = 0; i < PPL; ++i) {
      float t[E];
      load_act_piece<HT, E>(a.h, a.H, b, l + G * i, t);
#pragma unroll
      for (int k = 0; k < E; ++k) hv[i * E + k] = t[k];
    }
  }
  float acc[V];
#pragma unroll
  for (int k = 0; k < V; ++k) acc[k] = 0.f;
  float sse = 0.f, sae = 0.f, cnt = 0.f;
  for (int j = j0 + grp; j < j1; j += NG * RG_UD) {
    uint4 w[RG_UD][PPL];
    bool lv[RG_UD];
    int nc[RG_UD];
    float tc[RG_UD], bn[RG_UD];
#pragma unroll
    for (int u = 0; u < RG_UD; ++u) {
      lv[u] = live[u];
      nc[u] = n[u];
      tc[u] = t[u];
      bn[u] = live[u] ? a.bias[n[u]] : 0.f;
#pragma unroll
      for (int i = 0; i < PPL; ++i)
        w[u][i] = live[u] ? load_piece_raw<WT>(W, a.ldw, a.w_blocked, n[u], l + G * i) : make_uint4(0, 0, 0, 0);
    }
    idx(j + NG * RG_UD);
    float dot[RG_UD];
#pragma unroll
    for (int u = 0; u < RG_UD; ++u) {
      float d0 = 0.f;
#pragma unroll
      for (int i = 0; i < PPL; ++i) {
        float f[E];
        unpack_piece<WT>(w[u][i], f);
#pragma unroll
        for (int k = 0; k < E; ++k) d0 += hv[i * E + k] * f[k];
      }
      dot[u] = d0;
    }
#pragma unroll
    for (int off = G / 2; off > 0; off >>= 1)
#pragma unroll
      for (int u = 0; u < RG_UD; ++u) dot[u] += __shfl_xor(dot[u], off, G);
#pragma unroll
    for (int u = 0; u < RG_UD; ++u) {
      const int ju = j + u * NG;
      if (ju >= j1) break;
      float d = 0.f;
      if (lv[u]) {
        const float yh = m * (dot[u] + bn[u]);
        const float err = yh - tc[u];
        d = err * m;
        if (l == 0) {
          sse += err * err;
          sae += fabsf(err);
          cnt += (tc[u] + yh != 0.f) ? 1.f : 0.f;
          if (a.d_out) store_ct(a.d_out, a.d_dtype, (int64_t)b * a.ld_d + nc[u], d);
        }
      }
      if (l == 0 && a.delta_e) a.delta_e[lb + ju] = d;
#pragma unroll
      for (int i = 0; i < PPL; ++i) {
        float f[E];
        unpack_piece<WT>(w[u][i], f);
#pragma unroll
        for (int k = 0; k < E; ++k) acc[i * E + k] += d * f[k];
      }
    }
  }
  if (l == 0) {
    st[grp][0] = sse;
    st[grp][1] = sae;
    st[grp][2] = cnt;
  }
  // (fold) a row of one chunk keeps its sums in registers: nothing to hand off
  const bool solo = fold && jr.row_cptr[b + 1] - jr.row_cptr[b] == 1;
  float own[RG_XPT];
  reduce_groups<G, V, E, PPL>(acc, red, a.part, c, a.H, grp, l, fold, solo, own);
  float own_st = 0.f;
  if (threadIdx.x < 3) {
    float v = 0.f;
    for (int g = 0; g < NG; ++g) v += st[g][threadIdx.x];
    own_st = v;
    if (solo) {
    } else if (fold) {
      st_sc1(a.chunk_stats, (int64_t)c * 4 + threadIdx.x, v);
    } else {
      a.chunk_stats[(int64_t)c * 4 + threadIdx.x] = v;
    }
  }
  if (fold) dec_row_tail(a, jr, b, a_sh, mk_sh, a.enc_part != nullptr, solo, own, own_st, enc_arrive);
}

// (f16: 133 VGPRs, bf16: 163 -- 3 waves per SIMD.  Capped at 128 by amdgpu_waves_per_eu(4) the f16 form spills 20 B
// per lane and the ML-20M step goes 0.381 -> 0.524 ms, same box, profiles/r05_decoder_cap128_ab.jsonl; an LDS-resident
// hidden row instead of the per-lane pieces does not lower the peak.  Round 4: 162 VGPRs, 144 B spilled, 0.388 ->
// 0.523 ms)
template <typename WT, typename HT, int G, int PPL>
__global__ void __launch_bounds__(RG_THREADS) gather_decoder_kernel(OcfGatherArgs a, OcfRowsReduceArgs jr) {
  __shared__ float red[(RG_THREADS / G) * RG_MAX_H];
  decoder_chunk<WT, HT, G, PPL>(a, jr, blockIdx.x, blockIdx.x == 0, red, EncDecSync{});
}

// The encoder and the decoder as ONE launch (ocf_gather_encdec): workgroups [0, e.n_chunks) are the encoder's
// chunks, the rest the decoder's; a decoder chunk starts its row as soon as that row's encoder chunks are done
// (per-row arrival counters enc_arrive, reset by the row's last decoder chunk) instead of after the whole encoder
// launch.  Needs the decoder's folded row reduction (its last chunk per row resets the counter) and the same
// chunk table for both (train batches: inputs = targets).
template <typename WT, typename HT, int G, int PPL>
__global__ void __launch_bounds__(RG_THREADS) gather_encdec_kernel(OcfGatherArgs e, OcfGatherArgs d,
                                                                   OcfRowsReduceArgs jr, EncDecSync sy) {
  __shared__ float red[(RG_THREADS / G) * RG_MAX_H];
  const int bx = blockIdx.x;
  if (bx < e.n_chunks) encoder_chunk<WT, G, PPL, RG_UE>(e, bx, red, sy.enc_arrive);
  else decoder_chunk<WT, HT, G, PPL>(d, jr, bx - e.n_chunks, bx == e.n_chunks, red, sy);
}

// The row-resident form of the encoder -> decoder launch (ocf_gather_encdec, 16-bit weights; tuning
// "encdec_rowres"): ONE 1,024-thread workgroup per batch row runs the row's whole encoder sum, the hidden epilogue,
// the decoder over the row's targets and the hidden delta's reduction, with the partial sums reduced in LDS -- no
// chunk partials through memory, no per-row arrival counters, no workgroup waiting for another.  The chunked form
// (gather_encdec_kernel) ran the row's encoder and decoder as ~3 + ~3 workgroups of 256 threads each with those
// hand-offs, at 3 waves per SIMD.  Arithmetic per entry as in encoder_chunk / decoder_chunk; the sums run over the
// row's entries in another order (per lane group, then over the groups in a fixed order), so the results equal the
// chunked form's to fp32 rounding, not bit for bit.
#ifndef OCF_RR_UD
#define OCF_RR_UD 2
#endif
#ifndef OCF_RR_UE
#define OCF_RR_UE 4
#endif
constexpr int RR_UE = OCF_RR_UE;   // entries per group in flight in the encoder part
// ... in the decoder part: 2 (115 VGPRs); 3 spilled 44 B per lane at the 1,024-thread workgroup's 128 VGPRs and
// 4 148 B.  ML-20M, same box: chunked 0.3802, row-resident with 3 0.3770, with 2 0.3626 ms/step
// (profiles/r06_rowres/).  (64-lane groups x 1 piece at 16 bits with 4 / 5 entries in flight measured slower than
// 32 x 2 with 2: ML-20M 0.3799 / 0.3775 vs 0.3667, ML-1M 0.0635 / 0.0631 vs 0.0591, Netflix 1.9549 vs 1.8555
// ms/step, profiles/r06_rowres/rr_gd64_*)
constexpr int RR_UD = OCF_RR_UD;

// what a row-resident launch does (gather_rowres_kernel MODE)
enum { RR_FULL = 0,        // ocf_gather_encdec: encoder, hidden epilogue, decoder, hidden delta (GRAD_ACT)
       RR_ENC_RAW = 1,     // a feature-parallel rank's phase 0: the encoder's row sums (RAW, before the all-reduce)
       RR_DEC_RAW = 2 };   // ... phase 1: the hidden epilogue from the all-reduced sums, the decoder, the hidden
                           // delta's row sums (RAW, before the all-reduce) and the row stats

// the groups' per-lane vectors summed into red[wave][x]: the groups of one wave by lane shuffles (a fixed xor
// tree), then the waves' rows by the caller in wave order
template <int G, int V, int E, int PPL>
__device__ __forceinline__ void rr_wave_sums(float (&acc)[V], float (*red)[RG_MAX_H], int l, int lane, int w) {
#pragma unroll
  for (int off = G; off < 64; off <<= 1)
#pragma unroll
    for (int k = 0; k < V; ++k) acc[k] += __shfl_xor(acc[k], off, 64);
  if (lane < G) {
#pragma unroll
    for (int i = 0; i < PPL; ++i)
#pragma unroll
      for (int k = 0; k < E; ++k) red[w][(l + G * i) * E + k] = acc[i * E + k];
  }
}
// a workgroup barrier for LDS hand-offs only: __syncthreads would also wait for this wave's outstanding global loads
// (the decoder's first W_out rows, requested before the encoder's reduction to overlap it)
__device__ __forceinline__ void rr_lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
template <int NW>
__device__ __forceinline__ float rr_row_sum(const float (*red)[RG_MAX_H], int x) {
  float s0 = 0.f, s1 = 0.f;
#pragma unroll
  for (int w = 0; w < NW; w += 2) {
    s0 += red[w][x];
    s1 += red[w + 1][x];
  }
  return s0 + s1;
}
// ocf_splitk_bias_act's slab sum (ocf_elem.hip sum_slabs: the same order)
__device__ __forceinline__ float rr_sum_slabs(const float* s, int splits, int64_t sstride) {
  float v0 = 0.f, v1 = 0.f, v2 = 0.f, v3 = 0.f;
  int k = 0;
  for (; k + 4 <= splits; k += 4) {
    v0 += s[(int64_t)(k + 0) * sstride];
    v1 += s[(int64_t)(k + 1) * sstride];
    v2 += s[(int64_t)(k + 2) * sstride];
    v3 += s[(int64_t)(k + 3) * sstride];
  }
  for (; k < splits; ++k) v0 += s[(int64_t)k * sstride];
  return (v0 + v1) + (v2 + v3);
}

// e: the encoder's gather arguments (RR_FULL, RR_ENC_RAW); d: the decoder's (RR_FULL, RR_DEC_RAW; its rows /
// lboff / rp give the batch rows in every mode); r: the row reduction (GRAD_ACT for RR_FULL, RAW for the others);
// hb: the hidden epilogue over the all-reduced slabs (RR_DEC_RAW)
template <typename WT, typename HT, int G, int PPL, int T, int MODE>
__global__ void __launch_bounds__(T) gather_rowres_kernel(OcfGatherArgs e, OcfGatherArgs d, OcfRowsReduceArgs r,
                                                          OcfBiasActArgs hb) {
  constexpr int E = EPc<WT>::v;
  constexpr int V = PPL * E;
  constexpr int NG = T / G;
  constexpr int NW = T / 64;
  constexpr int XPT = (RG_MAX_H + T - 1) / T;   // hidden columns per thread in the row loops
  __shared__ float red[NW][RG_MAX_H];
  __shared__ float h_sh[RG_MAX_H];
  __shared__ float a_sh[RG_MAX_H];
  __shared__ uint8_t mk_sh[RG_MAX_H];
  __shared__ float st_sh[NG][3];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int grp = tid / G, l = tid % G;
  const OcfGatherArgs& q = MODE == RR_ENC_RAW ? e : d;     // (the batch rows)
  const int H = q.H;
  const int64_t rb = (int64_t)b * H;
  if (MODE == RR_FULL && d.zero_word && b == 0 && tid == 0)
    __hip_atomic_store(d.zero_word, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int row = b < r.B ? q.rows[b] : -1;
  const int64_t lb = b < r.B ? q.lboff[b] : 0;
  const int n_e = row >= 0 ? (int)(q.lboff[b + 1] - lb) : 0;
  // (RR_DEC_RAW: the hidden epilogue runs for every row, as ocf_splitk_bias_act did)
  if (n_e == 0 && MODE != RR_DEC_RAW) {   // padding rows, rows without entries: an empty row's outputs
    for (int x = tid; x < H; x += T) {
      if (MODE == RR_FULL) {
        store_ct(r.h_out, r.h_dtype, rb + x, 0.f);
        if (r.db_part) r.db_part[rb + x] = 0.f;
      } else {
        r.out[rb + x] = 0.f;
      }
    }
    if (MODE == RR_FULL) {
      if (tid < 4) r.stats_part[(int64_t)b * 4 + tid] = 0.f;
      if (tid == 0 && r.row_sse) r.row_sse[b] = 0.f;
    }
    return;
  }
  const int64_t s = n_e > 0 ? q.rp[row] : 0;
  // ---- encoder: hpre[x] = sum over the row's live inputs of x * W1[n][x]
  if constexpr (MODE != RR_DEC_RAW) {
    const WT* W = reinterpret_cast<const WT*>(e.W);
    float acc[V];
#pragma unroll
    for (int k = 0; k < V; ++k) acc[k] = 0.f;
    float xv[RR_UE];
    int nn[RR_UE];
    auto idx = [&](int j) {
#pragma unroll
      for (int u = 0; u < RR_UE; ++u) {
        const int ju = j + u * NG;
        const bool ok = ju < n_e;
        xv[u] = ok ? e.xval[lb + ju] : 0.f;
        nn[u] = ok ? e.col[s + ju] : 0;
      }
    };
    idx(grp);
    for (int j = grp; j < n_e; j += NG * RR_UE) {
      uint4 wv[RR_UE][PPL];
      float xc[RR_UE];
#pragma unroll
      for (int u = 0; u < RR_UE; ++u) {
        xc[u] = xv[u];
#pragma unroll
        for (int i = 0; i < PPL; ++i)
          wv[u][i] = xv[u] != 0.f ? load_piece_raw<WT>(W, e.ldw, e.w_blocked, nn[u], l + G * i) : make_uint4(0, 0, 0, 0);
      }
      idx(j + NG * RR_UE);
#pragma unroll
      for (int u = 0; u < RR_UE; ++u)
#pragma unroll
        for (int i = 0; i < PPL; ++i) {
          float f[E];
          unpack_piece<WT>(wv[u][i], f);
#pragma unroll
          for (int k = 0; k < E; ++k) acc[i * E + k] += xc[u] * f[k];
        }
    }
    rr_wave_sums<G, V, E, PPL>(acc, red, l, lane, w);
  }
  if constexpr (MODE == RR_ENC_RAW) {
    __syncthreads();
    for (int x = tid; x < H; x += T) r.out[rb + x] = rr_row_sum<NW>(red, x);
    return;
  }
  // the hidden epilogue's inputs, loaded before the decoder's first rows (a wait for them would otherwise also wait
  // for the rows requested after them): the bias, and (RR_DEC_RAW) the all-reduced sums
  BiasActParams p;
  if constexpr (MODE == RR_FULL) {
    p.bias = d.bias_h; p.act = d.act; p.keep = d.keep; p.seed = d.seed; p.stream = d.stream; p.mask_in = nullptr;
    p.mask_out = d.mask_out; p.a_out = d.a_out; p.h_out = const_cast<void*>(d.h); p.h_dtype = d.h_dtype;
    p.ld = H; p.m_real = d.m_real; p.n_real = d.n_real;
  } else {
    p.bias = hb.bias; p.act = hb.act; p.keep = hb.keep; p.seed = hb.seed; p.stream = hb.stream;
    p.mask_in = hb.mask_in; p.mask_out = hb.mask_out; p.a_out = hb.a_out; p.h_out = hb.h_out; p.h_dtype = hb.h_dtype;
    p.ld = hb.ld; p.m_real = hb.m_real; p.n_real = hb.n_real;
  }
  float bh[XPT], vin[XPT];
#pragma unroll
  for (int i = 0; i < XPT; ++i) {
    const int x = tid + i * T;
    const bool lv = x < H && b < p.m_real && x < p.n_real;
    bh[i] = lv ? p.bias[x] : 0.f;
    vin[i] = 0.f;
    if constexpr (MODE == RR_DEC_RAW)
      if (x < H) vin[i] = rr_sum_slabs(hb.slabs + (int64_t)b * hb.ld + x, hb.splits, hb.split_stride);
  }
  // the decoder's first entries: indices and W_out rows requested now, in flight across the encoder's reduction
  // and the hidden epilogue (they do not depend on h)
  const WT* Wd = reinterpret_cast<const WT*>(d.W);
  bool live[RR_UD];
  int n[RR_UD];
  float t[RR_UD];
  // branch-free: every load issued (indices clamped to the row, results masked at use), so the compiler can count
  // them and a wait for an early load does not wait for the rows requested after it
  // (an empty row, RR_DEC_RAW only: entry 0 of the tables stands in; nothing of it is used)
  const int64_t lbq = n_e > 0 ? lb : 0;
  auto idx_d = [&](int j) {
#pragma unroll
    for (int u = 0; u < RR_UD; ++u) {
      const int ju = j + u * NG;
      const int jc = max(min(ju, n_e - 1), 0);
      const uint8_t fl = d.flag[lbq + jc];
      const int nn = d.col[s + jc];
      live[u] = ju < n_e && fl;
      n[u] = live[u] ? nn : 0;                 // (not a live target: row 0, an L2 hit, instead of its own row)
      t[u] = d.val[s + jc];
    }
  };
  uint4 wv[RR_UD][PPL];
  float bn[RR_UD];
  auto load_d = [&]() {
#pragma unroll
    for (int u = 0; u < RR_UD; ++u) {
      bn[u] = d.bias[n[u]];
#pragma unroll
      for (int i = 0; i < PPL; ++i) wv[u][i] = load_piece_raw<WT>(Wd, d.ldw, d.w_blocked, n[u], l + G * i);
    }
  };
  idx_d(grp);
  load_d();
  if constexpr (MODE == RR_FULL) rr_lds_barrier();
  // ---- hidden epilogue (bias_act_value's arithmetic with the bias already loaded): a, mask, h stored for the
  //      backward pass
#pragma unroll
  for (int i = 0; i < XPT; ++i) {
    const int x = tid + i * T;
    if (x >= H) break;
    const int64_t ix = (int64_t)b * p.ld + x;
    const bool lv = b < p.m_real && x < p.n_real;
    float v = vin[i];
    if constexpr (MODE == RR_FULL) v = rr_row_sum<NW>(red, x);
    const float av = lv ? act_apply(p.act, v + bh[i]) : 0.f;
    float hvx = av;
    a_sh[x] = av;
    if (p.keep < 1.f) {
      uint8_t mk;
      if (p.mask_in) mk = p.mask_in[ix];
      else mk = (uint8_t)floorf(p.keep + philox_uniform(p.seed, p.stream, (uint64_t)ix));
      hvx = (av / p.keep) * (float)mk;
      if (p.mask_out) p.mask_out[ix] = mk;
      mk_sh[x] = mk;
    }
    if (p.a_out) p.a_out[ix] = av;
    if (p.h_out) store_ct(p.h_out, p.h_dtype, ix, hvx);
    h_sh[x] = (float)CvtT<HT>::to(hvx);
  }
  rr_lds_barrier();
  // ---- decoder: at every live target y = m (h . W_out[n] + b_out[n]), err = y - t, delta = err m;
  //      dh[x] = sum of delta * W_out[n][x]
  {
    const float m = d.aux;
    float acc[V];
#pragma unroll
    for (int k = 0; k < V; ++k) acc[k] = 0.f;
    float sse = 0.f, sae = 0.f, cnt = 0.f;
    for (int j = grp; j < n_e; j += NG * RR_UD) {
      // this iteration's entries (their W_out rows were requested at the end of the previous one)
      bool lv[RR_UD];
      int nc[RR_UD];
      float tc[RR_UD];
#pragma unroll
      for (int u = 0; u < RR_UD; ++u) {
        lv[u] = live[u];
        nc[u] = n[u];
        tc[u] = t[u];
      }
      idx_d(j + NG * RR_UD);
      // the hidden row's pieces from LDS one at a time (held in registers for the whole loop they spilled)
      float dot[RR_UD];
#pragma unroll
      for (int u = 0; u < RR_UD; ++u) dot[u] = 0.f;
#pragma unroll
      for (int i = 0; i < PPL; ++i) {
        float hh[E];
#pragma unroll
        for (int k = 0; k < E; ++k) hh[k] = h_sh[(l + G * i) * E + k];
#pragma unroll
        for (int u = 0; u < RR_UD; ++u) {
          float f[E];
          unpack_piece<WT>(wv[u][i], f);
#pragma unroll
          for (int k = 0; k < E; ++k) dot[u] += hh[k] * f[k];
        }
      }
#pragma unroll
      for (int off = G / 2; off > 0; off >>= 1)
#pragma unroll
        for (int u = 0; u < RR_UD; ++u) dot[u] += __shfl_xor(dot[u], off, G);
#pragma unroll
      for (int u = 0; u < RR_UD; ++u) {
        const int ju = j + u * NG;
        if (ju >= n_e) break;
        float dl = 0.f;
        if (lv[u]) {
          const float yh = m * (dot[u] + bn[u]);
          const float err = yh - tc[u];
          dl = err * m;
          if (l == 0) {
            sse += err * err;
            sae += fabsf(err);
            cnt += (tc[u] + yh != 0.f) ? 1.f : 0.f;
            if (d.d_out) store_ct(d.d_out, d.d_dtype, (int64_t)b * d.ld_d + nc[u], dl);
          }
        }
        if (l == 0 && d.delta_e) d.delta_e[lb + ju] = dl;
#pragma unroll
        for (int i = 0; i < PPL; ++i) {
          float f[E];
          unpack_piece<WT>(wv[u][i], f);
#pragma unroll
          for (int k = 0; k < E; ++k) acc[i * E + k] += dl * f[k];
        }
      }
      load_d();                        // the next iteration's rows (none past the row's end: live is false there)
    }
    if (l == 0) {
      st_sh[grp][0] = sse;
      st_sh[grp][1] = sae;
      st_sh[grp][2] = cnt;
    }
    __syncthreads();                 // (every wave is done reading red's encoder sums: the epilogue's barrier)
    rr_wave_sums<G, V, E, PPL>(acc, red, l, lane, w);
  }
  __syncthreads();
  // ---- the hidden delta (rows_reduce_kernel GRAD_ACT arithmetic; RR_DEC_RAW: the row sums) and the row's stats
  for (int x = tid; x < H; x += T) {
    const float v = rr_row_sum<NW>(red, x);
    if constexpr (MODE == RR_DEC_RAW) {
      r.out[rb + x] = v;
    } else {
      float dv = 0.f;
      if (x < r.n_real) {
        dv = v;
        if (r.keep < 1.f && r.mask_in) dv = dv * ((float)mk_sh[x] / r.keep);
        dv = dv * act_grad(r.act, a_sh[x]);
      }
      store_ct(r.h_out, r.h_dtype, rb + x, dv);
      if (r.db_part) r.db_part[rb + x] = dv * r.gscale;
    }
  }
  if (tid < 4) {
    float v = 0.f;
    if (tid < 3)
      for (int g = 0; g < NG; ++g) v += st_sh[g][tid];
    r.stats_part[(int64_t)b * 4 + tid] = v;
    if (tid == 0 && r.row_sse) r.row_sse[b] = v;
  }
}

// per batch row: fixed-order sum of its chunk partials, then the layer epilogue
__global__ void __launch_bounds__(256) rows_reduce_kernel(OcfRowsReduceArgs a) {
  const int b = blockIdx.x;
  const bool real = b < a.B;
  const int c0 = real ? a.row_cptr[b] : 0, c1 = real ? a.row_cptr[b + 1] : 0;
  for (int x = threadIdx.x; x < a.H; x += blockDim.x) {
    // 8 chunks' loads in flight, added in chunk order (the same sums: rows of many chunks -- Netflix's ~22 --
    // waited a round trip per chunk)
    float v = 0.f;
    for (int c = c0; c < c1; c += 8) {
      float q[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) q[k] = c + k < c1 ? a.part[(int64_t)(c + k) * a.H + x] : 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (c + k < c1) v += q[k];
    }
    if (a.mode == OCF_REDUCE_RAW) {
      a.out[(int64_t)b * a.H + x] = v;
    } else if (a.mode == OCF_REDUCE_BIAS_ACT) {
      BiasActParams p;
      p.bias = a.bias; p.act = a.act; p.keep = a.keep; p.seed = a.seed; p.stream = a.stream;
      p.mask_in = a.mask_in; p.mask_out = a.mask_out; p.a_out = a.a_out; p.h_out = a.h_out;
      p.h_dtype = a.h_dtype; p.ld = a.H; p.m_real = a.B; p.n_real = a.n_real;
      bias_act_store(p, b, x, v);
    } else {
      GradActParams p;
      p.a = a.a_in; p.mask = a.mask_in; p.keep = a.keep; p.act = a.act; p.d_out = a.h_out; p.d_dtype = a.h_dtype;
      p.ld = a.H; p.db_part = nullptr; p.gscale = a.gscale; p.m_real = a.B; p.n_real = a.n_real;
      const float d = grad_act_value(p, b, x, v);
      store_ct(a.h_out, a.h_dtype, (int64_t)b * a.H + x, d);
      if (a.db_part) a.db_part[(int64_t)b * a.H + x] = d * a.gscale;
    }
  }
  if (a.chunk_stats && threadIdx.x < 4) {
    float v = 0.f;
    if (threadIdx.x < 3)
      for (int c = c0; c < c1; c += 8) {
        float q[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) q[k] = c + k < c1 ? a.chunk_stats[(int64_t)(c + k) * 4 + threadIdx.x] : 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if (c + k < c1) v += q[k];
      }
    a.stats_part[(int64_t)b * 4 + threadIdx.x] = v;
    if (threadIdx.x == 0 && a.row_sse) a.row_sse[b] = v;
  }
}

// (group width G, pieces per lane PPL) for a row of H elements of WT: the widest group (<= 64
// lanes) that the row's 16-byte pieces fill
template <typename WT> bool gather_shape(int H, int& G, int& ppl) {
  const int pieces = H / EPc<WT>::v;
  // group width cap: 32 lanes x 2 pieces per entry beat 64 x 1 at H = 512 (ML-20M step: decoder
  // 72 -> 55 us, encoder 57 -> 50 us): twice the entries in flight per workgroup and one shuffle
  // step less per dot product.
  constexpr int gmax = 32;
  for (int g : {64, 32, 16})
    if (g <= gmax && pieces % g == 0 && pieces / g <= 4) {
      G = g;
      ppl = pieces / g;
      return true;
    }
  for (int g : {64, 32, 16})
    if (pieces % g == 0) {
      G = g;
      ppl = pieces / g;
      return ppl <= 3;
    }
  return false;
}

template <template <int, int> class L>
void by_shape(int G, int ppl, const OcfGatherArgs& a, hipStream_t s) {
  if (G == 64 && ppl == 1) L<64, 1>::go(a, s);
  else if (G == 64 && ppl == 2) L<64, 2>::go(a, s);
  else if (G == 32 && ppl == 1) L<32, 1>::go(a, s);
  else if (G == 32 && ppl == 2) L<32, 2>::go(a, s);
  else if (G == 16 && ppl == 4) L<16, 4>::go(a, s);
  else if (G == 32 && ppl == 4) L<32, 4>::go(a, s);   // fp32 weights, H = 512 (exact-fp32 mode at 500 units)
  else if (G == 32 && ppl == 3) L<32, 3>::go(a, s);
  else if (G == 16 && ppl == 1) L<16, 1>::go(a, s);
  else if (G == 16 && ppl == 3) L<16, 3>::go(a, s);
  else throw std::runtime_error("row gather: unsupported H / weight dtype combination");
}

template <typename WT> struct Enc {
  template <int G, int P> struct L {
    static void go(const OcfGatherArgs& a, hipStream_t s) {
      hipLaunchKernelGGL((gather_encoder_kernel<WT, G, P>), dim3(a.n_chunks), dim3(RG_THREADS), 0, s, a);
    }
  };
};
template <typename WT, typename HT> struct Dec {
  template <int G, int P> struct L {
    static void go(const OcfGatherArgs& a, hipStream_t s) {
      OcfRowsReduceArgs r{};
      if (a.jr && a.row_arrive) r = *a.jr;
      hipLaunchKernelGGL((gather_decoder_kernel<WT, HT, G, P>), dim3(a.n_chunks), dim3(RG_THREADS), 0, s, a, r);
    }
  };
};

template <typename WT, typename HT>
void launch_encdec(int G, int ppl, const OcfGatherArgs& e, const OcfGatherArgs& d, const EncDecSync& sy, hipStream_t s) {
  OcfRowsReduceArgs r = *d.jr;
  const dim3 grid(e.n_chunks + d.n_chunks), blk(RG_THREADS);
#define OCF_ED(GG, PP) hipLaunchKernelGGL((gather_encdec_kernel<WT, HT, GG, PP>), grid, blk, 0, s, e, d, r, sy)
  if (G == 64 && ppl == 1) OCF_ED(64, 1);
  else if (G == 64 && ppl == 2) OCF_ED(64, 2);
  else if (G == 32 && ppl == 1) OCF_ED(32, 1);
  else if (G == 32 && ppl == 2) OCF_ED(32, 2);
  else if (G == 16 && ppl == 4) OCF_ED(16, 4);
  else if (G == 32 && ppl == 4) OCF_ED(32, 4);
  else if (G == 32 && ppl == 3) OCF_ED(32, 3);
  else if (G == 16 && ppl == 1) OCF_ED(16, 1);
  else if (G == 16 && ppl == 3) OCF_ED(16, 3);
  else throw std::runtime_error("row gather: unsupported H / weight dtype combination");
#undef OCF_ED
}

template <typename WT, typename HT, int T, int MODE>
void launch_rowres_t(int G, int ppl, const OcfGatherArgs& e, const OcfGatherArgs& d, const OcfRowsReduceArgs& r,
                     const OcfBiasActArgs& hb, hipStream_t s) {
  const dim3 grid(r.Bp), blk(T);
#define OCF_RR(GG, PP) hipLaunchKernelGGL((gather_rowres_kernel<WT, HT, GG, PP, T, MODE>), grid, blk, 0, s, e, d, r, hb)
  if (G == 32 && ppl == 2) OCF_RR(32, 2);
  else if (G == 64 && ppl == 2) OCF_RR(64, 2);
  else if (G == 64 && ppl == 1) OCF_RR(64, 1);
  else if (G == 32 && ppl == 1) OCF_RR(32, 1);
  else if (G == 16 && ppl == 1) OCF_RR(16, 1);
  else throw std::runtime_error("row gather (row-resident): unsupported H / weight dtype combination");
#undef OCF_RR
}
// T threads per row: 1,024 for ocf_gather_encdec's rows (hundreds of entries), 256 for a feature rank's rows of a
// column shard (~1/G of them)
template <int MODE>
void launch_rowres(int dtype, int H, int T, const OcfGatherArgs& e, const OcfGatherArgs& d,
                   const OcfRowsReduceArgs& r, const OcfBiasActArgs& hb, hipStream_t s) {
  int G, ppl;
  if (dtype == OCF_F32) {
    G = 64;
    ppl = H / 256;
  } else if (!(dtype == OCF_F16 ? gather_shape<_Float16>(H, G, ppl) : gather_shape<__bf16>(H, G, ppl))) {
    throw std::runtime_error("row gather (row-resident): unsupported H");
  }
  auto go = [&](auto wt) {
    using WT = decltype(wt);
    if (T == 256) launch_rowres_t<WT, WT, 256, MODE>(G, ppl, e, d, r, hb, s);
    else launch_rowres_t<WT, WT, 1024, MODE>(G, ppl, e, d, r, hb, s);
  };
  if (dtype == OCF_F32) go(float{});
  else if (dtype == OCF_F16) go(_Float16{});
  else go(__bf16{});
}
// (H = 384 at 16 bits, 16 lanes x 3 pieces, would spill: the chunked forms)
bool rowres_shape_ok(int dtype, int H) { return dtype == OCF_F32 ? H % 256 == 0 : H != 384; }

void check_gather(const OcfGatherArgs& a, const char* who) {
  OCF_CHECK(a.rows && a.rp && a.col && a.lboff && a.ch_row && a.ch_j0 && a.ch_j1 && a.W && a.part,
            std::string(who) + ": null pointer");
  OCF_CHECK(a.H > 0 && a.H <= RG_MAX_H && a.H % 128 == 0, std::string(who) + ": H must be a multiple of 128, <= 512");
  OCF_CHECK(a.w_dtype == OCF_F32 || a.w_dtype == OCF_F16 || a.w_dtype == OCF_BF16, std::string(who) + ": w_dtype");
  OCF_CHECK(!a.w_blocked || a.w_dtype != OCF_F32, std::string(who) + ": blocked weights are 16-bit");
  OCF_CHECK(a.ldw >= a.H && a.ldw % 8 == 0, std::string(who) + ": ldw");
}

template <typename WT> void shape_or_throw(const OcfGatherArgs& a, int& G, int& ppl) {
  if (!gather_shape<WT>(a.H, G, ppl)) throw std::runtime_error("row gather: unsupported H " + std::to_string(a.H));
}

}  // namespace ocf

using namespace ocf;

extern "C" int ocf_gather_encoder(const OcfGatherArgs* args, void* stream) {
  OCF_TRY_BEGIN
  const OcfGatherArgs& a = *args;
  check_gather(a, "ocf_gather_encoder");
  OCF_CHECK(a.xval != nullptr, "ocf_gather_encoder: xval required");
  if (a.n_chunks == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  int G, ppl;
  if (a.w_dtype == OCF_F32) { shape_or_throw<float>(a, G, ppl); by_shape<Enc<float>::L>(G, ppl, a, s); }
  else if (a.w_dtype == OCF_F16) { shape_or_throw<_Float16>(a, G, ppl); by_shape<Enc<_Float16>::L>(G, ppl, a, s); }
  else { shape_or_throw<__bf16>(a, G, ppl); by_shape<Enc<__bf16>::L>(G, ppl, a, s); }
  OCF_HIP(hipGetLastError());
  OCF_TRY_END
}

extern "C" int ocf_gather_decoder(const OcfGatherArgs* args, void* stream) {
  OCF_TRY_BEGIN
  const OcfGatherArgs& a = *args;
  check_gather(a, "ocf_gather_decoder");
  OCF_CHECK(a.flag && a.val && a.h && a.bias && a.chunk_stats, "ocf_gather_decoder: flag/val/h/bias/chunk_stats required");
  OCF_CHECK(a.h_dtype == a.w_dtype, "ocf_gather_decoder: h and W must share the compute dtype");
  OCF_CHECK(!a.enc_part || (a.enc_cptr && a.bias_h && (a.keep >= 1.f || a.mask_out) && a.a_out),
            "ocf_gather_decoder: enc_part needs enc_cptr, bias_h, a_out and (with dropout) mask_out");
  OCF_CHECK(!a.jr == !a.row_arrive, "ocf_gather_decoder: jr and row_arrive go together");
  if (a.jr) {
    const OcfRowsReduceArgs& r = *a.jr;
    OCF_CHECK(r.mode == OCF_REDUCE_GRAD_ACT && r.part == a.part && r.chunk_stats == a.chunk_stats && r.H == a.H &&
                  r.row_cptr && r.h_out && r.a_in && r.stats_part && r.B <= r.Bp && (r.keep >= 1.f || r.mask_in),
              "ocf_gather_decoder: jr must be OCF_REDUCE_GRAD_ACT over this launch's part / chunk_stats (same H) "
              "with row_cptr, h_out, a_in, stats_part and (with dropout) mask_in");
  }
  if (a.n_chunks == 0) {
    OCF_CHECK(!a.jr, "ocf_gather_decoder: a folded row reduction needs at least one chunk");
    return 0;
  }
  hipStream_t s = (hipStream_t)stream;
  int G, ppl;
  if (a.w_dtype == OCF_F32) { shape_or_throw<float>(a, G, ppl); by_shape<Dec<float, float>::L>(G, ppl, a, s); }
  else if (a.w_dtype == OCF_F16) {
    shape_or_throw<_Float16>(a, G, ppl);
    by_shape<Dec<_Float16, _Float16>::L>(G, ppl, a, s);
  } else {
    shape_or_throw<__bf16>(a, G, ppl);
    by_shape<Dec<__bf16, __bf16>::L>(G, ppl, a, s);
  }
  OCF_HIP(hipGetLastError());
  OCF_TRY_END
}

namespace ocf {
int g_encdec_max_polls = 1 << 22;   // ocf_gather_encdec's bounded wait (ocf_set_tuning "encdec_max_polls")
// ocf_gather_encdec's row-resident form for 16-bit weights (ocf_set_tuning "encdec_rowres"; env OCF_ENCDEC_ROWRES)
int g_encdec_rowres = [] {
  const char* v = std::getenv("OCF_ENCDEC_ROWRES");
  return v ? std::atoi(v) : 1;
}();
}

extern "C" int ocf_gather_encdec(const OcfGatherArgs* enc, const OcfGatherArgs* dec, uint32_t* enc_arrive,
                                 void* stream) {
  OCF_TRY_BEGIN
  OCF_CHECK(enc && dec && enc_arrive, "ocf_gather_encdec: null arguments");
  const OcfGatherArgs& e = *enc;
  const OcfGatherArgs& d = *dec;
  check_gather(e, "ocf_gather_encdec (encoder)");
  check_gather(d, "ocf_gather_encdec (decoder)");
  OCF_CHECK(e.xval != nullptr, "ocf_gather_encdec: xval required");
  OCF_CHECK(d.flag && d.val && d.h && d.bias && d.chunk_stats, "ocf_gather_encdec: flag/val/h/bias/chunk_stats required");
  OCF_CHECK(d.h_dtype == d.w_dtype && e.w_dtype == d.w_dtype && e.H == d.H, "ocf_gather_encdec: one dtype and H");
  OCF_CHECK(d.enc_part == e.part && d.enc_cptr && d.bias_h && (d.keep >= 1.f || d.mask_out) && d.a_out,
            "ocf_gather_encdec: dec.enc_part must be enc.part, with enc_cptr, bias_h, a_out (and mask_out)");
  OCF_CHECK(d.jr && d.row_arrive, "ocf_gather_encdec: the decoder's folded row reduction (jr, row_arrive) is required");
  OCF_CHECK(e.ch_row == d.ch_row && e.ch_j0 == d.ch_j0 && e.ch_j1 == d.ch_j1 && e.n_chunks == d.n_chunks &&
                e.rows == d.rows && e.lboff == d.lboff && e.rp == d.rp,
            "ocf_gather_encdec: the encoder and the decoder must share the batch's chunk table");
  const OcfRowsReduceArgs& r = *d.jr;
  OCF_CHECK(r.mode == OCF_REDUCE_GRAD_ACT && r.part == d.part && r.chunk_stats == d.chunk_stats && r.H == d.H &&
                r.row_cptr && r.h_out && r.a_in && r.stats_part && r.B <= r.Bp && (r.keep >= 1.f || r.mask_in),
            "ocf_gather_encdec: jr must be OCF_REDUCE_GRAD_ACT over the decoder's part / chunk_stats");
  if (d.n_chunks == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  int G, ppl;
  // one workgroup per batch row: no hand-offs.  fp32 rows (2 KB at H = 512) as one 64-lane group per entry
  // (32 lanes x 4 pieces would not fit the 1,024-thread workgroup's 128 VGPRs)
  if (g_encdec_rowres && r.Bp > 0 && rowres_shape_ok(d.w_dtype, d.H)) {
    launch_rowres<RR_FULL>(d.w_dtype, d.H, 1024, e, d, r, OcfBiasActArgs{}, s);
    OCF_HIP(hipGetLastError());
    return 0;
  }
  EncDecSync sy{enc_arrive, async_error_word(), nullptr, 0, g_encdec_max_polls};
  sy.gen = next_encdec_generation();
  sy.gate = encdec_gate_word();
  if (d.w_dtype == OCF_F32) { shape_or_throw<float>(d, G, ppl); launch_encdec<float, float>(G, ppl, e, d, sy, s); }
  else if (d.w_dtype == OCF_F16) { shape_or_throw<_Float16>(d, G, ppl); launch_encdec<_Float16, _Float16>(G, ppl, e, d, sy, s); }
  else { shape_or_throw<__bf16>(d, G, ppl); launch_encdec<__bf16, __bf16>(G, ppl, e, d, sy, s); }
  OCF_HIP(hipGetLastError());
  OCF_TRY_END
}

namespace ocf {
// A feature-parallel rank's gathers in the row-resident form (ocf_rank_step phases 0 / 1, "encdec_rowres"):
// phase 0's encoder + RAW row reduction as one launch, phase 1's hidden epilogue (ocf_splitk_bias_act) + decoder +
// RAW row reduction + row stats as one launch.  false: the arguments do not fit the form (the caller issues the
// separate launches).  Rows of a column shard are short (~1/G of a row): 256 threads per row when the chunk table
// holds about one chunk per row.
bool rank_rowres_enc(const OcfGatherArgs& e, const OcfRowsReduceArgs& r, hipStream_t s) {
  if (!(g_encdec_rowres && rowres_shape_ok(e.w_dtype, e.H) && r.mode == OCF_REDUCE_RAW && r.out && r.H == e.H &&
        e.xval && r.Bp > 0 && r.B <= r.Bp && e.n_chunks > 0))
    return false;
  check_gather(e, "ocf_rank_step (row-resident encoder)");
  const int T = e.n_chunks <= 2 * r.B ? 256 : 1024;
  launch_rowres<RR_ENC_RAW>(e.w_dtype, e.H, T, e, e, r, OcfBiasActArgs{}, s);
  OCF_HIP(hipGetLastError());
  return true;
}
bool rank_rowres_dec(const OcfBiasActArgs& hb, const OcfGatherArgs& d, const OcfRowsReduceArgs& r, hipStream_t s) {
  if (!(g_encdec_rowres && rowres_shape_ok(d.w_dtype, d.H) && r.mode == OCF_REDUCE_RAW && r.out && r.H == d.H &&
        r.stats_part && r.Bp > 0 && r.B <= r.Bp && d.n_chunks > 0 && !d.enc_part && !d.jr && d.flag && d.val &&
        d.bias && hb.slabs && hb.splits >= 1 && hb.M == r.Bp && hb.N == d.H && hb.ld >= d.H && hb.bias &&
        d.h_dtype == d.w_dtype && hb.h_dtype == d.w_dtype && (hb.keep >= 1.f || hb.mask_out || hb.mask_in)))
    return false;
  check_gather(d, "ocf_rank_step (row-resident decoder)");
  const int T = d.n_chunks <= 2 * r.B ? 256 : 1024;
  launch_rowres<RR_DEC_RAW>(d.w_dtype, d.H, T, d, d, r, hb, s);
  OCF_HIP(hipGetLastError());
  return true;
}
}  // namespace ocf

extern "C" int ocf_rows_reduce(const OcfRowsReduceArgs* args, void* stream) {
  OCF_TRY_BEGIN
  const OcfRowsReduceArgs& a = *args;
  OCF_CHECK(a.part && a.row_cptr && a.H > 0 && a.B <= a.Bp, "ocf_rows_reduce: bad arguments");
  OCF_CHECK(a.mode != OCF_REDUCE_RAW || a.out, "ocf_rows_reduce: RAW needs out");
  OCF_CHECK(a.mode == OCF_REDUCE_RAW || a.h_out, "ocf_rows_reduce: BIAS_ACT / GRAD_ACT need h_out");
  OCF_CHECK(!a.chunk_stats || a.stats_part, "ocf_rows_reduce: chunk_stats needs stats_part");
  if (a.Bp == 0) return 0;
  hipLaunchKernelGGL(rows_reduce_kernel, dim3(a.Bp), dim3(256), 0, (hipStream_t)stream, a);
  OCF_HIP(hipGetLastError());
  OCF_TRY_END
}

// output-bias gradient from a dense delta: db[n] = gscale * sum_{b < B} d[b][n] (fixed order)
namespace ocf {
__global__ void __launch_bounds__(256) colsum_kernel(const void* d, int dtype, int64_t ld, int B, int N, float gscale,
                                                     float* out) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  float s0 = 0.f, s1 = 0.f;
  int b = 0;
  for (; b + 2 <= B; b += 2) {
    s0 += load_ct(d, dtype, (int64_t)b * ld + n);
    s1 += load_ct(d, dtype, (int64_t)(b + 1) * ld + n);
  }
  if (b < B) s0 += load_ct(d, dtype, (int64_t)b * ld + n);
  out[n] = (s0 + s1) * gscale;
}
}  // namespace ocf

extern "C" int ocf_colsum(const void* d, int dtype, int64_t ld, int B, int N, float gscale, float* out, void* stream) {
  OCF_TRY_BEGIN
  OCF_CHECK(d && out && ld >= N, "ocf_colsum: bad arguments");
  if (N == 0) return 0;
  hipLaunchKernelGGL(colsum_kernel, dim3((N + 255) / 256), dim3(256), 0, (hipStream_t)stream, d, dtype, ld, B, N, gscale,
                     out);
  OCF_HIP(hipGetLastError());
  OCF_TRY_END
}

// ---------------------------------------------------------------------------------------
// (M tile, K-step) buckets of a batch's sparse A operand for the persistent dW kernel.
// Pass 1: one wave per bucket (t, kt), lane = batch row b - 64 kt, counts.  Pass 2: one workgroup
// per tile writes each lane's tile segment at its wave-prefix offset (rows in order, entries in
// column order): deterministic, no atomics.
namespace ocf {

struct TbSeg {
  int64_t e0;   // first entry of row r's tile-t segment (column-sorted view)
  int n;        // entries in it
  int64_t lb;   // value index base of batch row b
};

__device__ __forceinline__ TbSeg tb_segment(const OcfTileBucketArgs& a, int t, int b) {
  TbSeg s{0, 0, 0};
  if (b >= a.krows) return s;
  const int r = a.rows[b];
  if (r < 0) return s;
  const int32_t* tp = a.tptr + (int64_t)r * (a.ntiles + 1) + t;
  s.e0 = a.rp[r] + tp[0];
  s.n = tp[1] - tp[0];
  s.lb = a.lboff[b];
  return s;
}

__device__ __forceinline__ int wave_incl_scan(int v, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int u = __shfl_up(v, d, 64);
    if (lane >= d) v += u;
  }
  return v;
}

__global__ void __launch_bounds__(256) tb_count_kernel(OcfTileBucketArgs a) {
  const int lane = threadIdx.x & 63;
  const int id = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (id >= a.gm * a.nk) return;
  const int t = id / a.nk, kt = id % a.nk;
  const TbSeg s = tb_segment(a, t, kt * 64 + lane);
  const int tot = __shfl(wave_incl_scan(s.n, lane), 63, 64);
  if (lane == 0) a.cnt[id] = tot;
}

// live-row record of tile t (ocf.h OCF_LIVE_REC) from a tag array, by one wave: rank k of a live row =
// live rows before it in the tile
__device__ __forceinline__ void live_record(const uint8_t* tags, uint8_t* rec, int rtag, int lane) {
  const bool l0 = tags[lane] == (uint8_t)rtag, l1 = tags[64 + lane] == (uint8_t)rtag;
  const uint64_t b0 = __ballot(l0), b1 = __ballot(l1), below = (1ull << lane) - 1;
  const int n0 = __popcll(b0);
  const int k0 = __popcll(b0 & below), k1 = n0 + __popcll(b1 & below);
  if (l0) rec[16 + (k0 & 7) * 16 + (k0 >> 3)] = (uint8_t)lane;
  if (l1) rec[16 + (k1 & 7) * 16 + (k1 >> 3)] = (uint8_t)(64 + lane);
  if (lane == 0) *reinterpret_cast<int*>(rec) = n0 + __popcll(b1);
}

// Row lists of tile t (ocf.h OcfTileBucketArgs row_ptr / row_ent), from the tile's buckets just
// written by this workgroup (entries in (K-step, batch row, column) order): a stable counting sort by
// column.  Per chunk of 256 entries an entry's rank among the earlier same-column entries is counted
// inside its wave by lane reads (no LDS traffic) plus the same-column counts of the earlier waves, so
// every column's list is in batch-row order without atomics deciding the order.
__device__ void tb_rows(const OcfTileBucketArgs& a, int t, int tile_base) {
  __shared__ int cnt_m[128], base_m[128], kofs[65];
  __shared__ int wcnt[4][128];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nk = a.nk, before = t * nk;
  if (tid < 128) cnt_m[tid] = 0;
  if (tid <= nk) kofs[tid] = 0;
  __syncthreads();
  if (tid < 64) {                       // bucket offsets of the tile, relative to its first entry
    const int v = tid < nk ? a.cnt[before + tid] : 0;
    const int incl = wave_incl_scan(v, tid);
    if (tid < nk) kofs[tid] = incl - v;
    if (tid == nk - 1) kofs[nk] = incl;
  }
  __syncthreads();
  const int n = kofs[nk];
  const int2* ent = reinterpret_cast<const int2*>(a.ent) + tile_base;
  const bool fits = (int64_t)tile_base + n <= a.cap;
  if (fits)
    for (int i = tid; i < n; i += 256) atomicAdd(&cnt_m[ent[i].y >> 8], 1);   // counts only: order-free
  __syncthreads();
  if (tid < 64) {                       // exclusive scan of the column counts, two columns per lane
    const int c0 = fits ? cnt_m[2 * tid] : 0, c1 = fits ? cnt_m[2 * tid + 1] : 0;
    const int incl = wave_incl_scan(c0 + c1, tid), ex = incl - c0 - c1;
    base_m[2 * tid] = ex;
    base_m[2 * tid + 1] = ex + c0;
    a.row_ptr[t * 128 + 2 * tid] = tile_base + ex;
    a.row_ptr[t * 128 + 2 * tid + 1] = tile_base + ex + c0;
    if (t == a.gm - 1 && tid == 63) a.row_ptr[a.gm * 128] = tile_base + incl;
  }
  __syncthreads();
  if (!fits) return;
  int2* rent = reinterpret_cast<int2*>(a.row_ent) + tile_base;
  for (int c0 = 0; c0 < n; c0 += 256) {
    const int i = c0 + tid;
    int2 e = make_int2(0, 0);
    int m = -1;
    if (i < n) {
      e = ent[i];
      m = e.y >> 8;
    }
    int r = 0, tot = 0;                 // same-column entries of this wave: before this lane / all
    for (int j = 0; j < 64; ++j) {
      const int mj = __builtin_amdgcn_readlane(m, j);
      const int eq = mj == m ? 1 : 0;
      tot += eq;
      r += j < lane ? eq : 0;
    }
    wcnt[w][tid & 127] = 0;
    wcnt[w][(tid & 127) ^ 64] = 0;
    __syncthreads();
    if (m >= 0) wcnt[w][m] = tot;       // every lane of the column writes the same count
    __syncthreads();
    if (m >= 0) {
      for (int v = 0; v < w; ++v) r += wcnt[v][m];
      int lo = 0, hi = nk - 1;          // the entry's K-step: the bucket holding position i
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (kofs[mid] <= i) lo = mid;
        else hi = mid - 1;
      }
      rent[base_m[m] + r] = make_int2(e.x, lo * 64 + (e.y & 255));
    }
    __syncthreads();
    if (tid < 128) base_m[tid] += wcnt[0][tid] + wcnt[1][tid] + wcnt[2][tid] + wcnt[3][tid];
    __syncthreads();
  }
}

// one workgroup per column tile t: its base = sum of the counts of all earlier buckets (a parallel
// fixed-order sum, cheap at a few thousand buckets, and no separate scan launch), then one wave per
// K-step writes its rows' segments at the wave-prefix offsets; the last workgroup writes bptr[total]
__global__ void __launch_bounds__(256) tb_fill_kernel(OcfTileBucketArgs a) {
  __shared__ int red[256];
  __shared__ int kt_cnt[64];
  const int t = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nb = a.gm * a.nk, before = t * a.nk;
  // live-row records of tile t (ocf.h OCF_LIVE_REC): wave 0 from the input tags, wave 1 from the
  // target tags; rank k of a live row = live rows before it in the tile
  if (w < 2 && (w == 0 ? a.live_in : a.live_out))
    live_record((w == 0 ? a.rtag_in : a.rtag_out) + (int64_t)t * 128,
                (w == 0 ? a.live_in : a.live_out) + (int64_t)t * OCF_LIVE_REC, a.rtag, lane);
  int s = 0;
  for (int i = tid; i < before; i += 256) s += a.cnt[i];
  red[tid] = s;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (tid < off) red[tid] += red[tid + off];
    __syncthreads();
  }
  const int tile_base = red[0];
  if (a.cnt_clear)   // the next batch's counters (ocf_scatter_batch tb_cnt), zeroed for it
    for (int i = tid; i < a.nk; i += 256) a.cnt_clear[before + i] = 0;
  if (t == a.gm - 1 && tid == 0) {
    int tot = tile_base;
    for (int i = before; i < nb; ++i) tot += a.cnt[i];
    a.bptr[nb] = tot;
  }
  for (int kt0 = 0; kt0 < a.nk; kt0 += 4) {
    const int kt = kt0 + w;
    // bucket offsets of this group of K-steps within the tile
    if (tid < 4 && kt0 + tid < a.nk) kt_cnt[tid] = a.cnt[before + kt0 + tid];
    __syncthreads();
    int koff = tile_base;
    for (int i = 0; i < kt0; ++i) koff += a.cnt[before + i];
    for (int i = 0; i < w; ++i) koff += kt_cnt[i];
    if (kt < a.nk) {
      const TbSeg sg = tb_segment(a, t, kt * 64 + lane);
      const int incl = wave_incl_scan(sg.n, lane);
      if (lane == 0) a.bptr[before + kt] = koff;
      const int64_t base = (int64_t)koff + incl - sg.n;
      if (base + sg.n <= a.cap)
        for (int j = 0; j < sg.n; ++j) {
          const int64_t e = sg.e0 + j;
          int2 v;
          v.x = (int)(sg.lb + a.lidx[e]);
          v.y = lane | ((a.col[e] - t * 128) << 8);
          reinterpret_cast<int2*>(a.ent)[base + j] = v;
        }
    }
    __syncthreads();
  }
  if (a.row_ptr) tb_rows(a, t, tile_base);
}

// ---- row lists straight from the scatter's per-column counts (ocf_row_lists) ------------------------
// row_ptr = exclusive scan of col_cnt in blocks of RL_CHUNK columns: rl_scan_kernel scans each block
// locally (coalesced int4 loads, wave scans + the block's wave totals) into lp[] and the block total
// into bsum[]; the later kernels add the block offsets, each computing the (<= 128) offsets in LDS
constexpr int RL_CHUNK = 4096;
constexpr int RL_REG = 32;      // lists up to this long are sorted in registers (K = 2,048 rows: ~11 per column)
constexpr int RL_LONG_BLOCKS = 128;   // workgroups of rl_sort_long_kernel (most batches queue no list)
__global__ void __launch_bounds__(1024) rl_scan_kernel(OcfRowListArgs a) {
  __shared__ int wtot[16];
  const int n = a.n_cols, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int* lp = a.cursor + n;
  int* bsum = a.cursor + 2 * n;
  const int i0 = blockIdx.x * RL_CHUNK + 4 * tid;
  if (blockIdx.x == 0 && tid == 0) a.cursor[2 * n + 128] = 0;   // this batch's long-list queue (rl_sort)
  int4 v = make_int4(0, 0, 0, 0);
  if (i0 < n) {                          // n % 128 == 0: a thread's 4 columns are all in range or none
    v = *reinterpret_cast<const int4*>(a.col_cnt + i0);
    *reinterpret_cast<int4*>(a.col_cnt + i0) = make_int4(0, 0, 0, 0);   // zeroed for the next batch
  }
  const int ts = v.x + v.y + v.z + v.w;
  const int incl = wave_incl_scan(ts, lane);
  if (lane == 63) wtot[w] = incl;
  __syncthreads();
  int off = 0;
  for (int k = 0; k < w; ++k) off += wtot[k];
  const int ex = off + incl - ts;
  if (i0 < n) *reinterpret_cast<int4*>(lp + i0) = make_int4(ex, ex + v.x, ex + v.x + v.y, ex + v.x + v.y + v.z);
  if (tid == 1023) bsum[blockIdx.x] = off + incl;
}

// exclusive prefix of the block totals into LDS (one wave, nb <= 128 blocks); returns the grand total
__device__ __forceinline__ int rl_block_offsets(const OcfRowListArgs& a, int* sboff) {
  const int nb = (a.n_cols + RL_CHUNK - 1) / RL_CHUNK;
  const int* bsum = a.cursor + 2 * a.n_cols;
  __shared__ int tot;
  if (threadIdx.x < 64) {
    const int l = threadIdx.x;
    const int v0 = 2 * l < nb ? bsum[2 * l] : 0, v1 = 2 * l + 1 < nb ? bsum[2 * l + 1] : 0;
    const int incl = wave_incl_scan(v0 + v1, l);
    sboff[2 * l] = incl - v0 - v1;
    sboff[2 * l + 1] = incl - v1;
    if (l == 63) tot = incl;
  }
  __syncthreads();
  return tot;
}

// one thread per entry: its column's next slot (unordered; rl_sort_kernel orders each list)
__global__ void __launch_bounds__(256) rl_fill_kernel(OcfRowListArgs a) {
  __shared__ int sboff[128];
  rl_block_offsets(a, sboff);
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= a.E) return;
  const int v = a.ecb[e];
  const int c = v & ((1 << 19) - 1), b = v >> 19;
  const int slot = a.cursor[a.n_cols + c] + sboff[c / RL_CHUNK] + atomicAdd(&a.cursor[c], 1);
  reinterpret_cast<int2*>(a.row_ent)[slot] = make_int2((int)e, b);
}

// short list (the common case): independent loads, an odd-even transposition sort in registers on the
// entry index (unique; the batch row rides along), independent stores
template <int S>
__device__ __forceinline__ void rl_reg_sort(int2* ent, int n) {
  int2 k[S];
#pragma unroll
  for (int i = 0; i < S; ++i) k[i] = i < n ? ent[i] : make_int2(0x7fffffff, 0);
#pragma unroll
  for (int p = 0; p < S; ++p)
#pragma unroll
    for (int i = p & 1; i + 1 < S; i += 2) {
      const bool sw = k[i + 1].x < k[i].x;
      const int2 a = k[i], b = k[i + 1];
      k[i] = sw ? b : a;
      k[i + 1] = sw ? a : b;
    }
#pragma unroll
  for (int i = 0; i < S; ++i)
    if (i < n) ent[i] = k[i];
}

// one thread per column of a 128-column tile: insertion sort of its list by entry index (entry indices
// grow with the batch row: the list ends in batch-row order, whatever order the fill left), cursor
// reset; waves 0 / 1 write the tile's live-row records
__global__ void __launch_bounds__(128) rl_sort_kernel(OcfRowListArgs a) {
  const int t = blockIdx.x, tid = threadIdx.x, m = t * 128 + tid;
  const int lane = tid & 63, w = tid >> 6;
  if (w == 0 && a.live_in) live_record(a.rtag_in + (int64_t)t * 128, a.live_in + (int64_t)t * OCF_LIVE_REC, a.rtag, lane);
  if (w == 1 && a.live_out)
    live_record(a.rtag_out + (int64_t)t * 128, a.live_out + (int64_t)t * OCF_LIVE_REC, a.rtag, lane);
  __shared__ int sboff[128];
  const int total = rl_block_offsets(a, sboff);
  const int* lp = a.cursor + a.n_cols;
  const int lo = lp[m] + sboff[m / RL_CHUNK];
  const int hi = m + 1 < a.n_cols ? lp[m + 1] + sboff[(m + 1) / RL_CHUNK] : total;
  a.row_ptr[m] = lo;
  if (m + 1 == a.n_cols) a.row_ptr[a.n_cols] = total;
  a.cursor[m] = 0;
  int2* ent = reinterpret_cast<int2*>(a.row_ent);
  const int n = hi - lo;
  // the sorting network's size follows the wave's longest short list (an S-entry network costs S^2 / 2
  // compare-exchanges whatever n is: 32 entries for every column took 22 us at ML-20M, ~1.4 per column)
  int nm = n <= RL_REG ? n : 0;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) nm = max(nm, __shfl_xor(nm, off, 64));
  if (n <= 1) return;                    // empty or single-entry lists are in order as filled
  if (n <= RL_REG) {
    if (nm <= 4) rl_reg_sort<4>(ent + lo, n);
    else if (nm <= 8) rl_reg_sort<8>(ent + lo, n);
    else if (nm <= 16) rl_reg_sort<16>(ent + lo, n);
    else rl_reg_sort<RL_REG>(ent + lo, n);
    return;
  }
  // long list (a column present in more than RL_REG batch rows): queued for rl_sort_long_kernel
  int* q = a.cursor + 2 * a.n_cols + 128;
  q[1 + atomicAdd(q, 1)] = m;
}

// Bitonic sort of x[0, n) by .x in a workgroup of NT threads (LDS), all-ascending form: each merge
// stage first compares i with i ^ (k - 1), then with i ^ j; a partner at or past n is a virtual +inf
// that never moves, so no padding is needed.  Every thread of the workgroup must call it.
template <int NT>
__device__ void wg_bitonic(int2* x, int n) {
  int P = 1;
  while (P < n) P <<= 1;
  for (int k = 2; k <= P; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < n; i += NT) {
        const int ij = j == (k >> 1) ? (i ^ (k - 1)) : (i ^ j);
        if (ij > i && ij < n) {
          const int2 a = x[i], b = x[ij];
          if (a.x > b.x) {
            x[i] = b;
            x[ij] = a;
          }
        }
      }
      __syncthreads();
    }
}

// one workgroup per queued long list: bitonic sort in LDS (a list holds at most one entry per batch
// row, <= RL_MAX_LIST); the queue length is read after rl_sort_kernel has finished
constexpr int RL_MAX_LIST = 4096;
__global__ void __launch_bounds__(256) rl_sort_long_kernel(OcfRowListArgs a) {
  __shared__ int2 buf[RL_MAX_LIST];
  const int* q = a.cursor + 2 * a.n_cols + 128;
  const int nq = q[0];
  int2* ent = reinterpret_cast<int2*>(a.row_ent);
  for (int qi = blockIdx.x; qi < nq; qi += gridDim.x) {
    const int m = q[1 + qi];
    const int lo = a.row_ptr[m], n = a.row_ptr[m + 1] - lo;
    for (int i = threadIdx.x; i < n; i += 256) buf[i] = ent[lo + i];
    __syncthreads();
    wg_bitonic<256>(buf, n);
    for (int i = threadIdx.x; i < n; i += 256) ent[lo + i] = buf[i];
    __syncthreads();
  }
}

// ---- epoch row lists (ocf_epoch_row_lists): the same lists for many batches, from the plan's tables ----
// Counting and placement are privatised per (batch, block of columns): the workgroup's waves walk the
// batch's rows (a wave per row, lanes over its entries) and count / place the entries of the block's
// columns with LDS atomics (global atomics on per-column counters ran at ~40 G/s: 355 + 429 us for an
// ML-20M epoch).  The column block is as wide as the LDS allows next to the batch's row table.
constexpr int ERL_THREADS = 1024;
constexpr int ERL_MAXB = 4096;
constexpr int ERL_LDS = 160 * 1024;

// columns per workgroup for batches of B rows: the rest of the LDS after the CSR starts and row offsets,
// at 16 bits per column (a column holds at most one entry per batch row, B <= 4,096: two counters share
// a 32-bit word and an atomic add of 1 << 16 (c & 1) never carries into the neighbour)
inline int erl_block_cols(int B) {
  const int64_t rest = ERL_LDS - (int64_t)B * 8 - (int64_t)(B + 1) * 4 - 64;
  return (int)std::min<int64_t>(65536, rest / 2 / 128 * 128);
}
inline size_t erl_lds_bytes(int B) { return (size_t)erl_block_cols(B) * 2 + (size_t)B * 8 + (size_t)(B + 1) * 4; }

constexpr int ERL_U = 8;   // entries per lane in flight in the count / fill walks

struct ErlLds {
  uint32_t* cnt; int64_t* src; int* off;   // cnt: 16-bit counters, two per word
};
__device__ __forceinline__ ErlLds erl_lds(int B) {
  extern __shared__ int64_t erl_dyn[];
  ErlLds l;
  l.src = erl_dyn;
  l.off = reinterpret_cast<int*>(erl_dyn + B);
  l.cnt = reinterpret_cast<uint32_t*>(l.off + B + 1);
  return l;
}
// stage batch s's CSR starts and batch-local row offsets in LDS
__device__ __forceinline__ void erl_stage(const OcfEpochRowListArgs& a, int s, const ErlLds& l) {
  const int bi = a.sel[s];
  const int64_t* lb = a.lboff + (int64_t)bi * (a.B + 1);
  for (int b = threadIdx.x; b <= a.B; b += ERL_THREADS) {
    l.off[b] = (int)lb[b];
    if (b < a.B) {
      const int r = a.rows[(int64_t)bi * a.B + b];
      l.src[b] = r >= 0 ? a.rp[r] : 0;
    }
  }
}

// per (column block, batch, row group): the block's column counts over the group's batch rows.  A batch's rows
// are split into n_rg groups (OcfEpochRowListArgs n_rg) when few batches are built at once: each workgroup
// walks one group instead of the whole batch (the count and fill walks are latency-bound chains of loads;
// with a window of 20 batches the grid held 60 workgroups).  Counts go to cnt[rg][s][column].
__device__ __forceinline__ int erl_rg(const OcfEpochRowListArgs& a) { return a.n_rg > 1 ? a.n_rg : 1; }
__global__ void __launch_bounds__(ERL_THREADS) erl_count_kernel(OcfEpochRowListArgs a, int cb) {
  const ErlLds l = erl_lds(a.B);
  const int s = blockIdx.y, rg = blockIdx.z, c0 = blockIdx.x * cb, nc = min(cb, a.n_cols - c0);
  const int nrg = erl_rg(a), b0 = rg * a.B / nrg, b1 = (rg + 1) * a.B / nrg;
  for (int i = threadIdx.x; i < nc / 2; i += ERL_THREADS) l.cnt[i] = 0u;   // nc % 128 == 0
  erl_stage(a, s, l);
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int b = b0 + w; b < b1; b += ERL_THREADS / 64) {
    const int n = l.off[b + 1] - l.off[b];
    const int* col = a.col + l.src[b];
    // ERL_U column loads in flight per lane (a one-load loop waited a round trip per 64 entries)
    for (int j0 = lane; j0 < n; j0 += 64 * ERL_U) {
      int cu[ERL_U];
#pragma unroll
      for (int u = 0; u < ERL_U; ++u) cu[u] = j0 + 64 * u < n ? col[j0 + 64 * u] - c0 : -1;
#pragma unroll
      for (int u = 0; u < ERL_U; ++u)
        if (cu[u] >= 0 && cu[u] < nc) atomicAdd(&l.cnt[cu[u] >> 1], 1u << (16 * (cu[u] & 1)));
    }
  }
  __syncthreads();
  // 16-bit counts (a column's list holds <= 4,096 entries), stored as the LDS holds them: two per word
  uint32_t* g = reinterpret_cast<uint32_t*>(a.cnt) + (((int64_t)rg * a.n_sel + s) * a.n_cols + c0) / 2;
  for (int i = threadIdx.x; i < nc / 2; i += ERL_THREADS) g[i] = l.cnt[i];
}

// the row pointers of every batch in two passes over blocks of 4,096 columns, grid (blocks, batches): a batch's
// scan in one workgroup walked its 138 K (Netflix: 480 K) columns serially, 65-185 us for a window of 20 batches
constexpr int ERL_SB = 4096;   // columns per scan block (1,024 threads x 4)
__device__ __forceinline__ int erl_nsb(const OcfEpochRowListArgs& a) { return (a.n_cols + ERL_SB - 1) / ERL_SB; }
// cnt layout: [n_rg][n_sel][n_cols] 16-bit counts (two per int), [n_sel][blocks] block totals, the long-list queue
__device__ __forceinline__ int* erl_btot(const OcfEpochRowListArgs& a) {
  return a.cnt + (int64_t)erl_rg(a) * a.n_sel * a.n_cols / 2;
}
__device__ __forceinline__ int* erl_queue(const OcfEpochRowListArgs& a) {
  return erl_btot(a) + (int64_t)a.n_sel * erl_nsb(a);
}

// the exclusive scan of a 4,096-column block's totals (4 per thread) from `base` into rp; the last block also
// writes rp[n]
__device__ __forceinline__ void erl_scan_block(int* rp, int4 v, int i0, int n, int base, bool last, int* wtot) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int ts = v.x + v.y + v.z + v.w;
  const int incl = wave_incl_scan(ts, lane);
  if (lane == 63) wtot[w] = incl;
  __syncthreads();
  int off = base;
  for (int k = 0; k < w; ++k) off += wtot[k];
  const int ex = off + incl - ts;
  if (i0 < n) {
    rp[i0] = ex;
    rp[i0 + 1] = ex + v.x;
    rp[i0 + 2] = ex + v.x + v.y;
    rp[i0 + 3] = ex + v.x + v.y + v.z;
  }
  if (last && tid == 1023) rp[n] = off + incl;
}

// pass 1, per (column block, batch): each column's count summed over the row groups (the groups' counts become
// their exclusive prefixes: the fill's cursor starts), the totals parked in row_ptr, the block's total.  ONE (a
// single block of <= 4,096 columns: ML-100K, Jester): the block's scan right here, no second pass
template <bool ONE>
__global__ void __launch_bounds__(1024) erl_gsum_kernel(OcfEpochRowListArgs a) {
  __shared__ int wtot[16];
  const int blk = blockIdx.x, s = blockIdx.y, n = a.n_cols, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nrg = erl_rg(a);
  const int64_t gstride = (int64_t)a.n_sel * n / 2;   // (32-bit words of two 16-bit counts)
  uint32_t* cnt = reinterpret_cast<uint32_t*>(a.cnt) + (int64_t)s * n / 2;
  int* rp = a.row_ptr + (int64_t)s * (n + 1);
  if (s == 0 && blk == 0 && tid == 0) erl_queue(a)[0] = 0;   // erl_sort's long-list queue
  const int i0 = blk * ERL_SB + 4 * tid;
  int4 v = make_int4(0, 0, 0, 0);
  if (i0 < n) {                         // n % 128 == 0: all 4 columns in range or none
    for (int g = 0; g < nrg; ++g) {
      uint2* q = reinterpret_cast<uint2*>(cnt + g * gstride + i0 / 2);
      const uint2 c = *q;
      // the group's counts become its exclusive prefixes (< 4,096: 16 bits)
      if (nrg > 1) *q = make_uint2((uint32_t)v.x | ((uint32_t)v.y << 16), (uint32_t)v.z | ((uint32_t)v.w << 16));
      v.x += (int)(c.x & 0xFFFFu); v.y += (int)(c.x >> 16); v.z += (int)(c.y & 0xFFFFu); v.w += (int)(c.y >> 16);
    }
    if (!ONE) { rp[i0] = v.x; rp[i0 + 1] = v.y; rp[i0 + 2] = v.z; rp[i0 + 3] = v.w; }
  }
  if (ONE) {
    erl_scan_block(rp, v, i0, n, 0, true, wtot);
    return;
  }
  int t = v.x + v.y + v.z + v.w;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
  if (lane == 0) wtot[w] = t;
  __syncthreads();
  if (tid == 0) {
    int bt = 0;
    for (int k = 0; k < 16; ++k) bt += wtot[k];
    erl_btot(a)[(int64_t)s * erl_nsb(a) + blk] = bt;
  }
}

// pass 2, per (column block, batch): the block's offset (the earlier blocks' totals), then the exclusive scan of
// its column totals into row_ptr; the last block writes row_ptr[n_cols]
__global__ void __launch_bounds__(1024) erl_scan_kernel(OcfEpochRowListArgs a) {
  __shared__ int wtot[16];
  __shared__ int base_s;
  const int blk = blockIdx.x, s = blockIdx.y, n = a.n_cols, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nsb = erl_nsb(a);
  int* rp = a.row_ptr + (int64_t)s * (n + 1);
  if (w == 0) {
    const int* bt = erl_btot(a) + (int64_t)s * nsb;
    int o = 0;
    for (int k = lane; k < blk; k += 64) o += bt[k];
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) o += __shfl_xor(o, d, 64);
    if (lane == 0) base_s = o;
  }
  const int i0 = blk * ERL_SB + 4 * tid;
  int4 v = make_int4(0, 0, 0, 0);
  if (i0 < n) v = make_int4(rp[i0], rp[i0 + 1], rp[i0 + 2], rp[i0 + 3]);   // the totals pass 1 parked here
  __syncthreads();
  erl_scan_block(rp, v, i0, n, base_s, blk == nsb - 1, wtot);
}

// per (column block, batch): every entry of the block's columns at its column's next slot (LDS cursors;
// unordered within a column, erl_sort_kernel orders each list)
#ifndef OCF_ERL_XCD
#define OCF_ERL_XCD 1
#endif
// OCF_ERL_XCD (default): a 1-D grid whose workgroups go to the 8 XCDs round robin, remapped so that the row groups
// of one (batch, column block) -- the workgroups writing the same part of row_ent -- run on one XCD side by side
// (their scattered 8-byte list writes then merge in that XCD's L2 instead of reaching memory as partial lines).
// Same box, 20-step windows: ML-20M 0.3870 -> 0.3835 ms/step, Netflix 1.958 -> 1.950 (profiles/r05_window/
// ab_fill_xcd.jsonl); 0: the (column block, batch, row group) grid
__global__ void __launch_bounds__(ERL_THREADS) erl_fill_kernel(OcfEpochRowListArgs a, int cb) {
  const ErlLds l = erl_lds(a.B);
  const int nrg = erl_rg(a);
  int s, rg, cbk;
  if (OCF_ERL_XCD) {
    const int ncb = (a.n_cols + cb - 1) / cb, T = ncb * a.n_sel * nrg, per = (T + 7) / 8;
    const int u = (int)(blockIdx.x % 8) * per + (int)(blockIdx.x / 8);
    if (u >= T) return;
    rg = u % nrg;
    cbk = (u / nrg) % ncb;
    s = u / (nrg * ncb);
  } else {
    s = blockIdx.y;
    rg = blockIdx.z;
    cbk = blockIdx.x;
  }
  const int c0 = cbk * cb, nc = min(cb, a.n_cols - c0);
  const int b0 = rg * a.B / nrg, b1 = (rg + 1) * a.B / nrg;
  if (nrg > 1) {      // the group's cursors start after the earlier groups' entries (erl_gsum_kernel)
    const uint32_t* pre = reinterpret_cast<const uint32_t*>(a.cnt) + (((int64_t)rg * a.n_sel + s) * a.n_cols + c0) / 2;
    for (int i = threadIdx.x; i < nc / 2; i += ERL_THREADS) l.cnt[i] = pre[i];
  } else {
    for (int i = threadIdx.x; i < nc / 2; i += ERL_THREADS) l.cnt[i] = 0u;
  }
  erl_stage(a, s, l);
  __syncthreads();
  const int* rp = a.row_ptr + (int64_t)s * (a.n_cols + 1);
  int2* ent = reinterpret_cast<int2*>(a.row_ent) + (a.ebase[s] - a.ebase0);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int b = b0 + w; b < b1; b += ERL_THREADS / 64) {
    const int e0 = l.off[b], n = l.off[b + 1] - e0;
    const int* col = a.col + l.src[b];
    // ERL_U entries per lane in flight: their columns, then their lists' starts (a one-entry loop waited two
    // dependent round trips per 64 entries: 456 us per 104-batch ML-20M epoch).  Slots within a list are
    // taken in any order; erl_sort_kernel orders every list afterwards.
    for (int j0 = lane; j0 < n; j0 += 64 * ERL_U) {
      int cu[ERL_U], st[ERL_U];
#pragma unroll
      for (int u = 0; u < ERL_U; ++u) cu[u] = j0 + 64 * u < n ? col[j0 + 64 * u] : -1;
#pragma unroll
      for (int u = 0; u < ERL_U; ++u) st[u] = (cu[u] >= c0 && cu[u] < c0 + nc) ? rp[cu[u]] : -1;
#pragma unroll
      for (int u = 0; u < ERL_U; ++u)
        if (st[u] >= 0) {
          const int r = cu[u] - c0, sh = 16 * (r & 1);
          const int pos = (int)((atomicAdd(&l.cnt[r >> 1], 1u << sh) >> sh) & 0xFFFFu);
          ent[st[u] + pos] = make_int2(e0 + j0 + 64 * u, b);
        }
    }
  }
}

// per (batch, 128-column tile): the tile's live record, every list sorted by entry
// index -- short lists in registers (rl_reg_sort), up to ERL_MID entries by the workgroup in LDS, longer
// ones (a column in more than ERL_MID batch rows) queued for erl_sort_long_kernel
constexpr int ERL_MID = 1024;
constexpr int ERL_LONG_MAX = 4096;
__global__ void __launch_bounds__(128) erl_sort_kernel(OcfEpochRowListArgs a) {
  __shared__ int2 buf[ERL_MID];
  __shared__ int nlong, n0s;
  __shared__ int longs[128];
  const int t = blockIdx.x, s = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int n_cols = a.n_cols, m = t * 128 + tid;
  const int* rp = a.row_ptr + (int64_t)s * (n_cols + 1);
  int2* ent = reinterpret_cast<int2*>(a.row_ent) + (a.ebase[s] - a.ebase0);
  const int lo = rp[m], n = rp[m + 1] - lo;
  if (tid == 0) nlong = 0;
  const uint64_t bal = __ballot(n > 0);
  if (w == 0 && lane == 0) n0s = __popcll(bal);
  __syncthreads();
  if (a.live) {
    uint8_t* rec = a.live + ((int64_t)s * (n_cols / 128) + t) * OCF_LIVE_REC;
    const int k = (w ? n0s : 0) + __popcll(bal & ((1ull << lane) - 1));
    if (n > 0) rec[16 + (k & 7) * 16 + (k >> 3)] = (uint8_t)tid;
    if (w == 1 && lane == 0) *reinterpret_cast<int*>(rec) = n0s + __popcll(bal);
  }
  int nm = n <= RL_REG ? n : 0;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) nm = max(nm, __shfl_xor(nm, off, 64));
  if (n > 1 && n <= RL_REG) {
    if (nm <= 4) rl_reg_sort<4>(ent + lo, n);
    else if (nm <= 8) rl_reg_sort<8>(ent + lo, n);
    else if (nm <= 16) rl_reg_sort<16>(ent + lo, n);
    else rl_reg_sort<RL_REG>(ent + lo, n);
  } else if (n > ERL_MID) {
    int* q = erl_queue(a);                               // long-list queue after the counters
    const int qi = atomicAdd(q, 1);
    q[1 + 2 * qi] = s;
    q[2 + 2 * qi] = m;
  } else if (n > RL_REG) {
    longs[atomicAdd(&nlong, 1)] = tid;
  }
  __syncthreads();
  for (int q = 0; q < nlong; ++q) {        // workgroup-uniform loop over the tile's mid-length lists
    const int mq = t * 128 + longs[q];
    const int lq = rp[mq], nq = rp[mq + 1] - lq;
    for (int i = tid; i < nq; i += 128) buf[i] = ent[lq + i];
    __syncthreads();
    wg_bitonic<128>(buf, nq);
    for (int i = tid; i < nq; i += 128) ent[lq + i] = buf[i];
    __syncthreads();
  }
}

// bitonic sort by .x across the S lanes of a segment (S | 64, segments aligned): lane i of the segment ends with
// the i-th smallest; every lane of the wave takes part (pad with INT_MAX keys)
template <int S>
__device__ __forceinline__ int2 seg_bitonic(int2 v, int i) {
#pragma unroll
  for (int k = 2; k <= S; k <<= 1)
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      int2 o;
      o.x = __shfl_xor(v.x, j, 64);
      o.y = __shfl_xor(v.y, j, 64);
      const bool up = (i & k) == 0, lower = (i & j) == 0;
      if (lower == up ? o.x < v.x : o.x > v.x) v = o;
    }
  return v;
}

// a wave's lists of up to 64 entries sorted in segments of S lanes (S = the longest of them, rounded up to a
// power of two): 64 / S lists per pass, every pass's loads issued before the first sort
template <int S>
__device__ __forceinline__ void erl_wave_lists(int2* ent, const int* s_lo, const int* s_n, int c0, int lane) {
  constexpr int PER = 64 / S, IT = (8 + PER - 1) / PER;
  const int seg = lane / S, sl = lane % S;
  int2 v[IT];
  bool mine[IT];
  int base[IT];
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int k = it * PER + seg;
    const int c = c0 + (k < 8 ? k : 0), nn = s_n[c];
    mine[it] = k < 8 && nn > 1 && nn <= 64 && sl < nn;
    base[it] = s_lo[c];
    v[it] = mine[it] ? ent[base[it] + sl] : make_int2(0x7fffffff, 0);
  }
#pragma unroll
  for (int it = 0; it < IT; ++it) v[it] = seg_bitonic<S>(v[it], sl);
#pragma unroll
  for (int it = 0; it < IT; ++it)
    if (mine[it]) ent[base[it] + sl] = v[it];
}

// erl_sort_kernel for builds of long lists on average (ML-100K / ML-1M: ~9-16 entries per column list), where a
// thread per list leaves most SIMDs idle (ML-100K: 6 K lists = 96 waves) and runs an odd-even network of ~500
// compare-exchanges in series per 32-entry list: 16 waves per 128-column tile, 8 columns per wave, the lists
// sorted across lanes (erl_wave_lists); 65-1,024 entries by the workgroup in LDS, longer ones queued as before.
// Same live records.
__global__ void __launch_bounds__(1024) erl_sort_wave_kernel(OcfEpochRowListArgs a) {
  __shared__ int2 buf[ERL_MID];
  __shared__ int s_lo[128], s_n[128], mids[128];
  __shared__ int nmid, n0s;
  const int t = blockIdx.x, s = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int n_cols = a.n_cols;
  const int* rp = a.row_ptr + (int64_t)s * (n_cols + 1);
  int2* ent = reinterpret_cast<int2*>(a.row_ent) + (a.ebase[s] - a.ebase0);
  int n = 0;
  if (tid < 128) {
    const int lo = rp[t * 128 + tid];
    n = rp[t * 128 + tid + 1] - lo;
    s_lo[tid] = lo;
    s_n[tid] = n;
  }
  if (tid == 0) nmid = 0;
  const uint64_t bal = __ballot(n > 0);
  if (w == 0 && lane == 0) n0s = __popcll(bal);
  __syncthreads();
  if (tid < 128) {
    if (a.live) {
      uint8_t* rec = a.live + ((int64_t)s * (n_cols / 128) + t) * OCF_LIVE_REC;
      const int k = (w ? n0s : 0) + __popcll(bal & ((1ull << lane) - 1));
      if (n > 0) rec[16 + (k & 7) * 16 + (k >> 3)] = (uint8_t)tid;
      if (w == 1 && lane == 0) *reinterpret_cast<int*>(rec) = n0s + __popcll(bal);
    }
    if (n > ERL_MID) {
      int* q = erl_queue(a);
      const int qi = atomicAdd(q, 1);
      q[1 + 2 * qi] = s;
      q[2 + 2 * qi] = t * 128 + tid;
    } else if (n > 64) {
      mids[atomicAdd(&nmid, 1)] = tid;
    }
  }
  // wave w: the tile's columns 8 w .. 8 w + 7
  const int c0 = 8 * w;
  int mx = lane < 8 ? s_n[c0 + lane] : 0;
  if (mx > 64) mx = 0;                   // (the workgroup's LDS pass)
#pragma unroll
  for (int o = 4; o > 0; o >>= 1) mx = max(mx, __shfl_xor(mx, o, 64));
  mx = __shfl(mx, 0, 64);
  if (mx > 32) erl_wave_lists<64>(ent, s_lo, s_n, c0, lane);
  else if (mx > 16) erl_wave_lists<32>(ent, s_lo, s_n, c0, lane);
  else if (mx > 8) erl_wave_lists<16>(ent, s_lo, s_n, c0, lane);
  else if (mx > 1) erl_wave_lists<8>(ent, s_lo, s_n, c0, lane);
  __syncthreads();
  for (int q = 0; q < nmid; ++q) {        // workgroup-uniform loop over the tile's mid-length lists
    const int c = mids[q], lq = s_lo[c], nq = s_n[c];
    for (int i = tid; i < nq; i += 1024) buf[i] = ent[lq + i];
    __syncthreads();
    wg_bitonic<1024>(buf, nq);
    for (int i = tid; i < nq; i += 1024) ent[lq + i] = buf[i];
    __syncthreads();
  }
}

// one workgroup per queued list of more than ERL_MID entries (<= ERL_LONG_MAX: one per batch row)
__global__ void __launch_bounds__(1024) erl_sort_long_kernel(OcfEpochRowListArgs a) {
  __shared__ int2 buf[ERL_LONG_MAX];
  const int* q = erl_queue(a);
  const int nq = q[0];
  for (int qi = blockIdx.x; qi < nq; qi += gridDim.x) {
    const int s = q[1 + 2 * qi], m = q[2 + 2 * qi];
    const int* rp = a.row_ptr + (int64_t)s * (a.n_cols + 1);
    int2* ent = reinterpret_cast<int2*>(a.row_ent) + (a.ebase[s] - a.ebase0);
    const int lo = rp[m], n = rp[m + 1] - lo;
    for (int i = threadIdx.x; i < n; i += 1024) buf[i] = ent[lo + i];
    __syncthreads();
    wg_bitonic<1024>(buf, n);
    for (int i = threadIdx.x; i < n; i += 1024) ent[lo + i] = buf[i];
    __syncthreads();
  }
}

}  // namespace ocf

extern "C" int ocf_epoch_row_lists(const OcfEpochRowListArgs* args, void* stream) {
  OCF_TRY_BEGIN
  const OcfEpochRowListArgs& a = *args;
  OCF_CHECK(a.rows && a.rp && a.col && a.lboff && a.sel && a.ebase && a.cnt && a.row_ptr && a.row_ent,
            "ocf_epoch_row_lists: null pointer");
  OCF_CHECK(a.n_cols > 0 && a.n_cols % 128 == 0, "ocf_epoch_row_lists: n_cols > 0, % 128");
  OCF_CHECK(a.B > 0 && a.B <= ERL_MAXB, "ocf_epoch_row_lists: 0 < B <= 4096 (one entry per batch row and column)");
  OCF_CHECK(a.n_sel >= 0 && a.n_sel <= 65535, "ocf_epoch_row_lists: 0 <= n_sel <= 65535");
  OCF_CHECK(a.n_rg >= 0 && a.n_rg <= 64 && a.n_rg <= a.B, "ocf_epoch_row_lists: 0 <= n_rg <= min(64, B)");
  if (a.n_sel == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const int cb = erl_block_cols(a.B), ncb = (a.n_cols + cb - 1) / cb;
  const size_t lds = erl_lds_bytes(a.B);
  static const bool lds_attr = [] {   // dynamic LDS above 64 KiB (gfx950: up to 160 KiB per workgroup)
    return hipFuncSetAttribute((const void*)erl_count_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, ERL_LDS) ==
               hipSuccess &&
           hipFuncSetAttribute((const void*)erl_fill_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, ERL_LDS) ==
               hipSuccess;
  }();
  OCF_CHECK(lds_attr, "ocf_epoch_row_lists: cannot raise the dynamic LDS limit");
  const int nrg = a.n_rg > 1 ? a.n_rg : 1;
  hipLaunchKernelGGL(erl_count_kernel, dim3(ncb, a.n_sel, nrg), dim3(ERL_THREADS), lds, s, a, cb);
  const int nsb = (a.n_cols + ERL_SB - 1) / ERL_SB;
  if (nsb == 1) {
    hipLaunchKernelGGL(erl_gsum_kernel<true>, dim3(1, a.n_sel), dim3(1024), 0, s, a);
  } else {
    hipLaunchKernelGGL(erl_gsum_kernel<false>, dim3(nsb, a.n_sel), dim3(1024), 0, s, a);
    hipLaunchKernelGGL(erl_scan_kernel, dim3(nsb, a.n_sel), dim3(1024), 0, s, a);
  }
  if (OCF_ERL_XCD) {
    const int64_t T = (int64_t)ncb * a.n_sel * nrg;
    hipLaunchKernelGGL(erl_fill_kernel, dim3((unsigned)((T + 7) / 8 * 8)), dim3(ERL_THREADS), lds, s, a, cb);
  } else {
    hipLaunchKernelGGL(erl_fill_kernel, dim3(ncb, a.n_sel, nrg), dim3(ERL_THREADS), lds, s, a, cb);
  }
  // lists of ~4+ entries on average: sorted across lanes (erl_sort_wave_kernel), else a thread per list
  if (a.entries >= 4 * (int64_t)a.n_sel * a.n_cols)
    hipLaunchKernelGGL(erl_sort_wave_kernel, dim3(a.n_cols / 128, a.n_sel), dim3(1024), 0, s, a);
  else
    hipLaunchKernelGGL(erl_sort_kernel, dim3(a.n_cols / 128, a.n_sel), dim3(128), 0, s, a);
  // the long-list pass only when a list can hold more than ERL_MID entries (max_list: the caller's bound)
  if (a.max_list <= 0 || a.max_list > ERL_MID)
    hipLaunchKernelGGL(erl_sort_long_kernel, dim3(64), dim3(1024), 0, s, a);
  OCF_HIP(hipGetLastError());
  OCF_TRY_END
}

extern "C" int ocf_row_lists(const OcfRowListArgs* args, void* stream) {
  OCF_TRY_BEGIN
  const OcfRowListArgs& a = *args;
  OCF_CHECK(a.ecb && a.col_cnt && a.cursor && a.row_ptr && a.row_ent, "ocf_row_lists: null pointer");
  OCF_CHECK(a.n_cols > 0 && a.n_cols % 128 == 0 && a.n_cols <= (1 << 19), "ocf_row_lists: 0 < n_cols <= 2^19, % 128");
  OCF_CHECK((!a.live_in || a.rtag_in) && (!a.live_out || a.rtag_out), "ocf_row_lists: live records need row tags");
  OCF_CHECK(!(a.live_in || a.live_out) || (a.rtag >= 1 && a.rtag <= 255), "ocf_row_lists: 1 <= rtag <= 255");
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(rl_scan_kernel, dim3((a.n_cols + RL_CHUNK - 1) / RL_CHUNK), dim3(1024), 0, s, a);
  if (a.E > 0) hipLaunchKernelGGL(rl_fill_kernel, dim3((unsigned)((a.E + 255) / 256)), dim3(256), 0, s, a);
  hipLaunchKernelGGL(rl_sort_kernel, dim3(a.n_cols / 128), dim3(128), 0, s, a);
  hipLaunchKernelGGL(rl_sort_long_kernel, dim3(RL_LONG_BLOCKS), dim3(256), 0, s, a);
  OCF_HIP(hipGetLastError());
  OCF_TRY_END
}

extern "C" int ocf_sparse_tiles(const OcfTileBucketArgs* args, void* stream) {
  OCF_TRY_BEGIN
  const OcfTileBucketArgs& a = *args;
  OCF_CHECK(a.rows && a.rp && a.tptr && a.col && a.lidx && a.lboff && a.cnt && a.bptr && a.ent,
            "ocf_sparse_tiles: null pointer");
  OCF_CHECK(a.gm >= 0 && a.nk >= 0 && a.gm <= a.ntiles && a.krows <= 64 * a.nk,
            "ocf_sparse_tiles: gm <= ntiles and krows <= 64 * nk required");
  OCF_CHECK(!a.row_ptr || (a.row_ent && a.nk <= 64), "ocf_sparse_tiles: row lists need row_ent and nk <= 64");
  const int nb = a.gm * a.nk;
  hipStream_t s = (hipStream_t)stream;
  OCF_CHECK(a.cnt_clear != a.cnt, "ocf_sparse_tiles: cnt_clear must not alias cnt");
  OCF_CHECK((!a.live_in || a.rtag_in) && (!a.live_out || a.rtag_out), "ocf_sparse_tiles: live records need row tags");
  OCF_CHECK(!(a.live_in || a.live_out) || (a.rtag >= 1 && a.rtag <= 255), "ocf_sparse_tiles: 1 <= rtag <= 255");
  if (nb > 0 && !a.counted) {
    hipLaunchKernelGGL(tb_count_kernel, dim3((nb + 3) / 4), dim3(256), 0, s, a);
    OCF_HIP(hipGetLastError());
  }
  if (nb > 0) {
    hipLaunchKernelGGL(tb_fill_kernel, dim3(a.gm), dim3(256), 0, s, a);
    OCF_HIP(hipGetLastError());
  } else {
    OCF_HIP(hipMemsetAsync(a.bptr, 0, sizeof(int32_t), s));
  }
  OCF_TRY_END
}
