// ocf_mlp_step (ocf.h): a small dense model's whole training step in one persistent launch.
//
// The dense path's step (split-K encoder, hidden-layer GEMMs, the masked-MSE decoder, the backward GEMMs
// with the fused optimizer, bias kernels, stats) is ~14 launches of 2-33 us on a model of 0.14 M
// parameters (train_jester.py's 200 -> 256 -> 256 -> 100, batch 128): every launch is a handful of
// workgroups waiting on latency, and the host spends longer issuing them than the GPU running them.
// Here a grid of up to 128 workgroups stays resident and walks the step's phases, each a set of 32 x 32
// output tiles (one per workgroup, the reduction dimension split over its four waves, MFMA from LDS;
// operands from the L2 / MALL-resident weights and activations), separated by grid barriers:
//   F_0 .. F_{L-1}  h_i = act(h_{i-1} W_i + b_i)                     (model.py:64-71)
//   OUT             y = M * (h_{L-1} W_L + b_L), e = y - T, delta_L = e * M, the step's statistics, the
//                   column sums of delta_L (model.py:81-86, train.py:49, 102-121)
//   BACK_L          stats; b_L's update; delta_{L-1} = (delta_L W_L^T) * act' (+ column sums); dW_L -> scratch
//   BACK_i          W_{i+1} updated from its scratch gradient (nothing reads it any more); b_i's update;
//                   delta_{i-1}; dW_i -> scratch
//   BACK_0          W_1 updated; b_0's update; dW_0 tiles update W_0 directly
// (Keras computes every gradient from the weights before the step, train.py:50-51: a layer's weights
// change only after the phase that last reads them.)  Gradients are carried unscaled (e * M) and the
// MSE's 2 / (B N) applied in fp32 at the update, as on the other paths.
#include <algorithm>
#include <cstring>
#include <type_traits>

#include "ocf_epilogues.h"
#include "ocf_internal.h"

namespace ocf {
namespace mlp {

constexpr int THREADS = 256;
constexpr int WAVES = THREADS / 64;
constexpr int MAXL = OCF_MAX_HIDDEN + 1;

// the word a masked operand element reads (stage() loads through addresses)
__device__ float g_zero[4];

// device copy of the arguments with the scratch carved out
struct P {
  int L, B, Bp, N, Np, k, act;
  int dim[MAXL + 1];      // padded widths: dim[0] = k Np, dim[i] = hidden_p[i-1], dim[L+1] = Np
  int real[MAXL + 1];     // real widths (dim[0]: k N counted per block)
  const float* x[3]; int64_t ld_x; const int64_t* rows;
  const float* om; const float* tg; int64_t ld_t;
  float* W[MAXL]; float* b[MAXL]; float* sW1[MAXL]; float* sW2[MAXL]; float* sb1[MAXL]; float* sb2[MAXL];
  void* sh[MAXL]; int sh_blk;
  OcfOptParams op;
  float* stats;
  float* h[MAXL];         // h[i]: [Bp][dim[i+1]] (i < L)
  float* d[MAXL + 1];     // d[i]: delta of layer i's output, [Bp][dim[i+1]] (i <= L)
  float* g[MAXL];         // g[i]: dW_i scratch (1 <= i <= L), W_i's layout
  float* colp[MAXL + 1];  // colp[i]: [Bp / 32][dim[i+1]] column sums of delta_i per 32-row tile (bias gradients)
  float* rowp;            // [Np / 32][Bp] per column-tile row sse
  float* totp;            // [tiles][waves][3] per output tile and wave sse / sae / count
  uint32_t* bar; uint32_t* err; int max_polls;
  uint64_t* trace;
};

// workgroup 0 records the constant-rate clock (diagnostics: ocf.h OcfMlpStepArgs trace)
__device__ __forceinline__ void mark(const P& p, int& n) {
  if (p.trace && blockIdx.x == 0 && threadIdx.x == 0 && n < 24) p.trace[n] = wall_clock64();
  ++n;
}

// ---- hand-offs between phases (MI355X_MICROARCH.md § inter-workgroup visibility, the first row of its
// table of sc1 hand-offs).  Every value one workgroup writes for another (activations, deltas, scratch
// gradients, column / row / tile partials) is stored write-through (sc1: a relaxed agent-scope store) and
// read with L1-bypassing sc1 loads (ldc / ldc4), so a barrier needs neither an L2 write-back on the producer
// nor an L1 invalidate on the consumer: every storing wave drains its stores (vmcnt(0)), the workgroup
// meets at a workgroup barrier, one lane adds to the arrival counter, and one lane polls that counter
// (sc1 loads) until every workgroup has arrived.  Each handed-off word is written once per launch, before
// any read of it; the launch starts with clean caches.
constexpr int SC1 = 16;   // cache-policy bits of an L1-bypassing (sc1) access
__device__ __forceinline__ void pub(float* q, float v) {
  __hip_atomic_store(q, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rs_of(const float* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, 0x7FFFFFFF, 0x00020000);
}
__device__ __forceinline__ float4 ldc4(const float* base, int64_t e) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs_of(base), (uint32_t)(e * 4), 0, SC1);
  float4 r;
  __builtin_memcpy(&r, &v, 16);
  return r;
}
__device__ __forceinline__ float ldc(const float* base, int64_t e) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs_of(base), (uint32_t)(e * 4), 0, SC1));
}

// grid barrier number nb (1, 2, ...) of the launch: bar[0] counts arrivals monotonically within the launch
// (barrier nb is passed when it reaches nb * grid); the last workgroup to leave the kernel resets it (exit()),
// so it is zero for the next launch.  Bounded: a workgroup that gives up (not all workgroups resident)
// records the error word and continues.
__device__ __forceinline__ void grid_sync(const P& p, int& tn, int& nb) {
  mark(p, tn);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");       // this wave's write-through stores have landed
  __syncthreads();
  ++nb;
  if (threadIdx.x == 0) {
    const uint32_t target = (uint32_t)nb * gridDim.x;
    __hip_atomic_fetch_add(&p.bar[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int it = 0;
    while (__hip_atomic_load(&p.bar[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++it > p.max_polls) {
        __hip_atomic_store(p.err, (uint32_t)OCF_ASYNC_MLP_BARRIER, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (no instruction: keeps the loads below the poll)
  __syncthreads();
  mark(p, tn);
}
__device__ __forceinline__ void grid_exit(const P& p, int nb) {
  if (threadIdx.x == 0) {
    const uint32_t all = (uint32_t)(nb + 1) * gridDim.x;
    if (__hip_atomic_fetch_add(&p.bar[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1 == all)
      __hip_atomic_store(&p.bar[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ---- one 32 x 32 tile of C = A B per workgroup, K split over the 4 waves (a wave's quarter of K in chunks of
// KC staged through the wave's own LDS region, then MFMA from LDS); the four partial tiles are summed in wave
// order through LDS.  A phase of the Jester model has 16-96 such tiles, so every workgroup of the grid has
// work and a wave walks one or two chunks instead of a workgroup walking the whole K.
// a(r, k) / b(n, k) return 4 consecutive fp32 elements along the operand's contiguous direction (r .. r+3 when
// A_RFAST / B_NFAST, else k .. k+3), rounded to CT when staged (as the MFMA operand staging of the other paths).
// Every lane issues all of a chunk's loads before it writes any (the accessors are branch-free).
constexpr int TT = 32;
template <typename CT> struct Lds {
  static constexpr int KC = sizeof(CT) == 2 ? 64 : 32;     // a wave's K chunk
  static constexpr int PAD = sizeof(CT) == 2 ? 8 : 4;
  static constexpr int STRIDE = KC + PAD;                  // row stride 144 B (16-bit) / 144 B (fp32)
  static constexpr int WAVE = 2 * TT * STRIDE;             // a wave's A + B chunk (elements)
  static constexpr int STAGE_BYTES = WAVES * WAVE * (int)sizeof(CT);
  static constexpr int RED_BYTES = WAVES * TT * (TT + 1) * 4;
  static constexpr int BYTES = (STAGE_BYTES > RED_BYTES ? STAGE_BYTES : RED_BYTES) + WAVES * TT * 4;
};

template <typename CT, bool FAST_R, typename F>
__device__ __forceinline__ void stage(CT* dst, int r0, int k0, int kc, F&& f) {
  constexpr int S = Lds<CT>::STRIDE, KC = Lds<CT>::KC, RUNS = TT * KC / 4 / 64;
  const int lane = threadIdx.x & 63;
  float4 v[RUNS];
#pragma unroll
  for (int j = 0; j < RUNS; ++j) {
    const int u = lane + 64 * j;
    int r, k;
    if (FAST_R) { r = 4 * (u % (TT / 4)); k = u / (TT / 4); }
    else { r = u / (KC / 4); k = 4 * (u % (KC / 4)); }
    v[j] = f(r0 + r, k0 + (k < kc ? k : 0));              // past the chunk's end: a valid address, unused
  }
#pragma unroll
  for (int j = 0; j < RUNS; ++j) {
    const int u = lane + 64 * j;
    const float e[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
    if (FAST_R) {
      const int r = 4 * (u % (TT / 4)), k = u / (TT / 4);
#pragma unroll
      for (int q = 0; q < 4; ++q) dst[(r + q) * S + k] = CvtT<CT>::to(e[q]);
    } else {
      const int r = u / (KC / 4), k = 4 * (u % (KC / 4));
#pragma unroll
      for (int q = 0; q < 4; ++q) dst[r * S + k + q] = CvtT<CT>::to(e[q]);
    }
  }
}

// the summed tile: thread t holds rows (t >> 5) + 8 j (j < 4) of column t & 31
struct Tile {
  float v[4];
};
__device__ __forceinline__ int out_row(int j) { return (threadIdx.x >> 5) + 8 * j; }
__device__ __forceinline__ int out_col() { return threadIdx.x & 31; }

template <typename CT, bool A_RFAST, bool B_NFAST, typename FA, typename FB>
__device__ __forceinline__ Tile wg_tile(char* lds, int m0, int n0, int K, FA&& a, FB&& b) {
  constexpr int S = Lds<CT>::STRIDE, KC = Lds<CT>::KC;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, r = lane & 31, hf = lane >> 5;
  CT* sA = reinterpret_cast<CT*>(lds) + wave * Lds<CT>::WAVE;
  CT* sB = sA + TT * S;
  const int kw = K / WAVES, kb = wave * kw;             // K % 64 == 0: kw is a multiple of 16
  ocf_f16v acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  for (int k0 = 0; k0 < kw; k0 += KC) {
    const int kc = kw - k0 < KC ? kw - k0 : KC;
    stage<CT, A_RFAST>(sA, m0, kb + k0, kc, a);
    stage<CT, B_NFAST>(sB, n0, kb + k0, kc, b);
    __syncthreads();
    if constexpr (sizeof(CT) == 2) {
      using V = typename std::conditional<std::is_same<CT, _Float16>::value, ocf_h8, ocf_b8>::type;
      for (int ks = 0; ks < kc; ks += 16) {
        V fa, fb;
        const int kk = ks + 8 * hf;
        __builtin_memcpy(&fa, sA + r * S + kk, 16);
        __builtin_memcpy(&fb, sB + r * S + kk, 16);
        if constexpr (std::is_same<CT, _Float16>::value)
          acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa, fb, acc, 0, 0, 0);
        else
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb, acc, 0, 0, 0);
      }
    } else {
      for (int ks = 0; ks < kc; ks += 2)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(sA[r * S + ks + hf], sB[r * S + ks + hf], acc, 0, 0, 0);
    }
    __syncthreads();
  }
  // the four K quarters, summed in wave order (C layout of v_mfma_f32_32x32x*: register q holds row
  // (q & 3) + 8 (q >> 2) + 4 hf, column r)
  float* red = reinterpret_cast<float*>(lds);
#pragma unroll
  for (int q = 0; q < 16; ++q) red[(wave * TT + (q & 3) + 8 * (q >> 2) + 4 * hf) * (TT + 1) + r] = acc[q];
  __syncthreads();
  Tile t;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int rr = out_row(j), cc = out_col();
    float s = red[rr * (TT + 1) + cc];
#pragma unroll
    for (int w = 1; w < WAVES; ++w) s += red[(w * TT + rr) * (TT + 1) + cc];
    t.v[j] = s;
  }
  __syncthreads();
  return t;
}

// the column sums of the summed tile over its 32 rows (a thread's rows, then the two half-waves, then the
// waves in order), written to dst[0..31] by threads 0..31
template <typename CT>
__device__ __forceinline__ void tile_colsum(char* lds, const Tile& t, float* dst) {
  float* cs = reinterpret_cast<float*>(lds + Lds<CT>::BYTES - WAVES * TT * 4);
  float s = (t.v[0] + t.v[1]) + (t.v[2] + t.v[3]);
  s += __shfl_xor(s, 32, 64);
  if ((threadIdx.x & 63) < 32) cs[(threadIdx.x >> 6) * TT + out_col()] = s;
  __syncthreads();
  if (threadIdx.x < TT) {
    float c = cs[threadIdx.x];
#pragma unroll
    for (int w = 1; w < WAVES; ++w) c += cs[w * TT + threadIdx.x];
    pub(&dst[threadIdx.x], c);
  }
}

__device__ __forceinline__ float4 ld4(const float* q) { return *reinterpret_cast<const float4*>(q); }

// ---- operand views
// layer-0 input of batch row b, padded columns c .. c+3 (one block: Np % 4 == 0); zero past the batch and in
// the block padding (element loads through selected addresses: no branches, the four loads go out together)
__device__ __forceinline__ float4 x4(const P& p, int b, int c) {
  const int blk = c / p.Np, n = c - blk * p.Np;
  const float* row = p.x[blk] + p.rows[b < p.B ? b : p.B - 1] * p.ld_x;
  float e[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) e[q] = *((b < p.B && n + q < p.N) ? row + n + q : g_zero);
  return make_float4(e[0], e[1], e[2], e[3]);
}
__device__ __forceinline__ int64_t shadow_index(const P& p, int i, int r, int c) {
  const int C = i == p.L ? p.dim[i] : p.dim[i + 1];
  if (!p.sh_blk) return (int64_t)r * C + c;
  return ((int64_t)(r >> 6) * (C >> 6) + (c >> 6)) * 4096 + (r & 63) * 64 + (c & 63);
}

// the update of a thread's 4 elements of weight i (rows r[q], column c of a [R][C] weight): the parameters and
// slots are loaded before the tile's GEMM (load), the update applied from its gradients after it (apply)
template <typename CT, int KIND>
struct TileUpdate {
  float w[4], a[4], bb[4];
  int64_t e[4];
  __device__ __forceinline__ void load(const P& p, int i, const int* r, int c) {
    const int C = i == p.L ? p.dim[i] : p.dim[i + 1];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      e[q] = (int64_t)r[q] * C + c;
      w[q] = p.W[i][e[q]];
      a[q] = p.sW1[i] ? p.sW1[i][e[q]] : 0.f;
      bb[q] = p.sW2[i] ? p.sW2[i][e[q]] : 0.f;
    }
  }
  __device__ __forceinline__ void apply(const P& p, int i, const float* g, const int* r, int c) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      opt_update_k<KIND>(p.op, g[q], w[q], a[q], bb[q]);
      p.W[i][e[q]] = w[q];
      if (p.sW1[i]) p.sW1[i][e[q]] = a[q];
      if (p.sW2[i]) p.sW2[i][e[q]] = bb[q];
      if constexpr (sizeof(CT) == 2)
        if (p.sh[i]) reinterpret_cast<CT*>(p.sh[i])[shadow_index(p, i, r[q], c)] = CvtT<CT>::to(w[q]);
    }
  }
};

// bias i: db[n] = gscale * sum over the Bp / 32 row tiles of the column partials the producer of delta_i wrote
// (tile order), then the update
template <int KIND>
__device__ __forceinline__ void bias_update(const P& p, int i, int gtid, int gthreads) {
  const int W = p.dim[i + 1], realw = p.real[i + 1], nb = p.Bp / TT;
  for (int n = gtid; n < realw; n += gthreads) {
    float v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = j < nb ? ldc(p.colp[i], (int64_t)j * W + n) : 0.f;
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) s += v[j];
    float w = p.b[i][n], a = p.sb1[i] ? p.sb1[i][n] : 0.f, bb = p.sb2[i] ? p.sb2[i][n] : 0.f;
    opt_update_k<KIND>(p.op, s * p.op.gscale, w, a, bb);
    p.b[i][n] = w;
    if (p.sb1[i]) p.sb1[i][n] = a;
    if (p.sb2[i]) p.sb2[i][n] = bb;
  }
}

// the elementwise update of weight i from its gradient g (every element: a padded element has g = 0 and
// zero slots, which every optimizer leaves unchanged), 4 per thread with the loads issued together
template <typename CT, int KIND>
__device__ __forceinline__ void update_from(const P& p, int i, const float* g, int64_t n, int gtid, int gthreads) {
  const int C = i == p.L ? p.dim[i] : p.dim[i + 1];
  for (int64_t e0 = (int64_t)gtid * 4; e0 < n; e0 += (int64_t)gthreads * 4) {
    const float4 gv = ldc4(g, e0);
    float4 w = *reinterpret_cast<const float4*>(p.W[i] + e0);
    float4 a = p.sW1[i] ? *reinterpret_cast<const float4*>(p.sW1[i] + e0) : make_float4(0.f, 0.f, 0.f, 0.f);
    float4 bb = p.sW2[i] ? *reinterpret_cast<const float4*>(p.sW2[i] + e0) : make_float4(0.f, 0.f, 0.f, 0.f);
    float* wf = reinterpret_cast<float*>(&w);
    float* af = reinterpret_cast<float*>(&a);
    float* bf = reinterpret_cast<float*>(&bb);
    const float* gf = reinterpret_cast<const float*>(&gv);
#pragma unroll
    for (int j = 0; j < 4; ++j) opt_update_k<KIND>(p.op, gf[j], wf[j], af[j], bf[j]);
    *reinterpret_cast<float4*>(p.W[i] + e0) = w;
    if (p.sW1[i]) *reinterpret_cast<float4*>(p.sW1[i] + e0) = a;
    if (p.sW2[i]) *reinterpret_cast<float4*>(p.sW2[i] + e0) = bb;
    if constexpr (sizeof(CT) == 2)
      if (p.sh[i]) {
        const int r = (int)(e0 / C), c = (int)(e0 % C);
#pragma unroll
        for (int j = 0; j < 4; ++j) reinterpret_cast<CT*>(p.sh[i])[shadow_index(p, i, r, c + j)] = CvtT<CT>::to(wf[j]);
      }
  }
}

template <typename CT, int KIND>
__global__ void __launch_bounds__(THREADS) mlp_step_kernel(P p) {
  __shared__ __attribute__((aligned(16))) char lds[Lds<CT>::BYTES];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int gtid = blockIdx.x * THREADS + threadIdx.x, gthreads = gridDim.x * THREADS;
  const int L = p.L, Bt = p.Bp / TT;
  const float gs = p.op.gscale;
  const int c = out_col();
  int tn = 0, nb = 0;
  mark(p, tn);

  // ---- forward: h_i = act(src W_i + b_i); padded rows / units are zero
  for (int i = 0; i < L; ++i) {
    const int K = p.dim[i], Wd = p.dim[i + 1], nt = Wd / TT;
    for (int t = blockIdx.x; t < Bt * nt; t += gridDim.x) {
      const int m0 = (t / nt) * TT, n0 = (t % nt) * TT;
      Tile v;
      if (i == 0)
        v = wg_tile<CT, false, true>(lds, m0, n0, K, [&](int m, int k) { return x4(p, m, k); },
                                     [&](int n, int k) { return ld4(p.W[0] + (int64_t)k * Wd + n); });
      else
        v = wg_tile<CT, false, true>(lds, m0, n0, K, [&](int m, int k) { return ldc4(p.h[i - 1], (int64_t)m * K + k); },
                                     [&](int n, int k) { return ld4(p.W[i] + (int64_t)k * Wd + n); });
      const int n = n0 + c;
      const float bias = p.b[i][n];
      const bool live_n = n < p.real[i + 1];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = m0 + out_row(j);
        pub(&p.h[i][(int64_t)m * Wd + n], (m < p.B && live_n) ? act_apply(p.act, v.v[j] + bias) : 0.f);
      }
    }
    grid_sync(p, tn, nb);
  }
  // ---- output layer + masked MSE: y = M (h W_L + b_L); e = y - T; delta_L = e M; per-tile statistics and
  // the column sums of delta_L (b_L's gradient)
  {
    const int K = p.dim[L], nt = p.Np / TT;
    for (int t = blockIdx.x; t < Bt * nt; t += gridDim.x) {
      const int m0 = (t / nt) * TT, n0 = (t % nt) * TT;
      const int n = n0 + c;
      const float bias = p.b[L][n];
      float mkv[4], ttv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {        // the mask / target loads in flight during the GEMM (clamped)
        const int m = m0 + out_row(j);
        const int64_t o = p.rows[m < p.B ? m : p.B - 1] * p.ld_t + (n < p.N ? n : 0);
        mkv[j] = p.om[o];
        ttv[j] = p.tg[o];
      }
      // W_L is stored transposed ([Np][K]): B(n, k) = W_L[n][k], contiguous along k
      const Tile v = wg_tile<CT, false, false>(lds, m0, n0, K,
                                               [&](int m, int k) { return ldc4(p.h[L - 1], (int64_t)m * K + k); },
                                               [&](int n, int k) { return ld4(p.W[L] + (int64_t)n * K + k); });
      Tile dl;
      float sse = 0.f, sae = 0.f, cnt = 0.f, rs[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = m0 + out_row(j);
        float d = 0.f, se = 0.f;
        if (m < p.B && n < p.N) {
          const float y = mkv[j] * (v.v[j] + bias);
          const float e = y - ttv[j];
          se = e * e;
          sse += se;
          sae += fabsf(e);
          cnt += (ttv[j] + y != 0.f) ? 1.f : 0.f;
          d = e * mkv[j];
        }
        pub(&p.d[L][(int64_t)m * p.Np + n], d);
        dl.v[j] = d;
        rs[j] = se;
      }
      // row sums over the tile's 32 columns (the 32 lanes of each half-wave), in a fixed butterfly order
      for (int o = 16; o > 0; o >>= 1)
#pragma unroll
        for (int j = 0; j < 4; ++j) rs[j] += __shfl_xor(rs[j], o, 64);
      if ((lane & 31) == 0)
#pragma unroll
        for (int j = 0; j < 4; ++j) pub(&p.rowp[(int64_t)(n0 / TT) * p.Bp + m0 + out_row(j)], rs[j]);
      for (int o = 32; o > 0; o >>= 1) {
        sse += __shfl_xor(sse, o, 64);
        sae += __shfl_xor(sae, o, 64);
        cnt += __shfl_xor(cnt, o, 64);
      }
      if (lane == 0) {
        const int64_t slot = (int64_t)t * WAVES + wave;
        pub(&p.totp[slot * 3 + 0], sse);
        pub(&p.totp[slot * 3 + 1], sae);
        pub(&p.totp[slot * 3 + 2], cnt);
      }
      tile_colsum<CT>(lds, dl, p.colp[L] + (int64_t)(m0 / TT) * p.Np + n0);
    }
    grid_sync(p, tn, nb);
  }
  // ---- backward, layer by layer from the output
  for (int i = L; i >= 0; --i) {
    const int Wi = p.dim[i + 1];                 // layer i's output width (padded)
    const int Ki = p.dim[i];                     // its input width
    // delta of layer i - 1's output: (delta_i W_i^T) * act'(h_{i-1}), with its column sums
    const int nd = i > 0 ? (Bt * (Ki / TT)) : 0;
    // dW_i: [input][output] (layer L: [output][input]) tiles, K = the batch rows
    const int gr = i == L ? Wi : Ki, gc = i == L ? Ki : Wi;
    const int ng = (gr / TT) * (gc / TT);
    // the phase's side work, which no tile of the phase reads: the update of W_{i+1} from its scratch gradient
    // (nothing reads W_{i+1} from here on), the step's statistics (i = L), b_i's update.  Done by the
    // workgroups without a tile when there are enough of them, else by every workgroup after its tiles.
    auto side = [&](int sid, int sthreads, bool last) {
      if (i + 1 <= L) {
        const int R = i + 1 == L ? p.dim[L + 1] : p.dim[i + 1], C = i + 1 == L ? p.dim[L] : p.dim[i + 2];
        update_from<CT, KIND>(p, i + 1, p.g[i + 1], (int64_t)R * C, sid, sthreads);
      }
      if (i == L && last && wave == 0) {
        // the step's statistics from the per-wave partials, in order
        const int slots = Bt * (p.Np / TT) * WAVES, ncb = p.Np / TT;
        float a[3] = {0.f, 0.f, 0.f};
        for (int t = lane; t < slots; t += 64)
          for (int k = 0; k < 3; ++k) a[k] += ldc(p.totp, (int64_t)t * 3 + k);
        for (int k = 0; k < 3; ++k)
          for (int o = 32; o > 0; o >>= 1) a[k] += __shfl_xor(a[k], o, 64);
        if (lane == 0) {
          p.stats[0] = a[0];
          p.stats[1] = a[1];
          p.stats[2] = a[2];
          p.stats[3] = 0.f;
        }
        for (int b = lane; b < p.Bp; b += 64) {
          float r = 0.f;
          for (int cb = 0; cb < ncb; ++cb) r += ldc(p.rowp, (int64_t)cb * p.Bp + b);
          p.stats[4 + b] = r;
        }
      }
      bias_update<KIND>(p, i, sid, sthreads);
    };
    const int T = nd + ng, idle = (int)gridDim.x - T;
    const bool side_idle = idle >= (int)gridDim.x / 4;
    if (side_idle && (int)blockIdx.x >= T)
      side(((int)blockIdx.x - T) * THREADS + threadIdx.x, idle * THREADS, blockIdx.x == gridDim.x - 1);
    for (int t = blockIdx.x; t < nd + ng; t += gridDim.x) {
      if (t < nd) {
        const int ct = Ki / TT, m0 = (t / ct) * TT, n0 = (t % ct) * TT;
        const int n = n0 + c;
        float hv[4];                    // in flight during the GEMM
#pragma unroll
        for (int j = 0; j < 4; ++j) hv[j] = ldc(p.h[i - 1], (int64_t)(m0 + out_row(j)) * Ki + n);
        Tile v;
        if (i == L)      // B(n = input unit, k = output unit) = W_L[k][n], contiguous along n
          v = wg_tile<CT, false, true>(lds, m0, n0, Wi, [&](int m, int k) { return ldc4(p.d[i], (int64_t)m * Wi + k); },
                                       [&](int n, int k) { return ld4(p.W[L] + (int64_t)k * Ki + n); });
        else             // B(n = input unit, k = output unit) = W_i[n][k], contiguous along k
          v = wg_tile<CT, false, false>(lds, m0, n0, Wi, [&](int m, int k) { return ldc4(p.d[i], (int64_t)m * Wi + k); },
                                        [&](int n, int k) { return ld4(p.W[i] + (int64_t)n * Wi + k); });
        Tile dv;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int m = m0 + out_row(j);
          dv.v[j] = (m < p.B && n < p.real[i]) ? v.v[j] * act_grad(p.act, hv[j]) : 0.f;
          pub(&p.d[i - 1][(int64_t)m * Ki + n], dv.v[j]);
        }
        tile_colsum<CT>(lds, dv, p.colp[i - 1] + (int64_t)(m0 / TT) * Ki + n0);
        continue;
      }
      const int u = t - nd, ct = gc / TT, m0 = (u / ct) * TT, n0 = (u % ct) * TT;
      int rr[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) rr[j] = m0 + out_row(j);
      TileUpdate<CT, KIND> up;
      if (i == 0) up.load(p, 0, rr, n0 + c);   // W_0's parameters and slots in flight during the GEMM
      Tile v;
      if (i == L)        // dW_L[n][j] = sum_b delta_L[b][n] h_{L-1}[b][j]
        v = wg_tile<CT, true, true>(lds, m0, n0, p.Bp, [&](int m, int k) { return ldc4(p.d[L], (int64_t)k * Wi + m); },
                                    [&](int n, int k) { return ldc4(p.h[L - 1], (int64_t)k * Ki + n); });
      else if (i > 0)    // dW_i[k][j] = sum_b h_{i-1}[b][k] delta_i[b][j]
        v = wg_tile<CT, true, true>(lds, m0, n0, p.Bp, [&](int m, int k) { return ldc4(p.h[i - 1], (int64_t)k * Ki + m); },
                                    [&](int n, int k) { return ldc4(p.d[i], (int64_t)k * Wi + n); });
      else               // dW_0[k][j] = sum_b x[b][k] delta_0[b][j]
        v = wg_tile<CT, true, true>(lds, m0, n0, p.Bp, [&](int m, int k) { return x4(p, k, m); },
                                    [&](int n, int k) { return ldc4(p.d[0], (int64_t)k * Wi + n); });
      if (i == 0) {      // nothing reads W_0 any more: update it from the tile (padded elements have zero gradient)
        float gv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) gv[j] = v.v[j] * gs;
        up.apply(p, 0, gv, rr, n0 + c);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) pub(&p.g[i][(int64_t)(m0 + out_row(j)) * gc + n0 + c], v.v[j] * gs);
      }
    }
    if (!side_idle) side(gtid, gthreads, blockIdx.x == gridDim.x - 1);
    if (i > 0) grid_sync(p, tn, nb);
  }
  grid_exit(p, nb);
  mark(p, tn);
}

struct Layout {
  size_t h[MAXL], d[MAXL + 1], g[MAXL], colp[MAXL + 1], rowp, totp, total;
};
Layout layout(const OcfMlpStepArgs& a, int* dim) {
  Layout w{};
  size_t off = 0;
  auto take = [&](size_t floats) {
    const size_t o = off;
    off += (floats * 4 + 255) / 256 * 256;
    return o;
  };
  const int L = a.n_hidden;
  for (int i = 0; i < L; ++i) w.h[i] = take((size_t)a.Bp * dim[i + 1]);
  for (int i = 0; i <= L; ++i) w.d[i] = take((size_t)a.Bp * dim[i + 1]);
  for (int i = 1; i <= L; ++i) w.g[i] = take((size_t)dim[i] * dim[i + 1]);
  for (int i = 0; i <= L; ++i) w.colp[i] = take((size_t)(a.Bp / TT) * dim[i + 1]);
  w.rowp = take((size_t)(a.Np / TT) * a.Bp);
  w.totp = take((size_t)(a.Bp / TT) * (a.Np / TT) * WAVES * 3);
  w.total = off;
  return w;
}

void dims_of(const OcfMlpStepArgs& a, int* dim, int* real) {
  const int L = a.n_hidden;
  dim[0] = a.k_blocks * a.Np;
  real[0] = a.k_blocks * a.N;
  for (int i = 0; i < L; ++i) {
    dim[i + 1] = a.hidden_p[i];
    real[i + 1] = a.hidden[i];
  }
  dim[L + 1] = a.Np;
  real[L + 1] = a.N;
}

void check(const OcfMlpStepArgs& a) {
  OCF_CHECK(a.n_hidden >= 1 && a.n_hidden <= OCF_MAX_HIDDEN, "ocf_mlp_step: n_hidden 1..OCF_MAX_HIDDEN");
  OCF_CHECK(a.Bp % 64 == 0 && a.Bp >= 64 && a.Bp <= 512 && a.B >= 1 && a.B <= a.Bp, "ocf_mlp_step: B <= Bp, Bp % 64 == 0, <= 512");
  OCF_CHECK(a.N >= 1 && a.Np % 64 == 0 && a.N <= a.Np, "ocf_mlp_step: N <= Np, Np % 64 == 0");
  OCF_CHECK(a.k_blocks >= 1 && a.k_blocks <= 3, "ocf_mlp_step: k_blocks 1..3");
  for (int i = 0; i < a.n_hidden; ++i)
    OCF_CHECK(a.hidden_p[i] % 64 == 0 && a.hidden[i] >= 1 && a.hidden[i] <= a.hidden_p[i],
              "ocf_mlp_step: hidden widths padded to multiples of 64");
  for (int j = 0; j < a.k_blocks; ++j) OCF_CHECK(a.x[j] != nullptr, "ocf_mlp_step: null input block");
  OCF_CHECK(a.rows && a.out_mask && a.targets && a.ld_x >= a.N && a.ld_t >= a.N, "ocf_mlp_step: batch arrays");
  for (int i = 0; i <= a.n_hidden; ++i) OCF_CHECK(a.W[i] && a.b[i], "ocf_mlp_step: null parameter");
  OCF_CHECK(a.opt.l2 == 0.f, "ocf_mlp_step: l2 must be 0 (the regulariser is not fused)");
  const bool slots = a.opt.kind == OCF_OPT_ADAGRAD || a.opt.kind == OCF_OPT_RMSPROP || a.opt.kind == OCF_OPT_ADAM;
  if (slots)
    for (int i = 0; i <= a.n_hidden; ++i)
      OCF_CHECK(a.sW1[i] && a.sb1[i] && (a.opt.kind != OCF_OPT_ADAM || (a.sW2[i] && a.sb2[i])),
                "ocf_mlp_step: optimizer slots");
  OCF_CHECK(a.stats && a.work && a.barrier, "ocf_mlp_step: stats / work / barrier");
}

template <typename CT>
void launch(const OcfMlpStepArgs& a, const P& p, int wgs, hipStream_t s) {
  switch (a.opt.kind) {
    case OCF_OPT_ADAGRAD: hipLaunchKernelGGL((mlp_step_kernel<CT, OCF_OPT_ADAGRAD>), dim3(wgs), dim3(THREADS), 0, s, p); break;
    case OCF_OPT_RMSPROP: hipLaunchKernelGGL((mlp_step_kernel<CT, OCF_OPT_RMSPROP>), dim3(wgs), dim3(THREADS), 0, s, p); break;
    case OCF_OPT_ADAM: hipLaunchKernelGGL((mlp_step_kernel<CT, OCF_OPT_ADAM>), dim3(wgs), dim3(THREADS), 0, s, p); break;
    default: hipLaunchKernelGGL((mlp_step_kernel<CT, 0>), dim3(wgs), dim3(THREADS), 0, s, p);
  }
  OCF_HIP(hipGetLastError());
}

}  // namespace mlp
}  // namespace ocf

using namespace ocf;

extern "C" int64_t ocf_mlp_step_workspace(const OcfMlpStepArgs* a) {
  try {
    OCF_CHECK(a != nullptr, "ocf_mlp_step_workspace: null arguments");
    int dim[mlp::MAXL + 1], real[mlp::MAXL + 1];
    OCF_CHECK(a->n_hidden >= 1 && a->n_hidden <= OCF_MAX_HIDDEN, "ocf_mlp_step: n_hidden 1..OCF_MAX_HIDDEN");
    mlp::dims_of(*a, dim, real);
    return (int64_t)mlp::layout(*a, dim).total;
  } catch (const std::exception& e) {
    set_error(e.what());
    return -1;
  }
}

extern "C" int ocf_mlp_step(const OcfMlpStepArgs* a, void* stream) {
  OCF_TRY_BEGIN
  OCF_CHECK(a != nullptr, "ocf_mlp_step: null arguments");
  mlp::check(*a);
  mlp::P p{};
  p.L = a->n_hidden; p.B = a->B; p.Bp = a->Bp; p.N = a->N; p.Np = a->Np; p.k = a->k_blocks; p.act = a->act;
  mlp::dims_of(*a, p.dim, p.real);
  const mlp::Layout w = mlp::layout(*a, p.dim);
  OCF_CHECK(a->work_bytes >= (int64_t)w.total, "ocf_mlp_step: workspace too small");
  char* ws = reinterpret_cast<char*>(a->work);
  for (int i = 0; i < p.L; ++i) p.h[i] = reinterpret_cast<float*>(ws + w.h[i]);
  for (int i = 0; i <= p.L; ++i) p.d[i] = reinterpret_cast<float*>(ws + w.d[i]);
  for (int i = 1; i <= p.L; ++i) p.g[i] = reinterpret_cast<float*>(ws + w.g[i]);
  for (int i = 0; i <= p.L; ++i) p.colp[i] = reinterpret_cast<float*>(ws + w.colp[i]);
  p.rowp = reinterpret_cast<float*>(ws + w.rowp);
  p.totp = reinterpret_cast<float*>(ws + w.totp);
  for (int j = 0; j < 3; ++j) p.x[j] = a->x[j];
  p.ld_x = a->ld_x; p.rows = a->rows; p.om = a->out_mask; p.tg = a->targets; p.ld_t = a->ld_t;
  for (int i = 0; i <= p.L; ++i) {
    p.W[i] = a->W[i]; p.b[i] = a->b[i]; p.sW1[i] = a->sW1[i]; p.sW2[i] = a->sW2[i]; p.sb1[i] = a->sb1[i];
    p.sb2[i] = a->sb2[i]; p.sh[i] = a->shadow[i];
  }
  p.sh_blk = a->shadow_blocked;
  p.op = a->opt;
  p.stats = a->stats;
  p.bar = a->barrier;
  p.err = async_error_word();
  p.max_polls = 1 << 22;
  p.trace = a->trace;
  // every workgroup must be resident for the grid barriers; by default one per tile of the busiest phase, at
  // most 128 (the barriers' arrivals grow with the grid)
  int tiles = 0;
  {
    const int bt = p.Bp / mlp::TT;
    for (int i = 0; i <= p.L; ++i) tiles = std::max(tiles, bt * (p.dim[i + 1] / mlp::TT));
    for (int i = p.L; i >= 0; --i)
      tiles = std::max(tiles, (i > 0 ? bt * (p.dim[i] / mlp::TT) : 0) + (p.dim[i] / mlp::TT) * (p.dim[i + 1] / mlp::TT));
  }
  int wgs = a->wgs > 0 ? a->wgs : std::min(tiles, 128);
  int cus = 0, dev = 0;
  OCF_HIP(hipGetDevice(&dev));
  OCF_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  OCF_CHECK(wgs <= cus, "ocf_mlp_step: wgs must not exceed the CU count (grid barriers)");
  hipStream_t s = (hipStream_t)stream;
  switch (a->compute_dtype) {
    case OCF_F16: mlp::launch<_Float16>(*a, p, wgs, s); break;
    case OCF_BF16: mlp::launch<__bf16>(*a, p, wgs, s); break;
    case OCF_F32: mlp::launch<float>(*a, p, wgs, s); break;
    default: throw std::runtime_error("ocf_mlp_step: bad compute dtype");
  }
  OCF_TRY_END
}
