// ocf_mlp_step (ocf.h): a small dense model's whole training step in one persistent launch.
//
// The dense path's step (split-K encoder, hidden-layer GEMMs, the masked-MSE decoder, the backward GEMMs
// with the fused optimizer, bias kernels, stats) is ~14 launches of 2-33 us on a model of 0.14 M
// parameters (train_jester.py's 200 -> 256 -> 256 -> 100, batch 128): every launch is a handful of
// workgroups waiting on latency, and the host spends longer issuing them than the GPU running them.
// Here a grid of a few dozen workgroups stays resident and walks the step's phases, each a set of
// 32 x 32 output tiles (one MFMA tile per wave, operands straight from the L2-resident weights and
// activations), separated by grid barriers:
//   F_0 .. F_{L-1}  h_i = act(h_{i-1} W_i + b_i)                     (model.py:64-71)
//   OUT             y = M * (h_{L-1} W_L + b_L), e = y - T, delta_L = e * M, the step's statistics
//                   (model.py:81-86, train.py:49, 102-121)
//   BACK_L          stats; db_L + its update; delta_{L-1} = (delta_L W_L^T) * act'; dW_L -> scratch
//   BACK_i          W_{i+1} updated from its scratch gradient (nothing reads it any more); db_i + update;
//                   delta_{i-1}; dW_i -> scratch
//   BACK_0          W_1 updated; db_0 + update; dW_0 tiles update W_0 directly
// (Keras computes every gradient from the weights before the step, train.py:50-51: a layer's weights
// change only after the phase that last reads them.)  Gradients are carried unscaled (e * M) and the
// MSE's 2 / (B N) applied in fp32 at the update, as on the other paths.
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
  float* rowp;            // [Np / 32][Bp] per column-tile row sse
  float* totp;            // [tiles][3] per output tile sse / sae / count
  uint32_t* bar; uint32_t* err; int max_polls;
  uint64_t* trace;
};

// workgroup 0 records the constant-rate clock (diagnostics: ocf.h OcfMlpStepArgs trace)
__device__ __forceinline__ void mark(const P& p, int& n) {
  if (p.trace && blockIdx.x == 0 && threadIdx.x == 0 && n < 24) p.trace[n] = wall_clock64();
  ++n;
}

// ---- grid barrier: arrive-count + generation (the last arrival clears the count and bumps the
// generation, so the words are ready for the next barrier and the next launch); agent-scope release /
// acquire so every workgroup's stores of the phase are visible to every XCD afterwards.  Bounded: a
// workgroup that gives up (not all workgroups resident) records the error word and continues.
__device__ __forceinline__ void grid_sync(const P& p, int& tn) {
  mark(p, tn);
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t gen = __hip_atomic_load(&p.bar[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const uint32_t arrived = __hip_atomic_fetch_add(&p.bar[0], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) + 1;
    if (arrived == gridDim.x) {
      __hip_atomic_store(&p.bar[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&p.bar[1], gen + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      int it = 0;
      while (__hip_atomic_load(&p.bar[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gen) {
        __builtin_amdgcn_s_sleep(1);
        if (++it > p.max_polls) {
          __hip_atomic_store(p.err, (uint32_t)OCF_ASYNC_MLP_BARRIER, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
  mark(p, tn);
}

// ---- one 64 x 64 tile of C = A B per workgroup: K in chunks of KC staged through LDS (every thread issues its
// 16 loads of a chunk together, in the source's contiguous direction), each wave then runs its 32 x 32
// quarter on MFMA from LDS.  a(m, k) / b(k, n) return fp32 values, rounded to CT when staged (as the MFMA
// operand staging of the other paths rounds them); A_MFAST / B_NFAST: the source is contiguous along m / n.
constexpr int TT = 64, KC = 64;
template <typename CT> struct Lds {
  static constexpr int PAD = sizeof(CT) == 2 ? 8 : 4;      // row stride 144 B (16-bit) / 272 B (fp32)
  static constexpr int STRIDE = KC + PAD;
  static constexpr int BYTES = 2 * TT * STRIDE * (int)sizeof(CT);
};

// f(r, k) returns the element's ADDRESS (always a readable location: masked elements point at a zero word), so
// all 16 loads of a thread go out together before any is used (a value-returning accessor with branches let
// the compiler serialise them: one L2 / MALL round trip per element)
template <typename CT, bool FAST_R, typename F>
__device__ __forceinline__ void stage(CT* dst, int r0, int k0, F&& f) {
  constexpr int S = Lds<CT>::STRIDE;
  const int tid = threadIdx.x;
  const float* ad[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int e = tid * 16 + j;
    const int r = FAST_R ? e % TT : e / KC, k = FAST_R ? e / TT : e % KC;
    ad[j] = f(r0 + r, k0 + k);
  }
  float v[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) v[j] = *ad[j];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int e = tid * 16 + j;
    const int r = FAST_R ? e % TT : e / KC, k = FAST_R ? e / TT : e % KC;
    dst[r * S + k] = CvtT<CT>::to(v[j]);
  }
}

template <typename CT, bool A_MFAST, bool B_NFAST, typename FA, typename FB>
__device__ __forceinline__ ocf_f16v wg_tile(char* lds, int m0, int n0, int K, FA&& a, FB&& b) {
  constexpr int S = Lds<CT>::STRIDE;
  CT* sA = reinterpret_cast<CT*>(lds);
  CT* sB = sA + TT * S;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, r = lane & 31, hf = lane >> 5;
  const int wm = 32 * (wave >> 1), wn = 32 * (wave & 1);
  ocf_f16v acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  for (int k0 = 0; k0 < K; k0 += KC) {
    stage<CT, A_MFAST>(sA, m0, k0, a);
    stage<CT, B_NFAST>(sB, n0, k0, [&](int n, int k) { return b(k, n); });
    __syncthreads();
    if constexpr (sizeof(CT) == 2) {
      using V = typename std::conditional<std::is_same<CT, _Float16>::value, ocf_h8, ocf_b8>::type;
#pragma unroll
      for (int ks = 0; ks < KC / 16; ++ks) {
        V fa, fb;
        const int kk = 16 * ks + 8 * hf;
        __builtin_memcpy(&fa, sA + (wm + r) * S + kk, 16);
        __builtin_memcpy(&fb, sB + (wn + r) * S + kk, 16);
        if constexpr (std::is_same<CT, _Float16>::value)
          acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa, fb, acc, 0, 0, 0);
        else
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb, acc, 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < KC; ks += 2)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(sA[(wm + r) * S + ks + hf], sB[(wn + r) * S + ks + hf], acc, 0, 0, 0);
    }
    __syncthreads();
  }
  return acc;
}
// accumulator register -> (row, col) of the workgroup tile (C layout of v_mfma_f32_32x32x*, the wave's quarter)
__device__ __forceinline__ int tile_row(int reg) {
  return 32 * ((threadIdx.x >> 6) >> 1) + (reg & 3) + 8 * (reg >> 2) + 4 * ((threadIdx.x & 63) >> 5);
}
__device__ __forceinline__ int tile_col() { return 32 * ((threadIdx.x >> 6) & 1) + (threadIdx.x & 31); }

// ---- operand views
// layer-0 input of batch row b, padded column c (block c / Np): its address, or the zero word when padding
__device__ __forceinline__ const float* x_ptr(const P& p, int b, int c) {
  const int blk = c / p.Np, n = c - blk * p.Np;
  const int64_t row = p.rows[b < p.B ? b : p.B - 1];
  return (b < p.B && n < p.N) ? p.x[blk] + row * p.ld_x + n : g_zero;
}
__device__ __forceinline__ int64_t shadow_index(const P& p, int i, int r, int c) {
  const int C = i == p.L ? p.dim[i] : p.dim[i + 1];
  if (!p.sh_blk) return (int64_t)r * C + c;
  return ((int64_t)(r >> 6) * (C >> 6) + (c >> 6)) * 4096 + (r & 63) * 64 + (c & 63);
}

// the update of the 16 elements of weight i an MFMA accumulator covers, from their gradients (rows r[q], column c
// of a [R][C] weight): every load first, then the updates and the stores
template <typename CT, int KIND>
__device__ __forceinline__ void update_tile(const P& p, int i, const float* g, const int* r, int c) {
  const int C = i == p.L ? p.dim[i] : p.dim[i + 1];
  float w[16], a[16], bb[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int64_t e = (int64_t)r[q] * C + c;
    w[q] = p.W[i][e];
    a[q] = p.sW1[i] ? p.sW1[i][e] : 0.f;
    bb[q] = p.sW2[i] ? p.sW2[i][e] : 0.f;
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int64_t e = (int64_t)r[q] * C + c;
    opt_update_k<KIND>(p.op, g[q], w[q], a[q], bb[q]);
    p.W[i][e] = w[q];
    if (p.sW1[i]) p.sW1[i][e] = a[q];
    if (p.sW2[i]) p.sW2[i][e] = bb[q];
    if constexpr (sizeof(CT) == 2)
      if (p.sh[i]) reinterpret_cast<CT*>(p.sh[i])[shadow_index(p, i, r[q], c)] = CvtT<CT>::to(w[q]);
  }
}

// bias i: db[n] = gscale * sum_b delta_i[b][n] (batch rows in order; loads 16 at a time), then the update
template <int KIND>
__device__ __forceinline__ void bias_update(const P& p, int i, int gtid, int gthreads) {
  const int W = p.dim[i + 1], realw = p.real[i + 1];
  for (int n = gtid; n < realw; n += gthreads) {
    float s = 0.f;
    for (int b0 = 0; b0 < p.Bp; b0 += 16) {       // padded rows hold zero deltas
      float v[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] = p.d[i][(int64_t)(b0 + j) * W + n];
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if (b0 + j < p.B) s += v[j];
    }
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
    const float4 gv = *reinterpret_cast<const float4*>(g + e0);
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
  int tn = 0;
  mark(p, tn);

  // ---- forward: h_i = act(src W_i + b_i); padded rows / units are zero
  for (int i = 0; i < L; ++i) {
    const int K = p.dim[i], Wd = p.dim[i + 1], nt = Wd / TT;
    for (int t = blockIdx.x; t < Bt * nt; t += gridDim.x) {
      const int m0 = (t / nt) * TT, n0 = (t % nt) * TT;
      ocf_f16v acc;
      if (i == 0)
        acc = wg_tile<CT, false, true>(lds, m0, n0, K, [&](int m, int k) { return x_ptr(p, m, k); },
                                       [&](int k, int n) { return p.W[0] + (int64_t)k * Wd + n; });
      else
        acc = wg_tile<CT, false, true>(lds, m0, n0, K, [&](int m, int k) { return p.h[i - 1] + (int64_t)m * K + k; },
                                       [&](int k, int n) { return p.W[i] + (int64_t)k * Wd + n; });
      const int n = n0 + tile_col();
      const float bias = p.b[i][n];
      const bool live_n = n < p.real[i + 1];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int m = m0 + tile_row(q);
        const float v = (m < p.B && live_n) ? act_apply(p.act, acc[q] + bias) : 0.f;
        p.h[i][(int64_t)m * Wd + n] = v;
      }
    }
    grid_sync(p, tn);
  }
  // ---- output layer + masked MSE: y = M (h W_L + b_L); e = y - T; delta_L = e M; per-tile statistics
  {
    const int K = p.dim[L], nt = p.Np / TT;
    for (int t = blockIdx.x; t < Bt * nt; t += gridDim.x) {
      const int m0 = (t / nt) * TT, n0 = (t % nt) * TT;
      // W_L is stored transposed ([Np][K]): B(k, n) = W_L[n][k], contiguous along k
      const ocf_f16v acc = wg_tile<CT, false, false>(lds, m0, n0, K,
                                                     [&](int m, int k) { return p.h[L - 1] + (int64_t)m * K + k; },
                                                     [&](int k, int n) { return p.W[L] + (int64_t)n * K + k; });
      const int n = n0 + tile_col();
      const float bias = p.b[L][n];
      float sse = 0.f, sae = 0.f, cnt = 0.f, rs[16], mkv[16], ttv[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) {       // the mask / target loads first (clamped rows: always in bounds)
        const int m = m0 + tile_row(q);
        const int64_t o = p.rows[m < p.B ? m : p.B - 1] * p.ld_t + (n < p.N ? n : 0);
        mkv[q] = p.om[o];
        ttv[q] = p.tg[o];
      }
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int m = m0 + tile_row(q);
        float dl = 0.f, se = 0.f;
        if (m < p.B && n < p.N) {
          const float mk = mkv[q], tt = ttv[q];
          const float y = mk * (acc[q] + bias);
          const float e = y - tt;
          se = e * e;
          sse += se;
          sae += fabsf(e);
          cnt += (tt + y != 0.f) ? 1.f : 0.f;
          dl = e * mk;
        }
        p.d[L][(int64_t)m * p.Np + n] = dl;
        rs[q] = se;
      }
      // row sums over the wave's 32 columns (the 32 lanes of each half-wave), in a fixed butterfly order
      for (int o = 16; o > 0; o >>= 1)
#pragma unroll
        for (int q = 0; q < 16; ++q) rs[q] += __shfl_xor(rs[q], o, 64);
      const int ct = n0 / 32 + (wave & 1);        // the wave's 32-column block
      if ((lane & 31) == 0)
#pragma unroll
        for (int q = 0; q < 16; ++q) p.rowp[(int64_t)ct * p.Bp + m0 + tile_row(q)] = rs[q];
      for (int o = 32; o > 0; o >>= 1) {
        sse += __shfl_xor(sse, o, 64);
        sae += __shfl_xor(sae, o, 64);
        cnt += __shfl_xor(cnt, o, 64);
      }
      if (lane == 0) {
        const int64_t slot = (int64_t)t * WAVES + wave;
        p.totp[slot * 3 + 0] = sse;
        p.totp[slot * 3 + 1] = sae;
        p.totp[slot * 3 + 2] = cnt;
      }
    }
    grid_sync(p, tn);
  }
  // ---- backward, layer by layer from the output
  for (int i = L; i >= 0; --i) {
    // the update of W_{i+1} from its scratch gradient: nothing reads W_{i+1} from here on
    if (i + 1 <= L) {
      const int R = i + 1 == L ? p.dim[L + 1] : p.dim[i + 1], C = i + 1 == L ? p.dim[L] : p.dim[i + 2];
      update_from<CT, KIND>(p, i + 1, p.g[i + 1], (int64_t)R * C, gtid, gthreads);
    }
    if (i == L && blockIdx.x == 0 && wave == 0) {
      // the step's statistics from the per-wave partials, in order
      const int slots = Bt * (p.Np / TT) * WAVES, ncb = p.Np / 32;
      float a[3] = {0.f, 0.f, 0.f};
      for (int t = lane; t < slots; t += 64)
        for (int k = 0; k < 3; ++k) a[k] += p.totp[(int64_t)t * 3 + k];
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
        for (int c = 0; c < ncb; ++c) r += p.rowp[(int64_t)c * p.Bp + b];
        p.stats[4 + b] = r;
      }
    }
    bias_update<KIND>(p, i, gtid, gthreads);
    const int Wi = p.dim[i + 1];                 // layer i's output width (padded)
    const int Ki = p.dim[i];                     // its input width
    // delta of layer i - 1's output: (delta_i W_i^T) * act'(h_{i-1})
    const int nd = i > 0 ? (Bt * (Ki / TT)) : 0;
    // dW_i: [input][output] (layer L: [output][input]) tiles, K = the batch rows
    const int gr = i == L ? Wi : Ki, gc = i == L ? Ki : Wi;
    const int ng = (gr / TT) * (gc / TT);
    for (int t = blockIdx.x; t < nd + ng; t += gridDim.x) {
      if (t < nd) {
        const int ct = Ki / TT, m0 = (t / ct) * TT, n0 = (t % ct) * TT;
        ocf_f16v acc;
        if (i == L)      // B(k = output unit, n = input unit) = W_L[k][n], contiguous along n
          acc = wg_tile<CT, false, true>(lds, m0, n0, Wi, [&](int m, int k) { return p.d[i] + (int64_t)m * Wi + k; },
                                         [&](int k, int n) { return p.W[L] + (int64_t)k * Ki + n; });
        else             // B(k = output unit, n = input unit) = W_i[n][k], contiguous along k
          acc = wg_tile<CT, false, false>(lds, m0, n0, Wi, [&](int m, int k) { return p.d[i] + (int64_t)m * Wi + k; },
                                          [&](int k, int n) { return p.W[i] + (int64_t)n * Wi + k; });
        const int n = n0 + tile_col();
        float hv[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) hv[q] = p.h[i - 1][(int64_t)(m0 + tile_row(q)) * Ki + n];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int m = m0 + tile_row(q);
          p.d[i - 1][(int64_t)m * Ki + n] = (m < p.B && n < p.real[i]) ? acc[q] * act_grad(p.act, hv[q]) : 0.f;
        }
        continue;
      }
      const int u = t - nd, ct = gc / TT, m0 = (u / ct) * TT, n0 = (u % ct) * TT;
      ocf_f16v acc;
      if (i == L)        // dW_L[n][j] = sum_b delta_L[b][n] h_{L-1}[b][j]
        acc = wg_tile<CT, true, true>(lds, m0, n0, p.Bp, [&](int m, int k) { return p.d[L] + (int64_t)k * Wi + m; },
                                      [&](int k, int n) { return p.h[L - 1] + (int64_t)k * Ki + n; });
      else if (i > 0)    // dW_i[k][j] = sum_b h_{i-1}[b][k] delta_i[b][j]
        acc = wg_tile<CT, true, true>(lds, m0, n0, p.Bp, [&](int m, int k) { return p.h[i - 1] + (int64_t)k * Ki + m; },
                                      [&](int k, int n) { return p.d[i] + (int64_t)k * Wi + n; });
      else               // dW_0[k][j] = sum_b x[b][k] delta_0[b][j]
        acc = wg_tile<CT, true, true>(lds, m0, n0, p.Bp, [&](int m, int k) { return x_ptr(p, k, m); },
                                      [&](int k, int n) { return p.d[0] + (int64_t)k * Wi + n; });
      const int c = n0 + tile_col();
      if (i == 0) {      // nothing reads W_0 any more: update it from the tile (padded elements have zero gradient)
        float gv[16];
        int rr[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          gv[q] = acc[q] * gs;
          rr[q] = m0 + tile_row(q);
        }
        update_tile<CT, KIND>(p, 0, gv, rr, c);
      } else {
#pragma unroll
        for (int q = 0; q < 16; ++q) p.g[i][(int64_t)(m0 + tile_row(q)) * gc + c] = acc[q] * gs;
      }
    }
    if (i > 0) grid_sync(p, tn);
  }
  mark(p, tn);
}

struct Layout {
  size_t h[MAXL], d[MAXL + 1], g[MAXL], rowp, totp, total;
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
  w.rowp = take((size_t)(a.Np / 32) * a.Bp);
  w.totp = take((size_t)(a.Bp / 64) * (a.Np / 64) * 4 * 3);
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
  // every workgroup must be resident for the grid barriers: a few dozen on 256 CUs
  int wgs = a->wgs > 0 ? a->wgs : 64;
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
