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
  float* colp[MAXL + 1];  // colp[i]: [Bp / 32][dim[i+1]] column sums of delta_i per 32-row block (bias gradients)
  float* am[MAXL];        // am[i], dm[i] (dropout only): layer i's activation before dropout, mask / keep
  float* dm[MAXL];
  float keep; uint64_t seed, stream; uint8_t* mask[MAXL];
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
// (barrier nb is passed when it reaches nb * grid); bar[1] counts the workgroups leaving the kernel and the
// last one resets both words (grid_exit), so they are zero for the next launch.  Bounded and fail-safe: a
// workgroup that gives up (not every workgroup resident) POISONS the barrier -- it sets bar[0]'s top bit with a
// compare-and-swap on the count it last saw, so the poison lands only while the barrier is still incomplete --
// and records OCF_ASYNC_MLP_BARRIER.  Every workgroup then finds the bit (its arrival's returned value or its
// polls), and grid_sync returns false: the caller leaves the kernel without any further write.  Nobody passes
// a poisoned barrier, so no weight, bias or slot is written after it; a residency failure shows at the first
// barrier (once every workgroup has arrived there, all are resident), before the first parameter write, so
// the step's parameters and slots stay untouched (tests/test_mlp_step_gpu.py::test_mlp_barrier_gives_up_safely).
// max_polls < 0 is fault injection for that test: workgroup 0 never arrives at the first barrier and poisons it.
constexpr uint32_t BAR_POISON = 0x80000000u;
__device__ __forceinline__ bool grid_sync(const P& p, int& tn, int& nb) {
  __shared__ int bar_ok;
  mark(p, tn);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");       // this wave's write-through stores have landed
  __syncthreads();
  ++nb;
  if (threadIdx.x == 0) {
    const uint32_t target = (uint32_t)nb * gridDim.x;
    const bool inject = p.max_polls < 0 && blockIdx.x == 0 && nb == 1;
    uint32_t v = inject ? __hip_atomic_load(&p.bar[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                        : __hip_atomic_fetch_add(&p.bar[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    int it = 0;
    bool ok;
    for (;;) {
      if (v & BAR_POISON) { ok = false; break; }
      if (v >= target) { ok = true; break; }
      if (inject || ++it > p.max_polls) {
        // give up: poison unless the count moved since v was read (then v holds the new count: test it again)
        if (__hip_atomic_compare_exchange_strong(&p.bar[0], &v, v | BAR_POISON, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT)) {
          __hip_atomic_store(p.err, (uint32_t)OCF_ASYNC_MLP_BARRIER, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          ok = false;
          break;
        }
        continue;
      }
      __builtin_amdgcn_s_sleep(1);
      v = __hip_atomic_load(&p.bar[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    bar_ok = ok ? 1 : 0;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (no instruction: keeps the loads below the poll)
  __syncthreads();
  mark(p, tn);
  return bar_ok != 0;
}
__device__ __forceinline__ void grid_exit(const P& p) {
  if (threadIdx.x == 0) {
    if (__hip_atomic_fetch_add(&p.bar[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u == gridDim.x) {
      __hip_atomic_store(&p.bar[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&p.bar[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ---- one 32 x 32 tile of C = A B per workgroup, K split over the four waves: each wave stages its quarter of
// K through its own LDS region in chunks of KC and the four partial tiles are summed in wave order through
// LDS.  (Keeping the next chunk's loads in flight during the MFMAs raised the kernel to ~300 VGPRs and cost
// Jester ~10 %: its waves walk one chunk.)  A phase of
// the Jester model has 16-96 such tiles, so every workgroup of the grid has work and a wave walks one or two
// chunks instead of a workgroup walking the whole K.  a(r, k) / b(n, k) return 4 consecutive fp32 elements
// along the operand's contiguous direction (r .. r+3 when A_RFAST / B_NFAST, else k .. k+3), rounded to CT
// when staged (as the MFMA operand staging of the other paths); every lane issues all of a chunk's loads
// before it writes any (the accessors are branch-free).  (A 64 x 64 shape with one quadrant per wave was
// measured for the wide GEMMs of ML-100K / ML-1M-sized models and removed: DESIGN.md §1.)
constexpr int TT = 32;
template <typename CT> struct Geo {
  static constexpr int KC = sizeof(CT) == 2 ? 64 : 32;     // K chunk
  static constexpr int PAD = sizeof(CT) == 2 ? 8 : 4;
  static constexpr int S = KC + PAD;                       // LDS row stride: 144 B
  static constexpr int STAGE = WAVES * 2 * TT * S * (int)sizeof(CT);   // four waves' A + B
  static constexpr int RED = WAVES * TT * (TT + 1) * 4;
  static constexpr int CS_OFF = STAGE > RED ? STAGE : RED;
  static constexpr int BYTES = CS_OFF + WAVES * TT * 4;
};

// one operand's chunk: R rows x KC, loaded by NP participants (the lanes of a wave) as RUNS float4 each
template <typename CT, bool FAST_R, int R, int NP>
struct Chunk {
  static constexpr int KC = Geo<CT>::KC, S = Geo<CT>::S, RUNS = R * KC / 4 / NP;
  float4 v[RUNS];
  __device__ __forceinline__ static void at(int u, int& r, int& k) {
    if (FAST_R) { r = 4 * (u % (R / 4)); k = u / (R / 4); }
    else { r = u / (KC / 4); k = 4 * (u % (KC / 4)); }
  }
  template <typename F>
  __device__ __forceinline__ void load(F& f, int r0, int k0, int kc, int pid) {
#pragma unroll
    for (int j = 0; j < RUNS; ++j) {
      int r, k;
      at(pid + NP * j, r, k);
      v[j] = f(r0 + r, k0 + (k < kc ? k : 0));            // past the chunk's end: a valid address, unused
    }
  }
  __device__ __forceinline__ void store(CT* dst, int pid) const {
#pragma unroll
    for (int j = 0; j < RUNS; ++j) {
      int r, k;
      at(pid + NP * j, r, k);
      const float e[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (FAST_R) dst[(r + q) * S + k] = CvtT<CT>::to(e[q]);
        else dst[r * S + k + q] = CvtT<CT>::to(e[q]);
      }
    }
  }
};

// acc += the 32 x 32 product of LDS rows sA[0..31] x sB[0..31] over kc (a multiple of 16)
template <typename CT>
__device__ __forceinline__ void mfma_chunk(ocf_f16v& acc, const CT* sA, const CT* sB, int kc) {
  constexpr int S = Geo<CT>::S;
  const int lane = threadIdx.x & 63, r = lane & 31, hf = lane >> 5;
  if constexpr (sizeof(CT) == 2) {
    using V = typename std::conditional<std::is_same<CT, _Float16>::value, ocf_h8, ocf_b8>::type;
    for (int ks = 0; ks < kc; ks += 16) {
      V fa, fb;
      __builtin_memcpy(&fa, sA + r * S + ks + 8 * hf, 16);
      __builtin_memcpy(&fb, sB + r * S + ks + 8 * hf, 16);
      if constexpr (std::is_same<CT, _Float16>::value)
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa, fb, acc, 0, 0, 0);
      else
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb, acc, 0, 0, 0);
    }
  } else {
    for (int ks = 0; ks < kc; ks += 2)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(sA[r * S + ks + hf], sB[r * S + ks + hf], acc, 0, 0, 0);
  }
}

// a thread's share of a finished tile: NE rows m[] of one column n
template <int NE> struct Frag {
  int n;
  int m[NE];
  float v[NE];
};

template <typename CT, bool A_RFAST, bool B_NFAST, typename FA, typename FB>
__device__ __forceinline__ Frag<4> tile_s(char* lds, int m0, int n0, int K, FA&& a, FB&& b) {
  constexpr int S = Geo<CT>::S, KC = Geo<CT>::KC;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  CT* sA = reinterpret_cast<CT*>(lds) + wave * 2 * TT * S;
  CT* sB = sA + TT * S;
  const int kw = K / WAVES, kb = wave * kw;             // K % 64 == 0: kw is a multiple of 16
  Chunk<CT, A_RFAST, TT, 64> ca;
  Chunk<CT, B_NFAST, TT, 64> cb;
  ocf_f16v acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  for (int k0 = 0; k0 < kw; k0 += KC) {
    const int kc = kw - k0 < KC ? kw - k0 : KC;
    ca.load(a, m0, kb + k0, kc, lane);
    cb.load(b, n0, kb + k0, kc, lane);
    ca.store(sA, lane);
    cb.store(sB, lane);
    __syncthreads();
    mfma_chunk<CT>(acc, sA, sB, kc);
    __syncthreads();
  }
  // the four K quarters, summed in wave order (C layout of v_mfma_f32_32x32x*: register q holds row
  // (q & 3) + 8 (q >> 2) + 4 hf, column lane & 31)
  float* red = reinterpret_cast<float*>(lds);
  const int r = lane & 31, hf = lane >> 5;
#pragma unroll
  for (int q = 0; q < 16; ++q) red[(wave * TT + (q & 3) + 8 * (q >> 2) + 4 * hf) * (TT + 1) + r] = acc[q];
  __syncthreads();
  Frag<4> f;
  f.n = n0 + (threadIdx.x & 31);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int rr = (threadIdx.x >> 5) + 8 * j, cc = threadIdx.x & 31;
    float s = red[rr * (TT + 1) + cc];
#pragma unroll
    for (int w = 1; w < WAVES; ++w) s += red[(w * TT + rr) * (TT + 1) + cc];
    f.m[j] = m0 + rr;
    f.v[j] = s;
  }
  __syncthreads();
  return f;
}

// the column sums of a fragment's tile over its 32 rows in a fixed order (a thread's rows, the two half-waves,
// the four waves through LDS), written to colp[row block][column] (ld W)
template <typename CT>
__device__ __forceinline__ void frag_colsum(char* lds, const Frag<4>& f, int m0, float* colp, int W) {
  float s = (f.v[0] + f.v[1]) + (f.v[2] + f.v[3]);
  s += __shfl_xor(s, 32, 64);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float* cs = reinterpret_cast<float*>(lds + Geo<CT>::CS_OFF);
  if (lane < 32) cs[wave * TT + lane] = s;
  __syncthreads();
  if (threadIdx.x < TT) {
    float c = cs[threadIdx.x];
#pragma unroll
    for (int w = 1; w < WAVES; ++w) c += cs[w * TT + threadIdx.x];
    pub(&colp[(int64_t)(m0 / TT) * W + f.n], c);
  }
}

__device__ __forceinline__ float4 ld4(const float* q) { return *reinterpret_cast<const float4*>(q); }

// ---- operand views
// layer-0 input of batch row b, padded columns c .. c+3 (one block: Np % 4 == 0): row rows[b] of the caller's
// [n][ld_x] arrays, zero past the batch and in the block padding (element loads through selected addresses: no
// branches)
__device__ __forceinline__ float4 x4(const P& p, int b, int c) {
  const int blk = c / p.Np, n = c - blk * p.Np;
  const float* row = p.x[blk] + p.rows[b < p.B ? b : p.B - 1] * p.ld_x;
  float e[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) e[q] = *((b < p.B && n + q < p.N) ? row + n + q : g_zero);
  return make_float4(e[0], e[1], e[2], e[3]);
}
// element offset of batch row m, column n of the output mask / targets
__device__ __forceinline__ int64_t t_off(const P& p, int m, int n) {
  return p.rows[m < p.B ? m : p.B - 1] * p.ld_t + (n < p.N ? n : 0);
}
__device__ __forceinline__ int64_t shadow_index(const P& p, int i, int r, int c) {
  const int C = i == p.L ? p.dim[i] : p.dim[i + 1];
  if (!p.sh_blk) return (int64_t)r * C + c;
  return ((int64_t)(r >> 6) * (C >> 6) + (c >> 6)) * 4096 + (r & 63) * 64 + (c & 63);
}

// the update of a thread's NE elements of weight i (rows r[q], column c of a [R][C] weight): the parameters and
// slots are loaded before the tile's GEMM (load), the update applied from its gradients after it (apply)
template <typename CT, int KIND, int NE>
struct TileUpdate {
  float w[NE], a[NE], bb[NE];
  __device__ __forceinline__ int64_t at(const P& p, int i, int r, int c) const {
    return (int64_t)r * (i == p.L ? p.dim[i] : p.dim[i + 1]) + c;
  }
  __device__ __forceinline__ void load(const P& p, int i, const int* r, int c) {
#pragma unroll
    for (int q = 0; q < NE; ++q) {
      const int64_t e = at(p, i, r[q], c);
      w[q] = p.W[i][e];
      a[q] = p.sW1[i] ? p.sW1[i][e] : 0.f;
      bb[q] = p.sW2[i] ? p.sW2[i][e] : 0.f;
    }
  }
  __device__ __forceinline__ void apply(const P& p, int i, const float* g, const int* r, int c) {
#pragma unroll
    for (int q = 0; q < NE; ++q) {
      const int64_t e = at(p, i, r[q], c);
      opt_update_k<KIND>(p.op, g[q], w[q], a[q], bb[q]);
      p.W[i][e] = w[q];
      if (p.sW1[i]) p.sW1[i][e] = a[q];
      if (p.sW2[i]) p.sW2[i][e] = bb[q];
      if constexpr (sizeof(CT) == 2)
        if (p.sh[i]) reinterpret_cast<CT*>(p.sh[i])[shadow_index(p, i, r[q], c)] = CvtT<CT>::to(w[q]);
    }
  }
};

// bias i: db[n] = gscale * sum over the Bp / 32 row blocks of the column partials the producer of delta_i wrote
// (block order), then the update
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

// ---- phase epilogues, for either tile shape
// hidden layer i's output: a = act(v + b), h = dropout(a) (model.py:64-73; the layer-wise path's Philox stream
// and formula: mask = floor(keep + U(seed, stream + i, m * W + n)), h = a / keep * mask)
template <int NE>
__device__ __forceinline__ void epi_forward(const P& p, int i, const Frag<NE>& f) {
  const int Wd = p.dim[i + 1], n = f.n;
  const float bias = p.b[i][n];
  const bool live_n = n < p.real[i + 1];
#pragma unroll
  for (int j = 0; j < NE; ++j) {
    const int m = f.m[j];
    const int64_t idx = (int64_t)m * Wd + n;
    const float a = (m < p.B && live_n) ? act_apply(p.act, f.v[j] + bias) : 0.f;
    float h = a;
    if (p.keep < 1.f) {
      const float mk = floorf(p.keep + philox_uniform(p.seed, p.stream + i, (uint64_t)idx));
      h = (a / p.keep) * mk;
      p.mask[i][idx] = (uint8_t)mk;                   // the caller's record (read after the launch)
      pub(&p.am[i][idx], a);
      pub(&p.dm[i][idx], mk / p.keep);
    }
    pub(&p.h[i][idx], h);
  }
}

// delta of hidden layer i's output from v = (delta_{i+1} W_{i+1}^T): v * (mask / keep) * act'(a)
template <int NE>
__device__ __forceinline__ void epi_delta(const P& p, int i, const Frag<NE>& f, Frag<NE>& dv, const float* av,
                                          const float* dmv) {
  const int Wd = p.dim[i + 1], n = f.n;
  dv.n = n;
#pragma unroll
  for (int j = 0; j < NE; ++j) {
    const int m = f.m[j];
    float d = 0.f;
    if (m < p.B && n < p.real[i + 1]) {
      d = f.v[j];
      if (p.keep < 1.f) d = d * dmv[j];
      d = d * act_grad(p.act, av[j]);
    }
    dv.m[j] = m;
    dv.v[j] = d;
    pub(&p.d[i][(int64_t)m * Wd + n], d);
  }
}

template <typename CT, int KIND>
__global__ void __launch_bounds__(THREADS) mlp_step_kernel(P p) {
  __shared__ __attribute__((aligned(16))) char lds[Geo<CT>::BYTES];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int gtid = blockIdx.x * THREADS + threadIdx.x, gthreads = gridDim.x * THREADS;
  const int L = p.L, Bt = p.Bp / TT;
  const float gs = p.op.gscale;
  const int c = threadIdx.x & 31;               // a thread's column in every tile; rows (threadIdx.x >> 5) + 8 j
  int tn = 0, nb = 0;
  mark(p, tn);

  // ---- forward: h_i = dropout(act(src W_i + b_i)); padded rows / units are zero
  for (int i = 0; i < L; ++i) {
    const int K = p.dim[i], Wd = p.dim[i + 1], nt = Wd / TT;
    auto Bw = [&](int n, int k) { return ld4(p.W[i] + (int64_t)k * Wd + n); };
    for (int t = blockIdx.x; t < Bt * nt; t += gridDim.x) {
      const int m0 = (t / nt) * TT, n0 = (t % nt) * TT;
      if (i == 0)      // (one accessor per call: a select inside it would split the chunk's loads)
        epi_forward(p, i, tile_s<CT, false, true>(lds, m0, n0, K, [&](int m, int k) { return x4(p, m, k); }, Bw));
      else
        epi_forward(p, i, tile_s<CT, false, true>(lds, m0, n0, K,
                                                  [&](int m, int k) { return ldc4(p.h[i - 1], (int64_t)m * K + k); }, Bw));
    }
    if (!grid_sync(p, tn, nb)) return grid_exit(p);
  }
  // ---- output layer + masked MSE: y = M (h W_L + b_L); e = y - T; delta_L = e M; per-tile statistics and
  // the column sums of delta_L (b_L's gradient).  W_L is stored transposed ([Np][K]): B(n, k) = W_L[n][k].
  {
    const int K = p.dim[L], nt = p.Np / TT;
    auto A = [&](int m, int k) { return ldc4(p.h[L - 1], (int64_t)m * K + k); };
    auto Bw = [&](int n, int k) { return ld4(p.W[L] + (int64_t)n * K + k); };
    for (int t = blockIdx.x; t < Bt * nt; t += gridDim.x) {
      const int m0 = (t / nt) * TT, n0 = (t % nt) * TT, n = n0 + c;
      const float bias = p.b[L][n];
      float mkv[4], ttv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {        // the mask / target loads fly during the GEMM
        const int64_t o = t_off(p, m0 + (threadIdx.x >> 5) + 8 * j, n);
        mkv[j] = p.om[o];
        ttv[j] = p.tg[o];
      }
      const Frag<4> v = tile_s<CT, false, false>(lds, m0, n0, K, A, Bw);
      Frag<4> dl;
      dl.n = n;
      float sse = 0.f, sae = 0.f, cnt = 0.f, rs[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = v.m[j];
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
        dl.m[j] = m;
        dl.v[j] = d;
        rs[j] = se;
      }
      // row sums over the tile's 32 columns (the 32 lanes of each half-wave), in a fixed butterfly order
      for (int o = 16; o > 0; o >>= 1)
#pragma unroll
        for (int j = 0; j < 4; ++j) rs[j] += __shfl_xor(rs[j], o, 64);
      if ((lane & 31) == 0)
#pragma unroll
        for (int j = 0; j < 4; ++j) pub(&p.rowp[(int64_t)(n0 / TT) * p.Bp + v.m[j]], rs[j]);
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
      frag_colsum<CT>(lds, dl, m0, p.colp[L], p.Np);
    }
    if (!grid_sync(p, tn, nb)) return grid_exit(p);
  }
  // ---- backward, layer by layer from the output
  for (int i = L; i >= 0; --i) {
    const int Wi = p.dim[i + 1];                 // layer i's output width (padded)
    const int Ki = p.dim[i];                     // its input width
    // delta of layer i - 1's output: (delta_i W_i^T) * dropout' * act'(a_{i-1}), with its column sums
    const int nd = i > 0 ? Bt * (Ki / TT) : 0;
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
      if (i == L && last) {
        // the step's statistics from the per-wave partials, by the whole workgroup in a fixed order: each wave
        // sums its stride of the slots (8 loads in flight), then the wave butterfly, then the waves through LDS
        const int slots = Bt * (p.Np / TT) * WAVES, ncb = p.Np / TT;
        float a[3] = {0.f, 0.f, 0.f};
        for (int t0 = threadIdx.x; t0 < slots; t0 += 8 * THREADS) {
          float v[8][3];
#pragma unroll
          for (int u = 0; u < 8; ++u)
#pragma unroll
            for (int k = 0; k < 3; ++k) {
              const int t = t0 + u * THREADS;
              v[u][k] = t < slots ? ldc(p.totp, (int64_t)t * 3 + k) : 0.f;
            }
#pragma unroll
          for (int u = 0; u < 8; ++u)
#pragma unroll
            for (int k = 0; k < 3; ++k) a[k] += v[u][k];
        }
        for (int k = 0; k < 3; ++k)
          for (int o = 32; o > 0; o >>= 1) a[k] += __shfl_xor(a[k], o, 64);
        float* ws = reinterpret_cast<float*>(lds + Geo<CT>::CS_OFF);
        __syncthreads();
        if (lane == 0)
          for (int k = 0; k < 3; ++k) ws[wave * 3 + k] = a[k];
        __syncthreads();
        if (threadIdx.x == 0) {
          for (int k = 0; k < 3; ++k) p.stats[k] = ((ws[k] + ws[3 + k]) + ws[6 + k]) + ws[9 + k];
          p.stats[3] = 0.f;
        }
        // per-row sums over the 32-column blocks, one thread per row, 8 loads in flight
        for (int b = threadIdx.x; b < p.Bp; b += THREADS) {
          float r = 0.f;
          for (int c0 = 0; c0 < ncb; c0 += 8) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = c0 + u < ncb ? ldc(p.rowp, (int64_t)(c0 + u) * p.Bp + b) : 0.f;
#pragma unroll
            for (int u = 0; u < 8; ++u) r += v[u];
          }
          p.stats[4 + b] = r;
        }
      }
      bias_update<KIND>(p, i, sid, sthreads);
    };
    const int T = nd + ng, idle = (int)gridDim.x - T;
    const bool side_idle = idle >= (int)gridDim.x / 4;
    if (side_idle && (int)blockIdx.x >= T)
      side(((int)blockIdx.x - T) * THREADS + threadIdx.x, idle * THREADS, blockIdx.x == gridDim.x - 1);
    for (int t = blockIdx.x; t < T; t += gridDim.x) {
      if (t < nd) {
        const int ct = Ki / TT, m0 = (t / ct) * TT, n0 = (t % ct) * TT, n = n0 + c;
        // the activation (and dropout scale) of layer i - 1 in flight during the GEMM
        float av[4], dmv[4];
        const float* asrc = p.keep < 1.f ? p.am[i - 1] : p.h[i - 1];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int64_t o = (int64_t)(m0 + (threadIdx.x >> 5) + 8 * j) * Ki + n;
          av[j] = ldc(asrc, o);
          dmv[j] = p.keep < 1.f ? ldc(p.dm[i - 1], o) : 1.f;
        }
        auto Ad = [&](int m, int k) { return ldc4(p.d[i], (int64_t)m * Wi + k); };
        Frag<4> v;
        if (i == L)      // B(n = input unit, k = output unit) = W_L[k][n], contiguous along n
          v = tile_s<CT, false, true>(lds, m0, n0, Wi, Ad, [&](int nn, int k) { return ld4(p.W[L] + (int64_t)k * Ki + nn); });
        else             // B(n = input unit, k = output unit) = W_i[n][k], contiguous along k
          v = tile_s<CT, false, false>(lds, m0, n0, Wi, Ad, [&](int nn, int k) { return ld4(p.W[i] + (int64_t)nn * Wi + k); });
        Frag<4> dv;
        epi_delta(p, i - 1, v, dv, av, dmv);
        frag_colsum<CT>(lds, dv, m0, p.colp[i - 1], Ki);
        continue;
      }
      const int u = t - nd, ct = gc / TT, m0 = (u / ct) * TT, n0 = (u % ct) * TT, n = n0 + c;
      int rr[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) rr[j] = m0 + (threadIdx.x >> 5) + 8 * j;
      TileUpdate<CT, KIND, 4> up;
      if (i == 0) up.load(p, 0, rr, n);             // W_0's parameters and slots in flight during the GEMM
      Frag<4> v;
      if (i == L)        // dW_L[n][j] = sum_b delta_L[b][n] h_{L-1}[b][j]
        v = tile_s<CT, true, true>(lds, m0, n0, p.Bp, [&](int m, int k) { return ldc4(p.d[L], (int64_t)k * Wi + m); },
                                   [&](int nn, int k) { return ldc4(p.h[L - 1], (int64_t)k * Ki + nn); });
      else if (i > 0)    // dW_i[k][j] = sum_b h_{i-1}[b][k] delta_i[b][j]
        v = tile_s<CT, true, true>(lds, m0, n0, p.Bp, [&](int m, int k) { return ldc4(p.h[i - 1], (int64_t)k * Ki + m); },
                                   [&](int nn, int k) { return ldc4(p.d[i], (int64_t)k * Wi + nn); });
      else               // dW_0[k][j] = sum_b x[b][k] delta_0[b][j]
        v = tile_s<CT, true, true>(lds, m0, n0, p.Bp, [&](int m, int k) { return x4(p, k, m); },
                                   [&](int nn, int k) { return ldc4(p.d[0], (int64_t)k * Wi + nn); });
      float gv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) gv[j] = v.v[j] * gs;
      if (i == 0) {      // nothing reads W_0 any more: update it from the tile (padded elements: zero gradient)
        up.apply(p, 0, gv, rr, n);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) pub(&p.g[i][(int64_t)rr[j] * gc + n], gv[j]);
      }
    }
    if (!side_idle) side(gtid, gthreads, blockIdx.x == gridDim.x - 1);
    if (i > 0 && !grid_sync(p, tn, nb)) return grid_exit(p);
  }
  grid_exit(p);
  mark(p, tn);
}

struct Layout {
  size_t h[MAXL], d[MAXL + 1], g[MAXL], colp[MAXL + 1], am[MAXL], dm[MAXL], rowp, totp, total;
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
  for (int i = 0; i < L; ++i) {
    const size_t n = a.keep < 1.f ? (size_t)a.Bp * dim[i + 1] : 0;
    w.am[i] = take(n);
    w.dm[i] = take(n);
  }
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
  OCF_CHECK(a.keep > 0.f && a.keep <= 1.f, "ocf_mlp_step: keep in (0, 1]");
  if (a.keep < 1.f)
    for (int i = 0; i < a.n_hidden; ++i) OCF_CHECK(a.mask[i] != nullptr, "ocf_mlp_step: dropout masks");
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

namespace ocf {
int g_mlp_max_polls = 1 << 22;   // ocf_mlp_step's bounded barrier wait (ocf_set_tuning "mlp_max_polls"; < 0: fault injection)
}

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
  for (int i = 0; i < p.L; ++i) {
    p.am[i] = reinterpret_cast<float*>(ws + w.am[i]);
    p.dm[i] = reinterpret_cast<float*>(ws + w.dm[i]);
    p.mask[i] = a->mask[i];
  }
  p.keep = a->keep; p.seed = a->seed; p.stream = a->stream;
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
  p.max_polls = g_mlp_max_polls;
  p.trace = a->trace;
  // every workgroup must be resident for the grid barriers; by default one per 32 x 32 tile of the busiest
  // phase, at most 128 (the barriers' arrivals grow with the grid) -- or one per CU (at most 256) when a phase
  // has more than 256 tiles (the wide output layers of the I-AutoRec models on the opt-in generator path)
  int tiles = 0;
  {
    const int bt = p.Bp / mlp::TT;
    for (int i = 0; i <= p.L; ++i) tiles = std::max(tiles, bt * (p.dim[i + 1] / mlp::TT));
    for (int i = p.L; i >= 0; --i)
      tiles = std::max(tiles, (i > 0 ? bt * (p.dim[i] / mlp::TT) : 0) + (p.dim[i] / mlp::TT) * (p.dim[i + 1] / mlp::TT));
  }
  int cus = 0, dev = 0;
  OCF_HIP(hipGetDevice(&dev));
  OCF_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  // (the default never exceeds the CU count: a partitioned device may have fewer CUs than tiles)
  int wgs = tiles > 256 ? std::min(cus, 256) : std::min({tiles, 128, cus});
  if (a->wgs > 0) {
    OCF_CHECK(a->wgs <= cus, "ocf_mlp_step: wgs must not exceed the CU count (grid barriers)");
    wgs = a->wgs;
  }
  hipStream_t s = (hipStream_t)stream;
  switch (a->compute_dtype) {
    case OCF_F16: mlp::launch<_Float16>(*a, p, wgs, s); break;
    case OCF_BF16: mlp::launch<__bf16>(*a, p, wgs, s); break;
    case OCF_F32: mlp::launch<float>(*a, p, wgs, s); break;
    default: throw std::runtime_error("ocf_mlp_step: bad compute dtype");
  }
  OCF_TRY_END
}
