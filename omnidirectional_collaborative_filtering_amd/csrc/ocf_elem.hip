// Split-K reductions fused with the layer epilogues, elementwise optimizers, stats reduction,
// and the library's error state.
#include <atomic>
#include <cstring>
#include <mutex>
#include <string>
#include <type_traits>

#include "ocf_epilogues.h"
#include "ocf_internal.h"

namespace ocf {

static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }

namespace {
std::mutex g_async_mu;
uint32_t* g_async_host = nullptr;   // hipHostMalloc'd, coherent: kernels store to it, the host polls it
uint32_t* g_async_dev = nullptr;
const char* async_error_text(uint32_t code) {
  switch (code) {
    case OCF_ASYNC_PAIR_WAIT:
      return "ocf_gemm_pair: an input-layer workgroup gave up waiting for the row reduction (sync word behind its "
             "target: the word was written by someone else, or the count passed does not match it) and skipped "
             "its update; the weights of that launch are not a valid step";
    case OCF_ASYNC_ENC_WAIT:
      return "ocf_gather_encdec: a decoder chunk gave up waiting for its row's encoder chunks; that step's "
             "decoder outputs are not valid";
    case OCF_ASYNC_MLP_BARRIER:
      return "ocf_mlp_step: a grid barrier gave up waiting (not every workgroup was resident); that step's "
             "weights are not valid";
    default:
      return "asynchronous kernel error";
  }
}
}  // namespace

uint32_t* async_error_word() {
  std::lock_guard<std::mutex> lk(g_async_mu);
  if (!g_async_dev) {
    void* h = nullptr;
    OCF_HIP(hipHostMalloc(&h, 64, hipHostMallocCoherent | hipHostMallocMapped | hipHostMallocPortable));
    std::memset(h, 0, 64);
    void* d = nullptr;
    OCF_HIP(hipHostGetDevicePointer(&d, h, 0));
    g_async_host = static_cast<uint32_t*>(h);
    g_async_dev = static_cast<uint32_t*>(d);
  }
  return g_async_dev;
}

namespace {
uint32_t* g_gate_dev = nullptr;
std::atomic<uint32_t> g_encdec_gen{0};
}  // namespace

uint32_t* encdec_gate_word() {
  std::lock_guard<std::mutex> lk(g_async_mu);
  return g_gate_dev;
}
uint32_t encdec_generation() { return g_encdec_gen.load(); }
uint32_t next_encdec_generation() {
  {
    std::lock_guard<std::mutex> lk(g_async_mu);
    if (!g_gate_dev) {
      void* d = nullptr;
      OCF_HIP(hipMalloc(&d, 64));
      OCF_HIP(hipMemset(d, 0, 64));
      OCF_HIP(hipDeviceSynchronize());
      g_gate_dev = static_cast<uint32_t*>(d);
    }
  }
  uint32_t g = g_encdec_gen.fetch_add(1u) + 1u;
  if (g == 0) g = g_encdec_gen.fetch_add(1u) + 1u;   // (wrapped: 0 means "no launch")
  return g;
}

void check_async_errors() {
  uint32_t* h = g_async_host;
  if (!h) return;
  const uint32_t code = __atomic_exchange_n(h, 0u, __ATOMIC_ACQ_REL);
  if (code) throw std::runtime_error(std::string("error from an earlier launch: ") + async_error_text(code));
}

}  // namespace ocf

extern "C" int ocf_check_async(void) {
  OCF_TRY_BEGIN
  OCF_TRY_END
}

namespace ocf {

// Split-K reductions: grid (N/64, M/4); 256 threads = 64 columns x 4 rows, one output element per
// thread, slabs summed in a fixed order (4 independent partial sums for memory-level parallelism).
__device__ __forceinline__ float sum_slabs(const float* s, int splits, int64_t sstride) {
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

__global__ void __launch_bounds__(256) splitk_bias_act_kernel(const float* slabs, int splits, int64_t sstride, int M,
                                                              int N, BiasActParams p) {
  const int col = blockIdx.x * 64 + (threadIdx.x & 63);
  const int m = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (col >= N || m >= M) return;
  bias_act_store(p, m, col, sum_slabs(slabs + (int64_t)m * p.ld + col, splits, sstride));
}

// db_part[blockIdx.y][col] = gscale * sum of the block's 4 rows (fixed order)
__global__ void __launch_bounds__(256) splitk_grad_act_kernel(const float* slabs, int splits, int64_t sstride, int M,
                                                              int N, GradActParams p, float* db_part) {
  __shared__ float part[4][64];
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + cl;
  const int m = blockIdx.y * 4 + rg;
  float d = 0.f;
  if (col < N && m < M) {
    d = grad_act_value(p, m, col, sum_slabs(slabs + (int64_t)m * p.ld + col, splits, sstride));
    store_ct(p.d_out, p.d_dtype, (int64_t)m * p.ld + col, d);
  }
  part[rg][cl] = d;
  __syncthreads();
  if (rg == 0 && col < N && db_part)
    db_part[(int64_t)blockIdx.y * p.ld + col] = ((part[0][cl] + part[1][cl]) + (part[2][cl] + part[3][cl])) * p.gscale;
}

__global__ void opt_kernel(float* p, const float* g, float* s1, float* s2, int64_t n, OcfOptParams o) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) {
    float w = p[i];
    float a = s1 ? s1[i] : 0.f;
    float b = s2 ? s2[i] : 0.f;
    opt_update(o, g[i] * o.gscale, w, a, b);
    p[i] = w;
    if (s1) s1[i] = a;
    if (s2) s2[i] = b;
  }
}

// ocf_opt_step_ex: gradient in fp32 or bf16 (the data-parallel reduce-scatter's shard, no widening copy),
// and the updated parameter rounded once more into the compute-dtype shadow (the same RNE rounding the
// fused EPI_OPTIM epilogue and a torch .to() apply), so a sharded update leaves the shadow shard ready
// for the all-gather
template <typename GT, typename ST>
__global__ void __launch_bounds__(256) opt_ex_kernel(float* p, const GT* g, float* s1, float* s2, ST* sh, int64_t n,
                                                     OcfOptParams o) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) {
    float w = p[i];
    float a = s1 ? s1[i] : 0.f;
    float b = s2 ? s2[i] : 0.f;
    opt_update(o, (float)g[i] * o.gscale, w, a, b);
    p[i] = w;
    if (s1) s1[i] = a;
    if (s2) s2[i] = b;
    if constexpr (!std::is_same<ST, float>::value) sh[i] = (ST)w;
  }
}

// grid n/64; 256 threads = 64 columns x 4 partial groups; fixed summation order
__global__ void __launch_bounds__(256) bias_opt_partials_kernel(float* bvec, const float* db_part, int parts,
                                                                int64_t ld, int n, float* s1, float* s2, float* g_out,
                                                                OcfOptParams o) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + cl;
  // the group's rows grp, grp + 4, ... added in that order, 16 loads in flight (a one-load-at-a-time loop
  // took 40 us for the 512 partial rows of a 2,048-row batch: an 8-way feature rank's hidden bias)
  constexpr int NB = 16;
  float part = 0.f;
  if (i < n)
    for (int k0 = grp; k0 < parts; k0 += 4 * NB) {
      float x[NB];
#pragma unroll
      for (int j = 0; j < NB; ++j) x[j] = k0 + 4 * j < parts ? db_part[(int64_t)(k0 + 4 * j) * ld + i] : 0.f;
#pragma unroll
      for (int j = 0; j < NB; ++j)
        if (k0 + 4 * j < parts) part += x[j];
    }
  red[grp][cl] = part;
  __syncthreads();
  if (grp != 0 || i >= n) return;
  const float g = (red[0][cl] + red[1][cl]) + (red[2][cl] + red[3][cl]);
  if (g_out) {           // data-parallel: hand the gradient to the all-reduce instead
    g_out[i] = g;
    return;
  }
  float w = bvec[i];
  float a = s1 ? s1[i] : 0.f;
  float b = s2 ? s2[i] : 0.f;
  o.gscale = 1.f;        // partials are already scaled
  opt_update(o, g, w, a, b);
  bvec[i] = w;
  if (s1) s1[i] = a;
  if (s2) s2[i] = b;
}

// grid 1 + M/4: block 0 = fixed-order totals of the per-tile stats; block b>0 = row SSE of rows
// 4(b-1)..4(b-1)+3, one wave per row (lane-strided over tiles, then a fixed butterfly).
__global__ void __launch_bounds__(256) stats_finalize_kernel(const float* sp, int n_parts, const float* rsp,
                                                             int n_tiles, int M, float* out) {
  const int tid = threadIdx.x;
  if (blockIdx.x == 0) {
    __shared__ float red[3][256];
    float a = 0.f, b = 0.f, c = 0.f;
    for (int i = tid; i < n_parts; i += 256) {
      a += sp[(int64_t)i * 4 + 0];
      b += sp[(int64_t)i * 4 + 1];
      c += sp[(int64_t)i * 4 + 2];
    }
    red[0][tid] = a; red[1][tid] = b; red[2][tid] = c;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
      if (tid < s)
        for (int k = 0; k < 3; ++k) red[k][tid] += red[k][tid + s];
      __syncthreads();
    }
    if (tid == 0) { out[0] = red[0][0]; out[1] = red[1][0]; out[2] = red[2][0]; out[3] = 0.f; }
    return;
  }
  if (!rsp) return;
  const int m = (blockIdx.x - 1) * 4 + (tid >> 6);
  const int lane = tid & 63;
  if (m >= M) return;
  float r = 0.f;
  for (int t = lane; t < n_tiles; t += 64) r += rsp[(int64_t)t * M + m];
  for (int off = 32; off > 0; off >>= 1) r += __shfl_xor(r, off);
  if (lane == 0) out[4 + m] = r;
}

// sum of squares, two passes with a fixed order: 1,024 block partials (block b: elements b*256 + i,
// strided by the grid, a fixed LDS tree), then one block adds them in order and accumulates
// scale * sum into out[0] (the l2 penalty of Keras' W_regularizer, model.py:66,82)
constexpr int SUMSQ_BLOCKS = 1024;
__global__ void __launch_bounds__(256) sumsq_partials_kernel(const float* x, int64_t n, float* ws) {
  __shared__ float red[256];
  float a = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)SUMSQ_BLOCKS * 256) a += x[i] * x[i];
  red[threadIdx.x] = a;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) ws[blockIdx.x] = red[0];
}
__global__ void __launch_bounds__(256) sumsq_final_kernel(const float* ws, float scale, float* out) {
  __shared__ float red[256];
  float a = 0.f;
  for (int i = threadIdx.x; i < SUMSQ_BLOCKS; i += 256) a += ws[i];
  red[threadIdx.x] = a;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] += scale * red[0];
}

}  // namespace ocf

using namespace ocf;

extern "C" int ocf_sumsq(const float* x, int64_t n, float scale, float* ws, float* out, void* stream) {
  OCF_TRY_BEGIN
  OCF_CHECK(x && ws && out, "ocf_sumsq: null pointer");
  hipLaunchKernelGGL(sumsq_partials_kernel, dim3(SUMSQ_BLOCKS), dim3(256), 0, (hipStream_t)stream, x, n, ws);
  hipLaunchKernelGGL(sumsq_final_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, ws, scale, out);
  OCF_HIP(hipGetLastError());
  OCF_TRY_END
}

extern "C" int ocf_timing_event_create(void** ev) {
  OCF_TRY_BEGIN
  OCF_CHECK(ev != nullptr, "ocf_timing_event_create: null pointer");
  hipEvent_t e = nullptr;
  OCF_HIP(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
  *ev = e;
  OCF_TRY_END
}
extern "C" int ocf_event_record(void* ev, void* stream) {
  OCF_TRY_BEGIN
  OCF_CHECK(ev != nullptr, "ocf_event_record: null event");
  OCF_HIP(hipEventRecord((hipEvent_t)ev, (hipStream_t)stream));
  OCF_TRY_END
}
extern "C" int ocf_event_elapsed_ms(void* start, void* stop, float* ms) {
  OCF_TRY_BEGIN
  OCF_CHECK(start && stop && ms, "ocf_event_elapsed_ms: null pointer");
  OCF_HIP(hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)stop));
  OCF_TRY_END
}
// (no pending-error check: a destructor's call must not consume an asynchronous error it cannot report)
extern "C" int ocf_event_destroy(void* ev) {
  if (ev && hipEventDestroy((hipEvent_t)ev) != hipSuccess) {
    set_error("ocf_event_destroy: hipEventDestroy failed");
    return 1;
  }
  return 0;
}

extern "C" int ocf_version(void) { return 1; }
extern "C" const char* ocf_last_error(void) { return g_last_error.c_str(); }

extern "C" int ocf_splitk_bias_act(const float* slabs, int splits, int64_t split_stride, int M, int N, int64_t ld,
                                   const float* bias, int act, float keep, uint64_t seed, uint64_t stream,
                                   const uint8_t* mask_in, uint8_t* mask_out, float* a_out, void* h_out, int h_dtype,
                                   int m_real, int n_real, void* hstream) {
  OCF_TRY_BEGIN
  OCF_CHECK(slabs && bias, "ocf_splitk_bias_act: null pointer");
  BiasActParams p;
  p.bias = bias; p.act = act; p.keep = keep; p.seed = seed; p.stream = stream; p.mask_in = mask_in;
  p.mask_out = mask_out; p.a_out = a_out; p.h_out = h_out; p.h_dtype = h_dtype; p.ld = ld;
  p.m_real = m_real; p.n_real = n_real;
  hipLaunchKernelGGL(splitk_bias_act_kernel, dim3((N + 63) / 64, (M + 3) / 4), dim3(256), 0, (hipStream_t)hstream,
                     slabs, splits, split_stride, M, N, p);
  OCF_HIP(hipGetLastError());
  OCF_TRY_END
}

extern "C" int ocf_splitk_grad_act(const float* slabs, int splits, int64_t split_stride, int M, int N, int64_t ld,
                                   const float* a_in, const uint8_t* mask, float keep, int act, void* d_out,
                                   int d_dtype, float* db, float gscale, int m_real, int n_real, void* hstream) {
  OCF_TRY_BEGIN
  OCF_CHECK(slabs && a_in && d_out, "ocf_splitk_grad_act: null pointer");
  GradActParams p;
  p.a = a_in; p.mask = mask; p.keep = keep; p.act = act; p.d_out = d_out; p.d_dtype = d_dtype; p.ld = ld;
  p.db_part = nullptr; p.gscale = gscale; p.m_real = m_real; p.n_real = n_real;
  hipLaunchKernelGGL(splitk_grad_act_kernel, dim3((N + 63) / 64, (M + 3) / 4), dim3(256), 0, (hipStream_t)hstream,
                     slabs, splits, split_stride, M, N, p, db);
  OCF_HIP(hipGetLastError());
  OCF_TRY_END
}

extern "C" int ocf_opt_step(float* p, const float* g, float* s1, float* s2, int64_t n, const OcfOptParams* opt,
                            void* stream) {
  OCF_TRY_BEGIN
  OCF_CHECK(p && g && opt, "ocf_opt_step: null pointer");
  if (n == 0) return 0;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(opt_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, p, g, s1, s2, n, *opt);
  OCF_HIP(hipGetLastError());
  OCF_TRY_END
}

extern "C" int ocf_opt_step_ex(const OcfOptStepArgs* a, void* stream) {
  OCF_TRY_BEGIN
  OCF_CHECK(a && a->p && a->g, "ocf_opt_step_ex: null pointer");
  OCF_CHECK(a->g_dtype == OCF_F32 || a->g_dtype == OCF_BF16, "ocf_opt_step_ex: gradients fp32 or bf16");
  OCF_CHECK(!a->shadow || a->shadow_dtype == OCF_F16 || a->shadow_dtype == OCF_BF16,
            "ocf_opt_step_ex: shadow f16 or bf16");
  if (a->n == 0) return 0;
  int64_t blocks = (a->n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipStream_t s = (hipStream_t)stream;
  auto go = [&](auto gt, auto st) {
    using GT = decltype(gt);
    using ST = decltype(st);
    hipLaunchKernelGGL((opt_ex_kernel<GT, ST>), dim3((unsigned)blocks), dim3(256), 0, s, a->p,
                       reinterpret_cast<const GT*>(a->g), a->s1, a->s2, reinterpret_cast<ST*>(a->shadow), a->n, a->opt);
  };
  const bool gb = a->g_dtype == OCF_BF16;
  if (!a->shadow) gb ? go(__bf16{}, 0.f) : go(0.f, 0.f);
  else if (a->shadow_dtype == OCF_F16) gb ? go(__bf16{}, _Float16{}) : go(0.f, _Float16{});
  else gb ? go(__bf16{}, __bf16{}) : go(0.f, __bf16{});
  OCF_HIP(hipGetLastError());
  OCF_TRY_END
}

extern "C" int ocf_bias_opt_from_partials(float* b, const float* db_part, int parts, int64_t ld, int n, float* s1,
                                          float* s2, float* g_out, const OcfOptParams* opt, void* stream) {
  OCF_TRY_BEGIN
  OCF_CHECK(b && db_part && opt, "ocf_bias_opt_from_partials: null pointer");
  if (n == 0) return 0;
  hipLaunchKernelGGL(bias_opt_partials_kernel, dim3((n + 63) / 64), dim3(256), 0, (hipStream_t)stream, b, db_part,
                     parts, ld, n, s1, s2, g_out, *opt);
  OCF_HIP(hipGetLastError());
  OCF_TRY_END
}

extern "C" int ocf_stats_finalize(const float* stats_part, int n_parts, const float* row_sse_part, int n_tiles, int M,
                                  float* out, void* stream) {
  OCF_TRY_BEGIN
  OCF_CHECK(stats_part && out, "ocf_stats_finalize: null pointer");
  hipLaunchKernelGGL(stats_finalize_kernel, dim3(1 + (M + 3) / 4), dim3(256), 0, (hipStream_t)stream, stats_part,
                     n_parts, row_sse_part, n_tiles, M, out);
  OCF_HIP(hipGetLastError());
  OCF_TRY_END
}
