// Split-K reductions fused with the layer epilogues, elementwise optimizers, stats reduction,
// and the library's error state.
#include <string>

#include "ocf_epilogues.h"
#include "ocf_internal.h"

namespace ocf {

static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }

// grid: N/64 column blocks; 256 threads = 64 columns x 4 row groups
__global__ void __launch_bounds__(256) splitk_bias_act_kernel(const float* slabs, int splits, int64_t sstride, int M,
                                                              int N, BiasActParams p) {
  const int col = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rg = threadIdx.x >> 6;
  if (col >= N) return;
  for (int m = rg; m < M; m += 4) {
    const float* s = slabs + (int64_t)m * p.ld + col;
    float v = 0.f;
    for (int k = 0; k < splits; ++k) v += s[(int64_t)k * sstride];
    bias_act_store(p, m, col, v);
  }
}

__global__ void __launch_bounds__(256) splitk_grad_act_kernel(const float* slabs, int splits, int64_t sstride, int M,
                                                              int N, GradActParams p, float* db) {
  __shared__ float part[4][64];
  const int cl = threadIdx.x & 63;
  const int col = blockIdx.x * 64 + cl;
  const int rg = threadIdx.x >> 6;
  float cs = 0.f;
  if (col < N) {
    for (int m = rg; m < M; m += 4) {
      const float* s = slabs + (int64_t)m * p.ld + col;
      float v = 0.f;
      for (int k = 0; k < splits; ++k) v += s[(int64_t)k * sstride];
      float d = grad_act_value(p, m, col, v);
      store_ct(p.d_out, p.d_dtype, (int64_t)m * p.ld + col, d);
      cs += d;
    }
  }
  part[rg][cl] = cs;
  __syncthreads();
  if (rg == 0 && col < N && db) db[col] = ((part[0][cl] + part[1][cl]) + (part[2][cl] + part[3][cl])) * p.gscale;
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

__global__ void bias_opt_partials_kernel(float* bvec, const float* db_part, int parts, int64_t ld, int n, float* s1,
                                         float* s2, float* g_out, OcfOptParams o) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float g = 0.f;
  for (int k = 0; k < parts; ++k) g += db_part[(int64_t)k * ld + i];
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

// one block: out[0..2] = fixed-order sums of the per-tile stats; out[4+m] = row SSE
__global__ void __launch_bounds__(256) stats_finalize_kernel(const float* sp, int n_parts, const float* rsp,
                                                             int n_tiles, int M, float* out) {
  __shared__ float red[3][256];
  const int tid = threadIdx.x;
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
  if (rsp)
    for (int m = tid; m < M; m += 256) {
      float r = 0.f;
      for (int t = 0; t < n_tiles; ++t) r += rsp[(int64_t)t * M + m];
      out[4 + m] = r;
    }
}

}  // namespace ocf

using namespace ocf;

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
  hipLaunchKernelGGL(splitk_bias_act_kernel, dim3((N + 63) / 64), dim3(256), 0, (hipStream_t)hstream, slabs, splits,
                     split_stride, M, N, p);
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
  hipLaunchKernelGGL(splitk_grad_act_kernel, dim3((N + 63) / 64), dim3(256), 0, (hipStream_t)hstream, slabs, splits,
                     split_stride, M, N, p, db);
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

extern "C" int ocf_bias_opt_from_partials(float* b, const float* db_part, int parts, int64_t ld, int n, float* s1,
                                          float* s2, float* g_out, const OcfOptParams* opt, void* stream) {
  OCF_TRY_BEGIN
  OCF_CHECK(b && db_part && opt, "ocf_bias_opt_from_partials: null pointer");
  if (n == 0) return 0;
  hipLaunchKernelGGL(bias_opt_partials_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, b, db_part,
                     parts, ld, n, s1, s2, g_out, *opt);
  OCF_HIP(hipGetLastError());
  OCF_TRY_END
}

extern "C" int ocf_stats_finalize(const float* stats_part, int n_parts, const float* row_sse_part, int n_tiles, int M,
                                  float* out, void* stream) {
  OCF_TRY_BEGIN
  OCF_CHECK(stats_part && out, "ocf_stats_finalize: null pointer");
  hipLaunchKernelGGL(stats_finalize_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, stats_part, n_parts,
                     row_sse_part, n_tiles, M, out);
  OCF_HIP(hipGetLastError());
  OCF_TRY_END
}
