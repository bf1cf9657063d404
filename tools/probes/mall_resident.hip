// Diagnostic probe: does the row gather's table (138,496 x 1 KB f16 rows, the W shadow) stay Infinity-Cache
// resident across a 1.2 GB optimizer-like stream (read + write of other arrays), depending on the stream's
// cache policy?  Sequence per measurement: gather (warm) -> stream (policy P) -> timed gather.
// The stream mirrors the dW launch: float4 loads and stores of two 0.6 GB arrays (p, a) with the buffer
// cache-policy bits P (0 = default, 2 = nt as in the dW kernels, 3 = nt + sc0, 18 = nt + sc1), plus an optional regular
// store of 1 KB rows into the gathered table itself (the shadow update).  Modes 6/7: between the two gathers of
// table 1, a gather of a second 138 MB table (the step's encoder and decoder tables alternate), with regular or
// non-temporal loads.
//   hipcc --offload-arch=gfx950 -O3 -o tools/probes/mall_resident tools/probes/mall_resident.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int NROWS = 138496;
constexpr int H = 512;
constexpr size_t STREAM_FLOATS = (size_t)150 * 1024 * 1024;   // 600 MB per array

template <bool NT = false>
__global__ void __launch_bounds__(256) gather(const _Float16* __restrict__ W, const int* __restrict__ idx, int E,
                                              float* out) {
  typedef unsigned int u4 __attribute__((ext_vector_type(4)));
  constexpr int G = 32, U = 4, NG = 8;
  const int grp = threadIdx.x / G, l = threadIdx.x % G;
  const int j0 = blockIdx.x * 256, j1 = min(E, j0 + 256);
  float acc = 0.f;
  for (int j = j0 + grp; j < j1; j += NG * U) {
    uint4 w[U][2];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int ju = j + u * NG;
      const int n = ju < j1 ? idx[ju] : -1;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const _Float16* src = W + (size_t)n * H + (l + G * i) * 8;
        if (n < 0) {
          w[u][i] = make_uint4(0, 0, 0, 0);
        } else if constexpr (NT) {
          const u4 v = __builtin_nontemporal_load(reinterpret_cast<const u4*>(src));
          w[u][i] = make_uint4(v.x, v.y, v.z, v.w);
        } else {
          w[u][i] = *reinterpret_cast<const uint4*>(src);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int i = 0; i < 2; ++i) acc += __uint_as_float(w[u][i].x) + __uint_as_float(w[u][i].w);
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int POL>
__global__ void __launch_bounds__(256) stream(float* P, float* A, size_t n4) {
  __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(P, 0, 0x7fffffff, 0x00020000);
  __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(A, 0, 0x7fffffff, 0x00020000);
  typedef float v4 __attribute__((ext_vector_type(4)));
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
    const uint32_t o = (uint32_t)(i * 16);   // i < n4: inside the 600 MB arrays
    v4 p = __builtin_amdgcn_raw_buffer_load_b128(rp, o, 0, POL);
    v4 a = __builtin_amdgcn_raw_buffer_load_b128(ra, o, 0, POL);
    a = a + p * p;
    p = p - 0.001f * p;
    __builtin_amdgcn_raw_buffer_store_b128(p, rp, o, 0, POL);
    __builtin_amdgcn_raw_buffer_store_b128(a, ra, o, 0, POL);
  }
}

// the shadow update: regular stores of 1 KB rows of the gathered table (rows idx[0..n))
__global__ void __launch_bounds__(256) shadow_rows(_Float16* W, const int* idx, int n) {
  const int r = blockIdx.x * 4 + threadIdx.x / 64, l = threadIdx.x % 64;
  if (r >= n) return;
  uint4* row = reinterpret_cast<uint4*>(W + (size_t)idx[r] * H);
  row[l] = make_uint4(r, l, 1, 2);
}

int main() {
  const int E = 172000;
  std::vector<int> hidx(E), hrows(92000);
  srand(11);
  for (auto& x : hidx) x = (int)(((unsigned)rand() * 2654435761u) % NROWS);
  for (auto& x : hrows) x = (int)(((unsigned)rand() * 2246822519u) % NROWS);
  _Float16 *W, *W2;
  int *idx, *rows;
  float *out, *P, *A;
  hipMalloc(&W, (size_t)NROWS * H * 2);
  hipMemset(W, 0, (size_t)NROWS * H * 2);
  hipMalloc(&W2, (size_t)NROWS * H * 2);
  hipMemset(W2, 0, (size_t)NROWS * H * 2);
  hipMalloc(&idx, E * 4);
  hipMemcpy(idx, hidx.data(), E * 4, hipMemcpyHostToDevice);
  hipMalloc(&rows, hrows.size() * 4);
  hipMemcpy(rows, hrows.data(), hrows.size() * 4, hipMemcpyHostToDevice);
  hipMalloc(&out, (size_t)E * 4);
  hipMalloc(&P, STREAM_FLOATS * 4);
  hipMalloc(&A, STREAM_FLOATS * 4);
  hipMemset(P, 0, STREAM_FLOATS * 4);
  hipMemset(A, 0, STREAM_FLOATS * 4);
  const int nb = (E + 255) / 256;
  const size_t n4 = STREAM_FLOATS / 4;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const char* names[] = {"none", "stream_default", "stream_nt", "stream_nt_sc0", "stream_nt+shadow_rows",
                         "stream_nt_sc1", "second_table", "second_table_nt"};
  for (int mode = 0; mode < 8; ++mode) {
    double us = 0.0;
    const int R = 10;
    for (int r = 0; r < R; ++r) {
      hipLaunchKernelGGL(gather<false>, dim3(nb), dim3(256), 0, 0, W, idx, E, out);   // warm
      if (mode == 1) hipLaunchKernelGGL(stream<0>, dim3(4096), dim3(256), 0, 0, P, A, n4);
      if (mode == 2 || mode == 4) hipLaunchKernelGGL(stream<2>, dim3(4096), dim3(256), 0, 0, P, A, n4);
      if (mode == 3) hipLaunchKernelGGL(stream<3>, dim3(4096), dim3(256), 0, 0, P, A, n4);
      if (mode == 4) hipLaunchKernelGGL(shadow_rows, dim3((92000 + 3) / 4), dim3(256), 0, 0, W, rows, 92000);
      if (mode == 5) hipLaunchKernelGGL(stream<18>, dim3(4096), dim3(256), 0, 0, P, A, n4);
      if (mode == 6) hipLaunchKernelGGL(gather<false>, dim3(nb), dim3(256), 0, 0, W2, idx, E, out);
      if (mode == 7) hipLaunchKernelGGL(gather<true>, dim3(nb), dim3(256), 0, 0, W2, idx, E, out);
      hipEventRecord(a);
      hipLaunchKernelGGL(gather<false>, dim3(nb), dim3(256), 0, 0, W, idx, E, out);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0.f;
      hipEventElapsedTime(&ms, a, b);
      us += ms * 1e3 / R;
    }
    printf("{\"after\": \"%s\", \"gather_us\": %.1f}\n", names[mode], us);
  }
  hipDeviceSynchronize();
  return 0;
}
