// Diagnostic probe: HBM read rate of the GEMM operand-staging pattern vs contiguous blocks.
// Each workgroup (256 threads) streams one 128-row x K-col f16 tile in K-steps of 64 columns,
// one step of loads in flight, loads -> LDS -> barrier (the gemm_kernel structure, no MFMA).
//   mode 0: row-major [N][K] tile: a step reads 128 B from each of 128 rows (rows K*2 B apart)
//   mode 1: blocked: a step's 128 x 64 tile is one contiguous 16 KB block
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void __launch_bounds__(256) stream_tiles(const uint4* __restrict__ w, int K, int mode, int ntiles,
                                                   float* sink) {
  __shared__ uint4 lds[2][1024];
  const int tid = threadIdx.x;
  const int nk = K / 64;
  float acc = 0.f;
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    for (int kt = 0; kt < nk; ++kt) {
      uint4 v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = tid + i * 256;          // chunk of 8 halves
        size_t idx;
        if (mode == 0) {
          const int r = c >> 3, kc = c & 7;   // 8 chunks per 128-B row segment
          idx = ((size_t)t * 128 + r) * (K / 8) + kt * 8 + kc;
        } else {
          idx = ((size_t)t * nk + kt) * 1024 + c;
        }
        v[i] = w[idx];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) lds[kt & 1][tid + i * 256] = v[i];
      __syncthreads();
      acc += __uint_as_float(lds[kt & 1][(tid * 7) & 1023].x);
    }
  }
  if (acc == 12345.f) sink[0] = acc;
}

int main() {
  const int N = 138496;
  for (int K : {512, 2048}) {
    size_t bytes = (size_t)N * K * 2;
    uint4* w;
    float* sink;
    hipMalloc(&w, bytes);
    hipMalloc(&sink, 4);
    hipMemset(w, 1, bytes);
    const int ntiles = N / 128;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int mode = 0; mode < 2; ++mode) {
      for (int grid : {512, 1024, ntiles}) {
        for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(stream_tiles, dim3(grid), dim3(256), 0, 0, w, K, mode, ntiles, sink);
        hipEventRecord(a);
        const int R = 10;
        for (int rep = 0; rep < R; ++rep)
          hipLaunchKernelGGL(stream_tiles, dim3(grid), dim3(256), 0, 0, w, K, mode, ntiles, sink);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        printf("K=%d mode=%d grid=%d  %.1f us  %.2f TB/s\n", K, mode, grid, ms * 1e3 / R, bytes / (ms / R * 1e-3) / 1e12);
      }
    }
    hipFree(w);
    hipFree(sink);
  }
  return 0;
}
