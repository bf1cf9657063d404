// Diagnostic probe: the rate of the row gathers' access pattern alone -- random whole rows of an f16
// weight shadow at the ML-20M shape (138,496 rows x 512 f16 = 1 KB), one row per rating entry,
// summed into a per-workgroup accumulator (the encoder gather without its epilogue).
//   G lanes per entry, PPL 16-byte pieces per lane (G * PPL * 16 = 1 KB), U entries in flight per group,
//   ENT entries per workgroup; E entries in total (uniform random rows).
// Prints one JSON line per shape: microseconds per launch (HIP events, mean of 20) and the rate at
// E KB per launch.
//   hipcc --offload-arch=gfx950 -O3 -o tools/probes/gather_rate tools/probes/gather_rate.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int NROWS = 138496;
constexpr int H = 512;

template <int G, int PPL, int U, int TPB>
__global__ void __launch_bounds__(TPB) gather(const _Float16* __restrict__ W, const int* __restrict__ idx, int E,
                                              int ent, float* out) {
  constexpr int NG = TPB / G;
  const int grp = threadIdx.x / G, l = threadIdx.x % G;
  const int j0 = blockIdx.x * ent, j1 = min(E, j0 + ent);
  float acc[PPL * 8];
#pragma unroll
  for (int k = 0; k < PPL * 8; ++k) acc[k] = 0.f;
  for (int j = j0 + grp; j < j1; j += NG * U) {
    uint4 w[U][PPL];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int ju = j + u * NG;
      const int n = ju < j1 ? idx[ju] : -1;
#pragma unroll
      for (int i = 0; i < PPL; ++i)
        w[u][i] = n >= 0 ? *reinterpret_cast<const uint4*>(W + (size_t)n * H + (l + G * i) * 8) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int i = 0; i < PPL; ++i) {
        _Float16 h[8];
        __builtin_memcpy(h, &w[u][i], 16);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[i * 8 + k] += (float)h[k];
      }
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < PPL * 8; ++k) s += acc[k];
  out[blockIdx.x * TPB + threadIdx.x] = s;
}

static char* g_flush = nullptr;          // 1 GiB streamed before every timed launch ("cold": MALL evicted)
constexpr size_t FLUSH = (size_t)1 << 30;

template <int G, int PPL, int U, int TPB>
void run(const char* name, const _Float16* W, const int* idx, int E, int ent, float* out, bool cold) {
  const int nb = (E + ent - 1) / ent;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((gather<G, PPL, U, TPB>), dim3(nb), dim3(TPB), 0, 0, W, idx, E, ent, out);
  const int R = 20;
  double us = 0.0;
  for (int r = 0; r < R; ++r) {
    if (cold) hipMemsetAsync(g_flush, r & 255, FLUSH, 0);
    hipEventRecord(a);
    hipLaunchKernelGGL((gather<G, PPL, U, TPB>), dim3(nb), dim3(TPB), 0, 0, W, idx, E, ent, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0.f;
    hipEventElapsedTime(&ms, a, b);
    us += ms * 1e3 / R;
  }
  printf("{\"shape\": \"%s\", \"cold\": %d, \"G\": %d, \"ppl\": %d, \"u\": %d, \"tpb\": %d, \"ent\": %d, \"E\": %d, "
         "\"blocks\": %d, \"us\": %.1f, \"TBs\": %.3f}\n",
         name, (int)cold, G, PPL, U, TPB, ent, E, nb, us, E * 1024.0 / (us * 1e-6) / 1e12);
}

int main() {
  std::vector<int> hidx(1 << 22);
  srand(7);
  for (auto& x : hidx) x = (int)(((unsigned)rand() * 2654435761u) % NROWS);
  _Float16* W;
  int* idx;
  float* out;
  hipMalloc(&W, (size_t)NROWS * H * 2);
  hipMemset(W, 0, (size_t)NROWS * H * 2);
  hipMalloc(&idx, hidx.size() * 4);
  hipMemcpy(idx, hidx.data(), hidx.size() * 4, hipMemcpyHostToDevice);
  hipMalloc(&out, (size_t)(1 << 20) * 512 * 4);   // >= blocks x TPB for every shape below
  hipMalloc(&g_flush, FLUSH);
  for (int cold : {0, 1})
    for (int E : {172000, 1 << 20}) {
      run<32, 2, 4, 256>("ours", W, idx, E, 256, out, cold);
      run<32, 2, 4, 256>("ours", W, idx, E, 64, out, cold);
      run<16, 4, 4, 256>("g16", W, idx, E, 256, out, cold);
      run<32, 2, 2, 256>("ours", W, idx, E, 128, out, cold);
      run<32, 2, 1, 256>("ours", W, idx, E, 32, out, cold);
    }
  hipDeviceSynchronize();
  return 0;
}
