// Diagnostic probe: the HBM rate of the fused optimizer's parameter stream alone (no GEMM), at the
// ML-20M weight shape (138,496 x 512 fp32 parameters + one fp32 Adagrad slot + an f16 shadow,
// 18 B per live element), to find the access shape the role-split dW kernel's stream should use.
//   shape "tile": a workgroup streams one 128-row x 128-col piece of a weight panel (512-B row
//                 pieces 2 KB apart: the dW kernel's 128x128 tiles), its live rows compacted
//   shape "row":  a workgroup streams whole 2-KB rows of a contiguous run of live rows
// Live rows: every row (dense) or a random 67 % (the ML-20M batch's live-row fraction).
// Gradients come from a 16 KB table (L1/L2-resident), so only the optimizer bytes touch HBM.
//   hipcc --offload-arch=gfx950 -O3 -o tools/probes/opt_stream tools/probes/opt_stream.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int HP = 512;          // row width (floats)
constexpr int NP = 138496;       // rows
typedef float ocf_v4 __attribute__((ext_vector_type(4)));

template <int AUX>
__device__ __forceinline__ float4 ld16(const float* base, size_t idx) {
  if constexpr (AUX == 0) {
    return *reinterpret_cast<const float4*>(base + idx);
  } else {
    const ocf_v4 v = __builtin_nontemporal_load(reinterpret_cast<const ocf_v4*>(base + idx));
    return make_float4(v.x, v.y, v.z, v.w);
  }
}
template <int AUX>
__device__ __forceinline__ void st16(float* base, size_t idx, float4 v) {
  if constexpr (AUX == 0) {
    *reinterpret_cast<float4*>(base + idx) = v;
  } else {
    const ocf_v4 w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<ocf_v4*>(base + idx));
  }
}

__device__ __forceinline__ void adagrad(float g, float& p, float& a) {
  a = a + g * g;
  p = p - 0.005f * g / (__builtin_sqrtf(a) + 1e-8f);
}

// row shape: rows[] = live rows (sorted); RPB rows per block; thread t: float4 column t % 128, rows
// t / 128 + (TPB / 128) * u
template <int TPB, int U, int NT>
__global__ void __launch_bounds__(TPB) stream_rows(const int* __restrict__ rows, int nlive, float* P, float* A,
                                                  _Float16* S, const float4* __restrict__ gt) {
  constexpr int RPP = TPB / 128;       // rows per pass
  constexpr int RPB = RPP * U;
  const int c = threadIdx.x & 127, r0 = threadIdx.x >> 7;
  const int base = blockIdx.x * RPB;
  float4 p[U], a[U];
  int rr[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int li = base + r0 + RPP * u;
    rr[u] = li < nlive ? rows[li] : -1;
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (rr[u] >= 0) {
      const size_t o = (size_t)rr[u] * HP + c * 4;
      p[u] = ld16<NT>(P, o);
      a[u] = ld16<NT>(A, o);
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (rr[u] < 0) continue;
    const size_t o = (size_t)rr[u] * HP + c * 4;
    const float4 g = gt[(rr[u] * 7 + c) & 1023];
    adagrad(g.x, p[u].x, a[u].x);
    adagrad(g.y, p[u].y, a[u].y);
    adagrad(g.z, p[u].z, a[u].z);
    adagrad(g.w, p[u].w, a[u].w);
    st16<NT>(P, o, p[u]);
    st16<NT>(A, o, a[u]);
    typedef _Float16 h4 __attribute__((ext_vector_type(4)));
    h4 s = {(_Float16)p[u].x, (_Float16)p[u].y, (_Float16)p[u].z, (_Float16)p[u].w};
    *reinterpret_cast<h4*>(S + o) = s;
  }
}

// tile shape: block = (panel, piece); rec[panel] = live rows of the panel (count + 128 indices);
// thread t: float4 column (t % 32) of the 128-col piece, live slots t / 32 + (TPB / 32) * j
template <int TPB, int U, int NT>
__global__ void __launch_bounds__(TPB) stream_tiles(const int* __restrict__ rec, float* P, float* A, _Float16* S,
                                                   const float4* __restrict__ gt) {
  constexpr int SPP = TPB / 32;        // slots per pass
  const int panel = blockIdx.x >> 2, piece = blockIdx.x & 3;
  const int* rc = rec + panel * 129;
  const int L = rc[0];
  const int c = (threadIdx.x & 31) + piece * 32, k0 = threadIdx.x >> 5;
  for (int j0 = 0; j0 < L; j0 += SPP * U) {
    float4 p[U], a[U];
    int rr[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = j0 + k0 + SPP * u;
      rr[u] = k < L ? panel * 128 + rc[1 + k] : -1;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (rr[u] >= 0) {
        const size_t o = (size_t)rr[u] * HP + c * 4;
        p[u] = ld16<NT>(P, o);
        a[u] = ld16<NT>(A, o);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (rr[u] < 0) continue;
      const size_t o = (size_t)rr[u] * HP + c * 4;
      const float4 g = gt[(rr[u] * 7 + c) & 1023];
      adagrad(g.x, p[u].x, a[u].x);
      adagrad(g.y, p[u].y, a[u].y);
      adagrad(g.z, p[u].z, a[u].z);
      adagrad(g.w, p[u].w, a[u].w);
      st16<NT>(P, o, p[u]);
      st16<NT>(A, o, a[u]);
      typedef _Float16 h4 __attribute__((ext_vector_type(4)));
      h4 s = {(_Float16)p[u].x, (_Float16)p[u].y, (_Float16)p[u].z, (_Float16)p[u].w};
      *reinterpret_cast<h4*>(S + o) = s;
    }
  }
}

__global__ void copy4(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    b[i] = a[i];
}

struct Bufs {
  float *P, *A;
  _Float16* S;
  float4* gt;
  int *rows_dense, *rows_live, *rec_dense, *rec_live;
  int n_dense, n_live;
};

template <typename F>
static float time_us(F f, int reps = 10) {
  for (int i = 0; i < 2; ++i) f();
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  for (int i = 0; i < reps; ++i) f();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1e3f / reps;
}

template <int TPB, int U, int NT>
static void run_rows(const Bufs& B, bool live) {
  const int n = live ? B.n_live : B.n_dense;
  const int* rows = live ? B.rows_live : B.rows_dense;
  const int rpb = TPB / 128 * U;
  const int grid = (n + rpb - 1) / rpb;
  const float us = time_us([&] {
    hipLaunchKernelGGL((stream_rows<TPB, U, NT>), dim3(grid), dim3(TPB), 0, 0, rows, n, B.P, B.A, B.S, B.gt);
  });
  const double bytes = (double)n * HP * 18;
  printf("{\"shape\": \"row\", \"live\": %d, \"tpb\": %d, \"u\": %d, \"nt\": %d, \"us\": %.1f, \"TBs\": %.3f}\n", live,
         TPB, U, NT, us, bytes / us / 1e6);
}

template <int TPB, int U, int NT>
static void run_tiles(const Bufs& B, bool live) {
  const int* rec = live ? B.rec_live : B.rec_dense;
  const int n = live ? B.n_live : B.n_dense;
  const int grid = NP / 128 * 4;
  const float us = time_us([&] {
    hipLaunchKernelGGL((stream_tiles<TPB, U, NT>), dim3(grid), dim3(TPB), 0, 0, rec, B.P, B.A, B.S, B.gt);
  });
  const double bytes = (double)n * HP * 18;
  printf("{\"shape\": \"tile\", \"live\": %d, \"tpb\": %d, \"u\": %d, \"nt\": %d, \"us\": %.1f, \"TBs\": %.3f}\n",
         live, TPB, U, NT, us, bytes / us / 1e6);
}

int main() {
  Bufs B;
  const size_t n = (size_t)NP * HP;
  hipMalloc(&B.P, n * 4);
  hipMalloc(&B.A, n * 4);
  hipMalloc(&B.S, n * 2);
  hipMalloc(&B.gt, 1024 * 16);
  hipMemset(B.P, 0, n * 4);
  hipMemset(B.A, 0, n * 4);
  std::vector<float> g(4096);
  for (int i = 0; i < 4096; ++i) g[i] = 1e-3f * ((i * 37) % 101 - 50);
  hipMemcpy(B.gt, g.data(), 4096 * 4, hipMemcpyHostToDevice);
  std::vector<int> dense(NP), live;
  std::vector<int> rec_d((size_t)NP / 128 * 129), rec_l((size_t)NP / 128 * 129);
  srand(1);
  for (int r = 0; r < NP; ++r) {
    dense[r] = r;
    if (rand() % 1000 < 669) live.push_back(r);
  }
  for (int t = 0; t < NP / 128; ++t) {
    int* d = &rec_d[(size_t)t * 129];
    int* l = &rec_l[(size_t)t * 129];
    d[0] = 128;
    l[0] = 0;
    for (int k = 0; k < 128; ++k) d[1 + k] = k;
  }
  for (int r : live) {
    int* l = &rec_l[(size_t)(r / 128) * 129];
    l[1 + l[0]++] = r % 128;
  }
  B.n_dense = NP;
  B.n_live = (int)live.size();
  hipMalloc(&B.rows_dense, NP * 4);
  hipMalloc(&B.rows_live, live.size() * 4);
  hipMalloc(&B.rec_dense, rec_d.size() * 4);
  hipMalloc(&B.rec_live, rec_l.size() * 4);
  hipMemcpy(B.rows_dense, dense.data(), NP * 4, hipMemcpyHostToDevice);
  hipMemcpy(B.rows_live, live.data(), live.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(B.rec_dense, rec_d.data(), rec_d.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(B.rec_live, rec_l.data(), rec_l.size() * 4, hipMemcpyHostToDevice);

  {
    float4* C;
    hipMalloc(&C, n * 4);
    const float us = time_us([&] {
      hipLaunchKernelGGL(copy4, dim3(256 * 16), dim3(256), 0, 0, reinterpret_cast<const float4*>(B.P), C, n / 4);
    });
    printf("{\"shape\": \"copy\", \"us\": %.1f, \"TBs\": %.3f}\n", us, n * 8.0 / us / 1e6);
    hipFree(C);
  }
  for (int live = 0; live < 2; ++live) {
    run_rows<256, 2, 0>(B, live);
    run_rows<256, 4, 0>(B, live);
    run_rows<256, 8, 0>(B, live);
    run_rows<512, 4, 0>(B, live);
    run_rows<256, 4, 1>(B, live);
    run_rows<256, 8, 1>(B, live);
    run_tiles<256, 4, 0>(B, live);
    run_tiles<256, 2, 0>(B, live);
    run_tiles<512, 4, 0>(B, live);
    run_tiles<256, 4, 1>(B, live);
  }
  return 0;
}
