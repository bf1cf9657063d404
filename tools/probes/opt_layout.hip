// Diagnostic probe: does the optimizer stream of the row-stream dW kernel get faster when a weight row's
// parameters and Adagrad slot are ONE contiguous record instead of two arrays?  ML-20M weight shape
// (138,496 rows x 512 fp32 + one fp32 slot + the 16-bit shadow, 18 B per live element), 66.9 % of the rows
// live (the ML-20M batch's live-row fraction), whole rows, one wave per row as in ocf_rows_dw.h.
//   SEP  p[Np][512], a[Np][512], s[Np][512] (the library's layout today)
//   IL2  [p | a] per row (4 KB), s separate
//   IL3  [p | a | s] per row (5 KB)
// Loads / stores with the nt policy on the fp32 streams (as the kernel); the shadow store plain or nt.
// Gradients come from a 16 KB table (L1/L2-resident), so only the optimizer bytes touch HBM.
//   hipcc --offload-arch=gfx950 -O3 -o tools/probes/opt_layout tools/probes/opt_layout.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int HP = 512;          // row width (floats)
constexpr int NP = 138496;       // rows
typedef float v4 __attribute__((ext_vector_type(4)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ v4 ldn(const float* p) { return __builtin_nontemporal_load(reinterpret_cast<const v4*>(p)); }
__device__ __forceinline__ void stn(float* p, v4 v) { __builtin_nontemporal_store(v, reinterpret_cast<v4*>(p)); }

__device__ __forceinline__ void adagrad(float g, float& p, float& a) {
  a = a + g * g;
  p = p - 0.005f * g / (__builtin_sqrtf(a) + 1e-8f);
}

// LAYOUT 0 SEP, 1 IL2, 2 IL3.  A wave walks rows wave_id, wave_id + waves, ... of the live list with the next
// row's loads issued before the current row's update (two rows in flight per wave, as the kernel's stage D / E).
template <int LAYOUT, int SNT>
__global__ void __launch_bounds__(256) stream(const int* __restrict__ rows, int nlive, float* P, float* A,
                                              _Float16* S, const v4* __restrict__ gt) {
  const int lane = threadIdx.x & 63;
  const int wave = blockIdx.x * 4 + (threadIdx.x >> 6), waves = gridDim.x * 4;
  // row record stride in floats and the offsets of a / s inside it
  constexpr size_t REC = LAYOUT == 0 ? HP : LAYOUT == 1 ? 2 * HP : 2 * HP + HP / 2;
  auto pp = [&](int r) { return LAYOUT == 0 ? P + (size_t)r * HP : P + (size_t)r * REC; };
  auto ap = [&](int r) { return LAYOUT == 0 ? A + (size_t)r * HP : P + (size_t)r * REC + HP; };
  auto sp = [&](int r) {
    return LAYOUT == 2 ? reinterpret_cast<_Float16*>(P + (size_t)r * REC + 2 * HP) : S + (size_t)r * HP;
  };
  int i = wave;
  if (i >= nlive) return;
  int r = rows[i];
  v4 p[2], a[2];
  for (int j = 0; j < 2; ++j) {
    p[j] = ldn(pp(r) + (lane + 64 * j) * 4);
    a[j] = ldn(ap(r) + (lane + 64 * j) * 4);
  }
  while (true) {
    const int in = i + waves;
    const int rn = in < nlive ? rows[in] : -1;
    v4 pn[2], an[2];
    if (rn >= 0)
      for (int j = 0; j < 2; ++j) {
        pn[j] = ldn(pp(rn) + (lane + 64 * j) * 4);
        an[j] = ldn(ap(rn) + (lane + 64 * j) * 4);
      }
    for (int j = 0; j < 2; ++j) {
      const v4 g = gt[(r * 7 + lane + 64 * j) & 1023];
      for (int e = 0; e < 4; ++e) {
        float pe = p[j][e], ae = a[j][e];
        adagrad(g[e], pe, ae);
        p[j][e] = pe;
        a[j][e] = ae;
      }
      stn(pp(r) + (lane + 64 * j) * 4, p[j]);
      stn(ap(r) + (lane + 64 * j) * 4, a[j]);
      h4 s = {(_Float16)p[j].x, (_Float16)p[j].y, (_Float16)p[j].z, (_Float16)p[j].w};
      h4* d = reinterpret_cast<h4*>(sp(r) + (lane + 64 * j) * 4);
      if constexpr (SNT) __builtin_nontemporal_store(s, d);
      else *d = s;
    }
    if (rn < 0) break;
    i = in;
    r = rn;
    for (int j = 0; j < 2; ++j) {
      p[j] = pn[j];
      a[j] = an[j];
    }
  }
}

template <typename F>
static float time_us(F f, int reps = 20) {
  for (int i = 0; i < 3; ++i) f();
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

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 3;
  const size_t n = (size_t)NP * HP;
  float *P, *A;
  _Float16* S;
  v4* gt;
  hipMalloc(&P, n * 4 * 3);       // big enough for every layout
  hipMalloc(&A, n * 4);
  hipMalloc(&S, n * 2);
  hipMalloc(&gt, 1024 * 16);
  hipMemset(P, 0, n * 12);
  hipMemset(A, 0, n * 4);
  std::vector<float> g(4096);
  for (int i = 0; i < 4096; ++i) g[i] = 1e-3f * ((i * 37) % 101 - 50);
  hipMemcpy(gt, g.data(), 4096 * 4, hipMemcpyHostToDevice);
  std::vector<int> live;
  srand(1);
  for (int r = 0; r < NP; ++r)
    if (rand() % 1000 < 669) live.push_back(r);
  int* rows;
  hipMalloc(&rows, live.size() * 4);
  hipMemcpy(rows, live.data(), live.size() * 4, hipMemcpyHostToDevice);
  const int nl = (int)live.size();
  const double bytes = (double)nl * HP * 18;
  const char* names[3] = {"SEP", "IL2", "IL3"};
  for (int rd = 0; rd < rounds; ++rd)
    for (int grid : {1024, 2048, 4096}) {
      auto run = [&](auto lay, auto snt) {
        constexpr int L = decltype(lay)::value, SN = decltype(snt)::value;
        const float us = time_us([&] {
          hipLaunchKernelGGL((stream<L, SN>), dim3(grid), dim3(256), 0, 0, rows, nl, P, A, S, gt);
        });
        printf("{\"layout\": \"%s\", \"shadow_nt\": %d, \"grid\": %d, \"round\": %d, \"us\": %.1f, \"TBs\": %.3f}\n",
               names[L], SN, grid, rd, us, bytes / us / 1e6);
      };
      using std::integral_constant;
      run(integral_constant<int, 0>{}, integral_constant<int, 0>{});
      run(integral_constant<int, 1>{}, integral_constant<int, 0>{});
      run(integral_constant<int, 2>{}, integral_constant<int, 0>{});
      run(integral_constant<int, 0>{}, integral_constant<int, 1>{});
      run(integral_constant<int, 1>{}, integral_constant<int, 1>{});
      run(integral_constant<int, 2>{}, integral_constant<int, 1>{});
    }
  return 0;
}
