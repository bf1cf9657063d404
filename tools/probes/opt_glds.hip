// Diagnostic probe: does staging the optimizer stream's parameter / slot loads through LDS-DMA
// (global_load_lds_dwordx4: no VGPR destination while in flight) raise its rate over the register-staged
// stream the row-stream dW kernel uses?  ML-20M weight shape (138,496 rows x 512 fp32 + one fp32 Adagrad slot
// + the 16-bit shadow, 18 B per live element), 66.9 % of the rows live, one wave per row as in ocf_rows_dw.h,
// the next row's loads issued before the current row's update.
//   REG   p / a of the next row into registers (the kernel's form; opt_layout.hip's SEP)
//   GLDS  p / a of the next row into the wave's LDS slot (2 slots per wave, 8 KB), read back at the update
// Gradients come from a 16 KB table (L1/L2-resident), so only the optimizer bytes touch HBM.
//   hipcc --offload-arch=gfx950 -O3 -o tools/probes/opt_glds tools/probes/opt_glds.hip
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

__device__ __forceinline__ void update_row(int r, int lane, v4* p, v4* a, float* P, float* A, _Float16* S,
                                           const v4* __restrict__ gt) {
  for (int j = 0; j < 2; ++j) {
    const v4 g = gt[(r * 7 + lane + 64 * j) & 1023];
    for (int e = 0; e < 4; ++e) {
      float pe = p[j][e], ae = a[j][e];
      adagrad(g[e], pe, ae);
      p[j][e] = pe;
      a[j][e] = ae;
    }
    stn(P + (size_t)r * HP + (lane + 64 * j) * 4, p[j]);
    stn(A + (size_t)r * HP + (lane + 64 * j) * 4, a[j]);
    h4 s = {(_Float16)p[j].x, (_Float16)p[j].y, (_Float16)p[j].z, (_Float16)p[j].w};
    *reinterpret_cast<h4*>(S + (size_t)r * HP + (lane + 64 * j) * 4) = s;
  }
}

__global__ void __launch_bounds__(256) stream_reg(const int* __restrict__ rows, int nlive, float* P, float* A,
                                                  _Float16* S, const v4* __restrict__ gt) {
  const int lane = threadIdx.x & 63;
  const int wave = blockIdx.x * 4 + (threadIdx.x >> 6), waves = gridDim.x * 4;
  int i = wave;
  if (i >= nlive) return;
  int r = rows[i];
  v4 p[2], a[2];
  for (int j = 0; j < 2; ++j) {
    p[j] = ldn(P + (size_t)r * HP + (lane + 64 * j) * 4);
    a[j] = ldn(A + (size_t)r * HP + (lane + 64 * j) * 4);
  }
  while (true) {
    const int in = i + waves;
    const int rn = in < nlive ? rows[in] : -1;
    v4 pn[2], an[2];
    if (rn >= 0)
      for (int j = 0; j < 2; ++j) {
        pn[j] = ldn(P + (size_t)rn * HP + (lane + 64 * j) * 4);
        an[j] = ldn(A + (size_t)rn * HP + (lane + 64 * j) * 4);
      }
    update_row(r, lane, p, a, P, A, S, gt);
    if (rn < 0) break;
    i = in;
    r = rn;
    for (int j = 0; j < 2; ++j) {
      p[j] = pn[j];
      a[j] = an[j];
    }
  }
}

// the wave's slot s: p (2 KB) then a (2 KB); one global_load_lds_dwordx4 moves 1 KB (64 lanes x 16 B)
template <int AUX>
__device__ __forceinline__ void glds_row(const float* P, const float* A, int r, float* slot, int lane) {
  for (int j = 0; j < 2; ++j) {
    __builtin_amdgcn_global_load_lds(P + (size_t)r * HP + (lane + 64 * j) * 4, slot + j * 256, 16, 0, AUX);
    __builtin_amdgcn_global_load_lds(A + (size_t)r * HP + (lane + 64 * j) * 4, slot + 512 + j * 256, 16, 0, AUX);
  }
}

template <int AUX>
__global__ void __launch_bounds__(256) stream_glds(const int* __restrict__ rows, int nlive, float* P, float* A,
                                                   _Float16* S, const v4* __restrict__ gt) {
  __shared__ __attribute__((aligned(16))) float lds[4][2][1024];    // [wave][slot][p 512 | a 512]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wave = blockIdx.x * 4 + w, waves = gridDim.x * 4;
  int i = wave;
  if (i >= nlive) return;
  int r = rows[i], cur = 0;
  glds_row<AUX>(P, A, r, lds[w][0], lane);
  while (true) {
    const int in = i + waves;
    const int rn = in < nlive ? rows[in] : -1;
    // the current row's four LDS-DMA loads (and the previous row's stores) have landed
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    v4 p[2], a[2];
    for (int j = 0; j < 2; ++j) {
      p[j] = *reinterpret_cast<const v4*>(&lds[w][cur][j * 256 + lane * 4]);
      a[j] = *reinterpret_cast<const v4*>(&lds[w][cur][512 + j * 256 + lane * 4]);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (rn >= 0) glds_row<AUX>(P, A, rn, lds[w][cur ^ 1], lane);   // the next row in flight during the update
    update_row(r, lane, p, a, P, A, S, gt);
    if (rn < 0) break;
    i = in;
    r = rn;
    cur ^= 1;
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
  hipMalloc(&P, n * 4);
  hipMalloc(&A, n * 4);
  hipMalloc(&S, n * 2);
  hipMalloc(&gt, 1024 * 16);
  hipMemset(P, 0, n * 4);
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
  for (int rd = 0; rd < rounds; ++rd)
    for (int grid : {1024, 2048, 4096}) {
      auto report = [&](const char* name, float us) {
        printf("{\"form\": \"%s\", \"grid\": %d, \"round\": %d, \"us\": %.1f, \"TBs\": %.3f}\n", name, grid, rd, us,
               bytes / us / 1e6);
      };
      report("REG", time_us([&] { hipLaunchKernelGGL(stream_reg, dim3(grid), dim3(256), 0, 0, rows, nl, P, A, S, gt); }));
      report("GLDS", time_us([&] { hipLaunchKernelGGL(stream_glds<0>, dim3(grid), dim3(256), 0, 0, rows, nl, P, A, S, gt); }));
      report("GLDS_NT", time_us([&] { hipLaunchKernelGGL(stream_glds<2>, dim3(grid), dim3(256), 0, 0, rows, nl, P, A, S, gt); }));
    }
  hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    printf("{\"error\": \"%s\"}\n", hipGetErrorString(e));
    return 1;
  }
  return 0;
}
