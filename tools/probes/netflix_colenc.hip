// Diagnostic probe ("read each live W row once, in column order"): the Netflix-width encoder
// product h_pre[b] = sum_n x[b][n] W[n] computed column by column, every live W row read once, against the row-
// gather order the library's encoder uses (one W row per rating entry; ~2.6 reads per live row per batch).
//   gather    per batch row, its entries in chunks of <= 256 (32 lanes x 2 pieces per entry, 4 entries in flight per
//             group), one fp32 partial per chunk, then the chunk partials of each row summed: the library's encoder
//   col<HS>   grid (R column ranges) x (512 / HS hidden slices): a thread per live column of the range reads the
//             column's HS-wide W slice once (HS / 8 16-byte loads) and adds x * w into an LDS [256][HS + 1] fp32
//             accumulator for each batch row of the column's list (LDS float atomics, rows padded by one word so
//             the lanes' rows land in different banks); the workgroup writes its [256][HS] partial, then the R range
//             partials of every (b, h) are summed in range order (a second launch)
// Synthetic data: 256 batch rows x 4,500 distinct random columns of 480,189 (Netflix I-AutoRec batch: ~1.15 M
// entries over ~437 K distinct columns), H = 512 f16.  Timed cold (1 GiB streamed before every launch, as in the
// training step, where the dW streams pass GBs between gathers); checked against an fp64 host product.
//   hipcc --offload-arch=gfx950 -O3 -o tools/probes/netflix_colenc tools/probes/netflix_colenc.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

constexpr int NROWS = 480189;
constexpr int H = 512;
constexpr int B = 256;
constexpr int PER_ROW = 4500;

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

// ---- the library's order: per batch row, chunks of <= 256 entries, a partial per chunk
constexpr int G = 32, PPL = 2, U = 4, TPB = 256;
__global__ void __launch_bounds__(TPB) gather_chunks(const _Float16* __restrict__ W, const int* __restrict__ col,
                                                     const float* __restrict__ val, const int* __restrict__ cb,
                                                     const int* __restrict__ ce, float* __restrict__ part) {
  constexpr int NG = TPB / G;
  __shared__ float red[NG][H];
  const int grp = threadIdx.x / G, l = threadIdx.x % G;
  const int j0 = cb[blockIdx.x], j1 = ce[blockIdx.x];
  float acc[PPL * 8];
#pragma unroll
  for (int k = 0; k < PPL * 8; ++k) acc[k] = 0.f;
  for (int j = j0 + grp; j < j1; j += NG * U) {
    uint4 w[U][PPL];
    float x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int ju = j + u * NG;
      const int n = ju < j1 ? col[ju] : -1;
      x[u] = ju < j1 ? val[ju] : 0.f;
#pragma unroll
      for (int i = 0; i < PPL; ++i)
        w[u][i] = n >= 0 ? *reinterpret_cast<const uint4*>(W + (size_t)n * H + (l + G * i) * 8) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int i = 0; i < PPL; ++i) {
        _Float16 hv[8];
        __builtin_memcpy(hv, &w[u][i], 16);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[i * 8 + k] += x[u] * (float)hv[k];
      }
  }
#pragma unroll
  for (int i = 0; i < PPL; ++i)
#pragma unroll
    for (int k = 0; k < 8; ++k) red[grp][(l + G * i) * 8 + k] = acc[i * 8 + k];
  __syncthreads();
  for (int hh = threadIdx.x; hh < H; hh += TPB) {
    float s = 0.f;
#pragma unroll
    for (int g = 0; g < NG; ++g) s += red[g][hh];
    part[(size_t)blockIdx.x * H + hh] = s;
  }
}
// per batch row: its chunk partials summed in chunk order
__global__ void __launch_bounds__(256) sum_chunks(const float* __restrict__ part, const int* __restrict__ rc,
                                                  float* __restrict__ out) {
  const int b = blockIdx.x;
  for (int hh = threadIdx.x; hh < H; hh += 256) {
    float s = 0.f;
    for (int c = rc[b]; c < rc[b + 1]; ++c) s += part[(size_t)c * H + hh];
    out[(size_t)b * H + hh] = s;
  }
}

// ---- column order: a thread per live column, the column's HS-wide W slice once, LDS accumulator per batch row
template <int HS>
__global__ void __launch_bounds__(256) col_enc(const _Float16* __restrict__ W, const int* __restrict__ live,
                                               const int* __restrict__ rb, const int* __restrict__ cptr,
                                               const int* __restrict__ eb, const float* __restrict__ ev,
                                               float* __restrict__ part) {
  constexpr int LD = HS + 1;
  extern __shared__ float acc[];   // [B][LD]
  const int r = blockIdx.x, s = blockIdx.y, h0 = s * HS;
  for (int i = threadIdx.x; i < B * LD; i += 256) acc[i] = 0.f;
  __syncthreads();
  const int k0 = rb[r], k1 = rb[r + 1];
  for (int k = k0 + threadIdx.x; k < k1; k += 256) {
    const int n = live[k];
    const int e0 = cptr[k], e1 = cptr[k + 1];
    uint4 w[HS / 8];
#pragma unroll
    for (int i = 0; i < HS / 8; ++i) w[i] = *reinterpret_cast<const uint4*>(W + (size_t)n * H + h0 + 8 * i);
    float wf[HS];
#pragma unroll
    for (int i = 0; i < HS / 8; ++i) {
      _Float16 hv[8];
      __builtin_memcpy(hv, &w[i], 16);
#pragma unroll
      for (int q = 0; q < 8; ++q) wf[8 * i + q] = (float)hv[q];
    }
    for (int e = e0; e < e1; ++e) {
      const int b = eb[e];
      const float x = ev[e];
      float* a = acc + b * LD;
#pragma unroll
      for (int q = 0; q < HS; ++q) atomicAdd(a + q, x * wf[q]);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < B * HS; i += 256) {
    const int b = i / HS, q = i % HS;
    part[((size_t)r * B + b) * H + h0 + q] = acc[b * LD + q];
  }
}
__global__ void __launch_bounds__(256) sum_ranges(const float* __restrict__ part, int R, float* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (size_t)B * H) return;
  float s = 0.f;
  for (int r = 0; r < R; ++r) s += part[(size_t)r * B * H + i];
  out[i] = s;
}

__global__ void flush_kernel(const float4* p, size_t n, float4* sink) {
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) a.x += p[i].x;
  if (a.x == 12345.f) sink[0] = a;
}

int main() {
  std::mt19937 rng(1);
  std::uniform_real_distribution<float> uw(-0.05f, 0.05f);
  std::vector<std::vector<int>> rows(B);
  for (int b = 0; b < B; ++b) {
    std::vector<int>& r = rows[b];
    while ((int)r.size() < PER_ROW) r.push_back((int)(rng() % NROWS));
    std::sort(r.begin(), r.end());
    r.erase(std::unique(r.begin(), r.end()), r.end());
  }
  // row-major batch: entries in random order within a row (the rating lists), values 1..5
  std::vector<int> col, cb, ce, rc(B + 1, 0);
  std::vector<float> val;
  for (int b = 0; b < B; ++b) {
    std::vector<int> r = rows[b];
    std::shuffle(r.begin(), r.end(), rng);
    const int s = (int)col.size();
    for (int n : r) {
      col.push_back(n);
      val.push_back((float)(1 + rng() % 5));
    }
    for (int c = s; c < (int)col.size(); c += 256) {
      cb.push_back(c);
      ce.push_back(std::min((int)col.size(), c + 256));
    }
    rc[b + 1] = (int)cb.size();
  }
  const int E = (int)col.size(), NCH = (int)cb.size();
  // column lists (CSC over live columns, batch rows ascending)
  std::vector<int> cnt(NROWS, 0);
  for (int n : col) ++cnt[n];
  std::vector<int> live, cptr(1, 0), slot(NROWS, -1);
  for (int n = 0; n < NROWS; ++n)
    if (cnt[n]) {
      slot[n] = (int)live.size();
      live.push_back(n);
      cptr.push_back(cptr.back() + cnt[n]);
    }
  const int L = (int)live.size();
  std::vector<int> eb(E), cur(cptr.begin(), cptr.end() - 1);
  std::vector<float> ev(E);
  for (int b = 0, j = 0; b < B; ++b)
    for (int k = 0; k < (int)rows[b].size(); ++k, ++j) {
      const int sl = slot[col[j]];
      eb[cur[sl]] = b;
      ev[cur[sl]] = val[j];
      ++cur[sl];
    }
  std::vector<_Float16> Wh((size_t)NROWS * H);
  for (auto& w : Wh) w = (_Float16)uw(rng);
  std::printf("{\"entries\": %d, \"live_columns\": %d, \"chunks\": %d, \"unique_W_MB\": %.1f, \"entry_W_MB\": %.1f}\n", E, L,
              NCH, L * (double)H * 2 / 1e6, E * (double)H * 2 / 1e6);
  // fp64 reference for 8 batch rows
  const int chk_rows[8] = {0, 1, 37, 100, 128, 200, 254, 255};
  std::vector<double> ref(8 * H, 0.0);
  {
    std::vector<int> off(B + 1, 0);
    for (int b = 0; b < B; ++b) off[b + 1] = off[b] + (int)rows[b].size();
    for (int t = 0; t < 8; ++t) {
      const int b = chk_rows[t];
      for (int j = off[b]; j < off[b + 1]; ++j)
        for (int hh = 0; hh < H; ++hh) ref[t * H + hh] += (double)val[j] * (double)(float)Wh[(size_t)col[j] * H + hh];
    }
  }
  _Float16* W;
  CK(hipMalloc(&W, Wh.size() * 2));
  CK(hipMemcpy(W, Wh.data(), Wh.size() * 2, hipMemcpyHostToDevice));
  auto up = [](const void* p, size_t bytes) {
    void* d;
    CK(hipMalloc(&d, std::max<size_t>(bytes, 4)));
    CK(hipMemcpy(d, p, bytes, hipMemcpyHostToDevice));
    return d;
  };
  int* d_col = (int*)up(col.data(), E * 4);
  float* d_val = (float*)up(val.data(), E * 4);
  int* d_cb = (int*)up(cb.data(), NCH * 4);
  int* d_ce = (int*)up(ce.data(), NCH * 4);
  int* d_rc = (int*)up(rc.data(), (B + 1) * 4);
  int* d_live = (int*)up(live.data(), L * 4);
  int* d_cptr = (int*)up(cptr.data(), (L + 1) * 4);
  int* d_eb = (int*)up(eb.data(), E * 4);
  float* d_ev = (float*)up(ev.data(), E * 4);
  float *part, *out;
  const int RMAX = 256;
  CK(hipMalloc(&part, std::max<size_t>((size_t)NCH, (size_t)RMAX * B) * H * 4));
  CK(hipMalloc(&out, (size_t)B * H * 4));
  const size_t FL = (size_t)1 << 30;
  float4 *fl, *sink;
  CK(hipMalloc(&fl, FL));
  CK(hipMemset(fl, 0, FL));
  CK(hipMalloc(&sink, 64));
  hipEvent_t a, m, z;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&m));
  CK(hipEventCreate(&z));
  auto check = [&](const char* name) {
    std::vector<float> o((size_t)B * H);
    CK(hipMemcpy(o.data(), out, o.size() * 4, hipMemcpyDeviceToHost));
    double worst = 0.0;
    for (int t = 0; t < 8; ++t)
      for (int hh = 0; hh < H; ++hh) {
        const double d = std::fabs(o[(size_t)chk_rows[t] * H + hh] - ref[t * H + hh]);
        worst = std::max(worst, d / (1.0 + std::fabs(ref[t * H + hh])));
      }
    return worst;
  };
  auto run = [&](const char* name, int R, auto launch1, auto launch2) {
    float t1 = 0.f, t2 = 0.f;
    const int reps = 10;
    for (int it = 0; it < reps + 2; ++it) {
      flush_kernel<<<4096, 256>>>(fl, FL / 16, sink);
      CK(hipEventRecord(a));
      launch1();
      CK(hipEventRecord(m));
      launch2();
      CK(hipEventRecord(z));
      CK(hipEventSynchronize(z));
      float x = 0.f, y = 0.f;
      CK(hipEventElapsedTime(&x, a, m));
      CK(hipEventElapsedTime(&y, m, z));
      if (it >= 2) {
        t1 += x;
        t2 += y;
      }
    }
    CK(hipGetLastError());
    std::printf("{\"order\": \"%s\", \"ranges\": %d, \"main_us\": %.1f, \"reduce_us\": %.1f, \"total_us\": %.1f, "
                "\"max_rel_err\": %.2e}\n",
                name, R, t1 / reps * 1e3, t2 / reps * 1e3, (t1 + t2) / reps * 1e3, check(name));
    std::fflush(stdout);
  };
  run("gather", 0, [&] { gather_chunks<<<NCH, TPB>>>(W, d_col, d_val, d_cb, d_ce, part); },
      [&] { sum_chunks<<<B, 256>>>(part, d_rc, out); });
  auto colrun = [&](auto kern, int HS, int R, const char* name) {
    std::vector<int> rb(R + 1);
    for (int r = 0; r <= R; ++r) rb[r] = (int)((int64_t)L * r / R);
    int* d_rb = (int*)up(rb.data(), (R + 1) * 4);
    const size_t lds = (size_t)B * (HS + 1) * 4;
    CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    run(name, R, [&] { kern<<<dim3(R, H / HS), 256, lds>>>(W, d_live, d_rb, d_cptr, d_eb, d_ev, part); },
        [&] { sum_ranges<<<B * H / 256, 256>>>(part, R, out); });
    CK(hipFree(d_rb));
  };
  for (int R : {32, 64, 128, 256}) colrun(col_enc<32>, 32, R, "col32");
  for (int R : {32, 64, 128}) colrun(col_enc<64>, 64, R, "col64");
  for (int R : {16, 32, 64}) colrun(col_enc<128>, 128, R, "col128");
  return 0;
}
