// Diagnostic probe: does the ORDER in which the row gathers walk a batch's entries change
// their HBM bytes at the Netflix width?  The encoder gather reads one 1-KB f16 W row per rating entry; at
// N = 480,189 users a 256-movie batch holds ~1.15 M entries over ~437 K distinct rows, so each row is read
// ~2.6 times, and the 492 MB table does not fit the 256 MiB Infinity Cache.  Same gather kernel as
// tools/probes/gather_rate.hip (32 lanes x 2 pieces per entry, 4 entries in flight per group, chunks of <= 256
// entries per workgroup), entries in different orders:
//   list      per batch row, the entries in rating-list order (random columns): the current encoder
//   rowsort   per batch row, sorted by column
//   range<R>  the columns cut into R ranges; chunk order (range, batch row): every batch row's entries of range r
//             (sorted) before any of range r + 1, so all rows walk the same W rows at about the same time
//   xcd<R>    as range<R>, but workgroup w runs on XCD w % 8 (round-robin dispatch): XCD x takes ranges x, x + 8,
//             ... in turn, so a range's repeated rows meet in one XCD's L2 instead of 8
// Timed "cold" (1 GiB streamed before every launch: the training step's dW streams pass GBs between gathers).
//   hipcc --offload-arch=gfx950 -O3 -o tools/probes/netflix_order tools/probes/netflix_order.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <string>
#include <vector>

constexpr int NROWS = 480189;
constexpr int H = 512;
constexpr int B = 256;
constexpr int PER_ROW = 4500;     // ratings per movie row (Netflix: 100.5 M / 17,770 = 5,654; ~80 % train)
constexpr int G = 32, PPL = 2, U = 4, TPB = 256, ENT = 256;

__global__ void __launch_bounds__(TPB) gather(const _Float16* __restrict__ W, const int* __restrict__ idx,
                                              const int* __restrict__ cb, const int* __restrict__ ce, float* out) {
  constexpr int NG = TPB / G;
  const int grp = threadIdx.x / G, l = threadIdx.x % G;
  const int j0 = cb[blockIdx.x], j1 = ce[blockIdx.x];
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

__global__ void flush_kernel(float4* p, size_t n, float4* sink) {
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const float4 v = p[i];
    a.x += v.x;
  }
  if (a.x == 12345.f) sink[0] = a;
}

struct Order {
  std::string name;
  std::vector<int> idx, cb, ce;
};

// chunks of <= ENT entries over consecutive runs [s, e) of idx
static void cut(Order& o, int s, int e) {
  for (int c = s; c < e; c += ENT) {
    o.cb.push_back(c);
    o.ce.push_back(std::min(e, c + ENT));
  }
}

int main(int argc, char** argv) {
  std::mt19937 rng(1);
  std::vector<std::vector<int>> rows(B);
  for (int b = 0; b < B; ++b) {
    std::vector<int>& r = rows[b];
    r.reserve(PER_ROW);
    while ((int)r.size() < PER_ROW) r.push_back((int)(rng() % NROWS));
    std::sort(r.begin(), r.end());
    r.erase(std::unique(r.begin(), r.end()), r.end());
  }
  std::vector<Order> orders;
  {
    Order o{"list"};
    for (int b = 0; b < B; ++b) {
      std::vector<int> r = rows[b];
      std::shuffle(r.begin(), r.end(), rng);
      const int s = (int)o.idx.size();
      o.idx.insert(o.idx.end(), r.begin(), r.end());
      cut(o, s, (int)o.idx.size());
    }
    orders.push_back(o);
  }
  {
    Order o{"rowsort"};
    for (int b = 0; b < B; ++b) {
      const int s = (int)o.idx.size();
      o.idx.insert(o.idx.end(), rows[b].begin(), rows[b].end());
      cut(o, s, (int)o.idx.size());
    }
    orders.push_back(o);
  }
  for (int R : {8, 16, 32, 64, 128}) {
    Order o{"range" + std::to_string(R)};
    for (int r = 0; r < R; ++r) {
      const int c0 = (int)((int64_t)NROWS * r / R), c1 = (int)((int64_t)NROWS * (r + 1) / R);
      for (int b = 0; b < B; ++b) {
        auto lo = std::lower_bound(rows[b].begin(), rows[b].end(), c0);
        auto hi = std::lower_bound(rows[b].begin(), rows[b].end(), c1);
        const int s = (int)o.idx.size();
        o.idx.insert(o.idx.end(), lo, hi);
        cut(o, s, (int)o.idx.size());
      }
    }
    orders.push_back(o);
  }
  for (int R : {64, 128, 256}) {
    // per XCD x: the chunks of ranges x, x+8, ... in (range, row) order; then interleave so chunk k of XCD x is
    // workgroup 8 k + x (padding with empty chunks where an XCD's list runs short)
    Order o{"xcd" + std::to_string(R)};
    std::vector<std::vector<std::pair<int, int>>> per(8);
    for (int r = 0; r < R; ++r) {
      const int c0 = (int)((int64_t)NROWS * r / R), c1 = (int)((int64_t)NROWS * (r + 1) / R);
      for (int b = 0; b < B; ++b) {
        auto lo = std::lower_bound(rows[b].begin(), rows[b].end(), c0);
        auto hi = std::lower_bound(rows[b].begin(), rows[b].end(), c1);
        const int s = (int)o.idx.size();
        o.idx.insert(o.idx.end(), lo, hi);
        for (int c = s; c < (int)o.idx.size(); c += ENT) per[r % 8].push_back({c, std::min((int)o.idx.size(), c + ENT)});
      }
    }
    size_t mx = 0;
    for (auto& p : per) mx = std::max(mx, p.size());
    for (size_t k = 0; k < mx; ++k)
      for (int x = 0; x < 8; ++x) {
        if (k < per[x].size()) {
          o.cb.push_back(per[x][k].first);
          o.ce.push_back(per[x][k].second);
        } else {
          o.cb.push_back(0);
          o.ce.push_back(0);
        }
      }
    orders.push_back(o);
  }
  size_t E = orders[0].idx.size();
  std::printf("{\"entries\": %zu, \"rows\": %d, \"table_MB\": %.1f}\n", E, NROWS, NROWS * (double)H * 2 / 1e6);
  _Float16* W;
  hipMalloc(&W, (size_t)NROWS * H * 2);
  hipMemset(W, 0, (size_t)NROWS * H * 2);
  const size_t FL = (size_t)1 << 30;
  float4 *fl, *sink;
  hipMalloc(&fl, FL);
  hipMemset(fl, 0, FL);
  hipMalloc(&sink, 64);
  int *idx, *cb, *ce;
  float* out;
  hipMalloc(&idx, E * 4 * 2);
  hipMalloc(&cb, 4 << 20);
  hipMalloc(&ce, 4 << 20);
  hipMalloc(&out, (size_t)(4 << 20) * TPB * 4 / 16);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (auto& o : orders) {
    hipMemcpy(idx, o.idx.data(), o.idx.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(cb, o.cb.data(), o.cb.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(ce, o.ce.data(), o.ce.size() * 4, hipMemcpyHostToDevice);
    const int nb = (int)o.cb.size();
    float tot = 0.f;
    const int reps = 10;
    for (int it = 0; it < reps + 2; ++it) {
      flush_kernel<<<4096, 256>>>(fl, FL / 16, sink);
      hipEventRecord(a);
      gather<<<nb, TPB>>>(W, idx, cb, ce, out);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0.f;
      hipEventElapsedTime(&ms, a, b);
      if (it >= 2) tot += ms;
    }
    const double us = tot / reps * 1e3;
    std::printf("{\"order\": \"%s\", \"chunks\": %d, \"us\": %.1f, \"GBps_at_entry_bytes\": %.0f}\n", o.name.c_str(), nb,
                us, o.idx.size() * 1024.0 / (us * 1e-6) / 1e9);
  }
  return 0;
}
