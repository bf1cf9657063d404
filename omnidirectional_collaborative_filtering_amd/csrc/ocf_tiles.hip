// The encoder as an MFMA contraction over column tiles (model.py:64-71, the first Dense layer's X W1 on a
// sparse batch): for regimes where a weight row carries many batch entries (Netflix width: ~2.6 entries per live
// column at B = 256; a feature-parallel rank's B x G = 2,048 global rows: ~19), the row gathers read each W1 row
// once PER ENTRY, so their bytes grow with the entries; here each 128-column tile of W1 is read once per
// workgroup row group and multiplied on the matrix cores by the batch's X tile, densified in LDS from the
// batch rows' column-sorted entries.
//
//   part[b][s][h] = sum over the columns n of split s (128-column tiles [t0_s, t1_s)) of X[b][n] W1[n][h]
//
// followed by the existing fixed-order row reduction (ocf_rows_reduce with row_cptr[b] = b S: BIAS_ACT on one
// GPU, RAW before a feature-parallel all-reduce).  X[b][n] = the live input value of batch row b's entry in
// column n (ocf_epoch_scatter's xval, 0 for an entry that is not an input), rounded to the compute dtype as
// every MFMA operand of the dense path is.
//
// Workgroup (256 threads, 4 waves) = (row group of 256 batch rows, hidden slice of 128, split s).  Per tile t:
//   * the W1 tile [128 columns][128 hidden] (32 KB, 16-bit shadow, row-major) is staged through LDS in its
//     natural row layout with the 256-B-row XOR swizzle and read as the MFMA B operand by the transposing
//     ds_read_b64_tr_b16 (8 consecutive columns of one hidden unit per lane);
//   * the X tile [256 rows][128 columns] lives in LDS (64 KB, row-swizzled for the ds_read_b128 A reads): thread
//     b owns row b and writes its <= 8 entries of the tile (the row's column-sorted view, 128-column tile
//     pointers), then clears exactly those positions after the tile's MFMAs;
//   * wave w computes rows [64 w, 64 w + 64) x the 128 hidden units: 2 x 4 tiles of v_mfma_f32_32x32x16, fp32
//     accumulators in registers across all tiles of the split.
// The next tile's W1 loads, its entries' values and the entry indices of the tile after it are issued before the
// current tile's MFMAs (a three-stage pipeline of the dependent chain tile pointer -> column / list index ->
// value), so one workgroup per CU keeps its HBM reads in flight.  Rows with more than ET_EMAX entries in a tile
// take a slow path for the rest (rare: ~1.2 entries per row per tile at Netflix width).
#include <hip/hip_runtime.h>

#include "ocf_epilogues.h"
#include "ocf_internal.h"

namespace ocf {
namespace et {

constexpr int BM = 256;      // batch rows per workgroup
constexpr int BH = 128;      // hidden units per workgroup
constexpr int BK = 128;      // columns per tile (the view's tile pointers)
constexpr int EMAX = 8;      // entries per row per tile held in registers
constexpr int ROWB = 256;    // bytes per LDS row of either image (128 x 16-bit)

typedef short s4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef __bf16 b8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

// X image: row b, 16-byte chunk ch (8 columns) at ROWB b + 16 (ch ^ (b & 15)) -- the A-operand row reads of 32
// consecutive rows then spread over all 64 banks
__device__ __forceinline__ int xoff(int b, int ch) { return ROWB * b + 16 * (ch ^ (b & 15)); }
// W image: column n (a row of the tile), 16-byte chunk ch (8 hidden units) at ROWB n + 16 (ch ^ sw(n)), the
// microarch guide's swizzle for 256-byte rows read both ways (cdna_hip_programming.md T10 (b))
__device__ __forceinline__ int woff(int n, int ch) {
  return ROWB * n + 16 * (ch ^ (((n & 3) << 2) | ((n >> 2) & 3)));
}

template <typename CT> struct Frag;
template <> struct Frag<_Float16> {
  using T = h8;
  __device__ static f16v mfma(T a, T b, f16v c) { return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0); }
};
template <> struct Frag<__bf16> {
  using T = b8;
  __device__ static f16v mfma(T a, T b, f16v c) { return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0); }
};

struct Rows {          // a thread's batch row
  int64_t rp0, lb;     // start of the dataset row in the view, the batch-local entry offset
  const int32_t* tp;   // the row's tile pointers (nullptr: no entries)
};

template <typename CT>
__global__ void __launch_bounds__(256) enc_tiles_kernel(OcfEncTileArgs a, int n_rg, int n_q, int tiles_per) {
  __shared__ __attribute__((aligned(16))) char lds[BM * ROWB + BK * ROWB];
  char* const xs = lds;
  char* const ws = lds + BM * ROWB;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // workgroups -> (row group, hidden slice, split): the row groups of one (slice, split) -- readers of the same
  // W1 tiles -- on one XCD (blockIdx round-robins over the 8 XCDs), so the second and later reads hit its L2
  const int bx = blockIdx.x, xcd = bx & 7, j = bx >> 3;
  const int rg = j % n_rg, q = (j / n_rg) * 8 + xcd;
  if (q >= n_q) return;
  const int S = a.splits, s = q % S, hs = q / S;
  const int t0 = s * tiles_per, t1 = min(a.n_tiles, t0 + tiles_per);
  if (t0 >= t1) {                                     // an empty split: zero partials
    for (int i = tid; i < BM * BH; i += 256) {
      const int b = rg * BM + i / BH;
      if (b < a.Bp) a.part[((int64_t)b * S + s) * a.H + hs * BH + (i % BH)] = 0.f;
    }
    return;
  }
  const int h0 = hs * BH;
  using F = Frag<CT>;
  using FT = typename F::T;
  // ---- this thread's batch row
  Rows me{0, 0, nullptr};
  {
    const int b = rg * BM + tid;
    if (b < a.B) {
      const int r = a.rows[b];
      if (r >= 0) {
        me.rp0 = a.rp[r];
        me.lb = a.lboff[b];
        me.tp = a.tptr + (int64_t)r * (a.n_tiles + 1);
      }
    }
  }
  // ---- W1 tile staging: 16 rows x 16 chunks per pass, 8 passes
  const int wrow = tid >> 4, wch = tid & 15;
  const char* Wb = reinterpret_cast<const char*>(a.W);
  auto wload = [&](int t, uint4 (&v)[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int64_t n = (int64_t)t * BK + wrow + 16 * i;
      v[i] = *reinterpret_cast<const uint4*>(Wb + (n * a.ldw + h0) * 2 + 16 * wch);
    }
  };
  auto wstore = [&](const uint4 (&v)[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) *reinterpret_cast<uint4*>(ws + woff(wrow + 16 * i, wch)) = v[i];
  };
  // ---- the entry chain: tile pointers (4 tiles ahead) -> columns / list indices (2 ahead) -> values (1 ahead)
  auto tpl = [&](int t) { return (me.tp && t <= t1) ? me.tp[t] : 0; };
  int tpA = tpl(t0), tpB = tpl(t0 + 1), tpC = tpl(t0 + 2), tpD = tpl(t0 + 3);   // tp[t], tp[t+1], ...
  int cl0[EMAX], li0[EMAX], n0;      // tile t+1's columns / list indices (for the values)
  int cl1[EMAX], li1[EMAX], n1;      // tile t+2's
  float xv[EMAX];                    // tile t+1's values
  int cw[EMAX], nw = 0;              // the positions this thread wrote for the current tile (to clear)
  bool over_w = false;
  auto idx = [&](int lo, int hi, int (&cl)[EMAX], int (&li)[EMAX]) {
    const int n = hi - lo;
#pragma unroll
    for (int e = 0; e < EMAX; ++e) {
      const bool ok = e < n;
      cl[e] = ok ? a.tcol[me.rp0 + lo + e] : 0;
      li[e] = ok ? a.tlidx[me.rp0 + lo + e] : 0;
    }
    return n;
  };
  auto vals = [&](int n, const int (&li)[EMAX]) {
#pragma unroll
    for (int e = 0; e < EMAX; ++e) xv[e] = e < n ? a.xval[me.lb + li[e]] : 0.f;
  };
  // write the tile's entries into row tid of the X image (t: the tile, lo: its first entry in the view)
  auto xwrite = [&](int t, int n, int lo, const int (&cl)[EMAX]) {
    nw = n < EMAX ? n : EMAX;
    over_w = n > EMAX;
    // (added, not stored: a duplicate rating's entries meet in one column, and the gathers sum over entries)
    auto put = [&](int kk, float x) {
      CT* p = reinterpret_cast<CT*>(xs + xoff(tid, kk >> 3) + 2 * (kk & 7));
      *p = CvtT<CT>::to(CvtT<CT>::from(*p) + x);
    };
#pragma unroll
    for (int e = 0; e < EMAX; ++e)
      if (e < n) {
        const int kk = cl[e] - t * BK;
        cw[e] = kk;
        put(kk, xv[e]);
      }
    for (int e = EMAX; e < n; ++e)                    // (rare) the rest of a long row
      put(a.tcol[me.rp0 + lo + e] - t * BK, a.xval[me.lb + a.tlidx[me.rp0 + lo + e]]);
  };
  auto xclear = [&]() {
    if (over_w) {
#pragma unroll
      for (int ch = 0; ch < 16; ++ch) *reinterpret_cast<uint4*>(xs + xoff(tid, ch)) = make_uint4(0, 0, 0, 0);
    } else {
#pragma unroll
      for (int e = 0; e < EMAX; ++e)
        if (e < nw) *reinterpret_cast<CT*>(xs + xoff(tid, cw[e] >> 3) + 2 * (cw[e] & 7)) = CvtT<CT>::to(0.f);
    }
  };
  // ---- prologue: clear the X image, stage tile t0
  for (int i = tid; i < BM * ROWB / 16; i += 256) reinterpret_cast<uint4*>(xs)[i] = make_uint4(0, 0, 0, 0);
  {
    uint4 v[8];
    wload(t0, v);
    n0 = idx(tpA, tpB, cl0, li0);
    vals(n0, li0);
    __syncthreads();
    wstore(v);
    xwrite(t0, n0, tpA, cl0);
  }
  // tile t0 + 1's indices and values, t0 + 2's indices
  n0 = idx(tpB, tpC, cl0, li0);
  n1 = idx(tpC, tpD, cl1, li1);
  vals(n0, li0);
  int tpE = tpl(t0 + 4);
  __syncthreads();
  // ---- MFMA state
  f16v acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int k = 0; k < 16; ++k) acc[i][c][k] = 0.f;
  const int r = lane & 31, hf = lane >> 5, g = lane >> 4, gi = lane & 15, gq = gi >> 2, gp = gi & 3;
  for (int t = t0; t < t1; ++t) {
    const bool more = t + 1 < t1;
    uint4 wn[8];
    if (more) wload(t + 1, wn);
    // (the entry chain of the tiles ahead is already in flight: values of t + 1, indices of t + 2)
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      FT fa[2], fb[4];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = 64 * wave + 32 * i + r;
        __builtin_memcpy(&fa[i], xs + xoff(row, 2 * ks + hf), 16);
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        s4 lo, hi;
        const int ch = 4 * c + 2 * (g & 1) + (gp >> 1);
        const int n0r = 16 * ks + 8 * (g >> 1) + gq;
        lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s4*)(ws + woff(n0r, ch) + 8 * (gp & 1)));
        hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s4*)(ws + woff(n0r + 4, ch) + 8 * (gp & 1)));
        short e[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        __builtin_memcpy(&fb[c], e, 16);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[i][c] = F::mfma(fa[i], fb[c], acc[i][c]);
    }
    if (!more) break;
    // next stage of the entry chain (issued before the barrier: its loads overlap the other waves' MFMAs)
    int cl2[EMAX], li2[EMAX];
    const int n2 = idx(tpD, tpE, cl2, li2);           // tile t + 3's indices
    const int tpF = tpl(t + 5);
    __syncthreads();                                  // every wave is done with tile t's images
    xclear();
    wstore(wn);
    xwrite(t + 1, n0, tpB, cl0);
    // rotate: t + 2 -> t + 1 (values now), t + 3 -> t + 2
    tpA = tpB; tpB = tpC; tpC = tpD; tpD = tpE; tpE = tpF;
    n0 = n1;
#pragma unroll
    for (int e = 0; e < EMAX; ++e) { cl0[e] = cl1[e]; li0[e] = li1[e]; cl1[e] = cl2[e]; li1[e] = li2[e]; }
    n1 = n2;
    vals(n0, li0);
    __syncthreads();
  }
  // ---- partials: C layout of v_mfma_f32_32x32x16 (register k: row (k & 3) + 8 (k >> 2) + 4 hf, column lane & 31)
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int b = rg * BM + 64 * wave + 32 * i + (k & 3) + 8 * (k >> 2) + 4 * hf;
      if (b < a.Bp) {
        float* dst = a.part + ((int64_t)b * S + s) * a.H + h0 + r;
#pragma unroll
        for (int c = 0; c < 4; ++c) dst[32 * c] = acc[i][c][k];
      }
    }
}

}  // namespace et
}  // namespace ocf

using namespace ocf;

extern "C" int ocf_encoder_tiles(const OcfEncTileArgs* args, void* stream) {
  OCF_TRY_BEGIN
  OCF_CHECK(args != nullptr, "ocf_encoder_tiles: null arguments");
  const OcfEncTileArgs& a = *args;
  OCF_CHECK(a.rows && a.rp && a.tptr && a.tcol && a.tlidx && a.lboff && a.xval && a.W && a.part,
            "ocf_encoder_tiles: null pointer");
  OCF_CHECK(a.w_dtype == OCF_F16 || a.w_dtype == OCF_BF16, "ocf_encoder_tiles: 16-bit weights only");
  OCF_CHECK(a.H > 0 && a.H % et::BH == 0, "ocf_encoder_tiles: H must be a multiple of 128");
  OCF_CHECK(a.ldw >= a.H && a.ldw % 8 == 0, "ocf_encoder_tiles: ldw");
  OCF_CHECK(a.B >= 0 && a.B <= a.Bp && a.Bp % 128 == 0, "ocf_encoder_tiles: B <= Bp, Bp a multiple of 128");
  OCF_CHECK(a.n_tiles >= 1 && a.splits >= 1, "ocf_encoder_tiles: n_tiles, splits >= 1");
  if (a.Bp == 0) return 0;
  const int n_rg = (a.Bp + et::BM - 1) / et::BM, n_hs = a.H / et::BH;
  const int tiles_per = (a.n_tiles + a.splits - 1) / a.splits;
  const int n_q = n_hs * a.splits;
  const int grid = n_rg * ((n_q + 7) / 8) * 8;
  hipStream_t s = (hipStream_t)stream;
  if (a.w_dtype == OCF_F16)
    hipLaunchKernelGGL(et::enc_tiles_kernel<_Float16>, dim3(grid), dim3(256), 0, s, a, n_rg, n_q, tiles_per);
  else
    hipLaunchKernelGGL(et::enc_tiles_kernel<__bf16>, dim3(grid), dim3(256), 0, s, a, n_rg, n_q, tiles_per);
  OCF_HIP(hipGetLastError());
  OCF_TRY_END
}
