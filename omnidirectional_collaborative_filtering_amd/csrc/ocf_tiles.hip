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
//   * the W1 tile [128 columns][128 hidden] (32 KB, 16-bit shadow, row-major) goes to LDS by direct-to-LDS loads
//     (global_load_lds_dwordx4: no registers, double-buffered, the next tile's in flight during this tile's
//     MFMAs) in its natural row layout with the 256-B-row XOR swizzle, and is read as the MFMA B operand by the
//     transposing ds_read_b64_tr_b16 (8 consecutive columns of one hidden unit per lane);
//   * the X tile [256 rows][128 columns] lives in LDS (64 KB, row-swizzled for the ds_read_b128 A reads): thread
//     b owns row b and writes its <= 8 entries of the tile (the row's column-sorted view, 128-column tile
//     pointers), then clears exactly those positions after the tile's MFMAs;
//   * wave w computes rows [64 w, 64 w + 64) x the 128 hidden units: 2 x 4 tiles of v_mfma_f32_32x32x16, fp32
//     accumulators in registers across all tiles of the split.
// The entries go through a branch-free pipeline (clamped addresses, masked results) of the dependent chain tile
// pointer (4 tiles ahead) -> column / list index (2 ahead) -> value (1 ahead), every stage's loads issued before
// the current tile's MFMAs, so one workgroup per CU keeps its reads in flight.  Rows with more than ET_EMAX entries in a tile
// take a slow path for the rest (rare: ~1.2 entries per row per tile at Netflix width).
#include <hip/hip_runtime.h>

#include <algorithm>

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

template <typename CT>
__global__ void __launch_bounds__(256) enc_tiles_kernel(OcfEncTileArgs a, int n_rg, int n_hs, int tiles_per) {
  // three separate LDS objects: the compiler then knows a direct-to-LDS load into one W buffer does not alias the
  // reads of the other or of the X image, and does not wait for it (vmcnt) before them
  __shared__ __attribute__((aligned(16))) char xs[BM * ROWB];
  __shared__ __attribute__((aligned(16))) char wsA[BK * ROWB];
  __shared__ __attribute__((aligned(16))) char wsB[BK * ROWB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // workgroups -> (split, row group, hidden slice): every workgroup of one split on one XCD (blockIdx round-robins
  // over the 8 XCDs) -- the row groups read the same W1 tiles, the hidden slices the same entries -- so only the
  // first read of each goes to HBM, the others hit the XCD's L2
  const int per = n_rg * n_hs;                        // workgroups per split
  const int bx = blockIdx.x, xcd = bx & 7, slot = bx >> 3;
  const int S = a.splits, s = (slot / per) * 8 + xcd, rem = slot % per, rg = rem / n_hs, hs = rem % n_hs;
  if (s >= S) return;
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
  // ---- this thread's batch row (rows without entries read row 0's pointers, masked: every load is branch-free)
  int64_t rp0 = 0, lb = 0;
  bool live = false;
  const int32_t* tp = a.tptr;
  {
    const int b = rg * BM + tid;
    const int rr = b < a.B ? a.rows[b] : -1;
    live = rr >= 0;
    if (live) {
      rp0 = a.rp[rr];
      lb = a.lboff[b];
      tp = a.tptr + (int64_t)rr * (a.n_tiles + 1);
    }
  }
  // ---- W1 tiles: direct-to-LDS loads (global_load_lds_dwordx4, no registers), two buffers.  Instruction i of wave
  // w fills 1 KB = rows n0 .. n0 + 3 (n0 = 4 (4 i + w)) of the image; lane L lands at slot L % 16 of row n0 + L / 16,
  // so it loads the global chunk that the swizzle puts there
  const char* Wb = reinterpret_cast<const char*>(a.W);
  auto wload = [&](int t, char* dst) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int n0 = 4 * (4 * i + wave), n = n0 + (lane >> 4), c = (lane & 15) ^ (((n & 3) << 2) | ((n >> 2) & 3));
      const char* src = Wb + (((int64_t)t * BK + n) * a.ldw + h0) * 2 + 16 * c;
      __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(dst + n0 * ROWB), 16, 0, 0);
    }
  };
  // ---- the entry chain, branch-free (clamped addresses, masked results): tile pointers 4 tiles ahead, the packed
  // (column in tile | list index << 7) of the entries 2 ahead, their values 1 ahead
  const int64_t last = a.nnz - 1, elast = a.n_entries - 1;
  auto tpl = [&](int t) { return live ? tp[min(t, t1)] : 0; };
  // (the loads' results are not touched here -- the caller packs them a stage later -- so nothing waits for them)
  auto idx = [&](int lo, int (&col)[EMAX], int (&li)[EMAX]) {
#pragma unroll
    for (int e = 0; e < EMAX; ++e) {
      const int64_t v = min(rp0 + lo + e, last);
      col[e] = a.tcol[v];
      li[e] = a.tlidx[v];
    }
  };
  auto pack = [&](int t, int n, const int (&col)[EMAX], const int (&li)[EMAX], int (&pk)[EMAX]) {
#pragma unroll
    for (int e = 0; e < EMAX; ++e) pk[e] = e < n ? ((col[e] - t * BK) & 127) | (li[e] << 7) : -1;
  };
  // (raw loads, masked where they are used: xwrite skips pk < 0 -- a select here would wait for the loads)
  auto vals = [&](const int (&pk)[EMAX], float (&xv)[EMAX]) {
#pragma unroll
    for (int e = 0; e < EMAX; ++e) xv[e] = a.xval[min(lb + (pk[e] >= 0 ? (pk[e] >> 7) : 0), elast)];
  };
  // (added, not stored: a duplicate rating's entries meet in one column, and the gathers sum over entries)
  auto put = [&](int kk, float x) {
    CT* p = reinterpret_cast<CT*>(xs + xoff(tid, kk >> 3) + 2 * (kk & 7));
    *p = CvtT<CT>::to(CvtT<CT>::from(*p) + x);
  };
  int cw[EMAX];                      // the positions written for the current tile (cleared after its MFMAs)
  bool over = false;
  auto xwrite = [&](int t, int n, int lo, const int (&pk)[EMAX], const float (&xv)[EMAX]) {
#pragma unroll
    for (int e = 0; e < EMAX; ++e) {
      cw[e] = pk[e];
      if (pk[e] >= 0) put(pk[e] & 127, xv[e]);
    }
    over = n > EMAX;
    for (int e = EMAX; e < n; ++e)                    // (rare) the rest of a long row
      put(a.tcol[rp0 + lo + e] - t * BK, a.xval[lb + a.tlidx[rp0 + lo + e]]);
  };
  auto xclear = [&]() {
    if (over) {
#pragma unroll
      for (int ch = 0; ch < 16; ++ch) *reinterpret_cast<uint4*>(xs + xoff(tid, ch)) = make_uint4(0, 0, 0, 0);
    } else {
#pragma unroll
      for (int e = 0; e < EMAX; ++e)
        if (cw[e] >= 0)
          *reinterpret_cast<CT*>(xs + xoff(tid, (cw[e] & 127) >> 3) + 2 * (cw[e] & 7)) = CvtT<CT>::to(0.f);
    }
  };
  // ---- prologue: clear the X image; tile t0 staged, t0 + 1's entries and values, t0 + 2's entries in flight
  for (int i = tid; i < BM * ROWB / 16; i += 256) reinterpret_cast<uint4*>(xs)[i] = make_uint4(0, 0, 0, 0);
  wload(t0, wsA);
  int tq[5];                                          // tp[t + 1 .. t + 5] while processing tile t
  const int tp0 = tpl(t0);
#pragma unroll
  for (int i = 0; i < 5; ++i) tq[i] = tpl(t0 + 1 + i);
  int P1[EMAX], P2[EMAX], C2[EMAX], L2[EMAX];
  float X1[EMAX];
  int n1 = tq[1] - tq[0], n2 = tq[2] - tq[1];
  {
    int P0[EMAX], C0[EMAX], L0[EMAX];
    float X0[EMAX];
    const int n0 = tq[0] - tp0;
    idx(tp0, C0, L0);
    pack(t0, n0, C0, L0, P0);
    vals(P0, X0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    xwrite(t0, n0, tp0, P0, X0);
    idx(tq[0], C0, L0);
    pack(t0 + 1, n1, C0, L0, P1);
  }
  idx(tq[1], C2, L2);
  pack(t0 + 2, n2, C2, L2, P2);
  vals(P1, X1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
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
  // one tile: t's MFMAs from wcur while t + 1's W1 tile streams into wnext; false after the split's last tile
  auto step = [&](int t, const char* wcur, char* wnext) -> bool {
    const bool more = t + 1 < t1;
    if (more) wload(t + 1, wnext);
    // tile t + 3's entries (tile pointers t + 3, t + 4; packed after this tile's MFMAs) and tile t + 6's pointer
    int C3[EMAX], L3[EMAX];
    const int n3 = tq[3] - tq[2];
    idx(tq[2], C3, L3);
    const int tnew = tpl(t + 6);
    const char* wsb = wcur;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      FT fa[2], fb[4];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = 64 * wave + 32 * i + r;
        fa[i] = *reinterpret_cast<const FT*>(xs + xoff(row, 2 * ks + hf));
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int ch = 4 * c + 2 * (g & 1) + (gp >> 1);
        const int nr = 16 * ks + 8 * (g >> 1) + gq;
        const s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s4*)(wsb + woff(nr, ch) + 8 * (gp & 1)));
        const s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s4*)(wsb + woff(nr + 4, ch) + 8 * (gp & 1)));
        const short e[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        __builtin_memcpy(&fb[c], e, 16);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[i][c] = F::mfma(fa[i], fb[c], acc[i][c]);
    }
    if (!more) return false;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tile t + 1's W1 image, t + 3's entries, t + 2's values
    __syncthreads();                                  // every wave is done with tile t's images
    xclear();
    xwrite(t + 1, n1, tq[0], P1, X1);
    __syncthreads();                                  // tile t + 1's X image complete
    // rotate: t + 2 -> t + 1, t + 3 -> t + 2; then t + 2's values (after the barrier: a barrier's release would
    // wait for them; in flight during the next tile's MFMAs instead)
    n1 = n2;
    n2 = n3;
#pragma unroll
    for (int e = 0; e < EMAX; ++e) P1[e] = P2[e];
    pack(t + 3, n3, C3, L3, P2);
#pragma unroll
    for (int i = 0; i < 4; ++i) tq[i] = tq[i + 1];
    tq[4] = tnew;
    vals(P1, X1);
    return true;
  };
  for (int t = t0; t < t1; t += 2) {                  // (two tiles per trip: each W1 buffer a static LDS object)
    if (!step(t, wsA, wsB) || !step(t + 1, wsB, wsA)) break;
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


// ---- the packed form.  The thread-per-row chain above reads, per tile and workgroup, one or two 64-B lines of the
// view (columns, list indices) and of xval per batch row: ~48 KB of scattered lines against the tile's 32 KB of W1,
// and once per hidden slice.  A pre-pass (three launches per batch) packs the batch's entries into buckets per (row
// group, tile) instead -- one 32-bit word per entry: row in group (8 bits) | column in tile (7 bits) | valid (1) |
// the input value in the compute dtype (16 bits), duplicates of a (row, column) merged into one word (their values
// added, the others left invalid) -- so the tile kernel reads each tile's entries as ~1.2 KB of contiguous words.
constexpr int PK_TB = 16;          // tiles per pre-pass workgroup (a thread per batch row of the group)

__device__ __forceinline__ int row_of(const OcfEncTileArgs& a, int b) { return b < a.B ? a.rows[b] : -1; }

// thread b's counts of its row's entries in tiles [t0, t0 + PK_TB) (0 past the last tile / for an empty row)
__device__ __forceinline__ void row_counts(const OcfEncTileArgs& a, int r, int t0, int (&tp)[PK_TB + 1]) {
#pragma unroll
  for (int j = 0; j <= PK_TB; ++j) tp[j] = 0;
  if (r < 0) return;
  const int32_t* p = a.tptr + (int64_t)r * (a.n_tiles + 1);
#pragma unroll
  for (int j = 0; j <= PK_TB; ++j) tp[j] = p[min(t0 + j, a.n_tiles)];
}

// cnt[rg][t] = entries of the row group's rows in tile t: a workgroup per (group, 16 tiles), a thread per row, the
// 256 rows summed per tile by the four waves' reductions (integer sums: order-free)
__global__ void __launch_bounds__(BM) pack_count_kernel(OcfEncTileArgs a, int32_t* cnt) {
  const int rg = blockIdx.y, t0 = blockIdx.x * PK_TB, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  __shared__ int tot[4][PK_TB];
  int tp[PK_TB + 1];
  row_counts(a, row_of(a, rg * BM + tid), t0, tp);
#pragma unroll
  for (int j = 0; j < PK_TB; ++j) {
    int c = tp[j + 1] - tp[j];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
    if (lane == 0) tot[wave][j] = c;
  }
  __syncthreads();
  if (tid < PK_TB && t0 + tid < a.n_tiles)
    cnt[(int64_t)rg * (a.n_tiles + 1) + t0 + tid] = tot[0][tid] + tot[1][tid] + tot[2][tid] + tot[3][tid];
}

// exclusive scan of one row group's counts (in place) -> bucket pointers; the group's base = the previous groups'
// totals (groups scanned in order by one workgroup each: group rg adds the totals of groups < rg from the bases)
__global__ void __launch_bounds__(1024) pack_scan_kernel(OcfEncTileArgs a, int32_t* cnt, int n_rg) {
  __shared__ int part[1024];
  __shared__ int base_sh;
  const int n = a.n_tiles;
  if (threadIdx.x == 0) base_sh = 0;
  __syncthreads();
  for (int rg = 0; rg < n_rg; ++rg) {
    int32_t* c = cnt + (int64_t)rg * (n + 1);
    const int per = (n + 1023) / 1024, i0 = threadIdx.x * per;
    int s = 0;
    for (int i = i0; i < min(n, i0 + per); ++i) s += c[i];
    part[threadIdx.x] = s;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {       // inclusive scan of the thread sums
      const int v = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
      __syncthreads();
      part[threadIdx.x] += v;
      __syncthreads();
    }
    int run = base_sh + (threadIdx.x ? part[threadIdx.x - 1] : 0);
    for (int i = i0; i < min(n, i0 + per); ++i) {
      const int v = c[i];
      c[i] = run;
      run += v;
    }
    __syncthreads();
    if (threadIdx.x == 1023) {
      c[n] = base_sh + part[1023];
      base_sh += part[1023];
    }
    __syncthreads();
  }
}

// each (batch row, tile)'s first word position: the bucket pointer + the entries of the group's rows before it in
// that tile (wave prefix sums + the waves before it): a workgroup per (group, 16 tiles), thread b = row b of the group
__global__ void __launch_bounds__(BM) pack_base_kernel(OcfEncTileArgs a, const int32_t* bptr, int32_t* base) {
  const int rg = blockIdx.y, t0 = blockIdx.x * PK_TB, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  __shared__ int tot[4][PK_TB];
  const int b = rg * BM + tid, r = row_of(a, b);
  int tp[PK_TB + 1];
  row_counts(a, r, t0, tp);
  int pre[PK_TB];
#pragma unroll
  for (int j = 0; j < PK_TB; ++j) {
    const int c = tp[j + 1] - tp[j];
    int v = c;                                          // inclusive scan over the wave's lanes
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int u = __shfl_up(v, off);
      if (lane >= off) v += u;
    }
    pre[j] = v - c;
    if (lane == 63) tot[wave][j] = v;
  }
  __syncthreads();
  if (b >= a.B) return;
#pragma unroll
  for (int j = 0; j < PK_TB; ++j) {
    if (t0 + j >= a.n_tiles) break;
    int w = 0;
    for (int k = 0; k < wave; ++k) w += tot[k][j];
    // (relative to the row's first entry of the tile: word position = base + entry position in the row's view)
    base[(int64_t)b * a.n_tiles + t0 + j] = bptr[(int64_t)rg * (a.n_tiles + 1) + t0 + j] + w + pre[j] - tp[j];
  }
}

// the words themselves, a thread per entry of the batch rows' views (grid: batch row x chunks of 1,024 entries):
// word position = base[b][tile] + the entry's position in the row's view; a run of one (row, column) -- duplicate
// ratings, adjacent in the column-sorted view -- becomes one word holding the run's sum and invalid words
constexpr int PK_CHUNK = 1024;
template <typename CT>
__global__ void __launch_bounds__(256) pack_words_kernel(OcfEncTileArgs a, const int32_t* base, uint32_t* ent) {
  const int b = blockIdx.y, r = row_of(a, b);
  if (r < 0) return;
  const int64_t rp0 = a.rp[r], len = a.rp[r + 1] - rp0, lb = a.lboff[b];
  const int32_t* bs = base + (int64_t)b * a.n_tiles;
  const int rl = b % BM;
#pragma unroll
  for (int k = 0; k < PK_CHUNK / 256; ++k) {
    const int64_t p = (int64_t)blockIdx.x * PK_CHUNK + 256 * k + threadIdx.x;
    if (p >= len) break;
    const int64_t e = rp0 + p;
    const int col = a.tcol[e], t = col / BK;
    const bool head = p == 0 || a.tcol[e - 1] != col;
    uint32_t w = 0;
    if (head) {
      float x = a.xval[lb + a.tlidx[e]];
      for (int64_t f = e + 1; f < rp0 + len && a.tcol[f] == col; ++f) x += a.xval[lb + a.tlidx[f]];
      const CT h = CvtT<CT>::to(x);
      uint16_t vb;
      __builtin_memcpy(&vb, &h, 2);
      w = (uint32_t)rl | ((uint32_t)(col - t * BK) << 8) | (1u << 15) | ((uint32_t)vb << 16);
    }
    ent[bs[t] + p] = w;
  }
}

constexpr int PEMAX = 4;   // bucket words per thread per tile held in registers (a bucket of <= 1,024 words)
constexpr int STEP_LOADS = 8 + 1 + PEMAX;   // VMEM instructions one step issues (W1 tile, a bucket pointer, words)

// W1 tiles three deep (two in flight during a tile's MFMAs: at one wave per SIMD a single 32-KB tile in flight left
// the loads' latency exposed); LDS = the X image + three W1 buffers = 160 KB
template <typename CT>
__global__ void __launch_bounds__(256) enc_tiles_packed_kernel(OcfEncTileArgs a, const int32_t* bptr,
                                                                const uint32_t* ent, int n_rg, int n_hs,
                                                                int tiles_per) {
  __shared__ __attribute__((aligned(16))) char xs[BM * ROWB];
  __shared__ __attribute__((aligned(16))) char wsA[BK * ROWB];
  __shared__ __attribute__((aligned(16))) char wsB[BK * ROWB];
  __shared__ __attribute__((aligned(16))) char wsC[BK * ROWB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int per = n_rg * n_hs;
  const int bx = blockIdx.x, xcd = bx & 7, slot = bx >> 3;
  const int S = a.splits, s = (slot / per) * 8 + xcd, rem = slot % per, rg = rem / n_hs, hs = rem % n_hs;
  if (s >= S) return;
  const int t0 = s * tiles_per, t1 = min(a.n_tiles, t0 + tiles_per);
  if (t0 >= t1) {
    for (int i = tid; i < BM * BH; i += 256) {
      const int b = rg * BM + i / BH;
      if (b < a.Bp) a.part[((int64_t)b * S + s) * a.H + hs * BH + (i % BH)] = 0.f;
    }
    return;
  }
  const int h0 = hs * BH;
  using F = Frag<CT>;
  using FT = typename F::T;
  const char* Wb = reinterpret_cast<const char*>(a.W);
  // every step issues the same loads (clamped to the split's last tile) so that one vmcnt count fits every step
  auto wload = [&](int t, char* dst) {
    t = min(t, t1 - 1);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int n0 = 4 * (4 * i + wave), n = n0 + (lane >> 4), c = (lane & 15) ^ (((n & 3) << 2) | ((n >> 2) & 3));
      const char* src = Wb + (((int64_t)t * BK + n) * a.ldw + h0) * 2 + 16 * c;
      __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(dst + n0 * ROWB), 16, 0, 0);
    }
  };
  const int32_t* bpr = bptr + (int64_t)rg * (a.n_tiles + 1);
  auto bpl = [&](int t) { return bpr[min(t, t1)]; };
  const int64_t elast = max(bptr[(int64_t)n_rg * (a.n_tiles + 1) - 1] - 1, 0);   // (every group's words - 1)
  // a tile's words (bucket [lo, hi)): thread tid takes words lo + tid + 256 j; raw clamped loads, masked where used
  auto eload = [&](int lo, uint32_t (&w)[PEMAX]) {
#pragma unroll
    for (int j = 0; j < PEMAX; ++j) w[j] = ent[min((int64_t)lo + tid + 256 * j, elast)];
  };
  auto wput = [&](uint32_t w, bool zero) {
    if (!(w & 0x8000u)) return;
    const int row = w & 255, kk = (w >> 8) & 127;
    *reinterpret_cast<uint16_t*>(xs + xoff(row, kk >> 3) + 2 * (kk & 7)) = zero ? (uint16_t)0 : (uint16_t)(w >> 16);
  };
  // write (zero = false) or clear (zero = true) a tile's words
  auto xput = [&](const uint32_t (&w)[PEMAX], int lo, int hi, bool zero) {
#pragma unroll
    for (int j = 0; j < PEMAX; ++j)
      if (lo + tid + 256 * j < hi) wput(w[j], zero);
    for (int i = lo + tid + 256 * PEMAX; i < hi; i += 256) wput(ent[i], zero);   // (rare) a bucket over 1,024
  };
  // ---- prologue: X image clear, tiles t0 and t0 + 1 in flight, tile t0's words written
  for (int i = tid; i < BM * ROWB / 16; i += 256) reinterpret_cast<uint4*>(xs)[i] = make_uint4(0, 0, 0, 0);
  int q0 = bpl(t0), q1 = bpl(t0 + 1), q2 = bpl(t0 + 2), q3 = bpl(t0 + 3), q4 = bpl(t0 + 4);   // bp(t) .. bp(t + 4)
  wload(t0, wsA);
  wload(t0 + 1, wsB);
  // the words of three consecutive tiles in arrays whose roles rotate with the W1 buffers (no register moves of
  // words still in flight at the loop's back edge)
  uint32_t WX[PEMAX], WY[PEMAX], WZ[PEMAX];
  eload(q0, WX);
  eload(q1, WY);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  xput(WX, q0, q1, false);
  __syncthreads();
  f16v acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int k = 0; k < 16; ++k) acc[i][c][k] = 0.f;
  const int r = lane & 31, hf = lane >> 5, g = lane >> 4, gi = lane & 15, gq = gi >> 2, gp = gi & 3;
  // one tile: t's MFMAs from wcur while t + 1 (issued a step ago) and t + 2 (now, into w2) stream in
  // (the bucket pointer first: moving it into the window waits for it alone, not for the tiles behind it)
  auto step = [&](int t, const char* wcur, char* w2, uint32_t (&W0)[PEMAX], const uint32_t (&W1)[PEMAX],
                  uint32_t (&W2)[PEMAX]) -> bool {
    const int q5 = bpl(t + 5);
    wload(t + 2, w2);
    eload(q2, W2);                                    // tile t + 2's words (bucket [q2, q3))
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      FT fa[2], fb[4];
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[i] = *reinterpret_cast<const FT*>(xs + xoff(64 * wave + 32 * i + r, 2 * ks + hf));
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int ch = 4 * c + 2 * (g & 1) + (gp >> 1);
        const int nr = 16 * ks + 8 * (g >> 1) + gq;
        const s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s4*)(wcur + woff(nr, ch) + 8 * (gp & 1)));
        const s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s4*)(wcur + woff(nr + 4, ch) + 8 * (gp & 1)));
        const short e[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        __builtin_memcpy(&fb[c], e, 16);
      }
#ifndef OCF_ET_NOMFMA
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[i][c] = F::mfma(fa[i], fb[c], acc[i][c]);
#else
      acc[0][0][ks] += (float)fa[0][0] + (float)fb[0][0] + (float)fa[1][1] + (float)fb[1][1] + (float)fb[2][2] +
                       (float)fb[3][3];
#endif
    }
    if (t + 1 >= t1) return false;
    // the previous step's loads (tile t + 1's W1 image and words, bp(t + 4)) are done; this step's may still fly.
    // The barriers here are bare s_barrier + lgkmcnt(0) (LDS writes visible): __syncthreads' workgroup release
    // would also wait for this step's direct-to-LDS loads (vmcnt(0)), i.e. undo the prefetch
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(STEP_LOADS) : "memory");
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // every wave is done with tile t's images
#ifndef OCF_ET_NOX
    xput(W0, q0, q1, true);                           // clear tile t's words
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // (a row's words of two tiles may share a position)
    xput(W1, q1, q2, false);                          // tile t + 1's
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#endif
    q0 = q1; q1 = q2; q2 = q3; q3 = q4; q4 = q5;
    return true;
  };
  for (int t = t0; t < t1; t += 3)                    // (three tiles per trip: each W1 buffer a static LDS object)
    if (!step(t, wsA, wsC, WX, WY, WZ) || !step(t + 1, wsB, wsA, WY, WZ, WX) || !step(t + 2, wsC, wsB, WZ, WX, WY))
      break;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");    // (the last steps' unused loads land before the exit)
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

namespace ocf {
int g_enc_tiles_pack = 1;   // ocf_set_tuning "enc_tiles_pack": the packed pre-pass (1) or the per-row chain (0)
}

namespace {
struct TileWork {   // the pre-pass scratch: bucket pointers [n_rg][n_tiles + 1], row bases [B][n_tiles], words
  int64_t cnt, base, ent, total;
};
TileWork tile_work(const OcfEncTileArgs& a) {
  const int64_t n_rg = (a.Bp + et::BM - 1) / et::BM;
  auto r = [](int64_t bytes) { return (bytes + 255) / 256 * 256; };
  TileWork w;
  w.cnt = 0;
  w.base = r(n_rg * (a.n_tiles + 1) * 4);
  w.ent = w.base + r((int64_t)std::max(a.B, 1) * a.n_tiles * 4);
  w.total = w.ent + r(std::max<int64_t>(a.n_entries, 1) * 4);
  return w;
}
}  // namespace

extern "C" int64_t ocf_encoder_tiles_workspace(const OcfEncTileArgs* a) {
  if (!a || a->Bp < 0 || a->B < 0 || a->n_tiles < 1 || a->n_entries < 0) return -1;
  return tile_work(*a).total;
}

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
  OCF_CHECK(a.nnz >= 1 && a.n_entries >= 1, "ocf_encoder_tiles: nnz, n_entries >= 1 (the clamp bounds)");
  if (a.Bp == 0) return 0;
  const int n_rg = (a.Bp + et::BM - 1) / et::BM, n_hs = a.H / et::BH;
  const int tiles_per = (a.n_tiles + a.splits - 1) / a.splits;
  OCF_CHECK(tiles_per <= 1024, "ocf_encoder_tiles: more than 1,024 tiles per split (raise splits)");
  const int grid = (a.splits + 7) / 8 * 8 * n_rg * n_hs;
  hipStream_t s = (hipStream_t)stream;
  const bool f16 = a.w_dtype == OCF_F16;
  if (g_enc_tiles_pack) {
    const int64_t need = ocf_encoder_tiles_workspace(&a);
    OCF_CHECK(a.work && a.work_bytes >= need, "ocf_encoder_tiles: workspace too small (ocf_encoder_tiles_workspace)");
    const TileWork tw = tile_work(a);
    char* wb = reinterpret_cast<char*>(a.work);
    int32_t* cnt = reinterpret_cast<int32_t*>(wb + tw.cnt);
    int32_t* base = reinterpret_cast<int32_t*>(wb + tw.base);
    uint32_t* ent = reinterpret_cast<uint32_t*>(wb + tw.ent);
    const dim3 pg((a.n_tiles + et::PK_TB - 1) / et::PK_TB, n_rg);
    int64_t max_len = a.max_row_len > 0 ? a.max_row_len : 0;
    OCF_CHECK(max_len > 0, "ocf_encoder_tiles: max_row_len (the longest batch row's view length) required");
    const dim3 wg((unsigned)((max_len + et::PK_CHUNK - 1) / et::PK_CHUNK), (unsigned)a.B);
#ifndef OCF_ET_NOPACK
    hipLaunchKernelGGL(et::pack_count_kernel, pg, dim3(et::BM), 0, s, a, cnt);
    hipLaunchKernelGGL(et::pack_scan_kernel, dim3(1), dim3(1024), 0, s, a, cnt, n_rg);
    hipLaunchKernelGGL(et::pack_base_kernel, pg, dim3(et::BM), 0, s, a, cnt, base);
#endif
    if (f16) {
#ifndef OCF_ET_NOPACK
      if (a.B) hipLaunchKernelGGL(et::pack_words_kernel<_Float16>, wg, dim3(256), 0, s, a, base, ent);
#endif
      hipLaunchKernelGGL(et::enc_tiles_packed_kernel<_Float16>, dim3(grid), dim3(256), 0, s, a, cnt, ent, n_rg, n_hs,
                         tiles_per);
    } else {
#ifndef OCF_ET_NOPACK
      if (a.B) hipLaunchKernelGGL(et::pack_words_kernel<__bf16>, wg, dim3(256), 0, s, a, base, ent);
#endif
      hipLaunchKernelGGL(et::enc_tiles_packed_kernel<__bf16>, dim3(grid), dim3(256), 0, s, a, cnt, ent, n_rg, n_hs,
                         tiles_per);
    }
  } else if (f16) {
    hipLaunchKernelGGL(et::enc_tiles_kernel<_Float16>, dim3(grid), dim3(256), 0, s, a, n_rg, n_hs, tiles_per);
  } else {
    hipLaunchKernelGGL(et::enc_tiles_kernel<__bf16>, dim3(grid), dim3(256), 0, s, a, n_rg, n_hs, tiles_per);
  }
  OCF_HIP(hipGetLastError());
  OCF_TRY_END
}
