// LDS-staged MFMA GEMM template for gfx950 (CDNA4), 64-wide waves.
//
//   C[M,N] (+)= A[M,K] * B[K,N]      fp32 accumulate, epilogue fused per tile
//
// Operands arrive in either of two global layouts and are staged to LDS images the MFMA
// fragments read directly:
//   "row" image  [R][BK]  (K contiguous)  <- A stored [M][K] / B stored [N][K]
//                fragment = ds_read_b128                         (f16/bf16: 8 k per lane)
//   "col" image  [BK][R]  (R contiguous)  <- A stored [K][M] / B stored [K][N]
//                fragment = 2 x ds_read_b64_tr_b16 (CDNA4 transposing LDS read)
// so no operand is ever transposed in HBM or in registers.  Source element type may differ from
// the compute type (fp32 master weights are converted to f16/bf16 while staging).
//
// Tile 128x128, 256 threads = 4 waves in 2x2, each wave 64x64 = 2x2 blocks of
// v_mfma_f32_32x32x16_{f16,bf16} (BK = 64) or v_mfma_f32_32x32x2_f32 (BK = 32, exact-f32 mode).
// Register-prefetch double buffering: one barrier per K-step (cdna_hip_programming.md T14).
#pragma once
#include "ocf_common.h"

namespace ocf {

constexpr int GT_BM = 128;
constexpr int GT_BN = 128;
constexpr int GT_THREADS = 256;

#ifndef OCF_FRAG_PREFETCH
#define OCF_FRAG_PREFETCH 1
#endif

template <typename CT> struct KInfo { static constexpr int BK = 64; };
template <> struct KInfo<float> { static constexpr int BK = 32; };

// byte strides of the two LDS image kinds (see bank analysis in DESIGN.md):
//   row image: BK*s + 16  -> 144 B = 9 x 16-B slots (odd): ds_read_b128 conflict-free
//   col image: R*s + 64   -> rows 16 banks apart: ds_read_b64_tr_b16 conflict-free (f16/bf16)
template <typename CT, int R, bool COL> struct Img {
  static constexpr int BK = KInfo<CT>::BK;
  static constexpr int ES = (int)sizeof(CT);
  static constexpr int STRIDE = COL ? (R * ES + (ES == 2 ? 64 : 16)) : (BK * ES + 16);
  static constexpr int BYTES = COL ? BK * STRIDE : R * STRIDE;
};

// ---------------------------------------------------------------------------------------
// global -> register -> LDS staging of one operand tile (R rows of the M/N dim x BK).
// Loads are buffer loads: a wave-uniform descriptor at the tile origin (SGPRs), a 32-bit byte
// offset per chunk fixed for the whole K-loop (VGPRs), and the K advance as the SGPR soffset.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7FFFFFFF, 0x00020000);
}

template <typename GT, typename CT, int R, bool COL> struct Stager {
  static constexpr int BK = KInfo<CT>::BK;
  static constexpr int CHUNKS = R * BK / 8;  // 8 elements per chunk
  static constexpr int NCH = CHUNKS / GT_THREADS;
  static_assert(NCH * GT_THREADS == CHUNKS, "tile/threads mismatch");
  GT v[NCH][8];

  // byte offset of this thread's chunk i from the tile origin at k = 0; ld in elements.
  // blk: the operand is stored 64x64-blocked (rows in blocks of 64, columns in blocks of 64, each
  // block 64 rows x 128 B contiguous, blocks row-major; 16-bit elements): a K-step tile is two
  // contiguous 8 KB blocks instead of 64-128 strided row pieces.
  __device__ __forceinline__ static uint32_t chunk_off(int64_t ld, int tid, int i, bool blk) {
    int c = tid + i * GT_THREADS;
    if (blk) {
      if (!COL) {  // [R][K]: r within the tile, kc = 16-B chunk of the 64-wide K-step
        int r = c / (BK / 8), kc = c % (BK / 8);
        return (uint32_t)((r >> 6) * ld * 128 + (r & 63) * 128 + kc * 16);
      } else {     // [K][R]: k within the K-step, 8 consecutive r
        int k = c / (R / 8), rr = (c % (R / 8)) * 8;
        return (uint32_t)((rr >> 6) * 8192 + k * 128 + (rr & 63) * 2);
      }
    }
    int64_t e;
    if (!COL) {  // [R][K] k-contiguous; chunk = 8 consecutive k of one row
      int r = c / (BK / 8), kc = c % (BK / 8);
      e = (int64_t)r * ld + kc * 8;
    } else {  // [K][R] r-contiguous; chunk = 8 consecutive r of one k
      int k = c / (R / 8), rc = c % (R / 8);
      e = (int64_t)k * ld + rc * 8;
    }
    return (uint32_t)(e * (int64_t)sizeof(GT));
  }
  // byte advance of the tile origin per K-step
  __device__ __forceinline__ static uint32_t step_bytes(int64_t ld, bool blk) {
    if (blk) return (uint32_t)(COL ? ld * 128 : 8192);
    return (uint32_t)((COL ? (int64_t)BK * ld : (int64_t)BK) * (int64_t)sizeof(GT));
  }
  // byte offset of the tile origin (rdim0 along R, k0 along K) in a 64x64-blocked array
  __device__ __forceinline__ static int64_t blocked_origin(int64_t ld, int rdim0, int k0) {
    return COL ? (int64_t)(k0 >> 6) * ld * 128 + (int64_t)(rdim0 >> 6) * 8192
               : (int64_t)(rdim0 >> 6) * ld * 128 + (int64_t)(k0 >> 6) * 8192;
  }

  template <int AUX>
  __device__ __forceinline__ void load_pol(__amdgpu_buffer_rsrc_t rs, int64_t ld, uint32_t soff, int tid, bool blk) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const uint32_t o = chunk_off(ld, tid, i, blk);
      if constexpr (sizeof(GT) == 4) {
        auto a = __builtin_amdgcn_raw_buffer_load_b128(rs, o, soff, AUX);
        auto b = __builtin_amdgcn_raw_buffer_load_b128(rs, o + 16, soff, AUX);
        __builtin_memcpy(&v[i][0], &a, 16);
        __builtin_memcpy(&v[i][4], &b, 16);
      } else {
        auto a = __builtin_amdgcn_raw_buffer_load_b128(rs, o, soff, AUX);
        __builtin_memcpy(&v[i][0], &a, 16);
      }
    }
  }
  // nt: wave-uniform choice of the non-temporal cache policy (the operand's last use in the step)
  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t rs, int64_t ld, uint32_t soff, int tid, bool nt,
                                       bool blk = false) {
    if (nt) load_pol<2>(rs, ld, soff, tid, blk);
    else load_pol<0>(rs, ld, soff, tid, blk);
  }

  __device__ __forceinline__ void store(char* img, int tid) const {
    using I = Img<CT, R, COL>;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      int c = tid + i * GT_THREADS;
      char* dst;
      if (!COL) {
        int r = c / (BK / 8), kc = c % (BK / 8);
        dst = img + r * I::STRIDE + kc * 8 * (int)sizeof(CT);
      } else {
        int k = c / (R / 8), rc = c % (R / 8);
        dst = img + k * I::STRIDE + rc * 8 * (int)sizeof(CT);
      }
      CT o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = CvtT<CT>::to((float)v[i][j]);
      if constexpr (sizeof(CT) == 2) {
        uint4 w;
        __builtin_memcpy(&w, o, 16);
        *reinterpret_cast<uint4*>(dst) = w;
      } else {
        float4 a = make_float4(o[0], o[1], o[2], o[3]);
        float4 b = make_float4(o[4], o[5], o[6], o[7]);
        reinterpret_cast<float4*>(dst)[0] = a;
        reinterpret_cast<float4*>(dst)[1] = b;
      }
    }
  }
};

// ---------------------------------------------------------------------------------------
// MFMA fragment readers
template <typename CT> struct Frag;
template <> struct Frag<_Float16> { using T = ocf_h8; };
template <> struct Frag<__bf16> { using T = ocf_b8; };

// f16/bf16: k-substep ks (16 k), block of 32 rows starting at rb within the image
template <typename CT, int R, bool COL>
__device__ __forceinline__ typename Frag<CT>::T read_frag16(const char* img, int rb, int ks, int lane) {
  using I = Img<CT, R, COL>;
  typename Frag<CT>::T f;
  if constexpr (!COL) {
    const char* p = img + (rb + (lane & 31)) * I::STRIDE + (16 * ks + 8 * (lane >> 5)) * 2;
    uint4 w = *reinterpret_cast<const uint4*>(p);
    __builtin_memcpy(&f, &w, 16);
  } else {
    // 16-lane group g reads a 4(k) x 16(r) block; lane 4q+p addresses row q, cols 4p..4p+3
    int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
    int r0 = rb + 16 * (g & 1);
    int k0 = 16 * ks + 8 * (g >> 1);
    const char* p = img + (k0 + q) * I::STRIDE + (r0 + 4 * pp) * 2;
    ocf_s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) ocf_s4*)(size_t)(p));
    ocf_s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) ocf_s4*)(size_t)(p + 4 * I::STRIDE));
    short s8[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    __builtin_memcpy(&f, s8, 16);
  }
  return f;
}

// f32: the whole BK=32 slice for one lane: 16 values, substep s uses element s
// (k index of (lane half h, substep s) is 16h + s -- same map for A and B)
template <int R, bool COL>
__device__ __forceinline__ void read_frag32(const char* img, int rb, int lane, float (&out)[16]) {
  using I = Img<float, R, COL>;
  int r = lane & 31, h = lane >> 5;
  if constexpr (!COL) {
    const char* p = img + (rb + r) * I::STRIDE + 16 * h * 4;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float4 w = reinterpret_cast<const float4*>(p)[q];
      out[4 * q + 0] = w.x; out[4 * q + 1] = w.y; out[4 * q + 2] = w.z; out[4 * q + 3] = w.w;
    }
  } else {
#pragma unroll
    for (int s = 0; s < 16; ++s)
      out[s] = *reinterpret_cast<const float*>(img + (16 * h + s) * I::STRIDE + (rb + r) * 4);
  }
}

// ---------------------------------------------------------------------------------------
// accumulator element -> (row, col) within the wave's 64x64 sub-tile
__device__ __forceinline__ int acc_row(int bi, int reg, int lane) {
  return 32 * bi + (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
}
__device__ __forceinline__ int acc_col(int bj, int lane) { return 32 * bj + (lane & 31); }

struct TileCtx {
  int m0, n0;    // tile origin (global)
  int wm, wn;    // wave origin within the tile (0 or 64)
  int lane, tid;
  int split;     // split-K index
  int tile_m, tile_n;
  char* lds;     // LDS scratch (operand buffers are free at epilogue time)
};

struct GemmShape {
  const void* A;
  const void* B;
  int64_t lda, ldb;
  int M, N, K;
  int kchunk;    // K elements per split (multiple of BK)
  int a_nt, b_nt;  // non-temporal operand loads
  int b_blk;       // B stored 64x64-blocked (16-bit compute-dtype shadows)
  int order;     // 0: n-fastest tile order, 1: m-fastest (XCD-local neighbours)
  // sparse A (gemm_kernel SPA): A = [K][M] built in LDS from a CSR's column-sorted view.  K index =
  // batch row b, M index = column n; value = sp_vals[sp_lboff[b] + list index] (0 = no entry)
  const int32_t* sp_rows; const int64_t* sp_rp; const int32_t* sp_tptr; const int32_t* sp_col;
  const int32_t* sp_lidx; const int64_t* sp_lboff; const float* sp_vals;
  int sp_ntiles, sp_krows;   // column tiles per CSR row; batch rows that exist (K beyond is padding)
  float* sp_colsum;          // nullable: out[m] = colsum_scale * sum_k A[k][m] (tile_n == 0 workgroups)
  float colsum_scale;
  // sparse A bucketed by (column tile, K-step) (ocf_sparse_tiles; optim_ws_kernel)
  const int32_t* sp_bptr; const int2* sp_ent;
};

// Fill the A image of one K-step from sparse entries: zero it, then 4 threads per batch row walk the
// row's entries of this 128-column tile (each (k, m) has at most one nonzero: duplicates and
// non-entries carry value 0 and are skipped).  Caller synchronises before and after.
template <typename CT, int R, int BK>
__device__ __forceinline__ void sparse_a_zero(char* img, int tid) {
  using I = Img<CT, R, true>;
  uint4* p = reinterpret_cast<uint4*>(img);
  constexpr int N16 = I::BYTES / 16;
  for (int i = tid; i < N16; i += GT_THREADS) p[i] = make_uint4(0, 0, 0, 0);
}
template <typename CT, int R, int BK>
__device__ __forceinline__ void sparse_a_fill(const GemmShape& sh, char* img, int k0, int m0, int tid) {
  using I = Img<CT, R, true>;
  const int k = tid >> 2, sub = tid & 3;
  if (k >= BK) return;
  const int b = k0 + k;
  if (b >= sh.sp_krows) return;
  const int r = sh.sp_rows[b];
  if (r < 0) return;
  const int t = m0 / R;
  const int32_t* tp = sh.sp_tptr + (int64_t)r * (sh.sp_ntiles + 1) + t;
  const int64_t base = sh.sp_rp[r];
  const int64_t lo = base + tp[0], hi = base + tp[1];
  const int64_t lb = sh.sp_lboff[b];
  for (int64_t e = lo + sub; e < hi; e += 4) {
    const float v = sh.sp_vals[lb + sh.sp_lidx[e]];
    if (v == 0.f) continue;
    const int m = sh.sp_col[e] - m0;
    *reinterpret_cast<CT*>(img + k * I::STRIDE + m * (int)sizeof(CT)) = CvtT<CT>::to(v);
  }
}

// one K-step of the wave's 64x64 sub-tile (2x2 blocks of 32x32) from the LDS operand images
// column c of a [K][M] LDS image summed over its BK rows in k order (the output-bias gradient):
// loads batched 16 at a time so the fixed-order add chain does not wait on each LDS read
template <typename CT, int BK>
__device__ __forceinline__ float colsum_kstep(const char* img, int stride, int c) {
  float s0 = 0.f;
#pragma unroll
  for (int k0 = 0; k0 < BK; k0 += 16) {
    CT v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = *reinterpret_cast<const CT*>(img + (k0 + j) * stride + c * (int)sizeof(CT));
#pragma unroll
    for (int j = 0; j < 16; ++j) s0 += (float)v[j];
  }
  return s0;
}

template <typename CT, bool ACOL, bool BCOL, int RA = GT_BM, int RB = GT_BN>
__device__ __forceinline__ void mfma_kstep(const char* bufA, const char* bufB, int wm, int wn, int lane,
                                           ocf_f16v (&acc)[2][2]) {
  constexpr int BK = KInfo<CT>::BK;
  if constexpr (sizeof(CT) == 2) {
#if OCF_FRAG_PREFETCH
    // all fragments of the K-step first (one LDS latency per step instead of one per 16-deep slice)
    typename Frag<CT>::T fa[BK / 16][2], fb[BK / 16][2];
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[ks][i] = read_frag16<CT, RA, ACOL>(bufA, wm + 32 * i, ks, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) fb[ks][j] = read_frag16<CT, RB, BCOL>(bufB, wn + 32 * j, ks, lane);
    }
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          if constexpr (std::is_same<CT, _Float16>::value)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[ks][i], fb[ks][j], acc[i][j], 0, 0, 0);
          else
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[ks][i], fb[ks][j], acc[i][j], 0, 0, 0);
        }
#else
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      typename Frag<CT>::T fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[i] = read_frag16<CT, RA, ACOL>(bufA, wm + 32 * i, ks, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) fb[j] = read_frag16<CT, RB, BCOL>(bufB, wn + 32 * j, ks, lane);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          if constexpr (std::is_same<CT, _Float16>::value)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[i], fb[j], acc[i][j], 0, 0, 0);
          else
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
        }
    }
#endif
  } else {
    float fa[2][16], fb[2][16];
#pragma unroll
    for (int i = 0; i < 2; ++i) read_frag32<RA, ACOL>(bufA, wm + 32 * i, lane, fa[i]);
#pragma unroll
    for (int j = 0; j < 2; ++j) read_frag32<RB, BCOL>(bufB, wn + 32 * j, lane, fb[j]);
#pragma unroll
    for (int s = 0; s < 16; ++s)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i][s], fb[j][s], acc[i][j], 0, 0, 0);
  }
}

template <typename CT, bool ACOL, bool BCOL, typename AGT, typename BGT> struct GemmCfg {
  using ImgA = Img<CT, GT_BM, ACOL>;
  using ImgB = Img<CT, GT_BN, BCOL>;
  static constexpr int BK = KInfo<CT>::BK;
  static constexpr int BUF = ImgA::BYTES + ImgB::BYTES;
  static constexpr int OPER_LDS = 2 * BUF;
};

// bijective XCD-aware remap (cdna_hip_programming.md T1): blocks with the same id % 8 run on
// one XCD; give each such class a contiguous range of logical tiles.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (orig >> 3);
}

template <typename CT, bool ACOL, bool BCOL, typename AGT, typename BGT, class Epi, int LDS_BYTES, bool SPA = false>
__global__ void __launch_bounds__(GT_THREADS)
gemm_kernel(GemmShape sh, typename Epi::Params ep) {
  using Cfg = GemmCfg<CT, ACOL, BCOL, AGT, BGT>;
  constexpr int BK = Cfg::BK;
  __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int gm = sh.M / GT_BM, gn = sh.N / GT_BN;
  const int ntile = gm * gn;
  const int nwg = ntile * gridDim.y;
  const int lin = xcd_remap(blockIdx.x + gridDim.x * blockIdx.y, nwg);
  const int split = lin / ntile;
  const int t = lin % ntile;
  const int tile_m = sh.order ? (t % gm) : (t / gn);
  const int tile_n = sh.order ? (t / gm) : (t % gn);
  const int m0 = tile_m * GT_BM, n0 = tile_n * GT_BN;
  const int k_begin = split * sh.kchunk;
  int k_end = k_begin + sh.kchunk;
  if (k_end > sh.K) k_end = sh.K;
  const int nk = (k_end - k_begin) / BK;

  const AGT* Ag = reinterpret_cast<const AGT*>(sh.A);
  const BGT* Bg = reinterpret_cast<const BGT*>(sh.B);
  // buffer descriptors at the tile origins (k = k_begin); K-steps advance through soffset
  const __amdgpu_buffer_rsrc_t ra =
      tile_rsrc(ACOL ? Ag + (int64_t)k_begin * sh.lda + m0 : Ag + (int64_t)m0 * sh.lda + k_begin);
  const bool bblk = sizeof(BGT) == 2 && sh.b_blk;
  const __amdgpu_buffer_rsrc_t rb =
      bblk ? tile_rsrc(reinterpret_cast<const char*>(Bg) +
                       Stager<BGT, CT, GT_BN, BCOL>::blocked_origin(sh.ldb, n0, k_begin))
           : tile_rsrc(BCOL ? Bg + (int64_t)k_begin * sh.ldb + n0 : Bg + (int64_t)n0 * sh.ldb + k_begin);

  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  // epilogue inputs that do not depend on the product (e.g. target buckets) are loaded here, so
  // their latency hides under the K-loop
  const typename Epi::Pre pre = Epi::prologue(ep, tile_m, tile_n, m0, n0, tid, sh);

  ocf_f16v acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto compute = [&](const char* bufA) {
    mfma_kstep<CT, ACOL, BCOL>(bufA, bufA + Cfg::ImgA::BYTES, wm, wn, lane, acc);
  };
  char* buf0 = lds;
  char* buf1 = lds + Cfg::BUF;

  // output-column sums of a [K][M] A for the tile_n == 0 workgroups (the output-bias gradient), in
  // fixed k order, from each K-step's A image once it is in LDS
  const bool colsum = ACOL && sh.sp_colsum && tile_n == 0;
  float csum = 0.f;
  auto sum_a = [&](const char* img) {
    if constexpr (ACOL) {
      if (colsum && tid < GT_BM) csum += colsum_kstep<CT, BK>(img, Img<CT, GT_BM, true>::STRIDE, tid);
    }
  };
  {
    Stager<AGT, CT, GT_BM, ACOL> sa;
    Stager<BGT, CT, GT_BN, BCOL> sb;
    const uint32_t sta = decltype(sa)::step_bytes(sh.lda, false), stb = decltype(sb)::step_bytes(sh.ldb, bblk);
    auto fill_a = [&](char* img, int kt) {   // SPA: zero + scatter the A image of K-step kt
      if constexpr (SPA) {
        sparse_a_zero<CT, GT_BM, BK>(img, tid);
        __syncthreads();
        sparse_a_fill<CT, GT_BM, BK>(sh, img, k_begin + kt * BK, m0, tid);
      }
    };
    if (nk > 0) {
      if constexpr (!SPA) sa.load(ra, sh.lda, 0, tid, sh.a_nt);
      sb.load(rb, sh.ldb, 0, tid, sh.b_nt, bblk);
      if constexpr (SPA) fill_a(buf0, 0);
      else sa.store(buf0, tid);
      sb.store(buf0 + Cfg::ImgA::BYTES, tid);
      __syncthreads();
      sum_a(buf0);
    }
    for (int kt = 0; kt < nk; ++kt) {
      const bool more = kt + 1 < nk;
      if (more) {
        if constexpr (!SPA) sa.load(ra, sh.lda, (kt + 1) * sta, tid, sh.a_nt);
        sb.load(rb, sh.ldb, (kt + 1) * stb, tid, sh.b_nt, bblk);
      }
      compute((kt & 1) ? buf1 : buf0);
      if (more) {
        char* nb = ((kt + 1) & 1) ? buf1 : buf0;
        if constexpr (SPA) fill_a(nb, kt + 1);
        else sa.store(nb, tid);
        sb.store(nb + Cfg::ImgA::BYTES, tid);
      }
      __syncthreads();
      if (more) sum_a(((kt + 1) & 1) ? buf1 : buf0);
    }
  }
  if (colsum && tid < GT_BM) sh.sp_colsum[m0 + tid] = csum * sh.colsum_scale;

  TileCtx c;
  c.m0 = m0; c.n0 = n0; c.wm = wm; c.wn = wn; c.lane = lane; c.tid = tid;
  c.split = split; c.tile_m = tile_m; c.tile_n = tile_n; c.lds = lds;
  Epi::apply(ep, acc, c, sh, pre);
}

}  // namespace ocf
