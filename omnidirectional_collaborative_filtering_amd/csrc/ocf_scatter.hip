// K1: sparse-rating -> dense-batch assembly (replaces data_reader.py:95-298).
//
// Flattened grid (one thread per batch entry, see scatter_flat_kernel).  The dataset lives in HBM as row-CSR in the reference's list
// order (row_ptr int64, col int32 = dense column index, val f32) plus an optional duplicate
// chain dup[e] = next entry of the same row with the same column (or -1), so that the
// reference's last-write-wins per array (data_reader.py:158-166, 250-266) is reproduced by a
// parallel scatter: an entry writes a *value* array only if no later entry of its chain
// writes that array.  Mask arrays all receive the same constant (aux) so they need no check.
//
// Entry roles:
//   train  (mode 0): input  = keep (reciprocal split, data_reader.py:130,158)
//                    target = !keep || pass_through (:161-166)
//   eval   (mode 1): source-1 entries are inputs only (:234-252),
//                    source-2 entries are targets only (:256-268)
// Outputs (all optional): dense f32 X / M_in / M_out / T / M_miss (the data_gen API arrays),
// the concatenated layer-0 input in the compute dtype, and the target entries bucketed by
// 128-column tile for the fused masked-MSE epilogue.
#include "ocf_internal.h"

namespace ocf {

__device__ __forceinline__ float reciprocal_cut(float s) { return (1.0f - s) / ((1.0f - s) + s); }

__device__ __forceinline__ bool keep_of(const ScatterArgs& a, int b, int64_t local_j, int64_t bo1, float cut) {
  if (a.keep1) return a.keep1[bo1 + local_j] != 0;
  if (a.s0 >= 1.0f) return true;
  float u = philox_uniform(a.seed, a.stream + 1, (uint64_t)(bo1 + local_j));
  return u >= cut;
}

__device__ __forceinline__ float row_cut(const ScatterArgs& a, int b) {
  if (a.keep1 || a.s0 >= 1.0f) return 0.f;
  float s = a.s0 + (a.s1 - a.s0) * philox_uniform(a.seed, a.stream, (uint64_t)b);
  return reciprocal_cut(s);
}

// role bits: 1 = input, 2 = target
__device__ __forceinline__ int role1(const ScatterArgs& a, int b, int64_t local_j, int64_t bo1, float cut) {
  if (a.mode == 1) return 1;
  bool k = keep_of(a, b, local_j, bo1, cut);
  return (k ? 1 : 0) | ((!k || a.pass_through) ? 2 : 0);
}

__device__ __forceinline__ void store_val(void* base, int dtype, int64_t idx, float v) {
  if (dtype == OCF_F32) reinterpret_cast<float*>(base)[idx] = v;
  else if (dtype == OCF_F16) reinterpret_cast<_Float16*>(base)[idx] = (_Float16)v;
  else reinterpret_cast<__bf16*>(base)[idx] = (__bf16)v;
}

// Flattened launch: one thread per batch entry held by this CSR, SC_THREADS entries per workgroup, so the
// load balances whatever the row lengths (full rows on one GPU, ~1/G of them per column shard).
// Blocks [0, nblk1) take source-1 entries, the rest source-2 entries.  A thread finds its batch row
// by binary search over the batch offsets staged in LDS.  The outputs were zeroed by
// hipMemsetAsync on the same stream before this launch.
#ifndef OCF_SC_THREADS
#define OCF_SC_THREADS 1024   // step A/B 0.5042 (1024) / 0.5078 (512) / 0.5073 (256) ms; scatter_flat 15.6 us either way
#endif
constexpr int SC_THREADS = OCF_SC_THREADS;

__device__ __forceinline__ int find_row(const int64_t* off, int B, int64_t e) {
  int lo = 0, hi = B;   // off[lo] <= e < off[hi]; empty rows are skipped because off[b] == off[b+1]
  while (hi - lo > 1) {
    int mid = (lo + hi) >> 1;
    if (off[mid] <= e) lo = mid;
    else hi = mid;
  }
  return lo;
}

// one batch entry e (of source 1 or 2) with the batch offsets staged in LDS
__device__ __forceinline__ void scatter_entry(const ScatterArgs& a, const int64_t* sh_off, bool src2, int64_t e) {
  const int B = a.B;
  const int b = find_row(sh_off, B, e);
  const int64_t j = e - sh_off[b];
  const float aux = a.aux;
  const int64_t xb = a.xin_block;
  if (!src2) {
    const int r1 = a.rows1[b];
    const int64_t s = a.rp1[r1];
    const int64_t i = s + j;
    const int64_t bo1 = a.boff1 ? a.boff1[b] : 0;
    const float cut = row_cut(a, b);
    const int c = a.col1[i];
    const float v = a.val1[i];
    const int role = role1(a, b, a.pos1 ? a.pos1[i] : j, bo1, cut);
    // later duplicates of the same column that also write the value arrays (last write wins)
    bool later_in = false, later_tg = false;
    if (a.dup1) {
      for (int f = a.dup1[i]; f >= 0; f = a.dup1[f]) {
        int rf = role1(a, b, a.pos1 ? a.pos1[f] : f - s, bo1, cut);
        later_in |= (rf & 1) != 0;
        later_tg |= (rf & 2) != 0;
      }
    }
    const int64_t o = (int64_t)b * a.ld + c;
    const int64_t ox = (int64_t)b * a.xin_ld + c;
    if (role & 1) {
      if (a.Min) a.Min[o] = aux;
      if (!later_in) {
        if (a.X) a.X[o] = v;
        if (a.xin) store_val(a.xin, a.xin_dtype, ox, v);
      }
      if (a.xin && a.feed == 1) store_val(a.xin, a.xin_dtype, ox + xb, aux);
    }
    if (a.xval1) a.xval1[e] = ((role & 1) && !later_in) ? v : 0.f;
    if (a.tb_cnt) atomicAdd(&a.tb_cnt[(c >> 7) * a.tb_nk + (b >> 6)], 1);   // ocf_sparse_tiles counts
    if (a.col_cnt) {                                                         // ocf_row_lists counts / keys
      atomicAdd(&a.col_cnt[c], 1);
      a.ecb[e] = c | (b << 19);
    }
    const bool live_tg = (role & 2) && !later_tg;
    if (role & 2) {
      if (a.Mout) a.Mout[o] = aux;
      if (live_tg && a.T) a.T[o] = v;
      if (live_tg && a.tile_cnt) atomicAdd(&a.tile_cnt[c >> 7], 1);
    }
    if (a.tflag1) a.tflag1[e] = live_tg ? 1 : 0;
    // row tags (ocf.h OcfScatterArgs rtag_*): same-value byte stores, no ordering needed
    if (a.rtag_in && (role & 1) && !later_in) a.rtag_in[c] = (uint8_t)a.rtag;
    if (a.rtag_out && live_tg) a.rtag_out[c] = (uint8_t)a.rtag;
    if (a.Mmiss) a.Mmiss[o] = aux;
    if (a.xin) {
      if (a.feed == 2) store_val(a.xin, a.xin_dtype, ox + xb, aux);
      if (a.both) store_val(a.xin, a.xin_dtype, ox + 2 * xb, aux);
    }
  } else {
    const int r2 = a.rows2[b];
    const int64_t i = a.rp2[r2] + j;
    const int c = a.col2[i];
    const float v = a.val2[i];
    const bool dead = a.dup2 && a.dup2[i] >= 0;   // every source-2 entry is a target
    const int64_t o = (int64_t)b * a.ld + c;
    const int64_t ox = (int64_t)b * a.xin_ld + c;
    if (a.Mout) a.Mout[o] = aux;
    if (!dead && a.T) a.T[o] = v;
    if (!dead && a.tile_cnt) atomicAdd(&a.tile_cnt[c >> 7], 1);
    if (a.tflag2) a.tflag2[e] = dead ? 0 : 1;
    if (a.Mmiss) a.Mmiss[o] = aux;
    if (a.xin) {
      if (a.feed == 2) store_val(a.xin, a.xin_dtype, ox + xb, aux);
      if (a.both) store_val(a.xin, a.xin_dtype, ox + 2 * xb, aux);
    }
  }
}


__global__ void __launch_bounds__(SC_THREADS) scatter_flat_kernel(ScatterArgs a, int nblk1) {
  extern __shared__ int64_t sh_off[];
  const bool src2 = (int)blockIdx.x >= nblk1;
  const int64_t* lboff = src2 ? a.lboff2 : (a.lboff1 ? a.lboff1 : a.boff1);
  for (int i = threadIdx.x; i <= a.B; i += SC_THREADS) sh_off[i] = lboff[i];
  __syncthreads();
  const int64_t e = (int64_t)(src2 ? (int)blockIdx.x - nblk1 : (int)blockIdx.x) * SC_THREADS + threadIdx.x;
  if (e >= (src2 ? a.E2 : a.E1)) return;
  scatter_entry(a, sh_off, src2, e);
}

// every selected batch of an epoch plan at once (ocf_epoch_scatter): base holds batch 0's pointers; slot s
// (epoch batch sel[s]) offsets them and writes its entries' xval / live-target flags at ebase[s].  Only those two
// per-entry outputs (the entry point refuses the dense ones), so an entry needs its value, its role and its
// duplicate chain: SE_U entries per thread, every entry's loads issued before any store, the batch rows' CSR
// starts and keep offsets staged in LDS once per workgroup.  (One entry per thread with the row -> row start ->
// value chain per entry: 37 us per ML-20M 20-batch window, 8 rounds of workgroups of ~3 round trips each.)
constexpr int SE_U = 4;
__global__ void __launch_bounds__(SC_THREADS) scatter_epoch_kernel(ScatterArgs base, OcfEpochScatterArgs ep) {
  extern __shared__ int64_t sh_off[];   // [B + 1] batch-local offsets, [B] CSR row starts, [B] keep offsets
  const int s = blockIdx.y, bi = ep.sel[s];
  ScatterArgs a = base;
  a.rows1 = base.rows1 + (int64_t)bi * base.B;
  a.lboff1 = base.lboff1 ? base.lboff1 + (int64_t)bi * (base.B + 1) : nullptr;
  a.boff1 = base.boff1 ? base.boff1 + (int64_t)bi * (base.B + 1) : nullptr;
  a.keep1 = base.keep1 ? base.keep1 + ep.keep_off[bi] : nullptr;
  a.stream = ep.stream_mul * (uint64_t)(bi + 1);
  a.E1 = ep.ebase[s + 1] - ep.ebase[s];
  float* xval = ep.xval + (ep.ebase[s] - ep.ebase0);
  uint8_t* tflag = ep.tflag + (ep.ebase[s] - ep.ebase0);
  const int B = a.B;
  const int64_t blk0 = (int64_t)blockIdx.x * SC_THREADS * SE_U;
  if (blk0 >= a.E1) return;                               // (a shorter batch than the grid's longest)
  int64_t* sh_src = sh_off + B + 1;
  int64_t* sh_bo = sh_src + B;
  const int64_t* lboff = a.lboff1 ? a.lboff1 : a.boff1;
  for (int i = threadIdx.x; i <= B; i += SC_THREADS) {
    sh_off[i] = lboff[i];
    if (i < B) {
      const int r = a.rows1[i];
      sh_src[i] = r >= 0 ? a.rp1[r] : 0;                 // (padding rows hold no entry)
      sh_bo[i] = a.boff1 ? a.boff1[i] : 0;
    }
  }
  __syncthreads();
  float v[SE_U];
  int role[SE_U];
  bool later_in[SE_U], later_tg[SE_U];
#pragma unroll
  for (int u = 0; u < SE_U; ++u) {
    const int64_t e = blk0 + (int64_t)u * SC_THREADS + threadIdx.x;
    v[u] = 0.f;
    role[u] = 0;
    later_in[u] = later_tg[u] = false;
    if (e < a.E1) {
      const int b = find_row(sh_off, B, e);
      const int64_t j = e - sh_off[b], st = sh_src[b], i = st + j, bo1 = sh_bo[b];
      const float cut = row_cut(a, b);
      v[u] = a.val1[i];
      role[u] = role1(a, b, a.pos1 ? a.pos1[i] : j, bo1, cut);
      if (a.dup1) {       // later duplicates of the same column that also write the value arrays (last write wins)
        for (int f = a.dup1[i]; f >= 0; f = a.dup1[f]) {
          const int rf = role1(a, b, a.pos1 ? a.pos1[f] : f - st, bo1, cut);
          later_in[u] |= (rf & 1) != 0;
          later_tg[u] |= (rf & 2) != 0;
        }
      }
    }
  }
#pragma unroll
  for (int u = 0; u < SE_U; ++u) {
    const int64_t e = blk0 + (int64_t)u * SC_THREADS + threadIdx.x;
    if (e < a.E1) {
      xval[e] = ((role[u] & 1) && !later_in[u]) ? v[u] : 0.f;
      tflag[e] = ((role[u] & 2) && !later_tg[u]) ? 1 : 0;
    }
  }
}

// exclusive scan of per-tile target counts -> bucket pointers; resets counts for next batch
__global__ void __launch_bounds__(1024) bucket_scan_kernel(int* tile_cnt, int* bk_ptr, int* bk_cur, int n_tiles) {
  __shared__ int part[1024];
  const int tid = threadIdx.x;
  const int per = (n_tiles + 1023) / 1024;
  const int lo = tid * per;
  int hi = lo + per;
  if (hi > n_tiles) hi = n_tiles;
  int s = 0;
  for (int i = lo; i < hi; ++i) s += tile_cnt[i];
  part[tid] = s;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {   // Hillis-Steele inclusive scan
    int v = tid >= off ? part[tid - off] : 0;
    __syncthreads();
    part[tid] += v;
    __syncthreads();
  }
  int run = tid ? part[tid - 1] : 0;
  for (int i = lo; i < hi; ++i) {
    bk_ptr[i] = run;
    bk_cur[i] = run;
    run += tile_cnt[i];
    tile_cnt[i] = 0;
  }
  if (tid == 1023) bk_ptr[n_tiles] = part[1023];
}

__global__ void __launch_bounds__(SC_THREADS) bucket_fill_kernel(ScatterArgs a, int nblk1) {
  extern __shared__ int64_t sh_off[];
  const bool src2 = (int)blockIdx.x >= nblk1;
  const int64_t* lboff = src2 ? a.lboff2 : (a.lboff1 ? a.lboff1 : a.boff1);
  const int B = a.B;
  for (int i = threadIdx.x; i <= B; i += SC_THREADS) sh_off[i] = lboff[i];
  __syncthreads();
  const int64_t e = (int64_t)(src2 ? (int)blockIdx.x - nblk1 : (int)blockIdx.x) * SC_THREADS + threadIdx.x;
  if (e >= (src2 ? a.E2 : a.E1)) return;
  const int b = find_row(sh_off, B, e);
  const int64_t j = e - sh_off[b];
  if (!src2) {
    if (a.mode != 0) return;
    const int64_t s = a.rp1[a.rows1[b]];
    const int64_t i = s + j;
    const int64_t bo1 = a.boff1 ? a.boff1[b] : 0;
    const float cut = row_cut(a, b);
    const int role = role1(a, b, a.pos1 ? a.pos1[i] : j, bo1, cut);
    if (!(role & 2)) return;
    if (a.dup1)
      for (int f = a.dup1[i]; f >= 0; f = a.dup1[f])
        if (role1(a, b, a.pos1 ? a.pos1[f] : f - s, bo1, cut) & 2) return;
    const int c = a.col1[i];
    int slot = atomicAdd(&a.bk_cur[c >> 7], 1);
    a.bk_rc[slot] = (b << 7) | (c & 127);
    a.bk_t[slot] = a.val1[i];
    a.bk_m[slot] = a.aux;
  } else {
    const int64_t i = a.rp2[a.rows2[b]] + j;
    if (a.dup2 && a.dup2[i] >= 0) return;
    const int c = a.col2[i];
    int slot = atomicAdd(&a.bk_cur[c >> 7], 1);
    a.bk_rc[slot] = (b << 7) | (c & 127);
    a.bk_t[slot] = a.val2[i];
    a.bk_m[slot] = a.aux;
  }
}

// ---- targets given as dense arrays (Model.train_on_batch / fit / evaluate on user arrays) -----
// An entry wherever T != 0 or M != 0, with its own (t, m).  One workgroup per 128-column tile walks the
// tile's B x 128 elements in (row, column) order: pass 1 counts, bucket_scan_kernel turns the counts into
// bucket pointers, pass 2 places each entry at its rank within the tile (a workgroup prefix sum) -- no
// atomics, so the bucket order (and the masked-MSE sums over it) is run-to-run identical.  (The first
// version took one global atomic per entry on its tile's counter: 74 + 75 us for a Jester batch, all
// 12,800 elements in one tile.)  rows (nullable): batch row b reads source row rows[b] (a device-resident
// dataset gathered by index, Model.fit).
constexpr int DT_THREADS = 1024;

__device__ __forceinline__ bool dense_entry(const float* T, const float* M, int64_t ld, const int64_t* rows, int B,
                                            int N, int t, int64_t i, float& tv, float& mv, int& b, int& n) {
  b = (int)(i >> 7);
  n = t * 128 + (int)(i & 127);
  if (b >= B || n >= N) return false;
  const int64_t o = (rows ? rows[b] : (int64_t)b) * ld + n;
  tv = T[o];
  mv = M[o];
  return tv != 0.f || mv != 0.f;
}

__device__ __forceinline__ int block_exclusive_scan(int v, int* sh, int& total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) sh[wave] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    int run = 0;
    for (int w = 0; w < DT_THREADS / 64; ++w) {
      const int c = sh[w];
      sh[w] = run;
      run += c;
    }
    sh[DT_THREADS / 64] = run;
  }
  __syncthreads();
  const int ex = sh[wave] + x - v;
  total = sh[DT_THREADS / 64];
  __syncthreads();
  return ex;
}

__global__ void __launch_bounds__(DT_THREADS) dense_targets_count_kernel(const float* T, const float* M, int64_t ld,
                                                                          const int64_t* rows, int B, int N,
                                                                          int* tile_cnt) {
  __shared__ int sh[DT_THREADS / 64 + 1];
  const int t = blockIdx.x;
  int c = 0;
  for (int64_t i = threadIdx.x; i < (int64_t)B * 128; i += DT_THREADS) {
    float tv, mv;
    int b, n;
    c += dense_entry(T, M, ld, rows, B, N, t, i, tv, mv, b, n) ? 1 : 0;
  }
  int total;
  block_exclusive_scan(c, sh, total);
  if (threadIdx.x == 0) tile_cnt[t] = total;
}

__global__ void __launch_bounds__(DT_THREADS) dense_targets_fill_kernel(const float* T, const float* M, int64_t ld,
                                                                         const int64_t* rows, int B, int N,
                                                                         const int* bk_ptr, int* bk_rc, float* bk_t,
                                                                         float* bk_m) {
  __shared__ int sh[DT_THREADS / 64 + 1];
  const int t = blockIdx.x;
  int base = bk_ptr[t];
  for (int64_t i0 = 0; i0 < (int64_t)B * 128; i0 += DT_THREADS) {
    float tv = 0.f, mv = 0.f;
    int b = 0, n = 0;
    const bool on = dense_entry(T, M, ld, rows, B, N, t, i0 + threadIdx.x, tv, mv, b, n);
    int total;
    const int r = block_exclusive_scan(on ? 1 : 0, sh, total);
    if (on) {
      const int slot = base + r;
      bk_rc[slot] = (b << 7) | (n & 127);
      bk_t[slot] = tv;
      bk_m[slot] = mv;
    }
    base += total;
  }
}

// pack dense f32 inputs [*][ld_src] (k blocks; batch row b = source row rows[b] when rows is given) into the
// compute-dtype layer-0 input
__global__ void pack_input_kernel(const float* s0, const float* s1, const float* s2, int64_t ld_src, int B, int N,
                                  void* xin, int dtype, int64_t xin_ld, int64_t xin_block, int B_pad,
                                  const int64_t* rows) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t tot = (int64_t)B_pad * xin_ld;
  if (i >= tot) return;
  int b = (int)(i / xin_ld);
  int64_t j = i % xin_ld;
  int blk = (int)(j / xin_block);
  int64_t n = j % xin_block;
  float v = 0.f;
  const float* src = blk == 0 ? s0 : (blk == 1 ? s1 : s2);
  if (b < B && n < N && src) v = src[(rows ? rows[b] : (int64_t)b) * ld_src + n];
  store_val(xin, dtype, i, v);
}

}  // namespace ocf

using namespace ocf;

extern "C" int ocf_epoch_scatter(const ScatterArgs* base, const OcfEpochScatterArgs* ep, void* stream) {
  OCF_TRY_BEGIN
  const ScatterArgs& a = *base;
  const OcfEpochScatterArgs& e = *ep;
  OCF_CHECK(a.mode == 0 && a.rows1 && a.rp1 && a.col1 && a.val1 && (a.lboff1 || a.boff1),
            "ocf_epoch_scatter: a train-mode base with source-1 tables");
  OCF_CHECK(!a.X && !a.Min && !a.Mout && !a.T && !a.Mmiss && !a.xin && !a.tile_cnt && !a.tb_cnt && !a.col_cnt &&
                !a.rtag_in && !a.rtag_out && !a.E2,
            "ocf_epoch_scatter: only the per-entry outputs (xval, live-target flags) are produced");
  OCF_CHECK(e.sel && e.ebase && e.xval && e.tflag && (!a.keep1 || e.keep_off), "ocf_epoch_scatter: null pointer");
  OCF_CHECK(e.n_sel >= 0 && e.n_sel <= 65535 && a.B >= 0 && a.B <= 4096, "ocf_epoch_scatter: sizes (B <= 4,096)");
  if (e.n_sel == 0 || e.max_e == 0) return 0;
  static const bool lds_attr = hipFuncSetAttribute((const void*)scatter_epoch_kernel,
                                                   hipFuncAttributeMaxDynamicSharedMemorySize,
                                                   (3 * 4096 + 1) * (int)sizeof(int64_t)) == hipSuccess;
  OCF_CHECK(lds_attr, "ocf_epoch_scatter: cannot raise the dynamic LDS limit");
  const int nblk = (int)((e.max_e + (int64_t)SC_THREADS * SE_U - 1) / ((int64_t)SC_THREADS * SE_U));
  hipLaunchKernelGGL(scatter_epoch_kernel, dim3(nblk, e.n_sel), dim3(SC_THREADS), (size_t)(3 * a.B + 1) * sizeof(int64_t),
                     (hipStream_t)stream, a, e);
  OCF_HIP(hipGetLastError());
  OCF_TRY_END
}

extern "C" int ocf_scatter_batch(const ScatterArgs* args, void* stream) {
  OCF_TRY_BEGIN
  const ScatterArgs& a = *args;
  hipStream_t s = (hipStream_t)stream;
  OCF_CHECK(a.B >= 0 && a.B <= a.B_pad, "ocf_scatter_batch: need 0 <= B <= B_pad");
  OCF_CHECK(a.mode == 0 || a.mode == 1, "ocf_scatter_batch: mode must be 0 (train) or 1 (eval)");
  OCF_CHECK((a.ld * 4) % 16 == 0, "ocf_scatter_batch: dense ld must be a multiple of 4 floats");
  if (a.xin) OCF_CHECK((a.xin_ld * (a.xin_dtype == OCF_F32 ? 4 : 2)) % 16 == 0, "ocf_scatter_batch: xin ld alignment");
  if (a.tile_cnt) OCF_CHECK(a.bk_ptr && a.bk_cur && a.bk_rc && a.bk_t && a.bk_m && a.n_tiles > 0,
                            "ocf_scatter_batch: bucket outputs incomplete");
  if (a.B_pad == 0) return 0;
  OCF_CHECK(a.B <= 16384, "ocf_scatter_batch: B too large for the LDS offset table");
  OCF_CHECK(a.E1 >= 0 && a.E2 >= 0, "ocf_scatter_batch: negative entry counts");
  OCF_CHECK(a.E2 == 0 || (a.rows2 && a.lboff2), "ocf_scatter_batch: source 2 needs rows2 / lboff2");
  OCF_CHECK(a.E1 == 0 || (a.rows1 && (a.lboff1 || a.boff1)), "ocf_scatter_batch: source 1 needs rows1 / offsets");
  OCF_CHECK(!a.col_cnt || (a.ecb && a.mode == 0 && a.B <= 4096 && a.N <= (1 << 19)),
            "ocf_scatter_batch: col_cnt needs ecb, mode 0, B <= 4096 and N <= 2^19");
  OCF_CHECK(!(a.rtag_in || a.rtag_out) || (a.rtag >= 1 && a.rtag <= 255),
            "ocf_scatter_batch: row tags need 1 <= rtag <= 255");
  // zero rows [0, B_pad) of every dense output (contiguous [B_pad][ld] blocks); outputs that sit back to back
  // in memory are cleared by one memset (each memset is a launch of its own)
  {
    const size_t blk = (size_t)a.B_pad * a.ld * 4;
    float* dense[5] = {a.X, a.Min, a.Mout, a.T, a.Mmiss};
    char* run = nullptr;
    size_t len = 0;
    for (float* d : dense) {
      if (!d) continue;
      char* c = reinterpret_cast<char*>(d);
      if (run && c == run + len) {
        len += blk;
        continue;
      }
      if (run) OCF_HIP(hipMemsetAsync(run, 0, len, s));
      run = c;
      len = blk;
    }
    if (run) OCF_HIP(hipMemsetAsync(run, 0, len, s));
  }
  if (a.xin && !a.xin_clean)
    OCF_HIP(hipMemsetAsync(a.xin, 0, (size_t)a.B_pad * a.xin_ld * (a.xin_dtype == OCF_F32 ? 4 : 2), s));
  const int nblk1 = (int)((a.E1 + SC_THREADS - 1) / SC_THREADS);
  const int nblk2 = (int)((a.E2 + SC_THREADS - 1) / SC_THREADS);
  const size_t shm = (size_t)(a.B + 1) * sizeof(int64_t);
  if (nblk1 + nblk2 > 0)
    hipLaunchKernelGGL(scatter_flat_kernel, dim3(nblk1 + nblk2), dim3(SC_THREADS), shm, s, a, nblk1);
  OCF_HIP(hipGetLastError());
  if (a.tile_cnt) {
    hipLaunchKernelGGL(bucket_scan_kernel, dim3(1), dim3(1024), 0, s, a.tile_cnt, a.bk_ptr, a.bk_cur, a.n_tiles);
    OCF_HIP(hipGetLastError());
    if (nblk1 + nblk2 > 0)
      hipLaunchKernelGGL(bucket_fill_kernel, dim3(nblk1 + nblk2), dim3(SC_THREADS), shm, s, a, nblk1);
    OCF_HIP(hipGetLastError());
  }
  OCF_TRY_END
}


extern "C" int ocf_dense_targets(const float* T, const float* M, int64_t ld, int B, int N, int n_tiles, int* tile_cnt,
                                 int* bk_ptr, int* bk_cur, int* bk_rc, float* bk_t, float* bk_m, const int64_t* rows,
                                 void* stream) {
  OCF_TRY_BEGIN
  hipStream_t s = (hipStream_t)stream;
  OCF_CHECK(T && M && tile_cnt && bk_ptr && bk_cur && bk_rc && bk_t && bk_m, "ocf_dense_targets: null pointer");
  OCF_CHECK(n_tiles * 128 >= N, "ocf_dense_targets: n_tiles too small");
  OCF_CHECK((int64_t)B * 128 < ((int64_t)1 << 31), "ocf_dense_targets: B too large");
  hipLaunchKernelGGL(dense_targets_count_kernel, dim3(n_tiles), dim3(DT_THREADS), 0, s, T, M, ld, rows, B, N, tile_cnt);
  hipLaunchKernelGGL(bucket_scan_kernel, dim3(1), dim3(1024), 0, s, tile_cnt, bk_ptr, bk_cur, n_tiles);
  hipLaunchKernelGGL(dense_targets_fill_kernel, dim3(n_tiles), dim3(DT_THREADS), 0, s, T, M, ld, rows, B, N, bk_ptr,
                     bk_rc, bk_t, bk_m);
  OCF_HIP(hipGetLastError());
  OCF_TRY_END
}

extern "C" int ocf_pack_input(const float* s0, const float* s1, const float* s2, int64_t ld_src, int B, int N, void* xin,
                              int dtype, int64_t xin_ld, int64_t xin_block, int B_pad, const int64_t* rows, void* stream) {
  OCF_TRY_BEGIN
  OCF_CHECK(xin && s0, "ocf_pack_input: null pointer");
  int64_t tot = (int64_t)B_pad * xin_ld;
  if (tot == 0) return 0;
  hipLaunchKernelGGL(pack_input_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, (hipStream_t)stream, s0, s1, s2,
                     ld_src, B, N, xin, dtype, xin_ld, xin_block, B_pad, rows);
  OCF_HIP(hipGetLastError());
  OCF_TRY_END
}
