// Row-list weight-gradient + optimizer kernel (EPI_OPTIM over a sparse batch operand), gfx950.
//
// The weight gradient of a first/last layer on a sparse batch is dW[m][:] = sum over the batch entries
// (v, k) of column m of v * B[k][:] (B = the hidden activations h or deltas dh, [K][N]); v is the
// live input (dW_in) or the output delta (dW_out).  At ML-20M a batch holds 0.5 % of the [K][M]
// operand, so the MFMA form (optim_ws_kernel) spends its matrix-core and LDS work on zeros; here the
// entries come as row lists (ocf_sparse_tiles row_ptr / row_ent: column m's entries in batch-row
// order) and one wave owns one weight row at a time:
//   lane l holds columns [l*CPL, l*CPL + CPL) of the row (CPL = N / 64), so every load / store of
//   the row is one contiguous N*4-byte (or N*2-byte shadow) wave access;
//   g = sum over the row's entries, in k order, of v * B[k][cols] (fp32 FMA, v and B as stored:
//   fp32 values, compute-dtype B), then the optimizer update of p / slots, the shadow write, and for
//   the output layer the column sum of v (the output-bias gradient) and its update.
// One wave per task of RW_BLOCK consecutive rows (ballot over the row lengths); with Adagrad and
// l2 == 0 rows without entries are skipped (zero gradient: identity update), otherwise every row is
// updated (g = 0).  A row's parameter / slot loads are issued with its entry list, so the row costs
// about two memory latencies; the many resident waves (small register footprint) keep HBM busy.
#pragma once
#include "ocf_epilogues.h"
#include "ocf_optim_ws.h"

namespace ocf {

constexpr int RW_THREADS = 256;

struct RowsDwArgs {
  float* p; float* s1; float* s2;
  int64_t ld;                 // parameter row stride (floats) = N
  int M, N;
  const void* B; int64_t ldb; // [K][ldb] compute dtype (or fp32)
  const int32_t* rowptr; const int2* rowent; const float* vals;
  OcfOptParams op;
  void* shadow; int shadow_dtype; bool shadow_blocked;
  float* colsum; float colsum_scale;
  int skip_empty;
};

constexpr int RW_BLOCK = 16;     // rows per wave task (one wave per task)
constexpr int RW_EB = 8;         // entries whose B rows are loaded together

// one weight row in flight: its parameters / slots (this lane's columns), entry range, the entry of
// this lane (< 64), and the first RW_EB entries' values and B pieces
template <typename BT, int CPL, int NS> struct RwRow {
  float p[CPL], a[CPL], b[NS == 2 ? CPL : 1];
  int m, lo, n;
  int2 en;
  float ve;
  BT bv[RW_EB][CPL];
  float vv[RW_EB];
};

template <typename BT, int KIND, int CPL>
__global__ void __launch_bounds__(RW_THREADS) optim_rows_kernel(RowsDwArgs ra, WsJobs jobs) {
  constexpr int NS = KIND == OCF_OPT_ADAM ? 2 : 1;
  static_assert(CPL % 2 == 0, "columns per lane");
  using Row = RwRow<BT, CPL, NS>;
  const int lane = threadIdx.x & 63;
  const int wave = blockIdx.x * (RW_THREADS / 64) + (threadIdx.x >> 6);
  const int nwaves = gridDim.x * (RW_THREADS / 64);
  {  // folded small jobs (bias updates, stats): one per wave
    const int nj = jobs.count();
    for (int j = wave; j < nj; j += nwaves) jobs.run<KIND>(j, lane);
  }
  const int r0 = wave * RW_BLOCK;
  if (r0 >= ra.M) return;
  const int c0 = lane * CPL;
  const BT* Bg = reinterpret_cast<const BT*>(ra.B);
  const __amdgpu_buffer_rsrc_t rp = wt_rsrc(ra.p), r1 = wt_rsrc(ra.s1), r2 = wt_rsrc(ra.s2);

  // 16-B buffer loads / stores with the optimizer streams' cache policy (CPL % 4 == 0), else 8-B
  auto ldv = [&](__amdgpu_buffer_rsrc_t r, const float* base, uint32_t ob, float* dst) {
    if constexpr (CPL % 4 == 0) {
#pragma unroll
      for (int c = 0; c < CPL; c += 4) {
        const float4 x = ld_pol16<OCF_OPT_LD_POL>(r, base, ob + c * 4);
        dst[c] = x.x; dst[c + 1] = x.y; dst[c + 2] = x.z; dst[c + 3] = x.w;
      }
    } else {
#pragma unroll
      for (int c = 0; c < CPL; c += 2) {
        const float2 x = *reinterpret_cast<const float2*>(reinterpret_cast<const char*>(base) + ob + c * 4);
        dst[c] = x.x; dst[c + 1] = x.y;
      }
    }
  };
  auto stv = [&](__amdgpu_buffer_rsrc_t r, float* base, uint32_t ob, const float* src) {
    if constexpr (CPL % 4 == 0) {
#pragma unroll
      for (int c = 0; c < CPL; c += 4)
        st_pol16<OCF_OPT_ST_POL>(r, base, ob + c * 4, make_float4(src[c], src[c + 1], src[c + 2], src[c + 3]));
    } else {
#pragma unroll
      for (int c = 0; c < CPL; c += 2)
        *reinterpret_cast<float2*>(reinterpret_cast<char*>(base) + ob + c * 4) = make_float2(src[c], src[c + 1]);
    }
  };
  auto off = [&](int m) { return (uint32_t)(((int64_t)m * ra.ld + c0) * 4); };   // < 2 GiB: host check
  // stage 1: parameters, slots and the entry list of a row (HBM)
  auto stage1 = [&](Row& r, int m, int lo, int n) {
    r.m = m; r.lo = lo; r.n = n;
    const uint32_t ob = off(m);
    ldv(rp, ra.p, ob, r.p);
    ldv(r1, ra.s1, ob, r.a);
    if constexpr (NS == 2) ldv(r2, ra.s2, ob, r.b);
    r.en = lane < n ? ra.rowent[lo + lane] : make_int2(0, 0);
  };
  // stage 2a: the values and B pieces of the row's first RW_EB entries (L2)
  auto load_ents = [&](Row& r, int e0) {
#pragma unroll
    for (int u = 0; u < RW_EB; ++u) {
      const int e = e0 + u;
      r.vv[u] = 0.f;
      if (e < r.n) {
        int k;
        if (e < 64) {
          k = __builtin_amdgcn_readlane(r.en.y, e);
          r.vv[u] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, r.ve), e));
        } else {
          const int2 x = ra.rowent[r.lo + e];
          k = x.y;
          r.vv[u] = ra.vals[x.x];
        }
        __builtin_memcpy(r.bv[u], Bg + (int64_t)k * ra.ldb + c0, sizeof(r.bv[u]));
      }
    }
  };
  auto stage2a = [&](Row& r) {
    r.ve = lane < r.n ? ra.vals[r.en.x] : 0.f;
    load_ents(r, 0);
  };
  // stage 2b: g = sum over the entries, in k order, of v * B[k][cols]; the update; the stores
  auto stage2b = [&](Row& r) {
    float g[CPL];
#pragma unroll
    for (int c = 0; c < CPL; ++c) g[c] = 0.f;
    float cs = 0.f;
    for (int e0 = 0; e0 < r.n; e0 += RW_EB) {
      if (e0 > 0) load_ents(r, e0);   // rows with more than RW_EB entries
#pragma unroll
      for (int u = 0; u < RW_EB; ++u) {
        if (e0 + u < r.n) {
#pragma unroll
          for (int c = 0; c < CPL; ++c) g[c] += r.vv[u] * (float)r.bv[u][c];
          cs += r.vv[u];
        }
      }
    }
    const OcfOptParams o = ra.op;
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      float bb = 0.f;
      if constexpr (NS == 2) bb = r.b[c];
      opt_update_k<KIND>(o, g[c] * o.gscale, r.p[c], r.a[c], bb);
      if constexpr (NS == 2) r.b[c] = bb;
    }
    const uint32_t ob = off(r.m);
    stv(rp, ra.p, ob, r.p);
    stv(r1, ra.s1, ob, r.a);
    if constexpr (NS == 2) stv(r2, ra.s2, ob, r.b);
    if (ra.shadow) {
      if (ra.shadow_blocked) {   // 64x64 blocks (CPL % 4 == 0, checked on the host)
        EpiOptim::Params sh{};
        sh.ld = ra.ld; sh.shadow = ra.shadow; sh.shadow_dtype = ra.shadow_dtype; sh.shadow_blocked = true;
#pragma unroll
        for (int c = 0; c + 3 < CPL; c += 4)
          EpiOptim::store_shadow(sh, r.m, c0 + c, make_float4(r.p[c], r.p[c + 1], r.p[c + 2], r.p[c + 3]));
      } else {
        char* dst = reinterpret_cast<char*>(ra.shadow) + ((int64_t)r.m * ra.ld + c0) * 2;
        uint16_t hv[CPL];
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
          if (ra.shadow_dtype == OCF_F16) {
            const _Float16 x = (_Float16)r.p[c];
            __builtin_memcpy(&hv[c], &x, 2);
          } else {
            const __bf16 x = (__bf16)r.p[c];
            __builtin_memcpy(&hv[c], &x, 2);
          }
        }
        __builtin_memcpy(dst, hv, sizeof(hv));
      }
    }
    if (ra.colsum && lane == 0) {   // output-bias gradient (column sum of the entries, k order) + update
      const float v = cs * ra.colsum_scale;
      ra.colsum[r.m] = v;
      if (jobs.cb_p) jobs.colsum_bias<KIND>(r.m, v, jobs.colsum_pre(r.m));
    }
  };

  // the task's row lengths (lanes < RW_BLOCK), then its rows through a two-row pipeline: the next
  // row's HBM loads are issued after the current row's L2 loads and before the current row waits
  int lo = 0, n = 0;
  if (lane < RW_BLOCK && r0 + lane < ra.M) {
    lo = ra.rowptr[r0 + lane];
    n = ra.rowptr[r0 + lane + 1] - lo;
    if (ra.colsum && n == 0 && ra.skip_empty) ra.colsum[r0 + lane] = 0.f;   // skipped rows: zero column sum
  }
  uint64_t todo = __ballot(lane < RW_BLOCK && r0 + lane < ra.M && (n > 0 || !ra.skip_empty));
  if (!todo) return;
  Row cur, nxt;
  {
    const int l = __builtin_ctzll(todo);
    todo &= todo - 1;
    stage1(cur, r0 + l, __builtin_amdgcn_readlane(lo, l), __builtin_amdgcn_readlane(n, l));
  }
  while (true) {
    stage2a(cur);
    const bool more = todo != 0;
    if (more) {
      const int l = __builtin_ctzll(todo);
      todo &= todo - 1;
      stage1(nxt, r0 + l, __builtin_amdgcn_readlane(lo, l), __builtin_amdgcn_readlane(n, l));
    }
    stage2b(cur);
    if (!more) break;
    cur = nxt;
  }
}

}  // namespace ocf
