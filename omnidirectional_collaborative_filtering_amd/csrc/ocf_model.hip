// Model-level C ABI (include/ocf.h "Model ABI"): SURVEY §8(b)'s ocf_ctx_create / ocf_forward /
// ocf_masked_mse / ocf_backward, with the existing ocf_opt_step as the update.  One omni_model
// (/root/reference/model.py:43-99) over caller-owned fp32 parameters in the padded Keras layout, dense
// batches in the reference's data_gen format (data_reader.py:354-361 input list, [B][N] fp32 arrays), the
// Keras MSE of train.py:49 and raw weight gradients -- what a binding that drives its own training loop
// needs, in five calls per step, without the engine's argument blocks.
//
// Every product runs on the library's MFMA kernels (ocf_gemm) with the epilogues the engine's dense path
// uses (split-K + ocf_splitk_bias_act / ocf_splitk_grad_act for few-tile layers, EPI_BIAS_ACT /
// EPI_GRAD_ACT otherwise, EPI_PREDICT, EPI_GRAD), so results agree with Engine's dense path run with raw
// gradients (parallel.DataParallel's step) up to the summation order of the bias sums.  The weights are
// read in fp32 by the GEMMs (staged to the compute dtype per tile), so a caller's elementwise update
// (ocf_opt_step) needs no shadow refresh.  The context owns only the per-batch activations, dropout masks
// and split-K slabs (allocated once, at create: nothing is allocated or synchronised per call).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "ocf_internal.h"

namespace ocf {

constexpr int MT = 128;   // GEMM tile: every padded dimension is a multiple of it
static int64_t ru(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

struct ModelCtx {
  OcfModelDesc d;
  int L;                     // hidden layers
  int cdt;
  int64_t Np, Bp, pad0;
  std::vector<int64_t> Hp;   // padded hidden widths
  std::vector<int> H;
  float keep;
  int splits0, splitsL;
  std::vector<int> splits_fwd, splits_bwd;
  // workspace
  void* xin = nullptr;                // [Bp][pad0] compute dtype
  std::vector<float*> a;              // [Bp][Hp] fp32 pre-dropout activations
  std::vector<void*> h, dh;           // [Bp][Hp] compute dtype
  std::vector<uint8_t*> mask;         // [Bp][Hp] dropout keep flags (keep < 1)
  std::vector<float*> db;             // [Bp/4][Hp] hidden-bias gradient partials
  void* d_out = nullptr;              // [Bp][Np] compute dtype output delta
  float* slabs = nullptr;
  std::vector<void*> allocs;
  int last_B = 0;                     // batch rows of the last forward (backward checks it)
  float last_keep = 1.f;              // its dropout keep probability (1 outside training)

  int bk() const { return cdt == OCF_F32 ? 32 : 64; }
  int pick_hidden(int64_t K, int64_t N) const {   // engine.Engine._pick_splits_hidden
    const int64_t tiles = (Bp / MT) * (N / MT);
    if (tiles >= 16) return 1;
    const int64_t ks = K / bk();
    int64_t s = std::max<int64_t>(1, std::min<int64_t>(ks, 64 / tiles));
    while (ks % s) --s;
    return (int)s;
  }
  int pick(int64_t K, int64_t N) const {          // engine.Engine._pick_splits
    const int64_t ks = K / bk(), tiles = (Bp / MT) * (N / MT);
    if (ks < 64 && tiles < 16) return pick_hidden(K, N);
    return (int)std::max<int64_t>(1, std::min<int64_t>(ks / 8, std::max<int64_t>(1, 512 / tiles)));
  }
  void* alloc(size_t bytes) {
    void* p = nullptr;
    OCF_HIP(hipMalloc(&p, bytes));
    OCF_HIP(hipMemset(p, 0, bytes));
    allocs.push_back(p);
    return p;
  }
  ~ModelCtx() {
    for (void* p : allocs) (void)hipFree(p);
  }
};

static size_t dt_size(int dt) { return dt == OCF_F32 ? 4 : 2; }

// padded shapes of W[i] (rows x cols) in the Keras (in, out) layout: in = k N_pad for layer 0, hidden
// widths padded to 128, out = N_pad for the output layer
static void model_dims(const OcfModelDesc& d, std::vector<int64_t>& rows, std::vector<int64_t>& cols) {
  const int64_t Np = ru(d.N, MT);
  std::vector<int64_t> dims{(int64_t)d.k_blocks * Np};
  for (int i = 0; i < d.n_hidden; ++i) dims.push_back(ru(d.hidden[i], MT));
  dims.push_back(Np);
  rows.assign(dims.begin(), dims.end() - 1);
  cols.assign(dims.begin() + 1, dims.end());
}

static void check_desc(const OcfModelDesc* d) {
  OCF_CHECK(d != nullptr, "ocf model: null descriptor");
  OCF_CHECK(d->n_hidden >= 1 && d->n_hidden <= OCF_MAX_HIDDEN, "ocf model: n_hidden must be 1..8");
  OCF_CHECK(d->N >= 1 && d->k_blocks >= 1 && d->k_blocks <= 3, "ocf model: N >= 1, k_blocks 1..3");
  for (int i = 0; i < d->n_hidden; ++i) OCF_CHECK(d->hidden[i] >= 1, "ocf model: hidden widths >= 1");
  OCF_CHECK(d->act >= OCF_ACT_LINEAR && d->act <= OCF_ACT_RELU, "ocf model: activation");
  OCF_CHECK(d->dropout >= 0.f && d->dropout < 1.f, "ocf model: dropout in [0, 1)");
  OCF_CHECK(d->compute_dtype == OCF_F32 || d->compute_dtype == OCF_F16 || d->compute_dtype == OCF_BF16,
            "ocf model: compute_dtype");
  OCF_CHECK(d->max_batch >= 1 && d->max_batch <= 65536, "ocf model: max_batch 1..65536");
}

static OcfGemmArgs gemm_base(const ModelCtx& c) {
  OcfGemmArgs g{};
  g.compute_dtype = c.cdt;
  g.a_dtype = c.cdt;
  g.splits = 1;
  g.keep = 1.f;
  return g;
}

static void gemm(const OcfGemmArgs& g, hipStream_t s) {
  OCF_CHECK(ocf_gemm(&g, s) == 0, ocf_last_error());
}

}  // namespace ocf

using namespace ocf;

extern "C" int ocf_model_dims(const OcfModelDesc* desc, int64_t* rows, int64_t* cols) {
  OCF_TRY_BEGIN
  check_desc(desc);
  OCF_CHECK(rows && cols, "ocf_model_dims: null output");
  std::vector<int64_t> r, c;
  model_dims(*desc, r, c);
  for (size_t i = 0; i < r.size(); ++i) {
    rows[i] = r[i];
    cols[i] = c[i];
  }
  OCF_TRY_END
}

extern "C" int ocf_ctx_create(const OcfModelDesc* desc, OcfCtx** out) {
  OCF_TRY_BEGIN
  check_desc(desc);
  OCF_CHECK(out != nullptr, "ocf_ctx_create: null output");
  *out = nullptr;
  const int L = desc->n_hidden;
  for (int i = 0; i <= L; ++i) OCF_CHECK(desc->W[i] && desc->b[i], "ocf_ctx_create: null parameter pointer");
  auto* c = new ModelCtx();
  try {
    c->d = *desc;
    c->L = L;
    c->cdt = desc->compute_dtype;
    c->Np = ru(desc->N, MT);
    c->Bp = ru(desc->max_batch, MT);
    c->pad0 = (int64_t)desc->k_blocks * c->Np;
    c->keep = 1.f - desc->dropout;
    for (int i = 0; i < L; ++i) {
      c->H.push_back(desc->hidden[i]);
      c->Hp.push_back(ru(desc->hidden[i], MT));
    }
    const int64_t Bp = c->Bp, HpL = c->Hp[L - 1];
    c->splits0 = c->pick(c->pad0, c->Hp[0]);
    c->splitsL = c->pick(c->Np, HpL);
    c->splits_fwd.assign(L, 1);
    c->splits_bwd.assign(L, 1);
    int64_t smax = std::max(c->splits0 * c->Hp[0], c->splitsL * HpL);
    for (int i = 1; i < L; ++i) {
      c->splits_fwd[i] = c->pick_hidden(c->Hp[i - 1], c->Hp[i]);
      c->splits_bwd[i] = c->pick_hidden(c->Hp[i], c->Hp[i - 1]);
      smax = std::max({smax, c->splits_fwd[i] * c->Hp[i], c->splits_bwd[i] * c->Hp[i - 1]});
    }
    const size_t cs = dt_size(c->cdt);
    c->xin = c->alloc(Bp * c->pad0 * cs);
    for (int i = 0; i < L; ++i) {
      c->a.push_back((float*)c->alloc(Bp * c->Hp[i] * 4));
      c->h.push_back(c->alloc(Bp * c->Hp[i] * cs));
      c->dh.push_back(c->alloc(Bp * c->Hp[i] * cs));
      c->mask.push_back(c->keep < 1.f ? (uint8_t*)c->alloc(Bp * c->Hp[i]) : nullptr);
      c->db.push_back((float*)c->alloc(Bp / 4 * c->Hp[i] * 4));
    }
    c->d_out = c->alloc(Bp * c->Np * cs);
    c->slabs = (float*)c->alloc(smax * Bp * 4);
  } catch (...) {
    delete c;
    throw;
  }
  *out = reinterpret_cast<OcfCtx*>(c);
  OCF_TRY_END
}

extern "C" int ocf_ctx_destroy(OcfCtx* ctx) {
  OCF_TRY_BEGIN
  delete reinterpret_cast<ModelCtx*>(ctx);
  OCF_TRY_END
}

// model.py:43-99: concatenate(inputs) -> L x (Dense + act + Dropout) -> Dense -> * output mask
extern "C" int ocf_forward(OcfCtx* ctx, const float* const* inputs, int64_t ld_in, int B, int training,
                           uint64_t step, const float* out_mask, int64_t ld_mask, float* pred, int64_t ld_pred,
                           uint8_t* const* masks_out, void* stream) {
  OCF_TRY_BEGIN
  auto* c = reinterpret_cast<ModelCtx*>(ctx);
  OCF_CHECK(c && inputs && pred, "ocf_forward: null pointer");
  OCF_CHECK(B >= 1 && B <= c->d.max_batch, "ocf_forward: B must be 1..max_batch");
  OCF_CHECK(ld_in >= c->d.N && ld_pred >= c->d.N && (!out_mask || ld_mask >= c->d.N), "ocf_forward: row strides");
  for (int i = 0; i < c->d.k_blocks; ++i) OCF_CHECK(inputs[i] != nullptr, "ocf_forward: null input block");
  hipStream_t s = (hipStream_t)stream;
  const int L = c->L;
  const int64_t Bp = c->Bp;
  const float keep = training ? c->keep : 1.f;
  const uint64_t sid = training ? step * 16 : 0;     // Engine.forward's Philox stream of the step's masks
  const float* in2 = c->d.k_blocks > 1 ? inputs[1] : nullptr;
  const float* in3 = c->d.k_blocks > 2 ? inputs[2] : nullptr;
  OCF_CHECK(ocf_pack_input(inputs[0], in2, in3, ld_in, B, c->d.N, c->xin, c->cdt, c->pad0, c->Np, (int)Bp, nullptr,
                           stream) == 0, ocf_last_error());
  // layer 0: split-K over the (k x N_pad)-wide input, the epilogue in the slab reduction
  {
    const int64_t Hp0 = c->Hp[0];
    OcfGemmArgs g = gemm_base(*c);
    g.A = c->xin; g.a_col = 0; g.lda = c->pad0;
    g.B = c->d.W[0]; g.b_dtype = OCF_F32; g.b_col = 1; g.ldb = Hp0;
    g.M = (int)Bp; g.N = (int)Hp0; g.K = (int)c->pad0;
    g.epi = OCF_EPI_SLAB; g.splits = c->splits0; g.out = c->slabs; g.ld_out = Hp0; g.split_stride = Bp * Hp0;
    gemm(g, s);
    OCF_CHECK(ocf_splitk_bias_act(c->slabs, c->splits0, Bp * Hp0, (int)Bp, (int)Hp0, Hp0, c->d.b[0], c->d.act, keep,
                                  c->d.seed, sid, nullptr, keep < 1.f ? c->mask[0] : nullptr, c->a[0], c->h[0], c->cdt,
                                  B, c->H[0], stream) == 0, ocf_last_error());
  }
  for (int i = 1; i < L; ++i) {
    const int64_t K = c->Hp[i - 1], N = c->Hp[i];
    OcfGemmArgs g = gemm_base(*c);
    g.A = c->h[i - 1]; g.a_col = 0; g.lda = K;
    g.B = c->d.W[i]; g.b_dtype = OCF_F32; g.b_col = 1; g.ldb = N;
    g.M = (int)Bp; g.N = (int)N; g.K = (int)K;
    if (c->splits_fwd[i] > 1) {
      g.epi = OCF_EPI_SLAB; g.splits = c->splits_fwd[i]; g.out = c->slabs; g.ld_out = N; g.split_stride = Bp * N;
      gemm(g, s);
      OCF_CHECK(ocf_splitk_bias_act(c->slabs, c->splits_fwd[i], Bp * N, (int)Bp, (int)N, N, c->d.b[i], c->d.act, keep,
                                    c->d.seed, sid + i, nullptr, keep < 1.f ? c->mask[i] : nullptr, c->a[i], c->h[i],
                                    c->cdt, B, c->H[i], stream) == 0, ocf_last_error());
      continue;
    }
    g.epi = OCF_EPI_BIAS_ACT; g.bias = c->d.b[i]; g.act = c->d.act; g.keep = keep; g.seed = c->d.seed;
    g.stream = sid + i; g.mask_out = keep < 1.f ? c->mask[i] : nullptr; g.a_out = c->a[i]; g.h_out = c->h[i];
    g.h_dtype = c->cdt; g.ld_out = N; g.m_real = B; g.n_real = c->H[i];
    gemm(g, s);
  }
  // output layer: pred = out_mask * (h W + b)   (model.py:81-86)
  {
    const int64_t HpL = c->Hp[L - 1];
    OcfGemmArgs g = gemm_base(*c);
    g.A = c->h[L - 1]; g.a_col = 0; g.lda = HpL;
    g.B = c->d.W[L]; g.b_dtype = OCF_F32; g.b_col = 1; g.ldb = c->Np;
    g.M = (int)Bp; g.N = (int)c->Np; g.K = (int)HpL;
    g.epi = OCF_EPI_PREDICT; g.bias = c->d.b[L]; g.pmask = out_mask; g.ld_pmask = out_mask ? ld_mask : 0;
    g.out = pred; g.ld_out = ld_pred; g.m_real = B; g.n_real = c->d.N;
    gemm(g, s);
  }
  if (masks_out && keep < 1.f)
    for (int i = 0; i < L; ++i)
      if (masks_out[i])
        OCF_HIP(hipMemcpy2DAsync(masks_out[i], c->H[i], c->mask[i], c->Hp[i], c->H[i], B, hipMemcpyDeviceToDevice, s));
  c->last_B = B;
  c->last_keep = keep;
  OCF_TRY_END
}

namespace ocf {

// per batch row: residual, its masked form, and the row's SSE / SAE / count_nonzero(T + yhat)
__global__ void __launch_bounds__(256) mse_rows_kernel(const float* pred, const float* T, const float* M, int64_t ld,
                                                       int N, float* grad, int64_t ld_g, float* row_stats, int B) {
  __shared__ float red[3][256];
  const int b = blockIdx.x;
  float sse = 0.f, sae = 0.f, cnt = 0.f;
  for (int n = threadIdx.x; n < N; n += 256) {
    const int64_t o = (int64_t)b * ld + n;
    const float y = pred[o], t = T[o];
    const float e = y - t;
    sse += e * e;
    sae += fabsf(e);
    cnt += (t + y != 0.f) ? 1.f : 0.f;
    if (grad) grad[(int64_t)b * ld_g + n] = M ? e * M[o] : e;
  }
  red[0][threadIdx.x] = sse;
  red[1][threadIdx.x] = sae;
  red[2][threadIdx.x] = cnt;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w)
      for (int k = 0; k < 3; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x < 3) row_stats[(int64_t)threadIdx.x * B + b] = red[threadIdx.x][0];
}

// totals over the rows in a fixed order: {sse, sae, count, loss = sse / (B N)}
__global__ void __launch_bounds__(256) mse_total_kernel(float* stats, int B, int N) {
  __shared__ double red[3][256];
  const float* rows = stats + 4;
  double v[3] = {0.0, 0.0, 0.0};
  for (int b = threadIdx.x; b < B; b += 256)
    for (int k = 0; k < 3; ++k) v[k] += (double)rows[(int64_t)k * B + b];
  for (int k = 0; k < 3; ++k) red[k][threadIdx.x] = v[k];
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w)
      for (int k = 0; k < 3; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    stats[0] = (float)red[0][0];
    stats[1] = (float)red[1][0];
    stats[2] = (float)red[2][0];
    stats[3] = (float)(red[0][0] / ((double)B * (double)N));
  }
}

// the output delta in the compute dtype, zero-padded to [Bp][Np]
__global__ void __launch_bounds__(256) delta_pack_kernel(const float* g, int64_t ld, int B, int N, void* d, int dt,
                                                         int64_t Np, int64_t Bp) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= Bp * Np) return;
  const int64_t b = i / Np, n = i % Np;
  const float v = (b < B && n < N) ? g[b * ld + n] : 0.f;
  if (dt == OCF_F32) reinterpret_cast<float*>(d)[i] = v;
  else if (dt == OCF_F16) reinterpret_cast<_Float16*>(d)[i] = (_Float16)v;
  else reinterpret_cast<__bf16*>(d)[i] = (__bf16)v;
}

}  // namespace ocf

// train.py:49 (Keras mean_squared_error on the masked prediction) and train.py:102-121's per-row sums
extern "C" int ocf_masked_mse(const float* pred, const float* T, const float* out_mask, int64_t ld, int B, int N,
                              float* out_grad, int64_t ld_grad, float* out_stats, void* stream) {
  OCF_TRY_BEGIN
  OCF_CHECK(pred && T && out_stats, "ocf_masked_mse: null pointer");
  OCF_CHECK(B >= 1 && N >= 1 && ld >= N && (!out_grad || ld_grad >= N), "ocf_masked_mse: sizes");
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(mse_rows_kernel, dim3(B), dim3(256), 0, s, pred, T, out_mask, ld, N, out_grad, ld_grad,
                     out_stats + 4, B);
  hipLaunchKernelGGL(mse_total_kernel, dim3(1), dim3(256), 0, s, out_stats, B, N);
  OCF_HIP(hipGetLastError());
  OCF_TRY_END
}

// the backward pass of the last ocf_forward (training or not) from the unscaled output gradient
extern "C" int ocf_backward(OcfCtx* ctx, const float* grad, int64_t ld_grad, int B, float gscale, float* const* gW,
                            float* const* gb, void* stream) {
  OCF_TRY_BEGIN
  auto* c = reinterpret_cast<ModelCtx*>(ctx);
  OCF_CHECK(c && grad && gW && gb, "ocf_backward: null pointer");
  OCF_CHECK(B == c->last_B, "ocf_backward: B differs from the last ocf_forward");
  OCF_CHECK(ld_grad >= c->d.N, "ocf_backward: ld_grad");
  const int L = c->L;
  for (int i = 0; i <= L; ++i) OCF_CHECK(gW[i] && gb[i], "ocf_backward: null gradient pointer");
  hipStream_t s = (hipStream_t)stream;
  const int64_t Bp = c->Bp, Np = c->Np, HpL = c->Hp[L - 1];
  const float keep = c->last_keep;
  hipLaunchKernelGGL(delta_pack_kernel, dim3((unsigned)((Bp * Np + 255) / 256)), dim3(256), 0, s, grad, ld_grad, B,
                     c->d.N, c->d_out, c->cdt, Np, Bp);
  OCF_HIP(hipGetLastError());
  // output bias: gscale * column sums of the delta (pad columns zero)
  OCF_HIP(hipMemsetAsync(gb[L], 0, Np * 4, s));
  OCF_CHECK(ocf_colsum(grad, OCF_F32, ld_grad, B, c->d.N, gscale, gb[L], stream) == 0, ocf_last_error());
  // output weights: gW[L] = gscale * h^T delta
  {
    OcfGemmArgs g = gemm_base(*c);
    g.A = c->h[L - 1]; g.a_col = 1; g.lda = HpL;
    g.B = c->d_out; g.b_dtype = c->cdt; g.b_col = 1; g.ldb = Np;
    g.M = (int)HpL; g.N = (int)Np; g.K = (int)Bp;
    g.epi = OCF_EPI_GRAD; g.out = gW[L]; g.ld_out = Np; g.h_dtype = OCF_F32;
    g.opt.gscale = gscale;
    gemm(g, s);
  }
  // last hidden delta: split-K (delta W_L^T), then act' * dropout and the bias partials
  {
    OcfGemmArgs g = gemm_base(*c);
    g.A = c->d_out; g.a_col = 0; g.lda = Np;
    g.B = c->d.W[L]; g.b_dtype = OCF_F32; g.b_col = 0; g.ldb = Np;
    g.M = (int)Bp; g.N = (int)HpL; g.K = (int)Np;
    g.epi = OCF_EPI_SLAB; g.splits = c->splitsL; g.out = c->slabs; g.ld_out = HpL; g.split_stride = Bp * HpL;
    gemm(g, s);
    OCF_CHECK(ocf_splitk_grad_act(c->slabs, c->splitsL, Bp * HpL, (int)Bp, (int)HpL, HpL, c->a[L - 1], keep < 1.f ? c->mask[L - 1] : nullptr,
                                  keep, c->d.act, c->dh[L - 1], c->cdt, c->db[L - 1], gscale, B, c->H[L - 1], stream) == 0,
              ocf_last_error());
  }
  int64_t parts_last = Bp / 4;
  for (int i = L - 1; i >= 1; --i) {
    // dh[i-1] = (dh[i] W_i^T) * act'(a[i-1]) * dropout; bias partials db[i-1]
    const int64_t Ko = c->Hp[i], No = c->Hp[i - 1];
    int64_t parts_next;
    OcfGemmArgs g = gemm_base(*c);
    g.A = c->dh[i]; g.a_col = 0; g.lda = Ko;
    g.B = c->d.W[i]; g.b_dtype = OCF_F32; g.b_col = 0; g.ldb = Ko;   // W_i [No][Ko] = B^T
    g.M = (int)Bp; g.N = (int)No; g.K = (int)Ko;
    if (c->splits_bwd[i] > 1) {
      g.epi = OCF_EPI_SLAB; g.splits = c->splits_bwd[i]; g.out = c->slabs; g.ld_out = No; g.split_stride = Bp * No;
      gemm(g, s);
      OCF_CHECK(ocf_splitk_grad_act(c->slabs, c->splits_bwd[i], Bp * No, (int)Bp, (int)No, No, c->a[i - 1],
                                    keep < 1.f ? c->mask[i - 1] : nullptr, keep, c->d.act, c->dh[i - 1], c->cdt, c->db[i - 1], gscale, B,
                                    c->H[i - 1], stream) == 0, ocf_last_error());
      parts_next = Bp / 4;
    } else {
      g.epi = OCF_EPI_GRAD_ACT; g.a_in = c->a[i - 1]; g.mask_in = keep < 1.f ? c->mask[i - 1] : nullptr; g.keep = keep; g.act = c->d.act;
      g.h_out = c->dh[i - 1]; g.h_dtype = c->cdt; g.ld_out = No; g.db_part = c->db[i - 1]; g.opt.gscale = gscale;
      g.m_real = B; g.n_real = c->H[i - 1];
      gemm(g, s);
      parts_next = Bp / MT;
    }
    // layer i's bias and weights
    OCF_CHECK(ocf_colsum(c->db[i], OCF_F32, c->Hp[i], (int)parts_last, (int)c->Hp[i], 1.f, gb[i], stream) == 0,
              ocf_last_error());
    OcfGemmArgs w = gemm_base(*c);
    w.A = c->h[i - 1]; w.a_col = 1; w.lda = No;
    w.B = c->dh[i]; w.b_dtype = c->cdt; w.b_col = 1; w.ldb = Ko;
    w.M = (int)No; w.N = (int)Ko; w.K = (int)Bp;
    w.epi = OCF_EPI_GRAD; w.out = gW[i]; w.ld_out = Ko; w.h_dtype = OCF_F32; w.opt.gscale = gscale;
    gemm(w, s);
    parts_last = parts_next;
  }
  OCF_CHECK(ocf_colsum(c->db[0], OCF_F32, c->Hp[0], (int)parts_last, (int)c->Hp[0], 1.f, gb[0], stream) == 0,
            ocf_last_error());
  {
    const int64_t Hp0 = c->Hp[0];
    OcfGemmArgs w = gemm_base(*c);
    w.A = c->xin; w.a_col = 1; w.lda = c->pad0;
    w.B = c->dh[0]; w.b_dtype = c->cdt; w.b_col = 1; w.ldb = Hp0;
    w.M = (int)c->pad0; w.N = (int)Hp0; w.K = (int)Bp;
    w.epi = OCF_EPI_GRAD; w.out = gW[0]; w.ld_out = Hp0; w.h_dtype = OCF_F32; w.opt.gscale = gscale;
    gemm(w, s);
  }
  OCF_TRY_END
}
