/*
 * libocf -- MI355X (gfx950) kernels for the autoencoder-CF training hot path.
 *
 * C ABI only: plain pointers, sizes and POD structs; no framework types.  Every function returns
 * 0 on success and a non-zero code on failure; ocf_last_error() gives the message (thread-local).
 * All device pointers are caller-owned (e.g. PyTorch-ROCm tensors passed by data_ptr()); the
 * library never allocates or synchronises per call.  Work is enqueued on the caller's
 * hipStream_t (passed as void*), so every entry point is graph-capturable.
 *
 * The reference (Epist/omnidirectional_collaborative_filtering, Python 2.7 + TF 1.3 / Keras 2.0.4)
 * has no FFI of its own: its hot path is the Python pair data_reader / omni_model driven by
 * train.py.  Each entry point below names the reference code it replaces; INTEGRATION.md shows
 * the ctypes binding a maintainer would add on the reference side.
 */
#ifndef OCF_H_
#define OCF_H_
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* element types */
#define OCF_DT_F32 0
#define OCF_DT_F16 1
#define OCF_DT_BF16 2

/* activations (model.py:34 default 'tanh'; train.py:52 'sigmoid') */
#define OCF_ACTV_LINEAR 0
#define OCF_ACTV_SIGMOID 1
#define OCF_ACTV_TANH 2
#define OCF_ACTV_RELU 3

/* optimizers (train.py:50-51 Adagrad; train_jester.py:61 'rmsprop'; north_star Adam) */
#define OCF_OPTK_SGD 0
#define OCF_OPTK_ADAGRAD 1
#define OCF_OPTK_RMSPROP 2
#define OCF_OPTK_ADAM 3

/* GEMM epilogues (ocf_gemm) */
#define OCF_EPI_SLAB 0       /* split-K fp32 partial slabs                                   */
#define OCF_EPI_BIAS_ACT 1   /* + bias, activation, dropout  (model.py:64-73)                */
#define OCF_EPI_GRAD_ACT 2   /* * dropout mask * act'(a), bias-grad column partials          */
#define OCF_EPI_GRAD 3       /* raw weight gradient (data-parallel path)                     */
#define OCF_EPI_OPTIM 4      /* fused optimizer update of the weight tile (train.py:50-51)  */
#define OCF_EPI_PREDICT 5    /* y = mask * (acc + b)   (model.py:82-86)                       */
#define OCF_EPI_MASKED_MSE 6 /* masked MSE loss/grad on bucketed targets (train.py:49)       */

/* Keras 2.0.4 optimizer scalars for one step (host computes lr incl. decay / Adam lr_t). */
typedef struct OcfOptParams {
  int kind;
  float lr, eps, rho, beta2, l2, gscale;
} OcfOptParams;

/*
 * ocf_scatter_batch -- replaces data_reader.build_sparse_batch (data_reader.py:95-200, mode 0)
 * and build_sparse_batch_fixed_split (data_reader.py:202-298, mode 1), dense representation.
 * Zeroes rows [0, B_pad) of every non-null output, scatters the batch, and (if tile_cnt != NULL)
 * buckets the target entries by 128-column tile for OCF_EPI_MASKED_MSE.
 */
typedef struct OcfScatterArgs {
  /* source 1: train CSR (mode 0) or eval-input CSR (mode 1) */
  const int64_t* rp1; const int32_t* col1; const float* val1; const int32_t* dup1;
  const int32_t* rows1;      /* [B] dataset row of each batch row, -1 = empty (None input)  */
  const uint8_t* keep1;      /* [nnz of batch] reciprocal-split keep flags (host NumPy RNG)  */
  const int64_t* boff1;      /* [B+1] batch-local entry offsets of source 1                  */
  float s0, s1;              /* data_sparsity range; used when keep1 == NULL (device RNG)   */
  uint64_t seed, stream;
  int mode;                  /* 0 train, 1 eval                                              */
  int pass_through;          /* pass_through_input_training (data_reader.py:161)             */
  /* source 2: eval-target CSR (mode 1) */
  const int64_t* rp2; const int32_t* col2; const float* val2; const int32_t* dup2;
  const int32_t* rows2;
  int B, B_pad, N;
  float aux;                 /* aux_var_value (train.py:47)                                  */
  /* dense fp32 outputs [B_pad][ld] (nullable) */
  float *X, *Min, *Mout, *T, *Mmiss;
  int64_t ld;
  /* concatenated layer-0 input [B_pad][xin_ld] in the compute dtype (nullable) */
  void* xin; int xin_dtype; int64_t xin_ld, xin_block;
  int feed;                  /* block 1: 0 none, 1 M_in (dropout/both), 2 M_miss (causal), 3 zeros */
  int both;                  /* block 2 = M_miss (auxilliary_mask_type 'both')               */
  /* target buckets (nullable) */
  int* tile_cnt; int* bk_ptr; int* bk_cur; int32_t* bk_rc; float* bk_t; float* bk_m;
  int n_tiles;
  /* column-sharded source 1 (feature parallelism): pos1[e] = position of entry e within its FULL
   * row, used to index keep1 / the device RNG so every shard sees the same reciprocal split
   * (nullable: position = e - row start) */
  const int32_t* pos1;
  /* flattened launch: entries of the batch held by this CSR (local offsets, = boff1 when the CSR
   * is not a column shard) and their counts; per-entry "live target" flags for the row-segment
   * target mode of OCF_EPI_MASKED_MSE (nullable) */
  const int64_t* lboff1; const int64_t* lboff2;
  int64_t E1, E2;
  uint8_t* tflag1; uint8_t* tflag2;
  /* 1: xin is already zero (nothing was written to it since it was last cleared), so the
   * [B_pad][xin_ld] memset is skipped */
  int xin_clean;
  /* per batch-local source-1 entry: its rating if it is a live input (the value X keeps after
   * duplicate resolution), else 0 -- the row-gather encoder's input (nullable) */
  float* xval1;
  /* (nullable) per-(128-column tile, 64-row K-step) entry counts of source 1 for ocf_sparse_tiles
   * (tb_cnt[(col >> 7) * tb_nk + (b >> 6)] += 1 per entry; the caller zeroes them beforehand) */
  int32_t* tb_cnt; int tb_nk;
  /* (nullable) per-column row tags: rtag_in[c] = rtag for every column c holding a live input of
   * the batch, rtag_out[c] = rtag for every column holding a live target (source 1, mode 0).  The
   * columns so tagged are a superset of the weight rows with a nonzero gradient this step
   * (OcfGemmArgs row_tag); the caller cycles rtag through 1..255 so no clearing pass is needed */
  uint8_t* rtag_in; uint8_t* rtag_out; int rtag;
  /* (nullable, mode 0) the batch's per-column entry counts and entry keys for ocf_row_lists:
   * col_cnt[c] += 1 and ecb[e] = c | b << 19 for every source-1 entry e (column c < 2^19, batch row
   * b < 4096); the caller zeroes col_cnt once, ocf_row_lists leaves it zeroed for the next batch */
  int32_t* col_cnt; int32_t* ecb;
} OcfScatterArgs;

int ocf_scatter_batch(const OcfScatterArgs* args, void* stream);

/* ocf_epoch_scatter -- ocf_scatter_batch's per-entry outputs (xval1: live input value, tflag1: live target)
 * for many train batches of an epoch plan in one launch: base is batch 0's OcfScatterArgs (mode 0, no
 * dense / xin / bucket / count / tag outputs, E2 = 0); batch sel[s] uses base's rows1 / lboff1 / boff1
 * offset by that batch, keep1 + keep_off[sel[s]], stream = stream_mul * (sel[s] + 1) (the per-step
 * generator's seeds) and writes xval / tflag at ebase[s] - ebase0 .. ebase[s + 1] - ebase0; max_e = max entries
 * of a batch.  ebase0 lets sel / ebase point into epoch-wide device tables (a window of consecutive batches
 * needs no upload): 0 when ebase starts at 0.
 * B <= 4,096.  Extension (no reference counterpart): the data_reader.py:95-200 batch assembly, per epoch. */
typedef struct OcfEpochScatterArgs {
  int n_sel; const int32_t* sel; const int64_t* ebase; int64_t max_e;
  const int64_t* keep_off; uint64_t stream_mul;
  float* xval; uint8_t* tflag;
  int64_t ebase0;                        /* subtracted from every ebase[s] */
} OcfEpochScatterArgs;
int ocf_epoch_scatter(const OcfScatterArgs* base, const OcfEpochScatterArgs* ep, void* stream);

/*
 * Row-gather products for sparse batches (csrc/ocf_sparse.hip): the encoder sum over a batch row's
 * live input entries, and the decoder's per-target forward / loss / delta with the delta times W_out
 * row accumulated for the hidden-layer delta (model.py:64-86, train.py:49).  Work is split into
 * chunks of <= 256 entries of one batch row (ch_row / ch_j0 / ch_j1: batch row and local entry range);
 * each chunk writes an fp32 partial [H] and ocf_rows_reduce sums a row's chunks in order.
 */
typedef struct OcfGatherArgs {
  const int32_t* rows;       /* [B] CSR row of each batch row (-1 = empty)                        */
  const int64_t* rp; const int32_t* col; const float* val;   /* the CSR holding the entries     */
  const int64_t* lboff;      /* [B+1] batch-local entry offsets of this CSR                       */
  const float* xval;         /* encoder: per batch-local entry input value, 0 = not a live input  */
  const uint8_t* flag;       /* decoder: per batch-local entry live-target flag                   */
  const int32_t* ch_row; const int32_t* ch_j0; const int32_t* ch_j1;
  int n_chunks;
  const void* W; int w_dtype; int64_t ldw; int w_blocked;   /* weights, one row per column n      */
  int H;                     /* padded hidden width (multiple of 128, <= 512)                     */
  float* part;               /* [n_chunks][H] fp32 partial sums                                   */
  /* decoder only */
  const void* h; int h_dtype;                 /* [Bp][H] hidden activations (compute dtype)       */
  const float* bias; float aux;               /* output bias, output-mask value (train.py:47)     */
  float* delta_e;            /* per batch-local entry delta err*m (nullable)                      */
  float* chunk_stats;        /* [n_chunks][4]: SSE, SAE, count_nonzero(T + yhat), 0               */
  void* d_out; int d_dtype; int64_t ld_d;     /* optional dense delta (zero elsewhere)            */
  /* decoder, optional (enc_part != NULL, one hidden layer): the hidden layer's bias / activation /
   * dropout applied here instead of by ocf_rows_reduce(OCF_REDUCE_BIAS_ACT) -- h[b] = dropout(act(the
   * encoder chunk partials enc_part[enc_cptr[b] .. enc_cptr[b+1]) summed in order + bias_h)), the same
   * arithmetic; the first chunk of each batch row also stores a_out, mask_out and h (h is then written) */
  const float* enc_part; const int32_t* enc_cptr; const float* bias_h; int act; float keep;
  uint64_t seed, stream; float* a_out; uint8_t* mask_out; int m_real, n_real;
  /* decoder, optional: a device word the launch sets to zero (a caller's flag cleared for free; the
   * engine no longer needs it: ocf_gemm_pair's counter never needs clearing) */
  uint64_t* zero_word;
  /* decoder, optional (jr and row_arrive both set): the hidden delta's row reduction (ocf_rows_reduce with
   * OCF_REDUCE_GRAD_ACT on *jr: the same sums and arithmetic, the chunk stats summed into the stats rows) done
   * in this launch by the last chunk of each batch row to finish.  The chunks store their partials and stats
   * write-through and count themselves in row_arrive[b] (device uint32 [Bp], zero when first passed: the
   * last chunk of a row resets it); rows without chunks (padding, no targets) get the zero delta.  jr->part
   * and jr->chunk_stats must be this launch's part and chunk_stats, jr->H its H. */
  const struct OcfRowsReduceArgs* jr; uint32_t* row_arrive;
} OcfGatherArgs;

int ocf_gather_encoder(const OcfGatherArgs* args, void* stream);
int ocf_gather_decoder(const OcfGatherArgs* args, void* stream);
/* ocf_gather_encdec -- ocf_gather_encoder(enc) then ocf_gather_decoder(dec) as ONE launch: a decoder chunk starts
 * as soon as its row's encoder chunks are done (per-row arrival counters) instead of after the whole encoder.
 * Requires: dec.enc_part == enc.part, dec.enc_cptr (the encoder's row_cptr), the decoder's folded row reduction
 * (dec.jr + dec.row_arrive: its last chunk per row resets the counter), the same chunk table in both (ch_row /
 * ch_j0 / ch_j1 / n_chunks: a train batch, inputs = targets) and the same H.  enc_arrive: device uint32 [Bp],
 * zero before the first call, left zero.  Same results as the two calls (the same sums in the same order).
 * Fail-safe: a decoder chunk's wait is bounded (ocf_set_tuning "encdec_max_polls"; < 0 injects a give-up on
 * batch row 0 for tests).  A chunk that gives up still counts itself in row_arrive, so the row's last chunk
 * returns both counters to zero, stores nothing else, closes the launch's hand-off gate (a library-internal
 * device word set to this launch's generation) and raises OCF_ASYNC_ENC_WAIT; every ocf_gemm_pair launch
 * issued after it (pair or dual-row form) reads the gate at entry and writes no parameter, slot, shadow, bias
 * or statistic.  The next ocf_* call reports the error once.  (An encoder chunk that arrives after the give-up
 * would leave its row's count behind: a host that sees OCF_ASYNC_ENC_WAIT clears enc_arrive and row_arrive
 * after synchronising, as engine.Engine does.) */
int ocf_gather_encdec(const OcfGatherArgs* enc, const OcfGatherArgs* dec, uint32_t* enc_arrive, void* stream);

/* ocf_encoder_tiles -- the encoder's X W1 (model.py:64-71) as an MFMA contraction over 128-column tiles of W1, for
 * batches whose weight rows carry many entries (Netflix width, feature-parallel ranks): each W1 tile is read once
 * per 256 batch rows (the row gathers read a W1 row per entry) and multiplied by the batch's X tile, densified in
 * LDS from the rows' column-sorted entries.  Writes split-K partials part[b][s][h] (s < splits: contiguous tile
 * ranges); the caller sums them with ocf_rows_reduce (row_cptr[b] = b * splits).  X = the live input values
 * (xval, list order; duplicates added) rounded to the compute dtype; fp32 accumulation. */
typedef struct OcfEncTileArgs {
  const int32_t* rows;    /* [B] dataset row per batch row (-1 = none)                                      */
  const int64_t* rp;      /* row pointers of the dataset CSR                                                */
  const int32_t* tptr;    /* [rows][n_tiles + 1] per-row tile pointers of the column-sorted view (RatingsCSR.tile_index) */
  const int32_t* tcol;    /* view: column of each entry (row-relative positions from rp)                    */
  const int32_t* tlidx;   /* view: the entry's index in the row's list order                                */
  const int64_t* lboff;   /* [B + 1] batch-local offset of each row's entries                              */
  const float* xval;      /* per batch-local entry: live input value (0 = not an input)                    */
  const void* W;          /* 16-bit weight shadow, row-major [n_tiles * 128][ldw]                           */
  int64_t ldw; int w_dtype;
  int B, Bp;              /* real batch rows, padded rows (multiple of 128)                                 */
  int n_tiles;            /* 128-column tiles                                                               */
  int H;                  /* hidden width (multiple of 128)                                                 */
  int splits;             /* tile ranges (split-K)                                                          */
  float* part;            /* [Bp][splits][H] fp32                                                           */
  int64_t nnz;            /* entries of the view, n_entries: entries of xval (bounds of the clamped loads)  */
  int64_t n_entries;
  void* work; int64_t work_bytes;   /* device scratch of ocf_encoder_tiles_workspace(args) bytes: the batch's
                                       entries packed per (256-row group, tile) by a pre-pass in the same call */
  int64_t max_row_len;    /* an upper bound of the batch rows' lengths (the pre-pass grid)                  */
} OcfEncTileArgs;
int64_t ocf_encoder_tiles_workspace(const OcfEncTileArgs* args);
int ocf_encoder_tiles(const OcfEncTileArgs* args, void* stream);

enum { OCF_REDUCE_RAW = 0, OCF_REDUCE_BIAS_ACT = 1, OCF_REDUCE_GRAD_ACT = 2 };

typedef struct OcfRowsReduceArgs {
  const float* part; const int32_t* row_cptr;  /* chunk partials, [B+1] first chunk of each row   */
  int B, Bp, H, mode;
  float* out;                /* RAW: [Bp][H] fp32 row sums                                        */
  /* BIAS_ACT (layer forward) / GRAD_ACT (delta through activation + dropout) */
  const float* bias; int act; float keep; uint64_t seed, stream;
  const uint8_t* mask_in; uint8_t* mask_out; float* a_out; const float* a_in;
  void* h_out; int h_dtype; int n_real;
  float* db_part; float gscale;             /* GRAD_ACT: [Bp][H] bias-gradient rows * gscale     */
  const float* chunk_stats; float* stats_part; float* row_sse;   /* decoder stats -> per row      */
} OcfRowsReduceArgs;

int ocf_rows_reduce(const OcfRowsReduceArgs* args, void* stream);

/* out[n] = gscale * sum_{b < B} d[b][n] for a dense [*][ld] array in dtype (output-bias gradient) */
int ocf_colsum(const void* d, int dtype, int64_t ld, int B, int N, float gscale, float* out, void* stream);

/* Target buckets from dense target / output-mask arrays (Model.train_on_batch / fit on user arrays):
 * an entry wherever T != 0 or M != 0, bucketed per 128-column tile in (row, column) order
 * (deterministic).  rows (nullable): batch row b is row rows[b] of T / M (a device-resident dataset). */
int ocf_dense_targets(const float* T, const float* M, int64_t ld, int B, int N, int n_tiles, int* tile_cnt,
                      int* bk_ptr, int* bk_cur, int32_t* bk_rc, float* bk_t, float* bk_m, const int64_t* rows,
                      void* stream);

/* Pack up to three dense fp32 [*][ld_src] inputs into the compute-dtype concatenated layer-0
 * input (model.py:47-56 concatenate); rows (nullable) as for ocf_dense_targets. */
int ocf_pack_input(const float* s0, const float* s1, const float* s2, int64_t ld_src, int B, int N, void* xin,
                   int dtype, int64_t xin_ld, int64_t xin_block, int B_pad, const int64_t* rows, void* stream);

/*
 * ocf_gemm -- one MFMA GEMM  C[M,N] = A[M,K] * B[K,N]  with a fused epilogue.  Replaces the TF
 * MatMul / BiasAdd / activation / Dropout / Mul / SquaredDifference / Assign ops Keras emits for
 * model.py:64-86 and train.py:49-51.  a_col: A stored [K][M] (else [M][K]); b_col: B stored [K][N]
 * (else [N][K]).  M, N multiples of 128; K a multiple of 64 (f16/bf16) or 32 (f32).
 */
typedef struct OcfGemmArgs {
  int compute_dtype;         /* f16 / bf16 MFMA (fp32 accumulate) or f32 MFMA (exact fp32)     */
  const void* A; int a_dtype; int a_col; int64_t lda;
  const void* B; int b_dtype; int b_col; int64_t ldb;
  int M, N, K;
  int splits;                /* split-K count (OCF_EPI_SLAB only)                               */
  int order;                 /* tile order: 0 n-fastest, 1 m-fastest                            */
  int epi;
  /* epilogue operands (meaning per epilogue; unused ones may be NULL/0) */
  float* out; int64_t ld_out; int64_t split_stride;          /* SLAB, GRAD, PREDICT; GRAD writes
                                                                 bf16 when h_dtype == OCF_BF16  */
  const float* bias;                                          /* BIAS_ACT, PREDICT, MSE       */
  int act; float keep; uint64_t seed, stream;                 /* BIAS_ACT, GRAD_ACT           */
  const uint8_t* mask_in; uint8_t* mask_out;                  /* dropout masks                */
  float* a_out; void* h_out; int h_dtype;                     /* BIAS_ACT outputs / GRAD_ACT  */
  const float* a_in;                                          /* GRAD_ACT: forward activation */
  float* db_part; int64_t ld_db;                              /* GRAD_ACT, MSE               */
  int m_real, n_real;
  float* p; float* s1; float* s2; OcfOptParams opt;           /* OPTIM                        */
  const float* pmask; int64_t ld_pmask;                       /* PREDICT output mask          */
  const int* bk_ptr; const int32_t* bk_rc; const float* bk_t; const float* bk_m;   /* MSE     */
  float* stats_part; float* row_sse_part;                     /* MSE                          */
  /* MSE row-segment target mode (used when bk_ptr == NULL): the target CSR's column-sorted view
   * (col/val/list index), its per-row tile pointers [rows][t_ntiles+1], the batch rows' CSR rows,
   * the batch-local entry offsets and the scatter's live-target flags; every target has mask t_aux */
  const int32_t* t_rows; const int64_t* t_rp; const int32_t* t_tptr; const int32_t* t_col; const float* t_val;
  const int32_t* t_lidx; const uint8_t* t_flag; const int64_t* t_lboff; int t_ntiles; float t_aux;
  /* OPTIM: also write the updated weights in the compute dtype (same layout as p, nullable), the
   * half-width shadow the next forward / backward GEMMs stream instead of the fp32 master copy */
  void* p_shadow;
  /* 1: load operand A / B with the non-temporal cache policy (its last use in the step, so it
   * should not displace reusable data from the Infinity Cache) */
  int a_nt, b_nt;
  /* B is a 16-bit compute-dtype array stored 64x64-blocked (blocks of 64 rows x 64 columns, each
   * 8 KB contiguous and row-major inside, blocks row-major; ldb = columns); OPTIM: write p_shadow in
   * that layout */
  int b_blocked, shadow_blocked;
  /* OPTIM / GRAD with a_col = 1: A ([K][M], K = batch row, M = column) is not read from memory but
   * built per K-step in LDS from a CSR's column-sorted view (RatingsCSR.tile_index): for batch row b
   * (CSR row sp_rows[b], b < sp_krows) and the M tile t, the entries [sp_rp[r] + sp_tptr[r][t],
   * sp_rp[r] + sp_tptr[r][t+1]) of sp_col / sp_lidx, with value sp_vals[sp_lboff[b] + lidx] (0 = none).
   * sp_colsum (nullable): opt.gscale * column sums of A (the output-bias gradient) */
  int a_sparse;
  const int32_t* sp_rows; const int64_t* sp_rp; const int32_t* sp_tptr; const int32_t* sp_col;
  const int32_t* sp_lidx; const int64_t* sp_lboff; const float* sp_vals;
  int sp_ntiles, sp_krows;
  float* sp_colsum;
  /* optional (OPTIM, 16-bit compute): the same sparse A bucketed by (M tile, K-step) by
   * ocf_sparse_tiles (sp_bptr [M/128 * K/64 + 1], sp_ent pairs (value index, k | m_local << 8));
   * with them the persistent role-split kernel runs (ocf_set_tuning "optim_ws") */
  const int32_t* sp_bptr; const int32_t* sp_ent;
  /* OPTIM: small jobs of the step done by the same launch (folded into the persistent kernel, else
   * launched separately on the same stream), each nullable by its first pointer:
   *   cb_p: bias optimizer on the sp_colsum outputs (the output-layer bias: cb_p[m] for m < M),
   *         = ocf_bias_opt_from_partials(cb_p, sp_colsum, 1, M, M, cb_s1, cb_s2, NULL, &cb_op)
   *   jb_part: = ocf_bias_opt_from_partials(jb_p, jb_part, jb_parts, jb_ld, jb_n, jb_s1, jb_s2, NULL, &jb_op)
   *   js_sp: = ocf_stats_finalize(js_sp, js_nparts, js_rs, js_ntiles, js_M, js_out) */
  float* cb_p; float* cb_s1; float* cb_s2; OcfOptParams cb_op;
  const float* jb_part; int jb_parts, jb_n; int64_t jb_ld; float* jb_p; float* jb_s1; float* jb_s2;
  OcfOptParams jb_op;
  const float* js_sp; const float* js_rs; float* js_out; int js_nparts, js_ntiles, js_M;
  /* OPTIM with Adagrad and l2 == 0 (nullable): live-row records of M's 128-row tiles (layout:
   * OCF_LIVE_REC below, built by ocf_sparse_tiles from the scatter's row tags).  Rows not listed
   * have an all-zero gradient (caller's guarantee); for them Keras' Adagrad update (a += 0;
   * p -= lr * 0 / (sqrt(a) + eps)) is the identity, so the kernel streams the parameter / slot /
   * shadow traffic of the listed rows only; results are bit-identical to the full update.  Used by
   * the role-split kernel, ignored by the generic one; rejected with any other optimizer or l2 != 0. */
  const uint8_t* row_live;
  /* OPTIM / a_col = 1, a_sparse (nullable): the same sparse A as row lists (OcfTileBucketArgs row_ptr /
   * row_ent; values sp_vals).  With them the weight gradient is computed row by row from the entries
   * (g[m][:] = sum over the entries (v, k) of column m, in k order, of v * B[k][:], fp32) and updated
   * in place by one wave per row -- no MFMA over the mostly-zero A; with Adagrad and l2 == 0 rows
   * without entries are skipped (identity update).  Requires N % 128 == 0, N <= 512. */
  const int32_t* sp_rowptr; const int32_t* sp_rowent;
  /* (nullable, OPTIM with the row-stream or role-split kernel) a folded ocf_rows_reduce in mode
   * OCF_REDUCE_GRAD_ACT: one job per batch row (a wave; the same per-element sums and epilogue), so the
   * decoder's delta reduction rides in a weight-gradient launch that does not read its outputs (dW_out)
   * and the launches that do (dW_in, its bias / stats jobs) follow.  The struct is copied at the call. */
  const OcfRowsReduceArgs* jr;
  /* row lists: the number of entries (0 = unknown).  With many entries per weight row (>= 4 per row on
   * average: feature-parallel global batches, dense datasets like ML-1M) the row-stream kernel loads each
   * row's entries as one vector (a lane per entry) and the B rows of a group of entries in one go. */
  int64_t sp_nent;
  /* MASKED_MSE dense target mode (nullable dn_t): targets / output masks as dense fp32 arrays, batch row b
   * at row dn_rows[b] (nullable: b) of [*][ld_dn], columns < n_real; an entry wherever t != 0 or m != 0.
   * Replaces the bucket pass of ocf_dense_targets for dense batches (Model.fit / train_on_batch). */
  const float* dn_t; const float* dn_m; int64_t ld_dn; const int64_t* dn_rows;
} OcfGemmArgs;

int ocf_gemm(const OcfGemmArgs* args, void* stream);

/*
 * ocf_gemm_pair -- ocf_gemm(a) then ocf_gemm(b) for the two weight updates of a one-hidden-layer step
 * (a = the output layer, with the decoder's folded row reduction jr; b = the input layer, whose operand B
 * and job inputs that reduction writes: train.py:50-51 for both kernels).  When both take the row-stream
 * kernel with the same instance they run as ONE launch: b's workgroups wait, in the kernel, for a's
 * row-reduction workgroups (agent-scope release / acquire on sync[0]), so the two row streams run back to
 * back without a kernel boundary.  On small weights (fewer than ~170 row tiles) whose two updates share
 * their row lists (sp_rowptr / sp_rowent / row_live equal: the generator's train batches) the launch is
 * the dual-row form instead: one wave walks column m's entry chain once and updates row m of both
 * matrices (ocf_set_tuning "rows_dual" 0: two launches).  sync (NULL = two launches): the hand-off
 * counter below.  Results are identical to the two ocf_gemm calls.
 *
 * The counter only grows, so nothing is reset between launches: word is a device uint64 that is zero
 * when first passed (one hipMemset after allocating it) and that only the library writes afterwards;
 * count is its host-side twin (zero with it): the producer workgroups counted on *word before this
 * launch.  A pair launch makes its input-layer workgroups wait for *word >= count + n_prod and
 * advances count by n_prod (the number of row-reduction workgroups); a call that falls back to two
 * launches leaves both unchanged.  The wait is bounded (ocf_set_tuning "pair_wait_polls"): a workgroup
 * that gives up skips its update and the next ocf_* call fails with OCF_ASYNC_PAIR_WAIT's message
 * (a word written by someone else, or a count that does not match it).
 */
typedef struct OcfPairSync {
  uint64_t* word;      /* device */
  uint64_t count;      /* host, in/out */
} OcfPairSync;
int ocf_gemm_pair(const OcfGemmArgs* a, const OcfGemmArgs* b, OcfPairSync* sync, void* stream);

/* codes of the asynchronous error word (kernels that detect a fault without stopping; reported by the
 * next entry point through its status and ocf_last_error()) */
#define OCF_ASYNC_PAIR_WAIT 1
#define OCF_ASYNC_MLP_BARRIER 2   /* ocf_mlp_step: a grid barrier gave up (workgroups not all resident) */
#define OCF_ASYNC_ENC_WAIT 3      /* ocf_gather_encdec: a decoder chunk gave up waiting for its row's encoder chunks */

/*
 * ocf_train_step_rows -- one whole single-GPU training step of a one-hidden-layer model on a sparse
 * (generator) batch, the Keras train_on_batch that fit_generator runs per step (train.py:157 ->
 * model.py:64-86 forward, train.py:49 masked MSE, train.py:50-51 Adagrad / RMSprop / Adam): the encoder
 * gather, the decoder gather (with the hidden layer's epilogue), dW_out (+ the folded row reduction jr
 * when jr_on, the output bias) and dW_in (+ the hidden bias, the step's stats), i.e.
 *   ocf_gather_encoder(&enc); ocf_gather_decoder(&dec); ocf_gemm(&dw_out with .jr = &jr); ocf_gemm(&dw_in)
 * in one library call (dw_out / dw_in through ocf_gemm_pair when pair_sync is set): each member is exactly
 * what the four calls take (the same checks run).  The host
 * keeps one of these per model and rewrites only the batch's table pointers and the step's Philox stream /
 * stats slot / optimizer constants between steps (engine.Engine.fast_train_step), so issuing a step costs
 * one call instead of building four argument blocks (the small configs' steps are host-bound otherwise).
 * dw_out.jr is ignored (jr_on selects the folded reduction).
 */
typedef struct OcfRowStepArgs {
  OcfGatherArgs enc;
  OcfGatherArgs dec;
  OcfGemmArgs dw_out;
  OcfGemmArgs dw_in;
  /* the decoder's row reduction: jr_on 1 = as jobs of dw_out (its jr), 2 = in the decoder launch (dec.jr;
   * dec.row_arrive set), 0 = none (dw_out.jr / dec.jr are ignored: the library points them at jr) */
  OcfRowsReduceArgs jr; int jr_on;
  /* (nullable) hipEvent_t recorded on `stream` before / after each launch: encoder, decoder, dW_out, dW_in
   * (the per-kernel timing bench.py reports; recorded only where set) */
  void* ev[8];
  /* (nullable) ocf_gemm_pair's hand-off counter: dW_out and dW_in as one launch (events 4 and 7 bracket
   * it); its count advances with every pair launch */
  OcfPairSync* pair_sync;
  /* (nullable) the encoder and the decoder as one launch (ocf_gather_encdec with this counter; needs jr_on = 2):
   * events 0 / 1 then bracket nothing, 2 / 3 the fused launch */
  uint32_t* enc_arrive;
} OcfRowStepArgs;
int ocf_train_step_rows(const OcfRowStepArgs* args, void* stream);

/*
 * ocf_rank_step -- one feature-parallel rank step (SURVEY.md 8(e) N-sharding: this rank owns a column
 * shard of W1's rows and W_out's, one hidden layer, generator batches) as one library call per phase,
 * the collectives between them issued by the host (train.py:157 per step; model.py:64-86 forward,
 * train.py:49-51 loss and update):
 *   phase 0  ocf_gather_encoder(enc); ocf_rows_reduce(enc_sum)        -> partial pre-activations; the host
 *            all-reduces them over the ranks
 *   phase 1  ocf_splitk_bias_act(hidden); ocf_gather_decoder(dec); ocf_rows_reduce(dec_sum) -> partial
 *            hidden deltas; ocf_stats_finalize(stats) on `side` -- the host starts the deltas' all-reduce
 *   phase 2  (on `side`, overlapping that all-reduce) ocf_gemm(dw_out); ocf_bias_opt_from_partials(out_bias)
 *   phase 3  (after the host waited for it) ocf_splitk_grad_act(hidden_grad); ocf_gemm(dw_in); `stream`
 *            waits for `side`
 * Each member is exactly what the single call takes (the same checks run).  side = NULL runs every phase on
 * `stream`; with side, fork[0..1] / join are hipEvent_t the library records (side waits on fork[k] recorded
 * on stream before phases 1 / 2; stream waits on join recorded on side in phase 3).  ev[8] (nullable):
 * events recorded on stream before / after phase 0, 1, 2 (on side when set), 3.  The host keeps one of
 * these per model and rewrites only the batch's table pointers, the dropout stream and the stats slot
 * between steps (engine.Engine.fast_rank_step), so a rank step costs four calls instead of ten argument
 * blocks built in Python. */
typedef struct OcfBiasActArgs {         /* ocf_splitk_bias_act's arguments, in order (without the stream) */
  const float* slabs; int splits; int64_t split_stride; int M, N; int64_t ld; const float* bias; int act;
  float keep; uint64_t seed, stream; const uint8_t* mask_in; uint8_t* mask_out; float* a_out; void* h_out;
  int h_dtype, m_real, n_real;
} OcfBiasActArgs;
typedef struct OcfGradActArgs {         /* ocf_splitk_grad_act's arguments, in order */
  const float* slabs; int splits; int64_t split_stride; int M, N; int64_t ld; const float* a_in;
  const uint8_t* mask; float keep; int act; void* d_out; int d_dtype; float* db; float gscale; int m_real, n_real;
} OcfGradActArgs;
typedef struct OcfStatsArgs {           /* ocf_stats_finalize's arguments, in order */
  const float* stats_part; int n_parts; const float* row_sse_part; int n_tiles, M; float* out;
} OcfStatsArgs;
typedef struct OcfBiasOptArgs {         /* ocf_bias_opt_from_partials' arguments, in order (opt by value) */
  float* b; const float* db_part; int parts; int64_t ld; int n; float* s1; float* s2; float* g_out;
  OcfOptParams opt;
} OcfBiasOptArgs;
typedef struct OcfRankStepArgs {
  OcfGatherArgs enc; OcfRowsReduceArgs enc_sum;
  OcfBiasActArgs hidden; OcfGatherArgs dec; OcfRowsReduceArgs dec_sum; OcfStatsArgs stats;
  OcfGemmArgs dw_out; OcfBiasOptArgs out_bias;
  OcfGradActArgs hidden_grad; OcfGemmArgs dw_in;
  void* side; void* fork[2]; void* join;
  void* ev[8];
} OcfRankStepArgs;
int ocf_rank_step(const OcfRankStepArgs* args, int phase, void* stream);

/* split-K reductions fused with the layer epilogue (see OCF_EPI_BIAS_ACT / OCF_EPI_GRAD_ACT).
 * ocf_splitk_grad_act writes bias-gradient partials db[M/4][ld] (one row per 4 batch rows,
 * already * gscale) for ocf_bias_opt_from_partials. */
int ocf_splitk_bias_act(const float* slabs, int splits, int64_t split_stride, int M, int N, int64_t ld,
                        const float* bias, int act, float keep, uint64_t seed, uint64_t stream,
                        const uint8_t* mask_in, uint8_t* mask_out, float* a_out, void* h_out, int h_dtype,
                        int m_real, int n_real, void* hstream);
int ocf_splitk_grad_act(const float* slabs, int splits, int64_t split_stride, int M, int N, int64_t ld,
                        const float* a_in, const uint8_t* mask, float keep, int act, void* d_out, int d_dtype,
                        float* db, float gscale, int m_real, int n_real, void* hstream);

/* ocf_opt_step -- elementwise Adagrad / RMSprop / Adam / SGD update (Keras 2.0.4 get_updates);
 * g is multiplied by opt.gscale.  Used for biases and after the data-parallel all-reduce. */
int ocf_opt_step(float* p, const float* g, float* s1, float* s2, int64_t n, const OcfOptParams* opt, void* stream);
/* ocf_opt_step_ex -- ocf_opt_step on a gradient in fp32 or bf16 (g_dtype OCF_F32 / OCF_BF16: a
 * data-parallel reduce-scatter shard as it arrives), optionally writing the updated parameter rounded
 * to the compute dtype into shadow (OCF_F16 / OCF_BF16, RNE; the 16-bit weight copy the row gathers
 * read), so the data-parallel step all-gathers only the 16-bit shard (extension; no reference
 * counterpart -- the reference runs on one device). */
typedef struct OcfOptStepArgs {
  float* p; const void* g; int g_dtype; float* s1; float* s2; int64_t n; OcfOptParams opt;
  void* shadow; int shadow_dtype;
} OcfOptStepArgs;
int ocf_opt_step_ex(const OcfOptStepArgs* args, void* stream);

/* bias update from per-row-tile column partials db_part[parts][ld] (fixed summation order). */
int ocf_bias_opt_from_partials(float* b, const float* db_part, int parts, int64_t ld, int n, float* s1, float* s2,
                               float* g_out, const OcfOptParams* opt, void* stream);

/* ocf_sumsq -- out[0] += scale * sum(x[i]^2) over n elements (fixed summation order; ws: scratch of
 * 1,024 floats).  The l2 kernel-regulariser term Keras adds to the logged loss
 * (/root/reference/model.py:66,82 W_regularizer=l2(l2_weight_regulatization)). */
int ocf_sumsq(const float* x, int64_t n, float scale, float* ws, float* out, void* stream);

/* reduce OCF_EPI_MASKED_MSE partials to out[4 + M] = {sse, sae, nnz(T+yhat), 0, row_sse[M]}. */
int ocf_stats_finalize(const float* stats_part, int n_parts, const float* row_sse_part, int n_tiles, int M,
                       float* out, void* stream);

/* ocf_sparse_tiles -- bucket a batch's sparse A operand (the OcfGemmArgs sp_* descriptor) by
 * (M tile t < gm, K-step kt < nk): bucket t*nk + kt holds, for the batch rows b in [64 kt, 64 kt + 64)
 * in order and each row's entries of tile t in column order, the pair (sp_lboff[b] + lidx,
 * (b - 64 kt) | (col - 128 t) << 8).  Deterministic (no atomics).  cnt: scratch [gm*nk]; bptr:
 * [gm*nk + 1]; ent: [cap][2] with cap >= the batch's entries in tiles < gm.  Built once per batch
 * and shared by both weight-gradient GEMMs (train split: inputs and targets share the descriptor).
 * Extension (no reference counterpart): feeds the persistent dW kernel. */
/* live-row record of one 128-row tile (OCF_LIVE_REC bytes): int32 L = number of live rows at byte 0,
 * then at byte 16 + (k % 8) * 16 + k / 8 the tile-local index of its k-th live row (ascending), k < L
 * (the 16 row slots one stream thread of the dW kernel owns are contiguous: one 16-B load). */
#define OCF_LIVE_REC 144

typedef struct OcfTileBucketArgs {
  const int32_t* rows; const int64_t* rp; const int32_t* tptr; const int32_t* col; const int32_t* lidx;
  const int64_t* lboff;
  int krows, ntiles, gm, nk;
  int32_t* cnt; int32_t* bptr; int32_t* ent;
  int64_t cap;
  /* counted = 1: cnt already holds the counts (ocf_scatter_batch tb_cnt), the count pass is skipped;
   * cnt_clear (nullable): [gm*nk] counts zeroed by the fill pass (the next batch's counters) */
  int counted; int32_t* cnt_clear;
  /* (nullable) live-row records (OCF_LIVE_REC bytes per tile, gm tiles) of the rows m < 128 gm whose
   * tag equals rtag: live_in from rtag_in, live_out from rtag_out (OcfScatterArgs row tags) */
  const uint8_t* rtag_in; const uint8_t* rtag_out; int rtag;
  uint8_t* live_in; uint8_t* live_out;
  /* (nullable) row lists, the transpose of the buckets: for row m < 128 gm, the entries of column m
   * ordered by batch row, as pairs (value index, k) at row_ent[row_ptr[m] .. row_ptr[m+1]) (row_ent:
   * [cap][2]; row_ptr: [128 gm + 1]).  Deterministic (no atomics in the ordering). */
  int32_t* row_ptr; int32_t* row_ent;
} OcfTileBucketArgs;
int ocf_sparse_tiles(const OcfTileBucketArgs* args, void* stream);

/* ocf_row_lists -- the batch's entries grouped by column (the row lists of OcfGemmArgs sp_rowptr /
 * sp_rowent) straight from the scatter's counts and keys, in parallel over the entries and columns
 * whatever the number of column tiles: row_ptr = exclusive scan of col_cnt (which is zeroed for the
 * next batch), each entry placed at its column's cursor, then every column's list sorted by entry
 * index (= batch-row order; deterministic).  cursor: scratch of 3 n_cols + 256 ints whose first n_cols
 * are zero on entry (and are left zero).  Lists longer than 32 entries (a column present in that many
 * batch rows; at most one entry per batch row, so <= 4,096) are sorted by a workgroup each in LDS.
 * With rtag_* / live_*, also the live-row records of ocf_sparse_tiles (OCF_LIVE_REC per 128 rows).
 * Extension (no reference counterpart): feeds the row-stream weight-gradient kernel. */
typedef struct OcfRowListArgs {
  const int32_t* ecb; int64_t E;
  int32_t* col_cnt; int32_t* cursor; int n_cols;
  int32_t* row_ptr; int32_t* row_ent;
  const uint8_t* rtag_in; const uint8_t* rtag_out; int rtag;
  uint8_t* live_in; uint8_t* live_out;
} OcfRowListArgs;
int ocf_row_lists(const OcfRowListArgs* args, void* stream);

/* ocf_epoch_row_lists -- the row lists of ocf_row_lists for many batches of an epoch plan at once
 * (one launch sequence per epoch instead of three small launches per step), built from the plan's
 * tables rather than a scatter: for each selected batch s (epoch batch sel[s]) and column m,
 *   row_ent[ebase[s] - ebase0 + row_ptr[s][m] .. ebase[s] - ebase0 + row_ptr[s][m+1]) = (batch-local entry, batch row)
 * of every source entry of the batch in column m, in entry (= batch-row) order, row_ptr[s] the exclusive
 * scan of the column counts (row_ptr[s][n_cols] = the batch's entry count), and with live non-null
 * the OCF_LIVE_REC records of the columns holding at least one entry (a superset of the columns with
 * a nonzero gradient: an Adagrad l2 = 0 update at g = 0 is the identity, so the row skip stays exact).
 * B <= 4,096; a batch's entries < 2^31.  n_rg (0 or 1: one; at most min(64, B)): row groups per batch --
 * the count / fill walks split each batch's rows over n_rg workgroups (more parallelism when few batches are
 * built at once; the lists are the same).  cnt: scratch of max(n_rg, 1) * n_sel * n_cols / 2 + n_sel * (n_cols / 4096
 * + 1) + 1 + 2 * (entries / 1025 + 1) ints (16-bit counts per row group, per-4,096-column block totals, then the
 * queue of lists over 1,024 entries).  n_cols % 128 == 0.  ebase0 (0 when ebase starts at 0) lets sel / ebase be a window of
 * epoch-wide device tables (consecutive batches: nothing to upload per build).
 * Extension (no reference counterpart): the data_reader.py:326-419 batch loop's structure, per epoch. */
typedef struct OcfEpochRowListArgs {
  int n_sel; int B; int n_cols;
  const int32_t* rows;                   /* [nb][B] CSR row of each batch row */
  const int64_t* rp; const int32_t* col; /* source CSR */
  const int64_t* lboff;                  /* [nb][B + 1] batch-local entry offsets */
  const int32_t* sel;                    /* [n_sel] epoch batch index of each slot */
  const int64_t* ebase;                  /* [n_sel + 1] slot offsets into row_ent (entries) */
  int32_t* cnt;
  int32_t* row_ptr;                      /* [n_sel][n_cols + 1] */
  int32_t* row_ent;                      /* [ebase[n_sel]][2] */
  uint8_t* live;                         /* [n_sel][n_cols / 128][OCF_LIVE_REC] or null */
  int n_rg;                              /* row groups per batch (0 / 1: one) */
  int64_t ebase0;                        /* subtracted from every ebase[s] */
  int max_list;                          /* bound on a column's entries in one batch (B without duplicate
                                            ratings), 0 = unknown: <= 1,024 skips the long-list sort pass */
  int64_t entries;                       /* the build's entries (ebase[n_sel] - ebase[0]; 0 = unknown): >= 4 per
                                            list on average sorts the lists across lanes instead of per thread */
} OcfEpochRowListArgs;
int ocf_epoch_row_lists(const OcfEpochRowListArgs* args, void* stream);

/* ocf_recip_keep -- the reference's reciprocal input/target split draws for a whole training epoch,
 * bit-identical to NumPy's legacy global RandomState (MT19937): per batch bi, the B row sparsities
 * s = np.random.uniform(s0, s1, B) (data_reader.py:120), then per row np.random.choice([0, 1], len,
 * p=[1-s, s]) (:130), i.e. nb * B + n_entries doubles in that order; keep[e] = 1 where the choice is 1
 * (the entry is an input).  key / pos: NumPy's state (np.random.get_state()[1], [2]) on entry, the state
 * after the draws on return (hand it back with np.random.set_state).  The stream is generated on the
 * device in parallel segments, each started by MT19937 jump-ahead (characteristic polynomial of the
 * recurrence, x^J mod phi); the call synchronises `stream` to read the end state back.
 *   boff  [nb][B + 1] (device) cumulative entry counts of each batch's rows (full rows: the draws'
 *         lengths); ebase [nb + 1] (device) first entry of each batch (cumulative over batches);
 *   keep  (device, nullable: only advance the state, e.g. data_sparsity [1, 1]) [n_entries] u8;
 *   doubles (host, nullable) receives the raw uniforms (tests);
 *   workspace: device scratch of ocf_recip_keep_workspace(nb, B, n_entries, pos) bytes. */
typedef struct OcfRecipKeepArgs {
  uint32_t key[624]; int32_t pos;
  int32_t nb; int32_t B; int64_t n_entries;
  const int64_t* boff; const int64_t* ebase;
  double s0; double s1;
  uint8_t* keep;
  double* doubles;
  void* workspace; int64_t workspace_bytes;
} OcfRecipKeepArgs;
int64_t ocf_recip_keep_workspace(int nb, int B, int64_t n_entries, int pos);
int ocf_recip_keep(OcfRecipKeepArgs* args, void* stream);
/* host twins of the same algorithm (segments, jump-ahead tree), for CPU tests: n doubles of
 * np.random.random_sample from the state (key, pos), advancing it; and a jump by n_blocks * 624 words
 * of a block-aligned state (pos = 624). */
int ocf_mt_host_random_sample(uint32_t* key, int32_t* pos, int64_t n, double* out);
int ocf_mt_host_jump(const uint32_t* key_in, int64_t n_blocks, uint32_t* key_out);

/*
 * Model ABI: one omni_model (/root/reference/model.py:43-99) trained by five calls per step,
 *   ocf_forward -> ocf_masked_mse -> ocf_backward -> ocf_opt_step (per parameter)
 * the Keras train_on_batch that fit_generator runs (train.py:157) split at the points a binding drives:
 * forward (model.py:64-86), the masked MSE and its per-row sums (train.py:49, 102-121), the backward pass to
 * raw fp32 gradients, and the elementwise Keras update (train.py:50-51).  Parameters and gradients are
 * caller-owned fp32 device arrays in the padded Keras layout: W[i] is rows[i] x cols[i] (ocf_model_dims:
 * layer 0 has k_blocks * roundup(N, 128) rows -- input block j's column n at row j * roundup(N, 128) + n --,
 * hidden widths and N rounded up to 128), b[i] has cols[i] elements, padding zero.  A context holds only
 * the per-batch activations / dropout masks / split-K slabs of up to max_batch rows (allocated by
 * ocf_ctx_create, the only call that allocates or synchronises).  Batches are the reference's dense data_gen
 * arrays (data_reader.py:354-361): k_blocks fp32 [B][N] input blocks (inputs, then the mask to feed /
 * missing-data mask, model.py:47-56 concatenate), the output mask and the targets.
 */
#define OCF_MAX_HIDDEN 8
typedef struct OcfModelDesc {
  int n_hidden;              /* hidden layers, 1..OCF_MAX_HIDDEN (model.py:64 layers)                    */
  int N;                     /* output width (items or users, data_reader.py:24-28)                     */
  int k_blocks;              /* input blocks 1..3 (1 + use_causal_info + 'both', model.py:47-56)        */
  int hidden[OCF_MAX_HIDDEN];
  int act;                   /* OCF_ACTV_* of the hidden layers (train.py:52 'sigmoid')                  */
  float dropout;             /* model.py:70 Dropout rate, 0 = none                                       */
  int compute_dtype;         /* OCF_DT_F32 (exact fp32) / OCF_DT_F16 / OCF_DT_BF16 MFMA operands          */
  int max_batch;             /* batch rows per call, at most                                             */
  uint64_t seed;             /* dropout mask stream (Philox; step s draws stream 16 s + layer)           */
  float* W[OCF_MAX_HIDDEN + 1];
  float* b[OCF_MAX_HIDDEN + 1];
} OcfModelDesc;
typedef struct OcfCtx OcfCtx;

/* padded shape of every W[i] (n_hidden + 1 entries each) */
int ocf_model_dims(const OcfModelDesc* desc, int64_t* rows, int64_t* cols);
int ocf_ctx_create(const OcfModelDesc* desc, OcfCtx** ctx);
int ocf_ctx_destroy(OcfCtx* ctx);
/* ocf_forward -- pred[b][n] = out_mask[b][n] * (h_L[b] . W_L[:, n] + b_L[n]) for b < B, n < N (model.py:81-86;
 * out_mask nullable = unmasked).  training: dropout with the masks of step `step` (else none); masks_out
 * (nullable array of n_hidden nullable device pointers): each layer's keep flags as u8 [B][hidden[i]]. */
int ocf_forward(OcfCtx* ctx, const float* const* inputs, int64_t ld_in, int B, int training, uint64_t step,
                const float* out_mask, int64_t ld_mask, float* pred, int64_t ld_pred, uint8_t* const* masks_out,
                void* stream);
/* ocf_masked_mse -- the Keras loss on the masked prediction (train.py:49): e = pred - T over [B][N];
 * out_stats (4 + 3 B floats): {sum e^2, sum |e|, count_nonzero(T + pred), loss = sum e^2 / (B N)}, then the
 * per-row sums e^2 [B], |e| [B], count_nonzero [B] (train.py:102-121's batch metrics); out_grad (nullable)
 * [B][ld_grad] = e * out_mask (out_mask nullable = 1): the loss gradient with respect to the unmasked output
 * divided by gscale = 2 / (B N) -- kept unscaled so 16-bit operands do not underflow. */
int ocf_masked_mse(const float* pred, const float* T, const float* out_mask, int64_t ld, int B, int N,
                   float* out_grad, int64_t ld_grad, float* out_stats, void* stream);
/* ocf_backward -- the gradients of the last ocf_forward (same B) from out_grad: gW[i] / gb[i] (shapes of
 * W[i] / b[i]) = gscale * the backward pass of model.py:64-86 (dropout masks of that forward). */
int ocf_backward(OcfCtx* ctx, const float* grad, int64_t ld_grad, int B, float gscale, float* const* gW,
                 float* const* gb, void* stream);

/*
 * ocf_mlp_step -- one whole training step of a SMALL dense model (train_jester.py's 200 -> 256 -> 256 -> 100,
 * Model.fit's batches: train_jester.py:44-79 with model.py:64-86, train.py:49 and the Keras update) in ONE
 * launch: a persistent grid of `wgs` workgroups runs the forward layers, the masked MSE with the step's
 * statistics, the backward pass and every weight / bias update as phases separated by grid barriers
 * (2 L + 1 barriers for L hidden layers).  Each phase's work is 32 x 32 output tiles, one per workgroup with
 * the reduction dimension split over its four waves, on MFMA (v_mfma_f32_32x32x16_{f16,bf16} on operands
 * rounded to the compute dtype, v_mfma_f32_32x32x2_f32 in the exact-fp32 mode); values handed from one phase
 * to the next are stored write-through; a layer's weights are updated only after the phase that still reads
 * them.  For models
 * whose weights fit in L2 (0.14 M parameters) the step is latency-bound: one launch instead of ~14.
 * The batch is gathered from device-resident arrays by row index (Model.fit's data path): input block j of
 * batch row b is x[j] + rows[b] * ld_x (N values), its output mask / targets out_mask / targets + rows[b] *
 * ld_t.  Rows b >= B are padding (zero).  Weights in the engine's padded layout: W[0] [k_blocks * Np][hidden_p[0]]
 * (block j's column n at row j * Np + n), W[i] [hidden_p[i-1]][hidden_p[i]], W[L] transposed [Np][hidden_p[L-1]];
 * b[i] the padded output width; optimizer slots alike (nullable per the optimizer); shadow[i] (nullable) the
 * compute-dtype copy of W[i] rewritten by the update (64 x 64-blocked with shadow_blocked).  l2 = 0.
 * stats: {sse, sae, count_nonzero(T + y), 0, row sse [Bp]} (the masked-MSE statistics).  work: scratch of
 * ocf_mlp_step_workspace bytes.  barrier: device uint32[2], zero before the first launch, left reusable.
 */
typedef struct OcfMlpStepArgs {
  int n_hidden;                                   /* L, 1..OCF_MAX_HIDDEN */
  int B, Bp;                                      /* batch rows; padded (multiple of 64, <= 512) */
  int N, Np, k_blocks;                            /* output width / padded (multiple of 64); input blocks */
  int hidden[OCF_MAX_HIDDEN], hidden_p[OCF_MAX_HIDDEN];   /* hidden widths, padded (multiples of 64) */
  const float* x[3]; int64_t ld_x; const int64_t* rows;
  const float* out_mask; const float* targets; int64_t ld_t;
  float* W[OCF_MAX_HIDDEN + 1]; float* b[OCF_MAX_HIDDEN + 1];
  float* sW1[OCF_MAX_HIDDEN + 1]; float* sW2[OCF_MAX_HIDDEN + 1];
  float* sb1[OCF_MAX_HIDDEN + 1]; float* sb2[OCF_MAX_HIDDEN + 1];
  void* shadow[OCF_MAX_HIDDEN + 1]; int shadow_blocked;
  int act, compute_dtype;
  OcfOptParams opt;                               /* gscale = 2 / (B N) */
  float* stats;
  void* work; int64_t work_bytes;
  uint32_t* barrier;
  int wgs;                                        /* persistent workgroups (0: one per tile of the busiest
                                                   * phase, at most 128; never more than the CU count) */
  uint64_t* trace;                                /* (nullable) device uint64[24]: workgroup 0's constant-rate
                                                   * clock (100 MHz) at the start and after each phase */
  /* Dropout after every hidden layer (model.py:72-73; keep = 1 - dropout_probability, 1 = none): the mask of
   * layer i's element (m, n) is floor(keep + U) with U the Philox uniform of (seed, stream + i, m * hidden_p[i]
   * + n), as the layer-wise path draws it; mask[i] (u8 [Bp][hidden_p[i]], required when keep < 1) receives it. */
  float keep; uint64_t seed, stream;
  uint8_t* mask[OCF_MAX_HIDDEN];
} OcfMlpStepArgs;
int64_t ocf_mlp_step_workspace(const OcfMlpStepArgs* args);
int ocf_mlp_step(const OcfMlpStepArgs* args, void* stream);

/* ocf_set_tuning -- process-wide kernel selection switches (no reference counterpart).
 *   "optim_ws": 1 (default; env OCF_OPTIM_WS=0 turns it off) = EPI_OPTIM weight-gradient GEMMs on
 *               [K][M] x [K][N] operands with 16-bit compute run on the persistent role-split kernel
 *               (ocf_optim_ws.h); 0 = the generic tile kernel.  Bit-identical results.
 *   "optim_ws_max_k": largest K (batch rows) sent to that kernel (default 256; beyond it the K-loop
 *               outgrows the optimizer stream it hides under and the generic kernel is faster).
 *   "enc_tiles_pack": ocf_encoder_tiles with its packed pre-pass (1, default) or each row's entries read by the
 *               tile kernel itself (0).
 *   "encdec_rowres": ocf_gather_encdec with 16-bit weights as one 1,024-thread workgroup per batch row (1: the
 *               row's encoder, hidden epilogue, decoder and delta reduction with LDS reductions, no hand-offs;
 *               results equal to fp32 summation order) or as the chunked launch (0); a negative value only
 *               reports the setting; env OCF_ENCDEC_ROWRES sets the initial value (default 1).
 *   "pair_wait_polls", "encdec_max_polls", "mlp_max_polls": the bounded in-kernel waits of ocf_gemm_pair,
 *               ocf_gather_encdec and ocf_mlp_step (polls of ~64 cycles); the last two take a negative value as
 *               fault injection for tests (a give-up on workgroup 0 / batch row 0).
 * previous (nullable) receives the old value. */
int ocf_set_tuning(const char* key, int value, int* previous);

/* ocf_check_async -- reports (status 1, ocf_last_error) and clears a pending asynchronous kernel error
 * (OCF_ASYNC_*) without launching anything: hosts call it after their last step's results are read back
 * (Engine.take_stats at every epoch end), so a fault in the last launches of a run cannot go unseen. */
int ocf_check_async(void);

/* Timing events for measurement (bench.py's HIP-event timing of the dominant launch; no reference counterpart).
 * ocf_timing_event_create makes an event with hipEventDisableSystemFence: recording it takes no system-scope
 * cache write-back and invalidate.  With the default flags (torch.cuda.Event) every record idled the stream
 * ~5.7 us and started the next launch on a flushed L2.  Such an event is only for ocf_event_elapsed_ms after a
 * device synchronisation; it orders nothing.  *ev receives the hipEvent_t. */
int ocf_timing_event_create(void** ev);
int ocf_event_record(void* ev, void* stream);
int ocf_event_elapsed_ms(void* start, void* stop, float* ms);
int ocf_event_destroy(void* ev);

int ocf_version(void);
const char* ocf_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* OCF_H_ */
