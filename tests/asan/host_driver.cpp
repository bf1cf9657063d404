// SURVEY §5 sanitizer leg: the host side of libocf (argument checks, error state, tuning switches, the
// model-ABI dimension logic, the workspace layouts, the MT19937 host twin and its jump-ahead) run under
// AddressSanitizer + UndefinedBehaviorSanitizer on the CPU.  Built by `make asan` in the csrc directory from
// the library's own translation units, host side only (the device code is the normal build's, embedded as is);
// run by tests/test_asan_host.py.  Nothing here touches a GPU: every call either fails its argument checks
// before a HIP call or is pure host logic.  Exit status 0 = every check passed (a sanitizer report aborts).
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/ocf.h"

static int g_fail = 0;
#define EXPECT(c, what)                                                                 \
  do {                                                                                  \
    if (!(c)) {                                                                         \
      std::fprintf(stderr, "FAIL %s:%d %s (last error: %s)\n", __FILE__, __LINE__, what, \
                   ocf_last_error());                                                   \
      ++g_fail;                                                                         \
    }                                                                                   \
  } while (0)

static bool last_error_has(const char* s) { return std::strstr(ocf_last_error(), s) != nullptr; }

static void tuning() {
  struct K { const char* key; int good; int bad; };
  const K keys[] = {{"optim_rows", 1, -99}, {"enc_tiles_pack", 1, -99}, {"rows_long", -1, -99}, {"rows_dual", 1, -99},
                    {"rows_dual_parts", 23, 99}, {"rows_dual_pf", -1, -99}, {"rows_dual_large", 1, -99},
                    {"rows_dual_count", 0, -99}, {"rows_small_waves", 4096, -99}, {"optim_ws", 1, -99},
                    {"pair_wait_polls", 1 << 22, 0}, {"encdec_max_polls", 1 << 22, 0}, {"mlp_max_polls", 1 << 22, 0},
                    {"optim_ws_max_k", 256, -99}, {"encdec_rowres", 1, -99}};
  for (const K& k : keys) {
    int prev = -12345;
    EXPECT(ocf_set_tuning(k.key, k.good, &prev) == 0, k.key);
    EXPECT(prev != -12345, "previous value reported");
    EXPECT(ocf_set_tuning(k.key, prev, nullptr) == 0, "restore");
    if (k.bad != -99) {
      EXPECT(ocf_set_tuning(k.key, k.bad, nullptr) == 1, "out-of-range value refused");
      EXPECT(last_error_has("ocf_set_tuning"), "message names the call");
    }
  }
  EXPECT(ocf_set_tuning("no_such_key", 1, nullptr) == 1 && last_error_has("no_such_key"), "unknown key");
  EXPECT(ocf_set_tuning(nullptr, 1, nullptr) == 1 && last_error_has("unknown key"), "null key");
}

static void argument_checks() {
  OcfGatherArgs g{};
  EXPECT(ocf_gather_encoder(&g, nullptr) == 1 && last_error_has("null pointer"), "encoder: null tables");
  EXPECT(ocf_gather_decoder(&g, nullptr) == 1, "decoder: null tables");
  EXPECT(ocf_gather_encdec(nullptr, &g, nullptr, nullptr) == 1 && last_error_has("null arguments"), "encdec: nulls");
  uint32_t arrive[4] = {};
  OcfGatherArgs e{};
  EXPECT(ocf_gather_encdec(&e, &g, arrive, nullptr) == 1, "encdec: empty descriptors");
  // a well-formed table with a bad H
  int dummy_i[8] = {};
  int64_t dummy_l[8] = {};
  float dummy_f[8] = {};
  g.rows = dummy_i; g.rp = dummy_l; g.col = dummy_i; g.lboff = dummy_l; g.ch_row = dummy_i; g.ch_j0 = dummy_i;
  g.ch_j1 = dummy_i; g.W = dummy_f; g.part = dummy_f; g.H = 500; g.ldw = 512; g.w_dtype = OCF_DT_F16;
  EXPECT(ocf_gather_encoder(&g, nullptr) == 1 && last_error_has("multiple of 128"), "encoder: H % 128");
  g.H = 512; g.ldw = 500;
  EXPECT(ocf_gather_encoder(&g, nullptr) == 1 && last_error_has("ldw"), "encoder: ldw");
  g.ldw = 512;
  EXPECT(ocf_gather_encoder(&g, nullptr) == 1 && last_error_has("xval"), "encoder: xval");
  OcfRowsReduceArgs r{};
  EXPECT(ocf_rows_reduce(&r, nullptr) == 1 && last_error_has("bad arguments"), "rows_reduce");
  OcfGemmArgs a{};
  EXPECT(ocf_gemm(&a, nullptr) == 1 && last_error_has("null operand"), "gemm: null operands");
  a.A = dummy_f; a.B = dummy_f; a.M = 100; a.N = 128; a.K = 64; a.compute_dtype = OCF_DT_F16;
  EXPECT(ocf_gemm(&a, nullptr) == 1 && last_error_has("multiples of 128"), "gemm: M % 128");
  EXPECT(ocf_gemm_pair(nullptr, &a, nullptr, nullptr) == 1, "gemm_pair: null");
  OcfPairSync sy{};
  EXPECT(ocf_gemm_pair(&a, &a, &sy, nullptr) == 1 && last_error_has("device word"), "gemm_pair: sync word");
  EXPECT(ocf_train_step_rows(nullptr, nullptr) == 1, "train_step_rows: null");
  EXPECT(ocf_rank_step(nullptr, 0, nullptr) == 1, "rank_step: null");
  OcfRecipKeepArgs rk{};
  rk.nb = -1;
  EXPECT(ocf_recip_keep(&rk, nullptr) == 1 && last_error_has("sizes"), "recip_keep: sizes");
  rk.nb = 2; rk.B = 4; rk.n_entries = 10;
  EXPECT(ocf_recip_keep(&rk, nullptr) == 1 && last_error_has("workspace"), "recip_keep: workspace");
  EXPECT(ocf_recip_keep_workspace(-1, 4, 10, 624) == -1, "recip_keep_workspace: negative");
  EXPECT(ocf_recip_keep_workspace(3, 256, 200000, 17) > 0, "recip_keep_workspace: layout");
  EXPECT(ocf_mlp_step(nullptr, nullptr) == 1, "mlp_step: null");
  OcfEncTileArgs et{};
  EXPECT(ocf_encoder_tiles(&et, nullptr) == 1 && last_error_has("null pointer"), "encoder_tiles: null tables");
  EXPECT(ocf_encoder_tiles_workspace(nullptr) == -1, "encoder_tiles_workspace: null");
  et.Bp = 256; et.n_tiles = 3753; et.n_entries = 1150000;
  EXPECT(ocf_encoder_tiles_workspace(&et) >= 3754 * 4 + 1150000 * 4, "encoder_tiles_workspace: layout");
  et.rows = dummy_i; et.rp = dummy_l; et.tptr = dummy_i; et.tcol = dummy_i; et.tlidx = dummy_i; et.lboff = dummy_l;
  et.xval = dummy_f; et.W = dummy_f; et.part = dummy_f; et.w_dtype = OCF_DT_F32;
  EXPECT(ocf_encoder_tiles(&et, nullptr) == 1 && last_error_has("16-bit"), "encoder_tiles: fp32 weights refused");
  et.w_dtype = OCF_DT_F16; et.H = 512; et.ldw = 512; et.B = 256; et.splits = 1; et.nnz = 10;
  EXPECT(ocf_encoder_tiles(&et, nullptr) == 1 && last_error_has("1,024 tiles"), "encoder_tiles: tiles per split");
  et.splits = 64;
  EXPECT(ocf_encoder_tiles(&et, nullptr) == 1 && last_error_has("workspace"), "encoder_tiles: workspace");
}

static void model_logic() {
  OcfModelDesc d{};
  int64_t rows[OCF_MAX_HIDDEN + 1], cols[OCF_MAX_HIDDEN + 1];
  EXPECT(ocf_model_dims(&d, rows, cols) == 1, "model_dims: empty description refused");
  d.n_hidden = 2; d.N = 100; d.k_blocks = 2; d.hidden[0] = 256; d.hidden[1] = 200; d.act = OCF_ACTV_TANH;
  d.compute_dtype = OCF_DT_BF16; d.max_batch = 128;
  EXPECT(ocf_model_dims(&d, rows, cols) == 0, "model_dims: train_jester.py's model");
  EXPECT(rows[0] == 2 * 128 && cols[0] == 256 && rows[1] == 256 && cols[1] == 256 && rows[2] == 256 &&
             cols[2] == 128, "model_dims: padded Keras layout");
  EXPECT(ocf_model_dims(&d, nullptr, cols) == 1, "model_dims: null output");
  d.k_blocks = 4;
  EXPECT(ocf_model_dims(&d, rows, cols) == 1, "model_dims: k_blocks 1..3");
  OcfMlpStepArgs m{};
  EXPECT(ocf_mlp_step_workspace(&m) == -1, "mlp workspace: n_hidden 0 refused");
  m.n_hidden = 2; m.Bp = 128; m.N = 100; m.Np = 128; m.k_blocks = 2;
  m.hidden[0] = m.hidden[1] = 256; m.hidden_p[0] = m.hidden_p[1] = 256; m.compute_dtype = OCF_DT_BF16;
  m.keep = 0.8f;
  const int64_t ws = ocf_mlp_step_workspace(&m);
  EXPECT(ws > 0 && ws % 256 == 0, "mlp workspace: layout of the Jester step");
}

// MT19937 host twin: doubles of np.random.random_sample from a state (key, pos) equal (a >> 5, b >> 6) of two
// consecutive std::mt19937 outputs from the same state, and a jump of n blocks equals drawing 312 n doubles.
static void mt_twin() {
  std::mt19937 ref(20260101u);
  for (int i = 0; i < 1000; ++i) ref();                       // an arbitrary mid-block position
  // libstdc++'s state text: the 624 words, then the position
  std::stringstream ss;
  ss << ref;
  std::vector<uint32_t> key(624);
  for (auto& w : key) ss >> w;
  int32_t pos = 0;
  ss >> pos;
  const int64_t n = 5000;
  std::vector<double> out(n);
  std::vector<uint32_t> k2 = key;
  int32_t p2 = pos;
  EXPECT(ocf_mt_host_random_sample(k2.data(), &p2, n, out.data()) == 0, "random_sample");
  bool same = true;
  for (int64_t i = 0; i < n; ++i) {
    const uint32_t a = ref() >> 5, b = ref() >> 6;
    same &= out[i] == (a * 67108864.0 + b) / 9007199254740992.0;
  }
  EXPECT(same, "random_sample equals std::mt19937's words");
  // jump: a block-aligned state (pos 624) advanced by 3 blocks, against 3 x 312 doubles drawn from it
  std::vector<uint32_t> kb = k2;
  int32_t pb = p2;
  std::vector<double> skip(624);
  if (pb != 624) EXPECT(ocf_mt_host_random_sample(kb.data(), &pb, (624 - pb) / 2, skip.data()) == 0, "align");
  EXPECT(pb == 624, "block-aligned");
  std::vector<uint32_t> jumped(624), stepped = kb;
  int32_t ps = pb;
  EXPECT(ocf_mt_host_jump(kb.data(), 3, jumped.data()) == 0, "jump");
  std::vector<double> burn(3 * 312);
  EXPECT(ocf_mt_host_random_sample(stepped.data(), &ps, 3 * 312, burn.data()) == 0, "step 3 blocks");
  EXPECT(ps == 624 && std::memcmp(jumped.data(), stepped.data(), 624 * 4) == 0, "jump == 3 blocks of draws");
  EXPECT(ocf_mt_host_jump(nullptr, 3, jumped.data()) == 1, "jump: null key");
  EXPECT(ocf_mt_host_jump(kb.data(), -1, jumped.data()) == 1, "jump: negative");
}

int main() {
  EXPECT(ocf_version() >= 1, "version");
  tuning();
  argument_checks();
  model_logic();
  mt_twin();
  EXPECT(ocf_check_async() == 0, "no asynchronous error pending");
  std::printf("host_driver: %s (%d failures)\n", g_fail ? "FAILED" : "ok", g_fail);
  return g_fail ? 1 : 0;
}
