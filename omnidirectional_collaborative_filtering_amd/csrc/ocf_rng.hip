// NumPy's legacy RandomState stream (MT19937) on the device: the reference's reciprocal-split draws
// (data_reader.py:120 np.random.uniform per batch, :130 np.random.choice per row) for a whole training
// epoch at once, bit-identical to NumPy, with NumPy's global state handed in and handed back.
//
// MT19937 is a linear recurrence over GF(2): word x_{k+624} = x_{k+397} ^ twist(x_k, x_{k+1}).  The
// window W_k = (x_k .. x_{k+623}) advances by F (one word).  The stream is cut into segments of
// SEG_BLOCKS blocks of 624 words; segment s starts from the window jumped ahead by s * SEG_BLOCKS * 624
// words, so all segments generate in parallel.  A jump by J words applies p(F) with
// p(x) = x^J mod phi(x), phi = the recurrence's characteristic polynomial (degree 19937, found once by
// Berlekamp-Massey on the generator's own output bits): W_{k+J} = sum_i p_i F^i W_k, i.e. the XOR of
// the windows at the steps whose coefficient is set.  F has a 31-dimensional kernel (the low 31 bits
// of the oldest word never reach the future), so the jumped window is exact except those bits; they
// are recomputed from words 396 and 623 by inverting the twist (fix_first), after which every window
// is the one NumPy would hold.  Segment windows come from a doubling tree of jumps (round r: windows
// [2^r, 2^(r+1)) from windows [0, 2^r) by x^(2^r * SEG_BLOCKS * 624)), ~log2(segments) launches.
//
// Doubles: NumPy's random_sample / next_double = ((w0 >> 5) * 2^26 + (w1 >> 6)) / 2^53 from two
// consecutive words; uniform(a, b) = a + (b - a) * u; choice([0, 1], p=[1-s, s]) = (u >= (1-s)/((1-s)+s))
// (cdf = cumsum(p) / its last element, searchsorted side='right').  Compiled with -ffp-contract=off,
// so the device's double arithmetic rounds exactly like NumPy's.
//
// The host twin (ocf_mt_host_*) runs the same segment/jump algorithm on the CPU for the CPU tests;
// the product path (data_reader.BatchGenerator) only calls ocf_recip_keep.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <vector>

#include "ocf_internal.h"

namespace ocf {
namespace mt {

constexpr int NW = 624;
constexpr uint32_t MATRIX_A = 0x9908b0dfu, UPPER = 0x80000000u, LOWER = 0x7fffffffu;
constexpr int DEG = 19937;
constexpr int PW = (DEG + 1 + 63) / 64;   // 312 64-bit words: polynomials of degree <= DEG
constexpr int SEG_LOG = 8;                 // segments of 256 blocks (159,744 words)
constexpr int SEG_BLOCKS = 1 << SEG_LOG;
constexpr int QMAX = 40;                   // Q_k = x^(624 * 2^k) mod phi, k < QMAX

__host__ __device__ __forceinline__ uint32_t twist(uint32_t a, uint32_t b) {
  const uint32_t y = (a & UPPER) | (b & LOWER);
  return (y >> 1) ^ ((y & 1u) ? MATRIX_A : 0u);
}

__host__ __device__ __forceinline__ uint32_t temper(uint32_t y) {
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}

// the low 31 bits of window word 0 from words 396 and 623: x_{k+623} = x_{k+396} ^ twist(x_{k-1}, x_k)
__host__ __device__ __forceinline__ uint32_t fix_first(uint32_t w0, uint32_t w396, uint32_t w623) {
  const uint32_t t = w623 ^ w396;
  const uint32_t lsb = t >> 31;                       // MATRIX_A has its top bit set, y >> 1 does not
  const uint32_t y = ((t ^ (lsb ? MATRIX_A : 0u)) << 1) | lsb;
  return (w0 & UPPER) | (y & LOWER);
}

__host__ __device__ __forceinline__ double to_double(uint32_t a, uint32_t b) {
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) / 9007199254740992.0;
}

// ---------------------------------------------------------------- host: polynomials over GF(2)
struct Poly {
  uint64_t w[PW];
};

static inline bool bit(const uint64_t* p, int64_t k) { return (p[k >> 6] >> (k & 63)) & 1u; }

static void next_block_host(const uint32_t* x, uint32_t* out) {   // x: 624-word window, out: next 624 words
  uint32_t buf[2 * NW];
  std::memcpy(buf, x, NW * 4);
  for (int i = 0; i < NW; ++i) buf[NW + i] = buf[397 + i] ^ twist(buf[i], buf[i + 1]);
  std::memcpy(out, buf + NW, NW * 4);
}

struct Tables {
  Poly phi;                     // characteristic polynomial, phi.w bit DEG set
  std::vector<Poly> q;          // q[k] = x^(624 * 2^k) mod phi
  bool ready = false;
};

static Tables& tables() {
  static Tables t;
  return t;
}
static std::mutex& tables_mutex() {
  static std::mutex m;
  return m;
}

// a ^= b << sh   (wide bitsets of nw words; b has nb words)
static inline void xor_shifted(uint64_t* a, int nwa, const uint64_t* b, int nb, int64_t sh) {
  const int64_t ws = sh >> 6;
  const int bs = (int)(sh & 63);
  for (int j = 0; j < nb; ++j) {
    if (!b[j]) continue;
    if (ws + j < nwa) a[ws + j] ^= b[j] << bs;
    if (bs && ws + j + 1 < nwa) a[ws + j + 1] ^= b[j] >> (64 - bs);
  }
}

static void reduce_wide(uint64_t* wide, int nw, const Poly& phi, Poly& out) {
  for (int64_t k = (int64_t)nw * 64 - 1; k >= DEG; --k)
    if (bit(wide, k)) xor_shifted(wide, nw, phi.w, PW, k - DEG);
  std::memcpy(out.w, wide, PW * 8);
  out.w[PW - 1] &= (DEG % 64) ? ((1ull << (DEG % 64)) - 1) : ~0ull;   // bits >= DEG are zero already
}

static inline uint64_t spread32(uint32_t v) {
  uint64_t x = v;
  x = (x | (x << 16)) & 0x0000FFFF0000FFFFull;
  x = (x | (x << 8)) & 0x00FF00FF00FF00FFull;
  x = (x | (x << 4)) & 0x0F0F0F0F0F0F0F0Full;
  x = (x | (x << 2)) & 0x3333333333333333ull;
  x = (x | (x << 1)) & 0x5555555555555555ull;
  return x;
}

static void sqr_mod(const Poly& a, const Poly& phi, Poly& out) {
  std::vector<uint64_t> wide(2 * PW, 0);
  for (int j = 0; j < PW; ++j) {
    wide[2 * j] = spread32((uint32_t)a.w[j]);
    wide[2 * j + 1] = spread32((uint32_t)(a.w[j] >> 32));
  }
  reduce_wide(wide.data(), 2 * PW, phi, out);
}

static void mulx_mod(Poly& a, const Poly& phi) {
  uint64_t carry = 0;
  for (int j = 0; j < PW; ++j) {
    const uint64_t c = a.w[j] >> 63;
    a.w[j] = (a.w[j] << 1) | carry;
    carry = c;
  }
  if (bit(a.w, DEG)) for (int j = 0; j < PW; ++j) a.w[j] ^= phi.w[j];
}

// Berlekamp-Massey over the low output bits of MT19937(5489): the connection polynomial C(x) of the
// shortest recurrence; phi(x) = x^L C(1/x)
static void find_phi(Poly& phi) {
  const int n = 2 * DEG + 64;
  std::vector<uint8_t> s(n);
  uint32_t st[NW];
  st[0] = 5489u;
  for (int i = 1; i < NW; ++i) st[i] = 1812433253u * (st[i - 1] ^ (st[i - 1] >> 30)) + (uint32_t)i;
  for (int t = 0; t < n; t += NW) {
    uint32_t nb[NW];
    next_block_host(st, nb);
    std::memcpy(st, nb, sizeof(st));
    for (int i = 0; i < NW && t + i < n; ++i) s[t + i] = temper(st[i]) & 1u;
  }
  const int W = (n + 63) / 64 + 2;
  std::vector<uint64_t> C(W, 0), Bp(W, 0), T(W);
  std::vector<uint64_t> rev(W, 0);   // rev bit (n-1-t) = s[t]
  for (int t = 0; t < n; ++t)
    if (s[t]) rev[(n - 1 - t) >> 6] |= 1ull << ((n - 1 - t) & 63);
  C[0] = Bp[0] = 1;
  int L = 0, m = 1;
  for (int t = 0; t < n; ++t) {
    // d = s[t] ^ sum_{i=1..L} C_i s[t-i];  s[t-i] = rev bit (n-1-t+i)
    uint64_t acc = s[t];
    const int64_t base = n - 1 - t;        // rev index of s[t]; C bit i pairs with rev bit base + i
    for (int wi = 0; wi * 64 <= L; ++wi) {
      uint64_t cw = C[wi];
      if (wi == 0) cw &= ~1ull;             // i >= 1
      const int hi_bits = L - wi * 64 + 1;  // C bits [wi*64, L]
      if (hi_bits < 64) cw &= (1ull << hi_bits) - 1;
      if (!cw) continue;
      const int64_t o = base + (int64_t)wi * 64;
      const int64_t ow = o >> 6;
      const int ob = (int)(o & 63);
      uint64_t rw = ow < W ? rev[ow] >> ob : 0;
      if (ob && ow + 1 < W) rw |= rev[ow + 1] << (64 - ob);
      acc ^= (uint64_t)__builtin_parityll(cw & rw);
    }
    if (!(acc & 1u)) {
      ++m;
    } else if (2 * L <= t) {
      T = C;
      xor_shifted(C.data(), W, Bp.data(), W, m);
      L = t + 1 - L;
      Bp = T;
      m = 1;
    } else {
      xor_shifted(C.data(), W, Bp.data(), W, m);
      ++m;
    }
  }
  if (L != DEG) throw std::runtime_error("MT19937 characteristic polynomial: unexpected degree " + std::to_string(L));
  std::memset(phi.w, 0, sizeof(phi.w));
  for (int i = 0; i <= L; ++i)
    if (bit(C.data(), i)) phi.w[(L - i) >> 6] |= 1ull << ((L - i) & 63);
}

// q[0 .. k] ready (computed once, grown on demand)
static const Tables& jump_tables(int k) {
  std::lock_guard<std::mutex> g(tables_mutex());
  Tables& t = tables();
  if (!t.ready) {
    find_phi(t.phi);
    Poly p;
    std::memset(p.w, 0, sizeof(p.w));
    p.w[0] = 1;
    for (int b = 9; b >= 0; --b) {   // x^624, 624 = 0b1001110000
      Poly sq;
      sqr_mod(p, t.phi, sq);
      p = sq;
      if ((624 >> b) & 1) mulx_mod(p, t.phi);
    }
    t.q.push_back(p);
    t.ready = true;
  }
  if (k >= QMAX) throw std::runtime_error("MT19937 jump beyond 624 * 2^40 words");
  while ((int)t.q.size() <= k) {
    Poly sq;
    sqr_mod(t.q.back(), t.phi, sq);
    t.q.push_back(sq);
  }
  return t;
}

// window W -> p(F) W (host)
static void jump_host(const uint32_t* in, const Poly& p, uint32_t* out) {
  uint32_t buf[2 * NW];
  uint32_t acc[NW];
  std::memcpy(buf, in, NW * 4);
  std::memset(acc, 0, sizeof(acc));
  for (int blk = 0; blk * NW < DEG; ++blk) {
    for (int i = 0; i < NW; ++i) buf[NW + i] = buf[397 + i] ^ twist(buf[i], buf[i + 1]);
    for (int i = 0; i < NW; ++i) {
      const int k = blk * NW + i;
      if (k >= DEG) break;
      if (bit(p.w, k))
        for (int j = 0; j < NW; ++j) acc[j] ^= buf[i + j];
    }
    std::memmove(buf, buf + NW, NW * 4);
  }
  acc[0] = fix_first(acc[0], acc[396], acc[623]);
  std::memcpy(out, acc, NW * 4);
}

// ---------------------------------------------------------------- device kernels
constexpr int JUMP_THREADS = 640;   // mt_init_kernel
constexpr int GEN_THREADS = 256;

// buf[624 .. 1248) = the block after the window buf[0 .. 624) (three dependency phases)
template <int NT>
__device__ __forceinline__ void next_block_lds(uint32_t* buf, int t) {
#pragma unroll
  for (int ph = 0; ph < 3; ++ph) {
    const int lo = ph == 0 ? 0 : (ph == 1 ? 227 : 454), hi = ph == 0 ? 227 : (ph == 1 ? 454 : NW);
    for (int i = lo + t; i < hi; i += NT) buf[NW + i] = buf[397 + i] ^ twist(buf[i], buf[i + 1]);
    __syncthreads();
  }
}

struct KeyArg {
  uint32_t w[NW];
};

__global__ void __launch_bounds__(JUMP_THREADS) mt_init_kernel(KeyArg key, uint32_t* win) {
  for (int i = threadIdx.x; i < NW; i += JUMP_THREADS) win[i] = key.w[i];
}

// dst[i] = Q (src[i]) for the n windows of 624 words: workgroup (i, g) regenerates the window sequence of
// job i and accumulates its share [JP_W g, JP_W (g + 1)) of the 624 words.  Q comes as the positions of
// its set coefficients, per block of 624 steps, each block's list padded to a multiple of 8 with a sentinel
// (JP_ZERO: it reads a zero region).  Lane l of the share XORs window word buf[k + w0 + l] of every listed
// k: eight positions per two broadcast LDS reads, their reads in flight together, consecutive lanes on
// consecutive banks.  (Measured per jump: a scalar walk of the coefficient bits by every wave 536 us; one
// workgroup per jump, two words per lane 255 us -- LDS-bandwidth bound, 780 KB of window reads per block.)
constexpr int JP_THREADS = 256;
constexpr int JP_SPLIT = 8;                // workgroups per jump
constexpr int JP_W = NW / JP_SPLIT;        // 78 words each
constexpr int JP_ZERO = 2 * NW;            // sentinel position: buf[JP_ZERO ..] holds zeros
static_assert(NW % JP_SPLIT == 0, "share");
__global__ void __launch_bounds__(JP_THREADS) mt_jump_kernel(const uint32_t* srcs, uint32_t* dsts, const int* pos,
                                                              const int* bptr, int npos) {
  __shared__ uint32_t buf[2 * NW + 2 * NW];
  __shared__ uint32_t fixw[2];
  extern __shared__ int sp[];
  const int t = threadIdx.x, g = blockIdx.y;
  const uint32_t* src = srcs + (size_t)blockIdx.x * NW;
  uint32_t* dst = dsts + (size_t)blockIdx.x * NW;
  for (int i = t; i < NW; i += JP_THREADS) buf[i] = src[i];
  for (int i = t; i < 2 * NW; i += JP_THREADS) buf[JP_ZERO + i] = 0u;
  for (int i = t; i < npos; i += JP_THREADS) sp[i] = pos[i];
  __syncthreads();
  uint32_t a = 0;
  // this lane's window word: the share's JP_W words; share 0 also follows words 396 and 623 (lanes JP_W,
  // JP_W + 1), which word 0's low bits are recomputed from
  const int w = t < JP_W ? g * JP_W + t : (g == 0 && t == JP_W ? 396 : (g == 0 && t == JP_W + 1 ? 623 : 0));
  for (int blk = 0; blk * NW < DEG; ++blk) {
    next_block_lds<JP_THREADS>(buf, t);
    const int q0 = bptr[blk], q1 = bptr[blk + 1];
    if (t < 128) {
      for (int q = q0; q < q1; q += 8) {
        const int4 k0 = *reinterpret_cast<const int4*>(sp + q);
        const int4 k1 = *reinterpret_cast<const int4*>(sp + q + 4);
        const uint32_t x0 = buf[k0.x + w], x1 = buf[k0.y + w], x2 = buf[k0.z + w], x3 = buf[k0.w + w];
        const uint32_t x4 = buf[k1.x + w], x5 = buf[k1.y + w], x6 = buf[k1.z + w], x7 = buf[k1.w + w];
        a ^= ((x0 ^ x1) ^ (x2 ^ x3)) ^ ((x4 ^ x5) ^ (x6 ^ x7));
      }
    }
    __syncthreads();
    for (int i = t; i < NW; i += JP_THREADS) buf[i] = buf[NW + i];
    __syncthreads();
  }
  if (g == 0 && (t == JP_W || t == JP_W + 1)) fixw[t - JP_W] = a;
  __syncthreads();
  if (t < JP_W) dst[w] = (g == 0 && t == 0) ? fix_first(a, fixw[0], fixw[1]) : a;
}

// segment s = seg0 + workgroup (window win[workgroup]): blocks [s * SEG_BLOCKS, ...) of the device part of the
// stream, tempered into out[L + 624 blk ..] (out nullable: only the end state wanted); segment 0 also writes
// the L = 624 - pos words left in the caller's block; block bq's raw words -> final_raw
__global__ void __launch_bounds__(GEN_THREADS) mt_gen_kernel(const uint32_t* win, int seg0, int64_t nblocks, int pos,
                                                              uint32_t* out, int64_t bq, uint32_t* final_raw) {
  __shared__ uint32_t buf[2 * NW];
  const int t = threadIdx.x;
  const int64_t s = seg0 + (int64_t)blockIdx.x;
  const int L = NW - pos;
  for (int i = t; i < NW; i += GEN_THREADS) buf[i] = win[(size_t)blockIdx.x * NW + i];
  __syncthreads();
  if (s == 0 && out)
    for (int i = t; i < L; i += GEN_THREADS) out[i] = temper(buf[pos + i]);
  const int64_t b0 = s * SEG_BLOCKS, b1 = min(b0 + SEG_BLOCKS, nblocks);
  for (int64_t blk = b0; blk < b1; ++blk) {
    next_block_lds<GEN_THREADS>(buf, t);
    for (int i = t; i < NW; i += GEN_THREADS) {
      const uint32_t x = buf[NW + i];
      if (out) out[L + blk * NW + i] = temper(x);
      if (blk == bq) final_raw[i] = x;
    }
    __syncthreads();
    for (int i = t; i < NW; i += GEN_THREADS) buf[i] = buf[NW + i];
    __syncthreads();
  }
}

__device__ __forceinline__ int64_t last_le(const int64_t* a, int64_t n, int64_t v) {   // last i < n: a[i] <= v
  int64_t lo = 0, hi = n;
  while (hi - lo > 1) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid] <= v) lo = mid;
    else hi = mid;
  }
  return lo;
}

// workgroups (x, bi): batch bi's entries, grid-stride over x; the batch's row offsets staged in LDS.  Batch
// bi's doubles are [bi*B + ebase[bi], ...): B row sparsities, then the entries' uniforms in batch order
// (data_reader.py:120 then :130 row by row)
constexpr int RK_THREADS = 256;
constexpr int RK_BLOCKS = 64;    // workgroups per batch
__global__ void __launch_bounds__(RK_THREADS) recip_keep_kernel(const uint32_t* words, const int64_t* boff,
                                                                 const int64_t* ebase, int B, double s0, double s1,
                                                                 uint8_t* keep) {
  extern __shared__ int64_t off[];
  const int64_t bi = blockIdx.y;
  for (int i = threadIdx.x; i <= B; i += RK_THREADS) off[i] = boff[bi * (B + 1) + i];
  __syncthreads();
  const int64_t eb = ebase[bi], E = off[B];
  const int64_t d0 = bi * (int64_t)B + eb;
  for (int64_t e = (int64_t)blockIdx.x * RK_THREADS + threadIdx.x; e < E; e += (int64_t)RK_BLOCKS * RK_THREADS) {
    const int64_t b = last_le(off, B, e);
    const int64_t dr = d0 + b, de = d0 + B + e;
    const double s = s0 + (s1 - s0) * to_double(words[2 * dr], words[2 * dr + 1]);
    const double cut = (1.0 - s) / ((1.0 - s) + s);
    keep[eb + e] = to_double(words[2 * de], words[2 * de + 1]) >= cut ? 1 : 0;
  }
}

// ---------------------------------------------------------------- plan shared by host and device paths
struct Plan {
  int64_t words;     // words consumed
  int L;             // words left in the caller's block (624 - pos)
  int64_t nblocks;   // device blocks generated (the one holding the last word included)
  int64_t bq;        // block holding the last consumed word (-1: it is in the caller's block)
  int S;             // segments
  int rounds;        // doubling-tree rounds
};

static Plan make_plan(int pos, int64_t words) {
  OCF_CHECK(pos >= 0 && pos <= NW, "MT19937 state: pos must be in [0, 624]");
  OCF_CHECK(words >= 0, "MT19937: negative draw count");
  Plan p;
  p.words = words;
  p.L = NW - pos;
  if (words <= p.L) {
    p.nblocks = 0;
    p.bq = -1;
  } else {
    p.bq = (words - p.L - 1) / NW;
    p.nblocks = p.bq + 1;
  }
  p.S = (int)std::max<int64_t>(1, (p.nblocks + SEG_BLOCKS - 1) / SEG_BLOCKS);
  p.rounds = 0;
  while ((1 << p.rounds) < p.S) ++p.rounds;
  return p;
}

static void end_state(const Plan& p, const uint32_t* key_in, int pos_in, const uint32_t* final_raw, uint32_t* key_out,
                      int32_t* pos_out) {
  if (p.bq < 0) {
    if (key_out != key_in) std::memcpy(key_out, key_in, NW * 4);
    *pos_out = pos_in + (int)p.words;
  } else {
    std::memcpy(key_out, final_raw, NW * 4);
    *pos_out = (int)((p.words - p.L - 1) % NW) + 1;
  }
}

// a jump polynomial as the device kernel reads it: set-coefficient positions, block by block (position
// k of block b stored as k - 624 b), each block padded to a multiple of 8 with JP_ZERO
struct JumpList {
  std::vector<int> pos;
  int bptr[34];
};

static JumpList jump_list(const Poly& q) {
  JumpList L;
  const int nblk = (DEG + NW - 1) / NW;
  for (int b = 0; b < nblk; ++b) {
    L.bptr[b] = (int)L.pos.size();
    for (int k = b * NW; k < std::min((b + 1) * NW, DEG); ++k)
      if (bit(q.w, k)) L.pos.push_back(k - b * NW);
    while (L.pos.size() % 8) L.pos.push_back(JP_ZERO);
  }
  for (int b = nblk; b < 34; ++b) L.bptr[b] = (int)L.pos.size();
  return L;
}

struct DevJump {
  const int* pos;
  const int* bptr;
  int npos;
};

struct DevTables {
  std::vector<DevJump> r;   // r[i]: Q_{SEG_LOG + i}
};

static std::vector<DevJump> device_jump_lists(int rounds) {
  static std::mutex mx;
  static std::vector<DevTables> per_dev;
  int dev = 0;
  OCF_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> g(mx);
  if ((int)per_dev.size() <= dev) per_dev.resize(dev + 1);
  DevTables& d = per_dev[dev];
  if ((int)d.r.size() < rounds) {
    const Tables& t = jump_tables(SEG_LOG + rounds - 1);
    for (int i = (int)d.r.size(); i < rounds; ++i) {
      const JumpList L = jump_list(t.q[SEG_LOG + i]);
      int* buf = nullptr;   // one allocation per polynomial, kept for the process (a few tens of KB)
      OCF_HIP(hipMalloc(&buf, (L.pos.size() + 34) * sizeof(int)));
      OCF_HIP(hipMemcpy(buf, L.pos.data(), L.pos.size() * sizeof(int), hipMemcpyHostToDevice));
      OCF_HIP(hipMemcpy(buf + L.pos.size(), L.bptr, 34 * sizeof(int), hipMemcpyHostToDevice));
      d.r.push_back(DevJump{buf, buf + L.pos.size(), (int)L.pos.size()});
    }
  }
  return std::vector<DevJump>(d.r.begin(), d.r.begin() + rounds);
}

static inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

struct WsLayout {
  size_t words, win, fin, total;
};

static WsLayout ws_layout(const Plan& p) {
  WsLayout w;
  w.words = 0;
  const size_t nwords = (size_t)p.L + (size_t)p.nblocks * NW;
  w.win = align256(nwords * 4);
  w.fin = w.win + align256((size_t)std::max(p.S, 2) * NW * 4);
  w.total = w.fin + align256(NW * 4);
  return w;
}

}  // namespace mt
}  // namespace ocf

using namespace ocf;
using namespace ocf::mt;

extern "C" int64_t ocf_recip_keep_workspace(int nb, int B, int64_t n_entries, int pos) {
  try {
    if (nb < 0 || B < 0 || n_entries < 0) return -1;
    const Plan p = make_plan(pos, 2 * ((int64_t)nb * B + n_entries));
    return (int64_t)ws_layout(p).total;
  } catch (const std::exception& e) {
    set_error(e.what());
    return -1;
  }
}

extern "C" int ocf_recip_keep(OcfRecipKeepArgs* a, void* stream) {
  OCF_TRY_BEGIN
  OCF_CHECK(a && a->nb >= 0 && a->B >= 0 && a->n_entries >= 0, "ocf_recip_keep: sizes");
  OCF_CHECK(a->n_entries < ((int64_t)1 << 40), "ocf_recip_keep: too many entries");
  hipStream_t s = (hipStream_t)stream;
  const int64_t draws = (int64_t)a->nb * a->B + a->n_entries;
  const Plan p = make_plan(a->pos, 2 * draws);
  const WsLayout w = ws_layout(p);
  OCF_CHECK(a->workspace && a->workspace_bytes >= (int64_t)w.total, "ocf_recip_keep: workspace too small");
  OCF_CHECK(!a->keep || (a->boff && a->ebase), "ocf_recip_keep: keep needs boff and ebase");
  if (p.words == 0) return 0;
  char* ws = reinterpret_cast<char*>(a->workspace);
  uint32_t* words = reinterpret_cast<uint32_t*>(ws);
  uint32_t* win = reinterpret_cast<uint32_t*>(ws + w.win);
  uint32_t* fin = reinterpret_cast<uint32_t*>(ws + w.fin);
  KeyArg key;
  std::memcpy(key.w, a->key, sizeof(key.w));
  hipLaunchKernelGGL(mt_init_kernel, dim3(1), dim3(JUMP_THREADS), 0, s, key, win);
  OCF_HIP(hipGetLastError());
  const bool stream_out = a->keep || a->doubles;
  if (stream_out) {
    // every segment: windows [2^r, 2^(r+1)) from windows [0, 2^r) by x^(2^r segments), r < rounds
    if (p.nblocks > 0) {
      const std::vector<DevJump> q = device_jump_lists(p.rounds);
      for (int r = 0; r < p.rounds; ++r) {
        const int half = 1 << r;
        const int jobs = std::min(half, p.S - half);
        hipLaunchKernelGGL(mt_jump_kernel, dim3(jobs, JP_SPLIT), dim3(JP_THREADS), q[r].npos * sizeof(int), s, win,
                           win + (size_t)half * NW, q[r].pos, q[r].bptr, q[r].npos);
        OCF_HIP(hipGetLastError());
      }
    }
    hipLaunchKernelGGL(mt_gen_kernel, dim3(p.S), dim3(GEN_THREADS), 0, s, win, 0, p.nblocks, a->pos, words, p.bq, fin);
    OCF_HIP(hipGetLastError());
  } else if (p.bq >= 0) {
    // only the end state (data_sparsity [1, 1]): jump straight to the segment holding the last word
    // (one jump per set bit of its index, ping-pong between two windows), generate that segment alone
    const int64_t sq = p.bq / SEG_BLOCKS;
    int top = 0;
    while ((sq >> top) > 1) ++top;
    const std::vector<DevJump> q = device_jump_lists(sq ? top + 1 : 0);
    int cur = 0;
    for (int k = 0; sq && k <= top; ++k)
      if ((sq >> k) & 1) {
        hipLaunchKernelGGL(mt_jump_kernel, dim3(1, JP_SPLIT), dim3(JP_THREADS), q[k].npos * sizeof(int), s,
                           win + (size_t)cur * NW, win + (size_t)(cur ^ 1) * NW, q[k].pos, q[k].bptr, q[k].npos);
        OCF_HIP(hipGetLastError());
        cur ^= 1;
      }
    hipLaunchKernelGGL(mt_gen_kernel, dim3(1), dim3(GEN_THREADS), 0, s, win + (size_t)cur * NW, (int)sq, p.nblocks,
                       a->pos, (uint32_t*)nullptr, p.bq, fin);
    OCF_HIP(hipGetLastError());
  }
  if (a->keep && a->n_entries > 0) {
    OCF_CHECK(a->B <= 16384, "ocf_recip_keep: B <= 16384 (the batch's row offsets are staged in LDS)");
    hipLaunchKernelGGL(recip_keep_kernel, dim3(RK_BLOCKS, a->nb), dim3(RK_THREADS), (size_t)(a->B + 1) * 8, s, words,
                       a->boff, a->ebase, a->B, a->s0, a->s1, a->keep);
    OCF_HIP(hipGetLastError());
  }
  if (a->doubles) {   // the raw uniform stream (tests): words -> doubles on the host side of the copy
    std::vector<uint32_t> h((size_t)p.words);
    OCF_HIP(hipMemcpyAsync(h.data(), words, (size_t)p.words * 4, hipMemcpyDeviceToHost, s));
    OCF_HIP(hipStreamSynchronize(s));
    for (int64_t j = 0; j < draws; ++j) a->doubles[j] = to_double(h[2 * j], h[2 * j + 1]);
  }
  uint32_t raw[NW];
  if (p.bq >= 0) OCF_HIP(hipMemcpyAsync(raw, fin, NW * 4, hipMemcpyDeviceToHost, s));
  // always: the keep flags (and the workspace the caller frees next) must be complete when the call
  // returns, also when every draw fits in the current 624-word block (no end-state copy to wait for)
  OCF_HIP(hipStreamSynchronize(s));
  end_state(p, a->key, a->pos, raw, a->key, &a->pos);
  OCF_TRY_END
}

// ---- host twin (CPU tests): the same plan, segment windows by the same doubling tree of jumps
extern "C" int ocf_mt_host_random_sample(uint32_t* key, int32_t* pos, int64_t n, double* out) {
  OCF_TRY_BEGIN
  OCF_CHECK(key && pos && (out || n == 0), "ocf_mt_host_random_sample: null pointer");
  const Plan p = make_plan(*pos, 2 * n);
  if (p.words == 0) return 0;
  std::vector<uint32_t> words((size_t)p.L + (size_t)p.nblocks * NW);
  std::vector<uint32_t> win((size_t)p.S * NW);
  std::memcpy(win.data(), key, NW * 4);
  if (p.nblocks > 0) {
    const Tables& t = jump_tables(SEG_LOG + std::max(p.rounds, 1) - 1);
    for (int r = 0; r < p.rounds; ++r) {
      const int half = 1 << r;
      for (int i = 0; i < half && i + half < p.S; ++i)
        jump_host(&win[(size_t)i * NW], t.q[SEG_LOG + r], &win[(size_t)(i + half) * NW]);
    }
  }
  uint32_t fin[NW];
  for (int i = 0; i < p.L; ++i) words[i] = temper(key[*pos + i]);
  for (int sgm = 0; sgm < p.S; ++sgm) {
    uint32_t cur[NW], nxt[NW];
    std::memcpy(cur, &win[(size_t)sgm * NW], NW * 4);
    const int64_t b0 = (int64_t)sgm * SEG_BLOCKS, b1 = std::min<int64_t>(b0 + SEG_BLOCKS, p.nblocks);
    for (int64_t blk = b0; blk < b1; ++blk) {
      next_block_host(cur, nxt);
      for (int i = 0; i < NW; ++i) words[p.L + blk * NW + i] = temper(nxt[i]);
      if (blk == p.bq) std::memcpy(fin, nxt, NW * 4);
      std::memcpy(cur, nxt, NW * 4);
    }
  }
  for (int64_t j = 0; j < n; ++j) out[j] = to_double(words[2 * j], words[2 * j + 1]);
  end_state(p, key, *pos, fin, key, pos);
  OCF_TRY_END
}

extern "C" int ocf_mt_host_jump(const uint32_t* key_in, int64_t n_blocks, uint32_t* key_out) {
  OCF_TRY_BEGIN
  OCF_CHECK(key_in && key_out && n_blocks >= 0, "ocf_mt_host_jump: arguments");
  int top = 0;
  while (top < 63 && (n_blocks >> (top + 1))) ++top;
  const Tables& t = jump_tables(top);
  uint32_t cur[NW];
  std::memcpy(cur, key_in, NW * 4);
  for (int k = 0; k <= top; ++k)
    if ((n_blocks >> k) & 1) {
      uint32_t nx[NW];
      jump_host(cur, t.q[k], nx);
      std::memcpy(cur, nx, NW * 4);
    }
  std::memcpy(key_out, cur, NW * 4);
  OCF_TRY_END
}
