// MT19937 jump-ahead (host): the state after J more words without generating them.
//
// The generator is linear over GF(2): the 19937-bit state advances by one word through a
// fixed matrix T with a primitive characteristic polynomial phi (degree 19937).  Then
// T^J = p(T) with p(x) = x^J mod phi, and p(T) s = XOR of T^i s over the set bits i of p.
// With the word sequence y_k of state s (y_0..y_623 = the window, y_{k+624} = y_{k+397} ^
// twist(y_k, y_{k+1})), T^i s is the window y_i..y_{i+623}, so word w of the jumped window
// is the XOR of y_{i+w} over the set bits i of p (only the top bit of word 0 is state; the
// caller asks for the window one word early when it needs that word whole).
//
//   phi: Berlekamp-Massey on 2 x 19937 output bits of any seeded generator, embedded as a
//        constant (mt_phi.h, tools/gen_mt_phi.cpp) and re-derived by the self-test;
//   p:   x^(J mod 624) by shifts times cached x^(624 2^k) over the set bits of J div 624,
//        products by carry-less multiplication with Barrett reduction (below);
//   numpy's state (key[624], pos) is the raw block holding the next word plus the offset.
//
// Used by the parity sampler to start many generators along one numpy / CPython stream.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <vector>
#if defined(__x86_64__)
#include <immintrin.h>
#endif

#include "common.h"
#if RSAMD_GEN_PHI  // tools/gen_mt_phi.cpp: writes the constants below from charpoly_bm
constexpr uint64_t kPhiWords[312] = {};
constexpr uint64_t kMuWords[312] = {};
constexpr int kPow2Embed = 0;
constexpr uint64_t kPow2Words[1][312] = {};
#else
#include "mt_phi.h"
#endif

namespace {

constexpr int kN = 624;
constexpr int kM = 397;
constexpr int kDeg = 19937;
constexpr int kWords = (kDeg + 64) / 64 + 1;  // polynomial words (degree <= kDeg)

inline uint32_t twist(uint32_t a, uint32_t b, uint32_t m) {
  const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
  return m ^ (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
}
inline uint32_t temper(uint32_t y) {
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

// GF(2)[x] polynomial, bit i = coefficient of x^i
using Poly = std::vector<uint64_t>;

inline int getbit(const Poly &p, int64_t i) { return static_cast<int>((p[i >> 6] >> (i & 63)) & 1u); }
inline void flipbit(Poly &p, int64_t i) { p[i >> 6] ^= 1ull << (i & 63); }

// p ^= q << s (words of q beyond p's size must be zero: degrees are bounded by the caller)
void xor_shifted(Poly &p, const Poly &q, int64_t s) {
  const int64_t ws = s >> 6;
  const int bs = static_cast<int>(s & 63);
  const int64_t np = static_cast<int64_t>(p.size());
  for (int64_t i = 0; i < static_cast<int64_t>(q.size()); ++i) {
    const uint64_t v = q[i];
    if (!v) continue;
    if (i + ws < np) p[i + ws] ^= v << bs;
    if (bs && i + ws + 1 < np) p[i + ws + 1] ^= v >> (64 - bs);
  }
}

// phi by Berlekamp-Massey (~50 ms): the generator of mt_phi.h and the self-test's check of it
const Poly &charpoly_bm() {
  static Poly phi;
  static std::once_flag once;
  std::call_once(once, [] {
    // bit 0 of successive outputs of a seeded generator (any seed: phi is primitive)
    const int64_t nb = 2 * kDeg + 4096;
    std::vector<uint8_t> s(static_cast<size_t>(nb));
    uint32_t mt[kN];
    mt[0] = 5489u;
    for (int i = 1; i < kN; ++i)
      mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + static_cast<uint32_t>(i);
    int pos = kN;
    for (int64_t t = 0; t < nb; ++t) {
      if (pos >= kN) {
        for (int i = 0; i < kN; ++i) mt[i] = twist(mt[i], mt[(i + 1) % kN], mt[(i + kM) % kN]);
        pos = 0;
      }
      s[static_cast<size_t>(t)] = static_cast<uint8_t>(temper(mt[pos++]) & 1u);
    }
    // Berlekamp-Massey over GF(2): C(x) = 1 + c1 x + ... + cL x^L, s_n = sum c_i s_{n-i}
    const int64_t nbm = 2 * kDeg;
    Poly C(2 * kWords, 0), B(2 * kWords, 0), T;
    C[0] = B[0] = 1;
    int64_t L = 0, m = 1;
    // reversed sequence bits, packed: bit j of rs = s_{nbm - 1 - j}
    Poly rs((nbm + 64) / 64 + 2, 0);
    for (int64_t j = 0; j < nbm; ++j)
      if (s[static_cast<size_t>(nbm - 1 - j)]) rs[j >> 6] |= 1ull << (j & 63);
    auto window = [&](int64_t bit) -> uint64_t {  // 64 bits of rs from `bit`
      const int64_t w = bit >> 6;
      const int b = static_cast<int>(bit & 63);
      uint64_t lo = rs[w] >> b;
      if (b) lo |= rs[w + 1] << (64 - b);
      return lo;
    };
    for (int64_t n = 0; n < nbm; ++n) {
      // d = sum_{i=0..L} c_i s_{n-i}; s_{n-i} = rs bit (nbm - 1 - n + i)
      uint64_t acc = 0;
      const int64_t base = nbm - 1 - n;
      for (int64_t w = 0; w <= (L >> 6); ++w) {
        uint64_t cw = C[w];
        if (w == (L >> 6)) {
          const int keep = static_cast<int>(L & 63) + 1;
          if (keep < 64) cw &= (1ull << keep) - 1;
        }
        if (cw) acc ^= cw & window(base + 64 * w);
      }
      const int d = __builtin_parityll(acc);
      if (!d) {
        ++m;
      } else if (2 * L <= n) {
        T = C;
        xor_shifted(C, B, m);
        L = n + 1 - L;
        B = T;
        m = 1;
      } else {
        xor_shifted(C, B, m);
        ++m;
      }
    }
    // C is the reciprocal of phi: phi(x) = x^L C(1/x)
    phi.assign(kWords, 0);
    for (int64_t i = 0; i <= L; ++i)
      if (getbit(C, i)) flipbit(phi, L - i);
    (void)T;
  });
  return phi;
}

// phi from mt_phi.h (the process never pays for Berlekamp-Massey)
const Poly &charpoly() {
  static const Poly phi = [] {
    Poly p(kWords, 0);
    for (int i = 0; i < 312; ++i) p[static_cast<size_t>(i)] = kPhiWords[i];
    return p;
  }();
  return phi;
}

// ---- fast arithmetic mod phi: carry-less products (PCLMULQDQ) and Barrett reduction ----------
// A residue is kR = 312 words (degree < kDeg = 19937 needs 19937 bits).  Over GF(2) Barrett
// reduction is exact: for deg a < 2 kDeg, a div phi = ((a div x^kDeg) * mu) div x^kDeg with
// mu = x^(2 kDeg) div phi, so a mod phi = (a + q phi) mod x^kDeg.  A product mod phi is then
// three carry-less products (one of them only its low half): ~0.2 ms, against ~13 ms for the
// bit-serial shifted-XOR form below (kept as the reference the self-test compares with).
constexpr int kR = (kDeg + 63) / 64;  // 312
using u64 = uint64_t;

inline void clmul_portable(u64 a, u64 b, u64 &lo, u64 &hi) {
  u64 l = 0, h = 0;
  for (int i = 0; i < 64; ++i)
    if ((b >> i) & 1u) {
      l ^= a << i;
      if (i) h ^= a >> (64 - i);
    }
  lo = l;
  hi = h;
}

#if defined(__x86_64__)
__attribute__((target("pclmul,sse4.1"))) void mul_words_clmul(const u64 *a, int na, const u64 *b,
                                                             int nb, u64 *out, int nout) {
  // out[0 .. nout) = low nout words of a * b (out zeroed by the caller)
  for (int i = 0; i < na; ++i) {
    if (!a[i]) continue;
    const __m128i av = _mm_set_epi64x(0, static_cast<long long>(a[i]));
    const int jmax = std::min(nb, nout - i);
    for (int j = 0; j < jmax; ++j) {
      const __m128i p = _mm_clmulepi64_si128(av, _mm_set_epi64x(0, static_cast<long long>(b[j])), 0x00);
      out[i + j] ^= static_cast<u64>(_mm_cvtsi128_si64(p));
      if (i + j + 1 < nout) out[i + j + 1] ^= static_cast<u64>(_mm_extract_epi64(p, 1));
    }
  }
}
bool have_clmul() {
  static const bool v = __builtin_cpu_supports("pclmul") && __builtin_cpu_supports("sse4.1");
  return v;
}
#else
void mul_words_clmul(const u64 *, int, const u64 *, int, u64 *, int) {}
bool have_clmul() { return false; }
#endif

void mul_words(const u64 *a, int na, const u64 *b, int nb, u64 *out, int nout) {
  std::memset(out, 0, sizeof(u64) * static_cast<size_t>(nout));
  if (have_clmul()) {
    mul_words_clmul(a, na, b, nb, out, nout);
    return;
  }
  for (int i = 0; i < na; ++i) {
    if (!a[i]) continue;
    for (int j = 0; j < nb && i + j < nout; ++j) {
      u64 lo, hi;
      clmul_portable(a[i], b[j], lo, hi);
      out[i + j] ^= lo;
      if (i + j + 1 < nout) out[i + j + 1] ^= hi;
    }
  }
}

// out[0 .. nout) = (a >> s) for a of na words
void shr_words(const u64 *a, int na, int64_t s, u64 *out, int nout) {
  const int64_t ws = s >> 6;
  const int bs = static_cast<int>(s & 63);
  for (int k = 0; k < nout; ++k) {
    const int64_t i = k + ws;
    u64 v = i < na ? a[i] >> bs : 0;
    if (bs && i + 1 < na) v |= a[i + 1] << (64 - bs);
    out[k] = v;
  }
}

struct Barrett {
  u64 phi[kR], mu[kR];
};

// mu = x^(2 kDeg) div phi by long division (the generator of mt_phi.h and the self-test)
Poly barrett_mu_bm(const Poly &phi) {
  Poly rem(2 * kR + 2, 0), mu(kR + 1, 0);
  flipbit(rem, 2 * static_cast<int64_t>(kDeg));
  for (int64_t i = 2 * static_cast<int64_t>(kDeg); i >= kDeg; --i)
    if (getbit(rem, i)) {
      flipbit(mu, i - kDeg);
      xor_shifted(rem, phi, i - kDeg);
    }
  mu.resize(kR);
  return mu;
}

const Barrett &barrett() {
  static const Barrett B = [] {
    Barrett b;
    for (int i = 0; i < kR; ++i) {
      b.phi[i] = kPhiWords[i];
      b.mu[i] = kMuWords[i];
    }
    return b;
  }();
  return B;
}

// r (kR words, degree < kDeg) = a mod phi for a product a of 2 kR words (degree < 2 kDeg - 1)
void barrett_reduce(const u64 *a, u64 *r) {
  const Barrett &B = barrett();
  u64 h[kR], t[2 * kR], q[kR], qp[kR];
  shr_words(a, 2 * kR, kDeg, h, kR);
  mul_words(h, kR, B.mu, kR, t, 2 * kR);
  shr_words(t, 2 * kR, kDeg, q, kR);
  mul_words(q, kR, B.phi, kR, qp, kR);  // low kR words of q phi
  for (int i = 0; i < kR; ++i) r[i] = a[i] ^ qp[i];
  r[kR - 1] &= (u64(1) << (kDeg - 64 * (kR - 1))) - 1u;
}

void mulmod_fast(const u64 *a, const u64 *b, u64 *r) {
  u64 p[2 * kR];
  mul_words(a, kR, b, kR, p, 2 * kR);
  barrett_reduce(p, r);
}

void sqrmod_fast(const u64 *a, u64 *r) {
  u64 p[2 * kR];
  std::memset(p, 0, sizeof(p));
  for (int i = 0; i < kR; ++i) {  // squaring spreads the bits: no cross terms over GF(2)
    u64 lo, hi;
    if (have_clmul()) {
      mul_words(a + i, 1, a + i, 1, p + 2 * i, 2);
      continue;
    }
    clmul_portable(a[i], a[i], lo, hi);
    p[2 * i] = lo;
    p[2 * i + 1] = hi;
  }
  barrett_reduce(p, r);
}

// x^(624 * 2^k) mod phi for k < 40: the first kPow2Embed from mt_phi.h (checked by the
// self-test), the rest built on demand (each a squaring of the one before): x^(624 JB) is the
// product over JB's set bits
constexpr int kPow2 = 40;
std::mutex g_pow2_mu;
// x^624 mod phi by times-x steps
std::vector<u64> x624() {
  std::vector<u64> p(kR, 0);
  p[0] = 1;
  for (int s = 0; s < kN; ++s) {
    u64 carry = 0;
    for (int i = 0; i < kR; ++i) {
      const u64 v = p[i];
      p[i] = (v << 1) | carry;
      carry = v >> 63;
    }
    if ((p[kR - 1] >> (kDeg - 64 * (kR - 1))) & 1u)
      for (int i = 0; i < kR; ++i) p[i] ^= kPhiWords[i];
  }
  return p;
}
const std::vector<u64> &pow2(int k) {
  static std::vector<std::vector<u64>> T;
  std::lock_guard<std::mutex> g(g_pow2_mu);
  if (T.empty()) {
    T.reserve(kPow2);  // no reallocation: references handed out stay valid
    for (int e = 0; e < kPow2Embed && e < kPow2; ++e) T.emplace_back(kPow2Words[e], kPow2Words[e] + kR);
  }
  if (T.empty()) {
    std::vector<u64> p(kR, 0);
    p[0] = 1;
    for (int s = 0; s < kN; ++s) {  // x^624 by times-x steps
      u64 carry = 0;
      for (int i = 0; i < kR; ++i) {
        const u64 v = p[i];
        p[i] = (v << 1) | carry;
        carry = v >> 63;
      }
      if ((p[kR - 1] >> (kDeg - 64 * (kR - 1))) & 1u)
        for (int i = 0; i < kR; ++i) p[i] ^= kPhiWords[i];
    }
    T.push_back(p);
  }
  while (static_cast<int>(T.size()) <= k) {
    std::vector<u64> q(kR, 0);
    sqrmod_fast(T.back().data(), q.data());
    T.push_back(q);
  }
  return T[static_cast<size_t>(k)];
}

// r = r^2 mod phi (deg r < kDeg)
void square_mod(Poly &r, const Poly &phi) {
  Poly sq(2 * kWords + 2, 0);
  for (int64_t i = 0; i < kWords; ++i) {
    const uint64_t v = r[i];
    if (!v) continue;
    for (int b = 0; b < 64; ++b)
      if ((v >> b) & 1u) flipbit(sq, 2 * (64 * i + b));
  }
  for (int64_t i = 2 * (kDeg - 1); i >= kDeg; --i)
    if (getbit(sq, i)) xor_shifted(sq, phi, i - kDeg);
  for (int64_t i = 0; i < kWords; ++i) r[i] = sq[i];
}

// r = r * x mod phi
void times_x_mod(Poly &r, const Poly &phi) {
  uint64_t carry = 0;
  for (int64_t i = 0; i < kWords; ++i) {
    const uint64_t v = r[i];
    r[i] = (v << 1) | carry;
    carry = v >> 63;
  }
  if (getbit(r, kDeg))
    for (int64_t i = 0; i < kWords; ++i) r[i] ^= phi[i];
}

}  // namespace

namespace rs {

void mt_jump_poly_slow(uint64_t J, std::vector<uint64_t> &out);

namespace {
std::vector<uint64_t> widen(const u64 *r) {
  std::vector<uint64_t> v(kWords, 0);
  std::memcpy(v.data(), r, sizeof(u64) * kR);
  return v;
}
void narrow(const std::vector<uint64_t> &p, u64 *r) {
  std::memset(r, 0, sizeof(u64) * kR);
  std::memcpy(r, p.data(), sizeof(u64) * std::min<size_t>(kR, p.size()));
}
}  // namespace

// x^J mod phi as little-endian 64-bit words (kDeg bits); J >= 0: x^(J mod 624) by shifts, times
// the cached x^(624 2^k) over the set bits of J div 624 (a handful of products instead of 64
// squarings)
void mt_jump_poly(uint64_t J, std::vector<uint64_t> &out) {
  if ((J / kN) >> kPow2) {  // beyond the cached powers (no caller comes near)
    mt_jump_poly_slow(J, out);
    return;
  }
  const Barrett &B = barrett();
  u64 r[kR] = {}, t[kR];
  r[0] = 1;
  for (uint64_t s = 0; s < J % kN; ++s) {
    u64 carry = 0;
    for (int i = 0; i < kR; ++i) {
      const u64 v = r[i];
      r[i] = (v << 1) | carry;
      carry = v >> 63;
    }
    if ((r[kR - 1] >> (kDeg - 64 * (kR - 1))) & 1u)
      for (int i = 0; i < kR; ++i) r[i] ^= B.phi[i];
  }
  const uint64_t q = J / kN;
  for (int k = 0; k < kPow2; ++k)
    if ((q >> k) & 1u) {
      mulmod_fast(r, pow2(k).data(), t);
      std::memcpy(r, t, sizeof(t));
    }
  out = widen(r);
}

// p = p^2 mod phi (x^J -> x^(2J))
void mt_poly_square(std::vector<uint64_t> &p) {
  u64 a[kR], r[kR];
  narrow(p, a);
  sqrmod_fast(a, r);
  p = widen(r);
}

// r = a * b mod phi (x^A, x^B -> x^(A+B))
void mt_poly_mulmod(const std::vector<uint64_t> &a, const std::vector<uint64_t> &b,
                    std::vector<uint64_t> &r) {
  u64 x[kR], y[kR], z[kR];
  narrow(a, x);
  narrow(b, y);
  mulmod_fast(x, y, z);
  r = widen(z);
}

// the bit-serial reference forms (self-test only)
void mt_jump_poly_slow(uint64_t J, std::vector<uint64_t> &out) {
  const Poly &phi = charpoly();
  Poly r(kWords, 0);
  r[0] = 1;
  for (int b = 63; b >= 0; --b) {
    square_mod(r, phi);
    if ((J >> b) & 1u) times_x_mod(r, phi);
  }
  out = r;
}
void mt_poly_mulmod_slow(const std::vector<uint64_t> &a, const std::vector<uint64_t> &b,
                         std::vector<uint64_t> &r) {
  const Poly &phi = charpoly();
  Poly pr(2 * kWords + 2, 0), bb(b.begin(), b.end());
  bb.resize(kWords, 0);
  for (int64_t i = 0; i < kWords; ++i) {
    const uint64_t v = i < static_cast<int64_t>(a.size()) ? a[i] : 0;
    if (!v) continue;
    for (int t = 0; t < 64; ++t)
      if ((v >> t) & 1u) xor_shifted(pr, bb, 64 * i + t);
  }
  for (int64_t i = 2 * (kDeg - 1); i >= kDeg; --i)
    if (getbit(pr, i)) xor_shifted(pr, phi, i - kDeg);
  r.assign(pr.begin(), pr.begin() + kWords);
}

// Window (y_0..y_623) advanced by the polynomial p: out[w] = XOR_{i: p_i} y_{i+w}.
void mt_apply_poly(const uint32_t *win, const std::vector<uint64_t> &p, uint32_t *out) {
  std::vector<uint32_t> y(static_cast<size_t>(kDeg + kN + 1));
  std::memcpy(y.data(), win, sizeof(uint32_t) * kN);
  for (size_t k = 0; k + kN < y.size(); ++k) y[k + kN] = twist(y[k], y[k + 1], y[k + kM]);
  uint32_t acc[kN] = {};
  for (int64_t i = 0; i < kDeg; ++i) {
    if (!getbit(p, i)) continue;
    const uint32_t *src = y.data() + i;
    for (int w = 0; w < kN; ++w) acc[w] ^= src[w];
  }
  std::memcpy(out, acc, sizeof(acc));
}

}  // namespace rs

// numpy / CPython state after `steps` more outputs: (key, pos) of the block holding the next
// word.  The jumped window starts one word early so that key[0] comes out whole.
extern "C" int rs_mt_jump(const uint32_t *key, int32_t pos, int64_t steps, uint32_t *key_out,
                          int32_t *pos_out) {
  if (!key || !key_out || !pos_out) return rs::fail(RS_EINVAL, "rs_mt_jump: null pointer");
  if (pos < 0 || pos > kN || steps < 0) return rs::fail(RS_EINVAL, "rs_mt_jump: bad state");
  if (steps == 0) {
    std::memmove(key_out, key, sizeof(uint32_t) * kN);
    *pos_out = pos;
    return RS_OK;
  }
  // absolute index of the last word drawn: W - 1 with W = pos + steps; its block b
  const int64_t W = static_cast<int64_t>(pos) + steps;
  const int64_t b = (W - 1) / kN;
  if (b == 0) {
    std::memmove(key_out, key, sizeof(uint32_t) * kN);
    *pos_out = static_cast<int32_t>(W);
    return RS_OK;
  }
  // window at index 624 b - 1: its words 1..623 plus one generated word are block b
  std::vector<uint64_t> p;
  rs::mt_jump_poly(static_cast<uint64_t>(kN * b - 1), p);
  uint32_t win[kN];
  rs::mt_apply_poly(key, p, win);
  uint32_t blk[kN];
  std::memcpy(blk, win + 1, sizeof(uint32_t) * (kN - 1));
  blk[kN - 1] = twist(win[0], win[1], win[kM]);  // y_{624}: window words 0, 1, 397
  std::memcpy(key_out, blk, sizeof(blk));
  *pos_out = static_cast<int32_t>(W - kN * b);
  return RS_OK;
}

// The fast forms (carry-less products, Barrett reduction, cached powers) against the bit-serial
// reference: x^j1, x^j2 and x^(j1 + j2) by both, and both products.
extern "C" int rs_mt_poly_selftest(int64_t j1, int64_t j2) {
  if (j1 < 0 || j2 < 0) return rs::fail(RS_EINVAL, "rs_mt_poly_selftest: negative exponent");
  std::vector<uint64_t> a, b, c, r, as, bs, cs, rs_;
  rs::mt_jump_poly(static_cast<uint64_t>(j1), a);
  rs::mt_jump_poly(static_cast<uint64_t>(j2), b);
  rs::mt_jump_poly(static_cast<uint64_t>(j1) + static_cast<uint64_t>(j2), c);
  rs::mt_poly_mulmod(a, b, r);
  rs::mt_jump_poly_slow(static_cast<uint64_t>(j1), as);
  rs::mt_jump_poly_slow(static_cast<uint64_t>(j2), bs);
  rs::mt_jump_poly_slow(static_cast<uint64_t>(j1) + static_cast<uint64_t>(j2), cs);
  rs::mt_poly_mulmod_slow(as, bs, rs_);
  std::vector<uint64_t> sq = a, sqs;
  rs::mt_poly_square(sq);
  rs::mt_jump_poly_slow(2 * static_cast<uint64_t>(j1), sqs);
  // the embedded phi and mu (mt_phi.h) against Berlekamp-Massey and long division, once
  static const bool consts_ok = [] {
    const Poly &bm = charpoly_bm(), &em = charpoly();
    const Poly mu = barrett_mu_bm(bm);
    bool ok = true;
    for (int i = 0; i < kR; ++i) ok = ok && bm[static_cast<size_t>(i)] == em[static_cast<size_t>(i)] &&
                                      mu[static_cast<size_t>(i)] == kMuWords[i];
    return ok;
  }();
  // the embedded x^(624 2^k) (mt_phi.h): x^624 by times-x steps, then squarings
  static const bool pow2_ok = [] {
    std::vector<u64> p = x624(), q(kR, 0);
    bool ok = true;
    for (int k = 0; k < kPow2Embed; ++k) {
      if (k) {
        sqrmod_fast(p.data(), q.data());
        p.swap(q);
      }
      ok = ok && std::equal(p.begin(), p.end(), kPow2Words[k]);
    }
    return ok;
  }();
  return (consts_ok && pow2_ok && r == c && a == as && b == bs && c == cs && rs_ == cs && sq == sqs) ? 1 : 0;
}
