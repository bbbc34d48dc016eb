// Host replays of the reference's random streams (bit-exact).
//
//  * numpy legacy RandomState (fun.py:306 np.random.choice(arange(N), 8, replace=False)):
//    MT19937 init_genrand seeding; choice(replace=False) == permutation(N)[:k], a
//    Fisher-Yates sweep i = N-1..1 with j = random_interval(i) (u32 & smear-mask, retry
//    while > i).  SURVEY.md 8(a) row a-R.
//  * CPython random (ransac.py:17 random.shuffle): init_by_array seeding; shuffle sweep
//    i = N-1..1 with j = randbelow(i+1), randbelow(n) = getrandbits(bitlen(n)) retried
//    while >= n, getrandbits(k) = u32 >> (32-k).  SURVEY.md 8(a) row a-8.
//
// The state (key[624], pos) is the one np.random.get_state() / random.getstate() expose,
// so the Python shims hand it in and write the advanced state back (drop-in fidelity).
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "common.h"

namespace {

constexpr int kN = 624;
constexpr int kM = 397;
constexpr uint32_t kMatrixA = 0x9908b0dfu;
constexpr uint32_t kUpper = 0x80000000u;
constexpr uint32_t kLower = 0x7fffffffu;

struct Mt {
  uint32_t key[kN];
  int pos;

  void load(const uint32_t *k, int32_t p) {
    std::memcpy(key, k, sizeof(key));
    pos = p;
  }
  void store(uint32_t *k, int32_t *p) const {
    std::memcpy(k, key, sizeof(key));
    *p = pos;
  }
  // The classic mt19937 twist (numpy mt19937_gen == CPython genrand_uint32 refill).
  void twist() {
    int i = 0;
    for (; i < kN - kM; ++i) {
      uint32_t y = (key[i] & kUpper) | (key[i + 1] & kLower);
      key[i] = key[i + kM] ^ (y >> 1) ^ ((0u - (y & 1u)) & kMatrixA);
    }
    for (; i < kN - 1; ++i) {
      uint32_t y = (key[i] & kUpper) | (key[i + 1] & kLower);
      key[i] = key[i + (kM - kN)] ^ (y >> 1) ^ ((0u - (y & 1u)) & kMatrixA);
    }
    uint32_t y = (key[kN - 1] & kUpper) | (key[0] & kLower);
    key[kN - 1] = key[kM - 1] ^ (y >> 1) ^ ((0u - (y & 1u)) & kMatrixA);
    pos = 0;
  }
  inline uint32_t next() {
    if (pos >= kN) twist();
    uint32_t y = key[pos++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
  }
};

void init_genrand(uint32_t *key, uint32_t s) {
  key[0] = s;
  for (int i = 1; i < kN; ++i)
    key[i] = 1812433253u * (key[i - 1] ^ (key[i - 1] >> 30)) + static_cast<uint32_t>(i);
}

inline uint32_t smear_mask(uint32_t v) {
  v |= v >> 1;
  v |= v >> 2;
  v |= v >> 4;
  v |= v >> 8;
  v |= v >> 16;
  return v;
}

inline int bit_length(uint32_t v) { return v ? 32 - __builtin_clz(v) : 0; }

}  // namespace

extern "C" int rs_np_seed(uint32_t seed, uint32_t *mt_key, int32_t *mt_pos) {
  if (!mt_key || !mt_pos) return rs::fail(RS_EINVAL, "rs_np_seed: null pointer");
  init_genrand(mt_key, seed);
  *mt_pos = kN;
  return RS_OK;
}

extern "C" int rs_py_seed(const uint32_t *words, int32_t n_words, uint32_t *mt_key,
                          int32_t *mt_pos) {
  if (!mt_key || !mt_pos || n_words < 0 || (n_words > 0 && !words))
    return rs::fail(RS_EINVAL, "rs_py_seed: bad arguments");
  // CPython random_seed(): an int seed 0 is the key [0]; init_by_array (mt19937ar.c).
  uint32_t zero = 0;
  const uint32_t *key = n_words ? words : &zero;
  const int len = n_words ? n_words : 1;
  uint32_t *mt = mt_key;
  init_genrand(mt, 19650218u);
  int i = 1, j = 0;
  for (int k = (kN > len ? kN : len); k; --k) {
    mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525u)) + key[j] +
            static_cast<uint32_t>(j);
    ++i;
    ++j;
    if (i >= kN) {
      mt[0] = mt[kN - 1];
      i = 1;
    }
    if (j >= len) j = 0;
  }
  for (int k = kN - 1; k; --k) {
    mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941u)) - static_cast<uint32_t>(i);
    ++i;
    if (i >= kN) {
      mt[0] = mt[kN - 1];
      i = 1;
    }
  }
  mt[0] = 0x80000000u;
  *mt_pos = kN;
  return RS_OK;
}

namespace {

// Block-tempered MT19937 stream: after each twist all 624 words are tempered at once (two
// vectorisable loops), so a draw is a buffer read.  (key, pos) keep numpy's / CPython's exact
// meaning: `out[j]` is the tempered `key[j]`, the next draw is out[pos].
struct MtStream {
  uint32_t key[kN];
  uint32_t out[kN];
  int pos;

  __attribute__((target_clones("avx2", "default"))) static void temper_all(const uint32_t *k,
                                                                           uint32_t *o) {
    for (int i = 0; i < kN; ++i) {
      uint32_t y = k[i];
      y ^= (y >> 11);
      y ^= (y << 7) & 0x9d2c5680u;
      y ^= (y << 15) & 0xefc60000u;
      y ^= (y >> 18);
      o[i] = y;
    }
  }
  __attribute__((target_clones("avx2", "default"))) static void twist_all(uint32_t *k) {
    for (int i = 0; i < kN - kM; ++i) {
      const uint32_t y = (k[i] & kUpper) | (k[i + 1] & kLower);
      k[i] = k[i + kM] ^ (y >> 1) ^ ((0u - (y & 1u)) & kMatrixA);
    }
    for (int i = kN - kM; i < kN - 1; ++i) {
      const uint32_t y = (k[i] & kUpper) | (k[i + 1] & kLower);
      k[i] = k[i + (kM - kN)] ^ (y >> 1) ^ ((0u - (y & 1u)) & kMatrixA);
    }
    const uint32_t y = (k[kN - 1] & kUpper) | (k[0] & kLower);
    k[kN - 1] = k[kM - 1] ^ (y >> 1) ^ ((0u - (y & 1u)) & kMatrixA);
  }
  void load(const uint32_t *k, int32_t p) {
    std::memcpy(key, k, sizeof(key));
    pos = p;
    temper_all(key, out);  // valid for the words at pos..623 of the current block
  }
  void store(uint32_t *k, int32_t *p) const {
    std::memcpy(k, key, sizeof(key));
    *p = pos;
  }
  inline uint32_t next() {
    if (__builtin_expect(pos >= kN, 0)) {
      twist_all(key);
      temper_all(key, out);
      pos = 0;
    }
    return out[pos++];
  }
};

// One Fisher-Yates hypothesis x = arange(n); for i = n-1..1: swap(x[i], x[j]) with j drawn
// by masked rejection, and the k-prefix of the result.  Position i is final after step i, so
// x[i] is only written back while i < k (the prefix); x[j] always receives the old x[i].
//
// Branch-free over the words of one "level" (i in (lo, hi], where the draw's mask / shift is
// fixed): every word is consumed as  acc = (draw(w) <= i);  j = acc ? draw(w) : i;  a swap
// that is a no-op for a rejected word;  i -= acc.  The loop-carried chain is one compare and
// one subtract per word, and the 25-50 % rejections cost no branch mispredictions.
//   numpy  (random_interval, masked):  draw(w) = w & mask,            level: i in (mask/2, mask]
//   CPython (randbelow(i+1), top bits): draw(w) = w >> (32 - bl(i+1)), level: i+1 in [2^(b-1), 2^b)
template <bool NUMPY>
inline void fisher_yates_prefix(MtStream &mt, std::vector<int32_t> &perm,
                                const std::vector<int32_t> &iota, int64_t n, int32_t k,
                                int32_t *out) {
  std::memcpy(perm.data(), iota.data(), sizeof(int32_t) * static_cast<size_t>(n));
  int32_t *x = perm.data();
  uint32_t i = static_cast<uint32_t>(n > 1 ? n - 1 : 0);
  const uint32_t uk = static_cast<uint32_t>(k);
  while (i >= 1) {
    uint32_t lo, mask = 0, sh = 0;
    if (NUMPY) {
      mask = smear_mask(i);  // random_interval(i): mask of i, fixed while i > mask / 2
      lo = mask >> 1;
    } else {
      const int b = bit_length(i + 1);  // randbelow(i + 1): getrandbits(b), fixed while
      sh = static_cast<uint32_t>(32 - b);  // i + 1 >= 2^(b-1)
      lo = (1u << (b - 1)) - 2u;  // i > lo  <=>  i + 1 >= 2^(b-1)
      if (b == 1) lo = 0;          // i = 0 never occurs here (loop condition)
    }
    while (i > lo) {
      const uint32_t w = mt.next();
      const uint32_t v = NUMPY ? (w & mask) : (w >> sh);
      const uint32_t acc = v <= i ? 1u : 0u;
      const uint32_t j = acc ? v : i;
      const int32_t t = x[i];
      if (i < uk) x[i] = x[j];
      x[j] = t;
      i -= acc;
    }
  }
  std::memcpy(out, x, sizeof(int32_t) * static_cast<size_t>(k));
}

}  // namespace

extern "C" int rs_np_choice_tuples(uint32_t *mt_key, int32_t *mt_pos, int64_t n, int32_t k,
                                   int64_t count, int32_t *out) {
  if (!mt_key || !mt_pos || (count > 0 && !out))
    return rs::fail(RS_EINVAL, "rs_np_choice_tuples: null pointer");
  if (k < 0 || count < 0) return rs::fail(RS_EINVAL, "negative dimensions are not allowed");
  if (k > n)  // numpy: "Cannot take a larger sample than population when 'replace=False'"
    return rs::fail(RS_EINVAL,
                    "Cannot take a larger sample than population when 'replace=False'");
  if (n > 0x7fffffffLL) return rs::fail(RS_EINVAL, "population too large");
  if (*mt_pos < 0 || *mt_pos > kN) return rs::fail(RS_EINVAL, "bad MT19937 position");
  MtStream mt;
  mt.load(mt_key, *mt_pos);
  std::vector<int32_t> perm(static_cast<size_t>(n > 0 ? n : 1)), iota(perm.size());
  for (int64_t i = 0; i < n; ++i) iota[static_cast<size_t>(i)] = static_cast<int32_t>(i);
  // numpy random_interval(max): draws u32 & smear(max) until <= max
  for (int64_t h = 0; h < count; ++h) fisher_yates_prefix<true>(mt, perm, iota, n, k, out + h * k);
  mt.store(mt_key, mt_pos);
  return RS_OK;
}

// Many independent numpy streams (one per image pair, config C4: np.random.seed(1000 + pair)
// then H x choice(N_b, k, replace=False)) replayed on host threads.  Streams with n < k are
// skipped: their outputs are zero and their state is unchanged (the pair batch flags them).
extern "C" int rs_np_choice_tuples_multi(int64_t B, const uint32_t *seeds, uint32_t *mt_keys,
                                         int32_t *mt_pos, const int64_t *ns, int32_t k,
                                         int64_t count, int32_t *out, int32_t threads) {
  if (B < 0 || k < 0 || count < 0) return rs::fail(RS_EINVAL, "negative dimensions are not allowed");
  if (B == 0) return RS_OK;
  if (!mt_keys || !mt_pos || !ns || (count > 0 && !out))
    return rs::fail(RS_EINVAL, "rs_np_choice_tuples_multi: null pointer");
  for (int64_t b = 0; b < B; ++b) {
    if (ns[b] > 0x7fffffffLL) return rs::fail(RS_EINVAL, "population too large");
    if (seeds) rs_np_seed(seeds[b], mt_keys + b * kN, mt_pos + b);  // np.random.seed(s_b)
    if (mt_pos[b] < 0 || mt_pos[b] > kN) return rs::fail(RS_EINVAL, "bad MT19937 position");
  }
  const int64_t per = count * k;
  std::atomic<int64_t> next{0};
  std::atomic<bool> oom{false};
  // no exception may leave a worker (std::terminate would take the host process down): an
  // allocation failure stops the whole batch and the call returns RS_ENOMEM
  auto work_streams = [&] {
    std::vector<int32_t> perm, iota;
    for (int64_t b; (b = next.fetch_add(1)) < B;) {
      int32_t *o = out + b * per;
      const int64_t n = ns[b];
      if (n < k) {
        std::fill(o, o + per, 0);
        continue;
      }
      MtStream mt;
      mt.load(mt_keys + b * kN, mt_pos[b]);
      perm.resize(static_cast<size_t>(n > 0 ? n : 1));
      iota.resize(perm.size());
      for (int64_t i = 0; i < n; ++i) iota[static_cast<size_t>(i)] = static_cast<int32_t>(i);
      for (int64_t h = 0; h < count; ++h) fisher_yates_prefix<true>(mt, perm, iota, n, k, o + h * k);
      mt.store(mt_keys + b * kN, mt_pos + b);
    }
  };
  auto work = [&]() noexcept {
    try {
      work_streams();
    } catch (...) {
      oom = true;
      next = B;
    }
  };
  // default: the hardware threads, at most 16 (a one-GPU share of a shared host)
  int nt = threads > 0 ? threads
                       : std::min(16, static_cast<int>(std::thread::hardware_concurrency()));
  nt = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>({static_cast<int64_t>(nt), B, 64})));
  std::vector<std::thread> pool;
  try {
    pool.reserve(static_cast<size_t>(nt));
    for (int i = 1; i < nt; ++i) pool.emplace_back(work);
  } catch (...) {
    // fewer threads than asked (thread creation or the pool's allocation failed): the
    // streams are handed out dynamically, so the ones that exist -- at least this one --
    // still draw every stream
  }
  work();
  for (auto &t : pool) t.join();
  return oom ? rs::fail(RS_ENOMEM, "rs_np_choice_tuples_multi: out of host memory") : RS_OK;
}

extern "C" int rs_py_shuffle_tuples(uint32_t *mt_key, int32_t *mt_pos, int64_t n, int32_t k,
                                    int64_t count, int32_t *out) {
  if (!mt_key || !mt_pos || (count > 0 && !out))
    return rs::fail(RS_EINVAL, "rs_py_shuffle_tuples: null pointer");
  if (n < k)  // ransac.py:13-14
    return rs::fail(RS_EINVAL,
                    "Cannot generate more indices than the amount of values in the set from "
                    "which they are extracted. n should therefore be smaller or equal to "
                    "set_length");
  if (k < 0 || count < 0 || n > 0x7fffffffLL) return rs::fail(RS_EINVAL, "bad dimensions");
  if (*mt_pos < 0 || *mt_pos > kN) return rs::fail(RS_EINVAL, "bad MT19937 position");
  MtStream mt;
  mt.load(mt_key, *mt_pos);
  std::vector<int32_t> perm(static_cast<size_t>(n > 0 ? n : 1)), iota(perm.size());
  for (int64_t i = 0; i < n; ++i) iota[static_cast<size_t>(i)] = static_cast<int32_t>(i);
  // randbelow(i + 1): getrandbits(bit_length(i + 1)) until < i + 1
  for (int64_t h = 0; h < count; ++h)
    fisher_yates_prefix<false>(mt, perm, iota, n, k, out + h * k);
  mt.store(mt_key, mt_pos);
  return RS_OK;
}
