// numpy-exact parity stream on the GPU: the tuples of rs_np_choice_tuples (fun.py:305-306,
// np.random.choice(N, 8, replace=False) = permutation(N)[:8]) without the serial host replay.
//
// One hypothesis is a Fisher-Yates sweep i = N-1 .. 1 whose step i draws u32 words until
// (w & mask(i)) <= i (numpy's random_interval).  Where hypotheses start in the word stream is
// a serial property of the stream; the rest is parallel.  Pipeline per segment of hypotheses:
//
//   1. k_mt_jump    MT19937 windows 2^k J words apart by x^(2^k J) mod phi (a doubling tree;
//                   the polynomials come from mt_jump.cpp, once per process);
//   2. k_mt_stream  one wave per window: the tempered word stream, materialised in HBM;
//   3. k_np_entry   per chunk of kW draws, the parse from EVERY entry state at once: parser
//                   states are i in 1..N-1, trajectories that meet merge, and they stay in
//                   cyclic order, so a sorted list with member ranges (lo) describes the map
//                   entry -> exit state.  Every wrap (hypothesis end) of every trajectory is
//                   logged with the member range it belongs to;
//   4. host         compose the per-chunk maps (C lookups) -> the true entry state per chunk;
//   5. k_np_filter  keep the logged wraps whose member range holds the true entry: these are
//                   exactly the hypothesis starts; k_np_starts gathers them in order;
//   6. k_np_tuples  one lane per hypothesis: re-parse its own words, keep the swap partners
//                   j_i, trace positions 0..k-1 back through the swaps -> the k indices.
//
// The final (key, pos) state is the stream block holding the next word, untempered on the
// host.  Exactness does not depend on any tuning constant; tests compare against the host
// replay (tests/test_gpu_np_sampler.py).
#include <hip/hip_runtime.h>
#include <array>
#include <chrono>
#include <memory>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <mutex>
#include <thread>
#include <vector>

#include "common.h"
#include "ctx.h"

namespace rs {
int hip_fail(hipError_t e, const char *what);
void mt_jump_poly(uint64_t J, std::vector<uint64_t> &out);
void mt_poly_square(std::vector<uint64_t> &p);
void mt_poly_mulmod(const std::vector<uint64_t> &a, const std::vector<uint64_t> &b,
                    std::vector<uint64_t> &r);
}  // namespace rs

#define HIP_TRY(expr)                                     \
  do {                                                    \
    hipError_t e_ = (expr);                               \
    if (e_ != hipSuccess) return rs::hip_fail(e_, #expr); \
  } while (0)

namespace {

constexpr int kN = 624;
constexpr int kM = 397;
constexpr uint32_t kUpper = 0x80000000u;
constexpr uint32_t kLower = 0x7fffffffu;
constexpr uint32_t kMatA = 0x9908b0dfu;
constexpr int kDeg = 19937;
constexpr int kPrefix = kDeg + kN - 1;       // words of a window's sequence a jump reads
constexpr int kPrefixAlloc = kN * ((kPrefix + kN - 1) / kN);  // generated in whole blocks
constexpr int kPhases = (kDeg + kN - 1) / kN;  // blocks holding a jump polynomial's bits (32)
constexpr int kJB = 1024;                    // stream blocks per generator (unless chunk-aligned)
constexpr int kLevels = 16;                  // jump levels: windows up to 2^16 generators apart
constexpr int kW = 1 << 24;                  // longest automatic parse chunk (draws)
constexpr int kWmax = 1 << 24;               // longest chunk (RSAMD_NP_KW)
constexpr int kWmin = 8192;                  // shortest parse chunk
constexpr int kEntryThreads = 512;
constexpr int kR = 20;                       // slots per thread: N - 1 <= 10240
constexpr int kMaxN1 = kEntryThreads * kR;
constexpr int kK = 64;                       // draws between compactions (<= N - 1 when dense)
// dense-phase batches of 64 draws between compactions (the one-slot and the multi-slot paths):
// a compaction costs ~8k cycles (block scans, barriers), merges are slow at large N.  Measured
// (round 2, C2 / N = 10 000 ms): one-slot 4 / 16 / 32 batches 7.90 / 7.75 / - and 41.4 / 38.6 /
// 36.6; multi-slot 1 / 4 / 8 batches 7.78 / 8.17 / 8.22 and 38.0 / 37.1 / 36.9 (re-measured in
// round 4 below).
#ifndef RSAMD_NFAST
#define RSAMD_NFAST 0   // A/B builds: batches between the one-slot path's compactions at C2 sizes
#endif
#ifndef RSAMD_NFASTM
#define RSAMD_NFASTM 0  // A/B builds: the same for the multi-slot path
#endif
__host__ __device__ constexpr int fast_batches(int n1) {
  return n1 >= 4096 ? 32 : (RSAMD_NFAST ? RSAMD_NFAST : 16);
}
// (with the one-instruction draw masks the multi-slot batches got cheap against a compaction:
// C2 entry kernel per launch, compaction every 1 / 2 / 4 / 8 / 16 batches: 430 / 412 / 406 /
// 409 / 410 us; one-slot every 8 / 16 / 32: 442 / 430 / 433, profiles/r04_np_ab3)
__host__ __device__ constexpr int fast_batches_multi(int n1) {
  return n1 >= 4096 ? 4 : (RSAMD_NFASTM ? RSAMD_NFASTM : 4);
}
constexpr int kRFast = 8;                    // slots per thread of the branch-free multi-slot path
#ifndef RSAMD_ONESLOT2
#define RSAMD_ONESLOT2 1  // two-bucket batches in the one-slot dense path (A/B builds: 0)
#endif
#ifndef RSAMD_MULTI2
#define RSAMD_MULTI2 1    // the same per slot in the multi-slot dense path (A/B builds: 0)
#endif
// numpy draw rule inside a two-bucket batch (s in [M/4 + 1, M], M = mask of the batch's first
// state): mask(s) = s | (M >> 1) -- M where s has the top bit of M, M >> 1 below it -- so a step
// is one v_bitop3 (w & (s | M/2)), a compare and a subtract-with-borrow instead of compare /
// select / and / compare / subtract.  Entry kernel at C2 (rocprofv3, two interleaved passes,
// profiles/r04_np_ab3): 550 -> 489 us per launch (A/B builds: 0)
#ifndef RSAMD_ORMASK
#define RSAMD_ORMASK 1
#endif
// the batch's 64 words broadcast from a per-wave LDS copy (ds_read_b128, four draws per read)
// instead of one v_readlane per draw: three vector instructions per draw.  489 -> 437 us
// (A/B builds: 0)
#ifndef RSAMD_WLDS
#define RSAMD_WLDS 1
#endif
#ifndef RSAMD_STREAM_PRIO
#define RSAMD_STREAM_PRIO 0  // k_mt_stream's waves at issue priority 3 (A/B knob: the second
                             // pass sped up, the entry beside it slowed 389 -> 450 us per
                             // launch; C2 parse 4.98 vs 4.97 ms: not kept)
#endif
#ifndef RSAMD_GEN2
#define RSAMD_GEN2 0  // the one-slot general batch with the wrap test off the chain (A/B builds: 1)
#endif
// (Measured and not kept: the same broadcast in the one-slot path's general batches, 433 ->
// 441 us, and with the wrap bookkeeping skipped where no state is <= 64, 450 us.)
// the dense phase's compaction specialised for one slot per thread (a ballot rank and the wave
// counts instead of the block scan; three barriers instead of five): 437 -> 432 us (A/B builds: 0)
#ifndef RSAMD_CMP1
#define RSAMD_CMP1 1
#endif
// Trajectories left when the dense parse hands a chunk to the tracking kernel, also the tracking
// kernel's list capacity (a template argument, <= 8 per wave of its 16).  The
// one-slot dense path costs ~N per draw and chunk, so large N hands over earlier: measured
// (probe, C2 / N = 10 000): 64 -> 6.40 / 36.6 ms, 128 -> 6.48 / 34.2 ms.
#ifndef RSAMD_HAND_SMALL
#define RSAMD_HAND_SMALL 64  // hand-over list for N - 1 < 4096 (A/B builds: 128)
#endif
__host__ __device__ constexpr int hand_of(int n1) { return n1 >= 4096 ? 128 : RSAMD_HAND_SMALL; }

constexpr uint32_t kSentinel = 0x80000000u;  // an empty slot: never reaches 0 within kW steps

__device__ __forceinline__ uint32_t twist(uint32_t a, uint32_t b) {
  const uint32_t y = (a & kUpper) | (b & kLower);
  return (y >> 1) ^ ((0u - (y & 1u)) & kMatA);
}
__device__ __forceinline__ uint32_t temper(uint32_t y) {
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}
// numpy random_interval(i): the draw is w & mask(i), mask = smallest 2^b - 1 >= i (i >= 1)
__device__ __forceinline__ uint32_t masked(uint32_t w, uint32_t i) {
  return w & (0xffffffffu >> __builtin_clz(i));
}
// The draw of state i under either stream's rule; the step accepts iff draw <= i.
//   numpy (PY = false): random_interval(i) = w & mask(i)                       (fun.py:305)
//   CPython (PY = true): randbelow(i + 1) = getrandbits(bit_length(i + 1)) = w >> clz(i + 1)
//                        (random.shuffle behind ransac.gen_rnd_indices, ransac.py:12-19)
template <bool PY>
__device__ __forceinline__ uint32_t draw_of(uint32_t w, uint32_t i) {
  if constexpr (PY) return w >> __builtin_clz(i + 1u);
  else return masked(w, i);
}

// ---- 1. jump tree level: window[g + half] = x^(half J) applied to window[g] ----------------
// y_t = y_{t-227} ^ twist(y_{t-624}, y_{t-623}); word w of the jumped window is the XOR of
// y_{i+w} over the set bits i of the polynomial.  Only the top bit of word 0 is MT state, so
// word 0 of a jumped window may carry wrong low bits: it is never emitted (k_mt_stream) and
// the recurrence reads only its top bit.
// Each jump is split into S parts over the (sorted) set bits, so that every level of the tree
// runs on all CUs: part q regenerates in LDS only the prefix y_0 .. y_{hi-1} its bits read,
// XORs its share (kJumpGroups groups of kJumpGroupThreads threads, a third of the bits each),
// and XOR-adds the partial window into the destination (zeroed beforehand) with vector atomics;
// a single part stores it.
// The XOR phase is LDS-bandwidth bound, so it reads aligned word PAIRS (ds_read_b64: 256 B per
// clock against 128 for ds_read_b32): thread l of a group owns the pair (2l, 2l + 1) for an even
// bit i, reading y_{i+2l}, y_{i+2l+1}; for an odd bit the aligned pair at i + 2l - 1 holds
// y_{i+2l-1}, y_{i+2l}, which belong to words 2l - 1 and 2l.  The four accumulators per thread
// are recombined through LDS at the end.  (b32 reads, three words per thread: C2 levels 7 / 8
// 85 / 155 us.)
constexpr int kJumpGroups = 3;
constexpr int kJumpGroupThreads = 320;   // >= 313 pair owners (l = 0 .. 312)
constexpr int kJumpThreads = kJumpGroups * kJumpGroupThreads;
// One launch per tree level: multiplier m = 1 .. nm of the level's base distance B (`half`),
// window[g + m B] = x^(m B J) applied to window[g] (radix nm + 1; the g0 chain uses nm = 1).
struct JumpSet {
  int nm;
  int off[7], nb[7], ne[7];  // per multiplier: offset into the bit lists, set bits, even ones
};
__global__ __launch_bounds__(kJumpThreads) void k_mt_jump(uint32_t *__restrict__ win, int half,
                                                         int G,
                                                         const int32_t *__restrict__ bits_base,
                                                         JumpSet js, int S) {
  // bits: the level's even set bits (ne of them, ascending), then its odd ones
  extern __shared__ uint32_t y[];  // up to kPrefixAlloc words (8-byte aligned)
  __shared__ uint32_t pe[kJumpGroups][kN], po[kJumpGroups][kN];
  const int per_m = half * S, mi = static_cast<int>(blockIdx.x) / per_m;
  const int rem = static_cast<int>(blockIdx.x) - mi * per_m;
  const int g = rem / S, q = rem % S, dst = g + (mi + 1) * half;
  if (mi >= js.nm || dst >= G) return;
  const int32_t *__restrict__ bits = bits_base + js.off[mi];
  const int nbits = js.nb[mi], ne = js.ne[mi];
  const int no = nbits - ne;
  const int e0 = static_cast<int>(static_cast<int64_t>(ne) * q / S);
  const int e1 = static_cast<int>(static_cast<int64_t>(ne) * (q + 1) / S);
  const int q0 = ne + static_cast<int>(static_cast<int64_t>(no) * q / S);
  const int q1 = ne + static_cast<int>(static_cast<int64_t>(no) * (q + 1) / S);
  if (e0 >= e1 && q0 >= q1) return;
  // words y_0 .. y_{hi-1} are read (a bit i is stored as 8 (i >> 1), its pair's byte offset)
  const int hi = 2 * (max(e1 > e0 ? bits[e1 - 1] : 0, q1 > q0 ? bits[q1 - 1] : 0) >> 3) + 2 + kN;
  const int tid = threadIdx.x;
  const int grp = __builtin_amdgcn_readfirstlane(tid / kJumpGroupThreads), lt = tid - grp * kJumpGroupThreads;
  for (int t = tid; t < kN; t += kJumpThreads) y[t] = win[static_cast<size_t>(g) * kN + t];
  __syncthreads();
  // the prefix a block of 624 words at a time, one barrier per block (the three dependent runs
  // of the recurrence are one thread's chain, as in k_mt_stream; 88 -> 33 barriers at most)
  for (int b0 = 0; b0 + kN < hi; b0 += kN) {
    if (tid < 227) {
      const uint32_t *o = y + b0;
      uint32_t *n = y + b0 + kN;
      const uint32_t n0 = o[tid + kM] ^ twist(o[tid], o[tid + 1]);
      const uint32_t n1 = n0 ^ twist(o[tid + 227], o[tid + 228]);
      n[tid] = n0;
      n[tid + 227] = n1;
      if (tid < 170) {
        const uint32_t nx = tid + 455 < kN ? o[tid + 455] : (o[kM] ^ twist(o[0], o[1]));
        n[tid + 454] = n1 ^ twist(o[tid + 454], nx);
      }
    }
    __syncthreads();
  }
  // pair owner l = lt (0 .. 312); reads stay below hi + 1 <= kPrefixAlloc (lane 312 of an even
  // bit reads y_{i+624}, y_{i+625}: words of the last generated block)
  const bool act = lt <= kN / 2;
  uint32_t a0 = 0, a1 = 0, c0 = 0, c1 = 0;  // even bits: words 2l, 2l+1; odd: 2l-1, 2l
  const char *yl = reinterpret_cast<const char *>(y) + 8 * lt;
  // the group's share of a sorted run of bits of one parity, 16 byte offsets per scalar load
  // batch, the next batch's load issued before this batch's LDS reads (its latency was exposed
  // once per batch), the offsets stored ready to add (no scalar shift / mask per bit)
  auto run = [&](int r0, int r1, uint32_t &x0, uint32_t &x1) {
    const int per = (r1 - r0 + kJumpGroups - 1) / kJumpGroups;
    const int b0 = r0 + grp * per, b1 = min(r1, b0 + per);
    int b = b0;
    if (b + 16 <= b1) {
      int ix[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) ix[k] = bits[b + k];
      // the first batch waited for here, so that inside the loop only the prefetch is pending
      // when the addresses are formed (scalar loads return out of order: the wait before the
      // XORs then covers the prefetch and the LDS reads together)
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
      for (; b + 16 <= b1; b += 16) {
        int nx[16];
        const bool more = b + 32 <= b1;
        if (more) {
#pragma unroll
          for (int k = 0; k < 16; ++k) nx[k] = bits[b + 16 + k];
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const uint2 v = *reinterpret_cast<const uint2 *>(yl + ix[k]);  // pair at i - (i & 1) + 2l
          x0 ^= v.x;
          x1 ^= v.y;
        }
        if (more) {
#pragma unroll
          for (int k = 0; k < 16; ++k) ix[k] = nx[k];
        }
      }
    }
    for (; b < b1; ++b) {
      const uint2 v = *reinterpret_cast<const uint2 *>(yl + bits[b]);
      x0 ^= v.x;
      x1 ^= v.y;
    }
  };
  if (act) {
    run(e0, e1, a0, a1);
    run(q0, q1, c0, c1);
    const uint32_t o0 = c0, o1 = c1;
    // word 2l: e0 ^ o1; word 2l+1: e1 (+ the next owner's o0); word 2l-1: o0
    const int w = 2 * lt;
    if (w < kN) pe[grp][w] = a0 ^ o1;
    if (w + 1 < kN) pe[grp][w + 1] = a1;
    if (w >= 1 && w - 1 < kN) po[grp][w - 1] = o0;
  }
  __syncthreads();
  // combine: word t = XOR over groups of pe[.][t] ^ po[.][t] (po[.][t] for odd t only)
  uint32_t *out = win + static_cast<size_t>(dst) * kN;
  for (int t = tid; t < kN; t += kJumpThreads) {
    uint32_t v = 0;
#pragma unroll
    for (int k = 0; k < kJumpGroups; ++k) v ^= pe[k][t] ^ ((t & 1) ? po[k][t] : 0u);
    if (S == 1) out[t] = v;
    else atomicXor(out + t, v);
  }
}

// The same jump with the window's sequence in a ring of four blocks instead of a 20 561-word
// prefix (RSAMD_JUMP_PREFIX=1 selects the prefix form): phase p generates block p + 3 and XORs
// the bits in block p (their reads span blocks p .. p + 2), one barrier per phase as before.
// 27.5 KB of LDS instead of 97 KB, so two workgroups share a CU.  Reads run linearly past the
// ring's end into a mirror of slot 0 (and slot 1's first two words): block b sits at slot b % 4,
// and the bits of phase p read at byte offset - (p / 4) 4 kN 4.
#ifndef RSAMD_JUMP_XOR3
#define RSAMD_JUMP_XOR3 1  // the ring form's XORs in pairs by v_bitop3 (A/B builds: 0; C5 jump 6.5 -> 6.1 ms)
#endif
constexpr int kRing = 4 * kN;
constexpr int kMirror = kN + 2;
struct JumpIdx16 {
  int v[16];
};
constexpr int kZeroPad = kN + 2;  // zeros the padding entries read (words 2 l, 2 l + 1 <= kN + 1)
__device__ __forceinline__ void jump_gen_block(uint32_t *y, int b, int tid) {
  // block b + 1 from block b (the three dependent runs on one thread, as in the prefix form)
  if (tid < 227) {
    const uint32_t *o = y + kN * (b & 3);
    const int sn = (b + 1) & 3;
    uint32_t *n = y + kN * sn;
    const uint32_t n0 = o[tid + kM] ^ twist(o[tid], o[tid + 1]);
    const uint32_t n1 = n0 ^ twist(o[tid + 227], o[tid + 228]);
    uint32_t n2 = 0;
    if (tid < 170) {
      const uint32_t nx = tid + 455 < kN ? o[tid + 455] : (o[kM] ^ twist(o[0], o[1]));
      n2 = n1 ^ twist(o[tid + 454], nx);
    }
    n[tid] = n0;
    n[tid + 227] = n1;
    if (tid < 170) n[tid + 454] = n2;
    if (sn == 0) {  // the mirror of slot 0
      y[kRing + tid] = n0;
      y[kRing + tid + 227] = n1;
      if (tid < 170) y[kRing + tid + 454] = n2;
    } else if (sn == 1 && tid < 2) {
      y[kRing + kN + tid] = n0;
    }
  }
}

__global__ __launch_bounds__(kJumpThreads, 8) void k_mt_jump_slide(uint32_t *__restrict__ win,
                                                                  int half, int G,
                                                                  const int32_t *__restrict__ bits_base,
                                                                  JumpSet js, int S) {
  // the ring, its mirror, then zeros (the padding entries of a run read them)
  __shared__ __attribute__((aligned(16))) uint32_t y[kRing + kMirror + kZeroPad];
  __shared__ uint32_t pe[kJumpGroups][kN], po[kJumpGroups][kN];
  const int per_m = half * S, mi = static_cast<int>(blockIdx.x) / per_m;
  const int rem = static_cast<int>(blockIdx.x) - mi * per_m;
  const int g = rem / S, q = rem % S, dst = g + (mi + 1) * half;
  if (mi >= js.nm || dst >= G) return;
  const int32_t *__restrict__ bits = bits_base + js.off[mi];
  const int nbits = js.nb[mi];
  const int32_t *__restrict__ tab = bits + nbits;     // run starts by (phase, parity)
  const int32_t *__restrict__ pad = tab + 2 * kPhases + 1;  // the padded runs
  // part q of S: phases [ph0, ph1) (every phase of a degree-19937 polynomial holds bits)
  const int ph0 = kPhases * q / S, ph1 = kPhases * (q + 1) / S;
  if (ph0 >= ph1) return;
  const int tid = threadIdx.x;
  const int grp = __builtin_amdgcn_readfirstlane(tid / kJumpGroupThreads), lt = tid - grp * kJumpGroupThreads;
  for (int t = tid; t < kN; t += kJumpThreads) {
    const uint32_t v = win[static_cast<size_t>(g) * kN + t];
    y[t] = v;
    y[kRing + t] = v;
  }
  for (int t = tid; t < kZeroPad; t += kJumpThreads) y[kRing + kMirror + t] = 0u;
  __syncthreads();
  jump_gen_block(y, 0, tid);
  __syncthreads();
  jump_gen_block(y, 1, tid);
  __syncthreads();
  const bool act = lt <= kN / 2;
  uint32_t a0 = 0, a1 = 0, c0 = 0, c1 = 0;  // even bits: words 2l, 2l+1; odd: 2l-1, 2l
  // a padded run in full batches of 16 (batch j to group j % 3), one 64-byte scalar load each,
  // the XORs in pairs
  auto run = [&](int r0, int r1, const char *yl, uint32_t &x0, uint32_t &x1) {
#pragma clang loop vectorize(disable) interleave(disable)
    for (int b = r0 + 16 * grp; b < r1; b += 16 * kJumpGroups) {
      const JumpIdx16 t = *reinterpret_cast<const JumpIdx16 *>(pad + b);
#pragma unroll
      for (int k = 0; k < 16; k += 2) {
        const uint2 u = *reinterpret_cast<const uint2 *>(yl + t.v[k]);
        const uint2 v = *reinterpret_cast<const uint2 *>(yl + t.v[k + 1]);
#if RSAMD_JUMP_XOR3
        asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(x0) : "v"(x0), "v"(u.x), "v"(v.x));
        asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(x1) : "v"(x1), "v"(u.y), "v"(v.y));
#else
        x0 ^= u.x ^ v.x;
        x1 ^= u.y ^ v.y;
#endif
      }
    }
  };
  for (int p = 0; p < ph1; ++p) {
    if (p + 3 <= ph1 + 1) jump_gen_block(y, p + 2, tid);  // block p + 3 (the last one read: ph1 + 1)
    if (p >= ph0 && act) {
      const char *yl = reinterpret_cast<const char *>(y) + 8 * lt - (p >> 2) * (4 * kRing);
      const int r0 = tab[2 * p], r1 = tab[2 * p + 1], r2 = tab[2 * p + 2];
      run(r0, r1, yl, a0, a1);
      run(r1, r2, yl, c0, c1);
    }
    __syncthreads();
  }
  if (act) {
    const int w = 2 * lt;
    if (w < kN) pe[grp][w] = a0 ^ c1;
    if (w + 1 < kN) pe[grp][w + 1] = a1;
    if (w >= 1 && w - 1 < kN) po[grp][w - 1] = c0;
  }
  __syncthreads();
  uint32_t *out = win + static_cast<size_t>(dst) * kN;
  for (int t = tid; t < kN; t += kJumpThreads) {
    uint32_t v = 0;
#pragma unroll
    for (int k = 0; k < kJumpGroups; ++k) v ^= pe[k][t] ^ ((t & 1) ? po[k][t] : 0u);
    if (S == 1) out[t] = v;
    else atomicXor(out + t, v);
  }
}

// ---- 2. stream: generator g owns blocks (g kJB, (g+1) kJB] plus words 1..623 of its window --
// Thread l < 227 owns the words l, l + 227 and (l < 170) l + 454 of every block, in registers:
//   new[l]       = old[l + 397] ^ twist(old[l], old[l + 1])
//   new[l + 227] = new[l]       ^ twist(old[l + 227], old[l + 228])
//   new[l + 454] = new[l + 227] ^ twist(old[l + 454], old[l + 455])   (new[0] for word 623)
// so the three dependent runs of the recurrence are one thread's sequential chain and a block
// needs ONE barrier: the old block is published in LDS (two buffers alternate), every thread
// reads the four neighbour words it needs (thread 169 also recomputes new[0]).  (Three runs of
// 227 / 227 / 170 threads with a barrier after each: 0.61 ms at C2; one wave per generator
// with wave-level fences: 1.45 ms.)
// Chunk-aligned layouts split a generator's run in two launches (k_mt_stream over blocks
// 1..XB of every generator, then XB+1.. on a second stream while the entry kernel parses the
// chunks' first draws): blo / bhi bound the blocks (relative to the window) this launch
// writes, and the raw words of block blo (pass 2) / bhi (pass 1) go through io.  G generators
// of JB blocks; with `ext` the last one runs on to the segment's end (Lb - 1).
__global__ __launch_bounds__(256) void k_mt_stream(const uint32_t *__restrict__ win,
                                                   uint32_t *__restrict__ stream, int64_t Lb,
                                                   int JB, int G, int ext, int blo, int bhi,
                                                   uint32_t *__restrict__ io) {
  __shared__ uint32_t bb[2][kN];
#if RSAMD_STREAM_PRIO
  // the second pass runs beside the entry kernel and, with the entry's steps down to three
  // instructions a draw, became the longer of the two (854 vs 765 us at C2): its waves are a
  // barrier-bound chain, so they take the SIMDs' issue first
  __builtin_amdgcn_s_setprio(3);
#endif
  const int g = blockIdx.x, l = threadIdx.x;
  const bool own = l < 227, own2 = l < 170;
  const int64_t b0 = static_cast<int64_t>(g) * JB;
  uint32_t o0 = 0, o1 = 0, o2 = 0;
  if (blo == 0) {
    const uint32_t *wg = win + static_cast<size_t>(g) * kN;
    if (own) {
      o0 = wg[l];
      o1 = wg[l + 227];
      if (own2) o2 = wg[l + 454];
      uint32_t *o = stream + b0 * kN;
      if (l > 0 || g == 0) o[l] = temper(o0);
      o[l + 227] = temper(o1);
      if (own2) o[l + 454] = temper(o2);
    }
  } else if (own) {
    const uint32_t *ig = io + static_cast<size_t>(g) * kN;
    o0 = ig[l];
    o1 = ig[l + 227];
    if (own2) o2 = ig[l + 454];
  }
  const int64_t gend = ext && g == G - 1 ? Lb - 1 : std::min<int64_t>(b0 + JB, Lb - 1);
  const int64_t bend = std::min<int64_t>(gend, b0 + bhi);
  int buf = 0;
  for (int64_t b = b0 + blo + 1; b <= bend; ++b) {
    uint32_t *ob = bb[buf];
    if (own) {
      ob[l] = o0;
      ob[l + 227] = o1;
      if (own2) ob[l + 454] = o2;
    }
    __syncthreads();
    if (own) {
      const uint32_t n0 = ob[l + kM] ^ twist(o0, ob[l + 1]);
      const uint32_t n1 = n0 ^ twist(o1, ob[l + 228]);
      uint32_t *o = stream + b * kN;
      o[l] = temper(n0);
      o[l + 227] = temper(n1);
      if (own2) {
        const uint32_t nx = l + 455 < kN ? ob[l + 455] : (ob[kM] ^ twist(ob[0], ob[1]));
        o2 = n1 ^ twist(o2, nx);
        o[l + 454] = temper(o2);
      }
      o0 = n0;
      o1 = n1;
    }
    buf ^= 1;
  }
  if (bend < gend && own) {  // pass 1 stopped early: the raw block for pass 2
    uint32_t *ig = io + static_cast<size_t>(g) * kN;
    ig[l] = o0;
    ig[l + 227] = o1;
    if (own2) ig[l + 454] = o2;
  }
}

// ---- 3. all-entry parse of one chunk ---------------------------------------------------------
struct EntryArgs {
  const uint32_t *draws;  // draw 0 of the segment
  int64_t D;              // draws in the segment
  int W;                  // draws per chunk
  int n1;                 // N - 1: parser states 1..n1, entry list index a <-> state n1 - a
  uint32_t *fin;          // [C][n1] final list: lo | state << 16
  int *fin_m;             // [C]
  uint2 *ev;              // [C][ecap] wraps: (draw after the wrap, lo | hi << 16)
  int *ev_n;              // [C]
  int *tpos;              // [C] draws parsed by the dense kernel (the sparse kernel resumes there)
  int ecap;
  int *err;
  long long *stats;       // RSAMD_DIAG builds only: per-chunk tracking statistics (else null)
  // split stream (chunk-aligned generators): the first launch of k_np_entry reads only the
  // chunk's first xlim draws (the first stream pass); a chunk still dense there pauses (its list
  // in fin, position in tpos, pause[c] = 1) and the resume launch (after the second pass)
  // carries it on
  int xlim, resume;
  int *pause;
};

// inclusive wave scan by DPP (row shifts, then the row broadcasts into the upper rows): six
// vector ops instead of six LDS permutes
__device__ __forceinline__ int wave_incl_scan(int x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return x;
}

__device__ __forceinline__ int block_excl_scan(int v, int *sh, int *total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int x = wave_incl_scan(v);  // (by LDS permutes: +4 us per C2 entry launch)
  if (lane == 63) sh[wid] = x;
  __syncthreads();
  int base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kEntryThreads / 64; ++w) {
    const int s = sh[w];
    base += w < wid ? s : 0;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return base + x - v;
}

// a value the compiler cannot prove wave-uniform (threadIdx-derived, LDS-loaded) that is
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint32_t uni(uint32_t v) {
  return static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(v)));
}

__device__ __forceinline__ uint32_t lane_rank(uint64_t bits) {
  return __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(bits >> 32),
                                   __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(bits), 0u));
}

// Chunk timeline of the parse (RSAMD_NP_TSTAMP=<file>, tools/np_timeline.py): per chunk
// kTs words of stamps -- 100 MHz real-time counter and shader-clock cycles at the entry kernel's
// start / end, the tracking kernel's start / end and the moment the chunk's trajectories are
// down to one per wave, with the draw positions and hardware ids.  Null in production: the
// product kernels carry the stamps (read through a relaxed load at each point, so no register
// holds the pointer), and a stamp never feeds a computed value.
__device__ unsigned long long *g_np_ts = nullptr;
constexpr int kTs = 16;
enum : int {
  kTsEntryR0 = 0, kTsEntryC0, kTsEntryR1, kTsEntryC1, kTsEntryT, kTsEntryM, kTsEntryHw,
  kTsTrackR0 = 8, kTsTrackC0, kTsSingleR, kTsSingleT, kTsTrackR1, kTsTrackC1, kTsTrackHw, kTsSingleC
};
__device__ __forceinline__ unsigned long long *np_ts() {
  return __atomic_load_n(&g_np_ts, __ATOMIC_RELAXED);
}
__device__ __forceinline__ unsigned long long hw_where() {  // HW_ID (wave, SIMD, CU, SE) | XCC_ID
  return (static_cast<unsigned long long>(__builtin_amdgcn_s_getreg((31 << 11) | 4)) << 8) |
         static_cast<unsigned long long>(__builtin_amdgcn_s_getreg((3 << 11) | 20) & 7);
}
__device__ __forceinline__ void np_stamp(int c, int slot_r, int slot_c) {
  if (unsigned long long *ts = np_ts()) {
    ts[static_cast<size_t>(c) * kTs + slot_r] = __builtin_amdgcn_s_memrealtime();
    ts[static_cast<size_t>(c) * kTs + slot_c] = __builtin_amdgcn_s_memtime();
  }
}
__device__ __forceinline__ void np_stamp_val(int c, int slot, unsigned long long v) {
  if (unsigned long long *ts = np_ts()) ts[static_cast<size_t>(c) * kTs + slot] = v;
}

// The one-slot path's general (wrap-capable) batch as one instruction stream (RSAMD_GEN3): per
// draw the next word's v_readlane and the wrap select sit where the compiler placed hazard waits
// (the wrap test reads the step's INPUT state: state 1 always accepts and wraps), so a draw is
// nine vector instructions and no s_nop.  Operand rules kept by hand: one scalar source per
// instruction (N1 in a VGPR), >= 2 instructions between an SGPR / VCC write and its read.
#ifndef RSAMD_GEN3
#define RSAMD_GEN3 1
#endif
#define RSD_S_(x) #x
#define RSD_S(x) RSD_S_(x)
#define RSD_GSTEP_BODY(K, SA)                                      \
  "v_cmp_eq_u32_e64 %[one], 1, %[sv]\n\t"                           \
  "v_ffbh_u32_e32 %[t], %[sv]\n\t"                                  \
  "v_lshrrev_b32_e64 %[t], %[t], -1\n\t"                            \
  "v_and_b32_e32 %[t], %[" SA "], %[t]\n\t"                         \
  "v_cmp_le_u32_e32 vcc, %[t], %[sv]\n\t"                           \
  "v_cndmask_b32_e64 %[wk], %[wk], " RSD_S(K) ", %[one]\n\t"
#define RSD_GSTEP(K, KN, SA, SB)                                   \
  RSD_GSTEP_BODY(K, SA)                                            \
  "v_readlane_b32 %[" SB "], %[wa], " RSD_S(KN) "\n\t"               \
  "v_subbrev_co_u32_e32 %[s2], vcc, 0, %[sv], vcc\n\t"              \
  "v_cndmask_b32_e64 %[sv], %[s2], %[n1], %[one]\n\t"
#define RSD_GSTEP_LAST(K, SA)                                      \
  RSD_GSTEP_BODY(K, SA)                                            \
  "s_nop 1\n\t"                                                    \
  "v_subbrev_co_u32_e32 %[s2], vcc, 0, %[sv], vcc\n\t"              \
  "v_cndmask_b32_e64 %[sv], %[s2], %[n1], %[one]\n\t"
__device__ __forceinline__ void general_batch_asm(uint32_t wa, uint32_t n1v, uint32_t &sv,
                                                  uint32_t &wk) {
  uint32_t t, s2, w0, w1;
  uint64_t one;
  asm volatile(
    "v_readlane_b32 %[w0], %[wa], 0\n\t"
    "s_nop 1\n\t"
    RSD_GSTEP(0, 1, "w0", "w1")
    RSD_GSTEP(1, 2, "w1", "w0")
    RSD_GSTEP(2, 3, "w0", "w1")
    RSD_GSTEP(3, 4, "w1", "w0")
    RSD_GSTEP(4, 5, "w0", "w1")
    RSD_GSTEP(5, 6, "w1", "w0")
    RSD_GSTEP(6, 7, "w0", "w1")
    RSD_GSTEP(7, 8, "w1", "w0")
    RSD_GSTEP(8, 9, "w0", "w1")
    RSD_GSTEP(9, 10, "w1", "w0")
    RSD_GSTEP(10, 11, "w0", "w1")
    RSD_GSTEP(11, 12, "w1", "w0")
    RSD_GSTEP(12, 13, "w0", "w1")
    RSD_GSTEP(13, 14, "w1", "w0")
    RSD_GSTEP(14, 15, "w0", "w1")
    RSD_GSTEP(15, 16, "w1", "w0")
    RSD_GSTEP(16, 17, "w0", "w1")
    RSD_GSTEP(17, 18, "w1", "w0")
    RSD_GSTEP(18, 19, "w0", "w1")
    RSD_GSTEP(19, 20, "w1", "w0")
    RSD_GSTEP(20, 21, "w0", "w1")
    RSD_GSTEP(21, 22, "w1", "w0")
    RSD_GSTEP(22, 23, "w0", "w1")
    RSD_GSTEP(23, 24, "w1", "w0")
    RSD_GSTEP(24, 25, "w0", "w1")
    RSD_GSTEP(25, 26, "w1", "w0")
    RSD_GSTEP(26, 27, "w0", "w1")
    RSD_GSTEP(27, 28, "w1", "w0")
    RSD_GSTEP(28, 29, "w0", "w1")
    RSD_GSTEP(29, 30, "w1", "w0")
    RSD_GSTEP(30, 31, "w0", "w1")
    RSD_GSTEP(31, 32, "w1", "w0")
    RSD_GSTEP(32, 33, "w0", "w1")
    RSD_GSTEP(33, 34, "w1", "w0")
    RSD_GSTEP(34, 35, "w0", "w1")
    RSD_GSTEP(35, 36, "w1", "w0")
    RSD_GSTEP(36, 37, "w0", "w1")
    RSD_GSTEP(37, 38, "w1", "w0")
    RSD_GSTEP(38, 39, "w0", "w1")
    RSD_GSTEP(39, 40, "w1", "w0")
    RSD_GSTEP(40, 41, "w0", "w1")
    RSD_GSTEP(41, 42, "w1", "w0")
    RSD_GSTEP(42, 43, "w0", "w1")
    RSD_GSTEP(43, 44, "w1", "w0")
    RSD_GSTEP(44, 45, "w0", "w1")
    RSD_GSTEP(45, 46, "w1", "w0")
    RSD_GSTEP(46, 47, "w0", "w1")
    RSD_GSTEP(47, 48, "w1", "w0")
    RSD_GSTEP(48, 49, "w0", "w1")
    RSD_GSTEP(49, 50, "w1", "w0")
    RSD_GSTEP(50, 51, "w0", "w1")
    RSD_GSTEP(51, 52, "w1", "w0")
    RSD_GSTEP(52, 53, "w0", "w1")
    RSD_GSTEP(53, 54, "w1", "w0")
    RSD_GSTEP(54, 55, "w0", "w1")
    RSD_GSTEP(55, 56, "w1", "w0")
    RSD_GSTEP(56, 57, "w0", "w1")
    RSD_GSTEP(57, 58, "w1", "w0")
    RSD_GSTEP(58, 59, "w0", "w1")
    RSD_GSTEP(59, 60, "w1", "w0")
    RSD_GSTEP(60, 61, "w0", "w1")
    RSD_GSTEP(61, 62, "w1", "w0")
    RSD_GSTEP(62, 63, "w0", "w1")
    RSD_GSTEP_LAST(63, "w1")
      : [sv] "+v"(sv), [wk] "+v"(wk), [t] "=&v"(t), [s2] "=&v"(s2), [w0] "=&s"(w0),
        [w1] "=&s"(w1), [one] "=&s"(one)
      : [wa] "v"(wa), [n1] "v"(n1v)
      : "vcc");
}

template <bool PY>
__global__ __launch_bounds__(kEntryThreads, 4) void k_np_entry(EntryArgs a,
                                                             const uint32_t *__restrict__ draws) {
  extern __shared__ uint16_t dyn[];
  __shared__ uint32_t wbuf[kK];
#if RSAMD_WLDS
  __shared__ __attribute__((aligned(16))) uint32_t wl[kEntryThreads];  // per-wave word copies
  const uint4 *wq = reinterpret_cast<const uint4 *>(wl + (threadIdx.x & ~63u));
#endif
  __shared__ int sh_red[kEntryThreads / 64];
  __shared__ int sh_evn;
  const int tid = threadIdx.x, lane = tid & 63;
  const int n1 = a.n1, n1p = (n1 + 1) & ~1;
  // the list (state, member-range start) in LDS, compacted in place (4 n1p bytes: two chunks
  // share a CU at every N; with a second pair of arrays as the compaction target, 8 n1p
  // bytes, N = 10 000 took 82.3 KB and one chunk per CU -- C5's entry ran in two rounds)
  uint16_t *st = dyn, *lo = dyn + n1p;
  const int c = blockIdx.x;
  const int64_t t0 = static_cast<int64_t>(c) * a.W;
  const int T = static_cast<int>(std::min<int64_t>(a.W, a.D - t0));
  const int TL = min(T, a.xlim);  // draws this launch may read
  if (a.resume && !a.pause[c]) return;
  const uint32_t *__restrict__ wp = draws + t0;
  uint2 *ev = a.ev + static_cast<size_t>(c) * a.ecap;
  const uint32_t N1 = static_cast<uint32_t>(n1);
  if (tid == 0) {
    np_stamp(c, kTsEntryR0, kTsEntryC0);
    np_stamp_val(c, kTsEntryHw, hw_where());
  }
  int m = n1, t = 0;
  if (a.resume) {  // the paused list, draw position and wrap count
    m = a.fin_m[c];
    t = a.tpos[c];
    // (a bound on everything the resume indexes by: a paused chunk's list and position came from
    // the first launch, a corrupt one fails the parse loudly instead of reading out of range)
    if (m < 1 || m > n1 || t < 0 || t > T) {
      if (tid == 0) atomicOr(a.err, 4);
      return;
    }
    for (int q = tid; q < m; q += kEntryThreads) {
      const uint32_t x = a.fin[static_cast<size_t>(c) * n1 + q];
      st[q] = static_cast<uint16_t>(x >> 16);
      lo[q] = static_cast<uint16_t>(x & 0xffffu);
    }
    if (tid == 0) sh_evn = a.ev_n[c];
  } else {
    for (int q = tid; q < n1; q += kEntryThreads) {
      st[q] = static_cast<uint16_t>(n1 - q);
      lo[q] = static_cast<uint16_t>(q);
    }
    if (tid == 0) sh_evn = 0;
  }
  __syncthreads();
  const int hand = hand_of(n1);
  const int nfast = fast_batches(n1), nfastm = fast_batches_multi(n1);
#ifdef RSAMD_DIAG
  // per path: cycles [0..2] (several slots / multi-slot fast / one-slot), compaction [3], draws [4..6]
  long long eg[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const long long e0 = __builtin_amdgcn_s_memtime();
  long long ec = e0;
#define RSD_ETICK(slot, draws)                                   \
  do {                                                          \
    const long long now_ = __builtin_amdgcn_s_memtime();       \
    eg[slot] += now_ - ec;                                      \
    if ((slot) < 3) eg[(slot) + 4] += (draws);                  \
    ec = now_;                                                  \
  } while (0)
#else
#define RSD_ETICK(slot, draws) \
  do {                         \
  } while (0)
#endif
  if (m > hand) {
    // dense phase: the whole workgroup, slots q = tid + r * kEntryThreads
    uint32_t s[kR];
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      const int q = tid + r * kEntryThreads;
      s[r] = q < m ? st[q] : kSentinel;
    }
    // the words of the next two 64-draw batches, lane l holding draw l of each, loaded one
    // batch ahead in every wave: the stream comes from HBM, and a load issued where it is
    // used cost ~40 cycles per draw (one HBM round trip per batch)
    uint32_t wa = t + lane < TL ? wp[t + lane] : 0u, wb = t + 64 + lane < TL ? wp[t + 64 + lane] : 0u;
    while (m > hand && t < TL) {
      const int kk = min(kK, TL - t);
      const int nr = (m + kEntryThreads - 1) / kEntryThreads;
      if (nr == 1 && kk == 64) {
        // one slot per thread (the common case after the first ~n1 draws): the 64 words in a
        // register of every wave, branch-free steps, a slot's wrap (at most one in 64 draws,
        // as n1 > 64) logged after the batch with one LDS atomic per wave
        // up to nfast batches between compactions (a slot's list neighbours, used by the wrap
        // log, change only at a compaction)
        for (int fb = 0; fb < nfast && TL - t >= 64; ++fb) {
          // (waves holding only empty slots skip the batch: sentinels stay sentinels)
          uint32_t sv = s[0], wk = 0xffffffffu;
#ifdef RSAMD_DIAG
          bool gen = false;  // this wave took the general (wrap-capable) batch
#endif
          if ((tid & ~63) < m) {
#if RSAMD_ONESLOT2
            // Two-bucket batch: when every lane's state stays within its bucket and the one
            // below for the 64 draws (and so cannot wrap), both draw rules are taken off the
            // chain and a step is select / compare / subtract (the general step: clz, shift,
            // and, compare, subtract, wrap test and select).  Sentinel slots qualify.
            uint32_t lw, lw2, sh = 0, M = 0;
            if constexpr (PY) {
              sh = static_cast<uint32_t>(__builtin_clz(sv + 1u));
              lw = (1u << (31u - sh)) - 1u;
              lw2 = sh < 30u ? (1u << (30u - sh)) - 1u : 0x7fffffffu;
            } else {
              M = 0xffffffffu >> __builtin_clz(sv);
              lw = (M >> 1) + 1u;
              lw2 = M > 1u ? (M >> 2) + 1u : 0x7fffffffu;
            }
            const bool fast = sv >= lw2 + 64u && lw2 >= 1u && lw2 != 0x7fffffffu;
            if (__ballot(!fast) == 0ull) {
              if (!PY && RSAMD_ORMASK) {
                const uint32_t M2 = M >> 1;
#if RSAMD_WLDS
                wl[tid] = wa;
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                  const uint4 q4 = wq[j];
                  sv -= (q4.x & (sv | M2)) <= sv ? 1u : 0u;
                  sv -= (q4.y & (sv | M2)) <= sv ? 1u : 0u;
                  sv -= (q4.z & (sv | M2)) <= sv ? 1u : 0u;
                  sv -= (q4.w & (sv | M2)) <= sv ? 1u : 0u;
                }
                __builtin_amdgcn_wave_barrier();
#else
#pragma unroll
                for (int k = 0; k < 64; ++k) {
                  const uint32_t w = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(wa), k));
                  sv -= (w & (sv | M2)) <= sv ? 1u : 0u;
                }
#endif
              } else {
#pragma unroll
                for (int k = 0; k < 64; ++k) {
                  const uint32_t w = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(wa), k));
                  const uint32_t uh = PY ? (w >> sh) : (w & M), ul = PY ? (w >> (sh + 1u)) : (w & (M >> 1));
                  const uint32_t u = sv >= lw ? uh : ul;
                  sv -= u <= sv ? 1u : 0u;
                }
              }
            } else
#endif
            {
#ifdef RSAMD_DIAG
              gen = true;
#endif
#if RSAMD_GEN3
              if constexpr (!PY) {
                uint32_t n1v;
                asm volatile("v_mov_b32 %0, %1" : "=v"(n1v) : "s"(N1));
                general_batch_asm(wa, n1v, sv, wk);
              } else
#endif
#if RSAMD_GEN2
              if constexpr (!PY) {
                // the wrap test off the chain: state 1 always accepts (mask 1) and wraps, so
                // the select reads a compare of the step's INPUT state, written instructions
                // earlier (no dependent hazard wait)
#pragma unroll
                for (int k = 0; k < 64; ++k) {
                  const uint32_t w = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(wa), k));
                  const bool one = sv == 1u;
                  const uint32_t s2 = sv - (masked(w, sv) <= sv ? 1u : 0u);
                  sv = one ? N1 : s2;
                  wk = one ? static_cast<uint32_t>(k) : wk;
                }
              } else
#endif
#pragma unroll
              for (int k = 0; k < 64; ++k) {
                const uint32_t w = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(wa), k));
                sv -= draw_of<PY>(w, sv) <= sv ? 1u : 0u;
                const bool z = sv == 0;
                sv = z ? N1 : sv;
                wk = z ? static_cast<uint32_t>(k) : wk;
              }
            }
          }
          s[0] = sv;
          const uint64_t wr = __ballot(wk != 0xffffffffu);
          if (wr) {
            int base = 0;
            if (lane == 0) base = atomicAdd(&sh_evn, __popcll(wr));
            base = __shfl(base, 0);
            if (wk != 0xffffffffu) {
              const int e = base + static_cast<int>(lane_rank(wr));
              if (e < a.ecap)
                ev[e] = make_uint2(static_cast<uint32_t>(t) + wk + 1u,
                                   lo[tid] | (static_cast<uint32_t>(lo[tid + 1 == m ? 0 : tid + 1]) << 16));
            }
          }
          t += 64;
          wa = wb;
          wb = t + 64 + lane < TL ? wp[t + 64 + lane] : 0u;
#ifdef RSAMD_DIAG
          if (gen) eg[7] += 1;  // general batches of this wave (thread 0's wave reports)
#endif
          RSD_ETICK(2, 64);
        }
      } else if (kk == 64 && nr <= kRFast) {
        // several slots per thread: branch-free steps, each slot's wrap (at most one in 64
        // draws, as n1 > 64) logged after the batch; up to nfastm batches between compactions
        // (member ranges change only at a compaction)
        for (int fb = 0; fb < nfastm && TL - t >= 64; ++fb) {
          uint32_t wk[kRFast];
#pragma unroll
          for (int r = 0; r < kRFast; ++r) wk[r] = 0xffffffffu;
#if RSAMD_MULTI2
          // slot by slot: a slot whose states all stay within their bucket and the one below
          // for the batch takes the two-bucket step (as the one-slot path), else the general one
#pragma unroll
          for (int r = 0; r < kRFast; ++r) {
            if (r >= nr) break;
            uint32_t sv = s[r], wkr = 0xffffffffu;
            uint32_t lw, lw2, sh = 0, M = 0;
            if constexpr (PY) {
              sh = static_cast<uint32_t>(__builtin_clz(sv + 1u));
              lw = (1u << (31u - sh)) - 1u;
              lw2 = sh < 30u ? (1u << (30u - sh)) - 1u : 0x7fffffffu;
            } else {
              M = 0xffffffffu >> __builtin_clz(sv);
              lw = (M >> 1) + 1u;
              lw2 = M > 1u ? (M >> 2) + 1u : 0x7fffffffu;
            }
            const bool fast = sv >= lw2 + 64u && lw2 >= 1u && lw2 != 0x7fffffffu;
            if (__ballot(!fast) == 0ull) {
              if (!PY && RSAMD_ORMASK) {
                const uint32_t M2 = M >> 1;
#if RSAMD_WLDS
                wl[tid] = wa;
                __builtin_amdgcn_wave_barrier();
#pragma unroll 4
                for (int j = 0; j < 16; ++j) {
                  const uint4 q4 = wq[j];
                  sv -= (q4.x & (sv | M2)) <= sv ? 1u : 0u;
                  sv -= (q4.y & (sv | M2)) <= sv ? 1u : 0u;
                  sv -= (q4.z & (sv | M2)) <= sv ? 1u : 0u;
                  sv -= (q4.w & (sv | M2)) <= sv ? 1u : 0u;
                }
                __builtin_amdgcn_wave_barrier();
#else
#pragma unroll 16
                for (int k = 0; k < 64; ++k) {
                  const uint32_t w = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(wa), k));
                  sv -= (w & (sv | M2)) <= sv ? 1u : 0u;
                }
#endif
              } else {
#pragma unroll 16
                for (int k = 0; k < 64; ++k) {
                  const uint32_t w = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(wa), k));
                  const uint32_t uh = PY ? (w >> sh) : (w & M), ul = PY ? (w >> (sh + 1u)) : (w & (M >> 1));
                  const uint32_t u = sv >= lw ? uh : ul;
                  sv -= u <= sv ? 1u : 0u;
                }
              }
            } else {
#pragma unroll 16
              for (int k = 0; k < 64; ++k) {
                const uint32_t w = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(wa), k));
                sv -= draw_of<PY>(w, sv) <= sv ? 1u : 0u;
                const bool z = sv == 0;
                sv = z ? N1 : sv;
                wkr = z ? static_cast<uint32_t>(k) : wkr;
              }
            }
            s[r] = sv;
            wk[r] = wkr;
          }
#else
#pragma unroll 1
          for (int k = 0; k < 64; ++k) {
            const uint32_t w = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(wa), k));
#pragma unroll
            for (int r = 0; r < kRFast; ++r) {
              if (r >= nr) break;
              uint32_t sv = s[r];
              sv -= draw_of<PY>(w, sv) <= sv ? 1u : 0u;
              const bool z = sv == 0;
              s[r] = z ? N1 : sv;
              wk[r] = z ? static_cast<uint32_t>(k) : wk[r];
            }
          }
#endif
#pragma unroll
          for (int r = 0; r < kRFast; ++r) {
            if (r >= nr) break;
            const uint64_t wr = __ballot(wk[r] != 0xffffffffu);
            if (wr) {
              int base = 0;
              if (lane == 0) base = atomicAdd(&sh_evn, __popcll(wr));
              base = __shfl(base, 0);
              if (wk[r] != 0xffffffffu) {
                const int q = tid + r * kEntryThreads;
                const int e = base + static_cast<int>(lane_rank(wr));
                if (e < a.ecap)
                  ev[e] = make_uint2(static_cast<uint32_t>(t) + wk[r] + 1u,
                                     lo[q] | (static_cast<uint32_t>(lo[q + 1 == m ? 0 : q + 1]) << 16));
              }
            }
          }
          t += 64;
          wa = wb;
          wb = t + 64 + lane < TL ? wp[t + 64 + lane] : 0u;
          RSD_ETICK(1, 64);
        }
      } else {
      if (tid < kk) wbuf[tid] = wa;
      __syncthreads();
      for (int k = 0; k < kk; ++k) {
        const uint32_t w = wbuf[k];
#pragma unroll
        for (int r = 0; r < kR; ++r) {
          if (r >= nr) break;
          uint32_t sv = s[r];
          sv -= draw_of<PY>(w, sv) <= sv ? 1u : 0u;
          if (sv == 0) {  // hypothesis end: log the wrap with this trajectory's member range
            sv = N1;
            const int q = tid + r * kEntryThreads;
            const int e = atomicAdd(&sh_evn, 1);
            if (e < a.ecap)
              ev[e] = make_uint2(static_cast<uint32_t>(t + k + 1),
                                 lo[q] | (static_cast<uint32_t>(lo[q + 1 == m ? 0 : q + 1]) << 16));
          }
          s[r] = sv;
        }
      }
      t += kk;
      wa = wb;
      wb = t + 64 + lane < TL ? wp[t + 64 + lane] : 0u;
      RSD_ETICK(0, kk);
      }
      // compaction: equal cyclic neighbours merge, the first of a run keeps its lo (the list
      // stays in cyclic order; where it starts does not matter, so no rotation to a run head:
      // two barriers and a block reduction fewer per compaction); all equal: one survivor
#if RSAMD_CMP1
      if (nr == 1) {
        // one slot per thread (m <= 512): a thread's own slot is its list entry, so the
        // neighbour test is one LDS read and the offsets a ballot rank plus the wave counts
        // (three barriers: the batches read no st entry of another thread)
        const uint32_t sv = s[0];
        if (tid < m) st[tid] = static_cast<uint16_t>(sv);
        __syncthreads();
        const bool keep = tid < m && static_cast<uint16_t>(sv) != st[tid == 0 ? m - 1 : tid - 1];
        const uint16_t lv = tid < m ? lo[tid] : 0;  // read before the barrier: written in place
        const uint64_t kb = __ballot(keep);
        if (lane == 0) sh_red[tid >> 6] = __popcll(kb);
        __syncthreads();
        int base = 0, total = 0;
#pragma unroll
        for (int w = 0; w < kEntryThreads / 64; ++w) {
          const int cw = sh_red[w];
          base += w < (tid >> 6) ? cw : 0;
          total += cw;
        }
        if (keep) {  // in place: o <= tid, and every read of st / lo is behind the barrier
          const int o = base + static_cast<int>(lane_rank(kb));
          st[o] = static_cast<uint16_t>(sv);
          lo[o] = lv;
        }
        // every trajectory in one state: one survivor covering every entry (entry 0 holds it)
        if (total == 0) total = 1;
        __syncthreads();
        m = total;
        s[0] = tid < m ? st[tid] : kSentinel;
        RSD_ETICK(3, 0);
        continue;
      }
#endif
      __syncthreads();
#pragma unroll
      for (int r = 0; r < kR; ++r) {
        if (r >= nr) break;
        const int q = tid + r * kEntryThreads;
        if (q < m) st[q] = static_cast<uint16_t>(s[r]);
      }
      __syncthreads();
      const int per = (m + kEntryThreads - 1) / kEntryThreads;  // <= kR (m <= kMaxN1)
      const int k0 = min(m, tid * per), k1 = min(m, k0 + per);
      // the thread's kept entries (state << 16 | lo) in registers, then written in place once
      // the scan's barriers have ordered every read before every write (o <= p)
      int cnt = 0;
      uint32_t kmask = 0u, kv[kR];
#pragma unroll
      for (int j = 0; j < kR; ++j) {
        const int p = k0 + j;
        kv[j] = 0u;
        if (p < k1) {
          const uint16_t x = st[p];
          if (x != st[p == 0 ? m - 1 : p - 1]) {
            kmask |= 1u << j;
            kv[j] = (static_cast<uint32_t>(x) << 16) | lo[p];
            ++cnt;
          }
        }
      }
      int total;
      int o = block_excl_scan(cnt, sh_red, &total);
#pragma unroll
      for (int j = 0; j < kR; ++j) {
        if ((kmask >> j) & 1u) {
          st[o] = static_cast<uint16_t>(kv[j] >> 16);
          lo[o] = static_cast<uint16_t>(kv[j] & 0xffffu);
          ++o;
        }
      }
      // every trajectory in one state: one survivor covering every entry (entry 0 holds it)
      if (total == 0) total = 1;
      __syncthreads();
      m = total;
#pragma unroll
      for (int r = 0; r < kR; ++r) {
        const int q = tid + r * kEntryThreads;
        s[r] = q < m ? st[q] : kSentinel;
      }
      RSD_ETICK(3, 0);
    }
#ifdef RSAMD_DIAG
    if (a.stats && tid == 0) {
      long long *o = a.stats + static_cast<size_t>(c) * 128 + 100;
      for (int k = 0; k < 7; ++k) o[k] = eg[k];
      o[7] = __builtin_amdgcn_s_memtime() - e0;
      o[8] = t;
      o[9] = m;
      o[10] = eg[7];
    }
#endif
    if (m > hand && t < T) {  // paused at the first stream pass's end: resumed after the second
      for (int q = tid; q < m; q += kEntryThreads)
        a.fin[static_cast<size_t>(c) * n1 + q] = lo[q] | (static_cast<uint32_t>(st[q]) << 16);
      if (tid == 0) {
        a.fin_m[c] = m;
        a.ev_n[c] = sh_evn;
        a.tpos[c] = t;
        a.pause[c] = 1;
      }
      return;
    }
    if (m > hand) {  // chunk done while still dense
      for (int q = tid; q < m; q += kEntryThreads)
        a.fin[static_cast<size_t>(c) * n1 + q] = lo[q] | (static_cast<uint32_t>(st[q]) << 16);
      if (tid == 0) {
        if (!a.resume) a.pause[c] = 0;
        a.fin_m[c] = m;
        a.ev_n[c] = min(sh_evn, a.ecap);
        if (sh_evn > a.ecap) atomicOr(a.err, 1);
        np_stamp(c, kTsEntryR1, kTsEntryC1);
        np_stamp_val(c, kTsEntryT, static_cast<unsigned long long>(t));
        np_stamp_val(c, kTsEntryM, static_cast<unsigned long long>(m));
      }
      return;
    }
  }
  // hand over to k_np_track: the (<= hand) live slots, the wrap count and the position
  __syncthreads();
  for (int q = tid; q < m; q += kEntryThreads)
    a.fin[static_cast<size_t>(c) * n1 + q] = lo[q] | (static_cast<uint32_t>(st[q]) << 16);
  if (tid == 0) {
    a.fin_m[c] = m;
    a.ev_n[c] = sh_evn;
    a.tpos[c] = t;
    if (!a.resume) a.pause[c] = 0;
    np_stamp(c, kTsEntryR1, kTsEntryC1);
    np_stamp_val(c, kTsEntryT, static_cast<unsigned long long>(t));
    np_stamp_val(c, kTsEntryM, static_cast<unsigned long long>(m));
  }
}

// ---- 3b. tracking phase of a chunk: the <= 64 trajectories left after the dense parse --------
// One workgroup per chunk, 8 waves; trajectory q (position q of the chunk's sorted list) runs on
// wave q % 8.  A trajectory advances by windows of 64 draws with the lanes as draws: lane l's
// state is s_l = i - (accepts among lanes < l) (wrapping from 1 to n1 at a hypothesis end), its
// step accepts iff draw_of(w_l, s_l) <= s_l.  The accept mask is the fixed point of
//     acc <- ballot(draw_of(w_l, i - rank_l(acc)) <= i - rank_l(acc)),
// iterated from "all accept": lane 0's state is always right, and once lanes < l are right lane
// l is, so the iteration reaches the sequential answer in at most 65 rounds (2.9 on average at
// N = 2000), and a fixed point IS that answer (induction over the lanes).  Windows cross bucket
// boundaries and hypothesis ends freely.
// Every kCheck draws the trajectories meet at a checkpoint: states that are equal there are the
// same trajectory from then on, so all but the first of each run of equal states (cyclic order
// is preserved by the parse) are dropped, and the survivor's member range extends to the next
// survivor's start.  Wraps are logged with the member range as in k_np_entry.
#ifndef RSAMD_TRACK_WAVES
#define RSAMD_TRACK_WAVES 16
#endif
constexpr int kTrackWaves = RSAMD_TRACK_WAVES;  // waves per chunk workgroup, >= 8 (A/B builds may override)
#ifndef RSAMD_KCHECK
#define RSAMD_KCHECK 4096
#endif
constexpr int kCheck = RSAMD_KCHECK;  // draws per checkpoint interval (A/B builds may override)
// multi-trajectory windows through fast_window (bucket constants on the vector unit) before
// window_step (A/B builds may override).  Measured (C2, tools/r04_np2.sh, two passes): parse
// 6.39 / 6.41 -> 6.28 / 6.26 ms.  The same for the single-trajectory windows of track_one was
// slower (6.74 / 6.75 ms: there the scalar unit is not the bound, the window's latency is, and
// the vector form adds to it)
#ifndef RSAMD_MULTI_VALU
#define RSAMD_MULTI_VALU 1
#endif
// (Measured and removed, round 4, commit "Parse A/B: lockstep chain groups": the chains of a
// wave in lockstep -- fixed-point rounds interleaved -- and 128-draw single-trajectory
// windows; commit "Parse A/B: seeded chunks": chunks parsed from 512 spread entries with the
// previous chunk's trajectories carried in -- entry 1.23 -> 0.85 ms at C2, but the carries'
// heavy tail (tools/seed_sim.c) cost 0.21-0.27 ms more and the parse stayed at 6.25-6.32 ms;
// DESIGN.md §5 "Round 4".)

template <bool PY, bool SMALL>
__device__ __forceinline__ uint32_t wrap_state(int si, int n1) {
  if (si > 0) return static_cast<uint32_t>(si);
  if constexpr (SMALL) return static_cast<uint32_t>(n1 - ((-si) % n1));
  else return static_cast<uint32_t>(si + n1);
}

// ---- one window of one trajectory -----------------------------------------------------------
// State i before the window, lane l holds draw l of the window (lanes >= Wn, outside wm, are
// never accepted).  Returns the accept mask; advances i; wraps (hypothesis ends) in *wr.
//
// Fast path: every state the window can reach lies in i's bucket or the one below (i - 63 >=
// the lower bucket's lowest state), so no hypothesis ends inside and lane l's draw is u_hi (i's
// rule) or u_lo (the lower rule) by whether its state i - rank_l is at least `lowest`: with
// v = i - u and rank_l = accepts among lanes < l, lane l accepts iff
//     rank_l <= (rank_l <= i - lowest ? v_hi : v_lo),
// and the accept mask is the fixed point of that test over rank_l(acc), from "accept unless
// v_hi < 0" (lanes < l right => lane l right, so it reaches the sequential answer, and any
// fixed point is that answer).
// General path (states below 2 x 64, hypothesis ends): the fixed point of
//     acc <- ballot(draw_of(w_l, s_l) <= s_l),  s_l = i - rank_l(acc) (wrapped into 1..n1),
// from "all accept".
// (Measured, tools/ubench/amb_bench2.hip, one wave alone: 5.1 cycles per draw; the one-bucket
// sure / ambiguous split with the ambiguous lanes resolved one by one on the scalar unit: 6.3.)
template <bool PY, bool SMALL>
__device__ __forceinline__ uint64_t window_step(uint32_t w, uint64_t wm, uint32_t &i, int n1,
                                                uint64_t &wr, uint32_t &sl_out) {
  uint32_t lowest, lowest2, sh = 0, M = 0;
  if constexpr (PY) {
    sh = static_cast<uint32_t>(__builtin_clz(i + 1u));
    lowest = (1u << (31u - sh)) - 1u;  // i + 1 in [2^(31-sh), 2^(32-sh) - 1]
    lowest2 = sh < 30u ? (1u << (30u - sh)) - 1u : 0x7fffffffu;
  } else {
    M = 0xffffffffu >> __builtin_clz(i);
    lowest = (M >> 1) + 1u;
    lowest2 = M > 1u ? (M >> 2) + 1u : 0x7fffffffu;
  }
  if (i >= lowest2 + 63u && lowest2 >= 1u) {
    const int c = static_cast<int>(i) - static_cast<int>(lowest);
    const int vh = static_cast<int>(i) - static_cast<int>(PY ? (w >> sh) : (w & M));
    const int vl = static_cast<int>(i) - static_cast<int>(PY ? (w >> (sh + 1u)) : (w & (M >> 1)));
    uint64_t acc = __ballot(vh >= 0) & wm, prev;
    do {
      prev = acc;
      const int rk = static_cast<int>(lane_rank(prev));
      acc = __ballot(rk <= (rk <= c ? vh : vl)) & wm;
    } while (acc != prev);
    i -= static_cast<uint32_t>(__popcll(acc));
    wr = 0;
    sl_out = 0;
    return acc;
  }
  uint64_t acc = wm, prev;
  uint32_t sl;
  do {
    prev = acc;
    sl = wrap_state<PY, SMALL>(static_cast<int>(i) - static_cast<int>(lane_rank(prev)), n1);
    acc = __ballot(draw_of<PY>(w, sl) <= sl) & wm;
  } while (acc != prev);
  wr = __ballot(sl == 1u) & acc;
  sl_out = sl;
  i = wrap_state<PY, SMALL>(static_cast<int>(i) - static_cast<int>(__popcll(acc)), n1);
  return acc;
}

// The fast two-bucket window of window_step for a FULL window (64 draws), with the bucket
// constants computed on the VECTOR unit: i is copied into a VGPR, the mask, the bucket's lowest
// state and the fast-path test are VALU, and the test reaches the scalar unit as one ballot.  A
// CU runs 16-32 busy tracking waves that share ONE scalar unit (1 instruction per cycle)
// against four SIMD-32 vector units (2 cycles per wave64 instruction each), and window_step
// spends ~35 scalar instructions per window against ~17 vector ones (ISA of the round-3
// kernel), so the scalar unit bounds the multi-trajectory phase; this form spends ~8 scalar and
// ~25 vector instructions.  Returns false (and leaves i alone) where the fast path does not
// hold; the caller then runs window_step.  Same fixed point, so the same accept mask.
// The two-bucket fixed point on REJECT masks (numpy rule): lane l's state is s_l = i - (accepts
// below l) = (i - l) + (rejects below l) -- one v_mbcnt pair with i - l as the addend -- and its
// draw is w_l & mask(s_l) = w_l & (s_l | M/2) inside the two buckets (one v_bitop3), so a round
// is mbcnt / mbcnt / bitop3 / compare with one hazard wait, against mbcnt / mbcnt / compare /
// select / compare with two.  From "every lane at state i" (rejects of the rank-0 guess); the
// same fixed point as the accept-mask form.  base = i - l (per lane), iu = i (uniform or its
// vector copy).  Returns the window's reject mask.
#ifndef RSAMD_REJFP
#define RSAMD_REJFP 1
#endif
#ifndef RSAMD_FWPRE
#define RSAMD_FWPRE 1  // fast_window's two-bucket test by leading-zero counts (A/B builds: 0)
#endif
__device__ __forceinline__ uint64_t rej_fixed_point(uint32_t w, uint32_t iu, uint32_t base,
                                                    uint32_t M2) {
  uint64_t r0 = __ballot((w & (iu | M2)) > iu), r1, r2;
  do {  // convergence checked every second round (a fixed point is stable)
    uint32_t sl = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(r0 >> 32),
                                            __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(r0), base));
    r1 = __ballot((w & (sl | M2)) > sl);
    sl = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(r1 >> 32),
                                   __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(r1), base));
    r2 = __ballot((w & (sl | M2)) > sl);
    r0 = r2;
  } while (r2 != r1);
  return r2;
}

// The same two-bucket fixed point from "all accept" (lane l at state base_l = i - l), with the
// state per lane in a VGPR: returns the window's reject mask.  Converged when two successive
// rounds agree, checked every second round.
#ifndef RSAMD_BLOCK4
#define RSAMD_BLOCK4 1  // single-trajectory blocks of four windows under one test (A/B: 0)
#endif
#ifndef RSAMD_PARTIAL
#define RSAMD_PARTIAL 0  // blocks run their first windows fast when only those stay in two buckets
                         // (A/B: 1; measured 4.52 against 4.44-4.46 ms per C2 parse, not kept)
#endif
#ifndef RSAMD_BLOCK4M
#define RSAMD_BLOCK4M 1  // the same blocks in the multi-trajectory intervals (A/B: 0)
#endif
#ifndef RSAMD_SINGLE_PRIO
#define RSAMD_SINGLE_PRIO 0  // s_setprio of the single-trajectory wave (A/B; measured: no gain)
#endif
__device__ __forceinline__ uint64_t rej_fixed_point_aa(uint32_t w, uint32_t base, uint32_t M2) {
  uint64_t r = __ballot((w & (base | M2)) > base), r1, r2;
  do {
    uint32_t sl = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(r >> 32),
                                            __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(r), base));
    r1 = __ballot((w & (sl | M2)) > sl);
    sl = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(r1 >> 32),
                                   __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(r1), base));
    r2 = __ballot((w & (sl | M2)) > sl);
    r = r2;
  } while (r2 != r1);
  return r2;
}
// The same fixed point checked after every round: fewer vector instructions per window where
// the waves are issue-bound (the multi-trajectory phase) rather than latency-bound
[[maybe_unused]] __device__ __forceinline__ uint64_t rej_fixed_point_aa1(uint32_t w, uint32_t base, uint32_t M2) {
  uint64_t r = __ballot((w & (base | M2)) > base), rn;
  for (;;) {
    const uint32_t sl = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(r >> 32),
                                                  __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(r), base));
    rn = __ballot((w & (sl | M2)) > sl);
    if (rn == r) return rn;
    r = rn;
  }
}
#ifndef RSAMD_MULTI_FP
#define RSAMD_MULTI_FP rej_fixed_point_aa  // multi-trajectory blocks (A/B: rej_fixed_point_aa1)
#endif
#ifndef RSAMD_SINGLE_FP
#define RSAMD_SINGLE_FP rej_fixed_point_aa  // one-per-wave blocks (A/B: rej_fixed_point_aa1)
#endif
// add + popcount(r) on the vector unit: the mask comes from a vector compare, so the count never
// takes the vector -> scalar -> vector round trip (s_bcnt1 then a VGPR operand: ~20 cycles more
// per window, tools/ubench/lat_bench.hip).  The s_nop pair covers the SGPR read after the VALU
// write, as the compiler places it before v_mbcnt.
__device__ __forceinline__ uint32_t vbcnt_add(uint64_t r, uint32_t add) {
  uint32_t o;
  asm volatile("s_nop 1\n v_bcnt_u32_b32 %0, %1, %2\n v_bcnt_u32_b32 %0, %3, %0"
               : "=&v"(o)
               : "s"(static_cast<uint32_t>(r)), "v"(add), "s"(static_cast<uint32_t>(r >> 32)));
  return o;
}

template <bool PY>
__device__ __forceinline__ bool fast_window(uint32_t w, uint32_t &i) {
  uint32_t iv;
  asm volatile("v_mov_b32 %0, %1" : "=v"(iv) : "s"(i));  // a vector copy of the uniform state
  uint32_t lowest, lowest2, sh = 0, M = 0;
  if constexpr (PY) {
    sh = static_cast<uint32_t>(__builtin_clz(iv + 1u));
    lowest = (1u << (31u - sh)) - 1u;
    lowest2 = sh < 30u ? (1u << (30u - sh)) - 1u : 0x7fffffffu;
  } else {
    M = 0xffffffffu >> __builtin_clz(iv);
    lowest = (M >> 1) + 1u;
    lowest2 = M > 1u ? (M >> 2) + 1u : 0x7fffffffu;
  }
#if RSAMD_FWPRE
  if constexpr (!PY && RSAMD_REJFP) {
    // two buckets hold the window iff i - 63 >= M/4 + 1 = 2^30 >> clz(i) (signed: i < 63 fails
    // too), tested by one compare whose ballot is the branch condition
    const uint32_t cz = static_cast<uint32_t>(__builtin_clz(iv));
    const int lw2 = static_cast<int>(0x40000000u >> cz);
    if (__ballot(static_cast<int>(iv) - 63 >= lw2) == 0ull) return false;  // uniform
    const uint32_t rej = static_cast<uint32_t>(__popcll(
        rej_fixed_point(w, iv, iv - static_cast<uint32_t>(threadIdx.x & 63), 0x7fffffffu >> cz)));
    i -= 64u - rej;
    return true;
  }
#endif
  const bool fast = iv >= lowest2 + 63u && lowest2 >= 1u && lowest2 != 0x7fffffffu;
  if (__builtin_amdgcn_ballot_w64(fast) == 0ull) return false;  // uniform: all lanes agree
  if constexpr (!PY && RSAMD_REJFP) {
    const uint32_t rej = static_cast<uint32_t>(__popcll(
        rej_fixed_point(w, iv, iv - static_cast<uint32_t>(threadIdx.x & 63), M >> 1)));
    i -= 64u - rej;
    return true;
  }
  const int c = static_cast<int>(iv) - static_cast<int>(lowest);
  const int vh = static_cast<int>(iv) - static_cast<int>(PY ? (w >> sh) : (w & M));
  const int vl = static_cast<int>(iv) - static_cast<int>(PY ? (w >> (sh + 1u)) : (w & (M >> 1)));
  // convergence checked every second round (a fixed point is stable)
  uint64_t a0 = __ballot(vh >= 0), a1, a2;
  do {
    int rk = static_cast<int>(lane_rank(a0));
    a1 = __ballot(rk <= (rk <= c ? vh : vl));
    rk = static_cast<int>(lane_rank(a1));
    a2 = __ballot(rk <= (rk <= c ? vh : vl));
    a0 = a2;
  } while (a2 != a1);
  i -= static_cast<uint32_t>(__popcll(a2));
  return true;
}

// One checkpoint interval [t, cp) of a single trajectory (the common case once a chunk's
// trajectories have merged down to at most one per wave): the tight loop.  Windows of 64 draws
// at fixed offsets, so their words are read from LDS four windows ahead into registers (the
// read never waits on the state).  While every state a window can reach lies in i's bucket or
// the one below, window_step's two-bucket fixed point decides it.  (Measured,
// tools/ubench/amb_bench2.hip: 5.1 cycles per draw for one wave alone, against 7.9 for the
// earlier 256-draw windows read from LDS at the top of each step.)
template <bool PY, bool SMALL>
__device__ __forceinline__ void track_window(int n1, int ecap, uint32_t w, int *s_evn, uint2 *ev,
                                             uint32_t &i, uint32_t range, int d, int cp) {
  const int lane = threadIdx.x & 63;
  const int Wn = min(64, cp - d);
  const uint64_t wm = Wn == 64 ? ~0ull : ((1ull << Wn) - 1ull);
  uint64_t wr;
  uint32_t sl;
  (void)window_step<PY, SMALL>(w, wm, i, n1, wr, sl);
  if (wr) {  // hypothesis ends: the next hypothesis starts at the following draw
    int eb = 0;
    if (lane == 0) eb = atomicAdd(s_evn, __popcll(wr));
    eb = __shfl(eb, 0);
    if (((wr >> lane) & 1ull)) {
      const int e = eb + static_cast<int>(lane_rank(wr));
      if (e < ecap) ev[e] = make_uint2(static_cast<uint32_t>(d + lane + 1), range);
    }
  }
}

template <bool PY, bool SMALL>
__device__ __forceinline__ uint32_t track_one(const EntryArgs &a, const uint32_t *sw, int *s_evn,
                                              uint2 *ev, uint32_t i, uint32_t range, int t,
                                              int cp) {
  const int lane = threadIdx.x & 63;
  const int n1 = uni(a.n1), ecap = uni(a.ecap);  // in SGPRs for the whole loop
  constexpr int kAhead = 4;
  // lanes beyond cp read words of the wrapped buffer: never accepted (wm)
  uint32_t q[kAhead];
#pragma unroll
  for (int k = 0; k < kAhead; ++k) q[k] = sw[(64 * k + lane) & (kCheck - 1)];
  // the scalar unit is shared by the CU's waves (two chunks, ~14 busy waves): keep the
  // per-window scalar work small -- the bucket constants are recomputed only when i leaves the
  // bucket, full windows skip the window mask, and the fixed point checks convergence every
  // second round (a fixed point is stable, so an extra round changes nothing).  C2 stream
  // 7.49 -> 6.82 ms (the same fixed point with per-window constants, window mask and a check
  // every round: window_step)
  uint32_t M = 0, sh = 0, lowest = 0, fast_min = 0xffffffffu;
  auto set_bucket = [&]() {
    uint32_t lowest2;
    if constexpr (PY) {
      sh = static_cast<uint32_t>(__builtin_clz(i + 1u));
      lowest = (1u << (31u - sh)) - 1u;
      lowest2 = sh < 30u ? (1u << (30u - sh)) - 1u : 0x7fffffffu;
    } else {
      M = 0xffffffffu >> __builtin_clz(i);
      lowest = (M >> 1) + 1u;
      lowest2 = M > 1u ? (M >> 2) + 1u : 0x7fffffffu;
    }
    fast_min = lowest2 >= 1u && lowest2 < 0x7fffffffu ? lowest2 + 63u : 0xffffffffu;
  };
  set_bucket();
  for (int d = t; d < cp; d += 64 * kAhead) {
    int kf = 0;  // windows of this block run with the state in a VGPR
#if RSAMD_BLOCK4
    if constexpr (!PY && RSAMD_REJFP) {
      // A block of kAhead full windows under ONE two-bucket test: every state the block can
      // reach (i .. i - 64 kAhead + 1) lies in i's bucket or the one below, where numpy's mask is
      // s | M/2, so no per-window bucket test is needed.  The state lives in a VGPR as
      // base = i - lane and advances by v_bcnt of the window's reject mask, so a window never
      // waits for a vector -> scalar round trip; the fixed point starts from "all accept" and
      // is checked every second round (tools/ubench/single_bench.hip, one wave alone: 5.6 ->
      // 3.9 cycles per draw; with the other chunk's waves beside it and s_setprio: 7.5 -> 3.8)
      // (a block whose lower states leave the two buckets runs its first kf windows so, where
      // kf = the full windows above the lower bucket's floor, then the rest window by window)
      const uint32_t Mb = 0xffffffffu >> __builtin_clz(i);
      const uint32_t l2b = Mb > 3u ? (Mb >> 2) + 1u : 0xffffffffu;
      kf = l2b != 0xffffffffu && i >= l2b + 63u ? static_cast<int>((i - l2b + 1u) >> 6) : 0;
      kf = min(min(kf, kAhead), (cp - d) >> 6);
      if (!RSAMD_PARTIAL && kf < kAhead) kf = 0;
      if (kf > 0) {
        const uint32_t M2 = Mb >> 1;
        uint32_t base = i - static_cast<uint32_t>(lane);
#pragma unroll
        for (int k = 0; k < kAhead; ++k) {
          if (k < kf) {
            const uint32_t w = q[k];
            q[k] = sw[(d - t + 64 * (kAhead + k) + lane) & (kCheck - 1)];
            base = vbcnt_add(RSAMD_SINGLE_FP(w, base, M2), base - 64u);
          }
        }
        i = uni(base);  // lane 0's base is i
        if (kf == kAhead) continue;
      }
    }
#endif
#pragma unroll
    for (int k = 0; k < kAhead; ++k) {
      if (k < kf) continue;  // run above in the block's fast part
      const uint32_t w = q[k];
      q[k] = sw[(d - t + 64 * (kAhead + k) + lane) & (kCheck - 1)];
      const int dk = d + 64 * k;
      if (dk + 64 <= cp) {
        if (i < lowest || i > (PY ? (lowest << 1) : (lowest << 1) - 1u)) set_bucket();  // left it
        if (i >= fast_min) {
          if constexpr (!PY && RSAMD_REJFP) {
            const uint32_t rej = static_cast<uint32_t>(__popcll(
                rej_fixed_point(w, i, i - static_cast<uint32_t>(lane), M >> 1)));
            i -= 64u - rej;
            continue;
          }
          const int c = static_cast<int>(i) - static_cast<int>(lowest);
          const int vh = static_cast<int>(i) - static_cast<int>(PY ? (w >> sh) : (w & M));
          const int vl = static_cast<int>(i) - static_cast<int>(PY ? (w >> (sh + 1u)) : (w & (M >> 1)));
          uint64_t a0 = __ballot(vh >= 0), a1, a2;
          do {
            int rk = static_cast<int>(lane_rank(a0));
            a1 = __ballot(rk <= (rk <= c ? vh : vl));
            rk = static_cast<int>(lane_rank(a1));
            a2 = __ballot(rk <= (rk <= c ? vh : vl));
            a0 = a2;
          } while (a2 != a1);
          i -= static_cast<uint32_t>(__popcll(a2));
          continue;
        }
      }
      if (dk < cp) {
        track_window<PY, SMALL>(n1, ecap, w, s_evn, ev, i, range, dk, cp);
        set_bucket();
      }
    }
  }
  return i;
}

// One checkpoint interval [t, cp) of R trajectories q = wv + r kTrackWaves (r < nq), a window
// of 64 draws per step.
template <int R, bool PY, bool SMALL>
__device__ __forceinline__ void track_interval(const EntryArgs &a, const uint32_t *sw,
                                               uint32_t *s_st, const uint32_t *s_lo, int *s_evn,
                                               uint2 *ev, int m, int wv, int nq, int t, int cp,
                                               long long *dg) {
  const int lane = threadIdx.x & 63;
  const int n1 = a.n1;
  uint32_t i[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int q = wv + (r < nq ? r : nq - 1) * kTrackWaves;
    i[r] = uni(s_st[q]);
  }
  // the member range of chain r, read from LDS only where a wrap is logged (rare): SGPRs are
  // what limits this kernel's residency (two 16-wave workgroups per CU need <= ~84)
  auto range_of = [&](int r) {
    const int q = wv + r * kTrackWaves;
    return s_lo[q] | (s_lo[q + 1 == m ? 0 : q + 1] << 16);
  };
  // one window of chain r at draw dk (Wn draws)
  auto one_window = [&](uint32_t w, int Wn, int dk, int r) {
#if RSAMD_MULTI_VALU
    if (Wn == 64 && fast_window<PY>(w, i[r])) return;
#endif
    // (the window mask only where the general step runs -- the opaque copy keeps the
    // compiler from hoisting it into every window: scalar instructions on the CU's shared
    // scalar unit)
    int wn_ = Wn;
    asm volatile("" : "+s"(wn_));
    const uint64_t wm = wn_ == 64 ? ~0ull : ((1ull << wn_) - 1ull);
    uint64_t wr;
    uint32_t sl;
    (void)window_step<PY, SMALL>(w, wm, i[r], n1, wr, sl);
    if (wr) {  // hypothesis ends: the next hypothesis starts at the following draw
      int eb = 0;
      if (lane == 0) eb = atomicAdd(s_evn, __popcll(wr));
      eb = __shfl(eb, 0);
      if (((wr >> lane) & 1ull)) {
        const int e = eb + static_cast<int>(lane_rank(wr));
        if (e < a.ecap) ev[e] = make_uint2(static_cast<uint32_t>(dk + lane + 1), range_of(r));
      }
    }
  };
  int d = t;
#if RSAMD_BLOCK4 && RSAMD_BLOCK4M
  if constexpr (!PY && RSAMD_REJFP) {
    // blocks of four full windows: a chain whose block stays within its bucket and the one below
    // runs the four windows with its state in a VGPR (as track_one; no scalar work per window on
    // the CU's shared scalar unit), the others window by window
    for (; d + 256 <= cp; d += 256) {
      uint32_t q[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) q[k] = sw[(d - t + 64 * k + lane) & (kCheck - 1)];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (r < nq) {
          const uint32_t Mb = 0xffffffffu >> __builtin_clz(i[r]);
          const uint32_t l2b = Mb > 3u ? (Mb >> 2) + 1u : 0xffffffffu;
          int kf = l2b != 0xffffffffu && i[r] >= l2b + 63u
                             ? min(4, static_cast<int>((i[r] - l2b + 1u) >> 6)) : 0;
          if (!RSAMD_PARTIAL && kf < 4) kf = 0;
          if (kf > 0) {
            const uint32_t M2 = Mb >> 1;
            uint32_t base = i[r] - static_cast<uint32_t>(lane);
#pragma unroll
            for (int k = 0; k < 4; ++k)
              if (k < kf) base = vbcnt_add(RSAMD_MULTI_FP(q[k], base, M2), base - 64u);
            i[r] = uni(base);
          }
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (k >= kf) one_window(q[k], 64, d + 64 * k, r);
        }
      }
    }
  }
#endif
  uint32_t wn = sw[(d - t + lane) & (kCheck - 1)];  // draws beyond cp are never accepted (lanes >= Wn)
  while (d < cp) {
    const int Wn = min(64, cp - d);
    const uint32_t w = wn;
    if (d + 64 < cp) wn = sw[(d + 64 - t + lane) & (kCheck - 1)];
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (r < nq) one_window(w, Wn, d, r);
#ifdef RSAMD_DIAG
    dg[0] += 1;
#endif
    d += Wn;
  }
#pragma unroll
  for (int r = 0; r < R; ++r)
    if (r < nq && lane == 0) s_st[wv + r * kTrackWaves] = i[r];
}

template <bool PY, bool SMALL, int CAP>  // CAP: list capacity = hand_of(n1)
__device__ __forceinline__ void np_track_body(const EntryArgs &a, const uint32_t *__restrict__ draws) {
  // the draws of the current checkpoint interval in LDS (all trajectories of the chunk read
  // them; a window's read is issued one window ahead), the next interval in flight in VGPRs
  __shared__ uint32_t s_w[2][kCheck];
  __shared__ uint32_t s_st[CAP], s_lo[CAP];
  __shared__ int s_m, s_evn;
  constexpr int kStride = 64 * kTrackWaves;
  constexpr int kPer = (kCheck + kStride - 1) / kStride;  // draws per thread per interval
  const int c = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = uni(tid >> 6);
  int m = a.fin_m[c];
  if (m > CAP) return;  // the chunk ended while dense: final already
  const int n1 = a.n1;
  const int64_t t0 = static_cast<int64_t>(c) * a.W;
  const int T = static_cast<int>(std::min<int64_t>(a.W, a.D - t0));
  int t = a.tpos[c];
  if (t >= T) return;
  if (t < 0 || m < 1) {  // a corrupt hand-over: fail the parse, index nothing
    if (threadIdx.x == 0) atomicOr(a.err, 4);
    return;
  }
  // (the busy wave is wave q % kTrackWaves for trajectory q; placing the trajectories by the
  // waves' hardware SIMD ids, the two chunks of a CU on opposite SIMDs: no gain, 6.46 vs 6.40 ms
  // at C2 with the SGPRs capped at 70 -- this kernel must stay within ~80 SGPRs, at 84-86 it
  // loses its second 16-wave workgroup per CU, +1.3 ms)
  const int wq = wv;
  const uint32_t *__restrict__ wp = draws + t0;
  uint2 *ev = a.ev + static_cast<size_t>(c) * a.ecap;
  // RSAMD_DIAG: windows (multi-slot path), cycles with one / several trajectories, wave-intervals
  // with one / several, intervals
  long long dg[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#ifdef RSAMD_DIAG
  const long long k0 = __builtin_amdgcn_s_memtime();
  const long long r0 = __builtin_amdgcn_s_memrealtime();
#endif
  if (tid < m) {
    const uint32_t f = a.fin[static_cast<size_t>(c) * n1 + tid];
    s_st[tid] = f >> 16;
    s_lo[tid] = f & 0xffffu;
  }
  if (tid == 0) {
    s_evn = a.ev_n[c];
    np_stamp(c, kTsTrackR0, kTsTrackC0);
    np_stamp_val(c, kTsTrackHw, hw_where());
    if (m <= kTrackWaves) {  // one trajectory per wave from the start
      np_stamp(c, kTsSingleR, kTsSingleC);
      np_stamp_val(c, kTsSingleT, static_cast<unsigned long long>(t));
    }
  }
  uint32_t nx[kPer];
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int j = k * kStride + tid, x = t + j;
    nx[k] = j < kCheck && x < T ? wp[x] : 0u;
  }
  int buf = 0;
  while (t < T) {
    const int cp = min(T, t + kCheck);
    uint32_t *sw = s_w[buf];
#pragma unroll
    for (int k = 0; k < kPer; ++k)
      if (k * kStride + tid < kCheck) sw[k * kStride + tid] = nx[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kPer; ++k) {  // the next interval's draws
      const int j = k * kStride + tid, x = cp + j;
      nx[k] = j < kCheck && x < T ? wp[x] : 0u;
    }
    // this wave's trajectories q = wv, wv + 8, ... advance together (independent fixed-point
    // chains interleaved: the latency of one round is shared by up to kTrackSlots of them)
    const int nq = m > wq ? (m - wq + kTrackWaves - 1) / kTrackWaves : 0;
#ifdef RSAMD_DIAG
    const long long c0 = __builtin_amdgcn_s_memtime();
#endif
    if (nq == 1) {
      // the single trajectory's wave is its chunk's critical path: issue priority over the
      // other chunk's waves on the SIMD (tools/ubench/single_bench.hip: a parse wave beside a
      // busy one 7.5 -> 5.2 cycles per draw at priority 3)
      if (RSAMD_SINGLE_PRIO) __builtin_amdgcn_s_setprio(RSAMD_SINGLE_PRIO);
      const uint32_t i1 = track_one<PY, SMALL>(
          a, sw, &s_evn, ev, uni(s_st[wq]), uni(s_lo[wq] | (s_lo[wq + 1 == m ? 0 : wq + 1] << 16)),
          t, cp);
      if (RSAMD_SINGLE_PRIO) __builtin_amdgcn_s_setprio(0);
      if (lane == 0) s_st[wq] = i1;
    }
    else if (nq == 2) track_interval<2, PY, SMALL>(a, sw, s_st, s_lo, &s_evn, ev, m, wq, 2, t, cp, dg);
    else if (nq > 2 && nq <= 4) track_interval<4, PY, SMALL>(a, sw, s_st, s_lo, &s_evn, ev, m, wq, nq, t, cp, dg);
    else if constexpr (CAP > 4 * kTrackWaves) {  // more than four per wave: the 128-entry list
      if (nq > 4) track_interval<8, PY, SMALL>(a, sw, s_st, s_lo, &s_evn, ev, m, wq, nq, t, cp, dg);
    }
#ifdef RSAMD_DIAG
    {
      const long long dc = __builtin_amdgcn_s_memtime() - c0;  // busy cycles of this wave
      if (nq == 1) dg[1] += dc, dg[3] += 1;
      else if (nq > 1) dg[2] += dc, dg[4] += 1;
      dg[5] += 1;
    }
#endif
    __syncthreads();
    if (wv == 0) {  // merge equal states (runs are contiguous in cyclic order)
      constexpr int kH = CAP / 64;
      uint32_t sq[kH], lq[kH];
      uint64_t eq[kH];
      int neq = 0;
#pragma unroll
      for (int h = 0; h < kH; ++h) {
        const int q = lane + 64 * h;
        const bool v = q < m;
        sq[h] = v ? s_st[q] : 0u;
        const uint32_t sp = v ? s_st[q == 0 ? m - 1 : q - 1] : 0u;
        lq[h] = v ? s_lo[q] : 0u;
        eq[h] = __ballot(v && m > 1 && sq[h] == sp);
        neq += static_cast<int>(__popcll(eq[h]));
      }
      const bool one = neq == m;  // every entry equals its predecessor: one trajectory left
      uint64_t kb[kH];
      bool keep[kH];
#pragma unroll
      for (int h = 0; h < kH; ++h) {
        const int q = lane + 64 * h;
        keep[h] = one ? q == 0 : (q < m && !((eq[h] >> lane) & 1ull));
        kb[h] = __ballot(keep[h]);
      }
      __builtin_amdgcn_wave_barrier();
      int base = 0;
#pragma unroll
      for (int h = 0; h < kH; ++h) {
        if (keep[h]) {
          const int dst = base + static_cast<int>(lane_rank(kb[h]));
          s_st[dst] = sq[h];
          s_lo[dst] = lq[h];
        }
        base += static_cast<int>(__popcll(kb[h]));
      }
      if (lane == 0) s_m = base;
    }
    __syncthreads();
    if (tid == 0 && m > kTrackWaves && s_m <= kTrackWaves) {  // down to one per wave
      np_stamp(c, kTsSingleR, kTsSingleC);
      np_stamp_val(c, kTsSingleT, static_cast<unsigned long long>(cp));
    }
    m = uni(s_m);
    t = cp;
    buf ^= 1;
  }
  if (tid < m) a.fin[static_cast<size_t>(c) * n1 + tid] = s_lo[tid] | (s_st[tid] << 16);
  if (tid == 0) {
    a.fin_m[c] = m;
    a.ev_n[c] = min(s_evn, a.ecap);
    if (s_evn > a.ecap) atomicOr(a.err, 1);
    np_stamp(c, kTsTrackR1, kTsTrackC1);
  }
#ifdef RSAMD_DIAG
  if (a.stats && lane == 0) {
    long long *o = a.stats + static_cast<size_t>(c) * 128 + wv * 6;
    for (int k = 0; k < 6; ++k) o[k] = dg[k];
    if (wv == 0) {
      a.stats[static_cast<size_t>(c) * 128 + 120] = __builtin_amdgcn_s_memtime() - k0;
      a.stats[static_cast<size_t>(c) * 128 + 121] = r0;  // start / end, 100 MHz real-time clock
      a.stats[static_cast<size_t>(c) * 128 + 122] = __builtin_amdgcn_s_memrealtime();
    }
  }
#else
  (void)dg;
#endif
}

// The tracking kernel must stay within ~80 SGPRs: at 84-86 it loses its second 16-wave
// workgroup per CU (+1.3 ms at C2).  The 64-entry kernel needs 70; the 128-entry one (large N)
// is capped at 72 (spilling ~20 SGPRs to VGPR lanes: 86 uncapped).
#ifndef RSAMD_TRACK_SGPR
#define RSAMD_TRACK_SGPR 0  // >0: cap the 64-entry tracking kernel's SGPRs (A/B builds)
#endif
template <bool PY, bool SMALL>
__global__ __launch_bounds__(64 * kTrackWaves)
#if RSAMD_TRACK_SGPR
__attribute__((amdgpu_num_sgpr(RSAMD_TRACK_SGPR)))
#endif
void k_np_track(EntryArgs a,
                                                                const uint32_t *__restrict__ draws) {
  np_track_body<PY, SMALL, 64>(a, draws);
}
template <bool PY>
__global__ __launch_bounds__(64 * kTrackWaves) __attribute__((amdgpu_num_sgpr(72))) void
k_np_track128(EntryArgs a, const uint32_t *__restrict__ draws) {
  np_track_body<PY, false, 128>(a, draws);
}

// ---- 5. keep the wraps of the true trajectory (in place, order preserved) -----------------
__global__ __launch_bounds__(64) void k_np_filter(uint2 *__restrict__ ev, const int *ev_n,
                                                  const int *ent, int *vcnt, int ecap) {
  const int c = blockIdx.x, l = threadIdx.x;
  const uint32_t a = static_cast<uint32_t>(ent[c]);
  const int n = ev_n[c];
  uint2 *e = ev + static_cast<size_t>(c) * ecap;
  int cnt = 0;
  // four 64-entry batches in flight per step (the loop waited one memory round trip per batch:
  // 35 us per C2 launch); in place is safe: a batch's kept entries land at or below its reads
  constexpr int kF = 4;
  for (int b = 0; b < n; b += 64 * kF) {
    uint2 x[kF];
#pragma unroll
    for (int f = 0; f < kF; ++f) {
      const int i = b + 64 * f + l;
      x[f] = i < n ? e[i] : make_uint2(0u, 0u);
    }
#pragma unroll
    for (int f = 0; f < kF; ++f) {
      const int i = b + 64 * f + l;
      const uint32_t lo = x[f].y & 0xffffu, hi = x[f].y >> 16;
      const bool ok = i < n && (lo < hi ? (a >= lo && a < hi) : (a >= lo || a < hi));
      const uint64_t bl = __ballot(ok);
      if (ok) e[cnt + static_cast<int>(lane_rank(bl))].x = x[f].x;
      cnt += __popcll(bl);
    }
  }
  if (l == 0) vcnt[c] = cnt;
}

// ---- 4. compose the chunk maps on the GPU ------------------------------------------------
// Chunk c's final list maps entry list index a (state n1 - a) to the state of the entry with the
// largest start lo <= a (cyclically: the largest lo overall if none); chunk 0 starts a
// hypothesis (a = 0).  A map is thus a step function of a: its entries rotated so that lo
// ascends, value v = n1 - state, below the first lo the last value.  Two maps compose on the
// first one's steps (g o f has f's steps, values g(v)), so a composition of consecutive chunks
// holds <= 64 steps at every level.  Per block of kComposeBlock chunks, all in LDS: the rows
// are staged (coalesced, every load in flight) and rotated, an up-sweep composes sibling pairs
// (a wave per node, a lane per step, a binary search of the sibling's steps), the down-sweep
// hands each node's entry to its left child and the left child's value of it to the right
// one; the block's root carries the entry to the next block.  (The serial walk of wave 0 --
// one ballot / find-last / readlane per chunk -- took 104 us for C2's 512 chunks and
// 0.3-0.6 ms for the 1 000-4 000 chunks of a split parse; it remains for blocks holding a
// chunk that ended dense, whose list may exceed 64 entries.)
constexpr int kComposeBlock = 256;
constexpr int kComposeNodes = 2 * kComposeBlock + 8;  // all levels of a block's tree
__device__ __forceinline__ int step_eval(const uint32_t *node, int m, int e) {
  int lo = 0, hi = m;  // the largest k with lo_k <= e (lo ascending), else m - 1
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (static_cast<int>(node[mid] & 0xffffu) <= e) lo = mid + 1;
    else hi = mid;
  }
  return static_cast<int>(node[lo > 0 ? lo - 1 : m - 1] >> 16);
}
// row_off (optional): where chunk c's list starts in fin (the gathered, packed maps of a
// sharded parse); null: row c at c * n1.
__global__ __launch_bounds__(1024) void k_np_compose(const uint32_t *__restrict__ fin,
                                                     const int *__restrict__ fin_m, int n1, int C,
                                                     int *__restrict__ ent,
                                                     const int64_t *__restrict__ row_off) {
  auto row = [&](int c) -> const uint32_t * {
    return fin + (row_off ? row_off[c] : static_cast<int64_t>(c) * n1);
  };
  __shared__ uint32_t pool[kComposeNodes * 64];  // tree nodes (the serial walk: its rows)
  __shared__ int nm[kComposeNodes], ne[kComposeNodes];  // steps and entry per node
  __shared__ int big, carry;
  const int tid = threadIdx.x, l = tid & 63, wv = tid >> 6;
  if (tid == 0) carry = 0;
  for (int c0 = 0; c0 < C; c0 += kComposeBlock) {
    const int nb = min(kComposeBlock, C - c0);
    if (tid == 0) big = 0;
    __syncthreads();
    for (int k = tid; k < nb; k += 1024) {
      nm[k] = fin_m[c0 + k];
      if (nm[k] > 64) big = 1;
    }
    __syncthreads();
    // the block's rows, every load of a thread in flight at once
    {
      constexpr int kPer = kComposeBlock * 64 / 1024;
      uint32_t v[kPer];
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        const int k = tid + j * 1024, r = k >> 6, q = k & 63;
        v[j] = r < nb && q < nm[r] && nm[r] <= 64 ? row(c0 + r)[q] : 0xffffffffu;
      }
#pragma unroll
      for (int j = 0; j < kPer; ++j) pool[tid + j * 1024] = v[j];
    }
    __syncthreads();
    // rotated so that lo ascends (a wave per row); tree rows hold lo | v << 16
    for (int r = wv; r < nb; r += 16) {
      const int m = nm[r];
      if (m > 64) continue;
      const uint32_t x = l < m ? pool[r * 64 + l] : 0xffffffffu;
      uint32_t mn = x & 0xffffu;
#pragma unroll
      for (int o = 32; o; o >>= 1) mn = min(mn, static_cast<uint32_t>(__shfl_xor(static_cast<int>(mn), o)));
      const uint64_t at = __ballot(l < m && (x & 0xffffu) == mn);
      const int p0 = __ffsll(static_cast<long long>(at)) - 1;
      __builtin_amdgcn_wave_barrier();
      if (l < m)
        pool[r * 64 + (l - p0 >= 0 ? l - p0 : l - p0 + m)] =
            big ? x : ((x & 0xffffu) | ((static_cast<uint32_t>(n1) - (x >> 16)) << 16));
    }
    __syncthreads();
    if (big) {  // the serial walk (rows: lo | state << 16)
      if (wv == 0) {
        int a = carry;
        for (int r = 0; r < nb; ++r) {
          const int c = c0 + r, m = nm[r];
          ne[r] = a;
          if (m <= 64) {
            const uint32_t x = l < m ? pool[r * 64 + l] : 0xffffffffu;
            const uint64_t le = __ballot(l < m && static_cast<int>(x & 0xffffu) <= a);
            const int idx = le ? 63 - __builtin_clzll(le) : m - 1;
            a = n1 - static_cast<int>(static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(x), idx)) >> 16);
            continue;
          }
          uint32_t kb = 0, kt = 0;
          bool hb = false, ht = false;
          for (int k = l; k < m; k += 64) {
            const uint32_t x = row(c)[k];
            const uint32_t lo = x & 0xffffu, key = (lo << 16) | (x >> 16);
            if (static_cast<int>(lo) <= a && (!hb || key > kb)) kb = key, hb = true;
            if (!ht || key > kt) kt = key, ht = true;
          }
          const uint64_t anyb = __ballot(hb);
          // keys of valid rows are distinct; invalid lanes hold 0 and lose every max below
          uint32_t mb = hb ? kb : 0u, mt = ht ? kt : 0u;
#pragma unroll
          for (int o = 32; o; o >>= 1) {
            mb = max(mb, static_cast<uint32_t>(__shfl_xor(static_cast<int>(mb), o)));
            mt = max(mt, static_cast<uint32_t>(__shfl_xor(static_cast<int>(mt), o)));
          }
          a = n1 - static_cast<int>((anyb ? mb : mt) & 0xffffu);
        }
        if (l == 0) carry = a;
      }
      __syncthreads();
      for (int k = tid; k < nb; k += 1024) ent[c0 + k] = ne[k];
      __syncthreads();
      continue;
    }
    // up-sweep: node j of a level composes nodes 2j (first) and 2j + 1 of the level below
    int nodes = nb, base = 0;
    while (nodes > 1) {
      const int nn = (nodes + 1) >> 1, nbase = base + nodes;
      for (int j = wv; j < nn; j += 16) {
        const int f = base + 2 * j, g = f + 1, mf = nm[f];
        if (l < mf) {
          const uint32_t x = pool[f * 64 + l];
          pool[(nbase + j) * 64 + l] =
              g < nbase ? (x & 0xffffu) | (static_cast<uint32_t>(step_eval(pool + g * 64, nm[g], static_cast<int>(x >> 16))) << 16)
                        : x;
        }
        if (l == 0) nm[nbase + j] = mf;
      }
      __syncthreads();
      base = nbase;
      nodes = nn;
    }
    // down-sweep from the root (at base) with the carried entry
    if (tid == 0) {
      ne[base] = carry;
      carry = step_eval(pool + base * 64, nm[base], carry);  // the next block's entry
    }
    __syncthreads();
    while (base > 0) {
      // the level below the current one: find its base and size by walking up from 0
      int cb = 0, cn = nb;
      while (cb + cn < base) {
        cb += cn;
        cn = (cn + 1) >> 1;
      }
      const int pn = (cn + 1) >> 1;
      for (int j = tid; j < pn; j += 1024) {
        const int e = ne[base + j], f = cb + 2 * j;
        ne[f] = e;
        if (2 * j + 1 < cn) ne[f + 1] = step_eval(pool + f * 64, nm[f], e);
      }
      __syncthreads();
      base = cb;
    }
    for (int k = tid; k < nb; k += 1024) ent[c0 + k] = ne[k];
    __syncthreads();
  }
}

// exclusive prefix sum of the per-chunk start counts; cnt[0] = min(H, total) hypotheses this
// segment delivers (the tuple kernel and the host read it)
__global__ __launch_bounds__(1024) void k_np_scan(const int *__restrict__ vcnt, int C,
                                                  int *__restrict__ off, int64_t H,
                                                  int64_t *__restrict__ got) {
  __shared__ int sh[16];
  __shared__ int carry;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (tid == 0) carry = 0;
  __syncthreads();
  for (int b = 0; b < C; b += 1024) {
    const int i = b + tid;
    const int v = i < C ? vcnt[i] : 0;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o);
      if (lane >= o) x += y;
    }
    if (lane == 63) sh[wid] = x;
    __syncthreads();
    int base = carry;
    for (int w = 0; w < wid; ++w) base += sh[w];
    if (i < C) off[i] = base + x - v;
    __syncthreads();
    if (tid == 1023) carry = base + x;
    __syncthreads();
  }
  if (tid == 0) *got = std::min<int64_t>(H, static_cast<int64_t>(carry));
}

// ---- 6. one wave per hypothesis: a window of W <= 64 words per step ------------------------
// Within a window every state keeps the mask of the first (W <= i - mask/2), so lane l's draw
// u_l = w_l & mask is accepted for sure if u_l <= i - l (its state is at least i - l), rejected
// for sure if u_l > i, and only the rare lanes in between are resolved in order.  Accepted
// lanes have consecutive states, so the swap partners J[state - 1] land in LDS together.  The
// trace keeps the k positions in wave-uniform registers: for state s >= 8 a position p < s can
// only move to s (when J[s - 1] == p), found by a ballot over 64 states at a time.
#ifndef RSAMD_TUP_WAVES
#define RSAMD_TUP_WAVES 4
#endif
constexpr int kTupWaves = RSAMD_TUP_WAVES;  // waves (hypotheses) per tuple workgroup
#ifndef RSAMD_TUP_BLK
#define RSAMD_TUP_BLK 128
#endif
// words per ring block (loaded one block ahead).  Measured (C2, k_np_tuples_wave per launch):
// direct global loads per window 872 us; blocks of 64 / 128 / 256 / 512 / 1024 words 691 / 684
// / 744 / 906 / 1099 us (the larger rings cost occupancy)
constexpr int kTupBlk = RSAMD_TUP_BLK;
constexpr int kTupRing = 2 * kTupBlk;       // words staged per wave
// u16 entries per wave after the ring: the swap partners J[s - 1] of the states s = 1..n1, then
// one dummy slot per lane (the rejected lanes of a two-bucket window store there, so the store
// needs no exec-mask change on the scalar unit)
// (RSAMD_TUPF: the table holds, instead of J, the first later state F[v] = min{s >= 8, s > v :
// J[s - 1] = v} for every partner value v -- the trace then follows F from each position, a
// few dependent reads instead of a ballot per 64 states -- plus J for the states 1..7.)
#ifndef RSAMD_TUPF
#define RSAMD_TUPF 1
#endif
// (entries 0..n1: the trace reads F at every state it reaches, n1 included)
__host__ __device__ constexpr int tup_jpad(int n1) { return (n1 + 2) & ~1; }
__host__ __device__ constexpr int tup_table(int n1) { return tup_jpad(n1) + 64 + (RSAMD_TUPF ? 8 : 0); }
__host__ __device__ constexpr int64_t tup_wave_bytes(int n1) {
  return static_cast<int64_t>(sizeof(uint32_t)) * kTupRing +
         static_cast<int64_t>(sizeof(uint16_t)) * tup_table(n1);
}
__host__ __device__ constexpr int64_t tup_lds_bytes(int n1) { return tup_wave_bytes(n1) * kTupWaves; }
// Waves per tuple workgroup for population n1: kTupWaves unless a smaller workgroup keeps at
// least a quarter more waves resident in a CU's 160 KB of LDS.  (C5, N = 10 000: 21 KB per
// wave, so 4-wave workgroups left ONE workgroup -- four waves, one per SIMD -- on a CU; 1-wave
// workgroups keep 7.  C2 keeps 4: 28 waves against at most 31.)
int64_t env_i64(const char *name);
inline int tup_waves_for(int n1) {
  static const int forced = static_cast<int>(env_i64("RSAMD_TUP_TW"));  // A/B: 1 .. kTupWaves
  if (forced >= 1 && forced <= kTupWaves) return forced;
  constexpr int64_t kLdsCu = 160 * 1024;
  const int64_t pw = tup_wave_bytes(n1);
  const int64_t base = (kLdsCu / (kTupWaves * pw)) * kTupWaves;
  int best = kTupWaves;
  int64_t bw = base;
  for (int t = kTupWaves - 1; t >= 1; --t) {
    const int64_t waves = (kLdsCu / (t * pw)) * t;
    if (waves > bw) {
      bw = waves;
      best = t;
    }
  }
  return 4 * bw >= 5 * base ? best : kTupWaves;
}
// ring blocks held in registers ahead of the one being parsed: the stream comes from HBM (far
// larger than the caches), and at large N the LDS table leaves one wave per SIMD, so one block
// ahead (two 64-draw windows) waited a full HBM round trip per block
#ifndef RSAMD_TUP_AHEAD
#define RSAMD_TUP_AHEAD 6
#endif
constexpr int kTupAhead = RSAMD_TUP_AHEAD;
#ifndef RSAMD_TUP_BLOCK2
#define RSAMD_TUP_BLOCK2 1  // two-window blocks with a VGPR state (A/B: 0)
#endif
#ifndef RSAMD_TUP_FP
#define RSAMD_TUP_FP rej_fixed_point_aa  // (A/B: rej_fixed_point_aa1)
#endif
#ifndef RSAMD_TUP_VWIN
#define RSAMD_TUP_VWIN 1  // general windows with a mask per lane (A/B: 0)
#endif


template <bool PY>
__global__ __launch_bounds__(64 * kTupWaves) void k_np_tuples_wave(
    const uint32_t *__restrict__ draws, const int64_t *__restrict__ starts,
    const int64_t *__restrict__ got, int64_t lo, int64_t hi, int n1, int kk,
    int32_t *__restrict__ out, int *err, int64_t nwords) {
  // per wave: a ring of kTupRing words of the hypothesis (blocks of kTupBlk words, kTupAhead
  // blocks in flight in registers), then the swap partners J (uint16 x tup_table(n1))
  extern __shared__ uint32_t tup_lds[];
  const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
  // hypotheses [lo, hi) of the segment (those the caller asked for), out row h - lo
  const int64_t h = lo + static_cast<int64_t>(blockIdx.x) * (blockDim.x >> 6) + wv;
  if (h >= hi || h >= *got) return;  // wave-uniform; the kernel has no workgroup barrier
  uint32_t *ring = tup_lds + static_cast<size_t>(wv) * (kTupRing + tup_table(n1) / 2);
  uint16_t *J = reinterpret_cast<uint16_t *>(ring + kTupRing);
  const int64_t a = starts[h], b = starts[h + 1];
  const uint32_t *__restrict__ src = draws + a;
  // read-ahead never leaves the stream allocation (nwords words from draws[0]), nor the
  // hypothesis by more than one window: the queue's look-ahead past the hypothesis's last word
  // (up to kTupAhead blocks, ~25 % of a C2 hypothesis) would fetch the next hypothesis's words
  // from HBM a second time (calibrated PMC, profiles/r06a_traffic.json: 1.46 GB per C2 run
  // against 1.11 GB of hypothesis words); clamped loads all read one word (one cache line)
  const int64_t lim = min(nwords - 1 - a, b - a + 63);
  auto ld = [&](int64_t x) { return src[x < lim ? x : lim]; };
  constexpr int kPerLane = kTupBlk / 64;
  uint32_t nb[kTupAhead][kPerLane];  // blocks 1 .. kTupAhead after the ring's newest
#pragma unroll
  for (int k = 0; k < kPerLane; ++k) ring[64 * k + l] = ld(64 * k + l);
#pragma unroll
  for (int q = 0; q < kTupAhead; ++q)
#pragma unroll
    for (int k = 0; k < kPerLane; ++k) nb[q][k] = ld((q + 1) * kTupBlk + 64 * k + l);
  int filled = kTupBlk;  // words of the hypothesis in the ring (relative to a)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const uint64_t below = (1ull << l) - 1ull;
  uint32_t i = static_cast<uint32_t>(n1);
  int o = 0;  // words parsed
  // A full 64-draw window in i's bucket and the one below (every state it can reach is at
  // least the lower bucket's lowest): the two-bucket fixed point of the tracking kernel
  // (fast_window), the bucket constants on the vector unit, the swap partners stored by every
  // lane (rejected lanes into their dummy slot).  PMC per C2 launch (r04d_pmc / r04d_pmc2):
  // SALU 3.28e8 -> 1.83e8, VALU 3.74e8 -> 4.03e8; 668 -> 591-611 us (profiles/r04d_tuples_ab.txt).
  const uint32_t jdummy = static_cast<uint32_t>(tup_jpad(n1)) + static_cast<uint32_t>(l);
#if RSAMD_TUPF
  uint16_t *F = J, *J7 = J + tup_jpad(n1) + 64;  // F[v] (0xffff: none), then J of states 1..7
  for (int x = l; x < tup_jpad(n1) / 2; x += 64) reinterpret_cast<uint32_t *>(F)[x] = 0xffffffffu;
  // F[v] = s for the lanes that store: the parse runs the states downwards, so a later window
  // simply overwrites; inside one window equal partners are resolved to the smallest state
  // (read back, the losers that should have won store again)
  auto fstore = [&](bool st, uint32_t v, uint32_t sl) {
    const uint32_t fi = st ? v : jdummy;
    F[fi] = static_cast<uint16_t>(sl);
    __builtin_amdgcn_wave_barrier();
    uint64_t bad = __ballot(st && F[fi] > sl);
    for (int r = 0; bad && r < 64; ++r) {  // each round settles at least one lane
      if ((bad >> l) & 1ull) F[fi] = static_cast<uint16_t>(sl);
      __builtin_amdgcn_wave_barrier();
      bad = __ballot(st && F[fi] > sl);
    }
  };
  // the read-back alone, for stores already made (rare path: a partner value twice in a window)
  [[maybe_unused]] auto fstore_fix = [&](bool st, uint32_t fi, uint32_t sl) {
    __builtin_amdgcn_wave_barrier();
    uint64_t bad = __ballot(st && F[fi] > sl);
    for (int r = 0; bad && r < 64; ++r) {
      if ((bad >> l) & 1ull) F[fi] = static_cast<uint16_t>(sl);
      __builtin_amdgcn_wave_barrier();
      bad = __ballot(st && F[fi] > sl);
    }
  };
#endif
  auto window2 = [&]() -> bool {
    uint32_t iv;
    asm volatile("v_mov_b32 %0, %1" : "=v"(iv) : "s"(i));
#if RSAMD_TUPF && RSAMD_FWPRE
    if constexpr (!PY && RSAMD_REJFP) {  // the tracking kernel's fast_window test and rounds
      const uint32_t cz = static_cast<uint32_t>(__builtin_clz(iv));
      if (__ballot(static_cast<int>(iv) - 63 >= static_cast<int>(0x40000000u >> cz)) == 0ull)
        return false;  // uniform
      const uint32_t wd = ring[(o + l) & (kTupRing - 1)];
      const uint32_t M2 = 0x7fffffffu >> cz, base = iv - static_cast<uint32_t>(l);
      const uint64_t rj = rej_fixed_point(wd, iv, base, M2);
      const uint32_t sl = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(rj >> 32),
                                                    __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(rj), base));
      const uint32_t v = wd & (sl | M2);
      fstore(v < sl, v, sl);
      i -= 64u - static_cast<uint32_t>(__popcll(rj));
      o += 64;
      return true;
    }
#endif
    uint32_t lowest, lowest2, sh = 0, M = 0;
    if constexpr (PY) {
      sh = static_cast<uint32_t>(__builtin_clz(iv + 1u));
      lowest = (1u << (31u - sh)) - 1u;
      lowest2 = sh < 30u ? (1u << (30u - sh)) - 1u : 0x7fffffffu;
    } else {
      M = 0xffffffffu >> __builtin_clz(iv);
      lowest = (M >> 1) + 1u;
      lowest2 = M > 1u ? (M >> 2) + 1u : 0x7fffffffu;
    }
    const bool ok = iv >= lowest2 + 63u && lowest2 >= 1u && lowest2 != 0x7fffffffu;
    if (__builtin_amdgcn_ballot_w64(ok) == 0ull) return false;  // uniform
    const uint32_t wd = ring[(o + l) & (kTupRing - 1)];
#if RSAMD_TUPF
    if constexpr (!PY && RSAMD_REJFP) {
      const uint32_t M2 = M >> 1, base = iv - static_cast<uint32_t>(l);
      const uint64_t rj = rej_fixed_point(wd, iv, base, M2);
      const uint32_t sl = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(rj >> 32),
                                                    __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(rj), base));
      const uint32_t v = wd & (sl | M2);  // the lane's draw = its swap partner when accepted
      fstore(v < sl, v, sl);              // (rejected lanes: v > sl)
      i -= 64u - static_cast<uint32_t>(__popcll(rj));
      o += 64;
      return true;
    }
#endif
    const uint32_t uh = PY ? (wd >> sh) : (wd & M), ul = PY ? (wd >> (sh + 1u)) : (wd & (M >> 1));
    const int c = static_cast<int>(iv) - static_cast<int>(lowest);
    const int vh = static_cast<int>(iv) - static_cast<int>(uh);
    const int vl = static_cast<int>(iv) - static_cast<int>(ul);
    uint64_t a0 = __ballot(vh >= 0), a1, a2;
    int rk;
    do {
      rk = static_cast<int>(lane_rank(a0));
      a1 = __ballot(rk <= (rk <= c ? vh : vl));
      rk = static_cast<int>(lane_rank(a1));
      a2 = __ballot(rk <= (rk <= c ? vh : vl));
      a0 = a2;
    } while (a2 != a1);
    // (rk = rank_l(a1) = rank_l(a2); recomputing it from an opaque a2 so that the loop does not
    // carry the lanes' predicates as exec-masked scalar copies measured the same, 604 vs 591 us)
    const bool hb = rk <= c;
    const bool ac = rk <= (hb ? vh : vl);
#if RSAMD_TUPF
    {
      const uint32_t sl = iv - static_cast<uint32_t>(rk), v = hb ? uh : ul;  // sl >= 32 here
      fstore(ac && v < sl, v, sl);
    }
#else
    J[ac ? iv - static_cast<uint32_t>(rk) - 1u : jdummy] = static_cast<uint16_t>(hb ? uh : ul);
#endif
    i -= static_cast<uint32_t>(__popcll(a2));
    o += 64;
    return true;
  };
  // one window of W <= 64 draws (states i .. i - W + 1 share the draw rule's mask / shift):
  // the general form, for the states below the two-bucket range and the hypothesis end
  auto window = [&]() {
    uint32_t L, msk = 0, sh = 0;
    if constexpr (PY) {
      sh = static_cast<uint32_t>(__builtin_clz(i + 1u));
      L = i + 2u - (1u << (31u - sh));
    } else {
      msk = 0xffffffffu >> __builtin_clz(i);
      L = i - (msk >> 1);
    }
    const int W = L < 64u ? static_cast<int>(L) : 64;
    const bool in = l < W;
    const uint32_t wd = ring[(o + l) & (kTupRing - 1)];
    const uint32_t u = in ? (PY ? (wd >> sh) : (wd & msk)) : 0xffffffffu;
    const uint32_t lo_s = i - static_cast<uint32_t>(l);
    uint64_t acc = __ballot(in && u <= lo_s);
    const bool am = in && u > lo_s && u <= i;
    const uint64_t amb = __ballot(am);
    if (amb) {
      // the ambiguous lanes by the fixed point acc <- ballot(u_l <= i - rank_l(acc)) (only they
      // can change; lanes < l right => lane l right, so it ends at the sequential answer), from
      // "every ambiguous lane accepts".  (One lane at a time on the scalar unit made the kernel
      // scalar-issue bound: 4.2e8 SALU per C2 launch.)
      const uint64_t sure = acc;
      uint64_t a = sure | amb, prev;
      do {
        prev = a;
        a = sure | __ballot(am && u <= i - lane_rank(prev));
      } while (a != prev);
      acc = a;
    }
#if RSAMD_TUPF
    {
      const bool ap = (acc >> l) & 1ull;
      const uint32_t sl = i - static_cast<uint32_t>(__popcll(acc & below));
      if (ap && sl <= 7u) J7[sl - 1u] = static_cast<uint16_t>(u);
      fstore(ap && sl >= 8u && u < sl, u, sl);
    }
#else
    if ((acc >> l) & 1ull)
      J[i - static_cast<uint32_t>(__popcll(acc & below)) - 1u] = static_cast<uint16_t>(u);
#endif
    i -= static_cast<uint32_t>(__popcll(acc));
    o += W;
  };
#if RSAMD_TUPF
  // The general window with a mask per lane (numpy rule): 64 draws whatever buckets they span,
  // the hypothesis end inside -- lane l's state s_l = i - rank_l(acc), its draw w_l & mask(s_l)
  // accepted iff <= s_l, lanes past the end (s_l < 1) never; the fixed point from "all
  // accept" is the sequential answer (lane 0 is right, and lane l is once lanes < l are).  The
  // single-mask window above stops at every bucket edge, so below the two-bucket range a
  // hypothesis took ~30 windows of a few draws each; this takes two or three.
  [[maybe_unused]] auto window_v = [&]() {
    const uint32_t wd = ring[(o + l) & (kTupRing - 1)];
    uint32_t iv;
    asm volatile("v_mov_b32 %0, %1" : "=v"(iv) : "s"(i));
    uint64_t acc = ~0ull, prev;
    uint32_t sl, u;
    do {
      prev = acc;
      sl = iv - lane_rank(prev);
      u = wd & (0xffffffffu >> __builtin_clz(sl | 1u));
      acc = __ballot(static_cast<int>(sl) >= 1 && u <= sl);
    } while (acc != prev);
    const bool ap = (acc >> l) & 1ull;
    if (ap && sl <= 7u) J7[sl - 1u] = static_cast<uint16_t>(u);
    fstore(ap && sl >= 8u && u < sl, u, sl);
    const uint64_t endb = __ballot(ap && sl == 1u);  // state 1 always accepts: the end
    i -= static_cast<uint32_t>(__popcll(acc));
    o += endb ? __ffsll(static_cast<long long>(endb)) : 64;
  };
#endif
  // The register queue rotates by unrolling (slot q is refilled in turn), never by moving a
  // register: a move of a load's destination would wait for that load.
  // (a two-bucket window never ends the hypothesis: only the general one is followed by the
  // test; unconditional refills let the compiler's wait counts keep five of six blocks in flight
  // -- the guarded form waited for every load at every refill -- which measured the same)
  for (;;) {
#pragma unroll
    for (int q = 0; q < kTupAhead; ++q) {
      while (o + 64 <= filled) {
#if RSAMD_TUP_BLOCK2 && RSAMD_TUPF && RSAMD_REJFP
        if constexpr (!PY) {
          // Two windows under one two-bucket test (all 128 states at least the lower bucket's
          // lowest), the state per lane in a VGPR advanced by v_bcnt (as the tracking kernel's
          // blocks), both windows' stores checked by one read-back: the scalar unit, not the
          // vector unit, bounded the window-by-window form (PMC: SALU 1.97e8 per C2 launch).
          uint32_t iv;
          asm volatile("v_mov_b32 %0, %1" : "=v"(iv) : "s"(i));
          const uint32_t cz = static_cast<uint32_t>(__builtin_clz(iv));
          if (o + 128 <= filled &&
              __ballot(static_cast<int>(iv) - 127 >= static_cast<int>(0x40000000u >> cz)) != 0ull) {
            const uint32_t M2 = 0x7fffffffu >> cz;
            uint32_t base = iv - static_cast<uint32_t>(l);
            const uint32_t wd0 = ring[(o + l) & (kTupRing - 1)];
            const uint32_t wd1 = ring[(o + 64 + l) & (kTupRing - 1)];
            const uint64_t r0 = RSAMD_TUP_FP(wd0, base, M2);
            const uint32_t sl0 = __builtin_amdgcn_mbcnt_hi(
                static_cast<uint32_t>(r0 >> 32), __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(r0), base));
            const uint32_t v0 = wd0 & (sl0 | M2);
            const bool st0 = v0 < sl0;
            const uint32_t fi0 = st0 ? v0 : jdummy;
            F[fi0] = static_cast<uint16_t>(sl0);
            base = vbcnt_add(r0, base - 64u);
            const uint64_t r1 = RSAMD_TUP_FP(wd1, base, M2);
            const uint32_t sl1 = __builtin_amdgcn_mbcnt_hi(
                static_cast<uint32_t>(r1 >> 32), __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(r1), base));
            const uint32_t v1 = wd1 & (sl1 | M2);
            const bool st1 = v1 < sl1;
            const uint32_t fi1 = st1 ? v1 : jdummy;
            F[fi1] = static_cast<uint16_t>(sl1);
            base = vbcnt_add(r1, base - 64u);
            __builtin_amdgcn_wave_barrier();
            // a later (smaller) state of window 1 may already have replaced window 0's entry: the
            // check is F <= sl, and a fix only ever lowers an entry
            const uint32_t c0 = F[fi0], c1 = F[fi1];
            if (__ballot((st0 && c0 > sl0) || (st1 && c1 > sl1))) {
              fstore_fix(st0, fi0, sl0);
              fstore_fix(st1, fi1, sl1);
            }
            i = __builtin_amdgcn_readfirstlane(base);  // lane 0's base is i
            o += 128;
            continue;
          }
        }
#endif
        if (window2()) continue;
#if RSAMD_TUPF && RSAMD_TUP_VWIN
        if constexpr (!PY) window_v();
        else window();
#else
        window();
#endif
        if (i == 0) goto parsed;
      }
      // the oldest block in flight lands in the ring; its slot loads the next
#pragma unroll
      for (int k = 0; k < kPerLane; ++k) ring[(filled + 64 * k + l) & (kTupRing - 1)] = nb[q][k];
#pragma unroll
      for (int k = 0; k < kPerLane; ++k)
        nb[q][k] = ld(filled + kTupAhead * kTupBlk + 64 * k + l);
      filled += kTupBlk;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
parsed:
  const int64_t d = a + o;
  if (d != b) {
    if (l == 0) atomicOr(err, 2);
    return;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // Trace positions 0..7 through the swaps in the order the shuffle's effect unwinds: states
  // 1..7 by the full transposition rule, then for s >= 8 ascending a position p < s moves to s
  // exactly when J[s - 1] == p.  64 states per step; one ballot per step tests all eight
  // positions at once (a hit is rare once s is large), and only a hit is resolved per position.
  uint32_t p[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) p[k] = static_cast<uint32_t>(k);
  const int s1 = n1 < 7 ? n1 : 7;
  for (int s = 1; s <= s1; ++s) {  // states below 8: the full transposition rule
#if RSAMD_TUPF
    const uint32_t j = J7[s - 1], us = static_cast<uint32_t>(s);
#else
    const uint32_t j = J[s - 1], us = static_cast<uint32_t>(s);
#endif
#pragma unroll
    for (int k = 0; k < 8; ++k) p[k] = p[k] == us ? j : (p[k] == j ? us : p[k]);
  }
#if RSAMD_TUPF
  // position k moves to F[p] (the first later state whose partner it is), then on from there;
  // lane k follows its chain (~ln(n1 / 8) steps)
  if (l < kk) {
    uint32_t v = p[0];
#pragma unroll
    for (int k = 1; k < 8; ++k) v = l == k ? p[k] : v;
    for (;;) {  // F[v] > v, so at most n1 steps; anything else is a corrupt table: loud
      const uint32_t nx = F[v];
      if (nx == 0xffffu) break;
      if (nx <= v || nx > static_cast<uint32_t>(n1)) {
        atomicOr(err, 4);
        break;
      }
      v = nx;
    }
    out[(h - lo) * kk + l] = static_cast<int32_t>(v);
  }
  return;
#endif
  for (int s0 = 8; s0 <= n1; s0 += 64) {
    const int s = s0 + l;
    const uint32_t jv = s <= n1 ? static_cast<uint32_t>(J[s - 1]) : 0xffffffffu;
    // any position hit: the minimum of jv ^ p[k] is zero (one vector compare, one ballot)
    uint32_t mn = jv ^ p[0];
#pragma unroll
    for (int k = 1; k < 8; ++k) mn = min(mn, jv ^ p[k]);
    if (!__ballot(mn == 0u)) continue;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      uint64_t bb = __ballot(jv == p[k]);
      while (bb) {
        const int f = __ffsll(static_cast<long long>(bb)) - 1;
        p[k] = static_cast<uint32_t>(s0 + f);
        bb = __ballot(jv == p[k]) & ~((2ull << f) - 1ull);
      }
    }
  }
  if (l < kk) {
    uint32_t v = p[0];
#pragma unroll
    for (int k = 1; k < 8; ++k) v = l == k ? p[k] : v;
    out[(h - lo) * kk + l] = static_cast<int32_t>(v);
  }
}

// ---- 7. what the host needs after a segment, in one copy ----------------------------------
struct NpResult {
  int64_t got;      // hypotheses delivered
  int64_t used;     // draws they consumed (starts[got])
  int32_t err, pad_;
  uint32_t blk[kN];  // tempered stream block holding the next draw (when pos + used > 624)
};

__global__ __launch_bounds__(64) void k_np_result(const uint32_t *__restrict__ stream,
                                                  const int64_t *__restrict__ starts, int pos,
                                                  const int *__restrict__ err,
                                                  NpResult *__restrict__ r) {
  const int l = threadIdx.x;
  const int64_t got = r->got;
  const int64_t used = got > 0 ? starts[got] : 0;
  const int64_t W = pos + used;
  if (W > kN) {
    const int64_t b = (W - 1) / kN;
    for (int t = l; t < kN; t += 64) r->blk[t] = stream[b * kN + t];
  }
  if (l == 0) {
    r->used = used;
    r->err = *err;
  }
}

// ---- host ------------------------------------------------------------------------------------
// Level polynomials as the jump kernel reads them: per polynomial its set bits below kDeg, the
// even ones first (ne of them), then the odd ones; all polynomials' lists concatenated.
struct JumpBits {
  std::vector<int32_t> all;
  std::vector<int> off, n, ne;
  void add(const std::vector<uint64_t> &p) {
    off.push_back(static_cast<int>(all.size()));
    const size_t n0 = all.size();
    for (int par = 0; par < 2; ++par) {
      for (int i = par; i < kDeg; i += 2)  // as the LDS byte offset of its aligned word pair
        if ((p[static_cast<size_t>(i) >> 6] >> (i & 63)) & 1u) all.push_back(8 * (i >> 1));
      if (par == 0) ne.push_back(static_cast<int>(all.size() - n0));
    }
    const int nb = static_cast<int>(all.size() - n0), nev = ne.back();
    n.push_back(nb);
    // k_mt_jump_slide's section after the slice: 2 kPhases + 1 starts, then the bits again by
    // (phase, parity) -- phase p, even; phase p, odd; phase p + 1, even ... -- each run padded to
    // a multiple of 16 with the phase's zero offset (its reads land on zeros: an XOR of 0), so
    // every batch of 16 is full.  Bit i is in phase i / kN <=> 8 (i >> 1) / (4 kN) (kN even).
    const size_t tab = all.size();
    all.resize(tab + 2 * kPhases + 1);
    const int pad0 = static_cast<int>(all.size());
    int ke = 0, ko = nev;
    for (int ph = 0; ph < kPhases; ++ph) {
      const int32_t zoff = 4 * (kRing + kMirror) + (ph >> 2) * (4 * kRing);
      for (int par = 0; par < 2; ++par) {
        all[tab + static_cast<size_t>(2 * ph + par)] = static_cast<int32_t>(all.size()) - pad0;
        int &k = par ? ko : ke;
        const int end = par ? nb : nev;
        int cnt = 0;
        while (k < end && all[n0 + static_cast<size_t>(k)] < 4 * (ph + 1) * kN) {
          all.push_back(all[n0 + static_cast<size_t>(k)]);
          ++k;
          ++cnt;
        }
        for (; cnt % 16; ++cnt) all.push_back(zoff);
      }
    }
    all[tab + 2 * kPhases] = static_cast<int32_t>(all.size()) - pad0;
  }
};

// A small process-wide cache of level polynomials, keyed by (kind, JB, levels).  Entries are
// immutable once built and are copied out under the mutex, so thread ranks of one process
// (ThreadComm) may ask concurrently; at most kJumpCache entries are kept (oldest dropped).
// With the fast arithmetic of mt_jump.cpp a new generator length costs a few ms of host time
// (x^(624 JB) from cached powers of x^624, then the tree's products).
constexpr size_t kJumpCache = 8;
std::mutex g_jump_mu;
double g_jump_host_ms = 0.0;  // host time spent building level polynomials (rs_np_host_stats)
int64_t g_jump_builds = 0;
void jump_bits_cached(int kind, int JB, int levels, JumpBits &out) {
  static std::vector<std::pair<std::array<int, 3>, std::shared_ptr<const JumpBits>>> cache;
  std::lock_guard<std::mutex> g(g_jump_mu);
  const std::array<int, 3> key{kind, JB, levels};
  for (auto &e : cache)
    if (e.first == key) {
      out = *e.second;
      return;
    }
  const auto t0 = std::chrono::steady_clock::now();
  auto jb = std::make_shared<JumpBits>();
  std::vector<uint64_t> p;
  rs::mt_jump_poly(static_cast<uint64_t>(kN) * static_cast<uint64_t>(JB), p);
  if (kind == 0) {
    // radix 2: level k is x^(2^k J), k < kLevels
    for (int k = 0; k < levels; ++k) {
      if (k) rs::mt_poly_square(p);
      jb->add(p);
    }
  } else {
    // radix R: level k's multipliers m = 1 .. R-1 are x^(m R^k J), index k (R-1) + m - 1;
    // even powers by squaring (cheaper than a product): b^2m = (b^m)^2, b^(2m+1) = b^2m b.
    // The levels are independent given their bases b_k = x^(R^k J) (b_{k+1} = b_k^R by
    // squarings when R is a power of two): each level's powers on a thread of its own, started
    // as soon as its base exists (C2: 4.7 -> ~2.7 ms of host time for a new generator length)
    std::vector<std::vector<std::vector<uint64_t>>> lv(static_cast<size_t>(levels));
    auto powers = [kind](const std::vector<uint64_t> &b, std::vector<std::vector<uint64_t>> &pw) {
      pw.assign(static_cast<size_t>(kind) + 1, {});
      pw[1] = b;
      auto step = [&pw](int m) {
        if (m % 2 == 0) {
          pw[static_cast<size_t>(m)] = pw[static_cast<size_t>(m / 2)];
          rs::mt_poly_square(pw[static_cast<size_t>(m)]);
        } else {
          rs::mt_poly_mulmod(pw[static_cast<size_t>(m - 1)], pw[1], pw[static_cast<size_t>(m)]);
        }
      };
      if (kind != 8) {
        for (int m = 2; m < kind; ++m) step(m);
        return;
      }
      // radix 8: after b^2, the chains b^4, b^5 and b^3, b^6, b^7 are independent (the second
      // on a helper thread: 1.6 -> 1.0 ms per level)
      step(2);
      std::thread t;
      try {
        t = std::thread([&step] { step(3); step(6); step(7); });
      } catch (...) {
        step(3);
        step(6);
        step(7);
      }
      step(4);
      step(5);
      if (t.joinable()) t.join();
    };
    const bool pow2 = (kind & (kind - 1)) == 0;
    std::vector<std::thread> th;
    for (int k = 0; k < levels; ++k) {
      bool spawned = false;
      if (k + 1 < levels && pow2) {
        try {
          th.emplace_back(powers, p, std::ref(lv[static_cast<size_t>(k)]));
          spawned = true;
        } catch (...) {  // no thread: this level here
        }
      }
      if (spawned) {
        for (int r = kind; r > 1; r >>= 1) rs::mt_poly_square(p);  // the next level's base
      } else {
        powers(p, lv[static_cast<size_t>(k)]);
        if (k + 1 < levels) {  // the next level's base b^R = b^(R-1) b
          std::vector<uint64_t> q;
          rs::mt_poly_mulmod(lv[static_cast<size_t>(k)][static_cast<size_t>(kind - 1)], p, q);
          p = q;
        }
      }
    }
    for (auto &t : th) t.join();
    for (int k = 0; k < levels; ++k)
      for (int m = 1; m < kind; ++m) jb->add(lv[static_cast<size_t>(k)][static_cast<size_t>(m)]);
  }
  if (cache.size() >= kJumpCache) cache.erase(cache.begin());
  cache.emplace_back(key, jb);
  out = *jb;
  g_jump_host_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  ++g_jump_builds;
}

// Radix-R tree levels (RSAMD_JRADIX, R <= 8): level k sends window g < R^k to g + m R^k
#ifndef RSAMD_JRADIX
#define RSAMD_JRADIX 8
#endif
constexpr int kJumpRadix = RSAMD_JRADIX;
static_assert(kJumpRadix >= 2 && kJumpRadix <= 8, "jump radix");

uint32_t untemper(uint32_t z) {
  uint32_t y = z ^ (z >> 18);
  y ^= (y << 15) & 0xefc60000u;
  uint32_t x = y;
  for (int r = 0; r < 5; ++r) x = y ^ ((x << 7) & 0x9d2c5680u);
  uint32_t u = x;
  for (int r = 0; r < 3; ++r) u = x ^ (u >> 11);
  return u;
}

// expected draws per hypothesis: sum over i of (mask(i) + 1) / (i + 1)
double expected_draws(int64_t n1, bool py) {
  double e = 0.0;
  for (int64_t i = 1; i <= n1; ++i) {
    uint64_t m = static_cast<uint64_t>(py ? i + 1 : i);  // CPython: 2^bit_length(i + 1) - 1
    m |= m >> 1;
    m |= m >> 2;
    m |= m >> 4;
    m |= m >> 8;
    m |= m >> 16;
    e += static_cast<double>(m + 1) / static_cast<double>(i + 1);
  }
  return e;
}

}  // namespace

// ==== sharded parse: the chunks of one stream split across ranks ==========
//
// Every rank runs the same deterministic layout: the segment's draws are C = world x Cr chunks
// of Wc draws, rank r owns chunks [r Cr, (r+1) Cr).  A rank
//   1. jumps its first MT19937 window to the generator holding its first word (the set bits of
//      g0 as level jumps, then the doubling tree over its own generators only), writes its
//      own words plus a margin (the hypothesis that straddles its end) and parses its chunks
//      from every entry state (k_np_entry / k_np_track, exactly as np_choice_device);
//   2. ships its chunk maps (the <= 64-entry lists entry -> exit, a blob of a few KB);
//   3. composes ALL chunks' maps (every rank, identically) into the true entry state of each
//      chunk and keeps its own chunks' wraps: its hypothesis starts, counted;
//   4. given the global offset of its first start (an all-gathered count scan) and the next
//      rank's first start, re-parses its own hypotheses into tuples; the rank holding the
//      start of hypothesis `got` reads the (key, pos) after the segment off its stream.
// Steps 2 -> 3 and 3 -> 4 are the all-gathers (Python, tsbb15_amd.parallel); nothing here
// depends on the transport.  World 1 gives the np_choice_device result, bit for bit.
namespace {

// own words per rank and segment (32 GiB, allocated by need).  C5 (N = 10 000, 1e6 hypotheses,
// 1.44e10 draws), measured per run: 2^31-word segments of 2^21-draw chunks 918 ms, 2^22 675,
// 2^23 612; 2^33-word segments of 2^23-draw chunks 442, of 2^24 368 (fewer chunks: the dense
// all-entry phase costs ~N per chunk; fewer segments: fewer rounds that drain)
constexpr int64_t kShardSegWords = int64_t(1) << 33;

// test / tuning knobs, read once per process: RSAMD_NP_SEGWORDS caps a rank's words per
// segment (tests of the multi-segment path), RSAMD_NP_KW fixes the chunk length (kWmin ..
// kWmax draws), RSAMD_NP_CPR the chunks per rank
int64_t env_i64(const char *name) {
  const char *e = std::getenv(name);
  return e ? std::atoll(e) : 0;
}
int64_t seg_words() {
  static const int64_t v = [] {
    const int64_t x = env_i64("RSAMD_NP_SEGWORDS");
    return x > 0 ? std::max<int64_t>(int64_t(1) << 16, std::min(x, int64_t(1) << 34)) : kShardSegWords;
  }();
  return v;
}
int knob_kw() {
  static const int v = [] {
    const int64_t x = env_i64("RSAMD_NP_KW");
    return x >= kWmin && x <= kWmax ? static_cast<int>(x) : 0;
  }();
  return v;
}
int64_t knob_cpr() {
  static const int64_t v = std::max<int64_t>(0, env_i64("RSAMD_NP_CPR"));
  return v;
}
// chunk-aligned generators and the two-pass stream (RSAMD_NP_SPLIT=0: off), read at every call
bool split_knob() {
  const char *e = std::getenv("RSAMD_NP_SPLIT");
  return !e || std::atoi(e) != 0;
}
constexpr int64_t kMapsMagic = 0x5253485044414d53LL;   // blob header tag

// start draw (relative to the rank's draw 0) of every kept wrap, in order; lead = 1 puts the
// segment's first hypothesis (draw 0, rank 0 only) in front
__global__ __launch_bounds__(256) void k_np_starts_local(const uint2 *__restrict__ ev,
                                                         const int *__restrict__ vcnt,
                                                         const int *__restrict__ off,
                                                         int64_t *__restrict__ starts, int ecap,
                                                         int W, int lead, int64_t scap, int *err) {
  const int c = blockIdx.x;
  const int n = vcnt[c];
  const int64_t base = lead + off[c];
  if (base + n > scap) {  // more starts than a hypothesis per n1 draws allows: a corrupt log
    if (threadIdx.x == 0) atomicOr(err, 8);
    return;
  }
  for (int i = threadIdx.x; i < n; i += 256)
    starts[base + i] = static_cast<int64_t>(c) * W + ev[static_cast<size_t>(c) * ecap + i].x;
  if (lead && c == 0 && threadIdx.x == 0) starts[0] = 0;
}

template <class T>
int sgrow(T *&p, int64_t &cap, int64_t need) {
  if (need <= cap) return RS_OK;
  if (p) (void)hipFree(p);
  p = nullptr;
  cap = 0;
  if (hipMalloc(reinterpret_cast<void **>(&p), sizeof(T) * static_cast<size_t>(need)) != hipSuccess)
    return rs::fail(RS_ENOMEM, "np shard: device allocation failed");
  cap = need;
  return RS_OK;
}

}  // namespace

// rs_np_timing marks: 0 start, 1 windows (jump) done, 2 first stream pass done, 3 entry done
// (with its resume launch, which waits for the second pass), 4 track done, 5 compose done,
// 6 starts done, 7 tuples done, 8 result copied.  Slots kNpMarks, kNpMarks + 1: the second
// stream pass on s2.
constexpr int kNpMarks = 9;

struct rs_np_shard {
  rs_ctx *ctx = nullptr;
  int world = 1, rank = 0, n1 = 0, cus = 256;
  int32_t k = 8;
  int64_t n = 0;
  bool py = false;
  // layout of the current segment (shard_layout)
  int64_t count = 0, Wc = 0, Cr = 0, C = 0, D = 0;
  int64_t s_lo = 0, g0 = 0, wbase = 0, Lb = 0, G = 0, nwords = 0;
  // generators of JB stream blocks (kJB, or the chunk length for chunk-aligned layouts, whose
  // last generator runs on to the segment's end: gext); xb > 0: the stream in two passes (blocks
  // 1..xb of every generator first), the entry kernel reading the first xlim draws of a chunk
  int JB = kJB, gext = 0, xb = 0, xlim = 0, bits_JB = 0;
  int ecap = 0, ecap_shift = 0;
  int state = 0;  // 0 idle, 1 parsed, 2 composed
  int64_t nstarts = 0, first_start = -1;
  std::vector<uint8_t> maps;  // this rank's chunk-map blob
  // device
  int32_t *d_bits = nullptr;
  std::vector<int> bit_off, bit_n, bit_ne;
  int32_t *d_rbits = nullptr;  // radix-tree level polynomials (jump_bits_cached)
  std::vector<int> rbit_off, rbit_n, rbit_ne;
  int rbits_JB = 0, rlevels = 0;
  uint32_t *d_win = nullptr, *d_chain = nullptr, *d_stream = nullptr, *d_fin = nullptr,
           *d_fin_all = nullptr;
  int *d_fin_m = nullptr, *d_fin_m_all = nullptr, *d_ev_n = nullptr, *d_ent = nullptr,
      *d_vcnt = nullptr, *d_off = nullptr, *d_err = nullptr, *d_tpos = nullptr, *d_pause = nullptr;
  uint32_t *d_io = nullptr;  // raw block of every generator between the two stream passes
  hipStream_t s2 = nullptr;  // the second stream pass
  hipEvent_t ev_a = nullptr, ev_b = nullptr;
  int64_t *d_row_off = nullptr, *d_starts = nullptr, *d_got = nullptr;
  uint2 *d_ev = nullptr;
  NpResult *d_res = nullptr;  // world 1 (np_choice_device): the segment's outcome in one copy
  // rs_np_timing: HIP events between the steps of a world-1 segment (kNpMarks on the context
  // stream, two around the second stream pass on s2); null unless timing was ever enabled
  bool timed = false;
  hipEvent_t tev[kNpMarks + 2] = {};
  // world 1: the segment's outcome copied to pinned memory behind ev_res, so the caller can
  // queue the evaluation before waiting for it (np_choice_enqueue / np_choice_finish)
  NpResult *h_res = nullptr;
  hipEvent_t ev_res = nullptr;
  int64_t pending = 0;  // hypotheses of an enqueued, not yet finished segment
  int64_t cap_win = 0, cap_chain = 0, cap_stream = 0, cap_fin = 0, cap_fin_all = 0, cap_fm = 0,
          cap_fm_all = 0, cap_ev = 0, cap_evn = 0, cap_ent = 0, cap_vcnt = 0, cap_off = 0,
          cap_tpos = 0, cap_row = 0, cap_starts = 0, cap_pause = 0, cap_io = 0;
};

namespace {

void shard_free(rs_np_shard *w) {
  void *ptrs[] = {w->d_bits, w->d_rbits, w->d_win,   w->d_chain, w->d_stream, w->d_fin,     w->d_fin_all,
                  w->d_fin_m, w->d_fin_m_all, w->d_ev_n, w->d_ent, w->d_vcnt, w->d_off,
                  w->d_err,  w->d_tpos,  w->d_row_off, w->d_starts, w->d_got, w->d_ev,
                  w->d_res};
  for (void *p : ptrs)
    if (p) (void)hipFree(p);
  if (w->d_pause) (void)hipFree(w->d_pause);
  if (w->d_io) (void)hipFree(w->d_io);
  if (w->ev_a) (void)hipEventDestroy(w->ev_a);
  if (w->ev_b) (void)hipEventDestroy(w->ev_b);
  for (hipEvent_t e : w->tev)
    if (e) (void)hipEventDestroy(e);
  if (w->ev_res) (void)hipEventDestroy(w->ev_res);
  if (w->h_res) (void)hipHostFree(w->h_res);
  // (w->s2 is the context's aux_stream: rs_ctx_destroy destroys it)
}

// kernel attributes for populations up to n1 (dynamic LDS of the entry and tuple kernels)
int shard_kernel_attrs(int n1) {
  static std::mutex mu;
  static int64_t entry_lds = 0, tup_lds = 0;
  static bool jump = false;
  std::lock_guard<std::mutex> g(mu);
  if (!jump) {
    HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void *>(k_mt_jump),
                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                static_cast<int>(sizeof(uint32_t) * kPrefixAlloc)));
    jump = true;
  }
  const int64_t lds = 4 * static_cast<int64_t>((n1 + 1) & ~1);  // k_np_entry: st, lo (uint16)
  if (lds > entry_lds) {
    HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void *>(k_np_entry<false>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds)));
    HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void *>(k_np_entry<true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds)));
    entry_lds = lds;
  }
  const int64_t tl = tup_lds_bytes(n1);
  if (tl > tup_lds) {
    HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void *>(k_np_tuples_wave<false>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(tl)));
    HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void *>(k_np_tuples_wave<true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(tl)));
    tup_lds = tl;
  }
  return RS_OK;
}

int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// a timing mark of rs_np_timing (no-op unless the segment is timed)
int tmark(rs_np_shard &w, int slot, hipStream_t s) {
  if (w.timed) HIP_TRY(hipEventRecord(w.tev[slot], s));
  return RS_OK;
}

}  // namespace

// Loads this file's code object on the current device (HIP loads a module at the first use of
// any of its kernels: ~10 ms for the parse kernels, paid by the first parity call otherwise).
int rs::np_preload() {
  hipFuncAttributes fa{};
  HIP_TRY(hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(k_np_track<false, false>)));
  return RS_OK;
}

namespace {

// The segment's layout for `count` more hypotheses from (., pos): identical on every rank with
// the same (n, count, pos, world, CUs); the compose step checks that it is.
int shard_layout(rs_np_shard &w, int32_t pos, int64_t count) {
  const double E = expected_draws(w.n1, w.py);
  const int64_t margin = 16 * w.n + 4096 + 8 * static_cast<int64_t>(std::ceil(E)) + kN;
  const int64_t own_cap = std::max<int64_t>(seg_words() - margin, 1 << 16);
  const int64_t hcap = std::max<int64_t>(
      1, static_cast<int64_t>(static_cast<double>(own_cap * w.world - 16 * w.n - 4096) / (E * 1.03)));
  const int64_t hs = std::min<int64_t>(count, hcap);
  const int64_t need = static_cast<int64_t>(std::ceil(hs * E * 1.03)) + 16 * w.n + 4096;
  const int64_t Dr = cdiv(need, w.world);
  // chunk length: every chunk in one resident round of k_np_track (16-wave workgroups, two
  // per CU) with equal lengths -- 2 x CUs chunks per rank for N - 1 < 4096; for larger N the
  // dense entry phase (cost ~ N per chunk) favours 1 x CUs.  Measured (C2, 1e5 tuples, one
  // GPU): 274 chunks of 2^20 9.9 ms, 508 of 565 248 8.3 ms, 765 of 376 832 9.9 ms.
  // A rank's share of a sharded segment is short: chunks below ~64 N draws spend most of
  // their time in the dense all-entry phase (~N draws per surviving trajectory), so the count
  // drops before the length does (C2 over 8 ranks, per-rank parse: 512 chunks of 73 728
  // draws 3.1 ms, 256 of 141 312 2.7 ms, 128 2.9 ms, 64 4.0 ms).
  // (N - 1 >= 4096 too: the entry kernel's 8 (N - 1) bytes of LDS still fit two workgroups per
  // CU at N = 10 000, so 2 x CUs chunks parse in one round, and the tracking kernel's serial
  // chains are shorter -- C5 per 1e6 hypotheses: 1 x CUs (chunks capped at 2^24 draws: 435 per
  // segment) 237.7 ms, 2 x CUs 226.9 ms, 3 x CUs 265.7 ms (entry in two rounds), gpurun_out r06g)
  const int64_t Cdef = static_cast<int64_t>(w.cus) * 2;
  const int64_t C0 = knob_cpr() ? knob_cpr()
                                : std::max<int64_t>(1, std::min<int64_t>(
                                                           Cdef, Dr / std::max<int64_t>(kWmin, 64 * w.n1)));
  // Chunk-aligned generators (N - 1 < 4096, chunks of at most two default generators): every
  // chunk starts a generator (J = the chunk length, a whole number of blocks), so the chunks'
  // first draws are generated in a short first pass and the rest on a second stream while the
  // entry kernel parses them (the stream's 0.33 ms beside the entry kernel at C2)
  const int64_t Lraw = cdiv(Dr, C0);
  const bool aligned = !knob_kw() && split_knob() && w.n1 < 4096 && Lraw >= kWmin &&
                       cdiv(Lraw, kN) <= 2 * kJB;
  const int64_t L = aligned ? cdiv(Lraw, kN) * kN : cdiv(Lraw, 4096) * 4096;
  w.Wc = knob_kw() ? knob_kw() : std::max<int64_t>(kWmin, std::min<int64_t>(kW, L));
  w.Cr = cdiv(Dr, w.Wc);
  w.C = w.Cr * w.world;
  w.D = w.C * w.Wc;
  w.count = hs;
  const int64_t own0 = static_cast<int64_t>(w.rank) * w.Cr * w.Wc;  // own draw 0
  w.s_lo = pos + own0;
  const int64_t s_end = w.s_lo + w.Cr * w.Wc + margin;
  // the first generator: every word the rank reads lies in a block it writes whole (a jumped
  // window's word 0 carries only its top bit)
  w.JB = aligned ? static_cast<int>(w.Wc / kN) : kJB;
  const int64_t J = static_cast<int64_t>(kN) * w.JB;
  w.g0 = w.rank == 0 ? 0 : (w.s_lo - kN) / J;
  if (w.g0 >> kLevels) return rs::fail(RS_EINVAL, "np shard: stream offset beyond the jump table");
  w.wbase = w.g0 * J;
  w.Lb = cdiv(s_end, kN) - w.g0 * w.JB;
  w.gext = aligned ? 1 : 0;
  w.G = aligned ? std::max<int64_t>(1, w.Lb / w.JB) : cdiv(w.Lb, w.JB);
  if (w.G > (int64_t(1) << kLevels)) return rs::fail(RS_EINVAL, "np shard: segment too long");
  // the first pass: every generator's blocks 1..xb, so that each chunk's first xlim draws
  // (offset oq into its generator) exist; a chunk whose dense phase goes further pauses
  const int64_t oq = (w.s_lo - w.wbase) % J;
  w.xb = 0;
  w.xlim = std::numeric_limits<int>::max();
  if (aligned && oq >= 1) {
    // (the dense phase ends within 23 360 draws at C2; RSAMD_NP_XDRAWS overrides: tests of the
    // pause / resume path.  The first pass runs alone, the second beside the entry kernel, which
    // waits for it before its resume launch: since the entry kernel got faster, a first pass of
    // 72 (N - 1) + 8 192 draws balances the two -- C2 parse 4.97-5.00 ms with 16 (N - 1) + 8 192,
    // 4.94 with 120k and 160k draws, profiles/r04_np_ab3)
    const int64_t xd = env_i64("RSAMD_NP_XDRAWS");
    const int64_t want = xd > 0 ? xd : 72 * static_cast<int64_t>(w.n1) + 8192;
    const int64_t xb = cdiv(want + oq, kN);
    if (xb < w.JB) {
      w.xb = static_cast<int>(xb);
      w.xlim = static_cast<int>((xb + 1) * kN - oq);
    }
  }
  w.nwords = w.Lb * kN - (w.s_lo - w.wbase);
  w.ecap_shift = 0;
  // host-side bounds of what the kernels index: every chunk's draws (and the straddling
  // hypothesis's margin) inside the generated words, the first pass inside a generator
  if (w.Cr * w.Wc + margin > w.nwords || w.Wc > std::numeric_limits<int>::max() / 2 ||
      (w.xb > 0 && w.xb >= w.JB))
    return rs::fail(RS_EINVAL, "np shard: segment layout exceeds the generated stream");
  return RS_OK;
}

// the ring form of the jump (k_mt_jump_slide) unless RSAMD_JUMP_PREFIX is set (A/B: the
// prefix form, one workgroup per CU)
#ifndef RSAMD_JUMP_SLIDE_WG
#define RSAMD_JUMP_SLIDE_WG 2  // ring-form jump parts per CU a level is sized for (A/B builds)
#endif
constexpr int kJumpSlideWg = RSAMD_JUMP_SLIDE_WG;
bool jump_slide() {
  static const bool v = std::getenv("RSAMD_JUMP_PREFIX") == nullptr;
  return v;
}
// (levels of fewer jumps than this keep the prefix form: one round either way, and the ring
// form's parts split by phases -- C2 level 1, 7 jumps: 16 us prefix, 22 us ring)
constexpr int kJumpSlideMin = 32;
void launch_jump(bool ring, unsigned grid, uint32_t *win, int half, int G, const int32_t *bits,
                 const JumpSet &js, int S, hipStream_t s) {
  if (ring)
    k_mt_jump_slide<<<grid, kJumpThreads, 0, s>>>(win, half, G, bits, js, S);
  else
    k_mt_jump<<<grid, kJumpThreads, sizeof(uint32_t) * kPrefixAlloc, s>>>(win, half, G, bits, js, S);
}

// windows of local generators 0 .. G-1 (global g0 ..) from the stream whose block 0 is key
int shard_windows(rs_np_shard &w, const uint32_t *key, hipStream_t s) {
  int st;
  if ((st = sgrow(w.d_win, w.cap_win, w.G * kN))) return st;
  // the radix-2 level polynomials of this generator length: only for a rank's first window
  // (g0 > 0: a chain of level jumps) or a radix-2 tree; world 1 (g0 = 0) never needs them
  if ((w.g0 != 0 || kJumpRadix == 2) && w.bits_JB != w.JB) {
    JumpBits jb;
    jump_bits_cached(0, w.JB, kLevels, jb);
    w.bit_off = jb.off;
    w.bit_n = jb.n;
    w.bit_ne = jb.ne;
    int64_t cap = 0;
    if (w.d_bits) (void)hipFree(w.d_bits);
    w.d_bits = nullptr;
    if ((st = sgrow(w.d_bits, cap, static_cast<int64_t>(jb.all.size())))) return st;
    HIP_TRY(hipMemcpy(w.d_bits, jb.all.data(), sizeof(int32_t) * jb.all.size(), hipMemcpyHostToDevice));
    w.bits_JB = w.JB;
  }
  if (w.g0 == 0) {
    HIP_TRY(hipMemcpyAsync(w.d_win, key, sizeof(uint32_t) * kN, hipMemcpyHostToDevice, s));
  } else {
    // a chain of level jumps, one per set bit of g0 (jumps commute)
    const int nb = __builtin_popcountll(static_cast<unsigned long long>(w.g0));
    if ((st = sgrow(w.d_chain, w.cap_chain, static_cast<int64_t>(nb + 1) * kN))) return st;
    HIP_TRY(hipMemcpyAsync(w.d_chain, key, sizeof(uint32_t) * kN, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemsetAsync(w.d_chain + kN, 0, sizeof(uint32_t) * kN * static_cast<size_t>(nb), s));
    int j = 0;
    for (int lv = 0; lv < kLevels; ++lv) {
      if (!((w.g0 >> lv) & 1)) continue;
      JumpSet js{};
      js.nm = 1;
      js.off[0] = w.bit_off[lv];
      js.nb[0] = w.bit_n[lv];
      js.ne[0] = w.bit_ne[lv];
      launch_jump(false, 64, w.d_chain + static_cast<size_t>(j) * kN, 1, 2, w.d_bits, js, 64, s);
      HIP_TRY(hipGetLastError());
      ++j;
    }
    HIP_TRY(hipMemcpyAsync(w.d_win, w.d_chain + static_cast<size_t>(j) * kN, sizeof(uint32_t) * kN,
                           hipMemcpyDeviceToDevice, s));
  }
  if (w.G > 1)
    HIP_TRY(hipMemsetAsync(w.d_win + kN, 0, sizeof(uint32_t) * kN * static_cast<size_t>(w.G - 1), s));
  // S parts per jump so that a level is one round of workgroups (one per CU: the prefix takes
  // 82 KB of LDS); two rounds cost a second prefix generation (C2 levels 3..8: 30 .. 168 us)
  if (kJumpRadix > 2) {
    // radix-R tree: level k sends window g < R^k to g + m R^k (m = 1 .. R-1) in one launch,
    // ceil(log_R G) levels instead of ceil(log2 G) (the small levels are latency, not work)
    int need = 0;
    for (int64_t B = 1; B < w.G; B *= kJumpRadix) ++need;
    if (w.rbits_JB != w.JB || w.rlevels < need) {
      JumpBits jr;
      jump_bits_cached(kJumpRadix, w.JB, need, jr);
      w.rbit_off = jr.off;
      w.rbit_n = jr.n;
      w.rbit_ne = jr.ne;
      int64_t cap = 0;
      if (w.d_rbits) (void)hipFree(w.d_rbits);
      w.d_rbits = nullptr;
      if ((st = sgrow(w.d_rbits, cap, static_cast<int64_t>(jr.all.size())))) return st;
      HIP_TRY(hipMemcpy(w.d_rbits, jr.all.data(), sizeof(int32_t) * jr.all.size(), hipMemcpyHostToDevice));
      w.rbits_JB = w.JB;
      w.rlevels = need;
    }
    int lv = 0;
    for (int64_t B = 1; B < w.G; B *= kJumpRadix, ++lv) {
      JumpSet js{};
      js.nm = kJumpRadix - 1;
      int64_t jumps = 0;
      for (int m = 1; m < kJumpRadix; ++m) {
        const size_t x = static_cast<size_t>(lv) * (kJumpRadix - 1) + (m - 1);
        js.off[m - 1] = w.rbit_off[x];
        js.nb[m - 1] = w.rbit_n[x];
        js.ne[m - 1] = w.rbit_ne[x];
        jumps += std::max<int64_t>(0, std::min<int64_t>(B, w.G - m * B));
      }
      const bool ring = jump_slide() && jumps >= kJumpSlideMin;
      const int64_t slots = static_cast<int64_t>(w.cus) * (ring ? kJumpSlideWg : 1);  // workgroups per round
      const int S = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(64, slots / std::max<int64_t>(1, jumps))));
      launch_jump(ring, static_cast<unsigned>(js.nm * B * S), w.d_win, static_cast<int>(B),
                  static_cast<int>(w.G), w.d_rbits, js, S, s);
      HIP_TRY(hipGetLastError());
    }
    return RS_OK;
  }
  for (int half = 1, lv = 0; half < w.G; half *= 2, ++lv) {
    const int jumps = static_cast<int>(std::min<int64_t>(half, w.G - half));
    const bool ring = jump_slide() && jumps >= kJumpSlideMin;
    const int S = std::max(1, std::min(64, w.cus * (ring ? kJumpSlideWg : 1) / jumps));
    JumpSet js{};
    js.nm = 1;
    js.off[0] = w.bit_off[lv];
    js.nb[0] = w.bit_n[lv];
    js.ne[0] = w.bit_ne[lv];
    launch_jump(ring, static_cast<unsigned>(half * S), w.d_win, half, static_cast<int>(w.G), w.d_bits,
                js, S, s);
    HIP_TRY(hipGetLastError());
  }
  return RS_OK;
}

// device set-up shared by both drivers: kernel attributes, the jump polynomials, counters
int shard_init(rs_np_shard &w) {
  HIP_TRY(hipSetDevice(w.ctx->device));
  int st;
  if ((st = shard_kernel_attrs(w.n1))) return st;
  if (!w.d_err) {
    int64_t c1 = 0, c2 = 0, c3 = 0;
    if ((st = sgrow(w.d_err, c1, 1)) || (st = sgrow(w.d_got, c2, 1)) || (st = sgrow(w.d_res, c3, 1)))
      return st;
    w.s2 = w.ctx->aux_stream;  // the context's own (rs_ctx_create)
    HIP_TRY(hipEventCreateWithFlags(&w.ev_a, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&w.ev_b, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&w.ev_res, hipEventDisableTiming));
    HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&w.h_res), sizeof(NpResult)));
  }
  return RS_OK;
}

// 1: the rank's own words (+ margin) for the segment laid out by shard_layout
int shard_stream(rs_np_shard &w, const uint32_t *key) {
  hipStream_t s = w.ctx->stream;
  int st;
  if ((st = sgrow(w.d_stream, w.cap_stream, w.Lb * kN))) return st;
  if ((st = shard_windows(w, key, s)) || (st = tmark(w, 1, s))) return st;
  const int G = static_cast<int>(w.G), JB = w.JB;
  if (w.xb > 0) {  // blocks 1..xb here, the rest on s2 beside the entry kernel (event ev_b)
    if ((st = sgrow(w.d_io, w.cap_io, w.G * kN))) return st;
    k_mt_stream<<<static_cast<unsigned>(G), 256, 0, s>>>(w.d_win, w.d_stream, w.Lb, JB, G, w.gext, 0,
                                                         w.xb, w.d_io);
    HIP_TRY(hipGetLastError());
    if ((st = tmark(w, 2, s))) return st;
    HIP_TRY(hipEventRecord(w.ev_a, s));
    HIP_TRY(hipStreamWaitEvent(w.s2, w.ev_a, 0));
    if ((st = tmark(w, kNpMarks, w.s2))) return st;
    k_mt_stream<<<static_cast<unsigned>(G), 256, 0, w.s2>>>(w.d_win, w.d_stream, w.Lb, JB, G, w.gext,
                                                            w.xb, std::numeric_limits<int>::max(), w.d_io);
    HIP_TRY(hipGetLastError());
    if ((st = tmark(w, kNpMarks + 1, w.s2))) return st;
    HIP_TRY(hipEventRecord(w.ev_b, w.s2));
  } else {
    k_mt_stream<<<static_cast<unsigned>(G), 256, 0, s>>>(w.d_win, w.d_stream, w.Lb, JB, G, w.gext, 0,
                                                         std::numeric_limits<int>::max(), nullptr);
    HIP_TRY(hipGetLastError());
    if ((st = tmark(w, 2, s)) || (st = tmark(w, kNpMarks, s)) || (st = tmark(w, kNpMarks + 1, s)))
      return st;
  }
  if ((st = sgrow(w.d_fin, w.cap_fin, w.Cr * w.n1)) || (st = sgrow(w.d_fin_m, w.cap_fm, w.Cr)) ||
      (st = sgrow(w.d_ev_n, w.cap_evn, w.Cr)) || (st = sgrow(w.d_tpos, w.cap_tpos, w.Cr)) ||
      (st = sgrow(w.d_vcnt, w.cap_vcnt, w.Cr)) || (st = sgrow(w.d_off, w.cap_off, w.Cr)) ||
      (st = sgrow(w.d_ent, w.cap_ent, w.Cr)) || (st = sgrow(w.d_pause, w.cap_pause, w.Cr)) ||
      // every hypothesis spans at least n1 draws: a bound on the own starts
      (st = sgrow(w.d_starts, w.cap_starts, w.Cr * w.Wc / std::max(1, w.n1) + 4)))
    return st;
  return RS_OK;
}

// 1: the all-entry parse of the rank's chunks, enqueued (wrap log of the current capacity)
int shard_enqueue_parse(rs_np_shard &w) {
  hipStream_t s = w.ctx->stream;
  int st;
  const double E = expected_draws(w.n1, w.py);
  w.ecap = static_cast<int>(std::min<int64_t>(
      w.Wc + 2 * w.n1, (static_cast<int64_t>(70.0 * w.Wc / E) + 4 * w.n1 + 4096) << w.ecap_shift));
  if ((st = sgrow(w.d_ev, w.cap_ev, w.Cr * w.ecap))) return st;
  HIP_TRY(hipMemsetAsync(w.d_err, 0, sizeof(int), s));
  const int Cr = static_cast<int>(w.Cr), Wc = static_cast<int>(w.Wc);
  const int64_t lds = 4 * static_cast<int64_t>((w.n1 + 1) & ~1);  // k_np_entry: st, lo (uint16)
  long long *d_stats = nullptr;
#ifdef RSAMD_DIAG
  // RSAMD_NP_STATS=<file>: per-chunk statistics of the entry kernel appended to <file>
  static int64_t cap_stats = 0;
  static long long *stats_buf = nullptr;
  if (std::getenv("RSAMD_NP_STATS")) {
    if ((st = sgrow(stats_buf, cap_stats, w.Cr * 128))) return st;
    HIP_TRY(hipMemsetAsync(stats_buf, 0, sizeof(long long) * w.Cr * 128, s));
    d_stats = stats_buf;
  }
#endif
  // RSAMD_NP_TSTAMP=<file>: the chunk timeline of this parse (g_np_ts), appended to <file>
  static const char *ts_path = std::getenv("RSAMD_NP_TSTAMP");
  static unsigned long long *ts_buf = nullptr;
  static int64_t ts_cap = 0;
  if (ts_path) {
    if ((st = sgrow(ts_buf, ts_cap, w.Cr * kTs))) return st;
    HIP_TRY(hipMemsetAsync(ts_buf, 0, sizeof(unsigned long long) * w.Cr * kTs, s));
    HIP_TRY(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_np_ts), &ts_buf, sizeof(ts_buf), 0,
                                   hipMemcpyHostToDevice, s));
  }
  EntryArgs ea{w.d_stream + (w.s_lo - w.wbase), w.Cr * w.Wc, Wc, w.n1, w.d_fin, w.d_fin_m,
               w.d_ev, w.d_ev_n, w.d_tpos, w.ecap, w.d_err, d_stats, w.xlim, 0, w.d_pause};
  const bool small = w.n1 < 64;  // several hypothesis ends in one tracking window
  // (split stream: the first launch reads the first pass's words; the second pass joins before
  // the resume launch, which carries on the chunks that paused)
  auto entry = [&](bool py) -> int {
    EntryArgs e2 = ea;
    (py ? k_np_entry<true> : k_np_entry<false>)<<<Cr, kEntryThreads, static_cast<size_t>(lds), s>>>(e2, e2.draws);
    HIP_TRY(hipGetLastError());
    if (w.xb > 0) {
      HIP_TRY(hipStreamWaitEvent(s, w.ev_b, 0));
      e2.resume = 1;
      e2.xlim = std::numeric_limits<int>::max();
      (py ? k_np_entry<true> : k_np_entry<false>)<<<Cr, kEntryThreads, static_cast<size_t>(lds), s>>>(e2, e2.draws);
      HIP_TRY(hipGetLastError());
    }
    return RS_OK;
  };
  if ((st = entry(w.py)) || (st = tmark(w, 3, s))) return st;
  if (w.py) {
    (small ? k_np_track<true, true>
           : (hand_of(w.n1) > 64 ? k_np_track128<true> : k_np_track<true, false>))<<<Cr, 64 * kTrackWaves, 0, s>>>(ea, ea.draws);
  } else {
    (small ? k_np_track<false, true>
           : (hand_of(w.n1) > 64 ? k_np_track128<false> : k_np_track<false, false>))<<<Cr, 64 * kTrackWaves, 0, s>>>(ea, ea.draws);
  }
  HIP_TRY(hipGetLastError());
  if ((st = tmark(w, 4, s))) return st;
  if (ts_path) {
    // header: n1, chunks, chunk length, draws, rank, world, then kTs words per chunk
    std::vector<unsigned long long> h(static_cast<size_t>(w.Cr) * kTs + 8, 0ull);
    const int64_t hd[8] = {w.n1, w.Cr, w.Wc, w.Cr * w.Wc, w.rank, w.world, kTs, 0};
    for (int k = 0; k < 8; ++k) h[k] = static_cast<unsigned long long>(hd[k]);
    HIP_TRY(hipMemcpyAsync(h.data() + 8, ts_buf, sizeof(unsigned long long) * w.Cr * kTs,
                           hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (FILE *f = std::fopen(ts_path, "ab")) {
      std::fwrite(h.data(), sizeof(unsigned long long), h.size(), f);
      std::fclose(f);
    }
  }
#ifdef RSAMD_DIAG
  if (d_stats) {
    std::vector<long long> hs(static_cast<size_t>(w.Cr) * 128 + 4);
    hs[0] = w.n1;
    hs[1] = w.Cr;
    hs[2] = w.Wc;
    hs[3] = w.Cr * w.Wc;
    HIP_TRY(hipMemcpyAsync(hs.data() + 4, d_stats, sizeof(long long) * w.Cr * 128, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (FILE *f = std::fopen(std::getenv("RSAMD_NP_STATS"), "ab")) {
      std::fwrite(hs.data(), sizeof(long long), hs.size(), f);
      std::fclose(f);
    }
  }
#endif
  return RS_OK;
}

// 3 (the true entry states in d_ent): the rank's wraps of the true trajectory, their count
// (scan into *got, at most cap) and start draws (d_starts, relative to the rank's draw 0)
int shard_enqueue_starts(rs_np_shard &w, int64_t cap, int64_t *got) {
  hipStream_t s = w.ctx->stream;
  const int Cr = static_cast<int>(w.Cr);
  k_np_filter<<<Cr, 64, 0, s>>>(w.d_ev, w.d_ev_n, w.d_ent + w.rank * w.Cr, w.d_vcnt, w.ecap);
  HIP_TRY(hipGetLastError());
  k_np_scan<<<1, 1024, 0, s>>>(w.d_vcnt, Cr, w.d_off, cap, got);
  HIP_TRY(hipGetLastError());
  k_np_starts_local<<<Cr, 256, 0, s>>>(w.d_ev, w.d_vcnt, w.d_off, w.d_starts, w.ecap,
                                       static_cast<int>(w.Wc), w.rank == 0 ? 1 : 0, w.cap_starts,
                                       w.d_err);
  HIP_TRY(hipGetLastError());
  return RS_OK;
}

// 4: the tuples of hypotheses [lo, hi) (rank-local start indices; waves at or beyond *got exit)
void shard_launch_tuples(rs_np_shard &w, int64_t lo, int64_t hi, const int64_t *got,
                         int32_t *d_out) {
  const int tw = tup_waves_for(w.n1);
  (w.py ? k_np_tuples_wave<true> : k_np_tuples_wave<false>)<<<static_cast<unsigned>(cdiv(hi - lo, tw)),
                                                               64 * tw,
                                                               static_cast<size_t>(tup_wave_bytes(w.n1) * tw),
                                                               w.ctx->stream>>>(
      w.d_stream + (w.s_lo - w.wbase), w.d_starts, got, lo, hi, w.n1, w.k, d_out, w.d_err,
      w.nwords);
}

int shard_parse(rs_np_shard &w, const uint32_t *key, int32_t pos, int64_t count) {
  hipStream_t s = w.ctx->stream;
  int st;
  if ((st = shard_init(w)) || (st = shard_layout(w, pos, count)) || (st = shard_stream(w, key)))
    return st;
  const int Cr = static_cast<int>(w.Cr);
  for (;;) {
    if ((st = shard_enqueue_parse(w))) return st;
    int err = 0;
    HIP_TRY(hipMemcpyAsync(&err, w.d_err, sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (err & 1) {  // wrap log overflow: a larger log, the same chunks again
      if (w.ecap >= w.Wc + 2 * w.n1) return rs::fail(RS_EDEVICE, "np shard: wrap log overflow");
      ++w.ecap_shift;
      continue;
    }
    if (err) return rs::fail(RS_EDEVICE, "np shard: parse error");
    break;
  }
  // 2: the chunk-map blob: header, fin_m[Cr], then each chunk's list
  std::vector<int> fm(static_cast<size_t>(Cr));
  HIP_TRY(hipMemcpy(fm.data(), w.d_fin_m, sizeof(int) * fm.size(), hipMemcpyDeviceToHost));
  const int width = std::min(w.n1, 64);
  std::vector<uint32_t> rows(static_cast<size_t>(Cr) * width);
  HIP_TRY(hipMemcpy2D(rows.data(), sizeof(uint32_t) * width, w.d_fin, sizeof(uint32_t) * w.n1,
                      sizeof(uint32_t) * width, static_cast<size_t>(Cr), hipMemcpyDeviceToHost));
  int64_t nent = 0;
  for (int q = 0; q < Cr; ++q) {
    if (fm[q] < 1 || fm[q] > w.n1) return rs::fail(RS_EDEVICE, "np shard: bad chunk map");
    nent += fm[q];
  }
  const int64_t hdr[8] = {kMapsMagic, w.rank, w.Cr, w.Wc, w.D, w.n1, nent, w.C};
  w.maps.assign(sizeof(hdr) + sizeof(int32_t) * Cr + sizeof(uint32_t) * nent, 0);
  uint8_t *o = w.maps.data();
  std::memcpy(o, hdr, sizeof(hdr));
  std::memcpy(o + sizeof(hdr), fm.data(), sizeof(int32_t) * Cr);
  uint32_t *e = reinterpret_cast<uint32_t *>(o + sizeof(hdr) + sizeof(int32_t) * Cr);
  for (int q = 0; q < Cr; ++q) {
    if (fm[q] <= width) {
      std::memcpy(e, rows.data() + static_cast<size_t>(q) * width, sizeof(uint32_t) * fm[q]);
    } else {  // the chunk ended dense: its whole list
      HIP_TRY(hipMemcpy(e, w.d_fin + static_cast<size_t>(q) * w.n1, sizeof(uint32_t) * fm[q],
                        hipMemcpyDeviceToHost));
    }
    e += fm[q];
  }
  w.state = 1;
  return RS_OK;
}

int shard_compose(rs_np_shard &w, const uint8_t *blobs, int64_t stride) {
  if (w.state < 1) return rs::fail(RS_EINVAL, "np shard: compose before parse");
  rs_ctx *c = w.ctx;
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = c->stream;
  int st;
  std::vector<int> fm_all(static_cast<size_t>(w.C));
  std::vector<int64_t> row(static_cast<size_t>(w.C));
  std::vector<uint32_t> ent;
  for (int r = 0; r < w.world; ++r) {
    const uint8_t *b = blobs + static_cast<size_t>(r) * stride;
    int64_t hdr[8];
    if (stride < static_cast<int64_t>(sizeof(hdr))) return rs::fail(RS_EINVAL, "np shard: short map blob");
    std::memcpy(hdr, b, sizeof(hdr));
    if (hdr[0] != kMapsMagic || hdr[1] != r)
      return rs::fail(RS_EINVAL, "np shard: map blobs must be the ranks' own, in rank order");
    if (hdr[2] != w.Cr || hdr[3] != w.Wc || hdr[4] != w.D || hdr[5] != w.n1 || hdr[7] != w.C)
      return rs::fail(RS_EINVAL, "np shard: ranks disagree on the segment layout");
    const int64_t nent = hdr[6];
    if (static_cast<int64_t>(sizeof(hdr) + sizeof(int32_t) * w.Cr + sizeof(uint32_t) * nent) > stride)
      return rs::fail(RS_EINVAL, "np shard: truncated map blob");
    const int32_t *fm = reinterpret_cast<const int32_t *>(b + sizeof(hdr));
    const uint32_t *e = reinterpret_cast<const uint32_t *>(b + sizeof(hdr) + sizeof(int32_t) * w.Cr);
    int64_t o = 0;
    for (int64_t q = 0; q < w.Cr; ++q) {
      const int m = fm[q];
      if (m < 1 || m > w.n1 || o + m > nent) return rs::fail(RS_EINVAL, "np shard: corrupt map blob");
      const int64_t cg = r * w.Cr + q;
      fm_all[static_cast<size_t>(cg)] = m;
      row[static_cast<size_t>(cg)] = static_cast<int64_t>(ent.size());
      ent.insert(ent.end(), e + o, e + o + m);
      o += m;
    }
  }
  if ((st = sgrow(w.d_fin_all, w.cap_fin_all, static_cast<int64_t>(ent.size()))) ||
      (st = sgrow(w.d_fin_m_all, w.cap_fm_all, w.C)) || (st = sgrow(w.d_row_off, w.cap_row, w.C)) ||
      (st = sgrow(w.d_ent, w.cap_ent, w.C)))
    return st;
  HIP_TRY(hipMemcpyAsync(w.d_fin_all, ent.data(), sizeof(uint32_t) * ent.size(), hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(w.d_fin_m_all, fm_all.data(), sizeof(int) * fm_all.size(), hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(w.d_row_off, row.data(), sizeof(int64_t) * row.size(), hipMemcpyHostToDevice, s));
  // 3: true entry state of every chunk, then this rank's wraps of the true trajectory
  k_np_compose<<<1, 1024, 0, s>>>(w.d_fin_all, w.d_fin_m_all, w.n1, static_cast<int>(w.C), w.d_ent,
                                  w.d_row_off);
  HIP_TRY(hipGetLastError());
  if ((st = shard_enqueue_starts(w, std::numeric_limits<int64_t>::max(), w.d_got))) return st;
  const int lead = w.rank == 0 ? 1 : 0;
  int64_t got = 0, first = -1;
  HIP_TRY(hipMemcpyAsync(&got, w.d_got, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  w.nstarts = got + lead;
  if (w.nstarts + 1 > w.cap_starts) return rs::fail(RS_EDEVICE, "np shard: start count out of range");
  if (w.nstarts > 0) {
    HIP_TRY(hipMemcpy(&first, w.d_starts, sizeof(int64_t), hipMemcpyDeviceToHost));
    first += static_cast<int64_t>(w.rank) * w.Cr * w.Wc;
  }
  w.first_start = first;
  w.state = 2;
  return RS_OK;
}

// 4: tuples of own hypotheses [base, hi) (global indices within the segment) into d_out;
// next_start: the following rank's first start (segment draw index), needed when hi reaches
// past the own starts; final_idx >= 0: the (key, pos) after hypothesis final_idx - 1.
int shard_tuples(rs_np_shard &w, int64_t base, int64_t hi, int64_t next_start, int64_t final_idx,
                 int32_t *d_out, uint32_t *key_out, int32_t *pos_out) {
  if (w.state < 2) return rs::fail(RS_EINVAL, "np shard: tuples before compose");
  const int64_t cnt = hi - base;
  if (base < 0 || cnt < 0 || cnt > w.nstarts) return rs::fail(RS_EINVAL, "np shard: hypothesis range out of range");
  if (cnt > 0 && !d_out) return rs::fail(RS_EINVAL, "np shard: null output");
  rs_ctx *c = w.ctx;
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = c->stream;
  const int64_t own0 = static_cast<int64_t>(w.rank) * w.Cr * w.Wc;
  if (cnt > 0) {
    if (cnt == w.nstarts) {  // the last own hypothesis ends at the next rank's first start
      if (next_start < 0) return rs::fail(RS_EINVAL, "np shard: the last hypothesis needs the next start");
      const int64_t nl = next_start - own0;
      if (nl <= 0 || nl > w.nwords)
        return rs::fail(RS_EDEVICE, "np shard: a hypothesis crosses beyond the rank's stream margin");
      HIP_TRY(hipMemcpy(w.d_starts + w.nstarts, &nl, sizeof(int64_t), hipMemcpyHostToDevice));
    }
    HIP_TRY(hipMemcpy(w.d_got, &cnt, sizeof(int64_t), hipMemcpyHostToDevice));
    HIP_TRY(hipMemsetAsync(w.d_err, 0, sizeof(int), s));
    shard_launch_tuples(w, 0, cnt, w.d_got, d_out);
    HIP_TRY(hipGetLastError());
    int err = 0;
    HIP_TRY(hipMemcpyAsync(&err, w.d_err, sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (err) return rs::fail(RS_EDEVICE, "np shard: hypothesis parse mismatch");
  }
  if (final_idx >= 0) {
    const int64_t j = final_idx - base;
    if (j < 0 || j >= w.nstarts) return rs::fail(RS_EINVAL, "np shard: final start not held by this rank");
    if (!key_out || !pos_out) return rs::fail(RS_EINVAL, "np shard: null state output");
    int64_t used = 0;
    HIP_TRY(hipMemcpy(&used, w.d_starts + j, sizeof(int64_t), hipMemcpyDeviceToHost));
    const int64_t W = w.s_lo + used;  // global word index of the next draw
    if (W > kN) {
      const int64_t b = (W - 1) / kN;
      const int64_t lb = b - w.g0 * w.JB;
      if (lb < (w.g0 ? 1 : 0) || lb >= w.Lb) return rs::fail(RS_EDEVICE, "np shard: final block outside the rank's stream");
      uint32_t blk[kN];
      HIP_TRY(hipMemcpy(blk, w.d_stream + lb * kN, sizeof(blk), hipMemcpyDeviceToHost));
      for (int i = 0; i < kN; ++i) key_out[i] = untemper(blk[i]);
      *pos_out = static_cast<int32_t>(W - b * kN);
    } else {
      *pos_out = static_cast<int32_t>(W);  // key unchanged (the caller's copy)
    }
  }
  return RS_OK;
}

// One world-1 segment after its stream: parse, compose, starts, tuples [lo, hi), the outcome
// (delivered count, draws used, errors, the stream block holding the next word) copied to the
// pinned w.h_res behind w.ev_res.  Nothing is waited for.
int shard_local_enqueue(rs_np_shard &w, int32_t pos, int64_t lo, int64_t hi, int32_t *d_out) {
  hipStream_t s = w.ctx->stream;
  int st;
  if ((st = shard_enqueue_parse(w))) return st;
  k_np_compose<<<1, 1024, 0, s>>>(w.d_fin, w.d_fin_m, w.n1, static_cast<int>(w.Cr), w.d_ent,
                                  nullptr);
  HIP_TRY(hipGetLastError());
  if ((st = tmark(w, 5, s))) return st;
  if ((st = shard_enqueue_starts(w, w.count, &w.d_res->got)) || (st = tmark(w, 6, s))) return st;
  if (hi > lo) {  // waves beyond the delivered count exit
    shard_launch_tuples(w, lo, hi, &w.d_res->got, d_out);
    HIP_TRY(hipGetLastError());
  }
  if ((st = tmark(w, 7, s))) return st;
  k_np_result<<<1, 64, 0, s>>>(w.d_stream, w.d_starts, pos, w.d_err, w.d_res);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(w.h_res, w.d_res, sizeof(NpResult), hipMemcpyDeviceToHost, s));
  if ((st = tmark(w, 8, s))) return st;
  HIP_TRY(hipEventRecord(w.ev_res, s));
  return RS_OK;
}

// Wait for the enqueued segment's outcome; its step times (rs_np_timing); *overflow: the wrap
// log overflowed (the same chunks must be parsed again with a larger log).
int shard_local_wait(rs_np_shard &w, bool *overflow) {
  HIP_TRY(hipEventSynchronize(w.ev_res));
  const NpResult &res = *w.h_res;
  if (w.timed) {  // this segment's steps, summed over the call's segments (rs_np_timing)
    float ms = 0.f;
    for (int k = 0; k + 1 < kNpMarks; ++k) {
      HIP_TRY(hipEventElapsedTime(&ms, w.tev[k], w.tev[k + 1]));
      w.ctx->np_ms[k] += ms;
    }
    HIP_TRY(hipEventElapsedTime(&ms, w.tev[kNpMarks], w.tev[kNpMarks + 1]));
    w.ctx->np_ms[kNpMarks - 1] += ms;
    HIP_TRY(hipEventElapsedTime(&ms, w.tev[0], w.tev[kNpMarks - 1]));
    w.ctx->np_ms[kNpMarks] += ms;
    // algorithmic HBM bytes of the segment: stream words written once, every parsed draw
    // read once by the chunk parse (entry + track), every hypothesis's draws read once by
    // the tuple kernel (words up to the last start)
    w.ctx->np_bytes[0] += 4.0 * static_cast<double>(w.Lb) * kN;
    w.ctx->np_bytes[1] += 4.0 * static_cast<double>(w.Cr * w.Wc);
    w.ctx->np_bytes[2] += 4.0 * static_cast<double>(res.used);
    w.ctx->np_segments += 1;
  }
  *overflow = (res.err & 1) != 0;
  if (*overflow && w.ecap >= w.Wc + 2 * w.n1) return rs::fail(RS_EDEVICE, "np sampler: wrap log overflow");
  return RS_OK;
}

// The finished segment's outcome: errors, delivered count, the advanced (key, pos).
int shard_local_outcome(rs_np_shard &w, uint32_t *key, int32_t *pos, int64_t *got_out) {
  const NpResult &res = *w.h_res;
  if (res.err & 2) return rs::fail(RS_EDEVICE, "np sampler: hypothesis parse mismatch");
  if (res.err) return rs::fail(RS_EDEVICE, "np sampler: corrupt chunk hand-over or start list");
  if (res.got < 1) return rs::fail(RS_EDEVICE, "np sampler: segment holds no complete hypothesis");
  // state after `used` draws: the block holding the last word drawn (rs_mt_jump's convention)
  const int64_t W = *pos + res.used;
  if (W > kN) {
    const int64_t b = (W - 1) / kN;
    for (int i = 0; i < kN; ++i) key[i] = untemper(res.blk[i]);
    *pos = static_cast<int32_t>(W - b * kN);
  } else {
    *pos = static_cast<int32_t>(W);
  }
  *got_out = res.got;
  return RS_OK;
}

// the segment's set-up through its stream (timing marks, layout, jump + stream launches)
int shard_local_begin(rs_np_shard &w, const uint32_t *key, int32_t pos, int64_t count) {
  int st;
  if ((st = shard_init(w))) return st;
  w.timed = w.ctx->np_timing != 0;
  if (w.timed && !w.tev[0])
    for (auto &e : w.tev) HIP_TRY(hipEventCreate(&e));
  if ((st = tmark(w, 0, w.ctx->stream)) || (st = shard_layout(w, pos, count)) ||
      (st = shard_stream(w, key)))
    return st;
  return RS_OK;
}

// World 1, all on the device (np_choice_device): one segment of at most `count` hypotheses
// from (key, pos) -- the same steps with the compose read straight from the device maps and
// one host synchronisation; its hypotheses [lo, hi) go to d_out as k-tuples; *got and
// (key, pos) advance.
int shard_run_local(rs_np_shard &w, uint32_t *key, int32_t *pos, int64_t count, int64_t lo,
                    int64_t hi, int32_t *d_out, int64_t *got_out) {
  int st;
  if ((st = shard_local_begin(w, key, *pos, count))) return st;
  for (;;) {
    bool overflow = false;
    if ((st = shard_local_enqueue(w, *pos, lo, hi, d_out)) || (st = shard_local_wait(w, &overflow)))
      return st;
    if (!overflow) break;
    ++w.ecap_shift;  // wrap log overflow: a larger log, the same chunks again
  }
  return shard_local_outcome(w, key, pos, got_out);
}

// The context's world-1 session for (n, k, py), created on first use.
int local_session(rs_ctx *c, int64_t n, int32_t k, bool py, rs_np_shard **out) {
  if (c->np_timing) {  // rs_np_timing reports this call's steps
    for (double &v : c->np_ms) v = 0.0;
    for (double &v : c->np_bytes) v = 0.0;
    c->np_segments = 0;
  }
  rs_np_shard *w = c->np_shard;
  if (w && (w->n != n || w->k != k || w->py != py)) {
    // another population (the drop-in's next pair): the session keeps its device buffers,
    // which only grow, and lays the next segment out for the new n (shard_layout)
    w->n = n;
    w->n1 = static_cast<int>(n - 1);
    w->k = k;
    w->py = py;
    w->state = 0;
  }
  if (!w) {
    int st;
    if ((st = rs_np_shard_create(c, n, k, 1, 0, py ? 1 : 0, &w))) return st;
    c->np_shard = w;
  }
  w->pending = 0;
  *out = w;
  return RS_OK;
}

}  // namespace

namespace rs {
int np_shard_tuples_device(rs_np_shard *w, int64_t base, int64_t hi, int64_t next_start,
                           int64_t final_idx, int32_t *d_out, uint32_t *key_out, int32_t *pos_out) {
  if (!w) return fail(RS_EINVAL, "null shard");
  return shard_tuples(*w, base, hi, next_start, final_idx, d_out, key_out, pos_out);
}

bool np_gpu_supported(int64_t n, int32_t k) { return k >= 1 && k <= 8 && k <= n && n - 1 <= kMaxN1; }

void np_shard_free(rs_ctx *c) {
  if (c->np_shard) {
    (void)rs_np_shard_destroy(c->np_shard);
    c->np_shard = nullptr;
  }
}

// The numpy (py: CPython) stream's next `count` choice(n, k) tuples, rows [skip, skip + take)
// into device memory, on the context stream; advances (key, pos).  Synchronous.  The
// context's world-1 session carries the buffers from call to call.
int np_choice_device(rs_ctx *c, uint32_t *key, int32_t *pos, int64_t n, int32_t k,
                     int64_t count, int32_t *d_out, bool py, int64_t skip, int64_t take) {
  if (take < 0) take = count - skip;
  if (skip < 0 || skip + take > count) return fail(RS_EINVAL, "np sampler: slice out of range");
  if (k < 1 || k > 8) return fail(RS_EINVAL, "np sampler: k must be in 1..8");
  if (k > n)
    return fail(RS_EINVAL, py ? "Cannot generate more indices than the amount of values in the set "
                                "from which they are extracted. n should therefore be smaller or "
                                "equal to set_length"
                              : "Cannot take a larger sample than population when 'replace=False'");
  if (n - 1 > kMaxN1) return fail(RS_EINVAL, "np sampler: population too large for the GPU parse");
  if (*pos < 0 || *pos > kN) return fail(RS_EINVAL, "bad MT19937 position");
  if (count == 0) return RS_OK;
  HIP_TRY(hipSetDevice(c->device));
  if (n <= 1) {  // a one-element shuffle draws nothing: every tuple is (0)
    HIP_TRY(hipMemsetAsync(d_out, 0, sizeof(int32_t) * static_cast<size_t>(take) * k, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return RS_OK;
  }
  rs_np_shard *w = nullptr;
  int st;
  if ((st = local_session(c, n, k, py, &w))) return st;
  int64_t done = 0;
  while (done < count) {
    // this segment's hypotheses [done, done + got) against the slice [skip, skip + take)
    const int64_t lo = std::max<int64_t>(skip - done, 0);
    const int64_t hi = std::max(lo, std::min<int64_t>(skip + take - done, count - done));
    int64_t got = 0;
    if ((st = shard_run_local(*w, key, pos, count - done, lo, hi,
                              hi > lo ? d_out + (done + lo - skip) * k : nullptr, &got)))
      return st;
    done += got;
  }
  return RS_OK;
}

// np_choice_device's one-segment case split in two, so that the caller can queue work that
// reads d_out before waiting: np_choice_enqueue queues all of one segment's steps when the
// whole `count` fits one segment (*queued; otherwise nothing is queued and the caller takes
// np_choice_device); np_choice_finish waits and advances (key, pos).  *rerun: the segment
// must be drawn again (a wrap-log overflow, or fewer hypotheses than asked) -- (key, pos)
// are unchanged and the caller repeats the call with np_choice_device, which handles both.
int np_choice_enqueue(rs_ctx *c, const uint32_t *key, int32_t pos, int64_t n, int32_t k,
                      int64_t count, int32_t *d_out, bool *queued) {
  *queued = false;
  if (!np_gpu_supported(n, k) || n <= 1 || count < 1 || pos < 0 || pos > kN) return RS_OK;
  HIP_TRY(hipSetDevice(c->device));
  rs_np_shard *w = nullptr;
  int st;
  if ((st = local_session(c, n, k, false, &w))) return st;
  if ((st = shard_init(*w))) return st;
  w->timed = c->np_timing != 0;
  if (w->timed && !w->tev[0])
    for (auto &e : w->tev) HIP_TRY(hipEventCreate(&e));
  if ((st = tmark(*w, 0, c->stream)) || (st = shard_layout(*w, pos, count))) return st;
  if (w->count < count) return RS_OK;  // more than one segment: nothing queued yet
  if ((st = shard_stream(*w, key)) || (st = shard_local_enqueue(*w, pos, 0, count, d_out)))
    return st;
  w->pending = count;
  *queued = true;
  return RS_OK;
}

int np_choice_finish(rs_ctx *c, uint32_t *key, int32_t *pos, bool *rerun) {
  *rerun = false;
  rs_np_shard *w = c->np_shard;
  if (!w || w->pending < 1) return fail(RS_EINVAL, "np sampler: no segment enqueued");
  const int64_t want = w->pending;
  w->pending = 0;
  bool overflow = false;
  int st;
  if ((st = shard_local_wait(*w, &overflow))) return st;
  if (overflow) {
    ++w->ecap_shift;  // the repeat gets the larger log
    *rerun = true;
    return RS_OK;
  }
  uint32_t k2[kN];
  int32_t p2 = *pos;
  std::memcpy(k2, key, sizeof(k2));
  int64_t got = 0;
  if ((st = shard_local_outcome(*w, k2, &p2, &got))) return st;
  if (got != want || std::getenv("RSAMD_NP_RERUN_TEST")) {  // the test hook takes this branch
    *rerun = true;
    return RS_OK;
  }
  std::memcpy(key, k2, sizeof(k2));
  *pos = p2;
  return RS_OK;
}
}  // namespace rs

namespace {
// Tuples of either stream into host memory through the context's scratch buffer.
int choice_tuples_gpu(rs_ctx *c, uint32_t *mt_key, int32_t *mt_pos, int64_t n, int32_t k,
                      int64_t count, int32_t *out, bool py) {
  if (!c || !mt_key || !mt_pos || (count > 0 && !out))
    return rs::fail(RS_EINVAL, "tuples_gpu: null pointer");
  if (count < 0 || k < 0) return rs::fail(RS_EINVAL, "negative dimensions are not allowed");
  if (count == 0) return RS_OK;
  int st;
  if ((st = rs::ensure_scratch(c, sizeof(int32_t) * static_cast<size_t>(count) * k))) return st;
  uint32_t key[kN];
  int32_t pos = *mt_pos;
  std::memcpy(key, mt_key, sizeof(key));
  if ((st = rs::np_choice_device(c, key, &pos, n, k, count, static_cast<int32_t *>(c->scratch),
                                 py)))
    return st;
  HIP_TRY(hipMemcpy(out, c->scratch, sizeof(int32_t) * static_cast<size_t>(count) * k,
                    hipMemcpyDeviceToHost));
  std::memcpy(mt_key, key, sizeof(key));
  *mt_pos = pos;
  return RS_OK;
}
}  // namespace

extern "C" int rs_np_choice_tuples_gpu(rs_ctx *c, uint32_t *mt_key, int32_t *mt_pos, int64_t n,
                                       int32_t k, int64_t count, int32_t *out) {
  return choice_tuples_gpu(c, mt_key, mt_pos, n, k, count, out, false);
}

extern "C" int rs_py_shuffle_tuples_gpu(rs_ctx *c, uint32_t *mt_key, int32_t *mt_pos, int64_t n,
                                        int32_t k, int64_t count, int32_t *out) {
  return choice_tuples_gpu(c, mt_key, mt_pos, n, k, count, out, true);
}

extern "C" int rs_np_shard_create(rs_ctx *c, int64_t n, int32_t k, int32_t world, int32_t rank,
                                  int32_t py, rs_np_shard **out) {
  if (!c || !out) return rs::fail(RS_EINVAL, "null pointer");
  *out = nullptr;
  if (world < 1 || rank < 0 || rank >= world) return rs::fail(RS_EINVAL, "np shard: bad rank / world");
  if (k < 1 || k > 8) return rs::fail(RS_EINVAL, "np sampler: k must be in 1..8");
  if (k > n)
    return rs::fail(RS_EINVAL, py ? "Cannot generate more indices than the amount of values in the set "
                                    "from which they are extracted. n should therefore be smaller or "
                                    "equal to set_length"
                                  : "Cannot take a larger sample than population when 'replace=False'");
  if (n < 2) return rs::fail(RS_EINVAL, "np shard: population must be at least 2");
  if (n - 1 > kMaxN1) return rs::fail(RS_EINVAL, "np sampler: population too large for the GPU parse");
  auto *w = new rs_np_shard();
  w->ctx = c;
  w->n = n;
  w->n1 = static_cast<int>(n - 1);
  w->k = k;
  w->world = world;
  w->rank = rank;
  w->py = py != 0;
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device) == hipSuccess && cus > 0)
    w->cus = cus;
  *out = w;
  return RS_OK;
}

extern "C" int rs_np_shard_destroy(rs_np_shard *w) {
  if (!w) return RS_OK;
  (void)hipSetDevice(w->ctx->device);
  (void)hipStreamSynchronize(w->ctx->stream);
  shard_free(w);
  delete w;
  return RS_OK;
}

extern "C" int rs_np_shard_parse(rs_np_shard *w, const uint32_t *mt_key, int32_t mt_pos,
                                 int64_t count, int64_t *layout) {
  if (!w || !mt_key) return rs::fail(RS_EINVAL, "null pointer");
  if (mt_pos < 0 || mt_pos > kN) return rs::fail(RS_EINVAL, "bad MT19937 position");
  if (count < 1) return rs::fail(RS_EINVAL, "np shard: count must be positive");
  w->state = 0;
  int st = shard_parse(*w, mt_key, mt_pos, count);
  if (st) return st;
  if (layout) {
    const int64_t v[6] = {w->count, w->C, w->Cr, w->Wc, w->D, static_cast<int64_t>(w->maps.size())};
    std::memcpy(layout, v, sizeof(v));
  }
  return RS_OK;
}

extern "C" int rs_np_shard_maps(rs_np_shard *w, uint8_t *out, int64_t cap, int64_t *nbytes) {
  if (!w || !nbytes) return rs::fail(RS_EINVAL, "null pointer");
  if (w->state < 1) return rs::fail(RS_EINVAL, "np shard: maps before parse");
  *nbytes = static_cast<int64_t>(w->maps.size());
  if (out) {
    if (cap < *nbytes) return rs::fail(RS_EINVAL, "np shard: map buffer too small");
    std::memcpy(out, w->maps.data(), w->maps.size());
  }
  return RS_OK;
}

extern "C" int rs_np_shard_compose(rs_np_shard *w, const uint8_t *blobs, int64_t stride,
                                   int64_t *nstarts, int64_t *first_start) {
  if (!w || !blobs || !nstarts || !first_start) return rs::fail(RS_EINVAL, "null pointer");
  const int st = shard_compose(*w, blobs, stride);
  if (st) return st;
  *nstarts = w->nstarts;
  *first_start = w->first_start;
  return RS_OK;
}

extern "C" int rs_np_shard_tuples(rs_np_shard *w, int64_t base, int64_t hi, int64_t next_start,
                                  int64_t final_idx, int32_t *out, uint32_t *key_out,
                                  int32_t *pos_out) {
  if (!w) return rs::fail(RS_EINVAL, "null shard");
  const int64_t cnt = hi - base;
  int32_t *d = nullptr;
  int st;
  if (cnt > 0) {
    if (!out) return rs::fail(RS_EINVAL, "null output");
    if ((st = rs::ensure_scratch(w->ctx, sizeof(int32_t) * static_cast<size_t>(cnt) * w->k))) return st;
    d = static_cast<int32_t *>(w->ctx->scratch);
  }
  if ((st = shard_tuples(*w, base, hi, next_start, final_idx, d, key_out, pos_out))) return st;
  if (cnt > 0)
    HIP_TRY(hipMemcpy(out, d, sizeof(int32_t) * static_cast<size_t>(cnt) * w->k, hipMemcpyDeviceToHost));
  return RS_OK;
}

// Host time the parse has spent building MT jump polynomials in this process (first calls at a
// new generator length), and how many level sets it built.
extern "C" int rs_np_timing(rs_ctx *c, int32_t enable, double *ms_out, double *bytes_out,
                            int64_t *segments) {
  if (!c) return rs::fail(RS_EINVAL, "null pointer");
  static_assert(kNpMarks + 1 == RS_NP_TIMING_SLOTS, "rs_np_timing slots");
  c->np_timing = enable ? 1 : 0;
  if (ms_out) std::memcpy(ms_out, c->np_ms, sizeof(c->np_ms));
  if (bytes_out) std::memcpy(bytes_out, c->np_bytes, sizeof(c->np_bytes));
  if (segments) *segments = c->np_segments;
  return RS_OK;
}

extern "C" int rs_np_host_stats(double *jump_ms, int64_t *builds) {
  if (!jump_ms || !builds) return rs::fail(RS_EINVAL, "rs_np_host_stats: null pointer");
  std::lock_guard<std::mutex> g(g_jump_mu);
  *jump_ms = g_jump_host_ms;
  *builds = g_jump_builds;
  return RS_OK;
}
