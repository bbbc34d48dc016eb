// Batched RANSAC-F over many image pairs in one pass (config C4: all pairs of the 36-view
// ring on a GPU).  The per-pair plan path (f8_plan.hip) is built for one large pair; C4 has
// hundreds of small ones (N <= 445, H = 1000), where one plan run per pair is launch- and
// sync-bound and fills a few percent of the chip.  Here every stage covers all pairs:
//
//   k_pairs_solve   lane per (pair, hypothesis): sample (Philox/Floyd keyed by seed_base +
//                   pair, counter h -- the same stream as a per-pair plan run with that seed --
//                   or host tuples), 8-point F (lab3.py:269-329), F stored SoA
//   k_pairs_count   wave per (pair, 64 hypotheses): lanes = hypotheses, the pair's points
//                   wave-uniform (scalar loads); reference-order float64 distance dist_ref
//                   (lab3.py:210-227, fun.py:316-317), so counts are the reference's exactly
//                   and no guard band / re-score pass is needed
//   k_pairs_select  workgroup per pair: c* = max count, the hypotheses with count == c* in
//                   index order, their np.std(d) / np.linalg.norm(d) (wave per candidate),
//                   the fun.py:320-328 replay, S_RANSAC of the winner
#include <hip/hip_runtime.h>

#include <cstring>
#include <initializer_list>
#include <vector>

#include "common.h"
#include "ctx.h"
#include "device_math.h"
#include "f8_kernels.h"

namespace rsd {

constexpr int kPairSelT = 512;          // select workgroup
constexpr int kPairSelW = kPairSelT / 64;

struct PairDevResult {  // == rs_pair_result
  double F[9];
  int64_t best_index;
  int64_t best_count;
  double best_std;
  double best_norm;
  int64_t n_candidates;
};

__global__ __launch_bounds__(256) void k_pairs_solve(const Pt *__restrict__ pts,
                                                     const int64_t *__restrict__ off, int B,
                                                     int H, int mode, uint64_t seed_base,
                                                     const int64_t *__restrict__ ids,
                                                     const int32_t *__restrict__ tuples,
                                                     double *__restrict__ Fsoa, int64_t ld) {
  const int64_t g = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (g >= ld) return;
  const int b = static_cast<int>(g / H), h = static_cast<int>(g - static_cast<int64_t>(b) * H);
  const int64_t o = off[b];
  const int n = static_cast<int>(off[b + 1] - o);
  double F[9];
  if (n < 8) {
#pragma unroll
    for (int k = 0; k < 9; ++k) F[k] = __builtin_nan("");
  } else {
    int idx[8];
    if (mode == RSD_SAMPLER_PHILOX) {
      const uint64_t sb = seed_base + static_cast<uint64_t>(ids ? ids[b] : b);
      floyd_sample<8>(sb, static_cast<uint64_t>(h), n, idx);
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) idx[k] = tuples[g * 8 + k];
    }
    double xl[8], yl[8], xr[8], yr[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const Pt p = pts[o + idx[k]];
      xl[k] = p.x1;
      yl[k] = p.y1;
      xr[k] = p.x2;
      yr[k] = p.y2;
    }
    fmatrix8(xl, yl, xr, yr, F);
  }
#pragma unroll
  for (int k = 0; k < 9; ++k) Fsoa[k * ld + g] = F[k];
}

// (and np.linalg.norm(d) of every hypothesis, for the selection's ties: the sum a wave per
// hypothesis forms -- 64 lane sums over the points i = l, l + 64, ..., combined by the xor
// butterfly (wsum) -- is the balanced pairwise sum of the lane sums in bit-reversed lane
// order.  A wave takes one of kCountChunks runs of those leaves, a complete subtree: its sum
// goes to nrmp[hypothesis][chunk] and k_pairs_select adds the chunks' subtrees in tree order
// (same bits).  Counts are added atomically (order-free).  Chunks: the largest pairs' point
// loops were the kernel's serial chains.)
constexpr int kCountChunks = 8;  // leaves per chunk: 64 / kCountChunks = 8 (a subtree)
__global__ __launch_bounds__(256) void k_pairs_count(const Pt *__restrict__ pts,
                                                     const int64_t *__restrict__ off, int B,
                                                     int H, const double *__restrict__ Fsoa,
                                                     int64_t ld, double thresh,
                                                     int *__restrict__ counts,
                                                     double *__restrict__ nrmp) {
  const int groups = (H + 63) >> 6;
  const int u = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  if (u >= B * groups * kCountChunks) return;
  const int ch = u % kCountChunks, ug = u / kCountChunks;
  const int b = ug / groups, grp = ug - b * groups;
  const int h = grp * 64 + (threadIdx.x & 63);
  const int64_t o = off[b];
  const int n = static_cast<int>(off[b + 1] - o);
  if (n < 8) return;  // no candidates: the counts stay 0
  const int64_t g = static_cast<int64_t>(b) * H + (h < H ? h : H - 1);
  double f[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) f[k] = Fsoa[k * ld + g];
  constexpr int kLeaves = 64 / kCountChunks, kLev = 3;  // log2(kLeaves)
  int cnt = 0;
  double acc[kLev], tot = 0.0;
  for (int q = 0; q < kLeaves; ++q) {
    const int k = ch * kLeaves + q;
    const int l = static_cast<int>(__builtin_bitreverse32(static_cast<uint32_t>(k)) >> 26);
    double s2 = 0.0;
    for (int i = l; i < n; i += 64) {
      const double d = dist_ref(f, pts[o + i]);
      cnt += d < thresh ? 1 : 0;
      s2 += d * d;
    }
    double carry = s2;  // leaf q closes the subtrees of its trailing one bits
    int lev = 0;
    for (; lev < kLev && ((q >> lev) & 1); ++lev) carry = acc[lev] + carry;
    if (lev < kLev) acc[lev] = carry;
    else tot = carry;
  }
  if (h < H) {
    if (cnt) atomicAdd(&counts[static_cast<int64_t>(b) * H + h], cnt);
    nrmp[(static_cast<int64_t>(b) * H + h) * kCountChunks + ch] = tot;
  }
}

__device__ __forceinline__ double wsum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__global__ __launch_bounds__(kPairSelT) void k_pairs_select(
    const Pt *__restrict__ pts, const int64_t *__restrict__ off, int H,
    const double *__restrict__ Fsoa, int64_t ld, const int *__restrict__ counts, double thresh,
    int *__restrict__ cand, const double *__restrict__ nrmp, double *__restrict__ cnorm,
    PairDevResult *__restrict__ res, int32_t *__restrict__ inl) {
  __shared__ int sh_i[kPairSelW];
  __shared__ int s_cstar, s_best;
  __shared__ int woff[kPairSelW];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t o = off[b];
  const int n = static_cast<int>(off[b + 1] - o);
  const int *cnt = counts + static_cast<int64_t>(b) * H;
  int *cb = cand + static_cast<int64_t>(b) * H;
  double *nb = cnorm + static_cast<int64_t>(b) * H;  // the candidates' norms, in list order
  // ---- c* ----
  int m = 0;
  for (int i = tid; i < H; i += kPairSelT) m = max(m, cnt[i]);
#pragma unroll
  for (int q = 32; q > 0; q >>= 1) m = max(m, __shfl_xor(m, q));
  if (lane == 0) sh_i[w] = m;
  __syncthreads();
  if (tid == 0) {
    int c = 0;
    for (int q = 0; q < kPairSelW; ++q) c = max(c, sh_i[q]);
    s_cstar = n >= 8 ? c : 0;
  }
  __syncthreads();
  const int cstar = s_cstar;
  // ---- ordered candidates: count == c* ----
  int nloc = 0;
  if (cstar > 0) {
    for (int base = 0; base < H; base += kPairSelT) {
      const int i = base + tid;
      const bool take = i < H && cnt[i] == cstar;
      const unsigned long long bal = __ballot(take);
      if (lane == 0) woff[w] = __popcll(bal);
      __syncthreads();
      int pre = nloc, tot = 0;
      for (int q = 0; q < kPairSelW; ++q) {
        if (q < w) pre += woff[q];
        tot += woff[q];
      }
      if (take) cb[pre + __popcll(bal & ((1ull << lane) - 1ull))] = i;
      nloc += tot;
      __syncthreads();
    }
  }
  // ---- np.linalg.norm(d) of every candidate: k_pairs_count's (same bits as a wave per
  // candidate; C4's ~1 000 tied candidates per pair took one wave pass each here) ----
  __syncthreads();  // (cb complete)
  for (int j = tid; j < nloc; j += kPairSelT) {  // the chunks' subtrees, in tree order
    const double *t = nrmp + (static_cast<int64_t>(b) * H + cb[j]) * kCountChunks;
    static_assert(kCountChunks == 8, "three levels above the chunks");
    nb[j] = sqrt(((t[0] + t[1]) + (t[2] + t[3])) + ((t[4] + t[5]) + (t[6] + t[7])));
  }
  __syncthreads();
  // ---- fun.py:320-328 replay over the c* candidates (wave 0).  The first one is always
  // taken; later ones replace the best only when best_std > norm(d_j), so the wave searches
  // 64 norms per load for the next such j (ballot) and computes np.std(d) (two-pass) only for
  // the candidates that become best.  C4's exact pairs tie at c* = N on ~all 1 000
  // hypotheses: this replaces ~1 000 serial global loads and 1 000 std passes per pair. ----
  if (w == 0) {
    auto std_of = [&](int j) {
      const int64_t g = static_cast<int64_t>(b) * H + cb[j];
      double f[9];
#pragma unroll
      for (int k = 0; k < 9; ++k) f[k] = Fsoa[k * ld + g];
      double s1 = 0.0;
      for (int i = lane; i < n; i += 64) s1 += dist_ref(f, pts[o + i]);
      s1 = wsum(s1);
      const double mean = s1 / static_cast<double>(n);
      double s3 = 0.0;
      for (int i = lane; i < n; i += 64) {
        const double v = dist_ref(f, pts[o + i]) - mean;
        s3 += v * v;
      }
      s3 = wsum(s3);
      return sqrt(s3 / static_cast<double>(n));
    };
    int best = -1;
    double bstd = 0.0;
    if (nloc > 0) {
      best = 0;
      bstd = std_of(0);
      int j0 = 1;
      while (j0 < nloc) {
        const int j = j0 + lane;
        const bool repl = j < nloc && bstd > nb[j];  // false for NaN on either side
        const unsigned long long bal = __ballot(repl);
        if (bal == 0ull) {
          j0 += 64;
          continue;
        }
        best = j0 + __ffsll(static_cast<long long>(bal)) - 1;
        bstd = std_of(best);
        j0 = best + 1;
      }
    }
    if (lane == 0) {
      s_best = best;
      PairDevResult r;
      if (best >= 0) {
        const int64_t g = static_cast<int64_t>(b) * H + cb[best];
        for (int k = 0; k < 9; ++k) r.F[k] = Fsoa[k * ld + g];
        r.best_index = cb[best];
        r.best_count = cstar;
        r.best_std = bstd;
        r.best_norm = nb[best];
      } else {
        for (int k = 0; k < 9; ++k) r.F[k] = __builtin_nan("");
        r.best_index = -1;
        r.best_count = 0;
        r.best_std = __builtin_nan("");
        r.best_norm = __builtin_nan("");
      }
      r.n_candidates = nloc;
      res[b] = r;
    }
  }
  __syncthreads();
  if (s_best < 0) return;
  // ---- S_RANSAC = flatnonzero(d < thresh), in order, at inl[off[b] ..] ----
  double f[9];
  {
    const int64_t g = static_cast<int64_t>(b) * H + cb[s_best];
#pragma unroll
    for (int k = 0; k < 9; ++k) f[k] = Fsoa[k * ld + g];
  }
  int done = 0;
  for (int base = 0; base < n; base += kPairSelT) {
    const int i = base + tid;
    const bool take = i < n && dist_ref(f, pts[o + i]) < thresh;
    const unsigned long long bal = __ballot(take);
    if (lane == 0) woff[w] = __popcll(bal);
    __syncthreads();
    int pre = done, tot = 0;
    for (int q = 0; q < kPairSelW; ++q) {
      if (q < w) pre += woff[q];
      tot += woff[q];
    }
    if (take) inl[o + pre + __popcll(bal & ((1ull << lane) - 1ull))] = i;
    done += tot;
    __syncthreads();
  }
}

}  // namespace rsd

using rs::fail;
using rs::hip_fail;

#define HIP_TRY(expr)                                 \
  do {                                                \
    hipError_t e_ = (expr);                           \
    if (e_ != hipSuccess) return hip_fail(e_, #expr); \
  } while (0)

static_assert(sizeof(rsd::PairDevResult) == sizeof(rs_pair_result), "rs_pair_result layout");

namespace rs {
// rs_pairs_f8_ransac's validation, upload and kernels, enqueued on the context stream without
// the download: the pair records and inlier lists stay in device memory (PairsDev), with
// `extra` bytes of scratch after them for the caller's next stages (rs_pairs_two_view).
int pairs_enqueue(rs_ctx *c, const double *p1, const double *p2, const int64_t *off, int64_t B,
                  int64_t H, int32_t mode, uint64_t seed_base, const int64_t *seed_ids,
                  const int32_t *host_tuples, double thresh, size_t extra, PairsDev *d) {
  if (!c || !off || !d) return fail(RS_EINVAL, "null pointer");
  if (B < 1 || B > (1 << 20)) return fail(RS_EINVAL, "bad pair count");
  if (H < 1 || H > (1 << 24) || B * H > (1LL << 31) - 64)
    return fail(RS_EINVAL, "bad hypothesis count");
  if (mode != RS_SAMPLER_PHILOX && mode != RS_SAMPLER_TUPLES) return fail(RS_EINVAL, "bad mode");
  if (mode == RS_SAMPLER_TUPLES && !host_tuples) return fail(RS_EINVAL, "tuple mode needs tuples");
  if (off[0] != 0) return fail(RS_EINVAL, "offsets must start at 0");
  for (int64_t b = 0; b < B; ++b)
    if (off[b + 1] < off[b] || off[b + 1] - off[b] > (1 << 24))
      return fail(RS_EINVAL, "offsets must be non-decreasing");
  const int64_t total = off[B];
  if (total > 0 && (!p1 || !p2)) return fail(RS_EINVAL, "null point arrays");
  if (mode == RS_SAMPLER_TUPLES)
    for (int64_t b = 0; b < B; ++b) {
      const int64_t n = off[b + 1] - off[b];
      if (n < 8) continue;
      const int32_t *t = host_tuples + b * H * 8;
      for (int64_t q = 0; q < H * 8; ++q)
        if (t[q] < 0 || t[q] >= n) return fail(RS_EINVAL, "tuple index out of range");
    }
  HIP_TRY(hipSetDevice(c->device));
  const int64_t ld = B * H, tp = total > 0 ? total : 1;
  auto al = [](size_t x) { return (x + 255) / 256 * 256; };
  const size_t sizes[] = {sizeof(rsd::Pt) * tp,         sizeof(int64_t) * (B + 1),
                          sizeof(double) * 9 * ld,      sizeof(int) * ld,
                          sizeof(int) * ld,             sizeof(double) * rsd::kCountChunks * ld,
                          sizeof(double) * ld,          sizeof(rsd::PairDevResult) * B,
                          sizeof(int32_t) * tp,
                          mode == RS_SAMPLER_TUPLES ? sizeof(int32_t) * 8 * ld : 0,
                          seed_ids ? sizeof(int64_t) * B : 0, extra};
  size_t tot = 0;
  for (size_t s : sizes) tot += al(s);
  int st = rs::ensure_scratch(c, tot + 256);
  if (st) return st;
  std::vector<char *> buf;
  char *p = static_cast<char *>(c->scratch);
  for (size_t s : sizes) {
    buf.push_back(p);
    p += al(s);
  }
  auto *d_pts = reinterpret_cast<rsd::Pt *>(buf[0]);
  auto *d_off = reinterpret_cast<int64_t *>(buf[1]);
  auto *d_F = reinterpret_cast<double *>(buf[2]);
  auto *d_counts = reinterpret_cast<int *>(buf[3]);
  auto *d_cand = reinterpret_cast<int *>(buf[4]);
  auto *d_nrm = reinterpret_cast<double *>(buf[5]);
  auto *d_cnorm = reinterpret_cast<double *>(buf[6]);
  auto *d_res = reinterpret_cast<rsd::PairDevResult *>(buf[7]);
  auto *d_inl = reinterpret_cast<int32_t *>(buf[8]);
  auto *d_tup = reinterpret_cast<int32_t *>(buf[9]);
  auto *d_ids = seed_ids ? reinterpret_cast<int64_t *>(buf[10]) : nullptr;
  if (total > 0) {
    std::vector<rsd::Pt> hp(total);
    for (int64_t i = 0; i < total; ++i) hp[i] = {p1[i], p1[total + i], p2[i], p2[total + i]};
    HIP_TRY(hipMemcpyAsync(d_pts, hp.data(), sizeof(rsd::Pt) * total, hipMemcpyHostToDevice,
                           c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));  // hp goes out of scope
  }
  HIP_TRY(hipMemcpyAsync(d_off, off, sizeof(int64_t) * (B + 1), hipMemcpyHostToDevice, c->stream));
  if (seed_ids)
    HIP_TRY(hipMemcpyAsync(d_ids, seed_ids, sizeof(int64_t) * B, hipMemcpyHostToDevice, c->stream));
  if (mode == RS_SAMPLER_TUPLES)
    HIP_TRY(hipMemcpyAsync(d_tup, host_tuples, sizeof(int32_t) * 8 * ld, hipMemcpyHostToDevice,
                           c->stream));
  hipLaunchKernelGGL(rsd::k_pairs_solve, dim3(static_cast<unsigned>((ld + 255) / 256)), dim3(256),
                     0, c->stream, d_pts, d_off, static_cast<int>(B), static_cast<int>(H), mode,
                     seed_base, d_ids, d_tup, d_F, ld);
  HIP_TRY(hipGetLastError());
  const int64_t units = B * ((H + 63) / 64) * rsd::kCountChunks;
  HIP_TRY(hipMemsetAsync(d_counts, 0, sizeof(int) * ld, c->stream));
  hipLaunchKernelGGL(rsd::k_pairs_count, dim3(static_cast<unsigned>((units + 3) / 4)), dim3(256),
                     0, c->stream, d_pts, d_off, static_cast<int>(B), static_cast<int>(H), d_F,
                     ld, thresh, d_counts, d_nrm);  // (every hypothesis's norm subtrees)
  HIP_TRY(hipGetLastError());
  hipLaunchKernelGGL(rsd::k_pairs_select, dim3(static_cast<unsigned>(B)), dim3(rsd::kPairSelT), 0,
                     c->stream, d_pts, d_off, static_cast<int>(H), d_F, ld, d_counts, thresh,
                     d_cand, d_nrm, d_cnorm, d_res, d_inl);
  HIP_TRY(hipGetLastError());
  d->pts = d_pts;
  d->off = d_off;
  d->res = d_res;
  d->inl = d_inl;
  d->total = total;
  d->extra = buf[11];
  return RS_OK;
}
}  // namespace rs

extern "C" int rs_pairs_f8_ransac(rs_ctx *c, const double *p1, const double *p2,
                                  const int64_t *off, int64_t B, int64_t H, int32_t mode,
                                  uint64_t seed_base, const int64_t *seed_ids,
                                  const int32_t *host_tuples, double thresh,
                                  rs_pair_result *out, int32_t *inliers) {
  if (!out || !inliers) return fail(RS_EINVAL, "null pointer");
  rs::PairsDev d{};
  const int st = rs::pairs_enqueue(c, p1, p2, off, B, H, mode, seed_base, seed_ids, host_tuples,
                                   thresh, 0, &d);
  if (st) return st;
  HIP_TRY(hipMemcpyAsync(out, d.res, sizeof(rs_pair_result) * B, hipMemcpyDeviceToHost, c->stream));
  if (d.total > 0)
    HIP_TRY(hipMemcpyAsync(inliers, d.inl, sizeof(int32_t) * d.total, hipMemcpyDeviceToHost,
                           c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return RS_OK;
}
