// RANSAC-F kernels for gfx950 (MI355X).  See DESIGN.md for the data layout and rooflines.
//
// Pipeline of one run (fun.py:298-328 unrolled into H concurrent hypotheses):
//   k_f8_solve    lane per hypothesis: sample (Philox/Floyd or host tuples) -> 8-point F
//                 (Householder LQ null vector + 3x3 Jacobi rank-2), F stored SoA in HBM
//   k_f8_count    lane per hypothesis x chunk of points: inlier count by the squared test
//                 e^2 < t^2 min(|l1|^2, |l2|^2) (points wave-uniform -> scalar loads)
//   k_f8_select   one workgroup: c* = max count, ordered list of hypotheses with count >=
//                 c* - 1 (guard slack)
//   k_f8_stats    wave per candidate: reference-order float64 d (lab3.py:210-227), count,
//                 np.std(d), np.linalg.norm(d)
//   k_f8_replay   one wave: the fun.py:320-328 rule over the ordered candidates
//   k_f8_inliers  one workgroup: S_RANSAC = flatnonzero(d < t) of the winner, in order
#include <hip/hip_runtime.h>

#include <algorithm>

#include "device_math.h"
#include "f8_kernels.h"

namespace rsd {

__device__ __forceinline__ int wave_uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

// ----------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_f8_solve(const Pt *__restrict__ pts, int n, int H,
                                                  int mode, uint64_t seed, uint64_t hyp_offset,
                                                  const int *__restrict__ tuples,
                                                  double *__restrict__ Fsoa, int64_t ld,
                                                  int *__restrict__ counts,
                                                  int *__restrict__ status) {
  const int h = blockIdx.x * blockDim.x + threadIdx.x;
  if (h >= H) return;
  if (counts) counts[h] = 0;  // the counting kernel accumulates into it
  if (status && h < 2) status[h] = 0;  // c*, n_candidates
  int idx[8];
  if (mode == RSD_SAMPLER_PHILOX) {
    floyd_sample<8>(seed, hyp_offset + static_cast<uint64_t>(h), n, idx);
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) idx[k] = tuples[static_cast<int64_t>(h) * 8 + k];
  }
  double xl[8], yl[8], xr[8], yr[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const Pt p = pts[idx[k]];
    xl[k] = p.x1;
    yl[k] = p.y1;
    xr[k] = p.x2;
    yr[k] = p.y2;
  }
  double F[9];
  fmatrix8(xl, yl, xr, yr, F);
#pragma unroll
  for (int k = 0; k < 9; ++k) Fsoa[k * ld + h] = F[k];
}

// ----------------------------------------------------------------------------------------
// Counting: unit u = (group g of 64 hypotheses, chunk c of points).  F lives in VGPRs (one
// hypothesis per lane); the point is the same for all 64 lanes, so its 32 B come through
// the scalar cache into SGPRs and feed the VALU as a free scalar operand.  21 float64 VALU
// ops per (hypothesis, point); no LDS, no cross-lane traffic.
// ----------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_f8_count(const Pt *__restrict__ pts, int n, int H,
                                                  const double *__restrict__ Fsoa, int64_t ld,
                                                  int chunk, int nchunks, double thr2,
                                                  int *__restrict__ counts) {
  const int lane = threadIdx.x & 63;
  const int u = wave_uniform(blockIdx.x * 4 + (threadIdx.x >> 6));
  const int ngroups = (H + 63) >> 6;
  if (u >= ngroups * nchunks) return;
  const int g = u / nchunks;
  const int c = u - g * nchunks;
  const int p0 = c * chunk;
  const int p1 = min(n, p0 + chunk);
  const int h = g * 64 + lane;
  const int hl = h < H ? h : H - 1;
  double f[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) f[k] = Fsoa[k * ld + hl];
  int cnt = 0;
#pragma unroll 2
  for (int i = p0; i < p1; ++i) {
    const Pt p = pts[i];
    const double l10 = fma(f[0], p.x2, fma(f[1], p.y2, f[2]));
    const double l11 = fma(f[3], p.x2, fma(f[4], p.y2, f[5]));
    const double l12 = fma(f[6], p.x2, fma(f[7], p.y2, f[8]));
    const double l20 = fma(f[0], p.x1, fma(f[3], p.y1, f[6]));
    const double l21 = fma(f[1], p.x1, fma(f[4], p.y1, f[7]));
    // e = x^T F y = l1 . x^ = l2 . y^ (both residual numerators are the same quantity)
    const double e = fma(l10, p.x1, fma(l11, p.y1, l12));
    const double n1 = fma(l10, l10, l11 * l11);
    const double n2 = fma(l20, l20, l21 * l21);
    // d < t  <=>  e^2 < t^2 min(n1, n2); false for NaN / zero-length lines as in numpy
    cnt += (e * e < thr2 * fmin(n1, n2)) ? 1 : 0;
  }
  if (h < H) atomicAdd(&counts[h], cnt);
}

// ----------------------------------------------------------------------------------------
// Selection over H counts in three grid-wide passes (no single-workgroup scan):
//   k_f8_max        c* = max count (block max -> one atomicMax per block)
//   k_f8_blockcount per block slice: number of hypotheses with count >= max(c* - slack, 1)
//   k_f8_compact    ordered compaction: block offset = sum of earlier block counts, then
//                   ballot/popcount prefix inside the block; the last block writes the total
// ----------------------------------------------------------------------------------------
__device__ __forceinline__ int block_reduce_max(int v, int *sh) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  int r = sh[0];
  for (int q = 1; q < (int)(blockDim.x >> 6); ++q) r = max(r, sh[q]);
  __syncthreads();
  return r;
}
__device__ __forceinline__ int block_reduce_sum(int v, int *sh) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  int r = 0;
  for (int q = 0; q < (int)(blockDim.x >> 6); ++q) r += sh[q];
  __syncthreads();
  return r;
}

__global__ __launch_bounds__(256) void k_f8_max(const int *__restrict__ counts, int H,
                                                int *__restrict__ status) {
  __shared__ int sh[4];
  int m = 0;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < H; i += gridDim.x * 256) m = max(m, counts[i]);
  m = block_reduce_max(m, sh);
  if (threadIdx.x == 0 && m > 0) atomicMax(&status[0], m);
}

__global__ __launch_bounds__(256) void k_f8_blockcount(const int *__restrict__ counts, int H,
                                                       int slack, int per_block,
                                                       const int *__restrict__ status,
                                                       int *__restrict__ bc) {
  __shared__ int sh[4];
  const int cmax = status[0];
  const int thr = max(cmax - slack, 1);
  const int b0 = blockIdx.x * per_block, b1 = min(H, b0 + per_block);
  int c = 0;
  if (cmax > 0)
    for (int i = b0 + threadIdx.x; i < b1; i += 256) c += counts[i] >= thr ? 1 : 0;
  c = block_reduce_sum(c, sh);
  if (threadIdx.x == 0) bc[blockIdx.x] = c;
}

__global__ __launch_bounds__(256) void k_f8_compact(const int *__restrict__ counts, int H,
                                                    int slack, int per_block,
                                                    int *__restrict__ status,
                                                    const int *__restrict__ bc,
                                                    int *__restrict__ cand) {
  __shared__ int sh[4];
  __shared__ int woff[4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int off = 0;
  for (int j = tid; j < (int)blockIdx.x; j += 256) off += bc[j];
  off = block_reduce_sum(off, sh);
  const int cmax = status[0];
  const int thr = max(cmax - slack, 1);
  const int b0 = blockIdx.x * per_block, b1 = min(H, b0 + per_block);
  if (cmax > 0 && bc[blockIdx.x] > 0) {
    for (int b = b0; b < b1; b += 256) {
      const int i = b + tid;
      const bool take = i < b1 && counts[i] >= thr;
      const unsigned long long bal = __ballot(take);
      if (lane == 0) woff[w] = __popcll(bal);
      __syncthreads();
      int base = off;
      for (int q = 0; q < w; ++q) base += woff[q];
      const int tot = woff[0] + woff[1] + woff[2] + woff[3];
      if (take) cand[base + __popcll(bal & ((1ull << lane) - 1ull))] = i;
      off += tot;
      __syncthreads();
    }
  }
  if (blockIdx.x == gridDim.x - 1 && tid == 0) status[1] = off + (cmax > 0 ? 0 : 0);
}

// ----------------------------------------------------------------------------------------
// Reference-order statistics, wave per candidate (grid-stride).
// ----------------------------------------------------------------------------------------
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ double block_sum_d(double v, double *sh) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  double r = 0.0;
  for (int q = 0; q < (int)(blockDim.x >> 6); ++q) r += sh[q];
  __syncthreads();
  return r;
}

// Workgroup (256 threads) per candidate, grid-stride over the device-side candidate count.
__global__ __launch_bounds__(256) void k_f8_stats(const Pt *__restrict__ pts, int n,
                                                  const double *__restrict__ Fsoa, int64_t ld,
                                                  const int *__restrict__ cand,
                                                  const int *__restrict__ status, double thresh,
                                                  int *__restrict__ ccount,
                                                  double *__restrict__ cstd,
                                                  double *__restrict__ cnorm) {
  __shared__ double shd[4];
  __shared__ int shi[4];
  const int tid = threadIdx.x;
  const int nc = status[1];
  for (int c = blockIdx.x; c < nc; c += gridDim.x) {
    const int h = cand[c];
    double f[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) f[k] = Fsoa[k * ld + h];
    double s1 = 0.0, s2 = 0.0;
    int cnt = 0;
    for (int i = tid; i < n; i += 256) {
      const double d = dist_ref(f, pts[i]);
      cnt += d < thresh ? 1 : 0;
      s1 += d;
      s2 += d * d;
    }
    s1 = block_sum_d(s1, shd);
    s2 = block_sum_d(s2, shd);
    cnt = block_reduce_sum(cnt, shi);
    const double mean = s1 / static_cast<double>(n);
    double s3 = 0.0;
    for (int i = tid; i < n; i += 256) {
      const double v = dist_ref(f, pts[i]) - mean;
      s3 += v * v;
    }
    s3 = block_sum_d(s3, shd);
    if (tid == 0) {
      ccount[c] = cnt;
      cstd[c] = sqrt(s3 / static_cast<double>(n));
      cnorm[c] = sqrt(s2);
    }
  }
}

// ----------------------------------------------------------------------------------------
// fun.py:320-328 over the ordered candidates.  Comparisons of non-negative doubles are done
// on their bit patterns (NaN keyed so that it never wins), scanning 64 candidates per
// coalesced load.
// ----------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t key_std(double s) {  // "best_std > x" is false for NaN
  return (s != s) ? 0ull : static_cast<uint64_t>(__double_as_longlong(s));
}
__device__ __forceinline__ uint64_t key_norm(double v) {  // "y > norm" is false for NaN
  return (v != v) ? ~0ull : static_cast<uint64_t>(__double_as_longlong(v));
}

__global__ __launch_bounds__(64) void k_f8_replay(const int *__restrict__ cand,
                                                  const int *__restrict__ status,
                                                  const int *__restrict__ counts,
                                                  const int *__restrict__ ccount,
                                                  const double *__restrict__ cstd,
                                                  const double *__restrict__ cnorm,
                                                  const double *__restrict__ Fsoa, int64_t ld,
                                                  F8DevResult *__restrict__ res) {
  const int lane = threadIdx.x;
  const int nc = status[1];
  int best = -1, bcount = 0;
  uint64_t bstd = 0ull;  // S_RANSAC = [], norm([]) = 0
  int mismatch = 0;
  for (int b = 0; b < nc; b += 64) {
    const int c = b + lane;
    int cc = 0;
    uint64_t ks = 0, kn = 0;
    if (c < nc) {
      cc = ccount[c];
      ks = key_std(cstd[c]);
      kn = key_norm(cnorm[c]);
      mismatch += (cc != counts[cand[c]]) ? 1 : 0;
    }
    const int lim = min(64, nc - b);
    for (int q = 0; q < lim; ++q) {
      const int qc = __shfl(cc, q);
      const uint64_t qs = __shfl(ks, q);
      const uint64_t qn = __shfl(kn, q);
      if (qc > bcount) {
        best = b + q;
        bcount = qc;
        bstd = qs;
      } else if (qc == bcount && bcount > 0 && bstd > qn) {
        best = b + q;
        bstd = qs;
      }
    }
  }
  mismatch = wave_sum_i(mismatch);
  if (lane == 0) {
    res->n_candidates = nc;
    res->max_count_fast = status[0];
    res->guard_mismatch = mismatch;
    if (best >= 0) {
      const int h = cand[best];
      res->best_index = h;
      res->best_count = bcount;
      res->best_std = cstd[best];
      res->best_norm = cnorm[best];
      res->best_cand = best;
      for (int k = 0; k < 9; ++k) res->F[k] = Fsoa[k * ld + h];
    } else {
      res->best_index = -1;
      res->best_count = 0;
      res->best_std = 0.0;
      res->best_norm = 0.0;
      res->best_cand = -1;
      for (int k = 0; k < 9; ++k) res->F[k] = 0.0;
    }
  }
}

// ----------------------------------------------------------------------------------------
// S_RANSAC of the winner: ascending indices with d < thresh (np.flatnonzero order).
// ----------------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_f8_inliers(const Pt *__restrict__ pts, int n,
                                                     double thresh,
                                                     F8DevResult *__restrict__ res) {
  __shared__ int woff[16];
  __shared__ int base_s;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const bool have = res->best_index >= 0;
  double f[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) f[k] = res->F[k];
  if (tid == 0) base_s = 0;
  __syncthreads();
  for (int b = 0; b < n; b += 1024) {
    const int i = b + tid;
    const bool take = have && i < n && dist_ref(f, pts[i]) < thresh;
    const unsigned long long bal = __ballot(take);
    const int before = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) woff[w] = __popcll(bal);
    __syncthreads();
    if (tid == 0) {
      int acc = base_s;
      for (int q = 0; q < 16; ++q) {
        const int t = woff[q];
        woff[q] = acc;
        acc += t;
      }
      base_s = acc;
    }
    __syncthreads();
    if (take) res->inliers[woff[w] + before] = i;
    __syncthreads();
  }
  if (tid == 0) res->n_inliers = base_s;
}

// ----------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_residuals(const Pt *__restrict__ pts, int n,
                                                   const double *__restrict__ F,
                                                   double *__restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double f[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) f[k] = F[k];
  double r1, r2;
  residuals_ref(f, pts[i], r1, r2);
  out[i] = r1;
  out[n + i] = r2;
}

// Pack (2,n) row-major p1, p2 into AoS points.
__global__ __launch_bounds__(256) void k_pack_points(const double *__restrict__ p1,
                                                     const double *__restrict__ p2, int n,
                                                     Pt *__restrict__ pts) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Pt p;
  p.x1 = p1[i];
  p.y1 = p1[n + i];
  p.x2 = p2[i];
  p.y2 = p2[n + i];
  pts[i] = p;
}

}  // namespace rsd

// ------------------------------------------------------------------------------------------
// Host launchers
// ------------------------------------------------------------------------------------------
namespace rsd {

hipError_t launch_pack_points(const double *p1, const double *p2, int n, Pt *pts,
                              hipStream_t s) {
  hipLaunchKernelGGL(k_pack_points, dim3((n + 255) / 256), dim3(256), 0, s, p1, p2, n, pts);
  return hipGetLastError();
}

hipError_t launch_f8_solve(const Pt *pts, int n, int H, int mode, uint64_t seed,
                           uint64_t hyp_offset, const int *tuples, double *Fsoa, int64_t ld,
                           int *counts, int *status, hipStream_t s) {
  hipLaunchKernelGGL(k_f8_solve, dim3((H + 255) / 256), dim3(256), 0, s, pts, n, H, mode, seed,
                     hyp_offset, tuples, Fsoa, ld, counts, status);
  return hipGetLastError();
}

hipError_t launch_f8_count(const Pt *pts, int n, int H, const double *Fsoa, int64_t ld,
                           int chunk, double thr2, int *counts, hipStream_t s) {
  const int nchunks = (n + chunk - 1) / chunk;
  const int units = ((H + 63) / 64) * nchunks;
  hipLaunchKernelGGL(k_f8_count, dim3((units + 3) / 4), dim3(256), 0, s, pts, n, H, Fsoa, ld,
                     chunk, nchunks, thr2, counts);
  return hipGetLastError();
}

hipError_t launch_f8_select(const int *counts, int H, int slack, int *cand, int *status,
                            hipStream_t s) {
  int *bc = status + 4;  // kSelectBlocks block counts live behind the status words
  const int per_block = (H + kSelectBlocks - 1) / kSelectBlocks;
  const int nb = (H + per_block - 1) / per_block;
  hipLaunchKernelGGL(k_f8_max, dim3(std::min(nb, 256)), dim3(256), 0, s, counts, H, status);
  hipLaunchKernelGGL(k_f8_blockcount, dim3(nb), dim3(256), 0, s, counts, H, slack, per_block,
                     status, bc);
  hipLaunchKernelGGL(k_f8_compact, dim3(nb), dim3(256), 0, s, counts, H, slack, per_block,
                     status, bc, cand);
  return hipGetLastError();
}

hipError_t launch_f8_stats(const Pt *pts, int n, const double *Fsoa, int64_t ld,
                           const int *cand, const int *status, double thresh, int *ccount,
                           double *cstd, double *cnorm, int grid, hipStream_t s) {
  hipLaunchKernelGGL(k_f8_stats, dim3(grid), dim3(256), 0, s, pts, n, Fsoa, ld, cand, status,
                     thresh, ccount, cstd, cnorm);
  return hipGetLastError();
}

hipError_t launch_f8_replay(const int *cand, const int *status, const int *counts,
                            const int *ccount, const double *cstd, const double *cnorm,
                            const double *Fsoa, int64_t ld, F8DevResult *res, hipStream_t s) {
  hipLaunchKernelGGL(k_f8_replay, dim3(1), dim3(64), 0, s, cand, status, counts, ccount, cstd,
                     cnorm, Fsoa, ld, res);
  return hipGetLastError();
}

hipError_t launch_f8_inliers(const Pt *pts, int n, double thresh, F8DevResult *res,
                             hipStream_t s) {
  hipLaunchKernelGGL(k_f8_inliers, dim3(1), dim3(1024), 0, s, pts, n, thresh, res);
  return hipGetLastError();
}

hipError_t launch_residuals(const Pt *pts, int n, const double *F, double *out,
                            hipStream_t s) {
  hipLaunchKernelGGL(k_residuals, dim3((n + 255) / 256), dim3(256), 0, s, pts, n, F, out);
  return hipGetLastError();
}

}  // namespace rsd
