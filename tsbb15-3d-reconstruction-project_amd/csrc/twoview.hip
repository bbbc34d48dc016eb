// Two-view geometry after the RANSAC loop, batched on the GPU:
//
//   k_triangulate_optimal  lane per point: lab3.triangulate_optimal (lab3.py:382-475)
//   k_resection            lane per camera: fun.camera_resectioning (fun.py:260-280)
//   k_essential            lane per pair: E = K^T F K (fun.getEAndK, fun.py:101)
//   k_relative_pose        quad per pair (lane per candidate pose): fun.relative_camera_pose
//                          (fun.py:209-258)
//   k_fmatrix_cameras / k_fmatrix_from_cameras: lab3.py:353-380 / 331-351
//   k_gold_standard        workgroup per pair: the gold-standard tail of fun.getFFromLabCode
//                          (fun.py:336-369) -- cameras from F_RANSAC, optimal triangulation of
//                          the inliers, least squares on lab3.fmatrix_residuals_gs
//                          (lab3.py:228-266) over (C1, X), F from the refined cameras.  The
//                          least-squares step is Levenberg-Marquardt run to convergence with
//                          the 3x3 point blocks eliminated (Schur complement on the 12 camera
//                          parameters); see oracle/twoview_ref.gold_standard_lm for why the
//                          reference's scipy TRF end point is not the target.
#include <hip/hip_runtime.h>

#include <cstring>
#include <initializer_list>
#include <vector>

#include "common.h"
#include "ctx.h"
#include "device_math.h"
#include "twoview_math.h"

namespace rsd {

__global__ __launch_bounds__(128) void k_triangulate_optimal(const double *__restrict__ C1s,
                                      const double *__restrict__ C2s,
                                      const double *__restrict__ x1, const double *__restrict__ x2,
                                      const int32_t *__restrict__ cam, int64_t n,
                                      double *__restrict__ X) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int k = cam ? cam[i] : 0;
  double C1[12], C2[12], Y[3];
#pragma unroll
  for (int q = 0; q < 12; ++q) {
    C1[q] = C1s[12 * k + q];
    C2[q] = C2s[12 * k + q];
  }
  triangulate_optimal(C1, C2, x1[i], x1[n + i], x2[i], x2[n + i], Y);
  X[3 * i + 0] = Y[0];
  X[3 * i + 1] = Y[1];
  X[3 * i + 2] = Y[2];
}

// fun.camera_resectioning: P = lambda K [R | t], K upper triangular with positive diagonal
// and K[2,2] = 1, R a rotation.  The decomposition is unique, so it is computed directly
// (RQ by twice-applied Gram-Schmidt from the last row, then the sign of det A), without the
// LAPACK sign conventions specRQ (fun.py:181-188) and the D fix-up (fun.py:267-279) undo.
__global__ __launch_bounds__(128) void k_resection(const double *__restrict__ P, int64_t B, double *__restrict__ K,
                            double *__restrict__ R, double *__restrict__ t) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= B) return;
  double a[3][3], b[3];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
#pragma unroll
    for (int c = 0; c < 3; ++c) a[r][c] = P[12 * i + 4 * r + c];
    b[r] = P[12 * i + 4 * r + 3];
  }
  double U[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}}, Q[3][3];
  for (int r = 2; r >= 0; --r) {
    double w[3] = {a[r][0], a[r][1], a[r][2]};
    for (int pass = 0; pass < 2; ++pass)
      for (int k = r + 1; k < 3; ++k) {
        const double p = w[0] * Q[k][0] + w[1] * Q[k][1] + w[2] * Q[k][2];
        U[r][k] += p;
        w[0] -= p * Q[k][0];
        w[1] -= p * Q[k][1];
        w[2] -= p * Q[k][2];
      }
    const double nrm = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    U[r][r] = nrm;
    Q[r][0] = w[0] / nrm;
    Q[r][1] = w[1] / nrm;
    Q[r][2] = w[2] / nrm;
  }
  const double detA = a[0][0] * (a[1][1] * a[2][2] - a[1][2] * a[2][1]) -
                      a[0][1] * (a[1][0] * a[2][2] - a[1][2] * a[2][0]) +
                      a[0][2] * (a[1][0] * a[2][1] - a[1][1] * a[2][0]);
  const double s = detA < 0.0 ? -1.0 : 1.0;
  // t = s U^-1 b (back substitution)
  double y[3];
  y[2] = b[2] / U[2][2];
  y[1] = (b[1] - U[1][2] * y[2]) / U[1][1];
  y[0] = (b[0] - U[0][1] * y[1] - U[0][2] * y[2]) / U[0][0];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      K[9 * i + 3 * r + c] = U[r][c] / U[2][2];
      R[9 * i + 3 * r + c] = s * Q[r][c];
    }
    t[3 * i + r] = s * y[r];
  }
}

__global__ __launch_bounds__(128) void k_essential(const double *__restrict__ K, int k_stride,
                            const double *__restrict__ F, int64_t B, double *__restrict__ E) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= B) return;
  double k[9], f[9], kt[9], T[9], e[9];
#pragma unroll
  for (int q = 0; q < 9; ++q) {
    k[q] = K[k_stride * i + q];
    f[q] = F[9 * i + q];
  }
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) kt[3 * r + c] = k[3 * c + r];
  mul33(kt, f, T);
  mul33(T, k, e);
#pragma unroll
  for (int q = 0; q < 9; ++q) E[9 * i + q] = e[q];
}

// fun.relative_camera_pose: specSVD(E) (U, V with det +1), candidates
// (V W U^T, v3), (V W^T U^T, v3), (V W U^T, -v3), (V W^T U^T, -v3), W = [[0,1,0],[-1,0,0],
// [0,0,1]]; the first whose optimally triangulated first correspondence has positive depth
// in both cameras wins (found = 1..4), else found = 0 (the reference returns None).  The
// candidate set does not depend on the SVD's sign / ordering freedom of the two equal
// singular values, so the pose is the reference's whenever exactly one candidate passes.
__global__ __launch_bounds__(128) void k_relative_pose(const double *__restrict__ Es, const double *__restrict__ y1,
                                const double *__restrict__ y2, int64_t Bn,
                                double *__restrict__ Rout, double *__restrict__ tout,
                                int32_t *__restrict__ found,
                                const int32_t *__restrict__ act = nullptr) {
  const int64_t gt = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int64_t i0 = gt >> 2;
  const int k = static_cast<int>(gt & 3);
  const bool live = i0 < Bn;
  const int64_t i = live ? i0 : Bn - 1;  // padding quads recompute the last pair, store nothing
  // (act: pairs with act[i] == 0 have no E -- rs_pairs_two_view's pairs without a consensus:
  // a stand-in E, no candidate passes, NaN pose and found 0)
  const bool skip = act && !act[i];
  double B[9], V[9];
#pragma unroll
  for (int q = 0; q < 9; ++q) B[q] = skip ? (q == 0 || q == 4 ? 1.0 : 0.0) : Es[9 * i + q];
  svd3_jacobi(B, V);
  double s[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) s[j] = B[j] * B[j] + B[3 + j] * B[3 + j] + B[6 + j] * B[6 + j];
  const int m = (s[0] <= s[1] && s[0] <= s[2]) ? 0 : (s[1] <= s[2] ? 1 : 2);
  int p = m == 0 ? 1 : 0, q = m == 2 ? 1 : 2;
  if (s[q] > s[p]) {  // descending, as LAPACK
    const int tmp = p;
    p = q;
    q = tmp;
  }
  double u1[3], u2[3], u3[3], v1[3], v2[3], v3[3];
  const double i1 = 1.0 / sqrt(s[p]), i2 = 1.0 / sqrt(s[q]);
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    u1[r] = B[3 * r + p] * i1;
    u2[r] = B[3 * r + q] * i2;
    v1[r] = V[3 * r + p];
    v2[r] = V[3 * r + q];
  }
  cross3(u1, u2, u3);
  cross3(v1, v2, v3);
  // V W U^T = -v2 u1^T + v1 u2^T + v3 u3^T;  V W^T U^T = v2 u1^T - v1 u2^T + v3 u3^T
  double Ra[9], Rb[9];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const double base = v3[r] * u3[c];
      const double x = v1[r] * u2[c] - v2[r] * u1[c];
      Ra[3 * r + c] = base + x;
      Rb[3 * r + c] = base - x;
    }
  // the four (R, t) candidates of fun.py:238-254, one per lane of the pair's quad, each with
  // its optimal triangulation of the first correspondence; the first that passes wins
  const double I34[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
  const double *Rk = (k & 1) ? Rb : Ra;
  const double sg = k < 2 ? 1.0 : -1.0;
  double C2[12];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    C2[4 * r + 0] = Rk[3 * r + 0];
    C2[4 * r + 1] = Rk[3 * r + 1];
    C2[4 * r + 2] = Rk[3 * r + 2];
    C2[4 * r + 3] = sg * v3[r];
  }
  double X[3];
  triangulate_optimal<true>(I34, C2, y1[2 * i], y1[2 * i + 1], y2[2 * i], y2[2 * i + 1], X);
  const double z2 = Rk[6] * X[0] + Rk[7] * X[1] + Rk[8] * X[2] + sg * v3[2];
  const bool pass = !skip && X[2] > 0.0 && z2 > 0.0;
  // quad lanes 4j..4j+3 hold k = 0..3 of one pair (the grid is a multiple of 4 lanes)
  const unsigned long long bal = __ballot(pass);
  const int q0 = (threadIdx.x & 63) & ~3;
  const unsigned quad = static_cast<unsigned>((bal >> q0) & 0xfull);
  const int which = quad ? __ffs(quad) : 0;  // first passing candidate, 1-based
  if (live && which == k + 1) {
#pragma unroll
    for (int q2 = 0; q2 < 9; ++q2) Rout[9 * i + q2] = Rk[q2];
#pragma unroll
    for (int r = 0; r < 3; ++r) tout[3 * i + r] = sg * v3[r];
  } else if (live && which == 0 && k == 0) {
#pragma unroll
    for (int q2 = 0; q2 < 9; ++q2) Rout[9 * i + q2] = __builtin_nan("");
#pragma unroll
    for (int r = 0; r < 3; ++r) tout[3 * i + r] = __builtin_nan("");
  }
  if (live && k == 0) found[i] = which;
}

__global__ __launch_bounds__(128) void k_fmatrix_cameras(const double *__restrict__ F, int64_t B,
                                  double *__restrict__ C1) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= B) return;
  double f[9], c[12];
#pragma unroll
  for (int q = 0; q < 9; ++q) f[q] = F[9 * i + q];
  fmatrix_cameras(f, c);
#pragma unroll
  for (int q = 0; q < 12; ++q) C1[12 * i + q] = c[q];
}

__global__ __launch_bounds__(128) void k_fmatrix_from_cameras(const double *__restrict__ C1s,
                                       const double *__restrict__ C2s, int64_t B,
                                       double *__restrict__ F) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= B) return;
  double a[12], b[12], f[9];
#pragma unroll
  for (int q = 0; q < 12; ++q) {
    a[q] = C1s[12 * i + q];
    b[q] = C2s[12 * i + q];
  }
  fmatrix_from_cameras(a, b, f);
#pragma unroll
  for (int q = 0; q < 9; ++q) F[9 * i + q] = f[q];
}

// ----------------------------------------------------------------------------------------
// Gold standard (fun.py:336-369), one workgroup per pair.
// ----------------------------------------------------------------------------------------
#ifndef RSAMD_GS_T
#define RSAMD_GS_T 256  // threads per pair (A/B: 64; r05c4a: 463 vs 561 us per C4 launch)
#endif
constexpr int kGsT = RSAMD_GS_T;
#ifndef RSAMD_GS_WAVE
#define RSAMD_GS_WAVE 1  // pairs of <= RSAMD_GS_WAVE_MAX inliers on one wave (A/B: 0)
#endif
#ifndef RSAMD_GS_WAVE_MAX
#define RSAMD_GS_WAVE_MAX 64
#endif
constexpr int kPerPt = 45;  // W (12x3), V (3x3 upper: 6), gx (3)

// Index of (r, c), r <= c, in a packed upper-triangular 12x12.
__device__ __forceinline__ int up12(int r, int c) { return r * 12 - (r * (r - 1)) / 2 + (c - r); }

// One halving step of a wave's reduce-scatter: lanes with bit o set keep the upper half of x
// and send the lower half to lane ^ o (the others the reverse), each adding what it receives.
template <int N>
__device__ __forceinline__ void rs_halve(const double (&x)[N], double (&y)[N / 2], int o) {
  const bool up = (threadIdx.x & o) != 0;
#pragma unroll
  for (int i = 0; i < N / 2; ++i) {
    const double send = up ? x[i] : x[i + N / 2];
    const double keep = up ? x[i + N / 2] : x[i];
    y[i] = keep + __shfl_xor(send, o);
  }
}

// The gold standard's barrier: a workgroup barrier, or for a one-wave pair (T == 64: the
// workgroup's other waves have left) a wave-level LDS fence -- no s_barrier across waves that
// have exited.  Points are owned by one thread in every phase, so only LDS is shared.
template <int T>
__device__ __forceinline__ void gs_sync() {
  if constexpr (T == 64) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  } else {
    __syncthreads();
  }
}

// Sum over the workgroup's T threads of K values per thread into out[0..K) (LDS).  Large K: a
// reduce-scatter inside each wave (six halving exchanges of the values padded to 128: 126
// exchanges instead of a 6-step butterfly per value, 6 K), lane l ending with the wave's sums
// of values 2 l and 2 l + 1; then the waves' partial sums added in wave order.
template <int K, int T>
__device__ __forceinline__ void block_reduce(double (&v)[K], double *scratch, double *out) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if constexpr (K > 16) {
    static_assert(K <= 128, "reduce-scatter holds 128 values");
    double x[128], a[64], b[32], c[16], d[8], e[4], f[2];
#pragma unroll
    for (int k = 0; k < 128; ++k) x[k] = k < K ? v[k] : 0.0;
    rs_halve<128>(x, a, 32);
    rs_halve<64>(a, b, 16);
    rs_halve<32>(b, c, 8);
    rs_halve<16>(c, d, 4);
    rs_halve<8>(d, e, 2);
    rs_halve<4>(e, f, 1);
    if constexpr (T == 64) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
        if (2 * lane + i < K) out[2 * lane + i] = f[i];
      gs_sync<T>();
    } else {
#pragma unroll
      for (int i = 0; i < 2; ++i) scratch[w * 128 + 2 * lane + i] = f[i];
      gs_sync<T>();
      for (int k = threadIdx.x; k < K; k += T) {
        double s = 0.0;
#pragma unroll
        for (int q = 0; q < T / 64; ++q) s += scratch[q * 128 + k];
        out[k] = s;
      }
      gs_sync<T>();
    }
  } else {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      double x = v[k];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
      if (lane == 0) scratch[w * K + k] = x;
    }
    gs_sync<T>();
    for (int k = threadIdx.x; k < K; k += T) {
      double s = 0.0;
#pragma unroll
      for (int q = 0; q < T / 64; ++q) s += scratch[q * K + k];
      out[k] = s;
    }
    gs_sync<T>();
  }
}

// The gold standard's sums on a one-wave pair (n <= 64 points, lane j = point j): the lanes'
// K values transposed through LDS (tr: n rows of K) and column k summed over the rows, in
// point order, by lane k -- n adds instead of block_reduce's reduce-scatter, whose 128 padded
// values spill to AGPRs at this kernel's register pressure (gold standard at C4: 437 -> 353
// us).  (The same for the 256-thread pairs up to 160 points, rows summed in two halves by two
// thread groups: 361 us, not kept -- a 116 KB row buffer for no gain.)
#ifndef RSAMD_GS_TR
#define RSAMD_GS_TR 1
#endif
template <int K>
__device__ __forceinline__ void wave_reduce_tr(double (&v)[K], double *tr, double *out, int n) {
  const int lane = threadIdx.x & 63;
  n = min(n, 64);  // rows: the lanes holding points (lane l sums points l, l + 64, ...)
  if (lane < n) {
#pragma unroll
    for (int k = 0; k < K; ++k) tr[lane * K + k] = v[k];
  }
  gs_sync<64>();
  for (int k = lane; k < K; k += 64) {
    double s = 0.0;
    for (int j = 0; j < n; ++j) s += tr[j * K + k];
    out[k] = s;
  }
  gs_sync<64>();
}

template <int K, int T>
__device__ __forceinline__ void gs_reduce(double (&v)[K], double *red, double *tr, double *out,
                                          int n) {
  if constexpr (T == 64 && RSAMD_GS_TR) wave_reduce_tr<K>(v, tr, out, n);
  else block_reduce<K, T>(v, red, out);
}

// Residuals of lab3.fmatrix_residuals_gs for one point and their Jacobians:
// a0 / a1 (12) = d r0 / d C1, d r1 / d C1;  Bj (4x3) = d r / d X.
__device__ __forceinline__ void gs_point(const double (&C)[12], const double *X, double plx,
                                         double ply, double prx, double pry, double (&r)[4],
                                         double (&a0)[12], double (&a1)[12], double (&Bj)[12]) {
  const double xh[4] = {X[0], X[1], X[2], 1.0};
  const double u = C[0] * xh[0] + C[1] * xh[1] + C[2] * xh[2] + C[3];
  const double v = C[4] * xh[0] + C[5] * xh[1] + C[6] * xh[2] + C[7];
  const double w = C[8] * xh[0] + C[9] * xh[1] + C[10] * xh[2] + C[11];
  const double iw = 1.0 / w, iw2 = iw * iw;
  r[0] = plx - u * iw;
  r[1] = ply - v * iw;
  r[2] = prx - X[0] / X[2];
  r[3] = pry - X[1] / X[2];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    a0[k] = -xh[k] * iw;
    a0[4 + k] = 0.0;
    a0[8 + k] = xh[k] * u * iw2;
    a1[k] = 0.0;
    a1[4 + k] = -xh[k] * iw;
    a1[8 + k] = xh[k] * v * iw2;
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    Bj[k] = -(C[k] * w - u * C[8 + k]) * iw2;
    Bj[3 + k] = -(C[4 + k] * w - v * C[8 + k]) * iw2;
  }
  const double iz = 1.0 / X[2];
  Bj[6] = -iz;
  Bj[7] = 0.0;
  Bj[8] = X[0] * iz * iz;
  Bj[9] = 0.0;
  Bj[10] = -iz;
  Bj[11] = X[1] * iz * iz;
}

__device__ __forceinline__ double gs_cost_point(const double (&C)[12], const double *X, double plx,
                                                double ply, double prx, double pry) {
  const double u = C[0] * X[0] + C[1] * X[1] + C[2] * X[2] + C[3];
  const double v = C[4] * X[0] + C[5] * X[1] + C[6] * X[2] + C[7];
  const double w = C[8] * X[0] + C[9] * X[1] + C[10] * X[2] + C[11];
  const double r0 = plx - u / w, r1 = ply - v / w;
  const double r2 = prx - X[0] / X[2], r3 = pry - X[1] / X[2];
  return r0 * r0 + r1 * r1 + r2 * r2 + r3 * r3;
}

// Inverse of the damped point block V + lam diag(V) (packed upper 6) -> packed upper 6.
__device__ __forceinline__ void inv_sym3(const double *V, double lam, double (&Vi)[6]) {
  const double a = V[0] * (1 + lam), b = V[1], c = V[2], d = V[3] * (1 + lam), e = V[4],
               f = V[5] * (1 + lam);
  const double c00 = d * f - e * e, c01 = c * e - b * f, c02 = b * e - c * d;
  const double c11 = a * f - c * c, c12 = b * c - a * e, c22 = a * d - b * b;
  const double id = 1.0 / (a * c00 + b * c01 + c * c02);
  Vi[0] = c00 * id;
  Vi[1] = c01 * id;
  Vi[2] = c02 * id;
  Vi[3] = c11 * id;
  Vi[4] = c12 * id;
  Vi[5] = c22 * id;
}

__device__ __forceinline__ void symv3(const double (&S)[6], const double *x, double *y) {
  y[0] = S[0] * x[0] + S[1] * x[1] + S[2] * x[2];
  y[1] = S[1] * x[0] + S[3] * x[1] + S[4] * x[2];
  y[2] = S[2] * x[0] + S[4] * x[1] + S[5] * x[2];
}

struct GsInfo {  // == rs_gs_info
  double cost_init;
  double cost;
  int32_t iterations;
  int32_t accepted;
  int32_t status;
  int32_t n;
};

// ---- reference-faithful gold standard (fun.py:358 as scipy runs it) ------------------------
// Residuals of lab3.fmatrix_residuals_gs (lab3.py:228-266) for one point k of the parameter
// vector (C1 row-major, X_k): left = pl - project(X_k, C1), right = pr - project(X_k, [I|0]).
// project (lab3.py:52-72) is np.dot(C, [X; 1]): OpenBLAS dgemm, whose microkernel accumulates
// over k = 0..3 with FMAs from zero, so row i is fma(c_i3, 1, fma(c_i2, x2, fma(c_i1, x1,
// c_i0 x0))) = fma(c_i2, x2, fma(c_i1, x1, c_i0 x0)) + c_i3 -- the same bits (checked against
// numpy in tests/test_gpu_twoview.py; tools/gs_trace_cpu.py shows that with these bits and
// the Jacobian's column-major layout scipy's TRF retraces the reference's path exactly).
__device__ __forceinline__ double dgemm_row(const double *c, double X0, double X1, double X2) {
  return __builtin_fma(c[2], X2, __builtin_fma(c[1], X1, c[0] * X0)) + c[3];
}
__device__ __forceinline__ void gs_res4(const double *C, double X0, double X1, double X2,
                                        double plx, double ply, double prx, double pry,
                                        double r[4]) {
#pragma clang fp contract(off)
  const double y0 = dgemm_row(C, X0, X1, X2);
  const double y1 = dgemm_row(C + 4, X0, X1, X2);
  const double y2 = dgemm_row(C + 8, X0, X1, X2);
  r[0] = plx - y0 / y2;
  r[1] = ply - y1 / y2;
  r[2] = prx - X0 / X2;
  r[3] = pry - X1 / X2;
}

// Thread per point k: the residual f(x) (rows k, n+k, 2n+k, 3n+k) and the 2-point forward
// differences scipy's approx_derivative forms for least_squares(jac='2-point'): column j is
// (f(x with x_j -> xp_j) - f(x)) / dx_j, xp and dx computed by the caller exactly as scipy
// does.  J is stored column-major (Jt[col][row], as scipy returns J_transposed.T): LSMR's
// products with J then run in the reference's order.  Entries a parameter cannot reach are
// left as the caller zeroed them (their forward differences are exactly 0).
__global__ __launch_bounds__(128) void k_gs_fd(const double *__restrict__ x,
                                               const double *__restrict__ xp,
                                               const double *__restrict__ dx,
                                               const double *__restrict__ pl,
                                               const double *__restrict__ pr, int64_t n,
                                               double *__restrict__ f, double *__restrict__ J) {
#pragma clang fp contract(off)
  const int64_t k = static_cast<int64_t>(blockIdx.x) * 128 + threadIdx.x;
  if (k >= n) return;
  const int64_t nr = 4 * n;
  double C[12];
#pragma unroll
  for (int j = 0; j < 12; ++j) C[j] = x[j];
  const double X0 = x[12 + 3 * k], X1 = x[13 + 3 * k], X2 = x[14 + 3 * k];
  const double plx = pl[k], ply = pl[n + k], prx = pr[k], pry = pr[n + k];
  double r0[4];
  gs_res4(C, X0, X1, X2, plx, ply, prx, pry, r0);
  const int64_t row[4] = {k, n + k, 2 * n + k, 3 * n + k};
#pragma unroll
  for (int q = 0; q < 4; ++q) f[row[q]] = r0[q];
  if (!J) return;
#pragma unroll
  for (int j = 0; j < 12; ++j) {  // camera parameters: the two left residuals of every point
    const double keep = C[j];
    C[j] = xp[j];
    double r[4];
    gs_res4(C, X0, X1, X2, plx, ply, prx, pry, r);
    C[j] = keep;
    J[j * nr + row[0]] = (r[0] - r0[0]) / dx[j];
    J[j * nr + row[1]] = (r[1] - r0[1]) / dx[j];
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) {  // this point's coordinates: its four residuals
    const int64_t col = 12 + 3 * k + c;
    double r[4];
    gs_res4(C, c == 0 ? xp[col] : X0, c == 1 ? xp[col] : X1, c == 2 ? xp[col] : X2, plx, ply,
            prx, pry, r);
#pragma unroll
    for (int q = 0; q < 4; ++q) J[col * nr + row[q]] = (r[q] - r0[q]) / dx[col];
  }
}

// One pair's gold standard by the workgroup's first T threads (T = 64: one wave)
template <int T>
__device__ __forceinline__ void gs_pair(
    const double *__restrict__ Fin, const double *__restrict__ pl, const double *__restrict__ pr,
    int64_t total, const int64_t *__restrict__ off, int max_iter, double *__restrict__ Xb,
    double *__restrict__ Xc, double *__restrict__ Wb, double *__restrict__ Fout,
    double *__restrict__ C1out, GsInfo *__restrict__ info, double *tr) {
  __shared__ double red[(T / 64) * 128];
  // the linearisation's sums land in sLin (U: 78, gc: 12, |r|^2): no copy out of sres
  __shared__ double sLin[91], sres[94], sC[12], sdc[12];
  double *const sU = sLin, *const sgc = sLin + 78;
  __shared__ double s_lam, s_nu, s_cost, s_cost0;
  __shared__ int s_state, s_it, s_acc, s_status;
  const int tid = threadIdx.x;
  const int64_t j0 = off[blockIdx.x];
  const int n = static_cast<int>(off[blockIdx.x + 1] - j0);
  const double *plx = pl + j0, *ply = pl + total + j0;
  const double *prx = pr + j0, *pry = pr + total + j0;
  double *X = Xb + 3 * j0, *XN = Xc + 3 * j0, *W = Wb + kPerPt * j0;
  const double I34[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};

  if (tid == 0) {
    double f[9], c[12];
    for (int q = 0; q < 9; ++q) f[q] = Fin[9 * blockIdx.x + q];
    fmatrix_cameras(f, c);
    for (int q = 0; q < 12; ++q) sC[q] = c[q];
    s_lam = 1e-3;
    s_nu = 2.0;
    s_it = 0;
    s_acc = 0;
    s_status = 0;
  }
  gs_sync<T>();
  double C[12];
#pragma unroll
  for (int q = 0; q < 12; ++q) C[q] = sC[q];
  for (int j = tid; j < n; j += T)
    triangulate_optimal<true>(C, I34, plx[j], ply[j], prx[j], pry[j], X + 3 * j);
  gs_sync<T>();

  bool relinearize = true;
  for (;;) {
    if (relinearize) {
      // ---- linearisation at (C, X): U (78), gc (12), cost; W, V, gx per point ----
      double acc[91];
#pragma unroll
      for (int k = 0; k < 91; ++k) acc[k] = 0.0;
      for (int j = tid; j < n; j += T) {
        double r[4], a0[12], a1[12], Bj[12];
        gs_point(C, X + 3 * j, plx[j], ply[j], prx[j], pry[j], r, a0, a1, Bj);
#pragma unroll
        for (int p = 0; p < 12; ++p)
#pragma unroll
          for (int q = p; q < 12; ++q) acc[up12(p, q)] += a0[p] * a0[q] + a1[p] * a1[q];
#pragma unroll
        for (int p = 0; p < 12; ++p) acc[78 + p] += a0[p] * r[0] + a1[p] * r[1];
        acc[90] += r[0] * r[0] + r[1] * r[1] + r[2] * r[2] + r[3] * r[3];
        double *w = W + kPerPt * j;
#pragma unroll
        for (int p = 0; p < 12; ++p)
#pragma unroll
          for (int k = 0; k < 3; ++k) w[3 * p + k] = a0[p] * Bj[k] + a1[p] * Bj[3 + k];
        int q = 36;
#pragma unroll
        for (int k = 0; k < 3; ++k)
#pragma unroll
          for (int l = k; l < 3; ++l)
            w[q++] = Bj[k] * Bj[l] + Bj[3 + k] * Bj[3 + l] + Bj[6 + k] * Bj[6 + l] +
                     Bj[9 + k] * Bj[9 + l];
#pragma unroll
        for (int k = 0; k < 3; ++k)
          w[42 + k] = Bj[k] * r[0] + Bj[3 + k] * r[1] + Bj[6 + k] * r[2] + Bj[9 + k] * r[3];
      }
      gs_reduce<91, T>(acc, red, tr, sLin, n);
      if (tid == 0) {
        s_cost = 0.5 * sLin[90];
        if (s_it == 0) s_cost0 = s_cost;
        s_it += 1;
      }
      gs_sync<T>();
      relinearize = false;
    }
    const double lam = s_lam;
    // ---- Schur complement on the camera block ----
    {
      double acc[90];
#pragma unroll
      for (int k = 0; k < 90; ++k) acc[k] = 0.0;
      for (int j = tid; j < n; j += T) {
        const double *w = W + kPerPt * j;
        double Vi[6];
        inv_sym3(w + 36, lam, Vi);
        double wv[12][3];
#pragma unroll
        for (int p = 0; p < 12; ++p) symv3(Vi, w + 3 * p, wv[p]);
#pragma unroll
        for (int p = 0; p < 12; ++p) {
#pragma unroll
          for (int q = p; q < 12; ++q)
            acc[up12(p, q)] += wv[p][0] * w[3 * q] + wv[p][1] * w[3 * q + 1] + wv[p][2] * w[3 * q + 2];
          acc[78 + p] += wv[p][0] * w[42] + wv[p][1] * w[43] + wv[p][2] * w[44];
        }
      }
      gs_reduce<90, T>(acc, red, tr, sres, n);
    }
    if (tid == 0) {
      // S = U + lam diag(U) - sum W Vi W^T;  rhs = -gc + sum W Vi gx;  Cholesky.  Fully
      // unrolled over a register copy of S (lower triangle, 78 doubles): the loop-carried
      // dependences are then FMA latencies, not LDS round trips.
      double L[78], y[12];
#pragma unroll
      for (int p = 0; p < 12; ++p)
#pragma unroll
        for (int q = 0; q <= p; ++q) {
          double v = sU[up12(q, p)] - sres[up12(q, p)];
          if (p == q) v += lam * sU[up12(p, p)];
          L[p * (p + 1) / 2 + q] = v;
        }
#pragma unroll
      for (int p = 0; p < 12; ++p) y[p] = -sgc[p] + sres[78 + p];
      bool ok = true;
      double dinv[12];
#pragma unroll
      for (int k = 0; k < 12; ++k) {
        double d = L[k * (k + 1) / 2 + k];
#pragma unroll
        for (int m = 0; m < k; ++m) d -= L[k * (k + 1) / 2 + m] * L[k * (k + 1) / 2 + m];
        ok = ok && d > 0.0;
        d = sqrt(d > 0.0 ? d : 1.0);
        dinv[k] = 1.0 / d;
        L[k * (k + 1) / 2 + k] = d;
#pragma unroll
        for (int i = k + 1; i < 12; ++i) {
          double v = L[i * (i + 1) / 2 + k];
#pragma unroll
          for (int m = 0; m < k; ++m) v -= L[i * (i + 1) / 2 + m] * L[k * (k + 1) / 2 + m];
          L[i * (i + 1) / 2 + k] = v * dinv[k];
        }
      }
#pragma unroll
      for (int i = 0; i < 12; ++i) {
        double v = y[i];
#pragma unroll
        for (int m = 0; m < i; ++m) v -= L[i * (i + 1) / 2 + m] * y[m];
        y[i] = v * dinv[i];
      }
#pragma unroll
      for (int i = 11; i >= 0; --i) {
        double v = y[i];
#pragma unroll
        for (int m = i + 1; m < 12; ++m) v -= L[m * (m + 1) / 2 + i] * y[m];
        y[i] = v * dinv[i];
      }
#pragma unroll
      for (int p = 0; p < 12; ++p) sdc[p] = ok ? y[p] : 0.0;
      s_state = ok ? 0 : 1;
    }
    gs_sync<T>();
    bool accepted = false, stop = false;
    if (s_state == 0) {
      // ---- point steps, candidate cost, predicted reduction, step / parameter norms ----
      double dc[12], Cn[12];
#pragma unroll
      for (int p = 0; p < 12; ++p) {
        dc[p] = sdc[p];
        Cn[p] = C[p] + dc[p];
      }
      double acc[4] = {0.0, 0.0, 0.0, 0.0};  // cost_n*2, x-part of pred*2, |dx|^2, |X|^2
      for (int j = tid; j < n; j += T) {
        const double *w = W + kPerPt * j;
        double Vi[6];
        inv_sym3(w + 36, lam, Vi);
        double g[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          double v = -w[42 + k];
#pragma unroll
          for (int p = 0; p < 12; ++p) v -= w[3 * p + k] * dc[p];
          g[k] = v;
        }
        double dx[3];
        symv3(Vi, g, dx);
        const double *x = X + 3 * j;
        double xn[3] = {x[0] + dx[0], x[1] + dx[1], x[2] + dx[2]};
        XN[3 * j + 0] = xn[0];
        XN[3 * j + 1] = xn[1];
        XN[3 * j + 2] = xn[2];
        acc[0] += gs_cost_point(Cn, xn, plx[j], ply[j], prx[j], pry[j]);
        const double dv0 = w[36], dv1 = w[39], dv2 = w[41];
        acc[1] += lam * (dx[0] * dv0 * dx[0] + dx[1] * dv1 * dx[1] + dx[2] * dv2 * dx[2]) -
                  (dx[0] * w[42] + dx[1] * w[43] + dx[2] * w[44]);
        acc[2] += dx[0] * dx[0] + dx[1] * dx[1] + dx[2] * dx[2];
        acc[3] += x[0] * x[0] + x[1] * x[1] + x[2] * x[2];
      }
      gs_reduce<4, T>(acc, red, tr, sres, n);
      if (tid == 0) {
        double pc = 0.0, dn = 0.0, cn = 0.0;
        for (int p = 0; p < 12; ++p) {
          pc += lam * dc[p] * sU[up12(p, p)] * dc[p] - dc[p] * sgc[p];
          dn += dc[p] * dc[p];
          cn += C[p] * C[p];
        }
        const double pred = 0.5 * (pc + sres[1]);
        const double cost_n = 0.5 * sres[0];
        const double cost = s_cost;
        const double rho = pred > 0.0 ? (cost - cost_n) / pred : -1.0;
        if (cost_n < cost && rho > 0.0) {
          const bool small_f = (cost - cost_n) <= 1e-15 * cost;
          const bool small_x = sqrt(dn + sres[2]) <= 1e-15 * (sqrt(cn + sres[3]) + 1e-15);
          s_state = (small_f || small_x) ? 3 : 2;
          s_acc += 1;
          s_cost = cost_n;
          const double t = 2.0 * rho - 1.0;
          const double f = 1.0 - t * t * t;
          s_lam = lam * (f > 1.0 / 3.0 ? f : 1.0 / 3.0);
          s_nu = 2.0;
          if (s_state == 3) s_status = 1;
        } else {
          s_state = 1;
          // rejected with a predicted decrease at the rounding level of the cost: more damping
          // only shrinks the step, so this is the minimum (parameters unchanged).  Stops the
          // ~15 rejections the lam > 1e32 exit would otherwise spend (status 2 either way).
          if (pred >= 0.0 && pred <= 1e-15 * cost) s_status = 2;
        }
      }
      gs_sync<T>();
    }
    if (s_state >= 2) {
      accepted = true;
      stop = s_state == 3;
#pragma unroll
      for (int p = 0; p < 12; ++p) C[p] += sdc[p];
      for (int j = tid; j < n; j += T) {
        X[3 * j + 0] = XN[3 * j + 0];
        X[3 * j + 1] = XN[3 * j + 1];
        X[3 * j + 2] = XN[3 * j + 2];
      }
    } else {  // rejected (or S not positive definite): more damping
      if (tid == 0) {
        s_lam = lam * s_nu;
        s_nu *= 2.0;
        if (s_lam > 1e32) s_status = 2;
      }
    }
    gs_sync<T>();
    if (stop || s_status == 2) break;
    if (accepted) {
      if (s_it >= max_iter) break;
      relinearize = true;
    }
  }
  if (tid == 0) {
    double f[9];
    fmatrix_from_cameras(C, I34, f);
    for (int q = 0; q < 9; ++q) Fout[9 * blockIdx.x + q] = f[q];
    if (C1out)
      for (int q = 0; q < 12; ++q) C1out[12 * blockIdx.x + q] = C[q];
    GsInfo g;
    g.cost_init = s_cost0;
    g.cost = s_cost;
    g.iterations = s_it;
    g.accepted = s_acc;
    g.status = s_status;
    g.n = n;
    info[blockIdx.x] = g;
  }
}

// Workgroup (T threads) per pair; a pair of at most 64 inliers runs on the first wave alone
// (wave-level reductions and fences, the other waves leave at once): the C4 pairs that bound
// the launch are small ones with many LM iterations, where the workgroup barriers and the
// cross-wave sums were most of an iteration
template <int T>
__global__ __launch_bounds__(T) void k_gold_standard(
    const double *__restrict__ Fin, const double *__restrict__ pl, const double *__restrict__ pr,
    int64_t total, const int64_t *__restrict__ off, int max_iter, double *__restrict__ Xb,
    double *__restrict__ Xc, double *__restrict__ Wb, double *__restrict__ Fout,
    double *__restrict__ C1out, GsInfo *__restrict__ info, const int32_t *__restrict__ act) {
  __shared__ double trbuf[RSAMD_GS_TR ? 64 * 91 : 1];  // wave_reduce_tr's rows
  const int tid = threadIdx.x;
  if (act && !act[blockIdx.x]) {  // (rs_pairs_two_view: a pair without a consensus)
    if (tid < 9) Fout[9 * blockIdx.x + tid] = __builtin_nan("");
    if (tid == 0) info[blockIdx.x] = GsInfo{0.0, 0.0, 0, 0, 0, 0};
    return;
  }
  if constexpr (T > 64 && RSAMD_GS_WAVE) {
    if (off[blockIdx.x + 1] - off[blockIdx.x] <= RSAMD_GS_WAVE_MAX) {
      if (tid >= 64) return;
      gs_pair<64>(Fin, pl, pr, total, off, max_iter, Xb, Xc, Wb, Fout, C1out, info, trbuf);
      return;
    }
  }
  gs_pair<T>(Fin, pl, pr, total, off, max_iter, Xb, Xc, Wb, Fout, C1out, info, trbuf);
}

// ---- rs_pairs_two_view: the pair records -> the gold standard, on the device ----------------
// (parallel._pairs_arrays' host steps between rs_pairs_f8_ransac and rs_gold_standard)
struct PairRec {  // == rs_pair_result
  double F[9];
  int64_t best_index, best_count;
  double best_std, best_norm;
  int64_t n_candidates;
};

// Which pairs refine (a consensus: best_index >= 0 and best_count > 0), where their inliers go
// in the gathered arrays (goff: exclusive scan of the counts in pair order, goff[B] = total)
// and F_RANSAC in the gold standard's (B, 9) layout.  One workgroup, 1 024 pairs a round.
__global__ __launch_bounds__(1024) void k_twoview_prep(const PairRec *__restrict__ res, int64_t B,
                                                       int64_t *__restrict__ goff,
                                                       int32_t *__restrict__ act,
                                                       double *__restrict__ Fin) {
  __shared__ long long sw[16];
  __shared__ long long s_carry;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (tid == 0) s_carry = 0;
  __syncthreads();
  for (int64_t b0 = 0; b0 < B; b0 += 1024) {
    const int64_t b = b0 + tid;
    long long v = 0;
    if (b < B) {
      const PairRec &r = res[b];
      const bool a = r.best_index >= 0 && r.best_count > 0;
      act[b] = a ? 1 : 0;
      v = a ? r.best_count : 0;
#pragma unroll
      for (int q = 0; q < 9; ++q) Fin[9 * b + q] = r.F[q];
    }
    long long x = v;  // inclusive wave scan
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const long long y = __shfl_up(x, d);
      if (lane >= d) x += y;
    }
    if (lane == 63) sw[w] = x;
    __syncthreads();
    long long pre = s_carry, tot = 0;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      pre += q < w ? sw[q] : 0;
      tot += sw[q];
    }
    if (b < B) goff[b] = pre + x - v;
    __syncthreads();
    if (tid == 0) s_carry += tot;
    __syncthreads();
  }
  if (tid == 0) goff[B] = s_carry;
}

// The refining pairs' inlier points, gathered in S_RANSAC order into the gold standard's
// (2, tp) arrays (row stride tp >= goff[B]): a wave per pair.
__global__ __launch_bounds__(64) void k_twoview_gather(const Pt *__restrict__ pts,
                                                       const int64_t *__restrict__ off,
                                                       const int32_t *__restrict__ inl,
                                                       const int64_t *__restrict__ goff,
                                                       const int32_t *__restrict__ act, int64_t tp,
                                                       double *__restrict__ pl,
                                                       double *__restrict__ pr) {
  const int64_t b = blockIdx.x;
  if (!act[b]) return;
  const int64_t o = off[b], g = goff[b], k = goff[b + 1] - g;
  for (int64_t j = threadIdx.x; j < k; j += 64) {
    const Pt P = pts[o + inl[o + j]];
    pl[g + j] = P.x1;
    pl[tp + g + j] = P.y1;
    pr[g + j] = P.x2;
    pr[tp + g + j] = P.y2;
  }
}

}  // namespace rsd

// ------------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------------
using rs::fail;
using rs::hip_fail;

#define HIP_TRY(expr)                                 \
  do {                                                \
    hipError_t e_ = (expr);                           \
    if (e_ != hipSuccess) return hip_fail(e_, #expr); \
  } while (0)

namespace {

size_t al(size_t b) { return (b + 255) / 256 * 256; }

// Carve `count` device buffers of the given byte sizes out of the context scratch.
int carve(rs_ctx *c, std::initializer_list<size_t> sizes, std::vector<char *> &out) {
  size_t tot = 0;
  for (size_t s : sizes) tot += al(s);
  int st = rs::ensure_scratch(c, tot + 256);
  if (st) return st;
  char *p = static_cast<char *>(c->scratch);
  out.clear();
  for (size_t s : sizes) {
    out.push_back(p);
    p += al(s);
  }
  return RS_OK;
}

int grid(int64_t n) { return static_cast<int>((n + 127) / 128); }

}  // namespace

static_assert(sizeof(rsd::GsInfo) == sizeof(rs_gs_info), "rs_gs_info layout");

extern "C" int rs_triangulate_optimal(rs_ctx *c, const double *C1, const double *C2,
                                      int64_t n_cam, const double *x1, const double *x2,
                                      const int32_t *cam, int64_t n, double *X_out) {
  if (!c || !C1 || !C2 || !x1 || !x2 || !X_out) return fail(RS_EINVAL, "null pointer");
  if (n_cam < 1) return fail(RS_EINVAL, "need at least one camera pair");
  if (n < 0 || n > (1LL << 28)) return fail(RS_EINVAL, "bad point count");
  if (n == 0) return RS_OK;
  if (cam)
    for (int64_t i = 0; i < n; ++i)
      if (cam[i] < 0 || cam[i] >= n_cam) return fail(RS_EINVAL, "camera index out of range");
  HIP_TRY(hipSetDevice(c->device));
  std::vector<char *> b;
  const size_t bc = sizeof(double) * 12 * n_cam, bx = sizeof(double) * 2 * n;
  int st = carve(c, {bc, bc, bx, bx, cam ? sizeof(int32_t) * n : 0, sizeof(double) * 3 * n}, b);
  if (st) return st;
  HIP_TRY(hipMemcpyAsync(b[0], C1, bc, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(b[1], C2, bc, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(b[2], x1, bx, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(b[3], x2, bx, hipMemcpyHostToDevice, c->stream));
  if (cam) HIP_TRY(hipMemcpyAsync(b[4], cam, sizeof(int32_t) * n, hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(rsd::k_triangulate_optimal, dim3(grid(n)), dim3(128), 0, c->stream,
                     reinterpret_cast<double *>(b[0]), reinterpret_cast<double *>(b[1]),
                     reinterpret_cast<double *>(b[2]), reinterpret_cast<double *>(b[3]),
                     cam ? reinterpret_cast<int32_t *>(b[4]) : nullptr, n,
                     reinterpret_cast<double *>(b[5]));
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(X_out, b[5], sizeof(double) * 3 * n, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return RS_OK;
}

extern "C" int rs_camera_resectioning(rs_ctx *c, const double *P, int64_t B, double *K,
                                      double *R, double *t) {
  if (!c || !P || !K || !R || !t) return fail(RS_EINVAL, "null pointer");
  if (B < 0 || B > (1LL << 26)) return fail(RS_EINVAL, "bad camera count");
  if (B == 0) return RS_OK;
  HIP_TRY(hipSetDevice(c->device));
  std::vector<char *> b;
  int st = carve(c, {sizeof(double) * 12 * B, sizeof(double) * 9 * B, sizeof(double) * 9 * B,
                     sizeof(double) * 3 * B}, b);
  if (st) return st;
  HIP_TRY(hipMemcpyAsync(b[0], P, sizeof(double) * 12 * B, hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(rsd::k_resection, dim3(grid(B)), dim3(128), 0, c->stream,
                     reinterpret_cast<double *>(b[0]), B, reinterpret_cast<double *>(b[1]),
                     reinterpret_cast<double *>(b[2]), reinterpret_cast<double *>(b[3]));
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(K, b[1], sizeof(double) * 9 * B, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(R, b[2], sizeof(double) * 9 * B, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(t, b[3], sizeof(double) * 3 * B, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return RS_OK;
}

extern "C" int rs_essential_from_f(rs_ctx *c, const double *K, int32_t one_k, const double *F,
                                   int64_t B, double *E) {
  if (!c || !K || !F || !E) return fail(RS_EINVAL, "null pointer");
  if (B < 0 || B > (1LL << 26)) return fail(RS_EINVAL, "bad batch size");
  if (B == 0) return RS_OK;
  HIP_TRY(hipSetDevice(c->device));
  const int64_t nk = one_k ? 1 : B;
  std::vector<char *> b;
  int st = carve(c, {sizeof(double) * 9 * nk, sizeof(double) * 9 * B, sizeof(double) * 9 * B}, b);
  if (st) return st;
  HIP_TRY(hipMemcpyAsync(b[0], K, sizeof(double) * 9 * nk, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(b[1], F, sizeof(double) * 9 * B, hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(rsd::k_essential, dim3(grid(B)), dim3(128), 0, c->stream,
                     reinterpret_cast<double *>(b[0]), one_k ? 0 : 9,
                     reinterpret_cast<double *>(b[1]), B, reinterpret_cast<double *>(b[2]));
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(E, b[2], sizeof(double) * 9 * B, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return RS_OK;
}

extern "C" int rs_relative_camera_pose(rs_ctx *c, const double *E, const double *y1,
                                       const double *y2, int64_t B, double *R, double *t,
                                       int32_t *found) {
  if (!c || !E || !y1 || !y2 || !R || !t || !found) return fail(RS_EINVAL, "null pointer");
  if (B < 0 || B > (1LL << 26)) return fail(RS_EINVAL, "bad batch size");
  if (B == 0) return RS_OK;
  HIP_TRY(hipSetDevice(c->device));
  std::vector<char *> b;
  int st = carve(c, {sizeof(double) * 9 * B, sizeof(double) * 2 * B, sizeof(double) * 2 * B,
                     sizeof(double) * 9 * B, sizeof(double) * 3 * B, sizeof(int32_t) * B}, b);
  if (st) return st;
  HIP_TRY(hipMemcpyAsync(b[0], E, sizeof(double) * 9 * B, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(b[1], y1, sizeof(double) * 2 * B, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(b[2], y2, sizeof(double) * 2 * B, hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(rsd::k_relative_pose, dim3(grid(4 * B)), dim3(128), 0, c->stream,
                     reinterpret_cast<double *>(b[0]), reinterpret_cast<double *>(b[1]),
                     reinterpret_cast<double *>(b[2]), B, reinterpret_cast<double *>(b[3]),
                     reinterpret_cast<double *>(b[4]), reinterpret_cast<int32_t *>(b[5]));
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(R, b[3], sizeof(double) * 9 * B, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(t, b[4], sizeof(double) * 3 * B, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(found, b[5], sizeof(int32_t) * B, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return RS_OK;
}

extern "C" int rs_fmatrix_cameras(rs_ctx *c, const double *F, int64_t B, double *C1) {
  if (!c || !F || !C1) return fail(RS_EINVAL, "null pointer");
  if (B < 0 || B > (1LL << 26)) return fail(RS_EINVAL, "bad batch size");
  if (B == 0) return RS_OK;
  HIP_TRY(hipSetDevice(c->device));
  std::vector<char *> b;
  int st = carve(c, {sizeof(double) * 9 * B, sizeof(double) * 12 * B}, b);
  if (st) return st;
  HIP_TRY(hipMemcpyAsync(b[0], F, sizeof(double) * 9 * B, hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(rsd::k_fmatrix_cameras, dim3(grid(B)), dim3(128), 0, c->stream,
                     reinterpret_cast<double *>(b[0]), B, reinterpret_cast<double *>(b[1]));
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(C1, b[1], sizeof(double) * 12 * B, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return RS_OK;
}

extern "C" int rs_fmatrix_from_cameras(rs_ctx *c, const double *C1, const double *C2, int64_t B,
                                       double *F) {
  if (!c || !C1 || !C2 || !F) return fail(RS_EINVAL, "null pointer");
  if (B < 0 || B > (1LL << 26)) return fail(RS_EINVAL, "bad batch size");
  if (B == 0) return RS_OK;
  HIP_TRY(hipSetDevice(c->device));
  std::vector<char *> b;
  int st = carve(c, {sizeof(double) * 12 * B, sizeof(double) * 12 * B, sizeof(double) * 9 * B}, b);
  if (st) return st;
  HIP_TRY(hipMemcpyAsync(b[0], C1, sizeof(double) * 12 * B, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(b[1], C2, sizeof(double) * 12 * B, hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(rsd::k_fmatrix_from_cameras, dim3(grid(B)), dim3(128), 0, c->stream,
                     reinterpret_cast<double *>(b[0]), reinterpret_cast<double *>(b[1]), B,
                     reinterpret_cast<double *>(b[2]));
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(F, b[2], sizeof(double) * 9 * B, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return RS_OK;
}

extern "C" int rs_gold_standard(rs_ctx *c, const double *F, const double *pl, const double *pr,
                                const int64_t *off, int64_t B, int32_t max_iter, double *F_gold,
                                double *C1_out, double *X_out, rs_gs_info *info) {
  if (!c || !F || !off || !F_gold || !info) return fail(RS_EINVAL, "null pointer");
  if (B < 1 || B > (1 << 24)) return fail(RS_EINVAL, "bad pair count");
  if (off[0] != 0) return fail(RS_EINVAL, "offsets must start at 0");
  for (int64_t b = 0; b < B; ++b)
    if (off[b + 1] < off[b] || off[b + 1] - off[b] > (1 << 24))
      return fail(RS_EINVAL, "offsets must be non-decreasing");
  const int64_t total = off[B];
  if (total > 0 && (!pl || !pr)) return fail(RS_EINVAL, "null point arrays");
  if (max_iter < 1 || max_iter > 100000) return fail(RS_EINVAL, "max_iter must be in [1, 1e5]");
  HIP_TRY(hipSetDevice(c->device));
  const int64_t tp = total > 0 ? total : 1;
  std::vector<char *> b;
  int st = carve(c, {sizeof(double) * 9 * B, sizeof(double) * 2 * tp, sizeof(double) * 2 * tp,
                     sizeof(int64_t) * (B + 1), sizeof(double) * 3 * tp, sizeof(double) * 3 * tp,
                     sizeof(double) * rsd::kPerPt * tp, sizeof(double) * 9 * B,
                     sizeof(double) * 12 * B, sizeof(rs_gs_info) * B}, b);
  if (st) return st;
  HIP_TRY(hipMemcpyAsync(b[0], F, sizeof(double) * 9 * B, hipMemcpyHostToDevice, c->stream));
  if (total > 0) {
    HIP_TRY(hipMemcpyAsync(b[1], pl, sizeof(double) * 2 * total, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(b[2], pr, sizeof(double) * 2 * total, hipMemcpyHostToDevice, c->stream));
  }
  HIP_TRY(hipMemcpyAsync(b[3], off, sizeof(int64_t) * (B + 1), hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(rsd::k_gold_standard<rsd::kGsT>, dim3(static_cast<unsigned>(B)), dim3(rsd::kGsT), 0,
                     c->stream, reinterpret_cast<double *>(b[0]),
                     reinterpret_cast<double *>(b[1]), reinterpret_cast<double *>(b[2]), tp,
                     reinterpret_cast<int64_t *>(b[3]), max_iter, reinterpret_cast<double *>(b[4]),
                     reinterpret_cast<double *>(b[5]), reinterpret_cast<double *>(b[6]),
                     reinterpret_cast<double *>(b[7]), reinterpret_cast<double *>(b[8]),
                     reinterpret_cast<rsd::GsInfo *>(b[9]), nullptr);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(F_gold, b[7], sizeof(double) * 9 * B, hipMemcpyDeviceToHost, c->stream));
  if (C1_out)
    HIP_TRY(hipMemcpyAsync(C1_out, b[8], sizeof(double) * 12 * B, hipMemcpyDeviceToHost, c->stream));
  if (X_out && total > 0)
    HIP_TRY(hipMemcpyAsync(X_out, b[4], sizeof(double) * 3 * total, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(info, b[9], sizeof(rs_gs_info) * B, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return RS_OK;
}

extern "C" int rs_gs_residuals_fd(rs_ctx *c, const double *x, const double *xp, const double *dx,
                                  const double *pl, const double *pr, int64_t n, double *f,
                                  double *J) {
  if (!c || !x || !pl || !pr || !f || (J && (!xp || !dx))) return fail(RS_EINVAL, "null pointer");
  if (n < 1 || n > (1LL << 20)) return fail(RS_EINVAL, "Wrong size of parameter vector");
  HIP_TRY(hipSetDevice(c->device));
  const int64_t np = 12 + 3 * n, nr = 4 * n;
  const size_t jb = J ? sizeof(double) * static_cast<size_t>(nr) * np : 0;
  std::vector<char *> b;
  int st = carve(c, {sizeof(double) * np, J ? sizeof(double) * np : 0, J ? sizeof(double) * np : 0,
                     sizeof(double) * 2 * n, sizeof(double) * 2 * n, sizeof(double) * nr, jb},
                 b);
  if (st) return st;
  HIP_TRY(hipMemcpyAsync(b[0], x, sizeof(double) * np, hipMemcpyHostToDevice, c->stream));
  if (J) {
    HIP_TRY(hipMemcpyAsync(b[1], xp, sizeof(double) * np, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(b[2], dx, sizeof(double) * np, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemsetAsync(b[6], 0, jb, c->stream));
  }
  HIP_TRY(hipMemcpyAsync(b[3], pl, sizeof(double) * 2 * n, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(b[4], pr, sizeof(double) * 2 * n, hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(rsd::k_gs_fd, dim3(static_cast<unsigned>((n + 127) / 128)), dim3(128), 0,
                     c->stream, reinterpret_cast<double *>(b[0]), reinterpret_cast<double *>(b[1]),
                     reinterpret_cast<double *>(b[2]), reinterpret_cast<double *>(b[3]),
                     reinterpret_cast<double *>(b[4]), n, reinterpret_cast<double *>(b[5]),
                     J ? reinterpret_cast<double *>(b[6]) : nullptr);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(f, b[5], sizeof(double) * nr, hipMemcpyDeviceToHost, c->stream));
  if (J) HIP_TRY(hipMemcpyAsync(J, b[6], jb, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return RS_OK;
}

static_assert(sizeof(rsd::PairRec) == sizeof(rs_pair_result), "rs_pair_result layout");

extern "C" int rs_pairs_two_view(rs_ctx *c, const double *p1, const double *p2, const int64_t *off,
                                 int64_t B, int64_t H, int32_t mode, uint64_t seed_base,
                                 const int64_t *seed_ids, const int32_t *host_tuples,
                                 double thresh, int32_t max_iter, const double *K,
                                 const double *y1, const double *y2, rs_pair_result *out,
                                 int32_t *inliers, double *F_gold, rs_gs_info *info, double *R,
                                 double *t, int32_t *found) {
  if (!out || !inliers || !F_gold || !info || !R || !t || !found)
    return fail(RS_EINVAL, "null pointer");
  if (K && (!y1 || !y2)) return fail(RS_EINVAL, "K needs y1 and y2");
  if (max_iter < 1 || max_iter > 100000) return fail(RS_EINVAL, "max_iter must be in [1, 1e5]");
  if (!off || B < 1 || B > (1 << 20)) return fail(RS_EINVAL, "bad pair count");
  // the offsets size this call's buffers (tp): validated before use (pairs_enqueue checks them
  // again for its own callers)
  if (off[0] != 0) return fail(RS_EINVAL, "offsets must start at 0");
  for (int64_t b = 0; b < B; ++b)
    if (off[b + 1] < off[b] || off[b + 1] - off[b] > (1 << 24))
      return fail(RS_EINVAL, "offsets must be non-decreasing");
  const int64_t tp = off[B] > 0 ? off[B] : 1;
  // the stages' buffers after the pair RANSAC's, then the output block (one download)
  const size_t sz[] = {sizeof(int64_t) * (B + 1), sizeof(int32_t) * B, sizeof(double) * 9 * B,
                       sizeof(double) * 2 * tp,   sizeof(double) * 2 * tp,
                       sizeof(double) * 3 * tp,   sizeof(double) * 3 * tp,
                       sizeof(double) * rsd::kPerPt * tp, sizeof(double) * 9,
                       sizeof(double) * 2 * B,    sizeof(double) * 2 * B, sizeof(double) * 9 * B};
  const size_t osz[] = {sizeof(double) * 9 * B, sizeof(rs_gs_info) * B, sizeof(double) * 9 * B,
                        sizeof(double) * 3 * B, sizeof(int32_t) * B};
  size_t extra = 0, oblk = 0;
  for (size_t x : sz) extra += al(x);
  for (size_t x : osz) oblk += al(x);
  rs::PairsDev d{};
  int st = rs::pairs_enqueue(c, p1, p2, off, B, H, mode, seed_base, seed_ids, host_tuples,
                             thresh, extra + oblk, &d);
  if (st) return st;
  std::vector<char *> b;
  char *p = d.extra;
  for (size_t x : sz) {
    b.push_back(p);
    p += al(x);
  }
  char *ob = p;
  std::vector<char *> o;
  for (size_t x : osz) {
    o.push_back(p);
    p += al(x);
  }
  auto *goff = reinterpret_cast<int64_t *>(b[0]);
  auto *act = reinterpret_cast<int32_t *>(b[1]);
  auto *Fin = reinterpret_cast<double *>(b[2]);
  auto *pl = reinterpret_cast<double *>(b[3]), *pr = reinterpret_cast<double *>(b[4]);
  auto *dK = reinterpret_cast<double *>(b[8]);
  auto *dy1 = reinterpret_cast<double *>(b[9]), *dy2 = reinterpret_cast<double *>(b[10]);
  auto *dE = reinterpret_cast<double *>(b[11]);
  auto *dFg = reinterpret_cast<double *>(o[0]);
  auto *dinfo = reinterpret_cast<rsd::GsInfo *>(o[1]);
  auto *dR = reinterpret_cast<double *>(o[2]), *dt = reinterpret_cast<double *>(o[3]);
  auto *dfound = reinterpret_cast<int32_t *>(o[4]);
  hipStream_t s = c->stream;
  if (K) {
    HIP_TRY(hipMemcpyAsync(dK, K, sizeof(double) * 9, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(dy1, y1, sizeof(double) * 2 * B, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(dy2, y2, sizeof(double) * 2 * B, hipMemcpyHostToDevice, s));
  }
  hipLaunchKernelGGL(rsd::k_twoview_prep, dim3(1), dim3(1024), 0, s,
                     static_cast<const rsd::PairRec *>(d.res), B, goff, act, Fin);
  hipLaunchKernelGGL(rsd::k_twoview_gather, dim3(static_cast<unsigned>(B)), dim3(64), 0, s,
                     static_cast<const rsd::Pt *>(d.pts), d.off, d.inl, goff, act, tp, pl, pr);
  hipLaunchKernelGGL(rsd::k_gold_standard<rsd::kGsT>, dim3(static_cast<unsigned>(B)), dim3(rsd::kGsT),
                     0, s, Fin, pl, pr, tp, goff, max_iter, reinterpret_cast<double *>(b[5]),
                     reinterpret_cast<double *>(b[6]), reinterpret_cast<double *>(b[7]), dFg,
                     nullptr, dinfo, act);
  if (K) {
    hipLaunchKernelGGL(rsd::k_essential, dim3(grid(B)), dim3(128), 0, s, dK, 0, dFg, B, dE);
    hipLaunchKernelGGL(rsd::k_relative_pose, dim3(grid(4 * B)), dim3(128), 0, s, dE, dy1, dy2, B,
                       dR, dt, dfound, act);
  }
  HIP_TRY(hipGetLastError());
  std::vector<char> host(static_cast<size_t>(p - ob));
  HIP_TRY(hipMemcpyAsync(out, d.res, sizeof(rs_pair_result) * B, hipMemcpyDeviceToHost, s));
  if (d.total > 0)
    HIP_TRY(hipMemcpyAsync(inliers, d.inl, sizeof(int32_t) * d.total, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(host.data(), ob, host.size(), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  std::memcpy(F_gold, host.data() + (o[0] - ob), osz[0]);
  std::memcpy(info, host.data() + (o[1] - ob), osz[1]);
  if (K) {
    std::memcpy(R, host.data() + (o[2] - ob), osz[2]);
    std::memcpy(t, host.data() + (o[3] - ob), osz[3]);
    std::memcpy(found, host.data() + (o[4] - ob), osz[4]);
  } else {
    for (int64_t i = 0; i < 9 * B; ++i) R[i] = __builtin_nan("");
    for (int64_t i = 0; i < 3 * B; ++i) t[i] = __builtin_nan("");
    std::memset(found, 0, sizeof(int32_t) * B);
  }
  return RS_OK;
}
