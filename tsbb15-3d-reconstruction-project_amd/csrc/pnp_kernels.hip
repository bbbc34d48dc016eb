// PnP-RANSAC with the algebraic DLT of pnp.py:132-160, consensus of ransac.py:93-111.
//
//   k_pnp_solve   lane per hypothesis: sample k >= 6 points of the `high` set (Philox/Floyd or
//                 host tuples from rs_py_shuffle_tuples), stream the 2k DLT rows
//                 vec(r_l x^T) (rows 0,1 of [y]_x) through Givens rotations into a 12x12
//                 upper-triangular R (78 doubles in VGPRs), smallest right singular vector by
//                 inverse iteration on R^T R, C0 = (A|b), tau = sign det A, polar factor of
//                 tau A by 3x3 Jacobi SVD, lambda = 3 tau / tr S, t = lambda b.
//   k_pnp_count   lane per hypothesis x chunk of `med` points (wave-uniform scalar loads):
//                 e = |pi(y) - pi(R x + t)|^2 <= thresh, evaluated division-free; pairs within
//                 a rigorous error band of the threshold re-tested in the reference's order.
//   k_pnp_select  one workgroup: first hypothesis with the largest count (strict ">"); for the
//                 P3P branch a mirrored-depth pose only where it clearly out-counts (x2) every
//                 front-facing one.
//   k_pnp_inliers consensus sets of the winner on `med` and `high` (reference order).
//
// The cv.solvePnPRansac drop-in (rs_pnp_ransac_cv) reuses solve / count with the test in
// PIXELS: the residual pi(y) - pi(R x + t) in C-normalised units is mapped through the upper
// 2x2 block of K, [[fx, s], [0, fy]] (K is affine on the image plane, so this IS the pixel
// reprojection error K pi(R x + t) - uv), and compared with reprojectionError^2.  The
// reference-mode metric is the identity (a, b, c) = (1, 0, 1), which leaves its arithmetic
// bit-unchanged.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <vector>

#include "common.h"
#include "ctx.h"
#include "device_math.h"
#include "f8_kernels.h"

namespace rsd {

// A 3D<->2D correspondence: world point (X, Y, Z) and pi(y) = (y0/y2, y1/y2).
struct PPt {
  double X, Y, Z, u, v, y0, y1, y2;
};

// Pixel metric: residual (du, dv) -> (a du + b dv, c dv).
struct PxMetric {
  double a, b, c;
};

}  // namespace rsd

#include "pnp_minimal.h"

namespace rsd {

constexpr int ridx(int j, int l) { return j * 12 - (j * (j - 1)) / 2 + (l - j); }


__device__ __forceinline__ void givens_row(double (&R)[78], double (&a)[12]) {
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    // rho = |(r, a_j)|, c = r / rho, s = a_j / rho from one reciprocal square root (a few ulp;
    // the DLT's parity bar is 1e-6 on R, t) instead of a correctly rounded sqrt and divide
    const double r = R[ridx(j, j)];
    const double q = fma(r, r, a[j] * a[j]);
    const bool live = q > 0.0;
    const double inv = live ? rsqrt_fast(live ? q : 1.0) : 0.0;
    const double c = live ? r * inv : 1.0;
    const double s = a[j] * inv;
    R[ridx(j, j)] = live ? q * inv : 0.0;
#pragma unroll
    for (int l = j + 1; l < 12; ++l) {
      const double rl = R[ridx(j, l)];
      R[ridx(j, l)] = fma(c, rl, s * a[l]);
      a[l] = fma(c, a[l], -s * rl);
    }
  }
}

__device__ __forceinline__ void dlt_rows(const PPt &p, double (&a0)[12], double (&a1)[12]) {
  // [y]_x rows 0 and 1 (lab3.cross_matrix): r0 = (0, -y2, y1), r1 = (y2, 0, -y0)
  const double r0[3] = {0.0, -p.y2, p.y1};
  const double r1[3] = {p.y2, 0.0, -p.y0};
  const double xh[4] = {p.X, p.Y, p.Z, 1.0};
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      a0[4 * i + j] = r0[i] * xh[j];
      a1[4 * i + j] = r1[i] * xh[j];
    }
}

// Smallest right singular vector of the matrix whose R factor is given: block inverse
// iteration on R^T R with two vectors and a 2x2 Rayleigh-Ritz step per sweep.  The Ritz
// vector converges at (s12 / s10)^2 per sweep instead of single-vector inverse iteration's
// (s12 / s11)^2, which a noisy minimal sample can hold near 1 (C3 samples, host prototype:
// a wave's slowest lane needs ~17 sweeps instead of ~100; deviation from numpy's SVD
// <= 2.3e-12).  Stops when the Ritz vector moves <= 1e-15.
__device__ __forceinline__ void tri_solve_rt_r(const double (&R)[78], const double (&dinv)[12],
                                               double (&v)[12]) {
#pragma unroll
  for (int j = 0; j < 12; ++j) {  // R^T z = v, in place
    double acc = v[j];
#pragma unroll
    for (int i = 0; i < j; ++i) acc = fma(-R[ridx(i, j)], v[i], acc);
    v[j] = acc * dinv[j];
  }
#pragma unroll
  for (int j = 11; j >= 0; --j) {  // R w = z, in place
    double acc = v[j];
#pragma unroll
    for (int l = j + 1; l < 12; ++l) acc = fma(-R[ridx(j, l)], v[l], acc);
    v[j] = acc * dinv[j];
  }
}

__device__ __forceinline__ double dot12(const double (&a)[12], const double (&b)[12]) {
  double s = 0.0;
#pragma unroll
  for (int j = 0; j < 12; ++j) s = fma(a[j], b[j], s);
  return s;
}

// |R u|^2, (R u).(R v), |R v|^2 for upper-triangular R
__device__ __forceinline__ void r_gram(const double (&R)[78], const double (&u)[12],
                                       const double (&v)[12], double &uu, double &uv,
                                       double &vv) {
  uu = 0.0;
  uv = 0.0;
  vv = 0.0;
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    double ru = 0.0, rv = 0.0;
#pragma unroll
    for (int l = j; l < 12; ++l) {
      ru = fma(R[ridx(j, l)], u[l], ru);
      rv = fma(R[ridx(j, l)], v[l], rv);
    }
    uu = fma(ru, ru, uu);
    uv = fma(ru, rv, uv);
    vv = fma(rv, rv, vv);
  }
}

__device__ __forceinline__ void orthonormalize2(double (&u)[12], double (&v)[12]) {
  const double iu = rsqrt_fast(dot12(u, u));
#pragma unroll
  for (int j = 0; j < 12; ++j) u[j] *= iu;
  const double p = dot12(u, v);
#pragma unroll
  for (int j = 0; j < 12; ++j) v[j] = fma(-p, u[j], v[j]);
  const double iv = rsqrt_fast(dot12(v, v));
#pragma unroll
  for (int j = 0; j < 12; ++j) v[j] *= iv;
}

__device__ __forceinline__ void smallest_right_sv(const double (&R)[78], double (&x)[12]) {
  double dinv[12];
#pragma unroll
  for (int j = 0; j < 12; ++j) dinv[j] = 1.0 / R[ridx(j, j)];
  // start: span(R^-1 e_11, R^-1 e_10)
  double u[12], v[12];
#pragma unroll
  for (int j = 11; j >= 0; --j) {
    double au = (j == 11) ? 1.0 : 0.0, av = (j == 10) ? 1.0 : 0.0;
#pragma unroll
    for (int l = j + 1; l < 12; ++l) {
      au = fma(-R[ridx(j, l)], u[l], au);
      av = fma(-R[ridx(j, l)], v[l], av);
    }
    u[j] = au * dinv[j];
    v[j] = av * dinv[j];
  }
  orthonormalize2(u, v);
#pragma unroll
  for (int j = 0; j < 12; ++j) x[j] = u[j];
  double prev_delta = 1.0;
  for (int it = 0; it < 200; ++it) {
    tri_solve_rt_r(R, dinv, u);
    tri_solve_rt_r(R, dinv, v);
    orthonormalize2(u, v);
    // Rayleigh-Ritz: smallest eigenvector y of G = (R [u v])^T (R [u v])
    double a, b, c;
    r_gram(R, u, v, a, b, c);
    const double hd = 0.5 * (a - c);
    const double lam = 0.5 * (a + c) - sqrt(fma(hd, hd, b * b));
    // (b, lam - a) and (lam - c, b) both span the eigenvector; take the longer
    double y0 = b, y1 = lam - a;
    const double z0 = lam - c, z1 = b;
    if (fma(z0, z0, z1 * z1) > fma(y0, y0, y1 * y1)) {
      y0 = z0;
      y1 = z1;
    }
    const double ny = fma(y0, y0, y1 * y1);
    if (!(ny > 0.0)) {  // G already diagonal: u or v
      y0 = a <= c ? 1.0 : 0.0;
      y1 = a <= c ? 0.0 : 1.0;
    } else {
      const double iy = rsqrt_fast(ny);
      y0 *= iy;
      y1 *= iy;
    }
    double w[12];
#pragma unroll
    for (int j = 0; j < 12; ++j) w[j] = fma(y0, u[j], y1 * v[j]);
    const double sgn = dot12(w, x) < 0.0 ? -1.0 : 1.0;
    double delta = 0.0;
#pragma unroll
    for (int j = 0; j < 12; ++j) {
      const double nv = sgn * w[j];
      delta = fmax(delta, fabs(nv - x[j]));
      x[j] = nv;
    }
    // converged (or NaN: the model scores zero); or at the rounding floor, where the Ritz
    // vector jitters at ~1e-15 instead of settling (it no longer halves its step)
    if (it > 0 && !(delta > 1e-15)) break;
    if (it > 1 && delta < 1e-13 && delta > 0.5 * prev_delta) break;
    prev_delta = delta;
  }
  // unit norm to full precision (a combination of an orthonormal pair, up to rounding)
  const double in = 1.0 / sqrt(dot12(x, x));
#pragma unroll
  for (int j = 0; j < 12; ++j) x[j] *= in;
}

// Three-vector variant (blk_smallest_right_sv3 below, on the block factor): a block of THREE
// vectors and a 3x3 Rayleigh-Ritz step per sweep: the Ritz
// vector converges at (s12 / s9)^2 per sweep.  The kernel's time is its slowest wave's, and a
// wave runs until its slowest lane converges: C3 samples (host prototype, 20 000 DLT samples of
// the C3 scene) need at most 46 sweeps of the two-vector block (mean 6.5, a wave's slowest 17
// on average) but 15 of the three-vector block (mean 4.8, a wave's slowest 8.9), at ~1.35x the
// work per sweep.  The basis is rotated onto the Ritz vectors every sweep (smallest first), so
// the 3x3 Gram matrix arrives nearly diagonal and its Jacobi eigen-solve ends after a sweep or
// two.  Stops when the Ritz vector moves <= 1e-15, or stagnates at the rounding floor.
__device__ __forceinline__ void jacobi_sym3(double (&G)[6], double (&Z)[9], int p, int q,
                                            bool &rotated) {
  // G packed (00, 11, 22, 01, 02, 12); rotate rows / columns p < q, accumulate Z's columns
  const int ipq = p == 0 ? (q == 1 ? 3 : 4) : 5;
  const int r = 3 - p - q;
  const int ipr = (p == 0 ? (r == 1 ? 3 : 4) : (r == 0 ? (p == 1 ? 3 : 4) : 5));
  const int iqr = (q == 1 ? (r == 0 ? 3 : 5) : (r == 0 ? 4 : 5));
  const double gpq = G[ipq], gpp = G[p], gqq = G[q];
  if (gpq * gpq > 1e-32 * fabs(gpp * gqq) && gpq != 0.0) {
    rotated = true;
    const double zeta = (gqq - gpp) * (0.5 * rcp_fast(gpq));
    const double az = fabs(zeta), z2 = fma(zeta, zeta, 1.0);
    const double t = az < 1e150 ? copysign(rcp_fast(az + z2 * rsqrt_fast(z2)), zeta)
                                : 0.5 * rcp_fast(zeta);
    const double c = rsqrt_fast(fma(t, t, 1.0)), s = c * t;
    G[p] = fma(-t, gpq, gpp);
    G[q] = fma(t, gpq, gqq);
    G[ipq] = 0.0;
    const double grp = G[ipr], grq = G[iqr];
    G[ipr] = c * grp - s * grq;
    G[iqr] = s * grp + c * grq;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const double zp = Z[3 * k + p], zq = Z[3 * k + q];
      Z[3 * k + p] = c * zp - s * zq;
      Z[3 * k + q] = s * zp + c * zq;
    }
  }
}

// Gram-Schmidt with one re-orthogonalisation ("twice is enough"): the inverse iterates are
// nearly parallel (on exact data they differ by ~1e16 along the null direction), and one
// classical pass leaves the remainder's rounding noise along u, which corrupts the 3x3 Ritz step.
__device__ __forceinline__ void orthonormalize3(double (&u)[12], double (&v)[12],
                                                double (&w)[12]) {
  const double iu = rsqrt_fast(dot12(u, u));
#pragma unroll
  for (int j = 0; j < 12; ++j) u[j] *= iu;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    const double p = dot12(u, v);
#pragma unroll
    for (int j = 0; j < 12; ++j) v[j] = fma(-p, u[j], v[j]);
  }
  const double iv = rsqrt_fast(dot12(v, v));
#pragma unroll
  for (int j = 0; j < 12; ++j) v[j] *= iv;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    const double pu = dot12(u, w), pv = dot12(v, w);
#pragma unroll
    for (int j = 0; j < 12; ++j) w[j] = fma(-pv, v[j], fma(-pu, u[j], w[j]));
  }
  const double iw = rsqrt_fast(dot12(w, w));
#pragma unroll
  for (int j = 0; j < 12; ++j) w[j] *= iw;
}

#ifndef RSAMD_PNP_MAXIT
#define RSAMD_PNP_MAXIT 200  // (A/B builds time the rest of the solve with 1)
#endif
// 3: block-structured factor + three-vector block (below); 2: the dense factor and the
// two-vector block (A/B builds)
#ifndef RSAMD_PNP_BLOCK
#define RSAMD_PNP_BLOCK 3
#endif
// The block iteration stops when the Ritz vector moves <= RSAMD_PNP_TOL (or stagnates at the
// rounding floor).  The samples' own conditioning sets how closely any two SVDs agree: over 400
// noisy C3 samples the GPU pose equals numpy's (oracle/pnp_ref.pnp_dlt) to max |dR| 4.6e-13
// (p99 8.9e-14) at 1e-15, 1e-13 and 1e-12 alike (test_dlt_minimal_samples_accuracy_against_
// numpy_svd), while the slowest trial's sweeps -- the kernel's time -- fall: C3 k_pnp_solve
// 0.075 / 0.068 / 0.065 ms (tools/pnp_tol_ab.sh).
#ifndef RSAMD_PNP_TOL
#define RSAMD_PNP_TOL 1e-12
#endif
#ifndef RSAMD_PNP_HOUSE6
#define RSAMD_PNP_HOUSE6 1  // six-point samples by Householder (blk_house6)
#endif
// Constraint enforcement (pnp.py:141-145): C0 = (A | b) -> (R, t).
__device__ __forceinline__ void enforce_pose(const double (&c0)[12], double (&Rm)[9],
                                             double (&t)[3]) {
  double A[9];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) A[3 * i + j] = c0[4 * i + j];
  const double det = A[0] * (A[4] * A[8] - A[5] * A[7]) - A[1] * (A[3] * A[8] - A[5] * A[6]) +
                     A[2] * (A[3] * A[7] - A[4] * A[6]);
  const double tau = det > 0.0 ? 1.0 : (det < 0.0 ? -1.0 : (det == 0.0 ? 0.0 : det));
  double B[9], V[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) B[i] = tau * A[i];
  svd3_jacobi(B, V);
  double s[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) s[j] = sqrt(B[j] * B[j] + B[3 + j] * B[3 + j] + B[6 + j] * B[6 + j]);
  const double is0 = 1.0 / s[0], is1 = 1.0 / s[1], is2 = 1.0 / s[2];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c)
      Rm[3 * r + c] = B[3 * r + 0] * is0 * V[3 * c + 0] + B[3 * r + 1] * is1 * V[3 * c + 1] +
                      B[3 * r + 2] * is2 * V[3 * c + 2];
  const double lam = 3.0 * tau / ((s[0] + s[1]) + s[2]);
  t[0] = lam * c0[3];
  t[1] = lam * c0[7];
  t[2] = lam * c0[11];
}

// ---- The DLT system's block structure ----------------------------------------------------
// The two rows of a correspondence are [y]_x rows 0 and 1 times x~ = (X, Y, Z, 1) (pnp.py:
// 132-160, dlt_rows): a0 = (0, -y2 x~, y1 x~), a1 = (y2 x~, 0, -y0 x~) in column blocks of four
// (P's rows 1, 2, 3).  With the a1 rows first the matrix is [[P, 0, Q], [0, S, T]], so A^T A has a
// zero block (0:4, 4:8) and so has its Cholesky factor R:
//   R = [[R1, 0, X1], [0, R2, X2], [0, 0, R3]]   (R1, R2, R3 4x4 upper triangular)
// An a1 row (p, 0, q) rotates into [R1 | X1] and leaves (0, 0, q') for R3; an a0 row (0, s, t)
// into [R2 | X2], leaving t'.  Givens streaming then costs 168 instead of 348 operations a row,
// R takes 62 doubles instead of 78, and R1 / R2 solve independently (R^T R is the same matrix
// as for the dense factor: the same singular vectors).
struct BlkR {
  double R1[10], X1[16], R2[10], X2[16], R3[10];
};
constexpr int t4(int j, int l) { return j * 4 - (j * (j - 1)) / 2 + (l - j); }

// one Givens pivot of the row's entry a (the pivot column's) against the diagonal r; returns
// (c, s) and the new diagonal (givens_row's arithmetic)
__device__ __forceinline__ void givens_cs(double &r, double aj, double &c, double &s) {
  const double q = fma(r, r, aj * aj);
  const bool live = q > 0.0;
  const double inv = live ? rsqrt_fast(live ? q : 1.0) : 0.0;
  c = live ? r * inv : 1.0;
  s = aj * inv;
  r = live ? q * inv : 0.0;
}

// row (p | q) into [Rk | Xk] (4x4 upper, 4x4), q' left in q
__device__ __forceinline__ void givens_blk(double (&Rk)[10], double (&Xk)[16], double (&p)[4],
                                           double (&q)[4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    double c, s;
    givens_cs(Rk[t4(j, j)], p[j], c, s);
#pragma unroll
    for (int l = j + 1; l < 4; ++l) {
      const double rl = Rk[t4(j, l)];
      Rk[t4(j, l)] = fma(c, rl, s * p[l]);
      p[l] = fma(c, p[l], -s * rl);
    }
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      const double xl = Xk[4 * j + l];
      Xk[4 * j + l] = fma(c, xl, s * q[l]);
      q[l] = fma(c, q[l], -s * xl);
    }
  }
}

__device__ __forceinline__ void givens_tri(double (&Rk)[10], double (&p)[4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    double c, s;
    givens_cs(Rk[t4(j, j)], p[j], c, s);
#pragma unroll
    for (int l = j + 1; l < 4; ++l) {
      const double rl = Rk[t4(j, l)];
      Rk[t4(j, l)] = fma(c, rl, s * p[l]);
      p[l] = fma(c, p[l], -s * rl);
    }
  }
}

// the two DLT rows of one correspondence into R
__device__ __forceinline__ void blk_add_point(BlkR &B, const PPt &p) {
  const double xh[4] = {p.X, p.Y, p.Z, 1.0};
  double a[4], b[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {  // a1 = (y2 x~, 0, -y0 x~)
    a[j] = p.y2 * xh[j];
    b[j] = -p.y0 * xh[j];
  }
  givens_blk(B.R1, B.X1, a, b);
  givens_tri(B.R3, b);
#pragma unroll
  for (int j = 0; j < 4; ++j) {  // a0 = (0, -y2 x~, y1 x~)
    a[j] = -p.y2 * xh[j];
    b[j] = p.y1 * xh[j];
  }
  givens_blk(B.R2, B.X2, a, b);
  givens_tri(B.R3, b);
}

// R^T z = v for one 4x4 block (forward), R w = z (backward); di = 1 / diag
__device__ __forceinline__ void tri4_t(const double (&Rk)[10], const double *di, double *v) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    double acc = v[j];
#pragma unroll
    for (int i = 0; i < j; ++i) acc = fma(-Rk[t4(i, j)], v[i], acc);
    v[j] = acc * di[j];
  }
}
__device__ __forceinline__ void tri4(const double (&Rk)[10], const double *di, double *v) {
#pragma unroll
  for (int j = 3; j >= 0; --j) {
    double acc = v[j];
#pragma unroll
    for (int l = j + 1; l < 4; ++l) acc = fma(-Rk[t4(j, l)], v[l], acc);
    v[j] = acc * di[j];
  }
}

// v <- (R^T R)^-1 v with the block factor
__device__ __forceinline__ void blk_solve(const BlkR &B, const double (&di)[12], double (&v)[12]) {
  tri4_t(B.R1, di, v);
  tri4_t(B.R2, di + 4, v + 4);
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    double acc = v[8 + c];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc = fma(-B.X1[4 * j + c], v[j], fma(-B.X2[4 * j + c], v[4 + j], acc));
    v[8 + c] = acc;
  }
  tri4_t(B.R3, di + 8, v + 8);
  tri4(B.R3, di + 8, v + 8);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    double a0 = v[j], a1 = v[4 + j];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      a0 = fma(-B.X1[4 * j + c], v[8 + c], a0);
      a1 = fma(-B.X2[4 * j + c], v[8 + c], a1);
    }
    v[j] = a0;
    v[4 + j] = a1;
  }
  tri4(B.R1, di, v);
  tri4(B.R2, di + 4, v + 4);
}

// r = R v
__device__ __forceinline__ void blk_mul(const BlkR &B, const double (&v)[12], double (&r)[12]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    double a0 = 0.0, a1 = 0.0, a2 = 0.0;
#pragma unroll
    for (int l = j; l < 4; ++l) {
      a0 = fma(B.R1[t4(j, l)], v[l], a0);
      a1 = fma(B.R2[t4(j, l)], v[4 + l], a1);
      a2 = fma(B.R3[t4(j, l)], v[8 + l], a2);
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      a0 = fma(B.X1[4 * j + c], v[8 + c], a0);
      a1 = fma(B.X2[4 * j + c], v[8 + c], a1);
    }
    r[j] = a0;
    r[4 + j] = a1;
    r[8 + j] = a2;
  }
}

// G = (R [u v w])^T (R [u v w]) accumulated a row of R at a time (no 12-vector temporaries:
// the kernel is at the register limit)
__device__ __forceinline__ void blk_gram3(const BlkR &B, const double (&u)[12],
                                          const double (&v)[12], const double (&w)[12],
                                          double (&G)[6]) {
#pragma unroll
  for (int i = 0; i < 6; ++i) G[i] = 0.0;
  auto acc = [&](double a, double b, double c) {
    G[0] = fma(a, a, G[0]);
    G[1] = fma(b, b, G[1]);
    G[2] = fma(c, c, G[2]);
    G[3] = fma(a, b, G[3]);
    G[4] = fma(a, c, G[4]);
    G[5] = fma(b, c, G[5]);
  };
#pragma unroll
  for (int blk = 0; blk < 3; ++blk) {
    const double *Rk = blk == 0 ? B.R1 : (blk == 1 ? B.R2 : B.R3);
    const double *Xk = blk == 0 ? B.X1 : B.X2;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      double a = 0.0, b = 0.0, c = 0.0;
#pragma unroll
      for (int l = j; l < 4; ++l) {
        a = fma(Rk[t4(j, l)], u[4 * blk + l], a);
        b = fma(Rk[t4(j, l)], v[4 * blk + l], b);
        c = fma(Rk[t4(j, l)], w[4 * blk + l], c);
      }
      if (blk < 2) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          a = fma(Xk[4 * j + q], u[8 + q], a);
          b = fma(Xk[4 * j + q], v[8 + q], b);
          c = fma(Xk[4 * j + q], w[8 + q], c);
        }
      }
      acc(a, b, c);
    }
  }
}

// smallest_right_sv3 on the block factor: the start span(R^-1 e_11, e_10, e_9), then the same
// three-vector block inverse iteration with the 3x3 Rayleigh-Ritz step
__device__ __forceinline__ void blk_smallest_right_sv3(const BlkR &B, double (&x)[12]) {
  double di[12];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    di[j] = 1.0 / B.R1[t4(j, j)];
    di[4 + j] = 1.0 / B.R2[t4(j, j)];
    di[8 + j] = 1.0 / B.R3[t4(j, j)];
  }
  double u[12], v[12], w[12];
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    u[j] = j == 11 ? 1.0 : 0.0;
    v[j] = j == 10 ? 1.0 : 0.0;
    w[j] = j == 9 ? 1.0 : 0.0;
  }
  // R^-1 e_k: R3 back-substitution, then blocks 1, 2 from the X coupling
  auto rinv = [&](double (&a)[12]) {
    tri4(B.R3, di + 8, a + 8);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      double a0 = 0.0, a1 = 0.0;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        a0 = fma(-B.X1[4 * j + c], a[8 + c], a0);
        a1 = fma(-B.X2[4 * j + c], a[8 + c], a1);
      }
      a[j] = a0;
      a[4 + j] = a1;
    }
    tri4(B.R1, di, a);
    tri4(B.R2, di + 4, a + 4);
  };
  rinv(u);
  rinv(v);
  rinv(w);
  orthonormalize3(u, v, w);
#pragma unroll
  for (int j = 0; j < 12; ++j) x[j] = u[j];
  double prev_delta = 1.0;
  for (int it = 0; it < RSAMD_PNP_MAXIT; ++it) {
    blk_solve(B, di, u);
    blk_solve(B, di, v);
    blk_solve(B, di, w);
    orthonormalize3(u, v, w);
    double G[6];
    blk_gram3(B, u, v, w, G);
    double Z[9] = {1.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0};
    for (int sw = 0; sw < 8; ++sw) {
      bool rotated = false;
      jacobi_sym3(G, Z, 0, 1, rotated);
      jacobi_sym3(G, Z, 0, 2, rotated);
      jacobi_sym3(G, Z, 1, 2, rotated);
      if (!rotated) break;
    }
    const int m0 = (G[0] <= G[1] && G[0] <= G[2]) ? 0 : (G[1] <= G[2] ? 1 : 2);
    const int m1 = m0 == 0 ? 1 : 0, m2 = m0 == 2 ? 1 : 2;
    double z0[3], z1[3], z2[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      z0[k] = m0 == 0 ? Z[3 * k] : (m0 == 1 ? Z[3 * k + 1] : Z[3 * k + 2]);
      z1[k] = m1 == 0 ? Z[3 * k] : Z[3 * k + 1];
      z2[k] = m2 == 1 ? Z[3 * k + 1] : Z[3 * k + 2];
    }
#pragma unroll
    for (int j = 0; j < 12; ++j) {
      const double a = fma(z0[0], u[j], fma(z0[1], v[j], z0[2] * w[j]));
      const double b = fma(z1[0], u[j], fma(z1[1], v[j], z1[2] * w[j]));
      const double c = fma(z2[0], u[j], fma(z2[1], v[j], z2[2] * w[j]));
      u[j] = a;
      v[j] = b;
      w[j] = c;
    }
    const double sgn = dot12(u, x) < 0.0 ? -1.0 : 1.0;
    double delta = 0.0;
#pragma unroll
    for (int j = 0; j < 12; ++j) {
      const double nv = sgn * u[j];
      delta = fmax(delta, fabs(nv - x[j]));
      x[j] = nv;
    }
    if (it > 0 && !(delta > RSAMD_PNP_TOL)) break;
    if (it > 1 && delta < 1e-13 && delta > 0.5 * prev_delta) break;
    prev_delta = delta;
  }
  const double in = 1.0 / sqrt(dot12(x, x));
#pragma unroll
  for (int j = 0; j < 12; ++j) x[j] *= in;
}

// Six correspondences (the minimal DLT sample) by Householder instead of row streaming.  Block 1
// is [P | Q] with rows y2 x~ | -y0 x~, block 2 is [S | T] with rows -y2 x~ | y1 x~, and S = -P:
// with P = H [R1; 0] (four reflections, applied to Q and T as well),
//   H^T [P | 0 | Q] = [[R1, 0, X1 = (H^T Q)_top], [0, 0, (H^T Q)_bot]],
//   H^T [0 | S | T] = [[0, -R1, (H^T T)_top], [0, 0, (H^T T)_bot]],
// so R2 = R1 and X2 = -(H^T T)_top (the second block's rows negated), and R3 is the QR of the four
// leftover rows.  ~700 operations for the sample instead of twelve streamed rows' ~3 300, and R1
// is shared (RSAMD_PNP_HOUSE6 = 0: the streaming form for k = 6 as well).
__device__ __forceinline__ void blk_house6(const PPt (&p)[6], BlkR &B) {
  double P[6][4], Q[6][4], T[6][4];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const double xh[4] = {p[i].X, p[i].Y, p[i].Z, 1.0};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      P[i][c] = p[i].y2 * xh[c];
      Q[i][c] = -p[i].y0 * xh[c];
      T[i][c] = p[i].y1 * xh[c];
    }
  }
  double diag[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    // reflection of column k, rows k..5: v = (1, x_{k+1..} / (alpha - beta)), tau = 2 / v^T v
    const double alpha = P[k][k];
    double sig = 0.0;
#pragma unroll
    for (int i = k + 1; i < 6; ++i) sig = fma(P[i][k], P[i][k], sig);
    const double nrm = sqrt(fma(alpha, alpha, sig));
    const bool refl = sig > 0.0;
    const double beta = refl ? (alpha >= 0.0 ? -nrm : nrm) : alpha;
    const double sc = refl ? 1.0 / (alpha - beta) : 0.0;
    double v[6];
#pragma unroll
    for (int i = k + 1; i < 6; ++i) v[i] = P[i][k] * sc;
    double vv = 1.0;
#pragma unroll
    for (int i = k + 1; i < 6; ++i) vv = fma(v[i], v[i], vv);
    const double tau = refl ? 2.0 / vv : 0.0;
    diag[k] = beta;
    // apply I - tau v v^T to the remaining columns of P and to Q, T
    auto apply = [&](double (&M)[6][4], int c) {
      double w = M[k][c];
#pragma unroll
      for (int i = k + 1; i < 6; ++i) w = fma(v[i], M[i][c], w);
      w *= tau;
      M[k][c] -= w;
#pragma unroll
      for (int i = k + 1; i < 6; ++i) M[i][c] = fma(-w, v[i], M[i][c]);
    };
#pragma unroll
    for (int c = k + 1; c < 4; ++c) apply(P, c);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      apply(Q, c);
      apply(T, c);
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
#pragma unroll
    for (int l = j; l < 4; ++l) {
      const double r = l == j ? diag[j] : P[j][l];
      B.R1[t4(j, l)] = r;
      B.R2[t4(j, l)] = r;
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      B.X1[4 * j + c] = Q[j][c];
      B.X2[4 * j + c] = -T[j][c];
    }
  }
#pragma unroll
  for (int i = 0; i < 10; ++i) B.R3[i] = 0.0;
#pragma unroll
  for (int i = 4; i < 6; ++i) {
    double a[4], b[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      a[c] = Q[i][c];
      b[c] = T[i][c];
    }
    givens_tri(B.R3, a);
    givens_tri(B.R3, b);
  }
}

__device__ __forceinline__ void blk_zero(BlkR &B) {
#pragma unroll
  for (int i = 0; i < 10; ++i) B.R1[i] = B.R2[i] = B.R3[i] = 0.0;
#pragma unroll
  for (int i = 0; i < 16; ++i) B.X1[i] = B.X2[i] = 0.0;
}

// cond = false: the reference DLT on the raw world points (pnp.py:132-160).
// cond = true (the cv.solvePnPRansac drop-in): the sample's world points are first centred on
// their centroid c and scaled to unit RMS distance s (Hartley conditioning), the DLT solves for
// the pose of X' = (X - c) / s, and t = s t' - R c maps it back.  Exact data give the same pose
// either way; on compact, distant point sets (near-affine views, BAdino2's noisy reconstruction:
// depth 5.7-6.1, spread ~0.3) the raw 12x12 system is too ill-conditioned to survive pixel noise.
template <bool Cond, class IndexAt>
__device__ __forceinline__ void pnp_solve_points(const PPt *pts, int k, IndexAt index_at,
                                                 double (&Rm)[9], double (&t)[3]) {
#if RSAMD_PNP_BLOCK == 3
  BlkR R;
  blk_zero(R);
#else
  double R[78];
#pragma unroll
  for (int i = 0; i < 78; ++i) R[i] = 0.0;
#endif
  double cx = 0.0, cy = 0.0, cz = 0.0, sc = 1.0;
  if (Cond) {
    for (int q = 0; q < k; ++q) {
      const PPt &p = pts[index_at(q)];
      cx += p.X;
      cy += p.Y;
      cz += p.Z;
    }
    cx /= k;
    cy /= k;
    cz /= k;
    double ss = 0.0;
    for (int q = 0; q < k; ++q) {
      const PPt &p = pts[index_at(q)];
      ss += (p.X - cx) * (p.X - cx) + (p.Y - cy) * (p.Y - cy) + (p.Z - cz) * (p.Z - cz);
    }
    sc = sqrt(ss / k);
    if (!(sc > 0.0)) sc = 1.0;
  }
  const double isc = 1.0 / sc;
#if RSAMD_PNP_BLOCK == 3 && RSAMD_PNP_HOUSE6
  if (k == 6) {
    PPt p6[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      p6[q] = pts[index_at(q)];
      if (Cond) {
        p6[q].X = (p6[q].X - cx) * isc;
        p6[q].Y = (p6[q].Y - cy) * isc;
        p6[q].Z = (p6[q].Z - cz) * isc;
      }
    }
    blk_house6(p6, R);
    k = 0;  // (the streaming loop below is skipped)
  }
#endif
  for (int q = 0; q < k; ++q) {
    PPt p = pts[index_at(q)];
    if (Cond) {
      p.X = (p.X - cx) * isc;
      p.Y = (p.Y - cy) * isc;
      p.Z = (p.Z - cz) * isc;
    }
#if RSAMD_PNP_BLOCK == 3
    blk_add_point(R, p);
#else
    double a0[12], a1[12];
    dlt_rows(p, a0, a1);
    givens_row(R, a0);
    givens_row(R, a1);
#endif
  }
  double c0[12];
#if RSAMD_PNP_BLOCK == 3
  blk_smallest_right_sv3(R, c0);
#else
  smallest_right_sv(R, c0);
#endif
  enforce_pose(c0, Rm, t);
  if (Cond) {
    t[0] = sc * t[0] - (Rm[0] * cx + Rm[1] * cy + Rm[2] * cz);
    t[1] = sc * t[1] - (Rm[3] * cx + Rm[4] * cy + Rm[5] * cz);
    t[2] = sc * t[2] - (Rm[6] * cx + Rm[7] * cy + Rm[8] * cz);
  }
}

constexpr int kMaxK = 16;

__global__ __launch_bounds__(256) void k_pnp_solve(const PPt *__restrict__ pts, int m, int H,
                                                   int k, int mode, uint64_t seed,
                                                   const int *__restrict__ tuples,
                                                   double *__restrict__ Psoa, int64_t ld,
                                                   int cond) {
  const int h = blockIdx.x * blockDim.x + threadIdx.x;
  if (h >= H) return;
  double Rm[9], t[3];
  if (mode == RSD_SAMPLER_PHILOX) {
    int s6[6];
    floyd_sample<6>(seed, static_cast<uint64_t>(h), m, s6);
    // select from the 6 registers without dynamic indexing
    auto at = [&](int q) {
      return q == 0 ? s6[0] : q == 1 ? s6[1] : q == 2 ? s6[2] : q == 3 ? s6[3] : q == 4 ? s6[4] : s6[5];
    };
    if (cond)
      pnp_solve_points<true>(pts, 6, at, Rm, t);
    else
      pnp_solve_points<false>(pts, 6, at, Rm, t);
  } else {
    const int *tup = tuples + static_cast<int64_t>(h) * k;
    pnp_solve_points<false>(pts, k, [&](int q) { return tup[q]; }, Rm, t);
  }
#pragma unroll
  for (int q = 0; q < 9; ++q) Psoa[q * ld + h] = Rm[q];
#pragma unroll
  for (int q = 0; q < 3; ++q) Psoa[(9 + q) * ld + h] = t[q];
}

// Minimal-sample poses for the cv.solvePnPRansac drop-in with OpenCV's RANSAC kernels: lane per
// hypothesis, a Philox sample of K points (K = 5: EPnP; K = 4: P3P on three, the fourth
// deciding).  Hypothesis `guess_slot` (>= 0) takes the caller's pose instead (the extrinsic
// guess, scored in the same order).  A failed solve writes NaN, which scores 0.
template <int K>
__global__ __launch_bounds__(64) void k_pnp_solve_min(const PPt *__restrict__ pts, int m, int H,
                                                      uint64_t seed, double *__restrict__ Psoa,
                                                      int64_t ld, int guess_slot,
                                                      const double *__restrict__ guess) {
  const int h = blockIdx.x * blockDim.x + threadIdx.x;
  if (h >= H) return;
  double Rm[9], t[3];
  double err = INFINITY;
  if (h == guess_slot) {
#pragma unroll
    for (int q = 0; q < 9; ++q) Rm[q] = guess[q];
#pragma unroll
    for (int q = 0; q < 3; ++q) t[q] = guess[9 + q];
    err = 0.0;
  } else {
    int idx[K];
    floyd_sample<K>(seed, static_cast<uint64_t>(h), m, idx);
    auto at = [&](int q) {
      int v = idx[0];
#pragma unroll
      for (int i = 1; i < K; ++i) v = q == i ? idx[i] : v;
      return pts[v];
    };
    if constexpr (K == 4)
      err = p3p_pose(at, Rm, t);
    else
      err = epnp_pose(at, K, Rm, t);
  }
  const double qn = __builtin_nan("");
  const bool ok = err < INFINITY;
#pragma unroll
  for (int q = 0; q < 9; ++q) Psoa[q * ld + h] = ok ? Rm[q] : qn;
#pragma unroll
  for (int q = 0; q < 3; ++q) Psoa[(9 + q) * ld + h] = ok ? t[q] : qn;
}

// The n = 3 branch of ransac_robust (ransac.py:81-82, 91-111): lane per trial, Lambda Twist
// P3P on the trial's three D_high correspondences (bearings (u, v, 1) / |.|), every pose it
// yields a hypothesis of its own, as the reference loops over p3p's poses (ransac.py:92) --
// slot j of trial i is model kP3pSlots i + j, so the strict-">" first-occurrence winner is the
// reference's trial-major, pose-minor order.  Up to four front-facing solutions, each followed
// by its mirrored-depth twin (the pose of a negative-scale camera, BAdino2's); empty slots are
// NaN, which scores no consensus.
constexpr int kP3pSlots = 8;
__global__ __launch_bounds__(64) void k_pnp_solve_p3p(const PPt *__restrict__ pts, int m, int H,
                                                      int mode, uint64_t seed,
                                                      const int *__restrict__ tuples,
                                                      double *__restrict__ Psoa, int64_t ld,
                                                      unsigned char *__restrict__ mirf) {
  const int h = blockIdx.x * blockDim.x + threadIdx.x;
  if (h >= H) return;
  int idx[3];
  if (mode == RSD_SAMPLER_PHILOX) {
    floyd_sample<3>(seed, static_cast<uint64_t>(h), m, idx);
  } else {
#pragma unroll
    for (int i = 0; i < 3; ++i) idx[i] = tuples[3 * static_cast<int64_t>(h) + i];
  }
  double X[3][3], y[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const PPt p = pts[idx[i]];
    X[i][0] = p.X;
    X[i][1] = p.Y;
    X[i][2] = p.Z;
    const double in = 1.0 / sqrt(p.u * p.u + p.v * p.v + 1.0);
    y[i][0] = p.u * in;
    y[i][1] = p.v * in;
    y[i][2] = in;
  }
  double Rs[kP3pSlots][9], ts[kP3pSlots][3];
  bool mir[kP3pSlots];
  const int ns = p3p_lambda_twist(X, y, Rs, ts, mir);
  const double qn = __builtin_nan("");
  const int64_t base = static_cast<int64_t>(kP3pSlots) * h;
  for (int s = 0; s < kP3pSlots; ++s) {
    const bool ok = s < ns;
#pragma unroll
    for (int q = 0; q < 9; ++q) Psoa[q * ld + base + s] = ok ? Rs[s][q] : qn;
#pragma unroll
    for (int q = 0; q < 3; ++q) Psoa[(9 + q) * ld + base + s] = ok ? ts[s][q] : qn;
    mirf[base + s] = ok && mir[s] ? 1 : 0;
  }
}

// EPnP over all m correspondences (method 1) or P3P on exactly four (method 2): single lane.
__global__ __launch_bounds__(64) void k_pnp_minimal_all(const PPt *__restrict__ pts, int m,
                                                        int method, double *__restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double Rm[9], t[3];
  auto at = [&](int q) { return pts[q]; };
  const double err = method == 2 ? p3p_pose(at, Rm, t) : epnp_pose(at, m, Rm, t);
  for (int q = 0; q < 9; ++q) out[q] = err < INFINITY ? Rm[q] : __builtin_nan("");
  for (int q = 0; q < 3; ++q) out[9 + q] = err < INFINITY ? t[q] : __builtin_nan("");
  out[12] = err;
}

// One-point DLT over all m correspondences (rs_pnp_dlt): single lane.
__global__ __launch_bounds__(64) void k_pnp_dlt_all(const PPt *__restrict__ pts, int m,
                                                    double *__restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  BlkR R;
  blk_zero(R);
  for (int q = 0; q < m; ++q) blk_add_point(R, pts[q]);
  double c0[12], Rm[9], t[3];
  blk_smallest_right_sv3(R, c0);
  enforce_pose(c0, Rm, t);
  for (int q = 0; q < 9; ++q) out[q] = Rm[q];
  for (int q = 0; q < 3; ++q) out[9 + q] = t[q];
}

// e = dpp_squared(y, R x + t) in the reference's arithmetic (ransac.py:21-35; calc_y_prim
// ransac.py:34-35): R x by numpy's matmul, which on the build container's OpenBLAS dgemm is the
// FMA chain fma(R_i2, z, fma(R_i1, y, R_i0 x)) (checked bit for bit against oracle/pnp_ref's
// pose_errors, tests/test_oracle_p3p.py), then + t, pi, diff, and the dot in order.
// P: R row-major (9), then t (3).
__device__ __forceinline__ bool pnp_inlier_ref(const double *P, const PPt &p, double thresh) {
#pragma clang fp contract(off)
  const double q0 = fma(P[2], p.Z, fma(P[1], p.Y, P[0] * p.X)) + P[9];
  const double q1 = fma(P[5], p.Z, fma(P[4], p.Y, P[3] * p.X)) + P[10];
  const double q2 = fma(P[8], p.Z, fma(P[7], p.Y, P[6] * p.X)) + P[11];
  const double a0 = p.u - q0 / q2, a1 = p.v - q1 / q2;
  const double a2 = p.y2 / p.y2 - q2 / q2;
  const double e = (a0 * a0 + a1 * a1) + a2 * a2;
  return thresh >= e;
}

// Consensus counts of ransac.py:96-105 (`thresh >= dpp_squared(y, R x + t)`, counted on D_med).
//
// The division-free test |M (u q2 - q0, v q2 - q1)|^2 <= thr q2^2 decides almost every
// (hypothesis, point); with Exact (the reference-mode metric, M = I) it is exact: a pair whose
// margin |D - thr q2^2| is within the rigorous error band below is re-tested in the reference's
// own arithmetic (pnp_inlier_ref: three divisions, numpy's order), so every count equals the
// reference-order count -- and so the winner's count equals its consensus set (k_pnp_inliers,
// the same arithmetic; the host checks best_count == n_med).
//
// The band (u = 2^-53, first-order error analysis, then x2 for the second-order terms).  With
// S_i = sum_j |R_ij x_j| + |t_i| <= L = rmax xmax + tmax (rmax the largest row 2-norm of R,
// Cauchy-Schwarz; xmax >= |x|_1 and umax >= max(|u|, |v|) over the call's points, from the host),
// Q = |q2|, d = (du, dv), D = |d|^2, a = |du| + |dv|:
//   * each q_i (either fma chain, the reference's with + t apart) is within 4u S_i of exact;
//   * fast: |d_i - A_i| <= 3u (umax S_2 + S_i) + u |d_i|, A_i = u_i q2* - q_i* the exact
//     residual; and e* q2^2 differs from |A|^2 by the relative 2 (3u S_2 / Q) of q2's error;
//   * reference: |a_i - a_i*| Q <= 4u (S_i + |q_i| / Q S_2) + u |q_i| + u |A_i| (the quotient's
//     and the difference's roundings), and the dot product adds 2u D;
//   * thr q2^2 is rounded twice (2u).
// Collected with g = 4.01u L (3 + umax + L / Q):  band = 2 (2 g a + 4 g^2 + u (D (8.1 + 6.1 L / Q)
// + 2.01 thr q2^2)).  If D - thr q2^2 > band the exact e exceeds thr by more than the
// reference's own error (outlier in both); below -band it is an inlier in both.  Q = 0, a NaN or
// an infinity makes the band non-finite, and the pair takes the reference test.  Per point the
// band costs a reciprocal estimate and ~8 FMAs (the per-hypothesis L and constants hoisted).
template <bool Exact>
__global__ __launch_bounds__(256) void k_pnp_count(const PPt *__restrict__ pts, int m, int H,
                                                   const double *__restrict__ Psoa, int64_t ld,
                                                   int chunk, int nchunks, double thresh,
                                                   PxMetric mt, double xmax, double umax,
                                                   int *__restrict__ counts) {
  const int lane = threadIdx.x & 63;
  const int u = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  const int ngroups = (H + 63) >> 6;
  if (u >= ngroups * nchunks) return;
  const int g = u / nchunks, c = u - g * nchunks;
  const int p0 = c * chunk, p1 = min(m, p0 + chunk);
  const int h = g * 64 + lane;
  const int hl = h < H ? h : H - 1;
  double P[12];
#pragma unroll
  for (int q = 0; q < 12; ++q) P[q] = Psoa[q * ld + hl];
  constexpr double kU = 0x1p-53;
  double L = 0.0, g0 = 0.0, g1 = 0.0;
  if (Exact) {
    double rmax = 0.0, tmax = 0.0;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      rmax = fmax(rmax, fma(P[3 * r], P[3 * r], fma(P[3 * r + 1], P[3 * r + 1], P[3 * r + 2] * P[3 * r + 2])));
      tmax = fmax(tmax, fabs(P[9 + r]));
    }
    // (a NaN pose makes D NaN, so its band is NaN and the reference test decides: false)
    L = fma(sqrt(rmax) * (1.0 + 8.0 * kU), xmax, tmax) * (1.0 + 4.0 * kU);
    g0 = 2.0 * (4.01 * kU) * L * (3.0 + umax);  // 2 g = g0 + g1 L / Q
    g1 = 2.0 * (4.01 * kU) * L;
  }
  int cnt = 0;
  for (int i = p0; i < p1; ++i) {
    const PPt p = pts[i];
    const double q0 = fma(P[0], p.X, fma(P[1], p.Y, fma(P[2], p.Z, P[9])));
    const double q1 = fma(P[3], p.X, fma(P[4], p.Y, fma(P[5], p.Z, P[10])));
    const double q2 = fma(P[6], p.X, fma(P[7], p.Y, fma(P[8], p.Z, P[11])));
    // |M (pi(y) - pi(q))|^2 <= thr  <=>  |M (u q2 - q0, v q2 - q1)|^2 <= thr q2^2, q2 != 0
    // (identity M in reference mode: the plain residual)
    const double du0 = fma(p.u, q2, -q0), dv = fma(p.v, q2, -q1);
    const double du = Exact ? du0 : fma(mt.a, du0, mt.b * dv), dvm = Exact ? dv : mt.c * dv;
    const double lhs = fma(du, du, dvm * dvm);
    const double rhs = thresh * (q2 * q2);
    bool in = q2 != 0.0 && lhs <= rhs;
    if (Exact) {
      const double Lr = L * __builtin_amdgcn_rcp(fabs(q2));
      const double g2 = fma(g1, Lr, g0);                          // 2 g
      const double a = fabs(du) + fabs(dv);
      const double band = fma(2.0 * g2, a + g2,                     // 2 (2 g a + 4 g^2 ...
                              (2.0 * kU) * fma(lhs, fma(6.1, Lr, 8.1), 2.01 * rhs));
      if (!(fabs(lhs - rhs) > band)) in = pnp_inlier_ref(P, p, thresh);
    }
    cnt += in ? 1 : 0;
  }
  if (h < H) atomicAdd(&counts[h], cnt);
}

struct PnpDevResult {
  double R[9];
  double t[3];
  int64_t best_index, best_count, n_med, n_high;
  int64_t inliers[];  // med then high
};

// (mirf, the P3P branch: each pose's mirrored-depth flag.  A mirrored pose -- all depths
// negated: the scene behind a positive-scale camera -- reprojects like its front-facing twin,
// so on a noisy near-planar scene the twin can out-count the true pose by a few points.  The
// winner is then the first best front-facing pose unless the best mirrored count is more than
// kMirrorCountWins times it: a negative-scale camera (BAdino2's) has no front-facing fit at all.)
constexpr int kMirrorCountWins = 2;
__device__ __forceinline__ void sel_better(int c, int i, int &bm, int &bi) {
  if (c > bm || (c == bm && i < bi)) {
    bm = c;
    bi = i;
  }
}
__device__ void pnp_select_block(const int *__restrict__ counts, int H,
                                 const double *__restrict__ Psoa, int64_t ld, PnpDevResult *res,
                                 const unsigned char *__restrict__ mirf) {
  __shared__ int sm[2][16], si[2][16];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int bm[2] = {0, 0}, bi[2] = {0x7fffffff, 0x7fffffff};  // front-facing, mirrored
  // 8 loads of four counts in flight per thread before the (order-free) max / first-index
  // comparisons (C3's 5e4 counts: two rounds of loads instead of seven; the select + inliers
  // launch measured 20.8 -> 19.5 us); counts and flags sit at 256-byte aligned scratch offsets
  const int H4 = H >> 2;
  const int4 *c4 = reinterpret_cast<const int4 *>(counts);
  const uchar4 *f4 = reinterpret_cast<const uchar4 *>(mirf);
  for (int i0 = tid; i0 < H4; i0 += 8 * 1024) {
    int4 c[8];
    uchar4 f[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + u * 1024;
      c[u] = i < H4 ? c4[i] : make_int4(-1, -1, -1, -1);
      f[u] = mirf && i < H4 ? f4[i] : make_uchar4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = 4 * (i0 + u * 1024);
      const int cc[4] = {c[u].x, c[u].y, c[u].z, c[u].w};
      const int ff[4] = {f[u].x, f[u].y, f[u].z, f[u].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (ff[e]) sel_better(cc[e], i + e, bm[1], bi[1]);
        else sel_better(cc[e], i + e, bm[0], bi[0]);
      }
    }
  }
  for (int i = 4 * H4 + tid; i < H; i += 1024) {  // the last H mod 4 counts
    if (mirf && mirf[i]) sel_better(counts[i], i, bm[1], bi[1]);
    else sel_better(counts[i], i, bm[0], bi[0]);
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const int om = __shfl_xor(bm[k], o), oi = __shfl_xor(bi[k], o);
      sel_better(om, oi, bm[k], bi[k]);
    }
    if (lane == 0) {
      sm[k][w] = bm[k];
      si[k][w] = bi[k];
    }
  }
  __syncthreads();
  if (tid == 0) {
    for (int k = 0; k < 2; ++k)
      for (int q = 1; q < 16; ++q) sel_better(sm[k][q], si[k][q], bm[k], bi[k]);
    const int cls = bm[1] > kMirrorCountWins * bm[0] ? 1 : 0;
    int bm0 = bm[cls], bi0 = bi[cls];
    if (!mirf) {  // one class: the first largest count over all hypotheses
      bm0 = bm[0];
      bi0 = bi[0];
    }
    // strict ">" against an initial best of 0 (ransac.py:108): zero consensus never wins
    if (bm0 > 0) {
      res->best_index = bi0;
      res->best_count = bm0;
      for (int q = 0; q < 9; ++q) res->R[q] = Psoa[q * ld + bi0];
      for (int q = 0; q < 3; ++q) res->t[q] = Psoa[(9 + q) * ld + bi0];
    } else {
      res->best_index = -1;
      res->best_count = 0;
      for (int q = 0; q < 9; ++q) res->R[q] = 0.0;
      for (int q = 0; q < 3; ++q) res->t[q] = 0.0;
    }
  }
}

// cv.solvePnPRansac's inlier test (OpenCV: projectPoints, dx^2 + dy^2 <= err^2) in pixels.
__device__ __forceinline__ bool pnp_inlier_px(const double (&Rm)[9], const double (&t)[3],
                                              const PPt &p, double thresh, const PxMetric &mt) {
  const double q0 = fma(Rm[0], p.X, fma(Rm[1], p.Y, fma(Rm[2], p.Z, t[0])));
  const double q1 = fma(Rm[3], p.X, fma(Rm[4], p.Y, fma(Rm[5], p.Z, t[1])));
  const double q2 = fma(Rm[6], p.X, fma(Rm[7], p.Y, fma(Rm[8], p.Z, t[2])));
  const double du0 = fma(p.u, q2, -q0), dv = fma(p.v, q2, -q1);
  const double du = fma(mt.a, du0, mt.b * dv), dvm = mt.c * dv;
  return q2 != 0.0 && fma(du, du, dvm * dvm) <= thresh * (q2 * q2);
}

template <class Pred>
__device__ void ordered_compact(int m, Pred pred, bool have, int64_t *out, int64_t *n_out,
                                int *woff, int *base_s) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (tid == 0) *base_s = 0;
  __syncthreads();
  for (int b = 0; b < m; b += 1024) {
    const int i = b + tid;
    const bool take = have && i < m && pred(i);
    const unsigned long long bal = __ballot(take);
    const int before = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) woff[w] = __popcll(bal);
    __syncthreads();
    if (tid == 0) {
      int acc = *base_s;
      for (int q = 0; q < 16; ++q) {
        const int tq = woff[q];
        woff[q] = acc;
        acc += tq;
      }
      *base_s = acc;
    }
    __syncthreads();
    if (take) out[woff[w] + before] = i;
    __syncthreads();
  }
  if (tid == 0) *n_out = *base_s;
  __syncthreads();
}

__device__ void pnp_inliers_block(const PPt *__restrict__ med, int m_med,
                                  const PPt *__restrict__ high, int m_high, double thresh,
                                  PnpDevResult *res) {
  __shared__ int woff[16];
  __shared__ int base_s;
  const bool have = res->best_index >= 0;
  double P[12];
#pragma unroll
  for (int q = 0; q < 9; ++q) P[q] = res->R[q];
#pragma unroll
  for (int q = 0; q < 3; ++q) P[9 + q] = res->t[q];
  if (m_med <= 512 && m_high <= 512 && blockDim.x == 1024) {
    // both sets in one pass: threads 0..511 test D_med's points, 512..1023 D_high's, each half
    // compacted in point order by its own wave prefix (one barrier pair instead of two)
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, half = tid >> 9, i = tid & 511;
    const int mm = half ? m_high : m_med;
    const PPt *src = half ? high : med;
    const bool take = have && i < mm && pnp_inlier_ref(P, src[i], thresh);
    const unsigned long long bal = __ballot(take);
    const int before = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) woff[w] = __popcll(bal);
    __syncthreads();
    if ((tid & 511) == 0) {
      int acc = 0;
      for (int q = 8 * half; q < 8 * half + 8; ++q) {
        const int tq = woff[q];
        woff[q] = acc;
        acc += tq;
      }
      if (half) res->n_high = acc;
      else res->n_med = acc;
    }
    __syncthreads();
    if (take) res->inliers[(half ? m_med : 0) + woff[w] + before] = i;
    return;
  }
  ordered_compact(
      m_med, [&](int i) { return pnp_inlier_ref(P, med[i], thresh); }, have, res->inliers,
      &res->n_med, woff, &base_s);
  ordered_compact(
      m_high, [&](int i) { return pnp_inlier_ref(P, high[i], thresh); }, have,
      res->inliers + m_med, &res->n_high, woff, &base_s);
}

// The winner and its consensus sets in one launch (one workgroup): k_pnp_select's choice, then
// the reference-order sets of pnp_inliers_block (one launch gap less per call).
__global__ __launch_bounds__(1024) void k_pnp_select_inliers(
    const int *__restrict__ counts, int H, const double *__restrict__ Psoa, int64_t ld,
    PnpDevResult *res, const unsigned char *__restrict__ mirf, const PPt *__restrict__ med,
    int m_med, const PPt *__restrict__ high, int m_high, double thresh) {
  pnp_select_block(counts, H, Psoa, ld, res, mirf);
  __syncthreads();  // the winner's record (thread 0's writes) before every thread reads it
  pnp_inliers_block(med, m_med, high, m_high, thresh, res);
}

// rs_pnp_ransac_cv: the pose of hypothesis `best` (chosen on the host by the adaptive
// replay), then its pixel-space consensus set in point order.
__global__ __launch_bounds__(1024) void k_pnp_inliers_px(const PPt *__restrict__ pts, int m,
                                                         const double *__restrict__ Psoa,
                                                         int64_t ld, int64_t best, int64_t count,
                                                         double thresh, PxMetric mt,
                                                         PnpDevResult *res) {
  __shared__ int woff[16];
  __shared__ int base_s;
  double Rm[9], t[3];
#pragma unroll
  for (int q = 0; q < 9; ++q) Rm[q] = Psoa[q * ld + best];
#pragma unroll
  for (int q = 0; q < 3; ++q) t[q] = Psoa[(9 + q) * ld + best];
  if (threadIdx.x == 0) {
    for (int q = 0; q < 9; ++q) res->R[q] = Rm[q];
    for (int q = 0; q < 3; ++q) res->t[q] = t[q];
    res->best_index = best;
    res->best_count = count;
    res->n_high = 0;
  }
  ordered_compact(
      m, [&](int i) { return pnp_inlier_px(Rm, t, pts[i], thresh, mt); }, true, res->inliers,
      &res->n_med, woff, &base_s);
}

__global__ __launch_bounds__(256) void k_pack_ppts(const double *__restrict__ X,
                                                   const double *__restrict__ y, int m,
                                                   PPt *__restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  PPt p;
  p.X = X[3 * i];
  p.Y = X[3 * i + 1];
  p.Z = X[3 * i + 2];
  p.y0 = y[3 * i];
  p.y1 = y[3 * i + 1];
  p.y2 = y[3 * i + 2];
  p.u = p.y0 / p.y2;  // norm_p (ransac.py:21-23)
  p.v = p.y1 / p.y2;
  out[i] = p;
}


// ---- Levenberg-Marquardt on the pixel reprojection error (cv.solvePnP SOLVEPNP_ITERATIVE's
// refinement stage, pnp.py:7-10 and the tables.py:141-147 call site) -------------------------
// One workgroup: every pass maps the points over the threads, each accumulating its share of
// J^T J (21 terms), J^T r (6) and the cost, reduced by wave shuffles and LDS; thread 0 solves the
// damped 6 x 6 system (Marquardt scaling, Cholesky) and steps.  The pose is updated on the left,
// R <- exp([d]x) R, t <- t + dt, so dq/dd = -[R x]x and dq/dt = I for q = R x + t; the pixel
// residual is K pi(q) - uv with K's fx, skew, cx, fy, cy (K / K[2][2], as projectPoints).  Only
// steps that lower the cost are taken (CvLevMarq), at most `max_jac` Jacobians and 8x as many
// trial passes; the loop ends when a taken step moves the parameters by less than eps relative.
struct LmK {
  double fx, s, cx, fy, cy;
};

constexpr int kLmThreads = 256;
constexpr int kLmAcc = 28;  // J^T J upper triangle (21), J^T r (6), |r|^2

__device__ void lm_block_sum(double (&v)[kLmAcc], double (*sh)[kLmAcc]) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < kLmAcc; ++k) {
    double x = v[k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    v[k] = x;
  }
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < kLmAcc; ++k) sh[wv][k] = v[k];
  __syncthreads();
  if (threadIdx.x == 0)
#pragma unroll
    for (int k = 0; k < kLmAcc; ++k) {
      double x = 0.0;
      for (int w = 0; w < kLmThreads / 64; ++w) x += sh[w][k];
      v[k] = x;
    }
}

// io: R (9), t (3), then scratch / results (4)
__global__ __launch_bounds__(kLmThreads) void k_pnp_lm(const double *__restrict__ X,
                                                        const double *__restrict__ uv, int n, LmK K,
                                                        double *__restrict__ io, int max_jac,
                                                        double eps) {
  __shared__ double sR[9], st[3], tR[9], tt[3];
  __shared__ double sh[kLmThreads / 64][kLmAcc];
  __shared__ int s_cmd;  // 0 Jacobian pass at the current pose, 1 trial pass, 2 stop
  const int tid = threadIdx.x;
  if (tid < 9) sR[tid] = io[tid];
  if (tid < 3) st[tid] = io[9 + tid];
  if (tid == 0) s_cmd = 0;
  __syncthreads();
  // thread 0's LM state
  double A[21] = {}, g[6] = {}, cost = 0.0, cost0 = 0.0, lambda = 1e-3, step2 = 0.0;
  int njac = 0, ntrial = 0, taken = 0;
  for (;;) {
    const int cmd = s_cmd;
    if (cmd == 2) break;
    double R[9], t[3];
#pragma unroll
    for (int k = 0; k < 9; ++k) R[k] = cmd == 0 ? sR[k] : tR[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) t[k] = cmd == 0 ? st[k] : tt[k];
    double acc[kLmAcc];
#pragma unroll
    for (int k = 0; k < kLmAcc; ++k) acc[k] = 0.0;
    for (int i = tid; i < n; i += kLmThreads) {
      const double *x = X + 3 * i;
      const double p0 = fma(R[0], x[0], fma(R[1], x[1], R[2] * x[2]));
      const double p1 = fma(R[3], x[0], fma(R[4], x[1], R[5] * x[2]));
      const double p2 = fma(R[6], x[0], fma(R[7], x[1], R[8] * x[2]));
      const double q0 = p0 + t[0], q1 = p1 + t[1], q2 = p2 + t[2];
      const double iz = 1.0 / q2, a = q0 * iz, b = q1 * iz;
      const double ru = fma(K.fx, a, fma(K.s, b, K.cx)) - uv[2 * i];
      const double rv = fma(K.fy, b, K.cy) - uv[2 * i + 1];
      acc[27] = fma(ru, ru, fma(rv, rv, acc[27]));
      if (cmd != 0) continue;
      // du/dq, dv/dq
      const double du0 = K.fx * iz, du1 = K.s * iz, du2 = -(K.fx * a + K.s * b) * iz;
      const double dv1 = K.fy * iz, dv2 = -K.fy * b * iz;
      // J = dres/dq [ -[p]x | I ],  -[p]x = [[0, p2, -p1], [-p2, 0, p0], [p1, -p0, 0]]
      double ju[6], jv[6];
      ju[0] = -du1 * p2 + du2 * p1;
      ju[1] = du0 * p2 - du2 * p0;
      ju[2] = -du0 * p1 + du1 * p0;
      ju[3] = du0;
      ju[4] = du1;
      ju[5] = du2;
      jv[0] = -dv1 * p2 + dv2 * p1;
      jv[1] = -dv2 * p0;
      jv[2] = dv1 * p0;
      jv[3] = 0.0;
      jv[4] = dv1;
      jv[5] = dv2;
      int k = 0;
#pragma unroll
      for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int c2 = r; c2 < 6; ++c2) acc[k++] += ju[r] * ju[c2] + jv[r] * jv[c2];
#pragma unroll
      for (int r = 0; r < 6; ++r) acc[21 + r] += ju[r] * ru + jv[r] * rv;
    }
    lm_block_sum(acc, sh);
    if (tid == 0) {
      const double c = 0.5 * acc[27];
      bool solve = false;
      if (cmd == 0) {  // the Jacobian at the current pose
        if (njac == 0) cost0 = c;
        cost = c;
#pragma unroll
        for (int k = 0; k < 21; ++k) A[k] = acc[k];
#pragma unroll
        for (int k = 0; k < 6; ++k) g[k] = acc[21 + k];
        ++njac;
        solve = isfinite(c);
        if (!solve) s_cmd = 2;
      } else {  // a trial pose
        ++ntrial;
        if (c < cost && isfinite(c)) {  // taken
          for (int k = 0; k < 9; ++k) sR[k] = tR[k];
          double pn = 0.0;
          for (int k = 0; k < 3; ++k) {
            st[k] = tt[k];
            pn += tt[k] * tt[k];
          }
          cost = c;
          lambda = fmax(lambda * 0.1, 1e-12);
          ++taken;
          // converged when the step is below eps relative to the parameters (|t| + rotation)
          s_cmd = (njac < max_jac && step2 > eps * eps * (pn + 1.0)) ? 0 : 2;
        } else {
          lambda *= 10.0;
          solve = lambda < 1e16 && ntrial < 8 * max_jac;
          if (!solve) s_cmd = 2;
        }
      }
      // (A + lambda diag(A)) d = -g by Cholesky; trial R' = exp([d0..2]x) R, t' = t + d3..5
      while (solve) {
        // (fully unrolled: every index static, the 6 x 6 stays in registers)
        double M[6][6], d[6];
#pragma unroll
        for (int r = 0; r < 6; ++r)
#pragma unroll
          for (int c2 = 0; c2 < 6; ++c2) {
            const int lo = r < c2 ? r : c2, hi = r < c2 ? c2 : r;
            M[r][c2] = A[lo * 6 - lo * (lo - 1) / 2 + (hi - lo)];
          }
#pragma unroll
        for (int r = 0; r < 6; ++r) M[r][r] *= 1.0 + lambda;
        bool ok = true;
#pragma unroll
        for (int j = 0; j < 6; ++j) {
          double sj = M[j][j];
#pragma unroll
          for (int l = 0; l < j; ++l) sj -= M[j][l] * M[j][l];
          ok = ok && sj > 0.0;
          M[j][j] = sqrt(sj > 0.0 ? sj : 1.0);
#pragma unroll
          for (int r = j + 1; r < 6; ++r) {
            double sr = M[r][j];
#pragma unroll
            for (int l = 0; l < j; ++l) sr -= M[r][l] * M[j][l];
            M[r][j] = sr / M[j][j];
          }
        }
        if (!ok) {  // singular even with damping: more damping, or stop
          lambda *= 10.0;
          if (!(lambda < 1e16)) {
            s_cmd = 2;
            solve = false;
          }
          continue;
        }
#pragma unroll
        for (int r = 0; r < 6; ++r) {  // L y = -g
          double sr = -g[r];
#pragma unroll
          for (int l = 0; l < r; ++l) sr -= M[r][l] * d[l];
          d[r] = sr / M[r][r];
        }
#pragma unroll
        for (int r = 5; r >= 0; --r) {  // L^T d = y
          double sr = d[r];
#pragma unroll
          for (int l = r + 1; l < 6; ++l) sr -= M[l][r] * d[l];
          d[r] = sr / M[r][r];
        }
        const double th2 = d[0] * d[0] + d[1] * d[1] + d[2] * d[2], th = sqrt(th2);
        const double sa = th2 < 1e-16 ? 1.0 - th2 / 6.0 : sin(th) / th;
        const double cb = th2 < 1e-16 ? 0.5 - th2 / 24.0 : (1.0 - cos(th)) / th2;
        const double W[9] = {0.0, -d[2], d[1], d[2], 0.0, -d[0], -d[1], d[0], 0.0};
        double E[9];
        for (int r = 0; r < 3; ++r)
          for (int c2 = 0; c2 < 3; ++c2) {
            double w2 = 0.0;
            for (int l = 0; l < 3; ++l) w2 += W[3 * r + l] * W[3 * l + c2];
            E[3 * r + c2] = (r == c2 ? 1.0 : 0.0) + sa * W[3 * r + c2] + cb * w2;
          }
        for (int r = 0; r < 3; ++r)
          for (int c2 = 0; c2 < 3; ++c2)
            tR[3 * r + c2] = E[3 * r] * sR[c2] + E[3 * r + 1] * sR[3 + c2] + E[3 * r + 2] * sR[6 + c2];
        for (int r = 0; r < 3; ++r) tt[r] = st[r] + d[3 + r];
        step2 = th2 + d[3] * d[3] + d[4] * d[4] + d[5] * d[5];
        s_cmd = 1;
        solve = false;
      }
    }
    __syncthreads();
  }
  if (tid == 0) {
    for (int k = 0; k < 9; ++k) io[k] = sR[k];
    for (int k = 0; k < 3; ++k) io[9 + k] = st[k];
    io[12] = cost0;
    io[13] = cost;
    io[14] = njac;
    io[15] = taken;
  }
}

}  // namespace rsd

// ------------------------------------------------------------------------------------------
using rs::fail;
using rs::hip_fail;

#define HIP_TRY(expr)                                 \
  do {                                                \
    hipError_t e_ = (expr);                           \
    if (e_ != hipSuccess) return hip_fail(e_, #expr); \
  } while (0)

static size_t align256(size_t b) { return (b + 255) / 256 * 256; }

// Bounds of the call's points for k_pnp_count<true>'s guard band: xmax >= |x|_1 and umax >=
// max(|y0 / y2|, |y1 / y2|) over all points (a non-finite point makes both infinite: every pair
// then takes the reference-order test).
static void pnp_band_bounds(const double *X, const double *y, int64_t m, double *xmax,
                            double *umax) {
  double a = 0.0, b = 0.0;
  bool bad = false;
  for (int64_t i = 0; i < m; ++i) {
    const double sx = std::fabs(X[3 * i]) + std::fabs(X[3 * i + 1]) + std::fabs(X[3 * i + 2]);
    const double u = y[3 * i] / y[3 * i + 2], v = y[3 * i + 1] / y[3 * i + 2];
    bad = bad || !std::isfinite(sx) || !std::isfinite(u) || !std::isfinite(v);
    a = std::max(a, sx);
    b = std::max(b, std::max(std::fabs(u), std::fabs(v)));
  }
  const double inf = std::numeric_limits<double>::infinity();
  *xmax = bad ? inf : a * (1.0 + 1e-15);
  *umax = bad ? inf : b * (1.0 + 1e-15);
}

extern "C" int rs_pnp_dlt(rs_ctx *c, const double *X, const double *y, int64_t m, double *R_out,
                          double *t_out) {
  if (!c || !X || !y || !R_out || !t_out) return fail(RS_EINVAL, "null pointer");
  if (m < 6) return fail(RS_EINVAL, "the DLT needs m >= 6 correspondences (pnp.py:134)");
  if (m > (1 << 24)) return fail(RS_EINVAL, "too many correspondences");
  HIP_TRY(hipSetDevice(c->device));
  const size_t bin = align256(sizeof(double) * 3 * m), bp = align256(sizeof(rsd::PPt) * m);
  int st = rs::ensure_scratch(c, 2 * bin + bp + 256);
  if (st) return st;
  char *base = static_cast<char *>(c->scratch);
  double *dX = reinterpret_cast<double *>(base), *dy = reinterpret_cast<double *>(base + bin);
  auto *dp = reinterpret_cast<rsd::PPt *>(base + 2 * bin);
  double *dout = reinterpret_cast<double *>(base + 2 * bin + bp);
  HIP_TRY(hipMemcpyAsync(dX, X, sizeof(double) * 3 * m, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(dy, y, sizeof(double) * 3 * m, hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(rsd::k_pack_ppts, dim3((m + 255) / 256), dim3(256), 0, c->stream, dX, dy,
                     static_cast<int>(m), dp);
  HIP_TRY(hipGetLastError());
  hipLaunchKernelGGL(rsd::k_pnp_dlt_all, dim3(1), dim3(64), 0, c->stream, dp,
                     static_cast<int>(m), dout);
  HIP_TRY(hipGetLastError());
  double out[12];
  HIP_TRY(hipMemcpyAsync(out, dout, sizeof(out), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  std::memcpy(R_out, out, sizeof(double) * 9);
  std::memcpy(t_out, out + 9, sizeof(double) * 3);
  return RS_OK;
}

extern "C" int rs_pnp_minimal(rs_ctx *c, const double *X, const double *y, int64_t m,
                              int32_t method, double *R_out, double *t_out, double *err_out) {
  if (!c || !X || !y || !R_out || !t_out) return fail(RS_EINVAL, "null pointer");
  if (method != RS_PNP_EPNP5 && method != RS_PNP_P3P) return fail(RS_EINVAL, "unknown solver");
  if (method == RS_PNP_P3P && m != 4)
    return fail(RS_EINVAL, "P3P takes exactly 4 correspondences (3 to solve, 1 to choose)");
  if (m < 4) return fail(RS_EINVAL, "EPnP needs m >= 4 correspondences");
  if (m > (1 << 24)) return fail(RS_EINVAL, "too many correspondences");
  HIP_TRY(hipSetDevice(c->device));
  const size_t bin = align256(sizeof(double) * 3 * m), bp = align256(sizeof(rsd::PPt) * m);
  int st = rs::ensure_scratch(c, 2 * bin + bp + 256);
  if (st) return st;
  char *base = static_cast<char *>(c->scratch);
  double *dX = reinterpret_cast<double *>(base), *dy = reinterpret_cast<double *>(base + bin);
  auto *dp = reinterpret_cast<rsd::PPt *>(base + 2 * bin);
  double *dout = reinterpret_cast<double *>(base + 2 * bin + bp);
  HIP_TRY(hipMemcpyAsync(dX, X, sizeof(double) * 3 * m, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(dy, y, sizeof(double) * 3 * m, hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(rsd::k_pack_ppts, dim3((m + 255) / 256), dim3(256), 0, c->stream, dX, dy,
                     static_cast<int>(m), dp);
  HIP_TRY(hipGetLastError());
  hipLaunchKernelGGL(rsd::k_pnp_minimal_all, dim3(1), dim3(64), 0, c->stream, dp,
                     static_cast<int>(m), static_cast<int>(method), dout);
  HIP_TRY(hipGetLastError());
  double out[13];
  HIP_TRY(hipMemcpyAsync(out, dout, sizeof(out), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  std::memcpy(R_out, out, sizeof(double) * 9);
  std::memcpy(t_out, out + 9, sizeof(double) * 3);
  if (err_out) *err_out = out[12];
  return RS_OK;
}

extern "C" int rs_pnp_ransac(rs_ctx *c, const double *X_med, const double *y_med, int64_t m_med,
                             const double *X_high, const double *y_high, int64_t m_high,
                             int32_t k, int64_t H, int32_t mode, uint64_t seed,
                             const int32_t *host_tuples, double thresh, rs_pnp_result *out,
                             int64_t *inl_med, int64_t *n_inl_med, int64_t *inl_high,
                             int64_t *n_inl_high) {
  if (!c || !X_med || !y_med || !X_high || !y_high || !out) return fail(RS_EINVAL, "null pointer");
  if (k != 3 && (k < 6 || k > rsd::kMaxK))
    return fail(RS_EINVAL, "sample size must be 3 (P3P) or in [6, 16] (the DLT)");
  if (mode == RS_SAMPLER_PHILOX && k != 6 && k != 3)
    return fail(RS_EINVAL, "Philox sampler draws k = 6 or k = 3");
  if (mode != RS_SAMPLER_PHILOX && mode != RS_SAMPLER_TUPLES) return fail(RS_EINVAL, "bad mode");
  if (m_high < k)
    return fail(RS_EINVAL,
                "Cannot generate more indices than the amount of values in the set from which "
                "they are extracted. n should therefore be smaller or equal to set_length");
  // n = 3: every P3P pose of a trial is a model of its own (k_pnp_solve_p3p)
  const int64_t Hm = k == 3 ? H * rsd::kP3pSlots : H;
  if (m_med < 1 || H < 1 || Hm > (1LL << 28) || m_med > (1 << 26) || m_high > (1 << 26))
    return fail(RS_EINVAL, "bad dimensions");
  if (mode == RS_SAMPLER_TUPLES) {
    if (!host_tuples) return fail(RS_EINVAL, "tuples required");
    for (int64_t i = 0; i < H * k; ++i)
      if (host_tuples[i] < 0 || host_tuples[i] >= m_high)
        return fail(RS_EINVAL, "tuple index out of range");
  }
  HIP_TRY(hipSetDevice(c->device));
  const int64_t ld = (Hm + 63) / 64 * 64;
  const size_t b_in_m = align256(sizeof(double) * 3 * m_med), b_in_h = align256(sizeof(double) * 3 * m_high);
  const size_t b_pm = align256(sizeof(rsd::PPt) * m_med), b_ph = align256(sizeof(rsd::PPt) * m_high);
  const size_t b_tup = align256(sizeof(int) * (mode == RS_SAMPLER_TUPLES ? H * k : 1));
  const size_t b_P = align256(sizeof(double) * 12 * ld), b_cnt = align256(sizeof(int) * ld);
  const size_t b_res = align256(sizeof(rsd::PnpDevResult) + sizeof(int64_t) * (m_med + m_high));
  const size_t b_mir = align256(k == 3 ? static_cast<size_t>(Hm) : 1);
  int st = rs::ensure_scratch(c, 2 * b_in_m + 2 * b_in_h + b_pm + b_ph + b_tup + b_P + b_cnt + b_res +
                                     b_mir);
  if (st) return st;
  char *p = static_cast<char *>(c->scratch);
  auto take = [&p](size_t b) {
    char *q = p;
    p += b;
    return q;
  };
  double *dXm = reinterpret_cast<double *>(take(b_in_m));
  double *dym = reinterpret_cast<double *>(take(b_in_m));
  double *dXh = reinterpret_cast<double *>(take(b_in_h));
  double *dyh = reinterpret_cast<double *>(take(b_in_h));
  auto *pm = reinterpret_cast<rsd::PPt *>(take(b_pm));
  auto *ph = reinterpret_cast<rsd::PPt *>(take(b_ph));
  int *dtup = reinterpret_cast<int *>(take(b_tup));
  double *dP = reinterpret_cast<double *>(take(b_P));
  int *dcnt = reinterpret_cast<int *>(take(b_cnt));
  auto *dres = reinterpret_cast<rsd::PnpDevResult *>(take(b_res));
  auto *dmir = reinterpret_cast<unsigned char *>(take(b_mir));  // P3P poses' mirrored flags
  hipStream_t s = c->stream;
  // the inputs staged contiguously in pinned memory (the layout of the scratch buffers up to the
  // tuples) and sent with one DMA copy; the call synchronises before returning, so the staging
  // is free again for the next call.  The same set as med and high (ransac.py's usual call,
  // D_med = D_high) is sent and packed once.
  const bool same = X_med == X_high && y_med == y_high && m_med == m_high;
  const size_t n_stage = 2 * b_in_m + 2 * b_in_h + b_pm + b_ph + b_tup;
  if ((st = rs::ensure_pinned(c, n_stage))) return st;
  char *hp = static_cast<char *>(c->pinned);
  std::memcpy(hp, X_med, sizeof(double) * 3 * m_med);
  std::memcpy(hp + b_in_m, y_med, sizeof(double) * 3 * m_med);
  size_t up = 2 * b_in_m;
  if (!same) {
    std::memcpy(hp + 2 * b_in_m, X_high, sizeof(double) * 3 * m_high);
    std::memcpy(hp + 2 * b_in_m + b_in_h, y_high, sizeof(double) * 3 * m_high);
    up = 2 * b_in_m + 2 * b_in_h;
  }
  HIP_TRY(hipMemcpyAsync(dXm, hp, up, hipMemcpyHostToDevice, s));
  if (mode == RS_SAMPLER_TUPLES) {
    const size_t to = 2 * b_in_m + 2 * b_in_h + b_pm + b_ph;  // dtup's offset, as in scratch
    std::memcpy(hp + to, host_tuples, sizeof(int) * H * k);
    HIP_TRY(hipMemcpyAsync(dtup, hp + to, sizeof(int) * H * k, hipMemcpyHostToDevice, s));
  }
  hipLaunchKernelGGL(rsd::k_pack_ppts, dim3((m_med + 255) / 256), dim3(256), 0, s, dXm, dym,
                     static_cast<int>(m_med), pm);
  if (same)
    ph = pm;
  else
    hipLaunchKernelGGL(rsd::k_pack_ppts, dim3((m_high + 255) / 256), dim3(256), 0, s, dXh, dyh,
                       static_cast<int>(m_high), ph);
  HIP_TRY(hipMemsetAsync(dcnt, 0, sizeof(int) * Hm, s));
  const bool timed = c->pnp_timing != 0;
  if (timed) HIP_TRY(hipEventRecord(c->pnp_ev[0], s));
  if (k == 3)
    hipLaunchKernelGGL(rsd::k_pnp_solve_p3p, dim3((H + 63) / 64), dim3(64), 0, s, ph,
                       static_cast<int>(m_high), static_cast<int>(H), mode, seed, dtup, dP, ld, dmir);
  else
    hipLaunchKernelGGL(rsd::k_pnp_solve, dim3((H + 255) / 256), dim3(256), 0, s, ph,
                       static_cast<int>(m_high), static_cast<int>(H), k, mode, seed, dtup, dP,
                       ld, 0);
  HIP_TRY(hipGetLastError());
  if (timed) HIP_TRY(hipEventRecord(c->pnp_ev[1], s));
  const int64_t groups = (Hm + 63) / 64;
  int64_t nch = std::max<int64_t>(1, std::min<int64_t>((8192 + groups - 1) / groups, (m_med + 63) / 64));
  const int chunk = static_cast<int>((m_med + nch - 1) / nch);
  nch = (m_med + chunk - 1) / chunk;
  const int64_t units = groups * nch;
  double xmax = 0.0, umax = 0.0;
  pnp_band_bounds(X_med, y_med, m_med, &xmax, &umax);
  hipLaunchKernelGGL(rsd::k_pnp_count<true>, dim3((units + 3) / 4), dim3(256), 0, s, pm,
                     static_cast<int>(m_med), static_cast<int>(Hm), dP, ld, chunk,
                     static_cast<int>(nch), thresh, rsd::PxMetric{1.0, 0.0, 1.0}, xmax, umax,
                     dcnt);
  HIP_TRY(hipGetLastError());
  if (timed) HIP_TRY(hipEventRecord(c->pnp_ev[2], s));
  hipLaunchKernelGGL(rsd::k_pnp_select_inliers, dim3(1), dim3(1024), 0, s, dcnt,
                     static_cast<int>(Hm), dP, ld, dres,
                     k == 3 ? static_cast<const unsigned char *>(dmir) : nullptr, pm,
                     static_cast<int>(m_med), ph, static_cast<int>(m_high), thresh);
  HIP_TRY(hipGetLastError());
  std::vector<char> host(sizeof(rsd::PnpDevResult) + sizeof(int64_t) * (m_med + m_high));
  HIP_TRY(hipMemcpyAsync(host.data(), dres, host.size(), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (timed) {
    float a = 0.f, b = 0.f;
    HIP_TRY(hipEventElapsedTime(&a, c->pnp_ev[0], c->pnp_ev[1]));
    HIP_TRY(hipEventElapsedTime(&b, c->pnp_ev[1], c->pnp_ev[2]));
    c->pnp_solve_ms = a;
    c->pnp_count_ms = b;
  }
  const auto *r = reinterpret_cast<const rsd::PnpDevResult *>(host.data());
  std::memcpy(out->R, r->R, sizeof(out->R));
  std::memcpy(out->t, r->t, sizeof(out->t));
  // n = 3: the trial of the winning pose (its slot: best_index % kP3pSlots on the device)
  out->best_index = k == 3 && r->best_index >= 0 ? r->best_index / rsd::kP3pSlots : r->best_index;
  // the counts are exact in the reference's arithmetic (k_pnp_count<true>), so the winner's
  // count IS the size of its consensus set on D_med (ransac.py:104,108)
  if (r->best_index >= 0 && r->n_med != r->best_count)
    return fail(RS_EDEVICE, "PnP consensus recount mismatch (best_count != |C_med|)");
  out->best_count = r->best_count;
  if (n_inl_med) *n_inl_med = r->n_med;
  if (n_inl_high) *n_inl_high = r->n_high;
  if (inl_med) std::memcpy(inl_med, r->inliers, sizeof(int64_t) * r->n_med);
  if (inl_high) std::memcpy(inl_high, r->inliers + m_med, sizeof(int64_t) * r->n_high);
  return RS_OK;
}

// Consensus counts of given poses (the scoring of ransac.py:96-105 without the sampling): the
// product counting kernel k_pnp_count<true>, so a count here is what rs_pnp_ransac would count
// for that pose.  poses: H x 12 (R row-major, then t).
extern "C" int rs_pnp_count_poses(rs_ctx *c, const double *X, const double *y, int64_t m,
                                  const double *poses, int64_t H, double thresh,
                                  int32_t *counts_out) {
  if (!c || !X || !y || !poses || !counts_out) return fail(RS_EINVAL, "null pointer");
  if (m < 1 || H < 1 || m > (1 << 26) || H > (1LL << 26)) return fail(RS_EINVAL, "bad dimensions");
  HIP_TRY(hipSetDevice(c->device));
  const int64_t ld = (H + 63) / 64 * 64;
  const size_t b_in = align256(sizeof(double) * 3 * m), b_p = align256(sizeof(rsd::PPt) * m);
  const size_t b_P = align256(sizeof(double) * 12 * ld), b_cnt = align256(sizeof(int) * ld);
  int st = rs::ensure_scratch(c, 2 * b_in + b_p + b_P + b_cnt);
  if (st) return st;
  char *p = static_cast<char *>(c->scratch);
  double *dX = reinterpret_cast<double *>(p);
  double *dy = reinterpret_cast<double *>(p + b_in);
  auto *pts = reinterpret_cast<rsd::PPt *>(p + 2 * b_in);
  double *dP = reinterpret_cast<double *>(p + 2 * b_in + b_p);
  int *dcnt = reinterpret_cast<int *>(p + 2 * b_in + b_p + b_P);
  std::vector<double> soa(static_cast<size_t>(12 * ld), 0.0);
  for (int64_t h = 0; h < H; ++h)
    for (int q = 0; q < 12; ++q) soa[static_cast<size_t>(q * ld + h)] = poses[12 * h + q];
  hipStream_t s = c->stream;
  HIP_TRY(hipMemcpyAsync(dX, X, sizeof(double) * 3 * m, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(dy, y, sizeof(double) * 3 * m, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(dP, soa.data(), sizeof(double) * soa.size(), hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(rsd::k_pack_ppts, dim3((m + 255) / 256), dim3(256), 0, s, dX, dy,
                     static_cast<int>(m), pts);
  HIP_TRY(hipMemsetAsync(dcnt, 0, sizeof(int) * H, s));
  const int64_t groups = (H + 63) / 64;
  int64_t nch = std::max<int64_t>(1, std::min<int64_t>((8192 + groups - 1) / groups, (m + 63) / 64));
  const int chunk = static_cast<int>((m + nch - 1) / nch);
  nch = (m + chunk - 1) / chunk;
  const int64_t units = groups * nch;
  double xmax = 0.0, umax = 0.0;
  pnp_band_bounds(X, y, m, &xmax, &umax);
  hipLaunchKernelGGL(rsd::k_pnp_count<true>, dim3((units + 3) / 4), dim3(256), 0, s, pts,
                     static_cast<int>(m), static_cast<int>(H), dP, ld, chunk,
                     static_cast<int>(nch), thresh, rsd::PxMetric{1.0, 0.0, 1.0}, xmax, umax,
                     dcnt);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(counts_out, dcnt, sizeof(int) * H, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  return RS_OK;
}

// OpenCV's RANSACUpdateNumIters (the adaptive stopping rule of cv::solvePnPRansac's RANSAC
// loop): iterations needed to draw one all-inlier sample of `model_points` with probability
// `p` at outlier ratio `ep`, never more than `max_iters`.
static int64_t ransac_update_num_iters(double p, double ep, int model_points, int64_t max_iters) {
  p = std::min(std::max(p, 0.0), 1.0);
  ep = std::min(std::max(ep, 0.0), 1.0);
  double num = std::max(1.0 - p, std::numeric_limits<double>::min());
  double denom = 1.0 - std::pow(1.0 - ep, model_points);
  if (denom < std::numeric_limits<double>::min()) return 0;
  num = std::log(num);
  denom = std::log(denom);
  return (denom >= 0.0 || -num >= static_cast<double>(max_iters) * (-denom))
             ? max_iters
             : static_cast<int64_t>(std::lrint(num / denom));
}

extern "C" int rs_pnp_ransac_cv(rs_ctx *c, const double *X, const double *uv, int64_t m,
                                const double *K, int64_t max_iters, uint64_t seed,
                                double reproj_err, double confidence, int32_t method,
                                const double *guess, rs_pnp_result *out, int64_t *inliers,
                                int64_t *n_inliers, int64_t *iters_used) {
  if (!c || !X || !uv || !K || !out) return fail(RS_EINVAL, "null pointer");
  if (method < RS_PNP_DLT6 || method > RS_PNP_P3P) return fail(RS_EINVAL, "unknown minimal solver");
  const int model_points = method == RS_PNP_DLT6 ? 6 : (method == RS_PNP_EPNP5 ? 5 : 4);
  if (m < model_points)
    return fail(RS_EINVAL, method == RS_PNP_DLT6 ? "the DLT minimal solver needs m >= 6 correspondences"
                                                : "the minimal solver needs more correspondences");
  if (m > (1 << 26) || max_iters < 1 || max_iters > (1LL << 28))
    return fail(RS_EINVAL, "bad dimensions");
  if (!(reproj_err >= 0.0) || !std::isfinite(reproj_err))
    return fail(RS_EINVAL, "reprojectionError must be finite and >= 0");
  if (K[3] != 0.0 || K[6] != 0.0 || K[7] != 0.0 || !(K[8] != 0.0))
    return fail(RS_EINVAL, "cameraMatrix must be upper triangular with K[2,2] != 0");
  const double k8 = K[8];
  const double fx = K[0] / k8, sk = K[1] / k8, cx = K[2] / k8, fy = K[4] / k8, cy = K[5] / k8;
  if (!(fx != 0.0) || !(fy != 0.0) || !std::isfinite(fx * fy * sk * cx * cy))
    return fail(RS_EINVAL, "cameraMatrix must have finite, nonzero fx and fy");
  HIP_TRY(hipSetDevice(c->device));
  // C-normalised homogeneous image points y = K^-1 (u, v, 1) for the DLT
  std::vector<double> yn(3 * m);
  for (int64_t i = 0; i < m; ++i) {
    const double y1 = (uv[2 * i + 1] - cy) / fy;
    yn[3 * i] = (uv[2 * i] - cx - sk * y1) / fx;
    yn[3 * i + 1] = y1;
    yn[3 * i + 2] = 1.0;
  }
  // with an extrinsic guess, hypothesis 0 is the guess and the samples follow
  const int64_t H = max_iters + (guess ? 1 : 0), ld = (H + 63) / 64 * 64;
  const size_t b_in = align256(sizeof(double) * 3 * m), b_p = align256(sizeof(rsd::PPt) * m);
  const size_t b_P = align256(sizeof(double) * 12 * ld), b_cnt = align256(sizeof(int) * ld);
  const size_t b_res = align256(sizeof(rsd::PnpDevResult) + sizeof(int64_t) * m);
  const size_t b_g = align256(sizeof(double) * 12);
  int st = rs::ensure_scratch(c, 2 * b_in + b_p + b_P + b_cnt + b_res + b_g);
  if (st) return st;
  char *p = static_cast<char *>(c->scratch);
  auto take = [&p](size_t b) {
    char *q = p;
    p += b;
    return q;
  };
  double *dX = reinterpret_cast<double *>(take(b_in));
  double *dy = reinterpret_cast<double *>(take(b_in));
  auto *pts = reinterpret_cast<rsd::PPt *>(take(b_p));
  double *dP = reinterpret_cast<double *>(take(b_P));
  int *dcnt = reinterpret_cast<int *>(take(b_cnt));
  auto *dres = reinterpret_cast<rsd::PnpDevResult *>(take(b_res));
  double *dguess = reinterpret_cast<double *>(take(b_g));
  hipStream_t s = c->stream;
  if (guess) HIP_TRY(hipMemcpyAsync(dguess, guess, sizeof(double) * 12, hipMemcpyHostToDevice, s));
  const rsd::PxMetric mt{fx, sk, fy};
  const double thresh = reproj_err * reproj_err;
  HIP_TRY(hipMemcpyAsync(dX, X, sizeof(double) * 3 * m, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(dy, yn.data(), sizeof(double) * 3 * m, hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(rsd::k_pack_ppts, dim3((m + 255) / 256), dim3(256), 0, s, dX, dy,
                     static_cast<int>(m), pts);
  HIP_TRY(hipMemsetAsync(dcnt, 0, sizeof(int) * H, s));
  const int gslot = guess ? 0 : -1;
  if (method == RS_PNP_DLT6) {
    hipLaunchKernelGGL(rsd::k_pnp_solve, dim3((H + 255) / 256), dim3(256), 0, s, pts,
                       static_cast<int>(m), static_cast<int>(H), 6, RS_SAMPLER_PHILOX, seed,
                       static_cast<const int *>(nullptr), dP, ld, 1);
    if (guess) {  // slot 0 (overwritten after the solve, in stream order): the guess
      for (int q = 0; q < 12; ++q)
        HIP_TRY(hipMemcpyAsync(dP + q * ld, dguess + q, sizeof(double), hipMemcpyDeviceToDevice, s));
    }
  } else if (method == RS_PNP_EPNP5) {
    hipLaunchKernelGGL(rsd::k_pnp_solve_min<5>, dim3((H + 63) / 64), dim3(64), 0, s, pts,
                       static_cast<int>(m), static_cast<int>(H), seed, dP, ld, gslot,
                       static_cast<const double *>(dguess));
  } else {
    hipLaunchKernelGGL(rsd::k_pnp_solve_min<4>, dim3((H + 63) / 64), dim3(64), 0, s, pts,
                       static_cast<int>(m), static_cast<int>(H), seed, dP, ld, gslot,
                       static_cast<const double *>(dguess));
  }
  HIP_TRY(hipGetLastError());
  const int64_t groups = (H + 63) / 64;
  int64_t nch = std::max<int64_t>(1, std::min<int64_t>((8192 + groups - 1) / groups, (m + 63) / 64));
  const int chunk = static_cast<int>((m + nch - 1) / nch);
  nch = (m + chunk - 1) / chunk;
  const int64_t units = groups * nch;
  hipLaunchKernelGGL(rsd::k_pnp_count<false>, dim3((units + 3) / 4), dim3(256), 0, s, pts,
                     static_cast<int>(m), static_cast<int>(H), dP, ld, chunk,
                     static_cast<int>(nch), thresh, mt, 0.0, 0.0, dcnt);
  HIP_TRY(hipGetLastError());
  std::vector<int> cnt(H);
  HIP_TRY(hipMemcpyAsync(cnt.data(), dcnt, sizeof(int) * H, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  // OpenCV's sequential loop over the same hypothesis order: a model replaces the best only
  // with goodCount > max(maxGoodCount, modelPoints - 1), and then shrinks the iteration budget
  int64_t niters = H, best = -1, it = 0;
  int good = 0;
  for (; it < niters; ++it) {
    const int g = cnt[it];
    if (g > std::max(good, model_points - 1)) {
      best = it;
      good = g;
      niters = ransac_update_num_iters(confidence, static_cast<double>(m - g) / m, model_points,
                                       niters);
    }
  }
  if (iters_used) *iters_used = it;
  if (best < 0) {
    std::memset(out, 0, sizeof(*out));
    out->best_index = -1;
    if (n_inliers) *n_inliers = 0;
    return RS_OK;
  }
  hipLaunchKernelGGL(rsd::k_pnp_inliers_px, dim3(1), dim3(1024), 0, s, pts, static_cast<int>(m),
                     dP, ld, best, static_cast<int64_t>(good), thresh, mt, dres);
  HIP_TRY(hipGetLastError());
  std::vector<char> host(sizeof(rsd::PnpDevResult) + sizeof(int64_t) * m);
  HIP_TRY(hipMemcpyAsync(host.data(), dres, host.size(), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  const auto *r = reinterpret_cast<const rsd::PnpDevResult *>(host.data());
  if (r->n_med != good) return fail(RS_EDEVICE, "pixel consensus recount mismatch");
  std::memcpy(out->R, r->R, sizeof(out->R));
  std::memcpy(out->t, r->t, sizeof(out->t));
  out->best_index = best;
  out->best_count = good;
  if (n_inliers) *n_inliers = r->n_med;
  if (inliers) std::memcpy(inliers, r->inliers, sizeof(int64_t) * r->n_med);
  return RS_OK;
}

extern "C" int rs_pnp_refine_lm(rs_ctx *c, const double *X, const double *uv, int64_t m,
                                const double *K, double *R_io, double *t_io, int32_t max_jac,
                                double *cost_out) {
  if (!c || !X || !uv || !K || !R_io || !t_io) return fail(RS_EINVAL, "null pointer");
  if (m < 3) return fail(RS_EINVAL, "the refinement needs m >= 3 correspondences");
  if (m > (1 << 24)) return fail(RS_EINVAL, "too many correspondences");
  if (max_jac < 1) return fail(RS_EINVAL, "max_jac must be >= 1");
  if (!(K[8] != 0.0)) return fail(RS_EINVAL, "K[2][2] must be nonzero");
  HIP_TRY(hipSetDevice(c->device));
  const size_t bx = align256(sizeof(double) * 3 * m), bu = align256(sizeof(double) * 2 * m);
  int st = rs::ensure_scratch(c, bx + bu + 256);
  if (st) return st;
  char *base = static_cast<char *>(c->scratch);
  double *dX = reinterpret_cast<double *>(base), *du = reinterpret_cast<double *>(base + bx);
  double *dio = reinterpret_cast<double *>(base + bx + bu);
  double io[16] = {};
  std::memcpy(io, R_io, sizeof(double) * 9);
  std::memcpy(io + 9, t_io, sizeof(double) * 3);
  HIP_TRY(hipMemcpyAsync(dX, X, sizeof(double) * 3 * m, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(du, uv, sizeof(double) * 2 * m, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(dio, io, sizeof(io), hipMemcpyHostToDevice, c->stream));
  const double k22 = K[8];
  const rsd::LmK kk{K[0] / k22, K[1] / k22, K[2] / k22, K[4] / k22, K[5] / k22};
  hipLaunchKernelGGL(rsd::k_pnp_lm, dim3(1), dim3(rsd::kLmThreads), 0, c->stream, dX, du,
                     static_cast<int>(m), kk, dio, static_cast<int>(max_jac),
                     static_cast<double>(std::numeric_limits<float>::epsilon()));
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(io, dio, sizeof(io), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  std::memcpy(R_io, io, sizeof(double) * 9);
  std::memcpy(t_io, io + 9, sizeof(double) * 3);
  if (cost_out) std::memcpy(cost_out, io + 12, sizeof(double) * 4);
  return RS_OK;
}

// HIP events around the solve and the count kernel of rs_pnp_ransac (the bench's C3 roofline):
// enable = 1 records them in the following calls (0 stops); returns the last call's times
// (-1 before any timed call).  No reference counterpart (ransac.py:93-105 is the loop timed).
extern "C" int rs_pnp_timing(rs_ctx *c, int32_t enable, double *solve_ms, double *count_ms) {
  if (!c || !solve_ms || !count_ms) return fail(RS_EINVAL, "null pointer");
  HIP_TRY(hipSetDevice(c->device));
  if (enable && !c->pnp_ev[0])
    for (auto &e : c->pnp_ev) HIP_TRY(hipEventCreate(&e));
  c->pnp_timing = enable ? 1 : 0;
  *solve_ms = c->pnp_solve_ms;
  *count_ms = c->pnp_count_ms;
  return RS_OK;
}
