// Device-side two-view geometry (float64), shared by the triangulation, relative-pose and
// gold-standard kernels (twoview.hip).  Each routine follows the reference function named in
// its comment; matrices are row-major, cameras 3x4.
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>

#include "device_math.h"

namespace rsd {

// ----------------------------------------------------------------------------------------
// small dense helpers
// ----------------------------------------------------------------------------------------
__device__ __forceinline__ void cross3(const double *a, const double *b, double *c) {
  c[0] = a[1] * b[2] - a[2] * b[1];
  c[1] = a[2] * b[0] - a[0] * b[2];
  c[2] = a[0] * b[1] - a[1] * b[0];
}

__device__ __forceinline__ double dot3(const double *a, const double *b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}

__device__ __forceinline__ double det3(const double *m) {
  return m[0] * (m[4] * m[8] - m[5] * m[7]) - m[1] * (m[3] * m[8] - m[5] * m[6]) +
         m[2] * (m[3] * m[7] - m[4] * m[6]);
}

// C = A B (3x3)
__device__ __forceinline__ void mul33(const double *A, const double *B, double *C) {
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c)
      C[3 * r + c] = A[3 * r + 0] * B[c] + A[3 * r + 1] * B[3 + c] + A[3 * r + 2] * B[6 + c];
}

// Unit null vector of a rank-2 3x3 matrix from the best-conditioned cross product of two of
// its rows (right null vector, M n = 0) or columns (left null vector, n^T M = 0).  Equals
// numpy's svd V[-1] / U[:, -1] up to sign.
__device__ __forceinline__ void null3(const double *M, bool left, double *n) {
  double v[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) v[i][j] = left ? M[3 * j + i] : M[3 * i + j];
  double c[3][3];
  cross3(v[0], v[1], c[0]);
  cross3(v[0], v[2], c[1]);
  cross3(v[1], v[2], c[2]);
  const double n0 = dot3(c[0], c[0]), n1 = dot3(c[1], c[1]), n2 = dot3(c[2], c[2]);
  const int k = (n0 >= n1 && n0 >= n2) ? 0 : (n1 >= n2 ? 1 : 2);
  const double nk = k == 0 ? n0 : (k == 1 ? n1 : n2);
  const double s = nk > 0.0 ? 1.0 / sqrt(nk) : 0.0;
  n[0] = c[k][0] * s;
  n[1] = c[k][1] * s;
  n[2] = c[k][2] * s;
}

// Unit null vector of a full-row-rank 3x4 camera (cofactor expansion), sign chosen so that
// n[3] >= 0 -- numpy's svd(C)[2][3] for C = [I | 0] (lab3.py:346).
__device__ __forceinline__ void camera_centre(const double *C, double *n) {
  double m[9];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    int q = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (c == j) continue;
      m[q] = C[c];
      m[3 + q] = C[4 + c];
      m[6 + q] = C[8 + c];
      ++q;
    }
    n[j] = ((j & 1) ? -1.0 : 1.0) * det3(m);
  }
  double s = sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2] + n[3] * n[3]);
  s = s > 0.0 ? 1.0 / s : 0.0;
  if (n[3] < 0.0) s = -s;
#pragma unroll
  for (int j = 0; j < 4; ++j) n[j] *= s;
}

// lab3.fmatrix_from_cameras (lab3.py:331-351): F = [C1 n]_x C1 C2^+,
// C2^+ = C2^T (C2 C2^T)^-1.
__device__ __forceinline__ void fmatrix_from_cameras(const double *C1, const double *C2,
                                                     double *F) {
  double n[4];
  camera_centre(C2, n);
  double e[3];
#pragma unroll
  for (int r = 0; r < 3; ++r)
    e[r] = C1[4 * r] * n[0] + C1[4 * r + 1] * n[1] + C1[4 * r + 2] * n[2] + C1[4 * r + 3] * n[3];
  double G[9], P[9];  // G = C2 C2^T, P = C1 C2^T
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      double g = 0.0, p = 0.0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        g += C2[4 * r + k] * C2[4 * c + k];
        p += C1[4 * r + k] * C2[4 * c + k];
      }
      G[3 * r + c] = g;
      P[3 * r + c] = p;
    }
  double Gi[9];
  Gi[0] = G[4] * G[8] - G[5] * G[7];
  Gi[1] = G[2] * G[7] - G[1] * G[8];
  Gi[2] = G[1] * G[5] - G[2] * G[4];
  Gi[3] = G[5] * G[6] - G[3] * G[8];
  Gi[4] = G[0] * G[8] - G[2] * G[6];
  Gi[5] = G[2] * G[3] - G[0] * G[5];
  Gi[6] = G[3] * G[7] - G[4] * G[6];
  Gi[7] = G[1] * G[6] - G[0] * G[7];
  Gi[8] = G[0] * G[4] - G[1] * G[3];
  const double id = 1.0 / (G[0] * Gi[0] + G[1] * Gi[3] + G[2] * Gi[6]);
#pragma unroll
  for (int i = 0; i < 9; ++i) Gi[i] *= id;
  double M[9];
  mul33(P, Gi, M);
  const double ex[9] = {0.0, -e[2], e[1], e[2], 0.0, -e[0], -e[1], e[0], 0.0};
  mul33(ex, M, F);
}

// lab3.fmatrix_cameras (lab3.py:353-380): C1 = [[e1]_x F | e1], e1 the unit left null
// vector of F (svd U[:, -1]); C2 = [I | 0] is implied.
__device__ __forceinline__ void fmatrix_cameras(const double *F, double *C1) {
  double e[3];
  null3(F, true, e);
  const double ex[9] = {0.0, -e[2], e[1], e[2], 0.0, -e[0], -e[1], e[0], 0.0};
  double A[9];
  mul33(ex, F, A);
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    C1[4 * r + 0] = A[3 * r + 0];
    C1[4 * r + 1] = A[3 * r + 1];
    C1[4 * r + 2] = A[3 * r + 2];
    C1[4 * r + 3] = e[r];
  }
}

#ifndef RSAMD_TRI_JTOL
#define RSAMD_TRI_JTOL 4e-16  // triangulate_linear's Jacobi rotation threshold (A/B: 1e-16)
#endif
// ----------------------------------------------------------------------------------------
// lab3.triangulate_linear (lab3.py:477-503): X = null vector of the 6x4 matrix
// [[x1]_x C1; [x2]_x C2] (numpy svd V[-1]) by one-sided Jacobi on its columns.
// ----------------------------------------------------------------------------------------
template <bool FAST>
__device__ __forceinline__ void triangulate_linear(const double *C1, const double *C2,
                                                   const double *x1, const double *x2,
                                                   double *X) {
  double B[6][4], V[4][4];
  const double *xs[2] = {x1, x2};
  const double *Cs[2] = {C1, C2};
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const double *x = xs[s];
    const double *C = Cs[s];
    const double ex[9] = {0.0, -x[2], x[1], x[2], 0.0, -x[0], -x[1], x[0], 0.0};
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c)
        B[3 * s + r][c] = ex[3 * r] * C[c] + ex[3 * r + 1] * C[4 + c] + ex[3 * r + 2] * C[8 + c];
  }
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) V[r][c] = r == c ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 20; ++sweep) {
    bool rotated = false;
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int q = p + 1; q < 4; ++q) {
        double a = 0.0, b = 0.0, g = 0.0;
#pragma unroll
        for (int r = 0; r < 6; ++r) {
          a += B[r][p] * B[r][p];
          b += B[r][q] * B[r][q];
          g += B[r][p] * B[r][q];
        }
        // (FAST: rotate while the columns' cosine is above ~2 eps.  At 1e-16, below the rounding
        // level of g, a converged matrix keeps rotating by rounding noise to the 20-sweep cap
        // in ~1 % of points, and a wave waits for its slowest lane; FAST takes 5-6 sweeps)
        if (fabs(g) > (FAST ? RSAMD_TRI_JTOL : 1e-16) * sqrt(a * b) && g != 0.0) {
          rotated = true;
          double c, s;
          if constexpr (FAST) {  // (fast reciprocals / square roots, as jacobi_rot)
            const double zeta = (b - a) * (0.5 * rcp_fast(g));
            const double az = fabs(zeta), z2 = fma(zeta, zeta, 1.0);
            const double t = az < 1e150 ? copysign(rcp_fast(az + z2 * rsqrt_fast(z2)), zeta)
                                        : 0.5 * rcp_fast(zeta);
            c = rsqrt_fast(fma(t, t, 1.0));
            s = c * t;
          } else {
            const double zeta = (b - a) / (2.0 * g);
            const double t = copysign(1.0, zeta) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
            c = 1.0 / sqrt(1.0 + t * t);
            s = c * t;
          }
#pragma unroll
          for (int r = 0; r < 6; ++r) {
            const double bp = B[r][p], bq = B[r][q];
            B[r][p] = c * bp - s * bq;
            B[r][q] = s * bp + c * bq;
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const double vp = V[r][p], vq = V[r][q];
            V[r][p] = c * vp - s * vq;
            V[r][q] = s * vp + c * vq;
          }
        }
      }
    if (!rotated) break;
  }
  int m = 0;
  double best = 0.0;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    double s = 0.0;
#pragma unroll
    for (int r = 0; r < 6; ++r) s += B[r][c] * B[r][c];
    if (c == 0 || s < best) {
      best = s;
      m = c;
    }
  }
  double v[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = m == 0 ? V[r][0] : m == 1 ? V[r][1] : m == 2 ? V[r][2] : V[r][3];
  X[0] = v[0] / v[3];
  X[1] = v[1] / v[3];
  X[2] = v[2] / v[3];
}

// ----------------------------------------------------------------------------------------
// numpy.roots semantics for a degree <= 6 real polynomial g[0] t^6 + ... + g[6]: leading
// zeros are stripped, trailing zeros give zero roots (appended last); the other roots by
// Aberth-Ehrlich iteration in complex float64.  Writes the real parts (lab3.py:442 takes
// np.real of every root) and returns how many there are.
//
// Start points: per edge of the Newton polygon (upper convex hull of (k, log|b_k|), b the
// ascending coefficients) m = k2 - k1 points on the circle |z| = (|b_k1| / |b_k2|)^(1/m), so
// roots of very different magnitude (here ~1e-12 .. ~1e8) each start near their own circle.
// A root is frozen once |p(z)| is within the rounding error of its Horner evaluation
// (8 eps sum |a_j| |z|^j) or its correction is below 2 eps |z|; 4-11 sweeps on the goldens.
// ----------------------------------------------------------------------------------------
// Generic degree-N form: g descending (g[0] the z^N coefficient).  Leading zeros lower the
// degree, trailing zeros are roots at 0 (not iterated): returns the iterated degree `deg`,
// with the roots in zr / zi[0 .. deg), and the number of zero roots in `trailing`.
#ifndef RSAMD_ABERTH_MAX
#define RSAMD_ABERTH_MAX 100  // sweep cap (A/B builds may lower it to time the tail)
#endif
// The same iteration with the roots in a run-time-indexed array (scratch memory): the form
// k_triangulate_optimal keeps, because the reference-faithful gold standard (scipy TRF from
// rs_triangulate_optimal's start) is chaotic in the last bits of that start
template <int N>
__device__ __forceinline__ int aberth_roots_serial(const double (&g)[N + 1], double (&zr)[N],
                                            double (&zi)[N], int &trailing) {
  trailing = 0;
  int lo = 0;
  while (lo < N + 1 && g[lo] == 0.0) ++lo;
  if (lo == N + 1) return 0;
  int hi = N;
  while (g[hi] == 0.0) --hi;
  trailing = N - hi;
  const int deg = hi - lo;
  double a[N + 1];  // monic, descending: z^deg + a[1] z^(deg-1) + ... + a[deg]
  for (int k = 0; k <= deg; ++k) a[k] = g[lo + k] / g[lo];
  if (deg > 0) {
    double lg[N + 1];  // log |b_k|, b_k = a[deg - k] (ascending)
    for (int k = 0; k <= deg; ++k) {
      const double v = fabs(a[deg - k]);
      lg[k] = v > 0.0 ? log(v) : -1.0e300;
    }
    int hull[N + 1], nh = 0;
    hull[nh++] = 0;
    for (int k = 1; k <= deg; ++k) {
      if (lg[k] == -1.0e300) continue;
      while (nh >= 2) {
        const int k1 = hull[nh - 2], k2 = hull[nh - 1];
        if ((lg[k2] - lg[k1]) * (k - k1) <= (lg[k] - lg[k1]) * (k2 - k1))
          --nh;
        else
          break;
      }
      hull[nh++] = k;
    }
    int q = 0;
    for (int e = 0; e + 1 < nh; ++e) {
      const int m = hull[e + 1] - hull[e];
      const double rad = exp((lg[hull[e]] - lg[hull[e + 1]]) / m);
      for (int u = 0; u < m; ++u) {
        const double ang = 6.283185307179586 * u / m + 6.283185307179586 * e / deg + 0.4;
        zr[q] = rad * cos(ang);
        zi[q] = rad * sin(ang);
        ++q;
      }
    }
    unsigned conv = 0, all = (1u << deg) - 1u;
    for (int it = 0; it < 100 && conv != all; ++it) {
      for (int k = 0; k < deg; ++k) {
        if (conv & (1u << k)) continue;
        const double xr = zr[k], xi = zi[k];
        const double az = sqrt(xr * xr + xi * xi);
        double pr = 1.0, pi = 0.0, dr = 0.0, di = 0.0, S = 1.0;
        for (int j = 1; j <= deg; ++j) {
          const double ndr = dr * xr - di * xi + pr, ndi = dr * xi + di * xr + pi;
          dr = ndr;
          di = ndi;
          const double npr = pr * xr - pi * xi + a[j], npi = pr * xi + pi * xr;
          pr = npr;
          pi = npi;
          S = S * az + fabs(a[j]);
        }
        if (sqrt(pr * pr + pi * pi) <= 8.0 * 2.220446049250313e-16 * S) {
          conv |= 1u << k;
          continue;
        }
        double rr, ri;  // p / p'
        const double den = dr * dr + di * di;
        if (den == 0.0) {
          rr = pr;
          ri = pi;
        } else {
          rr = (pr * dr + pi * di) / den;
          ri = (pi * dr - pr * di) / den;
        }
        double sr = 0.0, si = 0.0;  // sum_{j != k} 1 / (z_k - z_j)
        for (int j = 0; j < deg; ++j) {
          if (j == k) continue;
          const double ur = xr - zr[j], ui = xi - zi[j];
          const double dd = ur * ur + ui * ui;
          if (dd > 0.0) {
            sr += ur / dd;
            si -= ui / dd;
          }
        }
        const double qr = 1.0 - (rr * sr - ri * si), qi = -(rr * si + ri * sr);
        const double qd = qr * qr + qi * qi;
        double wr = rr, wi = ri;
        if (qd != 0.0) {
          wr = (rr * qr + ri * qi) / qd;
          wi = (ri * qr - rr * qi) / qd;
        }
        zr[k] = xr - wr;
        zi[k] = xi - wi;
        if (fabs(wr) + fabs(wi) <= 2.0 * 2.220446049250313e-16 * (fabs(zr[k]) + fabs(zi[k])))
          conv |= 1u << k;
      }
    }
  }
  return deg;
}

// v[i] for a run-time i < M by a select chain: the array stays in registers (an array indexed
// by a run-time value anywhere lives in scratch memory, and every Aberth sweep then waits on
// memory: k_relative_pose 100 us and the gold standard's triangulation at C4)
template <int M>
__device__ __forceinline__ double pick(const double (&v)[M], int i) {
  double r = v[0];
#pragma unroll
  for (int m = 1; m < M; ++m) r = i == m ? v[m] : r;
  return r;
}

template <int N>
__device__ __forceinline__ int aberth_roots(const double (&g)[N + 1], double (&zr)[N],
                                            double (&zi)[N], int &trailing) {
  trailing = 0;
  int lo = N + 1, hi = 0;
#pragma unroll
  for (int k = N; k >= 0; --k)
    if (g[k] != 0.0) lo = k;  // first non-zero coefficient
  if (lo == N + 1) return 0;
#pragma unroll
  for (int k = 0; k <= N; ++k)
    if (g[k] != 0.0) hi = k;  // last non-zero coefficient
  trailing = N - hi;
  const int deg = hi - lo;
  double a[N + 1];  // monic, descending: z^deg + a[1] z^(deg-1) + ... + a[deg]
  {
    const double g0 = pick(g, lo);
#pragma unroll
    for (int k = 0; k <= N; ++k) a[k] = k <= deg ? pick(g, lo + k) / g0 : 0.0;
  }
  if (deg > 0) {
    double lg[N + 1];  // log |b_k|, b_k = a[deg - k] (ascending)
#pragma unroll
    for (int k = 0; k <= N; ++k) {
      const double v = k <= deg ? fabs(pick(a, deg - k)) : 0.0;
      lg[k] = v > 0.0 ? log(v) : -1.0e300;
    }
    // upper convex hull of (k, lg[k]) as a bit set of its vertices (k = 0 .. deg)
    unsigned hull = 1u;
#pragma unroll
    for (int k = 1; k <= N; ++k) {
      if (k > deg || lg[k] == -1.0e300) continue;
      // pop while the last two vertices and k turn the wrong way
      for (;;) {
        const int k2 = 31 - __builtin_clz(hull);
        if (k2 == 0) break;
        const unsigned rest = hull & ~(1u << k2);
        const int k1 = 31 - __builtin_clz(rest);
        const double l1 = pick(lg, k1), l2 = pick(lg, k2);
        if ((l2 - l1) * (k - k1) <= (lg[k] - l1) * (k2 - k1))
          hull = rest;
        else
          break;
      }
      hull |= 1u << k;
    }
    // m = k2 - k1 start points per hull edge on |z| = (|b_k1| / |b_k2|)^(1/m); root q of the
    // edge e (0-based) at angle 2 pi u / m + 2 pi e / deg + 0.4, in edge order
    {
      int e = 0, k1 = 0;
      unsigned rest = hull & ~1u;
      double rad = 0.0;
      int m = 1, u = 0;
#pragma unroll
      for (int q = 0; q < N; ++q) {
        if (q < deg) {
          if (q == 0 || u == m) {  // next edge
            if (q > 0) {
              ++e;
              k1 += m;
            }
            const int k2 = __builtin_ctz(rest);
            rest &= rest - 1u;
            m = k2 - k1;
            rad = exp((pick(lg, k1) - pick(lg, k2)) / m);
            u = 0;
          }
          const double ang = 6.283185307179586 * u / m + 6.283185307179586 * e / deg + 0.4;
          double sa, ca;
          sincos(ang, &sa, &ca);  // (one range reduction for both)
          zr[q] = rad * ca;
          zi[q] = rad * sa;
          ++u;
        } else {
          zr[q] = 0.0;
          zi[q] = 0.0;
        }
      }
    }
    unsigned conv = 0, all = (1u << deg) - 1u;
    for (int it = 0; it < RSAMD_ABERTH_MAX && conv != all; ++it) {
#pragma unroll
      for (int k = 0; k < N; ++k) {
        if (k >= deg || (conv & (1u << k))) continue;
        const double xr = zr[k], xi = zi[k];
        const double az = sqrt(xr * xr + xi * xi);
        double pr = 1.0, pi = 0.0, dr = 0.0, di = 0.0, S = 1.0;
#pragma unroll
        for (int j = 1; j <= N; ++j) {
          if (j > deg) break;
          const double ndr = dr * xr - di * xi + pr, ndi = dr * xi + di * xr + pi;
          dr = ndr;
          di = ndi;
          const double npr = pr * xr - pi * xi + a[j], npi = pr * xi + pi * xr;
          pr = npr;
          pi = npi;
          S = S * az + fabs(a[j]);
        }
        if (sqrt(pr * pr + pi * pi) <= 8.0 * 2.220446049250313e-16 * S) {
          conv |= 1u << k;
          continue;
        }
        double rr, ri;  // p / p'
        const double den = dr * dr + di * di;
        if (den == 0.0) {
          rr = pr;
          ri = pi;
        } else {  // (one reciprocal, a few ulp: rcp_fast)
          const double iden = rcp_fast(den);
          rr = (pr * dr + pi * di) * iden;
          ri = (pi * dr - pr * di) * iden;
        }
        double sr = 0.0, si = 0.0;  // sum_{j != k} 1 / (z_k - z_j)
#pragma unroll
        for (int j = 0; j < N; ++j) {
          if (j == k || j >= deg) continue;
          const double ur = xr - zr[j], ui = xi - zi[j];
          const double dd = ur * ur + ui * ui;
          if (dd > 0.0) {
            const double idd = rcp_fast(dd);
            sr += ur * idd;
            si -= ui * idd;
          }
        }
        const double qr = 1.0 - (rr * sr - ri * si), qi = -(rr * si + ri * sr);
        const double qd = qr * qr + qi * qi;
        double wr = rr, wi = ri;
        if (qd != 0.0) {
          const double iqd = rcp_fast(qd);
          wr = (rr * qr + ri * qi) * iqd;
          wi = (ri * qr - rr * qi) * iqd;
        }
        zr[k] = xr - wr;
        zi[k] = xi - wi;
        if (fabs(wr) + fabs(wi) <= 2.0 * 2.220446049250313e-16 * (fabs(zr[k]) + fabs(zi[k])))
          conv |= 1u << k;
      }
    }
  }
  return deg;
}

template <bool FAST>
__device__ __forceinline__ int roots_real_parts(const double (&g)[7], double (&out)[6]) {
  double zr[6], zi[6];
  int trailing = 0;
  if constexpr (FAST) {
    const int deg = aberth_roots<6>(g, zr, zi, trailing);
    // the iterated roots, then `trailing` zero roots (zr is 0 beyond deg)
#pragma unroll
    for (int k = 0; k < 6; ++k) out[k] = k < deg ? zr[k] : 0.0;
    return deg + trailing;
  } else {
    const int deg = aberth_roots_serial<6>(g, zr, zi, trailing);
    for (int k = 0; k < deg; ++k) out[k] = zr[k];
    for (int k = 0; k < trailing; ++k) out[deg + k] = 0.0;
    return deg + trailing;
  }
}

// ----------------------------------------------------------------------------------------
// lab3.triangulate_optimal (lab3.py:382-475), f1 = f2 = 1: both points moved to the origin,
// epipoles rotated onto the x axis, the degree-6 polynomial of Klas Nordberg's code, cost at
// the real part of every root and at t = inf, the argmin (first NaN wins, as np.argmin), the
// closest points on the two lines, back-transfer, linear triangulation.
// ----------------------------------------------------------------------------------------
// FAST (k_relative_pose, which reads only the depth signs, and the LM gold standard
// k_gold_standard, whose start it is): register-resident roots, fast reciprocals and the 2-eps
// Jacobi stop -- the same points to rounding (the LM start's cost equals the reference start's to
// 1e-9, test_gpu_twoview.py), not bit for bit; else the arithmetic of rs_triangulate_optimal
// (the reference-faithful TRF path's start, bit-reproducible against lab3.triangulate_optimal's
// order).
template <bool FAST = false>
__device__ __forceinline__ void triangulate_optimal(const double *C1, const double *C2,
                                                    double x1, double y1, double x2, double y2,
                                                    double *X) {
  double F0[9];
  fmatrix_from_cameras(C1, C2, F0);
  // F = T1^T F0 T2 with T = [[1, 0, x], [0, 1, y], [0, 0, 1]]
  double F[9];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    F[3 * r + 0] = F0[3 * r + 0];
    F[3 * r + 1] = F0[3 * r + 1];
    F[3 * r + 2] = F0[3 * r + 0] * x2 + F0[3 * r + 1] * y2 + F0[3 * r + 2];
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) F[6 + c] = x1 * F[c] + y1 * F[3 + c] + F[6 + c];
  // epipoles (lab3.fmatrix_epipoles): e1 = U[:, -1], e2 = V[-1], dehomogenised, unit 2D
  double e1[3], e2[3];
  null3(F, true, e1);
  null3(F, false, e2);
  double u0 = e1[0] / e1[2], u1 = e1[1] / e1[2];
  double w0 = e2[0] / e2[2], w1 = e2[1] / e2[2];
  double nu = sqrt(u0 * u0 + u1 * u1), nw = sqrt(w0 * w0 + w1 * w1);
  u0 /= nu;
  u1 /= nu;
  w0 /= nw;
  w1 /= nw;
  const double R1[9] = {u0, u1, 0.0, -u1, u0, 0.0, 0.0, 0.0, 1.0};
  const double R2t[9] = {w0, -w1, 0.0, w1, w0, 0.0, 0.0, 0.0, 1.0};  // R2^T
  double T[9], G[9];
  mul33(F, R2t, T);
  mul33(R1, T, G);
  const double a = G[4], b = G[5], c = G[7], d = G[8];
  const double k1 = b * c - a * d;
  const double ac2 = a * a + c * c;
  double g[7];
  g[0] = a * c * k1;
  g[1] = ac2 * ac2 + k1 * (b * c + a * d);
  g[2] = 4 * ac2 * (a * b + c * d) + 2 * a * c * k1 + b * d * k1;
  g[3] = 2 * (4 * a * b * c * d + a * a * (3 * b * b) + c * c * (3 * d * d + b * b * 2));
  g[4] = -a * a * c * d + a * b * (4 * b * b + c * c + 4 * d * d - 2 * d * d) +
         2 * c * d * (2 * d * d + b * b * 3);
  g[5] = b * b * b * b - a * a * d * d + d * d * d * d + b * b * (c * c + 2 * d * d);
  g[6] = b * d * k1;
  double r[6];
  const int nr = roots_real_parts<FAST>(g, r);
  int best = -1;
  double bs = 0.0;
  bool nan_seen = false;
#pragma unroll
  for (int i = 0; i <= 6; ++i) {
    if (i > nr) break;
    double s;
    if (i < nr) {
      const double t = r[i];
      const double ct = c * t + d, at = a * t + b;
      s = t * t / (1 + t * t) + ct * ct / (at * at + ct * ct);
    } else {
      s = 1.0 + c * c / (a * a + c * c);
    }
    if (nan_seen) continue;
    if (s != s) {
      best = i;
      nan_seen = true;
    } else if (best < 0 || s < bs) {
      best = i;
      bs = s;
    }
  }
  double l1[3], l2[3];
  if (best < nr) {
    const double tm = pick(r, best);
    l1[0] = -(c * tm + d);
    l1[1] = a * tm + b;
    l1[2] = c * tm + d;
    l2[0] = tm;
    l2[1] = 1.0;
    l2[2] = -tm;
  } else {
    l1[0] = -c;
    l1[1] = a;
    l1[2] = c;
    l2[0] = 1.0;
    l2[1] = 0.0;
    l2[2] = -1.0;
  }
  const double q1[3] = {-l1[0] * l1[2], -l1[1] * l1[2], l1[0] * l1[0] + l1[1] * l1[1]};
  const double q2[3] = {-l2[0] * l2[2], -l2[1] * l2[2], l2[0] * l2[0] + l2[1] * l2[1]};
  // x_new = T R^T q;  R1^T = [[u0, -u1, 0], [u1, u0, 0], [0, 0, 1]]
  double p1[3], p2[3];
  p1[0] = u0 * q1[0] - u1 * q1[1];
  p1[1] = u1 * q1[0] + u0 * q1[1];
  p1[2] = q1[2];
  p1[0] += x1 * p1[2];
  p1[1] += y1 * p1[2];
  p2[0] = w0 * q2[0] - w1 * q2[1];
  p2[1] = w1 * q2[0] + w0 * q2[1];
  p2[2] = q2[2];
  p2[0] += x2 * p2[2];
  p2[1] += y2 * p2[2];
  triangulate_linear<FAST>(C1, C2, p1, p2, X);
}

}  // namespace rsd
