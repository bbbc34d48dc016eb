// Five-point essential matrix (Nister 2004) and E-RANSAC for gfx950 (SURVEY.md 8(a) row a-15;
// no reference counterpart: parity unpinned, known answers from the reference's BAdino2 scene,
// oracle/essential_ref.py).
//
// Convention of the reference (fun.py:12-21, lab3.fmatrix_residuals): y1^T E y2 = 0 for
// C-normalised points y1 (left) and y2 (right), E = R^T [t]_x for x2 = R x1 + t; pixel
// points x = K y, so F = K1^-T E K2^-1 satisfies x1^T F x2 = 0.
//
//   solve        three kernels per batch of minimal samples of 5 correspondences:
//                k_e5_build (lane per sample)
//                  1. Q (5 x 9), row i = vec(y1_i y2_i^T); Householder LQ of its rows, null
//                     basis {X, Y, Z, W} = H_0 .. H_4 e_{5..8}: E = x X + y Y + z Z + W
//                     (to memory);
//                  2. the ten cubics det E = 0 and 2 E E^T E - tr(E E^T) E = 0 over the 20
//                     monomials (Nister's order, kT3), to memory row by row;
//                k_e5_gj (32 lanes per sample, a column per lane): Gauss-Jordan with partial
//                  pivoting on the first ten columns -> [I | B];
//                k_e5_roots (16 lanes per sample, lane r owns root r)
//                  3. k = row(x^2 z) - z row(x^2), l = row(y^2 z) - z row(y^2),
//                     m = row(x y z) - z row(x y): linear in (x, y, 1), polynomial in z;
//                     det [k; l; m](z) has degree 10;
//                  4. its roots by Aberth-Ehrlich (the start points and freeze tests of
//                     twoview_math.h aberth_roots, the other roots read across the row by DPP),
//                     real ones polished by Newton; (x, y, 1) = the null vector of
//                     [k; l; m](z) (the row cross product with the largest third component);
//                writes up to 10 unit-norm E per sample, their F = K1^-T E K2^-1 (NaN slots
//                past the sample's count, so they count 0).  (One lane per sample for all of it
//                held the 10 x 20 system in 256 VGPRs + 256 AGPRs + 752 B of scratch.)
//   counting     k_e5_pack: a dense list of the real solutions' slots; k_f8_count
//                (f8_kernels.hip) over the models it names: the reference's residual
//                test d = max(|r1|, |r2|) < thresh of lab3.fmatrix_residuals in pixels.
//   k_e5_select  c* = the largest count; among the slots with c* the smallest residual norm
//                ||d||, d_i = max(|r1_i|, |r2_i|) over all points (the quantity the
//                reference's F loop compares on ties, fun.py:317-325), first slot on equal norms.
//                Then, in the same launch, the winner's consensus set in point order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "common.h"
#include "ctx.h"
#include "device_math.h"
#include "f8_kernels.h"
#include "twoview_math.h"

namespace rsd {

// monomial products: degree-1 [x, y, z, 1] x degree-1 -> degree-2
// [xx, xy, xz, x, yy, yz, y, zz, z, 1]; degree-2 x degree-1 -> Nister's 20 cubic monomials
// [x3, y3, x2y, xy2, x2z, x2, y2z, y2, xyz, xy | xz2, xz, x, yz2, yz, y, z3, z2, z, 1]
__constant__ constexpr int kT2[4][4] = {{0, 1, 2, 3}, {1, 4, 5, 6}, {2, 5, 7, 8}, {3, 6, 8, 9}};
__constant__ constexpr int kT3[10][4] = {{0, 2, 4, 5},    {2, 3, 8, 9},    {4, 8, 10, 11},
                                         {5, 9, 11, 12},  {3, 1, 6, 7},    {8, 6, 13, 14},
                                         {9, 7, 14, 15},  {10, 13, 16, 17}, {11, 14, 17, 18},
                                         {12, 15, 18, 19}};

constexpr int kE5Sol = 10;  // solution slots per sample

struct P1 {
  double c[4];
};
struct P2 {
  double c[10];
};

__device__ __forceinline__ P2 mul11(const P1 &a, const P1 &b) {
  P2 r;
#pragma unroll
  for (int i = 0; i < 10; ++i) r.c[i] = 0.0;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) r.c[kT2[i][j]] = fma(a.c[i], b.c[j], r.c[kT2[i][j]]);
  return r;
}

// acc += s * (a b), a of degree 2, b of degree 1
__device__ __forceinline__ void fma21(double (&acc)[20], double s, const P2 &a, const P1 &b) {
#pragma unroll
  for (int i = 0; i < 10; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[kT3[i][j]] = fma(s * a.c[i], b.c[j], acc[kT3[i][j]]);
}

// Null basis of the 5 x 9 epipolar constraint matrix by Householder LQ (rows reduced left to
// right); basis[j] = H_0 H_1 .. H_4 e_{5+j}, orthonormal.
__device__ __forceinline__ void e5_null_basis(double (&A)[5][9], double (&basis)[4][9]) {
  double tau[5];
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    double ss = 0.0;
#pragma unroll
    for (int j = k; j < 9; ++j) ss = fma(A[k][j], A[k][j], ss);
    const double nrm = sqrt(ss);
    const double akk = A[k][k];
    const double alpha = akk >= 0.0 ? -nrm : nrm;
    const double denom = nrm * (nrm + fabs(akk));
    const double tk = denom > 0.0 ? 1.0 / denom : 0.0;
    A[k][k] = akk - alpha;
    tau[k] = tk;
#pragma unroll
    for (int i = k + 1; i < 5; ++i) {
      double w = 0.0;
#pragma unroll
      for (int j = k; j < 9; ++j) w = fma(A[i][j], A[k][j], w);
      w *= tk;
#pragma unroll
      for (int j = k; j < 9; ++j) A[i][j] = fma(-w, A[k][j], A[i][j]);
    }
  }
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    double q[9];
#pragma unroll
    for (int j = 0; j < 9; ++j) q[j] = (j == 5 + b) ? 1.0 : 0.0;
#pragma unroll
    for (int k = 4; k >= 0; --k) {
      double w = 0.0;
#pragma unroll
      for (int j = k; j < 9; ++j) w = fma(A[k][j], q[j], w);
      w *= tau[k];
#pragma unroll
      for (int j = k; j < 9; ++j) q[j] = fma(-w, A[k][j], q[j]);
    }
#pragma unroll
    for (int j = 0; j < 9; ++j) basis[b][j] = q[j];
  }
}

// The ten cubic constraints (rows 0-8: 2 E E^T E - tr(E E^T) E, row 9: det E), each row of 20
// coefficients handed to sink(row, coefficients) as it is formed.
template <class Sink>
__device__ __forceinline__ void e5_constraints(const double (&basis)[4][9], Sink sink) {
  P1 E[9];
#pragma unroll
  for (int e = 0; e < 9; ++e) {
    E[e].c[0] = basis[0][e];
    E[e].c[1] = basis[1][e];
    E[e].c[2] = basis[2][e];
    E[e].c[3] = basis[3][e];
  }
  P2 EEt[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = i; j < 3; ++j) {
      P2 s = mul11(E[3 * i], E[3 * j]);
      const P2 s1 = mul11(E[3 * i + 1], E[3 * j + 1]);
      const P2 s2 = mul11(E[3 * i + 2], E[3 * j + 2]);
#pragma unroll
      for (int q = 0; q < 10; ++q) s.c[q] = (s.c[q] + s1.c[q]) + s2.c[q];
      EEt[i][j] = s;
      EEt[j][i] = s;
    }
  P2 tr;
#pragma unroll
  for (int q = 0; q < 10; ++q) tr.c[q] = (EEt[0][0].c[q] + EEt[1][1].c[q]) + EEt[2][2].c[q];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      double acc[20];
#pragma unroll
      for (int q = 0; q < 20; ++q) acc[q] = 0.0;
#pragma unroll
      for (int k = 0; k < 3; ++k) fma21(acc, 2.0, EEt[i][k], E[3 * k + j]);
      fma21(acc, -1.0, tr, E[3 * i + j]);
      sink(3 * i + j, acc);
    }
  double det[20];
#pragma unroll
  for (int q = 0; q < 20; ++q) det[q] = 0.0;
  const P2 c0 = mul11(E[4], E[8]), c0b = mul11(E[5], E[7]);  // E11 E22 - E12 E21
  const P2 c1 = mul11(E[3], E[8]), c1b = mul11(E[5], E[6]);  // E10 E22 - E12 E20
  const P2 c2 = mul11(E[3], E[7]), c2b = mul11(E[4], E[6]);  // E10 E21 - E11 E20
  fma21(det, 1.0, c0, E[0]);
  fma21(det, -1.0, c0b, E[0]);
  fma21(det, -1.0, c1, E[1]);
  fma21(det, 1.0, c1b, E[1]);
  fma21(det, 1.0, c2, E[2]);
  fma21(det, -1.0, c2b, E[2]);
  sink(9, det);
}

template <int A, int B>
__device__ __forceinline__ void polymul(const double (&a)[A], const double (&b)[B],
                                        double (&r)[A + B - 1]) {
#pragma unroll
  for (int i = 0; i < A + B - 1; ++i) r[i] = 0.0;
#pragma unroll
  for (int i = 0; i < A; ++i)
#pragma unroll
    for (int j = 0; j < B; ++j) r[i + j] = fma(a[i], b[j], r[i + j]);
}

// row(a) - z row(b) of the reduced system [I | B] (Bm holds B's rows 4..9): coefficients of x,
// y and 1, ascending in z
__device__ __forceinline__ void e5_row(const double (&Bm)[6][10], int a, int b, double (&px)[4],
                                       double (&py)[4], double (&p1)[5]) {
  const double *A = Bm[a - 4], *Bb = Bm[b - 4];
  px[0] = A[2];
  px[1] = A[1] - Bb[2];
  px[2] = A[0] - Bb[1];
  px[3] = -Bb[0];
  py[0] = A[5];
  py[1] = A[4] - Bb[5];
  py[2] = A[3] - Bb[4];
  py[3] = -Bb[3];
  p1[0] = A[9];
  p1[1] = A[8] - Bb[9];
  p1[2] = A[7] - Bb[8];
  p1[3] = A[6] - Bb[7];
  p1[4] = -Bb[6];
}

template <int N>
__device__ __forceinline__ double horner_asc(const double (&p)[N], double z) {
  double v = p[N - 1];
#pragma unroll
  for (int i = N - 2; i >= 0; --i) v = fma(v, z, p[i]);
  return v;
}

// The three rows k, l, m of one sample (linear in (x, y, 1), polynomial in z) from B's rows
// 4..9, and d(z) = det [k; l; m] (degree 10, ascending).
struct E5Polys {
  double kx[4], ky[4], k1[5], lx[4], ly[4], l1[5], mx[4], my[4], m1[5];
};

__device__ __forceinline__ void e5_polys(const double (&Bm)[6][10], E5Polys &P, double (&d)[11]) {
  e5_row(Bm, 4, 5, P.kx, P.ky, P.k1);
  e5_row(Bm, 6, 7, P.lx, P.ly, P.l1);
  e5_row(Bm, 8, 9, P.mx, P.my, P.m1);
  // det [k; l; m] = kx (ly m1 - l1 my) - ky (lx m1 - l1 mx) + k1 (lx my - ly mx)
  double t7a[8], t7b[8], t7[8], u[11];
  polymul(P.ly, P.m1, t7a);
  polymul(P.l1, P.my, t7b);
#pragma unroll
  for (int i = 0; i < 8; ++i) t7[i] = t7a[i] - t7b[i];
  polymul(P.kx, t7, d);
  polymul(P.lx, P.m1, t7a);
  polymul(P.l1, P.mx, t7b);
#pragma unroll
  for (int i = 0; i < 8; ++i) t7[i] = t7a[i] - t7b[i];
  polymul(P.ky, t7, u);
#pragma unroll
  for (int i = 0; i < 11; ++i) d[i] -= u[i];
  double t6a[7], t6b[7], t6[7];
  polymul(P.lx, P.my, t6a);
  polymul(P.ly, P.mx, t6b);
#pragma unroll
  for (int i = 0; i < 7; ++i) t6[i] = t6a[i] - t6b[i];
  polymul(P.k1, t6, u);
#pragma unroll
  for (int i = 0; i < 11; ++i) d[i] += u[i];
}

// The solution of one root z of d (Newton-polished on the real axis): (x, y, 1) = the row cross
// product of [k; l; m](z) with the largest third component (first on ties), E = x X + y Y +
// z Z + W from the null basis in memory, unit norm.  False when it degenerates.
// (d and the rows' polynomials read from memory, pg = k_e5_polys' column of the sample with
// stride ldp: the kernel's register peak was the 50 doubles held at once)
template <int N>
__device__ __forceinline__ double horner_mem(const double *p, int64_t ld, double z) {
  double q[N];
#pragma unroll
  for (int i = 0; i < N; ++i) q[i] = p[i * ld];
  return horner_asc(q, z);
}
__device__ __forceinline__ bool e5_solution(const double *pg, int64_t ldp, double z,
                                            const double *bas, int64_t ldb, double (&E)[9]) {
  double d[11];
#pragma unroll
  for (int i = 0; i < 11; ++i) d[i] = pg[i * ldp];
  // Newton polish on the real axis (the complex iteration may stop at its rounding floor)
  for (int it = 0; it < 3; ++it) {
    double fp = 10 * d[10];  // the derivative, ascending (i + 1) d[i + 1], by Horner
#pragma unroll
    for (int i = 8; i >= 0; --i) fp = fma(fp, z, (i + 1) * d[i + 1]);
    const double f = horner_asc(d, z);
    if (!(fp != 0.0)) break;
    const double step = f / fp;
    if (!(fabs(step) <= 1e-3 * fmax(1.0, fabs(z)))) break;
    z -= step;
  }
  const double *P = pg + 11 * ldp;  // kx ky k1 lx ly l1 mx my m1: 4 4 5 4 4 5 4 4 5 doubles
  const double A0[3] = {horner_mem<4>(P, ldp, z), horner_mem<4>(P + 4 * ldp, ldp, z),
                        horner_mem<5>(P + 8 * ldp, ldp, z)};
  const double A1[3] = {horner_mem<4>(P + 13 * ldp, ldp, z), horner_mem<4>(P + 17 * ldp, ldp, z),
                        horner_mem<5>(P + 21 * ldp, ldp, z)};
  const double A2[3] = {horner_mem<4>(P + 26 * ldp, ldp, z), horner_mem<4>(P + 30 * ldp, ldp, z),
                        horner_mem<5>(P + 34 * ldp, ldp, z)};
  double v0 = 0.0, v1 = 0.0, v2 = 0.0, bz = -1.0;
  auto cand = [&](const double (&a)[3], const double (&b)[3]) {
    const double c0 = a[1] * b[2] - a[2] * b[1];
    const double c1 = a[2] * b[0] - a[0] * b[2];
    const double c2 = a[0] * b[1] - a[1] * b[0];
    if (fabs(c2) > bz) {
      bz = fabs(c2);
      v0 = c0;
      v1 = c1;
      v2 = c2;
    }
  };
  cand(A0, A1);
  cand(A0, A2);
  cand(A1, A2);
  if (!(bz > 0.0)) return false;
  const double x = v0 / v2, y = v1 / v2;
  double nn = 0.0;
#pragma unroll
  for (int e = 0; e < 9; ++e) {
    E[e] = fma(x, bas[e * ldb], fma(y, bas[(9 + e) * ldb], fma(z, bas[(18 + e) * ldb], bas[(27 + e) * ldb])));
    nn = fma(E[e], E[e], nn);
  }
  if (!(nn > 0.0) || !isfinite(nn)) return false;
  const double in = 1.0 / sqrt(nn);
#pragma unroll
  for (int e = 0; e < 9; ++e) E[e] *= in;
  return true;
}

// (x, y) of the 16-lane row neighbour k to the left (DPP row_ror:k; every lane of the row
// must be active)
template <int K>
__device__ __forceinline__ void row_ror_pair(double xr, double xi, double &yr, double &yi) {
  auto rot = [](double v) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const unsigned lo = __builtin_amdgcn_update_dpp(0u, static_cast<unsigned>(b), 0x120 + K, 0xf, 0xf, false);
    const unsigned hi = __builtin_amdgcn_update_dpp(0u, static_cast<unsigned>(b >> 32), 0x120 + K, 0xf, 0xf, false);
    return __builtin_bit_cast(double, (static_cast<uint64_t>(hi) << 32) | lo);
  };
  yr = rot(xr);
  yi = rot(xi);
}

// sum over the other 15 lanes of the row of 1 / (z - z_j); lanes without a root hold NaN, which
// fails dd > 0 (as a coincident root does in aberth_roots)
template <int K>
__device__ __forceinline__ void aberth_sum(double xr, double xi, double &sr, double &si) {
  if constexpr (K < 16) {
    double yr, yi;
    row_ror_pair<K>(xr, xi, yr, yi);
    const double ur = xr - yr, ui = xi - yi;
    const double dd = ur * ur + ui * ui;
    if (dd > 0.0) {
      // the sum only shapes the step (the fixed point is p(z) = 0): v_rcp_f64 and one
      // Newton step instead of two IEEE divisions
      const double r0 = __builtin_amdgcn_rcp(dd);
      const double inv = r0 * fma(-dd, r0, 2.0);
      sr = fma(ur, inv, sr);
      si = fma(-ui, inv, si);
    }
    aberth_sum<K + 1>(xr, xi, sr, si);
  }
}

struct E5Args {
  const Pt *pts;            // pixel points (ransac) or C-normalised points (direct solve)
  int n, S, mode;           // mode: 0 Philox samples of the n points, 1 consecutive fives
  uint64_t seed;
  double Kin1[9], Kin2[9];  // pixel -> normalised (K^-1), identity for the direct solve
  double M1[9], M2[9];      // F = M1 E M2 (K1^-T, K2^-1)
  double *Esoa;             // 9 x ld models (ld >= 10 S), NaN past the sample's count
  double *Fsoa;             // 9 x ld (may be null)
  int *nsol;                // per sample (may be null)
  int64_t ld;
  // work between the three solve kernels (ldw >= S, sample-minor so each kernel's loads and
  // stores coalesce over its lanes): the 10 x 20 system (200 x ldw), the null basis
  // (36 x ldw), B's rows 4..9 (60 x ldw), Gauss-Jordan success (ldw)
  double *Mg, *Bas, *Bg;
  // d(z) and the three rows' polynomials per sample (k_e5_polys; 50 x ldw: d ascending, then
  // kx ky k1 lx ly l1 mx my m1 as in E5Polys), in Mg's space once Gauss-Jordan is done
  double *Pg;
  int *okg;
  int64_t ldw;
  // two-phase root finding (k_e5_roots): after `split` sweeps the samples whose roots are still
  // moving leave their root state (zr, zi, converged per lane: 3 x 16 doubles) in zst and their
  // index in defer_list; phase 2 resumes them packed four to a wave (split = 0: one phase)
  int split;
  int *defer_list, *defer_n;
  double *zst;
};

__device__ __forceinline__ void norm_pt(const double (&K)[9], double u, double v, double &x,
                                        double &y) {
  const double w = fma(K[6], u, fma(K[7], v, K[8]));
  x = fma(K[0], u, fma(K[1], v, K[2])) / w;
  y = fma(K[3], u, fma(K[4], v, K[5])) / w;
}

// (A) lane per sample: the sample, its 5 x 9 constraint matrix, the null basis (to memory) and
// the ten cubic constraints (to memory, row by row: the 10 x 20 system is 400 of the 512
// registers a lane has, so it is never held by one lane)
__global__ __launch_bounds__(64) void k_e5_build(E5Args a) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= a.S) return;
  int idx[5];
  if (a.mode == 0) {
    floyd_sample<5>(a.seed, static_cast<uint64_t>(s), a.n, idx);
  } else {
#pragma unroll
    for (int i = 0; i < 5; ++i) idx[i] = 5 * s + i;
  }
  double Q[5][9];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const Pt p = a.pts[idx[i]];
    double a0, a1, b0, b1;
    norm_pt(a.Kin1, p.x1, p.y1, a0, a1);
    norm_pt(a.Kin2, p.x2, p.y2, b0, b1);
    Q[i][0] = a0 * b0;
    Q[i][1] = a0 * b1;
    Q[i][2] = a0;
    Q[i][3] = a1 * b0;
    Q[i][4] = a1 * b1;
    Q[i][5] = a1;
    Q[i][6] = b0;
    Q[i][7] = b1;
    Q[i][8] = 1.0;
  }
  double basis[4][9];
  e5_null_basis(Q, basis);
#pragma unroll
  for (int b = 0; b < 4; ++b)
#pragma unroll
    for (int e = 0; e < 9; ++e) a.Bas[(9 * b + e) * a.ldw + s] = basis[b][e];
  double *M = a.Mg + s;
  const int64_t ldw = a.ldw;
  e5_constraints(basis, [&](int r, const double (&row)[20]) {
#pragma unroll
    for (int q = 0; q < 20; ++q) M[(20 * r + q) * ldw] = row[q];
  });
}

// (B) Gauss-Jordan on the first ten columns with partial pivoting, two samples per wave: lane j
// (< 20) of a 32-lane half holds column j of its sample's system; the pivot column's lane finds
// the pivot (the first largest |M[r][c]|, r >= c), and its column (the multipliers) and 1 /
// pivot are broadcast by shuffles.  Every element sees the same operations as a one-lane
// elimination: M[c][j] *= 1 / M[c][c], M[r][j] = fma(-M[r][c], M[c][j], M[r][j]).
__global__ __launch_bounds__(64) void k_e5_gj(E5Args a) {
  const int lane = threadIdx.x & 63, g = lane >> 5, j = lane & 31;
  const int s = blockIdx.x * 2 + g;
  const bool own = s < a.S && j < 20;
  const int64_t ldw = a.ldw;
  double col[10];
#pragma unroll
  for (int r = 0; r < 10; ++r) col[r] = own ? a.Mg[(20 * r + j) * ldw + s] : 0.0;
  bool ok = true;
#pragma unroll
  for (int c = 0; c < 10; ++c) {
    const int src = (g << 5) + c;
    int piv = c;
    double best = fabs(col[c]);
#pragma unroll
    for (int r = c + 1; r < 10; ++r) {
      const double v = fabs(col[r]);
      if (v > best) {
        best = v;
        piv = r;
      }
    }
    piv = __shfl(piv, src);
    best = __shfl(best, src);
    ok = ok && best > 0.0;
    // swap rows c and piv (a no-op on the reduced columns j < c, zero in both rows)
    double pc = col[c];
#pragma unroll
    for (int r = c + 1; r < 10; ++r) {
      const bool sw = r == piv;
      const double x = col[r];
      col[r] = sw ? pc : x;
      pc = sw ? x : pc;
    }
    col[c] = pc;
    const double inv = __shfl(1.0 / col[c], src);
    double f[10];
#pragma unroll
    for (int r = 0; r < 10; ++r) f[r] = __shfl(col[r], src);
    if (j > c) {
      col[c] *= inv;
#pragma unroll
      for (int r = 0; r < 10; ++r)
        if (r != c) col[r] = fma(-f[r], col[c], col[r]);
    } else if (j == c) {
#pragma unroll
      for (int r = 0; r < 10; ++r) col[r] = r == c ? 1.0 : 0.0;
    }
  }
  if (own && j >= 10)
#pragma unroll
    for (int r = 4; r < 10; ++r) a.Bg[(10 * (r - 4) + (j - 10)) * ldw + s] = col[r];
  if (own && j == 0) a.okg[s] = ok ? 1 : 0;
}

// (B') lane per sample: the rows' polynomials and d(z) = det [k; l; m] once per sample (the
// root kernel's 16 lanes of a sample computed them twice each: 32 copies, and B's 60 rows
// were its register peak)
static_assert(sizeof(E5Polys) == 39 * sizeof(double), "E5Polys is 39 packed doubles");
__global__ __launch_bounds__(64) void k_e5_polys(E5Args a) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= a.S) return;
  double Bm[6][10];
  const double *bg = a.Bg + s;
#pragma unroll
  for (int rr = 0; rr < 6; ++rr)
#pragma unroll
    for (int q = 0; q < 10; ++q) Bm[rr][q] = bg[(10 * rr + q) * a.ldw];
  E5Polys P;
  double d[11];
  e5_polys(Bm, P, d);
  double *o = a.Pg + s;
#pragma unroll
  for (int i = 0; i < 11; ++i) o[i * a.ldw] = d[i];
  const double *pp = P.kx;
#pragma unroll
  for (int j = 0; j < 39; ++j) o[(11 + j) * a.ldw] = pp[j];
}

// (C) 16 lanes per sample (a DPP row), lane r owns root r: the degree-10 polynomial of B's rows
// 4..9 (every lane of the row), its roots by Aberth-Ehrlich with the Newton-polygon start points
// of twoview_math.h aberth_roots (same start points, Horner steps and freeze tests, but every
// root of a sweep updated from the previous sweep's roots, read across the row by DPP), then
// lane r's real root to its solution (E from the null basis in memory, F = M1 E M2).  A sample's
// solutions take slots in root order; NaN in the slots past its count.  (A lane per sample:
// 346 us at C2 -- 313 waves for 1 024 SIMDs, each a serial chain of 10 roots.)
#ifndef RSD_E5_ROOTS_WAVES
#define RSD_E5_ROOTS_WAVES 2  // minimum waves per SIMD (157 VGPRs: 3; a cap at 4 spills and is slower) (A/B builds: tools/build_ab.sh)
#endif
// Two phases (a.split > 0): four samples share a wave and the wave sweeps until the slowest
// of them converges, so phase 1 stops after a.split sweeps and hands the rows still moving to
// phase 2, which resumes them from their saved roots packed densely (rows never interact --
// the sweep reads only its own row, converged roots stay frozen -- so the roots, and every
// solution, are the same as one phase's).
#ifdef RSAMD_DIAG
__device__ int *g_e5_stats = nullptr;  // per sample: row sweeps, wave sweeps, degree, ok, am[11]
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RSD_E5_ROOTS_WAVES))) void k_e5_roots(E5Args a, int phase) {
  const int r = threadIdx.x & 15;
  const int row_id = blockIdx.x * (blockDim.x >> 4) + (threadIdx.x >> 4);
  int s = row_id;
  bool live = s < a.S;  // the whole row runs the sweeps (DPP), dead rows are masked out
  if (phase == 2) {     // a deferred sample, or a dead row
    const int nd = *a.defer_n;
    if (static_cast<int>(blockIdx.x) * static_cast<int>(blockDim.x >> 4) >= nd) return;  // all dead
    live = row_id < nd;
    s = live ? a.defer_list[row_id] : a.S - 1;
  }
  const int sc = live ? s : a.S - 1;
  const bool ok = live && a.okg[sc];
  const double *pg = a.Pg + sc;  // d, then the rows' polynomials (k_e5_polys)
  double d[11];
#pragma unroll
  for (int i = 0; i < 11; ++i) d[i] = pg[i * a.ldw];
  // monic descending coefficients padded to degree 10: zero roots (trailing zeros of the
  // ascending d) shifted out, leading zeros kept (they add exact zeros in Horner)
  double g[11];
#pragma unroll
  for (int i = 0; i < 11; ++i) g[i] = ok ? d[10 - i] : 0.0;
  int trailing = 0;
#pragma unroll
  for (int i = 10; i >= 0; --i)
    if (g[i] == 0.0 && trailing == 10 - i) ++trailing;
  bool any = false;
#pragma unroll
  for (int i = 0; i < 11; ++i) any = any || g[i] != 0.0;
  if (!any) trailing = 0;
  for (int t = 0; t < trailing; ++t) {
#pragma unroll
    for (int i = 10; i > 0; --i) g[i] = g[i - 1];
    g[0] = 0.0;
  }
  double lead = 0.0;
  int lo = 11;
#pragma unroll
  for (int i = 10; i >= 0; --i)
    if (g[i] != 0.0) {
      lead = g[i];
      lo = i;
    }
  const int deg = any ? 10 - lo : 0;
  double am[11];
#pragma unroll
  for (int i = 0; i < 11; ++i) am[i] = any ? g[i] / lead : 0.0;
  // start point of root r: edge e of the Newton polygon (upper hull of (k, log |b_k|), b_k =
  // am[10 - k]) with m = k2 - k1 points on |z| = (|b_k1| / |b_k2|)^(1/m)
  double zr = __builtin_nan(""), zi = __builtin_nan("");
  // log |b_k| by lane k of the row, read across the row (one log per lane instead of eleven)
  double lgl;
  {
    double bk = am[0];
#pragma unroll
    for (int k = 1; k < 11; ++k) bk = r == k ? am[10 - k] : bk;
    bk = r == 0 ? am[10] : bk;
    const double v = fabs(bk);
    lgl = v > 0.0 && r < 11 ? log(v) : -1.0e300;
  }
  double lg[11];
#pragma unroll
  for (int k = 0; k < 11; ++k) lg[k] = __shfl(lgl, k, 16);
  if (r < deg) {
    int hull[11], nh = 0;
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
      if (r < q + m) {
        const double rad = exp((lg[hull[e]] - lg[hull[e + 1]]) / m);
        const double ang = 6.283185307179586 * (r - q) / m + 6.283185307179586 * e / deg + 0.4;
        zr = rad * cos(ang);
        zi = rad * sin(ang);
        break;
      }
      q += m;
    }
  }
  bool conv = !(r < deg);
  int it0 = 0, it1 = 100;
  double *zs = a.zst + (static_cast<int64_t>(sc) * 16 + r) * 3;
  if (phase == 1) it1 = a.split;
  if (phase == 2) {  // resume the saved sweep state
    zr = zs[0];
    zi = zs[1];
    conv = !live || zs[2] != 0.0;
    it0 = a.split;
  }
#ifdef RSAMD_DIAG
  int row_done = -1, wave_it = it0;  // sweeps until this row converged / the wave stopped
  const uint64_t rowmask = 0xffffull << (threadIdx.x & 48);
#endif
  for (int it = it0; it < it1; ++it) {
#ifdef RSAMD_DIAG
    if (row_done < 0 && !(__ballot(!conv) & rowmask)) row_done = it;
    wave_it = it + 1;
#endif
    if (!__ballot(!conv)) break;  // wave-uniform: every row keeps sweeping while one root moves
    double sr = 0.0, si = 0.0;  // sum_{j != r} 1 / (z_r - z_j), the previous sweep's z_j
    aberth_sum<1>(zr, zi, sr, si);
    if (!conv) {
      const double xr = zr, xi = zi;
      const double az = sqrt(xr * xr + xi * xi);
      double pr = 0.0, pi = 0.0, dr = 0.0, di = 0.0, S = 0.0;
#pragma unroll
      for (int j = 0; j < 11; ++j) {
        const double ndr = dr * xr - di * xi + pr, ndi = dr * xi + di * xr + pi;
        dr = ndr;
        di = ndi;
        const double npr = pr * xr - pi * xi + am[j], npi = pr * xi + pi * xr;
        pr = npr;
        pi = npi;
        S = S * az + fabs(am[j]);
      }
      if (sqrt(pr * pr + pi * pi) <= 8.0 * 2.220446049250313e-16 * S) {
        conv = true;
      } else {
        double rr_, ri_;  // p / p'
        const double den = dr * dr + di * di;
        if (den == 0.0) {
          rr_ = pr;
          ri_ = pi;
        } else {
          rr_ = (pr * dr + pi * di) / den;
          ri_ = (pi * dr - pr * di) / den;
        }
        const double qr = 1.0 - (rr_ * sr - ri_ * si), qi = -(rr_ * si + ri_ * sr);
        const double qd = qr * qr + qi * qi;
        double wr = rr_, wi = ri_;
        if (qd != 0.0) {
          wr = (rr_ * qr + ri_ * qi) / qd;
          wi = (ri_ * qr - rr_ * qi) / qd;
        }
        zr = xr - wr;
        zi = xi - wi;
        if (fabs(wr) + fabs(wi) <= 2.0 * 2.220446049250313e-16 * (fabs(zr) + fabs(zi))) conv = true;
      }
    }
  }
  if (phase == 1) {  // rows still moving go to phase 2 with their state
    const uint64_t rowm = 0xffffull << (threadIdx.x & 48);
    if (live && (__ballot(!conv) & rowm)) {
      zs[0] = zr;
      zs[1] = zi;
      zs[2] = conv ? 1.0 : 0.0;
      if (r == 0) a.defer_list[atomicAdd(a.defer_n, 1)] = s;
      return;
    }
  }
#ifdef RSAMD_DIAG
  if (g_e5_stats && live && r == 0) {
    int *o = g_e5_stats + 26 * static_cast<int64_t>(s);
    o[0] = row_done < 0 ? wave_it : row_done;
    o[1] = wave_it;
    o[2] = deg;
    o[3] = ok ? 1 : 0;
    double *od = reinterpret_cast<double *>(o + 4);  // the monic descending coefficients
#pragma unroll
    for (int i = 0; i < 11; ++i) od[i] = am[i];
  }
#endif
  // lane r's solution: real iterated roots (|Im| <= 1e-6 max(1, |Re|)) and the zero roots
  double E[9];
  bool valid = false;
  if (ok && r < deg + trailing && (r >= deg || fabs(zi) <= 1e-6 * fmax(1.0, fabs(zr)))) {
    // d and the rows' polynomials from memory (not kept live through the sweeps)
    const double *pg2 = pg;
    asm volatile("" : "+v"(pg2));
    valid = e5_solution(pg2, a.ldw, r < deg ? zr : 0.0, a.Bas + sc, a.ldw, E);
  }
  const uint64_t row = 0xffffull << (threadIdx.x & 48);
  const uint64_t vb = __ballot(valid) & row;
  const int ns = __popcll(vb);
  const int lane = threadIdx.x & 63;
  if (!live) return;
  if (r == 0 && a.nsol) a.nsol[s] = ns;
  auto store = [&](int j, const double (&V)[9]) {
    const int64_t slot = static_cast<int64_t>(s) * kE5Sol + j;
#pragma unroll
    for (int e = 0; e < 9; ++e) a.Esoa[e * a.ld + slot] = V[e];
    if (a.Fsoa) {
      double T[9];  // E M2
#pragma unroll
      for (int rr = 0; rr < 3; ++rr)
#pragma unroll
        for (int c = 0; c < 3; ++c)
          T[3 * rr + c] = fma(V[3 * rr], a.M2[c], fma(V[3 * rr + 1], a.M2[3 + c], V[3 * rr + 2] * a.M2[6 + c]));
#pragma unroll
      for (int rr = 0; rr < 3; ++rr)
#pragma unroll
        for (int c = 0; c < 3; ++c)
          a.Fsoa[(3 * rr + c) * a.ld + slot] =
              fma(a.M1[3 * rr], T[c], fma(a.M1[3 * rr + 1], T[3 + c], a.M1[3 * rr + 2] * T[6 + c]));
    }
  };
  if (valid) store(__popcll(vb & ((1ull << lane) - 1ull)), E);  // slots in root order
  if (r >= ns && r < kE5Sol) {  // NaN past the sample's solutions: those slots count 0
    const double qn = __builtin_nan("");
    const double Enan[9] = {qn, qn, qn, qn, qn, qn, qn, qn, qn};
    store(r, Enan);
  }
}

struct E5DevResult {
  double E[9], F[9];
  int64_t best_slot, best_count, n_inliers;
  int64_t inliers[];
};

// c* = max count (one workgroup; strict ">" against 0: no consensus, no winner).
__global__ __launch_bounds__(256) void k_e5_max(const int *__restrict__ counts, int64_t H,
                                                const int *__restrict__ hc, int *cmax) {
  __shared__ int sm[4];
  const int tid = threadIdx.x;
  H = hc ? min<int64_t>(H, *hc) : H;
  int bm = 0;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + tid; i < H;
       i += static_cast<int64_t>(gridDim.x) * 256)
    bm = max(bm, counts[i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) bm = max(bm, __shfl_xor(bm, o));
  if ((tid & 63) == 0) sm[tid >> 6] = bm;
  __syncthreads();
  if (tid == 0) atomicMax(cmax, max(max(sm[0], sm[1]), max(sm[2], sm[3])));  // *cmax zeroed first
}

// Counting only the real solutions: the map dense index -> slot of the real ones (*hc of
// them), so the counting and the tie-break read F through it.  A workgroup per 256 samples:
// the solutions of all earlier samples (int4 loads, a reduction; no device-wide scan pass),
// its samples' offsets by a block scan.  The dense order keeps the slot order, so "the smallest
// slot on equal norms" is "the smallest dense index".
// (Past kPackInline workgroups the earlier counts come from k_e5_bsum / k_e5_bscan instead:
// the inline reduction reads O(S^2 / 256) words.)
constexpr int kPackSamples = 256, kPackInline = 128;
__global__ __launch_bounds__(kPackSamples) void k_e5_pack(const int *__restrict__ nsol, int S,
                                                          const int *__restrict__ bbase,
                                                          int *__restrict__ slot_of,
                                                          int *__restrict__ hc,
                                                          int *__restrict__ zero2) {
  __shared__ int sw[kPackSamples / 64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (zero2 && blockIdx.x == 0 && tid < 2) zero2[tid] = 0;  // c* and the candidate count
  const int b0 = blockIdx.x * kPackSamples;  // a multiple of 4: int4 loads below b0
  int pre = 0;
  if (bbase) {
    pre = tid == 0 ? bbase[blockIdx.x] : 0;
  } else {
#pragma unroll 4
    for (int k = 4 * tid; k < b0; k += 4 * kPackSamples) {
      const int4 q = *reinterpret_cast<const int4 *>(nsol + k);
      pre += (q.x + q.y) + (q.z + q.w);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) pre += __shfl_xor(pre, o);
  if (lane == 0) sw[w] = pre;
  __syncthreads();
  int base = 0;
#pragma unroll
  for (int q = 0; q < kPackSamples / 64; ++q) base += sw[q];
  __syncthreads();
  const int sidx = b0 + tid;
  const int v = sidx < S ? nsol[sidx] : 0;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) sw[w] = x;
  __syncthreads();
  for (int q = 0; q < w; ++q) base += sw[q];
  const int o = base + x - v;
  for (int j = 0; j < v; ++j) slot_of[o + j] = sidx * kE5Sol + j;
  if (blockIdx.x == gridDim.x - 1 && tid == kPackSamples - 1) *hc = base + x;
}

// The counting models of the real solutions (dense index h -> slot): the float64 F for the
// guard re-test (Fd) and the fp32 unit-frame model with its decision constants (f32_model, as
// the F-RANSAC solve writes them)
__global__ __launch_bounds__(256) void k_e5_models(const int *__restrict__ slot_of,
                                                   const int *__restrict__ hc,
                                                   const double *__restrict__ Fsoa, int64_t ld,
                                                   Frame fr, double gT, double gDe, double gDn,
                                                   double *__restrict__ Fd,
                                                   float *__restrict__ F32soa,
                                                   float4 *__restrict__ G4,
                                                   int *__restrict__ counts,
                                                   int *__restrict__ gdone) {
  const int h = blockIdx.x * blockDim.x + threadIdx.x;
  if (h >= *hc) return;  // (the grid covers every slot: the real-solution count is on the device)
  counts[h] = 0;         // (the counting kernel adds into the first *hc counts only)
  if ((h & 63) == 0) gdone[h >> 6] = 0;  // its groups' completion counters (c* on the fly)
  const int64_t slot = slot_of[h];
  double F[9];
#pragma unroll
  for (int q = 0; q < 9; ++q) {
    F[q] = Fsoa[q * ld + slot];
    Fd[q * ld + h] = F[q];
  }
  f32_model(F, fr, gT, gDe, gDn, F32soa, G4, ld, h);
}

// solutions per workgroup of kPackSamples samples
__global__ __launch_bounds__(kPackSamples) void k_e5_bsum(const int *__restrict__ nsol, int S,
                                                          int *__restrict__ bsum) {
  __shared__ int sw[kPackSamples / 64];
  const int tid = threadIdx.x, sidx = blockIdx.x * kPackSamples + tid;
  int v = sidx < S ? nsol[sidx] : 0;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if ((tid & 63) == 0) sw[tid >> 6] = v;
  __syncthreads();
  if (tid == 0) {
    int t = 0;
#pragma unroll
    for (int q = 0; q < kPackSamples / 64; ++q) t += sw[q];
    bsum[blockIdx.x] = t;
  }
}

// exclusive scan of the nb workgroup sums in place (one workgroup, a run per thread)
__global__ __launch_bounds__(1024) void k_e5_bscan(int *__restrict__ bsum, int nb) {
  __shared__ int sw[16];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int per = (nb + 1023) / 1024, lo = min(nb, tid * per), hi = min(nb, lo + per);
  int v = 0;
  for (int k = lo; k < hi; ++k) v += bsum[k];
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) sw[w] = x;
  __syncthreads();
  int base = x - v;
  for (int q = 0; q < w; ++q) base += sw[q];
  for (int k = lo; k < hi; ++k) {
    const int t = bsum[k];
    bsum[k] = base;
    base += t;
  }
}

// The slots with the largest count c* (the candidates), appended in any order: one ballot and
// one atomic per wave.
__global__ __launch_bounds__(256) void k_e5_cands(const int *__restrict__ counts, int64_t H,
                                                  const int *__restrict__ hc,
                                                  const int *__restrict__ cmax, int *__restrict__ cand,
                                                  int *__restrict__ ncand) {
  const int c = *cmax;
  H = hc ? min<int64_t>(H, *hc) : H;
  const int lane = threadIdx.x & 63;
  for (int64_t b = static_cast<int64_t>(blockIdx.x) * blockDim.x; b < H;
       b += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t h = b + threadIdx.x;
    const bool take = c > 0 && h < H && counts[h] == c;
    const uint64_t bal = __ballot(take);
    if (!bal) continue;
    int base = 0;
    if (lane == 0) base = atomicAdd(ncand, static_cast<int>(__popcll(bal)));
    base = __shfl(base, 0);
    if (take) cand[base + __popcll(bal & ((1ull << lane) - 1ull))] = static_cast<int>(h);
  }
}

// ||d||^2 of every candidate, d_i = max(|r1_i|, |r2_i|) over all points (the quantity the
// reference's F loop compares on ties, fun.py:317-325): a wave per candidate, the points over
// the lanes, partial sums combined by a fixed butterfly (deterministic).  (A lane per slot
// summed 2 000 points serially: 476 us of the C2 E-RANSAC run.)  The summation order is NOT
// numpy's (np.linalg.norm's pairwise sum over the points) nor the earlier per-slot
// sequential one, so two candidates whose norms differ by a few ulp can rank differently
// from a numpy restatement; the E path has no reference counterpart (SURVEY a-15), so the
// tie-break is deterministic but unpinned at that level.
// ||d||^2 of the model at f (stride ld) over the points, by one wave (lanes over the points,
// a fixed butterfly)
__device__ __forceinline__ double e5_norm_wave(const Pt *__restrict__ pts, int n,
                                               const double *__restrict__ fp, int64_t ld) {
  const int lane = threadIdx.x & 63;
  double f[9];
#pragma unroll
  for (int q = 0; q < 9; ++q) f[q] = fp[q * ld];
  double ss = 0.0;
  for (int i = lane; i < n; i += 64) {
    const Pt p = pts[i];
    const double l10 = fma(f[0], p.x2, fma(f[1], p.y2, f[2]));
    const double l11 = fma(f[3], p.x2, fma(f[4], p.y2, f[5]));
    const double l12 = fma(f[6], p.x2, fma(f[7], p.y2, f[8]));
    const double l20 = fma(f[0], p.x1, fma(f[3], p.y1, f[6]));
    const double l21 = fma(f[1], p.x1, fma(f[4], p.y1, f[7]));
    const double e = fabs(fma(l10, p.x1, fma(l11, p.y1, l12)));
    const double d = fmax(e / sqrt(fma(l10, l10, l11 * l11)), e / sqrt(fma(l20, l20, l21 * l21)));
    ss = fma(d, d, ss);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o);
  return ss;
}

__global__ __launch_bounds__(256) void k_e5_norms(const Pt *__restrict__ pts, int n,
                                                  const int *__restrict__ cand,
                                                  const int *__restrict__ ncand,
                                                  const int *__restrict__ slot_of,
                                                  const double *__restrict__ Fsoa, int64_t ld,
                                                  double *__restrict__ norms) {
  const int lane = threadIdx.x & 63;
  const int nw = static_cast<int>(gridDim.x) * (blockDim.x >> 6);
  const int nc = *ncand;
  for (int k = static_cast<int>(blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6); k < nc; k += nw) {
    const double ss = e5_norm_wave(pts, n, Fsoa + slot_of[cand[k]], ld);  // dense index -> slot
    if (lane == 0) norms[k] = ss == ss ? ss : __builtin_inf();
  }
}

// k_e5_cands and k_e5_norms in one launch (c* from the counting kernel's group completion):
// a wave per 64 counts, and for each count equal to c* its slot appended and its norm by the
// same wave
__global__ __launch_bounds__(256) void k_e5_cand_norms(const int *__restrict__ counts, int64_t H,
                                                       const int *__restrict__ hc,
                                                       const int *__restrict__ cmax,
                                                       int *__restrict__ cand,
                                                       int *__restrict__ ncand,
                                                       const Pt *__restrict__ pts, int n,
                                                       const int *__restrict__ slot_of,
                                                       const double *__restrict__ Fsoa, int64_t ld,
                                                       double *__restrict__ norms) {
  const int c = *cmax;
  if (c <= 0) return;
  H = hc ? min<int64_t>(H, *hc) : H;
  const int lane = threadIdx.x & 63;
  const int64_t nwv = static_cast<int64_t>(gridDim.x) * (blockDim.x >> 6);
  for (int64_t b = (static_cast<int64_t>(blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 64;
       b < H; b += nwv * 64) {
    const int64_t h = b + lane;
    uint64_t bal = __ballot(h < H && counts[h] == c);
    while (bal) {
      const int f = __ffsll(static_cast<long long>(bal)) - 1;
      bal &= bal - 1ull;
      int k = 0;
      if (lane == 0) k = atomicAdd(ncand, 1);
      k = __shfl(k, 0);
      if (lane == 0) cand[k] = static_cast<int>(b + f);
      const double ss = e5_norm_wave(pts, n, Fsoa + slot_of[b + f], ld);
      if (lane == 0) norms[k] = ss == ss ? ss : __builtin_inf();
    }
  }
}

__device__ __forceinline__ void e5_inliers_body(const Pt *__restrict__ pts, int n, double thr2,
                                                E5DevResult *res);

// the winner among the candidates: the smallest norm, the smallest slot on equal norms; then
// its inlier list (e5_inliers_body)
__global__ __launch_bounds__(1024) void k_e5_select(const double *__restrict__ norms,
                                                    const int *__restrict__ cand,
                                                    const int *__restrict__ ncand,
                                                    const int *__restrict__ cmax,
                                                    const int *__restrict__ slot_of,
                                                    const double *__restrict__ Esoa,
                                                    const double *__restrict__ Fsoa, int64_t ld,
                                                    E5DevResult *res, const Pt *__restrict__ pts,
                                                    int n, double thr2) {
  __shared__ double sv[16];
  __shared__ int64_t si[16];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nc = *ncand;
  double bv = __builtin_inf();
  int64_t bi = INT64_MAX;
  for (int k = tid; k < nc; k += 1024) {
    const double v = norms[k];
    const int64_t i = cand[k];
    if (v < bv || (v == bv && i < bi)) {
      bv = v;
      bi = i;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double ov = __shfl_xor(bv, o);
    const int64_t oi = __shfl_xor(bi, o);
    if (ov < bv || (ov == bv && oi < bi)) {
      bv = ov;
      bi = oi;
    }
  }
  if (lane == 0) {
    sv[w] = bv;
    si[w] = bi;
  }
  __syncthreads();
  if (tid == 0) {
    for (int q = 1; q < 16; ++q)
      if (sv[q] < bv || (sv[q] == bv && si[q] < bi)) {
        bv = sv[q];
        bi = si[q];
      }
    const int c = *cmax;
    const bool ok = c > 0 && bi != INT64_MAX;
    const int64_t slot = ok ? (slot_of ? slot_of[bi] : bi) : -1;  // dense index -> slot
    res->best_slot = slot;
    res->best_count = ok ? c : 0;
    for (int q = 0; q < 9; ++q) {
      res->E[q] = ok ? Esoa[q * ld + slot] : 0.0;
      res->F[q] = ok ? Fsoa[q * ld + slot] : 0.0;
    }
  }
  // the winner's inlier list in the same launch (thread 0's record is visible after the barrier)
  __syncthreads();
  e5_inliers_body(pts, n, thr2, res);
}

__device__ __forceinline__ void e5_inliers_body(const Pt *__restrict__ pts, int n, double thr2,
                                                E5DevResult *res) {
  __shared__ int woff[16];
  __shared__ int base_s;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const bool have = res->best_slot >= 0;
  double f[9];
#pragma unroll
  for (int q = 0; q < 9; ++q) f[q] = res->F[q];
  if (tid == 0) base_s = 0;
  __syncthreads();
  for (int b = 0; b < n; b += 1024) {
    const int i = b + tid;
    bool take = false;
    if (have && i < n) {
      const Pt p = pts[i];
      const double l10 = fma(f[0], p.x2, fma(f[1], p.y2, f[2]));
      const double l11 = fma(f[3], p.x2, fma(f[4], p.y2, f[5]));
      const double l12 = fma(f[6], p.x2, fma(f[7], p.y2, f[8]));
      const double l20 = fma(f[0], p.x1, fma(f[3], p.y1, f[6]));
      const double l21 = fma(f[1], p.x1, fma(f[4], p.y1, f[7]));
      const double e = fma(l10, p.x1, fma(l11, p.y1, l12));
      const double n1 = fma(l10, l10, l11 * l11);
      const double n2 = fma(l20, l20, l21 * l21);
      take = e * e < thr2 * fmin(n1, n2);
    }
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

}  // namespace rsd

// ------------------------------------------------------------------------------------------
using rs::fail;
using rs::hip_fail;

#define HIP_TRY(expr)                                 \
  do {                                                \
    hipError_t e_ = (expr);                           \
    if (e_ != hipSuccess) return hip_fail(e_, #expr); \
  } while (0)

static size_t e5_align(size_t b) { return (b + 255) / 256 * 256; }
constexpr int kE5CountWaves = 6144;  // resident waves of k_f8_count32q (as the F-RANSAC plan)
// sweeps of the root finder's first phase (0: one phase).  Measured at C2 (20 000 samples,
// profiles/r04b_e5_split_ab.txt, two passes): one phase 0.440 / 0.446 ms per E-RANSAC run;
// split after 5 / 6 / 8 / 10 / 12 sweeps 0.52 / 0.52-0.54 / 0.50 / 0.46-0.47 / 0.48 ms -- the
// second phase's set-up (B rows, polynomial, start state) costs more than the drained sweeps
constexpr int kE5SplitDefault = 0;

// bytes of the three solve kernels' work buffers for S samples: the 10 x 20 system, null
// basis and B rows (296 doubles), Gauss-Jordan flags, the deferred list + count and the
// deferred rows' root state (48 doubles) of the two-phase root finder
static size_t e5_work_bytes(int64_t S) {
  return e5_align(sizeof(double) * 296 * static_cast<size_t>(S)) + e5_align(sizeof(int) * S) +
         e5_align(sizeof(int) * (S + 1)) + e5_align(sizeof(double) * 48 * static_cast<size_t>(S));
}

// sweeps before the root finder's rows still moving are repacked (RSAMD_E5_SPLIT; 0: one phase)
static int e5_split() {
  static const int v = [] {
    const char *e = std::getenv("RSAMD_E5_SPLIT");
    return e ? std::max(0, std::min(99, std::atoi(e))) : kE5SplitDefault;
  }();
  return v;
}

// the solve (k_e5_build, k_e5_gj, k_e5_roots) into a.Esoa / a.Fsoa, work buffers from `work`
static int launch_e5_solve(rsd::E5Args &a, char *work, hipStream_t s) {
  const int64_t S = a.S;
  a.ldw = S;
  a.Mg = reinterpret_cast<double *>(work);
  a.Bas = a.Mg + 200 * S;
  a.Bg = a.Bas + 36 * S;
  char *w2 = work + e5_align(sizeof(double) * 296 * static_cast<size_t>(S));
  a.okg = reinterpret_cast<int *>(w2);
  w2 += e5_align(sizeof(int) * S);
  a.defer_n = reinterpret_cast<int *>(w2);
  a.defer_list = a.defer_n + 1;
  w2 += e5_align(sizeof(int) * (S + 1));
  a.zst = reinterpret_cast<double *>(w2);
  a.split = e5_split();
  hipLaunchKernelGGL(rsd::k_e5_build, dim3((S + 63) / 64), dim3(64), 0, s, a);
  HIP_TRY(hipGetLastError());
  hipLaunchKernelGGL(rsd::k_e5_gj, dim3((S + 1) / 2), dim3(64), 0, s, a);
  HIP_TRY(hipGetLastError());
  a.Pg = a.Mg;  // the 10 x 20 systems are dead after Gauss-Jordan (200 >= 50 doubles per sample)
  hipLaunchKernelGGL(rsd::k_e5_polys, dim3((S + 63) / 64), dim3(64), 0, s, a);
  HIP_TRY(hipGetLastError());
  if (a.split > 0) {
    HIP_TRY(hipMemsetAsync(a.defer_n, 0, sizeof(int), s));
    hipLaunchKernelGGL(rsd::k_e5_roots, dim3((S + 15) / 16), dim3(256), 0, s, a, 1);
    HIP_TRY(hipGetLastError());
    // every row may have been deferred: the grid covers S rows, the rows past the deferred
    // count exit at once
    hipLaunchKernelGGL(rsd::k_e5_roots, dim3((S + 15) / 16), dim3(256), 0, s, a, 2);
  } else {
    hipLaunchKernelGGL(rsd::k_e5_roots, dim3((S + 15) / 16), dim3(256), 0, s, a, 0);
  }
  HIP_TRY(hipGetLastError());
  return RS_OK;
}

static bool inv3(const double *K, double *Ki) {
  const double det = K[0] * (K[4] * K[8] - K[5] * K[7]) - K[1] * (K[3] * K[8] - K[5] * K[6]) +
                     K[2] * (K[3] * K[7] - K[4] * K[6]);
  if (!(det != 0.0) || !std::isfinite(det)) return false;
  const double id = 1.0 / det;
  Ki[0] = (K[4] * K[8] - K[5] * K[7]) * id;
  Ki[1] = (K[2] * K[7] - K[1] * K[8]) * id;
  Ki[2] = (K[1] * K[5] - K[2] * K[4]) * id;
  Ki[3] = (K[5] * K[6] - K[3] * K[8]) * id;
  Ki[4] = (K[0] * K[8] - K[2] * K[6]) * id;
  Ki[5] = (K[2] * K[3] - K[0] * K[5]) * id;
  Ki[6] = (K[3] * K[7] - K[4] * K[6]) * id;
  Ki[7] = (K[1] * K[6] - K[0] * K[7]) * id;
  Ki[8] = (K[0] * K[4] - K[1] * K[3]) * id;
  return true;
}

extern "C" int rs_e5_solve(rs_ctx *c, const double *y1, const double *y2, int64_t S,
                           double *E_out, int32_t *nsol) {
  if (!c || !y1 || !y2 || !E_out || !nsol) return fail(RS_EINVAL, "null pointer");
  if (S < 1 || S > (1 << 24)) return fail(RS_EINVAL, "sample count out of range");
  HIP_TRY(hipSetDevice(c->device));
  const int64_t m = 5 * S, ld = rsd::kE5Sol * S;
  std::vector<rsd::Pt> hp(static_cast<size_t>(m));
  for (int64_t i = 0; i < m; ++i) {
    if (!(y1[3 * i + 2] != 0.0) || !(y2[3 * i + 2] != 0.0))
      return fail(RS_EINVAL, "homogeneous points need a nonzero third coordinate");
    hp[i] = rsd::Pt{y1[3 * i] / y1[3 * i + 2], y1[3 * i + 1] / y1[3 * i + 2],
                    y2[3 * i] / y2[3 * i + 2], y2[3 * i + 1] / y2[3 * i + 2]};
  }
  const size_t bp = e5_align(sizeof(rsd::Pt) * m), bE = e5_align(sizeof(double) * 9 * ld),
               bn = e5_align(sizeof(int) * S);
  int st = rs::ensure_scratch(c, bp + bE + bn + e5_work_bytes(S));
  if (st) return st;
  char *base = static_cast<char *>(c->scratch);
  auto *dp = reinterpret_cast<rsd::Pt *>(base);
  auto *dE = reinterpret_cast<double *>(base + bp);
  auto *dn = reinterpret_cast<int *>(base + bp + bE);
  char *work = base + bp + bE + bn;
  hipStream_t s = c->stream;
  HIP_TRY(hipMemcpyAsync(dp, hp.data(), sizeof(rsd::Pt) * m, hipMemcpyHostToDevice, s));
  rsd::E5Args a{};
  a.pts = dp;
  a.n = static_cast<int>(m);
  a.S = static_cast<int>(S);
  a.mode = 1;
  const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
  std::memcpy(a.Kin1, I, sizeof(I));
  std::memcpy(a.Kin2, I, sizeof(I));
  std::memcpy(a.M1, I, sizeof(I));
  std::memcpy(a.M2, I, sizeof(I));
  a.Esoa = dE;
  a.nsol = dn;
  a.ld = ld;
  if ((st = launch_e5_solve(a, work, s))) return st;
  std::vector<double> soa(static_cast<size_t>(9 * ld));
  HIP_TRY(hipMemcpyAsync(soa.data(), dE, sizeof(double) * 9 * ld, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(nsol, dn, sizeof(int) * S, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  for (int64_t q = 0; q < ld; ++q)
    for (int e = 0; e < 9; ++e) E_out[q * 9 + e] = soa[e * ld + q];
  return RS_OK;
}

extern "C" int rs_e5_ransac(rs_ctx *c, const double *p1, const double *p2, int64_t n,
                            const double *K1, const double *K2, int64_t S, uint64_t seed,
                            double thresh, rs_e5_result *out, int64_t *inliers,
                            int64_t *n_inliers) {
  if (!c || !p1 || !p2 || !K1 || !K2 || !out) return fail(RS_EINVAL, "null pointer");
  if (n < 5) return fail(RS_EINVAL, "the five-point solver needs n >= 5 correspondences");
  if (n > (1 << 26) || S < 1 || S > (1 << 24)) return fail(RS_EINVAL, "bad dimensions");
  if (!(thresh == thresh)) return fail(RS_EINVAL, "threshold is NaN");
  rsd::E5Args a{};
  if (!inv3(K1, a.Kin1) || !inv3(K2, a.Kin2)) return fail(RS_EINVAL, "singular camera matrix");
  for (int r = 0; r < 3; ++r)
    for (int q = 0; q < 3; ++q) {
      a.M1[3 * r + q] = a.Kin1[3 * q + r];  // K1^-T
      a.M2[3 * r + q] = a.Kin2[3 * r + q];  // K2^-1
    }
  HIP_TRY(hipSetDevice(c->device));
  const int64_t H = rsd::kE5Sol * S, ld = (H + 63) / 64 * 64;
  const size_t bin = e5_align(sizeof(double) * 2 * n), bp = e5_align(sizeof(rsd::Pt) * n);
  const size_t bE = e5_align(sizeof(double) * 9 * ld), bc = e5_align(sizeof(int) * ld);
  const size_t br = e5_align(sizeof(rsd::E5DevResult) + sizeof(int64_t) * n);
  const size_t bnorm = e5_align(sizeof(double) * ld);
  const size_t bpq = e5_align(sizeof(float) * 4 * ((n + 7) / 8 * 8));
  const size_t bF32 = e5_align(sizeof(float) * 9 * ld), bG4 = e5_align(sizeof(float4) * ld);
  int st = rs::ensure_scratch(c, 2 * bin + bp + 3 * bE + bc + br + bnorm + 256 + bpq + bF32 + bG4 +
                                     2 * e5_align(sizeof(int) * ld) + 2 * e5_align(sizeof(int) * S) +
                                     e5_align(sizeof(int) * (ld / 64 + 1)) + e5_work_bytes(S));
  if (st) return st;
  char *ptr = static_cast<char *>(c->scratch);
  auto take = [&ptr](size_t b) {
    char *q = ptr;
    ptr += b;
    return q;
  };
  double *d1 = reinterpret_cast<double *>(take(bin));
  double *d2 = reinterpret_cast<double *>(take(bin));
  auto *dp = reinterpret_cast<rsd::Pt *>(take(bp));
  double *dE = reinterpret_cast<double *>(take(bE));
  double *dF = reinterpret_cast<double *>(take(bE));
  int *dc = reinterpret_cast<int *>(take(bc));
  auto *dr = reinterpret_cast<rsd::E5DevResult *>(take(br));
  double *dnorm = reinterpret_cast<double *>(take(bnorm));
  int *dcmax = reinterpret_cast<int *>(take(256));  // c* (0), candidates (1), real solutions (2)
  int *dcand = reinterpret_cast<int *>(take(e5_align(sizeof(int) * ld)));
  int *dnsol = reinterpret_cast<int *>(take(e5_align(sizeof(int) * S)));
  int *dslot = reinterpret_cast<int *>(take(e5_align(sizeof(int) * ld)));
  int *doff = reinterpret_cast<int *>(take(e5_align(sizeof(int) * S)));  // workgroup bases
  int *dgdone = reinterpret_cast<int *>(take(e5_align(sizeof(int) * (ld / 64 + 1))));  // per group
  // fp32 counting: point-pair layout, dense float64 / fp32 models, decision constants
  auto *dpq = reinterpret_cast<float4 *>(take(bpq));
  double *dFd = reinterpret_cast<double *>(take(bE));
  float *dF32 = reinterpret_cast<float *>(take(bF32));
  auto *dG4 = reinterpret_cast<float4 *>(take(bG4));
  char *work = take(e5_work_bytes(S));
  hipStream_t s = c->stream;
  HIP_TRY(hipMemcpyAsync(d1, p1, sizeof(double) * 2 * n, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(d2, p2, sizeof(double) * 2 * n, hipMemcpyHostToDevice, s));
  // counting in fp32 with the float64 guard band (k_f8_count32q, the F-RANSAC product kernel:
  // counts identical to the float64 test's) unless the points give no unit frame
  rsd::Frame fr{};
  // (RSAMD_E5_FP64=1, a test hook: the plain float64 kernel, for the equal-counts test)
  const char *f64 = std::getenv("RSAMD_E5_FP64");
  const bool fp32 = rsd::unit_frame(p1, p2, n, fr) && !(f64 && f64[0] == '1');
  HIP_TRY(rsd::launch_pack_points_both(d1, d2, static_cast<int>(n), dp, fp32 ? &fr : nullptr, dpq, s));
  a.pts = dp;
  a.n = static_cast<int>(n);
  a.S = static_cast<int>(S);
  a.mode = 0;
  a.seed = seed;
  a.Esoa = dE;
  a.Fsoa = dF;
  a.nsol = dnsol;
  a.ld = ld;
  if ((st = launch_e5_solve(a, work, s))) return st;
#ifdef RSAMD_DIAG
  if (const char *path = std::getenv("RSAMD_E5_STATS")) {  // diagnostic builds: sweep counts
    int *dst = nullptr;
    HIP_TRY(hipMalloc(&dst, sizeof(int) * 26 * S));
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(rsd::g_e5_stats), &dst, sizeof(dst)));
    if ((st = launch_e5_solve(a, work, s))) return st;
    std::vector<int> h(static_cast<size_t>(26 * S));
    HIP_TRY(hipMemcpyAsync(h.data(), dst, sizeof(int) * h.size(), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    int *np = nullptr;
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(rsd::g_e5_stats), &np, sizeof(np)));
    HIP_TRY(hipFree(dst));
    if (FILE *f = std::fopen(path, "wb")) {
      std::fwrite(h.data(), sizeof(int), h.size(), f);
      std::fclose(f);
    }
  }
#endif
  // only the real solutions are counted: the map dslot (dense index -> slot, *hc entries)
  const int npack = static_cast<int>((S + rsd::kPackSamples - 1) / rsd::kPackSamples);
  int *dbsum = nullptr;
  if (npack > rsd::kPackInline) {
    dbsum = doff;
    hipLaunchKernelGGL(rsd::k_e5_bsum, dim3(npack), dim3(rsd::kPackSamples), 0, s, dnsol,
                       static_cast<int>(S), dbsum);
    hipLaunchKernelGGL(rsd::k_e5_bscan, dim3(1), dim3(1024), 0, s, dbsum, npack);
  }
  hipLaunchKernelGGL(rsd::k_e5_pack, dim3(npack), dim3(rsd::kPackSamples), 0, s, dnsol,
                     static_cast<int>(S), dbsum, dslot, dcmax + 2, dcmax);
  if (fp32) {
    // the real solutions' count stays on the device: the models kernel and the counting kernel
    // are sized for every slot and read it (no host round trip between the solve and the count)
    const rsd::Bounds gb = rsd::fp32_bounds(fr, thresh);
    hipLaunchKernelGGL(rsd::k_e5_models, dim3(static_cast<unsigned>((H + 255) / 256)), dim3(256), 0, s,
                       dslot, dcmax + 2, dF, ld, fr, gb.thr2, gb.De, gb.Dn, dFd, dF32, dG4, dc, dgdone);
    static const int slices = [] {  // RSAMD_E5_SLICES: slices per resident wave (A/B)
      const char *e = std::getenv("RSAMD_E5_SLICES");
      return e ? std::atoi(e) : 0;
    }();
    const rsd::Count32qShape sh =
        rsd::count32q_shape(static_cast<int>(n), static_cast<int>(H), kE5CountWaves, slices);
    HIP_TRY(rsd::launch_f8_count32q(dpq, dp, static_cast<int>(n), static_cast<int>(H), dF32, dFd, ld, sh,
                                    rsd::GuardW{thresh * thresh}, dc, s, dgdone, dcmax, dG4,
                                    dcmax + 2));  // (c* into dcmax[0] as groups complete)
  } else {
    HIP_TRY(hipMemsetAsync(dc, 0, sizeof(int) * H, s));
    // chunking of k_f8_count: >= 8 units of work per SIMD, chunks of >= 64 points (sized for
    // the expected ~4 real solutions per sample; the kernel stops at the device count)
    const int64_t groups = (std::max<int64_t>(1, 4 * S) + 63) / 64;
    int64_t nch = std::max<int64_t>(1, std::min<int64_t>((8192 + groups - 1) / groups, (n + 63) / 64));
    const int chunk = static_cast<int>((n + nch - 1) / nch);
    HIP_TRY(rsd::launch_f8_count(dp, static_cast<int>(n), static_cast<int>(H), dF, ld, chunk,
                                 thresh * thresh, dc, s, dcmax + 2, dslot));
  }
  if (fp32) {  // c* is in dcmax[0] already
    hipLaunchKernelGGL(rsd::k_e5_cand_norms, dim3(256), dim3(256), 0, s, dc, H, dcmax + 2, dcmax, dcand,
                       dcmax + 1, dp, static_cast<int>(n), dslot, dF, ld, dnorm);
  } else {
    hipLaunchKernelGGL(rsd::k_e5_max, dim3(static_cast<unsigned>(std::min<int64_t>((H + 255) / 256, 64))),
                       dim3(256), 0, s, dc, H, dcmax + 2, dcmax);
    hipLaunchKernelGGL(rsd::k_e5_cands, dim3(static_cast<unsigned>(std::min<int64_t>((H + 255) / 256, 1024))),
                       dim3(256), 0, s, dc, H, dcmax + 2, dcmax, dcand, dcmax + 1);
    hipLaunchKernelGGL(rsd::k_e5_norms, dim3(256), dim3(256), 0, s, dp, static_cast<int>(n), dcand,
                       dcmax + 1, dslot, dF, ld, dnorm);
  }
  // (the selection and the winner's inlier list: one single-workgroup launch)
  hipLaunchKernelGGL(rsd::k_e5_select, dim3(1), dim3(1024), 0, s, dnorm, dcand, dcmax + 1, dcmax,
                     dslot, dE, dF, ld, dr, dp, static_cast<int>(n), thresh * thresh);
  HIP_TRY(hipGetLastError());
  std::vector<char> host(sizeof(rsd::E5DevResult) + sizeof(int64_t) * n);
  HIP_TRY(hipMemcpyAsync(host.data(), dr, host.size(), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  const auto *r = reinterpret_cast<const rsd::E5DevResult *>(host.data());
  std::memcpy(out->E, r->E, sizeof(out->E));
  std::memcpy(out->F, r->F, sizeof(out->F));
  out->best_sample = r->best_slot >= 0 ? r->best_slot / rsd::kE5Sol : -1;
  out->best_solution = r->best_slot >= 0 ? r->best_slot % rsd::kE5Sol : -1;
  out->best_count = r->best_count;
  if (r->best_slot >= 0 && r->n_inliers != r->best_count)
    return fail(RS_EDEVICE, "consensus recount mismatch");
  if (n_inliers) *n_inliers = r->best_slot >= 0 ? r->n_inliers : 0;
  if (inliers && r->best_slot >= 0)
    std::memcpy(inliers, r->inliers, sizeof(int64_t) * r->n_inliers);
  return RS_OK;
}
