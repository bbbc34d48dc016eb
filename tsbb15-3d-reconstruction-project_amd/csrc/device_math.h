// Device-side numerics shared by the F and PnP kernels (gfx950, float64).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rsd {

// One correspondence, AoS 32 B: left image (x1, y1) = p1 column, right image (x2, y2) = p2
// column (fun.getFFromLabCode(p1, p2), convention p1^T F p2 = 0, lab3.py:195-196).
struct Pt {
  double x1, y1, x2, y2;
};

// Similarity frame of the fp32 counting kernel: x~ = (x - c_i) / s per image i, one common
// scale s so both line-length terms scale by s^2 and the min() test is frame invariant.
struct Frame {
  double s, cx1, cy1, cx2, cy2;
};

// Per-hypothesis decision (k_f8_count32q): constants live with each model (G4,
// written by the solve); only the float64 re-test threshold is global.
struct GuardW {
  double thr2_px;
};


// ----------------------------------------------------------------------------------------
// Philox4x32-10 counter-based generator (throughput-mode sampler).
// ----------------------------------------------------------------------------------------
__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint2 k) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
    const uint32_t lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
    c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
    k.x += 0x9E3779B9u;
    k.y += 0xBB67AE85u;
  }
  return c;
}

// Uniform k-subset of [0, n) by Floyd's algorithm with unbiased (Lemire) bounded draws.
// Hypothesis `h` of stream `seed` uses Philox counters (h, 0..); every k-subset is equally
// likely, as for np.random.choice(arange(n), k, replace=False).
template <int K>
__device__ __forceinline__ void floyd_sample(uint64_t seed, uint64_t h, int n, int (&idx)[K]) {
  const uint2 key = make_uint2(static_cast<uint32_t>(seed), static_cast<uint32_t>(seed >> 32));
  uint32_t ctr = 0;
  uint4 blk = philox4x32_10(
      make_uint4(static_cast<uint32_t>(h), static_cast<uint32_t>(h >> 32), ctr++, 0x5a17u), key);
  int used = 0;
  auto next = [&]() -> uint32_t {
    if (used == 4) {
      blk = philox4x32_10(
          make_uint4(static_cast<uint32_t>(h), static_cast<uint32_t>(h >> 32), ctr++, 0x5a17u),
          key);
      used = 0;
    }
    const uint32_t w = used == 0 ? blk.x : used == 1 ? blk.y : used == 2 ? blk.z : blk.w;
    ++used;
    return w;
  };
#pragma unroll
  for (int m = 0; m < K; ++m) {
    const uint32_t j = static_cast<uint32_t>(n - K + m);
    const uint32_t range = j + 1u;
    uint64_t prod = static_cast<uint64_t>(next()) * range;
    uint32_t low = static_cast<uint32_t>(prod);
    if (low < range) {
      const uint32_t thresh = (0u - range) % range;
      while (low < thresh) {
        prod = static_cast<uint64_t>(next()) * range;
        low = static_cast<uint32_t>(prod);
      }
    }
    const int t = static_cast<int>(prod >> 32);
    bool dup = false;
#pragma unroll
    for (int q = 0; q < m; ++q) dup |= (idx[q] == t);
    idx[m] = dup ? static_cast<int>(j) : t;
  }
}

// ----------------------------------------------------------------------------------------
// Reciprocal square root and reciprocal to float64 accuracy (a few ulp, not correctly
// rounded) from the hardware estimates v_rsq_f64 / v_rcp_f64 and two Newton steps: ~6
// dependent FMAs instead of the correctly rounded library sequences (range scaling, class
// checks, div_scale / div_fixup).  The minimal solves are latency bound, and their parity
// bar (1e-9 on F) is far above a few ulp.  x must be positive and finite.
// ----------------------------------------------------------------------------------------
__device__ __forceinline__ double rsqrt_fast(double x) {
  double y = __builtin_amdgcn_rsq(x);
  double r = fma(-x * y, y, 1.0);  // 1 - x y^2
  y = fma(0.5 * y, r, y);
  r = fma(-x * y, y, 1.0);
  return fma(0.5 * y, r, y);
}
__device__ __forceinline__ double rcp_fast(double x) {
  double y = __builtin_amdgcn_rcp(x);
  double e = fma(-x, y, 1.0);
  y = fma(y, e, y);
  e = fma(-x, y, 1.0);
  return fma(y, e, y);
}

// fp32 model of the counting kernel k_f8_count32q for the float64 F of hypothesis h: F~ = T1^T
// F T2 (T_i = [[s,0,cx_i],[0,s,cy_i],[0,0,1]]) scaled to max |F~_ij| = 1, into F32soa (9 x ld),
// and (G4 non-null) its decision constants from the guard bounds (T, De, Dn) of the frame
// (f8_kernels.hip above k_f8_count32q).
__device__ __forceinline__ void f32_model(const double (&F)[9], const Frame &fr, double gT,
                                          double gDe, double gDn, float *__restrict__ F32soa,
                                          float4 *__restrict__ G4, int64_t ld, int64_t h) {
  double G[9];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    G[3 * r + 0] = F[3 * r + 0] * fr.s;
    G[3 * r + 1] = F[3 * r + 1] * fr.s;
    G[3 * r + 2] = F[3 * r + 0] * fr.cx2 + F[3 * r + 1] * fr.cy2 + F[3 * r + 2];
  }
  double Ft[9];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    Ft[0 + c] = fr.s * G[0 + c];
    Ft[3 + c] = fr.s * G[3 + c];
    Ft[6 + c] = fr.cx1 * G[0 + c] + fr.cy1 * G[3 + c] + G[6 + c];
  }
  double mx = 0.0;
#pragma unroll
  for (int k = 0; k < 9; ++k) mx = fmax(mx, fabs(Ft[k]));
  const double kap = 1.0 / mx;  // F = 0 or non-finite -> NaN model, counts 0 on both paths
#pragma unroll
  for (int k = 0; k < 9; ++k) F32soa[k * ld + h] = static_cast<float>(Ft[k] * kap);
  if (G4) {
    // decision constants, AM-GM split point c = t~ sqrt(m at the frame centre) (any c > 0 is
    // rigorous; this one keeps the band near the exact-|e| band)
    const double u = 0x1p-24, T = gT, De = gDe, Dn = gDn;
    const double f02 = Ft[2] * kap, f12 = Ft[5] * kap, f20 = Ft[6] * kap, f21 = Ft[7] * kap;
    const double mc = fmin(f02 * f02 + f12 * f12, f20 * f20 + f21 * f21);
    // (rsqrt_fast / rcp_fast: a few ulp, far inside the 1 -/+ 4u and 1.02 margins)
    const double tm = T * fmax(mc, 1e-12);
    const double c = fmax(tm * rsqrt_fast(tm), 100.0 * De);
    const double r = De * rcp_fast(c);
    const double ip = rcp_fast(1.0 + r), im = rcp_fast(1.0 - r);
    const double alpha = T * (1.0 - u) * rcp_fast(1.0 + u) * ip * (1.0 - 4.0 * u);
    const double beta = T * (1.0 + u) * rcp_fast(1.0 - u) * im * (1.0 + 4.0 * u);
    const double ki = 1.02 * (De * c + De * De + T * Dn) * ip + 1e-30;
    const double ko = 1.02 * (T * Dn + De * c) * im + 1e-30;
    G4[h] = make_float4(static_cast<float>(ki), -static_cast<float>(ko), static_cast<float>(alpha),
                        static_cast<float>(beta));
  }
}

// ----------------------------------------------------------------------------------------
// One-sided Jacobi SVD of a 3x3 matrix (row-major M).  On exit the columns of B = M V are
// mutually orthogonal (their norms are the singular values) and V holds the right
// singular vectors as columns.
// ----------------------------------------------------------------------------------------
__device__ __forceinline__ void jacobi_rot(double (&B)[9], double (&V)[9], int p, int q,
                                           bool &rotated) {
  const double a = B[p] * B[p] + B[3 + p] * B[3 + p] + B[6 + p] * B[6 + p];
  const double b = B[q] * B[q] + B[3 + q] * B[3 + q] + B[6 + q] * B[6 + q];
  const double g = B[p] * B[q] + B[3 + p] * B[3 + q] + B[6 + p] * B[6 + q];
  if (g * g > 1e-30 * (a * b)) {  // |g| > 1e-15 sqrt(a b) without the square root
    rotated = true;
    const double zeta = (b - a) * (0.5 * rcp_fast(g));
    // t = sign(zeta) / (|zeta| + sqrt(1 + zeta^2)); 1 / (2 zeta) where zeta^2 would overflow
    const double az = fabs(zeta), z2 = fma(zeta, zeta, 1.0);
    const double t = az < 1e150 ? copysign(rcp_fast(az + z2 * rsqrt_fast(z2)), zeta)
                                : 0.5 * rcp_fast(zeta);
    const double c = rsqrt_fast(fma(t, t, 1.0));
    const double s = c * t;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const double bp = B[3 * r + p], bq = B[3 * r + q];
      B[3 * r + p] = c * bp - s * bq;
      B[3 * r + q] = s * bp + c * bq;
      const double vp = V[3 * r + p], vq = V[3 * r + q];
      V[3 * r + p] = c * vp - s * vq;
      V[3 * r + q] = s * vp + c * vq;
    }
  }
}

__device__ __forceinline__ void svd3_jacobi(double (&B)[9], double (&V)[9]) {
#pragma unroll
  for (int i = 0; i < 9; ++i) V[i] = (i % 4 == 0) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 12; ++sweep) {
    bool rotated = false;
    jacobi_rot(B, V, 0, 1, rotated);
    jacobi_rot(B, V, 0, 2, rotated);
    jacobi_rot(B, V, 1, 2, rotated);
    if (!rotated) break;
  }
}

// Nearest rank-2 matrix (lab3.py:321-324: U diag(s0, s1, 0) V): drop the term of the
// smallest singular value, F2 = sum_{j != min} b_j v_j^T.
__device__ __forceinline__ void enforce_rank2(const double (&Fs)[9], double (&F2)[9]) {
  double B[9], V[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) B[i] = Fs[i];
  svd3_jacobi(B, V);
  double s[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) s[j] = B[j] * B[j] + B[3 + j] * B[3 + j] + B[6 + j] * B[6 + j];
  const int m = (s[0] <= s[1] && s[0] <= s[2]) ? 0 : (s[1] <= s[2] ? 1 : 2);
  const double w0 = m == 0 ? 0.0 : 1.0, w1 = m == 1 ? 0.0 : 1.0, w2 = m == 2 ? 0.0 : 1.0;
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c)
      F2[3 * r + c] = w0 * B[3 * r + 0] * V[3 * c + 0] + w1 * B[3 * r + 1] * V[3 * c + 1] +
                      w2 * B[3 * r + 2] * V[3 * c + 2];
}

// Nearest rank-2 matrix by the smallest right singular vector: F2 = Fs (I - v v^T), the same
// matrix as U diag(s0, s1, 0) V^T.  v is the eigenvector of M = Fs^T Fs for its smallest
// eigenvalue l0: Newton from 0 on det(M - l I) = -l^3 + c2 l^2 - c1 l + c0 (monotone to the
// smallest root; 4.7 steps on average, <= 12 for 99.99 % of 8-point samples), then the
// largest column of adj(M - l0 I) = (l1 - l0)(l2 - l0) v v^T.  About 150 flops on a short
// dependent chain instead of 4-6 Jacobi sweeps.  Returns false (and leaves F2 alone) when
// Newton has not converged in 40 steps or the gap product is below 1e-12 c2^2 (near-double
// smallest singular value: the caller falls back to the Jacobi SVD).  Host prototype
// against numpy's SVD over 40 000 C2 samples: max deviation 2.4e-11 after normalisation,
// one fallback.
__device__ __forceinline__ bool enforce_rank2_adj(const double (&Fs)[9], double (&F2)[9]) {
  double M[9];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = r; c < 3; ++c) {
      const double v = fma(Fs[r], Fs[c], fma(Fs[3 + r], Fs[3 + c], Fs[6 + r] * Fs[6 + c]));
      M[3 * r + c] = v;
      M[3 * c + r] = v;
    }
  const double c2 = M[0] + M[4] + M[8];
  const double m01 = fma(M[4], M[8], -M[5] * M[5]);
  const double m02 = fma(M[0], M[8], -M[2] * M[2]);
  const double m12 = fma(M[0], M[4], -M[1] * M[1]);
  const double c1 = m01 + m02 + m12;
  const double c0 = M[0] * m01 - M[1] * fma(M[1], M[8], -M[5] * M[2]) +
                    M[2] * fma(M[1], M[5], -M[4] * M[2]);
  double lam = 0.0;
  bool conv = false;
  for (int it = 0; it < 40; ++it) {
    const double p = fma(fma(c2 - lam, lam, -c1), lam, c0);        // p(lam)
    const double ndp = fma(fma(3.0, lam, -2.0 * c2), lam, c1);     // -p'(lam) > 0 below l0
    const double st = p * rcp_fast(ndp);
    lam += st;
    if (fabs(st) <= 1e-15 * c2) {
      conv = true;
      break;
    }
  }
  if (!conv) return false;
  const double a00 = M[0] - lam, a11 = M[4] - lam, a22 = M[8] - lam;
  const double a01 = M[1], a02 = M[2], a12 = M[5];
  const double d0 = fma(a11, a22, -a12 * a12), d1 = fma(a00, a22, -a02 * a02),
               d2 = fma(a00, a11, -a01 * a01);
  double v0, v1, v2, dj;
  if (d0 >= d1 && d0 >= d2) {
    v0 = d0; v1 = fma(a12, a02, -a01 * a22); v2 = fma(a01, a12, -a11 * a02); dj = d0;
  } else if (d1 >= d2) {
    v0 = fma(a02, a12, -a01 * a22); v1 = d1; v2 = fma(a01, a02, -a00 * a12); dj = d1;
  } else {
    v0 = fma(a01, a12, -a02 * a11); v1 = fma(a02, a01, -a00 * a12); v2 = d2; dj = d2;
  }
  if (!(dj > 1e-12 * c2 * c2)) return false;  // also false for NaN
  const double inv = rsqrt_fast(fma(v0, v0, fma(v1, v1, v2 * v2)));
  v0 *= inv;
  v1 *= inv;
  v2 *= inv;
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    const double w = fma(Fs[3 * r], v0, fma(Fs[3 * r + 1], v1, Fs[3 * r + 2] * v2));  // Fs v
    F2[3 * r + 0] = fma(-w, v0, Fs[3 * r + 0]);
    F2[3 * r + 1] = fma(-w, v1, Fs[3 * r + 1]);
    F2[3 * r + 2] = fma(-w, v2, Fs[3 * r + 2]);
  }
  return true;
}

// ----------------------------------------------------------------------------------------
// Null vector of an R x C (R < C) matrix by Householder LQ: A Q = [L 0], null = Q e_{C-1}.
// The reflector of row k is stored in place of row k (entries k..C-1).  For R = C-1 and
// rank R this is the (unique up to sign) unit null vector, i.e. numpy svd's V[-1].
// ----------------------------------------------------------------------------------------
template <int R, int C>
__device__ __forceinline__ void lq_null_vector(double (&A)[R][C], double (&q)[C]) {
  double tau[R];
#pragma unroll
  for (int k = 0; k < R; ++k) {
    double ss = 0.0;
#pragma unroll
    for (int j = k; j < C; ++j) ss = fma(A[k][j], A[k][j], ss);
    const double nrm = ss > 0.0 ? ss * rsqrt_fast(ss) : 0.0;
    const double akk = A[k][k];
    const double alpha = akk >= 0.0 ? -nrm : nrm;
    const double denom = nrm * (nrm + fabs(akk));  // = v.v / 2
    const double tk = denom > 0.0 ? rcp_fast(denom) : 0.0;
    A[k][k] = akk - alpha;
    tau[k] = tk;
#pragma unroll
    for (int i = k + 1; i < R; ++i) {
      double w = 0.0;
#pragma unroll
      for (int j = k; j < C; ++j) w = fma(A[i][j], A[k][j], w);
      w *= tk;
#pragma unroll
      for (int j = k; j < C; ++j) A[i][j] = fma(-w, A[k][j], A[i][j]);
    }
  }
#pragma unroll
  for (int j = 0; j < C; ++j) q[j] = (j == C - 1) ? 1.0 : 0.0;
#pragma unroll
  for (int k = R - 1; k >= 0; --k) {
    double w = 0.0;
#pragma unroll
    for (int j = k; j < C; ++j) w = fma(A[k][j], q[j], w);
    w *= tau[k];
#pragma unroll
    for (int j = k; j < C; ++j) q[j] = fma(-w, A[k][j], q[j]);
  }
}

// numpy pairwise_sum order for exactly 8 contiguous values.
__device__ __forceinline__ double sum8(const double (&a)[8]) {
  return ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
}

// lab3.py:288-295 for N = 8: H = [[s, 0, ox], [0, s, oy], [0, 0, 1]], s = 1/L, o = -m/L.
__device__ __forceinline__ void scaling8(const double (&x)[8], const double (&y)[8], double &s,
                                         double &ox, double &oy) {
  const double xm = sum8(x) / 8.0;
  const double ym = sum8(y) / 8.0;
  double r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const double dx = x[j] - xm, dy = y[j] - ym;
    r[j] = __dadd_rn(__dmul_rn(dx, dx), __dmul_rn(dy, dy));
  }
  const double L = sqrt(0.0625 * sum8(r));  // 1./2./N with N = 8
  s = 1.0 / L;
  ox = -xm / L;
  oy = -ym / L;
}

// The 8-point algorithm of lab3.fmatrix_stls (lab3.py:269-329) on one minimal sample.
// xl, yl: left points (p1), xr, yr: right points (p2).  F row-major, pl^T F pr = 0.
__device__ __forceinline__ void fmatrix8(const double (&xl)[8], const double (&yl)[8],
                                         const double (&xr)[8], const double (&yr)[8],
                                         double (&F)[9]) {
  double s1, ox1, oy1, s2, ox2, oy2;
  scaling8(xl, yl, s1, ox1, oy1);
  scaling8(xr, yr, s2, ox2, oy2);
  double A[8][9];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    // map_homography (lab3.py:301-306): x*H00 + y*H01 + H02 with H01 = 0
    const double X = __dadd_rn(__dmul_rn(xl[k], s1), ox1);
    const double Y = __dadd_rn(__dmul_rn(yl[k], s1), oy1);
    const double x = __dadd_rn(__dmul_rn(xr[k], s2), ox2);
    const double y = __dadd_rn(__dmul_rn(yr[k], s2), oy2);
    // lab3.py:314: [X x, X y, X, Y x, Y y, Y, x, y, 1]
    A[k][0] = X * x;
    A[k][1] = X * y;
    A[k][2] = X;
    A[k][3] = Y * x;
    A[k][4] = Y * y;
    A[k][5] = Y;
    A[k][6] = x;
    A[k][7] = y;
    A[k][8] = 1.0;
  }
  double fs[9];
  lq_null_vector<8, 9>(A, fs);  // lab3.py:317-318: V[-1] of svd(A)
  double F2[9];
  if (!enforce_rank2_adj(fs, F2)) enforce_rank2(fs, F2);
  // lab3.py:327: F = S^T (F2 T); S = H(s1, ox1, oy1), T = H(s2, ox2, oy2)
  double M[9];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    M[3 * r + 0] = F2[3 * r + 0] * s2;
    M[3 * r + 1] = F2[3 * r + 1] * s2;
    M[3 * r + 2] = (F2[3 * r + 0] * ox2 + F2[3 * r + 1] * oy2) + F2[3 * r + 2];
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    F[0 + c] = s1 * M[0 + c];
    F[3 + c] = s1 * M[3 + c];
    F[6 + c] = (ox1 * M[0 + c] + oy1 * M[3 + c]) + M[6 + c];
  }
}

// Reference-order distance d = max(|res1|, |res2|) of lab3.fmatrix_residuals (lab3.py:
// 210-227) followed by fun.py:316 (NaN-propagating max).  No FMA contraction.
__device__ __forceinline__ double dist_ref(const double (&f)[9], const Pt &p) {
#pragma clang fp contract(off)
  const double l10 = (f[0] * p.x2 + f[1] * p.y2) + f[2];
  const double l11 = (f[3] * p.x2 + f[4] * p.y2) + f[5];
  const double l12 = (f[6] * p.x2 + f[7] * p.y2) + f[8];
  const double l20 = (f[0] * p.x1 + f[3] * p.y1) + f[6];
  const double l21 = (f[1] * p.x1 + f[4] * p.y1) + f[7];
  const double l22 = (f[2] * p.x1 + f[5] * p.y1) + f[8];
  const double l1s = sqrt(l10 * l10 + l11 * l11);
  const double l2s = sqrt(l20 * l20 + l21 * l21);
  const double r1 = ((l10 * p.x1 + l11 * p.y1) + l12) / l1s;
  const double r2 = ((l20 * p.x2 + l21 * p.y2) + l22) / l2s;
  const double a1 = fabs(r1), a2 = fabs(r2);
  return (a1 != a1 || a2 != a2) ? __longlong_as_double(0x7ff8000000000000LL)
                                : (a1 > a2 ? a1 : a2);
}

__device__ __forceinline__ void residuals_ref(const double (&f)[9], const Pt &p, double &r1,
                                              double &r2) {
#pragma clang fp contract(off)
  const double l10 = (f[0] * p.x2 + f[1] * p.y2) + f[2];
  const double l11 = (f[3] * p.x2 + f[4] * p.y2) + f[5];
  const double l12 = (f[6] * p.x2 + f[7] * p.y2) + f[8];
  const double l20 = (f[0] * p.x1 + f[3] * p.y1) + f[6];
  const double l21 = (f[1] * p.x1 + f[4] * p.y1) + f[7];
  const double l22 = (f[2] * p.x1 + f[5] * p.y1) + f[8];
  r1 = ((l10 * p.x1 + l11 * p.y1) + l12) / sqrt(l10 * l10 + l11 * l11);
  r2 = ((l20 * p.x2 + l21 * p.y2) + l22) / sqrt(l20 * l20 + l21 * l21);
}

}  // namespace rsd
