// Minimal PnP solvers for the cv.solvePnPRansac / cv.solvePnP drop-ins (tables.py:141-145,
// pnp.py:7-10), one GPU lane per pose:
//
//   epnp_pose   EPnP (Lepetit, Moreno-Noguer, Fua 2009) as OpenCV's SOLVEPNP_EPNP runs it --
//               the RANSAC kernel of cv::solvePnPRansac (5-point samples) and cv::solvePnP's
//               EPNP flag: four control points (centroid + principal axes scaled by
//               sqrt(eigenvalue / n)), barycentric coordinates, the 2n x 12 system M through
//               M^T M, its four smallest eigenvectors (cyclic Jacobi), betas by the three
//               linearisations (N = 4, 2, 3 null vectors), five Gauss-Newton steps each, the
//               camera-frame points, sign, and absolute orientation (Procrustes); the candidate
//               with the smallest mean reprojection error wins;
//   p3p_pose    Lambda Twist P3P (Persson & Nordberg 2018): the depths lambda of three points
//               solve lambda^T M_ij lambda = a_ij; a real root gamma of det(D1 + gamma D2) = 0
//               makes D0 = D1 + gamma D2 a degenerate conic, whose eigen-decomposition with the
//               known zero eigenvalue gives the two planes of lambda; each plane leaves a
//               quadratic in lambda_i / lambda_j; three Gauss-Newton steps on the distances;
//               R, t from the three point pairs.  The fourth point picks among the (<= 4)
//               solutions, as OpenCV's SOLVEPNP_P3P does.  (The reference's own p3p_twist,
//               pnp.py:61-121, stops after the eigen-decomposition; its cubic also takes
//               the gamma^1 and gamma^2 coefficients in swapped places.)
//
// Image points are C-normalised (u, v) = pi(K^-1 [px, py, 1]); world points (X, Y, Z).  The
// point source is an accessor pt(q) -> PPt, so the same code serves a sampled tuple and all m
// correspondences.
#pragma once

#include <cmath>

namespace rsd {

// A mirrored minimal pose (all depths negated) replaces the best front-facing one only when
// its error is below kMirrorWins times the front-facing error (on noise-free negative-scale
// views the ratio is ~1e-10; with noisy pixels a 4-point P3P mirror reached 0.27 of the
// front-facing error on positive-depth data, tests/test_gpu_pnp.py): OpenCV's EPnP / P3P return
// front-facing poses only, and the reprojection error x / z cannot tell the two apart on a
// near-degenerate sample.
constexpr double kMirrorWins = 1e-2;
__device__ inline bool mirror_wins(double e_mirror, double e_front) {
  return e_mirror < kMirrorWins * e_front || (e_front != e_front && e_mirror == e_mirror);
}

// cyclic Jacobi eigen-decomposition of a symmetric N x N matrix (row-major; destroyed):
// eigenvalues on the diagonal of A, eigenvectors in the columns of V
template <int N>
__device__ inline void sym_jacobi(double (&A)[N * N], double (&V)[N * N]) {
  for (int i = 0; i < N * N; ++i) V[i] = (i % (N + 1) == 0) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 30; ++sweep) {
    double off = 0.0, dia = 0.0;
    for (int p = 0; p < N; ++p) {
      dia += A[p * N + p] * A[p * N + p];
      for (int q = p + 1; q < N; ++q) off += A[p * N + q] * A[p * N + q];
    }
    if (!(off > 1e-30 * dia)) break;
    for (int p = 0; p < N - 1; ++p)
      for (int q = p + 1; q < N; ++q) {
        const double apq = A[p * N + q];
        if (apq == 0.0) continue;
        const double app = A[p * N + p], aqq = A[q * N + q];
        const double th = (aqq - app) / (2.0 * apq);
        const double t = (th >= 0.0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1.0));
        const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < N; ++k) {  // columns p, q
          const double akp = A[k * N + p], akq = A[k * N + q];
          A[k * N + p] = c * akp - s * akq;
          A[k * N + q] = s * akp + c * akq;
        }
        for (int k = 0; k < N; ++k) {  // rows p, q
          const double apk = A[p * N + k], aqk = A[q * N + k];
          A[p * N + k] = c * apk - s * aqk;
          A[q * N + k] = s * apk + c * aqk;
        }
        for (int k = 0; k < N; ++k) {
          const double vkp = V[k * N + p], vkq = V[k * N + q];
          V[k * N + p] = c * vkp - s * vkq;
          V[k * N + q] = s * vkp + c * vkq;
        }
      }
  }
}

// least squares min |A x - b| for a 6 x K system by Householder QR (K <= 5); false if rank
// deficient
template <int K>
__device__ inline bool lsq6(double (&A)[6][K], double (&b)[6], double (&x)[K]) {
  for (int k = 0; k < K; ++k) {
    double ss = 0.0;
    for (int i = k; i < 6; ++i) ss += A[i][k] * A[i][k];
    const double nrm = sqrt(ss);
    if (!(nrm > 0.0)) return false;
    const double alpha = A[k][k] > 0.0 ? -nrm : nrm;
    const double v0 = A[k][k] - alpha;
    // v = (v0, A[k+1..][k]); H = I - 2 v v^T / v^T v
    const double vtv = v0 * v0 + (ss - A[k][k] * A[k][k]);
    if (!(vtv > 0.0)) {
      A[k][k] = alpha;
      continue;
    }
    for (int j = k + 1; j < K; ++j) {
      double d = v0 * A[k][j];
      for (int i = k + 1; i < 6; ++i) d += A[i][k] * A[i][j];
      const double f = 2.0 * d / vtv;
      A[k][j] -= f * v0;
      for (int i = k + 1; i < 6; ++i) A[i][j] -= f * A[i][k];
    }
    double d = v0 * b[k];
    for (int i = k + 1; i < 6; ++i) d += A[i][k] * b[i];
    const double f = 2.0 * d / vtv;
    b[k] -= f * v0;
    for (int i = k + 1; i < 6; ++i) b[i] -= f * A[i][k];
    A[k][k] = alpha;
  }
  for (int k = K - 1; k >= 0; --k) {
    double s = b[k];
    for (int j = k + 1; j < K; ++j) s -= A[k][j] * x[j];
    if (!(A[k][k] != 0.0)) return false;
    x[k] = s / A[k][k];
  }
  return true;
}

__device__ inline void cross3(const double *a, const double *b, double *c) {
  c[0] = a[1] * b[2] - a[2] * b[1];
  c[1] = a[2] * b[0] - a[0] * b[2];
  c[2] = a[0] * b[1] - a[1] * b[0];
}
__device__ inline double dot3(const double *a, const double *b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}

// R = U V^T of the 3 x 3 matrix M (absolute orientation), det R = +1 (OpenCV's EPnP flips the
// last row when the product comes out a reflection)
__device__ inline void procrustes3(const double (&M)[9], double (&R)[9]) {
  double B[9], V[9];
  for (int i = 0; i < 9; ++i) B[i] = M[i];
  svd3_jacobi(B, V);  // B = U S (columns), V right singular vectors
  double U[9], s[3];
  for (int j = 0; j < 3; ++j) {
    s[j] = sqrt(B[j] * B[j] + B[3 + j] * B[3 + j] + B[6 + j] * B[6 + j]);
    const double is = s[j] > 0.0 ? 1.0 / s[j] : 0.0;
    for (int r = 0; r < 3; ++r) U[3 * r + j] = B[3 * r + j] * is;
  }
  // a zero singular value (planar or collinear configurations): complete U by the cross
  // product of the other two columns
  int z = s[0] <= s[1] && s[0] <= s[2] ? 0 : (s[1] <= s[2] ? 1 : 2);
  if (!(s[z] > 1e-300)) {
    const int a = (z + 1) % 3, b = (z + 2) % 3;
    const double ua[3] = {U[a], U[3 + a], U[6 + a]}, ub[3] = {U[b], U[3 + b], U[6 + b]};
    double c[3];
    cross3(ua, ub, c);
    for (int r = 0; r < 3; ++r) U[3 * r + z] = c[r];
  }
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c)
      R[3 * r + c] = U[3 * r] * V[3 * c] + U[3 * r + 1] * V[3 * c + 1] + U[3 * r + 2] * V[3 * c + 2];
  const double det = R[0] * (R[4] * R[8] - R[5] * R[7]) - R[1] * (R[3] * R[8] - R[5] * R[6]) +
                     R[2] * (R[3] * R[7] - R[4] * R[6]);
  if (det < 0.0)
    for (int c = 0; c < 3; ++c) R[6 + c] = -R[6 + c];
}

// ---- EPnP ----------------------------------------------------------------------------------
template <class PtAt>
__device__ inline double epnp_pose(PtAt pt, int n, double (&R)[9], double (&t)[3]) {
  // control points: centroid + principal axes
  double c0[3] = {0.0, 0.0, 0.0};
  for (int q = 0; q < n; ++q) {
    const PPt p = pt(q);
    c0[0] += p.X;
    c0[1] += p.Y;
    c0[2] += p.Z;
  }
  for (int k = 0; k < 3; ++k) c0[k] /= n;
  double C[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (int q = 0; q < n; ++q) {
    const PPt p = pt(q);
    const double d[3] = {p.X - c0[0], p.Y - c0[1], p.Z - c0[2]};
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) C[3 * r + c] += d[r] * d[c];
  }
  double Vc[9];
  svd3_jacobi(C, Vc);  // C V = U S: eigenvalues = column norms of C, eigenvectors = columns of V
  double ax[3][3], sc[3];  // axis j (unit), scale sqrt(lambda_j / n)
  for (int j = 0; j < 3; ++j) {
    const double lam = sqrt(C[j] * C[j] + C[3 + j] * C[3 + j] + C[6 + j] * C[6 + j]);
    sc[j] = sqrt(lam / n);
    for (int r = 0; r < 3; ++r) ax[j][r] = Vc[3 * r + j];
  }
  double cw[4][3];
  for (int r = 0; r < 3; ++r) cw[0][r] = c0[r];
  for (int j = 0; j < 3; ++j)
    for (int r = 0; r < 3; ++r) cw[1 + j][r] = c0[r] + sc[j] * ax[j][r];
  // barycentric coordinates: alpha_j = axis_j . (p - c0) / scale_j (the inverse of the
  // orthogonal control-point frame; a zero scale -- planar points -- gives 0, as a
  // pseudo-inverse does), alpha_0 = 1 - sum
  auto alphas = [&](const PPt &p, double (&a)[4]) {
    const double d[3] = {p.X - c0[0], p.Y - c0[1], p.Z - c0[2]};
    double s = 0.0;
    for (int j = 0; j < 3; ++j) {
      a[1 + j] = sc[j] > 0.0 ? dot3(ax[j], d) / sc[j] : 0.0;
      s += a[1 + j];
    }
    a[0] = 1.0 - s;
  };
  // M^T M of the rows [a_j, 0, -a_j u] and [0, a_j, -a_j v]
  double MtM[144];
  for (int i = 0; i < 144; ++i) MtM[i] = 0.0;
  for (int q = 0; q < n; ++q) {
    const PPt p = pt(q);
    double a[4];
    alphas(p, a);
    double r1[12], r2[12];
    for (int j = 0; j < 4; ++j) {
      r1[3 * j] = a[j];
      r1[3 * j + 1] = 0.0;
      r1[3 * j + 2] = -a[j] * p.u;
      r2[3 * j] = 0.0;
      r2[3 * j + 1] = a[j];
      r2[3 * j + 2] = -a[j] * p.v;
    }
    for (int r = 0; r < 12; ++r)
      for (int c = r; c < 12; ++c) MtM[12 * r + c] += r1[r] * r1[c] + r2[r] * r2[c];
  }
  for (int r = 0; r < 12; ++r)
    for (int c = 0; c < r; ++c) MtM[12 * r + c] = MtM[12 * c + r];
  double V[144];
  sym_jacobi<12>(MtM, V);
  // the four eigenvectors of the smallest eigenvalues, ascending (OpenCV's ut rows 11, 10, 9, 8)
  int ord[12];
  for (int i = 0; i < 12; ++i) ord[i] = i;
  for (int i = 1; i < 12; ++i)
    for (int j = i; j > 0 && MtM[13 * ord[j]] < MtM[13 * ord[j - 1]]; --j) {
      const int tmp = ord[j];
      ord[j] = ord[j - 1];
      ord[j - 1] = tmp;
    }
  double v[4][12];
  for (int i = 0; i < 4; ++i)
    for (int k = 0; k < 12; ++k) v[i][k] = V[12 * k + ord[i]];
  // L (6 x 10) and rho over the control-point pairs (0,1) (0,2) (0,3) (1,2) (1,3) (2,3)
  const int pa[6] = {0, 0, 0, 1, 1, 2}, pb[6] = {1, 2, 3, 2, 3, 3};
  double L[6][10], rho[6];
  for (int j = 0; j < 6; ++j) {
    double dv[4][3];
    for (int i = 0; i < 4; ++i)
      for (int k = 0; k < 3; ++k) dv[i][k] = v[i][3 * pa[j] + k] - v[i][3 * pb[j] + k];
    L[j][0] = dot3(dv[0], dv[0]);
    L[j][1] = 2.0 * dot3(dv[0], dv[1]);
    L[j][2] = dot3(dv[1], dv[1]);
    L[j][3] = 2.0 * dot3(dv[0], dv[2]);
    L[j][4] = 2.0 * dot3(dv[1], dv[2]);
    L[j][5] = dot3(dv[2], dv[2]);
    L[j][6] = 2.0 * dot3(dv[0], dv[3]);
    L[j][7] = 2.0 * dot3(dv[1], dv[3]);
    L[j][8] = 2.0 * dot3(dv[2], dv[3]);
    L[j][9] = dot3(dv[3], dv[3]);
    const double d0 = cw[pa[j]][0] - cw[pb[j]][0], d1 = cw[pa[j]][1] - cw[pb[j]][1],
                 d2 = cw[pa[j]][2] - cw[pb[j]][2];
    rho[j] = d0 * d0 + d1 * d1 + d2 * d2;
  }
  auto gauss_newton = [&](double (&b)[4]) {
    for (int it = 0; it < 5; ++it) {
      double A[6][4], r[6], dx[4];
      for (int j = 0; j < 6; ++j) {
        const double *l = L[j];
        A[j][0] = 2 * l[0] * b[0] + l[1] * b[1] + l[3] * b[2] + l[6] * b[3];
        A[j][1] = l[1] * b[0] + 2 * l[2] * b[1] + l[4] * b[2] + l[7] * b[3];
        A[j][2] = l[3] * b[0] + l[4] * b[1] + 2 * l[5] * b[2] + l[8] * b[3];
        A[j][3] = l[6] * b[0] + l[7] * b[1] + l[8] * b[2] + 2 * l[9] * b[3];
        r[j] = rho[j] - (l[0] * b[0] * b[0] + l[1] * b[0] * b[1] + l[2] * b[1] * b[1] +
                         l[3] * b[0] * b[2] + l[4] * b[1] * b[2] + l[5] * b[2] * b[2] +
                         l[6] * b[0] * b[3] + l[7] * b[1] * b[3] + l[8] * b[2] * b[3] +
                         l[9] * b[3] * b[3]);
      }
      if (!lsq6<4>(A, r, dx)) return;
      for (int k = 0; k < 4; ++k) b[k] += dx[k];
    }
  };
  // camera-frame pose of one beta vector; mean reprojection error (inf if degenerate)
  auto pose_of = [&](const double (&b)[4], bool mirror, double (&Ro)[9], double (&to)[3]) -> double {
    double cc[4][3];
    for (int j = 0; j < 4; ++j)
      for (int k = 0; k < 3; ++k)
        cc[j][k] = b[0] * v[0][3 * j + k] + b[1] * v[1][3 * j + k] + b[2] * v[2][3 * j + k] +
                   b[3] * v[3][3 * j + k];
    // sign: the first point in front of the camera (OpenCV's choice); with mirror set, the
    // other sign -- the camera frame of a P = K [R | t] carrying a negative scale, whose points
    // sit at z < 0 (BAdino2's cameras do)
    {
      double a[4];
      alphas(pt(0), a);
      const double z0 = a[0] * cc[0][2] + a[1] * cc[1][2] + a[2] * cc[2][2] + a[3] * cc[3][2];
      if ((z0 < 0.0) != mirror)
        for (int j = 0; j < 4; ++j)
          for (int k = 0; k < 3; ++k) cc[j][k] = -cc[j][k];
    }
    // Procrustes between the camera-frame points and the world points
    double pc0[3] = {0, 0, 0};
    for (int q = 0; q < n; ++q) {
      double a[4];
      alphas(pt(q), a);
      for (int k = 0; k < 3; ++k)
        pc0[k] += a[0] * cc[0][k] + a[1] * cc[1][k] + a[2] * cc[2][k] + a[3] * cc[3][k];
    }
    for (int k = 0; k < 3; ++k) pc0[k] /= n;
    double ABt[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int q = 0; q < n; ++q) {
      const PPt p = pt(q);
      double a[4];
      alphas(p, a);
      double pc[3];
      for (int k = 0; k < 3; ++k)
        pc[k] = a[0] * cc[0][k] + a[1] * cc[1][k] + a[2] * cc[2][k] + a[3] * cc[3][k] - pc0[k];
      const double pw[3] = {p.X - c0[0], p.Y - c0[1], p.Z - c0[2]};
      for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) ABt[3 * r + c] += pc[r] * pw[c];
    }
    procrustes3(ABt, Ro);
    for (int r = 0; r < 3; ++r)
      to[r] = pc0[r] - (Ro[3 * r] * c0[0] + Ro[3 * r + 1] * c0[1] + Ro[3 * r + 2] * c0[2]);
    double err = 0.0;
    for (int q = 0; q < n; ++q) {
      const PPt p = pt(q);
      const double x = Ro[0] * p.X + Ro[1] * p.Y + Ro[2] * p.Z + to[0];
      const double y = Ro[3] * p.X + Ro[4] * p.Y + Ro[5] * p.Z + to[1];
      const double z = Ro[6] * p.X + Ro[7] * p.Y + Ro[8] * p.Z + to[2];
      const double du = p.u - x / z, dv = p.v - y / z;
      err += sqrt(du * du + dv * dv);
    }
    err /= n;
    return err == err ? err : INFINITY;
  };
  // front-facing candidates (every point at z > 0 for the sign OpenCV picks) and mirrored ones
  // (the points behind the camera: a P = K [R | t] with a negative scale, BAdino2) are kept
  // apart; a mirrored pose wins only if clearly better (kMirrorWins), so on ordinary
  // positive-depth data the solver returns what OpenCV's EPnP returns
  double best = INFINITY, best_m = INFINITY, Rm[9], tm[3];
  for (int N = 1; N <= 3; ++N) {
    double b[4] = {0.0, 0.0, 0.0, 0.0};
    if (N == 1) {  // all four null vectors: b11 b12 b13 b14
      double A[6][4], r[6], x[4];
      for (int j = 0; j < 6; ++j) {
        A[j][0] = L[j][0];
        A[j][1] = L[j][1];
        A[j][2] = L[j][3];
        A[j][3] = L[j][6];
        r[j] = rho[j];
      }
      if (!lsq6<4>(A, r, x)) continue;
      const double s = x[0] < 0.0 ? -1.0 : 1.0;
      b[0] = sqrt(s * x[0]);
      if (!(b[0] > 0.0)) continue;
      b[1] = s * x[1] / b[0];
      b[2] = s * x[2] / b[0];
      b[3] = s * x[3] / b[0];
    } else if (N == 2) {  // b11 b12 b22
      double A[6][3], r[6], x[3];
      for (int j = 0; j < 6; ++j) {
        A[j][0] = L[j][0];
        A[j][1] = L[j][1];
        A[j][2] = L[j][2];
        r[j] = rho[j];
      }
      if (!lsq6<3>(A, r, x)) continue;
      if (x[0] < 0.0) {
        b[0] = sqrt(-x[0]);
        b[1] = x[2] < 0.0 ? sqrt(-x[2]) : 0.0;
      } else {
        b[0] = sqrt(x[0]);
        b[1] = x[2] > 0.0 ? sqrt(x[2]) : 0.0;
      }
      if (x[1] < 0.0) b[0] = -b[0];
    } else {  // b11 b12 b22 b13 b23
      double A[6][5], r[6], x[5];
      for (int j = 0; j < 6; ++j) {
        for (int k = 0; k < 5; ++k) A[j][k] = L[j][k];
        r[j] = rho[j];
      }
      if (!lsq6<5>(A, r, x)) continue;
      if (x[0] < 0.0) {
        b[0] = sqrt(-x[0]);
        b[1] = x[2] < 0.0 ? sqrt(-x[2]) : 0.0;
      } else {
        b[0] = sqrt(x[0]);
        b[1] = x[2] > 0.0 ? sqrt(x[2]) : 0.0;
      }
      if (x[1] < 0.0) b[0] = -b[0];
      if (!(b[0] != 0.0)) continue;
      b[2] = x[3] / b[0];
    }
    gauss_newton(b);
    for (int mirror = 0; mirror < 2; ++mirror) {
      double Rc[9], tc[3];
      const double e = pose_of(b, mirror != 0, Rc, tc);
      double &bb = mirror ? best_m : best;
      if (e < bb) {
        bb = e;
        for (int i = 0; i < 9; ++i) (mirror ? Rm : R)[i] = Rc[i];
        for (int i = 0; i < 3; ++i) (mirror ? tm : t)[i] = tc[i];
      }
    }
  }
  if (mirror_wins(best_m, best)) {
    for (int i = 0; i < 9; ++i) R[i] = Rm[i];
    for (int i = 0; i < 3; ++i) t[i] = tm[i];
    return best_m;
  }
  return best;
}

// ---- Lambda Twist P3P ----------------------------------------------------------------------
// real roots of c3 x^3 + c2 x^2 + c1 x + c0 (c3 != 0), Newton-polished; returns their number
__device__ inline int cubic_roots(double c3, double c2, double c1, double c0, double (&x)[3]) {
  const double a = c2 / c3, b = c1 / c3, c = c0 / c3;
  const double q = (a * a - 3.0 * b) / 9.0, r = (2.0 * a * a * a - 9.0 * a * b + 27.0 * c) / 54.0;
  int n;
  if (r * r < q * q * q) {  // three real roots (trigonometric)
    const double th = acos(fmin(1.0, fmax(-1.0, r / sqrt(q * q * q))));
    const double sq = -2.0 * sqrt(q);
    x[0] = sq * cos(th / 3.0) - a / 3.0;
    x[1] = sq * cos((th + 2.0 * M_PI) / 3.0) - a / 3.0;
    x[2] = sq * cos((th - 2.0 * M_PI) / 3.0) - a / 3.0;
    n = 3;
  } else {  // one real root (Cardano)
    const double A = -copysign(cbrt(fabs(r) + sqrt(r * r - q * q * q)), r);
    const double B = A != 0.0 ? q / A : 0.0;
    x[0] = (A + B) - a / 3.0;
    n = 1;
  }
  for (int i = 0; i < n; ++i)
    for (int it = 0; it < 2; ++it) {
      const double f = ((x[i] + a) * x[i] + b) * x[i] + c, fp = (3.0 * x[i] + 2.0 * a) * x[i] + b;
      if (fp != 0.0) x[i] -= f / fp;
    }
  return n;
}

// unit null vector of the symmetric 3 x 3 A: the largest cross product of two of its rows
__device__ inline void null3(const double (&A)[9], double (&v)[3]) {
  double c[3][3];
  cross3(A, A + 3, c[0]);
  cross3(A, A + 6, c[1]);
  cross3(A + 3, A + 6, c[2]);
  int k = 0;
  double best = dot3(c[0], c[0]);
  for (int i = 1; i < 3; ++i) {
    const double d = dot3(c[i], c[i]);
    if (d > best) {
      best = d;
      k = i;
    }
  }
  const double in = best > 0.0 ? 1.0 / sqrt(best) : 0.0;
  for (int r = 0; r < 3; ++r) v[r] = c[k][r] * in;
}

// Up to four poses from three correspondences (world X[i], unit bearings y[i]), each with its
// mirror (all depths negated); returns their number.
__device__ inline int p3p_lambda_twist(const double (&X)[3][3], const double (&y)[3][3],
                                       double (&Rs)[8][9], double (&ts)[8][3],
                                       bool (&mirrored)[8]) {
  const double b01 = dot3(y[0], y[1]), b02 = dot3(y[0], y[2]), b12 = dot3(y[1], y[2]);
  double d01[3], d02[3], d12[3];
  for (int k = 0; k < 3; ++k) {
    d01[k] = X[0][k] - X[1][k];
    d02[k] = X[0][k] - X[2][k];
    d12[k] = X[1][k] - X[2][k];
  }
  const double a01 = dot3(d01, d01), a02 = dot3(d02, d02), a12 = dot3(d12, d12);
  // D1 = a12 M01 - a01 M12, D2 = a12 M02 - a02 M12 (row-major, symmetric)
  const double D1[9] = {a12, -a12 * b01, 0.0, -a12 * b01, a12 - a01, a01 * b12, 0.0, a01 * b12, -a01};
  const double D2[9] = {a12, 0.0, -a12 * b02, 0.0, -a02, a02 * b12, -a12 * b02, a02 * b12, a12 - a02};
  auto col = [](const double (&D)[9], int j, double (&c)[3]) {
    c[0] = D[j];
    c[1] = D[3 + j];
    c[2] = D[6 + j];
  };
  double A0[3], A1[3], A2[3], B0[3], B1[3], B2[3], t0[3];
  col(D1, 0, A0);
  col(D1, 1, A1);
  col(D1, 2, A2);
  col(D2, 0, B0);
  col(D2, 1, B1);
  col(D2, 2, B2);
  // det(D1 + g D2) = c3 g^3 + c2 g^2 + c1 g + c0: g^2 takes one column of D1 and two of D2,
  // g^1 two columns of D1 and one of D2
  cross3(B1, B2, t0);
  const double c3 = dot3(B0, t0);
  double c2 = dot3(A0, t0);
  cross3(B2, B0, t0);
  c2 += dot3(A1, t0);
  cross3(B0, B1, t0);
  c2 += dot3(A2, t0);
  cross3(A1, A2, t0);
  const double c0 = dot3(A0, t0);
  double c1 = dot3(B0, t0);
  cross3(A2, A0, t0);
  c1 += dot3(B1, t0);
  cross3(A0, A1, t0);
  c1 += dot3(B2, t0);
  if (!(c3 != 0.0)) return 0;
  double g[3];
  const int ng = cubic_roots(c3, c2, c1, c0, g);
  const double a[3][3] = {{0.0, a01, a02}, {a01, 0.0, a12}, {a02, a12, 0.0}};
  const double bb[3][3] = {{1.0, b01, b02}, {b01, 1.0, b12}, {b02, b12, 1.0}};
  int ns = 0;
  for (int gi = 0; gi < ng; ++gi) {
    double D0[9];
    for (int i = 0; i < 9; ++i) D0[i] = D1[i] + g[gi] * D2[i];
    // eigen-decomposition with the known zero eigenvalue: sigma0 + sigma1 = trace, sigma0
    // sigma1 = the sum of the principal 2 x 2 minors
    const double T = D0[0] + D0[4] + D0[8];
    const double P = (D0[0] * D0[4] - D0[1] * D0[1]) + (D0[0] * D0[8] - D0[2] * D0[2]) +
                     (D0[4] * D0[8] - D0[5] * D0[5]);
    if (!(P < 0.0)) continue;  // the conic must be a real line pair (indefinite)
    const double sq = sqrt(T * T - 4.0 * P);
    const double s0 = T >= 0.0 ? 0.5 * (T + sq) : 0.5 * (T - sq);
    const double s1 = P / s0;
    double e0[3], e1[3];
    {
      double A[9];
      for (int i = 0; i < 9; ++i) A[i] = D0[i] - (i % 4 == 0 ? s0 : 0.0);
      null3(A, e0);
      for (int i = 0; i < 9; ++i) A[i] = D0[i] - (i % 4 == 0 ? s1 : 0.0);
      null3(A, e1);
    }
    for (int sg = 0; sg < 2; ++sg) {
      // sigma0 (e0.l)^2 + sigma1 (e1.l)^2 = 0: (e1 - tt e0) . lambda = 0
      const double tt = (sg ? -1.0 : 1.0) * sqrt(-s0 / s1);
      const double nv[3] = {e1[0] - tt * e0[0], e1[1] - tt * e0[1], e1[2] - tt * e0[2]};
      int k = 0;
      if (fabs(nv[1]) > fabs(nv[k])) k = 1;
      if (fabs(nv[2]) > fabs(nv[k])) k = 2;
      const int o1 = (k + 1) % 3, o2 = (k + 2) % 3;
      // lambda_k = w1 lambda_o1 + w2 lambda_o2; tau = lambda_o1 / lambda_o2
      const double w1 = -nv[o1] / nv[k], w2 = -nv[o2] / nv[k];
      const double aq = a[o1][o2], bq = bb[o1][o2], ap = a[k][o1], bp = bb[k][o1];
      const double q2 = aq * (w1 * w1 + 1.0 - 2.0 * bp * w1) - ap;
      const double q1 = aq * (2.0 * w1 * w2 - 2.0 * bp * w2) + 2.0 * ap * bq;
      const double q0 = aq * w2 * w2 - ap;
      const double disc = q1 * q1 - 4.0 * q2 * q0;
      if (!(disc >= 0.0) || q2 == 0.0) continue;
      const double sd = sqrt(disc);
      for (int rt = 0; rt < 2 && ns < 8; ++rt) {
        const double tau = (-q1 + (rt ? -sd : sd)) / (2.0 * q2);
        if (!(tau > 0.0)) continue;
        const double den = tau * tau - 2.0 * bq * tau + 1.0;
        if (!(den > 0.0)) continue;
        double lam[3];
        lam[o2] = sqrt(aq / den);
        lam[o1] = tau * lam[o2];
        lam[k] = w1 * lam[o1] + w2 * lam[o2];
        if (!(lam[0] > 0.0 && lam[1] > 0.0 && lam[2] > 0.0)) continue;
        // Gauss-Newton on lambda_i^2 + lambda_j^2 - 2 b_ij lambda_i lambda_j = a_ij
        for (int it = 0; it < 3; ++it) {
          const double r[3] = {lam[0] * lam[0] + lam[1] * lam[1] - 2.0 * b01 * lam[0] * lam[1] - a01,
                               lam[0] * lam[0] + lam[2] * lam[2] - 2.0 * b02 * lam[0] * lam[2] - a02,
                               lam[1] * lam[1] + lam[2] * lam[2] - 2.0 * b12 * lam[1] * lam[2] - a12};
          const double J[9] = {2.0 * (lam[0] - b01 * lam[1]), 2.0 * (lam[1] - b01 * lam[0]), 0.0,
                               2.0 * (lam[0] - b02 * lam[2]), 0.0, 2.0 * (lam[2] - b02 * lam[0]),
                               0.0, 2.0 * (lam[1] - b12 * lam[2]), 2.0 * (lam[2] - b12 * lam[1])};
          const double det = J[0] * (J[4] * J[8] - J[5] * J[7]) - J[1] * (J[3] * J[8] - J[5] * J[6]) +
                             J[2] * (J[3] * J[7] - J[4] * J[6]);
          if (!(fabs(det) > 0.0)) break;
          // lam -= J^-1 r (adjugate / det)
          const double inv[9] = {J[4] * J[8] - J[5] * J[7], J[2] * J[7] - J[1] * J[8], J[1] * J[5] - J[2] * J[4],
                                 J[5] * J[6] - J[3] * J[8], J[0] * J[8] - J[2] * J[6], J[2] * J[3] - J[0] * J[5],
                                 J[3] * J[7] - J[4] * J[6], J[1] * J[6] - J[0] * J[7], J[0] * J[4] - J[1] * J[3]};
          for (int i = 0; i < 3; ++i)
            lam[i] -= (inv[3 * i] * r[0] + inv[3 * i + 1] * r[1] + inv[3 * i + 2] * r[2]) / det;
        }
        // R from the point triangles: [P1 - P0, P2 - P0, cross] = R [X1 - X0, X2 - X0, cross];
        // the depths solve the distance equations up to one common sign, so the mirrored
        // triangle (points at z < 0: a camera matrix with a negative scale) is a solution too
        for (int mirror = 0; mirror < 2; ++mirror) {
        const double sgn = mirror ? -1.0 : 1.0;
        double P[3][3];
        for (int i = 0; i < 3; ++i)
          for (int c = 0; c < 3; ++c) P[i][c] = sgn * lam[i] * y[i][c];
        double xa[3], xb[3], xc[3], pa[3], pb[3], pc[3];
        for (int c = 0; c < 3; ++c) {
          xa[c] = X[1][c] - X[0][c];
          xb[c] = X[2][c] - X[0][c];
          pa[c] = P[1][c] - P[0][c];
          pb[c] = P[2][c] - P[0][c];
        }
        cross3(xa, xb, xc);
        cross3(pa, pb, pc);
        // Xm = [xa xb xc] (columns); R = Pm Xm^-1
        const double Xm[9] = {xa[0], xb[0], xc[0], xa[1], xb[1], xc[1], xa[2], xb[2], xc[2]};
        const double dx = Xm[0] * (Xm[4] * Xm[8] - Xm[5] * Xm[7]) - Xm[1] * (Xm[3] * Xm[8] - Xm[5] * Xm[6]) +
                          Xm[2] * (Xm[3] * Xm[7] - Xm[4] * Xm[6]);
        if (!(fabs(dx) > 0.0)) break;
        const double Xi[9] = {Xm[4] * Xm[8] - Xm[5] * Xm[7], Xm[2] * Xm[7] - Xm[1] * Xm[8], Xm[1] * Xm[5] - Xm[2] * Xm[4],
                              Xm[5] * Xm[6] - Xm[3] * Xm[8], Xm[0] * Xm[8] - Xm[2] * Xm[6], Xm[2] * Xm[3] - Xm[0] * Xm[5],
                              Xm[3] * Xm[7] - Xm[4] * Xm[6], Xm[1] * Xm[6] - Xm[0] * Xm[7], Xm[0] * Xm[4] - Xm[1] * Xm[3]};
        const double Pm[9] = {pa[0], pb[0], pc[0], pa[1], pb[1], pc[1], pa[2], pb[2], pc[2]};
        for (int r = 0; r < 3; ++r)
          for (int c = 0; c < 3; ++c)
            Rs[ns][3 * r + c] = (Pm[3 * r] * Xi[c] + Pm[3 * r + 1] * Xi[3 + c] + Pm[3 * r + 2] * Xi[6 + c]) / dx;
        for (int r = 0; r < 3; ++r)
          ts[ns][r] = P[0][r] - (Rs[ns][3 * r] * X[0][0] + Rs[ns][3 * r + 1] * X[0][1] + Rs[ns][3 * r + 2] * X[0][2]);
        mirrored[ns] = mirror != 0;
        ++ns;
        }
      }
    }
    break;  // one real root that gives a line pair carries every solution
  }
  return ns;
}

// P3P on points 0..2 of a four-point set; the fourth picks the solution with the smallest
// reprojection error.  Returns that error (inf: no solution).
template <class PtAt>
__device__ inline double p3p_pose(PtAt pt, double (&R)[9], double (&t)[3]) {
  double X[3][3], y[3][3];
  for (int i = 0; i < 3; ++i) {
    const PPt p = pt(i);
    X[i][0] = p.X;
    X[i][1] = p.Y;
    X[i][2] = p.Z;
    const double in = 1.0 / sqrt(p.u * p.u + p.v * p.v + 1.0);
    y[i][0] = p.u * in;
    y[i][1] = p.v * in;
    y[i][2] = in;
  }
  double Rs[8][9], ts[8][3];
  bool mir[8];
  const int ns = p3p_lambda_twist(X, y, Rs, ts, mir);
  const PPt p3 = pt(3);
  double best[2] = {INFINITY, INFINITY};  // front-facing, mirrored (see kMirrorWins)
  int arg[2] = {-1, -1};
  for (int s = 0; s < ns; ++s) {
    const double x = Rs[s][0] * p3.X + Rs[s][1] * p3.Y + Rs[s][2] * p3.Z + ts[s][0];
    const double yy = Rs[s][3] * p3.X + Rs[s][4] * p3.Y + Rs[s][5] * p3.Z + ts[s][1];
    const double z = Rs[s][6] * p3.X + Rs[s][7] * p3.Y + Rs[s][8] * p3.Z + ts[s][2];
    const double du = p3.u - x / z, dv = p3.v - yy / z;
    const double e = sqrt(du * du + dv * dv);
    const int k = mir[s] ? 1 : 0;
    if (e < best[k]) {
      best[k] = e;
      arg[k] = s;
    }
  }
  const int k = mirror_wins(best[1], best[0]) ? 1 : 0;
  if (arg[k] < 0) return INFINITY;
  for (int i = 0; i < 9; ++i) R[i] = Rs[arg[k]][i];
  for (int i = 0; i < 3; ++i) t[i] = ts[arg[k]][i];
  return best[k];
}

}  // namespace rsd
