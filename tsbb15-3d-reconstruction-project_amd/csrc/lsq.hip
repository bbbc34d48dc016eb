// lab3.fmatrix_stls for n > 8 correspondences (lab3.py:269-329): the least-squares null
// vector of the n x 9 design matrix.  One 1024-thread workgroup: Hartley-style scaling,
// Householder QR of A streamed from HBM (R is 9 x 9), one-sided Jacobi SVD of R (the right
// singular vectors of A are those of R), smallest singular vector -> rank 2 -> unscale.
#include <hip/hip_runtime.h>

#include <cstring>

#include "common.h"
#include "ctx.h"
#include "device_math.h"

namespace rsd {

constexpr int kT = 1024;

template <int K>
__device__ __forceinline__ void block_sum(double (&v)[K], double (*sh)[16]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    double x = v[k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    if (lane == 0) sh[k][w] = x;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) {
    double s = 0.0;
    for (int q = 0; q < kT / 64; ++q) s += sh[k][q];
    v[k] = s;
  }
  __syncthreads();
}

__global__ __launch_bounds__(kT) void k_fstls_lsq(const double *__restrict__ pl,
                                                  const double *__restrict__ pr, int n,
                                                  double *__restrict__ A,
                                                  double *__restrict__ F_out) {
  __shared__ double sh[10][16];
  __shared__ double R[9][9];
  __shared__ double fs_s[9];
  const int tid = threadIdx.x;
  // --- scaling homographies (lab3.py:288-295) ---
  double m[4] = {0, 0, 0, 0};
  for (int i = tid; i < n; i += kT) {
    m[0] += pl[i];
    m[1] += pl[n + i];
    m[2] += pr[i];
    m[3] += pr[n + i];
  }
  block_sum<4>(m, sh);
  const double xm1 = m[0] / n, ym1 = m[1] / n, xm2 = m[2] / n, ym2 = m[3] / n;
  double q[2] = {0, 0};
  for (int i = tid; i < n; i += kT) {
    const double a = pl[i] - xm1, b = pl[n + i] - ym1, c = pr[i] - xm2, d = pr[n + i] - ym2;
    q[0] += a * a + b * b;
    q[1] += c * c + d * d;
  }
  block_sum<2>(q, sh);
  const double L1 = sqrt(1.0 / 2.0 / n * q[0]), L2 = sqrt(1.0 / 2.0 / n * q[1]);
  const double s1 = 1.0 / L1, ox1 = -xm1 / L1, oy1 = -ym1 / L1;
  const double s2 = 1.0 / L2, ox2 = -xm2 / L2, oy2 = -ym2 / L2;
  // --- design matrix, column-major n x 9 (lab3.py:312-315) ---
  for (int i = tid; i < n; i += kT) {
    const double X = pl[i] * s1 + ox1, Y = pl[n + i] * s1 + oy1;
    const double x = pr[i] * s2 + ox2, y = pr[n + i] * s2 + oy2;
    A[0 * n + i] = X * x;
    A[1 * n + i] = X * y;
    A[2 * n + i] = X;
    A[3 * n + i] = Y * x;
    A[4 * n + i] = Y * y;
    A[5 * n + i] = Y;
    A[6 * n + i] = x;
    A[7 * n + i] = y;
    A[8 * n + i] = 1.0;
  }
  __syncthreads();
  // --- Householder QR, column by column ---
  for (int k = 0; k < 9; ++k) {
    double nn[1] = {0.0};
    for (int i = k + tid; i < n; i += kT) nn[0] += A[k * n + i] * A[k * n + i];
    block_sum<1>(nn, sh);
    const double nrm = sqrt(nn[0]);
    const double akk = A[k * n + k];
    const double alpha = akk >= 0.0 ? -nrm : nrm;
    const double denom = nrm * (nrm + fabs(akk));
    const double tau = denom > 0.0 ? 1.0 / denom : 0.0;
    __syncthreads();
    if (tid == 0) A[k * n + k] = akk - alpha;
    __syncthreads();
    double w[9];
#pragma unroll
    for (int j = 0; j < 9; ++j) w[j] = 0.0;
    for (int i = k + tid; i < n; i += kT) {
      const double v = A[k * n + i];
#pragma unroll
      for (int j = 0; j < 9; ++j)
        if (j > k) w[j] += v * A[j * n + i];
    }
    block_sum<9>(w, sh);
    for (int i = k + tid; i < n; i += kT) {
      const double v = A[k * n + i];
#pragma unroll
      for (int j = 0; j < 9; ++j)
        if (j > k) A[j * n + i] -= tau * w[j] * v;
    }
    __syncthreads();
    if (tid == 0) {
      R[k][k] = alpha;
      for (int j = 0; j < 9; ++j)
        if (j > k) R[k][j] = A[j * n + k];
        else if (j < k) R[k][j] = 0.0;
    }
    __syncthreads();
  }
  // --- one-sided Jacobi SVD of R (9 x 9), V accumulated; smallest singular vector ---
  if (tid == 0) {
    double B[9][9], V[9][9];
    for (int r = 0; r < 9; ++r)
      for (int c = 0; c < 9; ++c) {
        B[r][c] = R[r][c];
        V[r][c] = (r == c) ? 1.0 : 0.0;
      }
    for (int sweep = 0; sweep < 30; ++sweep) {
      bool rotated = false;
      for (int p = 0; p < 8; ++p)
        for (int qq = p + 1; qq < 9; ++qq) {
          double a = 0, b = 0, g = 0;
          for (int r = 0; r < 9; ++r) {
            a += B[r][p] * B[r][p];
            b += B[r][qq] * B[r][qq];
            g += B[r][p] * B[r][qq];
          }
          if (fabs(g) > 1e-15 * sqrt(a * b)) {
            rotated = true;
            const double zeta = (b - a) / (2.0 * g);
            const double t = copysign(1.0, zeta) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
            const double c = 1.0 / sqrt(1.0 + t * t), s = c * t;
            for (int r = 0; r < 9; ++r) {
              const double bp = B[r][p], bq = B[r][qq];
              B[r][p] = c * bp - s * bq;
              B[r][qq] = s * bp + c * bq;
              const double vp = V[r][p], vq = V[r][qq];
              V[r][p] = c * vp - s * vq;
              V[r][qq] = s * vp + c * vq;
            }
          }
        }
      if (!rotated) break;
    }
    int mi = 0;
    double best = 0.0;
    for (int c = 0; c < 9; ++c) {
      double ss = 0;
      for (int r = 0; r < 9; ++r) ss += B[r][c] * B[r][c];
      if (c == 0 || ss < best) {
        best = ss;
        mi = c;
      }
    }
    for (int r = 0; r < 9; ++r) fs_s[r] = V[r][mi];
    double fs[9], F2[9];
    for (int r = 0; r < 9; ++r) fs[r] = fs_s[r];
    enforce_rank2(fs, F2);
    double M[9];
    for (int r = 0; r < 3; ++r) {
      M[3 * r + 0] = F2[3 * r + 0] * s2;
      M[3 * r + 1] = F2[3 * r + 1] * s2;
      M[3 * r + 2] = (F2[3 * r + 0] * ox2 + F2[3 * r + 1] * oy2) + F2[3 * r + 2];
    }
    for (int c = 0; c < 3; ++c) {
      F_out[0 + c] = s1 * M[0 + c];
      F_out[3 + c] = s1 * M[3 + c];
      F_out[6 + c] = (ox1 * M[0 + c] + oy1 * M[3 + c]) + M[6 + c];
    }
  }
}

}  // namespace rsd

namespace rs {

int fmatrix_stls_lsq(rs_ctx *c, const double *pl, const double *pr, int64_t n, double *F_out) {
  if (n > (1LL << 26)) return fail(RS_EINVAL, "too many correspondences");
  hipError_t e = hipSetDevice(c->device);
  if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
  const size_t bp = sizeof(double) * 2 * n, bA = sizeof(double) * 9 * n;
  int st = ensure_scratch(c, 2 * bp + bA + 256);
  if (st) return st;
  char *base = static_cast<char *>(c->scratch);
  double *d_pl = reinterpret_cast<double *>(base);
  double *d_pr = reinterpret_cast<double *>(base + bp);
  double *d_A = reinterpret_cast<double *>(base + 2 * bp);
  double *d_F = reinterpret_cast<double *>(base + 2 * bp + bA);
  if ((e = hipMemcpyAsync(d_pl, pl, bp, hipMemcpyHostToDevice, c->stream)) != hipSuccess ||
      (e = hipMemcpyAsync(d_pr, pr, bp, hipMemcpyHostToDevice, c->stream)) != hipSuccess)
    return hip_fail(e, "hipMemcpyAsync");
  hipLaunchKernelGGL(rsd::k_fstls_lsq, dim3(1), dim3(rsd::kT), 0, c->stream, d_pl, d_pr,
                     static_cast<int>(n), d_A, d_F);
  if ((e = hipGetLastError()) != hipSuccess) return hip_fail(e, "k_fstls_lsq");
  if ((e = hipMemcpyAsync(F_out, d_F, sizeof(double) * 9, hipMemcpyDeviceToHost, c->stream)) !=
      hipSuccess)
    return hip_fail(e, "hipMemcpyAsync");
  if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return hip_fail(e, "sync");
  return RS_OK;
}

}  // namespace rs
