// The per-view SfM steps around PnP, batched on the GPU:
//
//   k_match_obs        lane per putative correspondence: the 2D<->3D matching loop of
//                      Tables.addNewView (tables.py:116-135) -- the FIRST observation of the
//                      last view, in its observations_index order, with ||obs - y1|| < tol;
//                      observations staged through LDS in tiles
//   k_new_points       lane per putative correspondence: Tables.addNewPoints
//                      (tables.py:161-175) -- E = fun.getEFromCameras(C1, C2) (fun.py:12-21),
//                      the gate |y1^T E y2| < gate, lab3.triangulate_optimal of the accepted
//   k_ba_residuals     lane per observation: EpsilonBA of Tables.BundleAdjustment2
//                      (tables.py:264-293), r = [u - c1.x / c3.x, v - c2.x / c3.x]
//   k_ba_jacobian      lane per observation: its 2x12 camera and 2x3 point Jacobian blocks
//                      (the nonzeros of Tables.sparsity_mask, tables.py:339-372)
#include <hip/hip_runtime.h>

#include <initializer_list>
#include <vector>

#include "common.h"
#include "ctx.h"
#include "device_math.h"
#include "twoview_math.h"

namespace rsd {

constexpr int kMatchTile = 512;

__global__ __launch_bounds__(256) void k_match_obs(const double *__restrict__ obs, int m,
                                                   const int64_t *__restrict__ obs_point,
                                                   const double *__restrict__ q, int n,
                                                   double tol, int64_t *__restrict__ out) {
  __shared__ double so[kMatchTile * 3];
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  double q0 = 0.0, q1 = 0.0, q2 = 0.0;
  if (i < n) {
    q0 = q[3 * i];
    q1 = q[3 * i + 1];
    q2 = q[3 * i + 2];
  }
  int found = -1;
  for (int base = 0; base < m; base += kMatchTile) {
    const int cnt = min(kMatchTile, m - base);
    __syncthreads();
    for (int k = threadIdx.x; k < 3 * cnt; k += blockDim.x) so[k] = obs[3 * base + k];
    __syncthreads();
    if (i < n && found < 0) {
      for (int k = 0; k < cnt; ++k) {
        const double d0 = so[3 * k] - q0, d1 = so[3 * k + 1] - q1, d2 = so[3 * k + 2] - q2;
        if (sqrt(d0 * d0 + d1 * d1 + d2 * d2) < tol) {
          found = base + k;
          break;
        }
      }
    }
  }
  if (i < n) out[i] = found >= 0 ? obs_point[found] : -1;
}

// fun.getEFromCameras: R = R2 R1^T, t = t2 - R2 R1^T t1, E = R^T [t]_x.
__device__ __forceinline__ void e_from_cameras(const double *C1, const double *C2, double *E) {
  double R[9];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c)
      R[3 * r + c] = C2[4 * r] * C1[4 * c] + C2[4 * r + 1] * C1[4 * c + 1] +
                     C2[4 * r + 2] * C1[4 * c + 2];
  double t[3];
#pragma unroll
  for (int r = 0; r < 3; ++r)
    t[r] = C2[4 * r + 3] - (R[3 * r] * C1[3] + R[3 * r + 1] * C1[7] + R[3 * r + 2] * C1[11]);
  const double tx[9] = {0.0, -t[2], t[1], t[2], 0.0, -t[0], -t[1], t[0], 0.0};
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c)
      E[3 * r + c] = R[r] * tx[c] + R[3 + r] * tx[3 + c] + R[6 + r] * tx[6 + c];
}

__global__ __launch_bounds__(128) void k_e_from_cameras(const double *__restrict__ C1s,
                                                        const double *__restrict__ C2s, int n,
                                                        double *__restrict__ E) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double a[12], b[12], e[9];
#pragma unroll
  for (int k = 0; k < 12; ++k) {
    a[k] = C1s[12 * i + k];
    b[k] = C2s[12 * i + k];
  }
  e_from_cameras(a, b, e);
#pragma unroll
  for (int k = 0; k < 9; ++k) E[9 * i + k] = e[k];
}

__global__ __launch_bounds__(128) void k_new_points(const double *__restrict__ Cs,
                                                    const double *__restrict__ y1,
                                                    const double *__restrict__ y2, int n,
                                                    double gate, int32_t *__restrict__ mask,
                                                    double *__restrict__ X) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double C1[12], C2[12], E[9];
#pragma unroll
  for (int k = 0; k < 12; ++k) {
    C1[k] = Cs[k];
    C2[k] = Cs[12 + k];
  }
  e_from_cameras(C1, C2, E);
  const double a[3] = {y1[3 * i], y1[3 * i + 1], y1[3 * i + 2]};
  const double b[3] = {y2[3 * i], y2[3 * i + 1], y2[3 * i + 2]};
  double Eb[3];
#pragma unroll
  for (int r = 0; r < 3; ++r) Eb[r] = E[3 * r] * b[0] + E[3 * r + 1] * b[1] + E[3 * r + 2] * b[2];
  const double e = a[0] * Eb[0] + a[1] * Eb[1] + a[2] * Eb[2];
  const bool ok = fabs(e) < gate;
  mask[i] = ok ? 1 : 0;
  double Y[3] = {__builtin_nan(""), __builtin_nan(""), __builtin_nan("")};
  if (ok) triangulate_optimal(C1, C2, a[0], a[1], b[0], b[1], Y);
  X[3 * i] = Y[0];
  X[3 * i + 1] = Y[1];
  X[3 * i + 2] = Y[2];
}

__global__ __launch_bounds__(256) void k_ba_residuals(
    const double *__restrict__ cams, const double *__restrict__ pts,
    const int32_t *__restrict__ ov, const int32_t *__restrict__ op,
    const double *__restrict__ uv, int n, double *__restrict__ r) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double *c = cams + 12 * ov[i];
  const double *p = pts + 3 * op[i];
  const double x0 = p[0], x1 = p[1], x2 = p[2];
  const double a = c[0] * x0 + c[1] * x1 + c[2] * x2 + c[3];
  const double b = c[4] * x0 + c[5] * x1 + c[6] * x2 + c[7];
  const double w = c[8] * x0 + c[9] * x1 + c[10] * x2 + c[11];
  r[2 * i] = uv[2 * i] - a / w;
  r[2 * i + 1] = uv[2 * i + 1] - b / w;
}

__global__ __launch_bounds__(256) void k_ba_jacobian(
    const double *__restrict__ cams, const double *__restrict__ pts,
    const int32_t *__restrict__ ov, const int32_t *__restrict__ op, int n,
    double *__restrict__ Jc, double *__restrict__ Jp) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double *c = cams + 12 * ov[i];
  const double *p = pts + 3 * op[i];
  const double xh[4] = {p[0], p[1], p[2], 1.0};
  const double a = c[0] * xh[0] + c[1] * xh[1] + c[2] * xh[2] + c[3];
  const double b = c[4] * xh[0] + c[5] * xh[1] + c[6] * xh[2] + c[7];
  const double w = c[8] * xh[0] + c[9] * xh[1] + c[10] * xh[2] + c[11];
  const double iw = 1.0 / w, iw2 = iw * iw;
  double *jc = Jc + 24 * static_cast<int64_t>(i);
  double *jp = Jp + 6 * static_cast<int64_t>(i);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    jc[k] = -xh[k] * iw;
    jc[4 + k] = 0.0;
    jc[8 + k] = xh[k] * a * iw2;
    jc[12 + k] = 0.0;
    jc[16 + k] = -xh[k] * iw;
    jc[20 + k] = xh[k] * b * iw2;
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    jp[k] = -(c[k] * w - a * c[8 + k]) * iw2;
    jp[3 + k] = -(c[4 + k] * w - b * c[8 + k]) * iw2;
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

namespace {

size_t al(size_t b) { return (b + 255) / 256 * 256; }

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

}  // namespace

extern "C" int rs_match_observations(rs_ctx *c, const double *obs, const int64_t *obs_point,
                                     int64_t m, const double *queries, int64_t n, double tol,
                                     int64_t *out) {
  if (!c || !out || (m > 0 && (!obs || !obs_point)) || (n > 0 && !queries))
    return fail(RS_EINVAL, "null pointer");
  if (m < 0 || n < 0 || m > (1 << 26) || n > (1 << 26)) return fail(RS_EINVAL, "bad sizes");
  if (n == 0) return RS_OK;
  HIP_TRY(hipSetDevice(c->device));
  const int64_t mm = m > 0 ? m : 1;
  std::vector<char *> b;
  int st = carve(c, {sizeof(double) * 3 * mm, sizeof(int64_t) * mm, sizeof(double) * 3 * n,
                     sizeof(int64_t) * n}, b);
  if (st) return st;
  if (m > 0) {
    HIP_TRY(hipMemcpyAsync(b[0], obs, sizeof(double) * 3 * m, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(b[1], obs_point, sizeof(int64_t) * m, hipMemcpyHostToDevice, c->stream));
  }
  HIP_TRY(hipMemcpyAsync(b[2], queries, sizeof(double) * 3 * n, hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(rsd::k_match_obs, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0,
                     c->stream, reinterpret_cast<double *>(b[0]), static_cast<int>(m),
                     reinterpret_cast<int64_t *>(b[1]), reinterpret_cast<double *>(b[2]),
                     static_cast<int>(n), tol, reinterpret_cast<int64_t *>(b[3]));
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(out, b[3], sizeof(int64_t) * n, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return RS_OK;
}

extern "C" int rs_e_from_cameras(rs_ctx *c, const double *C1, const double *C2, int64_t n,
                                 double *E) {
  if (!c || !C1 || !C2 || !E) return fail(RS_EINVAL, "null pointer");
  if (n < 0 || n > (1 << 26)) return fail(RS_EINVAL, "bad sizes");
  if (n == 0) return RS_OK;
  HIP_TRY(hipSetDevice(c->device));
  std::vector<char *> b;
  int st = carve(c, {sizeof(double) * 12 * n, sizeof(double) * 12 * n, sizeof(double) * 9 * n}, b);
  if (st) return st;
  HIP_TRY(hipMemcpyAsync(b[0], C1, sizeof(double) * 12 * n, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(b[1], C2, sizeof(double) * 12 * n, hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(rsd::k_e_from_cameras, dim3(static_cast<unsigned>((n + 127) / 128)),
                     dim3(128), 0, c->stream, reinterpret_cast<double *>(b[0]),
                     reinterpret_cast<double *>(b[1]), static_cast<int>(n),
                     reinterpret_cast<double *>(b[2]));
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(E, b[2], sizeof(double) * 9 * n, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return RS_OK;
}

extern "C" int rs_add_new_points(rs_ctx *c, const double *C1, const double *C2,
                                 const double *y1, const double *y2, int64_t n, double gate,
                                 int32_t *mask, double *X) {
  if (!c || !C1 || !C2 || !mask || !X || (n > 0 && (!y1 || !y2)))
    return fail(RS_EINVAL, "null pointer");
  if (n < 0 || n > (1 << 26)) return fail(RS_EINVAL, "bad sizes");
  if (n == 0) return RS_OK;
  HIP_TRY(hipSetDevice(c->device));
  std::vector<char *> b;
  int st = carve(c, {sizeof(double) * 24, sizeof(double) * 3 * n, sizeof(double) * 3 * n,
                     sizeof(int32_t) * n, sizeof(double) * 3 * n}, b);
  if (st) return st;
  HIP_TRY(hipMemcpyAsync(b[0], C1, sizeof(double) * 12, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(b[0] + sizeof(double) * 12, C2, sizeof(double) * 12,
                         hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(b[1], y1, sizeof(double) * 3 * n, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(b[2], y2, sizeof(double) * 3 * n, hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(rsd::k_new_points, dim3(static_cast<unsigned>((n + 127) / 128)), dim3(128),
                     0, c->stream, reinterpret_cast<double *>(b[0]),
                     reinterpret_cast<double *>(b[1]), reinterpret_cast<double *>(b[2]),
                     static_cast<int>(n), gate, reinterpret_cast<int32_t *>(b[3]),
                     reinterpret_cast<double *>(b[4]));
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(mask, b[3], sizeof(int32_t) * n, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(X, b[4], sizeof(double) * 3 * n, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return RS_OK;
}

static int ba_check(int64_t nC, int64_t nP, const int32_t *ov, const int32_t *op, int64_t n) {
  if (nC < 1 || nP < 0 || n < 0 || n > (1 << 26) || nC > (1 << 20) || nP > (1 << 26))
    return fail(RS_EINVAL, "bad sizes");
  for (int64_t i = 0; i < n; ++i)
    if (ov[i] < 0 || ov[i] >= nC || op[i] < 0 || op[i] >= nP)
      return fail(RS_EINVAL, "observation index out of range");
  return RS_OK;
}

extern "C" int rs_ba_residuals(rs_ctx *c, const double *cams, int64_t nC, const double *pts,
                               int64_t nP, const int32_t *obs_view, const int32_t *obs_point,
                               const double *uv, int64_t n, double *r) {
  if (!c || !cams || !r || (nP > 0 && !pts) || (n > 0 && (!obs_view || !obs_point || !uv)))
    return fail(RS_EINVAL, "null pointer");
  int st = ba_check(nC, nP, obs_view, obs_point, n);
  if (st) return st;
  if (n == 0) return RS_OK;
  HIP_TRY(hipSetDevice(c->device));
  std::vector<char *> b;
  const int64_t pp = nP > 0 ? nP : 1;
  st = carve(c, {sizeof(double) * 12 * nC, sizeof(double) * 3 * pp, sizeof(int32_t) * n,
                 sizeof(int32_t) * n, sizeof(double) * 2 * n, sizeof(double) * 2 * n}, b);
  if (st) return st;
  HIP_TRY(hipMemcpyAsync(b[0], cams, sizeof(double) * 12 * nC, hipMemcpyHostToDevice, c->stream));
  if (nP > 0)
    HIP_TRY(hipMemcpyAsync(b[1], pts, sizeof(double) * 3 * nP, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(b[2], obs_view, sizeof(int32_t) * n, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(b[3], obs_point, sizeof(int32_t) * n, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(b[4], uv, sizeof(double) * 2 * n, hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(rsd::k_ba_residuals, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256),
                     0, c->stream, reinterpret_cast<double *>(b[0]),
                     reinterpret_cast<double *>(b[1]), reinterpret_cast<int32_t *>(b[2]),
                     reinterpret_cast<int32_t *>(b[3]), reinterpret_cast<double *>(b[4]),
                     static_cast<int>(n), reinterpret_cast<double *>(b[5]));
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(r, b[5], sizeof(double) * 2 * n, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return RS_OK;
}

extern "C" int rs_ba_jacobian(rs_ctx *c, const double *cams, int64_t nC, const double *pts,
                              int64_t nP, const int32_t *obs_view, const int32_t *obs_point,
                              int64_t n, double *Jc, double *Jp) {
  if (!c || !cams || !Jc || !Jp || (nP > 0 && !pts) || (n > 0 && (!obs_view || !obs_point)))
    return fail(RS_EINVAL, "null pointer");
  int st = ba_check(nC, nP, obs_view, obs_point, n);
  if (st) return st;
  if (n == 0) return RS_OK;
  HIP_TRY(hipSetDevice(c->device));
  std::vector<char *> b;
  const int64_t pp = nP > 0 ? nP : 1;
  st = carve(c, {sizeof(double) * 12 * nC, sizeof(double) * 3 * pp, sizeof(int32_t) * n,
                 sizeof(int32_t) * n, sizeof(double) * 24 * n, sizeof(double) * 6 * n}, b);
  if (st) return st;
  HIP_TRY(hipMemcpyAsync(b[0], cams, sizeof(double) * 12 * nC, hipMemcpyHostToDevice, c->stream));
  if (nP > 0)
    HIP_TRY(hipMemcpyAsync(b[1], pts, sizeof(double) * 3 * nP, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(b[2], obs_view, sizeof(int32_t) * n, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(b[3], obs_point, sizeof(int32_t) * n, hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(rsd::k_ba_jacobian, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256),
                     0, c->stream, reinterpret_cast<double *>(b[0]),
                     reinterpret_cast<double *>(b[1]), reinterpret_cast<int32_t *>(b[2]),
                     reinterpret_cast<int32_t *>(b[3]), static_cast<int>(n),
                     reinterpret_cast<double *>(b[4]), reinterpret_cast<double *>(b[5]));
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(Jc, b[4], sizeof(double) * 24 * n, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(Jp, b[5], sizeof(double) * 6 * n, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return RS_OK;
}
