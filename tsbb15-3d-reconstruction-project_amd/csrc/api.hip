// C ABI (include/rsamd.h): contexts, F plans, single-shot lab3 ops.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "common.h"
#include "ctx.h"
#include "device_math.h"
#include "f8_kernels.h"

namespace rs {

static thread_local std::string g_err;

void set_error(const char *fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
}

int hip_fail(hipError_t e, const char *what) {
  set_error("%s: %s", what, hipGetErrorString(e));
  return e == hipErrorOutOfMemory ? RS_ENOMEM : RS_EDEVICE;
}

int ensure_scratch(rs_ctx *c, size_t bytes) {
  if (c->scratch_bytes >= bytes) return RS_OK;
  if (c->scratch) (void)hipFree(c->scratch);
  c->scratch = nullptr;
  c->scratch_bytes = 0;
  size_t want = std::max<size_t>(bytes, 1 << 20);
  hipError_t e = hipMalloc(&c->scratch, want);
  if (e != hipSuccess) return hip_fail(e, "hipMalloc(scratch)");
  c->scratch_bytes = want;
  return RS_OK;
}

int ensure_pinned(rs_ctx *c, size_t bytes) {
  if (c->pinned_bytes >= bytes) return RS_OK;
  if (c->pinned) (void)hipHostFree(c->pinned);
  c->pinned = nullptr;
  c->pinned_bytes = 0;
  size_t want = std::max<size_t>(bytes, 1 << 16);
  hipError_t e = hipHostMalloc(&c->pinned, want);
  if (e != hipSuccess) return hip_fail(e, "hipHostMalloc(staging)");
  c->pinned_bytes = want;
  return RS_OK;
}

}  // namespace rs

using rs::fail;
using rs::hip_fail;

#define HIP_TRY(expr)                                     \
  do {                                                    \
    hipError_t e_ = (expr);                               \
    if (e_ != hipSuccess) return hip_fail(e_, #expr);     \
  } while (0)

extern "C" const char *rs_last_error(void) { return rs::g_err.c_str(); }
extern "C" int rs_version(void) { return 100; }

extern "C" int rs_device_count(int *n) {
  if (!n) return fail(RS_EINVAL, "null pointer");
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess) {
    *n = 0;
    if (e == hipErrorNoDevice) return RS_OK;
    return hip_fail(e, "hipGetDeviceCount");
  }
  *n = c;
  return RS_OK;
}

extern "C" int rs_ctx_create(int device, rs_ctx **out) {
  if (!out) return fail(RS_EINVAL, "null pointer");
  *out = nullptr;
  int count = 0;
  hipError_t e = hipGetDeviceCount(&count);
  if (e != hipSuccess || count == 0)
    return fail(RS_ENODEV, "no HIP device visible (the MI355X path needs a GPU)");
  if (device < 0 || device >= count) return fail(RS_EINVAL, "device index out of range");
  HIP_TRY(hipSetDevice(device));
  rs_ctx *c = new rs_ctx();
  c->device = device;
  e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->aux_stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return hip_fail(e, "hipStreamCreate");
  }
  // the F-RANSAC and parity sampler code objects are loaded here rather than by the first
  // RANSAC call (HIP loads a module at the first use of one of its kernels; a no-op once the
  // process has them on this device)
  e = rsd::preload_f8();
  if (e != hipSuccess) {
    (void)hipStreamDestroy(c->aux_stream);
    (void)hipStreamDestroy(c->stream);
    delete c;
    return hip_fail(e, "code object load");
  }
  if (int st = rs::np_preload()) {
    (void)hipStreamDestroy(c->aux_stream);
    (void)hipStreamDestroy(c->stream);
    delete c;
    return st;
  }
  *out = c;
  return RS_OK;
}

extern "C" int rs_ctx_destroy(rs_ctx *c) {
  if (!c) return RS_OK;
  (void)hipSetDevice(c->device);
  (void)rs_comm_destroy(c);
  if (c->np_plan) rs_f8_plan_destroy(c->np_plan);
  rs::np_shard_free(c);
  if (c->scratch) (void)hipFree(c->scratch);
  if (c->pinned) (void)hipHostFree(c->pinned);
  for (auto &e : c->pnp_ev)
    if (e) (void)hipEventDestroy(e);
  if (c->aux_stream) (void)hipStreamDestroy(c->aux_stream);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return RS_OK;
}

extern "C" int rs_ctx_synchronize(rs_ctx *c) {
  if (!c) return fail(RS_EINVAL, "null context");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return RS_OK;
}

// ------------------------------------------------------------------------------------------
// lab3 primitives
// ------------------------------------------------------------------------------------------
extern "C" int rs_fmatrix_residuals(rs_ctx *c, const double *F, const double *x, const double *y,
                                    int64_t n, double *res_out) {
  if (!c || !F || !res_out || (n > 0 && (!x || !y))) return fail(RS_EINVAL, "null pointer");
  if (n < 0 || n > (1LL << 30)) return fail(RS_EINVAL, "bad point count");
  if (n == 0) return RS_OK;
  HIP_TRY(hipSetDevice(c->device));
  const size_t bpts = sizeof(double) * 4 * n, bpt = sizeof(rsd::Pt) * n, bout = sizeof(double) * 2 * n;
  int st = rs::ensure_scratch(c, bpts + bpt + bout + 128);
  if (st) return st;
  char *base = static_cast<char *>(c->scratch);
  double *d_xy = reinterpret_cast<double *>(base);
  rsd::Pt *d_pts = reinterpret_cast<rsd::Pt *>(base + bpts);
  double *d_out = reinterpret_cast<double *>(base + bpts + bpt);
  double *d_F = reinterpret_cast<double *>(base + bpts + bpt + bout);
  HIP_TRY(hipMemcpyAsync(d_xy, x, sizeof(double) * 2 * n, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(d_xy + 2 * n, y, sizeof(double) * 2 * n, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(d_F, F, sizeof(double) * 9, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(rsd::launch_pack_points(d_xy, d_xy + 2 * n, static_cast<int>(n), d_pts, c->stream));
  HIP_TRY(rsd::launch_residuals(d_pts, static_cast<int>(n), d_F, d_out, c->stream));
  HIP_TRY(hipMemcpyAsync(res_out, d_out, bout, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return RS_OK;
}

extern "C" int rs_fmatrix_stls_batch(rs_ctx *c, const double *pl, const double *pr, int64_t n,
                                     const int32_t *tuples, int64_t count, double *F_out) {
  if (!c || !pl || !pr || !tuples || !F_out) return fail(RS_EINVAL, "null pointer");
  if (n < 8 || count < 1 || count > (1LL << 28)) return fail(RS_EINVAL, "bad dimensions");
  for (int64_t i = 0; i < 8 * count; ++i)
    if (tuples[i] < 0 || tuples[i] >= n) return fail(RS_EINVAL, "tuple index out of range");
  HIP_TRY(hipSetDevice(c->device));
  const int64_t ld = (count + 63) / 64 * 64;
  const size_t bpts = sizeof(double) * 4 * n, bpt = sizeof(rsd::Pt) * n;
  const size_t btup = sizeof(int) * 8 * count, bF = sizeof(double) * 9 * ld;
  int st = rs::ensure_scratch(c, bpts + bpt + btup + bF + 256);
  if (st) return st;
  char *base = static_cast<char *>(c->scratch);
  double *d_xy = reinterpret_cast<double *>(base);
  rsd::Pt *d_pts = reinterpret_cast<rsd::Pt *>(base + bpts);
  int *d_tup = reinterpret_cast<int *>(base + bpts + bpt);
  double *d_F = reinterpret_cast<double *>(base + ((bpts + bpt + btup + 63) / 64) * 64);
  HIP_TRY(hipMemcpyAsync(d_xy, pl, sizeof(double) * 2 * n, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(d_xy + 2 * n, pr, sizeof(double) * 2 * n, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(d_tup, tuples, btup, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(rsd::launch_pack_points(d_xy, d_xy + 2 * n, static_cast<int>(n), d_pts, c->stream));
  HIP_TRY(rsd::launch_f8_solve(d_pts, static_cast<int>(n), static_cast<int>(count),
                               RS_SAMPLER_TUPLES, 0, 0, d_tup, d_F, ld, nullptr, nullptr,
                               c->stream));
  std::vector<double> soa(static_cast<size_t>(9 * ld));
  HIP_TRY(hipMemcpyAsync(soa.data(), d_F, bF, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  for (int64_t h = 0; h < count; ++h)
    for (int k = 0; k < 9; ++k) F_out[h * 9 + k] = soa[k * ld + h];
  return RS_OK;
}

extern "C" int rs_fmatrix_stls(rs_ctx *c, const double *pl, const double *pr, int64_t n,
                               double *F_out) {
  if (!c || !pl || !pr || !F_out) return fail(RS_EINVAL, "null pointer");
  if (n < 8) return fail(RS_EINVAL, "the 8-point algorithm needs at least 8 correspondences");
  if (n == 8) {
    const int32_t t[8] = {0, 1, 2, 3, 4, 5, 6, 7};
    return rs_fmatrix_stls_batch(c, pl, pr, n, t, 1, F_out);
  }
  return rs::fmatrix_stls_lsq(c, pl, pr, n, F_out);
}
