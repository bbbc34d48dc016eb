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
  if (e != hipSuccess) {
    delete c;
    return hip_fail(e, "hipStreamCreate");
  }
  *out = c;
  return RS_OK;
}

extern "C" int rs_ctx_destroy(rs_ctx *c) {
  if (!c) return RS_OK;
  (void)hipSetDevice(c->device);
  (void)rs_comm_destroy(c);
  if (c->np_plan) rs_f8_plan_destroy(c->np_plan);
  if (c->scratch) (void)hipFree(c->scratch);
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
// F plans
// ------------------------------------------------------------------------------------------
struct rs_f8_plan {
  rs_ctx *ctx = nullptr;
  int64_t n = 0, max_hyp = 0, ld = 0;
  double *d_p12 = nullptr;     // staging (2,n) p1 then (2,n) p2
  rsd::Pt *d_pts = nullptr;    // AoS points
  double *d_F = nullptr;       // 9 x ld SoA models
  int *d_counts = nullptr;     // fast counts
  int *d_tuples = nullptr;     // host tuples (parity mode)
  int *d_cand = nullptr;       // ordered candidate hypothesis ids
  int *d_status = nullptr;     // [c*, n_candidates]
  int *d_ccount = nullptr;
  double *d_cstd = nullptr, *d_cnorm = nullptr;
  rsd::F8DevResult *d_res = nullptr;
  // Runs are stream-ordered and may be issued back to back without a host round trip: each
  // run copies its result into its own pinned slot and records its own events.
  static constexpr int kSlots = 4, kEvRing = 64;
  rsd::F8DevResult *h_slot[kSlots] = {};  // pinned result slots
  rsd::F8DevResult *h_res = nullptr;      // slot of the last run
  hipEvent_t done[kSlots] = {};           // D2H of a slot complete
  size_t res_bytes = 0;
  hipEvent_t ring[kEvRing][4] = {};       // per-run kernel events (solve, count, tail)
  int64_t runs = 0;                       // runs issued on this plan
  int64_t last_H = 0;
  bool pending = false, have_result = false;
  int chunk_override = 0;
  // fp32 counting (k_f8_count32): frame, fp32 points and models
  float4 *d_pts32 = nullptr;
  float *d_F32 = nullptr;
  rsd::Frame frame{1.0, 0.0, 0.0, 0.0, 0.0};
  bool fp32_ok = false;   // finite points and a non-degenerate frame
  bool use_fp32 = true;   // RSAMD_COUNT=fp64 selects the float64 kernel
  int resident_waves = 8192;  // CUs x 4 SIMDs x 8 waves (RSAMD_WAVES overrides)
  int count_block = 8;        // points per scalar-load block (RSAMD_BLOCK = 4 | 8)
  bool prefetch = true;       // software-pipelined point loads (RSAMD_PREFETCH=0 off)
  bool packed = false;        // two hypotheses per lane, v_pk_fma_f32 (RSAMD_COUNT=pk)
  int pk_variant = 0;         // RSAMD_PKVAR: 0 (2-pt blocks, 8 waves/SIMD), 1 (6), 2 (4), 3
  int pk_waves = 8192;        // resident waves of the chosen variant
};

namespace {

// Absolute error bounds of the fp32 test in the unit frame (|x~| <= R); derivation in
// f8_kernels.hip above k_f8_count32.  Dl: a line component, De: e, Dn: a squared length.
rsd::Guard32 guard_constants(const rsd::Frame &fr, double thresh) {
  const double u = std::ldexp(1.0, -24), R = 1.0 + 1e-6, Lm = 2.0 * R + 1.0;
  const double Dl = 1.1 * u * (7.0 * R + 3.0);
  const double De =
      1.1 * (2.0 * (Dl * R * 1.001 + Lm * u * R) + Dl + u * (Lm + Dl) * (3.0 * R + 2.0) * 1.001);
  const double Dn = 1.1 * (2.0 * Dl * (2.0 * Lm + Dl) + 3.0 * u * (Lm + Dl) * (Lm + Dl) * 1.001);
  const double thr2 = (thresh / fr.s) * (thresh / fr.s);
  rsd::Guard32 g;
  g.thr2 = static_cast<float>(thr2);
  g.K1 = static_cast<float>(1.02 * 2.0 * De);
  g.Ku = static_cast<float>(1.02 * u);
  g.K0 = static_cast<float>(1.02 * (De * De + thr2 * (1.0 + 1e-6) * Dn));
  g.thr2_px = thresh * thresh;
  return g;
}

rsd::GuardPk guard_packed(const rsd::Frame &fr, double thresh) {
  const double u = std::ldexp(1.0, -24), R = 1.0 + 1e-6, Lm = 2.0 * R + 1.0;
  const double Dl = 1.1 * u * (7.0 * R + 3.0);
  const double De =
      1.1 * (2.0 * (Dl * R * 1.001 + Lm * u * R) + Dl + u * (Lm + Dl) * (3.0 * R + 2.0) * 1.001);
  const double Dn = 1.1 * (2.0 * Dl * (2.0 * Lm + Dl) + 3.0 * u * (Lm + Dl) * (Lm + Dl) * 1.001);
  const double thr2 = (thresh / fr.s) * (thresh / fr.s);
  const double c = std::sqrt(thr2);  // AM-GM split point for 2 De |e| <= De (e^2 / c + c)
  rsd::GuardPk g;
  g.thr2 = static_cast<float>(thr2);
  g.Ka = static_cast<float>(1.02 * (De / c * (1.0 + 2.0 * u) + u));
  g.Kb = static_cast<float>(1.02 * 2.0 * u);
  g.K0 = static_cast<float>(1.02 * (De * c + De * De + thr2 * (1.0 + 1e-6) * Dn));
  g.thr2_px = thresh * thresh;
  return g;
}

}  // namespace

static void plan_free(rs_f8_plan *p) {
  (void)hipFree(p->d_p12);
  (void)hipFree(p->d_pts);
  (void)hipFree(p->d_F);
  (void)hipFree(p->d_counts);
  (void)hipFree(p->d_tuples);
  (void)hipFree(p->d_cand);
  (void)hipFree(p->d_status);
  (void)hipFree(p->d_ccount);
  (void)hipFree(p->d_cstd);
  (void)hipFree(p->d_cnorm);
  (void)hipFree(p->d_res);
  (void)hipFree(p->d_pts32);
  (void)hipFree(p->d_F32);
  for (auto &h : p->h_slot)
    if (h) (void)hipHostFree(h);
  for (auto &e : p->done)
    if (e) (void)hipEventDestroy(e);
  for (auto &r : p->ring)
    for (auto &e : r)
      if (e) (void)hipEventDestroy(e);
}

extern "C" int rs_f8_plan_create(rs_ctx *c, int64_t n, int64_t max_hyp, rs_f8_plan **out) {
  if (!c || !out) return fail(RS_EINVAL, "null pointer");
  *out = nullptr;
  if (n < 8) return fail(RS_EINVAL, "Cannot take a larger sample than population when 'replace=False'");
  if (n > (1LL << 30) || max_hyp < 1 || max_hyp > (1LL << 30))
    return fail(RS_EINVAL, "plan dimensions out of range");
  HIP_TRY(hipSetDevice(c->device));
  auto *p = new rs_f8_plan();
  p->ctx = c;
  p->n = n;
  p->max_hyp = max_hyp;
  p->ld = (max_hyp + 63) / 64 * 64;
  p->res_bytes = sizeof(rsd::F8DevResult) + sizeof(int64_t) * static_cast<size_t>(n);
  if (const char *ch = std::getenv("RSAMD_CHUNK")) p->chunk_override = std::atoi(ch);
  if (const char *cm = std::getenv("RSAMD_COUNT")) {
    p->use_fp32 = std::strcmp(cm, "fp64") != 0;
    p->packed = std::strcmp(cm, "pk") == 0;  // "fp32" (default), "pk", "fp64"
  }
  {
    int cus = 256;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess)
      cus = 256;
    p->resident_waves = cus * 4 * 8 * 4;  // 4 slices per resident wave slot (sweep r01)
    if (const char *wv = std::getenv("RSAMD_WAVES")) p->resident_waves = std::max(1, std::atoi(wv));
    if (const char *bk = std::getenv("RSAMD_BLOCK")) p->count_block = std::atoi(bk) == 8 ? 8 : 4;
    if (const char *pf = std::getenv("RSAMD_PREFETCH")) p->prefetch = std::atoi(pf) != 0;
    if (const char *pv = std::getenv("RSAMD_PKVAR")) p->pk_variant = std::atoi(pv);
    const int minw = p->pk_variant == 1 || p->pk_variant == 3 ? 6 : (p->pk_variant == 2 ? 4 : 8);
    p->pk_waves = cus * 4 * minw;
    if (const char *wv = std::getenv("RSAMD_WAVES")) p->pk_waves = std::max(1, std::atoi(wv));
  }
  hipError_t e = hipSuccess;
#define ALLOC(ptr, bytes)                                  \
  if (e == hipSuccess) e = hipMalloc(&(ptr), (bytes));
  ALLOC(p->d_p12, sizeof(double) * 4 * n);
  ALLOC(p->d_pts, sizeof(rsd::Pt) * n);
  ALLOC(p->d_F, sizeof(double) * 9 * p->ld);
  ALLOC(p->d_counts, sizeof(int) * p->ld);
  ALLOC(p->d_tuples, sizeof(int) * 8 * p->ld);
  ALLOC(p->d_cand, sizeof(int) * p->ld);
  ALLOC(p->d_status, sizeof(int) * rsd::kStatusWords);
  ALLOC(p->d_ccount, sizeof(int) * p->ld);
  ALLOC(p->d_cstd, sizeof(double) * p->ld);
  ALLOC(p->d_cnorm, sizeof(double) * p->ld);
  ALLOC(p->d_res, p->res_bytes);
  ALLOC(p->d_pts32, sizeof(float4) * ((n + 7) & ~7LL));
  ALLOC(p->d_F32, sizeof(float) * 9 * p->ld);
#undef ALLOC
  for (auto &h : p->h_slot)
    if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void **>(&h), p->res_bytes);
  for (auto &ev : p->done)
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  for (auto &r : p->ring)
    for (auto &ev : r)
      if (e == hipSuccess) e = hipEventCreate(&ev);
  if (e != hipSuccess) {
    plan_free(p);
    delete p;
    return hip_fail(e, "rs_f8_plan_create");
  }
  *out = p;
  return RS_OK;
}

extern "C" int rs_f8_plan_destroy(rs_f8_plan *p) {
  if (!p) return RS_OK;
  (void)hipSetDevice(p->ctx->device);
  (void)hipStreamSynchronize(p->ctx->stream);
  plan_free(p);
  delete p;
  return RS_OK;
}

extern "C" int rs_f8_plan_set_points(rs_f8_plan *p, const double *p1, const double *p2) {
  if (!p || !p1 || !p2) return fail(RS_EINVAL, "null pointer");
  rs_ctx *c = p->ctx;
  HIP_TRY(hipSetDevice(c->device));
  const size_t b = sizeof(double) * 2 * p->n;
  HIP_TRY(hipMemcpyAsync(p->d_p12, p1, b, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(p->d_p12 + 2 * p->n, p2, b, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(rsd::launch_pack_points(p->d_p12, p->d_p12 + 2 * p->n, static_cast<int>(p->n),
                                  p->d_pts, c->stream));
  // unit frame of the fp32 counting kernel: per-image centres, one common scale
  const int64_t n = p->n;
  double lo[4], hi[4];
  bool finite = true;
  for (int k = 0; k < 4; ++k) {
    lo[k] = INFINITY;
    hi[k] = -INFINITY;
  }
  for (int64_t i = 0; i < n; ++i) {
    const double v[4] = {p1[i], p1[n + i], p2[i], p2[n + i]};
    for (int k = 0; k < 4; ++k) {
      finite &= std::isfinite(v[k]);
      lo[k] = std::min(lo[k], v[k]);
      hi[k] = std::max(hi[k], v[k]);
    }
  }
  rsd::Frame fr{0.0, 0.5 * (lo[0] + hi[0]), 0.5 * (lo[1] + hi[1]), 0.5 * (lo[2] + hi[2]),
                0.5 * (lo[3] + hi[3])};
  const double cen[4] = {fr.cx1, fr.cy1, fr.cx2, fr.cy2};
  for (int64_t i = 0; finite && i < n; ++i) {
    const double v[4] = {p1[i], p1[n + i], p2[i], p2[n + i]};
    for (int k = 0; k < 4; ++k) fr.s = std::max(fr.s, std::fabs(v[k] - cen[k]));
  }
  p->fp32_ok = finite && fr.s > 0.0 && std::isfinite(fr.s);
  if (p->fp32_ok) {
    fr.s *= 1.0 + 1e-12;  // |x~| <= 1 after the fp64 division
    p->frame = fr;
    HIP_TRY(rsd::launch_pack_points32(p->d_pts, static_cast<int>(n), fr, p->d_pts32, c->stream));
  }
  HIP_TRY(hipStreamSynchronize(c->stream));
  return RS_OK;
}

static int choose_chunk(const rs_f8_plan *p, int64_t H) {
  if (p->chunk_override > 0) return p->chunk_override;
  const int64_t groups = (H + 63) / 64;
  // aim for >= 8 units of work per SIMD (1024 SIMDs) without chunks below 64 points
  int64_t nchunks = (8192 + groups - 1) / groups;
  nchunks = std::max<int64_t>(1, std::min<int64_t>(nchunks, (p->n + 63) / 64));
  return static_cast<int>((p->n + nchunks - 1) / nchunks);
}

extern "C" int rs_f8_plan_run(rs_f8_plan *p, int64_t H, int32_t mode, uint64_t seed,
                              uint64_t hyp_offset, const int32_t *host_tuples, double thresh) {
  if (!p) return fail(RS_EINVAL, "null plan");
  if (H < 1 || H > p->max_hyp) return fail(RS_EINVAL, "hypothesis count out of plan range");
  if (mode != RS_SAMPLER_PHILOX && mode != RS_SAMPLER_TUPLES)
    return fail(RS_EINVAL, "unknown sampler mode");
  if (mode == RS_SAMPLER_TUPLES && !host_tuples) return fail(RS_EINVAL, "tuples required");
  if (!(thresh == thresh)) return fail(RS_EINVAL, "threshold is NaN");
  rs_ctx *c = p->ctx;
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = c->stream;
  const int n = static_cast<int>(p->n), h = static_cast<int>(H);
  if (mode == RS_SAMPLER_TUPLES) {
    for (int64_t i = 0; i < 8 * H; ++i)
      if (host_tuples[i] < 0 || host_tuples[i] >= p->n)
        return fail(RS_EINVAL, "tuple index out of range");
    HIP_TRY(hipMemcpyAsync(p->d_tuples, host_tuples, sizeof(int) * 8 * H,
                           hipMemcpyHostToDevice, s));
  }
  hipEvent_t *ev = p->ring[p->runs % rs_f8_plan::kEvRing];
  const int slot = static_cast<int>(p->runs % rs_f8_plan::kSlots);
  HIP_TRY(hipEventRecord(ev[0], s));
  const bool fp32 = p->use_fp32 && p->fp32_ok;
  HIP_TRY(rsd::launch_f8_solve(p->d_pts, n, h, mode, seed, hyp_offset, p->d_tuples, p->d_F,
                               p->ld, p->d_counts, p->d_status, s, p->d_F32,
                               fp32 ? &p->frame : nullptr));
  HIP_TRY(hipEventRecord(ev[1], s));
  if (fp32 && p->packed)
    HIP_TRY(rsd::launch_f8_count32p(p->d_pts32, p->d_pts, n, h, p->d_F32, p->d_F, p->ld,
                                    p->pk_waves, guard_packed(p->frame, thresh),
                                    p->d_counts, s, p->pk_variant));
  else if (fp32)
    HIP_TRY(rsd::launch_f8_count32(p->d_pts32, p->d_pts, n, h, p->d_F32, p->d_F, p->ld,
                                   p->resident_waves, guard_constants(p->frame, thresh),
                                   p->d_counts, s, p->count_block, p->prefetch));
  else
    HIP_TRY(rsd::launch_f8_count(p->d_pts, n, h, p->d_F, p->ld, choose_chunk(p, H),
                                 thresh * thresh, p->d_counts, s));
  HIP_TRY(hipEventRecord(ev[2], s));
  HIP_TRY(rsd::launch_f8_tail(p->d_pts, n, h, p->d_F, p->ld, p->d_counts, 1, thresh,
                              p->d_status, p->d_cand, p->d_ccount, p->d_cstd, p->d_cnorm,
                              p->d_res, s));
  HIP_TRY(hipEventRecord(ev[3], s));
  HIP_TRY(hipMemcpyAsync(p->h_slot[slot], p->d_res, p->res_bytes, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipEventRecord(p->done[slot], s));
  p->h_res = p->h_slot[slot];
  ++p->runs;
  p->last_H = H;
  p->pending = true;
  p->have_result = true;
  return RS_OK;
}

static int plan_wait(rs_f8_plan *p) {
  if (!p->have_result) return fail(RS_EINVAL, "no run has been issued on this plan");
  if (p->pending) {
    HIP_TRY(hipSetDevice(p->ctx->device));
    HIP_TRY(hipEventSynchronize(p->done[(p->runs - 1) % rs_f8_plan::kSlots]));
    HIP_TRY(hipStreamSynchronize(p->ctx->stream));
    p->pending = false;
  }
  return RS_OK;
}

extern "C" int rs_f8_plan_result(rs_f8_plan *p, rs_f8_result *out, int64_t *inliers, int64_t cap,
                                 int64_t *n_inliers) {
  if (!p || !out) return fail(RS_EINVAL, "null pointer");
  int st = plan_wait(p);
  if (st) return st;
  const rsd::F8DevResult *r = p->h_res;
  std::memcpy(out->F, r->F, sizeof(out->F));
  out->best_index = r->best_index;
  out->best_count = r->best_count;
  out->best_std = r->best_std;
  out->best_norm = r->best_norm;
  out->max_count_fast = r->max_count_fast;
  out->n_candidates = r->n_candidates;
  out->guard_mismatch = r->guard_mismatch;
  if (n_inliers) *n_inliers = r->n_inliers;
  if (inliers && cap > 0)
    std::memcpy(inliers, r->inliers, sizeof(int64_t) * std::min<int64_t>(cap, r->n_inliers));
  return RS_OK;
}

extern "C" int rs_f8_plan_candidates(rs_f8_plan *p, rs_f8_candidate *out, int64_t cap,
                                     int64_t *n_out) {
  if (!p || !n_out) return fail(RS_EINVAL, "null pointer");
  int st = plan_wait(p);
  if (st) return st;
  HIP_TRY(hipSetDevice(p->ctx->device));
  const int H = static_cast<int>(p->last_H);
  const int nb = rsd::select_blocks(H), pb = rsd::select_per_block(H);
  std::vector<int> bc(nb);
  HIP_TRY(hipMemcpy(bc.data(), p->d_status + 4, sizeof(int) * nb, hipMemcpyDeviceToHost));
  std::vector<int> cand, cc;
  std::vector<double> cs, cn;
  for (int b = 0; b < nb; ++b) {
    if (bc[b] == 0) continue;
    const size_t o = cand.size(), k = static_cast<size_t>(bc[b]);
    const int64_t slot = static_cast<int64_t>(b) * pb;
    cand.resize(o + k);
    cc.resize(o + k);
    cs.resize(o + k);
    cn.resize(o + k);
    HIP_TRY(hipMemcpy(&cand[o], p->d_cand + slot, sizeof(int) * k, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(&cc[o], p->d_ccount + slot, sizeof(int) * k, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(&cs[o], p->d_cstd + slot, sizeof(double) * k, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(&cn[o], p->d_cnorm + slot, sizeof(double) * k, hipMemcpyDeviceToHost));
  }
  const int nc = static_cast<int>(cand.size());
  int cmax = 0;
  for (int i = 0; i < nc; ++i) cmax = std::max(cmax, cc[i]);
  int64_t k = 0;
  for (int i = 0; i < nc; ++i) {
    if (cc[i] != cmax || cmax == 0) continue;
    if (out && k < cap) {
      rs_f8_candidate &o = out[k];
      o.index = cand[i];
      o.count = cc[i];
      o.std_d = cs[i];
      o.norm_d = cn[i];
      for (int q = 0; q < 9; ++q)
        HIP_TRY(hipMemcpy(&o.F[q], p->d_F + q * p->ld + cand[i], sizeof(double),
                          hipMemcpyDeviceToHost));
    }
    ++k;
  }
  *n_out = k;
  return RS_OK;
}

extern "C" int rs_f8_plan_counts(rs_f8_plan *p, int32_t *counts, int64_t H) {
  if (!p || !counts) return fail(RS_EINVAL, "null pointer");
  int st = plan_wait(p);
  if (st) return st;
  if (H > p->last_H) return fail(RS_EINVAL, "H exceeds the last run");
  HIP_TRY(hipSetDevice(p->ctx->device));
  HIP_TRY(hipMemcpy(counts, p->d_counts, sizeof(int) * H, hipMemcpyDeviceToHost));
  return RS_OK;
}

extern "C" int rs_f8_plan_models(rs_f8_plan *p, double *F_out, int64_t H) {
  if (!p || !F_out) return fail(RS_EINVAL, "null pointer");
  int st = plan_wait(p);
  if (st) return st;
  if (H > p->last_H) return fail(RS_EINVAL, "H exceeds the last run");
  HIP_TRY(hipSetDevice(p->ctx->device));
  std::vector<double> soa(static_cast<size_t>(9 * H));
  for (int k = 0; k < 9; ++k)
    HIP_TRY(hipMemcpy(soa.data() + k * H, p->d_F + k * p->ld, sizeof(double) * H,
                      hipMemcpyDeviceToHost));
  for (int64_t h = 0; h < H; ++h)
    for (int k = 0; k < 9; ++k) F_out[h * 9 + k] = soa[k * H + h];
  return RS_OK;
}

extern "C" int rs_f8_plan_kernel_ms(rs_f8_plan *p, double *score_ms, double *solve_ms,
                                    double *total_ms) {
  return rs_f8_plan_kernel_avg(p, 1, score_ms, solve_ms, total_ms);
}

extern "C" int rs_f8_plan_kernel_avg(rs_f8_plan *p, int64_t last_n, double *score_ms,
                                     double *solve_ms, double *total_ms) {
  if (!p) return fail(RS_EINVAL, "null plan");
  int st = plan_wait(p);
  if (st) return st;
  const int64_t k = std::max<int64_t>(1, std::min<int64_t>({last_n, p->runs,
                                                            (int64_t)rs_f8_plan::kEvRing}));
  double sa = 0, sb = 0, st_ = 0;
  for (int64_t r = p->runs - k; r < p->runs; ++r) {
    hipEvent_t *ev = p->ring[r % rs_f8_plan::kEvRing];
    float a = 0, b = 0, t = 0;
    HIP_TRY(hipEventElapsedTime(&a, ev[0], ev[1]));
    HIP_TRY(hipEventElapsedTime(&b, ev[1], ev[2]));
    HIP_TRY(hipEventElapsedTime(&t, ev[0], ev[3]));
    sa += a;
    sb += b;
    st_ += t;
  }
  if (solve_ms) *solve_ms = sa / k;
  if (score_ms) *score_ms = sb / k;
  if (total_ms) *total_ms = st_ / k;
  return RS_OK;
}

// ------------------------------------------------------------------------------------------
// numpy-exact one call (fun.getFFromLabCode loop)
// ------------------------------------------------------------------------------------------
extern "C" int rs_f8_ransac_np(rs_ctx *c, const double *p1, const double *p2, int64_t n,
                               int64_t H, uint32_t *mt_key, int32_t *mt_pos, double thresh,
                               rs_f8_result *out, int64_t *inliers, int64_t cap,
                               int64_t *n_inliers) {
  if (!c || !p1 || !p2 || !mt_key || !mt_pos || !out) return fail(RS_EINVAL, "null pointer");
  if (n < 8)
    return fail(RS_EINVAL, "Cannot take a larger sample than population when 'replace=False'");
  if (H < 1) return fail(RS_EINVAL, "hypothesis count must be positive");
  if (c->np_plan && (c->np_plan->n != n || c->np_plan->max_hyp < H)) {
    rs_f8_plan_destroy(c->np_plan);
    c->np_plan = nullptr;
  }
  int st;
  if (!c->np_plan && (st = rs_f8_plan_create(c, n, H, &c->np_plan))) return st;
  if ((st = rs_f8_plan_set_points(c->np_plan, p1, p2))) return st;
  std::vector<int32_t> tuples(static_cast<size_t>(8 * H));
  uint32_t key[RS_MT_N];
  int32_t pos = *mt_pos;
  std::memcpy(key, mt_key, sizeof(key));
  if ((st = rs_np_choice_tuples(key, &pos, n, 8, H, tuples.data()))) return st;
  if ((st = rs_f8_plan_run(c->np_plan, H, RS_SAMPLER_TUPLES, 0, 0, tuples.data(), thresh)))
    return st;
  if ((st = rs_f8_plan_result(c->np_plan, out, inliers, cap, n_inliers))) return st;
  std::memcpy(mt_key, key, sizeof(key));
  *mt_pos = pos;
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
