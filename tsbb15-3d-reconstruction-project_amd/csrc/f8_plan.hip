// F plans (include/rsamd.h "RANSAC-F"): one correspondence set resident in HBM, runs of H
// hypotheses issued back to back.  Replaces the fun.getFFromLabCode hypothesis loop
// (fun.py:298-328).
//
// Per-run buffer sets (kBufs) used in rotation.  By default everything runs on the context's
// HIP stream: rs_f8_plan_run(k) enqueues
//
//   k_f8_tail_solve  [selection tail of run k-1 | solve of run k]   (one launch)
//   k_f8_count32x    counts of run k (+ fused c*)
//
// and leaves run k's tail pending: it rides along with run k+1's solve, or is flushed alone
// by rs_f8_plan_result / set_points / destroy.  The tail (candidates, reference statistics,
// replay, S_RANSAC; latency bound, a few busy workgroups) and the solve (latency bound,
// ~1.5 waves per SIMD) thus share the machine instead of running back to back, with no
// cross-stream events (each event or wait is a packet the command processor retires
// between kernels; r01: ~3.5 us each).
//
// Optional overlap mode (RSAMD_OVERLAP=1, off by default: measured 2-4 % slower, DESIGN.md
// "Next"): run k's solve on a side stream ss, its count on the context stream and its tail
// on a third stream ts, chained by per-buffer-set events (ev_solve / ev_count / ev_tail); a
// set's solve waits for the tail of the run that used the set kBufs runs back, and the
// parity samplers wait for the set's last solve before they refill its tuples.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "common.h"
#include "ctx.h"
#include "device_math.h"
#include "f8_kernels.h"

using rs::fail;
using rs::hip_fail;

namespace {

// Per-run device buffers; two sets alternate between consecutive runs.
struct RunBufs {
  double *d_F = nullptr;       // 9 x ld SoA models (float64)
  float *d_F32 = nullptr;      // 9 x ld SoA models in the unit frame (fp32 counting)
  int *d_counts = nullptr;     // fast counts
  int *d_tuples = nullptr;     // host tuples (parity mode)
  int *d_cand = nullptr;       // candidate hypothesis ids, per-block segments
  int *d_status = nullptr;     // [c*, n_candidates, ., ., per-block candidate counts]
  int *d_ccount = nullptr;
  int *d_cfast = nullptr;      // fast counts of the candidates (guard_mismatch diagnostic)
  int *d_spec = nullptr;       // per select block: S_RANSAC of its first candidate
  int *d_spec_j = nullptr;     // per select block: that candidate's local index, or -1
  double *d_cstd = nullptr, *d_cnorm = nullptr;
  rsd::F8DevResult *d_res = nullptr;
  int *d_gdone = nullptr;      // per-group finish counters (fused c* in k_f8_count32x)
  float4 *d_G4 = nullptr;      // per-hypothesis decision constants (k_f8_count32q)
  // host tuples (parity mode fed from the host) are staged in a pinned buffer owned by the
  // set, so the caller's array may go away as soon as rs_f8_plan_run returns; ev_copy marks
  // the end of the H2D copy that last read it (waited for before the buffer is refilled)
  int *h_tuples = nullptr;
  int64_t cap_h_tuples = 0;
  hipEvent_t ev_copy = nullptr;
  bool copy_pending = false;
};

constexpr int kOverlapDefault = 0;  // rs_f8_plan::overlap unless RSAMD_OVERLAP is set

int env_int(const char *name, int dflt) {
  const char *v = std::getenv(name);
  return v ? std::atoi(v) : dflt;
}

}  // namespace

struct rs_f8_plan {
  rs_ctx *ctx = nullptr;
  int64_t n = 0, max_hyp = 0, ld = 0;
  int64_t cap_n = 0;           // points the per-point buffers hold (>= n; plan_retarget)
  double *d_p12 = nullptr;     // staging (2,n) p1 then (2,n) p2
  rsd::Pt *d_pts = nullptr;    // AoS float64 points
  float4 *d_pts32q = nullptr;  // the same, point-pair layout (k_f8_count32q)
  static constexpr int kBufs = 3, kSlots = 4, kEvRing = 64;
  RunBufs buf[kBufs];
  // Each run's tail writes its result header into its own pinned slot (through the host
  // mapping) and S_RANSAC into its buffer set's HBM result; rs_f8_plan_result waits for the
  // last run and copies S_RANSAC on demand.
  rsd::F8DevResult *h_slot[kSlots] = {};
  rsd::F8DevResult *h_slot_dev[kSlots] = {};
  int *h_inl[kSlots] = {};      // pinned S_RANSAC per slot (cap_n ints), written by the tail
  int *h_inl_dev[kSlots] = {};
  hipEvent_t ring[kEvRing][4] = {};  // count start/end; tail+solve launch start/end
  bool timed[kEvRing] = {};          // whether run r % kEvRing recorded its events
  int64_t runs = 0, last_H = 0;
  bool pending = false;              // stream work not yet waited for
  bool tail_pending = false;         // the last run's tail is not enqueued yet
  // Overlap mode (RSAMD_OVERLAP=1; kOverlapDefault otherwise): run k's solve on ss, its
  // count on the context stream, its tail on ts, chained by events, so the next run's solve and
  // this run's tail fill the CUs the counting kernel's drain leaves idle.  A buffer set's solve
  // waits for the tail of the run that used the set before (kBufs runs back).
  bool overlap = kOverlapDefault != 0;
  hipStream_t ss = nullptr, ts = nullptr;
  hipEvent_t ev_solve[kBufs] = {}, ev_count[kBufs] = {}, ev_tail[kBufs] = {};
  hipEvent_t ev_np = nullptr;  // parity mode: the parse queued before the solve (overlap)
  rsd::TailArgs tail{};              // ... its arguments
  // counting kernel: fp32 point-pair kernel with the float64 guard re-test (default), or the
  // plain float64 kernel (rs_f8_plan_set_count_precision; both give identical counts)
  rsd::Frame frame{1.0, 0.0, 0.0, 0.0, 0.0};
  bool fp32_ok = false;       // finite points and a non-degenerate frame
  bool use_fp32 = true;
  // HIP timing events per run (each is a marker packet between kernels): 0 none, 1 around the
  // counting kernel (default; the bench's roofline timing), 2 also the tail+solve launch
  int timing = 1;
  int timing_every = 1;       // RSAMD_TIMING_EVERY / rs_f8_plan_set_timing: time every k-th run
  int q_waves = 6144;         // resident waves of the fp32 kernel (RSAMD_WAVES)
  int q_slices = 0;           // slices per resident wave (RSAMD_QSLICES; 0: count32q_shape)
  int tail_cus = 256;         // CUs shared by the tail + solve launch
  int nospec = 0;             // RSAMD_NOSPEC=1 (test hook): the replay extracts S_RANSAC itself
  uint64_t *d_ts = nullptr;   // RSAMD_TSTAMP=<file>: wave timeline of the counting kernel
  const char *ts_path = nullptr;

  const RunBufs &last() const { return buf[(runs - 1) % kBufs]; }
};

#define HIP_TRY(expr)                                   \
  do {                                                  \
    hipError_t e_ = (expr);                             \
    if (e_ != hipSuccess) return hip_fail(e_, #expr);   \
  } while (0)

static void plan_free(rs_f8_plan *p) {
  (void)hipFree(p->d_p12);
  (void)hipFree(p->d_pts);
  (void)hipFree(p->d_pts32q);
  if (p->d_ts) {
    (void)rsd::set_count_timeline(nullptr);
    (void)hipFree(p->d_ts);
  }
  for (RunBufs &b : p->buf) {
    (void)hipFree(b.d_F);
    (void)hipFree(b.d_F32);
    (void)hipFree(b.d_counts);
    (void)hipFree(b.d_tuples);
    (void)hipFree(b.d_cand);
    (void)hipFree(b.d_status);
    (void)hipFree(b.d_ccount);
    (void)hipFree(b.d_cfast);
    (void)hipFree(b.d_spec);
    (void)hipFree(b.d_spec_j);
    (void)hipFree(b.d_cstd);
    (void)hipFree(b.d_cnorm);
    (void)hipFree(b.d_res);
    (void)hipFree(b.d_gdone);
    (void)hipFree(b.d_G4);
    if (b.h_tuples) (void)hipHostFree(b.h_tuples);
    if (b.ev_copy) (void)hipEventDestroy(b.ev_copy);
  }
  for (int k = 0; k < rs_f8_plan::kBufs; ++k) {
    if (p->ev_solve[k]) (void)hipEventDestroy(p->ev_solve[k]);
    if (p->ev_count[k]) (void)hipEventDestroy(p->ev_count[k]);
    if (p->ev_tail[k]) (void)hipEventDestroy(p->ev_tail[k]);
  }
  if (p->ev_np) (void)hipEventDestroy(p->ev_np);
  if (p->ss) (void)hipStreamDestroy(p->ss);
  if (p->ts) (void)hipStreamDestroy(p->ts);
  for (auto &h : p->h_slot)
    if (h) (void)hipHostFree(h);
  for (auto &h : p->h_inl)
    if (h) (void)hipHostFree(h);
  for (auto &r : p->ring)
    for (auto &e : r)
      if (e) (void)hipEventDestroy(e);
}

// the pinned S_RANSAC buffers of the result slots, cap ints each (the tail writes the winner's
// list through the host mapping; rs_f8_plan_result reads it without a copy)
static hipError_t alloc_h_inl(rs_f8_plan *p, int64_t cap) {
  hipError_t e = hipSuccess;
  for (int k = 0; k < rs_f8_plan::kSlots; ++k) {
    if (p->h_inl[k]) (void)hipHostFree(p->h_inl[k]);
    p->h_inl[k] = nullptr;
    p->h_inl_dev[k] = nullptr;
    if (e == hipSuccess)
      e = hipHostMalloc(reinterpret_cast<void **>(&p->h_inl[k]), sizeof(int) * static_cast<size_t>(cap));
    if (e == hipSuccess)
      e = hipHostGetDevicePointer(reinterpret_cast<void **>(&p->h_inl_dev[k]), p->h_inl[k], 0);
  }
  return e;
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
  p->cap_n = n;
  p->max_hyp = max_hyp;
  p->ld = (max_hyp + 63) / 64 * 64;
  const size_t res_bytes = sizeof(rsd::F8DevResult) + sizeof(int64_t) * static_cast<size_t>(n);
  if (const char *cm = std::getenv("RSAMD_COUNT"))  // tools: RSAMD_COUNT=fp64
    p->use_fp32 = std::strcmp(cm, "fp64") != 0;
  p->timing = env_int("RSAMD_TIMING", 1);
  p->timing_every = std::max(1, env_int("RSAMD_TIMING_EVERY", 1));
  {
    int cus = 256;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess)
      cus = 256;
    p->tail_cus = cus;
    p->q_waves = std::max(1, env_int("RSAMD_WAVES", rsd::count32q_resident_waves(c->device)));
    p->q_slices = env_int("RSAMD_QSLICES", 0);
  }
  hipError_t e = hipSuccess;
#define ALLOC(ptr, bytes) \
  if (e == hipSuccess) e = hipMalloc(&(ptr), (bytes));
  ALLOC(p->d_p12, sizeof(double) * 4 * n);
  ALLOC(p->d_pts, sizeof(rsd::Pt) * n);
  ALLOC(p->d_pts32q, sizeof(float4) * ((n + 7) & ~7LL));
  for (RunBufs &b : p->buf) {
    ALLOC(b.d_F, sizeof(double) * 9 * p->ld);
    ALLOC(b.d_F32, sizeof(float) * 9 * p->ld);
    ALLOC(b.d_counts, sizeof(int) * p->ld);
    ALLOC(b.d_tuples, sizeof(int) * 8 * p->ld);
    ALLOC(b.d_cand, sizeof(int) * p->ld);
    ALLOC(b.d_status, sizeof(int) * rsd::kStatusWords);
    ALLOC(b.d_ccount, sizeof(int) * p->ld);
    ALLOC(b.d_cfast, sizeof(int) * p->ld);
    ALLOC(b.d_spec, sizeof(int) * rsd::kSelectBlocks * static_cast<size_t>(n));
    ALLOC(b.d_spec_j, sizeof(int) * rsd::kSelectBlocks);
    ALLOC(b.d_cstd, sizeof(double) * p->ld);
    ALLOC(b.d_cnorm, sizeof(double) * p->ld);
    ALLOC(b.d_res, res_bytes);
    ALLOC(b.d_gdone, sizeof(int) * (p->ld / 64));
    ALLOC(b.d_G4, sizeof(float4) * p->ld);
  }
#undef ALLOC
  for (int k = 0; k < rs_f8_plan::kSlots; ++k) {
    if (e == hipSuccess)
      e = hipHostMalloc(reinterpret_cast<void **>(&p->h_slot[k]), sizeof(rsd::F8DevResult));
    if (e == hipSuccess)
      e = hipHostGetDevicePointer(reinterpret_cast<void **>(&p->h_slot_dev[k]), p->h_slot[k], 0);
  }
  if (e == hipSuccess) e = alloc_h_inl(p, p->cap_n);
  for (auto &r : p->ring)
    for (auto &ev : r)
      if (e == hipSuccess) e = hipEventCreate(&ev);
  p->overlap = env_int("RSAMD_OVERLAP", kOverlapDefault) != 0;
  if (p->overlap) {
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&p->ss, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&p->ts, hipStreamNonBlocking);
    for (int k = 0; k < rs_f8_plan::kBufs; ++k) {
      if (e == hipSuccess) e = hipEventCreateWithFlags(&p->ev_solve[k], hipEventDisableTiming);
      if (e == hipSuccess) e = hipEventCreateWithFlags(&p->ev_count[k], hipEventDisableTiming);
      if (e == hipSuccess) e = hipEventCreateWithFlags(&p->ev_tail[k], hipEventDisableTiming);
    }
  }
  p->nospec = env_int("RSAMD_NOSPEC", 0) != 0;
  p->ts_path = std::getenv("RSAMD_TSTAMP");
  if (p->ts_path) {
    const size_t tsb = sizeof(uint64_t) * rsd::kCountTsWords * (static_cast<size_t>(p->q_waves) * 64 + 1024);
    if (hipMalloc(&p->d_ts, tsb) == hipSuccess) {
      (void)hipMemset(p->d_ts, 0, tsb);
      (void)rsd::set_count_timeline(p->d_ts);
    }
  }
  if (e != hipSuccess) {
    plan_free(p);
    delete p;
    return hip_fail(e, "rs_f8_plan_create");
  }
  *out = p;
  return RS_OK;
}

static int plan_flush(rs_f8_plan *p);

// A new population for an existing plan (the drop-in's calls, one pair after another): the
// per-point buffers are reallocated only when n exceeds what they hold; the per-hypothesis
// buffers, events and pinned slots are kept (a fresh plan allocates ~20 buffers)
static int plan_retarget(rs_f8_plan *p, int64_t n) {
  if (n < 8) return fail(RS_EINVAL, "Cannot take a larger sample than population when 'replace=False'");
  if (n > (1LL << 30)) return fail(RS_EINVAL, "plan dimensions out of range");
  int st = plan_flush(p);  // runs in flight read the resident points and results
  if (st) return st;
  if (n > p->cap_n) {
    const int64_t cap = std::max<int64_t>(n, p->cap_n + p->cap_n / 4);
    (void)hipFree(p->d_p12);
    (void)hipFree(p->d_pts);
    (void)hipFree(p->d_pts32q);
    p->d_p12 = nullptr;
    p->d_pts = nullptr;
    p->d_pts32q = nullptr;
    hipError_t e = hipMalloc(&p->d_p12, sizeof(double) * 4 * cap);
    if (e == hipSuccess) e = hipMalloc(&p->d_pts, sizeof(rsd::Pt) * cap);
    if (e == hipSuccess) e = hipMalloc(&p->d_pts32q, sizeof(float4) * ((cap + 7) & ~7LL));
    for (RunBufs &b : p->buf) {
      (void)hipFree(b.d_spec);
      (void)hipFree(b.d_res);
      b.d_spec = nullptr;
      b.d_res = nullptr;
      if (e == hipSuccess) e = hipMalloc(&b.d_spec, sizeof(int) * rsd::kSelectBlocks * static_cast<size_t>(cap));
      if (e == hipSuccess)
        e = hipMalloc(&b.d_res, sizeof(rsd::F8DevResult) + sizeof(int64_t) * static_cast<size_t>(cap));
    }
    if (e == hipSuccess) e = alloc_h_inl(p, cap);
    if (e != hipSuccess) {
      // the old buffers are gone: mark the plan empty (a later retarget reallocates) and let
      // the caller drop it (rs_f8_ransac_np destroys its cached plan)
      p->cap_n = 0;
      p->n = 0;
      return hip_fail(e, "rs_f8_plan retarget");
    }
    p->cap_n = cap;
  }
  p->n = n;
  p->fp32_ok = false;  // set_points decides it for the new points
  return RS_OK;
}

// Enqueue the pending tail alone (no next run to ride along with), then wait for the stream.
static int plan_flush(rs_f8_plan *p) {
  HIP_TRY(hipSetDevice(p->ctx->device));
  if (p->tail_pending) {
    HIP_TRY(rsd::launch_f8_tail_solve(&p->tail, nullptr, p->ctx->stream));
    p->tail_pending = false;
  }
  if (p->overlap) {
    HIP_TRY(hipStreamSynchronize(p->ss));
    HIP_TRY(hipStreamSynchronize(p->ts));
  }
  HIP_TRY(hipStreamSynchronize(p->ctx->stream));
  p->pending = false;
  return RS_OK;
}

extern "C" int rs_f8_plan_destroy(rs_f8_plan *p) {
  if (!p) return RS_OK;
  (void)plan_flush(p);
  plan_free(p);
  delete p;
  return RS_OK;
}

extern "C" int rs_f8_plan_set_points(rs_f8_plan *p, const double *p1, const double *p2) {
  if (!p || !p1 || !p2) return fail(RS_EINVAL, "null pointer");
  int st = plan_flush(p);  // runs in flight read the resident points
  if (st) return st;
  rs_ctx *c = p->ctx;
  const int64_t n = p->n;
  const size_t b = sizeof(double) * 2 * n;
  HIP_TRY(hipMemcpyAsync(p->d_p12, p1, b, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(p->d_p12 + 2 * n, p2, b, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(rsd::launch_pack_points(p->d_p12, p->d_p12 + 2 * n, static_cast<int>(n), p->d_pts,
                                  c->stream));
  rsd::Frame fr{};
  p->fp32_ok = rsd::unit_frame(p1, p2, n, fr);
  if (p->fp32_ok) {
    p->frame = fr;
    HIP_TRY(rsd::launch_pack_points32q(p->d_pts, static_cast<int>(n), fr, p->d_pts32q,
                                       c->stream));
  }
  HIP_TRY(hipStreamSynchronize(c->stream));
  return RS_OK;
}

static int choose_chunk(const rs_f8_plan *p, int64_t H) {
  const int64_t groups = (H + 63) / 64;
  // aim for >= 8 units of work per SIMD (1024 SIMDs) without chunks below 64 points
  int64_t nchunks = (8192 + groups - 1) / groups;
  nchunks = std::max<int64_t>(1, std::min<int64_t>(nchunks, (p->n + 63) / 64));
  return static_cast<int>((p->n + nchunks - 1) / nchunks);
}

// One run.  dev_tuples: tuple mode with the tuples already written (in range, by the GPU
// parity stream) into the buffer set this run uses, so there is no host copy or check.
static int plan_run(rs_f8_plan *p, int64_t H, int32_t mode, uint64_t seed, uint64_t hyp_offset,
                    const int32_t *host_tuples, double thresh, bool dev_tuples) {
  if (!p) return fail(RS_EINVAL, "null plan");
  if (H < 1 || H > p->max_hyp) return fail(RS_EINVAL, "hypothesis count out of plan range");
  if (mode != RS_SAMPLER_PHILOX && mode != RS_SAMPLER_TUPLES)
    return fail(RS_EINVAL, "unknown sampler mode");
  if (mode == RS_SAMPLER_TUPLES && !host_tuples && !dev_tuples)
    return fail(RS_EINVAL, "tuples required");
  if (!(thresh == thresh)) return fail(RS_EINVAL, "threshold is NaN");
  if (mode == RS_SAMPLER_TUPLES && !dev_tuples)
    for (int64_t i = 0; i < 8 * H; ++i)
      if (host_tuples[i] < 0 || host_tuples[i] >= p->n)
        return fail(RS_EINVAL, "tuple index out of range");
  rs_ctx *c = p->ctx;
  HIP_TRY(hipSetDevice(c->device));
  const int n = static_cast<int>(p->n), h = static_cast<int>(H);
  RunBufs &b = p->buf[p->runs % rs_f8_plan::kBufs];
  hipEvent_t *ev = p->ring[p->runs % rs_f8_plan::kEvRing];
  const int tl = (p->runs % p->timing_every == 0) ? p->timing : 0;  // this run's timing level
  p->timed[p->runs % rs_f8_plan::kEvRing] = tl >= 1;
  const int slot = static_cast<int>(p->runs % rs_f8_plan::kSlots);
  const bool fp32 = p->use_fp32 && p->fp32_ok;
  hipStream_t ms = c->stream;
  const int bi = static_cast<int>(p->runs % rs_f8_plan::kBufs);
  // the solve's stream: ss in overlap mode, after the tail of this buffer set's previous run
  hipStream_t sv = p->overlap ? p->ss : ms;
  if (p->overlap) HIP_TRY(hipStreamWaitEvent(sv, p->ev_tail[bi], 0));

  if (mode == RS_SAMPLER_TUPLES && !dev_tuples) {
    // stage through the set's pinned buffer: the copy no longer reads caller memory after
    // this call returns (the caller may free or reuse its tuples at once)
    if (b.copy_pending) {
      HIP_TRY(hipEventSynchronize(b.ev_copy));
      b.copy_pending = false;
    }
    if (b.cap_h_tuples < 8 * H) {
      if (b.h_tuples) HIP_TRY(hipHostFree(b.h_tuples));
      b.h_tuples = nullptr;
      b.cap_h_tuples = 0;
      HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&b.h_tuples), sizeof(int) * 8 * p->ld));
      b.cap_h_tuples = 8 * p->ld;
    }
    if (!b.ev_copy) HIP_TRY(hipEventCreateWithFlags(&b.ev_copy, hipEventDisableTiming));
    std::memcpy(b.h_tuples, host_tuples, sizeof(int) * 8 * H);
    HIP_TRY(hipMemcpyAsync(b.d_tuples, b.h_tuples, sizeof(int) * 8 * H, hipMemcpyHostToDevice,
                           sv));
    HIP_TRY(hipEventRecord(b.ev_copy, sv));
    b.copy_pending = true;
  }
  // [tail of the previous run | solve of this run]: buffer set b was last read by run k-2,
  // whose tail is complete (stream order)
  rsd::SolveArgs sa{};
  sa.pts = p->d_pts;
  sa.n = n;
  sa.H = h;
  sa.mode = mode;
  sa.seed = seed;
  sa.hyp_offset = hyp_offset;
  sa.tuples = b.d_tuples;
  sa.Fsoa = b.d_F;
  sa.ld = p->ld;
  sa.counts = b.d_counts;
  sa.status = b.d_status;
  sa.F32soa = fp32 ? b.d_F32 : nullptr;
  sa.frame = fp32 ? p->frame : rsd::Frame{1.0, 0.0, 0.0, 0.0, 0.0};
  sa.gdone = b.d_gdone;
  if (fp32) {
    const rsd::Bounds gb = rsd::fp32_bounds(p->frame, thresh);
    sa.G4 = b.d_G4;
    sa.gT = gb.thr2;
    sa.gDe = gb.De;
    sa.gDn = gb.Dn;
  }
  if (tl >= 2) HIP_TRY(hipEventRecord(ev[2], sv));
  HIP_TRY(rsd::launch_f8_tail_solve(p->tail_pending ? &p->tail : nullptr, &sa, sv, p->tail_cus));
  p->tail_pending = false;
  if (tl >= 2) HIP_TRY(hipEventRecord(ev[3], sv));
  if (p->overlap) {
    HIP_TRY(hipEventRecord(p->ev_solve[bi], sv));
    HIP_TRY(hipStreamWaitEvent(ms, p->ev_solve[bi], 0));
  }

  // counts of this run
  if (tl >= 1) HIP_TRY(hipEventRecord(ev[0], ms));
  if (fp32) {
    // fused c*: the chunk that completes a hypothesis group folds its max into status[0]
    const rsd::Count32qShape sh = rsd::count32q_shape(n, h, p->q_waves, p->q_slices);
    HIP_TRY(rsd::launch_f8_count32q(p->d_pts32q, p->d_pts, n, h, b.d_F32, b.d_F, p->ld, sh,
                                    rsd::GuardW{thresh * thresh}, b.d_counts, ms, b.d_gdone,
                                    b.d_status, b.d_G4));
  } else {
    HIP_TRY(rsd::launch_f8_count(p->d_pts, n, h, b.d_F, p->ld, choose_chunk(p, H),
                                 thresh * thresh, b.d_counts, ms));
    HIP_TRY(rsd::launch_f8_max(b.d_counts, h, b.d_status, ms));
  }
  if (tl >= 1) HIP_TRY(hipEventRecord(ev[1], ms));

  // this run's tail rides along with the next run's solve (or plan_flush)
  rsd::TailArgs &ta = p->tail;
  ta = rsd::TailArgs{};
  ta.pts = p->d_pts;
  ta.n = n;
  ta.H = h;
  ta.slack = 1;
  ta.Fsoa = b.d_F;
  ta.ld = p->ld;
  ta.counts = b.d_counts;
  ta.status = b.d_status;
  ta.thresh = thresh;
  ta.cand = b.d_cand;
  ta.ccount = b.d_ccount;
  ta.cfast = b.d_cfast;
  ta.spec = b.d_spec;
  ta.spec_j = b.d_spec_j;
  ta.nospec = p->nospec;
  ta.cstd = b.d_cstd;
  ta.cnorm = b.d_cnorm;
  ta.res = b.d_res;
  ta.hres = p->h_slot_dev[slot];
  ta.hinl = p->h_inl_dev[slot];
  if (p->overlap) {
    // the tail on ts right after this run's count; the next run's count does not wait for it
    HIP_TRY(hipEventRecord(p->ev_count[bi], ms));
    HIP_TRY(hipStreamWaitEvent(p->ts, p->ev_count[bi], 0));
    HIP_TRY(rsd::launch_f8_tail_solve(&ta, nullptr, p->ts, p->tail_cus));
    HIP_TRY(hipEventRecord(p->ev_tail[bi], p->ts));
  } else {
    p->tail_pending = true;
  }
  ++p->runs;
  p->last_H = H;
  p->pending = true;
  return RS_OK;
}

extern "C" int rs_f8_plan_run(rs_f8_plan *p, int64_t H, int32_t mode, uint64_t seed,
                              uint64_t hyp_offset, const int32_t *host_tuples, double thresh) {
  return plan_run(p, H, mode, seed, hyp_offset, host_tuples, thresh, false);
}

// Parity mode with the numpy stream sampled on the GPU (np_sampler.hip) straight into the
// tuple buffer of the run about to be issued; advances (key, pos).  The sampler is synchronous
// on the context stream, and that buffer set was last read by run k-2's solve, which precedes
// it in stream order.  Populations beyond the GPU parse's range (and RSAMD_NP_HOST, a test
// hook) go through the host replay.
extern "C" int rs_f8_plan_run_np_slice(rs_f8_plan *p, int64_t H, int64_t start, int64_t count,
                                       uint32_t *key, int32_t *pos, double thresh) {
  if (!p || !key || !pos) return fail(RS_EINVAL, "null pointer");
  if (H < 1 || start < 0 || count < 1 || start + count > H)
    return fail(RS_EINVAL, "hypothesis slice out of range");
  if (count > p->max_hyp) return fail(RS_EINVAL, "hypothesis count out of plan range");
  int st;
  if (rs::np_gpu_supported(p->n, 8) && std::getenv("RSAMD_NP_HOST") == nullptr) {
    if (p->overlap) HIP_TRY(hipEventSynchronize(p->ev_solve[p->runs % rs_f8_plan::kBufs]));
    if (start == 0 && count == H && std::getenv("RSAMD_NP_SYNC") == nullptr) {
      // the whole draw in one segment: the run is queued behind the parse before the host
      // waits for the parse's outcome (no host gap between them); should the parse ask to be
      // drawn again (a wrap-log overflow), that run is superseded by the synchronous path below
      bool queued = false;
      RunBufs &b = p->buf[p->runs % rs_f8_plan::kBufs];
      if ((st = rs::np_choice_enqueue(p->ctx, key, *pos, p->n, 8, H, b.d_tuples, &queued)))
        return st;
      if (queued) {
        if (p->overlap) {  // the solve's stream reads the tuples after the parse
          if (!p->ev_np) HIP_TRY(hipEventCreateWithFlags(&p->ev_np, hipEventDisableTiming));
          HIP_TRY(hipEventRecord(p->ev_np, p->ctx->stream));
          HIP_TRY(hipStreamWaitEvent(p->ss, p->ev_np, 0));
        }
        const int run_st = plan_run(p, count, RS_SAMPLER_TUPLES, 0, 0, nullptr, thresh, true);
        bool rerun = false;
        if ((st = rs::np_choice_finish(p->ctx, key, pos, &rerun))) return st;
        if (run_st || !rerun) return run_st;
        if (p->overlap) HIP_TRY(hipEventSynchronize(p->ev_solve[p->runs % rs_f8_plan::kBufs]));
      }
    }
    RunBufs &b = p->buf[p->runs % rs_f8_plan::kBufs];
    if ((st = rs::np_choice_device(p->ctx, key, pos, p->n, 8, H, b.d_tuples, false, start, count)))
      return st;
    return plan_run(p, count, RS_SAMPLER_TUPLES, 0, static_cast<uint64_t>(start), nullptr, thresh,
                    true);
  }
  std::vector<int32_t> tuples(static_cast<size_t>(8 * H));
  if ((st = rs_np_choice_tuples(key, pos, p->n, 8, H, tuples.data()))) return st;
  return plan_run(p, count, RS_SAMPLER_TUPLES, 0, static_cast<uint64_t>(start),
                  tuples.data() + 8 * start, thresh, false);
}

// This rank's hypotheses [base, hi) of a sharded parse (rs_np_shard_*, step 4) straight into
// the tuple buffer of the run about to be issued, then that run; a rank holding no
// hypothesis only reads the final state (final_idx >= 0).  Candidate indices are run-local.
extern "C" int rs_f8_plan_run_np_shard(rs_f8_plan *p, rs_np_shard *sh, int64_t base, int64_t hi,
                                       int64_t next_start, int64_t final_idx, uint32_t *key_out,
                                       int32_t *pos_out, double thresh) {
  if (!p || !sh) return fail(RS_EINVAL, "null pointer");
  const int64_t count = hi - base;
  if (count > p->max_hyp) return fail(RS_EINVAL, "hypothesis count out of plan range");
  RunBufs &b = p->buf[p->runs % rs_f8_plan::kBufs];
  if (p->overlap) HIP_TRY(hipEventSynchronize(p->ev_solve[p->runs % rs_f8_plan::kBufs]));
  int st;
  if ((st = rs::np_shard_tuples_device(sh, base, hi, next_start, final_idx,
                                       count > 0 ? b.d_tuples : nullptr, key_out, pos_out)))
    return st;
  if (count < 1) return RS_OK;
  return plan_run(p, count, RS_SAMPLER_TUPLES, 0, static_cast<uint64_t>(base), nullptr, thresh, true);
}

extern "C" int rs_f8_plan_run_np(rs_f8_plan *p, int64_t H, uint32_t *key, int32_t *pos,
                                 double thresh) {
  return rs_f8_plan_run_np_slice(p, H, 0, H, key, pos, thresh);
}

// Complete the last run (its pending tail) and wait.  Accessors below then read its buffer
// set synchronously.
static int plan_wait(rs_f8_plan *p) {
  if (p->runs == 0) return fail(RS_EINVAL, "no run has been issued on this plan");
  return p->pending ? plan_flush(p) : RS_OK;
}

extern "C" int rs_f8_plan_result(rs_f8_plan *p, rs_f8_result *out, int64_t *inliers, int64_t cap,
                                 int64_t *n_inliers) {
  if (!p || !out) return fail(RS_EINVAL, "null pointer");
  int st = plan_wait(p);
  if (st) return st;
  const rsd::F8DevResult *r = p->h_slot[(p->runs - 1) % rs_f8_plan::kSlots];
  std::memcpy(out->F, r->F, sizeof(out->F));
  out->best_index = r->best_index;
  out->best_count = r->best_count;
  out->best_std = r->best_std;
  out->best_norm = r->best_norm;
  out->max_count_fast = r->max_count_fast;
  out->n_candidates = r->n_candidates;
  out->guard_mismatch = r->guard_mismatch;
  if (p->d_ts && p->ts_path) {  // diagnostics: append this run's wave timeline
    std::vector<uint64_t> t(rsd::kCountTsWords * (static_cast<size_t>(p->q_waves) * 64 + 1024));
    if (hipMemcpy(t.data(), p->d_ts, sizeof(uint64_t) * t.size(), hipMemcpyDeviceToHost) ==
        hipSuccess) {
      if (FILE *f = std::fopen(p->ts_path, "ab")) {
        std::fwrite(t.data(), sizeof(uint64_t), t.size(), f);
        std::fclose(f);
      }
    }
  }
  if (n_inliers) *n_inliers = r->n_inliers;
  const int64_t k = std::min<int64_t>(cap, r->n_inliers);
  if (inliers && k > 0) {
    if (const int *h = p->h_inl[(p->runs - 1) % rs_f8_plan::kSlots]) {  // written by the tail
      for (int64_t i = 0; i < k; ++i) inliers[i] = h[i];
    } else if (r->inl_row >= 0) {   // the winner's select block kept it (int32 row)
      std::vector<int32_t> row(static_cast<size_t>(k));
      HIP_TRY(hipMemcpy(row.data(), p->last().d_spec + r->inl_row * p->n, sizeof(int32_t) * k,
                        hipMemcpyDeviceToHost));
      for (int64_t i = 0; i < k; ++i) inliers[i] = row[static_cast<size_t>(i)];
    } else {
      HIP_TRY(hipMemcpy(inliers, p->last().d_res->inliers, sizeof(int64_t) * k,
                        hipMemcpyDeviceToHost));
    }
  }
  return RS_OK;
}

extern "C" int rs_f8_plan_candidates(rs_f8_plan *p, rs_f8_candidate *out, int64_t cap,
                                     int64_t *n_out) {
  if (!p || !n_out) return fail(RS_EINVAL, "null pointer");
  int st = plan_wait(p);
  if (st) return st;
  const RunBufs &b = p->last();
  const int H = static_cast<int>(p->last_H);
  int pb = 0;  // the select-block layout the tail used (status word 3)
  HIP_TRY(hipMemcpy(&pb, b.d_status + 3, sizeof(int), hipMemcpyDeviceToHost));
  if (pb < 1) return fail(RS_EINVAL, "no selection layout recorded for the last run");
  const int nb = (H + pb - 1) / pb;
  std::vector<int> bc(nb);
  HIP_TRY(hipMemcpy(bc.data(), b.d_status + 4, sizeof(int) * nb, hipMemcpyDeviceToHost));
  std::vector<int> cand, cc;
  std::vector<double> cs, cn;
  for (int k = 0; k < nb; ++k) {
    if (bc[k] == 0) continue;
    const size_t o = cand.size(), m = static_cast<size_t>(bc[k]);
    const int64_t seg = static_cast<int64_t>(k) * pb;
    cand.resize(o + m);
    cc.resize(o + m);
    cs.resize(o + m);
    cn.resize(o + m);
    HIP_TRY(hipMemcpy(&cand[o], b.d_cand + seg, sizeof(int) * m, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(&cc[o], b.d_ccount + seg, sizeof(int) * m, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(&cs[o], b.d_cstd + seg, sizeof(double) * m, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(&cn[o], b.d_cnorm + seg, sizeof(double) * m, hipMemcpyDeviceToHost));
  }
  int cmax = 0;
  for (int v : cc) cmax = std::max(cmax, v);
  int64_t k = 0;
  for (size_t i = 0; i < cand.size(); ++i) {
    if (cc[i] != cmax || cmax == 0) continue;
    if (out && k < cap) {
      rs_f8_candidate &o = out[k];
      o.index = cand[i];
      o.count = cc[i];
      o.std_d = cs[i];
      o.norm_d = cn[i];
      for (int q = 0; q < 9; ++q)
        HIP_TRY(hipMemcpy(&o.F[q], b.d_F + q * p->ld + cand[i], sizeof(double),
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
  HIP_TRY(hipMemcpy(counts, p->last().d_counts, sizeof(int) * H, hipMemcpyDeviceToHost));
  return RS_OK;
}

extern "C" int rs_f8_plan_models(rs_f8_plan *p, double *F_out, int64_t H) {
  if (!p || !F_out) return fail(RS_EINVAL, "null pointer");
  int st = plan_wait(p);
  if (st) return st;
  if (H > p->last_H) return fail(RS_EINVAL, "H exceeds the last run");
  std::vector<double> soa(static_cast<size_t>(9 * H));
  for (int k = 0; k < 9; ++k)
    HIP_TRY(hipMemcpy(soa.data() + k * H, p->last().d_F + k * p->ld, sizeof(double) * H,
                      hipMemcpyDeviceToHost));
  for (int64_t h = 0; h < H; ++h)
    for (int k = 0; k < 9; ++k) F_out[h * 9 + k] = soa[k * H + h];
  return RS_OK;
}

extern "C" int rs_f8_plan_kernel_avg(rs_f8_plan *p, int64_t last_n, double *score_ms,
                                     double *solve_ms, double *total_ms) {
  if (!p) return fail(RS_EINVAL, "null plan");
  int st = plan_wait(p);
  if (st) return st;
  if (p->timing < 1) return fail(RS_EINVAL, "timing events are disabled (RSAMD_TIMING=0)");
  const int64_t k = std::max<int64_t>(
      1, std::min<int64_t>({last_n, p->runs, static_cast<int64_t>(rs_f8_plan::kEvRing)}));
  double sa = 0, sb = 0, sc = 0;
  int64_t nt = 0;
  for (int64_t r = p->runs - k; r < p->runs; ++r) {
    if (!p->timed[r % rs_f8_plan::kEvRing]) continue;
    ++nt;
    hipEvent_t *ev = p->ring[r % rs_f8_plan::kEvRing];
    float a = 0, b = 0, t = 0;
    HIP_TRY(hipEventElapsedTime(&b, ev[0], ev[1]));  // counting kernel
    if (p->timing >= 2) {
      HIP_TRY(hipEventElapsedTime(&a, ev[2], ev[3]));  // previous tail + this solve
      HIP_TRY(hipEventElapsedTime(&t, ev[2], ev[1]));  // tail+solve start .. count end
    }
    sa += a;
    sb += b;
    sc += t;
  }
  if (nt == 0) return fail(RS_EINVAL, "no timed run among the requested ones");
  // the solve / whole-run times need timing level 2; reported as -1 otherwise
  if (solve_ms) *solve_ms = p->timing >= 2 ? sa / nt : -1.0;
  if (score_ms) *score_ms = sb / nt;
  if (total_ms) *total_ms = p->timing >= 2 ? sc / nt : -1.0;
  return RS_OK;
}

extern "C" int rs_f8_plan_set_count_precision(rs_f8_plan *p, int32_t fp64) {
  if (!p) return fail(RS_EINVAL, "null plan");
  int st = plan_flush(p);  // runs in flight use the current kernel's buffers
  if (st) return st;
  p->use_fp32 = fp64 == 0;
  return RS_OK;
}

extern "C" int rs_f8_plan_set_timing(rs_f8_plan *p, int32_t level, int32_t every) {
  if (!p) return fail(RS_EINVAL, "null plan");
  if (level < 0 || level > 2 || every < 1) return fail(RS_EINVAL, "bad timing level / period");
  p->timing = level;
  p->timing_every = every;
  return RS_OK;
}

extern "C" int rs_f8_plan_kernel_ms(rs_f8_plan *p, double *score_ms, double *solve_ms,
                                    double *total_ms) {
  return rs_f8_plan_kernel_avg(p, 1, score_ms, solve_ms, total_ms);
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
  if (c->np_plan && c->np_plan->max_hyp < H) {
    rs_f8_plan_destroy(c->np_plan);
    c->np_plan = nullptr;
  }
  int st;
  if (!c->np_plan && (st = rs_f8_plan_create(c, n, H, &c->np_plan))) return st;
  // another pair's population: the same plan, its per-point buffers grown if need be
  if (c->np_plan->n != n && (st = plan_retarget(c->np_plan, n))) {
    // a failed reallocation leaves the per-point buffers freed: drop the plan, so that the next
    // call builds a fresh one instead of running on null buffers
    rs_f8_plan_destroy(c->np_plan);
    c->np_plan = nullptr;
    return st;
  }
  if ((st = rs_f8_plan_set_points(c->np_plan, p1, p2))) return st;
  uint32_t key[RS_MT_N];
  int32_t pos = *mt_pos;
  std::memcpy(key, mt_key, sizeof(key));
  if ((st = rs_f8_plan_run_np(c->np_plan, H, key, &pos, thresh))) return st;
  if ((st = rs_f8_plan_result(c->np_plan, out, inliers, cap, n_inliers))) return st;
  std::memcpy(mt_key, key, sizeof(key));
  *mt_pos = pos;
  return RS_OK;
}
