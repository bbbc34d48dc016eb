// Context object behind the opaque rs_ctx handle.
#pragma once

#include <hip/hip_runtime.h>

#include "rsamd.h"


struct rs_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  // the parity parse's second stream (the second MT stream pass beside the entry kernel), one per
  // context, created with it: independent contexts never wait for each other's parse work
  hipStream_t aux_stream = nullptr;
  void *scratch = nullptr;     // grow-only device scratch for single-shot ops
  size_t scratch_bytes = 0;
  void *pinned = nullptr;      // grow-only pinned host staging of single-shot inputs (one DMA
  size_t pinned_bytes = 0;     // copy instead of several pageable ones; the ops synchronise)
  rs_f8_plan *np_plan = nullptr;  // cached plan of rs_f8_ransac_np
  rs_np_shard *np_shard = nullptr;  // world-1 parity-stream session (np_choice_device)
  void *comm = nullptr;        // ncclComm_t
  void *comm_buf = nullptr;    // device staging for collectives
  size_t comm_buf_bytes = 0;
  // rs_pnp_timing: HIP events around the PnP-RANSAC solve and count kernels of the next calls
  int pnp_timing = 0;
  hipEvent_t pnp_ev[3] = {};
  double pnp_solve_ms = -1.0, pnp_count_ms = -1.0;
  // rs_np_timing: HIP events between the parity-stream parse's steps (np_sampler.hip), the
  // last np_choice_device call's sums over its segments (RS_NP_TIMING_SLOTS ms, 3 byte counts)
  int np_timing = 0;
  double np_ms[RS_NP_TIMING_SLOTS] = {};
  double np_bytes[3] = {};
  int64_t np_segments = 0;
};

namespace rs {
int hip_fail(hipError_t e, const char *what);
int ensure_scratch(rs_ctx *c, size_t bytes);
int ensure_pinned(rs_ctx *c, size_t bytes);
void np_shard_free(rs_ctx *c);
int np_preload();  // the parse kernels' code object onto the current device (rs_ctx_create)
bool np_gpu_supported(int64_t n, int32_t k);  // within the GPU parse's population range
// The numpy (py: CPython) stream's next `count` choice(n, k) tuples; rows [skip, skip + take)
// (take < 0: to the end) are written to d_out (take * k int32); (key, pos) advance past all
// `count`.  Synchronous on the context stream.
int np_choice_enqueue(rs_ctx *c, const uint32_t *key, int32_t pos, int64_t n, int32_t k,
                      int64_t count, int32_t *d_out, bool *queued);
int np_choice_finish(rs_ctx *c, uint32_t *key, int32_t *pos, bool *rerun);
int np_choice_device(rs_ctx *c, uint32_t *key, int32_t *pos, int64_t n, int32_t k,
                     int64_t count, int32_t *d_out, bool py = false, int64_t skip = 0,
                     int64_t take = -1);
// Step 4 of a sharded parse (np_sampler.hip, rs_np_shard_*) into device memory.
int np_shard_tuples_device(rs_np_shard *w, int64_t base, int64_t hi, int64_t next_start,
                           int64_t final_idx, int32_t *d_out, uint32_t *key_out, int32_t *pos_out);
// The batched pair RANSAC (pairs.hip) enqueued without its download; the records (rs_pair_result
// layout), inlier lists and points stay on the device for the stages after it.
struct PairsDev {
  const void *pts;       // rsd::Pt per point (x1, y1, x2, y2), pair b at off[b]
  const int64_t *off;    // B + 1 offsets
  void *res;             // B records (rs_pair_result)
  int32_t *inl;          // S_RANSAC of pair b at inl[off[b] ..]
  int64_t total;         // off[B]
  char *extra;           // the caller's `extra` bytes of scratch (256-aligned)
};
int pairs_enqueue(rs_ctx *c, const double *p1, const double *p2, const int64_t *off, int64_t B,
                  int64_t H, int32_t mode, uint64_t seed_base, const int64_t *seed_ids,
                  const int32_t *host_tuples, double thresh, size_t extra, PairsDev *d);
int fmatrix_stls_lsq(rs_ctx *c, const double *pl, const double *pr, int64_t n, double *F_out);
}  // namespace rs
