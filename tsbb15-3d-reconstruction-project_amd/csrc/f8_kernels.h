// Launch interface of the RANSAC-F / PnP kernels (host side).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "device_math.h"

#define RSD_SAMPLER_PHILOX 0
#define RSD_SAMPLER_TUPLES 1

namespace rsd {


// Grid of the selection passes; the status buffer holds 4 words + kSelectBlocks counts.
constexpr int kSelectBlocks = 256;
constexpr int kStatusWords = 4 + kSelectBlocks;
constexpr int kTailThreads = 512;  // workgroup of the fused tail + solve launch

// Device-resident result of one F run; copied back to the host in one transfer together
// with the first n_inliers entries of `inliers`.
struct F8DevResult {
  double F[9];
  int64_t best_index;
  int64_t best_count;
  double best_std;
  double best_norm;
  int64_t max_count_fast;
  int64_t n_candidates;
  int64_t guard_mismatch;
  int64_t n_inliers;
  int64_t best_cand;
  int64_t inl_row;  // -1: S_RANSAC in inliers[]; else the select block whose spec row holds it

  int64_t inliers[];
};

// One run's solve (k_f8_solve / the solve half of k_f8_tail_solve).
struct SolveArgs {
  const Pt *pts;
  int n, H, mode;
  uint64_t seed, hyp_offset;
  const int *tuples;
  double *Fsoa;
  int64_t ld;
  int *counts;   // zeroed per hypothesis
  int *status;   // status words 0..3 zeroed
  float *F32soa; // unit-frame fp32 models (null: fp64 counting)
  Frame frame;
  int *gdone;    // per-group finish counters zeroed (fused c*)
  float4 *G4;    // per-hypothesis decision constants (k_f8_count32q), may be null
  double gT, gDe, gDn;  // their inputs: (t/s)^2 and the fp32 error bounds of e and m
};

// One run's selection tail (candidates, reference statistics, replay, S_RANSAC).
struct TailArgs {
  const Pt *pts;
  int n, H, slack, per_block;
  const double *Fsoa;
  int64_t ld;
  const int *counts;
  int *status;   // [c*, n_candidates, done counter, spare, per-block candidate counts]
  double thresh;
  int *cand, *ccount;
  int *cfast;          // fast count of each candidate (guard_mismatch without a gather)
  int *spec, *spec_j;  // per block: S_RANSAC of its first candidate (n ints), that index
  int nospec;          // RSAMD_NOSPEC=1: no speculative lists (the replay extracts S_RANSAC)
  double *cstd, *cnorm;
  F8DevResult *res;   // HBM result (header + S_RANSAC)
  F8DevResult *hres;  // pinned host header slot (device mapping), may be null
  int *hinl;          // pinned host S_RANSAC (int32, device mapping), may be null
};

hipError_t launch_pack_points(const double *p1, const double *p2, int n, Pt *pts,
                              hipStream_t s);
hipError_t launch_f8_solve(const Pt *pts, int n, int H, int mode, uint64_t seed,
                           uint64_t hyp_offset, const int *tuples, double *Fsoa, int64_t ld,
                           int *counts, int *status, hipStream_t s, float *F32soa = nullptr,
                           const Frame *frame = nullptr, int *gdone = nullptr);
// Point-pair packed fp32 counting (guard band + float64 re-test: counts bit-identical to
// launch_f8_count); ptsq in the k_pack_points32q layout.
hipError_t set_count_timeline(uint64_t *buf);  // RSAMD_TSTAMP diagnostics (null: off)
// words per wave of that timeline: real-time start / end, re-tests, HW_ID | XCC_ID,
// shader-clock start / end
constexpr int kCountTsWords = 6;
hipError_t launch_pack_points32q(const Pt *pts, int n, const Frame &fr, float4 *ptsq,
                                 hipStream_t s);
struct Count32qShape {
  int64_t per_wave;  // points of the (group, point) plane per wave (a multiple of 8)
  int64_t blocks;    // 256-thread workgroups launched
};
int count32q_resident_waves(int device);
// fp32 counting set-up (host): guard bounds of the unit frame, and the frame of the points
struct Bounds {
  double u, De, Dn, thr2;
};
Bounds fp32_bounds(const Frame &fr, double thresh);
bool unit_frame(const double *p1, const double *p2, int64_t n, Frame &fr);
Count32qShape count32q_shape(int n, int H, int waves, int slices_per_wave = 0);
hipError_t preload_f8();  // the F-RANSAC kernels' code object onto the current device
// pts (and with fr the point-pair layout ptsq) from the (2, n) arrays in one launch
hipError_t launch_pack_points_both(const double *p1, const double *p2, int n, Pt *pts,
                                   const Frame *fr, float4 *ptsq, hipStream_t s);
hipError_t launch_f8_count32q(const float4 *ptsq, const Pt *pts, int n, int H,
                              const float *F32soa, const double *Fsoa, int64_t ld,
                              const Count32qShape &sh, const GuardW &g, int *counts,
                              hipStream_t s, int *gdone, int *status, const float4 *G4,
                              const int *Hdev = nullptr);
hipError_t launch_f8_count(const Pt *pts, int n, int H, const double *Fsoa, int64_t ld,
                           int chunk, double thr2, int *counts, hipStream_t s,
                           const int *Hdev = nullptr, const int *Hmap = nullptr);
// Selection tail: c* (k_f8_max, unless the counting kernel fused it), candidates + reference
// statistics + (last block) replay and S_RANSAC.  Candidates live in per-block segments of
// `cand`.
int select_per_block(int H);
int select_blocks(int H);
hipError_t launch_f8_max(const int *counts, int H, int *status, hipStream_t s);
// Tail of one run and/or solve of the next in one launch (either may be null).
hipError_t launch_f8_tail_solve(TailArgs *ta, SolveArgs *sa, hipStream_t s,
                                int tail_cus = 0);
hipError_t launch_residuals(const Pt *pts, int n, const double *F, double *out, hipStream_t s);

}  // namespace rsd
