// Launch interface of the RANSAC-F / PnP kernels (host side).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define RSD_SAMPLER_PHILOX 0
#define RSD_SAMPLER_TUPLES 1

namespace rsd {

struct Pt;

// Grid of the selection passes; the status buffer holds 4 words + kSelectBlocks counts.
constexpr int kSelectBlocks = 256;
constexpr int kStatusWords = 4 + kSelectBlocks;

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
  int64_t pad_;
  int64_t inliers[];
};

hipError_t launch_pack_points(const double *p1, const double *p2, int n, Pt *pts,
                              hipStream_t s);
hipError_t launch_f8_solve(const Pt *pts, int n, int H, int mode, uint64_t seed,
                           uint64_t hyp_offset, const int *tuples, double *Fsoa, int64_t ld,
                           int *counts, int *status, hipStream_t s);
hipError_t launch_f8_count(const Pt *pts, int n, int H, const double *Fsoa, int64_t ld,
                           int chunk, double thr2, int *counts, hipStream_t s);
hipError_t launch_f8_select(const int *counts, int H, int slack, int *cand, int *status,
                            hipStream_t s);
hipError_t launch_f8_stats(const Pt *pts, int n, const double *Fsoa, int64_t ld,
                           const int *cand, const int *status, double thresh, int *ccount,
                           double *cstd, double *cnorm, int grid, hipStream_t s);
hipError_t launch_f8_replay(const int *cand, const int *status, const int *counts,
                            const int *ccount, const double *cstd, const double *cnorm,
                            const double *Fsoa, int64_t ld, F8DevResult *res, hipStream_t s);
hipError_t launch_f8_inliers(const Pt *pts, int n, double thresh, F8DevResult *res,
                             hipStream_t s);
hipError_t launch_residuals(const Pt *pts, int n, const double *F, double *out, hipStream_t s);

}  // namespace rsd
