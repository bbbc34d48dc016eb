// Context object behind the opaque rs_ctx handle.
#pragma once

#include <hip/hip_runtime.h>

#include "rsamd.h"

struct rs_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  void *scratch = nullptr;     // grow-only device scratch for single-shot ops
  size_t scratch_bytes = 0;
  rs_f8_plan *np_plan = nullptr;  // cached plan of rs_f8_ransac_np
  void *comm = nullptr;        // ncclComm_t
  void *comm_buf = nullptr;    // device staging for collectives
  size_t comm_buf_bytes = 0;
};

namespace rs {
int hip_fail(hipError_t e, const char *what);
int ensure_scratch(rs_ctx *c, size_t bytes);
int fmatrix_stls_lsq(rs_ctx *c, const double *pl, const double *pr, int64_t n, double *F_out);
}  // namespace rs
