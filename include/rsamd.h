/*
 * rsamd.h -- C ABI of the MI355X-native RANSAC-F / PnP hot path.
 *
 * Drop-in boundary for bioengstrom/tsbb15-3d-reconstruction-project (snapshot v0).  The
 * reference has no FFI: its boundary is the Python module surface.  Each
 * entry point below names the reference function it replaces; the Python shims in
 * tsbb15_amd/ (lab3.py, fun.py, ransac.py, pnp.py, cv.py) bind these through ctypes with the
 * reference's names, argument meaning and ValueError behaviour.
 *
 * Conventions
 *   - every function returns int status: RS_OK (0) or a negative RS_E* code; the message of
 *     the last failure on the calling thread is rs_last_error();
 *   - host pointers are caller-owned; the library never frees or keeps them;
 *   - point sets are row-major (2, n) float64 arrays: row 0 = x (column), row 1 = y (row);
 *   - a context owns one HIP device, one HIP stream and its device buffers; calls on one
 *     context are synchronous (except the *_plan_run launches, which are stream-ordered and
 *     completed by *_plan_result) and must not be issued concurrently from two threads.
 */
#ifndef RSAMD_H
#define RSAMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RS_OK 0
#define RS_EINVAL (-1)   /* shape / argument error  -> ValueError   */
#define RS_EDEVICE (-2)  /* HIP runtime failure     -> RuntimeError */
#define RS_ENODEV (-3)   /* no GPU visible          -> RuntimeError */
#define RS_ECOMM (-4)    /* RCCL failure            -> RuntimeError */
#define RS_ENOMEM (-5)   /* allocation failure      -> MemoryError  */

#define RS_MT_N 624      /* MT19937 state words */

const char *rs_last_error(void);
int rs_version(void);

/* ------------------------------------------------------------------------------------------
 * Host samplers (no device).  Bit-exact replays of the reference's random streams.
 * ---------------------------------------------------------------------------------------- */

/* numpy legacy RandomState: init_genrand(seed) -> key[624], pos = 624 (np.random.seed). */
int rs_np_seed(uint32_t seed, uint32_t *mt_key, int32_t *mt_pos);

/* `count` draws of np.random.choice(np.arange(n), k, replace=False) (fun.py:305-306), i.e.
 * permutation(n)[:k] by Fisher-Yates with masked-rejection random_interval.  Advances the
 * (key, pos) state in place exactly as numpy does.  out: (count, k) int32. */
int rs_np_choice_tuples(uint32_t *mt_key, int32_t *mt_pos, int64_t n, int32_t k, int64_t count,
                        int32_t *out);

/* B independent numpy streams at once on host threads (config C4: one stream per image pair,
 * np.random.seed(1000 + pair), then `count` x choice(n_b, k, replace=False)): mt_keys (B, 624),
 * mt_pos (B) advanced in place (with seeds non-null they are first set to np.random.seed(
 * seeds[b])), out (B, count, k).  Streams with n_b < k are skipped (zero output, state
 * unchanged).  threads <= 0: one per hardware thread, at most 16 (threads > 0: at most 64). */
int rs_np_choice_tuples_multi(int64_t B, const uint32_t *seeds, uint32_t *mt_keys,
                              int32_t *mt_pos, const int64_t *ns, int32_t k, int64_t count,
                              int32_t *out, int32_t threads);

/* CPython random.seed(int) with the int given as 32-bit little-endian words
 * (init_by_array) -> key[624], pos = 624. */
int rs_py_seed(const uint32_t *words, int32_t n_words, uint32_t *mt_key, int32_t *mt_pos);

/* `count` draws of ransac.gen_rnd_indices(n, k) (ransac.py:12-19): random.shuffle(
 * list(range(n)))[:k] with CPython's getrandbits rejection.  out: (count, k) int32. */
int rs_py_shuffle_tuples(uint32_t *mt_key, int32_t *mt_pos, int64_t n, int32_t k, int64_t count,
                         int32_t *out);

/* MT19937 jump-ahead: the (key, pos) state after `steps` more 32-bit outputs, computed as
 * x^J mod phi applied to the state (phi: the generator's characteristic polynomial), without
 * generating the words.  Same representation as np.random.get_state() / random.getstate():
 * key is the raw block holding the next word.  Replaces nothing in the reference; it is the
 * building block for starting many generators along one np.random / random stream. */
int rs_mt_jump(const uint32_t *mt_key, int32_t mt_pos, int64_t steps, uint32_t *key_out,
               int32_t *pos_out);

/* Self-test of the GF(2)[x] product mod phi behind the parity parse's radix-8 jump tree (level
 * polynomials x^(m 8^k J) as products, np_sampler.hip jump_polys_r): 1 iff
 * x^j1 * x^j2 mod phi == x^(j1 + j2) mod phi, 0 if not, RS_EINVAL for a negative exponent.
 * Host only; exported for the CPU test suite. */
int rs_mt_poly_selftest(int64_t j1, int64_t j2);

/* ------------------------------------------------------------------------------------------
 * Context: one per host thread; owns the device buffers, stream and RCCL communicator
 * ---------------------------------------------------------------------------------------- */
typedef struct rs_ctx rs_ctx;

int rs_device_count(int *n);
int rs_ctx_create(int device, rs_ctx **out);
int rs_ctx_destroy(rs_ctx *ctx);
int rs_ctx_synchronize(rs_ctx *ctx);

/* The same stream as rs_np_choice_tuples (k <= 8, n - 1 <= 10240), computed on the GPU of
 * `ctx`: MT19937 jump-ahead windows, the word stream in HBM, a chunked parse from every entry
 * state (hypothesis boundaries), then one lane per hypothesis for its k indices.  Same output
 * and (key, pos) advance, bit for bit; out is host memory (count, k) int32.
 * Replaces the serial host replay behind fun.py:305-306 in parity mode. */
int rs_np_choice_tuples_gpu(rs_ctx *ctx, uint32_t *mt_key, int32_t *mt_pos, int64_t n, int32_t k,
                            int64_t count, int32_t *out);

/* The same stream as rs_py_shuffle_tuples (ransac.gen_rnd_indices, ransac.py:12-19: CPython
 * random.shuffle with getrandbits rejection), k <= 8, n - 1 <= 10240, computed on the GPU by
 * the same pipeline with CPython's draw rule (w >> (32 - bit_length(i + 1)) <= i).  Same
 * output and (key, pos) advance, bit for bit; out is host memory (count, k) int32. */
int rs_py_shuffle_tuples_gpu(rs_ctx *ctx, uint32_t *mt_key, int32_t *mt_pos, int64_t n,
                             int32_t k, int64_t count, int32_t *out);

/* Sharded parity stream ("the host sampler must emit tuples in stream order
 * and hand each GPU its slice; that serial step is the scaling limiter").  The numpy (py = 0)
 * or CPython (py = 1) stream of fun.py:305-306 / ransac.py:12-19 is cut into world x Cr
 * chunks; rank r parses only its own chunks, and the ranks exchange two small records:
 *   rs_np_shard_parse    rank-local: jump to the rank's first word, generate its words, parse
 *                        its chunks from every entry state.  layout[6] = {hypotheses this
 *                        segment covers at most, C, Cr, Wc, draws, map blob bytes};
 *   rs_np_shard_maps     the rank's chunk maps as a blob                -> all-gather;
 *   rs_np_shard_compose  all ranks' blobs (rank order, `stride` bytes apart): the true entry
 *                        state of every chunk, then the rank's hypothesis starts: their number
 *                        and the first (segment draw index)          -> all-gather;
 *   rs_np_shard_tuples   the rank's hypotheses [base, hi) (global indices; base = starts of
 *                        lower ranks) as (hi - base, k) int32 rows, given the next rank's
 *                        first start; final_idx >= 0 on the rank holding start `got`: the
 *                        (key, pos) after the segment's `got` hypotheses (key_out untouched
 *                        when the state stays in the caller's block).
 * tsbb15_amd.parallel.np_sharded_segments runs the exchange; world 1 reproduces
 * rs_np_choice_tuples_gpu bit for bit. */
/* Host milliseconds this process has spent building MT19937 jump polynomials for the GPU parse
 * (once per new generator length; mt_jump.cpp's carry-less products), and the level sets built.
 * No reference counterpart: it accounts for the first-call cost of getFFromLabCode (fun.py:291). */
int rs_np_host_stats(double *jump_ms, int64_t *builds);

/* Step split of the GPU parse of the numpy stream (the sampling of fun.py:305-306): enable = 1
 * records HIP events between the steps of the following world-1 parses on this context (each
 * event is a marker between two kernels: a few microseconds each, so not in timed headline
 * runs).  Returns the last parse call's milliseconds summed over its segments, ms_out[10]:
 * 0 jump (MT windows), 1 first stream pass, 2 entry parse (with its resume launch, which waits
 * for the second pass), 3 tracking, 4 compose, 5 filter / scan / starts, 6 tuples, 7 result
 * copy, 8 the second stream pass (on the second stream, beside the entry parse), 9 the parse
 * from first to last mark; bytes_out[3]: algorithmic HBM bytes -- stream words written, chunk
 * draws read by the parse, hypothesis draws read by the tuple kernel; *segments. */
#define RS_NP_TIMING_SLOTS 10
int rs_np_timing(rs_ctx *ctx, int32_t enable, double *ms_out, double *bytes_out,
                 int64_t *segments);

typedef struct rs_np_shard rs_np_shard;
int rs_np_shard_create(rs_ctx *ctx, int64_t n, int32_t k, int32_t world, int32_t rank, int32_t py,
                       rs_np_shard **out);
int rs_np_shard_destroy(rs_np_shard *shard);
int rs_np_shard_parse(rs_np_shard *shard, const uint32_t *mt_key, int32_t mt_pos, int64_t count,
                      int64_t *layout);
int rs_np_shard_maps(rs_np_shard *shard, uint8_t *out, int64_t cap, int64_t *nbytes);
int rs_np_shard_compose(rs_np_shard *shard, const uint8_t *blobs, int64_t stride, int64_t *nstarts,
                        int64_t *first_start);
int rs_np_shard_tuples(rs_np_shard *shard, int64_t base, int64_t hi, int64_t next_start,
                       int64_t final_idx, int32_t *out, uint32_t *key_out, int32_t *pos_out);

/* ------------------------------------------------------------------------------------------
 * lab3 primitives on the GPU
 * ---------------------------------------------------------------------------------------- */

/* lab3.fmatrix_stls(pl, pr) (lab3.py:269-329): pl, pr (2, n), n >= 8; F_out (3,3) row-major,
 * pl^T F pr = 0.  n == 8 uses the batched minimal kernel, n > 8 the least-squares kernel. */
int rs_fmatrix_stls(rs_ctx *ctx, const double *pl, const double *pr, int64_t n, double *F_out);

/* Batched minimal solves: tuples (count, 8) index (2, n) point sets; F_out (count, 9). */
int rs_fmatrix_stls_batch(rs_ctx *ctx, const double *pl, const double *pr, int64_t n,
                          const int32_t *tuples, int64_t count, double *F_out);

/* lab3.fmatrix_residuals(F, x, y) (lab3.py:188-227): res_out (2, n). */
int rs_fmatrix_residuals(rs_ctx *ctx, const double *F, const double *x, const double *y,
                         int64_t n, double *res_out);

/* ------------------------------------------------------------------------------------------
 * RANSAC-F (fun.getFFromLabCode hypothesis loop, fun.py:298-328)
 * ---------------------------------------------------------------------------------------- */
#define RS_SAMPLER_PHILOX 0   /* throughput mode: counter-based Philox4x32-10 + Floyd   */
#define RS_SAMPLER_TUPLES 1   /* parity mode: host tuples (rs_np_choice_tuples stream)  */

typedef struct rs_f8_result {
  double F[9];            /* F_RANSAC, row-major (fun.py:322)                          */
  int64_t best_index;     /* hypothesis index within the run, -1 if none               */
  int64_t best_count;     /* len(S_RANSAC)                                             */
  double best_std;        /* d_RANSAC = np.std(d) of the winner (fun.py:323)           */
  double best_norm;       /* np.linalg.norm(d) of the winner                           */
  int64_t max_count_fast; /* c* of the counting kernel                                 */
  int64_t n_candidates;   /* hypotheses re-scored in float64 reference order           */
  int64_t guard_mismatch; /* candidates whose re-scored count differs from the fast one */
} rs_f8_result;

typedef struct rs_f8_candidate {
  int64_t index;          /* hypothesis index (run-local + hyp_offset)                 */
  int64_t count;          /* reference-order inlier count                              */
  double std_d;           /* np.std(d)                                                 */
  double norm_d;          /* np.linalg.norm(d)                                         */
  double F[9];
} rs_f8_candidate;

typedef struct rs_f8_plan rs_f8_plan;

/* A plan holds one correspondence set (n points) resident in HBM plus buffers for up to
 * max_hyp hypotheses per run. */
int rs_f8_plan_create(rs_ctx *ctx, int64_t n, int64_t max_hyp, rs_f8_plan **out);
int rs_f8_plan_destroy(rs_f8_plan *plan);
/* H2D upload of p1, p2 (2, n) row-major float64. */
int rs_f8_plan_set_points(rs_f8_plan *plan, const double *p1, const double *p2);
/* Enqueue one RANSAC run of H hypotheses: sample (mode), solve, count, select, re-score,
 * replay the fun.py:320-328 rule, extract inliers.  Philox mode draws hypothesis i from
 * counter (seed, hyp_offset + i); tuple mode reads host_tuples (H, 8) int32. */
int rs_f8_plan_run(rs_f8_plan *plan, int64_t H, int32_t mode, uint64_t seed, uint64_t hyp_offset,
                   const int32_t *host_tuples, double thresh);
/* Parity-mode run: the next H tuples of the numpy legacy stream (key, pos) -- the
 * rs_np_choice_tuples stream, fun.py:305-306 -- sampled on the GPU (np_sampler.hip) straight
 * into the run's tuple buffer, then the same pipeline as rs_f8_plan_run.  Advances
 * (key, pos) in place.  Populations beyond the GPU parse (n - 1 > 10240) use the host replay. */
int rs_f8_plan_run_np(rs_f8_plan *plan, int64_t H, uint32_t *mt_key, int32_t *mt_pos,
                      double thresh);
/* Hypotheses [start, start + count) of that H-hypothesis parity run (one rank's shard of the
 * fun.py:303-328 loop): the stream of all H hypotheses is parsed on the GPU,
 * only the slice's tuples are produced and evaluated (candidate indices are local; add start),
 * and (key, pos) advance past all H, exactly as rs_f8_plan_run_np. */
int rs_f8_plan_run_np_slice(rs_f8_plan *plan, int64_t H, int64_t start, int64_t count,
                            uint32_t *mt_key, int32_t *mt_pos, double thresh);
/* Parity mode, sharded: this rank's hypotheses [base, hi) of a sharded parse (rs_np_shard_*
 * after compose) produced straight into the run's tuple buffer, then the same pipeline as
 * rs_f8_plan_run (candidate indices are run-local: add base).  hi == base runs nothing and
 * only reads the final state (final_idx >= 0). */
int rs_f8_plan_run_np_shard(rs_f8_plan *plan, rs_np_shard *shard, int64_t base, int64_t hi,
                            int64_t next_start, int64_t final_idx, uint32_t *key_out,
                            int32_t *pos_out, double thresh);
/* Wait for the last run and copy its result; inliers (S_RANSAC, ascending) up to cap. */
int rs_f8_plan_result(rs_f8_plan *plan, rs_f8_result *out, int64_t *inliers, int64_t cap,
                      int64_t *n_inliers);
/* Candidates (count == max re-scored count) of the last run, ascending index, up to cap. */
int rs_f8_plan_candidates(rs_f8_plan *plan, rs_f8_candidate *out, int64_t cap, int64_t *n_out);
/* Per-hypothesis fast counts / models of the last run (test & diagnostics). */
/* Counting precision of later runs: fp64 != 0 selects the plain float64 counting kernel
 * (reference-order residuals, no fp32 filter); 0 (default) the fp32 kernel with its exact
 * float64 guard band.  Both give bit-identical counts; fp64 is the slower reference form. */
int rs_f8_plan_set_count_precision(rs_f8_plan *plan, int32_t fp64);
int rs_f8_plan_counts(rs_f8_plan *plan, int32_t *counts, int64_t H);
int rs_f8_plan_models(rs_f8_plan *plan, double *F_out, int64_t H);
/* Device time (ms, HIP events on the plan's stream) of the counting kernel, the solve kernel
 * and the whole run: of the last run, or averaged over the last `last_n` runs (<= 64).  Runs
 * may be issued back to back (each owns a result slot in pinned host memory: the header and
 * S_RANSAC, written by the run's last kernel); rs_f8_plan_result waits for the last. */
int rs_f8_plan_kernel_ms(rs_f8_plan *plan, double *score_ms, double *solve_ms, double *total_ms);
/* Timing events recorded by rs_f8_plan_run (each is a marker packet between two kernels,
 * ~3.5 us on MI355X): level 0 none, 1 around the counting kernel (default), 2 also around the
 * solve and the whole run (solve_ms / total_ms are -1 below level 2); `every` = record them on
 * every k-th run only (kernel_avg averages the timed runs among the last `last_n`). */
int rs_f8_plan_set_timing(rs_f8_plan *plan, int32_t level, int32_t every);
int rs_f8_plan_kernel_avg(rs_f8_plan *plan, int64_t last_n, double *score_ms, double *solve_ms,
                          double *total_ms);

/* One call: numpy-exact sampling (advancing mt_key/mt_pos in place) + GPU evaluation. */
int rs_f8_ransac_np(rs_ctx *ctx, const double *p1, const double *p2, int64_t n, int64_t H,
                    uint32_t *mt_key, int32_t *mt_pos, double thresh, rs_f8_result *out,
                    int64_t *inliers, int64_t cap, int64_t *n_inliers);

/* ------------------------------------------------------------------------------------------
 * PnP (pnp.py:132-160 DLT; ransac.py:37-113 consensus semantics)
 * ---------------------------------------------------------------------------------------- */
typedef struct rs_pnp_result {
  double R[9];
  double t[3];
  int64_t best_index;
  int64_t best_count;     /* D_med consensus size (ransac.py:104,108)                  */
} rs_pnp_result;

/* DLT pose from m >= 6 correspondences: X (m,3) world points, y (m,3) C-normalised
 * homogeneous image points (pnp.py:132-160).  R_out (3,3), t_out (3). */
int rs_pnp_dlt(rs_ctx *ctx, const double *X, const double *y, int64_t m, double *R_out,
               double *t_out);

/* RANSAC over minimal samples (ransac.py:37-113).  Tuples (H, k) index the `high` set;
 * consensus e = |pi(y) - pi(R x + t)|^2 <= thresh is counted on the `med` set.  mode as for
 * F; in tuple mode host_tuples come from rs_py_shuffle_tuples.  k in [6, 16]: the DLT
 * (pnp.py:132-160).  k = 3: the reference's p3p branch (ransac.py:81-82, 91-111), Lambda
 * Twist P3P with every pose of a trial scored (best_index is the trial).  The k = 3 winner is
 * chosen in two classes: the first (trial-major, pose-minor) front-facing pose with the largest
 * count, unless the best mirrored-depth pose counts more than twice as many (kMirrorCountWins =
 * 2; then the first such mirrored pose) -- so a mirrored pose with a higher count can lose.
 * Counts are exact in the reference's arithmetic (rs_pnp_count_poses), and the call fails with
 * RS_EDEVICE if the winner's count differs from its D_med consensus size.  Replaces
 * ransac.ransac_robust's loop (ransac.py:72-111). */
/* HIP events around rs_pnp_ransac's solve and count kernels (ransac.py:93-105's work): enable = 1
 * records them in the following calls; returns the last timed call's milliseconds (-1: none). */
int rs_pnp_timing(rs_ctx *ctx, int32_t enable, double *solve_ms, double *count_ms);
int rs_pnp_ransac(rs_ctx *ctx, const double *X_med, const double *y_med, int64_t m_med,
                  const double *X_high, const double *y_high, int64_t m_high, int32_t k,
                  int64_t H, int32_t mode, uint64_t seed, const int32_t *host_tuples,
                  double thresh, rs_pnp_result *out, int64_t *inl_med, int64_t *n_inl_med,
                  int64_t *inl_high, int64_t *n_inl_high);

/* Consensus counts of H given poses (H x 12: R row-major, then t) on m correspondences X (m,3),
 * y (m,3): the scoring of ransac.py:96-105 (`thresh >= dpp_squared(y, R x + t)`) with the same
 * kernel rs_pnp_ransac counts with -- division-free, pairs within a rigorous error band of the
 * threshold re-tested in the reference's arithmetic, so every count equals the reference-order
 * count.  counts_out: H int32. */
int rs_pnp_count_poses(rs_ctx *ctx, const double *X, const double *y, int64_t m,
                       const double *poses, int64_t H, double thresh, int32_t *counts_out);

/* Minimal solvers of the OpenCV drop-ins: RS_PNP_DLT6 the reference's DLT (pnp.py:132-160) on
 * 6-point samples, RS_PNP_EPNP5 EPnP on 5-point samples (OpenCV's solvePnPRansac kernel),
 * RS_PNP_P3P Lambda-Twist P3P on 4-point samples (3 solve, the 4th chooses; OpenCV's kernel
 * for 4 correspondences and for SOLVEPNP_P3P; the reference's unfinished p3p_twist,
 * pnp.py:61-121). */
#define RS_PNP_DLT6 0
#define RS_PNP_EPNP5 1
#define RS_PNP_P3P 2

/* EPnP over all m >= 4 correspondences (method RS_PNP_EPNP5) or P3P over exactly 4
 * (RS_PNP_P3P): X (m,3), y (m,3) C-normalised homogeneous image points; R_out (3,3), t_out
 * (3), err_out = mean reprojection error in normalised units (inf: no pose).  cv.solvePnP
 * with SOLVEPNP_EPNP / SOLVEPNP_P3P (pnp.py:7-10 calls cv.solvePnP). */
int rs_pnp_minimal(rs_ctx *ctx, const double *X, const double *y, int64_t m, int32_t method,
                   double *R_out, double *t_out, double *err_out);

/* Levenberg-Marquardt refinement of a pose (R row-major 3x3, t) on the PIXEL reprojection error
 * |K pi(R x + t) - uv|^2 over m correspondences: the refinement stage of cv.solvePnP with
 * SOLVEPNP_ITERATIVE (pnp.py:7-10) and of cv.solvePnPRansac (tables.py:141-147).  One GPU
 * workgroup; left-multiplied rotation steps, Marquardt damping, only cost-lowering steps taken,
 * at most max_jac Jacobians (OpenCV's CvLevMarq: 20), stop at a relative step below FLT_EPSILON.
 * R_io / t_io are updated in place; cost_out (4 doubles, may be null): initial and final
 * 0.5 |r|^2, Jacobians evaluated, steps taken. */
int rs_pnp_refine_lm(rs_ctx *ctx, const double *X, const double *uv, int64_t m, const double *K,
                     double *R_io, double *t_io, int32_t max_jac, double *cost_out);

/* cv.solvePnPRansac drop-in (tables.py:141-145 call site): world points X (m,3), PIXEL
 * image points uv (m,2), camera matrix K (3,3 row-major, upper triangular), zero distortion.
 * Up to max_iters hypotheses (Philox samples from `seed` of the method's minimal size: EPnP
 * on 5 points as OpenCV's kernel, P3P on 4, or the DLT on 6 with the sample's world points
 * centred and RMS-scaled) are solved and counted on the GPU with OpenCV's pixel test
 * |K pi(R x + t) - uv|^2 <= reproj_err^2; OpenCV's sequential loop (a model wins with
 * goodCount > max(best, model_points - 1), then RANSACUpdateNumIters(confidence, outlier
 * ratio, model_points, niters) shrinks the budget) is replayed over that hypothesis order.
 * guess (R row-major then t, 12 doubles, or null): scored first, as hypothesis 0 (the
 * extrinsic guess of useExtrinsicGuess).  out->best_index = -1 when nothing wins;
 * *iters_used = hypotheses the loop consumed; inliers (<= m) in point order. */
int rs_pnp_ransac_cv(rs_ctx *ctx, const double *X, const double *uv, int64_t m, const double *K,
                     int64_t max_iters, uint64_t seed, double reproj_err, double confidence,
                     int32_t method, const double *guess, rs_pnp_result *out, int64_t *inliers,
                     int64_t *n_inliers, int64_t *iters_used);

/* ------------------------------------------------------------------------------------------
 * Five-point essential matrix (Nister) and E-RANSAC.  No reference counterpart (SURVEY.md 8(a)
 * row a-15, north_star "5-point E"); the reference's convention: y1^T E y2 = 0, E = R^T [t]_x
 * (fun.py:12-21), F = K1^-T E K2^-1 in pixels.
 * ---------------------------------------------------------------------------------------- */
typedef struct rs_e5_result {
  double E[9];            /* winning essential matrix (unit Frobenius norm), row-major      */
  double F[9];            /* its pixel-space F = K1^-T E K2^-1                               */
  int64_t best_sample;    /* minimal sample of the winner, -1 if none                       */
  int64_t best_solution;  /* which of that sample's real solutions (0..9)                   */
  int64_t best_count;     /* consensus size                                                 */
} rs_e5_result;

/* All real solutions of S minimal samples: y1, y2 (5 S, 3) homogeneous C-normalised points,
 * sample s = rows 5s .. 5s+4.  E_out (S, 10, 9): unit-norm solutions, NaN past nsol[s]. */
int rs_e5_solve(rs_ctx *ctx, const double *y1, const double *y2, int64_t S, double *E_out,
                int32_t *nsol);

/* E-RANSAC over S Philox 5-point samples of n pixel correspondences p1, p2 ((2, n) each, the
 * layout of fun.py:298) with cameras K1, K2: every real solution is a hypothesis, scored with
 * the reference's F-RANSAC test (lab3.fmatrix_residuals, max(|r1|, |r2|) < thresh, fun.py:
 * 315-317); among the hypotheses with the largest count the smallest ||d|| (d_i =
 * max(|r1_i|, |r2_i|) over all points, fun.py:317) wins, the first on equal norms. */
int rs_e5_ransac(rs_ctx *ctx, const double *p1, const double *p2, int64_t n, const double *K1,
                 const double *K2, int64_t S, uint64_t seed, double thresh, rs_e5_result *out,
                 int64_t *inliers, int64_t *n_inliers);

/* ------------------------------------------------------------------------------------------
 * Batched RANSAC-F over many image pairs (config C4; fun.py:298-328 per pair)
 * ---------------------------------------------------------------------------------------- */
typedef struct rs_pair_result {
  double F[9];            /* F_RANSAC of the pair (NaN if none)                          */
  int64_t best_index;     /* winning hypothesis, -1 if none (N < 8 or no consensus)      */
  int64_t best_count;     /* len(S_RANSAC)                                               */
  double best_std;        /* d_RANSAC = np.std(d)                                        */
  double best_norm;       /* np.linalg.norm(d) of the winner                             */
  int64_t n_candidates;   /* hypotheses with count == c*                                 */
} rs_pair_result;

/* H hypotheses for each of B pairs in one pass.  p1, p2: (2, total) point sets of all pairs
 * concatenated, pair b = columns off[b] .. off[b+1]-1 (off: B+1 entries, off[0] = 0).
 * Philox mode: pair b draws from seed_base + id_b with counters 0..H-1 (the stream of
 * rs_f8_plan_run(seed = seed_base + id_b)), id_b = seed_ids[b] or b when seed_ids is NULL;
 * tuple mode: host_tuples (B, H, 8) int32.  Pairs with
 * N < 8 are skipped (best_index -1).  Counts use the reference-order float64 distance.
 * out (B); inliers (total) int32: S_RANSAC of pair b at inliers[off[b] .. off[b]+count-1]. */
int rs_pairs_f8_ransac(rs_ctx *ctx, const double *p1, const double *p2, const int64_t *off,
                       int64_t B, int64_t H, int32_t mode, uint64_t seed_base,
                       const int64_t *seed_ids, const int32_t *host_tuples, double thresh,
                       rs_pair_result *out,
                       int32_t *inliers);

/* ------------------------------------------------------------------------------------------
 * Two-view geometry after RANSAC (fun.py:91-102, 209-280, 336-369; lab3.py:331-475)
 * ---------------------------------------------------------------------------------------- */

/* lab3.triangulate_optimal (lab3.py:382-475), batched.  C1, C2: (n_cam, 3, 4) camera pairs;
 * x1, x2: (2, n) point sets (row 0 = x); cam: (n) int32 pair index per point, or NULL for
 * pair 0; X_out: (n, 3). */
int rs_triangulate_optimal(rs_ctx *ctx, const double *C1, const double *C2, int64_t n_cam,
                           const double *x1, const double *x2, const int32_t *cam, int64_t n,
                           double *X_out);

/* fun.camera_resectioning (fun.py:260-280, specRQ 181-188), batched: P (B, 3, 4) ->
 * K (B, 3, 3) upper triangular with K[2,2] = 1, R (B, 3, 3) rotation, t (B, 3). */
int rs_camera_resectioning(rs_ctx *ctx, const double *P, int64_t B, double *K, double *R,
                           double *t);

/* E = K^T F K of fun.getEAndK (fun.py:101), batched: F (B, 3, 3); K (B, 3, 3), or a single
 * (3, 3) K for all when one_k != 0. */
int rs_essential_from_f(rs_ctx *ctx, const double *K, int32_t one_k, const double *F, int64_t B,
                        double *E);

/* fun.relative_camera_pose (fun.py:209-258), batched: E (B, 3, 3); y1, y2 (B, 2) the
 * C-normalised first correspondence (main.py:63).  R (B, 3, 3), t (B, 3); found (B) = 1..4,
 * the candidate taken, or 0 where the reference returns None (R, t NaN). */
int rs_relative_camera_pose(rs_ctx *ctx, const double *E, const double *y1, const double *y2,
                            int64_t B, double *R, double *t, int32_t *found);

/* lab3.fmatrix_cameras (lab3.py:353-380): F (B, 3, 3) -> C1 (B, 3, 4); C2 = [I | 0]. */
int rs_fmatrix_cameras(rs_ctx *ctx, const double *F, int64_t B, double *C1);

/* lab3.fmatrix_from_cameras (lab3.py:331-351): C1, C2 (B, 3, 4) -> F (B, 3, 3). */
int rs_fmatrix_from_cameras(rs_ctx *ctx, const double *C1, const double *C2, int64_t B,
                            double *F);

typedef struct rs_gs_info {
  double cost_init;       /* 0.5 |r|^2 at the start (cameras of F_RANSAC, optimal points)  */
  double cost;            /* 0.5 |r|^2 at the end                                          */
  int32_t iterations;     /* linearisations                                                */
  int32_t accepted;       /* accepted LM steps                                             */
  int32_t status;         /* 0 max_iter, 1 converged (ftol/xtol 1e-15), 2 no further decrease */
  int32_t n;              /* inliers of the pair                                           */
} rs_gs_info;

/* The residual of lab3.fmatrix_residuals_gs (lab3.py:228-266) at the parameter vector x
 * (12 camera entries row-major, then n points xyz; f: 4n, order left x, left y, right x,
 * right y) and, when J is non-null, the forward-difference Jacobian scipy's
 * least_squares(jac='2-point') forms (fun.py:358): the (4n, 12 + 3n) Jacobian stored
 * column-major (J[j * 4n + i] = dF_i / dx_j, scipy's Fortran-ordered J_transposed.T), column
 * j = (f(x with x_j -> xp[j]) - f(x)) / dx[j]; xp and dx are the caller's (scipy's step rule).
 * The projection copies the FMA chain of one OpenBLAS dgemm microkernel (the one
 * OpenBLAS 0.3.29 DYNAMIC_ARCH picks on the build container's SkylakeX cores,
 * tests/golden/gs_trace_blas.json), so f equals the reference's residual bit for bit where
 * numpy runs that kernel; under another BLAS kernel (another CPU type, MKL, a threaded or
 * small-matrix path) the reference's own bits differ and the equality is not guaranteed --
 * the tests then skip the bit-equality assertions.  The host-side TRF iteration of the
 * reference-faithful gold standard calls this. */
int rs_gs_residuals_fd(rs_ctx *ctx, const double *x, const double *xp, const double *dx,
                       const double *pl, const double *pr, int64_t n, double *f, double *J);

/* The gold-standard tail of fun.getFFromLabCode (fun.py:336-369), batched over pairs:
 * F (B, 3, 3) = F_RANSAC per pair; pl, pr (2, total) the inlier points of all pairs
 * concatenated, pair b = columns off[b] .. off[b+1]-1 (off has B+1 entries, off[0] = 0).
 * Minimises lab3.fmatrix_residuals_gs over (C1, X) to convergence (LM, Schur complement).
 * F_gold (B, 3, 3); optional C1_out (B, 3, 4) and X_out (total, 3); info (B). */
int rs_gold_standard(rs_ctx *ctx, const double *F, const double *pl, const double *pr,
                     const int64_t *off, int64_t B, int32_t max_iter, double *F_gold,
                     double *C1_out, double *X_out, rs_gs_info *info);

/* Config C4 end to end (run_pairs with a refiner: fun.py:298-328, 336-369 and main.py:50-63 per
 * pair) in one call: rs_pairs_f8_ransac's stages, then for every pair with a consensus
 * (best_index >= 0 and best_count > 0) rs_gold_standard (max_iter) on its S_RANSAC points,
 * and -- when K (3, 3) is given -- E = K^T F_gold K and rs_relative_camera_pose on y1[b], y2[b]
 * (B, 2), the caller's C-normalised first correspondence of each pair.  Everything between the
 * stages stays on the device (the inlier points are gathered there): one upload, one download.
 * Outputs as the three calls': out (B), inliers (total), F_gold (B, 3, 3), info (B), R (B, 3, 3),
 * t (B, 3), found (B).  Pairs without a consensus: F_gold, R, t NaN, info zero, found 0; K NULL:
 * R, t NaN and found 0 for every pair. */
int rs_pairs_two_view(rs_ctx *ctx, const double *p1, const double *p2, const int64_t *off,
                      int64_t B, int64_t H, int32_t mode, uint64_t seed_base,
                      const int64_t *seed_ids, const int32_t *host_tuples, double thresh,
                      int32_t max_iter, const double *K, const double *y1, const double *y2,
                      rs_pair_result *out, int32_t *inliers, double *F_gold, rs_gs_info *info,
                      double *R, double *t, int32_t *found);

/* ------------------------------------------------------------------------------------------
 * Per-view SfM steps around PnP (tables.py, fun.py:12-21)
 * ---------------------------------------------------------------------------------------- */

/* The 2D<->3D matching loop of Tables.addNewView (tables.py:116-135): for each query (n, 3)
 * (C-normalised homogeneous y1), the point index obs_point[k] of the FIRST observation k of
 * obs (m, 3) -- the last view's observations in observations_index order -- with
 * ||obs_k - query|| < tol, else -1.  out: (n) int64. */
int rs_match_observations(rs_ctx *ctx, const double *obs, const int64_t *obs_point, int64_t m,
                          const double *queries, int64_t n, double tol, int64_t *out);

/* fun.getEFromCameras (fun.py:12-21), batched: C1, C2 (n, 3, 4) = [R | t] -> E (n, 3, 3). */
int rs_e_from_cameras(rs_ctx *ctx, const double *C1, const double *C2, int64_t n, double *E);

/* Tables.addNewPoints (tables.py:161-175) without the table bookkeeping: C1, C2 (3, 4) the two
 * views' [R | t]; y1, y2 (n, 3) C-normalised homogeneous putative correspondences.
 * mask (n) int32 = |y1^T E y2| < gate; X (n, 3) = lab3.triangulate_optimal of the accepted
 * (NaN where rejected). */
int rs_add_new_points(rs_ctx *ctx, const double *C1, const double *C2, const double *y1,
                      const double *y2, int64_t n, double gate, int32_t *mask, double *X);

/* EpsilonBA of Tables.BundleAdjustment2 (tables.py:264-293): cams (nC, 3, 4) as 12 free
 * parameters each, pts (nP, 3), observations (obs_view, obs_point int32, uv (n, 2)).
 * r (2n) = interleaved [u - c1.x / c3.x, v - c2.x / c3.x]. */
int rs_ba_residuals(rs_ctx *ctx, const double *cams, int64_t nC, const double *pts, int64_t nP,
                    const int32_t *obs_view, const int32_t *obs_point, const double *uv,
                    int64_t n, double *r);

/* Jacobian blocks of rs_ba_residuals per observation (the nonzeros of Tables.sparsity_mask,
 * tables.py:339-372): Jc (n, 2, 12) w.r.t. the camera's row-major entries, Jp (n, 2, 3). */
int rs_ba_jacobian(rs_ctx *ctx, const double *cams, int64_t nC, const double *pts, int64_t nP,
                   const int32_t *obs_view, const int32_t *obs_point, int64_t n, double *Jc,
                   double *Jp);

/* ------------------------------------------------------------------------------------------
 * Multi-GPU (RCCL over xGMI).  One process per GPU; the unique id travels out of band.
 * ---------------------------------------------------------------------------------------- */
#define RS_COMM_ID_BYTES 128
int rs_comm_unique_id(uint8_t *id_out);
int rs_comm_init(rs_ctx *ctx, int32_t nranks, int32_t rank, const uint8_t *id);
int rs_comm_destroy(rs_ctx *ctx);
/* All-gather of `bytes` per rank (host buffers; staged through HBM). */
int rs_comm_allgather(rs_ctx *ctx, const void *send, void *recv, int64_t bytes);
/* The RCCL this process runs: version (ncclGetVersion) and the path of the shared object
 * that provides it (up to cap bytes, NUL-terminated). */
int rs_comm_library(int32_t *version, char *path, int64_t cap);
/* Max-all-reduce of one int64 (c* across hypothesis shards). */
int rs_comm_allreduce_max_i64(rs_ctx *ctx, int64_t *value);

#ifdef __cplusplus
}
#endif

#endif /* RSAMD_H */
