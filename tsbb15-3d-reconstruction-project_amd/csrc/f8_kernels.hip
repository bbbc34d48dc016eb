// RANSAC-F kernels for gfx950 (MI355X).  See DESIGN.md for the data layout and rooflines.
//
// Pipeline of one run (fun.py:298-328 unrolled into H concurrent hypotheses):
//   k_f8_solve    lane per hypothesis: sample (Philox/Floyd or host tuples) -> 8-point F
//                 (Householder LQ null vector + 3x3 Jacobi rank-2), F stored SoA in HBM
//   k_f8_count    lane per hypothesis x chunk of points: inlier count by the squared test
//                 e^2 < t^2 min(|l1|^2, |l2|^2) (points wave-uniform -> scalar loads)
//   k_f8_select   one workgroup: c* = max count, ordered list of hypotheses with count >=
//                 c* - 1 (guard slack)
//   k_f8_stats    wave per candidate: reference-order float64 d (lab3.py:210-227), count,
//                 np.std(d), np.linalg.norm(d)
//   k_f8_replay   one wave: the fun.py:320-328 rule over the ordered candidates
//   k_f8_inliers  one workgroup: S_RANSAC = flatnonzero(d < t) of the winner, in order
#include <hip/hip_runtime.h>

#include <algorithm>

#include "device_math.h"
#include "f8_kernels.h"

namespace rsd {

__device__ __forceinline__ int wave_uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

// cnt + (this lane's bit of a wave mask): one v_addc_co_u32 with the SGPR mask as carry-in.
__device__ __forceinline__ int add_lane_bit(int cnt, unsigned long long mask) {
  int r;
  unsigned long long co;
  asm("v_addc_co_u32_e64 %0, %1, 0, %2, %3" : "=v"(r), "=s"(co) : "v"(cnt), "s"(mask));
  return r;
}

// Cross-workgroup hand-off inside one launch.  Each XCD has its own L2, so an agent-scope
// fence (__threadfence) writes back / invalidates L2 -- far too slow per segment.  Instead the
// shared values travel as agent-scope atomics (coherent across XCDs), each wave waits for its
// own to complete (vmcnt) before publishing with the counter atomic, and readers use
// agent-scope atomic loads.
template <class T>
__device__ __forceinline__ void st_agent(T *p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
__device__ __forceinline__ T ld_agent(const T *p) {
  return __hip_atomic_load(const_cast<T *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void wait_vmem() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// ----------------------------------------------------------------------------------------
// One hypothesis h of a run: sample, 8-point F (float64), its unit-frame fp32 copy, and the
// per-run zeroing the counting kernel and the selection tail rely on.
__device__ __forceinline__ void solve_one(const SolveArgs &a, int h) {
  const Pt *__restrict__ pts = a.pts;
  const int n = a.n, mode = a.mode;
  const uint64_t seed = a.seed, hyp_offset = a.hyp_offset;
  const int *__restrict__ tuples = a.tuples;
  double *__restrict__ Fsoa = a.Fsoa;
  const int64_t ld = a.ld;
  int *__restrict__ counts = a.counts;
  int *__restrict__ status = a.status;
  float *__restrict__ F32soa = a.F32soa;
  const Frame fr = a.frame;
  int *__restrict__ gdone = a.gdone;
  if (counts) counts[h] = 0;  // the counting kernel accumulates into it
  if (status && h == 0) {  // c*, n_candidates, tail done-counter, spare
#pragma unroll
    for (int k = 0; k < 4; ++k) status[k] = 0;
  }
  if (gdone && (h & 63) == 0) gdone[h >> 6] = 0;  // fused c*: per-group finish counters
  int idx[8];
  if (mode == RSD_SAMPLER_PHILOX) {
    floyd_sample<8>(seed, hyp_offset + static_cast<uint64_t>(h), n, idx);
  } else {
    // parity mode may queue this solve behind a parse it has not yet checked
    // (rs_f8_plan_run_np_slice): an index outside [0, n) reads point 0, never past the points;
    // such a run is discarded and run again
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int t = tuples[static_cast<int64_t>(h) * 8 + k];
      idx[k] = static_cast<unsigned>(t) < static_cast<unsigned>(n) ? t : 0;
    }
  }
  double xl[8], yl[8], xr[8], yr[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const Pt p = pts[idx[k]];
    xl[k] = p.x1;
    yl[k] = p.y1;
    xr[k] = p.x2;
    yr[k] = p.y2;
  }
  double F[9];
  fmatrix8(xl, yl, xr, yr, F);
#pragma unroll
  for (int k = 0; k < 9; ++k) Fsoa[k * ld + h] = F[k];
  if (F32soa) f32_model(F, fr, a.gT, a.gDe, a.gDn, F32soa, a.G4, ld, h);
}

__global__ __launch_bounds__(256) void k_f8_solve(SolveArgs a) {
  const int h = blockIdx.x * blockDim.x + threadIdx.x;
  if (h < a.H) solve_one(a, h);
}

// ----------------------------------------------------------------------------------------
// Counting: unit u = (group g of 64 hypotheses, chunk c of points).  F lives in VGPRs (one
// hypothesis per lane); the point is the same for all 64 lanes, so its 32 B come through
// the scalar cache into SGPRs and feed the VALU as a free scalar operand.  21 float64 VALU
// ops per (hypothesis, point); no LDS, no cross-lane traffic.
// ----------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_f8_count(const Pt *__restrict__ pts, int n, int H,
                                                  const double *__restrict__ Fsoa, int64_t ld,
                                                  int chunk, int nchunks, double thr2,
                                                  int *__restrict__ counts,
                                                  const int *__restrict__ Hdev,
                                                  const int *__restrict__ Hmap) {
  const int lane = threadIdx.x & 63;
  const int u = wave_uniform(blockIdx.x * 4 + (threadIdx.x >> 6));
  if (Hdev) H = min(H, *Hdev);  // a count known on the device only (grid sized for the bound H)
  const int ngroups = (H + 63) >> 6;
  if (u >= ngroups * nchunks) return;
  const int g = u / nchunks;
  const int c = u - g * nchunks;
  const int p0 = c * chunk;
  const int p1 = min(n, p0 + chunk);
  const int h = g * 64 + lane;
  const int hl0 = h < H ? h : H - 1;
  const int hl = Hmap ? Hmap[hl0] : hl0;  // counts[h] of model Hmap[h] (a dense list of models)
  double f[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) f[k] = Fsoa[k * ld + hl];
  int cnt = 0;
#pragma unroll 2
  for (int i = p0; i < p1; ++i) {
    const Pt p = pts[i];
    const double l10 = fma(f[0], p.x2, fma(f[1], p.y2, f[2]));
    const double l11 = fma(f[3], p.x2, fma(f[4], p.y2, f[5]));
    const double l12 = fma(f[6], p.x2, fma(f[7], p.y2, f[8]));
    const double l20 = fma(f[0], p.x1, fma(f[3], p.y1, f[6]));
    const double l21 = fma(f[1], p.x1, fma(f[4], p.y1, f[7]));
    // e = x^T F y = l1 . x^ = l2 . y^ (both residual numerators are the same quantity)
    const double e = fma(l10, p.x1, fma(l11, p.y1, l12));
    const double n1 = fma(l10, l10, l11 * l11);
    const double n2 = fma(l20, l20, l21 * l21);
    // d < t  <=>  e^2 < t^2 min(n1, n2); false for NaN / zero-length lines as in numpy
    cnt += (e * e < thr2 * fmin(n1, n2)) ? 1 : 0;
  }
  if (h < H) atomicAdd(&counts[h], cnt);
}

// ----------------------------------------------------------------------------------------
// fp32 counting with a rigorous fp64 guard band (k_f8_count32q, the product kernel).
//
// In the frame x~ = (x - c_i)/s (|x~| <= R = 1) with F~ = T1^T F T2 / max|.| the test
// e^2 < t^2 min(n1, n2) becomes e~^2 < T min(n~1, n~2), T = (t/s)^2, exactly (e scales with
// the model scale, n with its square, both line lengths with s^2).  Each fp32 operation and
// the fp64 -> fp32 rounding of F~ and of the points is bounded absolutely (f8_plan.hip
// fp32_bounds: De for e, Dn for a squared length), |e_c - e| <= De, |m_c - m| <= Dn,
// m = min(n1, n2), u = 2^-24.
//
// Decision (per-hypothesis constants, written by the solve into G4): with the AM-GM split
// 2De|e_c| <= De (e_c^2/c + c) at a per-hypothesis c (c = t~ sqrt(m at the frame centre),
// r = De/c) both sides are one packed fma of e and one packed multiply of m:
//   sure inlier  fl(e^2 + ki) < fl(alpha m):  e_c^2 + ki < alpha m_c (1+u)/(1-u), and with
//     alpha <= T (1-u)/((1+u)(1+r)), ki >= (De c + De^2 + T Dn)/(1+r):
//     e^2 <= e_c^2 (1+r) + De c + De^2 < T m_c - T Dn <= T m;
//   sure outlier fl(e^2 - ko) > fl(beta m) (>= 0):  e_c^2 > ko + beta m_c (1-u)/(1+u), and
//     with beta >= T (1+u)/((1-u)(1-r)), ko >= (T Dn + De c)/(1-r):
//     e^2 >= e_c^2 (1-r) - De c > T m_c + T Dn >= T m.
// (ki, -ko, alpha, beta) are one float4 per hypothesis (G4); ambiguous = XOR of the two
// ballots (fl(e^2 - ko) <= fl(e^2 + ki) and alpha <= beta).  An ambiguous (hypothesis, point)
// is re-tested in float64 in pixel units (test64, the k_f8_count expression), so the counts
// are bit-identical to k_f8_count's.  NaN (padding points, NaN models) fails every compare,
// as the float64 test fails.
//
// Point-pair packing.  Every v_pk_fma_f32 carries the SAME quantity of TWO consecutive points
// (2j and 2j+1 of a block of 8, one aligned SGPR pair per coordinate, k_pack_points32q):
//   a  = fma(F0, X2, fma(F1, Y2, F2))     b  = fma(F3, X2, fma(F4, Y2, F5))
//   l3 = fma(F6, X2, fma(F7, Y2, F8))     e  = fma(a, X1, fma(b, Y1, l3))
//   c  = fma(F0, X1, fma(F3, Y1, F6))     d  = fma(F1, X1, fma(F4, Y1, F7))
//   n1 = fma(a, a, b*b)   n2 = fma(c, c, d*d)   m = min(n1, n2) (two v_min)
//   P  = fma(e, e, ki)    Q  = fma(e, e, -ko)   R = alpha m   S = beta m
// Per point pair: 12 pk (a, b, l3, e, c, d) + 4 pk (n1, n2) + 2 min + 4 pk (P, Q, R, S) +
// 4 cmp + 2 add = 28 VALU, 14 per (64 hypotheses x point).  The splat coefficients are op_sel
// broadcasts inside one asm block per pair (pair_terms); the float64 re-test of an ambiguous
// pair runs right there.
//
// Work distribution.  The (group of 64 hypotheses) x (point) plane, flattened group-major, is
// cut into W equal contiguous slices (a multiple of 8 points), one per wave; a slice that
// crosses a group boundary runs as two segments, each with its own model load and one
// coalesced count atomic.  W is a multiple of the resident wave count (6 per SIMD), so every
// wave slot runs the same number of slices.  Waves of equal work still finish up to 2.5x
// apart (wave timeline, tools/count_timeline.py: not re-tests, not XCD, not SIMD occupancy),
// which is the launch's drain.  Measured and not kept: claiming chunks from per-XCD atomic
// head words (0.13-0.19 ms per C2 launch instead of ~0.1: a returning device-scope atomic per
// chunk queues behind thousands of pullers), 64 / 128-thread workgroups (same),
// progress-levelled s_setprio (same durations), and tile-major cells (a point tile x one
// hypothesis group per wave, so a workgroup's waves share scalar-cache lines: 0.108 vs 0.0995
// ms, slower ramp).  The scalar data cache misses 62 % of the point loads (PMC SQC_DCACHE_*),
// yet staging each wave's points through an LDS tile (broadcast ds_read_b128 into VGPR
// operands, 80 SGPRs / 62 VGPRs, 8 waves per SIMD) was slower too (0.104-0.106 ms).  Folding
// the guard band into per-hypothesis G constants (one compare chain per side, counts kept as
// bit planes) cut VALU by 6 % and left the time unchanged at C2 (0.1118 vs 0.1108 ms) and C5
// (4.35 vs 4.36 ms, tools/probe_c5_count.py): the issue slots are not what binds.  Slices
// shrinking with the wave index (slice w covering total x (1 - (1 - w/W)^p), so the last waves
// to start carry the least work) were slower too: 0.103-0.108 ms at p = 1.3-2.0 against
// 0.098-0.101 for equal slices, interleaved runs on one box (round 2).  Points loaded four at a
// time (16 SGPRs per load group: 90 SGPRs, 7-8 waves per SIMD) were not faster either:
// 97.0-99.3 us against 96.9-97.1 us, with 6 144 / 7 168 / 8 192 resident-wave launch shapes.
// A scalar-load double buffer (block i+8's two s_load_dwordx16 issued right after block i's
// data arrived, 16 s_mov_b64 per block to rotate) was not faster either (round 3, interleaved
// A/B: 98.1-103.4 us against 97.5-99.3 us; profiles/r03b_count_ab.txt): six resident waves
// per SIMD already cover the scalar cache's misses (SQC_DCACHE hit rate 36 %).  Two instruction-
// count variants, bit-exact against the full-size goldens, did not move it either (round 3,
// profiles/r03_count_variants.txt): sure-inlier counts as scalar bit planes (two v_addc fewer
// per pair, ~12 scalar ops more: 103-106 us, slower), and signed margins per point (E1 = P -
// alpha m, E2 = beta m - Q by one fma each, ambiguity iff E1 E2 >= 0 tested once per block by a
// running max3: no scalar work per pair, 30.75 instead of ~38 instructions per pair, in plain C
// or behind this asm core: 98-103 us against 98-100 us).  PMC of the product kernel
// (profiles/r03c_count_stall.txt): VALU instructions 79 % of the SIMD time at one quad-cycle
// each, 89 % of the SIMDs' time with waves resident; neither the total instruction count nor the
// scalar loads set the launch time -- the drain of unequal waves does (timeline, r03f: 26 % of
// the SIMD-time has <= 3 resident waves; the last ~20 us run on a falling fraction of them).
// Two ways to share the work dynamically, both bit-exact and both slower (round 3, same file):
// persistent 12-wave workgroups taking whole hypothesis groups from per-XCD heads, sub-chunks
// from an LDS counter, counts summed in LDS (109 us: the last groups leave one workgroup per CU
// running alone), and static slices over 75 % of the plane with the rest claimed in 32-128-point
// chunks from per-XCD heads (431-570 us: tens of thousands of returning device-scope atomics on
// eight words serialise).
// ----------------------------------------------------------------------------------------

// The float64 test of k_f8_count (pixel units) for one (hypothesis, point).
__device__ __forceinline__ bool test64(const double (&fd)[9], const Pt &q, double thr2) {
  const double a10 = fma(fd[0], q.x2, fma(fd[1], q.y2, fd[2]));
  const double a11 = fma(fd[3], q.x2, fma(fd[4], q.y2, fd[5]));
  const double a12 = fma(fd[6], q.x2, fma(fd[7], q.y2, fd[8]));
  const double a20 = fma(fd[0], q.x1, fma(fd[3], q.y1, fd[6]));
  const double a21 = fma(fd[1], q.x1, fma(fd[4], q.y1, fd[7]));
  const double ed = fma(a10, q.x1, fma(a11, q.y1, a12));
  const double m1 = fma(a10, a10, a11 * a11);
  const double m2 = fma(a20, a20, a21 * a21);
  return ed * ed < thr2 * fmin(m1, m2);
}

// Last-finisher reduction of one hypothesis group (64 lanes): the wave whose chunk brings
// gdone[grp] to npad reads the group's final counts and folds their max into status[0].  Every
// chunk's count atomics complete (vmcnt) before its gdone atomic, and the reader's atomic
// loads issue after its gdone atomic returned, so they see all of them.
__device__ __forceinline__ void group_done_max(int *counts, int *gdone, int *status, int grp,
                                               int len, int npad, int h, int H) {
  wait_vmem();
  int last = 0;
  if ((threadIdx.x & 63) == 0) last = (atomicAdd(&gdone[grp], len) + len == npad) ? 1 : 0;
  last = __shfl(last, 0);
  if (!last) return;
  int v = h < H ? ld_agent(&counts[h]) : 0;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
  if ((threadIdx.x & 63) == 0 && v > 0) atomicMax(&status[0], v);
}

#ifndef RSAMD_COUNT_LDS
#define RSAMD_COUNT_LDS 1  // per-workgroup group sums in LDS, one count atomic per group (A/B: 0)
#endif
constexpr int kCountGrpSlots = 8;  // hypothesis groups a workgroup sums in LDS (more: direct)
#ifndef RSAMD_COUNT_BT
#define RSAMD_COUNT_BT 256  // threads per counting workgroup (A/B: 512)
#endif
constexpr int kCountBT = RSAMD_COUNT_BT;
#ifndef RSAMD_RETEST_LANES
#define RSAMD_RETEST_LANES 1  // float64 re-test loads by the ambiguous lanes only (A/B: 0)
#endif

typedef float f2q __attribute__((ext_vector_type(2)));
// v_pk_mul_f32 with a broadcast half of a VGPR pair (OPSEL / OPSELHI pick, per result lane,
// the half of each source).
#define RSD_PKMUL_VB(d, a, b, OPSEL, OPSELHI)                                             \
  asm("v_pk_mul_f32 %0, %1, %2 op_sel:" OPSEL " op_sel_hi:" OPSELHI : "=v"(d) : "v"(a), "v"(b))

// The terms of one point pair (expressions and order as documented above); P01 = (F0, F1),
// P23 = (F2, F3), P45 = (F4, F5), P67 = (F6, F7), P8 = (F8, F8), KIO = (ki, -ko),
// ALB = (alpha, beta).
__device__ __forceinline__ void pair_terms(f2q P01, f2q P23, f2q P45, f2q P67, f2q P8, f2q KIO,
                                           f2q ALB, f2q X2, f2q Y2, f2q X1, f2q Y1, f2q &P,
                                           f2q &Q, f2q &R, f2q &S) {
#pragma clang fp contract(off)
  // One asm block from the point pair to (n1, n2, P, Q): the hazard recognizer treats every
  // inline asm as a possible transcendental and pads its consumers with an s_nop, so the
  // whole dependent chain is kept inside (plain VALU -> VALU dependencies interlock).
  // t0..t4 are reused in place: t0 = F1 y2 + F2 -> a -> P, t1 = F4 y2 + F5 -> b -> b^2 -> n1,
  // t2 = F7 y2 + F8 -> l3 -> b y1 + l3 -> e, t3 = F3 y1 + F6 -> c -> Q, t4 = F4 y1 + F7 -> d ->
  // d^2 -> n2.
  f2q t0, t1, t2, t3, t4;
  asm("v_pk_fma_f32 %[t0], %[P01], %[Y2], %[P23] op_sel:[1,0,0] op_sel_hi:[1,1,0]\n\t"
      "v_pk_fma_f32 %[t1], %[P45], %[Y2], %[P45] op_sel:[0,0,1] op_sel_hi:[0,1,1]\n\t"
      "v_pk_fma_f32 %[t2], %[P67], %[Y2], %[P8] op_sel:[1,0,0] op_sel_hi:[1,1,0]\n\t"
      "v_pk_fma_f32 %[t3], %[P23], %[Y1], %[P67] op_sel:[1,0,0] op_sel_hi:[1,1,0]\n\t"
      "v_pk_fma_f32 %[t4], %[P45], %[Y1], %[P67] op_sel:[0,0,1] op_sel_hi:[0,1,1]\n\t"
      "v_pk_fma_f32 %[t0], %[P01], %[X2], %[t0] op_sel:[0,0,0] op_sel_hi:[0,1,1]\n\t"  // a
      "v_pk_fma_f32 %[t1], %[P23], %[X2], %[t1] op_sel:[1,0,0] op_sel_hi:[1,1,1]\n\t"  // b
      "v_pk_fma_f32 %[t2], %[P67], %[X2], %[t2] op_sel:[0,0,0] op_sel_hi:[0,1,1]\n\t"  // l3
      "v_pk_fma_f32 %[t3], %[P01], %[X1], %[t3] op_sel:[0,0,0] op_sel_hi:[0,1,1]\n\t"  // c
      "v_pk_fma_f32 %[t4], %[P01], %[X1], %[t4] op_sel:[1,0,0] op_sel_hi:[1,1,1]\n\t"  // d
      "v_pk_fma_f32 %[t2], %[t1], %[Y1], %[t2]\n\t"                                      // b y1 + l3
      "v_pk_mul_f32 %[t1], %[t1], %[t1]\n\t"                                             // b^2
      "v_pk_mul_f32 %[t4], %[t4], %[t4]\n\t"                                             // d^2
      "v_pk_fma_f32 %[t2], %[t0], %[X1], %[t2]\n\t"                                      // e
      "v_pk_fma_f32 %[t1], %[t0], %[t0], %[t1]\n\t"                                      // n1
      "v_pk_fma_f32 %[t4], %[t3], %[t3], %[t4]\n\t"                                      // n2
      "v_pk_fma_f32 %[t0], %[t2], %[t2], %[KIO] op_sel:[0,0,0] op_sel_hi:[1,1,0]\n\t"  // P
      "v_pk_fma_f32 %[t3], %[t2], %[t2], %[KIO] op_sel:[0,0,1] op_sel_hi:[1,1,1]"        // Q
      : [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3), [t4] "=&v"(t4)
      : [P01] "v"(P01), [P23] "v"(P23), [P45] "v"(P45), [P67] "v"(P67), [P8] "v"(P8),
        [KIO] "v"(KIO), [X2] "s"(X2), [Y2] "s"(Y2), [X1] "s"(X1), [Y1] "s"(Y1));
  P = t0;
  Q = t3;
  // m = min(n1, n2): both are >= +0 or NaN, where the unsigned order of the bit patterns is
  // the float order and NaN loses, exactly as fminf (and no canonicalising v_max)
  typedef unsigned int u2 __attribute__((ext_vector_type(2)));
  const u2 mu = __builtin_elementwise_min(__builtin_bit_cast(u2, t1), __builtin_bit_cast(u2, t4));
  const f2q m = __builtin_bit_cast(f2q, mu);
  RSD_PKMUL_VB(R, m, ALB, "[0,0]", "[1,0]");  // alpha m
  RSD_PKMUL_VB(S, m, ALB, "[0,1]", "[1,1]");  // beta m
}

// Wave timeline of the counting kernel (start / end of each wave, 100 MHz real-time counter):
// set by the plan only under RSAMD_TSTAMP, for the launch-shape analysis.
__device__ uint64_t *g_count_ts = nullptr;

template <int BT>
__global__ __launch_bounds__(BT) void k_f8_count32q(const float4 *__restrict__ ptsq,
                                                     const Pt *__restrict__ pts, int n, int H,
                                                     const float *__restrict__ F32soa,
                                                     const double *__restrict__ Fsoa,
                                                     int64_t ld, int64_t per_wave, GuardW g,
                                                     int *__restrict__ counts,
                                                     int *__restrict__ gdone,
                                                     int *__restrict__ status,
                                                     const float4 *__restrict__ G4,
                                                     const int *__restrict__ Hdev) {
#pragma clang fp contract(off)
  typedef float f2 __attribute__((ext_vector_type(2)));
  const int lane = threadIdx.x & 63;
  // XCD-aware slice order: workgroups are dealt to the 8 XCDs round-robin, so workgroup b runs
  // on XCD b % 8; it takes slice block base(b % 8) + b / 8, which gives every XCD one contiguous
  // run of slices -- a hypothesis group's slices, and so its fp32 models and decision constants,
  // stay in one XCD's L2 instead of being fetched into two
  const int nb = static_cast<int>(gridDim.x), bx = static_cast<int>(blockIdx.x);
  const int xq = nb >> 3, xr = nb & 7, xc = bx & 7;
  const int bslot = xc * xq + min(xc, xr) + (bx >> 3);
  const int64_t w = wave_uniform(bslot * (BT / 64) + (threadIdx.x >> 6));
  const int npad = (n + 7) / 8 * 8;
  if (Hdev) {
    // the hypothesis count on the device (at most H, the bound the grid was sized for): the
    // slice length from it as count32q_shape would, so no host round trip before the launch
    H = min(H, *Hdev);
    const int64_t tot = static_cast<int64_t>((H + 63) >> 6) * npad;
    if (tot == 0) return;  // uniform over the grid, before any barrier
    const int64_t Wd = max<int64_t>(1, min<int64_t>(static_cast<int64_t>(nb) * (BT / 64), tot / 64));
    per_wave = ((tot + Wd - 1) / Wd + 7) / 8 * 8;
  }
  const int64_t total = static_cast<int64_t>((H + 63) >> 6) * npad;
  int64_t pos = w * per_wave;
  const int64_t end = min(total, pos + per_wave);
#if RSAMD_COUNT_LDS
  // The workgroup's slices are consecutive, so they cover a few hypothesis groups (two at C2):
  // their partial counts are summed in LDS, and the workgroup's last wave to finish adds each
  // group's 64 counts to HBM once and folds the group's completion (gdone, c*).  One 256-B
  // count atomic per workgroup and group instead of one per slice segment (WRITE_SIZE per C2
  // launch 3.99 MB for 0.4 MB of counts, profiles/r04k_pmc_k_f8_count.json); no barrier: the
  // finished waves never wait for the slow ones.
  __shared__ int s_cnt[kCountGrpSlots * 64];
  __shared__ int s_len[kCountGrpSlots];
  __shared__ int s_fin;
  const int g0 = static_cast<int>(min(total - 1, bslot * (BT / 64) * per_wave) / npad);
  for (int x = threadIdx.x; x < kCountGrpSlots * 64; x += BT) s_cnt[x] = 0;
  if (threadIdx.x < kCountGrpSlots) s_len[threadIdx.x] = 0;
  if (threadIdx.x == 0) s_fin = 0;
  __syncthreads();
#endif
  uint64_t *ts = g_count_ts;  // diagnostic wave timeline (RSAMD_TSTAMP), null in production
  const uint64_t t_start = ts ? __builtin_amdgcn_s_memrealtime() : 0ull;
  const uint64_t c_start = ts ? __builtin_amdgcn_s_memtime() : 0ull;  // shader clock
  int n_retest = 0;  // re-test branches taken (timeline diagnostics)
  while (pos < end) {
    const int grp = static_cast<int>(pos / npad);
    const int p0 = static_cast<int>(pos - static_cast<int64_t>(grp) * npad);
    const int p1 = static_cast<int>(min(static_cast<int64_t>(npad), p0 + (end - pos)));
    pos += p1 - p0;
    const int h = grp * 64 + lane;
    const int hl = h < H ? h : H - 1;
    float f[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) f[k] = F32soa[k * ld + hl];
    // coefficient pairs; broadcasts of one half are op_sel operands (pair_terms), so no
    // duplicated VGPRs
    const f2 P01 = {f[0], f[1]}, P23 = {f[2], f[3]}, P45 = {f[4], f[5]}, P67 = {f[6], f[7]};
    const f2 P8 = {f[8], f[8]};
    const float4 q = G4[hl];
    const f2 KIO = {q.x, q.y}, ALB = {q.z, q.w};
    int cnt = 0;
    for (int i = p0; i < p1; i += 8) {
      float4 blk[8];  // (x2[8], y2[8], x1[8], y1[8]) of points i..i+7
#pragma unroll
      for (int k = 0; k < 8; ++k) blk[k] = ptsq[i + k];
      const float *v = reinterpret_cast<const float *>(blk);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f2 X2 = {v[2 * j], v[2 * j + 1]}, Y2 = {v[8 + 2 * j], v[9 + 2 * j]};
        const f2 X1 = {v[16 + 2 * j], v[17 + 2 * j]}, Y1 = {v[24 + 2 * j], v[25 + 2 * j]};
        f2 P, Q, R, S;
        pair_terms(P01, P23, P45, P67, P8, KIO, ALB, X2, Y2, X1, Y1, P, Q, R, S);
        const unsigned long long i0 = __ballot(P.x < R.x), i1 = __ballot(P.y < R.y);
        const unsigned long long l0 = __ballot(Q.x <= S.x), l1 = __ballot(Q.y <= S.y);
        cnt = add_lane_bit(cnt, i0);  // sure inliers
        cnt = add_lane_bit(cnt, i1);
        const unsigned long long a0 = i0 ^ l0, a1 = i1 ^ l1;
        if ((a0 | a1) != 0ull) {  // rare: float64 re-test of the ambiguous lanes
          ++n_retest;
          // the opaque pointer keeps these loads (and their 18 VGPRs) inside the rare branch
          const double *fp = Fsoa + hl;
          asm volatile("" : "+v"(fp));
#if RSAMD_RETEST_LANES
          // only the ambiguous lanes fetch their float64 model (a 128-B line of each row holds
          // 16 hypotheses: a re-test touches the lines of its lanes, not all 36 of the group)
          if (((a0 | a1) >> lane) & 1ull) {
#endif
          double fdd[9];
#pragma unroll
          for (int k = 0; k < 9; ++k) fdd[k] = fp[k * ld];
          if ((a0 >> lane) & 1ull) cnt += test64(fdd, pts[i + 2 * j], g.thr2_px) ? 1 : 0;
          if ((a1 >> lane) & 1ull) cnt += test64(fdd, pts[i + 2 * j + 1], g.thr2_px) ? 1 : 0;
#if RSAMD_RETEST_LANES
          }
#endif
        }
      }
    }
#if RSAMD_COUNT_LDS
    if (grp - g0 < kCountGrpSlots) {
      atomicAdd(&s_cnt[(grp - g0) * 64 + lane], cnt);
      if (lane == 0) atomicAdd(&s_len[grp - g0], p1 - p0);
      continue;
    }
#endif
    if (h < H) atomicAdd(&counts[h], cnt);
    if (gdone) group_done_max(counts, gdone, status, grp, p1 - p0, npad, h, H);
  }
#if RSAMD_COUNT_LDS
  {
    // the last wave of the workgroup (its LDS adds, and every other wave's, are complete:
    // workgroup-scope acquire-release on the finish counter) flushes the group sums
    int last = 0;
    if (lane == 0)
      last = __hip_atomic_fetch_add(&s_fin, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP) ==
             BT / 64 - 1;
    last = __shfl(last, 0);
    if (last) {
      for (int k = 0; k < kCountGrpSlots; ++k) {
        const int len = __hip_atomic_load(&s_len[k], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (len == 0) continue;  // wave-uniform (an LDS word)
        const int grp = g0 + k, h = grp * 64 + lane;
        const int c = __hip_atomic_load(&s_cnt[k * 64 + lane], __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_WORKGROUP);
        if (h < H) atomicAdd(&counts[h], c);
        if (gdone) group_done_max(counts, gdone, status, grp, len, npad, h, H);
      }
    }
  }
#endif
  if (ts && lane == 0) {
    uint64_t *o = ts + kCountTsWords * w;
    o[0] = t_start;
    o[1] = __builtin_amdgcn_s_memrealtime();
    o[2] = static_cast<uint64_t>(n_retest);
    // where it ran: HW_ID (wave, SIMD, CU, SE fields) and XCC_ID
    o[3] = (static_cast<uint64_t>(__builtin_amdgcn_s_getreg((31 << 11) | 4)) << 8) |
           static_cast<uint64_t>(__builtin_amdgcn_s_getreg((3 << 11) | 20) & 7);
    // shader-clock cycles over the wave: with o[0..1] the wave's own clock (cycles / real time)
    o[4] = c_start;
    o[5] = __builtin_amdgcn_s_memtime();
  }
}

// Point-pair layout of k_f8_count32q: block b of 8 points is 32 floats
// (x2[8], y2[8], x1[8], y1[8]) in the unit frame; NaN padding.
__global__ __launch_bounds__(256) void k_pack_points32q(const Pt *__restrict__ pts, int n,
                                                        Frame fr, float *__restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= ((n + 7) & ~7)) return;
  float *o = out + 32 * (i >> 3) + (i & 7);
  if (i >= n) {
    const float qn = __builtin_nanf("");
    o[0] = o[8] = o[16] = o[24] = qn;
    return;
  }
  const Pt p = pts[i];
  const double is = 1.0 / fr.s;
  o[0] = static_cast<float>((p.x2 - fr.cx2) * is);
  o[8] = static_cast<float>((p.y2 - fr.cy2) * is);
  o[16] = static_cast<float>((p.x1 - fr.cx1) * is);
  o[24] = static_cast<float>((p.y1 - fr.cy1) * is);
}

// ----------------------------------------------------------------------------------------
// Selection over H counts in three grid-wide passes (no single-workgroup scan):
//   k_f8_max        c* = max count (block max -> one atomicMax per block)
//   k_f8_blockcount per block slice: number of hypotheses with count >= max(c* - slack, 1)
//   k_f8_compact    ordered compaction: block offset = sum of earlier block counts, then
//                   ballot/popcount prefix inside the block; the last block writes the total
// ----------------------------------------------------------------------------------------
__device__ __forceinline__ int block_reduce_max(int v, int *sh) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  int r = sh[0];
  for (int q = 1; q < (int)(blockDim.x >> 6); ++q) r = max(r, sh[q]);
  __syncthreads();
  return r;
}
__device__ __forceinline__ int block_reduce_sum(int v, int *sh) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  int r = 0;
  for (int q = 0; q < (int)(blockDim.x >> 6); ++q) r += sh[q];
  __syncthreads();
  return r;
}

__global__ __launch_bounds__(256) void k_f8_max(const int *__restrict__ counts, int H,
                                                int *__restrict__ status) {
  __shared__ int sh[4];
  int m = 0;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < H; i += gridDim.x * 256) m = max(m, counts[i]);
  m = block_reduce_max(m, sh);
  if (threadIdx.x == 0 && m > 0) atomicMax(&status[0], m);
}

// ----------------------------------------------------------------------------------------
// Reference-order statistics, wave per candidate (grid-stride).
// ----------------------------------------------------------------------------------------
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ double block_sum_d(double v, double *sh) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  double r = 0.0;
  for (int q = 0; q < (int)(blockDim.x >> 6); ++q) r += sh[q];
  __syncthreads();
  return r;
}

__device__ void replay_inliers(const Pt *__restrict__ pts, int n, const int *counts, int nb,
                               int per_block, const int *bc, const int *cand, const int *ccount,
                               const double *cstd, const double *cnorm,
                               const double *__restrict__ Fsoa, int64_t ld, int *status,
                               double thresh, F8DevResult *__restrict__ res,
                               F8DevResult *__restrict__ hres, const int *cfast,
                               const int *spec, const int *spec_j, int *__restrict__ hinl);

// Candidates + their reference-order statistics, one block per slice of hypotheses:
// every hypothesis of the slice with fast count >= max(c* - slack, 1) is appended in index
// order to the block's own segment cand[b * per_block + j] (bc[b] entries), then the block
// re-scores each of them with dist_ref: count, np.std(d) (two-pass), np.linalg.norm(d).
// Per select block: the candidates of its hypothesis range (count >= c* - slack), each with
// its exact reference-order count, std and norm (fun.py:316-321).  The distances of a
// candidate are computed once and kept in registers (n <= kRegPts * kTailThreads; larger n
// recomputes them in a second pass), the three sums share one LDS round, and the block's
// first candidate also writes its S_RANSAC = flatnonzero(d < t) to the block's `spec` row,
// so that the replay only copies the winner's list when the winner is such a candidate.
constexpr int kRegPts = 8;
constexpr int kLocalCands = 64;

__device__ void cand_stats_block(const TailArgs &a, int bid, int nblocks) {
  const Pt *__restrict__ pts = a.pts;
  const int n = a.n, H = a.H, slack = a.slack, per_block = a.per_block;
  const double *__restrict__ Fsoa = a.Fsoa;
  const int64_t ld = a.ld;
  const int *__restrict__ counts = a.counts;
  const int *__restrict__ status = a.status;
  int *__restrict__ status_rw = a.status;
  const double thresh = a.thresh;
  int *__restrict__ bc = a.status + 4;
  int *__restrict__ cand = a.cand;
  int *__restrict__ ccount = a.ccount;
  double *__restrict__ cstd = a.cstd;
  double *__restrict__ cnorm = a.cnorm;
  constexpr int NW = kTailThreads / 64;
  __shared__ double shd[2][NW];
  __shared__ double sh3[NW];  // s3 has its own row: other waves may still read shd / shi
  __shared__ int last_s;
  __shared__ int shi[NW];
  __shared__ int woff[NW];
  __shared__ int lcand[kLocalCands];
  __shared__ int qoff[kRegPts][NW];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int cmax = status[0];
  const int thr = max(cmax - slack, 1);
  const int b0 = bid * per_block, b1 = min(H, b0 + per_block);
  int *seg = cand + static_cast<int64_t>(bid) * per_block;
  int *segf = a.cfast + static_cast<int64_t>(bid) * per_block;
  int nloc = 0;
  if (cmax > 0) {
    for (int b = b0; b < b1; b += kTailThreads) {
      const int i = b + tid;
      const int c = i < b1 ? counts[i] : 0;
      const bool take = i < b1 && c >= thr;
      const unsigned long long bal = __ballot(take);
      if (lane == 0) woff[w] = __popcll(bal);
      __syncthreads();
      int base = nloc, tot = 0;
      for (int q = 0; q < NW; ++q) {
        if (q < w) base += woff[q];
        tot += woff[q];
      }
      if (take) {
        const int o = base + __popcll(bal & ((1ull << lane) - 1ull));
        st_agent(&seg[o], i);
        st_agent(&segf[o], c);
        if (o < kLocalCands) lcand[o] = i;
      }
      nloc += tot;
      __syncthreads();
    }
  }
  const bool in_regs = n <= kRegPts * kTailThreads;
  if (tid == 0) {
    st_agent(&bc[bid], nloc);
    st_agent(&a.spec_j[bid], (nloc > 0 && in_regs && !a.nospec) ? 0 : -1);
    if (bid == 0) st_agent(&status_rw[3], per_block);  // the layout, for rs_f8_plan_candidates
  }
  int *spec = a.spec + static_cast<int64_t>(bid) * n;
  for (int j = 0; j < nloc; ++j) {
    const int h = j < kLocalCands ? lcand[j] : ld_agent(&seg[j]);
    double f[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) f[k] = Fsoa[k * ld + h];
    double s1 = 0.0, s2 = 0.0, s3 = 0.0;
    int cnt = 0;
    double mean;
    if (in_regs) {
      double dv[kRegPts];
      unsigned long long bl[kRegPts];
#pragma unroll
      for (int q = 0; q < kRegPts; ++q) {
        const int i = tid + q * kTailThreads;
        double d = 0.0;
        bool in = false;
        if (i < n) {
          d = dist_ref(f, pts[i]);
          in = d < thresh;
          s1 += d;
          s2 += d * d;
        }
        dv[q] = d;
        cnt += in ? 1 : 0;
        bl[q] = __ballot(in);
      }
      s1 = wave_sum(s1);
      s2 = wave_sum(s2);
      cnt = wave_sum_i(cnt);
      if (lane == 0) {
        shd[0][w] = s1;
        shd[1][w] = s2;
        shi[w] = cnt;
#pragma unroll
        for (int q = 0; q < kRegPts; ++q) qoff[q][w] = __popcll(bl[q]);
      }
      __syncthreads();
      s1 = 0.0;
      s2 = 0.0;
      cnt = 0;
      for (int q = 0; q < NW; ++q) {  // block_sum_d / block_reduce_sum order
        s1 += shd[0][q];
        s2 += shd[1][q];
        cnt += shi[q];
      }
      mean = s1 / static_cast<double>(n);
      if (j == 0 && !a.nospec) {  // the block's speculative S_RANSAC, in index order
#pragma unroll
        for (int q = 0; q < kRegPts; ++q) {
          if ((bl[q] >> lane) & 1ull) {
            int o = __popcll(bl[q] & ((1ull << lane) - 1ull));
            for (int qq = 0; qq < kRegPts; ++qq)
              for (int ww = 0; ww < NW; ++ww)
                if (qq < q || (qq == q && ww < w)) o += qoff[qq][ww];
            st_agent(&spec[o], tid + q * kTailThreads);
          }
        }
      }
#pragma unroll
      for (int q = 0; q < kRegPts; ++q) {
        const int i = tid + q * kTailThreads;
        if (i < n) {
          const double v = dv[q] - mean;
          s3 += v * v;
        }
      }
    } else {
      for (int i = tid; i < n; i += kTailThreads) {
        const double d = dist_ref(f, pts[i]);
        cnt += d < thresh ? 1 : 0;
        s1 += d;
        s2 += d * d;
      }
      s1 = block_sum_d(s1, shd[0]);
      s2 = block_sum_d(s2, shd[0]);
      cnt = block_reduce_sum(cnt, shi);
      mean = s1 / static_cast<double>(n);
      for (int i = tid; i < n; i += kTailThreads) {
        const double v = dist_ref(f, pts[i]) - mean;
        s3 += v * v;
      }
    }
    s3 = block_sum_d(s3, sh3);  // its trailing barrier also retires shd / shi / qoff
    if (tid == 0) {
      const int64_t slot = static_cast<int64_t>(bid) * per_block + j;
      st_agent(&ccount[slot], cnt);
      st_agent(&cstd[slot], sqrt(s3 / static_cast<double>(n)));
      st_agent(&cnorm[slot], sqrt(s2));
    }
  }
  // the last block to finish runs the replay: every block's segment, counts, statistics and
  // speculative list are agent-scope stores completed (vmcnt) before its done-counter
  // increment
  wait_vmem();
  __syncthreads();
  if (tid == 0) last_s = atomicAdd(&status_rw[2], 1) == static_cast<int>(nblocks) - 1;
  __syncthreads();
  if (!last_s) return;
  replay_inliers(pts, n, counts, nblocks, per_block, bc, cand, ccount, cstd, cnorm, Fsoa, ld,
                 status_rw, thresh, a.res, a.hres, a.cfast, a.spec, a.spec_j, a.hinl);
}

// ----------------------------------------------------------------------------------------
// fun.py:320-328 over the ordered candidates.  Comparisons of non-negative doubles are done
// on their bit patterns (NaN keyed so that it never wins), scanning 64 candidates per
// coalesced load.
// ----------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t key_std(double s) {  // "best_std > x" is false for NaN
  return (s != s) ? 0ull : static_cast<uint64_t>(__double_as_longlong(s));
}
__device__ __forceinline__ uint64_t key_norm(double v) {  // "y > norm" is false for NaN
  return (v != v) ? ~0ull : static_cast<uint64_t>(__double_as_longlong(v));
}

// One kTailThreads workgroup (the last cand_stats block to finish): wave 0 replays
// fun.py:320-328 over the candidates in global index order (segments in block order), 64 per
// coalesced load; then the whole workgroup extracts S_RANSAC = flatnonzero(d < t) of the
// winner in order.  The result header goes to res (HBM) and, when given, to hres (the run's
// pinned host slot, written through the host mapping: no copy pass); the inlier list stays
// in res->inliers (HBM).
__device__ void replay_inliers(const Pt *__restrict__ pts, int n, const int *counts, int nb,
                               int per_block, const int *bc, const int *cand, const int *ccount,
                               const double *cstd, const double *cnorm,
                               const double *__restrict__ Fsoa, int64_t ld, int *status,
                               double thresh, F8DevResult *__restrict__ res,
                               F8DevResult *__restrict__ hres, const int *cfast,
                               const int *spec, const int *spec_j, int *__restrict__ hinl) {
  int *status_out = status;
  __shared__ int pref[kSelectBlocks + 1];
  __shared__ int woff[kTailThreads / 64];
  __shared__ int base_s;
  __shared__ double fsh[9];
  __shared__ int have_s;
  __shared__ int spec_row_s, nin_s;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // exclusive prefix of the per-block candidate counts (nb <= 256): one wave per 64 blocks,
  // then the 4 wave totals
  {
    const int v = tid < nb ? ld_agent(&bc[tid]) : 0;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o);
      if (lane >= o) x += y;
    }
    if (tid < kSelectBlocks) pref[tid] = x - v;   // wave-local exclusive
    if (lane == 63 && w < kSelectBlocks / 64) woff[w] = x;
    __syncthreads();
    if (tid < kSelectBlocks) {
      int add = 0;
      for (int q = 0; q < (tid >> 6); ++q) add += woff[q];
      pref[tid] += add;
    }
    if (tid == 0) {
      int tot = 0;
      for (int q = 0; q < kSelectBlocks / 64; ++q) tot += woff[q];
      pref[kSelectBlocks] = tot;
    }
    __syncthreads();
  }
  const int nc = pref[kSelectBlocks];
  if (w == 0) {
    int best = -1, bcount = 0;
    uint64_t bstd = 0ull;  // S_RANSAC = [], norm([]) = 0
    // the winner's record travels with the replay (no dependent loads after it)
    int bh = -1, brow = -1;
    double bsv = 0.0, bnv = 0.0;
    int mismatch = 0;
    for (int b = 0; b < nc; b += 64) {
      const int c = b + lane;
      int cc = 0, ch = -1, crow = -1;
      double sv = 0.0, nv = 0.0;
      if (c < nc) {
        int lo = 0, hi = nb - 1;  // block q with pref[q] <= c < pref[q+1]
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if (pref[mid] <= c) lo = mid; else hi = mid - 1;
        }
        const int64_t slot = static_cast<int64_t>(lo) * per_block + (c - pref[lo]);
        cc = ld_agent(&ccount[slot]);
        sv = ld_agent(&cstd[slot]);
        nv = ld_agent(&cnorm[slot]);
        ch = ld_agent(&cand[slot]);
        // its block's first candidate: its S_RANSAC is already in that block's spec row
        crow = ld_agent(&spec_j[lo]) == c - pref[lo] ? lo : -1;
        mismatch += (cc != ld_agent(&cfast[slot])) ? 1 : 0;
      }
      const uint64_t ks = key_std(sv), kn = key_norm(nv);
      const int lim = min(64, nc - b);
      for (int q = 0; q < lim; ++q) {
        const int qc = __shfl(cc, q);
        const uint64_t qs = __shfl(ks, q);
        const uint64_t qn = __shfl(kn, q);
        const int qh = __shfl(ch, q), qrow = __shfl(crow, q);
        const double qsv = __shfl(sv, q), qnv = __shfl(nv, q);
        bool take = false;
        if (qc > bcount) {
          take = true;
          bcount = qc;
        } else if (qc == bcount && bcount > 0 && bstd > qn) {
          take = true;
        }
        if (take) {
          best = b + q;
          bstd = qs;
          bh = qh;
          brow = qrow;
          bsv = qsv;
          bnv = qnv;
        }
      }
    }
    mismatch = wave_sum_i(mismatch);
    if (lane == 0) {
      const int cfast_max = status[0];
      double fw[9];
      if (best >= 0) {
#pragma unroll
        for (int k = 0; k < 9; ++k) fw[k] = Fsoa[k * ld + bh];
      } else {
#pragma unroll
        for (int k = 0; k < 9; ++k) fw[k] = 0.0;
      }
      const bool spec_ok = best >= 0 && brow >= 0;
      F8DevResult *outs[2] = {res, hres};
      for (int o = 0; o < 2; ++o) {
        F8DevResult *r = outs[o];
        if (!r) continue;
        r->n_candidates = nc;
        r->max_count_fast = cfast_max;
        r->guard_mismatch = mismatch;
        r->best_index = best >= 0 ? bh : -1;
        r->best_count = best >= 0 ? bcount : 0;
        r->best_std = best >= 0 ? bsv : 0.0;
        r->best_norm = best >= 0 ? bnv : 0.0;
        r->best_cand = best;
        r->inl_row = spec_ok ? brow : -1;
        if (spec_ok) r->n_inliers = bcount;
#pragma unroll
        for (int k = 0; k < 9; ++k) r->F[k] = fw[k];
      }
#pragma unroll
      for (int k = 0; k < 9; ++k) fsh[k] = fw[k];
      status_out[1] = nc;
      have_s = best >= 0 ? 1 : 0;
      spec_row_s = spec_ok ? brow : -1;
      nin_s = spec_ok ? bcount : 0;
      base_s = 0;
    }
  }
  __syncthreads();
  // the winner's S_RANSAC is its block's speculative list (rs_f8_plan_result reads it from
  // hinl, or copies the row: inl_row); otherwise extract it here
  if (spec_row_s >= 0) {
    if (hinl) {  // the list to the pinned host buffer (no copy pass after the run)
      const int *row = spec + static_cast<int64_t>(spec_row_s) * n;
      for (int i = tid; i < nin_s; i += kTailThreads) hinl[i] = ld_agent(&row[i]);
    }
    return;
  }
  const bool have = have_s != 0;
  double f[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) f[k] = fsh[k];
  for (int b = 0; b < n; b += kTailThreads) {
    const int i = b + tid;
    const bool take = have && i < n && dist_ref(f, pts[i]) < thresh;
    const unsigned long long bal = __ballot(take);
    const int before = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) woff[w] = __popcll(bal);
    __syncthreads();
    if (tid == 0) {
      int acc = base_s;
      for (int q = 0; q < kTailThreads / 64; ++q) {
        const int t = woff[q];
        woff[q] = acc;
        acc += t;
      }
      base_s = acc;
    }
    __syncthreads();
    if (take) {
      res->inliers[woff[w] + before] = i;
      if (hinl) hinl[woff[w] + before] = i;
    }
    __syncthreads();
  }
  if (tid == 0) {
    res->n_inliers = base_s;
    if (hres) hres->n_inliers = base_s;
  }
}

// ----------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_residuals(const Pt *__restrict__ pts, int n,
                                                   const double *__restrict__ F,
                                                   double *__restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double f[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) f[k] = F[k];
  double r1, r2;
  residuals_ref(f, pts[i], r1, r2);
  out[i] = r1;
  out[n + i] = r2;
}

// Pack (2,n) row-major p1, p2 into AoS points.
__global__ __launch_bounds__(256) void k_pack_points(const double *__restrict__ p1,
                                                     const double *__restrict__ p2, int n,
                                                     Pt *__restrict__ pts) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Pt p;
  p.x1 = p1[i];
  p.y1 = p1[n + i];
  p.x2 = p2[i];
  p.y2 = p2[n + i];
  pts[i] = p;
}

// both layouts in one launch (the E-RANSAC path: a launch fewer): pts as k_pack_points, and
// when fr is given the point-pair layout as k_pack_points32q, from the same doubles
__global__ __launch_bounds__(256) void k_pack_points_both(const double *__restrict__ p1,
                                                          const double *__restrict__ p2, int n,
                                                          Pt *__restrict__ pts, bool q, Frame fr,
                                                          float *__restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= ((n + 7) & ~7)) return;
  float *o = out + 32 * (i >> 3) + (i & 7);
  if (i >= n) {
    if (q) {
      const float qn = __builtin_nanf("");
      o[0] = o[8] = o[16] = o[24] = qn;
    }
    return;
  }
  Pt p;
  p.x1 = p1[i];
  p.y1 = p1[n + i];
  p.x2 = p2[i];
  p.y2 = p2[n + i];
  pts[i] = p;
  if (q) {
    const double is = 1.0 / fr.s;
    o[0] = static_cast<float>((p.x2 - fr.cx2) * is);
    o[8] = static_cast<float>((p.y2 - fr.cy2) * is);
    o[16] = static_cast<float>((p.x1 - fr.cx1) * is);
    o[24] = static_cast<float>((p.y1 - fr.cy1) * is);
  }
}

}  // namespace rsd

// ------------------------------------------------------------------------------------------
// Host launchers
// ------------------------------------------------------------------------------------------
namespace rsd {

// this file's code object onto the current device (rs_ctx_create: not at the first RANSAC)
hipError_t preload_f8() {
  hipFuncAttributes fa{};
  return hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(k_pack_points));
}

hipError_t launch_pack_points(const double *p1, const double *p2, int n, Pt *pts,
                              hipStream_t s) {
  hipLaunchKernelGGL(k_pack_points, dim3((n + 255) / 256), dim3(256), 0, s, p1, p2, n, pts);
  return hipGetLastError();
}

hipError_t launch_f8_solve(const Pt *pts, int n, int H, int mode, uint64_t seed,
                           uint64_t hyp_offset, const int *tuples, double *Fsoa, int64_t ld,
                           int *counts, int *status, hipStream_t s, float *F32soa,
                           const Frame *frame, int *gdone) {
  SolveArgs a{};
  a.pts = pts;
  a.n = n;
  a.H = H;
  a.mode = mode;
  a.seed = seed;
  a.hyp_offset = hyp_offset;
  a.tuples = tuples;
  a.Fsoa = Fsoa;
  a.ld = ld;
  a.counts = counts;
  a.status = status;
  a.F32soa = frame ? F32soa : nullptr;
  a.frame = frame ? *frame : Frame{1.0, 0.0, 0.0, 0.0, 0.0};
  a.gdone = gdone;
  hipLaunchKernelGGL(k_f8_solve, dim3((H + 255) / 256), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_f8_count(const Pt *pts, int n, int H, const double *Fsoa, int64_t ld,
                           int chunk, double thr2, int *counts, hipStream_t s, const int *Hdev,
                           const int *Hmap) {
  const int nchunks = (n + chunk - 1) / chunk;
  const int units = ((H + 63) / 64) * nchunks;
  hipLaunchKernelGGL(k_f8_count, dim3((units + 3) / 4), dim3(256), 0, s, pts, n, H, Fsoa, ld,
                     chunk, nchunks, thr2, counts, Hdev, Hmap);
  return hipGetLastError();
}

hipError_t set_count_timeline(uint64_t *buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_count_ts), &buf, sizeof(buf));
}

hipError_t launch_pack_points_both(const double *p1, const double *p2, int n, Pt *pts,
                                   const Frame *fr, float4 *ptsq, hipStream_t s) {
  hipLaunchKernelGGL(k_pack_points_both, dim3((n + 7 + 255) / 256), dim3(256), 0, s, p1, p2, n, pts,
                     fr != nullptr, fr ? *fr : Frame{}, reinterpret_cast<float *>(ptsq));
  return hipGetLastError();
}

hipError_t launch_pack_points32q(const Pt *pts, int n, const Frame &fr, float4 *ptsq,
                                 hipStream_t s) {
  hipLaunchKernelGGL(k_pack_points32q, dim3((n + 7 + 255) / 256), dim3(256), 0, s, pts, n, fr,
                     reinterpret_cast<float *>(ptsq));
  return hipGetLastError();
}

// Resident waves of k_f8_count32q: its ~106 SGPRs admit 6 waves per SIMD
// (floor(800 / (ceil(sgpr / 16) * 16 + 16)), MI355X_MICROARCH.md; the occupancy API reports 7,
// one block per CU too many for SGPR-heavy kernels; the wave timeline shows 6144 resident).
int count32q_resident_waves(int device) {
  int cus = 256;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
    cus = 256;
  return cus * 4 * 6;
}

// Absolute error bounds of the fp32 test in the unit frame (|x~| <= R); derivation above
// k_f8_count32q.  Dl: a line component, De: e, Dn: a squared length.
Bounds fp32_bounds(const Frame &fr, double thresh) {
  const double u = std::ldexp(1.0, -24), R = 1.0 + 1e-6, Lm = 2.0 * R + 1.0;
  const double Dl = 1.1 * u * (7.0 * R + 3.0);
  const double De =
      1.1 * (2.0 * (Dl * R * 1.001 + Lm * u * R) + Dl + u * (Lm + Dl) * (3.0 * R + 2.0) * 1.001);
  const double Dn = 1.1 * (2.0 * Dl * (2.0 * Lm + Dl) + 3.0 * u * (Lm + Dl) * (Lm + Dl) * 1.001);
  return {u, De, Dn, (thresh / fr.s) * (thresh / fr.s)};
}

// The unit frame of the fp32 counting kernel from the (2, n) pixel points: per-image centres,
// one common scale; false (no fp32 counting) for non-finite points or a degenerate frame.
bool unit_frame(const double *p1, const double *p2, int64_t n, Frame &fr) {
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
  fr = Frame{0.0, 0.5 * (lo[0] + hi[0]), 0.5 * (lo[1] + hi[1]), 0.5 * (lo[2] + hi[2]),
             0.5 * (lo[3] + hi[3])};
  const double cen[4] = {fr.cx1, fr.cy1, fr.cx2, fr.cy2};
  for (int64_t i = 0; finite && i < n; ++i) {
    const double v[4] = {p1[i], p1[n + i], p2[i], p2[n + i]};
    for (int k = 0; k < 4; ++k) fr.s = std::max(fr.s, std::fabs(v[k] - cen[k]));
  }
  if (!(finite && fr.s > 0.0 && std::isfinite(fr.s))) return false;
  fr.s *= 1.0 + 1e-12;  // |x~| <= 1 after the fp64 division
  return true;
}

Count32qShape count32q_shape(int n, int H, int waves, int slices_per_wave) {
  Count32qShape sh{};
  const int64_t npad = (n + 7) / 8 * 8;
  const int64_t total = static_cast<int64_t>((H + 63) / 64) * npad;
  // slices_per_wave x the resident waves (2 by default: A/B on C2 in r01 and r02, 2x ahead
  // of 1x, 2.67x and 5.3x by 1-6 %), at least 64 points each, a multiple of 8 points
  const int64_t k = slices_per_wave > 0 ? slices_per_wave : 2;
  int64_t W = std::max<int64_t>(1, std::min<int64_t>(k * waves, total / 64));
  int64_t per = (total + W - 1) / W;
  per = (per + 7) / 8 * 8;
  W = (total + per - 1) / per;
  sh.per_wave = per;
  sh.blocks = (W + kCountBT / 64 - 1) / (kCountBT / 64);
  return sh;
}

hipError_t launch_f8_count32q(const float4 *ptsq, const Pt *pts, int n, int H,
                              const float *F32soa, const double *Fsoa, int64_t ld,
                              const Count32qShape &sh, const GuardW &g, int *counts,
                              hipStream_t s, int *gdone, int *status, const float4 *G4,
                              const int *Hdev) {
  hipLaunchKernelGGL((k_f8_count32q<kCountBT>), dim3(static_cast<unsigned>(sh.blocks)), dim3(kCountBT), 0,
                     s, ptsq, pts, n, H, F32soa, Fsoa, ld, sh.per_wave, g, counts, gdone, status,
                     G4, Hdev);
  return hipGetLastError();
}

int select_per_block(int H) { return (H + kSelectBlocks - 1) / kSelectBlocks; }
int select_blocks(int H) {
  const int pb = select_per_block(H);
  return (H + pb - 1) / pb;
}

hipError_t launch_f8_max(const int *counts, int H, int *status, hipStream_t s) {
  hipLaunchKernelGGL(k_f8_max, dim3(select_blocks(H)), dim3(256), 0, s, counts, H, status);
  return hipGetLastError();
}

// The selection tail of run k-1 (blocks [0, ntail)) and the solve of run k (the rest) in one
// launch: both are latency bound and touch disjoint buffer sets, so they share the machine
// instead of running back to back.
__global__ __launch_bounds__(kTailThreads) void k_f8_tail_solve(TailArgs ta, int ntail,
                                                               SolveArgs sa) {
  if (static_cast<int>(blockIdx.x) < ntail) {
    cand_stats_block(ta, blockIdx.x, ntail);
  } else {
    const int h = (blockIdx.x - ntail) * kTailThreads + threadIdx.x;
    if (h < sa.H) solve_one(sa, h);
  }
}

hipError_t launch_f8_tail_solve(TailArgs *ta, SolveArgs *sa, hipStream_t s, int tail_cus) {
  int ntail = 0, nsolve = 0;
  TailArgs t{};
  SolveArgs v{};
  if (sa) {
    v = *sa;
    nsolve = (v.H + kTailThreads - 1) / kTailThreads;
  }
  if (ta) {
    t = *ta;
    // a solve workgroup (160 VGPRs) and a tail workgroup cannot share a CU, so the tail takes
    // the CUs the solve leaves free (>= 32 blocks) and every workgroup starts at once;
    // tail_blocks = 0 keeps the fixed 256-block split
    int nb = kSelectBlocks;
    if (tail_cus > 0) nb = std::min(kSelectBlocks, std::max(32, tail_cus - nsolve));
    t.per_block = (t.H + nb - 1) / nb;
    ntail = (t.H + t.per_block - 1) / t.per_block;
  }
  if (ntail + nsolve == 0) return hipSuccess;
  hipLaunchKernelGGL(k_f8_tail_solve, dim3(ntail + nsolve), dim3(kTailThreads), 0, s, t, ntail,
                     v);
  return hipGetLastError();
}

hipError_t launch_residuals(const Pt *pts, int n, const double *F, double *out,
                            hipStream_t s) {
  hipLaunchKernelGGL(k_residuals, dim3((n + 255) / 256), dim3(256), 0, s, pts, n, F, out);
  return hipGetLastError();
}

}  // namespace rsd
