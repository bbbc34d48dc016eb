// Cycles per 64-draw window of the tracking fast path (state kept in the top bucket of N = 2000:
// i is reset to 1999 whenever it drops below 1100), three formulations:
//   A: sure / ambiguous classification, ambiguous lanes resolved in order on the scalar unit
//   B: the same over 128-draw windows (two draws per lane)
//   C: fixed point of acc <- ballot(rank(acc) <= v) from sure | ambiguous
//   hipcc -O3 --offload-arch=gfx950 fast_bench.hip -o fast_bench && ./fast_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <vector>

__global__ void k_fill(uint32_t *w, int64_t n) {
  int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n) return;
  uint64_t x = 0x9e3779b97f4a7c15ull * (i + 1);
  x ^= x >> 31; x *= 0xbf58476d1ce4e5b9ull; x ^= x >> 27; x *= 0x94d049bb133111ebull; x ^= x >> 31;
  w[i] = static_cast<uint32_t>(x);
}

__device__ __forceinline__ uint32_t lane_rank(uint64_t bits) {
  return __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(bits >> 32),
                                   __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(bits), 0u));
}
__device__ __forceinline__ uint32_t uni(uint32_t v) {
  return static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(v)));
}

template <int V>
__global__ __launch_bounds__(64) void k_fast(const uint32_t *__restrict__ wp, int L, long long *out) {
  const int lane = threadIdx.x;
  __shared__ uint32_t lw[8192];
  for (int k = lane; k < 8192; k += 64) lw[k] = wp[k + blockIdx.x * 64];
  __syncthreads();
  uint32_t i = uni(1200 + (blockIdx.x * 7919u) % 700);
  long long amb_total = 0;
  const long long c0 = __builtin_amdgcn_s_memtime();
  constexpr int WW = V == 1 ? 128 : (V >= 3 ? 64 * (V - 1) : 64);
  uint32_t wn0 = lw[lane], wn1 = lw[64 + lane];
  constexpr int Q = V >= 3 ? V - 1 : 1;
  uint32_t wq[Q];
#pragma unroll
  for (int k = 0; k < Q; ++k) wq[k] = lw[64 * k + lane];
  for (int d = 0; d < L; d += WW) {
    const uint32_t w0 = wn0, w1 = wn1;
    wn0 = lw[(d + WW + lane) & 8191];
    if (V == 1) wn1 = lw[(d + WW + 64 + lane) & 8191];
    const uint32_t M = 2047u;
    if (V >= 3) {
      int vq[Q];
      uint64_t acc[Q];
#pragma unroll
      for (int k = 0; k < Q; ++k) {
        vq[k] = static_cast<int>(i) - static_cast<int>(wq[k] & M);
        wq[k] = lw[(d + WW + 64 * k + lane) & 8191];
        acc[k] = __ballot(vq[k] >= 0);
      }
      bool again;
      do {
        again = false;
        int base = 0;
        uint64_t nacc[Q];
#pragma unroll
        for (int k = 0; k < Q; ++k) {
          nacc[k] = __ballot(base + static_cast<int>(lane_rank(acc[k])) <= vq[k]);
          base += __popcll(acc[k]);
        }
#pragma unroll
        for (int k = 0; k < Q; ++k) {
          again |= nacc[k] != acc[k];
          acc[k] = nacc[k];
        }
        ++amb_total;
      } while (again);
      int tot = 0;
#pragma unroll
      for (int k = 0; k < Q; ++k) tot += __popcll(acc[k]);
      i -= tot;
    } else if (V == 0) {
      const int v = static_cast<int>(i) - static_cast<int>(w0 & M);
      uint64_t acc = __ballot(v >= lane);
      uint64_t amb = __ballot(v >= 0) & ~acc;
      amb_total += __popcll(amb);
      while (amb) {
        const int f = __ffsll(static_cast<long long>(amb)) - 1;
        const int rk = __popcll(acc & ((1ull << f) - 1ull));
        if (rk <= __builtin_amdgcn_readlane(v, f)) acc |= 1ull << f;
        amb &= amb - 1ull;
      }
      i -= __popcll(acc);
    } else if (V == 1) {
      const int v0 = static_cast<int>(i) - static_cast<int>(w0 & M);
      const int v1 = static_cast<int>(i) - static_cast<int>(w1 & M);
      uint64_t a0 = __ballot(v0 >= lane), a1 = __ballot(v1 >= lane + 64);
      uint64_t m0 = __ballot(v0 >= 0) & ~a0, m1 = __ballot(v1 >= 0) & ~a1;
      amb_total += __popcll(m0) + __popcll(m1);
      while (m0) {
        const int f = __ffsll(static_cast<long long>(m0)) - 1;
        const int rk = __popcll(a0 & ((1ull << f) - 1ull));
        if (rk <= __builtin_amdgcn_readlane(v0, f)) a0 |= 1ull << f;
        m0 &= m0 - 1ull;
      }
      const int p0 = __popcll(a0);
      while (m1) {
        const int f = __ffsll(static_cast<long long>(m1)) - 1;
        const int rk = p0 + __popcll(a1 & ((1ull << f) - 1ull));
        if (rk <= __builtin_amdgcn_readlane(v1, f)) a1 |= 1ull << f;
        m1 &= m1 - 1ull;
      }
      i -= p0 + __popcll(a1);
    } else {
      const int v = static_cast<int>(i) - static_cast<int>(w0 & M);
      uint64_t acc = __ballot(v >= 0), prev;
      do {
        prev = acc;
        acc = __ballot(static_cast<int>(lane_rank(prev)) <= v);
        ++amb_total;
      } while (acc != prev);
      i -= __popcll(acc);
    }
    if (i < 1100u) i = 1999u;
  }
  const long long c1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) {
    out[blockIdx.x * 4 + 0] = c1 - c0;
    out[blockIdx.x * 4 + 1] = amb_total;
    out[blockIdx.x * 4 + 2] = L / 64;  // 64-draw units
    out[blockIdx.x * 4 + 3] = i;
  }
}

template <int V>
void run(const uint32_t *dw, int L, int waves, long long *dout) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  k_fast<V><<<waves, 64>>>(dw, L, dout);
  (void)hipEventRecord(e0);
  k_fast<V><<<waves, 64>>>(dw, L, dout);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0; (void)hipEventElapsedTime(&ms, e0, e1);
  std::vector<long long> h(4 * waves);
  (void)hipMemcpy(h.data(), dout, 8 * h.size(), hipMemcpyDeviceToHost);
  double cyc = 0, amb = 0, win = 0;
  for (int b = 0; b < waves; ++b) { cyc += h[4 * b]; amb += h[4 * b + 1]; win += h[4 * b + 2]; }
  printf("V=%d waves=%5d: %.3f ms, %.1f cycles per 64 draws, %.2f amb (or rounds) per window, %.3g draws/s\n",
         V, waves, ms, cyc / win, amb / win * (V >= 3 ? V - 1 : (V == 1 ? 2 : 1)), (double)L * waves / (ms * 1e-3));
}

int main() {
  const int L = 1 << 18;
  uint32_t *dw; long long *dout;
  (void)hipMalloc(&dw, sizeof(uint32_t) * (8192 + 64 * 16384));
  (void)hipMalloc(&dout, sizeof(long long) * 4 * 16384);
  k_fill<<<(8192 + 64 * 16384 + 255) / 256, 256>>>(dw, 8192 + 64 * 16384);
  for (int waves : {256, 1024, 2048, 4096}) {
    run<0>(dw, L, waves, dout);
    run<1>(dw, L, waves, dout);
    run<2>(dw, L, waves, dout);
    run<3>(dw, L, waves, dout);
    run<5>(dw, L, waves, dout);
  }
  return 0;
}
