// Latency / throughput of the tracking window step (np_sampler.hip k_np_track): one trajectory
// per wave over L draws, windows of 64*Q draws, fixed-point accept mask.  Reports cycles per
// window (s_memtime), fixed-point rounds per window and draws per second.
//   hipcc -O3 --offload-arch=gfx950 track_bench.hip -o track_bench && ./track_bench
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

template <int Q>
__global__ __launch_bounds__(64) void k_track(const uint32_t *__restrict__ wp, int L, int n1,
                                              long long *out) {
  const int lane = threadIdx.x;
  uint32_t i = 1 + (blockIdx.x * 7919u) % n1;
  long long rounds = 0, wins = 0;
  const long long c0 = __builtin_amdgcn_s_memtime();
  uint32_t wn[Q];
#pragma unroll
  for (int k = 0; k < Q; ++k) wn[k] = wp[64 * k + lane];
  for (int d = 0; d < L; d += 64 * Q) {
    uint32_t w[Q];
#pragma unroll
    for (int k = 0; k < Q; ++k) { w[k] = wn[k]; wn[k] = wp[d + 64 * (Q + k) + lane]; }
    uint64_t acc[Q], prev[Q];
#pragma unroll
    for (int k = 0; k < Q; ++k) acc[k] = ~0ull;
    uint32_t sl[Q];
    bool again;
    do {
      int base = static_cast<int>(i);
#pragma unroll
      for (int k = 0; k < Q; ++k) {
        prev[k] = acc[k];
        int si = base - static_cast<int>(lane_rank(acc[k]));
        sl[k] = si > 0 ? si : si + n1;
        base -= static_cast<int>(__popcll(acc[k]));
      }
      again = false;
#pragma unroll
      for (int k = 0; k < Q; ++k) {
        acc[k] = __ballot((w[k] & (0xffffffffu >> __builtin_clz(sl[k]))) <= sl[k]);
        again |= acc[k] != prev[k];
      }
      ++rounds;
    } while (again);
    int acnt = 0;
#pragma unroll
    for (int k = 0; k < Q; ++k) acnt += __popcll(acc[k]);
    int si = static_cast<int>(i) - acnt;
    i = si > 0 ? si : si + n1;
    ++wins;
  }
  const long long c1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) {
    out[blockIdx.x * 4 + 0] = c1 - c0;
    out[blockIdx.x * 4 + 1] = rounds;
    out[blockIdx.x * 4 + 2] = wins;
    out[blockIdx.x * 4 + 3] = i;
  }
}


// Variant: initial guess acc0 = lanes accepted under s_l = i - floor(l * p), p = previous
// window's acceptance rate (numerically: the previous window's accept count / 64); the mask
// from the bucket of i or the one below (states >= 64 assumed for the benchmark).
__global__ __launch_bounds__(64) void k_track_g(const uint32_t *__restrict__ wp, int L, int n1,
                                                long long *out) {
  const int lane = threadIdx.x;
  uint32_t i = 1 + (blockIdx.x * 7919u) % n1;
  long long rounds = 0, wins = 0;
  const long long c0 = __builtin_amdgcn_s_memtime();
  uint32_t wn = wp[lane];
  int pa = 48;  // accepts in the previous window
  for (int d = 0; d < L; d += 64) {
    const uint32_t w = wn;
    wn = wp[d + 64 + lane];
    // guess: lane l accepted iff floor((l+1) pa / 64) > floor(l pa / 64)
    uint64_t acc = __ballot(((lane + 1) * pa >> 6) > (lane * pa >> 6)), prev;
    uint32_t sl;
    do {
      prev = acc;
      int si = static_cast<int>(i) - static_cast<int>(lane_rank(acc));
      sl = si > 0 ? si : si + n1;
      acc = __ballot((w & (0xffffffffu >> __builtin_clz(sl))) <= sl);
      ++rounds;
    } while (acc != prev);
    pa = __popcll(acc);
    int si = static_cast<int>(i) - pa;
    i = si > 0 ? si : si + n1;
    ++wins;
  }
  const long long c1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) {
    out[blockIdx.x * 4 + 0] = c1 - c0;
    out[blockIdx.x * 4 + 1] = rounds;
    out[blockIdx.x * 4 + 2] = wins;
    out[blockIdx.x * 4 + 3] = i;
  }
}

void run_g(const uint32_t *dw, int L, int waves, long long *dout) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  k_track_g<<<waves, 64>>>(dw, L, 1999, dout);
  hipEventRecord(e0);
  k_track_g<<<waves, 64>>>(dw, L, 1999, dout);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0; hipEventElapsedTime(&ms, e0, e1);
  std::vector<long long> h(4 * waves);
  hipMemcpy(h.data(), dout, 8 * h.size(), hipMemcpyDeviceToHost);
  double cyc = 0, rnd = 0, win = 0;
  for (int b = 0; b < waves; ++b) { cyc += h[4 * b]; rnd += h[4 * b + 1]; win += h[4 * b + 2]; }
  printf("G   waves=%5d L=%d: %.3f ms, %.1f cycles/window, %.2f rounds/window, %.1f cycles/round, %.3g draws/s\n",
         waves, L, ms, cyc / win, rnd / win, cyc / rnd, (double)L * waves / (ms * 1e-3));
}

template <int Q>
void run(const uint32_t *dw, int L, int waves, long long *dout) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  k_track<Q><<<waves, 64>>>(dw, L, 1999, dout);  // warm
  hipEventRecord(e0);
  k_track<Q><<<waves, 64>>>(dw, L, 1999, dout);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0; hipEventElapsedTime(&ms, e0, e1);
  std::vector<long long> h(4 * waves);
  hipMemcpy(h.data(), dout, 8 * h.size(), hipMemcpyDeviceToHost);
  double cyc = 0, rnd = 0, win = 0;
  for (int b = 0; b < waves; ++b) { cyc += h[4 * b]; rnd += h[4 * b + 1]; win += h[4 * b + 2]; }
  printf("Q=%d waves=%5d L=%d: %.3f ms, %.1f cycles/window, %.2f rounds/window, %.1f cycles/round, %.3g draws/s\n",
         Q, waves, L, ms, cyc / win, rnd / win, cyc / rnd, (double)L * waves / (ms * 1e-3));
}

int main() {
  const int L = 1 << 18;
  uint32_t *dw; long long *dout;
  hipMalloc(&dw, sizeof(uint32_t) * (L + 4096));
  hipMalloc(&dout, sizeof(long long) * 4 * 16384);
  k_fill<<<(L + 4096 + 255) / 256, 256>>>(dw, L + 4096);
  for (int waves : {256, 1024, 2048, 4096, 8192}) {
    run<1>(dw, L, waves, dout);
    run<2>(dw, L, waves, dout);
    run<4>(dw, L, waves, dout);
    run_g(dw, L, waves, dout);
  }
  return 0;
}
