// Single-trajectory parse, fixed windows, words prefetched in registers (independent of the
// state): V0 = k_np_track's track_one rules (256-draw two-bucket fixed point, 64-draw two-bucket
// fixed point, generic fixed point); V1 = 64-draw windows, one-bucket sure / ambiguous split
// (ambiguous lanes resolved in order on the scalar unit, fixed point over them if > kAmbSeq),
// else the 64-draw two-bucket fixed point, else generic.  Checked against a host parse.
//   hipcc -O3 --offload-arch=gfx950 amb_bench2.hip -o amb_bench2 && ./amb_bench2
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
__device__ __forceinline__ uint32_t wrap_state(int si, int n1) {
  return si > 0 ? static_cast<uint32_t>(si) : static_cast<uint32_t>(si + n1);
}

// generic window: fixed point from all-accept over wrapped states
__device__ __forceinline__ uint64_t generic(uint32_t w, uint32_t &i, int n1, long long &wraps) {
  uint64_t acc = ~0ull, prev;
  uint32_t sl;
  do {
    prev = acc;
    sl = wrap_state(static_cast<int>(i) - static_cast<int>(lane_rank(prev)), n1);
    acc = __ballot((w & (0xffffffffu >> __builtin_clz(sl))) <= sl);
  } while (acc != prev);
  wraps += __popcll(__ballot(sl == 1u) & acc);
  i = wrap_state(static_cast<int>(i) - static_cast<int>(__popcll(acc)), n1);
  return acc;
}

constexpr int kAmbSeq = 4;

template <int V>
__global__ __launch_bounds__(64) void k_run(const uint32_t *__restrict__ wp, int L, int n1,
                                            long long *out) {
  const int lane = threadIdx.x;
  uint32_t i = static_cast<uint32_t>(n1);
  long long wraps = 0, wins = 0;
  const long long c0 = __builtin_amdgcn_s_memtime();
  // register ring of 8 windows ahead
  constexpr int kAhead = 8;
  uint32_t ring[kAhead];
#pragma unroll
  for (int k = 0; k < kAhead; ++k) ring[k] = wp[64 * k + lane];
  int d = 0;
  while (d < L) {
    // windows d .. d + 64*kAhead are in the ring; consume them
#pragma unroll
    for (int k = 0; k < kAhead; ++k) {
      const uint32_t w = ring[k];
      ring[k] = wp[d + 64 * (kAhead + k) + lane];
      const uint32_t M = 0xffffffffu >> __builtin_clz(i);
      const uint32_t lowest = (M >> 1) + 1u;
      const uint32_t lowest2 = M > 1u ? (M >> 2) + 1u : 0x7fffffffu;
      if (V == 1 && i >= lowest + 63u) {
        const int v = static_cast<int>(i) - static_cast<int>(w & M);
        uint64_t acc = __ballot(v >= lane);
        uint64_t amb = __ballot(v >= 0) & ~acc;
        if (amb) {
          if (__popcll(amb) <= kAmbSeq) {
            do {
              const int f = __ffsll(static_cast<long long>(amb)) - 1;
              const int rk = __popcll(acc & ((1ull << f) - 1ull));
              if (rk <= __builtin_amdgcn_readlane(v, f)) acc |= 1ull << f;
              amb &= amb - 1ull;
            } while (amb);
          } else {
            acc |= amb;
            uint64_t prev;
            do {
              prev = acc;
              acc = __ballot(static_cast<int>(lane_rank(prev)) <= v);
            } while (acc != prev);
          }
        }
        i -= static_cast<uint32_t>(__popcll(acc));
      } else if (i >= lowest2 + 63u && lowest2 >= 1u) {
        const int c = static_cast<int>(i) - static_cast<int>(lowest);
        const int vh = static_cast<int>(i) - static_cast<int>(w & M);
        const int vl = static_cast<int>(i) - static_cast<int>(w & (M >> 1));
        uint64_t acc = __ballot(vh >= 0), prev;
        do {
          prev = acc;
          const int rk = static_cast<int>(lane_rank(prev));
          acc = __ballot(rk <= (rk <= c ? vh : vl));
        } while (acc != prev);
        i -= static_cast<uint32_t>(__popcll(acc));
      } else {
        (void)generic(w, i, n1, wraps);
      }
      ++wins;
    }
    d += 64 * kAhead;
  }
  const long long c1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) {
    out[blockIdx.x * 4 + 0] = c1 - c0;
    out[blockIdx.x * 4 + 1] = wins;
    out[blockIdx.x * 4 + 2] = wraps;
    out[blockIdx.x * 4 + 3] = i;
  }
}

int main() {
  const int L = 1 << 18;
  const int n1 = 1999;
  uint32_t *dw; long long *dout;
  hipMalloc(&dw, sizeof(uint32_t) * (L + 8192));
  hipMalloc(&dout, sizeof(long long) * 4 * 16384);
  k_fill<<<(L + 8192 + 255) / 256, 256>>>(dw, L + 8192);
  std::vector<uint32_t> hw(L + 8192);
  hipMemcpy(hw.data(), dw, 4 * hw.size(), hipMemcpyDeviceToHost);
  uint32_t s = n1; long long wr = 0;
  for (int t = 0; t < L; ++t) { uint32_t M = 0xffffffffu >> __builtin_clz(s); if ((hw[t] & M) <= s) { if (--s == 0) { s = n1; ++wr; } } }
  for (int v = 0; v < 2; ++v)
  for (int waves : {1, 512, 1024, 2048, 4096}) {
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    auto launch = [&] { if (v == 0) k_run<0><<<waves, 64>>>(dw, L, n1, dout); else k_run<1><<<waves, 64>>>(dw, L, n1, dout); };
    launch();
    hipEventRecord(e0); launch(); hipEventRecord(e1); hipEventSynchronize(e1);
    float ms = 0; hipEventElapsedTime(&ms, e0, e1);
    std::vector<long long> h(4 * waves);
    hipMemcpy(h.data(), dout, 8 * h.size(), hipMemcpyDeviceToHost);
    const bool ok = static_cast<uint32_t>(h[3]) == s && h[2] == wr;
    double cyc = 0;
    for (int b = 0; b < waves; ++b) cyc += h[4 * b];
    printf("V%d waves=%5d L=%d: %.3f ms, %.2f memtime/draw, %.2f ns/draw per wave, %.3g draws/s, %s\n", v, waves, L, ms,
           cyc / waves / L, ms * 1e6 / L, (double)L * waves / (ms * 1e-3), ok ? "exact" : "MISMATCH");
  }
  return 0;
}
