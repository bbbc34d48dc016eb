// Workgroup residency probe: 512 workgroups of T threads, each spinning ~2 ms, with LDS bytes
// L; reports how many start within the first 100 us (resident at once) per configuration.
//   hipcc -O3 --offload-arch=gfx950 resid_bench.hip -o resid_bench && ./resid_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

template <int T, int LDSW>
__global__ __launch_bounds__(T) void k_spin(long long *out, long long spin) {
  __shared__ unsigned lds[LDSW];
  const long long t0 = __builtin_amdgcn_s_memrealtime();
  lds[threadIdx.x % LDSW] = threadIdx.x;
  __syncthreads();
  long long t = t0;
  unsigned acc = lds[(threadIdx.x + 1) % LDSW];
  while (t - t0 < spin) { acc = acc * 1664525u + 1013904223u; t = __builtin_amdgcn_s_memrealtime(); }
  if (threadIdx.x == 0) { out[2 * blockIdx.x] = t0; out[2 * blockIdx.x + 1] = acc; }
}

template <int T, int LDSW>
void run(const char *name, long long *d) {
  const int G = 512;
  k_spin<T, LDSW><<<G, T>>>(d, 200000);  // 2 ms at 100 MHz
  hipDeviceSynchronize();
  std::vector<long long> h(2 * G);
  hipMemcpy(h.data(), d, 16 * G, hipMemcpyDeviceToHost);
  long long mn = h[0];
  for (int b = 0; b < G; ++b) mn = std::min(mn, h[2 * b]);
  int early = 0;
  for (int b = 0; b < G; ++b) early += (h[2 * b] - mn) < 10000 ? 1 : 0;  // 100 us
  printf("%-28s threads %4d lds %6d B: %d of %d start at once\n", name, T, LDSW * 4, early, G);
}

int main() {
  long long *d;
  hipMalloc(&d, 16 * 512);
  run<1024, 64>("1024 threads, tiny LDS", d);
  run<1024, 8448>("1024 threads, 33 KB LDS", d);
  run<768, 64>("768 threads", d);
  run<512, 8448>("512 threads, 33 KB LDS", d);
  run<256, 64>("256 threads", d);
  return 0;
}
