// The counting kernel's per-point instruction mix with all operands in registers (no memory):
// scalar fp32 (test32), packed fp32 (two hypotheses per lane), float64 (k_f8_count body).
// Prints points/s per chip and the implied cycles per wave-point at 2.4 GHz.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int NPT = 2048;

__global__ __launch_bounds__(256) void k_s32(const float *seed, int *out) {
  float f[9];
  for (int k = 0; k < 9; ++k) f[k] = seed[k] + threadIdx.x * 1e-6f;
  float x1 = seed[9], y1 = seed[10], x2 = seed[11], y2 = seed[12];
  const float thr2 = 1e-5f, K1 = 1e-5f, Ku = 6e-8f, K0 = 1e-10f;
  int cnt = 0;
  unsigned long long amb = 0;
  for (int i = 0; i < NPT; ++i) {
    x1 += 1e-4f; y2 -= 1e-4f;  // wave-uniform point changes (SALU-free: VGPR)
    const float l10 = fmaf(f[0], x2, fmaf(f[1], y2, f[2]));
    const float l11 = fmaf(f[3], x2, fmaf(f[4], y2, f[5]));
    const float l12 = fmaf(f[6], x2, fmaf(f[7], y2, f[8]));
    const float l20 = fmaf(f[0], x1, fmaf(f[3], y1, f[6]));
    const float l21 = fmaf(f[1], x1, fmaf(f[4], y1, f[7]));
    const float e = fmaf(l10, x1, fmaf(l11, y1, l12));
    const float n1 = fmaf(l10, l10, l11 * l11);
    const float n2 = fmaf(l20, l20, l21 * l21);
    const float ee = e * e, rhs = thr2 * fminf(n1, n2);
    const float d = ee - rhs;
    const float B = fmaf(fabsf(e), K1, fmaf(fmaf(rhs, 2.0f, ee), Ku, K0));
    cnt += (d < -B) ? 1 : 0;
    amb |= __ballot(fabsf(d) <= B);
  }
  out[blockIdx.x * 256 + threadIdx.x] = cnt + (int)(amb & 1);
}

__global__ __launch_bounds__(256) void k_pk(const float *seed, int *out) {
  f2 f[9];
  for (int k = 0; k < 9; ++k) f[k] = f2{seed[k] + threadIdx.x * 1e-6f, seed[k] - threadIdx.x * 1e-6f};
  float x1s = seed[9], y1s = seed[10], x2s = seed[11], y2s = seed[12];
  const f2 thr2 = 1e-5f, ka = 1e-3f, kb = 1e-7f, k0 = 1e-10f;
  int c0 = 0, c1 = 0;
  unsigned long long amb = 0;
  for (int i = 0; i < NPT; ++i) {
    x1s += 1e-4f; y2s -= 1e-4f;
    const f2 x1 = x1s, y1 = y1s, x2 = x2s, y2 = y2s;
    const f2 l10 = __builtin_elementwise_fma(f[0], x2, __builtin_elementwise_fma(f[1], y2, f[2]));
    const f2 l11 = __builtin_elementwise_fma(f[3], x2, __builtin_elementwise_fma(f[4], y2, f[5]));
    const f2 l12 = __builtin_elementwise_fma(f[6], x2, __builtin_elementwise_fma(f[7], y2, f[8]));
    const f2 l20 = __builtin_elementwise_fma(f[0], x1, __builtin_elementwise_fma(f[3], y1, f[6]));
    const f2 l21 = __builtin_elementwise_fma(f[1], x1, __builtin_elementwise_fma(f[4], y1, f[7]));
    const f2 e = __builtin_elementwise_fma(l10, x1, __builtin_elementwise_fma(l11, y1, l12));
    const f2 n1 = __builtin_elementwise_fma(l10, l10, l11 * l11);
    const f2 n2 = __builtin_elementwise_fma(l20, l20, l21 * l21);
    const f2 m = f2{fminf(n1.x, n2.x), fminf(n1.y, n2.y)};
    const f2 ee = e * e, rhs = thr2 * m, d = ee - rhs;
    const f2 B = __builtin_elementwise_fma(ee, ka, __builtin_elementwise_fma(rhs, kb, k0));
    c0 += (d.x < -B.x) ? 1 : 0;
    c1 += (d.y < -B.y) ? 1 : 0;
    amb |= __ballot(fabsf(d.x) <= B.x) | __ballot(fabsf(d.y) <= B.y);
  }
  out[blockIdx.x * 256 + threadIdx.x] = c0 + c1 + (int)(amb & 1);
}

__global__ __launch_bounds__(256) void k_d64(const double *seed, int *out) {
  double f[9];
  for (int k = 0; k < 9; ++k) f[k] = seed[k] + threadIdx.x * 1e-9;
  double x1 = seed[9], y1 = seed[10], x2 = seed[11], y2 = seed[12];
  int cnt = 0;
  for (int i = 0; i < NPT; ++i) {
    x1 += 1e-4; y2 -= 1e-4;
    const double l10 = fma(f[0], x2, fma(f[1], y2, f[2]));
    const double l11 = fma(f[3], x2, fma(f[4], y2, f[5]));
    const double l12 = fma(f[6], x2, fma(f[7], y2, f[8]));
    const double l20 = fma(f[0], x1, fma(f[3], y1, f[6]));
    const double l21 = fma(f[1], x1, fma(f[4], y1, f[7]));
    const double e = fma(l10, x1, fma(l11, y1, l12));
    const double n1 = fma(l10, l10, l11 * l11);
    const double n2 = fma(l20, l20, l21 * l21);
    cnt += (e * e < 2.25 * fmin(n1, n2)) ? 1 : 0;
  }
  out[blockIdx.x * 256 + threadIdx.x] = cnt;
}

template <class F>
void run(const char *name, F launch, int hyp_per_thread, int blocks) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  launch();
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  for (int r = 0; r < 10; ++r) launch();
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  ms /= 10;
  const double hp = (double)blocks * 256 * hyp_per_thread * NPT;  // hypothesis-points
  const double wave_pts = (double)blocks * 4 * NPT;
  printf("%-10s %7.3f ms  %8.3f Ghp/s  %6.1f cyc/wave-point/SIMD\n", name, ms, hp / ms / 1e6,
         ms * 1e-3 * 2.4e9 * 1024 / wave_pts);
}

int main() {
  const int blocks = 256 * 8 * 4;
  float *s32; double *s64; int *o;
  (void)hipMalloc(&s32, 64 * 4); (void)hipMalloc(&s64, 64 * 8); (void)hipMalloc(&o, blocks * 256 * 4);
  float h32[16]; double h64[16];
  for (int i = 0; i < 16; ++i) { h32[i] = 0.1f * (i + 1); h64[i] = 0.1 * (i + 1); }
  (void)hipMemcpy(s32, h32, sizeof(h32), hipMemcpyHostToDevice);
  (void)hipMemcpy(s64, h64, sizeof(h64), hipMemcpyHostToDevice);
  run("fp32", [&] { k_s32<<<blocks, 256>>>(s32, o); }, 1, blocks);
  run("pk32", [&] { k_pk<<<blocks, 256>>>(s32, o); }, 2, blocks);
  run("fp64", [&] { k_d64<<<blocks, 256>>>(s64, o); }, 1, blocks);
  return 0;
}
