// VALU issue-rate microbenchmark on gfx950: independent FMA chains per lane, with and
// without a wave-uniform (SGPR) operand, fp32 / packed fp32 / fp64.  Prints TFLOP/s.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITERS = 4096;

template <int CH>
__global__ __launch_bounds__(256) void k_f32(float *out, float a, const float *su) {
  float acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = threadIdx.x * 1e-3f + c;
  const float s = su[0];
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = fmaf(acc[c], a, s);
  }
  float r = 0;
  for (int c = 0; c < CH; ++c) r += acc[c];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <int CH>
__global__ __launch_bounds__(256) void k_f32v(float *out, float a) {  // all-VGPR operands
  float acc[CH], b[CH];
  for (int c = 0; c < CH; ++c) {
    acc[c] = threadIdx.x * 1e-3f + c;
    b[c] = threadIdx.x * 2e-3f - c;
  }
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = fmaf(acc[c], b[c], a);
  }
  float r = 0;
  for (int c = 0; c < CH; ++c) r += acc[c];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

typedef float float2v __attribute__((ext_vector_type(2)));
template <int CH>
__global__ __launch_bounds__(256) void k_pk(float *out, float a) {
  float2v acc[CH];
  const float2v av = {a, a * 0.5f};
  const float2v bv = {1e-3f, 2e-3f};
  for (int c = 0; c < CH; ++c) acc[c] = float2v{threadIdx.x * 1e-3f + c, (float)c};
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = __builtin_elementwise_fma(acc[c], av, bv);
  }
  float r = 0;
  for (int c = 0; c < CH; ++c) r += acc[c].x + acc[c].y;
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <int CH>
__global__ __launch_bounds__(256) void k_f64(double *out, double a, const double *su) {
  double acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = threadIdx.x * 1e-3 + c;
  const double s = su[0];
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = fma(acc[c], a, s);
  }
  double r = 0;
  for (int c = 0; c < CH; ++c) r += acc[c];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <class F>
void timeit(const char *name, F launch, double flops_per_thread, int blocks) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  launch();
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 10; ++r) launch();
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  ms /= 10;
  const double tf = flops_per_thread * blocks * 256.0 / (ms * 1e-3) / 1e12;
  printf("%-28s %8.3f ms  %8.2f TFLOP/s\n", name, ms, tf);
}

int main() {
  const int blocks = 256 * 8 * 4;  // 8 blocks of 4 waves per CU, 4 rounds
  float *o32;
  double *o64;
  float *s32;
  double *s64;
  hipMalloc(&o32, sizeof(float) * blocks * 256);
  hipMalloc(&o64, sizeof(double) * blocks * 256);
  hipMalloc(&s32, 64);
  hipMalloc(&s64, 64);
  hipMemset(s32, 0, 64);
  hipMemset(s64, 0, 64);
  timeit("f32 fma sgpr ch4", [&] { k_f32<4><<<blocks, 256>>>(o32, 0.999f, s32); }, 2.0 * ITERS * 4, blocks);
  timeit("f32 fma sgpr ch8", [&] { k_f32<8><<<blocks, 256>>>(o32, 0.999f, s32); }, 2.0 * ITERS * 8, blocks);
  timeit("f32 fma vgpr ch8", [&] { k_f32v<8><<<blocks, 256>>>(o32, 0.999f); }, 2.0 * ITERS * 8, blocks);
  timeit("f32 pk_fma ch4", [&] { k_pk<4><<<blocks, 256>>>(o32, 0.999f); }, 4.0 * ITERS * 4, blocks);
  timeit("f32 pk_fma ch8", [&] { k_pk<8><<<blocks, 256>>>(o32, 0.999f); }, 4.0 * ITERS * 8, blocks);
  timeit("f64 fma sgpr ch4", [&] { k_f64<4><<<blocks, 256>>>(o64, 0.999, s64); }, 2.0 * ITERS * 4, blocks);
  timeit("f64 fma sgpr ch8", [&] { k_f64<8><<<blocks, 256>>>(o64, 0.999, s64); }, 2.0 * ITERS * 8, blocks);
  return 0;
}
