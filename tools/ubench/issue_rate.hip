// Issue cost (SIMD cycles per wave64 instruction) of the instruction kinds in the counting
// kernels' inner loops on gfx950, with 8 waves per SIMD and 8 independent chains per wave.
// Each kernel runs a fixed inline-asm body (32 instructions per iteration); the clock comes
// from s_memtime / s_memrealtime inside the kernel, so cycles = time x clock / instructions.
//   hipcc -O3 --offload-arch=gfx950 issue_rate.hip -o issue_rate && ./issue_rate
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f2 __attribute__((ext_vector_type(2)));

#define X8(M) M(0) M(1) M(2) M(3) M(4) M(5) M(6) M(7)

enum Op {
  FMA_VVV, FMAC_S, PKFMA_VVV, PKFMA_S, PKMUL, PKADD_SEL, CMP_S, ADDC, AND, MIN, FMA64,
  NOPS
};
static const char *kNames[NOPS] = {
    "v_fma_f32 v,v,v,v",        "v_fmac_f32 v,s,v",           "v_pk_fma_f32 v,v,v,v",
    "v_pk_fma_f32 v,v,s,v",     "v_pk_mul_f32 v,v,v",         "v_pk_add_f32 v,s,v op_sel_hi",
    "v_cmp_lt_f32 s,v,v",       "v_addc_co_u32 v,s,0,v,s",    "v_and_b32 v,k,v",
    "v_min_f32 v,v,v",          "v_fma_f64 v,v,v,v"};
static const int kPerIter[NOPS] = {32, 32, 32, 32, 32, 32, 32, 32, 32, 32, 32};

template <int OP>
__global__ __launch_bounds__(256) void k_issue(float *out, long long *clk, int iters, float s0,
                                               float s1) {
  float a[8], b = threadIdx.x * 1e-7f, c = 1.0f + threadIdx.x * 1e-8f;
  f2 p[8], pb = {b, c}, pc = {c, b};
  double d[8], db = b, dc = c;
  unsigned long long m[8];
  int ci[8];
#define INIT(i)                          \
  a[i] = threadIdx.x * 1e-6f + i;        \
  p[i] = f2{a[i], a[i] * 0.5f};          \
  d[i] = a[i];                           \
  ci[i] = threadIdx.x + i;               \
  m[i] = 0x5555555555555555ull << i;
  X8(INIT)
  const f2 sp = {s0, s1};
  long long t0 = 0, r0 = 0;
  if (threadIdx.x == 0) {
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  for (int it = 0; it < iters; ++it) {
    if constexpr (OP == FMA_VVV) {
#define I(i) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
      X8(I) X8(I) X8(I) X8(I)
#undef I
    } else if constexpr (OP == FMAC_S) {
#define I(i) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(a[i]) : "s"(s0), "v"(c));
      X8(I) X8(I) X8(I) X8(I)
#undef I
    } else if constexpr (OP == PKFMA_VVV) {
#define I(i) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p[i]) : "v"(pb), "v"(pc));
      X8(I) X8(I) X8(I) X8(I)
#undef I
    } else if constexpr (OP == PKFMA_S) {
#define I(i) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p[i]) : "s"(sp), "v"(pc));
      X8(I) X8(I) X8(I) X8(I)
#undef I
    } else if constexpr (OP == PKMUL) {
#define I(i) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p[i]) : "v"(pb));
      X8(I) X8(I) X8(I) X8(I)
#undef I
    } else if constexpr (OP == PKADD_SEL) {
#define I(i) asm volatile("v_pk_add_f32 %0, %1, %0 op_sel_hi:[1,0]" : "+v"(p[i]) : "s"(sp));
      X8(I) X8(I) X8(I) X8(I)
#undef I
    } else if constexpr (OP == CMP_S) {
#define I(i) asm volatile("v_cmp_lt_f32 %0, %1, %2" : "=s"(m[i]) : "v"(a[i]), "v"(b));
      X8(I) X8(I) X8(I) X8(I)
#undef I
    } else if constexpr (OP == ADDC) {
#define I(i) \
  asm volatile("v_addc_co_u32 %0, %1, 0, %0, %2" : "+v"(ci[i]), "=s"(m[i]) : "s"(m[(i + 1) & 7]));
      X8(I) X8(I) X8(I) X8(I)
#undef I
    } else if constexpr (OP == AND) {
#define I(i) asm volatile("v_and_b32 %0, 0x7fffffff, %0" : "+v"(ci[i]));
      X8(I) X8(I) X8(I) X8(I)
#undef I
    } else if constexpr (OP == MIN) {
#define I(i) asm volatile("v_min_f32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
      X8(I) X8(I) X8(I) X8(I)
#undef I
    } else if constexpr (OP == FMA64) {
#define I(i) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(d[i]) : "v"(db), "v"(dc));
      X8(I) X8(I) X8(I) X8(I)
#undef I
    }
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    clk[0] = __builtin_amdgcn_s_memtime() - t0;
    clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
  float r = 0;
#define SUM(i) r += a[i] + p[i].x + p[i].y + (float)d[i] + (float)ci[i] + (float)(m[i] & 1);
  X8(SUM)
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <int OP>
void run(float *out, long long *clk, int cus, int waves_per_simd) {
  const int iters = 4000;
  const int blocks = cus * waves_per_simd;  // 256 threads = 4 waves = one per SIMD
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  k_issue<OP><<<blocks, 256>>>(out, clk, 10, 1.0f, 0.5f);
  hipEventRecord(e0);
  k_issue<OP><<<blocks, 256>>>(out, clk, iters, 1.0f, 0.5f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  long long h[2];
  hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost);
  const double ghz = (double)h[0] / (double)h[1] * 0.1;  // s_memrealtime is 100 MHz
  const double instr_per_simd = (double)waves_per_simd * iters * kPerIter[OP];
  const double cyc = ms * 1e-3 * ghz * 1e9 / instr_per_simd;
  printf("%-32s waves/SIMD %d  %.3f ms  clk %.2f GHz  %.2f cycles/instr\n", kNames[OP],
         waves_per_simd, ms, ghz, cyc);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
}

template <int OP>
void run_all(float *out, long long *clk, int cus) {
  run<OP>(out, clk, cus, 8);
  if (OP == FMA_VVV || OP == PKFMA_VVV || OP == PKFMA_S) run<OP>(out, clk, cus, 2);
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  float *out;
  long long *clk;
  hipMalloc(&out, sizeof(float) * cus * 8 * 256);
  hipMalloc(&clk, 16);
  run_all<FMA_VVV>(out, clk, cus);
  run_all<FMAC_S>(out, clk, cus);
  run_all<PKFMA_VVV>(out, clk, cus);
  run_all<PKFMA_S>(out, clk, cus);
  run_all<PKMUL>(out, clk, cus);
  run_all<PKADD_SEL>(out, clk, cus);
  run_all<CMP_S>(out, clk, cus);
  run_all<ADDC>(out, clk, cus);
  run_all<AND>(out, clk, cus);
  run_all<MIN>(out, clk, cus);
  run_all<FMA64>(out, clk, cus);
  return 0;
}
