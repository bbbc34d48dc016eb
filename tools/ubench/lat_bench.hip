// Dependent-chain latencies of the instructions a single-trajectory window of the parity
// parse is made of (one wave alone on the chip; s_memtime = shader cycles):
//   A  v_add_u32 chain                       B  four independent v_add_u32 streams
//   C  round v_cmp -> SGPR -> mbcnt lo/hi -> bitop3 -> v_cmp (the product's rej round)
//   D  round v_cmp -> SGPR -> mbcnt lo/hi (addend carries the threshold) -> v_cmp
//   E  VALU -> SGPR -> SALU (s_bcnt1, s_add) -> VALU (v_sub with the SGPR) round trip
//   F  D plus an s_cmp_lg_u64 / not-taken s_cbranch per round
//   G  D with the compare writing VCC (the mbcnt reading vcc_lo / vcc_hi)
//   H  two independent D chains interleaved (ILP across chains)
//   hipcc -O3 --offload-arch=gfx950 lat_bench.hip -o lat_bench && ./lat_bench
#include <hip/hip_runtime.h>
#include <cstdio>

#define R4(x) x x x x
#define R16(x) R4(x) R4(x) R4(x) R4(x)

template <int V>
__global__ __launch_bounds__(64) void k_lat(int iters, long long *out, unsigned *sink) {
  unsigned a = threadIdx.x, b = threadIdx.x * 3u, c = threadIdx.x * 5u, d = threadIdx.x * 7u;
  unsigned base = 100u - threadIdx.x, w = threadIdx.x * 0x9e3779b9u;
  unsigned long long s = 0;
  unsigned si = 1000u;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int k = 0; k < iters; ++k) {
    if constexpr (V == 0) {
      asm volatile(R16("v_add_u32 %0, %0, 1\n") : "+v"(a));
    } else if constexpr (V == 1) {
      asm volatile(R4("v_add_u32 %0, %0, 1\nv_add_u32 %1, %1, 1\nv_add_u32 %2, %2, 1\nv_add_u32 %3, %3, 1\n")
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    } else if constexpr (V == 2) {
      asm volatile(R16("v_cmp_gt_u32 s[40:41], %0, %1\n s_nop 1\n v_mbcnt_lo_u32_b32 %0, s40, %2\n"
                       " v_mbcnt_hi_u32_b32 %0, s41, %0\n v_bitop3_b32 %0, %0, %1, %2 bitop3:0xc8\n")
                   : "+v"(a), "+v"(w), "+v"(base) : : "s40", "s41");
    } else if constexpr (V == 3) {
      asm volatile(R16("v_cmp_gt_i32 s[40:41], 0, %0\n s_nop 1\n v_mbcnt_lo_u32_b32 %0, s40, %1\n"
                       " v_mbcnt_hi_u32_b32 %0, s41, %0\n")
                   : "+v"(a), "+v"(base) : : "s40", "s41");
    } else if constexpr (V == 4) {
      asm volatile(R16("v_cmp_gt_u32 s[40:41], %0, %1\n s_bcnt1_i32_b64 %2, s[40:41]\n s_add_u32 %2, %2, 7\n"
                       " v_sub_u32 %0, %2, %0\n")
                   : "+v"(a), "+v"(w), "+s"(si) : : "s40", "s41", "scc");
    } else if constexpr (V == 5) {
      asm volatile(R16("v_cmp_gt_i32 s[40:41], 0, %0\n s_nop 1\n v_mbcnt_lo_u32_b32 %0, s40, %1\n"
                       " v_mbcnt_hi_u32_b32 %0, s41, %0\n s_cmp_lg_u64 s[40:41], 0\n s_cbranch_scc0 1f\n1:\n")
                   : "+v"(a), "+v"(base) : : "s40", "s41", "scc");
    } else if constexpr (V == 6) {
      asm volatile(R16("v_cmp_gt_i32 vcc, 0, %0\n s_nop 1\n v_mbcnt_lo_u32_b32 %0, vcc_lo, %1\n"
                       " v_mbcnt_hi_u32_b32 %0, vcc_hi, %0\n")
                   : "+v"(a), "+v"(base) : : "vcc");
    } else if constexpr (V == 7) {
      asm volatile(R16("v_cmp_gt_i32 s[40:41], 0, %0\n v_cmp_gt_i32 s[42:43], 0, %2\n s_nop 0\n v_mbcnt_lo_u32_b32 %0, s40, %1\n"
                       " v_mbcnt_lo_u32_b32 %2, s42, %1\n v_mbcnt_hi_u32_b32 %0, s41, %0\n v_mbcnt_hi_u32_b32 %2, s43, %2\n")
                   : "+v"(a), "+v"(base), "+v"(b) : : "s40", "s41", "s42", "s43");
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[V] = t1 - t0;
  sink[threadIdx.x] = a + b + c + d + static_cast<unsigned>(s) + si + w;
}

int main() {
  long long *out;
  unsigned *sink;
  hipMalloc(&out, 16 * sizeof(long long));
  hipMalloc(&sink, 64 * sizeof(unsigned));
  const int iters = 4096;
  const char *names[] = {"A v_add chain (per instr)", "B 4 indep v_add (per instr)",
                         "C cmp-nop-mbcnt2-bitop3 round", "D cmp-nop-mbcnt2 round",
                         "E cmp-sbcnt-sadd-vsub round", "F D + s_cmp/s_cbranch",
                         "G D via vcc", "H two D chains interleaved (per round pair)"};
  const int per[] = {16, 16, 16, 16, 16, 16, 16, 16};
  long long h[16];
  for (int rep = 0; rep < 2; ++rep) {
    k_lat<0><<<1, 64>>>(iters, out, sink);
    k_lat<1><<<1, 64>>>(iters, out, sink);
    k_lat<2><<<1, 64>>>(iters, out, sink);
    k_lat<3><<<1, 64>>>(iters, out, sink);
    k_lat<4><<<1, 64>>>(iters, out, sink);
    k_lat<5><<<1, 64>>>(iters, out, sink);
    k_lat<6><<<1, 64>>>(iters, out, sink);
    k_lat<7><<<1, 64>>>(iters, out, sink);
    hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);
  }
  for (int v = 0; v < 8; ++v)
    printf("%-45s %7.2f cycles\n", names[v], static_cast<double>(h[v]) / (static_cast<double>(iters) * per[v]));
  return 0;
}
