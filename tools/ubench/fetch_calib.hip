// FETCH_SIZE / WRITE_SIZE calibration per access shape (MI355X_MICROARCH.md "HBM": on gfx950
// FETCH_SIZE reports half the bytes of a 16-B-per-lane coalesced read; other widths are
// uncalibrated).  Each kernel streams a known number of bytes exactly once (a 1 GiB buffer, far
// beyond the 256 MiB Infinity Cache), in the access shapes of this repository's kernels:
//   k_cal_ld<uint>    4 B/lane coalesced loads      (k_np_* stream reads, k_f8_count32q F32soa)
//   k_cal_ld<uint2>   8 B/lane coalesced loads      (float64 SoA model loads)
//   k_cal_ld<uint4>  16 B/lane coalesced loads      (k_f8_count32q G4 float4 constants)
//   k_cal_lds        wave-uniform 64-B scalar loads (k_f8_count32q points, s_load_dwordx16)
//   k_cal_st<uint>    4 B/lane coalesced stores     (k_mt_stream words)
//   k_cal_st<uint4>  16 B/lane coalesced stores
// Run under rocprofv3 --pmc FETCH_SIZE (then WRITE_SIZE in a pass of its own); the program
// prints the bytes each kernel moves, tools/fetch_calib.py divides.
//   hipcc -O3 --offload-arch=gfx950 fetch_calib.hip -o fetch_calib
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

template <class T>
__device__ __forceinline__ unsigned fold(const T &v);
template <>
__device__ __forceinline__ unsigned fold<unsigned>(const unsigned &v) { return v; }
template <>
__device__ __forceinline__ unsigned fold<uint2>(const uint2 &v) { return v.x ^ v.y; }
template <>
__device__ __forceinline__ unsigned fold<uint4>(const uint4 &v) { return v.x ^ v.y ^ v.z ^ v.w; }

template <class T>
__global__ __launch_bounds__(256) void k_cal_ld(const T *__restrict__ p, size_t n,
                                                unsigned *__restrict__ sink) {
  unsigned acc = 0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += 256ull * gridDim.x) acc ^= fold(p[i]);
  if (acc == 0x9e3779b9u) sink[threadIdx.x] = acc;  // never true for the zero buffer: no store
}

// wave-uniform 64-byte rows (16 dwords) through the scalar data cache
__global__ __launch_bounds__(256) void k_cal_lds(const unsigned *__restrict__ p, size_t rows,
                                                 unsigned *__restrict__ sink) {
  const unsigned w = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  const unsigned nw = gridDim.x * 4;
  unsigned acc = 0;
  for (size_t r = w; r < rows; r += nw) {
    const unsigned *q = p + 16 * r;
#pragma unroll
    for (int k = 0; k < 16; ++k) acc ^= q[k];
  }
  if (acc == 0x9e3779b9u) sink[threadIdx.x] = acc;
}

template <class T>
__global__ __launch_bounds__(256) void k_cal_st(T *__restrict__ p, size_t n, T v) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += 256ull * gridDim.x) p[i] = v;
}

int main() {
  const size_t bytes = size_t(1) << 30;
  void *buf = nullptr;
  unsigned *sink = nullptr;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&sink, 4096));
  CK(hipMemset(buf, 0, bytes));
  CK(hipDeviceSynchronize());
  const int grid = 256 * 16;  // 16 workgroups of 256 per CU
  const int reps = 3;
  std::printf("{\"bytes_per_launch\": %zu, \"reps\": %d, \"kernels\": [", bytes, reps);
  const char *sep = "";
  for (int r = 0; r < reps; ++r) {
    k_cal_ld<unsigned><<<grid, 256>>>(static_cast<const unsigned *>(buf), bytes / 4, sink);
    k_cal_ld<uint2><<<grid, 256>>>(static_cast<const uint2 *>(buf), bytes / 8, sink);
    k_cal_ld<uint4><<<grid, 256>>>(static_cast<const uint4 *>(buf), bytes / 16, sink);
    k_cal_lds<<<grid, 256>>>(static_cast<const unsigned *>(buf), bytes / 64, sink);
    k_cal_st<unsigned><<<grid, 256>>>(static_cast<unsigned *>(buf), bytes / 4, 0u);
    k_cal_st<uint4><<<grid, 256>>>(static_cast<uint4 *>(buf), bytes / 16, make_uint4(0, 0, 0, 0));
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
  }
  const char *names[] = {"k_cal_ld<unsigned int>", "k_cal_ld<HIP_vector_type<unsigned int, 2u> >",
                         "k_cal_ld<HIP_vector_type<unsigned int, 4u> >", "k_cal_lds",
                         "k_cal_st<unsigned int>", "k_cal_st<HIP_vector_type<unsigned int, 4u> >"};
  const char *shape[] = {"load 4 B/lane", "load 8 B/lane", "load 16 B/lane",
                         "scalar load 64 B/wave (s_load_dwordx16)", "store 4 B/lane",
                         "store 16 B/lane"};
  for (int k = 0; k < 6; ++k) {
    std::printf("%s{\"kernel\": \"%s\", \"shape\": \"%s\"}", sep, names[k], shape[k]);
    sep = ", ";
  }
  std::printf("]}\n");
  CK(hipFree(buf));
  CK(hipFree(sink));
  return 0;
}
