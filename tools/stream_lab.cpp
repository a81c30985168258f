// HBM streaming ceilings on one MI355X for the BN-kernel access pattern
// (two 16-B loads + one 16-B store per thread per row): plain vs nontemporal
// loads / stores, 1 or 4 rows in flight, grid 2048 / 4096 / 16384 blocks.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/stream_lab.cpp -o tools/stream_lab
//   ./tools/stream_lab [MiB per operand]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NTL, bool NTS, int UR>
__global__ __launch_bounds__(256) void two_in_one_out(const u32x4* __restrict__ a,
                                                      const u32x4* __restrict__ b,
                                                      u32x4* __restrict__ o, long long n) {
  const long long step = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += UR * step) {
    u32x4 x[UR], y[UR];
#pragma unroll
    for (int u = 0; u < UR; ++u) {
      const long long j = i + u * step;
      if (j < n) {
        x[u] = NTL ? __builtin_nontemporal_load(a + j) : a[j];
        y[u] = NTL ? __builtin_nontemporal_load(b + j) : b[j];
      }
    }
#pragma unroll
    for (int u = 0; u < UR; ++u) {
      const long long j = i + u * step;
      if (j < n) {
        const u32x4 v = x[u] + y[u];
        if (NTS)
          __builtin_nontemporal_store(v, o + j);
        else
          o[j] = v;
      }
    }
  }
}

template <bool NTL, bool NTS>
__global__ __launch_bounds__(256) void copy_k(const u32x4* __restrict__ a, u32x4* __restrict__ o,
                                              long long n) {
  const long long step = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += step) {
    const u32x4 v = NTL ? __builtin_nontemporal_load(a + i) : a[i];
    if (NTS)
      __builtin_nontemporal_store(v, o + i);
    else
      o[i] = v;
  }
}

template <typename F>
float timeit(F f) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int r = 0; r < 3; ++r) f();
  CK(hipEventRecord(e0, 0));
  const int reps = 20;
  for (int r = 0; r < reps; ++r) f();
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipGetLastError());
  return ms * 1e3f / reps;
}

int main(int argc, char** argv) {
  const long long mib = argc > 1 ? std::atoll(argv[1]) : 1568;  // ~ a 1024x56x56x256 bf16 tensor
  const long long bytes = mib << 20, n = bytes / 16;
  u32x4 *a, *b, *o;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMalloc(&o, bytes));
  CK(hipMemset(a, 1, bytes));
  CK(hipMemset(b, 2, bytes));
  for (int grid : {2048, 4096, 16384}) {
#define RUN2(NTL, NTS, UR)                                                                  \
  {                                                                                         \
    const float us = timeit([&] {                                                           \
      hipLaunchKernelGGL((two_in_one_out<NTL, NTS, UR>), dim3(grid), dim3(256), 0, 0, a, b, \
                         o, n);                                                             \
    });                                                                                     \
    std::printf("2-in-1-out grid %5d  nt-load %d nt-store %d  rows/iter %d: %8.1f us %5.2f TB/s\n", \
                grid, NTL, NTS, UR, us, 3.0 * bytes / us / 1e6);                            \
  }
    RUN2(false, false, 1)
    RUN2(false, true, 1)
    RUN2(true, false, 1)
    RUN2(true, true, 1)
    RUN2(false, false, 4)
    RUN2(false, true, 4)
#define RUNC(NTL, NTS)                                                                       \
  {                                                                                          \
    const float us = timeit(                                                                 \
        [&] { hipLaunchKernelGGL((copy_k<NTL, NTS>), dim3(grid), dim3(256), 0, 0, a, o, n); }); \
    std::printf("copy       grid %5d  nt-load %d nt-store %d:              %8.1f us %5.2f TB/s\n", \
                grid, NTL, NTS, us, 2.0 * bytes / us / 1e6);                                 \
  }
    RUNC(false, false)
    RUNC(false, true)
    RUNC(true, true)
  }
  return 0;
}
