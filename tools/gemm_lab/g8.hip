// GEMM lab: the 256x256x64 phased bf16 MFMA core that the implicit-GEMM
// convolution kernels build on, as a plain dense GEMM (C = A . B^T,
// A [M][K], B [N][K] bf16 row-major) so the main loop can be measured and
// checked in isolation on random data.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o g8 g8.hip && ./g8 [M N K reps]
//
// Structure (cdna_hip_programming.md §5 "the 256^2 phased template", derived
// here for K-halves instead of row halves):
//   * block 512 threads = 8 waves, 2 (M) x 4 (N); wave tile 128 x 64;
//     v_mfma_f32_16x16x32_bf16 (acc 8 x 4 fragments = 128 VGPRs);
//   * a K-tile (64 k) is staged as four 16 KB PIECES: (A, k 0-31), (B, k 0-31),
//     (A, k 32-63), (B, k 32-63), each [256 rows][64 B], filled by
//     global_load_lds_dwordx4 (2 per thread); two LDS buffers (128 KB);
//   * 4 phases per K-tile, 16 MFMAs each: (k0, rows 0-63), (k0, rows 64-127),
//     (k1, rows 0-63), (k1, rows 64-127) of the wave tile; phase p issues piece
//     p of the NEXT K-tile, and prefetches the next phase's fragments into the
//     other register set while its own MFMAs run;
//   * counted vmcnt(4) + one raw s_barrier at phases 1 and 3 only: two pieces
//     (4 DMAs per wave) stay in flight across every barrier;
//   * LDS image: 64-B rows, 16-B chunk c of row r stored at slot c ^ f(r),
//     f = {0,2,3,1}[(r>>2)&3]: conflict-free ds_read_b128 for the 16x16x32
//     operand map (lane l: row l&15, chunk l>>4) over all four lane groups.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

namespace {

#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void glds16(const void* src, const void* lds_dst) {
  const uint32_t base = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)lds_dst);
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(base)
               : "m0");
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void barrier() {
  asm volatile("s_barrier" ::: "memory");
}

__device__ __forceinline__ f32x4 mfma16(const uint4& a, const uint4& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

__device__ __forceinline__ int swz(int r) {  // r: row within its 16-row block
  return (0x1320 >> (4 * ((r >> 2) & 3))) & 3;  // {0,2,3,1}
}

__device__ __forceinline__ uint4 lds_read16(const unsigned char* p) {
  return *reinterpret_cast<const uint4*>(p);
}

__device__ __forceinline__ int xcd_linear(int L, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int x = L & 7, i = L >> 3;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

constexpr int BM = 256, BN = 256, NTH = 512;
constexpr int PIECE = 16384;          // 256 rows x 64 B
constexpr int BUF = 4 * PIECE;        // one K-tile
constexpr int LDS_BYTES = 2 * BUF;    // two K-tiles

template <int V>
__global__ __launch_bounds__(NTH, 1) void g8_kernel(const uint16_t* __restrict__ A,
                                                    const uint16_t* __restrict__ B,
                                                    float* __restrict__ C, int M, int N, int K,
                                                    int m_tiles) {
  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 2, wn = wave & 3;
  const int L = xcd_linear(blockIdx.x, gridDim.x);
  const int mt = L % m_tiles, nt = L / m_tiles;
  const int m0 = mt * BM, n0 = nt * BN;
  const int NT = K / 64;
  (void)NT;

  // loader: instruction i (0,1) of wave w covers piece rows (i*8 + w)*16 .. +16;
  // lane l -> row (l>>2), LDS slot l&3 holding global chunk (l&3) ^ swz(row)
  const int lrow = lane >> 2, lslot = lane & 3;
  const int gch = lslot ^ swz(lrow);
  const unsigned char* a_src[2];
  const unsigned char* b_src[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = (i * 8 + wave) * 16 + lrow;
    a_src[i] = reinterpret_cast<const unsigned char*>(A) + ((long long)(m0 + r) * K) * 2 + gch * 16;
    b_src[i] = reinterpret_cast<const unsigned char*>(B) + ((long long)(n0 + r) * K) * 2 + gch * 16;
  }
  auto issue = [&](int t, int p) {  // piece p of K-tile t
    unsigned char* dst = smem + (t & 1) * BUF + p * PIECE;
    const int koff = t * 128 + (p >> 1) * 64;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      glds16(((p & 1) ? b_src[i] : a_src[i]) + koff, dst + (i * 8 + wave) * 1024);
  };

  // fragment read offset of this lane inside any 16-row block
  const int foff = (lane & 15) * 64 + (((lane >> 4) ^ swz(lane & 15)) << 4);
  const int a_row0 = wm * 128, b_row0 = wn * 64;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  uint4 a1[4], a2[4], b1[4], b2[4];
  auto readA = [&](uint4 (&dst)[4], int t, int kh, int mh) {
    const unsigned char* base = smem + (t & 1) * BUF + (kh * 2) * PIECE + (a_row0 + mh * 64) * 64 + foff;
#pragma unroll
    for (int i = 0; i < 4; ++i) dst[i] = lds_read16(base + i * 1024);
  };
  auto readB = [&](uint4 (&dst)[4], int t, int kh) {
    const unsigned char* base = smem + (t & 1) * BUF + (kh * 2 + 1) * PIECE + b_row0 * 64 + foff;
#pragma unroll
    for (int j = 0; j < 4; ++j) dst[j] = lds_read16(base + j * 1024);
  };
  auto mma = [&](const uint4 (&a)[4], const uint4 (&b)[4], int mh) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[mh * 4 + i][j] = mfma16(a[i], b[j], acc[mh * 4 + i][j]);
    __builtin_amdgcn_s_setprio(0);
  };

  if constexpr (V == 1) {
    // prologue: K-tile 0, pieces 0..3; pieces 0,1 landed before the first reads
  #pragma unroll
    for (int p = 0; p < 4; ++p) issue(0, p);
    wait_vmcnt<4>();
    barrier();
    readA(a1, 0, 0, 0);
    readB(b1, 0, 0);

    for (int t = 0; t < NT; ++t) {
      const bool more = t + 1 < NT;
      // phase 0: (k0, rows 0-63) with a1 b1; prefetch A(k0, rows 64-127)
      if (more) issue(t + 1, 0);
      readA(a2, t, 0, 1);
      __builtin_amdgcn_sched_barrier(0);
      mma(a1, b1, 0);
      __builtin_amdgcn_sched_barrier(0);
      // phase 1: (k0, rows 64-127) with a2 b1; prefetch the k1 fragments
      // (pieces 2,3 of K-tile t: retire them, then the barrier)
      if (more) {
        issue(t + 1, 1);
        wait_vmcnt<4>();
      } else {
        wait_vmcnt<0>();
      }
      barrier();
      readA(a1, t, 1, 0);
      readB(b2, t, 1);
      __builtin_amdgcn_sched_barrier(0);
      mma(a2, b1, 1);
      __builtin_amdgcn_sched_barrier(0);
      // phase 2: (k1, rows 0-63) with a1 b2; prefetch A(k1, rows 64-127)
      if (more) issue(t + 1, 2);
      readA(a2, t, 1, 1);
      __builtin_amdgcn_sched_barrier(0);
      mma(a1, b2, 0);
      __builtin_amdgcn_sched_barrier(0);
      // phase 3: (k1, rows 64-127) with a2 b2; prefetch K-tile t+1's phase-0
      // fragments (its pieces 0,1)
      if (more) {
        issue(t + 1, 3);
        wait_vmcnt<4>();
        barrier();
        readA(a1, t + 1, 0, 0);
        readB(b1, t + 1, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      mma(a2, b2, 1);
      __builtin_amdgcn_sched_barrier(0);
    }

  } else if constexpr (V == 3) {
    // V3: ping-pong.  Waves 0-3 (rows 0-127) and 4-7 (rows 128-255) form two
    // groups, one wave of each per SIMD; group 1 runs one s_barrier behind
    // group 0, so while one group's wave issues its 16 MFMAs the other
    // group's wave on the same SIMD reads its fragments and issues its DMA
    // (cdna_hip_programming.md, the 256^2 template's staggered groups).
    // Phase (t, p): k-half kh = p>>1, row half mh = p&1; reads its own
    // fragments, issues piece p of K-tile t+1, s_barrier, lgkmcnt(0), MFMAs,
    // s_barrier.  A piece is retired by a counted vmcnt at the START of the
    // phase BEFORE the one that reads it (one barrier more than unstaggered).
    const int grp = __builtin_amdgcn_readfirstlane(wave >> 2);  // scalar branch around s_barrier
    uint4 af[4], bfv[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) issue(0, p);
    wait_vmcnt<4>();
    barrier();
    if (grp == 1) barrier();  // stagger
    for (int t = 0; t < NT; ++t) {
      const bool more = t + 1 < NT;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const int kh = p >> 1, mh = p & 1;
        if (p == 1) {
          if (more) wait_vmcnt<2>(); else wait_vmcnt<0>();
        }
        if (p == 3 && more) wait_vmcnt<2>();
        readA(af, t, kh, mh);
        if (mh == 0) readB(bfv, t, kh);
        if (more) issue(t + 1, p);
        barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        mma(af, bfv, mh);
        __builtin_amdgcn_sched_barrier(0);
        barrier();
      }
    }
    if (grp == 0) barrier();  // same barrier count in both groups
  } else {
    // V2: a ring of 4 half-tile slot pairs (A, B pieces of 32 k each): half-
    // tile h computes in phases 2h (rows 0-63) and 2h+1 (rows 64-127); A_j is
    // issued after the barrier of phase 2j-5, B_j in phase 2j-4, so every
    // piece has 3-4 phases to land (vs 2); a slot pair is refilled once the
    // barrier two phases after its last fragment read has passed.
    const int NH = 2 * NT;
    auto issueA = [&](int j) {
      unsigned char* dst = smem + (j & 3) * (2 * PIECE);
      const int koff = (j >> 1) * 128 + (j & 1) * 64;
#pragma unroll
      for (int i = 0; i < 2; ++i) glds16(a_src[i] + koff, dst + (i * 8 + wave) * 1024);
    };
    auto issueB = [&](int j) {
      unsigned char* dst = smem + (j & 3) * (2 * PIECE) + PIECE;
      const int koff = (j >> 1) * 128 + (j & 1) * 64;
#pragma unroll
      for (int i = 0; i < 2; ++i) glds16(b_src[i] + koff, dst + (i * 8 + wave) * 1024);
    };
    auto rdA = [&](uint4 (&dst)[4], int h, int mh) {
      const unsigned char* base = smem + (h & 3) * (2 * PIECE) + (a_row0 + mh * 64) * 64 + foff;
#pragma unroll
      for (int i = 0; i < 4; ++i) dst[i] = lds_read16(base + i * 1024);
    };
    auto rdB = [&](uint4 (&dst)[4], int h) {
      const unsigned char* base = smem + (h & 3) * (2 * PIECE) + PIECE + b_row0 * 64 + foff;
#pragma unroll
      for (int j = 0; j < 4; ++j) dst[j] = lds_read16(base + j * 1024);
    };
    // pieces issued after B_j (A_{j+1}.. up to what the schedule has issued)
    // prologue: A0 B0 A1 B1 A2
    issueA(0);
    issueB(0);
    if (NH > 1) { issueA(1); issueB(1); }
    if (NH > 2) issueA(2);
    if (NH > 2) wait_vmcnt<6>(); else if (NH > 1) wait_vmcnt<4>(); else wait_vmcnt<0>();
    barrier();
    rdA(a1, 0, 0);
    rdB(b1, 0);
    for (int h = 0; h < NH; h += 2) {
      // ---- half-tile h (b1), then h+1 (b2)
      // phase 2h
      if (h + 2 < NH) issueB(h + 2);
      rdA(a2, h, 1);
      __builtin_amdgcn_sched_barrier(0);
      mma(a1, b1, 0);
      __builtin_amdgcn_sched_barrier(0);
      // phase 2h+1: half-tile h+1 must have landed (NH is even: h+1 exists)
      if (h + 2 < NH) wait_vmcnt<4>(); else wait_vmcnt<0>();
      barrier();
      if (h + 3 < NH) issueA(h + 3);
      rdA(a1, h + 1, 0);
      rdB(b2, h + 1);
      __builtin_amdgcn_sched_barrier(0);
      mma(a2, b1, 1);
      __builtin_amdgcn_sched_barrier(0);
      // phase 2h+2
      if (h + 3 < NH) issueB(h + 3);
      rdA(a2, h + 1, 1);
      __builtin_amdgcn_sched_barrier(0);
      mma(a1, b2, 0);
      __builtin_amdgcn_sched_barrier(0);
      // phase 2h+3
      if (h + 2 < NH) {
        if (h + 3 < NH) wait_vmcnt<4>(); else wait_vmcnt<0>();
        barrier();
        if (h + 4 < NH) issueA(h + 4);
        rdA(a1, h + 2, 0);
        rdB(b1, h + 2);
      }
      __builtin_amdgcn_sched_barrier(0);
      mma(a2, b2, 1);
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  // epilogue: lane holds D[4*(l>>4)+r][l&15] of each 16x16 block
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + a_row0 + i * 16 + 4 * (lane >> 4) + r;
        const int n = n0 + b_row0 + j * 16 + (lane & 15);
        C[(long long)m * N + n] = acc[i][j][r];
      }
}

__global__ void ref_kernel(const uint16_t* A, const uint16_t* B, float* C, int M, int N, int K,
                           int rows) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  const int m = blockIdx.y;
  if (n >= N || m >= rows) return;
  float s = 0.f;
  for (int k = 0; k < K; ++k)
    s += __uint_as_float((uint32_t)A[(long long)m * K + k] << 16) *
         __uint_as_float((uint32_t)B[(long long)n * K + k] << 16);
  C[(long long)m * N + n] = s;
}

__global__ void fill_kernel(uint16_t* p, long long n, uint32_t seed) {
  long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  for (; i < n; i += (long long)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    const float f = ((x & 0xFFFFFF) / 8388608.0f) - 1.0f;  // [-1, 1)
    p[i] = (uint16_t)(__float_as_uint(f) >> 16);
  }
}

}  // namespace

int main(int argc, char** argv) {
  int M = argc > 1 ? atoi(argv[1]) : 8192;
  int N = argc > 2 ? atoi(argv[2]) : 8192;
  int K = argc > 3 ? atoi(argv[3]) : 8192;
  int reps = argc > 4 ? atoi(argv[4]) : 20;
  if (M % BM || N % BN || K % 64) {
    fprintf(stderr, "M, N multiples of 256, K of 64\n");
    return 2;
  }
  uint16_t *A, *B;
  float *C, *R;
  CHECK(hipMalloc(&A, (size_t)M * K * 2));
  CHECK(hipMalloc(&B, (size_t)N * K * 2));
  CHECK(hipMalloc(&C, (size_t)M * N * 4));
  const int rows = 64;
  CHECK(hipMalloc(&R, (size_t)rows * N * 4));
  fill_kernel<<<1024, 256>>>(A, (long long)M * K, 17u);
  fill_kernel<<<1024, 256>>>(B, (long long)N * K, 91u);
  CHECK(hipFuncSetAttribute((const void*)g8_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            LDS_BYTES));
  CHECK(hipFuncSetAttribute((const void*)g8_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            LDS_BYTES));
  const int m_tiles = M / BM, tiles = m_tiles * (N / BN);
  int rc_all = 0;
  CHECK(hipFuncSetAttribute((const void*)g8_kernel<3>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            LDS_BYTES));
  for (int v = 1; v <= 3; ++v) {
  auto run = [&]() {
    if (v == 1) g8_kernel<1><<<tiles, NTH, LDS_BYTES>>>(A, B, C, M, N, K, m_tiles);
    else if (v == 2) g8_kernel<2><<<tiles, NTH, LDS_BYTES>>>(A, B, C, M, N, K, m_tiles);
    else g8_kernel<3><<<tiles, NTH, LDS_BYTES>>>(A, B, C, M, N, K, m_tiles);
  };
  CHECK(hipMemset(C, 0, (size_t)M * N * 4));
  run();
  CHECK(hipDeviceSynchronize());
  // check the first `rows` rows and a band in the last tile row
  ref_kernel<<<dim3((N + 255) / 256, rows), 256>>>(A, B, R, M, N, K, rows);
  CHECK(hipDeviceSynchronize());
  std::vector<float> hc((size_t)rows * N), hr((size_t)rows * N);
  CHECK(hipMemcpy(hc.data(), C, hc.size() * 4, hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(hr.data(), R, hr.size() * 4, hipMemcpyDeviceToHost));
  double maxerr = 0, maxref = 0;
  for (size_t i = 0; i < hc.size(); ++i) {
    maxerr = fmax(maxerr, fabs((double)hc[i] - hr[i]));
    maxref = fmax(maxref, fabs((double)hr[i]));
  }
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) run();
  CHECK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) run();
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / reps;
  const double tf = 2.0 * M * N * K / (us * 1e-6) / 1e12;
  printf("g8 v%d M=%d N=%d K=%d: %.1f us  %.0f TF/s  maxerr %.3g (max |ref| %.3g) %s\n", v, M, N,
         K, us, tf, maxerr, maxref, maxerr <= 1e-3 * maxref + 1e-2 ? "OK" : "MISMATCH");
  if (!(maxerr <= 1e-3 * maxref + 1e-2)) rc_all = 1;
  }
  return rc_all;
}
