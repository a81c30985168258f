// Depthwise KxK convolution on NHWC bf16 activations (QuickNet stem and
// blur-pool transitions).  MIOpen falls back to naive/grouped kernels for
// depthwise NHWC bf16, which made these the slowest ops in QuickNetLarge.
//
// Depthwise conv has no reduction over channels, so it is pure bandwidth:
// every kernel maps one thread to 8 channels (one 16-B vector) of one pixel
// and keeps fp32 accumulators.  Weights are fp32 [C][K*K] (the physical
// layout of a (C,1,K,K) parameter in both contiguous and channels_last
// formats); forward/dgrad stage them transposed [K*K][C] in LDS so each tap
// is one broadcast-free vector read.
//
//   zk_dw_fwd    y[b,ho,wo,c]  = sum_t x[b, ho*s-pt+kh, wo*s-pl+kw, c] * w[c,t]
//   zk_dw_dgrad  dx[b,h,w,c]   = sum_t dy[b,(h+pt-kh)/s,(w+pl-kw)/s,c] * w[c,t]
//                                (gather form, only exact stride multiples)
//   zk_dw_wgrad  dw[c,t]      += sum_{b,ho,wo} dy[b,ho,wo,c] * x[b,hi,wi,c]
//                                (block-level LDS reduction, one fp32 atomic
//                                per (c,t) per block; dw may be the flat
//                                gradient buffer itself)
// Zero padding ('same' / 'valid' resolved by the caller into pt/pl).
#include "../common.h"

namespace {

__device__ __forceinline__ void ld8(const uint16_t* p, float (&v)[8]) {
  const uint4 q = *reinterpret_cast<const uint4*>(p);
  const uint32_t u[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[2 * k] = zk::bf16_to_f32((uint16_t)(u[k] & 0xffff));
    v[2 * k + 1] = zk::bf16_to_f32((uint16_t)(u[k] >> 16));
  }
}

__device__ __forceinline__ void st8(uint16_t* p, const float (&v)[8]) {
  *reinterpret_cast<uint4*>(p) =
      make_uint4(zk::pack_bf16x2(v[0], v[1]), zk::pack_bf16x2(v[2], v[3]),
                 zk::pack_bf16x2(v[4], v[5]), zk::pack_bf16x2(v[6], v[7]));
}

int grid_for(long long work) {
  long long b = (work + 255) / 256;
  if (b > 16384) b = 16384;
  return b < 1 ? 1 : (int)b;
}

// Transposed weights [KK][C] in LDS.
template <int K>
__device__ __forceinline__ void stage_weights(const float* __restrict__ w, float* ws, int C) {
  constexpr int KK = K * K;
  for (int i = threadIdx.x; i < KK * C; i += blockDim.x) {
    const int c = i / KK, t = i % KK;
    ws[t * C + c] = w[i];
  }
  __syncthreads();
}

template <int K>
__global__ __launch_bounds__(256) void dw_fwd_kernel(const uint16_t* __restrict__ x,
                                                     const float* __restrict__ w,
                                                     uint16_t* __restrict__ y, int B, int H,
                                                     int W, int C, int Ho, int Wo, int s,
                                                     int pt, int pl) {
  extern __shared__ float ws[];
  stage_weights<K>(w, ws, C);
  const int CG = C / 8;
  const long long total = (long long)B * Ho * Wo * CG;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int cg = (int)(i % CG);
    const long long pix = i / CG;
    const int wo = (int)(pix % Wo);
    const int ho = (int)((pix / Wo) % Ho);
    const int b = (int)(pix / ((long long)Wo * Ho));
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int kh = 0; kh < K; ++kh) {
      const int hi = ho * s - pt + kh;
      if (hi < 0 || hi >= H) continue;
#pragma unroll
      for (int kw = 0; kw < K; ++kw) {
        const int wi = wo * s - pl + kw;
        if (wi < 0 || wi >= W) continue;
        float v[8];
        ld8(x + (((long long)b * H + hi) * W + wi) * C + cg * 8, v);
        const float* wt = ws + (kh * K + kw) * C + cg * 8;
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] = fmaf(v[k], wt[k], acc[k]);
      }
    }
    st8(y + pix * C + cg * 8, acc);
  }
}

template <int K>
__global__ __launch_bounds__(256) void dw_dgrad_kernel(const uint16_t* __restrict__ dy,
                                                       const float* __restrict__ w,
                                                       uint16_t* __restrict__ dx, int B, int H,
                                                       int W, int C, int Ho, int Wo, int s,
                                                       int pt, int pl) {
  extern __shared__ float ws[];
  stage_weights<K>(w, ws, C);
  const int CG = C / 8;
  const long long total = (long long)B * H * W * CG;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int cg = (int)(i % CG);
    const long long pix = i / CG;
    const int wi = (int)(pix % W);
    const int hi = (int)((pix / W) % H);
    const int b = (int)(pix / ((long long)W * H));
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int kh = 0; kh < K; ++kh) {
      const int nh = hi + pt - kh;
      if (nh < 0 || nh % s) continue;
      const int ho = nh / s;
      if (ho >= Ho) continue;
#pragma unroll
      for (int kw = 0; kw < K; ++kw) {
        const int nw = wi + pl - kw;
        if (nw < 0 || nw % s) continue;
        const int wo = nw / s;
        if (wo >= Wo) continue;
        float g[8];
        ld8(dy + (((long long)b * Ho + ho) * Wo + wo) * C + cg * 8, g);
        const float* wt = ws + (kh * K + kw) * C + cg * 8;
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] = fmaf(g[k], wt[k], acc[k]);
      }
    }
    st8(dx + pix * C + cg * 8, acc);
  }
}

// Block = 256 threads = R rows x CG channel groups (256 % CG == 0).
template <int K>
__global__ __launch_bounds__(256) void dw_wgrad_kernel(const uint16_t* __restrict__ dy,
                                                       const uint16_t* __restrict__ x,
                                                       float* __restrict__ dw,
                                                       float* __restrict__ slab, int B, int H,
                                                       int W, int C, int Ho, int Wo, int s,
                                                       int pt, int pl) {
  constexpr int KK = K * K;
  const int CG = C / 8;
  const int R = 256 / CG;
  const int cg = threadIdx.x % CG;
  const int row = threadIdx.x / CG;
  const long long P = (long long)B * Ho * Wo;
  float acc[KK][8];
#pragma unroll
  for (int t = 0; t < KK; ++t)
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[t][k] = 0.f;
  for (long long p = (long long)blockIdx.x * R + row; p < P; p += (long long)gridDim.x * R) {
    const int wo = (int)(p % Wo);
    const int ho = (int)((p / Wo) % Ho);
    const int b = (int)(p / ((long long)Wo * Ho));
    float g[8];
    ld8(dy + p * C + cg * 8, g);
#pragma unroll
    for (int kh = 0; kh < K; ++kh) {
      const int hi = ho * s - pt + kh;
      if (hi < 0 || hi >= H) continue;
#pragma unroll
      for (int kw = 0; kw < K; ++kw) {
        const int wi = wo * s - pl + kw;
        if (wi < 0 || wi >= W) continue;
        float v[8];
        ld8(x + (((long long)b * H + hi) * W + wi) * C + cg * 8, v);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[kh * K + kw][k] = fmaf(g[k], v[k], acc[kh * K + kw][k]);
      }
    }
  }
  __shared__ float red[256][9];
#pragma unroll
  for (int t = 0; t < KK; ++t) {
#pragma unroll
    for (int k = 0; k < 8; ++k) red[threadIdx.x][k] = acc[t][k];
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += 256) {
      const int g = c / 8, k = c % 8;
      float sum = 0.f;
      for (int r = 0; r < R; ++r) sum += red[r * CG + g][k];
      if (slab)  // deterministic mode: per-block partials, fixed-order reduce
        slab[(long long)blockIdx.x * C * KK + (long long)c * KK + t] = sum;
      else
        atomicAdd(dw + (long long)c * KK + t, sum);
    }
    __syncthreads();
  }
}

}  // namespace

ZK_EXPORT int zk_dw_fwd(const void* x, const float* w, void* y, int B, int H, int W, int C,
                        int Ho, int Wo, int k, int s, int pt, int pl, hipStream_t st) {
  if (C % 8 || k != 3 || C * 9 * 4 > 64 * 1024) return (int)hipErrorInvalidValue;
  const long long work = (long long)B * Ho * Wo * (C / 8);
  hipLaunchKernelGGL(dw_fwd_kernel<3>, dim3(grid_for(work)), dim3(256), C * 9 * 4, st,
                     (const uint16_t*)x, w, (uint16_t*)y, B, H, W, C, Ho, Wo, s, pt, pl);
  ZK_CHECK_LAUNCH();
  return 0;
}

ZK_EXPORT int zk_dw_dgrad(const void* dy, const float* w, void* dx, int B, int H, int W, int C,
                          int Ho, int Wo, int k, int s, int pt, int pl, hipStream_t st) {
  if (C % 8 || k != 3 || C * 9 * 4 > 64 * 1024) return (int)hipErrorInvalidValue;
  const long long work = (long long)B * H * W * (C / 8);
  hipLaunchKernelGGL(dw_dgrad_kernel<3>, dim3(grid_for(work)), dim3(256), C * 9 * 4, st,
                     (const uint16_t*)dy, w, (uint16_t*)dx, B, H, W, C, Ho, Wo, s, pt, pl);
  ZK_CHECK_LAUNCH();
  return 0;
}

// Blocks of zk_dw_wgrad (the slab of the deterministic mode is [blocks][C*9]).
ZK_EXPORT int zk_dw_wgrad_blocks(int B, int Ho, int Wo, int C) {
  const int CG = C / 8;
  if (C % 8 || CG > 256 || 256 % CG) return -1;
  const int R = 256 / CG;
  const long long P = (long long)B * Ho * Wo;
  long long blocks = (P + R - 1) / R;
  return (int)(blocks > 1024 ? 1024 : blocks);
}

// dw [C][9] += per-channel 3x3 weight gradient; fp32 atomics, or with slab
// (deterministic mode) per-block partials summed by zk_wgrad_slab_reduce.
ZK_EXPORT int zk_dw_wgrad(const void* dy, const void* x, float* dw, void* slab, int B, int H,
                          int W, int C, int Ho, int Wo, int k, int s, int pt, int pl,
                          hipStream_t st) {
  const int CG = C / 8;
  if (C % 8 || k != 3 || CG > 256 || 256 % CG) return (int)hipErrorInvalidValue;
  const int blocks = zk_dw_wgrad_blocks(B, Ho, Wo, C);
  hipLaunchKernelGGL(dw_wgrad_kernel<3>, dim3(blocks), dim3(256), 0, st,
                     (const uint16_t*)dy, (const uint16_t*)x, dw, (float*)slab, B, H, W, C, Ho,
                     Wo, s, pt, pl);
  ZK_CHECK_LAUNCH();
  return 0;
}
