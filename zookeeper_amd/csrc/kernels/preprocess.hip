// Fused input preprocessing: uint8 NHWC (3 channels) -> bf16 NHWC,
// out = (x - mean[c]) / std[c], with an optional per-image horizontal flip
// decided by a hash of (seed, image index).  One pass over the batch:
// reads 3 B/pixel, writes 6 B/pixel (HBM-bound).
#include "../common.h"

namespace {

// One thread = 4 consecutive output pixels of one row (12 input bytes,
// 24 output bytes).  W must be a multiple of 4.
__global__ __launch_bounds__(256) void normalize_flip_c3(
    const uint8_t* __restrict__ in, uint16_t* __restrict__ out, int B, int H, int W,
    float m0, float m1, float m2, float r0, float r1, float r2, int do_flip,
    unsigned long long seed) {
  const int groups_per_row = W >> 2;
  const long long total = (long long)B * H * groups_per_row;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int g = (int)(t % groups_per_row);
    const long long row = t / groups_per_row;  // b*H + h
    const int b = (int)(row / H);
    const bool flip = do_flip && (zk::hash_u32(seed * 1000003ull + (unsigned)b) & 1u);
    // Output pixels [4g, 4g+4) come from input pixels [4g', 4g'+4) reversed
    // when flipped, where 4g' = W - 4 - 4g.
    const int src_g = flip ? (groups_per_row - 1 - g) : g;
    const uint32_t* src =
        reinterpret_cast<const uint32_t*>(in + (row * W + 4LL * src_g) * 3);
    uint32_t w0 = src[0], w1 = src[1], w2 = src[2];
    uint8_t px[12];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      px[i] = (w0 >> (8 * i)) & 0xff;
      px[4 + i] = (w1 >> (8 * i)) & 0xff;
      px[8 + i] = (w2 >> (8 * i)) & 0xff;
    }
    float o[12];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int sp = flip ? 3 - p : p;
      o[3 * p + 0] = ((float)px[3 * sp + 0] - m0) * r0;
      o[3 * p + 1] = ((float)px[3 * sp + 1] - m1) * r1;
      o[3 * p + 2] = ((float)px[3 * sp + 2] - m2) * r2;
    }
    uint2* dst = reinterpret_cast<uint2*>(out + (row * W + 4LL * g) * 3);
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      dst[q] = make_uint2(zk::pack_bf16x2(o[4 * q + 0], o[4 * q + 1]),
                          zk::pack_bf16x2(o[4 * q + 2], o[4 * q + 3]));
    }
  }
}

}  // namespace

ZK_EXPORT int zk_normalize_flip_c3(const void* in, void* out, int B, int H, int W,
                                   const float* mean, const float* std_, int do_flip,
                                   unsigned long long seed, hipStream_t stream) {
  if (W % 4 != 0) return (int)hipErrorInvalidValue;
  const long long work = (long long)B * H * (W / 4);
  int blocks = (int)((work + 255) / 256);
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(normalize_flip_c3, dim3(blocks), dim3(256), 0, stream,
                     (const uint8_t*)in, (uint16_t*)out, B, H, W, mean[0], mean[1], mean[2],
                     1.f / std_[0], 1.f / std_[1], 1.f / std_[2], do_flip, seed);
  ZK_CHECK_LAUNCH();
  return 0;
}
