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

// normalize_flip_c3 plus the fused stem's padded input in the same pass:
// xp bf16 [B][Hp][Wp][4] (channel 3 and the borders zero, image at rows
// [pt, pt + H), columns [pl, pl + W); ops/stem.py zk_stem_pack_input3 layout).
// One thread = one pair of xp pixels (16 B of xp, up to 12 B of out); the
// values are bit-identical to normalize_flip_c3 followed by the pack.
__global__ __launch_bounds__(256) void normalize_flip_pack_c3(
    const uint8_t* __restrict__ in, uint16_t* __restrict__ out, uint4* __restrict__ xp, int B,
    int H, int W, int Hp, int Wp, int pt, int pl, float m0, float m1, float m2, float r0,
    float r1, float r2, int do_flip, unsigned long long seed) {
  const int Wp2 = Wp >> 1;
  const long long total = (long long)B * Hp * Wp2;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int wq = (int)(i % Wp2);
    const long long r = i / Wp2;
    const int hp = (int)(r % Hp);
    const int b = (int)(r / Hp);
    const int h = hp - pt, w = 2 * wq - pl;
    uint32_t o[4] = {0u, 0u, 0u, 0u};
    uint16_t v[2][3];
    bool ok[2] = {false, false};
    if (h >= 0 && h < H) {
      const bool flip = do_flip && (zk::hash_u32(seed * 1000003ull + (unsigned)b) & 1u);
      const long long row = (long long)b * H + h;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int wk = w + k;
        if (wk < 0 || wk >= W) continue;
        ok[k] = true;
        const uint8_t* px = in + (row * W + (flip ? W - 1 - wk : wk)) * 3;
        const float c0 = ((float)px[0] - m0) * r0;
        const float c1 = ((float)px[1] - m1) * r1;
        const float c2 = ((float)px[2] - m2) * r2;
        const uint32_t p01 = zk::pack_bf16x2(c0, c1);
        const uint32_t p2 = zk::pack_bf16x2(c2, 0.f) & 0xffffu;
        o[2 * k] = p01;
        o[2 * k + 1] = p2;
        v[k][0] = (uint16_t)(p01 & 0xffffu);
        v[k][1] = (uint16_t)(p01 >> 16);
        v[k][2] = (uint16_t)p2;
      }
      uint16_t* dst = out + (row * W + w) * 3;
      if (ok[0] && ok[1] && (w & 1) == 0) {
        uint32_t* d32 = reinterpret_cast<uint32_t*>(dst);  // 12 B, 4-B aligned (w even)
        d32[0] = v[0][0] | ((uint32_t)v[0][1] << 16);
        d32[1] = v[0][2] | ((uint32_t)v[1][0] << 16);
        d32[2] = v[1][1] | ((uint32_t)v[1][2] << 16);
      } else {
#pragma unroll
        for (int k = 0; k < 2; ++k)
          if (ok[k]) {
            dst[3 * k] = v[k][0];
            dst[3 * k + 1] = v[k][1];
            dst[3 * k + 2] = v[k][2];
          }
      }
    }
    xp[i] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

}  // namespace

ZK_EXPORT int zk_normalize_flip_pack_c3(const void* in, void* out, void* xp, int B, int H, int W,
                                        int Hp, int Wp, int pt, int pl, const float* mean,
                                        const float* std_, int do_flip, unsigned long long seed,
                                        hipStream_t stream) {
  if (Wp % 2 != 0 || pt < 0 || pl < 0 || Hp < pt + H || Wp < pl + W)
    return (int)hipErrorInvalidValue;
  const long long work = (long long)B * Hp * (Wp / 2);
  long long blocks = (work + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(normalize_flip_pack_c3, dim3((int)blocks), dim3(256), 0, stream,
                     (const uint8_t*)in, (uint16_t*)out, (uint4*)xp, B, H, W, Hp, Wp, pt, pl,
                     mean[0], mean[1], mean[2], 1.f / std_[0], 1.f / std_[1], 1.f / std_[2],
                     do_flip, seed);
  ZK_CHECK_LAUNCH();
  return 0;
}

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
