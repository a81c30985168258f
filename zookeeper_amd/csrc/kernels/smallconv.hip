// Small-K convolutions on MFMA (v_mfma_f32_16x16x32_bf16): convs whose whole
// reduction K = KH*KW*Cin is at most 64 — the layers that read the image or a
// thin feature map: BinaryNet's first conv (3x3 valid over 1 or 3 channels,
// +-1 kernel, examples/larq_experiment.py:62-69), QuickNet's stem conv
// (3x3/2 over 3 channels) and its 16 -> 64 1x1 conv (and that conv's data
// gradient, which is again a K = 64 1x1 conv).
//
// The big implicit-GEMM kernels (igemm.hip) stream K in 64-channel chunks
// through an LDS-DMA ring; here the whole K of a 128-pixel tile fits one LDS
// image, so each block builds it once (an im2col gather of bf16 values,
// padding taps and k >= K as zeros) and runs all its MFMAs from LDS:
//
//   forward  D[co][pixel] = W[co][k] . col[pixel][k]    lane = pixel, 4
//            consecutive channels per lane -> 8-B bf16 stores;
//   wgrad    D[co][k] += dY[pixel][co]^T . col[pixel][k] over a split-K chunk
//            of pixels (both operands staged [row][pixel] in LDS so a lane
//            reads 8 consecutive pixels), then fp32 atomics into the OHWI
//            gradient, masked by |w| <= clip (the ste_sign kernel STE; +inf
//            for a float kernel).
//
// Cout is a multiple of 16 up to 128; K <= 64 (KP = 32 or 64 padded).
#include "mfma_common.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

struct SKGeom {
  int B, H, W, Cin, Ho, Wo, Cout, KH, KW, s, pt, pl, K;
};

constexpr int SK_BM = 128;  // pixels per block / per split-K stage

__device__ __forceinline__ f32x4 mfma16(const uint4& a, const uint4& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// im2col(p, k) of output pixel (b, ho, wo): zero for padding taps and k >= K.
__device__ __forceinline__ uint16_t col_value(const uint16_t* __restrict__ x, const SKGeom& g,
                                              int b, int ho, int wo, int k) {
  if (k >= g.K) return 0;
  const int c = k % g.Cin, t = k / g.Cin;
  const int kw = t % g.KW, kh = t / g.KW;
  const int hi = ho * g.s - g.pt + kh, wi = wo * g.s - g.pl + kw;
  if (hi < 0 || hi >= g.H || wi < 0 || wi >= g.W) return 0;
  return x[(((long long)b * g.H + hi) * g.W + wi) * g.Cin + c];
}

template <int KP>
__global__ __launch_bounds__(256) void smallk_fwd_kernel(const uint16_t* __restrict__ x,
                                                         const uint16_t* __restrict__ wp,
                                                         uint16_t* __restrict__ y, SKGeom g) {
  constexpr int RS = KP + 8;  // LDS row stride in elements (16-B aligned, staggers banks)
  __shared__ __attribute__((aligned(16))) uint16_t sW[128 * RS];
  __shared__ __attribute__((aligned(16))) uint16_t sX[SK_BM * RS];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const long long P = (long long)g.B * g.Ho * g.Wo;
  const long long p0 = (long long)blockIdx.x * SK_BM;
  const int nct = g.Cout >> 4;
  for (int e = tid; e < g.Cout * (KP / 8); e += 256) {
    const int co = e / (KP / 8), j = e % (KP / 8);
    *reinterpret_cast<uint4*>(&sW[co * RS + j * 8]) = reinterpret_cast<const uint4*>(wp)[e];
  }
  for (int e = tid; e < SK_BM * KP; e += 256) {
    const int r = e / KP, k = e % KP;
    const long long p = p0 + r;
    uint16_t v = 0;
    if (p < P) {
      const int wo = (int)(p % g.Wo);
      const long long q = p / g.Wo;
      v = col_value(x, g, (int)(q / g.Ho), (int)(q % g.Ho), wo, k);
    }
    sX[r * RS + k] = v;
  }
  __syncthreads();

  const int r16 = lane & 15, kq = lane >> 4;
  f32x4 acc[8][2];
#pragma unroll
  for (int c = 0; c < 8; ++c)
#pragma unroll
    for (int t = 0; t < 2; ++t) acc[c][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < KP / 32; ++ks) {
    uint4 bx[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
      bx[t] = *reinterpret_cast<const uint4*>(&sX[(wave * 32 + t * 16 + r16) * RS + ks * 32 + kq * 8]);
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      if (c < nct) {
        const uint4 a = *reinterpret_cast<const uint4*>(&sW[(c * 16 + r16) * RS + ks * 32 + kq * 8]);
#pragma unroll
        for (int t = 0; t < 2; ++t) acc[c][t] = mfma16(a, bx[t], acc[c][t]);
      }
    }
  }
  // D[co][pixel]: column (pixel) = lane & 15, rows (channels) 4*(lane>>4) + reg
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const long long p = p0 + wave * 32 + t * 16 + r16;
    if (p >= P) continue;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      if (c < nct) {
        const uint2 o = make_uint2(zk::pack_bf16x2(acc[c][t][0], acc[c][t][1]),
                                   zk::pack_bf16x2(acc[c][t][2], acc[c][t][3]));
        *reinterpret_cast<uint2*>(y + p * g.Cout + c * 16 + 4 * kq) = o;
      }
    }
  }
}

template <int KP>
__global__ __launch_bounds__(256) void smallk_wgrad_kernel(const uint16_t* __restrict__ dy,
                                                           const uint16_t* __restrict__ x,
                                                           const float* __restrict__ w,
                                                           float* __restrict__ dw, SKGeom g,
                                                           int kps, float clip) {
  constexpr int PS = SK_BM + 8;  // pixel stride of the transposed images (16-B aligned rows)
  __shared__ __attribute__((aligned(16))) uint16_t sD[128 * PS];  // dY^T [co][pixel]
  __shared__ __attribute__((aligned(16))) uint16_t sC[KP * PS];   // col^T [k][pixel]
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const long long P = (long long)g.B * g.Ho * g.Wo;
  const long long kbeg = (long long)blockIdx.x * kps;
  if (kbeg >= P) return;
  const long long kend = min(P, kbeg + kps);
  const int nct = g.Cout >> 4, nkt = KP / 16, ntile = nct * nkt;
  const int cv = g.Cout >> 3;  // 16-B vectors per dY row
  const int r16 = lane & 15, kq = lane >> 4;
  f32x4 acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (long long c0 = kbeg; c0 < kend; c0 += SK_BM) {
    __syncthreads();  // the previous stage's fragment reads are done
    for (int e = tid; e < SK_BM * cv; e += 256) {
      const int r = e / cv, j = e % cv;
      const long long p = c0 + r;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (p < kend) v = *reinterpret_cast<const uint4*>(dy + p * g.Cout + j * 8);
      const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        sD[(j * 8 + 2 * i) * PS + r] = (uint16_t)(vv[i] & 0xffff);
        sD[(j * 8 + 2 * i + 1) * PS + r] = (uint16_t)(vv[i] >> 16);
      }
    }
    for (int e = tid; e < SK_BM * KP; e += 256) {
      const int r = e % SK_BM, k = e / SK_BM;
      const long long p = c0 + r;
      uint16_t v = 0;
      if (p < kend) {
        const int wo = (int)(p % g.Wo);
        const long long q = p / g.Wo;
        v = col_value(x, g, (int)(q / g.Ho), (int)(q % g.Ho), wo, k);
      }
      sC[k * PS + r] = v;
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < SK_BM / 32; ++ks) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int t = wave + 4 * i;
        if (t < ntile) {
          const int ct = t / nkt, kt = t % nkt;
          const uint4 a = *reinterpret_cast<const uint4*>(&sD[(ct * 16 + r16) * PS + ks * 32 + kq * 8]);
          const uint4 b = *reinterpret_cast<const uint4*>(&sC[(kt * 16 + r16) * PS + ks * 32 + kq * 8]);
          acc[i] = mfma16(a, b, acc[i]);
        }
      }
    }
  }
  // D[co][k]: column k = lane & 15 of the tile, rows co = 4*(lane>>4) + reg
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int t = wave + 4 * i;
    if (t >= ntile) continue;
    const int ct = t / nkt, kt = t % nkt;
    const int k = kt * 16 + r16;
    if (k >= g.K) continue;
    const int c = k % g.Cin, tt = k / g.Cin;
    const int kw = tt % g.KW, kh = tt / g.KW;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int co = ct * 16 + 4 * kq + e;
      const long long idx = (((long long)co * g.KH + kh) * g.KW + kw) * g.Cin + c;
      if (fabsf(w[idx]) <= clip) atomicAdd(dw + idx, acc[i][e]);
    }
  }
}

bool sk_ok(const SKGeom& g) {
  return g.Cout > 0 && g.Cout % 16 == 0 && g.Cout <= 128 && g.K >= 1 && g.K <= 64 &&
         g.s >= 1 && (long long)g.B * g.Ho * g.Wo < (1LL << 31);
}

}  // namespace

// y bf16 [B][Ho][Wo][Cout] = x ⊛ W;  x bf16 [B][H][W][Cin];  wp bf16
// [Cout][KP] with KP = 32 (K <= 32) or 64 (K <= 64), k = (kh*KW + kw)*Cin + c,
// zero beyond K.  Zero padding (TF same / valid via pt, pl, Ho, Wo).
ZK_EXPORT int zk_smallk_conv_fwd(const void* x, const void* wp, void* y, int B, int H, int W,
                                 int Cin, int Ho, int Wo, int Cout, int KH, int KW, int s, int pt,
                                 int pl, hipStream_t st) {
  SKGeom g{B, H, W, Cin, Ho, Wo, Cout, KH, KW, s, pt, pl, KH * KW * Cin};
  if (!sk_ok(g)) return (int)hipErrorInvalidValue;
  const long long P = (long long)B * Ho * Wo;
  const unsigned blocks = (unsigned)((P + SK_BM - 1) / SK_BM);
  if (g.K <= 32)
    hipLaunchKernelGGL(smallk_fwd_kernel<32>, dim3(blocks), dim3(256), 0, st,
                       (const uint16_t*)x, (const uint16_t*)wp, (uint16_t*)y, g);
  else
    hipLaunchKernelGGL(smallk_fwd_kernel<64>, dim3(blocks), dim3(256), 0, st,
                       (const uint16_t*)x, (const uint16_t*)wp, (uint16_t*)y, g);
  ZK_CHECK_LAUNCH();
  return 0;
}

// dw fp32 OHWI [Cout][KH][KW][Cin] += dY^T ⊛ x where |w| <= clip (w: the
// latent fp32 kernel, OHWI); dy bf16 [B][Ho][Wo][Cout].  Split-K over pixel
// chunks, fp32 atomics (target_blocks <= 0: 1024 blocks).
ZK_EXPORT int zk_smallk_conv_wgrad(const void* dy, const void* x, const void* w, void* dw, int B,
                                   int H, int W, int Cin, int Ho, int Wo, int Cout, int KH, int KW,
                                   int s, int pt, int pl, float clip, int target_blocks,
                                   hipStream_t st) {
  SKGeom g{B, H, W, Cin, Ho, Wo, Cout, KH, KW, s, pt, pl, KH * KW * Cin};
  if (!sk_ok(g)) return (int)hipErrorInvalidValue;
  const long long P = (long long)B * Ho * Wo;
  if (target_blocks <= 0) target_blocks = 1024;
  long long kps = (P + target_blocks - 1) / target_blocks;
  kps = (kps + SK_BM - 1) / SK_BM * SK_BM;
  const unsigned blocks = (unsigned)((P + kps - 1) / kps);
  if (g.K <= 32)
    hipLaunchKernelGGL(smallk_wgrad_kernel<32>, dim3(blocks), dim3(256), 0, st,
                       (const uint16_t*)dy, (const uint16_t*)x, (const float*)w, (float*)dw, g,
                       (int)kps, clip);
  else
    hipLaunchKernelGGL(smallk_wgrad_kernel<64>, dim3(blocks), dim3(256), 0, st,
                       (const uint16_t*)dy, (const uint16_t*)x, (const float*)w, (float*)dw, g,
                       (int)kps, clip);
  ZK_CHECK_LAUNCH();
  return 0;
}
