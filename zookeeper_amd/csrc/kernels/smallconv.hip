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

// PW: a 1x1 stride-1 unpadded conv (QuickNet's 16 -> 64 stem conv and its data
// gradient): the im2col row of a pixel is its Cin contiguous channels, copied
// with 16-B loads (Cin % 8 == 0) instead of the per-element tap gather.
template <int KP, bool PW>
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
  if (PW) {
    for (int e = tid; e < SK_BM * (KP / 8); e += 256) {
      const int r = e / (KP / 8), k8 = (e % (KP / 8)) * 8;
      const long long p = p0 + r;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (p < P && k8 < g.Cin) v = *reinterpret_cast<const uint4*>(x + p * g.Cin + k8);
      *reinterpret_cast<uint4*>(&sX[r * RS + k8]) = v;
    }
  } else {
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

// NC: Cout / 16 when known at compile time (0: runtime, up to 8) -- the
// fixed tile count keeps the fragment loads from being hoisted into ~230
// VGPRs (one wave per SIMD) as the runtime-bounded loops were.
template <int KP, bool PW, int NC>
__global__ __launch_bounds__(256) void smallk_wgrad_kernel(const uint16_t* __restrict__ dy,
                                                           const uint16_t* __restrict__ x,
                                                           const float* __restrict__ w,
                                                           float* __restrict__ dw,
                                                           float* __restrict__ slab, SKGeom g,
                                                           int kps, float clip) {
  constexpr int PS = SK_BM + 8;  // pixel stride of the transposed images (16-B aligned rows)
  __shared__ __attribute__((aligned(16))) uint16_t sD[128 * PS];  // dY^T [co][pixel]
  __shared__ __attribute__((aligned(16))) uint16_t sC[KP * PS];   // col^T [k][pixel]
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const long long P = (long long)g.B * g.Ho * g.Wo;
  const long long kbeg = (long long)blockIdx.x * kps;
  if (kbeg >= P) return;
  const long long kend = min(P, kbeg + kps);
  constexpr int nkt = KP / 16;
  constexpr int MAXT = NC ? (NC * nkt + 3) / 4 : 8;  // tiles per wave
  const int nct = NC ? NC : g.Cout >> 4, ntile = nct * nkt;
  const int cv = g.Cout >> 3;  // 16-B vectors per dY row
  const int r16 = lane & 15, kq = lane >> 4;
  f32x4 acc[MAXT];
#pragma unroll
  for (int i = 0; i < MAXT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Software-pipelined staging: stage s+1's dY (and, 1x1, x) vectors are
  // loaded into registers while stage s's MFMAs run; the transposed 2-B LDS
  // stores happen after the barrier that retires stage s's fragment reads.
  constexpr int DV = NC ? NC : 8;  // 16-B dY vectors per thread per stage (Cout/16)
  constexpr int XV = KP / 8 * SK_BM / 256;  // 16-B x vectors per thread (1x1 path)
  uint4 rd[DV], rx[XV > 0 ? XV : 1];
  auto load_stage = [&](long long c0) {
#pragma unroll
    for (int u = 0; u < DV; ++u) {
      const int e = tid + 256 * u;
      const int r = e / cv, j = e % cv;
      const long long p = c0 + r;
      rd[u] = make_uint4(0u, 0u, 0u, 0u);
      if (e < SK_BM * cv && p < kend) rd[u] = *reinterpret_cast<const uint4*>(dy + p * g.Cout + j * 8);
    }
    if (PW) {
      constexpr int xv = KP / 8;
#pragma unroll
      for (int u = 0; u < XV; ++u) {
        const int e = tid + 256 * u;
        const int r = e / xv, j = e % xv;
        const long long p = c0 + r;
        rx[u] = make_uint4(0u, 0u, 0u, 0u);
        if (p < kend && j * 8 < g.Cin) rx[u] = *reinterpret_cast<const uint4*>(x + p * g.Cin + j * 8);
      }
    }
  };
  auto scatter = [&](uint16_t* S, const uint4& v, int r, int j) {
    const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      S[(j * 8 + 2 * i) * PS + r] = (uint16_t)(vv[i] & 0xffff);
      S[(j * 8 + 2 * i + 1) * PS + r] = (uint16_t)(vv[i] >> 16);
    }
  };
  load_stage(kbeg);
  for (long long c0 = kbeg; c0 < kend; c0 += SK_BM) {
    __syncthreads();  // the previous stage's fragment reads are done
#pragma unroll
    for (int u = 0; u < DV; ++u) {
      const int e = tid + 256 * u;
      if (e < SK_BM * cv) scatter(sD, rd[u], e / cv, e % cv);
    }
    if (PW) {
#pragma unroll
      for (int u = 0; u < XV; ++u) {
        const int e = tid + 256 * u;
        scatter(sC, rx[u], e / (KP / 8), e % (KP / 8));
      }
    } else {
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
    }
    if (c0 + SK_BM < kend) load_stage(c0 + SK_BM);
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < SK_BM / 32; ++ks) {
#pragma unroll
      for (int i = 0; i < MAXT; ++i) {
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
  for (int i = 0; i < MAXT; ++i) {
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
      if (slab)  // deterministic mode: this block's partial, reduced in a fixed order
        slab[(long long)blockIdx.x * g.Cout * g.K + idx] = acc[i][e];
      else if (fabsf(w[idx]) <= clip)
        atomicAdd(dw + idx, acc[i][e]);
    }
  }
}

// ---------------------------------------------------------------------------
// Row-band kernels for image-reading 3x3 convs (Cin 1 or 3, K <= 32): a block
// owns R whole output rows of one image (R*Wo ~ 256 pixels) and stages the
// (R-1)*s + 3 input rows it reads in LDS with 16-B copies, so the im2col
// gather is LDS reads with compile-time tap decomposition -- no per-element
// 64-bit index divisions and no 2-byte global gathers (the generic kernels
// above spent 3-4 ms/step on QuickNet's 224x224 stem conv for that reason).
//
//   forward  B operand = col[pixel][k] gathered per lane (k = 8*(lane>>4)+j),
//            A = packed weights held in registers for the whole block;
//   wgrad    A = dY^T (8 consecutive pixels of one channel, from an LDS copy
//            of the band's dY rows), B = col^T gathered per lane; per-block
//            fp32 partials, summed in a fixed order by band_wgrad_reduce
//            (deterministic, no atomics).
// ---------------------------------------------------------------------------

struct BandGeom {
  int R;          // output rows per band
  int nbands;     // bands per image
  int rows;       // staged input rows per band = (R-1)*s + KS
  int rowlen;     // W*Cin elements per input row
};

template <int CIN, int KS>
__device__ __forceinline__ void band_stage_input(const uint16_t* __restrict__ x, uint16_t* sIn,
                                                 const SKGeom& g, const BandGeom& bg, int b,
                                                 int hi0) {
  const int tid = threadIdx.x;
  if ((bg.rowlen & 7) == 0) {
    // 4 independent 16-B loads in flight per thread before their LDS stores
    const int vpr = bg.rowlen >> 3, total = bg.rows * vpr;
    for (int e0 = tid; e0 < total; e0 += 1024) {
      uint4 val[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = e0 + 256 * u;
        const int r = e / vpr, v = e - r * vpr, hi = hi0 + r;
        val[u] = make_uint4(0u, 0u, 0u, 0u);
        if (e < total && hi >= 0 && hi < g.H)
          val[u] = *reinterpret_cast<const uint4*>(x + ((long long)b * g.H + hi) * bg.rowlen +
                                                   v * 8);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = e0 + 256 * u;
        if (e < total) reinterpret_cast<uint4*>(sIn)[e] = val[u];
      }
    }
  } else {
    const int total = bg.rows * bg.rowlen;
    for (int e = tid; e < total; e += 256) {
      const int r = e / bg.rowlen, v = e - r * bg.rowlen, hi = hi0 + r;
      sIn[e] = (hi >= 0 && hi < g.H) ? x[((long long)b * g.H + hi) * bg.rowlen + v] : 0;
    }
  }
}

template <int CIN, int KS, int NC>
__global__ __launch_bounds__(256) void band_fwd_kernel(const uint16_t* __restrict__ x,
                                                       const uint16_t* __restrict__ wp,
                                                       uint16_t* __restrict__ y, SKGeom g,
                                                       BandGeom bg) {
  constexpr int K = KS * KS * CIN;
  static_assert(K <= 32, "band kernels take K <= 32");
  extern __shared__ __attribute__((aligned(16))) uint16_t sIn[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r16 = lane & 15, kq = lane >> 4;
  const int b = blockIdx.x / bg.nbands, ho0 = (blockIdx.x % bg.nbands) * bg.R;
  band_stage_input<CIN, KS>(x, sIn, g, bg, b, ho0 * g.s - g.pt);
  // this lane's 8 taps k = 8*kq + j: LDS offset relative to (row r*s, column wo*s - pl)
  int koff[8], kcol[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = kq * 8 + j;
    const int c = k % CIN, t = k / CIN, kw = t % KS, kh = t / KS;
    koff[j] = kh * bg.rowlen + kw * CIN + c;
    kcol[j] = (k < K) ? kw : -100000;  // k >= K: always out of range -> 0
  }
  constexpr int nct = NC;  // Cout / 16
  uint4 wa[NC];
#pragma unroll
  for (int ct = 0; ct < NC; ++ct)
    if (ct < nct) wa[ct] = *reinterpret_cast<const uint4*>(wp + (ct * 16 + r16) * 32 + kq * 8);
  __syncthreads();
  const int rv = min(bg.R, g.Ho - ho0), npix = rv * g.Wo;
  for (int p16 = wave * 16; p16 < npix; p16 += 64) {
    const int pb = p16 + r16;
    uint32_t pk[4] = {0u, 0u, 0u, 0u};
    if (pb < npix) {
      const int r = pb / g.Wo, wo = pb - r * g.Wo;
      const int base = r * g.s * bg.rowlen, c0 = wo * g.s - g.pl;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int wi = c0 + kcol[j];
        const uint32_t v = (wi >= 0 && wi < g.W) ? sIn[base + c0 * CIN + koff[j]] : 0u;
        pk[j >> 1] |= v << (16 * (j & 1));
      }
    }
    const uint4 bx = make_uint4(pk[0], pk[1], pk[2], pk[3]);
    // MFMAs outside the per-lane branch (lanes past the band's end carry zeros)
    f32x4 d[NC];
#pragma unroll
    for (int ct = 0; ct < NC; ++ct)
      if (ct < nct) d[ct] = mfma16(wa[ct], bx, f32x4{0.f, 0.f, 0.f, 0.f});
    if (pb < npix) {
      uint16_t* out = y + (((long long)b * g.Ho + ho0) * g.Wo + pb) * g.Cout + 4 * kq;
#pragma unroll
      for (int ct = 0; ct < NC; ++ct)
        if (ct < nct)
          *reinterpret_cast<uint2*>(out + ct * 16) =
              make_uint2(zk::pack_bf16x2(d[ct][0], d[ct][1]), zk::pack_bf16x2(d[ct][2], d[ct][3]));
    }
  }
}

template <int CIN, int KS, int NC>
__global__ __launch_bounds__(256) void band_wgrad_kernel(const uint16_t* __restrict__ dy,
                                                         const uint16_t* __restrict__ x,
                                                         float* __restrict__ part, SKGeom g,
                                                         BandGeom bg, int bands_per_block) {
  constexpr int K = KS * KS * CIN;
  static_assert(K <= 32, "band kernels take K <= 32");
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* sIn = smem;
  uint16_t* sD = smem + ((bg.rows * bg.rowlen + 7) & ~7);  // [pixel][Cout]
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r16 = lane & 15, kq = lane >> 4;
  constexpr int nct = NC;  // Cout / 16
  // this lane's B-operand taps: k = kt*16 + r16
  int koff[2], kcol[2];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const int k = kt * 16 + r16;
    const int c = k % CIN, t = k / CIN, kw = t % KS, kh = t / KS;
    koff[kt] = kh * bg.rowlen + kw * CIN + c;
    kcol[kt] = (k < K) ? kw : -100000;
  }
  f32x4 acc[NC][2];
#pragma unroll
  for (int i = 0; i < NC; ++i)
#pragma unroll
    for (int t = 0; t < 2; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int total_bands = g.B * bg.nbands;
  const int first = blockIdx.x * bands_per_block;
  const int last = min(total_bands, first + bands_per_block);
  for (int band = first; band < last; ++band) {
    const int b = band / bg.nbands, ho0 = (band % bg.nbands) * bg.R;
    const int rv = min(bg.R, g.Ho - ho0), npix = rv * g.Wo;
    __syncthreads();  // previous band's reads are done
    band_stage_input<CIN, KS>(x, sIn, g, bg, b, ho0 * g.s - g.pt);
    {
      // dY rows of the band are contiguous: npix * Cout elements
      const uint16_t* src = dy + ((long long)b * g.Ho + ho0) * g.Wo * g.Cout;
      const int nv = npix * g.Cout / 8;
      for (int e0 = tid; e0 < nv; e0 += 1024) {
        uint4 val[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (e0 + 256 * u < nv) val[u] = reinterpret_cast<const uint4*>(src)[e0 + 256 * u];
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (e0 + 256 * u < nv) reinterpret_cast<uint4*>(sD)[e0 + 256 * u] = val[u];
      }
    }
    __syncthreads();
    for (int p32 = wave * 32; p32 < npix; p32 += 128) {
      // 8 consecutive pixels p32 + 8*kq + j of this lane
      int base[8], c0[8];
      bool ok[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int p = p32 + kq * 8 + j;
        ok[j] = p < npix;
        const int r = p / g.Wo, wo = p - r * g.Wo;
        base[j] = r * g.s * bg.rowlen;
        c0[j] = wo * g.s - g.pl;
      }
      uint4 bcol[2];
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        uint32_t pk[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int wi = c0[j] + kcol[kt];
          const uint32_t v =
              (ok[j] && wi >= 0 && wi < g.W) ? sIn[base[j] + c0[j] * CIN + koff[kt]] : 0u;
          pk[j >> 1] |= v << (16 * (j & 1));
        }
        bcol[kt] = make_uint4(pk[0], pk[1], pk[2], pk[3]);
      }
#pragma unroll
      for (int ct = 0; ct < NC; ++ct) {
        if (ct < nct) {
          uint32_t pk[4] = {0u, 0u, 0u, 0u};
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int p = p32 + kq * 8 + j;
            const uint32_t v = ok[j] ? sD[p * g.Cout + ct * 16 + r16] : 0u;
            pk[j >> 1] |= v << (16 * (j & 1));
          }
          const uint4 a = make_uint4(pk[0], pk[1], pk[2], pk[3]);
#pragma unroll
          for (int kt = 0; kt < 2; ++kt) acc[ct][kt] = mfma16(a, bcol[kt], acc[ct][kt]);
        }
      }
    }
  }
  // the 4 waves' D[co][k] summed in LDS in wave order (column k = kt*16 +
  // (lane & 15), rows co = ct*16 + 4*kq + e), then one coalesced partial per block
  float* red = reinterpret_cast<float*>(smem);
  __syncthreads();
  for (int w = 0; w < 4; ++w) {
    if (wave == w) {
#pragma unroll
      for (int ct = 0; ct < NC; ++ct)
        if (ct < nct)
#pragma unroll
          for (int kt = 0; kt < 2; ++kt)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              float* d = red + (ct * 16 + 4 * kq + e) * 32 + kt * 16 + r16;
              *d = (w == 0) ? acc[ct][kt][e] : *d + acc[ct][kt][e];
            }
    }
    __syncthreads();
  }
  float* out = part + (long long)blockIdx.x * g.Cout * 32;
  for (int i = tid; i < g.Cout * 32; i += 256) out[i] = red[i];
}

// dw[co][k] (OHWI, fp32) += sum of the per-block partials, masked by |w| <= clip,
// in two fixed-order passes wide enough to keep many loads in flight (one
// pass of ~1000 dependent partial loads per thread ran ~70 us):
//   pass 1: block (o-chunk of 64, slice of 32 parts) -> part2[slice][o]
//   pass 2: thread o sums the slices in order and applies the mask.
constexpr int BR_SLICE = 32;

__global__ __launch_bounds__(256) void band_wgrad_reduce1(const float* __restrict__ part,
                                                          int nparts, int n,
                                                          float* __restrict__ part2) {
  __shared__ float red[4][64];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int o = blockIdx.x * 64 + lane, p0 = blockIdx.y * BR_SLICE;
  float v[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int p = p0 + wave + 4 * u;
    v[u] = (o < n && p < nparts) ? part[(long long)p * n + o] : 0.f;
  }
  red[wave][lane] = ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));
  __syncthreads();
  if (wave == 0 && o < n)
    part2[(long long)blockIdx.y * n + o] =
        ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
}

__global__ __launch_bounds__(256) void band_wgrad_reduce2(const float* __restrict__ part2,
                                                          int nslices, int Cout, int K,
                                                          const float* __restrict__ w,
                                                          float* __restrict__ dw, float clip) {
  const int o = blockIdx.x * 256 + threadIdx.x;  // index into [Cout][32]
  const int n = Cout * 32;
  if (o >= n) return;
  float t = 0.f;
  for (int sl = 0; sl < nslices; ++sl) t += part2[(long long)sl * n + o];
  const int co = o >> 5, k = o & 31;
  if (k < K) {
    const int i = co * K + k;
    if (fabsf(w[i]) <= clip) dw[i] += t;
  }
}

bool band_ok(const SKGeom& g) {
  return (g.Cin == 1 || g.Cin == 3) && g.KH == 3 && g.KW == 3 &&
         (g.Cout == 16 || g.Cout == 32 || g.Cout == 64 || g.Cout == 128) && g.s >= 1 &&
         g.s <= 4 && (long long)g.B * g.Ho * g.Wo < (1LL << 31);
}

BandGeom band_geom(const SKGeom& g) {
  BandGeom bg;
  bg.R = max(1, min(g.Ho, 256 / max(1, g.Wo)));
  bg.nbands = (g.Ho + bg.R - 1) / bg.R;
  bg.rows = (bg.R - 1) * g.s + g.KH;
  bg.rowlen = g.W * g.Cin;
  return bg;
}

size_t band_in_bytes(const BandGeom& bg) {
  return (size_t)((bg.rows * bg.rowlen + 7) & ~7) * 2;
}

// 1x1, stride 1, no padding, Cin % 8 == 0: the contiguous-row fast path
bool sk_pw(const SKGeom& g) {
  return g.KH == 1 && g.KW == 1 && g.s == 1 && g.pt == 0 && g.pl == 0 && g.Ho == g.H &&
         g.Wo == g.W && g.Cin % 8 == 0;
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
  const bool pw = sk_pw(g);
#define ZK_SK_FWD(KPV, PWV)                                                                      \
  hipLaunchKernelGGL((smallk_fwd_kernel<KPV, PWV>), dim3(blocks), dim3(256), 0, st,              \
                     (const uint16_t*)x, (const uint16_t*)wp, (uint16_t*)y, g)
  if (g.K <= 32) {
    if (pw) ZK_SK_FWD(32, true); else ZK_SK_FWD(32, false);
  } else {
    if (pw) ZK_SK_FWD(64, true); else ZK_SK_FWD(64, false);
  }
#undef ZK_SK_FWD
  ZK_CHECK_LAUNCH();
  return 0;
}

// dw fp32 OHWI [Cout][KH][KW][Cin] += dY^T ⊛ x where |w| <= clip (w: the
// latent fp32 kernel, OHWI); dy bf16 [B][Ho][Wo][Cout].  Split-K over pixel
// chunks (target_blocks <= 0: 1024 blocks), fp32 atomics -- or, with slab
// (deterministic mode), per-block partials [blocks][Cout*K] (zeroed by the
// caller; zk_smallk_conv_wgrad_blocks sizes it) summed by zk_wgrad_slab_reduce.
ZK_EXPORT int zk_smallk_conv_wgrad_blocks(int B, int Ho, int Wo, int target_blocks) {
  const long long P = (long long)B * Ho * Wo;
  if (target_blocks <= 0) target_blocks = 1024;
  long long kps = (P + target_blocks - 1) / target_blocks;
  kps = (kps + SK_BM - 1) / SK_BM * SK_BM;
  return (int)((P + kps - 1) / kps);
}

ZK_EXPORT int zk_smallk_conv_wgrad(const void* dy, const void* x, const void* w, void* dw,
                                   void* slab, int B, int H, int W, int Cin, int Ho, int Wo,
                                   int Cout, int KH, int KW, int s, int pt, int pl, float clip,
                                   int target_blocks, hipStream_t st) {
  SKGeom g{B, H, W, Cin, Ho, Wo, Cout, KH, KW, s, pt, pl, KH * KW * Cin};
  if (!sk_ok(g)) return (int)hipErrorInvalidValue;
  const long long P = (long long)B * Ho * Wo;
  if (target_blocks <= 0) target_blocks = 1024;
  long long kps = (P + target_blocks - 1) / target_blocks;
  kps = (kps + SK_BM - 1) / SK_BM * SK_BM;
  const unsigned blocks = (unsigned)((P + kps - 1) / kps);
  const bool pw = sk_pw(g);
#define ZK_SK_WG(KPV, PWV, NCV)                                                                  \
  hipLaunchKernelGGL((smallk_wgrad_kernel<KPV, PWV, NCV>), dim3(blocks), dim3(256), 0, st,       \
                     (const uint16_t*)dy, (const uint16_t*)x, (const float*)w, (float*)dw,       \
                     (float*)slab, g, (int)kps, clip)
#define ZK_SK_WG_NC(KPV, PWV)                \
  switch (g.Cout >> 4) {                     \
    case 1: ZK_SK_WG(KPV, PWV, 1); break;    \
    case 2: ZK_SK_WG(KPV, PWV, 2); break;    \
    case 4: ZK_SK_WG(KPV, PWV, 4); break;    \
    case 8: ZK_SK_WG(KPV, PWV, 8); break;    \
    default: ZK_SK_WG(KPV, PWV, 0); break;   \
  }
  if (g.K <= 32) {
    if (pw) { ZK_SK_WG_NC(32, true) } else { ZK_SK_WG_NC(32, false) }
  } else {
    if (pw) { ZK_SK_WG_NC(64, true) } else { ZK_SK_WG_NC(64, false) }
  }
#undef ZK_SK_WG_NC
#undef ZK_SK_WG
  ZK_CHECK_LAUNCH();
  return 0;
}

// Row-band 3x3 conv over a 1- or 3-channel map (K <= 32): same contract as
// zk_smallk_conv_fwd (wp bf16 [Cout][32]).  Returns hipErrorInvalidValue for
// shapes it does not take (see band_ok / zk_band_conv_ok).
ZK_EXPORT int zk_band_conv_ok(int B, int H, int W, int Cin, int Ho, int Wo, int Cout, int KH,
                              int KW, int s) {
  SKGeom g{B, H, W, Cin, Ho, Wo, Cout, KH, KW, s, 0, 0, KH * KW * Cin};
  if (!band_ok(g)) return 0;
  const BandGeom bg = band_geom(g);
  const size_t dbytes = (size_t)bg.R * Wo * Cout * 2;
  return band_in_bytes(bg) + dbytes <= 96 * 1024 ? 1 : 0;
}

ZK_EXPORT int zk_band_conv_fwd(const void* x, const void* wp, void* y, int B, int H, int W,
                               int Cin, int Ho, int Wo, int Cout, int KH, int KW, int s, int pt,
                               int pl, hipStream_t st) {
  SKGeom g{B, H, W, Cin, Ho, Wo, Cout, KH, KW, s, pt, pl, KH * KW * Cin};
  if (!zk_band_conv_ok(B, H, W, Cin, Ho, Wo, Cout, KH, KW, s)) return (int)hipErrorInvalidValue;
  const BandGeom bg = band_geom(g);
  const size_t lds = band_in_bytes(bg);
  const dim3 grid((unsigned)(B * bg.nbands));
#define ZK_BF(CI, NCV)                                                                           \
  hipLaunchKernelGGL((band_fwd_kernel<CI, 3, NCV>), grid, dim3(256), lds, st, (const uint16_t*)x, \
                     (const uint16_t*)wp, (uint16_t*)y, g, bg)
#define ZK_BF_NC(CI)                   \
  switch (Cout) {                      \
    case 16: ZK_BF(CI, 1); break;      \
    case 32: ZK_BF(CI, 2); break;      \
    case 64: ZK_BF(CI, 4); break;      \
    default: ZK_BF(CI, 8); break;      \
  }
  if (Cin == 3) { ZK_BF_NC(3) } else { ZK_BF_NC(1) }
#undef ZK_BF_NC
#undef ZK_BF
  ZK_CHECK_LAUNCH();
  return 0;
}

// Partial-row count the wgrad below needs scratch for (fp32 [n][Cout][32]).
ZK_EXPORT int zk_band_conv_wgrad_parts(int B, int Ho, int Wo, int target_blocks) {
  const int R = max(1, min(Ho, 256 / max(1, Wo)));
  const int total = B * ((Ho + R - 1) / R);
  if (target_blocks <= 0) target_blocks = 1024;
  const int bpb = (total + target_blocks - 1) / target_blocks;
  const int blocks = (total + bpb - 1) / bpb;
  return blocks + (blocks + 31) / 32;  // per-block partials + the reduction's slice sums
}

// dw fp32 OHWI += dY^T (*) x masked by |w| <= clip; part: scratch of
// zk_band_conv_wgrad_parts(...) * Cout * 32 floats.  Deterministic.
ZK_EXPORT int zk_band_conv_wgrad(const void* dy, const void* x, const void* w, void* dw,
                                 void* part, int B, int H, int W, int Cin, int Ho, int Wo,
                                 int Cout, int KH, int KW, int s, int pt, int pl, float clip,
                                 int target_blocks, hipStream_t st) {
  SKGeom g{B, H, W, Cin, Ho, Wo, Cout, KH, KW, s, pt, pl, KH * KW * Cin};
  if (!zk_band_conv_ok(B, H, W, Cin, Ho, Wo, Cout, KH, KW, s)) return (int)hipErrorInvalidValue;
  const BandGeom bg = band_geom(g);
  if (target_blocks <= 0) target_blocks = 1024;
  const int total = B * bg.nbands;
  const int bpb = (total + target_blocks - 1) / target_blocks;
  const int blocks = (total + bpb - 1) / bpb;
  size_t lds = band_in_bytes(bg) + (size_t)bg.R * Wo * Cout * 2;
  if (lds < (size_t)Cout * 32 * 4) lds = (size_t)Cout * 32 * 4;  // the wave reduction reuses it
#define ZK_BW(CI, NCV)                                                                        \
  hipLaunchKernelGGL((band_wgrad_kernel<CI, 3, NCV>), dim3(blocks), dim3(256), lds, st,        \
                     (const uint16_t*)dy, (const uint16_t*)x, (float*)part, g, bg, bpb)
#define ZK_BW_NC(CI)                   \
  switch (Cout) {                      \
    case 16: ZK_BW(CI, 1); break;      \
    case 32: ZK_BW(CI, 2); break;      \
    case 64: ZK_BW(CI, 4); break;      \
    default: ZK_BW(CI, 8); break;      \
  }
  if (Cin == 3) { ZK_BW_NC(3) } else { ZK_BW_NC(1) }
#undef ZK_BW_NC
#undef ZK_BW
  ZK_CHECK_LAUNCH();
  const int n = Cout * 32, nslices = (blocks + BR_SLICE - 1) / BR_SLICE;
  float* part2 = (float*)part + (long long)blocks * n;  // the tail of the scratch
  hipLaunchKernelGGL(band_wgrad_reduce1, dim3((n + 63) / 64, nslices), dim3(256), 0, st,
                     (const float*)part, blocks, n, part2);
  ZK_CHECK_LAUNCH();
  hipLaunchKernelGGL(band_wgrad_reduce2, dim3((n + 255) / 256), dim3(256), 0, st,
                     (const float*)part2, nslices, Cout, g.K, (const float*)w, (float*)dw, clip);
  ZK_CHECK_LAUNCH();
  return 0;
}

namespace {

// Weight operand of the small-K / band convs: out[n][k] (bf16, row stride KP)
// = w[n*sn + k1*t1 + k2*t2 + k3*t3] for k = (k1*d2 + k2)*d3 + k3 < d1*d2*d3,
// zero up to KP; sign: the ste_sign kernel (w >= 0 -> +1, else -1).  One
// launch instead of the framework's fill + cast + strided copy.
__global__ __launch_bounds__(256) void sk_pack_kernel(const float* __restrict__ w,
                                                      uint16_t* __restrict__ out, int N, int KP,
                                                      int d2, int d3, int K, long long sn,
                                                      long long t1, long long t2, long long t3,
                                                      int sign) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)N * KP) return;
  const int n = (int)(i / KP), k = (int)(i % KP);
  float v = 0.f;
  if (k < K) {
    const int k3 = k % d3, k2 = (k / d3) % d2, k1 = k / (d3 * d2);
    v = w[n * sn + k1 * t1 + k2 * t2 + k3 * t3];
    if (sign) v = v >= 0.f ? 1.f : -1.f;
  }
  out[i] = zk::f32_to_bf16(v);
}

}  // namespace

ZK_EXPORT int zk_smallk_pack(const void* w, void* out, int N, int KP, int d1, int d2, int d3,
                             long long sn, long long t1, long long t2, long long t3, int sign,
                             hipStream_t st) {
  const int K = d1 * d2 * d3;
  if (N < 1 || d1 < 1 || d2 < 1 || d3 < 1 || K > KP) return (int)hipErrorInvalidValue;
  const long long n = (long long)N * KP;
  hipLaunchKernelGGL(sk_pack_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                     (const float*)w, (uint16_t*)out, N, KP, d2, d3, K, sn, t1, t2, t3, sign);
  ZK_CHECK_LAUNCH();
  return 0;
}
