// Fused ImageNet stem: conv KxK/2 (Cin <= 4) -> BN -> ReLU -> maxpool 3x3/2
// [-> BN] for BinaryResNet-E18 / ResNet-50 (7x7/2, 3 -> 64, 224x224).
//
// MIOpen runs this 3-channel conv with generic kernels and the BN / ReLU /
// pool as separate passes over the 112x112x64 activation; here:
//
//   forward   zk_stem_pack_input   x bf16 [B][H][W][Cin] -> xp bf16 [B][Hp][Wp][4]
//                                  (zero border = 'same' padding, channel 3 = 0)
//             zk_stem_pack_weight  w fp32 OHWI -> ws bf16 [KH][Cout][32]
//             zk_stem_conv_fwd     MFMA implicit GEMM, K = KH x (8 px x 4 ch):
//                                  every (pixel, kh) row is ONE contiguous,
//                                  16-B aligned 64-B segment of xp -> LDS-DMA
//                                  ring as in igemm.hip; epilogue: bf16 y1 and
//                                  per-block BN partial sums of the stored values
//             zk_bn_finalize_partials  partial sums -> BN coefficients
//             zk_stem_pool_fwd     relu(BN1(y1)) -> 3x3/2 max pool (+argmax tap)
//                                  and per-block partial sums for BN2
//   backward  zk_stem_pool_bwd_sums  BN1 backward sums from the pooled side
//                                  (the pool gradient is sparse: one tap each)
//             zk_stem_dy1          dense dy1 = k1 * relu'(u) * scatter(dp) + k0 - k3*y1
//             zk_stem_wgrad        MFMA implicit GEMM dW = dy1^T . windows(xp),
//                                  split-K, fp32 atomics into the OHWI gradient
#include "mfma_common.h"

namespace {

struct StemGeom {
  int B, H, W, Cin, Cout, KH, KW, s, pt, pl, Ho, Wo, Hp, Wp;
};

constexpr int SEG = 64;  // bytes of one (pixel, kh) K-row: 8 pixels x 4 ch bf16

// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void stem_pack_input_kernel(const uint16_t* __restrict__ x,
                                                              uint2* __restrict__ xp,
                                                              StemGeom g) {
  const long long total = (long long)g.B * g.Hp * g.Wp;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int wp = (int)(i % g.Wp);
    const long long r = i / g.Wp;
    const int hp = (int)(r % g.Hp);
    const int b = (int)(r / g.Hp);
    const int h = hp - g.pt, w = wp - g.pl;
    uint16_t v[4] = {0, 0, 0, 0};
    if (h >= 0 && h < g.H && w >= 0 && w < g.W) {
      const uint16_t* src = x + (((long long)b * g.H + h) * g.W + w) * g.Cin;
      for (int c = 0; c < g.Cin; ++c) v[c] = src[c];
    }
    xp[i] = make_uint2(v[0] | ((uint32_t)v[1] << 16), v[2] | ((uint32_t)v[3] << 16));
  }
}

// Cin == 3 with an even left pad: two padded pixels per thread -- their 12
// input bytes are three aligned dwords (w even), their 16 output bytes one
// aligned uint4 -- instead of three 2-byte loads and one 8-byte store per
// pixel (the load instruction count bound the one-pixel form).
__global__ __launch_bounds__(256) void stem_pack_input3_kernel(const uint16_t* __restrict__ x,
                                                               uint4* __restrict__ xp,
                                                               StemGeom g) {
  const int Wp2 = g.Wp / 2;
  const long long total = (long long)g.B * g.Hp * Wp2;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int wq = (int)(i % Wp2);
    const long long r = i / Wp2;
    const int hp = (int)(r % g.Hp);
    const int b = (int)(r / g.Hp);
    const int h = hp - g.pt, w = 2 * wq - g.pl;  // w even
    uint32_t o[4] = {0u, 0u, 0u, 0u};
    if (h >= 0 && h < g.H) {
      const uint16_t* row = x + ((long long)b * g.H + h) * g.W * 3;
      if (w >= 0 && w + 1 < g.W) {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(row + (long long)w * 3);
        const uint32_t d0 = src[0], d1 = src[1], d2 = src[2];  // c0 c1 | c2 c0' | c1' c2'
        o[0] = d0;
        o[1] = d1 & 0xffffu;
        o[2] = (d1 >> 16) | (d2 << 16);
        o[3] = d2 >> 16;
      } else {
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const int wk = w + k;
          if (wk >= 0 && wk < g.W) {
            const uint16_t* px = row + (long long)wk * 3;
            o[2 * k] = px[0] | ((uint32_t)px[1] << 16);
            o[2 * k + 1] = px[2];
          }
        }
      }
    }
    xp[i] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

// w fp32 [Cout][KH][KW][Cin] -> ws bf16 [KH][Cout][32]: j = kw*4 + c
__global__ void stem_pack_weight_kernel(const float* __restrict__ w, uint16_t* __restrict__ ws,
                                        StemGeom g) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int total = g.KH * g.Cout * 32;
  if (i >= total) return;
  const int j = i % 32, co = (i / 32) % g.Cout, kh = i / (32 * g.Cout);
  const int kw = j / 4, c = j % 4;
  float v = 0.f;
  if (kw < g.KW && c < g.Cin) v = w[((co * g.KH + kh) * g.KW + kw) * g.Cin + c];
  ws[i] = zk::f32_to_bf16(v);
}

// ---------------------------------------------------------------------------
// conv forward: tile BM pixels x 64 output channels, K-step = one kh row.
// ---------------------------------------------------------------------------
template <int BM, int WM, int WN, int NS>
__global__ __launch_bounds__(WM * WN * 64, 1) void stem_conv_fwd_kernel(
    const unsigned char* __restrict__ xp, const unsigned char* __restrict__ ws,
    uint16_t* __restrict__ y, float* __restrict__ part, StemGeom g, int m_tiles) {
  constexpr int BN = 64, CB = SEG, NWAVES = WM * WN;
  constexpr int SPR = CB / 16, RPI = 1024 / CB, SH = 2;
  constexpr int A_INS = BM / RPI / NWAVES, B_INS = BN / RPI / NWAVES;
  static_assert(A_INS >= 1 && B_INS >= 1, "tile");
  constexpr int LPS = A_INS + B_INS;
  constexpr int STAGE = (BM + BN) * CB;
  constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 32, TN = WTN / 32;

  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave / WN, wn = wave % WN;
  const int L = xcd_linear(blockIdx.x, gridDim.x);
  const int mtile = L % m_tiles, ntile = L / m_tiles;
  if (ntile >= g.Cout / BN) return;
  const long long M = (long long)g.B * g.Ho * g.Wo;
  const long long m0 = (long long)mtile * BM;
  const int n0 = ntile * BN;
  const unsigned char* zp = reinterpret_cast<const unsigned char*>(g_zero_page);
  const int lrow = lane / SPR, lslot = lane % SPR;

  const unsigned char* a_src[A_INS];
  const long long rowb = (long long)g.Wp * 8;  // bytes per padded image row
#pragma unroll
  for (int j = 0; j < A_INS; ++j) {
    const int r = (j * NWAVES + wave) * RPI + lrow;
    const int sw = lslot ^ ((r >> SH) & (SPR - 1));
    const long long m = m0 + r;
    if (m < M) {
      const int wo = (int)(m % g.Wo);
      const long long q = m / g.Wo;
      const int ho = (int)(q % g.Ho), b = (int)(q / g.Ho);
      a_src[j] = xp + ((long long)b * g.Hp + (long long)ho * g.s) * rowb +
                 (long long)wo * g.s * 8 + sw * 16;
    } else {
      a_src[j] = nullptr;
    }
  }
  auto issue = [&](int kh) {
    unsigned char* st = smem + (kh % NS) * STAGE;
#pragma unroll
    for (int j = 0; j < A_INS; ++j) {
      const unsigned char* src = a_src[j] ? a_src[j] + kh * rowb : zp;
      ZK_GLDS16(src, st + (j * NWAVES + wave) * 1024);
    }
#pragma unroll
    for (int j = 0; j < B_INS; ++j) {
      const int r = (j * NWAVES + wave) * RPI + lrow;
      const int sw = lslot ^ ((r >> SH) & (SPR - 1));
      ZK_GLDS16(ws + ((long long)kh * g.Cout + n0 + r) * CB + sw * 16,
                st + BM * CB + (j * NWAVES + wave) * 1024);
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  const int r32 = lane & 31, h = lane >> 5;
  const int NK = g.KH;
#pragma unroll
  for (int p = 0; p < NS - 1; ++p)
    if (p < NK) issue(p);
  for (int ks = 0; ks < NK; ++ks) {
    if (ks + NS - 2 < NK)
      wait_vmcnt<LPS * (NS - 2)>();
    else
      wait_vmcnt<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (ks + NS - 1 < NK) issue(ks + NS - 1);
    const unsigned char* st = smem + (ks % NS) * STAGE;
#pragma unroll
    for (int sub = 0; sub < CB / 32; ++sub) {
      const int chunk = 2 * sub + h;
      uint4 af[TM], bfr[TN];
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        const int row = wm * WTM + a * 32 + r32;
        af[a] = *reinterpret_cast<const uint4*>(st + row * CB +
                                                ((chunk ^ ((row >> SH) & (SPR - 1))) * 16));
      }
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int row = wn * WTN + b * 32 + r32;
        bfr[b] = *reinterpret_cast<const uint4*>(st + BM * CB + row * CB +
                                                 ((chunk ^ ((row >> SH) & (SPR - 1))) * 16));
      }
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) acc[a][b] = mfma_bf16(af[a], bfr[b], acc[a][b]);
    }
  }

  // epilogue: bf16 y1 + partial sums of the STORED values.  D[pixel][co]:
  // lane = channel, registers = pixels, so the per-channel sums are in-lane
  // adds plus one exchange between the two wave halves.
  float csum[TN], csq[TN];
#pragma unroll
  for (int b = 0; b < TN; ++b) csum[b] = csq[b] = 0.f;
#pragma unroll
  for (int a = 0; a < TM; ++a) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const long long mc = m0 + wm * WTM + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      const bool live = mc < M;
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const uint16_t hv = zk::f32_to_bf16(acc[a][b][r]);
        const float v = live ? zk::bf16_to_f32(hv) : 0.f;
        csum[b] += v;
        csq[b] += v * v;
        if (live) y[mc * g.Cout + n0 + wn * WTN + b * 32 + r32] = hv;
      }
    }
  }
  __builtin_amdgcn_s_barrier();
  float* red = reinterpret_cast<float*>(smem);  // [WM][2][BN]
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    const float s1 = csum[b] + __shfl_xor(csum[b], 32, 64);
    const float s2 = csq[b] + __shfl_xor(csq[b], 32, 64);
    if (h == 0) {
      const int nl = wn * WTN + b * 32 + r32;
      red[(wm * 2 + 0) * BN + nl] = s1;
      red[(wm * 2 + 1) * BN + nl] = s2;
    }
  }
  __syncthreads();
  for (int c = tid; c < 2 * BN; c += NWAVES * 64) {
    const int which = c / BN, nl = c % BN;
    float tot = 0.f;
#pragma unroll
    for (int i = 0; i < WM; ++i) tot += red[(i * 2 + which) * BN + nl];
    part[((long long)mtile * 2 + which) * g.Cout + n0 + nl] = tot;
  }
}

// ---------------------------------------------------------------------------
// partial sums [nb][2][C] (fp32) -> BN coefficients [4][C] (scale, shift,
// mean, rstd) + Keras-momentum running statistics (Bessel-corrected var).
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void bn_finalize_partials_kernel(
    const T* __restrict__ part, int nb, int C, double P, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, float momentum, float* __restrict__ rmean,
    float* __restrict__ rvar, float* __restrict__ coef) {
  const int c = blockIdx.x;
  double s1 = 0, s2 = 0;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) {
    s1 += (double)part[((long long)i * 2) * C + c];
    s2 += (double)part[((long long)i * 2 + 1) * C + c];
  }
  __shared__ double r1[256], r2[256];
  r1[threadIdx.x] = s1;
  r2[threadIdx.x] = s2;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      r1[threadIdx.x] += r1[threadIdx.x + o];
      r2[threadIdx.x] += r2[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double mean = r1[0] / P;
    double var = r2[0] / P - mean * mean;
    if (var < 0) var = 0;
    const float rstd = (float)(1.0 / sqrt(var + (double)eps));
    const float gm = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
    coef[c] = gm * rstd;
    coef[C + c] = bt - (float)mean * gm * rstd;
    coef[2 * C + c] = (float)mean;
    coef[3 * C + c] = rstd;
    if (rmean) {
      const double unb = P > 1 ? var * P / (P - 1) : var;
      rmean[c] = momentum * rmean[c] + (1.f - momentum) * (float)mean;
      rvar[c] = momentum * rvar[c] + (1.f - momentum) * (float)unb;
    }
  }
}

// First pass of the two-pass finalize: [nb][n] fp32 partial rows -> [G][n]
// fp64 (block b sums a contiguous range of rows, each thread one column over
// every (256/n)-th row: coalesced rows instead of one strided column per
// block; fixed order, deterministic).  n | 256.
__global__ __launch_bounds__(256) void partials_colsum_kernel(const float* __restrict__ part,
                                                              int nb, int n, int rows_per_block,
                                                              double* __restrict__ out) {
  const int col = threadIdx.x % n, rg = threadIdx.x / n, RG = 256 / n;
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(nb, r0 + rows_per_block);
  double s = 0;
  for (int r = r0 + rg; r < r1; r += RG) s += part[(long long)r * n + col];
  __shared__ double red[256];
  red[threadIdx.x] = s;
  __syncthreads();
  if (rg == 0) {
    for (int k = 1; k < RG; ++k) s += red[k * n + col];
    out[(long long)blockIdx.x * n + col] = s;
  }
}

// partial sums [nb][n] -> out[n] (fp32, accumulated in fp64)
__global__ __launch_bounds__(256) void reduce_partials_kernel(const float* __restrict__ part,
                                                              int nb, int n,
                                                              float* __restrict__ out) {
  const int j = blockIdx.x;
  double s = 0;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) s += part[(long long)i * n + j];
  __shared__ double r[256];
  r[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) r[threadIdx.x] += r[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[j] = (float)r[0];
}

__device__ __forceinline__ void ld8(const uint16_t* p, float (&v)[8]) {
  const uint4 q = *reinterpret_cast<const uint4*>(p);
  const uint32_t u[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[2 * k] = zk::bf16_to_f32((uint16_t)(u[k] & 0xffff));
    v[2 * k + 1] = zk::bf16_to_f32((uint16_t)(u[k] >> 16));
  }
}

__device__ __forceinline__ uint4 pack8(const float (&v)[8]) {
  return make_uint4(zk::pack_bf16x2(v[0], v[1]), zk::pack_bf16x2(v[2], v[3]),
                    zk::pack_bf16x2(v[4], v[5]), zk::pack_bf16x2(v[6], v[7]));
}

struct PoolGeom {
  int B, H, W, C, Ho, Wo, k, s, pt, pl;
};

// Block reduction of per-thread channel-group sums into part[blockIdx][2][C];
// block = R rows x CG channel groups.
__device__ __forceinline__ void block_partials(const float (&s1)[8], const float (&s2)[8],
                                               float* part, int C) {
  __shared__ float red[2][256][9];
  const int CG = C / 8, R = 256 / CG;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    red[0][threadIdx.x][k] = s1[k];
    red[1][threadIdx.x][k] = s2[k];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < 2 * C; c += blockDim.x) {
    const int which = c / C, ch = c % C, gq = ch / 8, k = ch % 8;
    float t = 0.f;
    for (int r = 0; r < R; ++r) t += red[which][r * CG + gq][k];
    part[((long long)blockIdx.x * 2 + which) * C + ch] = t;
  }
}

// The pool kernels index pool outputs / channel groups in 32 bits (the
// launchers check the bounds; 64-bit div/mod per output dominated them) and
// take the pool stride / window as template constants when they are the
// ImageNet stems' 3x3/2 (S_ = K_ = 0: from the geometry).

// relu(scale*y1+shift) -> k x k / s max pool ('same', -inf padding); argmax
// tap (0..k*k-1, first maximum); BN2 partial sums of the stored bf16 output.
template <int S_, int K_>
__global__ __launch_bounds__(256) void stem_pool_fwd_kernel(
    const uint16_t* __restrict__ y1, const float* __restrict__ coef, uint16_t* __restrict__ p,
    uint8_t* __restrict__ arg, float* __restrict__ part, PoolGeom g) {
  const int s = S_ ? S_ : g.s, kk = K_ ? K_ : g.k;
  const int CG = g.C / 8, R = 256 / CG;
  const int cg = threadIdx.x % CG;
  float a[8], sh[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    a[k] = coef[cg * 8 + k];
    sh[k] = coef[g.C + cg * 8 + k];
  }
  float s1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int P2 = g.B * g.Ho * g.Wo;
  for (int o = blockIdx.x * R + threadIdx.x / CG; o < P2; o += gridDim.x * R) {
    const int ow = o % g.Wo, q = o / g.Wo;
    const int oh = q % g.Ho, b = q / g.Ho;
    float best[8];
    uint32_t bi[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      best[k] = -1.f;
      bi[k] = 0;
    }
    if constexpr (K_ > 0) {
      // all taps' loads in flight first, then the max scan
      constexpr int KK = K_ * K_;
      uint4 tv[KK];
      uint32_t valid = 0;
#pragma unroll
      for (int t = 0; t < KK; ++t) {
        const int hi = oh * s - g.pt + t / K_, wi = ow * s - g.pl + t % K_;
        const bool ok = hi >= 0 && hi < g.H && wi >= 0 && wi < g.W;
        valid |= (uint32_t)ok << t;
        tv[t] = ok ? *reinterpret_cast<const uint4*>(
                         y1 + ((long long)(b * g.H + hi) * g.W + wi) * g.C + cg * 8)
                   : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int t = 0; t < KK; ++t) {
        if (!((valid >> t) & 1u)) continue;
        float v[8];
        ld8(reinterpret_cast<const uint16_t*>(&tv[t]), v);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float u = fmaxf(fmaf(a[k], v[k], sh[k]), 0.f);
          if (u > best[k]) {
            best[k] = u;
            bi[k] = t;
          }
        }
      }
    } else {
      for (int th = 0; th < kk; ++th) {
        const int hi = oh * s - g.pt + th;
        if (hi < 0 || hi >= g.H) continue;
        for (int tw = 0; tw < kk; ++tw) {
          const int wi = ow * s - g.pl + tw;
          if (wi < 0 || wi >= g.W) continue;
          float v[8];
          ld8(y1 + ((long long)(b * g.H + hi) * g.W + wi) * g.C + cg * 8, v);
          const uint32_t t = th * kk + tw;
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const float u = fmaxf(fmaf(a[k], v[k], sh[k]), 0.f);
            if (u > best[k]) {
              best[k] = u;
              bi[k] = t;
            }
          }
        }
      }
    }
    const uint4 pk = pack8(best);
    const long long off = (long long)o * g.C + cg * 8;
    *reinterpret_cast<uint4*>(p + off) = pk;
    *reinterpret_cast<uint2*>(arg + off) =
        make_uint2(bi[0] | (bi[1] << 8) | (bi[2] << 16) | (bi[3] << 24),
                   bi[4] | (bi[5] << 8) | (bi[6] << 16) | (bi[7] << 24));
    float stored[8];
    ld8(reinterpret_cast<const uint16_t*>(&pk), stored);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      s1[k] += stored[k];
      s2[k] += stored[k] * stored[k];
    }
  }
  if (part) block_partials(s1, s2, part, g.C);
}

// BN1 backward sums (sum du, sum du*yhat) from the pooled side: every pool
// output routes dp to its argmax tap q, du(q) = dp * [u(q) > 0].  The pooled
// value p IS u(q) = gamma*yhat(q) + beta when positive (bf16-rounded), so
// yhat(q) = (p - beta) / gamma needs no gather of y1.  A thread holding a
// channel with |beta| > 8|gamma| (where p's rounding would be amplified) or
// gamma = 0 takes the exact path instead: y1 at the argmax tap, gathered
// with whole-tap vector loads.
template <int S_, int K_>
__global__ __launch_bounds__(256) void stem_pool_bwd_sums_kernel(
    const uint16_t* __restrict__ dp, const uint8_t* __restrict__ arg,
    const uint16_t* __restrict__ y1, const uint16_t* __restrict__ pooled,
    const float* __restrict__ coef, float* __restrict__ part, PoolGeom g) {
  const int s = S_ ? S_ : g.s, kk = K_ ? K_ : g.k;
  const int CG = g.C / 8, R = 256 / CG;
  const int cg = threadIdx.x % CG;
  float mean[8], rstd[8], bet[8], igm[8];
  bool gather = false;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float a = coef[cg * 8 + k], sh = coef[g.C + cg * 8 + k];
    mean[k] = coef[2 * g.C + cg * 8 + k];
    rstd[k] = coef[3 * g.C + cg * 8 + k];
    const float gm = a / rstd[k];  // gamma
    bet[k] = fmaf(a, mean[k], sh);  // beta
    igm[k] = gm != 0.f ? 1.f / gm : 0.f;
    gather |= !(fabsf(gm) > 0.f && fabsf(bet[k]) <= 8.f * fabsf(gm));
  }
  float s1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int P2 = g.B * g.Ho * g.Wo;
  for (int o = blockIdx.x * R + threadIdx.x / CG; o < P2; o += gridDim.x * R) {
    const long long off = (long long)o * g.C + cg * 8;
    float gv[8], pv[8], yh[8];
    ld8(dp + off, gv);
    ld8(pooled + off, pv);
#pragma unroll
    for (int k = 0; k < 8; ++k) yh[k] = (pv[k] - bet[k]) * igm[k];
    if (gather) {
      const int ow = o % g.Wo, q = o / g.Wo;
      const int oh = q % g.Ho, b = q / g.Ho;
      const uint2 av = *reinterpret_cast<const uint2*>(arg + off);
      const uint32_t aw[2] = {av.x, av.y};
      for (int th = 0; th < kk; ++th) {
        const int hi = oh * s - g.pt + th;
        if (hi < 0 || hi >= g.H) continue;
        for (int tw = 0; tw < kk; ++tw) {
          const int wi = ow * s - g.pl + tw;
          if (wi < 0 || wi >= g.W) continue;
          const uint32_t t = th * kk + tw;
          bool any = false;
#pragma unroll
          for (int k = 0; k < 8; ++k) any |= ((aw[k >> 2] >> (8 * (k & 3))) & 0xff) == t;
          if (!any) continue;
          float v[8];
          ld8(y1 + ((long long)(b * g.H + hi) * g.W + wi) * g.C + cg * 8, v);
#pragma unroll
          for (int k = 0; k < 8; ++k)
            if (((aw[k >> 2] >> (8 * (k & 3))) & 0xff) == t) yh[k] = (v[k] - mean[k]) * rstd[k];
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float du = pv[k] > 0.f ? gv[k] : 0.f;
      s1[k] += du;
      s2[k] += du * yh[k];
    }
  }
  block_partials(s1, s2, part, g.C);
}

// Dense BN1/ReLU/pool backward: dy1(q) = k1 * du(q) + k0 - k3 * y1(q) with
// du(q) = relu'(u(q)) * sum of dp over the pool outputs whose argmax is q.
// One thread per (pool cell, 8 channels) writes the s x s input pixels of its
// stride cell; with k <= s + 1 every such pixel is covered only by the pool
// outputs (oh-1..oh) x (ow-1..ow) (pt, pl <= s - 1), whose argmax / dp are
// loaded once, unconditionally.
template <int S_, int K_>
__global__ __launch_bounds__(256) void stem_dy1_kernel(
    const uint16_t* __restrict__ dp, const uint8_t* __restrict__ arg,
    const uint16_t* __restrict__ y1, const float* __restrict__ coef,
    const float* __restrict__ bcoef, uint16_t* __restrict__ dy1, PoolGeom g) {
  const int s = S_ ? S_ : g.s, kk = K_ ? K_ : g.k;
  const int CG = g.C / 8, lg = __builtin_ctz(CG);  // CG divides 256: a power of two
  const int total = g.B * g.Ho * g.Wo * CG;
  // the grid stride is a multiple of CG, so every thread keeps one channel group
  const int cg = (blockIdx.x * blockDim.x + threadIdx.x) & (CG - 1);
  float a1[8], s1v[8], k1[8], k0[8], k3[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int c = cg * 8 + k;
    a1[k] = coef[c];
    s1v[k] = coef[g.C + c];
    k1[k] = bcoef[c];
    k0[k] = bcoef[g.C + c];
    k3[k] = bcoef[2 * g.C + c];
  }
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int o = i >> lg;
    const int ow = o % g.Wo, q = o / g.Wo;
    const int oh = q % g.Ho, b = q / g.Ho;
    // candidate outputs (oh-1+dy, ow-1+dx), dy, dx in {0, 1}
    uint32_t aw[2][2][2];
    float gv[2][2][8];
#pragma unroll
    for (int dy = 0; dy < 2; ++dy)
#pragma unroll
      for (int dx = 0; dx < 2; ++dx) {
        const int ch = oh - 1 + dy, cw = ow - 1 + dx;
        if (ch >= 0 && cw >= 0) {
          const long long oo = ((long long)(b * g.Ho + ch) * g.Wo + cw) * g.C + cg * 8;
          const uint2 av = *reinterpret_cast<const uint2*>(arg + oo);
          aw[dy][dx][0] = av.x;
          aw[dy][dx][1] = av.y;
          ld8(dp + oo, gv[dy][dx]);
        } else {
          aw[dy][dx][0] = aw[dy][dx][1] = 0xFFFFFFFFu;  // tap 255: never matches
#pragma unroll
          for (int k = 0; k < 8; ++k) gv[dy][dx][k] = 0.f;
        }
      }
    // the stride cell's y1 rows: loads in flight before the routing math
    constexpr int SC = S_ > 0 ? S_ * S_ : 4;
    uint4 yq[SC];
    if constexpr (S_ > 0) {
#pragma unroll
      for (int c2 = 0; c2 < SC; ++c2) {
        const int hh = oh * s - g.pt + c2 / S_, ww = ow * s - g.pl + c2 % S_;
        yq[c2] = (hh >= 0 && hh < g.H && ww >= 0 && ww < g.W)
                     ? *reinterpret_cast<const uint4*>(
                           y1 + ((long long)(b * g.H + hh) * g.W + ww) * g.C + cg * 8)
                     : make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int sy = 0; sy < s; ++sy) {
      const int hh = oh * s - g.pt + sy;
      if (hh < 0 || hh >= g.H) continue;
#pragma unroll
      for (int sx = 0; sx < s; ++sx) {
        const int ww = ow * s - g.pl + sx;
        if (ww < 0 || ww >= g.W) continue;
        float du[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int dy = 0; dy < 2; ++dy) {
          const int th = hh - ((oh - 1 + dy) * s - g.pt);
          if (th < 0 || th >= kk) continue;
#pragma unroll
          for (int dx = 0; dx < 2; ++dx) {
            const int tw = ww - ((ow - 1 + dx) * s - g.pl);
            if (tw < 0 || tw >= kk) continue;
            const uint32_t t = th * kk + tw;
#pragma unroll
            for (int k = 0; k < 8; ++k)
              if (((aw[dy][dx][k >> 2] >> (8 * (k & 3))) & 0xff) == t) du[k] += gv[dy][dx][k];
          }
        }
        const long long pix = ((long long)(b * g.H + hh) * g.W + ww) * g.C + cg * 8;
        float yv[8], o8[8];
        if constexpr (S_ > 0)
          ld8(reinterpret_cast<const uint16_t*>(&yq[sy * S_ + sx]), yv);
        else
          ld8(y1 + pix, yv);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float u = fmaf(a1[k], yv[k], s1v[k]);
          o8[k] = k1[k] * (u > 0.f ? du[k] : 0.f) + k0[k] - k3[k] * yv[k];
        }
        *reinterpret_cast<uint4*>(dy1 + pix) = pack8(o8);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// stem weight gradient: dW[co][kh][j] = sum_p dy1[p][co] * xp-window(p, kh)[j]
//   A = dy1 rows (Cout*2 B), B = 8 window segments of 64 B per pixel (the
//   8th reads the zero page when KH < 8); both read transposed from LDS.
// ---------------------------------------------------------------------------
template <int BK, int NS>
__global__ __launch_bounds__(256, 1) void stem_wgrad_kernel(
    const uint16_t* __restrict__ dy1, const unsigned char* __restrict__ xp,
    float* __restrict__ dw, float* __restrict__ slab, StemGeom g, int k_per_split) {
  constexpr int BM = 64, BN = 256, WM = 1, WN = 4, NWAVES = 4;
  constexpr int RA = BM * 2, RBB = BN * 2;
  constexpr int SA = BK * RA, SB = BK * RBB;
  static_assert(SA % (1024 * NWAVES) == 0 && SB % (1024 * NWAVES) == 0, "stage");
  constexpr int A_INS = SA / 1024 / NWAVES, B_INS = SB / 1024 / NWAVES;
  constexpr int LPS = A_INS + B_INS, STAGE = SA + SB;
  constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 32, TN = WTN / 32;

  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = 0, wn = wave;
  const int P = g.B * g.Ho * g.Wo;
  const int kbeg = blockIdx.x * k_per_split;
  if (kbeg >= P) return;
  const int kend = min(P, kbeg + k_per_split);
  const int NK = (kend - kbeg + BK - 1) / BK;
  const unsigned char* dyb = reinterpret_cast<const unsigned char*>(dy1);
  const unsigned char* zp = reinterpret_cast<const unsigned char*>(g_zero_page);
  const float invWo = 1.0f / (float)g.Wo, invHo = 1.0f / (float)g.Ho;
  const long long rowb = (long long)g.Wp * 8;

  int a_row[A_INS], a_byte[A_INS];
#pragma unroll
  for (int j = 0; j < A_INS; ++j) {
    const int off = ((j * NWAVES + wave) * 64 + lane) * 16;
    a_row[j] = off / RA;
    a_byte[j] = (((off % RA) >> 4) ^ tr_swz<RA>(a_row[j])) << 4;
  }
  int b_row[B_INS], b_kh[B_INS], b_in[B_INS];
#pragma unroll
  for (int j = 0; j < B_INS; ++j) {
    const int off = ((j * NWAVES + wave) * 64 + lane) * 16;
    b_row[j] = off / RBB;
    const int chunk = ((off % RBB) >> 4) ^ tr_swz<RBB>(b_row[j]);  // 0..31
    b_kh[j] = chunk >> 2;                                          // 64-B segment = kh
    b_in[j] = (chunk & 3) * 16;
  }
  auto issue = [&](int ks) {
    unsigned char* st = smem + (ks % NS) * STAGE;
    const int k0 = kbeg + ks * BK;
#pragma unroll
    for (int j = 0; j < A_INS; ++j) {
      const int p = k0 + a_row[j];
      ZK_GLDS16(p < kend ? dyb + (long long)p * RA + a_byte[j] : zp,
                st + (j * NWAVES + wave) * 1024);
    }
#pragma unroll
    for (int j = 0; j < B_INS; ++j) {
      const int p = k0 + b_row[j];
      const unsigned char* src = zp;
      if (p < kend && b_kh[j] < g.KH) {
        const int q1 = fdiv(p, g.Wo, invWo);
        const int wo = p - q1 * g.Wo;
        const int b = fdiv(q1, g.Ho, invHo);
        const int ho = q1 - b * g.Ho;
        src = xp + ((long long)b * g.Hp + (long long)ho * g.s + b_kh[j]) * rowb +
              (long long)wo * g.s * 8 + b_in[j];
      }
      ZK_GLDS16(src, st + SA + (j * NWAVES + wave) * 1024);
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
#pragma unroll
  for (int p = 0; p < NS - 1; ++p)
    if (p < NK) issue(p);
  for (int ks = 0; ks < NK; ++ks) {
    if (ks + NS - 2 < NK)
      wait_vmcnt<LPS * (NS - 2)>();
    else
      wait_vmcnt<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (ks + NS - 1 < NK) issue(ks + NS - 1);
    const unsigned char* st = smem + (ks % NS) * STAGE;
#pragma unroll
    for (int sub = 0; sub < BK / 16; ++sub) {
      uint4 af[TM], bfr[TN];
#pragma unroll
      for (int a = 0; a < TM; ++a) af[a] = tr_frag_swz<RA>(st, sub * 16, wm * WTM + a * 32, lane);
#pragma unroll
      for (int b = 0; b < TN; ++b)
        bfr[b] = tr_frag_swz<RBB>(st + SA, sub * 16, wn * WTN + b * 32, lane);
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) acc[a][b] = mfma_bf16(af[a], bfr[b], acc[a][b]);
    }
  }
  // epilogue: column n = kh*32 + kw*4 + c -> OHWI dW[co][kh][kw][c]
  const int h = lane >> 5, r32 = lane & 31;
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = wm * WTM + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int n = wn * WTN + b * 32 + r32;
        const int kh = n >> 5, kw = (n >> 2) & 7, c = n & 3;
        if (kh < g.KH && kw < g.KW && c < g.Cin && co < g.Cout) {
          const int idx = ((co * g.KH + kh) * g.KW + kw) * g.Cin + c;
          if (slab)  // deterministic mode: per-split partials, fixed-order reduce
            slab[(long long)blockIdx.x * g.Cout * g.KH * g.KW * g.Cin + idx] = acc[a][b][r];
          else
            atomicAdd(dw + idx, acc[a][b][r]);
        }
      }
    }
}

template <typename K>
int set_lds(K kern, int bytes) {
  static bool done = false;
  if (!done) {
    hipError_t e =
        hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e != hipSuccess) return (int)e;
    done = true;
  }
  return 0;
}

constexpr int kMaxPoolParts = 4096;

int pool_grid(long long P2, int C) {
  const long long R = 256 / (C / 8);
  long long b = (P2 + R - 1) / R;
  if (b > kMaxPoolParts) b = kMaxPoolParts;
  return b < 1 ? 1 : (int)b;
}

bool stem_ok(const StemGeom& g) {
  return g.Cin >= 1 && g.Cin <= 4 && g.KW <= 8 && g.KH <= 8 && g.Cout % 64 == 0 &&
         g.Wp % 2 == 0 && g.s % 2 == 0 && (g.Wo - 1) * g.s + 8 <= g.Wp && (g.Ho - 1) * g.s + g.KH <= g.Hp;
}

}  // namespace

ZK_EXPORT int zk_stem_pack_input(const void* x, void* xp, int B, int H, int W, int Cin, int Hp,
                                 int Wp, int pt, int pl, hipStream_t st) {
  StemGeom g{B, H, W, Cin, 0, 0, 0, 0, pt, pl, 0, 0, Hp, Wp};
  if (Cin > 4) return (int)hipErrorInvalidValue;
  long long total = (long long)B * Hp * Wp;
  if (Cin == 3 && W % 2 == 0 && Wp % 2 == 0 && pl % 2 == 0 &&
      ((uintptr_t)x & 3) == 0 && ((uintptr_t)xp & 15) == 0) {
    total /= 2;  // two padded pixels per thread
    long long blocks = (total + 255) / 256;
    if (blocks > 16384) blocks = 16384;
    hipLaunchKernelGGL(stem_pack_input3_kernel, dim3((int)blocks), dim3(256), 0, st,
                       (const uint16_t*)x, (uint4*)xp, g);
    ZK_CHECK_LAUNCH();
    return 0;
  }
  long long blocks = (total + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(stem_pack_input_kernel, dim3((int)blocks), dim3(256), 0, st,
                     (const uint16_t*)x, (uint2*)xp, g);
  ZK_CHECK_LAUNCH();
  return 0;
}

ZK_EXPORT int zk_stem_pack_weight(const float* w, void* ws, int Cout, int KH, int KW, int Cin,
                                  hipStream_t st) {
  StemGeom g{0, 0, 0, Cin, Cout, KH, KW, 0, 0, 0, 0, 0, 0, 0};
  const int total = KH * Cout * 32;
  hipLaunchKernelGGL(stem_pack_weight_kernel, dim3((total + 255) / 256), dim3(256), 0, st, w,
                     (uint16_t*)ws, g);
  ZK_CHECK_LAUNCH();
  return 0;
}

// part: [m_tiles][2][Cout] fp32 (returns m_tiles through *nparts)
ZK_EXPORT int zk_stem_conv_fwd(const void* xp, const void* ws, void* y, void* part, int B,
                               int Cin, int Cout, int KH, int KW, int s, int Ho, int Wo, int Hp,
                               int Wp, int variant, int* nparts, hipStream_t st) {
  StemGeom g{B, 0, 0, Cin, Cout, KH, KW, s, 0, 0, Ho, Wo, Hp, Wp};
  if (!stem_ok(g)) return (int)hipErrorInvalidValue;
  const long long M = (long long)B * Ho * Wo;
#define ZK_STEM_FWD(BM, WM, WN, NS)                                                         \
  {                                                                                         \
    auto kern = stem_conv_fwd_kernel<BM, WM, WN, NS>;                                       \
    const int lds = NS * (BM + 64) * SEG;                                                   \
    if (int e = set_lds(kern, lds)) return e;                                               \
    const int mt = (int)((M + BM - 1) / BM);                                                \
    if (nparts) *nparts = mt;                                                               \
    hipLaunchKernelGGL(kern, dim3(mt * (Cout / 64)), dim3(WM * WN * 64), lds, st,           \
                       (const unsigned char*)xp, (const unsigned char*)ws, (uint16_t*)y,    \
                       (float*)part, g, mt);                                                \
    break;                                                                                  \
  }
  // default: 128-pixel tiles at ImageNet batch >= ~330 (tools/tune_stem.py,
  // batch 512: 450 us vs 555 us for the 256-pixel tiles tuned at batch 256)
  if (variant < 0) variant = M >= 4 * 1024 * 1024 ? 3 : 0;
  switch (variant) {
    case 0: ZK_STEM_FWD(256, 4, 1, 3)
    case 1: ZK_STEM_FWD(128, 2, 2, 4)
    case 2: ZK_STEM_FWD(256, 2, 2, 4)
    case 3: ZK_STEM_FWD(128, 2, 2, 3)
    default: return (int)hipErrorInvalidValue;
  }
#undef ZK_STEM_FWD
  ZK_CHECK_LAUNCH();
  return 0;
}

ZK_EXPORT int zk_stem_max_pool_parts() { return kMaxPoolParts; }

ZK_EXPORT int zk_stem_max_parts(int B, int Ho, int Wo) {
  // upper bound of m_tiles over the variants (BM >= 128)
  return (int)(((long long)B * Ho * Wo + 127) / 128);
}

ZK_EXPORT int zk_bn_finalize_partials(const void* part, int nb, int C, double P,
                                      const void* gamma, const void* beta, float eps,
                                      float momentum, void* rmean, void* rvar, void* coef,
                                      hipStream_t st) {
  hipLaunchKernelGGL(bn_finalize_partials_kernel<float>, dim3(C), dim3(256), 0, st,
                     (const float*)part, nb, C, P, (const float*)gamma, (const float*)beta, eps,
                     momentum, (float*)rmean, (float*)rvar, (float*)coef);
  ZK_CHECK_LAUNCH();
  return 0;
}

// zk_bn_finalize_partials for many partial rows (the stem conv writes one
// per 128- or 256-pixel tile: ~25-50k at batch 512): a coalesced first pass
// into ws ([256][2C] fp64, zk_bn_finalize_ws_bytes) then the finalize over
// 256 rows.  Falls back to the one-pass form when 2C does not divide 256.
ZK_EXPORT long long zk_bn_finalize_ws_bytes(int C) { return 256LL * 2 * C * 8; }

ZK_EXPORT int zk_bn_finalize_partials_ws(const void* part, int nb, int C, double P,
                                         const void* gamma, const void* beta, float eps,
                                         float momentum, void* rmean, void* rvar, void* coef,
                                         void* ws, hipStream_t st) {
  const int n = 2 * C;
  if (!ws || n > 256 || 256 % n || nb < 1024)
    return zk_bn_finalize_partials(part, nb, C, P, gamma, beta, eps, momentum, rmean, rvar, coef,
                                   st);
  constexpr int G = 256;
  const int rpb = (nb + G - 1) / G;
  hipLaunchKernelGGL(partials_colsum_kernel, dim3(G), dim3(256), 0, st, (const float*)part, nb,
                     n, rpb, (double*)ws);
  hipLaunchKernelGGL(bn_finalize_partials_kernel<double>, dim3(C), dim3(256), 0, st,
                     (const double*)ws, G, C, P, (const float*)gamma, (const float*)beta, eps,
                     momentum, (float*)rmean, (float*)rvar, (float*)coef);
  ZK_CHECK_LAUNCH();
  return 0;
}

ZK_EXPORT int zk_reduce_partials(const void* part, int nb, int n, void* out, hipStream_t st) {
  hipLaunchKernelGGL(reduce_partials_kernel, dim3(n), dim3(256), 0, st, (const float*)part, nb,
                     n, (float*)out);
  ZK_CHECK_LAUNCH();
  return 0;
}

// part may be null (no BN after the pool).  Returns the number of partial
// rows written through *nparts.
ZK_EXPORT int zk_stem_pool_fwd(const void* y1, const void* coef, void* p, void* arg, void* part,
                               int B, int H, int W, int C, int Ho, int Wo, int k, int s, int pt,
                               int pl, int* nparts, hipStream_t st) {
  if (C % 8 || 256 % (C / 8) || k * k > 255 || (long long)B * Ho * Wo >= (1LL << 31))
    return (int)hipErrorInvalidValue;
  PoolGeom g{B, H, W, C, Ho, Wo, k, s, pt, pl};
  const int grid = pool_grid((long long)B * Ho * Wo, C);
  if (nparts) *nparts = grid;
  auto kern = (s == 2 && k == 3) ? stem_pool_fwd_kernel<2, 3> : stem_pool_fwd_kernel<0, 0>;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, st, (const uint16_t*)y1, (const float*)coef,
                     (uint16_t*)p, (uint8_t*)arg, (float*)part, g);
  ZK_CHECK_LAUNCH();
  return 0;
}

// pooled: the pool output p of zk_stem_pool_fwd (relu'd BN-1 values at the
// argmax taps), read instead of gathering y1 there.
ZK_EXPORT int zk_stem_pool_bwd_sums(const void* dp, const void* arg, const void* y1,
                                    const void* pooled, const void* coef, void* part, int B, int H,
                                    int W, int C, int Ho, int Wo, int k, int s, int pt, int pl,
                                    int* nparts, hipStream_t st) {
  if (C % 8 || 256 % (C / 8) || (long long)B * Ho * Wo >= (1LL << 31))
    return (int)hipErrorInvalidValue;
  PoolGeom g{B, H, W, C, Ho, Wo, k, s, pt, pl};
  const int grid = pool_grid((long long)B * Ho * Wo, C);
  if (nparts) *nparts = grid;
  auto kern =
      (s == 2 && k == 3) ? stem_pool_bwd_sums_kernel<2, 3> : stem_pool_bwd_sums_kernel<0, 0>;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, st, (const uint16_t*)dp,
                     (const uint8_t*)arg, (const uint16_t*)y1, (const uint16_t*)pooled,
                     (const float*)coef, (float*)part, g);
  ZK_CHECK_LAUNCH();
  return 0;
}

ZK_EXPORT int zk_stem_dy1(const void* dp, const void* arg, const void* y1, const void* coef,
                          const void* bcoef, void* dy1, int B, int H, int W, int C, int Ho,
                          int Wo, int k, int s, int pt, int pl, hipStream_t st) {
  // scatter-block form: needs k <= s + 1, pads < s, and the stride cells to
  // cover the input (Ho*s >= H + pt)
  if (C % 8 || 256 % (C / 8) || k > s + 1 || pt >= s || pl >= s || pt < 0 || pl < 0 ||
      (long long)Ho * s < H + pt || (long long)Wo * s < W + pl)
    return (int)hipErrorInvalidValue;
  const long long work = (long long)B * Ho * Wo * (C / 8);
  if (work >= (1LL << 31)) return (int)hipErrorInvalidValue;
  PoolGeom g{B, H, W, C, Ho, Wo, k, s, pt, pl};
  long long blocks = (work + 255) / 256;
  if (blocks > 32768) blocks = 32768;
  auto kern = (s == 2 && k == 3) ? stem_dy1_kernel<2, 3> : stem_dy1_kernel<0, 0>;
  hipLaunchKernelGGL(kern, dim3((int)blocks), dim3(256), 0, st, (const uint16_t*)dp,
                     (const uint8_t*)arg, (const uint16_t*)y1, (const float*)coef,
                     (const float*)bcoef, (uint16_t*)dy1, g);
  ZK_CHECK_LAUNCH();
  return 0;
}

// Splits (blocks) of zk_stem_wgrad: its deterministic-mode slab is
// [splits][Cout*KH*KW*Cin] fp32.
ZK_EXPORT int zk_stem_wgrad_splits(int B, int Ho, int Wo, int target_blocks) {
  const long long P = (long long)B * Ho * Wo;
  if (target_blocks <= 0) target_blocks = 1024;
  long long kps = (P + target_blocks - 1) / target_blocks;
  kps = (kps + 31) / 32 * 32;
  return (int)((P + kps - 1) / kps);
}

// dw: fp32 OHWI [Cout][KH][KW][Cin], accumulated (zeroed by the caller or the
// flat gradient buffer) with fp32 atomics, or with slab (deterministic mode,
// zeroed by the caller) as per-split partials for zk_wgrad_slab_reduce.
// Cout must be 64.
ZK_EXPORT int zk_stem_wgrad(const void* dy1, const void* xp, void* dw, void* slab, int B,
                            int Cin, int Cout, int KH, int KW, int s, int Ho, int Wo, int Hp,
                            int Wp, int target_blocks, hipStream_t st) {
  StemGeom g{B, 0, 0, Cin, Cout, KH, KW, s, 0, 0, Ho, Wo, Hp, Wp};
  if (!stem_ok(g) || Cout != 64) return (int)hipErrorInvalidValue;
  const long long P = (long long)B * Ho * Wo;
  if (P >= (1 << 24)) return (int)hipErrorInvalidValue;
  constexpr int BK = 32, NS = 3;
  auto kern = stem_wgrad_kernel<BK, NS>;
  const int lds = NS * BK * (64 + 256) * 2;
  if (int e = set_lds(kern, lds)) return e;
  if (target_blocks <= 0) target_blocks = 1024;
  long long kps = (P + target_blocks - 1) / target_blocks;
  kps = (kps + BK - 1) / BK * BK;
  const long long splits = (P + kps - 1) / kps;
  hipLaunchKernelGGL(kern, dim3((unsigned)splits), dim3(256), lds, st, (const uint16_t*)dy1,
                     (const unsigned char*)xp, (float*)dw, (float*)slab, g, (int)kps);
  ZK_CHECK_LAUNCH();
  return 0;
}
