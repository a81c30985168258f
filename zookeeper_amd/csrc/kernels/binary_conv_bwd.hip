// Backward of the binary convolution on MFMA (gfx950, bf16 in / fp32 acc).
//
// With the straight-through estimator the gradients of a ±1 x ±1 conv are
// real-valued GEMMs whose other operand is exactly ±1 (exact in bf16):
//
//   dgrad  dX[m=(b,hi,wi), n=ci] = sum_{t, co} dY[(b,ho,wo), co] * S[co,t,ci]
//          (ho,wo) = ((hi+pt-kh)/s, (wi+pl-kw)/s) when integral and in range
//          epilogue: dx = dX * 1{|x| <= clip} (STE mask bits) + dres  -> bf16
//   wgrad  dW[co, (t,ci)] = sum_{p=(b,ho,wo)} dY[p, co] * sign(x)[p shifted by t, ci]
//          epilogue: * 1{|w| <= clip} (kernel STE), fp32 atomics (split-K)
//
// Both are implicit GEMMs on v_mfma_f32_32x32x16_bf16 with LDS-staged tiles:
//   * dgrad: A = gathered dY rows (K = Cout contiguous), B = S^T stored
//     [t][ci][co] (K contiguous) -> fragments are 16-B ds_read_b128 rows;
//   * wgrad: K = pixels is the outer (strided) dimension of both operands,
//     so tiles are staged [k][m] / [k][n] with coalesced 16-B loads and the
//     MFMA fragments are read with the gfx950 transposing LDS read
//     ds_read_b64_tr_b16.  The sign(x) operand is never materialised: the
//     loader reads the packed sign bits (1 bit/element) and expands 32 of
//     them to 32 bf16 ±1 values straight into LDS (16x less HBM traffic).
// Tiles: 256 threads = 4 waves in a WM x WN grid, each wave TM x TN 32x32
// MFMA tiles, BK = 32, register-prefetch double buffering.
#include "../common.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int NT = 256;
constexpr int BK = 32;

struct Geom {
  int B, H, W, Cin, Ho, Wo, Cout, kh, kw, s, pt, pl;
};

__device__ __forceinline__ f32x16 mfma32(const uint4& a, const uint4& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// ===========================================================================
// dgrad
// ===========================================================================
template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(NT, 2) void bconv_dgrad_kernel(
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ wt,
    const uint32_t* __restrict__ mask, const uint16_t* __restrict__ dres,
    uint16_t* __restrict__ dx, Geom g) {
  static_assert(WM * WN == 4, "4 waves");
  constexpr int WTM = BM / WM, WTN = BN / WN;  // wave tile
  constexpr int TM = WTM / 32, TN = WTN / 32;
  constexpr int LDK = BK + 8;                  // padded row (80 B): conflict-free b128 reads
  constexpr int A_CH = BM * BK / 8 / NT;       // 16-B chunks per thread
  constexpr int B_CH = BN * BK / 8 / NT;
  static_assert(A_CH >= 1 && B_CH >= 1, "tile too small");

  __shared__ __attribute__((aligned(16))) uint16_t As[BM * LDK];
  __shared__ __attribute__((aligned(16))) uint16_t Bs[BN * LDK];

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int wm = wave / WN, wn = wave % WN;
  const long long M = (long long)g.B * g.H * g.W;
  const long long m0 = (long long)blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int T = g.kh * g.kw;
  const int kchunks = g.Cout / BK;  // Cout % 32 == 0

  // Loader: chunk i -> (row = i / 4, c8 = i % 4) (4 chunks of 8 bf16 per 32-wide row).
  int a_row[A_CH], a_c8[A_CH], a_b[A_CH], a_h[A_CH], a_w[A_CH];
#pragma unroll
  for (int j = 0; j < A_CH; ++j) {
    const int i = tid + j * NT;
    a_row[j] = i >> 2;
    a_c8[j] = i & 3;
    const long long m = m0 + a_row[j];
    if (m < M) {
      a_w[j] = (int)(m % g.W);
      const long long r = m / g.W;
      a_h[j] = (int)(r % g.H);
      a_b[j] = (int)(r / g.H);
    } else {
      a_b[j] = -1;
      a_h[j] = a_w[j] = 0;
    }
  }
  uint4 ra[A_CH], rb[B_CH];
  auto load = [&](int kc) {
    const int t = kc / kchunks;
    const int co0 = (kc % kchunks) * BK;
    const int th = t / g.kw, tw = t % g.kw;
#pragma unroll
    for (int j = 0; j < A_CH; ++j) {
      uint4 v = make_uint4(0, 0, 0, 0);
      if (a_b[j] >= 0) {
        const int hn = a_h[j] + g.pt - th, wn_ = a_w[j] + g.pl - tw;
        if (hn >= 0 && wn_ >= 0 && hn % g.s == 0 && wn_ % g.s == 0) {
          const int ho = hn / g.s, wo = wn_ / g.s;
          if (ho < g.Ho && wo < g.Wo)
            v = *reinterpret_cast<const uint4*>(
                dy + (((long long)a_b[j] * g.Ho + ho) * g.Wo + wo) * g.Cout + co0 + 8 * a_c8[j]);
        }
      }
      ra[j] = v;
    }
#pragma unroll
    for (int j = 0; j < B_CH; ++j) {
      const int i = tid + j * NT;
      const int row = i >> 2, c8 = i & 3;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (n0 + row < g.Cin)
        v = *reinterpret_cast<const uint4*>(wt + ((long long)t * g.Cin + n0 + row) * g.Cout +
                                            co0 + 8 * c8);
      rb[j] = v;
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int j = 0; j < A_CH; ++j)
      *reinterpret_cast<uint4*>(&As[a_row[j] * LDK + 8 * a_c8[j]]) = ra[j];
#pragma unroll
    for (int j = 0; j < B_CH; ++j) {
      const int i = tid + j * NT;
      *reinterpret_cast<uint4*>(&Bs[(i >> 2) * LDK + 8 * (i & 3)]) = rb[j];
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
  const int nk = T * kchunks;
  load(0);
  for (int kc = 0; kc < nk; ++kc) {
    if (kc) __syncthreads();
    store();
    __syncthreads();
    if (kc + 1 < nk) load(kc + 1);
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      uint4 af[TM], bfr[TN];
#pragma unroll
      for (int a = 0; a < TM; ++a)
        af[a] = *reinterpret_cast<const uint4*>(
            &As[(wm * WTM + a * 32 + r32) * LDK + ks * 16 + 8 * h]);
#pragma unroll
      for (int b = 0; b < TN; ++b)
        bfr[b] = *reinterpret_cast<const uint4*>(
            &Bs[(wn * WTN + b * 32 + r32) * LDK + ks * 16 + 8 * h]);
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) acc[a][b] = mfma32(af[a], bfr[b], acc[a][b]);
    }
  }

  // Epilogue: STE mask + residual gradient, bf16 store.
  const int CW = g.Cin >> 5;
#pragma unroll
  for (int a = 0; a < TM; ++a) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = wm * WTM + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      const long long m = m0 + row;
      if (m >= M) continue;
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int n = n0 + wn * WTN + b * 32 + r32;
        if (n >= g.Cin) continue;
        float v = acc[a][b][r];
        if (mask && !((mask[m * CW + (n >> 5)] >> (n & 31)) & 1u)) v = 0.f;
        if (dres) v += zk::bf16_to_f32(dres[m * g.Cin + n]);
        dx[m * g.Cin + n] = zk::f32_to_bf16(v);
      }
    }
  }
}

// ===========================================================================
// wgrad
// ===========================================================================
// Transposed fragment read: lane gets column (c0 + l&15) of rows k0..k0+3
// from a [k][m] bf16 tile with row stride `ld` elements.
__device__ __forceinline__ s16x4 tr_read(const uint16_t* base, int ld, int row, int col) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(base + row * ld + col));
}

// 32x32x16 operand (8 k-values of one row/column) from a [k][m] LDS tile:
// lane l: group g = l>>4, i = l&15, q = i>>2, p = i&3; read s covers k rows
// 8*(g>>1) + 4s + q, columns 16*(g&1) + 4p .. +3 (relative to the 32-col tile).
__device__ __forceinline__ uint4 tr_frag(const uint16_t* tile, int ld, int k0, int c0, int lane) {
  const int gq = lane >> 4, i = lane & 15;
  const int q = i >> 2, p = i & 3;
  const int row = k0 + 8 * (gq >> 1) + q;
  const int col = c0 + 16 * (gq & 1) + 4 * p;
  const s16x4 lo = tr_read(tile, ld, row, col);
  const s16x4 hi = tr_read(tile, ld, row + 4, col);
  const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(uint4, v);
}

template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(NT, 2) void bconv_wgrad_kernel(
    const uint16_t* __restrict__ dy, const uint32_t* __restrict__ xbits,
    const float* __restrict__ w, float* __restrict__ dw, Geom g, int pad_ones, float clip,
    long long k_per_split) {
  static_assert(WM * WN == 4, "4 waves");
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  constexpr int LDA = BM + 8, LDB = BN + 8;      // padded rows
  constexpr int A_CH = BK * BM / 8 / NT;         // 16-B chunks of dY per thread
  constexpr int BWORDS = BK * (BN / 32);         // packed words of a B stage
  static_assert(A_CH >= 1, "tile");

  __shared__ __attribute__((aligned(16))) uint16_t As[BK * LDA];
  __shared__ __attribute__((aligned(16))) uint16_t Bs[BK * LDB];

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int wm = wave / WN, wn = wave % WN;
  const long long P = (long long)g.B * g.Ho * g.Wo;
  const int m0 = blockIdx.x * BM;                 // co
  const int ntile_per_tap = g.Cin / BN;
  const int t = blockIdx.y / ntile_per_tap;       // tap
  const int ci0 = (blockIdx.y % ntile_per_tap) * BN;
  const int th = t / g.kw, tw = t % g.kw;
  const long long kbeg = (long long)blockIdx.z * k_per_split;
  long long kend = kbeg + k_per_split;
  if (kend > P) kend = P;
  const int CW = g.Cin >> 5;

  uint4 ra[A_CH];
  uint32_t rb = 0;
  int rb_valid = 0;
  auto load = [&](long long k0) {
#pragma unroll
    for (int j = 0; j < A_CH; ++j) {
      const int i = tid + j * NT;
      const int kr = i / (BM / 8), c8 = i % (BM / 8);
      const long long p = k0 + kr;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (p < kend && m0 + 8 * c8 < g.Cout)
        v = *reinterpret_cast<const uint4*>(dy + p * g.Cout + m0 + 8 * c8);
      ra[j] = v;
    }
    rb_valid = 0;
    if (tid < BWORDS) {
      const int kr = tid / (BN / 32), wd = tid % (BN / 32);
      const long long p = k0 + kr;
      uint32_t v = 0;
      if (p < kend) {
        const int wo = (int)(p % g.Wo);
        const long long r = p / g.Wo;
        const int ho = (int)(r % g.Ho);
        const int b = (int)(r / g.Ho);
        const int hi = ho * g.s - g.pt + th, wi = wo * g.s - g.pl + tw;
        if (hi >= 0 && hi < g.H && wi >= 0 && wi < g.W) {
          v = xbits[(((long long)b * g.H + hi) * g.W + wi) * CW + (ci0 >> 5) + wd];
          rb_valid = 1;
        } else if (pad_ones) {
          v = 0xFFFFFFFFu;  // +1 padding
          rb_valid = 1;
        }  // zero padding: the row contributes nothing (expanded as 0, not -1)
      }
      rb = v;
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int j = 0; j < A_CH; ++j) {
      const int i = tid + j * NT;
      const int kr = i / (BM / 8), c8 = i % (BM / 8);
      *reinterpret_cast<uint4*>(&As[kr * LDA + 8 * c8]) = ra[j];
    }
    if (tid < BWORDS) {
      const int kr = tid / (BN / 32), wd = tid % (BN / 32);
      uint16_t* dst = &Bs[kr * LDB + 32 * wd];
      // Expand 32 sign bits into 32 bf16 (+1 = 0x3F80, -1 = 0xBF80); rows past
      // the split end and zero-padded taps are 0 (no contribution).
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint32_t v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int k = q * 8 + e * 2;
          const uint32_t lo = rb_valid ? (((rb >> k) & 1) ? 0x3F80u : 0xBF80u) : 0u;
          const uint32_t hi = rb_valid ? (((rb >> (k + 1)) & 1) ? 0x3F80u : 0xBF80u) : 0u;
          v[e] = lo | (hi << 16);
        }
        *reinterpret_cast<uint4*>(dst + 8 * q) = make_uint4(v[0], v[1], v[2], v[3]);
      }
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  if (kbeg < kend) {
    load(kbeg);
    for (long long k0 = kbeg; k0 < kend; k0 += BK) {
      if (k0 != kbeg) __syncthreads();
      store();
      __syncthreads();
      if (k0 + BK < kend) load(k0 + BK);
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
        uint4 af[TM], bfr[TN];
#pragma unroll
        for (int a = 0; a < TM; ++a) af[a] = tr_frag(As, LDA, ks * 16, wm * WTM + a * 32, lane);
#pragma unroll
        for (int b = 0; b < TN; ++b) bfr[b] = tr_frag(Bs, LDB, ks * 16, wn * WTN + b * 32, lane);
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b) acc[a][b] = mfma32(af[a], bfr[b], acc[a][b]);
      }
    }
  }

  // Epilogue: kernel STE mask, split-K accumulation with fp32 atomics into
  // dW [Cout][T][Cin] (OHWI, the channels_last layout of the latent kernel).
  const int h = lane >> 5, r32 = lane & 31;
#pragma unroll
  for (int a = 0; a < TM; ++a) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = m0 + wm * WTM + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (co >= g.Cout) continue;
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int ci = ci0 + wn * WTN + b * 32 + r32;
        const long long idx = ((long long)co * (g.kh * g.kw) + t) * g.Cin + ci;
        const float v = acc[a][b][r];
        if (fabsf(w[idx]) <= clip) atomicAdd(dw + idx, v);
      }
    }
  }
}

}  // namespace

// wt: ±1 bf16 [T][Cin][Cout]; mask/dres optional.  Requires Cout % 32 == 0,
// Cin % 64 == 0.
ZK_EXPORT int zk_bconv_dgrad(const void* dy, const void* wt, const void* mask, const void* dres,
                             void* dx, int B, int H, int W, int Cin, int Ho, int Wo, int Cout,
                             int kh, int kw, int stride, int pt, int pl, hipStream_t stream) {
  if (Cout % BK || Cin % 64) return (int)hipErrorInvalidValue;
  Geom g{B, H, W, Cin, Ho, Wo, Cout, kh, kw, stride, pt, pl};
  const long long M = (long long)B * H * W;
  if (Cin % 128 == 0) {
    dim3 grid((unsigned)((M + 127) / 128), Cin / 128);
    hipLaunchKernelGGL((bconv_dgrad_kernel<128, 128, 2, 2>), grid, dim3(NT), 0, stream,
                       (const uint16_t*)dy, (const uint16_t*)wt, (const uint32_t*)mask,
                       (const uint16_t*)dres, (uint16_t*)dx, g);
  } else {
    dim3 grid((unsigned)((M + 127) / 128), Cin / 64);
    hipLaunchKernelGGL((bconv_dgrad_kernel<128, 64, 4, 1>), grid, dim3(NT), 0, stream,
                       (const uint16_t*)dy, (const uint16_t*)wt, (const uint32_t*)mask,
                       (const uint16_t*)dres, (uint16_t*)dx, g);
  }
  ZK_CHECK_LAUNCH();
  return 0;
}

// dw fp32 [Cout][T][Cin] must be zeroed by the caller.  Requires Cout % 64
// == 0 and Cin % 64 == 0.
ZK_EXPORT int zk_bconv_wgrad(const void* dy, const void* xbits, const void* w, void* dw, int B,
                             int H, int W, int Cin, int Ho, int Wo, int Cout, int kh, int kw,
                             int stride, int pt, int pl, int pad_ones, float clip,
                             int target_blocks, hipStream_t stream) {
  if (Cout % 64 || Cin % 64) return (int)hipErrorInvalidValue;
  Geom g{B, H, W, Cin, Ho, Wo, Cout, kh, kw, stride, pt, pl};
  const long long P = (long long)B * Ho * Wo;
  const int T = kh * kw;
  const int BMv = (Cout % 128 == 0) ? 128 : 64;
  const int BNv = (Cin % 128 == 0) ? 128 : 64;
  const long long tiles = (long long)(Cout / BMv) * T * (Cin / BNv);
  long long splits = (target_blocks + tiles - 1) / tiles;
  const long long max_splits = (P + 255) / 256;  // keep >= 256 pixels per split
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  long long kps = (P + splits - 1) / splits;
  kps = (kps + BK - 1) / BK * BK;
  splits = (P + kps - 1) / kps;
  dim3 grid(Cout / BMv, (unsigned)(T * (Cin / BNv)), (unsigned)splits);
#define ZK_WG(bm, bn, wm, wn)                                                                \
  hipLaunchKernelGGL((bconv_wgrad_kernel<bm, bn, wm, wn>), grid, dim3(NT), 0, stream,         \
                     (const uint16_t*)dy, (const uint32_t*)xbits, (const float*)w, (float*)dw, \
                     g, pad_ones, clip, kps)
  if (BMv == 128 && BNv == 128)
    ZK_WG(128, 128, 2, 2);
  else if (BMv == 128)
    ZK_WG(128, 64, 4, 1);
  else if (BNv == 128)
    ZK_WG(64, 128, 1, 4);
  else
    ZK_WG(64, 64, 2, 2);
#undef ZK_WG
  ZK_CHECK_LAUNCH();
  return 0;
}
