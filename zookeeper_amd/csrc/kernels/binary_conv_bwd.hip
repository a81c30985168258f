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
// Both are implicit GEMMs on v_mfma_f32_32x32x16_bf16, LDS-staged, BK = 64,
// register-prefetch double buffering (global loads for stage k+1 are issued
// before the MFMAs of stage k), 4 waves per workgroup.
//
//   * dgrad computes the TRANSPOSED product D[ci][pixel] = S^T . dY^T (A and
//     B fragments swapped) so every lane owns one pixel and 4 consecutive
//     channels per accumulator group: the fused epilogue (STE mask word,
//     residual gradient, bf16 store) moves 8 B per access instead of 2 B.
//     Operands are K-contiguous (dY rows: Cout; S^T stored [t][ci][co]) ->
//     fragments are ds_read_b128 rows of 144-B padded LDS rows.
//   * wgrad: K = pixels is the strided dimension of both operands, so tiles
//     are staged [k][m] / [k][n] with coalesced 16-B loads and fragments are
//     read with the gfx950 transposing LDS read ds_read_b64_tr_b16.  The
//     sign(x) operand is never materialised: the loader reads the packed sign
//     bits and expands 32 of them into 32 bf16 ±1 values in LDS.  N runs over
//     (tap, ci) flattened and a 192-wide tile spans several taps when Cin is
//     small, so the 64-channel stage still gets 3 MFMA tiles per wave.
#include "../common.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int NT = 256;

struct Geom {
  int B, H, W, Cin, Ho, Wo, Cout, kh, kw, s, pt, pl;
};

// XCD-aware block mapping (speed only, never correctness).  Blocks are
// dealt round-robin over the 8 XCDs, so blocks L and L+8 share an L2.  For a
// gx x gy grid with gy | 8, give every XCD one fixed N-tile (`ny`) and a
// contiguous share of the M-tiles: the B panel of that N-tile then stays
// resident in that XCD's L2 instead of being re-fetched by all 8.
__device__ __forceinline__ void xcd_remap_2d(int gx, int gy, int& mx, int& ny) {
  const int L = blockIdx.x + gx * blockIdx.y;
  if (gy <= 8 && (8 % gy) == 0 && ((long long)gx * gy) % 8 == 0) {
    const int xcd = L & 7, k = L >> 3;
    const int groups = 8 / gy;
    ny = xcd % gy;
    mx = (xcd / gy) + groups * k;
  } else {
    mx = blockIdx.x;
    ny = blockIdx.y;
  }
}

__device__ __forceinline__ f32x16 mfma32(const uint4& a, const uint4& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// ===========================================================================
// dgrad:  tile BM pixels x BN input channels; waves WM x WN
// ===========================================================================
template <int BM, int BN, int WM, int WN, int BK, int OCC>
__global__ __launch_bounds__(NT, OCC) void bconv_dgrad_kernel(
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ wt,
    const uint32_t* __restrict__ mask, const uint16_t* __restrict__ dres,
    uint16_t* __restrict__ dx, Geom g) {
  static_assert(WM * WN == 4, "4 waves");
  constexpr int WTM = BM / WM, WTN = BN / WN;  // wave tile (pixels x channels)
  constexpr int TM = WTM / 32, TN = WTN / 32;
  constexpr int LDK = BK + 8;                  // 144-B rows
  constexpr int CPR = BK / 8;                  // 16-B chunks per row
  constexpr int A_CH = BM * CPR / NT;
  constexpr int B_CH = BN * CPR / NT;
  static_assert(A_CH >= 1 && B_CH >= 1, "tile too small");

  __shared__ __attribute__((aligned(16))) uint16_t As[BM * LDK];
  __shared__ __attribute__((aligned(16))) uint16_t Bs[BN * LDK];

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int wm = wave / WN, wn = wave % WN;
  int mtile, ntile;
  xcd_remap_2d(gridDim.x, gridDim.y, mtile, ntile);
  // Stride-s dgrad is split into s*s parity classes of input pixels
  // (blockIdx.z); a class only receives the taps whose offset matches its
  // parity, so no MFMA work is spent on structurally-zero taps.
  const int s = g.s;
  const int ph = blockIdx.z / s, pw = blockIdx.z % s;
  const int Hc = (g.H - ph + s - 1) / s, Wc = (g.W - pw + s - 1) / s;
  const long long M = (long long)g.B * Hc * Wc;  // pixels of this class
  const long long m0 = (long long)mtile * BM;
  if (m0 >= M) return;
  const int n0 = ntile * BN;
  const int kchunks = g.Cout / BK;
  int th_list[3], tw_list[3], nth = 0, ntw = 0;
  for (int k = 0; k < g.kh && nth < 3; ++k)
    if ((ph + g.pt - k) % s == 0) th_list[nth++] = k;
  for (int k = 0; k < g.kw && ntw < 3; ++k)
    if ((pw + g.pl - k) % s == 0) tw_list[ntw++] = k;
  const int T = nth * ntw;

  int a_b[A_CH], a_h[A_CH], a_w[A_CH];
#pragma unroll
  for (int j = 0; j < A_CH; ++j) {
    const int row = (tid + j * NT) / CPR;
    const long long m = m0 + row;
    if (m < M) {
      const int jw = (int)(m % Wc);
      const long long r = m / Wc;
      a_h[j] = (int)(r % Hc) * s + ph;
      a_w[j] = jw * s + pw;
      a_b[j] = (int)(r / Hc);
    } else {
      a_b[j] = -1;
      a_h[j] = a_w[j] = 0;
    }
  }
  uint4 ra[A_CH], rb[B_CH];
  auto load = [&](int kc) {
    const int ti = kc / kchunks;
    const int co0 = (kc % kchunks) * BK;
    const int th = th_list[ti / ntw], tw = tw_list[ti % ntw];
    const int t = th * g.kw + tw;
#pragma unroll
    for (int j = 0; j < A_CH; ++j) {
      const int c8 = (tid + j * NT) % CPR;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (a_b[j] >= 0) {
        const int hn = a_h[j] + g.pt - th, wn_ = a_w[j] + g.pl - tw;  // divisible by s
        if (hn >= 0 && wn_ >= 0) {
          const int ho = hn / s, wo = wn_ / s;
          if (ho < g.Ho && wo < g.Wo)
            v = *reinterpret_cast<const uint4*>(
                dy + (((long long)a_b[j] * g.Ho + ho) * g.Wo + wo) * g.Cout + co0 + 8 * c8);
        }
      }
      ra[j] = v;
    }
#pragma unroll
    for (int j = 0; j < B_CH; ++j) {
      const int i = tid + j * NT;
      const int row = i / CPR, c8 = i % CPR;
      rb[j] = *reinterpret_cast<const uint4*>(wt + ((long long)t * g.Cin + n0 + row) * g.Cout +
                                              co0 + 8 * c8);
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int j = 0; j < A_CH; ++j) {
      const int i = tid + j * NT;
      *reinterpret_cast<uint4*>(&As[(i / CPR) * LDK + 8 * (i % CPR)]) = ra[j];
    }
#pragma unroll
    for (int j = 0; j < B_CH; ++j) {
      const int i = tid + j * NT;
      *reinterpret_cast<uint4*>(&Bs[(i / CPR) * LDK + 8 * (i % CPR)]) = rb[j];
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
  if (nk > 0) load(0);
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
      // Transposed product: rows = channels (B), columns = pixels (A).
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) acc[a][b] = mfma32(bfr[b], af[a], acc[a][b]);
    }
  }

  // Epilogue: lane = pixel, 4 consecutive channels per register group.
  const int CW = g.Cin >> 5;
#pragma unroll
  for (int a = 0; a < TM; ++a) {
    const long long mc = m0 + wm * WTM + a * 32 + r32;
    if (mc >= M) continue;
    const int jw = (int)(mc % Wc);
    const long long rr = mc / Wc;
    const long long m =
        ((rr / Hc) * g.H + (long long)(rr % Hc) * s + ph) * g.W + (long long)jw * s + pw;
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int nb = n0 + wn * WTN + b * 32;  // 32-aligned: one mask word
      const uint32_t mw = mask ? mask[m * CW + (nb >> 5)] : 0xFFFFFFFFu;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int nl = 8 * q + 4 * h;  // channel offset within the 32-block
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          v[e] = ((mw >> (nl + e)) & 1u) ? acc[a][b][4 * q + e] : 0.f;
        const long long off = m * g.Cin + nb + nl;
        if (dres) {
          const uint2 d = *reinterpret_cast<const uint2*>(dres + off);
          v[0] += zk::bf16_to_f32((uint16_t)(d.x & 0xffff));
          v[1] += zk::bf16_to_f32((uint16_t)(d.x >> 16));
          v[2] += zk::bf16_to_f32((uint16_t)(d.y & 0xffff));
          v[3] += zk::bf16_to_f32((uint16_t)(d.y >> 16));
        }
        *reinterpret_cast<uint2*>(dx + off) =
            make_uint2(zk::pack_bf16x2(v[0], v[1]), zk::pack_bf16x2(v[2], v[3]));
      }
    }
  }
}

// ===========================================================================
// wgrad:  tile BM output channels x BN (tap, ci) columns; K = pixels
// ===========================================================================
__device__ __forceinline__ s16x4 tr_read(const uint16_t* base, int ld, int row, int col) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(base + row * ld + col));
}

// 32x32x16 operand (8 k-values of one row/column) from a [k][m] LDS tile:
// lane l: group g = l>>4, i = l&15, q = i>>2, p = i&3; read s covers k rows
// 8*(g>>1) + 4s + q, columns 16*(g&1) + 4p .. +3 of the 32-wide block.
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

template <int BM, int BN, int WM, int WN, int BK, int OCC>
__global__ __launch_bounds__(NT, OCC) void bconv_wgrad_kernel(
    const uint16_t* __restrict__ dy, const uint32_t* __restrict__ xbits,
    const float* __restrict__ w, float* __restrict__ dw, Geom g, int pad_ones, float clip,
    long long k_per_split) {
  static_assert(WM * WN == 4, "4 waves");
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  constexpr int LDA = BM + 8, LDB = BN + 8;
  constexpr int A_CH = BK * BM / 8 / NT;     // 16-B chunks of dY per thread
  constexpr int WPR = BN / 32;               // packed words per B row
  constexpr int B_W = (BK * WPR + NT - 1) / NT;
  static_assert(A_CH >= 1, "tile");

  __shared__ __attribute__((aligned(16))) uint16_t As[BK * LDA];
  __shared__ __attribute__((aligned(16))) uint16_t Bs[BK * LDB];

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int wm = wave / WN, wn = wave % WN;
  const long long P = (long long)g.B * g.Ho * g.Wo;
  // XCD-aware mapping: all (co, n) tiles of one K-split run on one XCD, so
  // the split's dY rows and sign bits are fetched into a single L2.
  int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  {
    const int gx = gridDim.x, gy = gridDim.y, gz = gridDim.z;
    if (gz % 8 == 0) {
      const long long L = blockIdx.x + (long long)gx * (blockIdx.y + (long long)gy * blockIdx.z);
      const int xcd = (int)(L & 7);
      const long long k = L >> 3;
      const long long tiles = (long long)gx * gy;
      bz = xcd + 8 * (int)(k / tiles);
      const int tile = (int)(k % tiles);
      bx = tile % gx;
      by = tile / gx;
    }
  }
  const int m0 = bx * BM;   // co
  const int n0 = by * BN;   // flattened (t, ci)
  const long long kbeg = (long long)bz * k_per_split;
  long long kend = kbeg + k_per_split;
  if (kend > P) kend = P;
  const int CW = g.Cin >> 5;

  // Per-thread B word columns are fixed: word wd of the tile -> tap / word.
  int b_tap[B_W], b_wrd[B_W];
#pragma unroll
  for (int j = 0; j < B_W; ++j) {
    const int i = tid + j * NT;
    const int wd = i % WPR;
    const int n = n0 + 32 * wd;
    b_tap[j] = n / g.Cin;
    b_wrd[j] = (n % g.Cin) >> 5;
  }

  uint4 ra[A_CH];
  uint32_t rb[B_W];
  uint32_t rb_ok = 0;
  auto load = [&](long long k0) {
#pragma unroll
    for (int j = 0; j < A_CH; ++j) {
      const int i = tid + j * NT;
      const int kr = i / (BM / 8), c8 = i % (BM / 8);
      const long long p = k0 + kr;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (p < kend) v = *reinterpret_cast<const uint4*>(dy + p * g.Cout + m0 + 8 * c8);
      ra[j] = v;
    }
    rb_ok = 0;
#pragma unroll
    for (int j = 0; j < B_W; ++j) {
      const int i = tid + j * NT;
      uint32_t v = 0;
      if (i < BK * WPR) {
        const long long p = k0 + i / WPR;
        if (p < kend) {
          const int wo = (int)(p % g.Wo);
          const long long r = p / g.Wo;
          const int ho = (int)(r % g.Ho);
          const int b = (int)(r / g.Ho);
          const int t = b_tap[j];
          const int hi = ho * g.s - g.pt + t / g.kw, wi = wo * g.s - g.pl + t % g.kw;
          if (hi >= 0 && hi < g.H && wi >= 0 && wi < g.W) {
            v = xbits[(((long long)b * g.H + hi) * g.W + wi) * CW + b_wrd[j]];
            rb_ok |= 1u << j;
          } else if (pad_ones) {
            v = 0xFFFFFFFFu;
            rb_ok |= 1u << j;
          }  // zero padding: contributes 0 (not -1)
        }
      }
      rb[j] = v;
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int j = 0; j < A_CH; ++j) {
      const int i = tid + j * NT;
      const int kr = i / (BM / 8), c8 = i % (BM / 8);
      *reinterpret_cast<uint4*>(&As[kr * LDA + 8 * c8]) = ra[j];
    }
#pragma unroll
    for (int j = 0; j < B_W; ++j) {
      const int i = tid + j * NT;
      if (i >= BK * WPR) continue;
      const int kr = i / WPR, wd = i % WPR;
      uint16_t* dst = &Bs[kr * LDB + 32 * wd];
      const bool ok = (rb_ok >> j) & 1u;
      const uint32_t bits = rb[j];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint32_t v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int k = q * 8 + e * 2;
          const uint32_t lo = ok ? (((bits >> k) & 1) ? 0x3F80u : 0xBF80u) : 0u;
          const uint32_t hi = ok ? (((bits >> (k + 1)) & 1) ? 0x3F80u : 0xBF80u) : 0u;
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

  // Epilogue: kernel STE mask, split-K fp32 atomics into dW [Cout][T*Cin]
  // (OHWI, the channels_last layout of the latent kernel); each
  // wave-instruction adds 2 x 128 contiguous bytes.
  const int h = lane >> 5, r32 = lane & 31;
  const int NTOT = g.kh * g.kw * g.Cin;
#pragma unroll
  for (int a = 0; a < TM; ++a) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = m0 + wm * WTM + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int n = n0 + wn * WTN + b * 32 + r32;
        const long long idx = (long long)co * NTOT + n;
        if (fabsf(w[idx]) <= clip) atomicAdd(dw + idx, acc[a][b][r]);
      }
    }
  }
}

}  // namespace

// ---------------------------------------------------------------------------
// Host entry points.  `variant` selects a tile configuration (-1 = the
// built-in heuristic, tuned on MI355X with tools/tune_bconv.py).
// ---------------------------------------------------------------------------
namespace {

template <int BM, int BN, int WM, int WN, int BK, int OCC>
int launch_dgrad(const void* dy, const void* wt, const void* mask, const void* dres, void* dx,
                 const Geom& g, hipStream_t stream) {
  if (g.Cout % BK || g.Cin % BN) return (int)hipErrorInvalidValue;
  const long long Mc = (long long)g.B * ((g.H + g.s - 1) / g.s) * ((g.W + g.s - 1) / g.s);
  hipLaunchKernelGGL((bconv_dgrad_kernel<BM, BN, WM, WN, BK, OCC>),
                     dim3((unsigned)((Mc + BM - 1) / BM), g.Cin / BN, g.s * g.s), dim3(NT), 0,
                     stream,
                     (const uint16_t*)dy, (const uint16_t*)wt, (const uint32_t*)mask,
                     (const uint16_t*)dres, (uint16_t*)dx, g);
  return 0;
}

template <int BM, int BN, int WM, int WN, int BK, int OCC>
int launch_wgrad(const void* dy, const void* xbits, const void* w, void* dw, const Geom& g,
                 int pad_ones, float clip, int target_blocks, hipStream_t stream) {
  const int NTOT = g.kh * g.kw * g.Cin;
  if (g.Cout % BM || NTOT % BN) return (int)hipErrorInvalidValue;
  const long long P = (long long)g.B * g.Ho * g.Wo;
  const long long tiles = (long long)(g.Cout / BM) * (NTOT / BN);
  long long splits = (target_blocks + tiles - 1) / tiles;
  const long long max_splits = (P + 8 * BK - 1) / (8 * BK);  // >= 8 K-steps per split
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  long long kps = (P + splits - 1) / splits;
  kps = (kps + BK - 1) / BK * BK;
  splits = (P + kps - 1) / kps;
  if (splits >= 8) splits = (splits + 7) / 8 * 8;  // XCD mapping wants gz % 8 == 0
  hipLaunchKernelGGL((bconv_wgrad_kernel<BM, BN, WM, WN, BK, OCC>),
                     dim3(g.Cout / BM, (unsigned)(NTOT / BN), (unsigned)splits), dim3(NT), 0,
                     stream, (const uint16_t*)dy, (const uint32_t*)xbits, (const float*)w,
                     (float*)dw, g, pad_ones, clip, kps);
  return 0;
}

int dgrad_variant(int v, const void* dy, const void* wt, const void* mask, const void* dres,
                  void* dx, const Geom& g, hipStream_t st) {
  switch (v) {
    case 0: return launch_dgrad<128, 128, 2, 2, 64, 2>(dy, wt, mask, dres, dx, g, st);
    case 1: return launch_dgrad<256, 64, 4, 1, 64, 2>(dy, wt, mask, dres, dx, g, st);
    case 2: return launch_dgrad<128, 64, 2, 2, 64, 3>(dy, wt, mask, dres, dx, g, st);
    case 3: return launch_dgrad<64, 64, 2, 2, 64, 4>(dy, wt, mask, dres, dx, g, st);
    case 4: return launch_dgrad<128, 64, 4, 1, 64, 3>(dy, wt, mask, dres, dx, g, st);
    case 5: return launch_dgrad<128, 128, 2, 2, 32, 2>(dy, wt, mask, dres, dx, g, st);
    case 6: return launch_dgrad<128, 64, 2, 2, 32, 4>(dy, wt, mask, dres, dx, g, st);
    case 7: return launch_dgrad<64, 64, 2, 2, 32, 4>(dy, wt, mask, dres, dx, g, st);
    default: return (int)hipErrorInvalidValue;
  }
}

int wgrad_variant(int v, const void* dy, const void* xb, const void* w, void* dw, const Geom& g,
                  int po, float clip, int tb, hipStream_t st) {
  switch (v) {
    case 0: return launch_wgrad<128, 192, 2, 2, 64, 2>(dy, xb, w, dw, g, po, clip, tb, st);
    case 1: return launch_wgrad<64, 192, 2, 2, 64, 2>(dy, xb, w, dw, g, po, clip, tb, st);
    case 2: return launch_wgrad<128, 64, 2, 2, 64, 3>(dy, xb, w, dw, g, po, clip, tb, st);
    case 3: return launch_wgrad<64, 64, 2, 2, 64, 4>(dy, xb, w, dw, g, po, clip, tb, st);
    case 4: return launch_wgrad<128, 192, 2, 2, 32, 2>(dy, xb, w, dw, g, po, clip, tb, st);
    case 5: return launch_wgrad<64, 192, 2, 2, 32, 3>(dy, xb, w, dw, g, po, clip, tb, st);
    case 6: return launch_wgrad<128, 64, 2, 2, 32, 4>(dy, xb, w, dw, g, po, clip, tb, st);
    case 7: return launch_wgrad<64, 64, 2, 2, 32, 4>(dy, xb, w, dw, g, po, clip, tb, st);
    default: return (int)hipErrorInvalidValue;
  }
}

}  // namespace

// wt: ±1 bf16 [T][Cin][Cout]; mask / dres optional.  Requires Cout % 64 == 0
// and Cin % 64 == 0.
ZK_EXPORT int zk_bconv_dgrad(const void* dy, const void* wt, const void* mask, const void* dres,
                             void* dx, int B, int H, int W, int Cin, int Ho, int Wo, int Cout,
                             int kh, int kw, int stride, int pt, int pl, int variant,
                             hipStream_t stream) {
  if (Cout % 64 || Cin % 64) return (int)hipErrorInvalidValue;
  Geom g{B, H, W, Cin, Ho, Wo, Cout, kh, kw, stride, pt, pl};
  // Tuned on MI355X (tools/tune_bconv.py, E18 shapes, batch 256): the
  // 64x64 / BK=32 tile at 4 workgroups per CU wins every shape.
  if (variant < 0) variant = 7;
  const int rc = dgrad_variant(variant, dy, wt, mask, dres, dx, g, stream);
  if (rc) return rc;
  ZK_CHECK_LAUNCH();
  return 0;
}

// dw fp32 [Cout][T][Cin] must be zeroed by the caller.  Requires Cout % 64
// == 0 and Cin % 64 == 0.
ZK_EXPORT int zk_bconv_wgrad(const void* dy, const void* xbits, const void* w, void* dw, int B,
                             int H, int W, int Cin, int Ho, int Wo, int Cout, int kh, int kw,
                             int stride, int pt, int pl, int pad_ones, float clip,
                             int target_blocks, int variant, hipStream_t stream) {
  if (Cout % 64 || Cin % 64) return (int)hipErrorInvalidValue;
  Geom g{B, H, W, Cin, Ho, Wo, Cout, kh, kw, stride, pt, pl};
  const int NTOT = kh * kw * Cin;
  if (variant < 0) {
    // Tuned on MI355X (tools/tune_bconv.py): strided layers and the
    // 64-channel stage prefer smaller tiles, deep layers the 128x192 tile.
    if (NTOT % 192 != 0)
      variant = 3;
    else if (stride > 1)
      variant = 3;
    else if (Cout == 64)
      variant = 5;
    else
      variant = (Cout >= 256) ? 4 : 0;
  }
  if (target_blocks <= 0) {
    // Tuned split-K sizes (tools/tune_bconv.py): variants 3/5 like 1024-2048
    // workgroups, the 128x192 tiles 512.
    target_blocks = (variant == 0 || variant == 4) ? 512 : (variant == 3 ? 2048 : 1024);
  }
  const int rc = wgrad_variant(variant, dy, xbits, w, dw, g, pad_ones, clip, target_blocks,
                               stream);
  if (rc) return rc;
  ZK_CHECK_LAUNCH();
  return 0;
}
