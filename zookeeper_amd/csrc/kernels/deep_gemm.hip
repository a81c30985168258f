// Phased 256x256 MFMA implicit GEMM for the data gradient of the deep-stage
// stride-1 3x3 binary convolutions (C >= 256: BinaryResNet-E18 / QuickNet
// stages 3-4), gfx950.
//
//   dx[p][ci] = mask(x)[p][ci] * sum_{tap, co} dY[p - shift(tap)][co] * S[tap][ci][co]
//             + dres[p][ci]
//
// A K = 9 * Cout GEMM per output pixel (M = pixels, N = Cin).  The generic
// implicit GEMM (igemm.hip) runs it with one barrier per 64-deep K-step and a
// 2-stage ring: 0.6-0.9 PF/s.  This kernel is the dense-GEMM schedule of
// tools/gemm_lab/g8.hip (cdna_hip_programming.md §5, the phased 256^2
// template) with the conv's gather in its loader:
//   * block 512 threads = 8 waves, 2 (ci) x 4 (pixels); wave tile 128 ci x 64
//     pixels as 8 x 4 accumulators of v_mfma_f32_16x16x32_bf16, computed
//     transposed (A = weight rows, B = dY pixel rows) so that in the epilogue a
//     lane owns one pixel and 4 consecutive channels (8-B mask / residual /
//     dx accesses);
//   * a K-tile (64 output channels of one tap) is staged as four 16 KB pieces
//     [256 rows][64 B] -- (S, k 0-31), (dY, k 0-31), (S, k 32-63), (dY, k
//     32-63) -- by global_load_lds_dwordx4, two LDS buffers (128 KB); dY rows
//     are gathered per lane (tap shift; rows outside the image read the zero
//     page), so padding costs no masking;
//   * 4 phases per K-tile, 16 MFMAs each; phase p issues piece p of the NEXT
//     K-tile and reads the next phase's fragments into the other register
//     set while its own MFMAs run; counted vmcnt(4) + one raw s_barrier at
//     phases 1 and 3 only, so two pieces stay in flight across every barrier;
//   * LDS image: 64-B rows, 16-B chunk c of row r at slot c ^ f(r), f =
//     {0,2,3,1}[(r>>2)&3]: conflict-free ds_read_b128 for the 16x16x32 operand
//     map (lane l: row l&15, chunk l>>4); the DMA writes LDS linearly, so the
//     swizzle is applied to the source chunk.
// Reference anchor: the QuantConv2D stack whose backward this is
// (/root/reference/examples/larq_experiment.py:62-99).
#include "mfma_common.h"
#include "splitk_tree.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int DP_PIECE = 16384;         // 256 rows x 64 B
constexpr int DP_BUF = 4 * DP_PIECE;    // one K-tile
constexpr int DP_LDS = 2 * DP_BUF;      // two K-tiles: 128 KB
constexpr int DP_NT = 512;

__device__ __forceinline__ int dp_swz(int r) {  // r: row within its 16-row block
  return (0x1320 >> (4 * ((r >> 2) & 3))) & 3;  // {0,2,3,1}
}

__device__ __forceinline__ f32x4 dp_mfma(const uint4& a, const uint4& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

__device__ __forceinline__ void dp_barrier() { asm volatile("s_barrier" ::: "memory"); }

struct DeepDgradArgs {
  const uint16_t* dy;    // [B][Ho][Wo][Cout]
  const uint16_t* wt;    // S^T [kh*kw][Cin][Cout] bf16
  const uint32_t* mask;  // STE mask bits [B*H*W][Cin/32] (optional)
  const uint16_t* dres;  // residual gradient [B][H][W][Cin] (optional)
  uint16_t* dx;          // [B][H][W][Cin]
  int B, H, W, Cin, Cout;
  int Ho, Wo, kh, kw, s, pt, pl;
  int m_tiles;           // 256-pixel tiles of the largest stride-parity class
};

// BNC: input channels per block (256; the launcher instantiates only that):
// the weight pieces hold BNC rows, a wave's A rows are BNC / 2 in two phase
// halves of FA = BNC / 64 fragments.
template <int BNC>
__global__ __launch_bounds__(DP_NT, 1) void dgrad_deep_kernel(DeepDgradArgs a) {
  constexpr int WP = BNC * 64;              // weight piece bytes
  constexpr int BUF = 2 * WP + 2 * DP_PIECE;
  constexpr int WINS = BNC / 16 / 8;        // weight-piece glds per wave
  constexpr int FA = BNC / 64;              // A fragments per phase half
  constexpr int OFF_K1 = WP + DP_PIECE;     // buffer layout: W k0 | dY k0 | W k1 | dY k1
  constexpr int VM2 = WINS + 2;             // vm ops per wave of one (S, dY) piece pair
  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 2, wn = wave & 3;  // ci half, pixel quarter
  // XCD-aware order: consecutive logical ids = pixel tiles of one ci tile
  const int L = xcd_linear(blockIdx.x, gridDim.x);
  const int mt = L % a.m_tiles, ct = L / a.m_tiles;
  // stride-parity class (blockIdx.y) of the input pixels: h = hc*s + ph.  Its
  // taps are th = th0 + i*s (i < nth), reading output row ho = hc + dh0 - i
  const int s = a.s;
  const int ph = blockIdx.y / s, pw = blockIdx.y - (blockIdx.y / s) * s;
  const int Hc = (a.H - ph + s - 1) / s, Wc = (a.W - pw + s - 1) / s;
  const int th0 = (ph + a.pt) % s, tw0 = (pw + a.pl) % s;
  const int nth = (a.kh - th0 + s - 1) / s, ntw = (a.kw - tw0 + s - 1) / s;
  const int dh0 = (ph + a.pt - th0) / s, dw0 = (pw + a.pl - tw0) / s;
  const long long P = (long long)a.B * Hc * Wc;  // pixels of the class
  const long long m0 = (long long)mt * 256;
  if (m0 >= P || nth <= 0 || ntw <= 0) return;  // block-uniform
  const int n0 = ct * BNC;
  const int KC = a.Cout >> 6;  // K-tiles per tap
  const int NKT = nth * ntw * KC;
  const long long rowb = (long long)a.Cout * 2;  // bytes per dY / S row

  // ---- loader: instruction i of wave w fills piece rows (i*8 + w)*16 ..
  // +15; lane l -> row l >> 2, LDS slot l & 3 holding global chunk
  // (l & 3) ^ f(row)
  const int lrow = lane >> 2, lslot = lane & 3;
  const int gch = lslot ^ dp_swz(lrow);
  const unsigned char* zp = reinterpret_cast<const unsigned char*>(g_zero_page) + gch * 16;
  const unsigned char* wsrc[WINS];  // S row ci, tap 0, k 0
  const unsigned char* dsrc[2];     // dY row of tap (th0, tw0), k 0
  uint32_t vh[2], vw[2];            // bit i / j: tap (i, j)'s dY row / column is inside the image
#pragma unroll
  for (int i = 0; i < WINS; ++i) {
    const int r = (i * 8 + wave) * 16 + lrow;
    wsrc[i] = reinterpret_cast<const unsigned char*>(a.wt) + (long long)(n0 + r) * rowb + gch * 16;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = (i * 8 + wave) * 16 + lrow;
    const long long m = m0 + r;
    vh[i] = vw[i] = 0;
    dsrc[i] = reinterpret_cast<const unsigned char*>(a.dy) + gch * 16;
    if (m < P) {
      const int wc = (int)(m % Wc);
      const long long q = m / Wc;
      const int hc = (int)(q % Hc);
      const long long b = q / Hc;
      const int ho0 = hc + dh0, wo0 = wc + dw0;
      for (int t = 0; t < nth; ++t) vh[i] |= (uint32_t)((unsigned)(ho0 - t) < (unsigned)a.Ho) << t;
      for (int t = 0; t < ntw; ++t) vw[i] |= (uint32_t)((unsigned)(wo0 - t) < (unsigned)a.Wo) << t;
      dsrc[i] += ((b * a.Ho + ho0) * a.Wo + wo0) * rowb;
    }
  }
  const long long wtap = (long long)a.Cin * rowb;  // S bytes per tap
  // piece p of K-tile kt into buffer kt & 1: p even = S, odd = dY; p >> 1 =
  // which 32 output channels of the 64
  auto issue = [&](int kt, int p) {
    const int ti = kt / KC, kc = kt - ti * KC;
    const int ih = ti / ntw, iw = ti - ih * ntw;  // tap (th0 + ih*s, tw0 + iw*s)
    const int tap = (th0 + ih * s) * a.kw + tw0 + iw * s;
    const int koff = kc * 128 + (p >> 1) * 64;
    unsigned char* buf = smem + (kt & 1) * BUF + (p >> 1) * OFF_K1;
    if ((p & 1) == 0) {
#pragma unroll
      for (int i = 0; i < WINS; ++i)
        glds16(wsrc[i] + tap * wtap + koff, buf + (i * 8 + wave) * 1024);
    } else {
      const long long toff = -((long long)ih * a.Wo + iw) * rowb;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const bool ok = (vh[i] >> ih) & (vw[i] >> iw) & 1u;
        glds16(ok ? dsrc[i] + toff + koff : zp, buf + WP + (i * 8 + wave) * 1024);
      }
    }
  };

  // ---- fragments: lane l reads row l & 15, chunk l >> 4 of a 16-row block
  const int foff = (lane & 15) * 64 + (((lane >> 4) ^ dp_swz(lane & 15)) << 4);
  const int arow0 = wm * (BNC / 2), brow0 = wn * 64;
  f32x4 acc[2 * FA][4];
#pragma unroll
  for (int i = 0; i < 2 * FA; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  uint4 a1[FA], a2[FA], b1[4], b2[4];
  auto readA = [&](uint4 (&d)[FA], int kt, int kh, int mh) {
    const unsigned char* base =
        smem + (kt & 1) * BUF + kh * OFF_K1 + (arow0 + mh * (BNC / 4)) * 64 + foff;
#pragma unroll
    for (int i = 0; i < FA; ++i) d[i] = *reinterpret_cast<const uint4*>(base + i * 1024);
  };
  auto readB = [&](uint4 (&d)[4], int kt, int kh) {
    const unsigned char* base = smem + (kt & 1) * BUF + kh * OFF_K1 + WP + brow0 * 64 + foff;
#pragma unroll
    for (int j = 0; j < 4; ++j) d[j] = *reinterpret_cast<const uint4*>(base + j * 1024);
  };
  auto mma = [&](const uint4 (&x)[FA], const uint4 (&y)[4], int mh) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < FA; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[mh * FA + i][j] = dp_mfma(x[i], y[j], acc[mh * FA + i][j]);
    __builtin_amdgcn_s_setprio(0);
  };

  // ---- main loop (tools/gemm_lab/g8.hip V1): prologue stages K-tile 0 and
  // waits for its first two pieces
#pragma unroll
  for (int p = 0; p < 4; ++p) issue(0, p);
  wait_vmcnt<VM2>();
  dp_barrier();
  readA(a1, 0, 0, 0);
  readB(b1, 0, 0);
  for (int kt = 0; kt < NKT; ++kt) {
    const bool more = kt + 1 < NKT;
    // phase 0: (k0, first half of the wave's ci rows) with a1 b1
    if (more) issue(kt + 1, 0);
    readA(a2, kt, 0, 1);
    __builtin_amdgcn_sched_barrier(0);
    mma(a1, b1, 0);
    __builtin_amdgcn_sched_barrier(0);
    // phase 1: (k0, second half) with a2 b1; pieces 2, 3 of K-tile kt land
    if (more) {
      issue(kt + 1, 1);
      wait_vmcnt<VM2>();
    } else {
      wait_vmcnt<0>();
    }
    dp_barrier();
    readA(a1, kt, 1, 0);
    readB(b2, kt, 1);
    __builtin_amdgcn_sched_barrier(0);
    mma(a2, b1, 1);
    __builtin_amdgcn_sched_barrier(0);
    // phase 2: (k1, first half) with a1 b2
    if (more) issue(kt + 1, 2);
    readA(a2, kt, 1, 1);
    __builtin_amdgcn_sched_barrier(0);
    mma(a1, b2, 0);
    __builtin_amdgcn_sched_barrier(0);
    // phase 3: (k1, second half) with a2 b2; pieces 0, 1 of K-tile kt + 1 land
    if (more) {
      issue(kt + 1, 3);
      wait_vmcnt<VM2>();
      dp_barrier();
      readA(a1, kt + 1, 0, 0);
      readB(b1, kt + 1, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    mma(a2, b2, 1);
    __builtin_amdgcn_sched_barrier(0);
  }

  // ---- epilogue: acc[i][j] reg e = D[ci][pixel], ci = n0 + arow0 + 16 i +
  // 4 (lane >> 4) + e, class pixel m = m0 + brow0 + 16 j + (lane & 15)
  const int CW = a.Cin >> 5;
  const int cq = 4 * (lane >> 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const long long m = m0 + brow0 + 16 * j + (lane & 15);
    if (m >= P) continue;
    long long pix = m;  // input pixel index
    if (s != 1) {
      const int wc = (int)(m % Wc);
      const long long q = m / Wc;
      pix = ((q / Hc) * a.H + (q % Hc) * s + ph) * a.W + (long long)wc * s + pw;
    }
    uint32_t mw[FA];
    uint2 dv[2 * FA];
#pragma unroll
    for (int i = 0; i < 2 * FA; ++i) {
      const int ci = n0 + arow0 + 16 * i + cq;
      if ((i & 1) == 0) mw[i >> 1] = a.mask ? a.mask[pix * CW + (ci >> 5)] : 0xFFFFFFFFu;
      dv[i] = a.dres ? *reinterpret_cast<const uint2*>(a.dres + pix * a.Cin + ci)
                     : make_uint2(0u, 0u);
    }
#pragma unroll
    for (int i = 0; i < 2 * FA; ++i) {
      const int ci = n0 + arow0 + 16 * i + cq;
      const uint32_t bits = mw[i >> 1] >> (ci & 31);
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = ((bits >> e) & 1u) ? acc[i][j][e] : 0.f;
      v[0] += zk::bf16_to_f32((uint16_t)(dv[i].x & 0xffff));
      v[1] += zk::bf16_to_f32((uint16_t)(dv[i].x >> 16));
      v[2] += zk::bf16_to_f32((uint16_t)(dv[i].y & 0xffff));
      v[3] += zk::bf16_to_f32((uint16_t)(dv[i].y >> 16));
      *reinterpret_cast<uint2*>(a.dx + pix * a.Cin + ci) =
          make_uint2(zk::pack_bf16x2(v[0], v[1]), zk::pack_bf16x2(v[2], v[3]));
    }
  }
}

// ===========================================================================
// Weight gradient of the same layers (variant 60 of the wgrad dispatch):
//
//   dW[co][tap][ci] = mask(|w| <= clip) * sum_p dY[p][co] * sx[p + shift(tap)][ci]
//
// M = Cout, N = 9 * Cin (a 256-wide N tile = 256 input channels of one tap),
// K = output pixels, split over blocks (the 9-36 tiles of a deep layer are far
// fewer than the 256 CUs).  Same block shape and 4-phase schedule as the
// data gradient; both operands are [pixel][channel] rows, so a K-tile piece is
// 32 pixel rows x 512 B (256 channels) and the 16x16x32 fragments (8
// consecutive pixels of one channel per lane) come from transposed LDS reads
// (ds_read_b64_tr_b16, two per fragment).  Image: 512-B rows, 16-B chunk c of
// row r at slot c ^ tr_swz<512>(r) -- conflict-free for the transposed reads
// (each 32-lane group reads 8 rows x 32 B).  sx rows of taps outside the
// image read a 512-B pad row (zeros, or bf16 +1 for pad_values=1); dY rows
// past the split read zeros.  Epilogue: the kernel STE mask and fp32 atomics
// into dW, or this split's partial into the level-0 slab of the in-launch
// fixed-order split-K tree (splitk_tree.h; the default), or plain stores into
// a slab reduced by igemm.hip's wgrad_reduce_kernel (tree off).
// ===========================================================================
__device__ __attribute__((aligned(512))) uint4 g_dz_page[32];  // 512 B of zeros

struct DeepWgradArgs {
  const uint16_t* dy;  // [B][H][W][Cout]
  const uint16_t* sx;  // sign(x) bf16 +-1 [B][H][W][Cin]
  const float* w;      // latent kernel [Cout][9][Cin] (STE mask)
  float* dw;           // [Cout][9][Cin] accumulated (atomic mode)
  float* slab;         // [splits][Cout][9 Cin] (slab mode) or null
  int B, H, W, Cin, Cout, pad_ones;
  float clip;
  int kps;             // pixels per split (multiple of 64)
  int co_tiles, ci_tiles;
  SkTree tree;         // tree mode (tree.dwn > 0): in-launch split-K combine
};

__device__ __forceinline__ uint4 wp_frag(const unsigned char* piece, int c0, int lane) {
  // 8 consecutive pixels (rows 8g .. 8g+7 of the piece) of channel c0 + (lane & 15)
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int r0 = 8 * g + q, r1 = r0 + 4;
  const int slot = (c0 >> 3) | (p >> 1), inner = (p & 1) * 8;
  const int o0 = r0 * 512 + ((slot ^ tr_swz<512>(r0)) << 4) + inner;
  const int o1 = r1 * 512 + ((slot ^ tr_swz<512>(r1)) << 4) + inner;
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s16x4*)(uintptr_t)(const __attribute__((address_space(3))) void*)(piece + o0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s16x4*)(uintptr_t)(const __attribute__((address_space(3))) void*)(piece + o1));
  const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(uint4, v);
}

__global__ __launch_bounds__(DP_NT, 1) void wgrad_deep_kernel(DeepWgradArgs a) {
  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 2, wn = wave & 3;  // co half, ci quarter
  // consecutive logical ids: the tiles of one split (same pixel rows in L2)
  const int L = xcd_linear(blockIdx.x, gridDim.x);
  const int tiles = a.co_tiles * 9 * a.ci_tiles;
  const int split = L / tiles, tile = L - split * tiles;
  const int cot = tile % a.co_tiles, rest = tile / a.co_tiles;
  const int tap = rest % 9, cit = rest / 9;
  const int co0 = cot * 256, ci0 = cit * 256;
  const int th = tap / 3, tw = tap - th * 3;
  const int P = a.B * a.H * a.W;
  const int kbeg = split * a.kps;
  if (kbeg >= P) return;  // block-uniform
  const int kend = min(P, kbeg + a.kps);
  const int NKT = (kend - kbeg + 63) >> 6;
  const float invW = 1.0f / (float)a.W, invH = 1.0f / (float)a.H;

  // loader: instruction i (0, 1) of wave w fills piece rows (i*8 + w)*2 + (lane >> 5);
  // LDS slot lane & 31 holds global chunk (lane & 31) ^ tr_swz<512>(row)
  const int slot = lane & 31;
  int lrow[2], gofs[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    lrow[i] = (i * 8 + wave) * 2 + (lane >> 5);
    gofs[i] = (slot ^ tr_swz<512>(lrow[i])) * 16;
  }
  const unsigned char* dyb = reinterpret_cast<const unsigned char*>(a.dy) + co0 * 2;
  const unsigned char* sxb = reinterpret_cast<const unsigned char*>(a.sx) + ci0 * 2;
  const unsigned char* zpage = reinterpret_cast<const unsigned char*>(g_dz_page);
  const unsigned char* ppage =
      a.pad_ones ? reinterpret_cast<const unsigned char*>(g_ones_page_bf16) : zpage;
  const long long dyrow = (long long)a.Cout * 2, sxrow = (long long)a.Cin * 2;
  // piece p of K-tile kt into buffer kt & 1: p even = dY (A), odd = sx (B);
  // p >> 1 = which 32 pixels of the 64
  auto issue = [&](int kt, int p) {
    unsigned char* dst = smem + (kt & 1) * DP_BUF + p * DP_PIECE;
    const int pbase = kbeg + kt * 64 + (p >> 1) * 32;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int px = pbase + lrow[i];
      const unsigned char* src = zpage + gofs[i];
      if (px < kend) {
        if ((p & 1) == 0) {
          src = dyb + (long long)px * dyrow + gofs[i];
        } else {
          const int q1 = fdiv(px, a.W, invW);
          const int w = px - q1 * a.W;
          const int b = fdiv(q1, a.H, invH);
          const int h = q1 - b * a.H;
          const int hi = h - 1 + th, wi = w - 1 + tw;
          src = ((unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W)
                    ? sxb + (((long long)b * a.H + hi) * a.W + wi) * sxrow + gofs[i]
                    : ppage + gofs[i];
        }
      }
      glds16(src, dst + (i * 8 + wave) * 1024);
    }
  };

  const int arow0 = wm * 128, brow0 = wn * 64;
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  uint4 a1[4], a2[4], b1[4], b2[4];
  auto readA = [&](uint4 (&d)[4], int kt, int kh, int mh) {
    const unsigned char* piece = smem + (kt & 1) * DP_BUF + (kh * 2) * DP_PIECE;
#pragma unroll
    for (int i = 0; i < 4; ++i) d[i] = wp_frag(piece, arow0 + mh * 64 + i * 16, lane);
  };
  auto readB = [&](uint4 (&d)[4], int kt, int kh) {
    const unsigned char* piece = smem + (kt & 1) * DP_BUF + (kh * 2 + 1) * DP_PIECE;
#pragma unroll
    for (int j = 0; j < 4; ++j) d[j] = wp_frag(piece, brow0 + j * 16, lane);
  };
  auto mma = [&](const uint4 (&x)[4], const uint4 (&y)[4], int mh) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[mh * 4 + i][j] = dp_mfma(x[i], y[j], acc[mh * 4 + i][j]);
    __builtin_amdgcn_s_setprio(0);
  };

#pragma unroll
  for (int p = 0; p < 4; ++p) issue(0, p);
  wait_vmcnt<4>();
  dp_barrier();
  readA(a1, 0, 0, 0);
  readB(b1, 0, 0);
  for (int kt = 0; kt < NKT; ++kt) {
    const bool more = kt + 1 < NKT;
    if (more) issue(kt + 1, 0);
    readA(a2, kt, 0, 1);
    __builtin_amdgcn_sched_barrier(0);
    mma(a1, b1, 0);
    __builtin_amdgcn_sched_barrier(0);
    if (more) {
      issue(kt + 1, 1);
      wait_vmcnt<4>();
    } else {
      wait_vmcnt<0>();
    }
    dp_barrier();
    readA(a1, kt, 1, 0);
    readB(b2, kt, 1);
    __builtin_amdgcn_sched_barrier(0);
    mma(a2, b1, 1);
    __builtin_amdgcn_sched_barrier(0);
    if (more) issue(kt + 1, 2);
    readA(a2, kt, 1, 1);
    __builtin_amdgcn_sched_barrier(0);
    mma(a1, b2, 0);
    __builtin_amdgcn_sched_barrier(0);
    if (more) {
      issue(kt + 1, 3);
      wait_vmcnt<4>();
      dp_barrier();
      readA(a1, kt + 1, 0, 0);
      readB(b1, kt + 1, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    mma(a2, b2, 1);
    __builtin_amdgcn_sched_barrier(0);
  }

  // ---- epilogue: acc[i][j] reg e = D[co][ci], co = co0 + arow0 + 16 i +
  // 4 (lane >> 4) + e, ci = ci0 + brow0 + 16 j + (lane & 15)
  const long long NTOT = 9LL * a.Cin;
  const bool treed = a.tree.dwn > 0;
  float* sl = a.slab ? a.slab + (long long)split * a.Cout * NTOT : nullptr;
  const int ci = ci0 + brow0 + (lane & 15);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int co = co0 + arow0 + 16 * i + 4 * (lane >> 4) + e;
      const long long row = (long long)co * NTOT + (long long)tap * a.Cin + ci;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const long long idx = row + 16 * j;
        if (treed) {
          if (a.tree.levels > 0)
            skt_store(a.tree, split, idx, acc[i][j][e]);
          else if (fabsf(a.w[idx]) <= a.clip)
            a.dw[idx] += acc[i][j][e];  // one split: this block owns the element
        } else if (sl) {
          sl[idx] = acc[i][j][e];
        } else if (fabsf(a.w[idx]) <= a.clip) {
          atomicAdd(a.dw + idx, acc[i][j][e]);
        }
      }
    }
  if (treed && a.tree.levels > 0)
    skt_combine<DP_NT, 256, 256>(a.tree, tile, split, co0, (long long)tap * a.Cin + ci0, NTOT,
                                 a.dw, a.w, a.clip, reinterpret_cast<int*>(smem));
}

bool g_dp_attr = false;
bool g_wp_attr = false;

}  // namespace

// Split plan of zk_wgrad_deep_impl: pixels per split (multiple of 64) and
// the split count.  target_blocks <= 0: 512.
static void wgrad_deep_plan(long long P, int tiles, int target_blocks, long long& kps,
                            int& splits) {
  if (target_blocks <= 0) target_blocks = 512;
  long long s = (target_blocks + tiles - 1) / tiles;
  const long long max_s = (P + 4 * 64 - 1) / (4 * 64);  // >= 4 K-tiles per split
  if (s > max_s) s = max_s;
  if (s < 1) s = 1;
  kps = (P + s - 1) / s;
  kps = (kps + 63) / 64 * 64;
  splits = (int)((P + kps - 1) / kps);
}

// Entry used by igemm.hip's wgrad dispatch (variant 60): stride-1 3x3 'same'
// weight gradient with Cin % 256 == 0 and Cout % 256 == 0.  slab (optional,
// slab_bytes >= *need): per-split partials for the fixed-order reduce;
// otherwise STE-masked fp32 atomics into dw.  need (non-null): slab bytes
// only.  *splits: the slab count (0: atomics).
int zk_wgrad_deep_impl(const void* dy, const void* sx, const void* w, void* dw, int B, int H,
                       int W, int Cin, int Cout, int pad_ones, float clip, int target_blocks,
                       void* slab, long long slab_bytes, long long* need, int* splits, bool dry,
                       bool tree, hipStream_t st) {
  if (Cin % 256 || Cout % 256 || B < 1 || H < 1 || W < 1) return (int)hipErrorInvalidValue;
  const long long P = (long long)B * H * W;
  if (P >= (1 << 24)) return (int)hipErrorInvalidValue;  // fdiv range
  const int tiles = (Cout / 256) * 9 * (Cin / 256);
  long long kps = 0;
  int ns = 0;
  wgrad_deep_plan(P, tiles, target_blocks, kps, ns);
  const long long dwn = (long long)Cout * 9 * Cin;
  long long sb = (long long)ns * dwn * 4;
  SkTree t{};
  long long tf = 0, tc = 0;
  const bool tree_plan = tree && skt_plan(ns, tiles, dwn, t, tf, tc);
  if (tree_plan) sb = tf * 4;
  if (need) {
    *need = sb;
    return 0;
  }
  int* cnt = nullptr;
  const bool treed = tree_plan && (t.levels == 0 || (slab && slab_bytes >= sb)) &&
                     (dry || (cnt = skt_counters(st)) != nullptr);
  if (!treed && slab && slab_bytes < (long long)ns * dwn * 4) slab = nullptr;
  if (splits) *splits = (!treed && slab) ? ns : 0;  // > 0: the caller reduces the slab
  if (dry) return 0;
  if (treed) {
    t.slab = t.levels > 0 ? (float*)slab : nullptr;
    t.cnt = cnt;
    slab = nullptr;
  } else {
    t = SkTree{};
  }
  if (!g_wp_attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)wgrad_deep_kernel,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, DP_LDS);
    if (e != hipSuccess) return (int)e;
    g_wp_attr = true;
  }
  DeepWgradArgs a{(const uint16_t*)dy, (const uint16_t*)sx, (const float*)w, (float*)dw,
                  (float*)slab, B, H, W, Cin, Cout, pad_ones, clip, (int)kps, Cout / 256,
                  Cin / 256, t};
  (void)hipGetLastError();
  hipLaunchKernelGGL(wgrad_deep_kernel, dim3((unsigned)(tiles * ns)), dim3(DP_NT), DP_LDS, st, a);
  return (int)hipGetLastError();
}

// Entry used by igemm.hip's dgrad dispatch (variant 60): data gradient of a
// conv with kh, kw <= 3, stride 1 or 2 (one grid row per stride-parity class
// of the input pixels), Cin % 256 == 0 (the dispatch's rule: the 128-channel
// block form lost to conv3rw / igemm there and was removed,
// profiles/r4/removed_variants.md), Cout % 64 == 0; mask / dres optional.
// dry: validate only.
int zk_dgrad_deep_impl(const void* dy, const void* wt, const void* mask, const void* dres, void* dx,
                       int B, int H, int W, int Cin, int Cout, int Ho, int Wo, int kh, int kw,
                       int s, int pt, int pl, bool dry, hipStream_t st) {
  if (Cin % 256 || Cout % 64 || Cout < 64 || B < 1 || H < 1 || W < 1 || Ho < 1 || Wo < 1)
    return (int)hipErrorInvalidValue;
  if (kh < 1 || kh > 3 || kw < 1 || kw > 3 || s < 1 || s > 2 || pt < 0 || pl < 0 || pt >= kh ||
      pl >= kw)
    return (int)hipErrorInvalidValue;
  const long long P = (long long)B * H * W;
  if (P * Cin >= (1LL << 40) || (long long)B * Ho * Wo * Cout >= (1LL << 40))
    return (int)hipErrorInvalidValue;
  constexpr int bnc = 256;
  // the largest parity class: ceil(H / s) x ceil(W / s) pixels per image
  const long long Pc = (long long)B * ((H + s - 1) / s) * ((W + s - 1) / s);
  const long long m_tiles = (Pc + 255) / 256;
  const long long blocks = m_tiles * (Cin / bnc);
  if (blocks >= (1LL << 31)) return (int)hipErrorInvalidValue;
  if (dry) return 0;
  DeepDgradArgs a{(const uint16_t*)dy, (const uint16_t*)wt, (const uint32_t*)mask,
                  (const uint16_t*)dres, (uint16_t*)dx, B, H, W, Cin, Cout, Ho, Wo, kh, kw,
                  s, pt, pl, (int)m_tiles};
  const dim3 grid((unsigned)blocks, (unsigned)(s * s));
  (void)hipGetLastError();
  constexpr int lds = 2 * (2 * 256 * 64 + 2 * DP_PIECE);
  if (!g_dp_attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)dgrad_deep_kernel<256>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return (int)e;
    g_dp_attr = true;
  }
  hipLaunchKernelGGL(dgrad_deep_kernel<256>, grid, dim3(DP_NT), lds, st, a);
  return (int)hipGetLastError();
}
