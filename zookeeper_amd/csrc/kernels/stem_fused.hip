// Recompute-fused ImageNet stem (7x7/2 conv, Cin <= 4 -> 64, BN, ReLU,
// 3x3/2 max pool) for gfx950.  stem.hip materialises the 112x112x64 conv
// output y1 (822 MB at batch 512) and a dense dy1 of the same size: written
// once, read three times.  Here neither tensor exists; the conv is cheap
// (K = 7 rows x 32) and is recomputed from the 4-channel padded image xp in
// each of the three passes that need it:
//
//   F1  zk_stem_fwd_stats   conv -> BN-1 partial sums (per block)
//   F2  zk_stem_fwd_pool    conv -> BN-1 + ReLU -> 3x3/2 max pool: pooled p,
//                           argmax tap, y1 at the argmax (ya), BN-2 partials
//   B1  zk_stem_pool_bwd_sums_ya   BN-1 backward sums from (dp, ya)
//   B2  zk_stem_bwd_fused   conv -> dy1 = k1 relu'(u) route(dp) + k0 - k3 y1
//                           -> weight gradient (MFMA), per-block slabs
//
// Every pass runs the same tile machinery: a persistent block walks spatial
// tiles of conv outputs; a tile's input is a LINE BUFFER of xp rows (the
// (pixel, kh) K-rows of all its pixels overlap: 8 x 16 outputs read 21 x 38
// input pixels = 8 KB instead of the 56 KB im2col image), loaded by
// global_load_lds one tile ahead.  The conv is D[co][px] = W[co][k] X[px][k]
// on v_mfma_f32_32x32x16_bf16 with the 64 x 7 x 32 weights resident in LDS
// (lane = pixel, 4 consecutive channels per register group).  Line-buffer
// rows are padded so that the 16-B K-chunk of pixel m sits at 16 m + const
// (mod 256): the B-operand reads of 32 consecutive pixels are bank-conflict
// free, and so are the transposed reads of the weight gradient.
//
// Numerics match stem.hip: y1 is rounded to bf16 before every use (the MFMA
// chain per output is identical in all passes, so F1, F2 and B2 see the same
// y1), the pool compares relu(a*y1 + b) in fp32 and keeps the first maximum.
#include "mfma_common.h"

namespace {

constexpr int SC = 64;                    // stem output channels
constexpr int SKH = 7;                    // kernel rows (7x7 stems)
constexpr int W_BYTES = SKH * SC * 64;    // [kh][co][32 bf16] = 28 KB

struct FGeom {
  int B, Cin, KW, Ho, Wo, Hp, Wp;  // conv: stride 2, 7 x KW, xp [B][Hp][Wp][4]
  int H2, W2, pt2, pl2;            // 3x3/2 max pool over the Ho x Wo conv output
};

// Line buffer of a TR x TC tile of conv outputs: xp rows [2 r0, 2 r0 + ROWS),
// pixels [2 c0, 2 c0 + 2 TC + 6), each row padded to RB bytes.
template <int TR, int TC>
struct LBuf {
  static constexpr int ROWS = 2 * (TR - 1) + SKH;
  static constexpr int BASE = (2 * TC + 6) * 8;
  // RB = 8 TC (mod 128) makes chunk(m) = 16 m + const (mod 256); for odd TC
  // use 8 (TC + 1) to keep rows 16-B aligned (a few 2-way conflicts).
  static constexpr int TGT = (8 * ((TC % 2) ? TC + 1 : TC)) % 128;
  static constexpr int RB = BASE + (((TGT - BASE) % 128) + 128) % 128;
  static constexpr int CHUNKS = ROWS * RB / 16;
  static constexpr int BYTES = (CHUNKS + 63) / 64 * 64 * 16;  // whole wave-instructions
  static_assert(RB % 16 == 0, "line-buffer rows must stay 16-B aligned");
};

// Issue the line buffer of the tile whose first conv output is (b, r0, c0).
// Rows / pixels outside xp (and the row padding) read the zero page.
template <int TR, int TC, int NT>
__device__ __forceinline__ void issue_lbuf(unsigned char* lb, const unsigned char* xp,
                                           const FGeom& g, int b, int r0, int c0, int tid) {
  using L = LBuf<TR, TC>;
  const unsigned char* zp = reinterpret_cast<const unsigned char*>(g_zero_page);
  const int wave = tid >> 6, lane = tid & 63;
  const long long rowb = (long long)g.Wp * 8;
  const int yr0 = 2 * r0, xc0 = 2 * c0;
#pragma unroll
  for (int j = 0; j < (L::CHUNKS + NT - 1) / NT; ++j) {
    const int q0 = j * NT + wave * 64;  // wave-uniform
    if (q0 < L::CHUNKS) {
      const int off = (q0 + lane) * 16;
      const int row = off / L::RB, cb = off - row * L::RB;
      const int yr = yr0 + row, xc = xc0 + (cb >> 3);
      const unsigned char* src = zp;
      if (cb < L::BASE && yr >= 0 && yr < g.Hp && xc >= 0 && xc + 1 < g.Wp)
        src = xp + ((long long)b * g.Hp + yr) * rowb + (long long)xc * 8;
      glds16(src, lb + q0 * 16);
    }
  }
}

// Weights ws [kh][co][32] bf16 -> LDS with the 16-B chunk of row co at slot
// chunk ^ ((co >> 2) & 3) (the A-operand reads of 32 rows are conflict free).
template <int NT>
__device__ __forceinline__ void load_weights(unsigned char* wl, const unsigned char* ws,
                                             int tid) {
  for (int i = tid; i < W_BYTES / 16; i += NT) {
    const int row = i >> 2, slot = i & 3, co = row & (SC - 1);
    const uint4 v = *reinterpret_cast<const uint4*>(ws + row * 64 + ((slot ^ ((co >> 2) & 3)) << 4));
    *reinterpret_cast<uint4*>(wl + i * 16) = v;
  }
}

// Conv of TN 32-pixel groups starting at tile pixel px0 (pixel m = r TC + c
// of the tile; m >= TR*TC are dummies that read pixel 0):
// acc[a][t][r] = y1[co = 32a + 8(r>>2) + 4h + (r&3)][px0 + 32t + lane%32].
template <int TR, int TC, int TN>
__device__ __forceinline__ void conv_tile(const unsigned char* wl, const unsigned char* lb,
                                          int px0, int lane, f32x16 (&acc)[2][TN]) {
  using L = LBuf<TR, TC>;
  const int r32 = lane & 31, h = lane >> 5;
  int segb[TN];
#pragma unroll
  for (int t = 0; t < TN; ++t) {
    int px = px0 + 32 * t + r32;
    if (px >= TR * TC) px = 0;
    const int rr = px / TC, cc = px - rr * TC;
    segb[t] = 2 * rr * L::RB + 16 * cc + 16 * h;
  }
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int t = 0; t < TN; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][t][r] = 0.f;
  int wrow[2];
#pragma unroll
  for (int a = 0; a < 2; ++a) wrow[a] = (32 * a + r32) * 64;
  const int wsw = (r32 >> 2) & 3;  // (co >> 2) & 3 for co = 32a + r32
#pragma unroll
  for (int kh = 0; kh < SKH; ++kh) {
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      const int chunk = 2 * sub + h;
      uint4 af[2], bf[TN];
#pragma unroll
      for (int a = 0; a < 2; ++a)
        af[a] = *reinterpret_cast<const uint4*>(wl + kh * SC * 64 + wrow[a] + ((chunk ^ wsw) << 4));
#pragma unroll
      for (int t = 0; t < TN; ++t)
        bf[t] = *reinterpret_cast<const uint4*>(lb + segb[t] + kh * L::RB + 32 * sub);
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int t = 0; t < TN; ++t) acc[a][t] = mfma_bf16(af[a], bf[t], acc[a][t]);
    }
  }
}

// Weight fragments of all 64 channels for every K-substep, in registers
// (112 VGPRs): w[kh][sub][a] = chunk 2 sub + h of row 32a + lane%32 of kernel
// row kh.
__device__ __forceinline__ void load_wfrags(const unsigned char* ws, int lane,
                                            uint4 (&w)[SKH][2][2]) {
  const int r32 = lane & 31, h = lane >> 5;
#pragma unroll
  for (int kh = 0; kh < SKH; ++kh)
#pragma unroll
    for (int sub = 0; sub < 2; ++sub)
#pragma unroll
      for (int a = 0; a < 2; ++a)
        w[kh][sub][a] = *reinterpret_cast<const uint4*>(
            ws + (kh * SC + 32 * a + r32) * 64 + (2 * sub + h) * 16);
}

// conv_tile with the A operand (weights) from registers: one LDS read per
// two MFMAs.
template <int TR, int TC>
__device__ __forceinline__ void conv_tile_wreg(const uint4 (&w)[SKH][2][2],
                                               const unsigned char* lb, int px0, int lane,
                                               f32x16 (&acc)[2]) {
  using L = LBuf<TR, TC>;
  const int r32 = lane & 31, h = lane >> 5;
  int px = px0 + r32;
  if (px >= TR * TC) px = 0;
  const int rr = px / TC, cc = px - rr * TC;
  const int segb = 2 * rr * L::RB + 16 * cc + 16 * h;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[a][r] = 0.f;
#pragma unroll
  for (int kh = 0; kh < SKH; ++kh)
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      const uint4 bf = *reinterpret_cast<const uint4*>(lb + segb + kh * L::RB + 32 * sub);
#pragma unroll
      for (int a = 0; a < 2; ++a) acc[a] = mfma_bf16(w[kh][sub][a], bf, acc[a]);
    }
}

__device__ __forceinline__ float bf16r(float v) { return zk::bf16_to_f32(zk::f32_to_bf16(v)); }

__device__ __forceinline__ void unpack8(const uint4& q, float (&v)[8]) {
  const uint32_t u[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[2 * k] = zk::bf16_to_f32((uint16_t)(u[k] & 0xffff));
    v[2 * k + 1] = zk::bf16_to_f32((uint16_t)(u[k] >> 16));
  }
}

__device__ __forceinline__ uint4 pack8f(const float (&v)[8]) {
  return make_uint4(zk::pack_bf16x2(v[0], v[1]), zk::pack_bf16x2(v[2], v[3]),
                    zk::pack_bf16x2(v[4], v[5]), zk::pack_bf16x2(v[6], v[7]));
}

__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

// Top of a tile: this wave's line-buffer DMA (and any stores) retired, then
// the barrier makes every wave's DMA visible.
__device__ __forceinline__ void tile_barrier() {
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

// Reduce-scatter of 32 values over the 32 lanes of a wave half (lane r ends
// with the half's total of value r).
template <int N>
__device__ __forceinline__ void rs_step32(float (&v)[32], int r32) {
  const bool upper = (r32 & N) != 0;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const float send = upper ? v[i] : v[i + N];
    const float keep = upper ? v[i + N] : v[i];
    v[i] = keep + __shfl_xor(send, N, 64);
  }
}
__device__ __forceinline__ float rs32(float (&v)[32], int r32) {
  rs_step32<16>(v, r32);
  rs_step32<8>(v, r32);
  rs_step32<4>(v, r32);
  rs_step32<2>(v, r32);
  rs_step32<1>(v, r32);
  return v[0];
}

// ===========================================================================
// F1: BN-1 statistics of y1 (bf16-rounded) without storing it.
// Tile 8 x 16 outputs, 4 waves x 32 pixels, line buffer double-buffered.
// part[block][2][64] (sum, sum of squares).
// ===========================================================================
constexpr int F1_TR = 8, F1_TC = 16;
constexpr int F1_LB = LBuf<F1_TR, F1_TC>::BYTES;
constexpr int F1_LDS = 2 * F1_LB;

__global__ __launch_bounds__(256, 2) void stem_fwd_stats_kernel(
    const unsigned char* __restrict__ xp, const unsigned char* __restrict__ ws,
    float* __restrict__ part, FGeom g, int tiles_w, int tiles_img, int ntiles) {
  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
  unsigned char* lbuf0 = smem;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r32 = lane & 31, h = lane >> 5;
  const int blk = xcd_linear(blockIdx.x, gridDim.x), nblk = gridDim.x;

  auto tile_pos = [&](int T, int& b, int& r0, int& c0) {
    b = T / tiles_img;
    const int rem = T - b * tiles_img;
    const int th = rem / tiles_w;
    r0 = th * F1_TR;
    c0 = (rem - th * tiles_w) * F1_TC;
  };
  if (blk < ntiles) {
    int b, r0, c0;
    tile_pos(blk, b, r0, c0);
    issue_lbuf<F1_TR, F1_TC, 256>(lbuf0, xp, g, b, r0, c0, tid);
  }
  uint4 wf[SKH][2][2];
  load_wfrags(ws, lane, wf);

  typedef float f32x2 __attribute__((ext_vector_type(2)));
  f32x2 cs[16], cq[16];  // value pairs (a = 0, 1) of register r: packed adds / FMAs
#pragma unroll
  for (int r = 0; r < 16; ++r) cs[r] = cq[r] = (f32x2){0.f, 0.f};

  int it = 0;
  for (int T = blk; T < ntiles; T += nblk, ++it) {
    const int cur = it & 1;
    tile_barrier();
    int b, r0, c0;
    tile_pos(T, b, r0, c0);
    if (T + nblk < ntiles) {
      int bn, rn, cn;
      tile_pos(T + nblk, bn, rn, cn);
      issue_lbuf<F1_TR, F1_TC, 256>(lbuf0 + (cur ^ 1) * F1_LB, xp, g, bn, rn, cn, tid);
    }
    f32x16 acc[2];
    conv_tile_wreg<F1_TR, F1_TC>(wf, lbuf0 + cur * F1_LB, 32 * wave, lane, acc);
    // statistics of the fp32 accumulators (the stored-bf16 rounding of
    // stem.hip is below the statistics' own summation error)
    if (r0 + F1_TR > g.Ho || c0 + F1_TC > g.Wo) {  // partial tile (uniform)
      const int px = 32 * wave + r32;
      const bool live = r0 + px / F1_TC < g.Ho && c0 + px % F1_TC < g.Wo;
      if (!live) {
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[0][r] = acc[1][r] = 0.f;
      }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const f32x2 v = {acc[0][r], acc[1][r]};
      cs[r] += v;
      cq[r] += v * v;
    }
  }

  // channel co = 32a + 8(r>>2) + 4h + (r&3): reduce over the 32 pixel lanes
  float v[32];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    v[r] = cs[r].x;
    v[16 + r] = cs[r].y;
  }
  const float s_sum = rs32(v, r32);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    v[r] = cq[r].x;
    v[16 + r] = cq[r].y;
  }
  const float s_sq = rs32(v, r32);
  // lane r32 holds value index i = r32 = a*16 + r
  const int a = r32 >> 4, r = r32 & 15;
  const int co = 32 * a + 8 * (r >> 2) + 4 * h + (r & 3);
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);  // [4 waves][2][64]
  red[(wave * 2 + 0) * SC + co] = s_sum;
  red[(wave * 2 + 1) * SC + co] = s_sq;
  __syncthreads();
  if (tid < 2 * SC) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) t += red[w * 2 * SC + tid];
    part[(long long)blockIdx.x * 2 * SC + tid] = t;
  }
}

// ===========================================================================
// F2: conv -> relu(BN-1) -> 3x3/2 max pool.  Tile = 8 x 7 pool outputs, whose
// windows cover a 17 x 15 conv region (255 pixels + 1 dummy = 8 waves x 32).
// Writes p (pooled), arg (tap of the first maximum), ya (y1 there) and
// per-block BN-2 partial sums of p.  y1 of the region is staged in LDS
// ([pixel][channel] bf16, chunk slot ^ ((m >> 1) & 7)).  One block per CU,
// the line buffer double-buffered and issued a whole tile ahead; every wave
// issues exactly three output stores per tile (pool outputs outside the
// image store to a sink), so the next tile waits for its line buffer with
// vmcnt(3) instead of draining the stores.
// ===========================================================================
constexpr int F2_PR = 8, F2_PC = 7;
constexpr int F2_TR = 2 * F2_PR + 1, F2_TC = 2 * F2_PC + 1;
constexpr int F2_LB = LBuf<F2_TR, F2_TC>::BYTES;
constexpr int F2_YT = 256 * 128;
constexpr int F2_NT = 512;
constexpr int F2_LDS = W_BYTES + 2 * F2_LB + F2_YT;
static_assert(F2_TR * F2_TC <= 256, "F2 region");
static_assert(F2_PR * F2_PC * 8 <= F2_NT, "one pool item per thread");
static_assert(F2_LDS <= 160 * 1024, "F2 LDS");

__device__ __attribute__((aligned(16))) uint4 g_pool_sink[2];

__global__ __launch_bounds__(F2_NT, 1) void stem_fwd_pool_kernel(
    const unsigned char* __restrict__ xp, const unsigned char* __restrict__ ws,
    const float* __restrict__ coef1, uint16_t* __restrict__ p, uint8_t* __restrict__ arg,
    uint16_t* __restrict__ ya, float* __restrict__ part, FGeom g, int tiles_w, int tiles_img,
    int ntiles) {
  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
  unsigned char* wl = smem;
  unsigned char* lb0 = smem + W_BYTES;
  unsigned char* yt = smem + W_BYTES + 2 * F2_LB;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r32 = lane & 31, h = lane >> 5;
  const int blk = xcd_linear(blockIdx.x, gridDim.x), nblk = gridDim.x;
  const int cg = tid & 7;  // channel group of this thread in the pool phase
  const int po = tid >> 3;
  const int pi = po / F2_PC, pj = po - (po / F2_PC) * F2_PC;
  const bool pitem = po < F2_PR * F2_PC;
  float a1[8], s1[8], sg[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    a1[k] = coef1[cg * 8 + k];
    s1[k] = coef1[SC + cg * 8 + k];
    sg[k] = a1[k] < 0.f ? -1.f : 1.f;
  }
  uint4 flip;  // bf16 sign bits of the channels with a < 0
  {
    uint32_t f[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      f[q] = (a1[2 * q] < 0.f ? 0x8000u : 0u) | (a1[2 * q + 1] < 0.f ? 0x80000000u : 0u);
    flip = make_uint4(f[0], f[1], f[2], f[3]);
  }
  auto tile_pos = [&](int T, int& b, int& oh0, int& ow0) {
    b = T / tiles_img;
    const int rem = T - b * tiles_img;
    const int th = rem / tiles_w;
    oh0 = th * F2_PR;
    ow0 = (rem - th * tiles_w) * F2_PC;
  };
  load_weights<F2_NT>(wl, ws, tid);
  if (blk < ntiles) {
    int b, oh0, ow0;
    tile_pos(blk, b, oh0, ow0);
    issue_lbuf<F2_TR, F2_TC, F2_NT>(lb0, xp, g, b, 2 * oh0 - g.pt2, 2 * ow0 - g.pl2, tid);
  }

  float bs1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, bs2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int it = 0;
  for (int T = blk; T < ntiles; T += nblk, ++it) {
    const int cur = it & 1;
    // line buffer of T retired (the previous tile's 3 stores may stay in
    // flight); the barrier also ends the previous pool phase's reads of yt
    if (it == 0)
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(3) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    int b, oh0, ow0;
    tile_pos(T, b, oh0, ow0);
    if (T + nblk < ntiles) {
      int bn, on, wn;
      tile_pos(T + nblk, bn, on, wn);
      issue_lbuf<F2_TR, F2_TC, F2_NT>(lb0 + (cur ^ 1) * F2_LB, xp, g, bn, 2 * on - g.pt2,
                                      2 * wn - g.pl2, tid);
    }
    f32x16 acc[2][1];
    conv_tile<F2_TR, F2_TC, 1>(wl, lb0 + cur * F2_LB, 32 * wave, lane, acc);
    // y1 (bf16) -> yt[m][co]: 4 consecutive channels per 8-B store
    {
      const int m = 32 * wave + r32;
      const int swz = (m >> 1) & 7;
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int chunk = 4 * a + q;
          const uint2 v = make_uint2(zk::pack_bf16x2(acc[a][0][4 * q], acc[a][0][4 * q + 1]),
                                     zk::pack_bf16x2(acc[a][0][4 * q + 2], acc[a][0][4 * q + 3]));
          *reinterpret_cast<uint2*>(yt + m * 128 + ((chunk ^ swz) << 4) + 8 * h) = v;
        }
    }
    lds_barrier();
    // pool: one (pool output, channel group) per thread, branch-free
    {
      const int hr0 = 2 * oh0 - g.pt2, wc0 = 2 * ow0 - g.pl2;  // conv coords of region (0, 0)
      const int i = pitem ? pi : 0, j = pitem ? pj : 0;
      const int oh = oh0 + i, ow = ow0 + j;
      const bool live = pitem && oh < g.H2 && ow < g.W2;
      // relu(a y + s) is monotone in y (increasing for a >= 0, else
      // decreasing), so the first maximum of the window is the first maximum
      // of y ^ sign(a) (a sign flip on the packed bf16); ties at relu's 0 do
      // not matter (they route no gradient).  Out-of-image taps read -inf.
      uint4 tv[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int m = (2 * i + t / 3) * F2_TC + 2 * j + t % 3;
        tv[t] = *reinterpret_cast<const uint4*>(yt + m * 128 + ((cg ^ ((m >> 1) & 7)) << 4));
      }
#pragma unroll
      for (int t = 0; t < 9; ++t) {  // y -> y * sign(a) on the packed bf16
        tv[t].x ^= flip.x;
        tv[t].y ^= flip.y;
        tv[t].z ^= flip.z;
        tv[t].w ^= flip.w;
      }
      const bool interior = hr0 + 2 * i >= 0 && hr0 + 2 * i + 2 < g.Ho && wc0 + 2 * j >= 0 &&
                            wc0 + 2 * j + 2 < g.Wo;
      if (!interior) {
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          const int hc = hr0 + 2 * i + t / 3, wc = wc0 + 2 * j + t % 3;
          if (!(hc >= 0 && hc < g.Ho && wc >= 0 && wc < g.Wo))
            tv[t] = make_uint4(0xFF80FF80u, 0xFF80FF80u, 0xFF80FF80u, 0xFF80FF80u);  // -inf
        }
      }
      float best[8], yb[8];
      uint32_t bi[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) bi[k] = 0;
      unpack8(tv[0], best);
#pragma unroll
      for (int t = 1; t < 9; ++t) {
        float v[8];
        unpack8(tv[t], v);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const bool gt = v[k] > best[k];
          best[k] = gt ? v[k] : best[k];
          bi[k] = gt ? (uint32_t)t : bi[k];
        }
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        yb[k] = best[k] * sg[k];
        best[k] = fmaxf(fmaf(a1[k], yb[k], s1[k]), 0.f);
      }
      const uint4 pk = pack8f(best);
      const long long off = (((long long)b * g.H2 + oh) * g.W2 + ow) * SC + cg * 8;
      uint4* dp_ = live ? reinterpret_cast<uint4*>(p + off) : &g_pool_sink[0];
      uint4* dy_ = live ? reinterpret_cast<uint4*>(ya + off) : &g_pool_sink[1];
      uint2* da_ = live ? reinterpret_cast<uint2*>(arg + off) : reinterpret_cast<uint2*>(&g_pool_sink[0]);
      *dp_ = pk;
      *dy_ = pack8f(yb);
      *da_ = make_uint2(bi[0] | (bi[1] << 8) | (bi[2] << 16) | (bi[3] << 24),
                        bi[4] | (bi[5] << 8) | (bi[6] << 16) | (bi[7] << 24));
      float st[8];
      unpack8(pk, st);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float v = live ? st[k] : 0.f;
        bs1[k] += v;
        bs2[k] += v * v;
      }
    }
  }
  if (!part) return;
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);  // [512][2][8]
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    red[(tid * 2 + 0) * 8 + k] = bs1[k];
    red[(tid * 2 + 1) * 8 + k] = bs2[k];
  }
  __syncthreads();
  if (tid < 2 * SC) {
    const int which = tid / SC, c = tid % SC, g8 = c >> 3, k = c & 7;
    float t = 0.f;
    for (int r = g8; r < F2_NT; r += 8) t += red[(r * 2 + which) * 8 + k];
    part[((long long)blockIdx.x * 2 + which) * SC + c] = t;
  }
}

// ===========================================================================
// B2: conv (recomputed) -> dy1 -> weight gradient.  Tile 8 x 16 conv outputs
// (4 x 8 pool stride cells).  Per tile:
//   a) conv -> y1 bf16 into yt [m][co] (transposed-read swizzle of the wgrad)
//   b) one thread per (stride cell, 8 channels): du = sum of dp over the (up
//      to 4) pool outputs whose argmax is the pixel (dp / arg of the tile's
//      5 x 9 candidate pool outputs staged in LDS), dy1 = k1 [u > 0] du + k0
//      - k3 y1 (0 outside the image), in place in yt
//   c) dW[co][kh*32 + j] += dy1^T X: 4 waves = 2 pixel halves x 2 channel
//      halves, 7 accumulators (one per kh) each
// Line buffer and routing stage double-buffered (issued one tile ahead).
// At the end each block writes its dW partial to slab[block] (plain stores)
// and zk_stem_wgrad_reduce sums the slabs into dW.
// ===========================================================================
constexpr int B2_TR = 8, B2_TC = 16;
constexpr int B2_LB = LBuf<B2_TR, B2_TC>::BYTES;
constexpr int RT_OH = B2_TR / 2 + 1, RT_OW = B2_TC / 2 + 1;  // 5 x 9 candidate pool outputs
constexpr int RT_N = RT_OH * RT_OW;
constexpr int RT_DP = RT_N * 128;                    // dp rows (64 bf16)
constexpr int RT_CHUNKS = RT_N * (128 + 64) / 16;    // + arg rows (64 B)
constexpr int B2_RT = (RT_CHUNKS + 63) / 64 * 64 * 16;
constexpr int B2_YT = 128 * 128;
constexpr int B2_CF = 5 * SC * 4;
constexpr int B2_LDS = W_BYTES + 2 * B2_LB + 2 * B2_RT + B2_YT + B2_CF;
static_assert(B2_LDS <= 80 * 1024, "two B2 blocks per CU");
constexpr int B2_NSLAB = SC * SKH * 32;  // dW partial per block [co][kh*32 + j]

// routing stage of the tile at (b, r0, c0): pool outputs (ohb + i, owb + j)
template <int NT>
__device__ __forceinline__ void issue_route(unsigned char* rt, const uint16_t* dp,
                                            const uint8_t* arg, const FGeom& g, int b, int r0,
                                            int c0, int tid) {
  const unsigned char* zp = reinterpret_cast<const unsigned char*>(g_zero_page);
  const int wave = tid >> 6, lane = tid & 63;
  const int ohb = r0 / 2 - 1 + g.pt2, owb = c0 / 2 - 1 + g.pl2;
#pragma unroll
  for (int j = 0; j < (RT_CHUNKS + NT - 1) / NT; ++j) {
    const int q0 = j * NT + wave * 64;
    if (q0 < RT_CHUNKS) {
      const int q = q0 + lane;
      const unsigned char* src = zp;
      if (q < RT_N * 8) {
        const int o = q >> 3, part = q & 7;
        const int oh = ohb + o / RT_OW, ow = owb + o % RT_OW;
        if (oh >= 0 && oh < g.H2 && ow >= 0 && ow < g.W2)
          src = reinterpret_cast<const unsigned char*>(dp) +
                (((long long)b * g.H2 + oh) * g.W2 + ow) * 128 + part * 16;
      } else if (q < RT_CHUNKS) {
        const int qa = q - RT_N * 8;
        const int o = qa >> 2, part = qa & 3;
        const int oh = ohb + o / RT_OW, ow = owb + o % RT_OW;
        if (oh >= 0 && oh < g.H2 && ow >= 0 && ow < g.W2)
          src = reinterpret_cast<const unsigned char*>(arg) +
                (((long long)b * g.H2 + oh) * g.W2 + ow) * 64 + part * 16;
      }
      glds16(src, rt + q0 * 16);
    }
  }
}

// 32x32x16 operand: 8 consecutive pixels (k) of column j (0..31) of kernel
// row kh, read transposed from the line buffer (see tr_frag_swz).
__device__ __forceinline__ uint4 tr_frag_lb(const unsigned char* lb, int k0, int kh, int lane) {
  using L = LBuf<B2_TR, B2_TC>;
  const int gq = lane >> 4, i = lane & 15;
  const int q = i >> 2, pp = i & 3;
  const int row = k0 + 8 * (gq >> 1) + q;  // pixel; row + 4 stays in the same tile row
  const int colb = (16 * (gq & 1) + 4 * pp) * 2;
  const int o0 = (2 * (row >> 4) + kh) * L::RB + 16 * (row & 15) + colb;
  const int o1 = o0 + 64;  // pixel row + 4
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(uintptr_t)(const __attribute__((
          address_space(3))) void*)(lb + o0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(uintptr_t)(const __attribute__((
          address_space(3))) void*)(lb + o1));
  const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(uint4, v);
}

__global__ __launch_bounds__(256, 2) void stem_bwd_fused_kernel(
    const unsigned char* __restrict__ xp, const unsigned char* __restrict__ ws,
    const uint16_t* __restrict__ dp, const uint8_t* __restrict__ arg,
    const float* __restrict__ coef1, const float* __restrict__ bcoef1, float* __restrict__ slab,
    FGeom g, int tiles_w, int tiles_img, int ntiles) {
  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
  unsigned char* wl = smem;
  unsigned char* lbuf0 = smem + W_BYTES;
  unsigned char* rtb0 = smem + W_BYTES + 2 * B2_LB;
  unsigned char* yt = smem + W_BYTES + 2 * B2_LB + 2 * B2_RT;
  float* cf = reinterpret_cast<float*>(yt + B2_YT);  // [5][64]: a1, s1, k1, k0, k3
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r32 = lane & 31, h = lane >> 5;
  const int blk = xcd_linear(blockIdx.x, gridDim.x), nblk = gridDim.x;

  auto tile_pos = [&](int T, int& b, int& r0, int& c0) {
    b = T / tiles_img;
    const int rem = T - b * tiles_img;
    const int th = rem / tiles_w;
    r0 = th * B2_TR;
    c0 = (rem - th * tiles_w) * B2_TC;
  };
  if (blk < ntiles) {
    int b, r0, c0;
    tile_pos(blk, b, r0, c0);
    issue_lbuf<B2_TR, B2_TC, 256>(lbuf0, xp, g, b, r0, c0, tid);
    issue_route<256>(rtb0, dp, arg, g, b, r0, c0, tid);
  }
  load_weights<256>(wl, ws, tid);
  for (int i = tid; i < 5 * SC; i += 256)
    cf[i] = i < 2 * SC ? coef1[i] : bcoef1[i - 2 * SC];

  // phase c: wave w owns kernel rows 2w, 2w+1 (wave 3: row 6) for all 64
  // channels and all 128 pixels of the tile
  const int kh0 = 2 * wave, nkh = wave < 3 ? 2 : 1;
  f32x16 accw[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) accw[a][j][r] = 0.f;

  // phase-b thread roles
  const int cell = tid >> 3, cgp = tid & 7;
  const int cr = cell >> 3, cc = cell & 7;

  int it = 0;
  for (int T = blk; T < ntiles; T += nblk, ++it) {
    const int cur = it & 1;
    tile_barrier();
    int b, r0, c0;
    tile_pos(T, b, r0, c0);
    if (T + nblk < ntiles) {
      int bn, rn, cn;
      tile_pos(T + nblk, bn, rn, cn);
      issue_lbuf<B2_TR, B2_TC, 256>(lbuf0 + (cur ^ 1) * B2_LB, xp, g, bn, rn, cn, tid);
      issue_route<256>(rtb0 + (cur ^ 1) * B2_RT, dp, arg, g, bn, rn, cn, tid);
    }
    // ---- a) conv -> yt
    {
      f32x16 acc[2][1];
      conv_tile<B2_TR, B2_TC, 1>(wl, lbuf0 + cur * B2_LB, 32 * wave, lane, acc);
      const int m = 32 * wave + r32;
      const int swz = tr_swz<128>(m);
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int chunk = 4 * a + q;
          const uint2 v = make_uint2(zk::pack_bf16x2(acc[a][0][4 * q], acc[a][0][4 * q + 1]),
                                     zk::pack_bf16x2(acc[a][0][4 * q + 2], acc[a][0][4 * q + 3]));
          *reinterpret_cast<uint2*>(yt + m * 128 + ((chunk ^ swz) << 4) + 8 * h) = v;
        }
    }
    lds_barrier();
    // ---- b) dy1 in place
    {
      const unsigned char* rt = rtb0 + cur * B2_RT;
      const int ohb = r0 / 2 - 1 + g.pt2, owb = c0 / 2 - 1 + g.pl2;
      uint32_t aw[2][2][2];
      uint4 gq[2][2];  // dp of the candidates, packed bf16
      bool cv[2][2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int o = (cr + i) * RT_OW + cc + j;
          const int oh = ohb + cr + i, ow = owb + cc + j;
          cv[i][j] = oh >= 0 && oh < g.H2 && ow >= 0 && ow < g.W2;
          const uint2 av = *reinterpret_cast<const uint2*>(rt + RT_DP + o * 64 + cgp * 8);
          aw[i][j][0] = av.x;
          aw[i][j][1] = av.y;
          gq[i][j] = *reinterpret_cast<const uint4*>(rt + o * 128 + cgp * 16);
        }
      // the four pixels' y1 and the channel coefficients, loads up front
      uint4 yq[4];
#pragma unroll
      for (int pq = 0; pq < 4; ++pq) {
        const int m = (2 * cr + (pq >> 1)) * B2_TC + 2 * cc + (pq & 1);
        yq[pq] = *reinterpret_cast<const uint4*>(yt + m * 128 + ((cgp ^ tr_swz<128>(m)) << 4));
      }
      const float4* c4 = reinterpret_cast<const float4*>(cf + cgp * 8);
      float ca[8], cs[8], k1[8], k0[8], k3[8];
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        const float4 v0 = c4[hf], v1 = c4[SC / 4 + hf], v2 = c4[2 * SC / 4 + hf],
                     v3 = c4[3 * SC / 4 + hf], v4 = c4[4 * SC / 4 + hf];
        ca[4 * hf] = v0.x; ca[4 * hf + 1] = v0.y; ca[4 * hf + 2] = v0.z; ca[4 * hf + 3] = v0.w;
        cs[4 * hf] = v1.x; cs[4 * hf + 1] = v1.y; cs[4 * hf + 2] = v1.z; cs[4 * hf + 3] = v1.w;
        k1[4 * hf] = v2.x; k1[4 * hf + 1] = v2.y; k1[4 * hf + 2] = v2.z; k1[4 * hf + 3] = v2.w;
        k0[4 * hf] = v3.x; k0[4 * hf + 1] = v3.y; k0[4 * hf + 2] = v3.z; k0[4 * hf + 3] = v3.w;
        k3[4 * hf] = v4.x; k3[4 * hf + 1] = v4.y; k3[4 * hf + 2] = v4.z; k3[4 * hf + 3] = v4.w;
      }
      float gv[2][2][8];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) unpack8(gq[i][j], gv[i][j]);
#pragma unroll
      for (int pq = 0; pq < 4; ++pq) {
        const int dy = pq >> 1, dx = pq & 1;
        const int hh = r0 + 2 * cr + dy, ww = c0 + 2 * cc + dx;
        float du[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            // tap of this pixel in the window of pool output (ohb+cr+i, owb+cc+j);
            // the range test is uniform (pt2, pl2), the candidate's validity not
            const int th = dy + 2 - g.pt2 - 2 * i, tw = dx + 2 - g.pl2 - 2 * j;
            if (th < 0 || th > 2 || tw < 0 || tw > 2) continue;
            const uint32_t t = th * 3 + tw;
            const uint32_t tm = cv[i][j] ? t : 0xFFu;  // 0xFF never matches a tap
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              const bool hit = ((aw[i][j][k >> 2] >> (8 * (k & 3))) & 0xff) == tm;
              du[k] += hit ? gv[i][j][k] : 0.f;
            }
          }
        const int m = (2 * cr + dy) * B2_TC + 2 * cc + dx;
        float yv[8], o8[8];
        unpack8(yq[pq], yv);
        const bool live = hh < g.Ho && ww < g.Wo;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float u = fmaf(ca[k], yv[k], cs[k]);
          const float v = k1[k] * (u > 0.f ? du[k] : 0.f) + k0[k] - k3[k] * yv[k];
          o8[k] = live ? v : 0.f;
        }
        *reinterpret_cast<uint4*>(yt + m * 128 + ((cgp ^ tr_swz<128>(m)) << 4)) = pack8f(o8);
      }
    }
    lds_barrier();
    // ---- c) weight gradient
    {
      const unsigned char* lbc = lbuf0 + cur * B2_LB;
#pragma unroll 2
      for (int s = 0; s < 8; ++s) {
        const int k0 = 16 * s;
        uint4 af[2];
#pragma unroll
        for (int a = 0; a < 2; ++a) af[a] = tr_frag_swz<128>(yt, k0, 32 * a, lane);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          if (j < nkh) {  // wave-uniform
            const uint4 bfr = tr_frag_lb(lbc, k0, kh0 + j, lane);
#pragma unroll
            for (int a = 0; a < 2; ++a) accw[a][j] = mfma_bf16(af[a], bfr, accw[a][j]);
          }
        }
      }
    }
  }

  // one plain-stored dW partial per block: slab[block][co][kh*32 + j]
  float* sl = slab + (long long)blockIdx.x * B2_NSLAB;
  constexpr int NR = SKH * 32;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    if (j >= nkh) continue;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = 32 * a + 8 * (r >> 2) + 4 * h + (r & 3);
        sl[co * NR + (kh0 + j) * 32 + r32] = accw[a][j][r];
      }
  }
}

// dw OHWI [64][KH][KW][Cin] += sum over blocks of slab[blk][co][kh*32 + kw*4 + c],
// in a fixed order (run-to-run identical): pass 1 sums every gridDim.y-th slab
// into tmp[blockIdx.y], pass 2 sums the groups in order and adds into dW.
constexpr int B2_GROUPS = 32;

__global__ __launch_bounds__(256) void stem_wgrad_reduce_kernel(const float* __restrict__ slab,
                                                                int nblk,
                                                                float* __restrict__ tmp) {
  const int i = blockIdx.x * 256 + threadIdx.x;  // over SC * SKH * 32
  if (i >= B2_NSLAB) return;
  float t[4] = {0.f, 0.f, 0.f, 0.f};
  int s = blockIdx.y;
  for (; s + 3 * (int)gridDim.y < nblk; s += 4 * gridDim.y) {
#pragma unroll
    for (int u = 0; u < 4; ++u) t[u] += slab[(long long)(s + u * gridDim.y) * B2_NSLAB + i];
  }
  for (; s < nblk; s += gridDim.y) t[0] += slab[(long long)s * B2_NSLAB + i];
  tmp[(long long)blockIdx.y * B2_NSLAB + i] = (t[0] + t[1]) + (t[2] + t[3]);
}

__global__ __launch_bounds__(256) void stem_wgrad_reduce2_kernel(const float* __restrict__ tmp,
                                                                 int groups,
                                                                 float* __restrict__ dw, int KW,
                                                                 int Cin) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= B2_NSLAB) return;
  const int j = i & 31, kh = (i >> 5) % SKH, co = i / (SKH * 32);
  const int kw = j >> 2, c = j & 3;
  if (kw >= KW || c >= Cin) return;
  float t = 0.f;
  for (int g = 0; g < groups; ++g) t += tmp[(long long)g * B2_NSLAB + i];
  dw[((co * SKH + kh) * KW + kw) * Cin + c] += t;
}

// B1 from the pooled side with the exact y1 at the argmax (F2's ya):
// du = dp [a1 ya + s1 > 0], sums of du and du * (ya - mean) * rstd.
__global__ __launch_bounds__(256) void stem_pool_bwd_sums_ya_kernel(
    const uint16_t* __restrict__ dp, const uint16_t* __restrict__ ya,
    const float* __restrict__ coef, float* __restrict__ part, long long P2) {
  const int cg = threadIdx.x & 7;
  float a[8], sh[8], mean[8], rstd[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    a[k] = coef[cg * 8 + k];
    sh[k] = coef[SC + cg * 8 + k];
    mean[k] = coef[2 * SC + cg * 8 + k];
    rstd[k] = coef[3 * SC + cg * 8 + k];
  }
  float s1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (long long o = blockIdx.x * 32LL + (threadIdx.x >> 3); o < P2; o += gridDim.x * 32LL) {
    const long long off = o * SC + cg * 8;
    float gv[8], yv[8];
    unpack8(*reinterpret_cast<const uint4*>(dp + off), gv);
    unpack8(*reinterpret_cast<const uint4*>(ya + off), yv);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float du = fmaf(a[k], yv[k], sh[k]) > 0.f ? gv[k] : 0.f;
      s1[k] += du;
      s2[k] += du * (yv[k] - mean[k]) * rstd[k];
    }
  }
  __shared__ float red[2][256][9];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    red[0][threadIdx.x][k] = s1[k];
    red[1][threadIdx.x][k] = s2[k];
  }
  __syncthreads();
  if (threadIdx.x < 2 * SC) {
    const int which = threadIdx.x / SC, ch = threadIdx.x % SC, gq = ch >> 3, k = ch & 7;
    float t = 0.f;
    for (int r = gq; r < 256; r += 8) t += red[which][r][k];
    part[((long long)blockIdx.x * 2 + which) * SC + ch] = t;
  }
}

int g_cus = 0;
int cu_count() {
  if (!g_cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        g_cus <= 0)
      g_cus = 256;
  }
  return g_cus;
}

template <typename K>
int set_lds_once(K kern, int bytes) {
  static bool done = false;
  if (!done) {
    hipError_t e =
        hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e != hipSuccess) return (int)e;
    done = true;
  }
  return 0;
}

bool fgeom_ok(const FGeom& g) {
  return g.B > 0 && g.Cin >= 1 && g.Cin <= 4 && g.KW >= 1 && g.KW <= 8 && g.Ho > 0 && g.Wo > 0 &&
         (g.Ho - 1) * 2 + SKH <= g.Hp && (g.Wo - 1) * 2 + 8 <= g.Wp && g.pt2 >= 0 && g.pt2 <= 1 &&
         g.pl2 >= 0 && g.pl2 <= 1 && g.H2 == (g.Ho + g.pt2 + 1) / 2 &&  // 3x3/2 'same'
         g.W2 == (g.Wo + g.pl2 + 1) / 2 && (long long)g.B * g.H2 * g.W2 < (1LL << 31);
}

int grid_for(long long ntiles, int per_cu) {
  long long gsz = (long long)cu_count() * per_cu;
  if (gsz > ntiles) gsz = ntiles;
  return gsz < 1 ? 1 : (int)gsz;
}

}  // namespace

// Number of per-block partial rows / slabs a pass writes (host-side sizing).
ZK_EXPORT int zk_stem_fused_blocks(int which, int B, int Ho, int Wo, int H2, int W2) {
  long long nt;
  if (which == 1) {  // F2: pool tiles, one block per CU
    nt = (long long)B * ((H2 + F2_PR - 1) / F2_PR) * ((W2 + F2_PC - 1) / F2_PC);
    return grid_for(nt, 1);
  }
  nt = (long long)B * ((Ho + 7) / 8) * ((Wo + 15) / 16);  // F1 / B2: conv tiles
  return grid_for(nt, 2);
}

ZK_EXPORT int zk_stem_fused_slab_floats() { return B2_NSLAB; }
// extra slab rows zk_stem_bwd_fused needs beyond one per block (reduction groups)
ZK_EXPORT int zk_stem_fused_slab_extra() { return B2_GROUPS; }

ZK_EXPORT int zk_stem_fwd_stats(const void* xp, const void* ws, void* part, int B, int Cin,
                                int KW, int Ho, int Wo, int Hp, int Wp, int H2, int W2, int pt2,
                                int pl2, int* nparts, hipStream_t st) {
  FGeom g{B, Cin, KW, Ho, Wo, Hp, Wp, H2, W2, pt2, pl2};
  if (!fgeom_ok(g)) return (int)hipErrorInvalidValue;
  const int tw = (Wo + F1_TC - 1) / F1_TC, th = (Ho + F1_TR - 1) / F1_TR;
  const long long nt = (long long)B * th * tw;
  if (nt >= (1LL << 31)) return (int)hipErrorInvalidValue;
  const int grid = grid_for(nt, 2);
  if (nparts) *nparts = grid;
  if (int e = set_lds_once(stem_fwd_stats_kernel, F1_LDS)) return e;
  hipLaunchKernelGGL(stem_fwd_stats_kernel, dim3(grid), dim3(256), F1_LDS, st,
                     (const unsigned char*)xp, (const unsigned char*)ws, (float*)part, g, tw,
                     th * tw, (int)nt);
  ZK_CHECK_LAUNCH();
  return 0;
}

ZK_EXPORT int zk_stem_fwd_pool(const void* xp, const void* ws, const void* coef1, void* p,
                               void* arg, void* ya, void* part, int B, int Cin, int KW, int Ho,
                               int Wo, int Hp, int Wp, int H2, int W2, int pt2, int pl2,
                               int* nparts, hipStream_t st) {
  FGeom g{B, Cin, KW, Ho, Wo, Hp, Wp, H2, W2, pt2, pl2};
  if (!fgeom_ok(g)) return (int)hipErrorInvalidValue;
  const int tw = (W2 + F2_PC - 1) / F2_PC, th = (H2 + F2_PR - 1) / F2_PR;
  const long long nt = (long long)B * th * tw;
  if (nt >= (1LL << 31)) return (int)hipErrorInvalidValue;
  const int grid = grid_for(nt, 1);
  if (nparts) *nparts = grid;
  if (int e = set_lds_once(stem_fwd_pool_kernel, F2_LDS)) return e;
  hipLaunchKernelGGL(stem_fwd_pool_kernel, dim3(grid), dim3(F2_NT), F2_LDS, st,
                     (const unsigned char*)xp, (const unsigned char*)ws, (const float*)coef1,
                     (uint16_t*)p, (uint8_t*)arg, (uint16_t*)ya, (float*)part, g, tw, th * tw,
                     (int)nt);
  ZK_CHECK_LAUNCH();
  return 0;
}

ZK_EXPORT int zk_stem_pool_bwd_sums_ya(const void* dp, const void* ya, const void* coef1,
                                       void* part, long long P2, int* nparts, hipStream_t st) {
  long long grid = (P2 + 31) / 32;
  if (grid > 4096) grid = 4096;
  if (grid < 1) grid = 1;
  if (nparts) *nparts = (int)grid;
  hipLaunchKernelGGL(stem_pool_bwd_sums_ya_kernel, dim3((int)grid), dim3(256), 0, st,
                     (const uint16_t*)dp, (const uint16_t*)ya, (const float*)coef1, (float*)part,
                     P2);
  ZK_CHECK_LAUNCH();
  return 0;
}

// slab: [zk_stem_fused_blocks(0, ...) + zk_stem_fused_slab_extra()]
// [zk_stem_fused_slab_floats()] fp32 scratch; dw: OHWI fp32 gradient,
// accumulated.
ZK_EXPORT int zk_stem_bwd_fused(const void* xp, const void* ws, const void* dp, const void* arg,
                                const void* coef1, const void* bcoef1, void* slab, void* dw,
                                int B, int Cin, int KW, int Ho, int Wo, int Hp, int Wp, int H2,
                                int W2, int pt2, int pl2, hipStream_t st) {
  FGeom g{B, Cin, KW, Ho, Wo, Hp, Wp, H2, W2, pt2, pl2};
  if (!fgeom_ok(g)) return (int)hipErrorInvalidValue;
  const int tw = (Wo + B2_TC - 1) / B2_TC, th = (Ho + B2_TR - 1) / B2_TR;
  const long long nt = (long long)B * th * tw;
  if (nt >= (1LL << 31)) return (int)hipErrorInvalidValue;
  const int grid = grid_for(nt, 2);
  if (int e = set_lds_once(stem_bwd_fused_kernel, B2_LDS)) return e;
  hipLaunchKernelGGL(stem_bwd_fused_kernel, dim3(grid), dim3(256), B2_LDS, st,
                     (const unsigned char*)xp, (const unsigned char*)ws, (const uint16_t*)dp,
                     (const uint8_t*)arg, (const float*)coef1, (const float*)bcoef1,
                     (float*)slab, g, tw, th * tw, (int)nt);
  ZK_CHECK_LAUNCH();
  const int groups = grid < B2_GROUPS ? grid : B2_GROUPS;
  float* tmp = (float*)slab + (long long)grid * B2_NSLAB;
  hipLaunchKernelGGL(stem_wgrad_reduce_kernel, dim3((B2_NSLAB + 255) / 256, groups), dim3(256), 0,
                     st, (const float*)slab, grid, tmp);
  ZK_CHECK_LAUNCH();
  hipLaunchKernelGGL(stem_wgrad_reduce2_kernel, dim3((B2_NSLAB + 255) / 256), dim3(256), 0, st,
                     (const float*)tmp, groups, (float*)dw, KW, Cin);
  ZK_CHECK_LAUNCH();
  return 0;
}
