// Persistent binary forward for the 64 -> 64-channel 3x3 stride-1 'same'
// convolutions (BinaryResNet-E18 stage 1, QuickNet's first section) on MX-FP4
// MFMA, for gfx950.
//
// y[m][co] = sum over the 9 taps and 64 input channels of sign(x) * sign(W)
// (exact integers, |y| <= 576) as int16, plus the per-channel sum and sum of
// squares for the following BatchNorm -- the same outputs, bit for bit, as
// igemm.hip's conv3 forward (igemm_conv3_kernel<true, ..., F4>, 285-317 us
// at batch 1536: 37.6k short-lived blocks, each with its own prologue, three
// barriered K-steps, 64 two-byte stores per lane and 128 int64 statistics
// atomics).  Here (MI355X, batch 1536 per GPU):
//   * persistent blocks (2 per CU, 4 waves) walk 256-pixel tiles (64 pixels
//     per wave); the union of the three kernel rows' input windows (256 + 2 W
//     + 2 flattened pixels x 32 B of e2m1 signs) streams into a three-stage
//     LDS ring by global_load_lds two tiles ahead (one barrier per tile);
//   * the 18 KB weight image stays in LDS for the whole launch; per tile a
//     wave reads each of the 18 weight fragments once and issues 36
//     v_mfma_scale_f32_32x32x64_f8f6f4 (D[co][pixel]: lane = pixel);
//   * padded taps read a pad row (zeros or e2m1 +1) through a per-lane
//     address select on scalar edge masks;
//   * the epilogue stays in fp32 (v_pk_add / v_pk_fma): the statistics
//     accumulate in fp32 registers (exact: integers below 2^24, flushed to
//     integers every BF_FLUSH tiles) and the int16 outputs come from the
//     float bits after adding 1.5 * 2^23, paired by v_perm, exchanged by
//     v_permlane32_swap into 16-B slots and staged through a per-wave LDS
//     area so every global store writes whole 128-B rows;
//   * the statistics are reduced once per flush: a reduce-scatter over the
//     lanes, one LDS pass at the end, 128 int64 atomics per block.
// Reference: the QuantConv2D -> BatchNorm pairs of
// /root/reference/examples/larq_experiment.py:71-91.
#include "mfma_common.h"

namespace {

constexpr int BF_C = 64;        // input and output channels
constexpr int BF_TM = 256;      // pixels per tile (4 waves x 64)
constexpr int BF_NT = 256;      // threads per block
constexpr int BF_ROW = 32;      // bytes per pixel (64 e2m1 nibbles)
constexpr int BF_WMAX = 60;     // widest image: the stage holds the union of the
                                // three kernel rows' windows, BF_TM + 2 W + 2 rows
constexpr int BF_CHMAX = 2 * (BF_TM + 2 * BF_WMAX + 2);   // 16-B chunks per stage (756)
constexpr int BF_ROUNDS = (BF_CHMAX + BF_NT - 1) / BF_NT;  // DMA rounds (3)
constexpr int BF_STAGE = BF_ROUNDS * BF_NT * 16;           // 12 KB
constexpr int BF_NS = 3;                            // ring: issued two tiles ahead
constexpr int BF_WBYTES = 9 * BF_C * BF_ROW;        // weight image, 18 KB
constexpr int BF_WOFF = BF_NS * BF_STAGE;
constexpr int BF_PADOFF = BF_WOFF + BF_WBYTES;      // 16-B pad fragment
constexpr int BF_YOFF = BF_PADOFF + 16;             // output staging, 4 KB per wave
constexpr int BF_LDS = BF_YOFF + 4 * 32 * 128;
constexpr int BF_FLUSH = 24;   // tiles between statistics flushes: 2 pixels per
                               // lane and tile, 24 * 2 * 576^2 < 2^24
static_assert(2 * BF_LDS <= 160 * 1024, "two blocks per CU");

typedef float f32x2 __attribute__((ext_vector_type(2)));

// Swizzle of the two 16-B halves of a staged pixel row: rows 8..15 of every
// 16 swap them, so the fragment reads of 16 consecutive rows (same half) hit
// 16 distinct 16-B bank slots.
__device__ __forceinline__ int bf_swz(int row) { return (row >> 3) & 1; }

// Reduce-scatter of 32 ints over the 32 lanes of a wave half (lane r ends
// with the half's total of value r).
template <int N>
__device__ __forceinline__ void rsi_step(int (&v)[32], int r32) {
  const bool upper = (r32 & N) != 0;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const int send = upper ? v[i] : v[i + N];
    const int keep = upper ? v[i + N] : v[i];
    v[i] = keep + __shfl_xor(send, N, 64);
  }
}
__device__ __forceinline__ int rsi32(int (&v)[32], int r32) {
  rsi_step<16>(v, r32);
  rsi_step<8>(v, r32);
  rsi_step<4>(v, r32);
  rsi_step<2>(v, r32);
  rsi_step<1>(v, r32);
  return v[0];
}

// s_waitcnt vmcnt(n) for a wave-uniform n in [0, 24]
__device__ __forceinline__ void bf_wait(int n) {
  switch (n) {
#define ZK_BFW(k) \
  case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    ZK_BFW(1) ZK_BFW(2) ZK_BFW(3) ZK_BFW(4) ZK_BFW(5) ZK_BFW(6) ZK_BFW(7) ZK_BFW(8)
    ZK_BFW(9) ZK_BFW(10) ZK_BFW(11) ZK_BFW(12) ZK_BFW(13) ZK_BFW(14) ZK_BFW(15) ZK_BFW(16)
    ZK_BFW(17) ZK_BFW(18) ZK_BFW(19) ZK_BFW(20) ZK_BFW(21) ZK_BFW(22) ZK_BFW(23) ZK_BFW(24)
#undef ZK_BFW
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

// Diagnostic build only (-DZK_BFWD_STAMPS, tools/bfwd_stamps.cpp): per wave,
// the shader cycles (s_memtime) of each phase of the tile loop.
#ifdef ZK_BFWD_STAMPS
__device__ unsigned long long g_bf_stamps[2048 * 4][6];
#define BF_ST_BEGIN \
  unsigned long long zb_t = __builtin_readcyclecounter(), zb[6] = {0, 0, 0, 0, 0, 0};
#define BF_ST(k)                                                   \
  {                                                                \
    const unsigned long long t_ = __builtin_readcyclecounter();    \
    zb[k] += t_ - zb_t;                                            \
    zb_t = t_;                                                     \
  }
#define BF_ST_STORE                                                        \
  if ((threadIdx.x & 63) == 0 && blockIdx.x < 2048)                        \
    for (int k_ = 0; k_ < 6; ++k_) g_bf_stamps[blockIdx.x * 4 + (threadIdx.x >> 6)][k_] = zb[k_];
#else
#define BF_ST_BEGIN
#define BF_ST(k)
#define BF_ST_STORE
#endif

struct BfArgs {
  const unsigned char* x4;   // [M][32] e2m1 sign image (channel 2j: low nibble of byte j)
  const unsigned char* w4;   // [9][64][32] e2m1 weight signs
  short* y;                  // [M][64] int16
  unsigned long long* stats;  // [stripes][2][64] int64 (sum; sum of squares)
  int M, H, W, stripes, ntiles;
  int pad_ones;
  float inv_w, inv_h;
};

// Statistics flush: the fp32 per-lane accumulators (exact integers) -> the
// per-lane running totals of value r32 of this wave half.
__device__ __forceinline__ void bf_flush(f32x16 (&cs)[2], f32x16 (&cq)[2], int r32,
                                         long long& tsum, unsigned long long& tsq) {
  int v[32];
#pragma unroll
  for (int i = 0; i < 32; ++i) v[i] = (int)cs[i >> 4][i & 15];
  tsum += rsi32(v, r32);
#pragma unroll
  for (int i = 0; i < 32; ++i) v[i] = (int)(unsigned)cq[i >> 4][i & 15];
  tsq += (unsigned)rsi32(v, r32);
#pragma unroll
  for (int e = 0; e < 2; ++e) cs[e] = cq[e] = f32x16{};
}

template <bool RELU>
__global__ __launch_bounds__(BF_NT, 2) void bfwd64_kernel(BfArgs a) {
  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, h = lane >> 5;
  const int blk = xcd_linear(blockIdx.x, gridDim.x), nblk = gridDim.x;
  const int n = blk < a.ntiles ? (a.ntiles - 1 - blk) / nblk + 1 : 0;
  const unsigned char* zp = reinterpret_cast<const unsigned char*>(g_zero_page);
  const int Mb = a.M * BF_ROW;

  // weight image [t][co][32 B] -> LDS (halves swizzled like the pixel rows),
  // plus the pad fragment
  unsigned char* wl = smem + BF_WOFF;
  for (int q = tid; q < BF_WBYTES / 16; q += BF_NT) {
    const int row = q >> 1, c = q & 1;
    *reinterpret_cast<uint4*>(wl + row * BF_ROW + ((c ^ bf_swz(row)) << 4)) =
        *reinterpret_cast<const uint4*>(a.w4 + q * 16);
  }
  if (tid < 4)
    reinterpret_cast<uint32_t*>(smem + BF_PADOFF)[tid] = a.pad_ones ? 0x22222222u : 0u;

  // DMA plan: stage row r <-> flattened pixel m0 - W - 1 + r (the union of
  // the three kernel rows' windows); chunk q = j * 256 + tid -> byte offset
  // from the tile's first pixel (LDS slot half c holds source half c ^ swz)
  const int nch = 2 * (BF_TM + 2 * a.W + 2);
  int kb[BF_ROUNDS];
  int nd = 0;  // DMA instructions of this wave per stage
#pragma unroll
  for (int j = 0; j < BF_ROUNDS; ++j) {
    const int q = j * BF_NT + tid;
    nd += j * BF_NT + wave * 64 < nch;
    const int row = q >> 1, c = q & 1;
    kb[j] = q < nch ? (row - a.W - 1) * BF_ROW + ((c ^ bf_swz(row)) << 4)
                    : -(1 << 30);  // past the stage: the zero page
  }
  auto issue = [&](int jt) {  // stage of this block's tile jt
    const int m0b = (blk + jt * nblk) * BF_TM * BF_ROW;
    unsigned char* st = smem + (jt % BF_NS) * BF_STAGE;
#pragma unroll
    for (int j = 0; j < BF_ROUNDS; ++j) {
      const int q0 = j * BF_NT + wave * 64;  // wave-uniform
      if (q0 < nch) {
        const int off = m0b + kb[j];
        glds16((unsigned)off < (unsigned)Mb ? a.x4 + off : zp, st + q0 * 16);
      }
    }
  };
  if (n > 0) issue(0);
  if (n > 1) issue(1);

  // per-lane constants of the fragment reads: tap (th, tw) of pixel 64 wave +
  // 32 u + r32 is stage row 64 wave + 32 u + (r32 + th W + tw), at byte
  // 2 KB * wave + 1 KB * u + lo[t]
  int lo[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int row = r32 + (t / 3) * a.W + t % 3;
    lo[t] = row * BF_ROW + ((h ^ bf_swz(row)) << 4);
  }
  const int wlo = (r32 * BF_ROW) + ((h ^ bf_swz(r32)) << 4);  // weight row 32 e + r32
  unsigned char* ys = smem + BF_YOFF + wave * (32 * 128);     // this wave's output rows

  f32x16 cs[2] = {}, cq[2] = {};
  long long tsum = 0;
  unsigned long long tsq = 0;
  const int ns = a.y ? 8 : 0;  // global stores per wave and tile
  BF_ST_BEGIN
  for (int it = 0; it < n; ++it) {
    // this tile's stage has landed: issued at the top of tile it - 2 (or
    // before the loop), it is followed by the stores of tiles it - 2 and
    // it - 1 and the DMA of tile it + 1 (counted in issue order)
    bf_wait(it == 0 ? (n > 1 ? nd : 0)
                    : (it == 1 ? ns : 2 * ns) + (it + 1 < n ? nd : 0));
    BF_ST(0)
    __syncthreads();
    BF_ST(1)
    // every wave is past tile it - 1, whose stage the DMA of tile it + 2 reuses
    if (it + 2 < n) issue(it + 2);
    const int m0 = (blk + it * nblk) * BF_TM;
    const bool full = m0 + BF_TM <= a.M;
    const int sb = (it % BF_NS) * BF_STAGE + wave * (64 * BF_ROW);
    // this lane's two pixels and their edge flags
    bool top[2], bot[2], lft[2], rgt[2], live[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int m = m0 + 64 * wave + 32 * u + r32;
      live[u] = m < a.M;
      const int q1 = fdiv(m, a.W, a.inv_w);
      const int ww = m - q1 * a.W;
      const int hh = q1 - fdiv(q1, a.H, a.inv_h) * a.H;
      top[u] = hh > 0;
      bot[u] = hh < a.H - 1;
      lft[u] = ww > 0;
      rgt[u] = ww < a.W - 1;
    }
    BF_ST(2)
    // ---- 9 taps x 2 channel halves x 2 pixel groups
    f32x16 acc[2][2];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int th = t / 3, tw = t % 3;
      uint4 wv[2];
#pragma unroll
      for (int e = 0; e < 2; ++e)
        wv[e] = *reinterpret_cast<const uint4*>(wl + (t * BF_C + 32 * e) * BF_ROW + wlo);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        bool ok = live[u];
        if (th == 0) ok = ok && top[u];
        if (th == 2) ok = ok && bot[u];
        if (tw == 0) ok = ok && lft[u];
        if (tw == 2) ok = ok && rgt[u];
        const int off = ok ? sb + u * (32 * BF_ROW) + lo[t] : BF_PADOFF;
        const uint4 b = *reinterpret_cast<const uint4*>(smem + off);
#pragma unroll
        for (int e = 0; e < 2; ++e) acc[u][e] = mfma_fp4(wv[e], b, t ? acc[u][e] : f32x16{});
      }
    }
    BF_ST(3)
    // ---- epilogue in packed fp32: statistics, int16 rows staged through LDS
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        f32x16 c = acc[u][e];
        if (RELU) {
#pragma unroll
          for (int r = 0; r < 16; ++r) c[r] = fmaxf(c[r], 0.f);
        }
        if (!full) {
#pragma unroll
          for (int r = 0; r < 16; ++r) c[r] = live[u] ? c[r] : 0.f;
        }
        uint32_t bits[16];
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          const f32x2 v = {c[r], c[r + 1]};
          f32x2 s2 = {cs[e][r], cs[e][r + 1]};
          f32x2 q2 = {cq[e][r], cq[e][r + 1]};
          s2 += v;
          q2 = __builtin_elementwise_fma(v, v, q2);
          cs[e][r] = s2[0];
          cs[e][r + 1] = s2[1];
          cq[e][r] = q2[0];
          cq[e][r + 1] = q2[1];
          // + 1.5 * 2^23: the low 16 bits of the float are the integer.  Scalar
          // adds on purpose: spelled as one f32x2 add, hipcc (ROCm 7.2) packs
          // the wrong halves below -- it reused element 0's bits for element 1
          // (profiles/r6/bfwd.md).
          bits[r] = __builtin_bit_cast(uint32_t, c[r] + 12582912.f);
          bits[r + 1] = __builtin_bit_cast(uint32_t, c[r + 1] + 12582912.f);
        }
        // registers r = 4 q + i hold channels 32 e + 8 q + 4 h + i; after the
        // swap lane (p, h) holds 16-B slot 4 e + 2 pq + h of pixel p, staged
        // at slot ^ (p & 7) (conflict-free 8-lane write groups)
#pragma unroll
        for (int pq = 0; pq < 2; ++pq) {
          uint32_t d[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int r = 4 * (2 * pq + (k >> 1)) + 2 * (k & 1);
            d[k] = __builtin_amdgcn_perm(bits[r + 1], bits[r], 0x05040100u);
          }
          const auto s0 = __builtin_amdgcn_permlane32_swap(d[0], d[2], false, false);
          const auto s1 = __builtin_amdgcn_permlane32_swap(d[1], d[3], false, false);
          const int slot = 4 * e + 2 * pq + h;
          *reinterpret_cast<uint4*>(ys + r32 * 128 + ((slot ^ (r32 & 7)) << 4)) =
              make_uint4(s0[0], s1[0], s0[1], s1[1]);
        }
      }
      // whole 128-B rows: instruction k stores pixels 8 k .. 8 k + 7 of the
      // group (lane l: pixel 8 k + l / 8, slot l % 8)
      const int mg = m0 + 64 * wave + 32 * u;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int p = 8 * k + (lane >> 3), sl = lane & 7;
        const uint4 v = *reinterpret_cast<const uint4*>(ys + p * 128 + ((sl ^ (p & 7)) << 4));
        if (a.y && mg + p < a.M)
          *reinterpret_cast<uint4*>(a.y + (long long)(mg + p) * BF_C + sl * 8) = v;
      }
    }
    BF_ST(4)
    if ((it + 1) % BF_FLUSH == 0) bf_flush(cs, cq, r32, tsum, tsq);
    BF_ST(5)
  }
  BF_ST_STORE
  bf_flush(cs, cq, r32, tsum, tsq);

  // ---- statistics: lane r32 of each half holds value r32 of the half
  const int e = r32 >> 4, r = r32 & 15;
  const int co = 32 * e + 8 * (r >> 2) + 4 * h + (r & 3);
  __syncthreads();
  long long* red = reinterpret_cast<long long*>(smem);  // [4 waves][2][64]
  red[(wave * 2 + 0) * BF_C + co] = tsum;
  red[(wave * 2 + 1) * BF_C + co] = (long long)tsq;
  __syncthreads();
  if (tid < 2 * BF_C) {
    const int which = tid / BF_C, c = tid % BF_C;
    long long tot = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) tot += red[(w * 2 + which) * BF_C + c];
    const int stripe = a.stripes > 1 ? (int)(blockIdx.x % a.stripes) : 0;
    atomicAdd(a.stats + ((long long)stripe * 2 + which) * BF_C + c, (unsigned long long)tot);
  }
}
int bf_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
  }
  return cus;
}

}  // namespace

// Shape check of zk_bfwd64_fp4: 3x3 stride 1 'same', 64 -> 64 channels, the
// image at most BF_WMAX wide (the stage holds 256 + 2 W + 2 rows) and the
// flattened pixel count inside the float-reciprocal division range (the
// statistics are exact at any size: fp32 below 2^24 between flushes, 32-bit
// lane reductions below 2^32, 64-bit totals).
ZK_EXPORT int zk_bfwd64_supported(int B, int H, int W, int Cin, int Cout, int kh, int kw,
                                  int stride, int pt, int pl) {
  const long long M = (long long)B * H * W;
  if (Cin != BF_C || Cout != BF_C || kh != 3 || kw != 3 || stride != 1 || pt != 1 || pl != 1)
    return 0;
  return M > 0 && M < (1LL << 24) && W <= BF_WMAX ? 1 : 0;
}

// y int16 [B][H][W][64] = 3x3 'same' binary conv of the e2m1 sign image x4
// [B][H][W][32 B] with the e2m1 weights w4 [9][64][32 B] (+ReLU), padding
// +1 (pad_ones) or 0; stats [stripes][2][64] int64 += per-channel sum and sum
// of squares of y (block b adds into copy b % stripes).
ZK_EXPORT int zk_bfwd64_fp4(const void* x4, const void* w4, void* y, void* stats, int B, int H,
                            int W, int pad_ones, int relu, int stripes, hipStream_t st) {
  if (!zk_bfwd64_supported(B, H, W, BF_C, BF_C, 3, 3, 1, 1, 1)) return (int)hipErrorInvalidValue;
  BfArgs a{};
  a.x4 = (const unsigned char*)x4;
  a.w4 = (const unsigned char*)w4;
  a.y = (short*)y;
  a.stats = (unsigned long long*)stats;
  a.M = B * H * W;
  a.H = H;
  a.W = W;
  a.stripes = stripes;
  a.ntiles = (a.M + BF_TM - 1) / BF_TM;
  a.pad_ones = pad_ones;
  a.inv_w = 1.f / (float)W;
  a.inv_h = 1.f / (float)H;
  static bool attr = false;
  if (!attr) {
    for (const void* f : {(const void*)bfwd64_kernel<false>, (const void*)bfwd64_kernel<true>}) {
      const hipError_t e =
          hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, BF_LDS);
      if (e != hipSuccess) return (int)e;
    }
    attr = true;
  }
  int grid = 2 * bf_cus();
  if (grid > a.ntiles) grid = a.ntiles;
  if (relu)
    hipLaunchKernelGGL(bfwd64_kernel<true>, dim3(grid), dim3(BF_NT), BF_LDS, st, a);
  else
    hipLaunchKernelGGL(bfwd64_kernel<false>, dim3(grid), dim3(BF_NT), BF_LDS, st, a);
  ZK_CHECK_LAUNCH();
  return 0;
}
