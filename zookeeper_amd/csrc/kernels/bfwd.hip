// Persistent binary forward for the 3x3 stride-1 'same' convolutions with 64
// or 128 input channels (BinaryResNet-E18 stages 1-2, QuickNet's first
// sections) on MX-FP4 MFMA, for gfx950.
//
// y[m][co] = sum over the 9 taps and Cin input channels of sign(x) * sign(W)
// (exact integers, |y| <= 9 Cin) as int16, plus the per-channel sum and sum of
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
// Cin = 128 (BfCfg<128, 8, 2, 32>): one 8-wave block per CU, 512-pixel
// tiles, two-stage ring; each block owns one 64-channel slice of the output
// (its 36 KB weight image in LDS), so the input is read once per slice.
// Reference: the QuantConv2D -> BatchNorm pairs of
// /root/reference/examples/larq_experiment.py:71-91.
#include "mfma_common.h"

namespace {

typedef float f32x2 __attribute__((ext_vector_type(2)));

// Tile / LDS plan of one instantiation: CIN input channels (64 or 128), NW
// waves per block (64 pixels each), NS-stage input ring, images at most WMAX
// wide.  Each block computes one 64-channel slice of the output.
template <int CIN_, int NW_, int NS_, int WMAX_>
struct BfCfg {
  static constexpr int CIN = CIN_, NW = NW_, NS = NS_, WMAX = WMAX_;
  static constexpr int NT = NW * 64;                 // threads per block
  static constexpr int TM = NW * 64;                 // pixels per tile
  static constexpr int ROW = CIN / 2;                // bytes per pixel row (e2m1)
  static constexpr int CH = ROW / 16;                // 16-B chunks per row
  static constexpr int KC = CIN / 64;                // MFMA K-chunks per tap
  static constexpr int RPB = 256 / ROW;              // rows per 256-B bank window
  static constexpr int CHMAX = CH * (TM + 2 * WMAX + 2);   // chunks of the widest stage
  static constexpr int ROUNDS = (CHMAX + NT - 1) / NT;     // DMA rounds per stage
  static constexpr int STAGE = ROUNDS * NT * 16;
  static constexpr int WBYTES = 9 * 64 * ROW;        // weight image of one output slice
  static constexpr int WOFF = NS * STAGE;
  static constexpr int PADOFF = WOFF + WBYTES;       // 16-B pad fragment
  static constexpr int YOFF = PADOFF + 16;           // output staging, 4 KB per wave
  static constexpr int LDS = YOFF + NW * 32 * 128;
  static constexpr int OCC = (2 * LDS <= 160 * 1024) ? 2 : 1;  // blocks per CU
  // tiles between statistics flushes: 2 pixels per lane and tile, the fp32
  // sums of squares exact below 2^24
  static constexpr int FLUSH = (1 << 24) / (2 * (9 * CIN) * (9 * CIN));
  static_assert(LDS <= 160 * 1024, "LDS");
  static_assert(FLUSH >= 1, "flush interval");
  // Swizzle of a staged row's 16-B chunks: the fragment reads of 16
  // consecutive rows (same chunk) hit 16 distinct 16-B bank slots.
  __device__ static __forceinline__ int swz(int row) { return (row / RPB) % CH; }
};
using Bf64 = BfCfg<64, 4, 3, 60>;    // 2 blocks per CU, 256-pixel tiles, 3-stage ring
using Bf128 = BfCfg<128, 8, 2, 32>;  // 1 block per CU, 512-pixel tiles, 2-stage ring

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
__device__ unsigned long long g_bf_stamps[2048 * 8][6];
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
    for (int k_ = 0; k_ < 6; ++k_)                                         \
      g_bf_stamps[blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)][k_] = zb[k_];
#else
#define BF_ST_BEGIN
#define BF_ST(k)
#define BF_ST_STORE
#endif

struct BfArgs {
  const unsigned char* x4;   // [M][Cin/2] e2m1 sign image (channel 2j: low nibble of byte j)
  const unsigned char* w4;   // [9][Cout][Cin/2] e2m1 weight signs
  short* y;                  // [M][Cout] int16
  unsigned long long* stats;  // [stripes][2][Cout] int64 (sum; sum of squares)
  int M, H, W, Cout, nsl, stripes, ntiles;
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

// vm ops a wave issued after the DMA of its tile `it` (issue order: the
// prologue's LA stages, then per tile the DMA of tile + LA after the barrier
// and the tile's ns stores; nd DMA instructions per stage)
template <int LA>
__device__ __forceinline__ int bf_after(int it, int n, int nd, int ns) {
  int after = 0;
  if (it < LA) {
#pragma unroll
    for (int j = 1; j < LA; ++j) after += (it + j < LA && it + j < n) ? nd : 0;
    for (int k = 0; k < it; ++k) after += (k + LA < n ? nd : 0) + ns;
  } else {
    after += ns;
#pragma unroll
    for (int d = 1; d < LA; ++d) {
      const int k = it - LA + d;
      after += (k + LA < n ? nd : 0) + ns;
    }
  }
  return after;
}

template <class C, bool RELU>
__global__ __launch_bounds__(C::NT, C::OCC) void bfwd_kernel(BfArgs a) {
  constexpr int NT = C::NT, TM = C::TM, ROW = C::ROW, CH = C::CH, KC = C::KC;
  constexpr int LA = C::NS - 1;  // tiles of DMA lookahead
  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, h = lane >> 5;
  // logical block: output slice L % nsl, tile stream L / nsl
  const int L = xcd_linear(blockIdx.x, gridDim.x);
  const int slice = L % a.nsl, blk = L / a.nsl, nblk = gridDim.x / a.nsl;
  const int n = blk < a.ntiles ? (a.ntiles - 1 - blk) / nblk + 1 : 0;
  const unsigned char* zp = reinterpret_cast<const unsigned char*>(g_zero_page);
  const int Mb = a.M * ROW;

  // this slice's weight image [t][64 co][ROW] -> LDS (chunks swizzled like
  // the pixel rows), plus the pad fragment
  unsigned char* wl = smem + C::WOFF;
  for (int q = tid; q < C::WBYTES / 16; q += NT) {
    const int row = q / CH, c = q % CH;  // row = t * 64 + co
    const int t = row >> 6, co = row & 63;
    *reinterpret_cast<uint4*>(wl + row * ROW + ((c ^ C::swz(row)) << 4)) =
        *reinterpret_cast<const uint4*>(a.w4 + ((long long)t * a.Cout + slice * 64 + co) * ROW +
                                        c * 16);
  }
  if (tid < 4)
    reinterpret_cast<uint32_t*>(smem + C::PADOFF)[tid] = a.pad_ones ? 0x22222222u : 0u;

  // DMA plan: stage row r <-> flattened pixel m0 - W - 1 + r (the union of
  // the three kernel rows' windows); chunk q = j * NT + tid -> byte offset
  // from the tile's first pixel (LDS slot c holds source chunk c ^ swz(row))
  const int nch = CH * (TM + 2 * a.W + 2);
  int kb[C::ROUNDS];
  int nd = 0;  // DMA instructions of this wave per stage
#pragma unroll
  for (int j = 0; j < C::ROUNDS; ++j) {
    const int q = j * NT + tid;
    nd += j * NT + wave * 64 < nch;
    const int row = q / CH, c = q % CH;
    kb[j] = q < nch ? (row - a.W - 1) * ROW + ((c ^ C::swz(row)) << 4)
                    : -(1 << 30);  // past the stage: the zero page
  }
  auto issue = [&](int jt) {  // stage of this block's tile jt
    const int m0b = (blk + jt * nblk) * TM * ROW;
    unsigned char* st = smem + (jt % C::NS) * C::STAGE;
#pragma unroll
    for (int j = 0; j < C::ROUNDS; ++j) {
      const int q0 = j * NT + wave * 64;  // wave-uniform
      if (q0 < nch) {
        const int off = m0b + kb[j];
        glds16((unsigned)off < (unsigned)Mb ? a.x4 + off : zp, st + q0 * 16);
      }
    }
  };
#pragma unroll
  for (int j = 0; j < LA; ++j)
    if (j < n) issue(j);

  // per-lane constants of the fragment reads: chunk 2 kc + h of tap (th, tw)
  // of pixel 64 wave + 32 u + r32 is stage row 64 wave + 32 u + (r32 + th W +
  // tw), at byte 64 ROW * wave + 32 ROW * u + lo[t][kc]
  int lo[9][KC];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int row = r32 + (t / 3) * a.W + t % 3;
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) lo[t][kc] = row * ROW + (((2 * kc + h) ^ C::swz(row)) << 4);
  }
  int wlo[KC];  // weight row 32 e + r32 (t * 64 + 32 e: the same swizzle)
#pragma unroll
  for (int kc = 0; kc < KC; ++kc) wlo[kc] = r32 * ROW + (((2 * kc + h) ^ C::swz(r32)) << 4);
  unsigned char* ys = smem + C::YOFF + wave * (32 * 128);  // this wave's output rows
  short* ybase = a.y ? a.y + slice * 64 : nullptr;

  f32x16 cs[2] = {}, cq[2] = {};
  long long tsum = 0;
  unsigned long long tsq = 0;
  const int ns = a.y ? 8 : 0;  // global stores per wave and tile
  BF_ST_BEGIN
  for (int it = 0; it < n; ++it) {
    // this tile's stage has landed
    bf_wait(bf_after<LA>(it, n, nd, ns));
    BF_ST(0)
    __syncthreads();
    BF_ST(1)
    // every wave is past tile it - 1, whose stage the DMA of tile it + LA reuses
    if (it + LA < n) issue(it + LA);
    const int m0 = (blk + it * nblk) * TM;
    const bool full = m0 + TM <= a.M;
    const int sb = (it % C::NS) * C::STAGE + wave * (64 * ROW);
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
    // ---- 9 taps x KC K-chunks x 2 channel halves x 2 pixel groups
    f32x16 acc[2][2];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int th = t / 3, tw = t % 3;
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) {
        uint4 wv[2];
#pragma unroll
        for (int e = 0; e < 2; ++e)
          wv[e] = *reinterpret_cast<const uint4*>(wl + (t * 64 + 32 * e) * ROW + wlo[kc]);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          bool ok = live[u];
          if (th == 0) ok = ok && top[u];
          if (th == 2) ok = ok && bot[u];
          if (tw == 0) ok = ok && lft[u];
          if (tw == 2) ok = ok && rgt[u];
          const int off = ok ? sb + u * (32 * ROW) + lo[t][kc] : C::PADOFF;
          const uint4 b = *reinterpret_cast<const uint4*>(smem + off);
#pragma unroll
          for (int e = 0; e < 2; ++e)
            acc[u][e] = mfma_fp4(wv[e], b, (t || kc) ? acc[u][e] : f32x16{});
        }
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
      // whole 128-B slice rows: instruction k stores pixels 8 k .. 8 k + 7 of
      // the group (lane l: pixel 8 k + l / 8, slot l % 8)
      const int mg = m0 + 64 * wave + 32 * u;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int p = 8 * k + (lane >> 3), sl = lane & 7;
        const uint4 v = *reinterpret_cast<const uint4*>(ys + p * 128 + ((sl ^ (p & 7)) << 4));
        if (ybase && mg + p < a.M)
          *reinterpret_cast<uint4*>(ybase + (long long)(mg + p) * a.Cout + sl * 8) = v;
      }
    }
    BF_ST(4)
    if ((it + 1) % C::FLUSH == 0) bf_flush(cs, cq, r32, tsum, tsq);
    BF_ST(5)
  }
  BF_ST_STORE
  bf_flush(cs, cq, r32, tsum, tsq);

  // ---- statistics: lane r32 of each half holds value r32 of the half
  const int e = r32 >> 4, r = r32 & 15;
  const int co = 32 * e + 8 * (r >> 2) + 4 * h + (r & 3);
  __syncthreads();
  long long* red = reinterpret_cast<long long*>(smem);  // [NW waves][2][64]
  red[(wave * 2 + 0) * 64 + co] = tsum;
  red[(wave * 2 + 1) * 64 + co] = (long long)tsq;
  __syncthreads();
  if (tid < 128) {
    const int which = tid / 64, c = tid % 64;
    long long tot = 0;
#pragma unroll
    for (int w = 0; w < C::NW; ++w) tot += red[(w * 2 + which) * 64 + c];
    const int stripe = a.stripes > 1 ? (int)(blockIdx.x % a.stripes) : 0;
    atomicAdd(a.stats + ((long long)stripe * 2 + which) * a.Cout + slice * 64 + c,
              (unsigned long long)tot);
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

template <class C>
int bf_launch(const BfArgs& a0, int relu, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    for (const void* f : {(const void*)bfwd_kernel<C, false>, (const void*)bfwd_kernel<C, true>}) {
      const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               C::LDS);
      if (e != hipSuccess) return (int)e;
    }
    attr = true;
  }
  BfArgs a = a0;
  a.ntiles = (a.M + C::TM - 1) / C::TM;
  // blocks per slice: the resident count split over the slices, at most one
  // per tile
  int bps = C::OCC * bf_cus() / a.nsl;
  if (bps < 1) bps = 1;
  if (bps > a.ntiles) bps = a.ntiles;
  const dim3 grid(bps * a.nsl);
  if (relu)
    hipLaunchKernelGGL((bfwd_kernel<C, true>), grid, dim3(C::NT), C::LDS, st, a);
  else
    hipLaunchKernelGGL((bfwd_kernel<C, false>), grid, dim3(C::NT), C::LDS, st, a);
  return 0;
}

}  // namespace

// Shape check of zk_bfwd_fp4: 3x3 stride 1 'same', Cin 64 (W <= 60) or 128
// (W <= 32; the stage holds TM + 2 W + 2 rows), Cout a multiple of 64 (one
// 64-channel slice per block), and the flattened pixel count inside the
// float-reciprocal division range (the statistics are exact at any size:
// fp32 below 2^24 between flushes, 32-bit lane reductions below 2^32, 64-bit
// totals).
ZK_EXPORT int zk_bfwd_supported(int B, int H, int W, int Cin, int Cout, int kh, int kw,
                                int stride, int pt, int pl) {
  const long long M = (long long)B * H * W;
  if (kh != 3 || kw != 3 || stride != 1 || pt != 1 || pl != 1) return 0;
  if (Cout <= 0 || Cout % 64 || Cout > 1024) return 0;
  if (M <= 0 || M >= (1LL << 24)) return 0;
  if (Cin == 64) return W <= Bf64::WMAX ? 1 : 0;
  if (Cin == 128) return W <= Bf128::WMAX ? 1 : 0;
  return 0;
}

// y int16 [B][H][W][Cout] = 3x3 'same' binary conv of the e2m1 sign image x4
// [B][H][W][Cin/2 B] with the e2m1 weights w4 [9][Cout][Cin/2 B] (+ReLU),
// padding +1 (pad_ones) or 0; stats [stripes][2][Cout] int64 += per-channel
// sum and sum of squares of y (block b adds into copy b % stripes).  y null:
// statistics only.
ZK_EXPORT int zk_bfwd_fp4(const void* x4, const void* w4, void* y, void* stats, int B, int H,
                          int W, int Cin, int Cout, int pad_ones, int relu, int stripes,
                          hipStream_t st) {
  if (!zk_bfwd_supported(B, H, W, Cin, Cout, 3, 3, 1, 1, 1)) return (int)hipErrorInvalidValue;
  BfArgs a{};
  a.x4 = (const unsigned char*)x4;
  a.w4 = (const unsigned char*)w4;
  a.y = (short*)y;
  a.stats = (unsigned long long*)stats;
  a.M = B * H * W;
  a.H = H;
  a.W = W;
  a.Cout = Cout;
  a.nsl = Cout / 64;
  a.stripes = stripes;
  a.pad_ones = pad_ones;
  a.inv_w = 1.f / (float)W;
  a.inv_h = 1.f / (float)H;
  const int rc = Cin == 64 ? bf_launch<Bf64>(a, relu, st) : bf_launch<Bf128>(a, relu, st);
  if (rc) return rc;
  ZK_CHECK_LAUNCH();
  return 0;
}
