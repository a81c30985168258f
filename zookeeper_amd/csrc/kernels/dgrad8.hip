// Persistent, phase-pipelined data gradient of 3x3 / kxk stride-1 binary
// convolutions (and the float 'same' convs that reuse it): the 256-pixel tile
// implicit GEMM of igemm.hip rebuilt on the 16x16x32 MFMA core measured in
// tools/gemm_lab/g8.hip.
//
//   D[ci][pixel] = sum_{tap t, co} S^T[t][ci][co] * dY[pixel - shift(t)][co]
//   dx = D * STE-mask(x) + dres   (bf16; mask / dres optional)
//
// Why a new kernel (profiles/r3/b_gemm_roofline_b1024_baseline.md, PMC in
// profiles/r3/): the round-2 kernels ran one tile per block with one barrier
// per K-step and vmcnt(0) at every step (2-stage rings), so each block paid
// the DMA latency at every step and once more for its epilogue; on the
// short-K 64 / 128-channel layers (K = 576 / 1152) the waves spent ~65 % of
// their lifetime waiting (SQ_WAIT_ANY + SQ_WAIT_INST_ANY) and MFMA sat at
// ~21 % busy.  Here:
//
//   * persistent blocks (grid = CUs x blocks/CU) walk their tiles and the
//     LDS-DMA ring never drains between tiles: the next tile's first
//     half-tiles are in flight while the current tile's epilogue runs;
//   * a K "half-tile" is 32 output channels of one tap: an A piece (BCI
//     weight rows x 64 B) and a B piece (256 gathered dY pixel rows x 64 B);
//     a ring of 4 half-tile slots, half-tile h + 3 issued right after the
//     barrier of half-tile h, so every piece has two half-tiles of MFMA work
//     to land (counted vmcnt, raw s_barrier: the ring stays in flight across
//     barriers);
//   * LDS rows of 64 B with the 16-B chunk swizzle {0,2,3,1}[(r>>2)&3]:
//     conflict-free ds_read_b128 for the 16x16x32 operand map;
//   * fragments double-buffered in registers: the next half-tile's (or
//     sub-phase's) fragments are read while this one's MFMAs issue;
//   * the product is D[ci][pixel]: a lane owns one pixel and 4 consecutive
//     input channels per register group -> 8-B mask-bit / residual / dx
//     epilogue accesses.
//
// Tiles: BCI input channels x 256 pixels, 8 waves (WM x WN).  NPH = 2 splits
// each half-tile's MFMAs over two sub-phases (halves of the wave's channel
// rows) so only half of the A fragments are live (the 256-channel tile's 128
// accumulator registers leave no room for a second full set).
#include "mfma_common.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma16(const uint4& a, const uint4& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// chunk swizzle of row r (within its 16-row block) for 64-B LDS rows
__device__ __forceinline__ int swz64(int r) { return (0x1320 >> (4 * ((r >> 2) & 3))) & 3; }

__device__ __forceinline__ void sbarrier() { asm volatile("s_barrier" ::: "memory"); }

__device__ __forceinline__ uint4 lds16(const unsigned char* p) {
  return *reinterpret_cast<const uint4*>(p);
}

struct D8Args {
  const uint16_t* dy;    // [B][Ho][Wo][Cout] bf16
  const uint16_t* wt;    // [T][Cin][Cout] bf16 (+-1)
  const uint32_t* mask;  // [B][H][W][Cin/32] STE mask bits of x (optional)
  const uint16_t* dres;  // [B][H][W][Cin] residual gradient (optional)
  uint16_t* dx;          // [B][H][W][Cin]
  int B, H, W, Cin, Ho, Wo, Cout, kh, kw, pt, pl;
  int n_tiles, tiles;    // channel tiles per pixel tile, total tiles
};

constexpr int BPX = 256;  // pixels per tile

template <int BCI, int WM, int WN, int NPH, int MINB, bool PP = false>
__global__ __launch_bounds__(512, MINB) void dgrad8_kernel(D8Args a) {
  static_assert(WM * WN == 8, "8 waves");
  constexpr int WTM = BCI / WM;          // channel rows per wave
  constexpr int WTN = BPX / WN;          // pixels per wave
  constexpr int FAT = WTM / 16;          // A fragments per half-tile
  constexpr int FA = FAT / NPH;          // ... per sub-phase
  constexpr int FB = WTN / 16;           // B fragments per half-tile
  static_assert(FA >= 1 && FB >= 1 && FAT % NPH == 0, "wave tile");
  constexpr int APIECE = BCI * 64, BPIECE = BPX * 64, SLOT = APIECE + BPIECE;
  constexpr int AROWI = BCI / 16;        // A load instructions per half-tile (all waves)
  constexpr int NA = (AROWI + 7) / 8;    // per wave (small tiles: duplicated rows)
  constexpr int NB = BPX / 16 / 8;       // B load instructions per wave
  constexpr int LPH = NA + NB;           // DMAs per wave per half-tile

  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave / WN, wn = wave % WN;
  const int lrow = lane >> 2;                  // row within a 16-row load block
  const int gch = (lane & 3) ^ swz64(lrow);    // global 16-B chunk this lane loads
  const int foff = (lane & 15) * 64 + (((lane >> 4) ^ swz64(lane & 15)) << 4);

  const int grid = gridDim.x;
  const int lb = xcd_linear(blockIdx.x, grid);
  if (lb >= a.tiles) return;
  const int my_tiles = (a.tiles - lb + grid - 1) / grid;
  const int KC2 = a.Cout >> 5;                 // 32-channel chunks per tap
  const int T = a.kh * a.kw;
  const int NH = T * KC2;                      // half-tiles per tile (even: Cout % 64 == 0)
  const int Htot = my_tiles * NH;
  const long long M = (long long)a.B * a.H * a.W;
  const int RB = a.Cout * 2;                   // bytes per dY row
  const unsigned char* dyb = reinterpret_cast<const unsigned char*>(a.dy);
  const unsigned char* wtb = reinterpret_cast<const unsigned char*>(a.wt);
  const unsigned char* zp = reinterpret_cast<const unsigned char*>(g_zero_page) + gch * 16;

  // ---- issue side: loader state of the tile being issued
  int issue_k = -1;
  long long b_base[NB];   // dY byte offset of (pixel, tap 0, chunk gch); < 0: no pixel
  uint32_t b_hm[NB], b_wm[NB];
  int a_n0 = 0;
  auto setup_tile = [&](int k) {
    const int tile = lb + k * grid;
    const int mt = tile / a.n_tiles, ct = tile % a.n_tiles;
    a_n0 = ct * BCI;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const long long m = (long long)mt * BPX + (i * 8 + wave) * 16 + lrow;
      b_base[i] = -1;
      b_hm[i] = b_wm[i] = 0;
      if (m < M) {
        const int wi = (int)(m % a.W);
        const long long q = m / a.W;
        const int hi = (int)(q % a.H), b = (int)(q / a.H);
        const int ho0 = hi + a.pt, wo0 = wi + a.pl;  // dY pixel of tap (0, 0)
        for (int t = 0; t < a.kh; ++t) b_hm[i] |= (uint32_t)(ho0 - t >= 0 && ho0 - t < a.Ho) << t;
        for (int t = 0; t < a.kw; ++t) b_wm[i] |= (uint32_t)(wo0 - t >= 0 && wo0 - t < a.Wo) << t;
        b_base[i] = (((long long)b * a.Ho + ho0) * a.Wo + wo0) * RB + gch * 16;
      }
    }
  };
  auto issue = [&](int h) {  // half-tile h (global over this block's tiles) -> slot h & 3
    const int k = h / NH, j = h - k * NH;
    if (k != issue_k) {
      setup_tile(k);
      issue_k = k;
    }
    const int t = j / KC2, kc = j - t * KC2;
    const int th = t / a.kw, tw = t - th * a.kw;
    unsigned char* slot = smem + (h & 3) * SLOT;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int blk = (i * 8 + wave) % AROWI;
      const int ci = a_n0 + blk * 16 + lrow;
      glds16(wtb + ((long long)(t * a.Cin + ci) * a.Cout) * 2 + kc * 64 + gch * 16,
             slot + blk * 1024);
    }
    const long long toff = ((long long)th * a.Wo + tw) * RB - kc * 64;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const bool ok = b_base[i] >= 0 && ((b_hm[i] >> th) & (b_wm[i] >> tw) & 1u);
      glds16(ok ? dyb + (b_base[i] - toff) : zp, slot + APIECE + (i * 8 + wave) * 1024);
    }
  };

  // ---- compute side
  f32x4 acc[FAT][FB];
#pragma unroll
  for (int i = 0; i < FAT; ++i)
#pragma unroll
    for (int j = 0; j < FB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto rdA = [&](uint4 (&dst)[FA], int h, int q) {
    const unsigned char* base = smem + (h & 3) * SLOT + (wm * WTM + q * FA * 16) * 64 + foff;
#pragma unroll
    for (int f = 0; f < FA; ++f) dst[f] = lds16(base + f * 1024);
  };
  auto rdB = [&](uint4 (&dst)[FB], int h) {
    const unsigned char* base = smem + (h & 3) * SLOT + APIECE + (wn * WTN) * 64 + foff;
#pragma unroll
    for (int f = 0; f < FB; ++f) dst[f] = lds16(base + f * 1024);
  };
  auto mma = [&](const uint4 (&af)[FA], const uint4 (&bf)[FB], int q) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int f = 0; f < FA; ++f)
#pragma unroll
      for (int g = 0; g < FB; ++g)
        acc[q * FA + f][g] = mfma16(af[f], bf[g], acc[q * FA + f][g]);
    __builtin_amdgcn_s_setprio(0);
  };
  // wait until half-tile h has landed (pieces issued after it: h+1, and h+2
  // when it exists -- h+2 is issued after this wait in the same phase)
  auto wait_landed = [&](int h) {
    if (h + 1 < Htot)
      wait_vmcnt<LPH>();
    else
      wait_vmcnt<0>();
  };

  auto epilogue = [&](int k) {
    const int tile = lb + k * grid;
    const int mt = tile / a.n_tiles, ct = tile % a.n_tiles;
    const int n0 = ct * BCI + wm * WTM;
    const int CW = a.Cin >> 5;
#pragma unroll
    for (int g = 0; g < FB; ++g) {
      const long long m = (long long)mt * BPX + wn * WTN + g * 16 + (lane & 15);
      if (m >= M) continue;
      uint32_t mw[FAT];
      uint2 dv[FAT];
#pragma unroll
      for (int f = 0; f < FAT; ++f) {
        const int ci = n0 + f * 16 + 4 * (lane >> 4);
        mw[f] = a.mask ? a.mask[m * CW + (ci >> 5)] >> (ci & 31) : 0xFu;
        dv[f] = a.dres ? *reinterpret_cast<const uint2*>(a.dres + m * a.Cin + ci)
                       : make_uint2(0u, 0u);
      }
#pragma unroll
      for (int f = 0; f < FAT; ++f) {
        const int ci = n0 + f * 16 + 4 * (lane >> 4);
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = ((mw[f] >> r) & 1u) ? acc[f][g][r] : 0.f;
        v[0] += zk::bf16_to_f32((uint16_t)(dv[f].x & 0xffff));
        v[1] += zk::bf16_to_f32((uint16_t)(dv[f].x >> 16));
        v[2] += zk::bf16_to_f32((uint16_t)(dv[f].y & 0xffff));
        v[3] += zk::bf16_to_f32((uint16_t)(dv[f].y >> 16));
        *reinterpret_cast<uint2*>(a.dx + m * a.Cin + ci) =
            make_uint2(zk::pack_bf16x2(v[0], v[1]), zk::pack_bf16x2(v[2], v[3]));
      }
    }
#pragma unroll
    for (int i = 0; i < FAT; ++i)
#pragma unroll
      for (int j = 0; j < FB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };

  if constexpr (PP) {
    // Ping-pong schedule (NPH = 2): waves 0-3 and 4-7 are two groups, one
    // wave of each per SIMD; group 1 runs one s_barrier behind group 0, so
    // one group's 16-MFMA cluster issues while the other group's wave on the
    // same SIMD reads its fragments and issues its DMA (the lab's V3:
    // 1.23 PF/s at 4096^3 vs 1.05-1.15 for the register-double-buffered
    // forms).  Phase (h, q): reads its own fragments (A rows half q; B at
    // q = 0, kept for q = 1), issues the A (q = 0) or B (q = 1) piece of
    // half-tile h + 2, s_barrier, lgkmcnt(0), MFMAs, s_barrier.  Half-tile
    // h + 1 is retired by a counted vmcnt at the start of phase (h, 1): one
    // phase before its first reads (the groups are a barrier apart).
    static_assert(NPH == 2, "ping-pong: two sub-phases per half-tile");
    const int grp = __builtin_amdgcn_readfirstlane(wave >> 2);
    uint4 af[FA], bf[FB];
    auto issueA = [&](int h) {
      const int k = h / NH, j = h - k * NH;
      if (k != issue_k) {
        setup_tile(k);
        issue_k = k;
      }
      const int t = j / KC2, kc = j - t * KC2;
      unsigned char* slot = smem + (h & 3) * SLOT;
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int blk = (i * 8 + wave) % AROWI;
        const int ci = a_n0 + blk * 16 + lrow;
        glds16(wtb + ((long long)(t * a.Cin + ci) * a.Cout) * 2 + kc * 64 + gch * 16,
               slot + blk * 1024);
      }
    };
    auto issueB = [&](int h) {  // after issueA(h): the loader state is h's tile
      const int k = h / NH, j = h - k * NH;
      const int t = j / KC2, kc = j - t * KC2;
      const int th = t / a.kw, tw = t - th * a.kw;
      unsigned char* slot = smem + (h & 3) * SLOT;
      const long long toff = ((long long)th * a.Wo + tw) * RB - kc * 64;
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const bool ok = b_base[i] >= 0 && ((b_hm[i] >> th) & (b_wm[i] >> tw) & 1u);
        glds16(ok ? dyb + (b_base[i] - toff) : zp, slot + APIECE + (i * 8 + wave) * 1024);
      }
      (void)k;
    };
    // prologue: half-tiles 0 and 1 issued and landed; group 1 one barrier behind
    issueA(0);
    issueB(0);
    if (Htot > 1) {
      issueA(1);
      issueB(1);
    }
    wait_vmcnt<0>();
    sbarrier();
    if (grp == 1) sbarrier();
    for (int h = 0; h < Htot; ++h) {
      // ---- phase (h, 0)
      rdA(af, h, 0);
      rdB(bf, h);
      if (h + 2 < Htot) issueA(h + 2);
      sbarrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      mma(af, bf, 0);
      __builtin_amdgcn_sched_barrier(0);
      sbarrier();
      // ---- phase (h, 1): retire half-tile h+1 first (read from phase (h+1, 0))
      if (h + 2 < Htot)
        wait_vmcnt<NA>();  // A_{h+2} stays in flight
      else
        wait_vmcnt<0>();
      rdA(af, h, 1);
      if (h + 2 < Htot) issueB(h + 2);
      sbarrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      mma(af, bf, 1);
      __builtin_amdgcn_sched_barrier(0);
      sbarrier();
      if ((h + 1) % NH == 0) epilogue(h / NH);
    }
    if (grp == 0) sbarrier();  // equal barrier counts in both groups
    return;
  }

  // fragment registers: two B sets (alternating half-tiles), A sets per
  // sub-phase (NPH = 1: two sets alternating half-tiles; NPH = 2: the
  // current sub-phase's and the next one's)
  uint4 aX[FA], aY[FA], bX[FB], bY[FB];

  // prologue: half-tiles 0, 1, 2 in flight; half-tile 0 landed
  issue(0);
  if (Htot > 1) issue(1);
  if (Htot > 2) issue(2);
  if (Htot > 2)
    wait_vmcnt<2 * LPH>();
  else if (Htot > 1)
    wait_vmcnt<LPH>();
  else
    wait_vmcnt<0>();
  sbarrier();
  rdA(aX, 0, 0);
  rdB(bX, 0);

  // Two half-tiles per iteration (Htot is even), register sets static.
  for (int h = 0; h < Htot; h += 2) {
    if constexpr (NPH == 1) {
      // ---- half-tile h: MFMA on (aX, bX); read h+1 into (aY, bY)
      wait_landed(h + 1);
      sbarrier();
      if (h + 3 < Htot) issue(h + 3);
      rdA(aY, h + 1, 0);
      rdB(bY, h + 1);
      __builtin_amdgcn_sched_barrier(0);
      mma(aX, bX, 0);
      __builtin_amdgcn_sched_barrier(0);
      // ---- half-tile h+1: MFMA on (aY, bY); read h+2 into (aX, bX)
      if (h + 2 < Htot) {
        wait_landed(h + 2);
        sbarrier();
        if (h + 4 < Htot) issue(h + 4);
        rdA(aX, h + 2, 0);
        rdB(bX, h + 2);
      }
      __builtin_amdgcn_sched_barrier(0);
      mma(aY, bY, 0);
      __builtin_amdgcn_sched_barrier(0);
    } else {
      // ---- half-tile h (B = bX): sub-phase 0 (aX), sub-phase 1 (aY)
      rdA(aY, h, 1);
      __builtin_amdgcn_sched_barrier(0);
      mma(aX, bX, 0);
      __builtin_amdgcn_sched_barrier(0);
      wait_landed(h + 1);
      sbarrier();
      if (h + 3 < Htot) issue(h + 3);
      rdA(aX, h + 1, 0);
      rdB(bY, h + 1);
      __builtin_amdgcn_sched_barrier(0);
      mma(aY, bX, 1);
      __builtin_amdgcn_sched_barrier(0);
      // ---- half-tile h+1 (B = bY)
      rdA(aY, h + 1, 1);
      __builtin_amdgcn_sched_barrier(0);
      mma(aX, bY, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (h + 2 < Htot) {
        wait_landed(h + 2);
        sbarrier();
        if (h + 4 < Htot) issue(h + 4);
        rdA(aX, h + 2, 0);
        rdB(bX, h + 2);
      }
      __builtin_amdgcn_sched_barrier(0);
      mma(aY, bY, 1);
      __builtin_amdgcn_sched_barrier(0);
    }
    if ((h + 2) % NH == 0) epilogue(h / NH);
  }
}

// Slot ring of 4 half-tiles.
template <int BCI>
constexpr int d8_lds() {
  return 4 * (BCI * 64 + BPX * 64);
}

template <int BCI, int WM, int WN, int NPH, int MINB, bool PP = false>
int d8_launch(const D8Args& args0, int num_cus, hipStream_t st, bool persistent = true) {
  D8Args args = args0;
  constexpr int LDS = d8_lds<BCI>();
  static_assert(LDS * MINB <= 160 * 1024, "LDS");
  auto kern = dgrad8_kernel<BCI, WM, WN, NPH, MINB, PP>;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)kern,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  const long long M = (long long)args.B * args.H * args.W;
  const long long m_tiles = (M + BPX - 1) / BPX;
  args.n_tiles = args.Cin / BCI;
  const long long tiles = m_tiles * args.n_tiles;
  if (tiles >= (1LL << 31)) return (int)hipErrorInvalidValue;
  args.tiles = (int)tiles;
  long long grid = persistent ? (long long)num_cus * MINB : tiles;
  if (grid > tiles) grid = tiles;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(512), LDS, st, args);
  return 0;
}

int g_num_cus = 0;

}  // namespace

// Stride-1 data gradient on the persistent phased core (igemm.hip's variant
// 60+ dispatch).  Requirements: stride 1, Cout % 64 == 0, Cin % BCI == 0,
// kh, kw <= 4.  variant: 60 = 64-channel tiles, 61 = 128, 62 = 256.
// dry: validate only.
int zk_dgrad8_impl(const void* dy, const void* wt, const void* mask, const void* dres, void* dx,
                   int B, int H, int W, int Cin, int Ho, int Wo, int Cout, int kh, int kw,
                   int stride, int pt, int pl, int variant, bool dry, hipStream_t st) {
  const int bci = variant == 60 ? 64 : variant == 61 ? 128 : (variant >= 62 && variant <= 65) ? 256 : 0;
  if (!bci || stride != 1 || Cout % 64 || Cin % bci || kh > 4 || kw > 4 ||
      (long long)B * Ho * Wo * Cout >= (1LL << 40))
    return (int)hipErrorInvalidValue;
  if (dry) return 0;
  if (g_num_cus == 0) {
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, dev) != hipSuccess) return (int)hipErrorInvalidDevice;
    g_num_cus = p.multiProcessorCount;
  }
  D8Args a{(const uint16_t*)dy, (const uint16_t*)wt, (const uint32_t*)mask, (const uint16_t*)dres,
           (uint16_t*)dx, B, H, W, Cin, Ho, Wo, Cout, kh, kw, pt, pl, 0, 0};
  switch (variant) {
    case 60: return d8_launch<64, 1, 8, 1, 2>(a, g_num_cus, st);
    case 61: return d8_launch<128, 1, 8, 1, 1>(a, g_num_cus, st);
    case 62: return d8_launch<256, 2, 4, 2, 1>(a, g_num_cus, st);
    case 63: return d8_launch<256, 2, 4, 2, 1, true>(a, g_num_cus, st);
    // one tile per block (no persistence): A/B of the schedules
    case 64: return d8_launch<256, 2, 4, 2, 1, true>(a, g_num_cus, st, false);
    case 65: return d8_launch<256, 2, 4, 2, 1>(a, g_num_cus, st, false);
    default: return (int)hipErrorInvalidValue;
  }
}
