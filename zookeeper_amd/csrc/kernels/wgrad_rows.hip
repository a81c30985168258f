// Row-streaming weight gradient of a 3x3 stride-1 'same' convolution
// (64 / 128-channel stages of BinaryResNet-E18, QuickNet, ResNet-50):
//
//   dW[co][kh][kw][ci] += mask(|w| <= clip) *
//       sum_{n,h,w} dY[n][h][w][co] * S[n][h+kh-1][w+kw-1][ci]
//
// S is the bf16 +-1 sign image, or (SIGN) the bf16 activation x itself, whose
// sign is taken in registers after the LDS read (one v_and_or per bf16 pair:
// +-1.0 from the sign bit; producers never store -0, zero -> +1 as larq's
// ste_sign).  With SIGN the padding is +1 (pad_values=1, the BinaryResNet /
// QuickNet convolutions): the zero page becomes +1 like any zero.
//
// Why a new schedule: the conv3 tile kernel (igemm.hip,
// variant 20) re-loads each S pixel row for every kernel row and keeps only
// ~2 small K-steps in flight per CU: at batch 1536 its stage-1 call ran at
// 1.4 TB/s and 5 % MFMA busy (profiles/r4/i_e18_b1536_pmc.md).
//
// Design:
//   * a block owns one 64(co) x 64(ci) x 9-tap tile and a contiguous range of
//     "steps"; a step is R image rows of one image (R * W = 112 pixels = 7
//     MFMA K-steps of 16).  Per step, LDS-DMA (global_load_lds_dwordx4, 16 B
//     per lane, per-lane gathered sources) stages the step's dY rows and the
//     S window: R + 2 rows (one halo row above and below) of W + 2 pixels
//     (one halo column each side); halo pixels and the rows above / below the
//     image come from the padding page.  Three slots, two steps in flight
//     across each step's raw s_barrier, counted vmcnt.
//   * LDS images are "planes" of 32 channels: [plane][pixel][32 ch], 64 B per
//     pixel.  A transposed fragment read (ds_read_b64_tr_b16) of 4 consecutive
//     pixels then covers the 4 quarters of a 256-B bank row: conflict-free
//     without a swizzle -- so tap (kh, kw) of S is the fragment at the
//     window's (row + kh, column + kw): base + kh * row_bytes + kw * 64, an
//     immediate offset.  A K-step costs 2 address adds per lane instead of a
//     gathered address per tap (the first version of this kernel was
//     VALU-issue-bound on exactly that: ~12 VALU per MFMA; one wave per SIMD
//     hides ~5 beside a 32-cycle MFMA, MI355X_MICROARCH.md issue costs).
//   * 4 waves, each 32(co) x 32(ci) x 9 taps: one dY fragment feeds 9 MFMAs
//     (v_mfma_f32_32x32x16_bf16); K-step kk + 1's fragments are read while
//     kk's MFMAs run.
//   * split-K over steps; the per-block partial tiles are combined INSIDE the
//     launch by a fixed-order tree (groups of 8, the last-arriving block of a
//     group sums its children in index order; agent-scope release / acquire,
//     cdna_hip_programming.md "In-launch split-K reduction") -- no reduce
//     launch, bit-reproducible whatever the arrival order.  The root applies
//     the kernel STE mask and adds into dW (the flat fp32 gradient buffer).
//
// Reference: the QuantConv2D stack whose weight gradients these are
// (/root/reference/examples/larq_experiment.py:62-99).
#include <climits>

#include "mfma_common.h"

// The in-launch tree's fence-free publish (relaxed agent-scope stores,
// vmcnt(0), relaxed counter atomic, sc1 loads without an acquire) relies on
// gfx950's sc1 write-through behaviour: refuse other targets.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "wgrad_rows.hip: the fence-free split-K publish protocol is specific to gfx950"
#endif

namespace {

constexpr int WR_NT = 256;     // 4 waves
constexpr int WR_G = 8;        // tree fan-in
constexpr int WR_MAXLV = 8;
constexpr int WR_RW = 112;     // pixels per step
constexpr int WR_NK = WR_RW / 16;
constexpr int WR_NSLOT = 3;
constexpr int WR_SC1 = 16;     // buffer-op cache policy: sc1 (agent-coherent)

// Operand modes of S: the bf16 image (OP_IMG: a +-1 sign image, or a float
// activation), the bf16 activation whose sign is taken in registers
// (OP_SIGN), or the e2m1 (FP4) sign image the binary forward already reads
// (OP_FP4): staged at a quarter of the bytes and expanded in LDS
// (v_cvt_scalef32_pk_bf16_fp4, one instruction per bf16 pair) one step ahead,
// so padding keeps its value (0 or +1) and the forward need not write a bf16
// sign image for these layers.
enum { OP_IMG = 0, OP_SIGN = 1, OP_FP4 = 2 };

// Window rows are padded to whole KB in LDS (RB, R4B) so that every 1-KB
// LDS-DMA piece lies in one window row: a piece's source row, and whether it
// is a padding row above / below the image, are wave-uniform (scalar
// selects); per lane only the static halo / row-padding lanes differ (one
// select): ~3 VALU per DMA piece instead of ~15.
template <int W, int OP>
struct WrGeo {
  static constexpr int R = WR_RW / W;           // image rows per step
  static constexpr int PW = W + 2;              // S window row (pixels, with the halo)
  static constexpr int RB = (PW * 64 + 1023) / 1024 * 1024;  // bf16 row pitch, one plane
  static constexpr int SPLANE = (R + 2) * RB;   // window rows h0-1 .. h0+R
  static constexpr int SBYTES = 2 * SPLANE;     // bf16 window, 2 planes of 32 channels
  static constexpr int R4B = (PW * 32 + 1023) / 1024 * 1024;  // e2m1 row pitch (32 B / pixel)
  static constexpr int S4BYTES = (R + 2) * R4B;
  static constexpr int DPLANE = WR_RW * 64;
  static constexpr int DBYTES = 2 * DPLANE;     // 14 KB of dY ...
  static constexpr int SOFF = 16 * 1024;        // ... in a 16-KB region: the S window at 16 KB
  // staged per step: dY + the S window (bf16, or e2m1 for OP_FP4), in 4-KB
  // units: a slot is 4 KB x NI, and DMA instruction k of every wave covers
  // bytes [4k, 4k + 4) KB (1 KB per wave): k < KD dY, then KS window units
  static constexpr int STAGED = ((OP == OP_FP4 ? S4BYTES : SBYTES) + 4095) / 4096 * 4096;
  static constexpr int SROW = OP == OP_FP4 ? R4B : RB;  // staged row pitch
  static constexpr int RBK = SROW / 1024;       // DMA pieces per staged row (1, 2, 4)
  static constexpr int KD = SOFF / 4096, KS = STAGED / 4096;
  static constexpr int TOT = 4 * (KD + KS);     // DMA pieces (1 KB)
  static constexpr int NI = TOT / 4;            // DMA pieces per wave per step
  static constexpr int SLOT = TOT * 1024;
  // OP_FP4: two expanded bf16 windows after the slots (step j's, step j+1's)
  static constexpr int SBF = WR_NSLOT * SLOT;
  static constexpr int FLAG = SBF + (OP == OP_FP4 ? 2 * SBYTES : 0);  // arrival word
  static constexpr int LDS = FLAG + 16;
  // OP_FP4 expansion: 16-B bf16 chunks of the real window pixels
  static constexpr int CPR = PW * 4;            // chunks per row of one plane
  static constexpr int CHUNKS = 2 * (R + 2) * CPR;
  static_assert(WR_RW % W == 0 && LDS <= 160 * 1024 && DBYTES <= SOFF && 4 % RBK == 0,
                "row-stream geometry");
};

// Rows above / below the image: DMA'd from these (zero, bf16 +1, e2m1 +1
// pairs), one image row of up to WR_MAXCIN channels long.  Filled once by
// wr_pad_init_kernel.
constexpr int WR_MAXCIN = 256;
constexpr int WR_PADROW = 56 * WR_MAXCIN * 2;
__device__ __attribute__((aligned(1024))) uint32_t g_wr_pad[3][WR_PADROW / 4];

__global__ void wr_pad_init_kernel() {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < WR_PADROW / 4) {
    g_wr_pad[0][i] = 0u;
    g_wr_pad[1][i] = 0x3F803F80u;
    g_wr_pad[2][i] = 0x22222222u;
  }
}

struct WrArgs {
  const uint16_t* dy;  // [B][H][W][Cout] bf16
  const uint16_t* sx;  // [B][H][W][Cin] bf16 (OP_IMG / OP_SIGN) or [B][H][W][Cin/2] e2m1 (OP_FP4)
  const float* w;      // [Cout][9][Cin] latent weights (kernel STE mask), or null
  float* dw;           // [Cout][9][Cin] fp32, accumulated
  float* slab;         // tree levels 0 .. levels-1, full-dW layout per node
  int* cnt;            // arrival counters (zero before the first launch; self-resetting)
  int B, H, W, Cin, Cout;
  int nsteps, sps, splits;
  int co_tiles, ci_tiles;
  int pad_ones;
  float clip;
  int levels;
  int nodes[WR_MAXLV];
  long long slab_off[WR_MAXLV];  // floats
  int cnt_off[WR_MAXLV];
  long long* dbg;      // LAB 7: per-wave cycle totals (wait + barrier, issue, compute)
};

__device__ __forceinline__ __attribute__((address_space(3))) s16x4* lds_s16x4(
    const unsigned char* smem, int off) {
  return (__attribute__((address_space(3))) s16x4*)(uintptr_t)(
      const __attribute__((address_space(3))) void*)(smem + off);
}

// global_load_lds_dwordx4 into LDS byte address lds (wave-uniform: M0)
__device__ __forceinline__ void glds16_at(const void* src, unsigned lds) {
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(lds) : "m0");
}

// 8 k-values of one column from two per-lane LDS addresses (rows q and q + 4
// of the lane's 4-row group, as tr_frag_swz)
__device__ __forceinline__ uint4 tr_read2(const unsigned char* smem, int o0, int o1) {
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(lds_s16x4(smem, o0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(lds_s16x4(smem, o1));
  const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(uint4, v);
}

// +-1.0 bf16 pair from the sign bits of a bf16 pair: one v_and_or_b32 with the
// +1.0 pair held in a VGPR (`ones`, opaque to the compiler so it does not fold
// the select back into an and + or with two literals)
__device__ __forceinline__ uint32_t sign_bf16x2(uint32_t v, uint32_t ones) {
  return (v & 0x80008000u) | (ones & 0x7FFF7FFFu);
}

// Unit schedules of the main loop (a unit = one S fragment: K-step kk, tap t)
// of the two pair members M 0 / 1: taps 0-3 / 5-8 of every K-step, tap 4 of
// K-steps 0-3 / 4-6: 32 / 31 units.
__host__ __device__ constexpr int wr_units(int m) { return m == 0 ? 32 : 31; }
// (closed forms, so unrolled loops fold them to constants: M 0 has 5 units
// per K-step below kk 4 and 4 above, M 1 the reverse)
__host__ __device__ constexpr int wr_unit_kk(int m, int n) {
  return m == 0 ? (n < 20 ? n / 5 : 4 + (n - 20) / 4) : (n < 16 ? n / 4 : 4 + (n - 16) / 5);
}
__host__ __device__ constexpr int wr_unit_tap(int m, int n) {
  return m == 0 ? (n < 20 ? n % 5 : (n - 20) % 4)
                : (n < 16 ? 5 + n % 4 : ((n - 16) % 5 == 4 ? 4 : 5 + (n - 16) % 5));
}
// accumulator slot of tap t, and back (M 1 keeps tap 4 in slot 0)
__host__ __device__ constexpr int wr_tap_slot(int m, int t) {
  return m == 1 ? (t == 4 ? 0 : t - 4) : t;
}
__host__ __device__ constexpr int wr_slot_tap(int m, int s) {
  return m == 1 ? (s == 0 ? 4 : s + 4) : s;
}
static_assert(wr_unit_kk(0, 31) == 6 && wr_unit_tap(0, 31) == 3 && wr_unit_tap(0, 4) == 4 &&
                  wr_unit_kk(1, 30) == 6 && wr_unit_tap(1, 30) == 4 && wr_unit_tap(1, 3) == 8 &&
                  wr_unit_kk(1, 4) == 1,
              "unit schedule");

// LAB: ablation builds for tools/wgrad_lab.py (0 = the kernel; 1 loads only,
// 2 compute only, 3 compute only without MFMAs, 4 compute only without the S
// fragment reads; results are garbage in 1-4)
// FD: how many MFMAs ahead each S fragment is read (one wave per SIMD: only
// this lookahead hides the LDS latency)
// A wave's tile is 64 (co) x 32 (ci); the two waves of a ci half split the
// step's 63 (K-step, tap) units by taps (wr_unit_*), so each S fragment read
// feeds both co halves; their tap-4 partials are combined through LDS.
// (Measured against 32 x 32 x 9-tap wave tiles: stage 1 sign operand 417 vs
// 491 us; profiles/r5/removed_variants.md.)
template <int W, int OP, int LAB = 0, int FD0 = 0>
__global__ __launch_bounds__(WR_NT, 1) void wgrad_rows_kernel(WrArgs a) {
  // lookahead: 5 units (10 S + up to 4 dY reads in flight, under the 15
  // lgkmcnt can count)
  constexpr int FD = FD0 > 0 ? FD0 : 5;
  using G = WrGeo<W, OP>;
  constexpr int R = G::R, PW = G::PW, RB = G::RB, NI = G::NI;
  constexpr bool FP4 = OP == OP_FP4, SIGN = OP == OP_SIGN;
  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wn = wave & 1;
  const int tiles = a.co_tiles * a.ci_tiles;
  const int L = xcd_linear(blockIdx.x, gridDim.x);
  const int split = L / tiles, tile = L % tiles;
  const int co0 = (tile % a.co_tiles) * 64, ci0 = (tile / a.co_tiles) * 64;
  const int j0 = split * a.sps;
  const int j1 = min(a.nsteps, j0 + a.sps);
  const int H = a.H;

  const unsigned char* dyb = reinterpret_cast<const unsigned char*>(a.dy);
  const unsigned char* sxb = reinterpret_cast<const unsigned char*>(a.sx);
  // padding rows (and pixel) source: zeros, or +1 (bf16 / e2m1) with pad_ones
  // (OP_SIGN: zeros, whose sign is +1)
  const int padk = !a.pad_ones || SIGN ? 0 : (FP4 ? 2 : 1);
  const unsigned char* padp = reinterpret_cast<const unsigned char*>(g_wr_pad[padk]);
  constexpr bool do_load = LAB < 2 || LAB > 4, do_mma = LAB != 1;
  // the next step's LDS-DMA pieces spread over the MFMA units (LAB 8: all
  // issued at the top of the step, before the first MFMA)
  constexpr bool spread = LAB != 8;
  constexpr bool lab_reads = LAB != 4, lab_mfma = LAB != 3;

  // LDS-DMA pieces: piece t = k * 4 + wave covers slot bytes [t KB, t KB +
  // 1 KB).  k < KD: dY; then window units: staged window row r(k, wave) =
  // (k - KD) * 4 / RBK + wave / RBK -- compile-time but for a wave-uniform
  // term.  Per lane, loff[k] = its source offset from the step's first dY
  // pixel / first S row (the row offset folded in), or WR_HALO for a lane
  // that reads the pad page (halo pixel, row padding).
  constexpr int WR_HALO = INT_MIN;
  int loff[NI];
  const long long srow = (long long)W * a.Cin * (FP4 ? 1 : 4) / 2;  // image row bytes
#pragma unroll
  for (int k = 0; k < NI; ++k) {
    const int b = (k * 4 + wave) * 1024 + lane * 16;
    loff[k] = WR_HALO;
    if (k < G::KD) {
      if (b < G::DBYTES) {
        const int plane = b / G::DPLANE, rem = b % G::DPLANE;
        const int p = rem >> 6, ch = (rem & 63) >> 4;
        loff[k] = (p * a.Cout + co0 + plane * 32 + ch * 8) * 2;
      } else {
        loff[k] = 0;  // the unused dY tail: any valid bytes
      }
    } else {
      const int bs = b - G::SOFF;
      int wr, col, choff;
      if constexpr (FP4) {  // [window row][pixel][32 B]: the tile's 64 channels as nibbles
        wr = bs / G::R4B;
        col = (bs % G::R4B) >> 5;
        choff = ci0 / 2 + ((bs & 31) >> 4) * 16;
      } else {  // [plane][window row][pixel][32 channels]
        const int plane = bs / G::SPLANE, rem = bs % G::SPLANE;
        wr = rem / RB;
        col = (rem % RB) >> 6;
        choff = (ci0 + plane * 32 + ((rem & 63) >> 4) * 8) * 2;
      }
      if (col >= 1 && col <= W && wr <= R + 1)
        loff[k] = (int)((wr - 1) * srow) + (col - 1) * (a.Cin * (FP4 ? 1 : 4) / 2) + choff;
    }
  }
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const long long dy_step = (long long)WR_RW * a.Cout * 2;
  const long long sx_step = (long long)WR_RW * a.Cin * (FP4 ? 1 : 4) / 2;
  // stage dY of step jd and the S window of step js into `slot` (OP_FP4
  // stages the window one step ahead: js = jd + 1).  The loop issues two
  // steps ahead unconditionally: steps out of range are clamped to real ones
  // (valid addresses; what they stage is never used).
  struct Stage {
    const unsigned char* dyp;  // the step's first dY pixel
    const unsigned char* sxp;  // the step's first S row
    bool top, bot;             // window row 0 / R + 1 is outside the image
    int dst;                   // LDS byte offset of this wave's piece 0
  };
  auto prep = [&](int jd, int js, int slot) -> Stage {
    Stage t;
    jd = min(max(jd, 0), a.nsteps - 1);
    js = min(max(js, 0), a.nsteps - 1);
    t.dyp = dyb + (long long)jd * dy_step;
    t.sxp = sxb + (long long)js * sx_step;
    const int h0 = (int)(((long long)js * R) % H);
    t.top = h0 == 0;
    t.bot = h0 + R == H;
    t.dst = slot * G::SLOT + wave_u * 1024;
    return t;
  };
  const unsigned lds0 = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)smem;
  auto piece = [&](const Stage& t, int k) {
    if constexpr (!do_load) return;
    const unsigned char* base;
    if (k < G::KD) {
      base = t.dyp;
    } else {
      // staged row of this piece (wave-uniform) and its window row
      const int r = (k - G::KD) * (4 / G::RBK) + wave_u / G::RBK;
      const int wr = FP4 ? r : r % (R + 2);
      // a padding row: the pad page, offset back by the row offset folded in loff
      const bool pad = (wr == 0 && t.top) || (wr == R + 1 && t.bot);
      base = pad ? padp - (wr - 1) * srow : t.sxp;
    }
    const unsigned char* src = loff[k] == WR_HALO ? padp : base + loff[k];
    glds16_at(src, lds0 + t.dst + k * 4096);
  };
  auto issue = [&](int jd, int js, int slot) {
    const Stage t = prep(jd, js, slot);
#pragma unroll
    for (int k = 0; k < NI; ++k) piece(t, k);
  };

  // OP_FP4: expand the e2m1 window staged in `slot` into bf16 window buffer
  // `buf`, chunk c (of CPT) of this thread: 4 B of nibbles -> 16 B of bf16
  // (8 channels of one pixel); chunks cover the real window pixels only
  constexpr int CPT = (G::CHUNKS + WR_NT - 1) / WR_NT;  // chunks per thread
  constexpr int CPP = (R + 2) * G::CPR;                  // chunks per plane
  auto expand_read = [&](int slot, int c) -> uint32_t {
    const int o = min(c * WR_NT + tid, G::CHUNKS - 1);
    const int plane = o / CPP, rem = o % CPP;
    const int row = rem / G::CPR, q = rem % G::CPR;
    return *reinterpret_cast<const uint32_t*>(smem + slot * G::SLOT + G::SOFF + row * G::R4B +
                                              (q >> 2) * 32 + plane * 16 + (q & 3) * 4);
  };
  // (lanes past the last chunk redo the last one: same bytes, no branch)
  auto expand_write = [&](int buf, int c, uint32_t v) {
    const int o = min(c * WR_NT + tid, G::CHUNKS - 1);
    const int plane = o / CPP, rem = o % CPP;
    const int row = rem / G::CPR, q = rem % G::CPR;
    typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
    uint4 out;
    out.x = __builtin_bit_cast(uint32_t, (bf2)__builtin_amdgcn_cvt_scalef32_pk_bf16_fp4(v, 1.0f, 0));
    out.y = __builtin_bit_cast(uint32_t, (bf2)__builtin_amdgcn_cvt_scalef32_pk_bf16_fp4(v, 1.0f, 1));
    out.z = __builtin_bit_cast(uint32_t, (bf2)__builtin_amdgcn_cvt_scalef32_pk_bf16_fp4(v, 1.0f, 2));
    out.w = __builtin_bit_cast(uint32_t, (bf2)__builtin_amdgcn_cvt_scalef32_pk_bf16_fp4(v, 1.0f, 3));
    *reinterpret_cast<uint4*>(smem + G::SBF + buf * G::SBYTES + plane * G::SPLANE + row * RB +
                              (q >> 2) * 64 + (q & 3) * 16) = out;
  };

  // fragment offsets: lane group gq = lane >> 4 reads pixels p = kk*16 +
  // 8*(gq>>1) + q (and + 4) of the step, 4 channels at (gq&1)*16 + 4p of its
  // 32-channel plane.  dY: offDp + hh*DPLANE + kk KB.  S: the pixel's window position
  // r*RB + (w + 1)*64 - 64 = p*64 + r*(RB - W*64) with r = p / W: a
  // compile-time offset from offS0 except where the lanes of one K-step
  // straddle an image row (then r differs by one across lanes: offS0 +
  // RB - W*64 for those lanes, xS).
  const int gq = lane >> 4, qi = lane & 15, qq = qi >> 2, pq = qi & 3;
  const int colb = (gq & 1) * 32 + pq * 8;
  const int p0 = 8 * (gq >> 1) + qq;  // 0 .. 11
  const int offDp = p0 * 64 + colb;  // co half hh: + hh * DPLANE
  const int offS0 = wn * G::SPLANE + p0 * 64 + colb;  // from the S window base
  int xS[WR_NK][2];  // per (kk, hf): offS0 + (RB - W*64) * (r - r_min) (where lanes straddle)
#pragma unroll
  for (int kk = 0; kk < WR_NK; ++kk)
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const int q0 = kk * 16 + 4 * hf;
      xS[kk][hf] = offS0 + (RB - W * 64) * ((q0 + p0) / W - q0 / W);
    }

  uint32_t ones;
  asm volatile("v_mov_b32 %0, 0x3f803f80" : "=v"(ones));
  long long* dbg = LAB == 7 ? a.dbg + ((long long)blockIdx.x * 4 + wave) * 8 : nullptr;
  // LAB 7: wall clock when this block leaves (after its tree work)
  auto lab_end = [&]() {
    if constexpr (LAB == 7)
      if (lane == 0) dbg[7] = wall_clock64();
  };
  const int h = lane >> 5, r32 = lane & 31;
  const long long NT9 = 9LL * a.Cin;
  const long long DWN = (long long)a.Cout * NT9;
  const int ci = ci0 + wn * 32 + r32;

  // The main loop and the partial-tile stores, per pair member M (waves 0,
  // 1: M 0; waves 2, 3: M 1) of the ci half wn, in a wave-uniform branch
  // around all of it, so each path keeps its own accumulators in registers
  // (no copies at the join).  A wave covers both co halves (64 x 32) on taps
  // 0-3 (M 0) or 5-8 (M 1) of every K-step and tap 4 of K-steps 0-3 (M 0) or
  // 4-6 (M 1): 32 / 31 (K-step, tap) units of two MFMAs that share one S
  // fragment; the two tap-4 partials are combined through LDS in a fixed
  // order.  Returns false if the block is done (no tree work).
  auto body = [&](auto mc) -> bool {
    constexpr int M = decltype(mc)::value;
    constexpr int NH = 2;                  // co halves per wave
    constexpr int NT = 5;                  // taps held
    constexpr int NU = wr_units(M);        // units per step
    f32x16 acc[NH][NT];
#pragma unroll
    for (int hh = 0; hh < NH; ++hh)
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[hh][t][e] = 0.f;

    long long t_wait = 0, t_issue = 0, t_mma = 0, t_prev = 0, t_start = 0;
    if constexpr (LAB == 7) {
      t_prev = clock64();
      t_start = wall_clock64();
    }
    // slot of step j: (j - j0 + FP4) % 3 (OP_FP4: a prologue slot holds the
    // window of step j0, each later slot dY(j) + the window of step j + 1)
    if constexpr (FP4) {
      issue(-1, j0, 0);
      issue(j0, j0 + 1, 1);
      issue(j0 + 1, j0 + 2, 2);
      wait_vmcnt<2 * NI>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
#pragma unroll
      for (int c = 0; c < CPT; ++c) expand_write(j0 & 1, c, expand_read(0, c));
    } else {
      issue(j0, j0, 0);
      issue(j0 + 1, j0 + 1, 1);
    }
    for (int j = j0; j < j1; ++j) {
      const int slot = (j - j0 + (FP4 ? 1 : 0)) % WR_NSLOT;
      if constexpr (LAB == 7) {
        const long long t = clock64();
        t_mma += t - t_prev;
        t_prev = t;
      }
      wait_vmcnt<NI>();  // step j landed (this wave's pieces); j + 1 in flight
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if constexpr (LAB == 7) {
        const long long t = clock64();
        t_wait += t - t_prev;
        t_prev = t;
      }
      // step j + 2 into the slot step j - 1 used (every wave is past it)
      const Stage nx = prep(j + 2, j + 2 + (FP4 ? 1 : 0), (j + 2 - j0 + (FP4 ? 1 : 0)) % WR_NSLOT);
      if constexpr (!spread || !do_mma) {
#pragma unroll
        for (int k = 0; k < NI; ++k) piece(nx, k);
      }
      if constexpr (LAB == 7) {
        const long long t = clock64();
        t_issue += t - t_prev;
        t_prev = t;
      }
      if constexpr (!do_mma) continue;
      const int base = slot * G::SLOT;
      const int sbase = FP4 ? G::SBF + (j & 1) * G::SBYTES : base + G::SOFF;
      // OP_FP4: the window of step j + 1 is expanded for the next iteration
      // (unconditionally: after the last step it fills a buffer nobody reads).
      // Each S fragment is read FD units ahead into a small rotating buffer
      // (one wave per SIMD: only this lookahead hides the LDS latency; few
      // registers, so the accumulators never leave their registers).
      constexpr int NB = FD + 1;
      uint4 fb[NB], fa[3][NH];
      uint32_t xv[2] = {0u, 0u};
      auto read_b = [&](int n) {
        const int kk = wr_unit_kk(M, n), t = wr_unit_tap(M, n), kh = t / 3, kw = t % 3;
        if constexpr (!lab_reads) {
          fb[n % NB] = make_uint4(n, kk, t, lane);
          return;
        }
        int o[2];
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          const int q0 = kk * 16 + 4 * hf;
          // lanes p0 = 0 .. 11 of this K-step in one image row: a constant offset
          const bool one_row = q0 / W == (q0 + 11) / W;
          o[hf] = (one_row ? sbase + offS0 : sbase + xS[kk][hf]) + q0 * 64 + (q0 / W) * (RB - W * 64) +
                  kh * RB + kw * 64;
        }
        fb[n % NB] = tr_read2(smem, o[0], o[1]);
      };
      auto read_a = [&](int kk) {
#pragma unroll
        for (int hh = 0; hh < NH; ++hh) {
          const int aD = base + hh * G::DPLANE + offDp + kk * 1024;
          fa[kk % 3][hh] = tr_read2(smem, aD, aD + 256);
        }
      };
      // (a unit whose K-step differs from its predecessor's reads that K-step's dY)
      auto first_of_kk = [](int n) { return n == 0 || wr_unit_kk(M, n) != wr_unit_kk(M, n - 1); };
#pragma unroll
      for (int n = 0; n < FD; ++n) {
        if (first_of_kk(n)) read_a(wr_unit_kk(M, n));
        read_b(n);
      }
      // FP4 expansion chunks spread over the units: chunk c read at unit
      // c * XS, converted and stored XS / 2 units later
      constexpr int XS = NU / CPT >= 2 ? NU / CPT : 2;
#pragma unroll
      for (int n = 0; n < NU; ++n) {
        if constexpr (spread && do_mma) {
          // DMA piece k at unit k * DS
          constexpr int DS = NU / NI;
          static_assert(DS >= 1, "DMA spread");
          if (n % DS == 0 && n / DS < NI) piece(nx, n / DS);
        }
        if (n + FD < NU) {
          if (first_of_kk(n + FD)) read_a(wr_unit_kk(M, n + FD));
          read_b(n + FD);
        }
        if constexpr (FP4) {
          if (n % XS == 0 && n / XS < CPT) xv[(n / XS) & 1] = expand_read(slot, n / XS);
          if (n % XS == XS / 2 && n / XS < CPT) expand_write((j + 1) & 1, n / XS, xv[(n / XS) & 1]);
        }
        uint4 b = fb[n % NB];
        if constexpr (SIGN) {
          b.x = sign_bf16x2(b.x, ones);
          b.y = sign_bf16x2(b.y, ones);
          b.z = sign_bf16x2(b.z, ones);
          b.w = sign_bf16x2(b.w, ones);
        }
        const int kk = wr_unit_kk(M, n), ti = wr_tap_slot(M, wr_unit_tap(M, n));
        if constexpr (lab_mfma) {
#pragma unroll
          for (int hh = 0; hh < NH; ++hh) acc[hh][ti] = mfma_bf16(fa[kk % 3][hh], b, acc[hh][ti]);
        } else {
          asm volatile("" ::"v"(b.x), "v"(b.y), "v"(b.z), "v"(b.w));
        }
        // keep the issue order: reads FD units ahead (the scheduler would
        // otherwise sink them next to their MFMA and expose the LDS latency)
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (FP4) {
        // chunks beyond the units' slots: finish them here
#pragma unroll
        for (int c = (NU + XS - 1) / XS; c < CPT; ++c)
          expand_write((j + 1) & 1, c, expand_read(slot, c));
      }
    }

    wait_vmcnt<0>();  // the DMA issued past the last step (its LDS is reused below)
    if constexpr (LAB == 7) {
      t_mma += clock64() - t_prev;
      if (lane == 0) {
        dbg[0] = t_wait;
        dbg[1] = t_issue;
        dbg[2] = t_mma;
        dbg[3] = j1 - j0;
        dbg[4] = t_start;
        dbg[5] = wall_clock64();
        dbg[6] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11));  // HW_REG_XCC_ID
      }
    }
    {
      // tap 4: member 1 hands its partial to member 0 through LDS (fixed
      // order: member 0's + member 1's); 8 KB per wave
      float4* cb = reinterpret_cast<float4*>(smem);
      __syncthreads();  // every wave is past its last LDS read of the loop
      if constexpr (M == 1) {
#pragma unroll
        for (int hh = 0; hh < 2; ++hh)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            cb[((wn * 2 + hh) * 4 + q) * 64 + lane] =
                make_float4(acc[hh][0][4 * q], acc[hh][0][4 * q + 1], acc[hh][0][4 * q + 2],
                            acc[hh][0][4 * q + 3]);
      }
      __syncthreads();
      if constexpr (M == 0) {
#pragma unroll
        for (int hh = 0; hh < 2; ++hh)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float4 v = cb[((wn * 2 + hh) * 4 + q) * 64 + lane];
            acc[hh][4][4 * q] += v.x;
            acc[hh][4][4 * q + 1] += v.y;
            acc[hh][4][4 * q + 2] += v.z;
            acc[hh][4][4 * q + 3] += v.w;
          }
      }
    }
    // ---- this wave's final partial taps: D[co][ci] of tap t: co = co0 + 32*cw
    // + (e&3) + 8*(e>>2) + 4*(lane>>5) with cw = hh, ci = ci0 +
    // wn*32 + (lane&31).  Member 1's tap 4 went to member 0.
    constexpr int TLO = M == 1 ? 1 : 0;
    if (a.levels == 0) {  // one split: straight into dW
#pragma unroll
      for (int hh = 0; hh < NH; ++hh)
#pragma unroll
        for (int ti = TLO; ti < NT; ++ti)
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int t = wr_slot_tap(M, ti);
            const int co = co0 + hh * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
            const long long idx = (long long)co * NT9 + (long long)t * a.Cin + ci;
            if (!a.w || fabsf(a.w[idx]) <= a.clip) a.dw[idx] += acc[hh][ti][e];
          }
      return false;
    }
    // Partial tiles cross XCDs (each has its own L2): slab stores and loads
    // are agent-scope (sc1: written through to, and read from, the coherent
    // level), so publishing needs only the stores' completion before the
    // counter atomic -- no agent-scope release / acquire fence, which writes
    // back / invalidates the WHOLE L2 of the XCD (buffer_wbl2 / buffer_inv)
    // and, with 32 blocks per XCD arriving together, serialised into ~180 us
    // at b1536.
    float* sl = a.slab + a.slab_off[0] + (long long)split * DWN;
#pragma unroll
    for (int hh = 0; hh < NH; ++hh)
#pragma unroll
      for (int ti = TLO; ti < NT; ++ti)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int t = wr_slot_tap(M, ti);
          const int co = co0 + hh * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
          __hip_atomic_store(sl + (long long)co * NT9 + (long long)t * a.Cin + ci, acc[hh][ti][e],
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    return true;
  };
  const bool more = wave < 2 ? body(std::integral_constant<int, 0>{})
                             : body(std::integral_constant<int, 1>{});
  if (!more) {
    lab_end();
    return;
  }

  // ---- fixed-order tree over the splits of this tile
  volatile int* flag = reinterpret_cast<volatile int*>(smem + G::FLAG);
  int node = split;
  for (int l = 1; l <= a.levels; ++l) {
    const int parent = node / WR_G;
    const int first = parent * WR_G;
    const int nchild = min(WR_G, a.nodes[l - 1] - first);
    // publish this block's slab: every wave's (write-through) stores complete
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      int* c = a.cnt + a.cnt_off[l] + tile * a.nodes[l] + parent;
      const int t = __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = t == nchild - 1;
      if (last) __hip_atomic_store(c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
      *flag = last;
    }
    __syncthreads();
    if (!*flag) {
      lab_end();
      return;
    }
    node = parent;
    // sum the children in index order.  This tile's 64 x 9 x 64 floats are
    // 9216 float4, 36 per thread, taken 4 at a time from all 8 children at
    // once (32 loads in flight per thread: the reducer is latency-bound
    // otherwise).  Missing children (the last group) re-read the group's last
    // child and are dropped by a select, not a branch around the load.
    const float* src = a.slab + a.slab_off[l - 1];
    const bool root = l == a.levels;
    float* dst = root ? a.dw : a.slab + a.slab_off[l] + (long long)node * DWN;
    __amdgpu_buffer_rsrc_t rs[WR_G];
#pragma unroll
    for (int c = 0; c < WR_G; ++c)
      rs[c] = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(src + (long long)(first + min(c, nchild - 1)) * DWN), (short)0,
          (int)(DWN * 4), 0x00020000);
    for (int i0 = 0; i0 < 36; i0 += 4) {
      int idx[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = (i0 + u) * WR_NT + tid;
        const int co = e / 144, rem = e - co * 144;
        idx[u] = ((co0 + co) * 9 + (rem >> 4)) * a.Cin + ci0 + (rem & 15) * 4;
      }
      float4 v[4][WR_G];
#pragma unroll
      for (int c = 0; c < WR_G; ++c)
#pragma unroll
        for (int u = 0; u < 4; ++u)
          v[u][c] = __builtin_bit_cast(
              float4, __builtin_amdgcn_raw_buffer_load_b128(rs[c], idx[u] * 4, 0, WR_SC1));
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float4 t = v[u][0];
#pragma unroll
        for (int c = 1; c < WR_G; ++c) {
          const bool in = c < nchild;
          t.x += in ? v[u][c].x : 0.f;
          t.y += in ? v[u][c].y : 0.f;
          t.z += in ? v[u][c].z : 0.f;
          t.w += in ? v[u][c].w : 0.f;
        }
        if (root) {
          float4 d = *reinterpret_cast<float4*>(dst + idx[u]);
          if (a.w) {
            const float4 wv = *reinterpret_cast<const float4*>(a.w + idx[u]);
            d.x += fabsf(wv.x) <= a.clip ? t.x : 0.f;
            d.y += fabsf(wv.y) <= a.clip ? t.y : 0.f;
            d.z += fabsf(wv.z) <= a.clip ? t.z : 0.f;
            d.w += fabsf(wv.w) <= a.clip ? t.w : 0.f;
          } else {
            d.x += t.x;
            d.y += t.y;
            d.z += t.z;
            d.w += t.w;
          }
          *reinterpret_cast<float4*>(dst + idx[u]) = d;
        } else {
          float* o = dst + idx[u];
          __hip_atomic_store(o + 0, t.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(o + 1, t.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(o + 2, t.z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(o + 3, t.w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
  }
  lab_end();
}

int g_wr_lab = 0;  // zk_wgrad_rows_lab
long long* g_wr_dbg = nullptr;

struct WrPlan {
  int nsteps, sps, splits, tiles, levels;
  int nodes[WR_MAXLV];
  long long slab_off[WR_MAXLV];
  int cnt_off[WR_MAXLV];
  long long slab_floats, cnt_ints;
};

// Supported: W in {56, 28} (a step = 112 pixels = R whole image rows), H % R
// == 0 (steps never straddle images), channels in multiples of 64, Cin <=
// WR_MAXCIN (the pad-row pages; the 64 / 128-channel stages this serves).
bool wr_plan(int B, int H, int W, int Cin, int Cout, int target_blocks, WrPlan& p) {
  if (B < 1 || H < 1 || Cin % 64 || Cout % 64 || Cin > WR_MAXCIN || Cout > 1024) return false;
  if (W != 56 && W != 28) return false;
  const int R = WR_RW / W;
  if (H % R) return false;
  if ((long long)B * H * W * Cin >= (1LL << 40) || (long long)B * H * W * Cout >= (1LL << 40))
    return false;
  const long long ns = (long long)B * H / R;
  if (ns >= (1LL << 30)) return false;
  p.nsteps = (int)ns;
  p.tiles = (Cout / 64) * (Cin / 64);
  if (target_blocks <= 0) target_blocks = 256;
  int s = target_blocks / p.tiles;
  if (s < 1) s = 1;
  p.sps = (p.nsteps + s - 1) / s;
  if (p.sps < 2) p.sps = 2;
  p.splits = (p.nsteps + p.sps - 1) / p.sps;
  p.levels = 0;
  p.nodes[0] = p.splits;
  int n = p.splits;
  while (n > 1) {
    n = (n + WR_G - 1) / WR_G;
    if (++p.levels >= WR_MAXLV) return false;
    p.nodes[p.levels] = n;
  }
  for (int l = p.levels + 1; l < WR_MAXLV; ++l) p.nodes[l] = 0;
  const long long dwn = (long long)Cout * 9 * Cin;
  long long so = 0;
  int co = 0;
  for (int l = 0; l < WR_MAXLV; ++l) {
    p.slab_off[l] = so;
    p.cnt_off[l] = co;
    if (l < p.levels) so += (long long)p.nodes[l] * dwn;    // levels 0 .. levels-1 stored
    if (l >= 1 && l <= p.levels) co += p.nodes[l] * p.tiles;  // counters of levels 1 .. levels
  }
  p.slab_floats = so;
  p.cnt_ints = co;
  return true;
}

// the pad-row pages, once per device (before the first launch on it)
hipError_t wr_pad_ready(hipStream_t st) {
  static bool done[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return hipErrorInvalidDevice;
  if (!done[dev]) {
    hipLaunchKernelGGL(wr_pad_init_kernel, dim3((WR_PADROW / 4 + 255) / 256), dim3(256), 0, st);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    done[dev] = true;
  }
  return hipSuccess;
}

template <int W, int OP, int LAB = 0, int FD = 0>
hipError_t wr_launch(const WrArgs& a, unsigned grid, hipStream_t st) {
  constexpr int lds = WrGeo<W, OP>::LDS;
  {
    const hipError_t e = wr_pad_ready(st);
    if (e != hipSuccess) return e;
  }
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)wgrad_rows_kernel<W, OP, LAB, FD>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize,
                                             lds);
    if (e != hipSuccess) return e;
    attr = true;
  }
  (void)hipGetLastError();
  hipLaunchKernelGGL((wgrad_rows_kernel<W, OP, LAB, FD>), dim3(grid), dim3(WR_NT), lds,
                     st, a);
  return hipGetLastError();
}

}  // namespace

// Ablation switch of the lab (tools/wgrad_lab.py): 0 normal, 1 loads only,
// 2 compute only, 3 compute only without the MFMAs (LDS reads only), 4
// compute only without the S fragment reads (results are garbage in 1-4),
// 6 lookahead 4, 7 cycle accounting
// into dbg ([blocks][4 waves][8]), 8 the step's DMA issued in one burst.
ZK_EXPORT int zk_wgrad_rows_lab(int mode, void* dbg) {
  g_wr_lab = mode;
  g_wr_dbg = (long long*)dbg;
  return 0;
}

// Workspace of zk_wgrad_rows for one shape: slab floats and counter ints
// (both 0 when a single split writes dW directly).  Returns 0 if the shape
// is supported, -1 otherwise.
ZK_EXPORT int zk_wgrad_rows_plan(int B, int H, int W, int Cin, int Cout, int target_blocks,
                                 long long* slab_bytes, long long* cnt_bytes) {
  WrPlan p;
  if (!wr_plan(B, H, W, Cin, Cout, target_blocks, p)) return -1;
  if (slab_bytes) *slab_bytes = p.slab_floats * 4;
  if (cnt_bytes) *cnt_bytes = p.cnt_ints * 4;
  return 0;
}

// dw [Cout][3][3][Cin] fp32 += mask(|w| <= clip) * (3x3 stride-1 'same'
// weight gradient of dy [B][H][W][Cout] against the operand sx), by operand
// mode op:
//   0: sx is a bf16 image (the +-1 sign image, or a float activation);
//      padding reads +1 (pad_ones) or 0;
//   1: sx is the bf16 activation, sign taken in registers; needs pad_ones
//      (the padding, a zero, becomes +1);
//   2: sx is the e2m1 (FP4) +-1 sign image [B][H][W][Cin/2 bytes] (channel
//      2j in the low nibble of byte j, zk_sign_pack's layout); padding +1
//      (pad_ones) or 0.
// w null: no kernel STE mask.  slab / cnt: zk_wgrad_rows_plan's bytes;
// cnt must be zero before the first launch and is left zero by every launch
// (one counter buffer per stream: launches on one stream never overlap).
ZK_EXPORT int zk_wgrad_rows(const void* dy, const void* sx, const void* w, void* dw, void* slab,
                            long long slab_bytes, void* cnt, long long cnt_bytes, int B, int H,
                            int W, int Cin, int Cout, int pad_ones, int op, float clip,
                            int target_blocks, hipStream_t st) {
  WrPlan p;
  if (!wr_plan(B, H, W, Cin, Cout, target_blocks, p)) return (int)hipErrorInvalidValue;
  if (op < OP_IMG || op > OP_FP4 || (op == OP_SIGN && !pad_ones)) return (int)hipErrorInvalidValue;
  if (p.levels > 0 && (!slab || !cnt || slab_bytes < p.slab_floats * 4 ||
                       cnt_bytes < p.cnt_ints * 4))
    return (int)hipErrorInvalidValue;
  if (!dy || !sx || !dw) return (int)hipErrorInvalidValue;
  WrArgs a{};
  a.dy = (const uint16_t*)dy;
  a.sx = (const uint16_t*)sx;
  a.w = (const float*)w;
  a.dw = (float*)dw;
  a.slab = (float*)slab;
  a.cnt = (int*)cnt;
  a.B = B;
  a.H = H;
  a.W = W;
  a.Cin = Cin;
  a.Cout = Cout;
  a.nsteps = p.nsteps;
  a.sps = p.sps;
  a.splits = p.splits;
  a.co_tiles = Cout / 64;
  a.ci_tiles = Cin / 64;
  a.pad_ones = pad_ones;
  a.clip = clip;
  a.levels = p.levels;
  for (int l = 0; l < WR_MAXLV; ++l) {
    a.nodes[l] = p.nodes[l];
    a.slab_off[l] = p.slab_off[l];
    a.cnt_off[l] = p.cnt_off[l];
  }
  const unsigned grid = (unsigned)(p.tiles * p.splits);
  a.dbg = g_wr_dbg;
  if (g_wr_lab && W == 56 && op == OP_SIGN) {  // lab ablations (tools/wgrad_lab.py)
    switch (g_wr_lab) {
      case 1: return (int)wr_launch<56, OP_SIGN, 1>(a, grid, st);
      case 2: return (int)wr_launch<56, OP_SIGN, 2>(a, grid, st);
      case 3: return (int)wr_launch<56, OP_SIGN, 3>(a, grid, st);
      case 4: return (int)wr_launch<56, OP_SIGN, 4>(a, grid, st);
      case 6: return (int)wr_launch<56, OP_SIGN, 0, 4>(a, grid, st);
      case 7: return (int)wr_launch<56, OP_SIGN, 7>(a, grid, st);
      case 8: return (int)wr_launch<56, OP_SIGN, 8>(a, grid, st);
      default: return (int)hipErrorInvalidValue;
    }
  }
  if (g_wr_lab == 7 && W == 56) {
    if (op == OP_IMG) return (int)wr_launch<56, OP_IMG, 7>(a, grid, st);
    return (int)wr_launch<56, OP_FP4, 7>(a, grid, st);
  }
  switch (op * 2 + (W == 56)) {
    case OP_IMG * 2 + 1: return (int)wr_launch<56, OP_IMG>(a, grid, st);
    case OP_SIGN * 2 + 1: return (int)wr_launch<56, OP_SIGN>(a, grid, st);
    case OP_FP4 * 2 + 1: return (int)wr_launch<56, OP_FP4>(a, grid, st);
    case OP_IMG * 2: return (int)wr_launch<28, OP_IMG>(a, grid, st);
    case OP_SIGN * 2: return (int)wr_launch<28, OP_SIGN>(a, grid, st);
    default: return (int)wr_launch<28, OP_FP4>(a, grid, st);
  }
}
