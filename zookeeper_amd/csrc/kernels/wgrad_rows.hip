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
#include "mfma_common.h"

namespace {

constexpr int WR_NT = 256;     // 4 waves
constexpr int WR_G = 8;        // tree fan-in
constexpr int WR_MAXLV = 8;
constexpr int WR_RW = 112;     // pixels per step
constexpr int WR_NK = WR_RW / 16;
constexpr int WR_NSLOT = 3;

template <int W>
struct WrGeo {
  static constexpr int R = WR_RW / W;           // image rows per step
  static constexpr int PW = W + 2;              // S window row pitch (pixels)
  static constexpr int RB = PW * 64;            // S window row bytes in one plane
  static constexpr int SPLANE = (R + 2) * RB;   // window rows h0-1 .. h0+R
  static constexpr int SBYTES = 2 * SPLANE;
  static constexpr int DPLANE = WR_RW * 64;
  static constexpr int DBYTES = 2 * DPLANE;     // 14 KB
  static constexpr int DINS = DBYTES / 1024;
  static constexpr int TOT = (DINS + (SBYTES + 1023) / 1024 + 3) / 4 * 4;  // DMA pieces
  static constexpr int NI = TOT / 4;            // DMA pieces per wave per step
  static constexpr int SLOT = TOT * 1024;
  static constexpr int FLAG = WR_NSLOT * SLOT;  // arrival broadcast word
  static constexpr int LDS = FLAG + 16;
  static_assert(WR_RW % W == 0 && LDS <= 160 * 1024, "row-stream geometry");
};

struct WrArgs {
  const uint16_t* dy;  // [B][H][W][Cout] bf16
  const uint16_t* sx;  // [B][H][W][Cin] bf16 (sign image, or the activation with SIGN)
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

// LAB: ablation builds for tools/wgrad_lab.py (0 = the kernel; 1 loads only,
// 2 compute only, 3 compute only without MFMAs, 4 compute only without the S
// fragment reads; results are garbage in 1-4)
// FD: how many MFMAs ahead each S fragment is read (one wave per SIMD: only
// this lookahead hides the LDS latency)
template <int W, bool SIGN, int LAB = 0, int FD = 6>
__global__ __launch_bounds__(WR_NT, 1) void wgrad_rows_kernel(WrArgs a) {
  using G = WrGeo<W>;
  constexpr int R = G::R, PW = G::PW, RB = G::RB, NI = G::NI;
  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles = a.co_tiles * a.ci_tiles;
  const int L = xcd_linear(blockIdx.x, gridDim.x);
  const int split = L / tiles, tile = L % tiles;
  const int co0 = (tile % a.co_tiles) * 64, ci0 = (tile / a.co_tiles) * 64;
  const int j0 = split * a.sps;
  const int j1 = min(a.nsteps, j0 + a.sps);
  const int H = a.H;

  const unsigned char* dyb = reinterpret_cast<const unsigned char*>(a.dy);
  const unsigned char* sxb = reinterpret_cast<const unsigned char*>(a.sx);
  const unsigned char* zp = reinterpret_cast<const unsigned char*>(g_zero_page);
  const unsigned char* pp =
      (a.pad_ones && !SIGN) ? reinterpret_cast<const unsigned char*>(g_ones_page_bf16) : zp;
  constexpr bool do_load = LAB < 2, do_mma = LAB != 1;
  constexpr bool lab_reads = LAB != 4, lab_mfma = LAB != 3;

  // per-lane LDS-DMA sources of a slot's NI pieces per wave (piece t = k*4 +
  // wave covers slot bytes [t KB, t KB + 1 KB)): a byte offset (multiple of
  // 16) from the step's first dY / S pixel, with a code in its low 4 bits:
  // 0 = dY, 1 + wr = S window row wr, 14 = padding page (halo column),
  // 15 = slot tail (zeros)
  int src[NI];
#pragma unroll
  for (int k = 0; k < NI; ++k) {
    const int b = (k * 4 + wave) * 1024 + lane * 16;
    if (b < G::DBYTES) {
      const int plane = b / G::DPLANE, rem = b % G::DPLANE;
      const int p = rem >> 6, ch = (rem & 63) >> 4;
      src[k] = (p * a.Cout + co0 + plane * 32 + ch * 8) * 2;
    } else if (b - G::DBYTES < G::SBYTES) {
      const int bs = b - G::DBYTES;
      const int plane = bs / G::SPLANE, rem = bs % G::SPLANE;
      const int wr = rem / RB, col = (rem % RB) >> 6, ch = (rem & 63) >> 4;
      if (col >= 1 && col <= W)
        src[k] = ((((wr - 1) * W + col - 1) * a.Cin + ci0 + plane * 32 + ch * 8) * 2) | (1 + wr);
      else
        src[k] = 14;
    } else {
      src[k] = 15;
    }
  }
  const long long dy_step = (long long)WR_RW * a.Cout * 2;
  const long long sx_step = (long long)WR_RW * a.Cin * 2;
  auto issue = [&](int j, int slot) {
    if constexpr (!do_load) return;
    const unsigned char* dyp = dyb + (long long)j * dy_step;
    const unsigned char* sxp = sxb + (long long)j * sx_step;
    const int h0 = (int)(((long long)j * R) % H);
    const int top = h0 == 0 ? 1 : -100;           // window row 0 is above the image
    const int bot = h0 + R == H ? R + 2 : -100;   // window row R + 1 is below it
    unsigned char* dst = smem + slot * G::SLOT + wave * 1024;
    // branch-free source selection (selects, no divergent branches)
    const uint64_t dyu = (uint64_t)(uintptr_t)dyp, sxu = (uint64_t)(uintptr_t)sxp;
    const uint64_t ppu = (uint64_t)(uintptr_t)pp, zpu = (uint64_t)(uintptr_t)zp;
#pragma unroll
    for (int k = 0; k < NI; ++k) {
      const int kd = src[k] & 15, off = src[k] & ~15;
      const bool pad = kd >= 14 || kd == top || kd == bot;
      const uint64_t real = (kd == 0 ? dyu : sxu) + (uint64_t)(int64_t)off;
      const uint64_t fill = kd == 15 ? zpu : ppu;
      ZK_GLDS16((const void*)(uintptr_t)(pad ? fill : real), dst + k * 4096);
    }
  };

  // fragment offsets: lane group gq = lane >> 4 reads pixels p = kk*16 +
  // 8*(gq>>1) + q (and + 4) of the step, 4 channels at (gq&1)*16 + 4p of its
  // 32-channel plane.  dY: offD + kk KB.  S: the pixel's window position
  // (r*PW + w) * 64 = (p + 2r) * 64 with r = p / W: a compile-time offset
  // from offS0 except where the lanes of one K-step straddle an image row
  // (then r differs by one across lanes: offS0 + 128 for those lanes, xS).
  const int gq = lane >> 4, qi = lane & 15, qq = qi >> 2, pq = qi & 3;
  const int colb = (gq & 1) * 32 + pq * 8;
  const int p0 = 8 * (gq >> 1) + qq;  // 0 .. 11
  const int offD = wm * G::DPLANE + p0 * 64 + colb;
  const int offS0 = G::DBYTES + wn * G::SPLANE + p0 * 64 + colb;
  int xS[WR_NK][2];  // per (kk, hf): offS0 + 128 * (r - r_min) (used where lanes straddle)
#pragma unroll
  for (int kk = 0; kk < WR_NK; ++kk)
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const int q0 = kk * 16 + 4 * hf;
      xS[kk][hf] = offS0 + 128 * ((q0 + p0) / W - q0 / W);
    }

  uint32_t ones;
  asm volatile("v_mov_b32 %0, 0x3f803f80" : "=v"(ones));
  f32x16 acc[9];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[t][e] = 0.f;

  long long t_wait = 0, t_issue = 0, t_mma = 0, t_prev = 0, t_start = 0;
  if constexpr (LAB == 7) {
    t_prev = clock64();
    t_start = wall_clock64();
  }
  if (j0 < j1) issue(j0, 0);
  if (j0 + 1 < j1) issue(j0 + 1, 1);
  for (int j = j0; j < j1; ++j) {
    const int slot = (j - j0) % WR_NSLOT;
    if constexpr (LAB == 7) {
      const long long t = clock64();
      t_mma += t - t_prev;
      t_prev = t;
    }
    if (j + 1 < j1)
      wait_vmcnt<NI>();  // step j landed (this wave's pieces); j + 1 in flight
    else
      wait_vmcnt<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if constexpr (LAB == 7) {
      const long long t = clock64();
      t_wait += t - t_prev;
      t_prev = t;
    }
    if (j + 2 < j1) issue(j + 2, (j + 2 - j0) % WR_NSLOT);
    if constexpr (LAB == 7) {
      const long long t = clock64();
      t_issue += t - t_prev;
      t_prev = t;
    }
    if constexpr (!do_mma) continue;
    const int base = slot * G::SLOT;
    // the step's 63 MFMAs (K-step kk = i / 9, tap t = i % 9) with each
    // fragment read FD MFMAs ahead into a small rotating buffer (one wave per
    // SIMD: only this lookahead hides the LDS latency; few registers, so the
    // accumulators never leave their registers)
    constexpr int NB = FD + 1, NM = WR_NK * 9;
    uint4 fb[NB], fa[2];
    auto read_b = [&](int i) {
      const int kk = i / 9, t = i % 9, kh = t / 3, kw = t % 3;
      if constexpr (!lab_reads) {
        fb[i % NB] = make_uint4(i, kk, t, lane);
        return;
      }
      int o[2];
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        const int q0 = kk * 16 + 4 * hf;
        // lanes p0 = 0 .. 11 of this K-step in one image row: a constant offset
        const bool one_row = q0 / W == (q0 + 11) / W;
        o[hf] = (one_row ? base + offS0 : base + xS[kk][hf]) + (q0 + 2 * (q0 / W)) * 64 +
                kh * RB + kw * 64;
      }
      fb[i % NB] = tr_read2(smem, o[0], o[1]);
    };
    auto read_a = [&](int kk) {
      const int aD = base + offD + kk * 1024;
      fa[kk % 2] = tr_read2(smem, aD, aD + 256);
    };
    read_a(0);
#pragma unroll
    for (int i = 0; i < FD; ++i) read_b(i);
#pragma unroll
    for (int i = 0; i < NM; ++i) {
      if (i + FD < NM) {
        if ((i + FD) % 9 == 0) read_a((i + FD) / 9);
        read_b(i + FD);
      }
      uint4 b = fb[i % NB];
      if constexpr (SIGN) {
        b.x = sign_bf16x2(b.x, ones);
        b.y = sign_bf16x2(b.y, ones);
        b.z = sign_bf16x2(b.z, ones);
        b.w = sign_bf16x2(b.w, ones);
      }
      if constexpr (lab_mfma)
        acc[i % 9] = mfma_bf16(fa[(i / 9) % 2], b, acc[i % 9]);
      else
        asm volatile("" ::"v"(b.x), "v"(b.y), "v"(b.z), "v"(b.w));
      // keep the issue order: reads FD MFMAs ahead (the scheduler would
      // otherwise sink them next to their MFMA and expose the LDS latency)
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  if constexpr (LAB == 7) {
    t_mma += clock64() - t_prev;
    if (lane == 0) {
      long long* d = a.dbg + ((long long)blockIdx.x * 4 + wave) * 8;
      d[0] = t_wait;
      d[1] = t_issue;
      d[2] = t_mma;
      d[3] = j1 - j0;
      d[4] = t_start;
      d[5] = wall_clock64();
      d[6] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11));  // HW_REG_XCC_ID
      d[7] = clock64();
    }
  }
  // ---- epilogue: D[co][ci] of tap t in acc[t]: co = co0 + wm*32 + (e&3) +
  // 8*(e>>2) + 4*(lane>>5), ci = ci0 + wn*32 + (lane&31)
  const int h = lane >> 5, r32 = lane & 31;
  const long long NT9 = 9LL * a.Cin;
  const int ci = ci0 + wn * 32 + r32;
  if (a.levels == 0) {  // one split: straight into dW
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int co = co0 + wm * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
        const long long idx = (long long)co * NT9 + (long long)t * a.Cin + ci;
        if (!a.w || fabsf(a.w[idx]) <= a.clip) a.dw[idx] += acc[t][e];
      }
    return;
  }
  const long long DWN = (long long)a.Cout * NT9;
  {
    float* sl = a.slab + a.slab_off[0] + (long long)split * DWN;
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int co = co0 + wm * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
        sl[(long long)co * NT9 + (long long)t * a.Cin + ci] = acc[t][e];
      }
  }

  // ---- fixed-order tree over the splits of this tile
  volatile int* flag = reinterpret_cast<volatile int*>(smem + G::FLAG);
  int node = split;
  for (int l = 1; l <= a.levels; ++l) {
    const int parent = node / WR_G;
    const int first = parent * WR_G;
    const int nchild = min(WR_G, a.nodes[l - 1] - first);
    // publish this block's slab: every wave's stores done, one agent release
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      int* c = a.cnt + a.cnt_off[l] + tile * a.nodes[l] + parent;
      const int t = __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = t == nchild - 1;
      if (last) {
        __hip_atomic_store(c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      *flag = last;
    }
    __syncthreads();
    if (!*flag) return;
    node = parent;
    // sum the children in index order; this tile's 64 x 9 x 64 floats as
    // 9216 float4, 36 per thread, in 3 chunks of 12
    const float* src = a.slab + a.slab_off[l - 1];
    const bool root = l == a.levels;
    float* dst = root ? a.dw : a.slab + a.slab_off[l] + (long long)node * DWN;
    for (int i0 = 0; i0 < 36; i0 += 12) {
      int idx[12];
#pragma unroll
      for (int i = 0; i < 12; ++i) {
        const int e = (i0 + i) * WR_NT + tid;
        const int co = e / 144, rem = e - co * 144;
        idx[i] = ((co0 + co) * 9 + (rem >> 4)) * a.Cin + ci0 + (rem & 15) * 4;
      }
      float4 s[12];
#pragma unroll
      for (int i = 0; i < 12; ++i) s[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int c = 0; c < nchild; ++c) {
        const float* cs = src + (long long)(first + c) * DWN;
#pragma unroll
        for (int i = 0; i < 12; ++i) {
          const float4 v = *reinterpret_cast<const float4*>(cs + idx[i]);
          s[i].x += v.x;
          s[i].y += v.y;
          s[i].z += v.z;
          s[i].w += v.w;
        }
      }
#pragma unroll
      for (int i = 0; i < 12; ++i) {
        if (root) {
          float4 d = *reinterpret_cast<float4*>(dst + idx[i]);
          if (a.w) {
            const float4 wv = *reinterpret_cast<const float4*>(a.w + idx[i]);
            d.x += fabsf(wv.x) <= a.clip ? s[i].x : 0.f;
            d.y += fabsf(wv.y) <= a.clip ? s[i].y : 0.f;
            d.z += fabsf(wv.z) <= a.clip ? s[i].z : 0.f;
            d.w += fabsf(wv.w) <= a.clip ? s[i].w : 0.f;
          } else {
            d.x += s[i].x;
            d.y += s[i].y;
            d.z += s[i].z;
            d.w += s[i].w;
          }
          *reinterpret_cast<float4*>(dst + idx[i]) = d;
        } else {
          *reinterpret_cast<float4*>(dst + idx[i]) = s[i];
        }
      }
    }
  }
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
// == 0 (steps never straddle images), channels in multiples of 64.
bool wr_plan(int B, int H, int W, int Cin, int Cout, int target_blocks, WrPlan& p) {
  if (B < 1 || H < 1 || Cin % 64 || Cout % 64 || Cin > 1024 || Cout > 1024) return false;
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

template <int W, bool SIGN, int LAB = 0, int FD = 6>
hipError_t wr_launch(const WrArgs& a, unsigned grid, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)wgrad_rows_kernel<W, SIGN, LAB, FD>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize,
                                             WrGeo<W>::LDS);
    if (e != hipSuccess) return e;
    attr = true;
  }
  (void)hipGetLastError();
  hipLaunchKernelGGL((wgrad_rows_kernel<W, SIGN, LAB, FD>), dim3(grid), dim3(WR_NT), WrGeo<W>::LDS,
                     st, a);
  return hipGetLastError();
}

}  // namespace

// Ablation switch of the lab (tools/wgrad_lab.py): 0 normal, 1 loads only,
// 2 compute only, 3 compute only without the MFMAs (LDS reads only), 4
// compute only without the S fragment reads (results are garbage in 1-4),
// 5 / 6 lookahead 3 / 7, 7 cycle accounting into dbg ([blocks][4 waves][4]).
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
// weight gradient of dy [B][H][W][Cout] against sx [B][H][W][Cin]).
//   sign_act = 0: sx is the bf16 +-1 image; padding reads +1 (pad_ones) or 0;
//   sign_act = 1: sx is the bf16 activation, sign taken in registers; needs
//                 pad_ones (the padding, a zero, becomes +1).
// w null: no kernel STE mask.  slab / cnt: zk_wgrad_rows_plan's bytes;
// cnt must be zero before the first launch and is left zero by every launch
// (one counter buffer per stream: launches on one stream never overlap).
ZK_EXPORT int zk_wgrad_rows(const void* dy, const void* sx, const void* w, void* dw, void* slab,
                            long long slab_bytes, void* cnt, long long cnt_bytes, int B, int H,
                            int W, int Cin, int Cout, int pad_ones, int sign_act, float clip,
                            int target_blocks, hipStream_t st) {
  WrPlan p;
  if (!wr_plan(B, H, W, Cin, Cout, target_blocks, p)) return (int)hipErrorInvalidValue;
  if (sign_act && !pad_ones) return (int)hipErrorInvalidValue;
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
  if (g_wr_lab && W == 56 && sign_act) {  // lab ablations (tools/wgrad_lab.py)
    switch (g_wr_lab) {
      case 1: return (int)wr_launch<56, true, 1>(a, grid, st);
      case 2: return (int)wr_launch<56, true, 2>(a, grid, st);
      case 3: return (int)wr_launch<56, true, 3>(a, grid, st);
      case 4: return (int)wr_launch<56, true, 4>(a, grid, st);
      case 5: return (int)wr_launch<56, true, 0, 3>(a, grid, st);
      case 6: return (int)wr_launch<56, true, 0, 7>(a, grid, st);
      case 7: return (int)wr_launch<56, true, 7>(a, grid, st);
      default: return (int)hipErrorInvalidValue;
    }
  }
  if (W == 56) return (int)(sign_act ? wr_launch<56, true>(a, grid, st) : wr_launch<56, false>(a, grid, st));
  return (int)(sign_act ? wr_launch<28, true>(a, grid, st) : wr_launch<28, false>(a, grid, st));
}
