// Implicit-GEMM convolution main loop for gfx950: LDS-DMA (global_load_lds)
// multi-stage ring, XOR-swizzled LDS image, 32x32 MFMA, transposed output.
//
// One template serves the binary-conv data gradient (bf16 operands,
// v_mfma_f32_32x32x16_bf16).  The GEMM view of a KH x KW conv:
//
//   D[n][m] = sum_{tap t} sum_{k} Wt[t][n][k] * Act[pixel(m, t)][k]
//
//   dgrad: m = input pixel (of one stride-parity class), n = ci, k = co,
//          Act = dY gathered at ((hi+pt-th)/s, (wi+pl-tw)/s), Wt = S^T [T][Cin][Cout]
//
// Design (cdna_hip_programming.md §5, MI355X_MICROARCH.md §LDS):
//   * the activation rows are gathered per lane: every lane of a
//     global_load_lds_dwordx4 supplies its own source address, so the
//     implicit-GEMM gather costs nothing extra over a dense GEMM; rows that
//     fall into the zero padding read a zero page instead;
//   * the LDS image is linear per wave-instruction (glds writes base +
//     lane*16) and conflict-free for the ds_read_b128 fragment reads by an
//     XOR swizzle applied to the SOURCE chunk: slot = chunk ^ ((row >> SH) &
//     (SPR-1)) - over every 16-lane group of ds_read_b128 the 16 rows land
//     on 16 distinct 16-B bank slots;
//   * NS-stage ring: NS-1 K-steps in flight; each K-step waits with a
//     counted vmcnt for its own stage only, then one raw s_barrier (no
//     __syncthreads: its implied vmcnt(0) would drain the ring);
//   * the product is computed transposed (MFMA A = weight rows, MFMA B =
//     pixel rows) so every lane owns one pixel and 4 consecutive channels
//     per register group: the epilogue moves 8 B per access;
//   * XCD-aware tile order: consecutive M tiles of one N tile share an XCD.
#include "mfma_common.h"
#include "splitk_tree.h"

// bfwd.hip: the persistent 3x3 binary forward (Cin 64 / 128)
extern "C" int zk_bfwd_supported(int B, int H, int W, int Cin, int Cout, int kh, int kw,
                                 int stride, int pt, int pl);
extern "C" int zk_bfwd_fp4(const void* x4, const void* w4, void* y, void* stats, int B, int H,
                           int W, int Cin, int Cout, int pad_ones, int relu, int stripes,
                           hipStream_t st);

// deep_gemm.hip: phased 256x256 wgrad of the stride-1 3x3 convs with Cin and
// Cout % 256 == 0 (variant 60 of the wgrad dispatch)
int zk_wgrad_deep_impl(const void* dy, const void* sx, const void* w, void* dw, int B, int H,
                       int W, int Cin, int Cout, int pad_ones, float clip, int target_blocks,
                       void* slab, long long slab_bytes, long long* need, int* splits, bool dry,
                       bool tree, hipStream_t st);

namespace {

// Support queries (zk_igemm_*_supported): every launcher validates the
// geometry for its tile, then returns 0 WITHOUT launching while this is set.
// Host-only; lets the test suite enumerate the valid (variant, shape) pairs
// on a machine without a GPU.
thread_local bool g_dry_run = false;

struct IGeom {
  int B, H, W, Cin, Ho, Wo, Cout, kh, kw, s, pt, pl;
};

// ===========================================================================
// Convolution-shaped implicit GEMM, transposed product D[n][pixel]:
//   FWD=false (dgrad): pixels = input pixels of one stride-parity class
//     (blockIdx.y), n = ci, K = (tap, co), A = dY, B = S^T [T][Cin][Cout];
//     epilogue: STE mask bits, + dres, bf16 dx.
//   FWD=true (binary forward): pixels = output pixels, n = co,
//     K = (tap, ci), A = sign(x) bf16 +-1, B = sign(W) bf16 [T][Cout][Cin];
//     padded taps read the zero / +1 page; the fp32 accumulators hold exact
//     integers.  Epilogue: optional ReLU, int16 y, per-channel sum and
//     sum of squares (int32 in-wave, int64 block atomics).
// ===========================================================================
struct ConvArgs {
  const uint16_t* act;   // dY (dgrad) / sign(x) (fwd)
  const uint16_t* wgt;   // [T][N][K-channels] bf16 +-1
  const uint32_t* mask;  // dgrad: STE mask bits of x (optional)
  const uint16_t* dres;  // dgrad: residual gradient (optional)
  void* out;             // dgrad: dx bf16 / fwd: y int16
  unsigned long long* stats;  // fwd: [stripes][2][Cout] int64 (sum, sum of squares)
  int pad_ones, relu;    // fwd
  int stripes;           // copies of stats / psums; block b adds into copy b % stripes
  // dgrad (optional): fused BN-backward reduction of the PREVIOUS block, whose
  // output gradient is exactly the dx this kernel writes (identity shortcut,
  // single consumer): psums[0][c][stripe] += sum dx, [1][c][stripe] += sum dx * yhat
  // (channel-major copies, the layout zk_bn_bwd_coef reads),
  // yhat = (ypred - pmean[c]) * prstd[c] -- the zk_bn_bwd_reduce of that block.
  const int16_t* ypred;
  const float* pmean;
  const float* prstd;
  float* psums;
  // float forward through the LDS epilogue (a 1x1 conv as this GEMM, optional):
  // the next BatchNorm's statistics of the stored bf16 outputs,
  // fstats[stripe][0][c] += sum y, [1][c] += sum y^2 (fp64, stripe = block % stripes)
  double* fstats;
  // float dgrad through the LDS epilogue (optional): the backward sums of the
  // BatchNorm whose output gradient is exactly the dx stored here (float BN,
  // bf16 input bxb [P][Cin], coefficients bcoef [4][Cin] = scale, shift,
  // mean, rstd): bsums[mtile][0][c] = sum g', [mtile][1][c] = sum g' * xhat
  // over the block's pixels (plain stores, one row per M tile: stripes >=
  // m_tiles), g' = dx * relu mask (brelu 0: none, 1: recomputed from bxb, 2:
  // the bits bmask [P][Cin/8]); zk_bn_bwd_tiles_reduce folds the rows in a
  // fixed order into the channel-major copies zk_bn_bwd_coef reads.
  const uint16_t* bxb;
  const float* bcoef;
  const uint8_t* bmask;
  int brelu;
  float* bsums;
  // LDS epilogue (optional): dres is masked by these bits [P][Cin/8] before
  // it is added (a ResNet tail's residual gradient g * relu mask, handed over
  // as g and the mask instead of a materialised tensor)
  const uint8_t* dmask;
};

// Host-side kernel options, set from Python (ops/options.py -> zk_set_option;
// the Runtime component owns the values, no environment variables):
//   tile_huge (key 0, bitmask): which batch >= 1024 tile rules apply --
//     1: 28x28x128 wgrad on conv3 64x64, 2: 256-input-channel wgrad 256x256 x 3
//     stages, 4: 64 -> 128 transition wgrad at 1024 blocks, 8: 7x7x512 wgrad on
//     128x128, 16: 28x28x128 dgrad variant 27,
//     32: 3x3 256x256 dgrads with the register epilogue (14, not 45).
//     Default 48 (16 | 32; bit 32 since round 5): each wgrad rule wins
//     alone (tools/tune_bconv.py --batch 1024) but costs 0.4-0.9 % of the E18
//     step, where those kernels overlap the data-gradient chain on the side
//     stream (bench A/B, 40 steps each: none 43.7k, 1 43.5k, 2 43.5k, 4 43.6k,
//     8 43.3k, 16 43.8k img/s).
//   deterministic (key 2): split-K weight gradients through slabs reduced in
//     a fixed order (no float atomics).
//   dgrad_rw (key 3): the row-window kernel (conv3rw.hip, variant 50) for the
//     64 -> 64 stride-1 3x3 data gradient by default.
int g_opt_tile_huge = 48;
int g_opt_deterministic = 0;
int g_opt_dgrad_rw = 1;
// wgrad_slab_mb (key 5): cap on the split-K slab bytes of one weight gradient
// (splits <= cap / |dW|); 0 = no cap (splits from the block target alone).
// Default 32 MB (ops/options.py has the measurements).
int g_opt_wgrad_slab_mb = 32;
// lab only (key 9): the fp4 forward skips its int16 y stores (statistics only)
int g_opt_lab_fwd_no_y = 0;
// dgrad_deep (key 6): the phased kernel (deep_gemm.hip, variant 60) for
// stride-1 3x3 data gradients with Cin % 256 == 0 (igemm_dgrad_impl): 1 for
// the float convs, 2 also for the binary (STE-mask) ones, 0 never.
int g_opt_dgrad_deep = 1;
// wgrad_deep (key 7): the same for stride-1 3x3 weight gradients with
// Cin % 256 == 0 and Cout % 256 == 0 (variant 60 of the wgrad dispatch).
int g_opt_wgrad_deep = 1;
// epilogue_prefetch (key 8): the LDS-epilogue dgrad prefetches its residual /
// BN-input loads in groups of 4 chunks before they are needed.
int g_opt_epilogue_prefetch = 1;
// wgrad_tree (key 10): split-K weight gradients combined inside the launch
// by the fixed-order tree (splitk_tree.h) instead of slab + wgrad_reduce_kernel
// (off by default: ~1 % slower in the E18 step, profiles/r6/wgrad_tree.md).
int g_opt_wgrad_tree = 0;

// splits limited by the slab cap (plan_wgrad / plan_wgrad3)
inline long long cap_splits(long long splits, long long dw_bytes) {
  if (g_opt_wgrad_slab_mb <= 0 || dw_bytes <= 0) return splits;
  long long cap = ((long long)g_opt_wgrad_slab_mb << 20) / dw_bytes;
  if (cap < 1) cap = 1;
  return splits < cap ? splits : cap;
}

bool huge_tiles_env(int bit = 31) { return (g_opt_tile_huge & bit) != 0; }

// Reduce-scatter of 32 values over the 32 lanes of each wave half: after
// the 5 butterfly steps lane r holds the half's total of value r (31
// exchanges per lane instead of 32 full 5-step reductions).
template <int N>
__device__ __forceinline__ void rs_step(float (&v)[32], int r32) {
  constexpr int OFF = N;  // exchange distance == values kept
  const bool upper = (r32 & OFF) != 0;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const float send = upper ? v[i] : v[i + N];
    const float keep = upper ? v[i + N] : v[i];
    v[i] = keep + __shfl_xor(send, OFF, 64);
  }
}

// dgrad epilogue for one 32-channel block of a wave's tile (lane = pixel,
// 4 consecutive channels per register group): STE mask, + residual
// gradient, bf16 dx, and (args.psums) the fused BN-backward sums of the
// stored values.  pix[a] < 0: no pixel for this lane in row-group a.
template <int TM>
__device__ __forceinline__ void dgrad_store_block(const ConvArgs& args, const IGeom& g,
                                                  const f32x16 (&acc)[TM], const long long (&pix)[TM],
                                                  int nb, int h, int r32) {
  uint16_t* dx = reinterpret_cast<uint16_t*>(args.out);
  const int CW = g.Cin >> 5;
  uint32_t mw[TM];
#pragma unroll
  for (int a = 0; a < TM; ++a)
    mw[a] = (args.mask && pix[a] >= 0) ? args.mask[pix[a] * CW + (nb >> 5)] : 0xFFFFFFFFu;
  // channel-major copies [2][Cin][stripes] (zk_bn_bwd_coef)
  float* ps = nullptr;
  if (args.psums) ps = args.psums + (args.stripes > 1 ? blockIdx.x % args.stripes : 0);
  float vals[32];  // value j = s*16 + q*4 + e: sum (s = 0) / sum * yhat (s = 1) of channel (q, e)
#pragma unroll
  for (int j = 0; j < 32; ++j) vals[j] = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int nl = 8 * q + 4 * h;
    float mu[4] = {0.f, 0.f, 0.f, 0.f}, rs[4] = {0.f, 0.f, 0.f, 0.f};
    if (ps) {
      const float4 m4 = *reinterpret_cast<const float4*>(args.pmean + nb + nl);
      const float4 r4 = *reinterpret_cast<const float4*>(args.prstd + nb + nl);
      mu[0] = m4.x; mu[1] = m4.y; mu[2] = m4.z; mu[3] = m4.w;
      rs[0] = r4.x; rs[1] = r4.y; rs[2] = r4.z; rs[3] = r4.w;
    }
#pragma unroll
    for (int a = 0; a < TM; ++a) {
      if (pix[a] < 0) continue;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = ((mw[a] >> (nl + e)) & 1u) ? acc[a][4 * q + e] : 0.f;
      const long long off = pix[a] * g.Cin + nb + nl;
      if (args.dres) {
        const uint2 d = *reinterpret_cast<const uint2*>(args.dres + off);
        v[0] += zk::bf16_to_f32((uint16_t)(d.x & 0xffff));
        v[1] += zk::bf16_to_f32((uint16_t)(d.x >> 16));
        v[2] += zk::bf16_to_f32((uint16_t)(d.y & 0xffff));
        v[3] += zk::bf16_to_f32((uint16_t)(d.y >> 16));
      }
      const uint2 o = make_uint2(zk::pack_bf16x2(v[0], v[1]), zk::pack_bf16x2(v[2], v[3]));
      *reinterpret_cast<uint2*>(dx + off) = o;
      if (ps) {
        const uint2 yv = *reinterpret_cast<const uint2*>(args.ypred + off);
        const int16_t* yy = reinterpret_cast<const int16_t*>(&yv);
        const uint32_t ow[2] = {o.x, o.y};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float gv = zk::bf16_to_f32((uint16_t)(ow[e >> 1] >> (16 * (e & 1))));  // as stored
          vals[q * 4 + e] += gv;
          vals[16 + q * 4 + e] += gv * ((float)yy[e] - mu[e]) * rs[e];
        }
      }
    }
  }
  if (ps) {
    // the 32 lanes of a wave half hold the same 16 channels (other pixels)
    rs_step<16>(vals, r32);
    rs_step<8>(vals, r32);
    rs_step<4>(vals, r32);
    rs_step<2>(vals, r32);
    rs_step<1>(vals, r32);
    const int c = nb + 8 * ((r32 >> 2) & 3) + 4 * h + (r32 & 3);
    atomicAdd(ps + (long long)((r32 >> 4) * g.Cin + c) * args.stripes, vals[0]);
  }
}

// Coalesced dgrad epilogue through LDS (LE variants; no fused BN sums).
// The masked fp32 fragments (lane = pixel, 4 consecutive channels per
// register group) are staged half a tile of pixel rows at a time (row
// groups a < TM/2, then the rest: [BM/2][BN] fp32 = BM * BN * 2 bytes,
// 16-B chunk k of staged row r at slot k ^ (r % (BN/4))); then each thread
// moves 8 channels = one 16-B bf16 chunk, consecutive lanes along a pixel
// row, so dx stores and residual-gradient loads are whole contiguous rows
// instead of 8 B per lane spread over 32 rows.  Same arithmetic as the
// register epilogue (masked fp32 + residual, one rounding).  pix(m) maps a
// tile row to its pixel.  The ring is free once every wave is past its last
// fragment read (first barrier).
template <int BM, int BN, int WM, int NT, int TM, int TN, bool EPF, typename PixFn>
__device__ __forceinline__ void dgrad_store_lds(const ConvArgs& args, const IGeom& g,
                                                const f32x16 (&acc)[TM][TN], unsigned char* smem,
                                                long long m0, long long M, int n0, int wm,
                                                int wcol0, int h, int r32, int tid, PixFn pix) {
  constexpr int WTM = BM / WM, HT = TM / 2;
  constexpr int NCH = BN / 4;  // 16-B fp32 chunks per staged row
  static_assert(TM % 2 == 0 && (NCH & (NCH - 1)) == 0 && NCH >= 8, "LDS epilogue tiling");
  const uint32_t* mask = args.mask;
  uint32_t mw[TM][TN];
  if (mask) {
    const int CW = g.Cin >> 5;
#pragma unroll
    for (int a = 0; a < TM; ++a) {
      const long long m = m0 + wm * WTM + a * 32 + r32;
      const bool live = m < M;
      const long long pm = live ? pix(m) : 0;
#pragma unroll
      for (int b = 0; b < TN; ++b)
        mw[a][b] = live ? mask[pm * CW + ((n0 + wcol0 + b * 32) >> 5)] : 0u;
    }
  }
  uint16_t* dx = reinterpret_cast<uint16_t*>(args.out);
  const uint16_t* dres = args.dres;
  // args.fstats / args.bsums: this thread's 8 channels are fixed (NT is a
  // multiple of BN/8)
  static_assert(NT % (BN / 8) == 0, "LDS epilogue: fixed channel chunk per thread");
  const bool fst = args.fstats != nullptr;
  const bool bsm = args.bsums != nullptr;
  float fs1[8], fs2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) fs1[k] = fs2[k] = 0.f;
  // bsums: the BN coefficients of this thread's 8 channels
  float bsc[8], bsh[8], bmu[8], brs[8];
  if (bsm) {
    const int c0 = n0 + 8 * (tid % (BN / 8));
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      bsc[k] = args.bcoef[c0 + k];
      bsh[k] = args.bcoef[g.Cin + c0 + k];
      bmu[k] = args.bcoef[2 * g.Cin + c0 + k];
      brs[k] = args.bcoef[3 * g.Cin + c0 + k];
    }
  }
  // the store pass of a half tile: ITER 16-B chunks per thread; their
  // residual-gradient / BN-input loads are issued before the half is staged
  // (latency hidden behind the staging and the barrier instead of exposed
  // once per chunk)
  constexpr int ITER = (BM / 2) * (BN / 8) / NT;
  static_assert((BM / 2) * (BN / 8) % NT == 0, "LDS epilogue: chunks per thread");
  // chunks whose loads are in flight together (EPF off: one, as loaded at use)
  constexpr int PF = !EPF ? 1 : ITER > 4 ? 4 : ITER;
  static_assert(ITER % PF == 0, "LDS epilogue: prefetch groups");
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    long long offs[PF];
    uint4 dq[PF], xq[PF];
    uint32_t mq[PF], dm[PF];
    // loads of chunks it0 .. it0 + PF - 1
    auto prefetch = [&](int it0) {
#pragma unroll
      for (int u = 0; u < PF; ++u) {
        const int i = tid + (it0 + u) * NT;
        const int lr = i / (BN / 8), j = i % (BN / 8);
        const int row = (lr / (WTM / 2)) * WTM + (p * HT + (lr % (WTM / 2)) / 32) * 32 + lr % 32;
        const long long m = m0 + row;
        offs[u] = m < M ? pix(m) * g.Cin + n0 + 8 * j : -1;
        const long long o = offs[u] < 0 ? 0 : offs[u];
        dq[u] = (dres && offs[u] >= 0) ? *reinterpret_cast<const uint4*>(dres + o)
                                       : make_uint4(0u, 0u, 0u, 0u);
        xq[u] = (bsm && offs[u] >= 0) ? *reinterpret_cast<const uint4*>(args.bxb + o)
                                      : make_uint4(0u, 0u, 0u, 0u);
        mq[u] = (bsm && args.brelu == 2 && offs[u] >= 0) ? args.bmask[o >> 3] : 0xFFu;
        dm[u] = (args.dmask && offs[u] >= 0) ? args.dmask[o >> 3] : 0xFFu;
      }
    };
    prefetch(0);
    __syncthreads();  // the ring (p = 0) / the previous half's tile is free
#pragma unroll
    for (int aa = 0; aa < HT; ++aa) {
      const int a = p * HT + aa;
      const int lr = wm * (WTM / 2) + aa * 32 + r32;
      unsigned char* rb = smem + lr * (BN * 4);
      const int sw = lr & (NCH - 1);
#pragma unroll
      for (int b = 0; b < TN; ++b) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int nl = 8 * q + 4 * h;
          float4 v;
          float* vp = reinterpret_cast<float*>(&v);
#pragma unroll
          for (int e = 0; e < 4; ++e)
            vp[e] = (!mask || ((mw[a][b] >> (nl + e)) & 1u)) ? acc[a][b][4 * q + e] : 0.f;
          const int k = (wcol0 + b * 32 + nl) >> 2;
          *reinterpret_cast<float4*>(rb + ((k ^ sw) << 4)) = v;
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
      const int u = it % PF;
      if (u == 0 && it > 0) prefetch(it);
      const int i = tid + it * NT;
      const int lr = i / (BN / 8), j = i % (BN / 8);
      const long long off = offs[u];
      if (off < 0) continue;
      const unsigned char* rb = smem + lr * (BN * 4);
      const int sw = lr & (NCH - 1);
      const float4 f0 = *reinterpret_cast<const float4*>(rb + (((2 * j) ^ sw) << 4));
      const float4 f1 = *reinterpret_cast<const float4*>(rb + (((2 * j + 1) ^ sw) << 4));
      float v[8] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
      if (dres) {
        const uint4 d = dq[u];
        const uint32_t dd[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float lo = zk::bf16_to_f32((uint16_t)(dd[k] & 0xffff));
          const float hi = zk::bf16_to_f32((uint16_t)(dd[k] >> 16));
          v[2 * k] += (dm[u] >> (2 * k)) & 1u ? lo : 0.f;
          v[2 * k + 1] += (dm[u] >> (2 * k + 1)) & 1u ? hi : 0.f;
        }
      }
      const uint4 o = make_uint4(zk::pack_bf16x2(v[0], v[1]), zk::pack_bf16x2(v[2], v[3]),
                                 zk::pack_bf16x2(v[4], v[5]), zk::pack_bf16x2(v[6], v[7]));
      *reinterpret_cast<uint4*>(dx + off) = o;
      if (bsm) {
        // the BN-backward sums over the stored gradient (zk_bn_bwd_reduce of
        // the BN whose output this dx is the whole gradient of)
        const uint32_t xw[4] = {xq[u].x, xq[u].y, xq[u].z, xq[u].w};
        const uint32_t ow[4] = {o.x, o.y, o.z, o.w};
        const uint32_t mb = mq[u];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float xk = zk::bf16_to_f32((uint16_t)(xw[k >> 1] >> (16 * (k & 1))));
          float gk = zk::bf16_to_f32((uint16_t)(ow[k >> 1] >> (16 * (k & 1))));  // as stored
          // ReLU mask as the forward stored it: bf16(scale * x + shift) > 0
          // (norm_pool.hip bn_pre / relu_live), or the stored bits
          const bool live = args.brelu == 1
                                ? (int16_t)zk::f32_to_bf16(bsc[k] * xk + bsh[k] + 0.f) > 0
                                : ((mb >> k) & 1u) != 0;
          gk = live ? gk : 0.f;
          fs1[k] += gk;
          fs2[k] += gk * (xk - bmu[k]) * brs[k];
        }
      }
      if (fst) {
        const uint32_t ow[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float r = zk::bf16_to_f32((uint16_t)(ow[k >> 1] >> (16 * (k & 1))));  // as stored
          fs1[k] += r;
          fs2[k] += r * r;
        }
      }
    }
  }
  if (bsm) {
    // as the statistics below, into this M tile's fp32 channel-major copy
    constexpr int JC = BN / 8, RPT = NT / JC;
    static_assert(NT * 16 * 4 <= BM * BN * 2, "LDS epilogue: sums exchange");
    float* red = reinterpret_cast<float*>(smem);
    __syncthreads();  // every thread is past its staged-tile reads
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      red[tid * 16 + k] = fs1[k];
      red[tid * 16 + 8 + k] = fs2[k];
    }
    __syncthreads();
    const long long copy = m0 / BM;  // this block's M tile (stride 1: one parity class)
    for (int c = tid; c < 2 * BN; c += NT) {
      const int which = c / BN, nl = c % BN, j = nl >> 3, k = nl & 7;
      float t = 0.f;
#pragma unroll 4
      for (int r = 0; r < RPT; ++r) t += red[(r * JC + j) * 16 + which * 8 + k];
      args.bsums[(copy * 2 + which) * g.Cin + n0 + nl] = t;
    }
  }
  if (fst) {
    // threads tid = r * JC + j hold chunk j: sum their rows through LDS
    // (16 floats per thread), then one fp64 atomic per channel and statistic
    constexpr int JC = BN / 8, RPT = NT / JC;
    static_assert(NT * 16 * 4 <= BM * BN * 2, "LDS epilogue: statistics exchange");
    float* red = reinterpret_cast<float*>(smem);
    __syncthreads();  // every thread is past its staged-tile reads
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      red[tid * 16 + k] = fs1[k];
      red[tid * 16 + 8 + k] = fs2[k];
    }
    __syncthreads();
    const int stripe = args.stripes > 1 ? (int)(blockIdx.x % args.stripes) : 0;
    double* so = args.fstats + (long long)stripe * 2 * g.Cin;
    for (int c = tid; c < 2 * BN; c += NT) {
      const int which = c / BN, nl = c % BN, j = nl >> 3, k = nl & 7;
      float t = 0.f;
#pragma unroll 4
      for (int r = 0; r < RPT; ++r) t += red[(r * JC + j) * 16 + which * 8 + k];
      // the block's partial rounded to a fixed grid (2^-20 for sums, 2^-8 for
      // sums of squares): every addend is an integer number of grid units and
      // the totals stay far below 2^53 units, so the fp64 atomics are exact
      // and their order cannot change the statistics (bit-reproducible)
      const double q = which ? 256.0 : 1048576.0;
      atomicAdd(so + which * g.Cin + n0 + nl, rint((double)t * q) / q);
    }
  }
}

template <bool FWD, int BM, int BN, int WM, int WN, int NS, int CB, bool F4 = false,
          bool OB = false, bool LE = false, bool EPF = true>
__global__ __launch_bounds__(WM * WN * 64, 1) void igemm_conv_kernel(ConvArgs args, IGeom g,
                                                                     int m_tiles) {
  constexpr int NWAVES = WM * WN;
  // CB = bytes of K per row per stage (128 = 64 bf16, 64, or 32)
  constexpr int SPR = CB / 16;            // 16-B slots per row
  constexpr int RPI = 1024 / CB;          // rows per wave-instruction
  constexpr int SH = (CB == 128) ? 1 : (CB == 64) ? 2 : 3;  // swizzle shift (see header)
  static_assert(!F4 || FWD, "e2m1 operands: the +-1 x +-1 forward only");
  static_assert(!OB || (FWD && !F4), "bf16 output: the float (bf16 x bf16) forward");
  constexpr int A_INS = BM / RPI / NWAVES;  // glds per wave per stage
  constexpr int B_INS = BN / RPI / NWAVES;
  static_assert(A_INS >= 1 && B_INS >= 1 && BM % (RPI * NWAVES) == 0 &&
                    BN % (RPI * NWAVES) == 0,
                "tile / wave mismatch");
  constexpr int LPS = A_INS + B_INS;  // vm ops per wave per stage
  constexpr int STAGE = (BM + BN) * CB;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  static_assert(!FWD || TM <= 4, "in-wave int32 sums of squares need TM <= 4");

  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int wm = wave / WN, wn = wave % WN;
  const int NCH = FWD ? g.Cout : g.Cin;   // GEMM N
  const int KCH = FWD ? g.Cin : g.Cout;   // channels per tap along K

  // ---- tile coordinates (XCD-aware: the M tiles of one N tile are
  // consecutive logical ids, so they share an L2 with that N tile's weights)
  const int nwg = gridDim.x;
  const int L = xcd_linear(blockIdx.x, nwg);
  const int n_tiles = NCH / BN;
  const int mtile = L % m_tiles;
  const int ntile = L / m_tiles;
  if (ntile >= n_tiles) return;
  const int s = g.s;
  const int ph = FWD ? 0 : blockIdx.y / s, pw = FWD ? 0 : blockIdx.y % s;
  const int Hc = FWD ? g.Ho : (g.H - ph + s - 1) / s;
  const int Wc = FWD ? g.Wo : (g.W - pw + s - 1) / s;
  const long long M = (long long)g.B * Hc * Wc;
  const long long m0 = (long long)mtile * BM;
  if (m0 >= M) return;
  const int n0 = ntile * BN;

  // taps: all of them (fwd) or those of this parity class (dgrad):
  // th = th0 + i*s (no runtime-indexed arrays, which would live in scratch)
  const int ts = FWD ? 1 : s;
  const int th0 = FWD ? 0 : (ph + g.pt) % s, tw0 = FWD ? 0 : (pw + g.pl) % s;
  const int nth = (g.kh - th0 + ts - 1) / ts, ntw = (g.kw - tw0 + ts - 1) / ts;
  const int T = nth * ntw;
  const int RB = F4 ? KCH / 2 : KCH * 2;  // bytes per activation / weight row
  const int kchunks = RB / CB;
  const int NK = T * kchunks;

  // ---- per-lane loader rows (A: pixels).  Every tap of a row is the row's
  // tap-0 source plus a uniform offset (fwd: +(ih*W + iw) pixels, dgrad:
  // -(ih*Wo + iw) pixels), valid iff bit ih of a_hm and bit iw of a_wm are
  // set: the per-tap address work is a shift, an and and a select.
  const int lrow = lane / SPR, lslot = lane % SPR;
  const unsigned char* actb = reinterpret_cast<const unsigned char*>(args.act);
  const unsigned char* wtb = reinterpret_cast<const unsigned char*>(args.wgt);
  const unsigned char* zp = reinterpret_cast<const unsigned char*>(g_zero_page);
  const unsigned char* padp =
      (FWD && args.pad_ones)
          ? (F4 ? reinterpret_cast<const unsigned char*>(g_ones_page_fp4)
                : reinterpret_cast<const unsigned char*>(g_ones_page_bf16))
          : zp;
  const unsigned char* a_base[A_INS];  // tap-0 source (may point outside: masked)
  const unsigned char* a_pad[A_INS];   // padding page (+ swizzled slot)
  uint32_t a_hm[A_INS], a_wm[A_INS];
#pragma unroll
  for (int j = 0; j < A_INS; ++j) {
    const int r = (j * NWAVES + wave) * RPI + lrow;
    const int sw = lslot ^ ((r >> SH) & (SPR - 1));
    const long long m = m0 + r;
    a_hm[j] = a_wm[j] = 0;
    a_base[j] = zp;
    a_pad[j] = zp + sw * 16;  // tail rows: zeros
    if (m < M) {
      const int jw = (int)(m % Wc);
      const long long rr = m / Wc;
      const int jh = (int)(rr % Hc);
      const int b = (int)(rr / Hc);
      a_pad[j] = padp + sw * 16;
      if (FWD) {
        const int h0 = jh * s - g.pt + th0, w0 = jw * s - g.pl + tw0;
        for (int i = 0; i < nth; ++i) a_hm[j] |= (uint32_t)(h0 + i >= 0 && h0 + i < g.H) << i;
        for (int i = 0; i < ntw; ++i) a_wm[j] |= (uint32_t)(w0 + i >= 0 && w0 + i < g.W) << i;
        a_base[j] = actb + (((long long)b * g.H + h0) * g.W + w0) * RB + sw * 16;
      } else {
        // tap index i: ho = (jh*s + ph + pt - th0)/s - i
        const int ho0 = (jh * s + ph + g.pt - th0) / s, wo0 = (jw * s + pw + g.pl - tw0) / s;
        for (int i = 0; i < nth; ++i) a_hm[j] |= (uint32_t)(ho0 - i >= 0 && ho0 - i < g.Ho) << i;
        for (int i = 0; i < ntw; ++i) a_wm[j] |= (uint32_t)(wo0 - i >= 0 && wo0 - i < g.Wo) << i;
        a_base[j] = actb + (((long long)b * g.Ho + ho0) * g.Wo + wo0) * RB + sw * 16;
      }
    }
  }
  int b_sw[B_INS];
#pragma unroll
  for (int j = 0; j < B_INS; ++j) {
    const int r = (j * NWAVES + wave) * RPI + lrow;
    b_sw[j] = lslot ^ ((r >> SH) & (SPR - 1));
  }

  // Source pointers of the current tap (recomputed when the tap changes).
  const unsigned char* a_src[A_INS];
  int a_step[A_INS];  // CB for a real row, 0 for a padding page
  const unsigned char* b_src[B_INS];
  auto set_tap = [&](int ti) {
    const int ih = ti / ntw, iw = ti % ntw;
    const int th = th0 + ih * ts, tw = tw0 + iw * ts;
    const int t = th * g.kw + tw;
    const long long off =
        (FWD ? ((long long)ih * g.W + iw) : -((long long)ih * g.Wo + iw)) * RB;
#pragma unroll
    for (int j = 0; j < A_INS; ++j) {
      const bool ok = (a_hm[j] >> ih) & (a_wm[j] >> iw) & 1u;
      a_src[j] = ok ? a_base[j] + off : a_pad[j];
      a_step[j] = ok ? CB : 0;
    }
#pragma unroll
    for (int j = 0; j < B_INS; ++j) {
      const int r = (j * NWAVES + wave) * RPI + lrow;
      b_src[j] = wtb + ((long long)t * NCH + n0 + r) * RB + b_sw[j] * 16;
    }
  };
  // Issue the glds of K-step ks into ring slot ks % NS.
  int cur_tap = -1;
  auto issue = [&](int ks) {
    const int ti = ks / kchunks, kc = ks % kchunks;
    if (ti != cur_tap) {
      set_tap(ti);
      cur_tap = ti;
    }
    unsigned char* st = smem + (ks % NS) * STAGE;
    const int koff = kc * CB;
#pragma unroll
    for (int j = 0; j < A_INS; ++j)
      ZK_GLDS16(a_src[j] + kc * a_step[j], st + (j * NWAVES + wave) * 1024);
#pragma unroll
    for (int j = 0; j < B_INS; ++j)
      ZK_GLDS16(b_src[j] + koff, st + BM * CB + (j * NWAVES + wave) * 1024);
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  const int r32 = lane & 31, h = lane >> 5;
  // fragment read offsets (bytes within a stage) for k-substep 0
  int a_off[TM], b_off[TN];
#pragma unroll
  for (int a = 0; a < TM; ++a) a_off[a] = (wm * WTM + a * 32 + r32) * CB;
#pragma unroll
  for (int b = 0; b < TN; ++b) b_off[b] = BM * CB + (wn * WTN + b * 32 + r32) * CB;

  // prologue: NS-1 stages in flight
#pragma unroll
  for (int p = 0; p < NS - 1; ++p)
    if (p < NK) issue(p);

  for (int ks = 0; ks < NK; ++ks) {
    // wait for this wave's loads of stage ks, then the barrier makes every
    // wave's loads visible and frees slot (ks-1) % NS for re-issue.
    if (ks + NS - 2 < NK)
      wait_vmcnt<LPS * (NS - 2)>();
    else
      wait_vmcnt<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (ks + NS - 1 < NK) issue(ks + NS - 1);

    const unsigned char* st = smem + (ks % NS) * STAGE;
    // fragment reads are double-buffered across the k-substeps: the reads of
    // substep sub+1 are in flight while the MFMAs of substep sub issue.
    constexpr int NSUB = CB / 32;
    uint4 af[2][TM], bfr[2][TN];
    auto read_frags = [&](int sub, int set) {
      const int chunk = 2 * sub + h;
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        const int row = wm * WTM + a * 32 + r32;
        af[set][a] = *reinterpret_cast<const uint4*>(
            st + a_off[a] + ((chunk ^ ((row >> SH) & (SPR - 1))) * 16));
      }
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int row = wn * WTN + b * 32 + r32;
        bfr[set][b] = *reinterpret_cast<const uint4*>(
            st + b_off[b] + ((chunk ^ ((row >> SH) & (SPR - 1))) * 16));
      }
    };
    read_frags(0, 0);
#pragma unroll
    for (int sub = 0; sub < NSUB; ++sub) {
      if (sub + 1 < NSUB) read_frags(sub + 1, (sub + 1) & 1);
      // keep the next substep's reads ahead of this substep's MFMAs (the
      // scheduler would otherwise sink them to reuse the registers)
      __builtin_amdgcn_sched_barrier(0);
      const int cs = sub & 1;
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b)
          // fwd: D[pixel][co] (lane = channel: in-lane BN statistics);
          // dgrad: D[ci][pixel] (lane = pixel: 8-B mask/residual epilogue)
          acc[a][b] = FWD ? (F4 ? mfma_fp4(af[cs][a], bfr[cs][b], acc[a][b])
                                : mfma_bf16(af[cs][a], bfr[cs][b], acc[a][b]))
                          : mfma_bf16(bfr[cs][b], af[cs][a], acc[a][b]);
    }
  }

  if constexpr (FWD && OB) {
    // ---- float forward epilogue: bf16 y (+ReLU), lane = output channel,
    // registers = pixels (64-B contiguous per wave half and register)
    uint16_t* y = reinterpret_cast<uint16_t*>(args.out);
#pragma unroll
    for (int a = 0; a < TM; ++a) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const long long mc = m0 + wm * WTM + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (mc >= M) continue;
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          float v = acc[a][b][r];
          if (args.relu) v = fmaxf(v, 0.f);
          y[mc * g.Cout + n0 + wn * WTN + b * 32 + r32] = zk::f32_to_bf16(v);
        }
      }
    }
  } else if constexpr (FWD) {
    // ---- forward epilogue: lane = output channel, registers = pixels;
    // the fp32 accumulators hold exact integers (|v| <= K)
    int16_t* y = reinterpret_cast<int16_t*>(args.out);
    int csum[TN], csq[TN];
#pragma unroll
    for (int b = 0; b < TN; ++b) csum[b] = csq[b] = 0;
#pragma unroll
    for (int a = 0; a < TM; ++a) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const long long mc = m0 + wm * WTM + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const bool live = mc < M;
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          int t = (int)acc[a][b][r];
          if (args.relu) t = t > 0 ? t : 0;
          if (!live) t = 0;
          csum[b] += t;
          csq[b] += t * t;  // < 2^32 as unsigned for TM <= 4, K <= 4608
          if (live && y) y[mc * g.Cout + n0 + wn * WTN + b * 32 + r32] = (int16_t)t;
        }
      }
    }
    // statistics: the two wave halves hold the same channels, then the WM
    // waves sharing these channels combine in LDS; one int64 atomic each.
    __builtin_amdgcn_s_barrier();  // all waves are done with the ring
    int* red = reinterpret_cast<int*>(smem);  // [WM][2][BN]
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int s1 = csum[b] + __shfl_xor(csum[b], 32, 64);
      const int s2 = csq[b] + __shfl_xor(csq[b], 32, 64);
      if (h == 0) {
        const int nl = wn * WTN + b * 32 + r32;
        red[(wm * 2 + 0) * BN + nl] = s1;
        red[(wm * 2 + 1) * BN + nl] = s2;
      }
    }
    __syncthreads();
    // striped copies: thousands of blocks adding into one [2][Cout] array
    // serialise on its cache lines (the stage-1 forward was bound by it)
    const int stripe = args.stripes > 1 ? (int)(blockIdx.x % args.stripes) : 0;
    unsigned long long* st_out = args.stats + (long long)stripe * 2 * g.Cout;
    for (int c = tid; c < 2 * BN; c += NWAVES * 64) {
      const int which = c / BN, nl = c % BN;
      long long tot = 0;
#pragma unroll
      for (int i = 0; i < WM; ++i) {
        const int v = red[(i * 2 + which) * BN + nl];
        tot += which ? (long long)(unsigned int)v : (long long)v;  // squares: unsigned
      }
      atomicAdd(st_out + which * g.Cout + n0 + nl, (unsigned long long)tot);
    }
  } else {
    // ---- dgrad epilogue: lane = pixel, 4 consecutive channels per group
    if (args.psums) {
      // + the previous block's fused BN-backward sums (dgrad_store_block)
      long long pix[TM];
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        const long long mc = m0 + wm * WTM + a * 32 + r32;
        pix[a] = -1;
        if (mc < M) {
          const int jw = (int)(mc % Wc);
          const long long rr = mc / Wc;
          pix[a] = ((rr / Hc) * g.H + (long long)(rr % Hc) * s + ph) * g.W + (long long)jw * s + pw;
        }
      }
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        f32x16 ab[TM];
#pragma unroll
        for (int a = 0; a < TM; ++a) ab[a] = acc[a][b];
        dgrad_store_block<TM>(args, g, ab, pix, n0 + wn * WTN + b * 32, h, r32);
      }
    } else if constexpr (LE) {
      static_assert(BM * BN * 2 <= NS * STAGE, "LDS epilogue: the ring holds half the tile");
      const int W = g.W, H = g.H;
      dgrad_store_lds<BM, BN, WM, NWAVES * 64, TM, TN, EPF>(
          args, g, acc, smem, m0, M, n0, wm, wn * WTN, h, r32, tid,
          [=](long long mc) -> long long {
            if (s == 1) return mc;
            const int jw = (int)(mc % Wc);
            const long long rr = mc / Wc;
            return ((rr / Hc) * H + (long long)(rr % Hc) * s + ph) * W + (long long)jw * s + pw;
          });
    } else {
      uint16_t* dx = reinterpret_cast<uint16_t*>(args.out);
      const uint32_t* mask = args.mask;
      const uint16_t* dres = args.dres;
      const int CW = g.Cin >> 5;
      // all mask / residual loads of the tile before the stores (see the
      // conv3 epilogue)
      long long pix[TM];
      uint32_t mw[TM][TN];
      uint2 dv[TM][TN][4];
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        const long long mc = m0 + wm * WTM + a * 32 + r32;
        pix[a] = -1;
        if (mc < M) {
          const int jw = (int)(mc % Wc);
          const long long rr = mc / Wc;
          pix[a] = ((rr / Hc) * g.H + (long long)(rr % Hc) * s + ph) * g.W + (long long)jw * s + pw;
        }
        const long long m = pix[a];
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          const int nb = n0 + wn * WTN + b * 32;
          mw[a][b] = !mask ? 0xFFFFFFFFu : m >= 0 ? mask[m * CW + (nb >> 5)] : 0u;
#pragma unroll
          for (int q = 0; q < 4; ++q)
            dv[a][b][q] = (dres && m >= 0)
                              ? *reinterpret_cast<const uint2*>(dres + m * g.Cin + nb + 8 * q + 4 * h)
                              : make_uint2(0u, 0u);
        }
      }
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        const long long m = pix[a];
        if (m < 0) continue;
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          const int nb = n0 + wn * WTN + b * 32;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int nl = 8 * q + 4 * h;
            float v[4];
#pragma unroll
            for (int e = 0; e < 4; ++e)
              v[e] = ((mw[a][b] >> (nl + e)) & 1u) ? acc[a][b][4 * q + e] : 0.f;
            const uint2 d = dv[a][b][q];  // zero without a residual
            v[0] += zk::bf16_to_f32((uint16_t)(d.x & 0xffff));
            v[1] += zk::bf16_to_f32((uint16_t)(d.x >> 16));
            v[2] += zk::bf16_to_f32((uint16_t)(d.y & 0xffff));
            v[3] += zk::bf16_to_f32((uint16_t)(d.y >> 16));
            *reinterpret_cast<uint2*>(dx + m * g.Cin + nb + nl) =
                make_uint2(zk::pack_bf16x2(v[0], v[1]), zk::pack_bf16x2(v[2], v[3]));
          }
        }
      }
    }
  }
}

// ===========================================================================
// 3x3 stride-1 'same' convolutions with horizontal tap reuse ("conv3").
//
// The three taps tw of one kernel row th read the SAME activation rows
// shifted by one pixel: with pixels flattened over (b, h, w), tap (th, tw)
// of output pixel m reads row m + dh(th)*W + dw(tw), dw in {-1, 0, 1}.  So a
// K-step loads BM + 2 activation rows ONCE (plus the three taps' weight
// rows) and the MFMAs of tap tw read LDS rows shifted by dw + 1 — a third of
// the activation LDS-fill bytes of igemm_conv_kernel.  Rows that belong to
// another image row / image (left/right/top/bottom padding) are loaded
// unconditionally and their fragments zeroed per lane (validity bit masks).
//   FWD:  q = m + (th-1)*W + (tw-1)       DGRAD: q = m + (1-th)*W + (1-tw)
// ===========================================================================
template <bool FWD, int BM, int BN, int WM, int WN, int NS, int CB, bool F4 = false>
__global__ __launch_bounds__(WM * WN * 64, 1) void igemm_conv3_kernel(ConvArgs args, IGeom g,
                                                                      int m_tiles) {
  constexpr int NWAVES = WM * WN;
  constexpr int SPR = CB / 16, RPI = 1024 / CB, SH = (CB == 128) ? 1 : (CB == 64) ? 2 : 3;
  static_assert(!F4 || FWD, "e2m1 operands: the +-1 x +-1 forward only");
  constexpr int A_INS = (BM + 2 + RPI * NWAVES - 1) / (RPI * NWAVES);  // glds per wave
  constexpr int AR = A_INS * RPI * NWAVES;                             // A rows staged
  // weight rows of the three taps, padded to whole load instructions (the
  // tail lanes load the zero page into the pad rows)
  constexpr int B_INS = (3 * BN + RPI * NWAVES - 1) / (RPI * NWAVES);
  constexpr int BR = B_INS * RPI * NWAVES;
  constexpr int LPS = A_INS + B_INS;
  constexpr int STAGE = (AR + BR) * CB;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  static_assert(!FWD || TM <= 4, "in-wave int32 sums of squares need TM <= 4");

  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave / WN, wn = wave % WN;
  const int NCH = FWD ? g.Cout : g.Cin, KCH = FWD ? g.Cin : g.Cout;
  const int L = xcd_linear(blockIdx.x, gridDim.x);
  const int n_tiles = NCH / BN;
  const int mtile = L % m_tiles, ntile = L / m_tiles;
  if (ntile >= n_tiles) return;
  const int H = g.H, W = g.W;
  const long long M = (long long)g.B * H * W;
  const long long m0 = (long long)mtile * BM;
  if (m0 >= M) return;
  const int n0 = ntile * BN;
  const int RB = F4 ? KCH / 2 : KCH * 2, kchunks = RB / CB, NK = 3 * kchunks;
  const unsigned char* actb = reinterpret_cast<const unsigned char*>(args.act);
  const unsigned char* wtb = reinterpret_cast<const unsigned char*>(args.wgt);
  const unsigned char* zp = reinterpret_cast<const unsigned char*>(g_zero_page);
  const unsigned char* padp =
      (FWD && args.pad_ones) ? reinterpret_cast<const unsigned char*>(g_ones_page_bf16) : zp;
  const int lrow = lane / SPR, lslot = lane % SPR;
  const int r32 = lane & 31, h = lane >> 5;

  // per-lane validity of the wave's output pixels: bit th of vh[a], bit tw of vw[a]
  uint32_t vh[TM], vw[TM];
#pragma unroll
  for (int a = 0; a < TM; ++a) {
    const long long m = m0 + wm * WTM + a * 32 + r32;
    vh[a] = vw[a] = 0;
    if (m < M) {
      const int w = (int)(m % W), hh = (int)((m / W) % H);
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        const int dh = FWD ? t - 1 : 1 - t;
        vh[a] |= (uint32_t)(hh + dh >= 0 && hh + dh < H) << t;
        vw[a] |= (uint32_t)(w + dh >= 0 && w + dh < W) << t;  // dw(t) == dh(t)
      }
    }
  }

  auto issue = [&](int ks) {
    const int th = ks / kchunks, kc = ks % kchunks;
    const int dh = FWD ? th - 1 : 1 - th;
    unsigned char* st = smem + (ks % NS) * STAGE;
    const long long base = m0 + (long long)dh * W - 1;  // LDS row 0
#pragma unroll
    for (int j = 0; j < A_INS; ++j) {
      const int r = (j * NWAVES + wave) * RPI + lrow;
      const int sw = lslot ^ ((r >> SH) & (SPR - 1));
      const long long q = base + r;
      // padding taps / tail rows are masked on the fragments; this only
      // keeps every address inside the tensor
      const unsigned char* src = (q >= 0 && q < M) ? actb + q * RB + kc * CB + sw * 16
                                                   : zp + sw * 16;
      ZK_GLDS16(src, st + (j * NWAVES + wave) * 1024);
    }
#pragma unroll
    for (int j = 0; j < B_INS; ++j) {
      const int r = (j * NWAVES + wave) * RPI + lrow;  // 0 .. BR-1
      const int tw = r / BN, n = r % BN;
      const int t = th * 3 + tw;
      const int sw = lslot ^ ((n >> SH) & (SPR - 1));
      ZK_GLDS16(r < 3 * BN ? wtb + ((long long)t * NCH + n0 + n) * RB + kc * CB + sw * 16
                           : zp + sw * 16,
                st + AR * CB + (j * NWAVES + wave) * 1024);
    }
  };
  (void)padp;
  // value of a padding tap's fragment: 0, or bf16 +1 pairs for pad_values=1
  const uint32_t padv = (FWD && args.pad_ones) ? (F4 ? 0x22222222u : 0x3F803F80u) : 0u;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  // dgrad epilogue operands (STE mask words, residual gradient) are loaded
  // BEFORE the main loop: their HBM latency overlaps the prologue DMAs and
  // the K-steps instead of following the last MFMA (the short-K 64 / 128-
  // channel layers spent a third of each block waiting for them).
  constexpr int PTM = FWD ? 1 : TM, PTN = FWD ? 1 : TN;
  uint32_t pmw[PTM][PTN];
  uint2 pdv[PTM][PTN][4];
  if constexpr (!FWD) {
    if (!args.psums) {
      const uint32_t* mask = args.mask;
      const uint16_t* dres = args.dres;
      const int CW = g.Cin >> 5;
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        const long long m = m0 + wm * WTM + a * 32 + r32;
        const bool live = m < M;
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          const int nb = n0 + wn * WTN + b * 32;
          pmw[a][b] = !mask ? 0xFFFFFFFFu : live ? mask[m * CW + (nb >> 5)] : 0u;
#pragma unroll
          for (int q = 0; q < 4; ++q)
            pdv[a][b][q] = (dres && live)
                               ? *reinterpret_cast<const uint2*>(dres + m * g.Cin + nb + 8 * q + 4 * h)
                               : make_uint2(0u, 0u);
        }
      }
    }
  }

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
    const int th = ks / kchunks;
    uint32_t okh[TM];
#pragma unroll
    for (int a = 0; a < TM; ++a) okh[a] = (vh[a] >> th) & 1u;
    // (tw, substep) flattened, fragment reads double-buffered
    constexpr int NSUB = CB / 32, NIT = 3 * NSUB;
    uint4 af[2][TM], bfr[2][TN];
    auto read_frags = [&](int it, int set) {
      const int tw = it / NSUB, sub = it % NSUB;
      const int chunk = 2 * sub + h;
      const int dw1 = FWD ? tw : 2 - tw;  // dw + 1: LDS row shift of this tap
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        const int row = wm * WTM + a * 32 + r32 + dw1;
        uint4 v = *reinterpret_cast<const uint4*>(
            st + row * CB + ((chunk ^ ((row >> SH) & (SPR - 1))) * 16));
        const bool ok = okh[a] & (vw[a] >> tw) & 1u;
        if (!ok) v = make_uint4(padv, padv, padv, padv);  // padding tap: 0 or +1
        af[set][a] = v;
      }
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int n = wn * WTN + b * 32 + r32;
        bfr[set][b] = *reinterpret_cast<const uint4*>(
            st + AR * CB + (tw * BN + n) * CB + ((chunk ^ ((n >> SH) & (SPR - 1))) * 16));
      }
    };
    read_frags(0, 0);
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      if (it + 1 < NIT) read_frags(it + 1, (it + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
      const int cs = it & 1;
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b)
          acc[a][b] = FWD ? (F4 ? mfma_fp4(af[cs][a], bfr[cs][b], acc[a][b])
                                : mfma_bf16(af[cs][a], bfr[cs][b], acc[a][b]))
                          : mfma_bf16(bfr[cs][b], af[cs][a], acc[a][b]);
    }
  }

  if constexpr (FWD) {
    // ---- forward epilogue (as igemm_conv_kernel): lane = channel
    int16_t* y = reinterpret_cast<int16_t*>(args.out);
    int csum[TN], csq[TN];
#pragma unroll
    for (int b = 0; b < TN; ++b) csum[b] = csq[b] = 0;
#pragma unroll
    for (int a = 0; a < TM; ++a) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const long long mc = m0 + wm * WTM + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const bool live = mc < M;
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          int t = (int)acc[a][b][r];
          if (args.relu) t = t > 0 ? t : 0;
          if (!live) t = 0;
          csum[b] += t;
          csq[b] += t * t;
          if (live && y) y[mc * g.Cout + n0 + wn * WTN + b * 32 + r32] = (int16_t)t;
        }
      }
    }
    __builtin_amdgcn_s_barrier();
    int* red = reinterpret_cast<int*>(smem);  // [WM][2][BN]
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int s1 = csum[b] + __shfl_xor(csum[b], 32, 64);
      const int s2 = csq[b] + __shfl_xor(csq[b], 32, 64);
      if (h == 0) {
        const int nl = wn * WTN + b * 32 + r32;
        red[(wm * 2 + 0) * BN + nl] = s1;
        red[(wm * 2 + 1) * BN + nl] = s2;
      }
    }
    __syncthreads();
    const int stripe = args.stripes > 1 ? (int)(blockIdx.x % args.stripes) : 0;
    unsigned long long* st_out = args.stats + (long long)stripe * 2 * g.Cout;
    for (int c = tid; c < 2 * BN; c += NWAVES * 64) {
      const int which = c / BN, nl = c % BN;
      long long tot = 0;
#pragma unroll
      for (int i = 0; i < WM; ++i) {
        const int v = red[(i * 2 + which) * BN + nl];
        tot += which ? (long long)(unsigned int)v : (long long)v;
      }
      atomicAdd(st_out + which * g.Cout + n0 + nl, (unsigned long long)tot);
    }
  } else {
    // ---- dgrad epilogue (stride 1: the pixel index is the row index)
    if (args.psums) {
      // + the previous block's fused BN-backward sums (dgrad_store_block)
      long long pix[TM];
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        const long long m = m0 + wm * WTM + a * 32 + r32;
        pix[a] = m < M ? m : -1;
      }
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        f32x16 ab[TM];
#pragma unroll
        for (int a = 0; a < TM; ++a) ab[a] = acc[a][b];
        dgrad_store_block<TM>(args, g, ab, pix, n0 + wn * WTN + b * 32, h, r32);
      }
    } else {
      uint16_t* dx = reinterpret_cast<uint16_t*>(args.out);
      // mask words / residual gradient: prefetched before the main loop
      const auto& mw = pmw;
      const auto& dv = pdv;
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        const long long m = m0 + wm * WTM + a * 32 + r32;
        if (m >= M) continue;
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          const int nb = n0 + wn * WTN + b * 32;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int nl = 8 * q + 4 * h;
            float v[4];
#pragma unroll
            for (int e = 0; e < 4; ++e)
              v[e] = ((mw[a][b] >> (nl + e)) & 1u) ? acc[a][b][4 * q + e] : 0.f;
            const uint2 d = dv[a][b][q];  // zero without a residual
            v[0] += zk::bf16_to_f32((uint16_t)(d.x & 0xffff));
            v[1] += zk::bf16_to_f32((uint16_t)(d.x >> 16));
            v[2] += zk::bf16_to_f32((uint16_t)(d.y & 0xffff));
            v[3] += zk::bf16_to_f32((uint16_t)(d.y >> 16));
            *reinterpret_cast<uint2*>(dx + m * g.Cin + nb + nl) =
                make_uint2(zk::pack_bf16x2(v[0], v[1]), zk::pack_bf16x2(v[2], v[3]));
          }
        }
      }
    }
  }
}

// conv3 applies to 3x3, stride 1, pads (1, 1) ('same'), pad value 0.
bool conv3_ok(const IGeom& g, int /*pad_ones: handled on the fragments*/) {
  return g.kh == 3 && g.kw == 3 && g.s == 1 && g.pt == 1 && g.pl == 1 && g.Ho == g.H &&
         g.Wo == g.W;
}

template <bool FWD, int BM, int BN, int WM, int WN, int NS, int CB, bool F4 = false>
int launch_conv3(const ConvArgs& args, const IGeom& g, hipStream_t stream) {
  const int NCH = FWD ? g.Cout : g.Cin, KCH = FWD ? g.Cin : g.Cout;
  const int RB = F4 ? KCH / 2 : KCH * 2;
  if (RB % CB || NCH % BN || !conv3_ok(g, args.pad_ones)) return (int)hipErrorInvalidValue;
  if (g_dry_run) return 0;
  constexpr int NW = WM * WN, RPI = 1024 / CB;
  constexpr int AR = (BM + 2 + RPI * NW - 1) / (RPI * NW) * RPI * NW;
  constexpr int BR = (3 * BN + RPI * NW - 1) / (RPI * NW) * RPI * NW;
  constexpr int LDS = NS * (AR + BR) * CB;
  static_assert(LDS <= 160 * 1024, "LDS");
  auto kern = igemm_conv3_kernel<FWD, BM, BN, WM, WN, NS, CB, F4>;
  ConvArgs ka = args;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)kern,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  const long long M = (long long)g.B * g.H * g.W;
  const int m_tiles = (int)((M + BM - 1) / BM);
  hipLaunchKernelGGL(kern, dim3((unsigned)((long long)m_tiles * (NCH / BN))), dim3(NW * 64), LDS,
                     stream, ka, g, m_tiles);
  return 0;
}

// Optional fused BN-backward reduction of the previous block (ConvArgs::psums).
struct BnSum {
  const void* ypred;
  const void* mean;
  const void* rstd;
  void* sums;
  int stripes;
  void* fstats = nullptr;  // LE variants only: ConvArgs::fstats (float forward statistics)
  int ypred_bf16 = 0;      // ypred bf16 (the stem's pooled BN-2 input): variant 50 only
  // LE variants only: ConvArgs::bxb / bcoef / bmask / brelu / bsums (float BN backward sums)
  const void* bxb = nullptr;
  const void* bcoef = nullptr;
  const void* bmask = nullptr;
  int brelu = 0;
  void* bsums = nullptr;
  const void* dmask = nullptr;  // LE variants only: ConvArgs::dmask
};

template <int BM, int BN, int WM, int WN, int NS, int CB = 128, bool LE = false>
int launch_igemm_dgrad(const void* dy, const void* wt, const void* mask, const void* dres,
                       void* dx, const IGeom& g, const BnSum& bs, hipStream_t stream) {
  if (LE && bs.sums) return (int)hipErrorInvalidValue;  // fused BN sums: register epilogue
  if (!LE && (bs.fstats || bs.bsums || bs.dmask))
    return (int)hipErrorInvalidValue;  // LDS epilogue only
  if ((g.Cout * 2) % CB || g.Cin % BN || g.s > 2 || g.kh > 4 || g.kw > 4)
    return (int)hipErrorInvalidValue;
  if (g_dry_run) return 0;
  constexpr int LDS = NS * (BM + BN) * CB;
  static_assert(LDS <= 160 * 1024, "LDS");
  // LE: the epilogue's residual / BN-input loads prefetched in groups
  // (runtime.epilogue_prefetch) or issued at each chunk
  auto kern = !LE || g_opt_epilogue_prefetch
                  ? igemm_conv_kernel<false, BM, BN, WM, WN, NS, CB, false, false, LE, true>
                  : igemm_conv_kernel<false, BM, BN, WM, WN, NS, CB, false, false, LE, false>;
  static bool attr[2] = {false, false};
  if (!attr[g_opt_epilogue_prefetch ? 1 : 0]) {
    hipError_t e = hipFuncSetAttribute((const void*)kern,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    if (e != hipSuccess) return (int)e;
    attr[g_opt_epilogue_prefetch ? 1 : 0] = true;
  }
  const int Hc = (g.H + g.s - 1) / g.s, Wc = (g.W + g.s - 1) / g.s;
  const long long Mc = (long long)g.B * Hc * Wc;
  const int m_tiles = (int)((Mc + BM - 1) / BM);
  const long long blocks = (long long)m_tiles * (g.Cin / BN);
  if (bs.bsums && (g.s != 1 || m_tiles > bs.stripes)) return (int)hipErrorInvalidValue;
  ConvArgs args{(const uint16_t*)dy, (const uint16_t*)wt, (const uint32_t*)mask,
                (const uint16_t*)dres, dx, nullptr, 0, 0, bs.stripes,
                (const int16_t*)bs.ypred, (const float*)bs.mean, (const float*)bs.rstd,
                (float*)bs.sums};
  args.fstats = (double*)bs.fstats;
  args.bxb = (const uint16_t*)bs.bxb;
  args.bcoef = (const float*)bs.bcoef;
  args.bmask = (const uint8_t*)bs.bmask;
  args.brelu = bs.brelu;
  args.bsums = (float*)bs.bsums;
  args.dmask = (const uint8_t*)bs.dmask;
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks, g.s * g.s), dim3(WM * WN * 64), LDS, stream,
                     args, g, m_tiles);
  return 0;
}

template <int BM, int BN, int WM, int WN, int NS, int CB = 128, bool F4 = false>
int launch_igemm_fwd(const void* sx, const void* wf, void* y, void* stats, const IGeom& g,
                     int pad_ones, int relu, int stripes, hipStream_t stream) {
  const int RB = F4 ? g.Cin / 2 : g.Cin * 2;
  if (RB % CB || g.Cout % BN) return (int)hipErrorInvalidValue;
  if (g_dry_run) return 0;
  constexpr int LDS = NS * (BM + BN) * CB;
  static_assert(LDS <= 160 * 1024, "LDS");
  auto kern = igemm_conv_kernel<true, BM, BN, WM, WN, NS, CB, F4>;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)kern,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  const long long Mo = (long long)g.B * g.Ho * g.Wo;
  const int m_tiles = (int)((Mo + BM - 1) / BM);
  const long long blocks = (long long)m_tiles * (g.Cout / BN);
  ConvArgs args{(const uint16_t*)sx, (const uint16_t*)wf, nullptr, nullptr, y,
                (unsigned long long*)stats, pad_ones, relu, stripes};
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks, 1), dim3(WM * WN * 64), LDS, stream, args, g,
                     m_tiles);
  return 0;
}

// Float forward (bf16 x bf16 -> bf16 y), any stride <= 2 / kernel <= 4x4:
// the binary-forward kernel with the bf16 epilogue.
template <int BM, int BN, int WM, int WN, int NS, int CB = 128>
int launch_igemm_fwd_bf16(const void* x, const void* wf, void* y, const IGeom& g, int relu,
                          hipStream_t stream) {
  if ((g.Cin * 2) % CB || g.Cout % BN || g.s > 2 || g.kh > 4 || g.kw > 4)
    return (int)hipErrorInvalidValue;
  if (g_dry_run) return 0;
  constexpr int LDS = NS * (BM + BN) * CB;
  static_assert(LDS <= 160 * 1024, "LDS");
  auto kern = igemm_conv_kernel<true, BM, BN, WM, WN, NS, CB, false, true>;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)kern,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  const long long Mo = (long long)g.B * g.Ho * g.Wo;
  const int m_tiles = (int)((Mo + BM - 1) / BM);
  const long long blocks = (long long)m_tiles * (g.Cout / BN);
  ConvArgs args{(const uint16_t*)x, (const uint16_t*)wf, nullptr, nullptr, y, nullptr, 0, relu,
                1};
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks, 1), dim3(WM * WN * 64), LDS, stream, args, g,
                     m_tiles);
  return 0;
}

int igemm_fwd_bf16_variant(int v, const void* x, const void* wf, void* y, const IGeom& g,
                           int relu, hipStream_t st) {
#define ZK_IGB(...) return launch_igemm_fwd_bf16<__VA_ARGS__>(x, wf, y, g, relu, st)
  switch (v) {
    case 0: ZK_IGB(128, 128, 2, 2, 2);
    case 1: ZK_IGB(256, 128, 4, 2, 2);
    case 2: ZK_IGB(128, 64, 2, 2, 2);
    case 3: ZK_IGB(256, 256, 4, 2, 2, 128);
    case 4: ZK_IGB(128, 64, 2, 2, 4, 64);
    case 5: ZK_IGB(256, 64, 4, 1, 2);
    default: return (int)hipErrorInvalidValue;
  }
#undef ZK_IGB
}

int igemm_fwd_variant(int v, const void* sx, const void* wf, void* y, void* stats,
                      const IGeom& g, int po, int relu, int ns, hipStream_t st) {
#define ZK_IGF(...) return launch_igemm_fwd<__VA_ARGS__>(sx, wf, y, stats, g, po, relu, ns, st)
  switch (v) {
    case 0: ZK_IGF(128, 128, 2, 2, 2);
    case 1: ZK_IGF(128, 128, 2, 2, 4, 64);
    case 2: ZK_IGF(256, 128, 4, 2, 2);
    case 3: ZK_IGF(128, 256, 2, 2, 2);
    case 4: ZK_IGF(128, 64, 2, 2, 2);
    case 5: ZK_IGF(128, 64, 2, 2, 3);
    case 6: ZK_IGF(256, 64, 4, 1, 2);
    case 7: ZK_IGF(128, 64, 2, 2, 4, 64);
    case 8: ZK_IGF(256, 64, 4, 1, 4, 64);
    case 9: ZK_IGF(64, 64, 2, 2, 2);
    case 10: ZK_IGF(128, 128, 2, 2, 4);
    case 11: ZK_IGF(256, 128, 4, 2, 4, 64);
    case 12: ZK_IGF(256, 256, 4, 2, 3, 64);
    case 13: ZK_IGF(256, 256, 2, 4, 3, 64);
    case 14: ZK_IGF(256, 256, 4, 2, 2, 128);
#define ZK_IGF3(...)                                                                    \
  {                                                                                     \
    ConvArgs a{(const uint16_t*)sx, (const uint16_t*)wf, nullptr, nullptr, y,           \
               (unsigned long long*)stats, po, relu, ns};                               \
    return launch_conv3<true, __VA_ARGS__>(a, g, st);                                   \
  }
    case 20: ZK_IGF3(256, 64, 4, 1, 2, 128)
    case 21: ZK_IGF3(256, 64, 4, 1, 3, 64)
    case 22: ZK_IGF3(128, 64, 2, 2, 2, 128)
    case 23: ZK_IGF3(128, 128, 2, 2, 2, 64)
    case 24: ZK_IGF3(256, 128, 4, 2, 2, 64)
    case 25: ZK_IGF3(256, 256, 4, 2, 2, 64)
    case 26: ZK_IGF3(128, 128, 2, 2, 3, 64)
    case 27: ZK_IGF3(256, 64, 4, 1, 2, 64)
#undef ZK_IGF3
    default: return (int)hipErrorInvalidValue;
  }
#undef ZK_IGF
}

// MX-FP4 forward tiles (e2m1 operands, RB = Cin/2 bytes per row): CB must
// divide Cin/2, so Cin = 64 runs 32-B K rows (SH = 3 swizzle), Cin = 128
// 64-B rows, Cin >= 256 64- or 128-B rows.  One MFMA covers 64 channels of
// one tap, 4x the K of a bf16 K-step over the same LDS bytes.
int igemm_fwd4_variant(int v, const void* sx, const void* wf, void* y, void* stats,
                       const IGeom& g, int po, int relu, int ns, hipStream_t st) {
  if (v == 40) {  // persistent 3x3 kernel (bfwd.hip)
    if (!zk_bfwd_supported(g.B, g.H, g.W, g.Cin, g.Cout, g.kh, g.kw, g.s, g.pt, g.pl) ||
        g.Ho != g.H || g.Wo != g.W)
      return (int)hipErrorInvalidValue;
    if (g_dry_run) return 0;
    return zk_bfwd_fp4(sx, wf, y, stats, g.B, g.H, g.W, g.Cin, g.Cout, po, relu, ns, st);
  }
#define ZK_IGF4(BM, BN, WM, WN, NS, CB) \
  return launch_igemm_fwd<BM, BN, WM, WN, NS, CB, true>(sx, wf, y, stats, g, po, relu, ns, st)
#define ZK_IGF43(BM, BN, WM, WN, NS, CB)                                                  \
  {                                                                                       \
    ConvArgs a{(const uint16_t*)sx, (const uint16_t*)wf, nullptr, nullptr, y,             \
               (unsigned long long*)stats, po, relu, ns};                                 \
    return launch_conv3<true, BM, BN, WM, WN, NS, CB, true>(a, g, st);                    \
  }
  switch (v) {
    // any stride (igemm_conv_kernel)
    case 0: ZK_IGF4(128, 128, 2, 2, 2, 32);
    case 1: ZK_IGF4(128, 128, 2, 2, 2, 64);
    case 2: ZK_IGF4(128, 128, 2, 2, 2, 128);
    case 3: ZK_IGF4(256, 128, 4, 2, 2, 128);
    case 4: ZK_IGF4(128, 64, 2, 1, 2, 32);
    case 5: ZK_IGF4(256, 256, 4, 2, 2, 128);
    case 6: ZK_IGF4(128, 128, 2, 2, 3, 64);
    case 7: ZK_IGF4(256, 128, 4, 2, 2, 64);
    case 8: ZK_IGF4(128, 64, 2, 1, 2, 64);
    case 9: ZK_IGF4(128, 64, 2, 1, 2, 128);
    // 3x3 stride 1 with horizontal tap reuse (igemm_conv3_kernel)
    case 20: ZK_IGF43(128, 64, 2, 1, 2, 32)
    case 21: ZK_IGF43(256, 64, 2, 1, 2, 32)
    case 22: ZK_IGF43(128, 128, 2, 2, 2, 64)
    case 23: ZK_IGF43(256, 128, 4, 2, 2, 64)
    case 24: ZK_IGF43(128, 128, 2, 2, 2, 128)
    case 25: ZK_IGF43(128, 256, 2, 2, 2, 64)
    case 26: ZK_IGF43(256, 256, 4, 2, 2, 64)
    case 27: ZK_IGF43(256, 64, 4, 1, 2, 64)
    case 28: ZK_IGF43(128, 64, 2, 1, 3, 32)
    default: return (int)hipErrorInvalidValue;
  }
#undef ZK_IGF43
#undef ZK_IGF4
}

int igemm_dgrad_variant(int v, const void* dy, const void* wt, const void* mask,
                        const void* dres, void* dx, const IGeom& g, const BnSum& bs,
                        hipStream_t st) {
#define ZK_IGD(...) return launch_igemm_dgrad<__VA_ARGS__>(dy, wt, mask, dres, dx, g, bs, st)
  if ((bs.fstats || bs.bsums || bs.dmask) && (v < 40 || v > 48))
    return (int)hipErrorInvalidValue;  // LE variants only
  switch (v) {
    case 0: ZK_IGD(128, 128, 2, 2, 2);        // 64 KB: 2 WG/CU
    case 1: ZK_IGD(128, 128, 2, 2, 4, 64);    // 64 KB, 3 K-steps of 32 in flight
    case 2: ZK_IGD(256, 128, 4, 2, 2);        // 8 waves, 96 KB
    case 3: ZK_IGD(128, 256, 2, 2, 2);        // wave tile 64x128, 96 KB
    case 4: ZK_IGD(128, 64, 2, 2, 2);         // 48 KB: 3 WG/CU
    case 5: ZK_IGD(128, 64, 2, 2, 3);         // 72 KB: 2 WG/CU
    case 6: ZK_IGD(256, 64, 4, 1, 2);         // 80 KB: 2 WG/CU
    case 7: ZK_IGD(128, 64, 2, 2, 4, 64);     // 48 KB, 3 in flight
    case 8: ZK_IGD(256, 64, 4, 1, 4, 64);     // 80 KB, 3 in flight
    case 9: ZK_IGD(64, 64, 2, 2, 2);          // 32 KB
    case 10: ZK_IGD(128, 128, 2, 2, 4);       // 128 KB, 1 WG/CU
    case 11: ZK_IGD(256, 128, 4, 2, 4, 64);   // 8 waves, 96 KB
    case 12: ZK_IGD(256, 256, 4, 2, 3, 64);   // 8 waves, 96 KB: 2x bytes/FLOP of 128x128
    case 13: ZK_IGD(256, 256, 2, 4, 3, 64);
    case 14: ZK_IGD(256, 256, 4, 2, 2, 128);  // 128 KB
    // three K-steps of 32 channels in flight
    case 15: ZK_IGD(256, 256, 4, 2, 4, 64);   // 128 KB
    case 16: ZK_IGD(256, 128, 4, 2, 4, 64);   // 96 KB
    case 17: ZK_IGD(128, 256, 2, 4, 4, 64);   // 96 KB
    // coalesced LDS-staged epilogue (dgrad_store_lds): whole-row dx stores
    case 40: ZK_IGD(128, 128, 2, 2, 2, 128, true);
    case 41: ZK_IGD(128, 128, 2, 2, 4, 64, true);
    case 42: ZK_IGD(128, 64, 2, 2, 2, 128, true);
    case 43: ZK_IGD(128, 64, 2, 2, 4, 64, true);
    case 44: ZK_IGD(256, 128, 4, 2, 2, 128, true);
    case 45: ZK_IGD(256, 256, 4, 2, 2, 128, true);
    case 46: ZK_IGD(256, 128, 4, 2, 4, 64, true);
    case 47: ZK_IGD(128, 256, 2, 4, 4, 64, true);
    case 48: ZK_IGD(128, 64, 2, 2, 3, 128, true);
#define ZK_IGD3(...)                                                                    \
  {                                                                                     \
    ConvArgs a{(const uint16_t*)dy, (const uint16_t*)wt, (const uint32_t*)mask,         \
               (const uint16_t*)dres, dx, nullptr, 0, 0, bs.stripes,                    \
               (const int16_t*)bs.ypred, (const float*)bs.mean, (const float*)bs.rstd,  \
               (float*)bs.sums};                                                        \
    return launch_conv3<false, __VA_ARGS__>(a, g, st);                                  \
  }
    case 20: ZK_IGD3(256, 64, 4, 1, 2, 128)
    case 21: ZK_IGD3(256, 64, 4, 1, 3, 64)
    case 22: ZK_IGD3(128, 64, 2, 2, 2, 128)
    case 23: ZK_IGD3(128, 128, 2, 2, 2, 64)
    case 24: ZK_IGD3(256, 128, 4, 2, 2, 64)
    case 25: ZK_IGD3(256, 256, 4, 2, 2, 64)
    case 26: ZK_IGD3(128, 128, 2, 2, 3, 64)
    case 27: ZK_IGD3(256, 64, 4, 1, 2, 64)
    // deeper rings with 32-B channel chunks (padded weight rows)
    case 28: ZK_IGD3(256, 64, 4, 1, 4, 32)
    case 29: ZK_IGD3(256, 64, 4, 1, 3, 32)
    case 30: ZK_IGD3(128, 64, 2, 2, 4, 32)
    case 32: ZK_IGD3(256, 64, 4, 1, 4, 64)
    case 33: ZK_IGD3(128, 128, 2, 2, 4, 32)
    case 34: ZK_IGD3(256, 128, 4, 2, 3, 32)
#undef ZK_IGD3
    default: return (int)hipErrorInvalidValue;
  }
#undef ZK_IGD
}


// ===========================================================================
// wgrad:  dW[co][n = (t, ci)] = sum_p dY[p][co] * sx[pixel(p, t)][ci]
//   K = output pixels (split over blockIdx-derived splits), both operands are
//   [pixel][channel] row images in LDS read with ds_read_b64_tr_b16.
//   sx = sign(x) as bf16 +-1 [B][H][W][Cin] (written by zk_sign_pack);
//   padded taps read the zero page (pad_values 0) or the +1 page.
// ===========================================================================
template <int BM, int BN, int WM, int WN, int BK, int NS>
__global__ __launch_bounds__(WM * WN * 64, 1) void igemm_wgrad_kernel(
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ sx,
    const float* __restrict__ w, float* __restrict__ dw, float* __restrict__ slab, IGeom g,
    int pad_ones, float clip, int k_per_split, int m_tiles, int n_tiles, SkTree tree) {
  constexpr int NWAVES = WM * WN;
  constexpr int RA = BM * 2, RBB = BN * 2;      // bytes per pixel row of A / B
  constexpr int SA = BK * RA, SB = BK * RBB;    // bytes per stage
  static_assert(SA % (1024 * NWAVES) == 0 && SB % (1024 * NWAVES) == 0, "stage / waves");
  constexpr int A_INS = SA / 1024 / NWAVES, B_INS = SB / 1024 / NWAVES;
  constexpr int LPS = A_INS + B_INS;
  constexpr int STAGE = SA + SB;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 32, TN = WTN / 32;

  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int wm = wave / WN, wn = wave % WN;

  // logical id: consecutive ids = tiles of one split (share dY / sx rows in
  // one XCD's L2)
  const int L = xcd_linear(blockIdx.x, gridDim.x);
  const int tiles = m_tiles * n_tiles;
  const int split = L / tiles, tile = L % tiles;
  const int m0 = (tile % m_tiles) * BM;  // co
  const int n0 = (tile / m_tiles) * BN;  // flattened (t, ci)
  const int P = g.B * g.Ho * g.Wo;
  const int kbeg = split * k_per_split;
  if (kbeg >= P) return;
  int kend = kbeg + k_per_split;
  if (kend > P) kend = P;
  const int NK = (kend - kbeg + BK - 1) / BK;

  const unsigned char* dyb = reinterpret_cast<const unsigned char*>(dy);
  const unsigned char* sxb = reinterpret_cast<const unsigned char*>(sx);
  const unsigned char* zp = reinterpret_cast<const unsigned char*>(g_zero_page);
  const unsigned char* pp = pad_ones ? reinterpret_cast<const unsigned char*>(g_ones_page_bf16)
                                     : zp;
  const float invWo = 1.0f / (float)g.Wo, invHo = 1.0f / (float)g.Ho;

  // Per-lane fixed parts of the loader: (row within stage, byte within row)
  int a_row[A_INS], a_byte[A_INS];
#pragma unroll
  for (int j = 0; j < A_INS; ++j) {
    const int off = ((j * NWAVES + wave) * 64 + lane) * 16;
    a_row[j] = off / RA;
    const int slot = (off % RA) >> 4;
    a_byte[j] = m0 * 2 + ((slot ^ tr_swz<RA>(a_row[j])) << 4);
  }
  int b_row[B_INS], b_th[B_INS], b_tw[B_INS], b_cib[B_INS];
#pragma unroll
  for (int j = 0; j < B_INS; ++j) {
    const int off = ((j * NWAVES + wave) * 64 + lane) * 16;
    b_row[j] = off / RBB;
    const int slot = (off % RBB) >> 4;
    const int n = n0 + ((slot ^ tr_swz<RBB>(b_row[j])) << 3);  // first column of the chunk
    const int t = n / g.Cin;
    b_th[j] = t / g.kw - g.pt;
    b_tw[j] = t % g.kw - g.pl;
    b_cib[j] = (n % g.Cin) * 2;
  }
  auto issue = [&](int ks) {
    unsigned char* st = smem + (ks % NS) * STAGE;
    const int k0 = kbeg + ks * BK;
#pragma unroll
    for (int j = 0; j < A_INS; ++j) {
      const int p = k0 + a_row[j];
      const unsigned char* src =
          p < kend ? dyb + (long long)p * (g.Cout * 2) + a_byte[j] : zp;
      ZK_GLDS16(src, st + (j * NWAVES + wave) * 1024);
    }
#pragma unroll
    for (int j = 0; j < B_INS; ++j) {
      const int p = k0 + b_row[j];
      const unsigned char* src = zp;
      if (p < kend) {
        const int q1 = fdiv(p, g.Wo, invWo);
        const int wo = p - q1 * g.Wo;
        const int b = fdiv(q1, g.Ho, invHo);
        const int ho = q1 - b * g.Ho;
        const int hi = ho * g.s + b_th[j], wi = wo * g.s + b_tw[j];
        if (hi >= 0 && hi < g.H && wi >= 0 && wi < g.W)
          src = sxb + (((long long)b * g.H + hi) * g.W + wi) * (g.Cin * 2) + b_cib[j];
        else
          src = pp;
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
    const unsigned char* stb = st + SA;
    // double-buffered transposed fragment reads (see igemm_conv_kernel)
    constexpr int NSUB = BK / 16;
    uint4 af[2][TM], bfr[2][TN];
    auto read_frags = [&](int sub, int set) {
#pragma unroll
      for (int a = 0; a < TM; ++a)
        af[set][a] = tr_frag_swz<RA>(st, sub * 16, wm * WTM + a * 32, lane);
#pragma unroll
      for (int b = 0; b < TN; ++b)
        bfr[set][b] = tr_frag_swz<RBB>(stb, sub * 16, wn * WTN + b * 32, lane);
    };
    read_frags(0, 0);
#pragma unroll
    for (int sub = 0; sub < NSUB; ++sub) {
      if (sub + 1 < NSUB) read_frags(sub + 1, (sub + 1) & 1);
      // keep the next substep's reads ahead of this substep's MFMAs (the
      // scheduler would otherwise sink them to reuse the registers)
      __builtin_amdgcn_sched_barrier(0);
      const int cs = sub & 1;
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) acc[a][b] = mfma_bf16(af[cs][a], bfr[cs][b], acc[a][b]);
    }
  }

  // epilogue.  Tree mode (tree.slab): this split's partial into the level-0
  // slab, then the in-launch fixed-order combine (splitk_tree.h); a single
  // split adds straight into dW.  Slab mode: plain stores into
  // slab[split][Cout][T*Cin] for wgrad_reduce_kernel.  Otherwise: kernel STE
  // mask and fp32 atomics straight into dW.
  const int h = lane >> 5, r32 = lane & 31;
  const int NTOT = g.kh * g.kw * g.Cin;
  const bool treed = tree.slab != nullptr || (tree.levels == 0 && tree.dwn > 0);
  float* sl = slab ? slab + (long long)split * g.Cout * NTOT : nullptr;
#pragma unroll
  for (int a = 0; a < TM; ++a) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = m0 + wm * WTM + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int n = n0 + wn * WTN + b * 32 + r32;
        const long long idx = (long long)co * NTOT + n;
        if (treed) {
          if (tree.levels > 0)
            skt_store(tree, split, idx, acc[a][b][r]);
          else if (!w || fabsf(w[idx]) <= clip)
            dw[idx] += acc[a][b][r];  // one split: this block owns the element
        } else if (sl) {
          sl[idx] = acc[a][b][r];
        } else if (fabsf(w[idx]) <= clip) {
          atomicAdd(dw + idx, acc[a][b][r]);
        }
      }
    }
  }
  if (treed && tree.levels > 0)
    skt_combine<NWAVES * 64, BM, BN>(tree, tile, split, m0, n0, NTOT, dw, w, clip,
                                     reinterpret_cast<int*>(smem));
}

// dW[i] += [|w[i]| <= clip] * sum_s slab[s][i], the splits summed in index
// order.  One float4 column per thread, the split loads 8 at a time (the sum
// stays sequential): a streaming pass over the slabs at HBM rate.  (Round 5's
// form -- 16 columns x 16 split lanes per block and an LDS reduction, ~37k
// blocks for a 2.4 M-float dW -- ran at ~0.5 TB/s: ~70 us per layer.)
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float4* __restrict__ slab,
                                                           int splits, long long n4,
                                                           const float4* __restrict__ w,
                                                           float clip, float4* __restrict__ dw) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
  int sp = 0;
  for (; sp + 8 <= splits; sp += 8) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = slab[(long long)(sp + u) * n4 + i];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      t.x += v[u].x;
      t.y += v[u].y;
      t.z += v[u].z;
      t.w += v[u].w;
    }
  }
  for (; sp < splits; ++sp) {
    const float4 v = slab[(long long)sp * n4 + i];
    t.x += v.x;
    t.y += v.y;
    t.z += v.z;
    t.w += v.w;
  }
  const float4 wv = w ? w[i] : make_float4(0.f, 0.f, 0.f, 0.f);  // no w: no mask
  float4 d = dw[i];
  d.x += fabsf(wv.x) <= clip ? t.x : 0.f;
  d.y += fabsf(wv.y) <= clip ? t.y : 0.f;
  d.z += fabsf(wv.z) <= clip ? t.z : 0.f;
  d.w += fabsf(wv.w) <= clip ? t.w : 0.f;
  dw[i] = d;
}

struct WgradPlan {
  int m_tiles, n_tiles, splits, kps;
};

// slab: the split-K partials go to slabs (capped by wgrad_slab_mb); otherwise
// fp32 atomics into dW, where the split count follows the block target alone.
template <int BM, int BN, int BK>
bool plan_wgrad(const IGeom& g, int target_blocks, WgradPlan& p, bool slab) {
  const int NTOT = g.kh * g.kw * g.Cin;
  if (g.Cout % BM || NTOT % BN || g.Cin % 8) return false;
  const long long P = (long long)g.B * g.Ho * g.Wo;
  if (P >= (1 << 24)) return false;  // fdiv range
  p.m_tiles = g.Cout / BM;
  p.n_tiles = NTOT / BN;
  const long long tiles = (long long)p.m_tiles * p.n_tiles;
  long long splits = (target_blocks + tiles - 1) / tiles;
  const long long max_splits = (P + 4 * BK - 1) / (4 * BK);  // >= 4 K-steps per split
  if (splits > max_splits) splits = max_splits;
  if (slab) splits = cap_splits(splits, (long long)g.Cout * NTOT * 4);
  if (splits < 1) splits = 1;
  long long kps = (P + splits - 1) / splits;
  kps = (kps + BK - 1) / BK * BK;
  p.splits = (int)((P + kps - 1) / kps);
  p.kps = (int)kps;
  return true;
}

template <int BM, int BN, int WM, int WN, int BK, int NS>
int launch_igemm_wgrad(const void* dy, const void* sx, const void* w, void* dw, const IGeom& g,
                       int pad_ones, float clip, int target_blocks, void* ws, long long ws_bytes,
                       long long* ws_needed, hipStream_t stream) {
  WgradPlan p;
  if (!plan_wgrad<BM, BN, BK>(g, target_blocks, p, ws_needed != nullptr || ws != nullptr))
    return (int)hipErrorInvalidValue;
  const int NTOT = g.kh * g.kw * g.Cin;
  const long long slab_bytes = (long long)p.splits * g.Cout * NTOT * 4;
  if (ws_needed) {  // size query only: the tree's levels when it applies
    SkTree t;
    long long tf = 0, tc = 0;
    const long long tiles = (long long)p.m_tiles * p.n_tiles;
    *ws_needed = (g_opt_wgrad_tree && skt_plan(p.splits, (int)tiles, (long long)g.Cout * NTOT, t,
                                               tf, tc))
                     ? tf * 4
                     : slab_bytes;
    return 0;
  }
  constexpr int LDS = NS * BK * (BM + BN) * 2;
  static_assert(LDS <= 160 * 1024, "LDS");
  auto kern = igemm_wgrad_kernel<BM, BN, WM, WN, BK, NS>;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)kern,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  const long long tiles = (long long)p.m_tiles * p.n_tiles;
  // the in-launch tree when its slab and counters are available, else the
  // slab + wgrad_reduce_kernel pair
  SkTree tree{};
  long long tree_floats = 0, tree_cnt = 0;
  int* cnt = nullptr;
  const bool tree_ok = g_opt_wgrad_tree && ws && NTOT % 4 == 0 &&
                       skt_plan(p.splits, (int)tiles, (long long)g.Cout * NTOT, tree,
                                tree_floats, tree_cnt) &&
                       ws_bytes >= tree_floats * 4 && (cnt = skt_counters(stream)) != nullptr;
  float* slab = nullptr;
  if (tree_ok) {
    tree.slab = tree.levels > 0 ? (float*)ws : nullptr;
    tree.cnt = cnt;
  } else {
    tree = SkTree{};
    slab = (ws && ws_bytes >= slab_bytes && NTOT % 4 == 0) ? (float*)ws : nullptr;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)(tiles * p.splits)), dim3(WM * WN * 64), LDS, stream,
                     (const uint16_t*)dy, (const uint16_t*)sx, (const float*)w, (float*)dw, slab,
                     g, pad_ones, clip, p.kps, p.m_tiles, p.n_tiles, tree);
  if (slab) {
    const long long n4 = (long long)g.Cout * NTOT / 4;
    const long long blocks = (n4 + 255) / 256;
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, stream,
                       (const float4*)slab, p.splits, n4, (const float4*)w, clip, (float4*)dw);
  }
  return 0;
}

// ===========================================================================
// conv3 weight gradient (3x3, stride 1, 'same'): the three taps of TH kernel
// rows per block, one dy load per K-step for all of them.
//
// K runs over "extended" pixel positions e = (b*H + h)*(W+2) + w + 1: every
// image row carries a halo column on both sides.  Tap (th, tw) of output e
// reads sx at extended position e + tw - 1 of image row h + th - 1, i.e. LDS
// row k + tw of kernel row th's staged segment (BK + 2 rows from e0 - 1).
// Halo / out-of-image sx rows are loaded from the zero (+1) page and the dy
// rows of halo positions from the zero page, so no fragment is masked.
// Per K-step: BK dy rows + TH segments of BK + 2 sx rows feed 3*TH taps:
// dy is read 3/TH times per layer instead of 9, sx 3 times instead of 9.
// The halo costs 2/(W+2) of the K-steps.  Output as igemm_wgrad_kernel.
// ===========================================================================
template <int BM, int BN, int WM, int WN, int BK, int NS, int TH, int OCC>
__global__ __launch_bounds__(WM * WN * 64, OCC) void igemm_wgrad3_kernel(
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ sx,
    const float* __restrict__ w, float* __restrict__ dw, float* __restrict__ slab, IGeom g,
    int pad_ones, float clip, int k_per_split, int m_tiles, int n_tiles) {
  constexpr int NWAVES = WM * WN, NT = 3 * TH, TG = 3 / TH;
  static_assert(TH == 1 || TH == 3, "kernel rows per block");
  constexpr int RA = BM * 2, RBB = BN * 2;
  constexpr int SA = BK * RA;
  static_assert(SA % (1024 * NWAVES) == 0, "A stage / waves");
  constexpr int A_INS = SA / 1024 / NWAVES;
  constexpr int SEG = (BK + 2) * RBB;  // one kernel row's sx segment
  static_assert(SEG % 256 == 0, "segments keep the swizzle period");
  constexpr int B_KB = (TH * SEG + 1023) / 1024;
  constexpr int B_INS = (B_KB + NWAVES - 1) / NWAVES;  // tail lanes: zero page
  constexpr int SB = B_INS * NWAVES * 1024;
  constexpr int LPS = A_INS + B_INS;
  constexpr int STAGE = SA + SB;
  constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 32, TN = WTN / 32;

  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave / WN, wn = wave % WN;

  // consecutive logical ids: the tiles (and kernel-row groups) of one split
  const int L = xcd_linear(blockIdx.x, gridDim.x);
  const int tiles = m_tiles * n_tiles * TG;
  const int split = L / tiles, tile = L % tiles;
  const int thg = tile % TG, mn = tile / TG;
  const int m0 = (mn % m_tiles) * BM;  // co
  const int n0 = (mn / m_tiles) * BN;  // ci
  const int WE = g.W + 2;
  const int E = g.B * g.H * WE;
  const int kbeg = split * k_per_split;
  if (kbeg >= E) return;
  const int kend = min(E, kbeg + k_per_split);
  const int NK = (kend - kbeg + BK - 1) / BK;

  const unsigned char* dyb = reinterpret_cast<const unsigned char*>(dy);
  const unsigned char* sxb = reinterpret_cast<const unsigned char*>(sx);
  const unsigned char* zp = reinterpret_cast<const unsigned char*>(g_zero_page);
  const unsigned char* pp = pad_ones ? reinterpret_cast<const unsigned char*>(g_ones_page_bf16)
                                     : zp;
  const float invWE = 1.0f / (float)WE, invH = 1.0f / (float)g.H;

  int a_row[A_INS], a_byte[A_INS];
#pragma unroll
  for (int j = 0; j < A_INS; ++j) {
    const int off = ((j * NWAVES + wave) * 64 + lane) * 16;
    a_row[j] = off / RA;
    const int slot = (off % RA) >> 4;
    a_byte[j] = m0 * 2 + ((slot ^ tr_swz<RA>(a_row[j])) << 4);
  }
  int b_row[B_INS], b_th[B_INS], b_byte[B_INS];  // b_th < 0: tail lane
#pragma unroll
  for (int j = 0; j < B_INS; ++j) {
    const int off = ((j * NWAVES + wave) * 64 + lane) * 16;
    b_th[j] = -1;
    b_row[j] = b_byte[j] = 0;
    if (off < TH * SEG) {
      const int t = off / SEG, o = off % SEG;
      b_th[j] = thg * TH + t;
      b_row[j] = o / RBB;
      b_byte[j] = n0 * 2 + ((((o % RBB) >> 4) ^ tr_swz<RBB>(b_row[j])) << 4);
    }
  }
  auto issue = [&](int ks) {
    unsigned char* st = smem + (ks % NS) * STAGE;
    const int e0 = kbeg + ks * BK;
#pragma unroll
    for (int j = 0; j < A_INS; ++j) {
      const int e = e0 + a_row[j];
      const unsigned char* src = zp;  // halo column / past the split: no contribution
      if (e < kend) {
        const int q = fdiv(e, WE, invWE);
        const int c = e - q * WE - 1;
        if (c >= 0 && c < g.W) src = dyb + ((long long)q * g.W + c) * (g.Cout * 2) + a_byte[j];
      }
      ZK_GLDS16(src, st + (j * NWAVES + wave) * 1024);
    }
#pragma unroll
    for (int j = 0; j < B_INS; ++j) {
      const unsigned char* src = zp;
      if (b_th[j] >= 0) {
        src = pp;  // padding tap
        const int e = e0 - 1 + b_row[j];
        if (e >= 0 && e < E) {
          const int q = fdiv(e, WE, invWE);  // b*H + h
          const int c = e - q * WE - 1;
          const int hh = q - fdiv(q, g.H, invH) * g.H + b_th[j] - 1;
          if (c >= 0 && c < g.W && hh >= 0 && hh < g.H)
            src = sxb + ((long long)(q + b_th[j] - 1) * g.W + c) * (g.Cin * 2) + b_byte[j];
        }
      }
      ZK_GLDS16(src, st + SA + (j * NWAVES + wave) * 1024);
    }
  };

  f32x16 acc[NT][TM][TN];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][a][b][r] = 0.f;

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
    const unsigned char* stb = st + SA;
#pragma unroll
    for (int sub = 0; sub < BK / 16; ++sub) {
      uint4 af[TM];
#pragma unroll
      for (int a = 0; a < TM; ++a) af[a] = tr_frag_swz<RA>(st, sub * 16, wm * WTM + a * 32, lane);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        // tap (t / 3, tw = t % 3): segment t / 3 shifted by tw rows
        uint4 bfr[TN];
#pragma unroll
        for (int b = 0; b < TN; ++b)
          bfr[b] = tr_frag_swz<RBB>(stb + (t / 3) * SEG, sub * 16 + t % 3,
                                    wn * WTN + b * 32, lane);
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b) acc[t][a][b] = mfma_bf16(af[a], bfr[b], acc[t][a][b]);
      }
    }
  }

  const int h = lane >> 5, r32 = lane & 31;
  const int NTOT = 9 * g.Cin;
  float* sl = slab ? slab + (long long)split * g.Cout * NTOT : nullptr;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int tap = (thg * TH + t / 3) * 3 + t % 3;
#pragma unroll
    for (int a = 0; a < TM; ++a) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = m0 + wm * WTM + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          const long long idx =
              (long long)co * NTOT + tap * g.Cin + n0 + wn * WTN + b * 32 + r32;
          if (sl)
            sl[idx] = acc[t][a][b][r];
          else if (fabsf(w[idx]) <= clip)
            atomicAdd(dw + idx, acc[t][a][b][r]);
        }
      }
    }
  }
}

template <int BM, int BN, int BK, int TH>
bool plan_wgrad3(const IGeom& g, int target_blocks, WgradPlan& p, bool slab) {
  if (!conv3_ok(g, 0) || g.Cout % BM || g.Cin % BN) return false;
  const long long E = (long long)g.B * g.H * (g.W + 2);
  if (E >= (1 << 24)) return false;  // fdiv range
  p.m_tiles = g.Cout / BM;
  p.n_tiles = g.Cin / BN;
  const long long tiles = (long long)p.m_tiles * p.n_tiles * (3 / TH);
  long long splits = (target_blocks + tiles - 1) / tiles;
  const long long max_splits = (E + 4 * BK - 1) / (4 * BK);
  if (splits > max_splits) splits = max_splits;
  if (slab) splits = cap_splits(splits, (long long)g.Cout * g.kh * g.kw * g.Cin * 4);
  if (splits < 1) splits = 1;
  long long kps = (E + splits - 1) / splits;
  kps = (kps + BK - 1) / BK * BK;
  p.splits = (int)((E + kps - 1) / kps);
  p.kps = (int)kps;
  return true;
}

template <int BM, int BN, int WM, int WN, int BK, int NS, int TH, int OCC>
int launch_igemm_wgrad3(const void* dy, const void* sx, const void* w, void* dw, const IGeom& g,
                        int pad_ones, float clip, int target_blocks, void* ws, long long ws_bytes,
                        long long* ws_needed, hipStream_t stream) {
  WgradPlan p;
  if (!plan_wgrad3<BM, BN, BK, TH>(g, target_blocks, p, ws_needed != nullptr || ws != nullptr))
    return (int)hipErrorInvalidValue;
  const int NTOT = 9 * g.Cin;
  const long long slab_bytes = (long long)p.splits * g.Cout * NTOT * 4;
  if (ws_needed) {
    *ws_needed = slab_bytes;
    return 0;
  }
  constexpr int NW = WM * WN;
  constexpr int SB = ((TH * (BK + 2) * BN * 2 + 1023) / 1024 + NW - 1) / NW * NW * 1024;
  constexpr int LDS = NS * (BK * BM * 2 + SB);
  static_assert(LDS <= 160 * 1024, "LDS");
  auto kern = igemm_wgrad3_kernel<BM, BN, WM, WN, BK, NS, TH, OCC>;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)kern,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  float* slab = (ws && ws_bytes >= slab_bytes && NTOT % 4 == 0) ? (float*)ws : nullptr;
  const long long tiles = (long long)p.m_tiles * p.n_tiles * (3 / TH);
  hipLaunchKernelGGL(kern, dim3((unsigned)(tiles * p.splits)), dim3(NW * 64), LDS, stream,
                     (const uint16_t*)dy, (const uint16_t*)sx, (const float*)w, (float*)dw, slab,
                     g, pad_ones, clip, p.kps, p.m_tiles, p.n_tiles);
  if (slab) {
    const long long n4 = (long long)g.Cout * NTOT / 4;
    const long long blocks = (n4 + 255) / 256;
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, stream,
                       (const float4*)slab, p.splits, n4, (const float4*)w, clip, (float4*)dw);
  }
  return 0;
}

int igemm_wgrad_variant(int v, const void* dy, const void* sx, const void* w, void* dw,
                        const IGeom& g, int po, float clip, int tb, void* ws, long long wsb,
                        long long* need, hipStream_t st) {
#define ZK_IGW(...) \
  return launch_igemm_wgrad<__VA_ARGS__>(dy, sx, w, dw, g, po, clip, tb, ws, wsb, need, st)
#define ZK_IGW3(...) \
  return launch_igemm_wgrad3<__VA_ARGS__>(dy, sx, w, dw, g, po, clip, tb, ws, wsb, need, st)
  if (v == 60) {  // deep_gemm.hip phased 256x256 kernel + its fixed-order split-K combine
    if (!conv3_ok(g, 0)) return (int)hipErrorInvalidValue;
    int splits = 0;
    const int rc = zk_wgrad_deep_impl(dy, sx, w, dw, g.B, g.H, g.W, g.Cin, g.Cout, po, clip, tb,
                                      ws, wsb, need, &splits, need != nullptr || g_dry_run,
                                      g_opt_wgrad_tree != 0, st);
    if (rc || need || g_dry_run || splits == 0) return rc;  // splits 0: combined in-launch
    const long long n4 = (long long)g.Cout * 9 * g.Cin / 4;
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st,
                       (const float4*)ws, splits, n4, (const float4*)w, clip, (float4*)dw);
    return 0;
  }
  switch (v) {
    // conv3 family <BM, BN, WM, WN, BK, NS, TH, OCC>
    case 20: ZK_IGW3(64, 64, 2, 2, 32, 4, 3, 1);
    case 21: ZK_IGW3(64, 64, 2, 2, 32, 4, 1, 2);
    case 22: ZK_IGW3(128, 64, 2, 2, 32, 3, 1, 2);
    case 23: ZK_IGW3(128, 128, 2, 2, 32, 2, 1, 1);
    case 24: ZK_IGW3(64, 128, 2, 2, 32, 3, 1, 2);
    case 25: ZK_IGW3(64, 64, 2, 2, 64, 3, 3, 1);
    case 26: ZK_IGW3(128, 128, 2, 2, 32, 3, 1, 1);
    case 27: ZK_IGW3(64, 64, 2, 2, 32, 3, 3, 2);
    case 28: ZK_IGW3(128, 64, 2, 2, 64, 2, 1, 2);
    // two waves of 64 x 32 (the dy fragment feeds two MFMAs per sx fragment)
    case 29: ZK_IGW3(64, 64, 1, 2, 32, 4, 3, 1);
    case 30: ZK_IGW3(64, 64, 1, 2, 32, 3, 3, 1);
    case 32: ZK_IGW3(128, 64, 2, 2, 32, 3, 3, 1);
    case 33: ZK_IGW3(64, 64, 1, 2, 32, 4, 1, 2);
    case 34: ZK_IGW3(128, 64, 1, 2, 32, 3, 1, 2);
    case 0: ZK_IGW(128, 128, 2, 2, 32, 2);
    case 1: ZK_IGW(128, 128, 2, 2, 32, 4);
    case 2: ZK_IGW(128, 192, 2, 2, 32, 3);
    case 3: ZK_IGW(64, 192, 2, 2, 32, 4);
    case 4: ZK_IGW(128, 128, 2, 2, 64, 2);
    case 5: ZK_IGW(64, 128, 2, 2, 32, 4);
    case 6: ZK_IGW(128, 256, 2, 2, 32, 2);
    case 7: ZK_IGW(64, 64, 2, 2, 32, 4);
    case 8: ZK_IGW(256, 256, 4, 2, 32, 2);   // 8 waves, 64 KB
    case 9: ZK_IGW(256, 256, 2, 4, 32, 2);
    case 10: ZK_IGW(256, 128, 4, 2, 32, 2);
    case 11: ZK_IGW(128, 256, 2, 4, 32, 2);
    case 12: ZK_IGW(256, 256, 4, 2, 32, 3);  // 96 KB
    default: return (int)hipErrorInvalidValue;
  }
#undef ZK_IGW
#undef ZK_IGW3
}

}  // namespace

// deep_gemm.hip: phased 256x256 (256x128) dgrad of the stride-1 3x3 convs
// with Cin % 128 == 0 (variant 60)
int zk_dgrad_deep_impl(const void* dy, const void* wt, const void* mask, const void* dres, void* dx,
                       int B, int H, int W, int Cin, int Cout, int Ho, int Wo, int kh, int kw,
                       int s, int pt, int pl, bool dry, hipStream_t st);

// conv3rw.hip: row-window dgrad of the 64 -> 64 stride-1 3x3 conv (variant 50)
int zk_conv3rw_dgrad_impl(const void* dy, const void* wt, const void* mask, const void* dres,
                          void* dx, int B, int H, int W, int Cin, int Cout, const void* ypred,
                          const void* pmean, const void* prstd, void* psums, int stripes,
                          int ypred_bf16, bool dry, hipStream_t st);

namespace {
int igemm_dgrad_impl(const void* dy, const void* wt, const void* mask, const void* dres, void* dx,
                     const IGeom& g, const BnSum& bs, int variant, hipStream_t stream) {
  if (variant < 0) {
    // Tuned on MI355X (tools/tune_bconv.py --only igemm, E18 shapes, batch
    // 256): 128x128 at 2 WG/CU for Cin >= 128 (8-wave 256x128 for the
    // 256-channel stride-1 layers), 128x64 with a 4-deep 64-B ring for Cin=64.
    // 256x256 (v14) halves the LDS-fill bytes per FLOP; it pays where the
    // grid still has ~200 tiles (the 256-channel stride-1 layers).  conv3
    // (20+: horizontal tap reuse) for the other stride-1 3x3 layers.
    // Batch >= 512 (profiles/r1av_bconv_tuning_b512.md): 256x256 also wins
    // for the 512-channel stride-1 and 256-channel stride-2 layers (7x7 x 512
    // images: 154 -> 121 us); smaller batches keep the batch-256 choices.
    // 1x1 GEMMs (ResNet-50's bottleneck convs: K = 64..2048, mostly bound
    // by the output bytes) and the 256x256 tiles use the coalesced
    // LDS-staged epilogue (40+) unless the fused BN sums need the register
    // one (tools/tune_pw.py, batch 512: 56x56 N256 K64 387 -> 334 us,
    // 14x14 N1024 K256 144 -> 127 us, 28x28 N128 K512 139 -> 120 us).
    const int Cin = g.Cin, stride = g.s;
    const bool c3 = conv3_ok(g, 0);
    const bool le = bs.sums == nullptr;  // (bs.bsums: LE variants, checked at the launch)
    // 3x3 256x256 tiles at batch >= 1024: the register epilogue (14) when
    // tile_huge bit 32 is set (batch 1536 standalone, tools/tune_bconv.py:
    // 14x14x256 383 vs 414 us, 7x7x512 398 vs 418 us, 14x14 256->512 stride 2
    // 215 vs 269 us; in-step QuickNet-Large b1024 27.63k / 27.64k vs 27.16k /
    // 27.12k img/s, E18 b1536 49.69k / 49.96k vs 50.15k / 49.80k)
    const int v256 =
        (le && !(g.kh == 3 && g.B >= 1024 && huge_tiles_env(32))) ? 45 : 14;
    if (g_opt_dgrad_deep && le && !bs.fstats && !bs.bsums && !bs.dmask && c3 &&
        Cin % 256 == 0 && g.Cout % 64 == 0 && (!mask || g_opt_dgrad_deep >= 2))
      // phased 256x256 schedule (deep_gemm.hip).  Measured at batch 1536 it
      // ties the 256x256 implicit GEMM (14x14x256: 428-484 vs 495 us; 7x7x512
      // 432-462 vs 406 us) and loses for 128 channels (769 vs 594 us) and the
      // stride-2 transitions, so only the stride-1 >= 256-channel layers take it
      // by default (profiles/r4/b_deep_gemm.md).  In the step (round 5,
      // interleaved A/B): the float convs keep it (ResNet-50 without the deep
      // kernels 10.71k vs 10.91k img/s); the binary ones (STE mask epilogue)
      // do not (E18 with it off 51.6k vs 51.3k)
      variant = 60;
    else if (le && g.kh == 1 && g.kw == 1 && stride == 1 && Cin % 64 == 0)
      // 256x256 only for deep K: with K < 1024 the 128x128 4-stage ring (41)
      // is 12-25 % faster at batch 512 and 1024, with and without a residual
      // (tools/tune_pw.py, profiles/r6/pw_tiles.md: 56x56 N256 K64 b1024
      // 1033 -> 832 us, 14x14 N1024 K256 345 -> 331, 7x7 N2048 K512 232 -> 203)
      variant = Cin % 256 == 0 ? (g.Cout >= 1024 ? 45 : 41) : Cin % 128 == 0 ? 41 : 43;
    else if (Cin == 256 && stride == 1)
      variant = v256;
    else if (Cin >= 256 && Cin % 256 == 0 && g.B >= 512)
      variant = v256;
    else if (c3 && Cin == 512)
      variant = 24;
    else if (c3 && Cin == 128)
      variant = g.B >= 1024 && huge_tiles_env(16) ? 27 : 23;  // batch 1024: 323 vs 338 us
    else if (c3 && Cin == 64)
      // row-window kernel for 64 -> 64 (stage 1 of E18 / QuickNet, batch
      // 1024: 430 vs 513-574 us for variant 27; profiles/r3/f_conv3rw.md)
      variant = (g_opt_dgrad_rw && g.Cout == 64 && g.W <= 64) ? 50 : 27;
    else if (Cin % 128 == 0)
      variant = 0;
    else
      variant = 7;
  }
  if (variant == 60) {  // deep_gemm.hip (explicit, or the default above)
    if (bs.fstats || bs.sums || bs.bsums || bs.dmask) return (int)hipErrorInvalidValue;
    return zk_dgrad_deep_impl(dy, wt, mask, dres, dx, g.B, g.H, g.W, g.Cin, g.Cout, g.Ho, g.Wo,
                              g.kh, g.kw, g.s, g.pt, g.pl, g_dry_run, stream);
  }
  if (variant == 50) {  // conv3rw.hip (explicit, or the default above)
    if (bs.fstats || bs.bsums || bs.dmask) return (int)hipErrorInvalidValue;
    if (g.s != 1 || g.kh != 3 || g.kw != 3 || g.pt != 1 || g.pl != 1 || g.Ho != g.H ||
        g.Wo != g.W)
      return (int)hipErrorInvalidValue;
    return zk_conv3rw_dgrad_impl(dy, wt, mask, dres, dx, g.B, g.H, g.W, g.Cin, g.Cout, bs.ypred,
                                 bs.mean, bs.rstd, bs.sums, bs.stripes, bs.ypred_bf16, g_dry_run,
                                 stream);
  }
  // bf16 predecessor outputs: only the row-window epilogue converts them
  if (bs.ypred_bf16) return (int)hipErrorInvalidValue;
  const int rc = igemm_dgrad_variant(variant, dy, wt, mask, dres, dx, g, bs, stream);
  if (rc) return rc;
  if (!g_dry_run) ZK_CHECK_LAUNCH();
  return 0;
}
}  // namespace

// Same contract as zk_bconv_dgrad (binary_conv_bwd.hip): wt ±1 bf16
// [T][Cin][Cout], mask / dres optional, Cout % 64 == 0, Cin % BN == 0.
ZK_EXPORT int zk_igemm_dgrad(const void* dy, const void* wt, const void* mask, const void* dres,
                             void* dx, int B, int H, int W, int Cin, int Ho, int Wo, int Cout,
                             int kh, int kw, int stride, int pt, int pl, int variant,
                             hipStream_t stream) {
  IGeom g{B, H, W, Cin, Ho, Wo, Cout, kh, kw, stride, pt, pl};
  return igemm_dgrad_impl(dy, wt, mask, dres, dx, g, BnSum{nullptr, nullptr, nullptr, nullptr, 1},
                          variant, stream);
}

// zk_igemm_dgrad + the previous block's BN-backward reduction fused into the
// epilogue: sums [2][Cin][stripes] fp32 (channel-major) += (sum dx, sum dx * (ypred - mean) *
// rstd) over the stored bf16 dx (ypred int16 [B][H][W][Cin]; mean / rstd
// [Cin]).  Valid when dx is that block's whole output gradient.
ZK_EXPORT int zk_igemm_dgrad_bnsum(const void* dy, const void* wt, const void* mask,
                                   const void* dres, void* dx, const void* ypred, const void* mean,
                                   const void* rstd, void* sums, int stripes, int ypred_bf16,
                                   int B, int H, int W, int Cin, int Ho, int Wo, int Cout, int kh,
                                   int kw, int stride, int pt, int pl, int variant,
                                   hipStream_t stream) {
  IGeom g{B, H, W, Cin, Ho, Wo, Cout, kh, kw, stride, pt, pl};
  if (!ypred || !mean || !rstd || !sums || Cin % 32) return (int)hipErrorInvalidValue;
  return igemm_dgrad_impl(dy, wt, mask, dres, dx, g,
                          BnSum{ypred, mean, rstd, sums, stripes < 1 ? 1 : stripes, nullptr,
                                ypred_bf16 ? 1 : 0},
                          variant, stream);
}

// Float 1x1 forward as this GEMM (roles renamed as in ops/pointwise.py:
// x = "dy" [P][K], W = "wt" [N][K], y = "dx" [P][N] bf16) with the next
// BatchNorm's statistics of the stored outputs: fstats [stripes][2][N] fp64
// += (sum y, sum y^2) (zeroed by the caller; zk_bn_finalize_f64_parts sums the
// stripes).  Only the LDS-epilogue variants carry the statistics: any other
// (default or explicit) choice returns hipErrorInvalidValue and the caller
// keeps the separate statistics pass.
ZK_EXPORT int zk_igemm_dgrad_fstats(const void* dy, const void* wt, void* dx, void* fstats,
                                    int stripes, int B, int H, int W, int Cin, int Ho, int Wo,
                                    int Cout, int kh, int kw, int stride, int pt, int pl,
                                    int variant, hipStream_t stream) {
  IGeom g{B, H, W, Cin, Ho, Wo, Cout, kh, kw, stride, pt, pl};
  if (!fstats || Cin % 8) return (int)hipErrorInvalidValue;
  return igemm_dgrad_impl(dy, wt, nullptr, nullptr, dx, g,
                          BnSum{nullptr, nullptr, nullptr, nullptr, stripes < 1 ? 1 : stripes,
                                fstats},
                          variant, stream);
}

// zk_igemm_dgrad with the LDS-epilogue extras (a tile with the LDS epilogue
// only: any other choice returns hipErrorInvalidValue and the caller keeps
// the separate passes):
//  * dres_mask (optional): bits [P][Cin/8] masking dres before it is added;
//  * sums (optional): the backward sums of the float BatchNorm whose output
// gradient dx is (its whole gradient): sums [stripes][2][Cin] fp32, row m =
// the M tile m's (sum g', sum g' * (xb - mean) * rstd) (plain stores: stripes
// >= the tiles of any LDS-epilogue variant, BM >= 128, so >= ceil(B*H*W /
// 128); the rows of unused tiles must be zero: zk_bn_bwd_tiles_reduce folds
// all stripes rows in a fixed order and re-zeroes them) with g' = the
// stored dx times the BN's ReLU mask (relu 0: none, 1: recomputed from xb
// and the forward scale / shift, 2: bits mask [P][Cin/8]); xb bf16
// [B][H][W][Cin] is the BN input, coef [4][Cin] = scale, shift, mean, rstd.
ZK_EXPORT int zk_igemm_dgrad_ex(const void* dy, const void* wt, const void* dres,
                                const void* dres_mask, void* dx, const void* xb,
                                const void* coef, const void* mask, int relu, void* sums,
                                int stripes, int B, int H, int W, int Cin, int Ho, int Wo,
                                int Cout, int kh, int kw, int stride, int pt, int pl, int variant,
                                hipStream_t stream) {
  IGeom g{B, H, W, Cin, Ho, Wo, Cout, kh, kw, stride, pt, pl};
  if (Cin % 8 || (dres_mask && !dres) || (!sums && !dres_mask)) return (int)hipErrorInvalidValue;
  if (sums && (!xb || !coef || relu < 0 || relu > 2 || (relu == 2 && !mask) || stride != 1))
    return (int)hipErrorInvalidValue;
  BnSum bs{nullptr, nullptr, nullptr, nullptr, stripes < 1 ? 1 : stripes};
  if (sums) {
    bs.bxb = xb;
    bs.bcoef = coef;
    bs.bmask = mask;
    bs.brelu = relu;
    bs.bsums = sums;
  }
  bs.dmask = dres_mask;
  return igemm_dgrad_impl(dy, wt, nullptr, dres, dx, g, bs, variant, stream);
}

namespace {
void wgrad_defaults(const IGeom& g, int& variant, int& target_blocks) {
  if (variant < 0) {
    // Tuned on MI355X (tools/tune_bconv.py --only igw, E18 shapes, batch 256)
    // (slab split-K reduction).  3x3 stride-1 'same' layers with 64 / 128
    // input channels: the conv3 kernel (profiles/r1at_wgrad3_tuning.md:
    // 56x56x64 145 -> 107 us, 28x28x128 102 -> 96 us at batch 256); the
    // 256 / 512-channel layers stay on 128x128 tiles (no gain there).
    // Batch >= 512 (profiles/r1av_bconv_tuning_b512.md): twice the blocks for
    // the 128-channel layers (28x28x128: 262 -> 183 us), and 256x256 tiles
    // with 512 blocks for the 256-input-channel 3x3 layers (14x14x256:
    // 235 -> 168 us; 256 -> 512 stride 2: 130 -> 106 us).
    // Batch >= 1024, opt-in (tile_huge option, see huge_tiles_env; standalone
    // tools/tune_bconv.py --batch 1024): 28x28x128 on the 64x64 three-row
    // conv3 tiles (406 -> 347 us), 256-input-channel layers on 256x256 x 3
    // stages at 1024 blocks (417 -> 349 us), the 64 -> 128 transition at 1024
    // blocks (329 -> 222 us), 7x7x512 on 128x128 at 2048 blocks (392 vs 400).
    const bool c3 = conv3_ok(g, 0);
    const bool big = g.B >= 512, huge = g.B >= 1024;
    if (g_opt_wgrad_deep && c3 && g.Cin % 256 == 0 && g.Cout % 256 == 0) {
      variant = 60;  // phased 256x256 schedule (deep_gemm.hip)
      if (target_blocks <= 0) target_blocks = 512;
    } else if (c3 && g.Cin == 64 && g.Cout % 64 == 0) {
      variant = 20;
      if (target_blocks <= 0) target_blocks = 512;
    } else if (huge && huge_tiles_env(1) && c3 && g.Cin == 128 && g.Cout % 64 == 0) {
      variant = 20;
      if (target_blocks <= 0) target_blocks = 512;
    } else if (c3 && g.Cin == 128 && g.Cout % 128 == 0) {
      variant = 28;
      if (target_blocks <= 0) target_blocks = big ? 1024 : 512;
    } else if (huge && huge_tiles_env(2) && g.kh == 3 && g.kw == 3 && g.Cin == 256 &&
               g.Cout % 256 == 0) {
      variant = 12;
      if (target_blocks <= 0) target_blocks = 1024;
    } else if (big && g.kh == 3 && g.kw == 3 && g.Cin == 256 && g.Cout % 256 == 0) {
      variant = 8;
      if (target_blocks <= 0) target_blocks = 512;
    } else if (big && !(huge && huge_tiles_env(8)) && g.kh == 3 && g.kw == 3 && g.Cin == 512 &&
               g.Cout % 256 == 0) {
      // 7x7x512 at batch 512: 256x256 tiles, 384 blocks 198 us vs 128x128
      // at 2048 blocks 217-221 us (tools/tune_bconv.py --tbs 128..768)
      variant = 8;
      if (target_blocks <= 0) target_blocks = 384;
    } else if (g.Cin == 64 && g.s == 2 && g.Cout % 128 == 0 && (9 * g.Cin) % 192 == 0) {
      variant = 2;
      if (target_blocks <= 0) target_blocks = huge && huge_tiles_env(4) ? 1024 : 512;
    } else if (g.Cin == 64 || g.Cout % 128 != 0) {
      variant = 7;
      if (target_blocks <= 0) target_blocks = 2048;
    } else {
      variant = 4;  // 128x128, 64-pixel K-steps
      if (target_blocks <= 0)
        target_blocks = (g.Cout >= 512 && g.s == 1) ? 2048
                        : (g.Cin >= 256 || g.Cout >= 512 || big) ? 1024 : 512;
    }
  }
  if (target_blocks <= 0) target_blocks = 1024;
}
}  // namespace

// dW fp32 [Cout][T][Cin] accumulated in place (zeroed by the caller or the
// flat gradient buffer itself).  sx: sign(x) bf16 +-1 [B][H][W][Cin].
// workspace (optional, zk_igemm_wgrad_ws_bytes) switches the split-K
// reduction from fp32 atomics to per-split slabs + one reduce kernel.
ZK_EXPORT int zk_igemm_wgrad(const void* dy, const void* sx, const void* w, void* dw, int B,
                             int H, int W, int Cin, int Ho, int Wo, int Cout, int kh, int kw,
                             int stride, int pt, int pl, int pad_ones, float clip,
                             int target_blocks, int variant, void* workspace,
                             long long ws_bytes, hipStream_t stream) {
  IGeom g{B, H, W, Cin, Ho, Wo, Cout, kh, kw, stride, pt, pl};
  wgrad_defaults(g, variant, target_blocks);
  const int rc = igemm_wgrad_variant(variant, dy, sx, w, dw, g, pad_ones, clip, target_blocks,
                                     workspace, ws_bytes, nullptr, stream);
  if (rc) return rc;
  if (!g_dry_run) ZK_CHECK_LAUNCH();
  return 0;
}

// dw[i] += [|w[i]| <= clip] * sum_s slab[s][i] (w null: no mask), summed in a
// fixed order: the deterministic-mode reduction of every split-K weight
// gradient (igemm, small-K convs, depthwise, stem).  n % 4 == 0.
ZK_EXPORT int zk_wgrad_slab_reduce(const void* slab, int splits, long long n, const void* w,
                                   float clip, void* dw, hipStream_t stream) {
  if (n % 4 || splits < 1) return (int)hipErrorInvalidValue;
  const long long n4 = n / 4;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, stream,
                     (const float4*)slab, splits, n4, (const float4*)w, clip, (float4*)dw);
  ZK_CHECK_LAUNCH();
  return 0;
}

// Workspace bytes zk_igemm_wgrad needs for slab mode (-1: shape unsupported).
ZK_EXPORT long long zk_igemm_wgrad_ws_bytes(int B, int Cin, int H, int W, int Ho, int Wo,
                                            int Cout, int kh, int kw, int stride, int pt, int pl,
                                            int target_blocks, int variant) {
  IGeom g{B, H, W, Cin, Ho, Wo, Cout, kh, kw, stride, pt, pl};
  wgrad_defaults(g, variant, target_blocks);
  long long need = -1;
  if (igemm_wgrad_variant(variant, nullptr, nullptr, nullptr, nullptr, g, 0, 0.f,
                          target_blocks, nullptr, 0, &need, nullptr) != 0)
    return -1;
  return need;
}

// Binary forward on MFMA: y int16 [B][Ho][Wo][Cout] = conv(sign x, sign W)
// (+ReLU), stats [stat_stripes][2][Cout] int64 += (sum y, sum y^2) (zeroed
// by the caller; the copies are summed by zk_bn_finalize).
// sx: bf16 +-1 [B][H][W][Cin]; wf: bf16 +-1 [T][Cout][Cin].
ZK_EXPORT int zk_igemm_fwd(const void* sx, const void* wf, void* y, void* stats, int B, int H,
                           int W, int Cin, int Cout, int kh, int kw, int stride, int pt, int pl,
                           int Ho, int Wo, int pad_ones, int relu, int variant, int stat_stripes,
                           hipStream_t stream) {
  IGeom g{B, H, W, Cin, Ho, Wo, Cout, kh, kw, stride, pt, pl};
  if (variant < 0) {
    // Tuned on MI355X (tools/tune_bconv.py --only igf, E18 shapes, batch 256)
    const bool c3 = conv3_ok(g, pad_ones);
    if (c3 && Cout == 64)
      variant = 27;  // conv3: horizontal tap reuse
    else if (c3 && Cout == 128)
      variant = 27;
    else if (c3 && Cout == 512)
      variant = 24;
    else if (Cin == 64 || Cout % 128 != 0)
      variant = (Cout == 64) ? 8 : 7;
    else if (Cout == 256)
      variant = 14;  // 256x256: half the LDS-fill bytes per FLOP, ~200 tiles
    else
      variant = 0;
  }
  const int rc =
      igemm_fwd_variant(variant, sx, wf, y, stats, g, pad_ones, relu, stat_stripes, stream);
  if (rc) return rc;
  if (!g_dry_run) ZK_CHECK_LAUNCH();
  return 0;
}

// Binary forward on MX-FP4 MFMA (v_mfma_f32_32x32x64_f8f6f4, e2m1 operands):
// the contract of zk_igemm_fwd with 4-bit sign images -- sx4: e2m1 +-1
// [B][H][W][Cin/2 bytes] (channel 2j in the low nibble of byte j; zk_sign_pack
// / the BN epilogues write it), wf4: [T][Cout][Cin/2] (zk_weight_pack).
// Cin % 64 == 0.  4x the MFMA rate and a quarter of the operand bytes of the
// bf16 form, the same exact integer outputs and statistics.
ZK_EXPORT int zk_igemm_fwd_fp4(const void* sx4, const void* wf4, void* y, void* stats, int B,
                               int H, int W, int Cin, int Cout, int kh, int kw, int stride, int pt,
                               int pl, int Ho, int Wo, int pad_ones, int relu, int variant,
                               int stat_stripes, hipStream_t stream) {
  IGeom g{B, H, W, Cin, Ho, Wo, Cout, kh, kw, stride, pt, pl};
  if (Cin % 64 || Cout % 64) return (int)hipErrorInvalidValue;
  if (variant < 0) {
    const bool c3 = conv3_ok(g, pad_ones);
    // Tuned on MI355X (tools/tune_bconv.py --only igf4, E18 shapes, batch 256);
    // at batch 512 the 256x256 tiles also win for Cin >= 256 once the output
    // image has >= 25088 pixels (7x7x512: 47 -> 38 us; 256 -> 512 stride 2:
    // 37 -> 27 us; profiles/r1av_bconv_tuning_b512.md).
    const long long Po = (long long)g.B * g.Ho * g.Wo;
    const bool wide = Cin % 256 == 0 && Cout % 256 == 0 && Po >= 25088;
    if (c3 && (Cin == 64 || Cin == 128) && Cout == Cin && Ho == H && Wo == W &&
        zk_bfwd_supported(B, H, W, Cin, Cout, kh, kw, stride, pt, pl))
      // persistent, LDS-resident weights (bfwd.hip, profiles/r6/bfwd.md): batch
      // 1536, 56x56x64 285 -> 151 us, 28x28x128 204 -> 109 us
      variant = 40;
    else if (c3 && Cin == 64)
      variant = 20;
    else if (c3 && Cin == 256 && Cout % 256 == 0)
      variant = 26;
    else if (c3 && wide)
      variant = 26;
    else if (!c3 && wide)
      variant = 5;
    else if (c3 && Cin >= 256 && Cout % 128 == 0)
      variant = 23;
    else if (c3)
      variant = 27;
    else if (Cin == 64)
      variant = Cout % 128 == 0 ? 0 : 4;
    else if (Cin == 128)
      variant = Cout % 128 == 0 ? 6 : 8;
    else
      variant = Cout % 128 == 0 ? 1 : 8;
  }
  // lab switch (option 9, tools/one_conv.py --no-y): statistics only, no y
  // stores -- the cost of the int16 output in the fp4 forward
  const int rc = igemm_fwd4_variant(variant, sx4, wf4, g_opt_lab_fwd_no_y ? nullptr : y, stats, g,
                                    pad_ones, relu, stat_stripes, stream);
  if (rc) return rc;
  if (!g_dry_run) ZK_CHECK_LAUNCH();
  return 0;
}

// Float forward convolution on MFMA: y bf16 [B][Ho][Wo][Cout] = x ⊛ W (+ReLU);
// x bf16 [B][H][W][Cin], wf bf16 [T][Cout][Cin] (T = kh*kw, tap-major).
// Any stride <= 2 and kernel <= 4x4 (ResNet-50's strided 3x3 / 1x1 convs);
// Cin % 64 == 0, Cout % 64 == 0.
ZK_EXPORT int zk_igemm_fwd_bf16(const void* x, const void* wf, void* y, int B, int H, int W,
                                int Cin, int Cout, int kh, int kw, int stride, int pt, int pl,
                                int Ho, int Wo, int relu, int variant, hipStream_t stream) {
  IGeom g{B, H, W, Cin, Ho, Wo, Cout, kh, kw, stride, pt, pl};
  if (variant < 0) {
    const long long Mo = (long long)B * Ho * Wo;
    if (Cout % 256 == 0 && Cin % 64 == 0 && Mo * (Cout / 256) >= 256 * 256)
      variant = 3;  // 256x256: half the LDS-fill bytes per FLOP when the grid stays full
    else if (Cout % 128 == 0)
      variant = Mo >= 65536 ? 1 : 0;
    else
      variant = 2;
  }
  const int rc = igemm_fwd_bf16_variant(variant, x, wf, y, g, relu, stream);
  if (rc) return rc;
  if (!g_dry_run) ZK_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------
// Support queries: 1 if the tile variant accepts the geometry, 0 if not
// (nothing is launched; no GPU needed).  variant -1 = the tuned default.
namespace {
struct DryRun {
  DryRun() { g_dry_run = true; }
  ~DryRun() { g_dry_run = false; }
};
}  // namespace

ZK_EXPORT int zk_igemm_dgrad_supported(int B, int H, int W, int Cin, int Ho, int Wo, int Cout,
                                       int kh, int kw, int stride, int pt, int pl, int variant) {
  DryRun dr;
  return zk_igemm_dgrad(nullptr, nullptr, nullptr, nullptr, nullptr, B, H, W, Cin, Ho, Wo, Cout,
                        kh, kw, stride, pt, pl, variant, nullptr) == 0;
}

ZK_EXPORT int zk_igemm_fwd_bf16_supported(int B, int H, int W, int Cin, int Cout, int kh,
                                          int kw, int stride, int pt, int pl, int Ho, int Wo,
                                          int variant) {
  DryRun dr;
  return zk_igemm_fwd_bf16(nullptr, nullptr, nullptr, B, H, W, Cin, Cout, kh, kw, stride, pt, pl,
                           Ho, Wo, 0, variant, nullptr) == 0;
}

ZK_EXPORT int zk_igemm_fwd_supported(int B, int H, int W, int Cin, int Cout, int kh, int kw,
                                     int stride, int pt, int pl, int Ho, int Wo, int pad_ones,
                                     int variant, int fp4) {
  DryRun dr;
  if (fp4)
    return zk_igemm_fwd_fp4(nullptr, nullptr, nullptr, nullptr, B, H, W, Cin, Cout, kh, kw, stride,
                            pt, pl, Ho, Wo, pad_ones, 0, variant, 1, nullptr) == 0;
  return zk_igemm_fwd(nullptr, nullptr, nullptr, nullptr, B, H, W, Cin, Cout, kh, kw, stride, pt,
                      pl, Ho, Wo, pad_ones, 0, variant, 1, nullptr) == 0;
}

// Host-side kernel options (see g_opt_* above; ops/options.py).  Returns 0,
// or -1 for an unknown key.
ZK_EXPORT int zk_set_option(int key, int value) {
  switch (key) {
    case 0: g_opt_tile_huge = value; return 0;
    case 2: g_opt_deterministic = value; return 0;
    case 3: g_opt_dgrad_rw = value; return 0;
    case 5: g_opt_wgrad_slab_mb = value; return 0;
    case 6: g_opt_dgrad_deep = value; return 0;
    case 7: g_opt_wgrad_deep = value; return 0;
    case 8: g_opt_epilogue_prefetch = value; return 0;
    case 9: g_opt_lab_fwd_no_y = value; return 0;
    case 10: g_opt_wgrad_tree = value; return 0;
    default: return -1;
  }
}

ZK_EXPORT int zk_get_option(int key) {
  switch (key) {
    case 0: return g_opt_tile_huge;
    case 2: return g_opt_deterministic;
    case 3: return g_opt_dgrad_rw;
    case 5: return g_opt_wgrad_slab_mb;
    case 6: return g_opt_dgrad_deep;
    case 7: return g_opt_wgrad_deep;
    case 8: return g_opt_epilogue_prefetch;
    case 9: return g_opt_lab_fwd_no_y;
    case 10: return g_opt_wgrad_tree;
    default: return -1;
  }
}
