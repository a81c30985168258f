// Row-window data gradient of the 64 -> 64-channel stride-1 3x3 'same'
// binary conv (BinaryResNet-E18 / QuickNet stage 1: 56x56x64), gfx950.
//
//   dx[b][h][w][ci] = mask(x) * sum_{kh,kw,co} dY[b][h+1-kh][w+1-kw][co] * S[kh][kw][ci][co]
//                     + dres[b][h][w][ci]
//
// The implicit-GEMM kernels (igemm.hip conv3) stage, per K-step, BM+2 dY rows
// for one kernel row plus the three taps' weight rows: ~57 KB per K-step for
// 1.5k MFMA cycles, fill latency exposed with one block per CU (measured
// 0.43-0.46 PF/s, 2.5x the HBM floor; profiles/r3/e_conv3_wave_tile_variants.md).
// Here instead:
//   * the whole weight tensor S^T [9][64 ci][64 co] (72 KB) is loaded into LDS
//     once per persistent block and stays resident;
//   * a block owns a contiguous range of work items (image b, group of 4
//     output rows); dY image rows live in a 10-slot LDS ring (slot = row % 10):
//     a group reads rows h0-1 .. h0+4, and while it computes, the 4 rows the
//     next group adds (h0+5 .. h0+8) stream in by LDS-DMA
//     (global_load_lds_dwordx4), one row per wave -- every dY row is fetched
//     once per block instead of three times per tile;
//   * all 9 taps x 64 co of a group are MFMAs over LDS-resident operands
//     (v_mfma_f32_16x16x32_bf16, transposed product D[ci][pixel]: A = weight
//     rows, B = dY pixel rows, so a lane owns one pixel and 4 consecutive
//     channels in the epilogue); 8 waves (2 per SIMD, so one wave's epilogue
//     and DMA overlap the other's MFMAs): wave w takes ci half (w & 1) and
//     every 4th 16-pixel block from (w >> 1) -> <= 4 blocks x 2 ci blocks;
//   * LDS rows are 128 B (64 channels); 16-B chunk c of pixel (or ci) p sits at
//     slot c ^ rw_swz(p) (conflict-free ds_read_b128 at every tap shift, see
//     rw_swz).  The DMA writes LDS linearly, so the swizzle is applied to the
//     SOURCE address.
//   * padding taps (rows -1 / H, columns -1 / W) read a 256-B zero chunk.
// Persistent grid: one block per CU (LDS ~144 KB at W = 56).
#include "mfma_common.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// Lab-only ablation bits (tools/gemm_lab/rw_lab.hip builds with -DRW_ABL=n;
// the library always builds 0): 1 no epilogue, 2 no row prefetch, 4 no MFMA,
// 8 no dY fragment reads.
#ifndef RW_ABL
#define RW_ABL 0
#endif

constexpr int RW_TR = 4;                         // output rows per work item
constexpr int RW_NW = 8;                         // waves per block (2 per SIMD)
constexpr int RW_MB = 4;                         // 16-pixel blocks per wave (stride RW_NW/2)
constexpr int RW_RING = 10;                      // dY row slots (TR + 2 + TR)
constexpr int RW_WBYTES = 9 * 64 * 128;          // resident weights
constexpr int RW_ZERO = RW_WBYTES;               // 256 B of zeros
constexpr int RW_RING_OFF = RW_WBYTES + 1024;    // ring base, 1 KB aligned

// STE mask word of "every channel live" (the mask-less call)
__device__ uint32_t g_rw_ones[4] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};

struct RWArgs {
  const uint16_t* dy;    // [B][H][W][64]
  const uint16_t* wt;    // S^T [9][64 ci][64 co]
  const uint32_t* mask;  // STE bits [B*H*W][2] (optional)
  const uint16_t* dres;  // residual gradient [B][H][W][64] (optional)
  uint16_t* dx;          // [B][H][W][64]
  int B, H, W, ngroups, ipb, slot;
  // optional: the predecessor block's BN-backward reduction over the stored
  // dx (its output gradient): psums[0][c][stripe] += sum dx,
  // [1][c][stripe] += sum dx * (ypred - mean[c]) * rstd[c]  (ypred int16, or bf16
  // with ypred_bf16, [B][H][W][64])
  const int16_t* ypred;
  const float* pmean;
  const float* prstd;
  float* psums;
  int stripes;
  int ypred_bf16;  // ypred holds bf16 values (the stem's pooled BN-2 input), not int16
};

// vmcnt(0) through the builtin (expcnt / lgkmcnt left at their maxima), so
// the compiler's own wait tracking knows every earlier load and store has
// retired: after the asm-volatile form it still assumed the previous item's
// epilogue loads outstanding and drained vmcnt again at the next item's
// start -- right after issuing the row DMA, which it then waited for.
__device__ __forceinline__ void rw_drain() { __builtin_amdgcn_s_waitcnt(0x0F70); }

__device__ __forceinline__ f32x4 mfma16(const uint4& a, const uint4& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// Chunk swizzle key of 128-B row r (pixel column or weight row ci): the
// 16-B chunk c is stored at c ^ rw_swz(r).  A ds_read_b128 lane group holds 8
// pixels reading chunk c and 8 reading chunk c+1 (k = 8*(lane>>4)+j), the
// pixels 16 consecutive columns at any tap shift; with an even key (c and
// c+1 never meet) cycling over 4 values per 8 columns, every such group
// lands on 16 distinct bank slots (checked exhaustively over all shifts and
// both group shapes; the plain (r>>1)&7 key was 2-way on odd shifts:
// SQ_LDS_BANK_CONFLICT 2.1 cycles per LDS instruction).
__device__ __forceinline__ int rw_swz(int r) { return ((r >> 1) & 3) << 1; }

// Weight rows: ci(j, r) = nh*32 + (r >> 2)*8 + j*4 + (r & 3) for A-fragment
// row r of ci block j (so the epilogue lane owns 8 consecutive channels, 16-B
// stores); a lane group then holds ci = 8q + 4j + e with q in {0,3} reading
// chunk c and q in {1,2} reading c+1: an even key from bits 1 and 4 of ci
// keeps the 16 reads on distinct bank slots.
__device__ __forceinline__ int rw_swz_w(int ci) {
  return (((ci >> 1) & 1) << 1) | (((ci >> 4) & 1) << 2);
}

// One wave DMAs dY row hr of image b into its ring slot (1 KB = 8 pixels per
// instruction; lanes past the row's end load the zero page into the slot's
// padding).
__device__ __forceinline__ void rw_load_row(const RWArgs& a, unsigned char* smem, int b, int hr,
                                            int lane, int k0 = 0, int kstep = 1) {
  unsigned char* slot = smem + RW_RING_OFF + (hr % RW_RING) * a.slot;
  const uint16_t* src = a.dy + ((long long)b * a.H + hr) * a.W * 64;
  const int nblk = (a.W + 7) >> 3;
  for (int k = k0; k < nblk; k += kstep) {
    const int J = k * 64 + lane, p = J >> 3, q = J & 7;
    const int c = q ^ rw_swz(p);
    const void* s = (p < a.W) ? (const void*)(src + p * 64 + c * 8) : (const void*)g_zero_page;
    glds16(s, slot + k * 1024);
  }
}

__global__ __launch_bounds__(RW_NW * 64, 1) void conv3rw_dgrad_kernel(RWArgs a) {
  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int nitems = a.B * a.ngroups;
  const int i0 = blockIdx.x * a.ipb;
  if (i0 >= nitems) return;  // block-uniform
  const int i1 = min(nitems, i0 + a.ipb);
  if (tid < 16) reinterpret_cast<uint4*>(smem + RW_ZERO)[tid] = make_uint4(0u, 0u, 0u, 0u);
  // resident weights: 72 x 1 KB, wave w takes blocks w, w + 4, ...
  for (int k = wave; k < 72; k += RW_NW) {
    const int J = k * 64 + lane, row = J >> 3, q = J & 7, ci = row & 63;
    glds16(a.wt + row * 64 + ((q ^ rw_swz_w(ci)) * 8), smem + k * 1024);
  }
  const int nh = wave & 1, mh = wave >> 1, r16 = lane & 15, kq = lane >> 4;  // mh: 0..3
  // A-fragment LDS offsets of this lane (tap 0, chunk kc*4 + kq): ci = nh*32 + j*16 + r16
  int aoff[2][2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int ci = nh * 32 + (r16 >> 2) * 8 + j * 4 + (r16 & 3);
#pragma unroll
    for (int kc = 0; kc < 2; ++kc) aoff[j][kc] = ci * 128 + (((kc * 4 + kq) ^ rw_swz_w(ci)) * 16);
  }

  // fused BN-backward sums of this lane's 8 channels, over all its pixels
  const bool bnsum = a.psums != nullptr;
  float s1[8], s2[8], mu[8], rs[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    s1[e] = s2[e] = 0.f;
    mu[e] = bnsum ? a.pmean[nh * 32 + kq * 8 + e] : 0.f;
    rs[e] = bnsum ? a.prstd[nh * 32 + kq * 8 + e] : 0.f;
  }

  // The previous item's packed dx chunks, stored one block per tap during
  // the next item's MFMAs (measured equal to storing them at once, 427-433 us
  // either way at batch 1024; kept: it spreads the write stream).
  uint4 pend[RW_MB];
  long long poff[RW_MB];
#pragma unroll
  for (int i = 0; i < RW_MB; ++i) poff[i] = -1;

  for (int it = i0; it < i1; ++it) {
    const int b = it / a.ngroups, g = it - b * a.ngroups, h0 = g * RW_TR;
    // Every wave waited for its own DMA (this item's rows) before its previous
    // epilogue, so a bare barrier publishes them -- no vmcnt drain here, which
    // would also wait for the previous epilogue's dx stores.
    __builtin_amdgcn_s_barrier();
    if (it == i0 || g == 0) {
      // first item of the block or of an image: load rows h0-1 .. h0+4 now
      for (int r = wave; r < RW_TR + 2; r += RW_NW) {
        const int hr = h0 - 1 + r;
        if (hr >= 0 && hr < a.H) rw_load_row(a, smem, b, hr, lane);
      }
      rw_drain();  // these rows (and, first time, the weights) are in LDS
      __builtin_amdgcn_s_barrier();
    }
    // the next group's 4 new rows, one per wave (same image only)
    if (it + 1 < i1 && g + 1 < a.ngroups) {
      // row (wave & 3) of the 4, its even / odd 1-KB pieces by waves < 4 / >= 4
      const int hr = h0 + RW_TR + 1 + (wave & 3);
      if (hr < a.H && !(RW_ABL & 2)) rw_load_row(a, smem, b, hr, lane, wave >> 2, 2);
    }

    const int rv = min(RW_TR, a.H - h0), npx = rv * a.W;
    // this lane's pixel in each of its RW_MB 16-pixel blocks mb = 4i + mh
    int pr[RW_MB], pw[RW_MB];
#pragma unroll
    for (int i = 0; i < RW_MB; ++i) {
      const int p = ((RW_NW / 2) * i + mh) * 16 + r16;
      pr[i] = p / a.W;
      pw[i] = p - pr[i] * a.W;
      if (p >= npx) pr[i] = -1000;  // invalid: every tap reads the zero chunk
    }
    // epilogue operands (STE mask byte, 16 B of residual gradient) requested
    // now and consumed after the MFMAs, which hide their latency
    uint32_t mw[RW_MB];
    uint4 dr[RW_MB], yp[RW_MB];
    long long pgo[RW_MB];
    // Unconditional loads from a valid address (pixel 0 for lanes without a
    // pixel, a constant page without mask / dres) and no use before the
    // epilogue: a predicated load, or one whose value is shifted right away,
    // made the compiler drain vmcnt here -- which also waited for the row DMA
    // just issued.
    const uint32_t* mbase = a.mask ? a.mask : g_rw_ones;
    const uint16_t* dbase = a.dres ? a.dres : reinterpret_cast<const uint16_t*>(g_zero_page);
#pragma unroll
    for (int i = 0; i < RW_MB; ++i) {
      const bool ok = pr[i] >= 0;
      const long long pc = ok ? ((long long)b * a.H + h0 + pr[i]) * a.W + pw[i] : 0;
      pgo[i] = ok ? pc : -1;
      mw[i] = mbase[a.mask ? pc * 2 + nh : 0];
      dr[i] = *reinterpret_cast<const uint4*>(dbase + (a.dres ? pc * 64 + nh * 32 + kq * 8 : 0));
      yp[i] = *reinterpret_cast<const uint4*>(
          bnsum ? reinterpret_cast<const uint16_t*>(a.ypred) + pc * 64 + nh * 32 + kq * 8
                : reinterpret_cast<const uint16_t*>(g_zero_page));
    }
    f32x4 acc[RW_MB][2];
#pragma unroll
    for (int i = 0; i < RW_MB; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};

    // per block i and kernel row kh: LDS base of the dY row h0 + pr + 1 - kh
    // (-1: row outside the image or no pixel); the ring slot from the
    // block-uniform h0 % 10 -- no per-lane division, no branches
    const int s0 = h0 % RW_RING;
    int rb[RW_MB][3];
#pragma unroll
    for (int i = 0; i < RW_MB; ++i)
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        const int rr = pr[i] + 1 - kh;
        int sl = s0 + rr;
        sl += sl < 0 ? RW_RING : 0;
        sl -= sl >= RW_RING ? RW_RING : 0;
        const bool ok = (unsigned)(h0 + rr) < (unsigned)a.H;
        rb[i][kh] = ok ? RW_RING_OFF + sl * a.slot : -1;
      }

#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int kh = t / 3, kw = t % 3;
      if (t < RW_MB && poff[t] >= 0) *reinterpret_cast<uint4*>(a.dx + poff[t]) = pend[t];
      int boff[RW_MB], bsw[RW_MB];  // pixel row base and its chunk swizzle key (zero chunk: key 0)
#pragma unroll
      for (int i = 0; i < RW_MB; ++i) {
        const int wc = pw[i] + 1 - kw;
        const bool ok = rb[i][kh] >= 0 && (unsigned)wc < (unsigned)a.W;
        boff[i] = ok ? rb[i][kh] + wc * 128 : RW_ZERO;
        bsw[i] = ok ? rw_swz(wc) : 0;
      }
#pragma unroll
      for (int kc = 0; kc < 2; ++kc) {
        const uint4 a0 = *reinterpret_cast<const uint4*>(smem + t * 8192 + aoff[0][kc]);
        const uint4 a1 = *reinterpret_cast<const uint4*>(smem + t * 8192 + aoff[1][kc]);
        const int ch = kc * 4 + kq;
        // all 8 blocks unconditionally (blocks past the item read the zero
        // chunk): no branches between the fragment reads and the MFMAs
        uint4 bv[RW_MB];
#pragma unroll
        for (int i = 0; i < RW_MB; ++i)
          bv[i] = (RW_ABL & 8) ? make_uint4(a0.x ^ i, a0.y, a1.z, boff[i] ^ bsw[i])
                               : *reinterpret_cast<const uint4*>(smem + boff[i] + ((ch ^ bsw[i]) * 16));
#pragma unroll
        for (int i = 0; i < RW_MB; ++i) {
          if constexpr ((RW_ABL & 4) != 0) {
            acc[i][0][0] += __builtin_bit_cast(float, bv[i].x & 0x3fffffffu);
            acc[i][1][0] += __builtin_bit_cast(float, bv[i].y & 0x3fffffffu);
          } else {
            acc[i][0] = mfma16(a0, bv[i], acc[i][0]);
            acc[i][1] = mfma16(a1, bv[i], acc[i][1]);
          }
        }
      }
    }

    // the next item's rows (and this item's epilogue operands) have landed:
    // wait now, while only the previous epilogue's stores -- long since
    // issued -- are ahead of them
    rw_drain();
    // epilogue: lane = pixel, rows 4*kq .. +3 of each 16-ci block
#pragma unroll
    for (int i = 0; i < RW_MB; ++i) {
      poff[i] = -1;
      if (pgo[i] < 0) continue;
      if constexpr ((RW_ABL & 1) != 0) {  // lab: keep the MFMAs live, skip the stores
        if (acc[i][0][0] == 12345.f && acc[i][1][1] == 54321.f) a.dx[pgo[i]] = 1;
        continue;
      }
      // this lane's 8 consecutive channels nh*32 + kq*8 + (0..7): block j holds 4j..4j+3
      float v[8];
      const uint32_t bits = mw[i] >> (kq * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = ((bits >> e) & 1u) ? acc[i][e >> 2][e & 3] : 0.f;
      const uint32_t d4[4] = {dr[i].x, dr[i].y, dr[i].z, dr[i].w};
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += zk::bf16_to_f32((uint16_t)(d4[e >> 1] >> (16 * (e & 1))));
      pend[i] = make_uint4(zk::pack_bf16x2(v[0], v[1]), zk::pack_bf16x2(v[2], v[3]),
                           zk::pack_bf16x2(v[4], v[5]), zk::pack_bf16x2(v[6], v[7]));
      if (bnsum) {
        // sums of the values as stored (bf16), as the separate reduce would see them
        const uint32_t pw4[4] = {pend[i].x, pend[i].y, pend[i].z, pend[i].w};
        const uint32_t y4[4] = {yp[i].x, yp[i].y, yp[i].z, yp[i].w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float gv = zk::bf16_to_f32((uint16_t)(pw4[e >> 1] >> (16 * (e & 1))));
          const uint16_t yb = (uint16_t)(y4[e >> 1] >> (16 * (e & 1)));
          const float yv = a.ypred_bf16 ? zk::bf16_to_f32(yb) : (float)(int16_t)yb;
          s1[e] += gv;
          s2[e] += gv * (yv - mu[e]) * rs[e];
        }
      }
      poff[i] = pgo[i] * 64 + nh * 32 + kq * 8;
    }
  }
#pragma unroll
  for (int i = 0; i < RW_MB; ++i)
    if (poff[i] >= 0) *reinterpret_cast<uint4*>(a.dx + poff[i]) = pend[i];
  if (bnsum) {
    // the 16 lanes of a kq group hold the same 8 channels (other pixels)
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) {
        s1[e] += __shfl_xor(s1[e], off, 64);
        s2[e] += __shfl_xor(s2[e], off, 64);
      }
    if (a.stripes >= (int)gridDim.x) {
      // one copy per block (plain stores; zk_bn_bwd_coef sums the copies in
      // a fixed order): the 4 waves sharing a channel half combine through
      // LDS in wave order -- run-to-run bit-reproducible
      __syncthreads();  // every wave is past its last ring / weight read
      float* red = reinterpret_cast<float*>(smem);  // [wave][2][32]
      if (r16 == 0) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          red[(wave * 2 + 0) * 32 + kq * 8 + e] = s1[e];
          red[(wave * 2 + 1) * 32 + kq * 8 + e] = s2[e];
        }
      }
      __syncthreads();
      if (wave == 0) {  // channel-major copies [2][64][stripes] (zk_bn_bwd_coef)
#pragma unroll
        for (int v = lane; v < 128; v += 64) {
          const int which = v >> 6, c = v & 63, half = c >> 5, cc = c & 31;
          float t = 0.f;
#pragma unroll
          for (int m = 0; m < RW_NW / 2; ++m) t += red[((2 * m + half) * 2 + which) * 32 + cc];
          a.psums[(long long)(which * 64 + c) * a.stripes + blockIdx.x] = t;
        }
      }
    } else if (r16 == 0) {
      const long long copy = blockIdx.x % a.stripes;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = nh * 32 + kq * 8 + e;
        atomicAdd(a.psums + (long long)c * a.stripes + copy, s1[e]);
        atomicAdd(a.psums + (long long)(64 + c) * a.stripes + copy, s2[e]);
      }
    }
  }
  rw_drain();  // no DMA outstanding at exit
}

int g_num_cus = 0;
int g_lds_attr = 0;

}  // namespace

// Entry used by igemm.hip's dgrad dispatch (variant 50).  Stride-1 'same'
// 3x3, Cin = Cout = 64, 1 <= W <= 64; psums (optional): the predecessor's
// fused BN-backward sums (per-lane registers over the whole persistent range,
// one atomic per channel and lane group at the end).  dry: validate only.
int zk_conv3rw_dgrad_impl(const void* dy, const void* wt, const void* mask, const void* dres,
                          void* dx, int B, int H, int W, int Cin, int Cout, const void* ypred,
                          const void* pmean, const void* prstd, void* psums, int stripes,
                          int ypred_bf16, bool dry, hipStream_t st) {
  if (Cin != 64 || Cout != 64 || W < 1 || W > 64 || H < 1 || B < 1) return (int)hipErrorInvalidValue;
  if (psums && (!ypred || !pmean || !prstd)) return (int)hipErrorInvalidValue;
  if ((long long)B * H * W * 64 >= (1LL << 40)) return (int)hipErrorInvalidValue;
  const int slot = ((W + 7) / 8) * 1024;
  const int lds = RW_RING_OFF + RW_RING * slot;
  if (lds > 160 * 1024) return (int)hipErrorInvalidValue;
  if (dry) return 0;
  if (g_num_cus == 0) {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    g_num_cus = n > 0 ? n : 256;
  }
  if (lds > g_lds_attr) {
    // as much dynamic LDS as this geometry needs
    const hipError_t e = hipFuncSetAttribute((const void*)conv3rw_dgrad_kernel,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return (int)e;
    g_lds_attr = lds;
  }
  RWArgs a{(const uint16_t*)dy, (const uint16_t*)wt, (const uint32_t*)mask,
           (const uint16_t*)dres, (uint16_t*)dx, B, H, W, (H + RW_TR - 1) / RW_TR, 0, slot,
           (const int16_t*)ypred, (const float*)pmean, (const float*)prstd, (float*)psums,
           stripes < 1 ? 1 : stripes, ypred_bf16};
  const int nitems = B * a.ngroups;
  a.ipb = (nitems + g_num_cus - 1) / g_num_cus;
  const int grid = (nitems + a.ipb - 1) / a.ipb;
  (void)hipGetLastError();  // a stale error of an unrelated earlier call is not ours
  hipLaunchKernelGGL(conv3rw_dgrad_kernel, dim3(grid), dim3(RW_NW * 64), lds, st, a);
  return (int)hipGetLastError();
}
