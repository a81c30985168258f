// Recompute-fused ImageNet stem (7x7/2 conv, Cin <= 4 -> 64, BN, ReLU,
// 3x3/2 max pool) for gfx950.  stem.hip materialises the 112x112x64 conv
// output y1 (822 MB at batch 512) and a dense dy1 of the same size: written
// once, read three times.  Here neither tensor exists; the conv is cheap
// (K = 7 rows x 32) and is recomputed from the 4-channel padded image xp in
// each of the two passes that need it:
//
//   F   zk_stem_fwd_fused   conv -> BN-1 partial sums AND the 3x3/2 max pool
//                           of y1 * sign(gamma1): argmax tap, y1 there (ya)
//   P   zk_stem_pool_relu   p = relu(a1 ya + s1), BN-2 partial sums
//   B0  zk_stem_bn2_bwd_sums       BN-2 backward dx (dp) + the BN-1 backward
//                                  sums from (dp, ya), one pass
//   B2  zk_stem_bwd_fused   conv -> dy1 = k1 relu'(u) route(dp) + k0 - k3 y1
//                           -> weight gradient (MFMA), per-block slabs
//
// F and B2 are two-role software pipelines, one 512-thread block per CU:
// four "matrix" waves run the MFMA work (conv, weight gradient) of one tile
// while four VALU waves run the element work (pool / dy1 routing) of the
// previous tile and issue the LDS-DMA rings, one barrier per tile.  Waves w
// and w + 4 share a SIMD, so every SIMD pairs an MFMA stream with a VALU
// stream; rounds 1-5 alternated the phases inside every wave (B2 1.93 ms, F1 +
// F2 1.80 ms per E18 step at batch 1536).  A tile's input is a LINE BUFFER of
// xp rows (the (pixel, kh) K-rows of all its pixels overlap: 8 x 16 outputs
// read 21 x 38 input pixels = 8 KB instead of the 56 KB im2col image).  The
// conv is D[co][px] = W[co][k] X[px][k] on v_mfma_f32_32x32x16_bf16 with each
// matrix wave's 32 x 224 weights in VGPRs (lane = pixel, 4 consecutive
// channels per register group).  Line-buffer rows are padded so that the
// 16-B K-chunk of pixel m sits at 16 m + const (mod 256): the B-operand reads
// of consecutive pixels are bank-conflict free, and so are the transposed
// reads of the weight gradient.
//
// Numerics: y1 is rounded to bf16 before every use (the MFMA chain per output
// is identical in F and B2, so both see the same y1); the pool keeps the
// first maximum of y1 * sign(gamma1), which is the first maximum of
// relu(a1 y1 + s1) up to ties at relu's 0 (which route no gradient); the
// BN-1 statistics are of the fp32 accumulators.
#include <utility>

#include "mfma_common.h"

namespace {

constexpr int SC = 64;                    // stem output channels
constexpr int SKH = 7;                    // kernel rows (7x7 stems)

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

// counted wait on this wave's own vector-memory operations (n <= 15, wave-uniform)
__device__ __forceinline__ void wait_vmcnt_dyn(int n) {
  switch (n) {
#define ZK_VMC(k) \
  case k:         \
    asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); \
    break;
    ZK_VMC(0) ZK_VMC(1) ZK_VMC(2) ZK_VMC(3) ZK_VMC(4) ZK_VMC(5) ZK_VMC(6) ZK_VMC(7)
    ZK_VMC(8) ZK_VMC(9) ZK_VMC(10) ZK_VMC(11) ZK_VMC(12) ZK_VMC(13) ZK_VMC(14)
#undef ZK_VMC
    default: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
  }
}

// LDS-DMA of the line buffer of the tile whose first conv output is (b, r0,
// c0); rows / pixels outside xp and the row padding read the zero page.  The
// window row and pixel column of each of a thread's 16-B chunks do not depend
// on the tile: the plan decodes them once, and a tile's issue costs a few
// adds, a bounds test and a 32-bit pixel index per chunk (decoding them per
// tile cost ~2,500 shader cycles per tile in B2's route waves:
// tools/stem_stamps.cpp).
template <class L, int NT>
struct LinePlan {
  static constexpr int NJ = (L::CHUNKS + NT - 1) / NT;
  int rc[NJ];  // (window row << 16) | pixel column; -1: row padding (zero page)
  int n;       // DMA instructions this wave issues
  __device__ explicit LinePlan(int tid) {
    const int wave = (tid >> 6) % (NT / 64), lane = tid & 63;
    n = 0;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int q0 = j * NT + wave * 64;
      const int off = (q0 + lane) * 16;
      const int row = off / L::RB, cb = off - row * L::RB;
      rc[j] = cb < L::BASE ? (row << 16) | (cb >> 3) : -1;
      n += q0 < L::CHUNKS;
    }
  }
  __device__ __forceinline__ void issue(unsigned char* lb, const unsigned char* xp, const FGeom& g,
                                        int b, int r0, int c0) const {
    const unsigned char* zp = reinterpret_cast<const unsigned char*>(g_zero_page);
    const int wave = (threadIdx.x >> 6) % (NT / 64);
    const int bh = b * g.Hp, yr0 = 2 * r0, xc0 = 2 * c0;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int q0 = j * NT + wave * 64;  // wave-uniform
      if (q0 < L::CHUNKS) {
        const int yr = yr0 + (rc[j] >> 16), xc = xc0 + (rc[j] & 0xFFFF);
        const bool v = rc[j] >= 0 && (unsigned)yr < (unsigned)g.Hp && xc >= 0 && xc + 1 < g.Wp;
        const unsigned pix = (unsigned)((bh + yr) * g.Wp + xc);
        glds16(v ? xp + (unsigned long long)pix * 8 : zp, lb + q0 * 16);
      }
    }
  }
};

// acc[u] = sum over the 14 K-steps (kh, sub) of W[kh][sub] x B(pixel group
// u), B fragments read from a line buffer with row pitch RB at byte offsets
// seg0 / seg1.  The fragments stream PF K-steps ahead of their MFMAs: with one
// matrix wave per SIMD nothing else hides the LDS latency, and the compiler's
// own schedule kept only one step in flight (the kernels then ran at ~28 % of
// the MFMA rate).  The read / MFMA interleave is pinned with
// sched_group_barrier (masks: 0x100 DS read, 0x008 MFMA).
//   NV > 0: NV independent VALU instructions that follow the call in program
// order (the previous conv's statistics and keys) are pulled in beside each
// step's MFMA pair -- an MFMA hides ~5 single-issue VALU of its own wave
// (MI355X_MICROARCH.md, issue costs).
template <int RB, int PF, int NV = 0>
__device__ __forceinline__ void conv2_wreg(const uint4 (&w)[SKH][2], const unsigned char* lbc,
                                           int seg0, int seg1, f32x16 (&acc)[2]) {
  constexpr int NS = 2 * SKH;
  uint4 ring[PF][2];
#pragma unroll
  for (int p = 0; p < PF; ++p) {
    ring[p][0] = *reinterpret_cast<const uint4*>(lbc + seg0 + (p >> 1) * RB + 32 * (p & 1));
    ring[p][1] = *reinterpret_cast<const uint4*>(lbc + seg1 + (p >> 1) * RB + 32 * (p & 1));
  }
  __builtin_amdgcn_sched_group_barrier(0x100, 2 * PF, 0);
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const uint4 b0 = ring[s % PF][0], b1 = ring[s % PF][1];
    if (s + PF < NS) {
      const int t = s + PF;
      ring[s % PF][0] = *reinterpret_cast<const uint4*>(lbc + seg0 + (t >> 1) * RB + 32 * (t & 1));
      ring[s % PF][1] = *reinterpret_cast<const uint4*>(lbc + seg1 + (t >> 1) * RB + 32 * (t & 1));
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
    }
    acc[0] = mfma_bf16(w[s >> 1][s & 1], b0, s ? acc[0] : f32x16{});  // C = 0 first
    acc[1] = mfma_bf16(w[s >> 1][s & 1], b1, s ? acc[1] : f32x16{});
    if constexpr (NV > 0) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, NV / 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, NV - NV / 2, 0);
    } else {
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
    }
  }
}

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
// F: conv -> BN-1 statistics AND the 3x3/2 max pool, in one pass.
// The pool needs no BN-1 coefficients: relu(a y + s) is monotone in y in the
// direction of a = gamma1 * rstd, i.e. of gamma1, which is known before the
// batch statistics exist.  The first maximum of relu(a y + s) over a window
// is the first maximum of y * sign(gamma1) (ties at relu's 0 route no
// gradient), so this pass writes ya (y1 at that tap, bf16) and arg (the tap)
// while it accumulates the statistics; p = relu(a ya + s) and BN-2's partial
// sums follow in the elementwise zk_stem_pool_relu once BN-1 is finalised.
// (Rounds 1-5 ran the conv twice: statistics, then BN-1 + pool.)
//
// Tile = 8 x 7 pool outputs <- a 17 x 15 conv region (255 pixels + 1
// dummy = 8 groups of 32).  Pixels are numbered owned-first: m < 224 are the
// 16 x 14 outputs the tile owns for the statistics; 224..254 the halo row and
// column it shares with the next tile (group 7, counted only in the last tile
// of a row / column); 255 a dummy.  4 waves, 2 blocks per CU: wave w computes
// channel half a = w & 1 of pixel groups 4 (w >> 1) .. +3 with its 32 x 224
// weights in VGPRs (one B read per MFMA).  y1 goes to LDS as int16 order keys
// of y * sign(gamma1) (the two's complement of the bf16 sign-magnitude, so
// -0 == +0); the pool takes one 32-bit max per tap over (key << 16 | 15 - tap):
// keys are distinct, the max is the first maximum, and max is order-free.
// ===========================================================================
constexpr int F_PR = 8, F_PC = 7;                        // pool outputs per tile
constexpr int F_TR = 2 * F_PR + 1, F_TC = 2 * F_PC + 1;  // 17 x 15 conv region
constexpr int F_OR = 2 * F_PR, F_OC = 2 * F_PC;          // 16 x 14 owned outputs
constexpr int F_NOWN = F_OR * F_OC;                      // 224 = 7 pixel groups
static_assert(F_TR * F_TC < 256 && F_NOWN == 7 * 32, "F region");

struct FLB {  // line buffer of the 17 x 15 region
  static constexpr int ROWS = 2 * (F_TR - 1) + SKH;  // 39 xp rows
  static constexpr int BASE = (2 * F_TC + 6) * 8;     // 36 pixels of 8 B
  // 2 RB = 16 F_OC (mod 256): the K-chunk of owned pixel m sits at 16 m
  // (mod 256), so the B reads of 16 consecutive pixels are conflict free
  static constexpr int RB = BASE + ((((8 * F_OC) % 128 - BASE) % 128) + 128) % 128;
  static constexpr int CHUNKS = ROWS * RB / 16;
  static constexpr int BYTES = (CHUNKS + 63) / 64 * 64 * 16;
  static_assert(RB % 16 == 0 && (2 * RB) % 256 == (16 * F_OC) % 256, "F line buffer");
};
constexpr int F_YT = 256 * 128;  // y1 keys [pixel][64 channels]

// LDS row of pixel m: rows 2k / 2k+1 swap when bit 1 of m is set, so the pool
// reads of pixels m and m + 2 fall in opposite 128-B bank halves; 16-B slot
// s ^ f_swz(m), a bijection of m mod 8 whose bit 2 ignores bit 2 of m: the
// ds_write_b128 stores of 8 consecutive pixels and the pool reads of pixels
// m and m + 4 (opposite channel halves) are conflict free.
__device__ __forceinline__ int f_off(int m, int slot) {
  const int row = m ^ ((m >> 1) & 1);
  const int swz = ((m & 3) << 1) | ((m >> 2) & 1);
  return row * 128 + ((slot ^ swz) << 4);
}

// region coordinates of pixel m / pixel number of region (rr, cc)
__device__ __forceinline__ void f_pix(int m, int& rr, int& cc) {
  if (m < F_NOWN) {
    rr = m / F_OC;
    cc = m - rr * F_OC;
  } else if (m < F_NOWN + F_TC) {
    rr = F_OR;
    cc = m - F_NOWN;
  } else if (m < F_NOWN + F_TC + F_OR) {
    rr = m - (F_NOWN + F_TC);
    cc = F_OC;
  } else {
    rr = 0;  // dummy: reads pixel 0, never counted or pooled
    cc = 0;
  }
}
__device__ __forceinline__ int f_m(int rr, int cc) {
  return rr < F_OR ? (cc < F_OC ? rr * F_OC + cc : F_NOWN + F_TC + rr) : F_NOWN + cc;
}

// Diagnostic build only (-DZK_STEM_STAMPS, tools/stem_stamps.cpp): per wave,
// the shader cycles spent working and waiting at the interval barrier of the
// two-role pipelines (s_memtime), for the role balance.
#ifdef ZK_STEM_STAMPS
__device__ unsigned long long g_stem_stamps[2][1024 * 8][3];
#define ZK_STAMP_BEGIN unsigned long long zs_t = __builtin_readcyclecounter(), zs_work = 0, zs_wait = 0, zs_mem = 0;
#define ZK_STAMP_WORK                                 \
  {                                                   \
    const unsigned long long t_ = __builtin_readcyclecounter(); \
    zs_work += t_ - zs_t;                             \
    zs_t = t_;                                        \
  }
#define ZK_STAMP_WAIT                                 \
  {                                                   \
    const unsigned long long t_ = __builtin_readcyclecounter(); \
    zs_wait += t_ - zs_t;                             \
    zs_t = t_;                                        \
  }
#define ZK_STAMP_MEM                                  \
  {                                                   \
    const unsigned long long t_ = __builtin_readcyclecounter(); \
    zs_mem += t_ - zs_t;                              \
    zs_t = t_;                                        \
  }
#define ZK_STAMP_STORE(k)                                                  \
  if ((threadIdx.x & 63) == 0 && blockIdx.x < 1024) {                      \
    g_stem_stamps[k][blockIdx.x * 8 + (threadIdx.x >> 6)][0] = zs_work;    \
    g_stem_stamps[k][blockIdx.x * 8 + (threadIdx.x >> 6)][1] = zs_wait;    \
    g_stem_stamps[k][blockIdx.x * 8 + (threadIdx.x >> 6)][2] = zs_mem;     \
  }
#else
#define ZK_STAMP_BEGIN
#define ZK_STAMP_WORK
#define ZK_STAMP_WAIT
#define ZK_STAMP_MEM
#define ZK_STAMP_STORE(k)
#endif

typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
// bf16 pair -> int16 order keys: negative values get their magnitude bits
// flipped (an involution).  -0 sorts below +0; the conv never produces -0
// (its fp32 accumulators start at +0 and x + (-x) = +0).
__device__ __forceinline__ uint32_t key16x2(uint32_t d) {
  const s16x2 x = __builtin_bit_cast(s16x2, d);
  const s16x2 s = x >> (s16x2){15, 15};
  return d ^ (__builtin_bit_cast(uint32_t, s) & 0x7FFF7FFFu);
}

// Position (image b, tile row th, tile column tw) of a block's tiles
// T = T0, T0 + nblk, ...: the divisions happen once per stream, next() is a
// few scalar adds (three divisions per interval were most of the pipelines'
// scalar instructions).
struct TileWalk {
  int b, th, tw;
  int db, dh, dw, tiles_w, tiles_h;
  __device__ TileWalk(int T0, int nblk, int tiles_w_, int tiles_h_)
      : tiles_w(tiles_w_), tiles_h(tiles_h_) {
    const int img = tiles_w * tiles_h;
    b = T0 / img;
    const int rem = T0 - b * img;
    th = rem / tiles_w;
    tw = rem - th * tiles_w;
    db = nblk / img;
    const int r2 = nblk - db * img;
    dh = r2 / tiles_w;
    dw = r2 - dh * tiles_w;
  }
  __device__ __forceinline__ void next() {
    tw += dw;
    int c = tw >= tiles_w;
    tw -= c ? tiles_w : 0;
    th += dh + c;
    c = th >= tiles_h;
    th -= c ? tiles_h : 0;
    b += db + c;
  }
};

struct FTile {
  const unsigned char* lbc;  // this tile's line buffer
  unsigned char* yt;         // this tile's key image
  int hr0, wc0;              // conv coordinates of region (0, 0)
  bool last_r, last_c;       // last tile of its row / column of tiles
};

// BN-1 statistics of two 32-pixel groups (first group index G0) and their
// keys into yt.  FAST: every owned pixel in the image, no halo counted (the
// 7 owned groups, group 7 skipped); else the per-pixel test.
template <bool FAST, int G0>
__device__ __forceinline__ void f_post(const FTile& t, const FGeom& g, const f32x16 (&acc)[2],
                                       int a, int r32, int h, float (&cs)[16], float (&cq)[16]) {
  if constexpr (FAST) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (G0 + u >= 7) continue;  // the halo group (compile-time)
#pragma unroll
      for (int r = 0; r < 16; r += 2) {
        const f32x2 v = {acc[u][r], acc[u][r + 1]};
        f32x2 s2 = {cs[r], cs[r + 1]}, q2 = {cq[r], cq[r + 1]};
        s2 += v;
        q2 = __builtin_elementwise_fma(v, v, q2);
        cs[r] = s2.x;
        cs[r + 1] = s2.y;
        cq[r] = q2.x;
        cq[r + 1] = q2.y;
      }
    }
  } else {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int m = 32 * (G0 + u) + r32;
      int rr, cc;
      f_pix(m, rr, cc);
      const int hc = t.hr0 + rr, wc = t.wc0 + cc;
      const bool counted = m < 255 && hc >= 0 && hc < g.Ho && wc >= 0 && wc < g.Wo &&
                           (rr < F_OR || t.last_r) && (cc < F_OC || t.last_c);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float v = counted ? acc[u][r] : 0.f;
        cs[r] += v;
        cq[r] = fmaf(v, v, cq[r]);
      }
    }
  }
  // y1 * sign(gamma1) -> LDS keys: per register pair (q, q+1) one permlane32
  // swap per dword gives each lane a whole 16-B slot (cdna_hip_programming.md T21)
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int m = 32 * (G0 + u) + r32;
#pragma unroll
    for (int pq = 0; pq < 2; ++pq) {
      uint32_t d[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r = 4 * (2 * pq + (e >> 1)) + 2 * (e & 1);
        d[e] = key16x2(zk::pack_bf16x2(acc[u][r], acc[u][r + 1]));
      }
      const auto s0 = __builtin_amdgcn_permlane32_swap(d[0], d[2], false, false);
      const auto s1 = __builtin_amdgcn_permlane32_swap(d[1], d[3], false, false);
      *reinterpret_cast<uint4*>(t.yt + f_off(m, 4 * a + 2 * pq + h)) =
          make_uint4(s0[0], s1[0], s0[1], s1[1]);
    }
  }
}

// One tile of a matrix wave: conv of its 4 pixel groups (channel half a),
// then the statistics and keys.  HALO: this wave's groups are 4..7.
template <bool FAST, bool HALO>
__device__ __forceinline__ void f_matrix_tile(const FTile& t, const FGeom& g,
                                              const uint4 (&w)[SKH][2], const int (&segb)[4],
                                              int a, int r32, int h, float (&cs)[16],
                                              float (&cq)[16]) {
  constexpr int G0 = HALO ? 4 : 0;
  f32x16 acc0[2], acc1[2];
  conv2_wreg<FLB::RB, 3>(w, t.lbc, segb[0], segb[1], acc0);
  conv2_wreg<FLB::RB, 3, 8>(w, t.lbc, segb[2], segb[3], acc1);
  f_post<FAST, G0>(t, g, acc0, a, r32, h, cs, cq);
  f_post<FAST, G0 + 2>(t, g, acc1, a, r32, h, cs, cq);
}

__device__ __attribute__((aligned(16))) uint4 g_pool_sink[2];

// F runs as a two-role software pipeline, one 512-thread block per CU:
// waves 4-7 ("matrix" waves) compute the conv, the statistics and the y1 keys
// of tile i while waves 0-3 ("pool" waves) pool tile i - 1, store its ya / arg
// and issue the line-buffer DMA two tiles ahead.  Wave w and wave w + 4 share
// a SIMD: the MFMA stream of one overlaps the VALU stream of the other.
constexpr int F_NLB = 3, F_NYT = 2;
constexpr int F_LDS = F_NLB * FLB::BYTES + F_NYT * F_YT;
static_assert(F_LDS <= 160 * 1024, "F pipeline LDS");

__global__ __launch_bounds__(512, 2) void stem_fwd_fused_kernel(
    const unsigned char* __restrict__ xp, const unsigned char* __restrict__ ws,
    const float* __restrict__ gamma1, uint16_t* __restrict__ ya, uint8_t* __restrict__ arg,
    float* __restrict__ part, FGeom g, int tiles_w, int tiles_h, int ntiles) {
  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
  unsigned char* lbr = smem;                          // [3][FLB::BYTES]
  unsigned char* ytr = smem + F_NLB * FLB::BYTES;     // [2][F_YT]
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r32 = lane & 31, h = lane >> 5;
  const int blk = xcd_linear(blockIdx.x, gridDim.x), nblk = gridDim.x;
  const int n = blk < ntiles ? (ntiles - 1 - blk) / nblk + 1 : 0;  // this block's tiles
  const bool pooler = wave < 4;
  const int mw = wave & 3, a = mw & 1, g0 = 4 * (mw >> 1);  // matrix waves: channel half, first group

  auto issue_lb = [&](const LinePlan<FLB, 256>& pl, const TileWalk& t, int j) {
    pl.issue(lbr + (j % F_NLB) * FLB::BYTES, xp, g, t.b, 2 * F_PR * t.th - g.pt2,
             2 * F_PC * t.tw - g.pl2);
  };

  float cs[16], cq[16];  // matrix waves: BN-1 sums / squares of this lane's 16 channels
  if (pooler) {
    // pool items it = tid + 256 k (k = 0, 1; k = 1 only in waves 0-2): pool
    // output po = it >> 3 of the tile, channels 8 cg .. 8 cg + 7
    const int cg = tid & 7;
    uint32_t pflip[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const int c = 8 * cg + 2 * d;
      pflip[d] = gamma1 ? ((gamma1[c] < 0.f ? 0x8000u : 0u) | (gamma1[c + 1] < 0.f ? 0x80000000u : 0u))
                        : 0u;
    }
    uint32_t toff[2][5];  // the 9 tap offsets of each item, two 16-bit halves per register
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int po = (tid >> 3) + 32 * k;
      const int i = po / F_PC, j = po - (po / F_PC) * F_PC;
#pragma unroll
      for (int t = 0; t < 10; t += 2) {
        uint32_t v = 0;
#pragma unroll
        for (int e = 0; e < 2; ++e)
          if (t + e < 9 && po < F_PR * F_PC)
            v |= (uint32_t)f_off(f_m(2 * i + (t + e) / 3, 2 * j + (t + e) % 3), cg) << (16 * e);
        toff[k][t / 2] = v;
      }
    }
    const LinePlan<FLB, 256> lplan(tid);
    TileWalk wdma(blk, nblk, tiles_w, tiles_h), wpool(blk, nblk, tiles_w, tiles_h);
    if (n > 0) issue_lb(lplan, wdma, 0);
    wdma.next();
    if (n > 1) issue_lb(lplan, wdma, 1);
    wdma.next();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int n_lb = lplan.n;
    const int nst = wave < 3 ? 4 : 2;  // ya / arg stores per tile
    ZK_STAMP_BEGIN
    for (int ii = 0; ii <= n; ++ii) {
      int issued = 0;
      if (ii + 2 < n) {
        issue_lb(lplan, wdma, ii + 2);
        wdma.next();
        issued = n_lb;
      }
      if (ii >= 1) {
        const unsigned char* yt = ytr + ((ii - 1) % F_NYT) * F_YT;
        const int b = wpool.b, th = wpool.th, tw = wpool.tw;
        wpool.next();
        const int hr0 = 2 * F_PR * th - g.pt2, wc0 = 2 * F_PC * tw - g.pl2;
        // tile inside the image: every tap in the image, every pool output live
        const bool tile_in = hr0 >= 0 && hr0 + F_TR <= g.Ho && wc0 >= 0 && wc0 + F_TC <= g.Wo &&
                             F_PR * th + F_PR <= g.H2 && F_PC * tw + F_PC <= g.W2;
        // ---- pool: one (pool output, 8 channels) item per thread and k
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          if (k == 1 && wave == 3) continue;  // 56 outputs x 8 = 448 items (uniform)
          const int po = (tid >> 3) + 32 * k;
          const int i = po / F_PC, j = po - (po / F_PC) * F_PC;
          const int oh = F_PR * th + i, ow = F_PC * tw + j;
          uint4 tv[9];
#pragma unroll
          for (int t = 0; t < 9; ++t)
            tv[t] = *reinterpret_cast<const uint4*>(yt + ((toff[k][t >> 1] >> (16 * (t & 1))) & 0xFFFFu));
          if (!tile_in) {  // a tile at the image border (uniform); then per item
            const bool interior = hr0 + 2 * i >= 0 && hr0 + 2 * i + 2 < g.Ho && wc0 + 2 * j >= 0 &&
                                  wc0 + 2 * j + 2 < g.Wo;
            if (!interior) {
#pragma unroll
            for (int t = 0; t < 9; ++t) {
              const int hc = hr0 + 2 * i + t / 3, wc = wc0 + 2 * j + t % 3;
              if (!(hc >= 0 && hc < g.Ho && wc >= 0 && wc < g.Wo))
                tv[t] = make_uint4(0x80008000u, 0x80008000u, 0x80008000u, 0x80008000u);  // -inf
            }
            }
          }
          int best[8];
#pragma unroll
          for (int t = 0; t < 9; ++t) {
            const uint32_t u[4] = {tv[t].x, tv[t].y, tv[t].z, tv[t].w};
#pragma unroll
            for (int d = 0; d < 4; ++d) {
              const int lo = (int)((u[d] << 16) | (uint32_t)(15 - t));
              const int hi = (int)((u[d] & 0xFFFF0000u) | (uint32_t)(15 - t));
              best[2 * d] = t == 0 ? lo : max(best[2 * d], lo);
              best[2 * d + 1] = t == 0 ? hi : max(best[2 * d + 1], hi);
            }
          }
          // arg: 15 - (low byte); ya: the key halves, un-keyed and un-flipped
          const uint32_t t01 = __builtin_amdgcn_perm((uint32_t)best[1], (uint32_t)best[0], 0x0c0c0400u);
          const uint32_t t23 = __builtin_amdgcn_perm((uint32_t)best[3], (uint32_t)best[2], 0x0c0c0400u);
          const uint32_t t45 = __builtin_amdgcn_perm((uint32_t)best[5], (uint32_t)best[4], 0x0c0c0400u);
          const uint32_t t67 = __builtin_amdgcn_perm((uint32_t)best[7], (uint32_t)best[6], 0x0c0c0400u);
          const uint2 av = make_uint2(__builtin_amdgcn_perm(t23, t01, 0x05040100u) ^ 0x0F0F0F0Fu,
                                      __builtin_amdgcn_perm(t67, t45, 0x05040100u) ^ 0x0F0F0F0Fu);
          uint32_t yv[4];
#pragma unroll
          for (int d = 0; d < 4; ++d)
            yv[d] = key16x2(__builtin_amdgcn_perm((uint32_t)best[2 * d + 1], (uint32_t)best[2 * d],
                                                  0x07060302u)) ^ pflip[d];
          const bool live = tile_in || (oh < g.H2 && ow < g.W2);  // po < 56 always here
          const long long off = (((long long)b * g.H2 + oh) * g.W2 + ow) * SC + cg * 8;
          uint4* dy_ = live ? reinterpret_cast<uint4*>(ya + off) : &g_pool_sink[0];
          uint2* da_ = live ? reinterpret_cast<uint2*>(arg + off) : reinterpret_cast<uint2*>(&g_pool_sink[1]);
          *dy_ = make_uint4(yv[0], yv[1], yv[2], yv[3]);
          *da_ = av;
        }
        issued += nst;
      }
      // everything issued before this interval (line buffer ii + 1, the
      // previous tile's stores) landed
      ZK_STAMP_WORK
      wait_vmcnt_dyn(issued);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      ZK_STAMP_MEM
      __builtin_amdgcn_s_barrier();
      ZK_STAMP_WAIT
    }
    ZK_STAMP_STORE(0)
  } else {
    // weights of channel half a, w[kh][sub] = K-chunk 2 sub + h of row
    // co = 32 a + r32, negated where gamma1[co] < 0 (exact in bf16): the MFMA
    // then yields y1 * sign(gamma1) itself, and so do its statistics (the sums
    // get the sign back at the end, the squares need none)
    const uint32_t wneg = gamma1 && gamma1[32 * a + r32] < 0.f ? 0x80008000u : 0u;
    uint4 w[SKH][2];
#pragma unroll
    for (int kh = 0; kh < SKH; ++kh)
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        const uint4 v = *reinterpret_cast<const uint4*>(ws + (kh * SC + 32 * a + r32) * 64 +
                                                        (2 * sub + h) * 16);
        w[kh][sub] = make_uint4(v.x ^ wneg, v.y ^ wneg, v.z ^ wneg, v.w ^ wneg);
      }
    int segb[4];  // B-operand byte offsets of this lane's pixel in the 4 groups
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      int rr, cc;
      f_pix(32 * (g0 + t) + r32, rr, cc);
      segb[t] = 2 * rr * FLB::RB + 16 * cc + 16 * h;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) cs[r] = cq[r] = 0.f;
    TileWalk wmat(blk, nblk, tiles_w, tiles_h);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    ZK_STAMP_BEGIN
    for (int ii = 0; ii <= n; ++ii) {
      if (ii < n) {
        const int th = wmat.th, tw = wmat.tw;
        wmat.next();
        const int hr0 = 2 * F_PR * th - g.pt2, wc0 = 2 * F_PC * tw - g.pl2;
        const unsigned char* lbc = lbr + (ii % F_NLB) * FLB::BYTES;
        unsigned char* yt = ytr + (ii % F_NYT) * F_YT;
        const bool last_r = th == tiles_h - 1, last_c = tw == tiles_w - 1;
        const bool fast = hr0 >= 0 && hr0 + F_OR <= g.Ho && wc0 >= 0 && wc0 + F_OC <= g.Wo &&
                          !(last_r && hr0 + F_OR < g.Ho) && !(last_c && wc0 + F_OC < g.Wo);
        // one straight-line body per (statistics path, halo wave): the second
        // conv's MFMAs and the first pair's statistics / keys share a basic
        // block, so the scheduler can interleave them
        const FTile ft{lbc, yt, hr0, wc0, last_r, last_c};
        if (fast) {
          if (g0) f_matrix_tile<true, true>(ft, g, w, segb, a, r32, h, cs, cq);
          else f_matrix_tile<true, false>(ft, g, w, segb, a, r32, h, cs, cq);
        } else {
          if (g0) f_matrix_tile<false, true>(ft, g, w, segb, a, r32, h, cs, cq);
          else f_matrix_tile<false, false>(ft, g, w, segb, a, r32, h, cs, cq);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // y1 keys stored
      ZK_STAMP_WORK
      __builtin_amdgcn_s_barrier();
      ZK_STAMP_WAIT
    }
    ZK_STAMP_STORE(0)
  }

  // statistics: lane r32 of each half ends with the half's total of value r32
  // (r32 < 16: sum of channel(r32), else sum of squares of channel(r32 - 16))
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);  // [pixel half of the matrix waves][2][64]
  if (!pooler) {
    float v[32];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      v[r] = cs[r];
      v[16 + r] = cq[r];
    }
    const float tot = rs32(v, r32);
    const int which = r32 >> 4, r = r32 & 15;
    const int co = 32 * a + 8 * (r >> 2) + 4 * h + (r & 3);
    const bool neg = which == 0 && gamma1 && gamma1[co] < 0.f;  // sums of y1 * sign(gamma1)
    red[((mw >> 1) * 2 + which) * SC + co] = neg ? -tot : tot;
  }
  __syncthreads();
  if (part && tid < 2 * SC) part[(long long)blockIdx.x * 2 * SC + tid] = red[tid] + red[2 * SC + tid];
}

// p = relu(a1 ya + s1) (bf16, as the pool's output) and BN-2 partial sums of
// the rounded p: part[block][2][64].
__global__ __launch_bounds__(256) void stem_pool_relu_kernel(const uint16_t* __restrict__ ya,
                                                             const float* __restrict__ coef,
                                                             uint16_t* __restrict__ p,
                                                             float* __restrict__ part,
                                                             long long P2) {
  const int cg = threadIdx.x & 7;
  float a[8], sh[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    a[k] = coef[cg * 8 + k];
    sh[k] = coef[SC + cg * 8 + k];
  }
  float s1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (long long o = blockIdx.x * 32LL + (threadIdx.x >> 3); o < P2; o += gridDim.x * 32LL) {
    const long long off = o * SC + cg * 8;
    float yv[8], pv[8];
    unpack8(*reinterpret_cast<const uint4*>(ya + off), yv);
#pragma unroll
    for (int k = 0; k < 8; ++k) pv[k] = fmaxf(fmaf(a[k], yv[k], sh[k]), 0.f);
    const uint4 pk = pack8f(pv);
    *reinterpret_cast<uint4*>(p + off) = pk;
    float st[8];
    unpack8(pk, st);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      s1[k] += st[k];
      s2[k] = fmaf(st[k], st[k], s2[k]);
    }
  }
  if (!part) return;
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
constexpr int B2_NSLAB = SC * SKH * 32;  // dW partial per block [co][kh*32 + j]

// B2's y1 / dy1 image yt [128 pixels][64 channels]: 16-B slot s of row r at
// s ^ b2_swz(r).  b2_swz is a bijection of r mod 8 (the ds_write_b128 stores
// of 8 consecutive pixels are conflict free) whose bit 2 differs between rows
// r and r + 2 for r = 0, 1 (mod 4) (the transposed reads of rows r .. r + 3
// fall in disjoint slot blocks per 128-B bank half).
__device__ __forceinline__ int b2_swz(int r) { return ((((r >> 1) ^ (r >> 2)) & 1) << 2) | (r & 3); }
__device__ __forceinline__ int b2_off(int r, int slot) { return r * 128 + ((slot ^ b2_swz(r)) << 4); }

// 32x32x16 operand (8 consecutive pixels k of channel column c0 + ..) from yt
// (as tr_frag_swz, with b2_swz)
__device__ __forceinline__ uint4 tr_frag_b2(const unsigned char* yt, int k0, int c0, int lane) {
  const int gq = lane >> 4, i = lane & 15;
  const int q = i >> 2, p = i & 3;
  const int row = k0 + 8 * (gq >> 1) + q;
  const int colb = (c0 + 16 * (gq & 1) + 4 * p) * 2;
  const int slot = colb >> 4, inner = colb & 15;
  const int o0 = b2_off(row, slot) + inner, o1 = b2_off(row + 4, slot) + inner;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(uintptr_t)(const __attribute__((
          address_space(3))) void*)(yt + o0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(uintptr_t)(const __attribute__((
          address_space(3))) void*)(yt + o1));
  const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(uint4, v);
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

// B2 runs as a two-role software pipeline, one 512-thread block per CU:
// waves 0-3 ("route" waves, VALU) compute dy1 of tile j (phase b) and issue
// every LDS-DMA, while waves 4-7 ("matrix" waves, MFMA) run the conv of tile
// j + 1 (phase a) and the weight gradient of tile j - 1 (phase c) in the same
// barrier interval.  The CU issues wave w and wave w + 4 on one SIMD, so each
// SIMD pairs a VALU stream with an MFMA stream (MI355X_MICROARCH.md: the two
// pipes run concurrently) instead of alternating the phases in every wave.
// Rings: line buffers 5 (issued two intervals ahead, read by phases a and c),
// routing stages 3, y1 / dy1 images 3.  One barrier per interval.
constexpr int B3_NLB = 5, B3_NRT = 3, B3_NYT = 3;
constexpr int B3_LDS = B3_NLB * B2_LB + B3_NRT * B2_RT + B3_NYT * B2_YT + 2 * SC * 4;
static_assert(B3_LDS <= 160 * 1024, "B2 pipeline LDS");

template <int KB, int S>
__device__ __forceinline__ void b2_wg_load(const unsigned char* yt, const unsigned char* lbc,
                                           int wa, int lane, uint4& fa, uint4 (&fb)[4]) {
  fa = tr_frag_b2(yt, 16 * S, 32 * wa, lane);
#pragma unroll
  for (int e = 0; e < 3; ++e) fb[e] = tr_frag_lb(lbc, 16 * S, KB + e, lane);
  if constexpr ((S >> 2) == (KB >> 2)) fb[3] = tr_frag_lb(lbc, 16 * S, 3, lane);
}

template <int KB, int S>
__device__ __forceinline__ void b2_wg_step(const unsigned char* yt, const unsigned char* lbc,
                                           int wa, int lane, uint4 (&fa)[2], uint4 (&fb)[2][4],
                                           f32x16 (&accw)[4]) {
  constexpr int K = S & 1;
  constexpr bool R3 = (S >> 2) == (KB >> 2);
  if constexpr (S + 1 < 8) {
    b2_wg_load<KB, S + 1>(yt, lbc, wa, lane, fa[K ^ 1], fb[K ^ 1]);
  }
#pragma unroll
  for (int e = 0; e < 3; ++e) accw[e] = mfma_bf16(fa[K], fb[K][e], accw[e]);
  if constexpr (R3) accw[3] = mfma_bf16(fa[K], fb[K][3], accw[3]);
}

template <int KB, int... S>
__device__ __forceinline__ void b2_wg_steps(const unsigned char* yt, const unsigned char* lbc,
                                            int wa, int lane, uint4 (&fa)[2], uint4 (&fb)[2][4],
                                            f32x16 (&accw)[4], std::integer_sequence<int, S...>) {
  (b2_wg_step<KB, S>(yt, lbc, wa, lane, fa, fb, accw), ...);
}

// Phase c of one tile for a matrix wave with kernel rows KB .. KB + 2 (all 8
// pixel steps) and its half of kernel row 3 (steps KB .. KB + 3): the A
// (dy1^T) and B (X) fragments of step s + 1 are read while step s's MFMAs
// run (see conv2_wreg; left to the compiler's schedule here: pinning it
// with sched_group_barrier cost 14 VGPRs of spills).
template <int KB>
__device__ __forceinline__ void b2_wgrad_tile(const unsigned char* yt, const unsigned char* lbc,
                                              int wa, int lane, f32x16 (&accw)[4]) {
  uint4 fa[2], fb[2][4];
  b2_wg_load<KB, 0>(yt, lbc, wa, lane, fa[0], fb[0]);
  b2_wg_steps<KB>(yt, lbc, wa, lane, fa, fb, accw, std::make_integer_sequence<int, 8>{});
}

// LDS-DMA of the routing stage of the tile at (b, r0, c0): dp rows (128 B)
// and arg rows (64 B) of its 5 x 9 candidate pool outputs; outside the image
// the zero page.  Candidate offsets, chunk part and dp / arg kind are decoded
// once per thread.
template <int NT>
struct RoutePlan {
  static constexpr int NJ = (RT_CHUNKS + NT - 1) / NT;
  int code[NJ];  // (arg << 24) | (row << 16) | (col << 8) | part; -1: no chunk
  int n;
  __device__ explicit RoutePlan(int tid) {
    const int wave = (tid >> 6) % (NT / 64), lane = tid & 63;
    n = 0;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int q0 = j * NT + wave * 64, q = q0 + lane;
      n += q0 < RT_CHUNKS;
      if (q < RT_N * 8) {
        const int o = q >> 3;
        code[j] = ((o / RT_OW) << 16) | ((o % RT_OW) << 8) | (q & 7);
      } else if (q < RT_CHUNKS) {
        const int qa = q - RT_N * 8, o = qa >> 2;
        code[j] = (1 << 24) | ((o / RT_OW) << 16) | ((o % RT_OW) << 8) | (qa & 3);
      } else {
        code[j] = -1;
      }
    }
  }
  __device__ __forceinline__ void issue(unsigned char* rt, const uint16_t* dp, const uint8_t* arg,
                                        const FGeom& g, int b, int r0, int c0) const {
    const unsigned char* zp = reinterpret_cast<const unsigned char*>(g_zero_page);
    const int wave = (threadIdx.x >> 6) % (NT / 64);
    const int ohb = r0 / 2 - 1 + g.pt2, owb = c0 / 2 - 1 + g.pl2, bh = b * g.H2;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int q0 = j * NT + wave * 64;  // wave-uniform
      if (q0 < RT_CHUNKS) {
        const int c = code[j];
        const int oh = ohb + ((c >> 16) & 0xFF), ow = owb + ((c >> 8) & 0xFF);
        const bool v = c >= 0 && (unsigned)oh < (unsigned)g.H2 && (unsigned)ow < (unsigned)g.W2;
        const unsigned pix = (unsigned)((bh + oh) * g.W2 + ow);
        const unsigned char* src =
            (c >> 24) ? reinterpret_cast<const unsigned char*>(arg) + (unsigned long long)pix * 64
                      : reinterpret_cast<const unsigned char*>(dp) + (unsigned long long)pix * 128;
        glds16(v ? src + (c & 0xFF) * 16 : zp, rt + q0 * 16);
      }
    }
  }
};

template <int PT2, int PL2>
__global__ __launch_bounds__(512, 2) void stem_bwd_fused_kernel(
    const unsigned char* __restrict__ xp, const unsigned char* __restrict__ ws,
    const uint16_t* __restrict__ dp, const uint8_t* __restrict__ arg,
    const float* __restrict__ coef1, const float* __restrict__ bcoef1, float* __restrict__ slab,
    FGeom g, int tiles_w, int tiles_img, int ntiles) {
  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
  unsigned char* lbr = smem;                                   // [5][B2_LB]
  unsigned char* rtr = lbr + B3_NLB * B2_LB;                   // [3][B2_RT]
  unsigned char* ytr = rtr + B3_NRT * B2_RT;                   // [3][B2_YT]
  float* cf = reinterpret_cast<float*>(ytr + B3_NYT * B2_YT);  // BN-1 a1, s1
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r32 = lane & 31, h = lane >> 5;
  const int blk = xcd_linear(blockIdx.x, gridDim.x), nblk = gridDim.x;
  const int n = blk < ntiles ? (ntiles - 1 - blk) / nblk + 1 : 0;  // this block's tiles
  const bool route = wave < 4;

  const int tiles_h = tiles_img / tiles_w;
  auto issue_lb = [&](const LinePlan<LBuf<B2_TR, B2_TC>, 256>& pl, const TileWalk& t, int j) {
    pl.issue(lbr + (j % B3_NLB) * B2_LB, xp, g, t.b, t.th * B2_TR, t.tw * B2_TC);
  };
  auto issue_rt = [&](const RoutePlan<256>& pl, const TileWalk& t, int j) {
    pl.issue(rtr + (j % B3_NRT) * B2_RT, dp, arg, g, t.b, t.th * B2_TR, t.tw * B2_TC);
  };

  // matrix-wave indices (used after the loops too)
  const int mw = wave & 3, ma = mw & 1, mg0 = 2 * (mw >> 1);
  const int wa = mw >> 1, kb = 4 * (mw & 1);
  f32x16 accw[4];
  if (route) {
    // ---- route waves: stride cell (cr, cc), channels 8 cgp ..; BN-backward
    // coefficients in registers (k3 negated)
    const int cell = tid >> 3, cgp = tid & 7;
    const int cr = cell >> 3, cc = cell & 7;
    float k1[8], k0[8], k3[8];  // BN-1's a1, s1: in LDS (registers are the limit)
    for (int i = tid; i < 2 * SC; i += 256) cf[i] = coef1[i];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = cgp * 8 + k;
      k1[k] = bcoef1[c];
      k0[k] = bcoef1[SC + c];
      k3[k] = -bcoef1[2 * SC + c];
    }
    const LinePlan<LBuf<B2_TR, B2_TC>, 256> lplan(tid);
    const RoutePlan<256> rplan(tid);
    TileWalk wlb(blk, nblk, tiles_w, tiles_h), wrt(blk, nblk, tiles_w, tiles_h),
        wb(blk, nblk, tiles_w, tiles_h);
    if (n > 0) issue_lb(lplan, wlb, 0);
    wlb.next();
    if (n > 1) issue_lb(lplan, wlb, 1);
    wlb.next();
    if (n > 0) issue_rt(rplan, wrt, 0);
    wrt.next();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    ZK_STAMP_BEGIN
    for (int i = 0; i < n + 2; ++i) {
      // DMA two intervals ahead for the conv, one for the routing stage
      int issued = 0;
      if (i + 2 < n) {
        issue_lb(lplan, wlb, i + 2);
        wlb.next();
        issued += lplan.n;
      }
      if (i + 1 < n) {
        issue_rt(rplan, wrt, i + 1);
        wrt.next();
        issued += rplan.n;
      }
      // ---- b) dy1 of tile i - 1 in place: du = sum of dp over the candidate
      // pool outputs whose argmax tap is the pixel; with the pool padding
      // (PT2, PL2) static, the candidates of each of the cell's 4 pixels and
      // their taps are compile-time (9 tests per cell).  Candidates outside
      // the image read the zero page: dp 0 adds nothing whatever the tap.
      if (i >= 1 && i <= n) {
        const int j = i - 1;
        const int r0 = wb.th * B2_TR, c0 = wb.tw * B2_TC;
        wb.next();
        const unsigned char* rt = rtr + (j % B3_NRT) * B2_RT;
        unsigned char* yt = ytr + (j % B3_NYT) * B2_YT;
        uint32_t aw[2][2][2];
        uint4 gq[2][2];
#pragma unroll
        for (int ii = 0; ii < 2; ++ii)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) {
            const int o = (cr + ii) * RT_OW + cc + jj;
            const uint2 av = *reinterpret_cast<const uint2*>(rt + RT_DP + o * 64 + cgp * 8);
            aw[ii][jj][0] = av.x;
            aw[ii][jj][1] = av.y;
            gq[ii][jj] = *reinterpret_cast<const uint4*>(rt + o * 128 + cgp * 16);
          }
        uint4 yq[4];
#pragma unroll
        for (int pq = 0; pq < 4; ++pq) {
          const int m = (2 * cr + (pq >> 1)) * B2_TC + 2 * cc + (pq & 1);
          yq[pq] = *reinterpret_cast<const uint4*>(yt + b2_off(m, cgp));
        }
        float ca[8], cs[8];
        {
          const float4* c4 = reinterpret_cast<const float4*>(cf + cgp * 8);
          const float4 a0 = c4[0], a1 = c4[1], s0 = c4[SC / 4], s1 = c4[SC / 4 + 1];
          ca[0] = a0.x; ca[1] = a0.y; ca[2] = a0.z; ca[3] = a0.w;
          ca[4] = a1.x; ca[5] = a1.y; ca[6] = a1.z; ca[7] = a1.w;
          cs[0] = s0.x; cs[1] = s0.y; cs[2] = s0.z; cs[3] = s0.w;
          cs[4] = s1.x; cs[5] = s1.y; cs[6] = s1.z; cs[7] = s1.w;
        }
        const bool interior = r0 + B2_TR <= g.Ho && c0 + B2_TC <= g.Wo;  // uniform
#pragma unroll
        for (int pq = 0; pq < 4; ++pq) {
          const int dy = pq >> 1, dx = pq & 1;
          float du[8];
          bool any = false;
#pragma unroll
          for (int ii = 0; ii < 2; ++ii) {
            const int th = dy + 2 - PT2 - 2 * ii;
            if (th < 0 || th > 2) continue;  // compile-time
#pragma unroll
            for (int jj = 0; jj < 2; ++jj) {
              const int tw = dx + 2 - PL2 - 2 * jj;
              if (tw < 0 || tw > 2) continue;  // compile-time
              const uint32_t t = th * 3 + tw;
              const uint32_t gw[4] = {gq[ii][jj].x, gq[ii][jj].y, gq[ii][jj].z, gq[ii][jj].w};
#pragma unroll
              for (int k = 0; k < 8; ++k) {
                const bool hit = ((aw[ii][jj][k >> 2] >> (8 * (k & 3))) & 0xffu) == t;
                const uint32_t wv = gw[k >> 1];
                const float gv = __uint_as_float((k & 1) ? (wv & 0xFFFF0000u) : (wv << 16));
                const float add = hit ? gv : 0.f;
                du[k] = any ? du[k] + add : add;
              }
              any = true;
            }
          }
          float yv[8], o8[8];
          unpack8(yq[pq], yv);
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const float u = fmaf(ca[k], yv[k], cs[k]);
            o8[k] = fmaf(k1[k], u > 0.f ? du[k] : 0.f, fmaf(k3[k], yv[k], k0[k]));
          }
          if (!interior) {
            const bool live = r0 + 2 * cr + dy < g.Ho && c0 + 2 * cc + dx < g.Wo;
#pragma unroll
            for (int k = 0; k < 8; ++k) o8[k] = live ? o8[k] : 0.f;
          }
          const int m = (2 * cr + dy) * B2_TC + 2 * cc + dx;
          *reinterpret_cast<uint4*>(yt + b2_off(m, cgp)) = pack8f(o8);
        }
      }
      ZK_STAMP_WORK
      // the previous interval's DMAs (line buffer i + 1, routing stage i) landed
      wait_vmcnt_dyn(issued);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // dy1 stores done
      ZK_STAMP_MEM
      __builtin_amdgcn_s_barrier();
      ZK_STAMP_WAIT
    }
    ZK_STAMP_STORE(1)
  } else {
    // ---- matrix waves: mw computes the conv of channel half ma for pixel
    // groups mg0, mg0 + 1 with its 32 x 224 weights in VGPRs, and the phase-c
    // units (wa, rows kb .. kb + 2 all steps; row 3 on steps kb .. kb + 3)
    uint4 w[SKH][2];
#pragma unroll
    for (int kh = 0; kh < SKH; ++kh)
#pragma unroll
      for (int sub = 0; sub < 2; ++sub)
        w[kh][sub] = *reinterpret_cast<const uint4*>(ws + (kh * SC + 32 * ma + r32) * 64 +
                                                     (2 * sub + h) * 16);
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int r = 0; r < 16; ++r) accw[e][r] = 0.f;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    ZK_STAMP_BEGIN
    for (int i = 0; i < n + 2; ++i) {
      // ---- a) conv of tile i -> its y1 image
      if (i < n) {
        const unsigned char* lbc = lbr + (i % B3_NLB) * B2_LB;
        unsigned char* yt = ytr + (i % B3_NYT) * B2_YT;
        using L = LBuf<B2_TR, B2_TC>;
        int segb[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int px = 32 * (mg0 + u) + r32;  // tile pixel: row px / 16, column px % 16
          segb[u] = 2 * (px / B2_TC) * L::RB + 16 * (px % B2_TC) + 16 * h;
        }
        f32x16 acc[2];
        conv2_wreg<L::RB, 2>(w, lbc, segb[0], segb[1], acc);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int m = 32 * (mg0 + u) + r32;
#pragma unroll
          for (int pq = 0; pq < 2; ++pq) {
            uint32_t d[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int r = 4 * (2 * pq + (e >> 1)) + 2 * (e & 1);
              d[e] = zk::pack_bf16x2(acc[u][r], acc[u][r + 1]);
            }
            const auto s0 = __builtin_amdgcn_permlane32_swap(d[0], d[2], false, false);
            const auto s1 = __builtin_amdgcn_permlane32_swap(d[1], d[3], false, false);
            *reinterpret_cast<uint4*>(yt + b2_off(m, 4 * ma + 2 * pq + h)) =
                make_uint4(s0[0], s1[0], s0[1], s1[1]);
          }
        }
      }
      // ---- c) weight gradient of tile i - 2, 28 MFMAs per wave
      if (i >= 2) {
        const int j = i - 2;
        const unsigned char* lbc = lbr + (j % B3_NLB) * B2_LB;
        const unsigned char* yt = ytr + (j % B3_NYT) * B2_YT;
        if (kb)
          b2_wgrad_tile<4>(yt, lbc, wa, lane, accw);
        else
          b2_wgrad_tile<0>(yt, lbc, wa, lane, accw);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // y1 stores done
      ZK_STAMP_WORK
      __builtin_amdgcn_s_barrier();
      ZK_STAMP_WAIT
    }
    ZK_STAMP_STORE(1)
  }

  // one plain-stored dW partial per block: slab[block][co][kh*32 + j]; the
  // row-3 halves of waves (2wa, 2wa+1) meet in LDS first
  __syncthreads();
  float* cmb = reinterpret_cast<float*>(smem);  // [2 wa][16 r][64 lanes]
  if (!route && kb) {
#pragma unroll
    for (int r = 0; r < 16; ++r) cmb[(wa * 16 + r) * 64 + lane] = accw[3][r];
  }
  __syncthreads();
  if (!route && !kb) {
#pragma unroll
    for (int r = 0; r < 16; ++r) accw[3][r] += cmb[(wa * 16 + r) * 64 + lane];
  }
  if (!route) {
    float* sl = slab + (long long)blockIdx.x * B2_NSLAB;
    constexpr int NR = SKH * 32;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = 32 * wa + 8 * (r >> 2) + 4 * h + (r & 3);
#pragma unroll
      for (int e = 0; e < 3; ++e) sl[co * NR + (kb + e) * 32 + r32] = accw[e][r];
      if (!kb) sl[co * NR + 3 * 32 + r32] = accw[3][r];
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

// BN-2 backward dx and B1 in one pass: dp = bf16(k1 g + k0 - k3 p) (as
// norm_pool.hip's bn_bwd_dx_bf16), then du = dp [a1 ya + s1 > 0] and the
// BN-1 sums of du and du (ya - mean1) rstd1 of that rounded dp.  Saves B1's
// re-read of dp.  bcoef2 [3][64]; coef1 [4][64]; part[block][2][64].
__global__ __launch_bounds__(256) void stem_bn2_bwd_sums_kernel(
    const uint16_t* __restrict__ g, const uint16_t* __restrict__ p,
    const uint16_t* __restrict__ ya, const float* __restrict__ bcoef2,
    const float* __restrict__ coef, uint16_t* __restrict__ dp, float* __restrict__ part,
    long long P2) {
  const int cg = threadIdx.x & 7;
  float k1[8], k0[8], k3[8], a[8], sh[8], mean[8], rstd[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int c = cg * 8 + k;
    k1[k] = bcoef2[c];
    k0[k] = bcoef2[SC + c];
    k3[k] = bcoef2[2 * SC + c];
    a[k] = coef[c];
    sh[k] = coef[SC + c];
    mean[k] = coef[2 * SC + c];
    rstd[k] = coef[3 * SC + c];
  }
  float s1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (long long o = blockIdx.x * 32LL + (threadIdx.x >> 3); o < P2; o += gridDim.x * 32LL) {
    const long long off = o * SC + cg * 8;
    float gv[8], pv[8], yv[8], dv[8];
    unpack8(*reinterpret_cast<const uint4*>(g + off), gv);
    unpack8(*reinterpret_cast<const uint4*>(p + off), pv);
    unpack8(*reinterpret_cast<const uint4*>(ya + off), yv);
#pragma unroll
    for (int k = 0; k < 8; ++k) dv[k] = k1[k] * gv[k] + k0[k] - k3[k] * pv[k];
    const uint4 dq = pack8f(dv);
    *reinterpret_cast<uint4*>(dp + off) = dq;
    unpack8(dq, dv);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float du = fmaf(a[k], yv[k], sh[k]) > 0.f ? dv[k] : 0.f;
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
  if (which == 1) {  // F: pool tiles, one pipelined block per CU
    nt = (long long)B * ((H2 + F_PR - 1) / F_PR) * ((W2 + F_PC - 1) / F_PC);
    return grid_for(nt, 1);
  }
  nt = (long long)B * ((Ho + 7) / 8) * ((Wo + 15) / 16);  // B2: conv tiles, one block per CU
  return grid_for(nt, 1);
}

ZK_EXPORT int zk_stem_fused_slab_floats() { return B2_NSLAB; }
// extra slab rows zk_stem_bwd_fused needs beyond one per block (reduction groups)
ZK_EXPORT int zk_stem_fused_slab_extra() { return B2_GROUPS; }

// gamma1: BN-1 scale (nullptr: none, all directions +); part: [blocks][2][64]
// BN-1 partial sums or nullptr; ya (bf16) / arg (u8): [B][H2][W2][64].
ZK_EXPORT int zk_stem_fwd_fused(const void* xp, const void* ws, const void* gamma1, void* ya,
                                void* arg, void* part, int B, int Cin, int KW, int Ho, int Wo,
                                int Hp, int Wp, int H2, int W2, int pt2, int pl2, int* nparts,
                                hipStream_t st) {
  FGeom g{B, Cin, KW, Ho, Wo, Hp, Wp, H2, W2, pt2, pl2};
  if (!fgeom_ok(g)) return (int)hipErrorInvalidValue;
  const int tw = (W2 + F_PC - 1) / F_PC, th = (H2 + F_PR - 1) / F_PR;
  const long long nt = (long long)B * th * tw;
  if (nt >= (1LL << 31)) return (int)hipErrorInvalidValue;
  const int grid = grid_for(nt, 1);
  if (nparts) *nparts = grid;
  if (int e = set_lds_once(stem_fwd_fused_kernel, F_LDS)) return e;
  hipLaunchKernelGGL(stem_fwd_fused_kernel, dim3(grid), dim3(512), F_LDS, st,
                     (const unsigned char*)xp, (const unsigned char*)ws, (const float*)gamma1,
                     (uint16_t*)ya, (uint8_t*)arg, (float*)part, g, tw, th, (int)nt);
  ZK_CHECK_LAUNCH();
  return 0;
}

// p = relu(coef1[0] ya + coef1[1]) (bf16) over P2 x 64; part: [<= 4096][2][64]
// BN-2 partial sums of p or nullptr.
ZK_EXPORT int zk_stem_pool_relu(const void* ya, const void* coef1, void* p, void* part,
                                long long P2, int* nparts, hipStream_t st) {
  long long grid = (P2 + 31) / 32;
  if (grid > 4096) grid = 4096;
  if (grid < 1) grid = 1;
  if (nparts) *nparts = (int)grid;
  hipLaunchKernelGGL(stem_pool_relu_kernel, dim3((int)grid), dim3(256), 0, st,
                     (const uint16_t*)ya, (const float*)coef1, (uint16_t*)p, (float*)part, P2);
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

// dp = BN-2 backward of g (bcoef2 [3][64], p the BN-2 input) and the BN-1
// partial sums of B1 (coef1 [4][64], ya) in one pass; part: [<= 4096][2][64].
ZK_EXPORT int zk_stem_bn2_bwd_sums(const void* g, const void* p, const void* ya,
                                   const void* bcoef2, const void* coef1, void* dp, void* part,
                                   long long P2, int* nparts, hipStream_t st) {
  long long grid = (P2 + 31) / 32;
  if (grid > 4096) grid = 4096;
  if (grid < 1) grid = 1;
  if (nparts) *nparts = (int)grid;
  hipLaunchKernelGGL(stem_bn2_bwd_sums_kernel, dim3((int)grid), dim3(256), 0, st,
                     (const uint16_t*)g, (const uint16_t*)p, (const uint16_t*)ya,
                     (const float*)bcoef2, (const float*)coef1, (uint16_t*)dp, (float*)part, P2);
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
  const int grid = grid_for(nt, 1);  // one pipelined 512-thread block per CU
  static bool lds_set = false;
  if (!lds_set) {
    for (const void* k : {(const void*)stem_bwd_fused_kernel<0, 0>, (const void*)stem_bwd_fused_kernel<0, 1>,
                          (const void*)stem_bwd_fused_kernel<1, 0>, (const void*)stem_bwd_fused_kernel<1, 1>}) {
      hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, B3_LDS);
      if (e != hipSuccess) return (int)e;
    }
    lds_set = true;
  }
  auto kern = g.pt2 ? (g.pl2 ? stem_bwd_fused_kernel<1, 1> : stem_bwd_fused_kernel<1, 0>)
                    : (g.pl2 ? stem_bwd_fused_kernel<0, 1> : stem_bwd_fused_kernel<0, 0>);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(512), B3_LDS, st,
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
