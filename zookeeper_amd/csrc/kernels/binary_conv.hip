// Binary convolution on bit-packed operands for gfx950 (MI355X).
//
// Forward of a Larq-style QuantConv2D with ste_sign input and kernel
// quantizers, as an implicit GEMM
//      M = B*Ho*Wo output pixels,  N = Cout,  K = kh*kw*Cin  (bits)
// on packed words (bit i of word w = sign bit of channel 32w+i, 1 = +1):
//      y[m,n] = sum_valid_taps  sum_words (32 - 2*popc(a ^ b))
// i.e. the ±1 dot product computed with v_xor_b32 + v_bcnt_u32_b32 (popcount
// with accumulate) on LDS-staged bit tiles.  No ±1 tensor is ever
// materialised; operands are 16x (vs bf16) / 32x (vs fp32) smaller.
//
// Padding.  Larq's default pads the *quantized* input with 0 (not ±1).  The
// main loop stays branch-free: padded taps load a = 0, which adds popc(b) =
// P[n][t] to the xor-popcount sum; the epilogue removes it using the
// per-(channel, tap) popcounts P of the packed kernel and the per-pixel count
// of valid taps:
//      y = 32*CW*nvalid - 2*S + 2*sum_{t invalid} P[n][t].
// With pad_value = +1 (QuickNet) padded words are all-ones and every tap is
// valid: y = 32*CW*T - 2*S.
//
// Epilogue fusions: optional ReLU (QuickNet applies it before BN), exact
// int16 output (|y| <= 9*Cin fits), and the BatchNorm batch statistics
// sum(y) and sum(y^2) as exact int64 atomics (deterministic, no fp rounding).
//
// Tiling (v1): 256 threads = 4 waves, tile 128 pixels x 64 channels, each
// thread an 8x4 register micro-tile of int32 accumulators; one K-step = one
// kernel tap (all CW = Cin/32 words), A and B tap tiles staged through LDS
// ([word][pixel] / [word][channel] so a thread reads its 8 pixels and 4
// channels with 2 + 1 ds_read_b128), next tap prefetched into registers
// while the current one is consumed.
#include "../common.h"

namespace {

constexpr int BM = 128;
constexpr int BN = 64;
constexpr int NT = 256;

// --------------------------------------------------------------------------
// sign / STE-mask packing of activations: x bf16 [P][C] -> bits, mask [P][C/32]
// --------------------------------------------------------------------------
__global__ __launch_bounds__(256) void sign_pack_kernel(const uint16_t* __restrict__ x,
                                                        uint32_t* __restrict__ bits,
                                                        uint32_t* __restrict__ mask,
                                                        uint16_t* __restrict__ xs,
                                                        uint4* __restrict__ xs4,
                                                        long long nwords, float clip) {
  for (long long w = blockIdx.x * (long long)blockDim.x + threadIdx.x; w < nwords;
       w += (long long)gridDim.x * blockDim.x) {
    const uint4* src = reinterpret_cast<const uint4*>(x + 32 * w);
    uint32_t b = 0, mk = 0, n4[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint4 v = src[q];
      uint32_t u[4] = {v.x, v.y, v.z, v.w};
      uint32_t o[4];
      n4[q] = 0;
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        o[h] = 0;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const float f = zk::bf16_to_f32((uint16_t)(u[h] >> (16 * s)));
          const int i = q * 8 + h * 2 + s;
          b |= (uint32_t)(f >= 0.f) << i;
          mk |= (uint32_t)(fabsf(f) <= clip) << i;
          o[h] |= (f >= 0.f ? 0x3F80u : 0xBF80u) << (16 * s);
          n4[q] |= zk::fp4_sign(f) << (4 * (h * 2 + s));
        }
      }
      // sign(x) as bf16 +-1: the operand of the MFMA weight gradient
      if (xs) reinterpret_cast<uint4*>(xs + 32 * w)[q] = make_uint4(o[0], o[1], o[2], o[3]);
    }
    if (bits) bits[w] = b;
    if (mask) mask[w] = mk;
    // sign(x) as e2m1 nibbles: the operand of the MX-FP4 forward
    if (xs4) xs4[w] = make_uint4(n4[0], n4[1], n4[2], n4[3]);
  }
}

// --------------------------------------------------------------------------
// Kernel packing: w fp32 [Cout][T][Cin] (OHWI) -> wbits [Cout][T][CW],
// wpop [Cout][T] (popcount per tap; zeroed by the caller), and (optional)
// wt: the ±1 kernel as bf16, transposed to [T][Cin][Cout] for the dgrad
// GEMM (K = Cout contiguous).  One thread per packed word (8 float4 loads).
// --------------------------------------------------------------------------
__global__ __launch_bounds__(256) void weight_pack_kernel(const float* __restrict__ w,
                                                          uint32_t* __restrict__ wbits,
                                                          int* __restrict__ wpop,
                                                          uint16_t* __restrict__ wt,
                                                          uint16_t* __restrict__ wf,
                                                          long long nwords, int CW, int T,
                                                          int Cout) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= nwords) return;
  const float4* src = reinterpret_cast<const float4*>(w + 32 * i);
  uint32_t b = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const float4 v = src[q];
    b |= (uint32_t)(v.x >= 0.f) << (4 * q);
    b |= (uint32_t)(v.y >= 0.f) << (4 * q + 1);
    b |= (uint32_t)(v.z >= 0.f) << (4 * q + 2);
    b |= (uint32_t)(v.w >= 0.f) << (4 * q + 3);
  }
  if (wbits) {
    wbits[i] = b;
    atomicAdd(wpop + i / CW, __popc(b));
  }
  if (wf) {  // [T][Cout][Cin]: the forward GEMM's K-contiguous operand
    const int wd = (int)(i % CW);
    const long long ct = i / CW;
    const int t = (int)(ct % T), co = (int)(ct / T);
    uint4* dst = reinterpret_cast<uint4*>(wf + (((long long)t * Cout + co) * CW + wd) * 32);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint32_t o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = 8 * q + 2 * e;
        o[e] = (((b >> k) & 1) ? 0x3F80u : 0xBF80u) | ((((b >> (k + 1)) & 1) ? 0x3F80u : 0xBF80u) << 16);
      }
      dst[q] = make_uint4(o[0], o[1], o[2], o[3]);
    }
  }
  if (wt) {
    const int wd = (int)(i % CW);
    const long long ct = i / CW;
    const int t = (int)(ct % T), co = (int)(ct / T);
    const int Cin = CW * 32;
    uint16_t* dst = wt + ((long long)t * Cin + wd * 32) * Cout + co;
#pragma unroll 8
    for (int k = 0; k < 32; ++k) dst[(long long)k * Cout] = ((b >> k) & 1) ? 0x3F80 : 0xBF80;
  }
}

// Tiled variant for the MFMA path (no bits): one block per (tap, 64 ci, 64
// co) tile, staged through LDS so both the forward layout wf [T][Cout][Cin]
// and the transposed dgrad layout wt [T][Cin][Cout] are written with
// coalesced 16-B stores (the per-word kernel writes wt with 2-B scattered
// stores at stride Cout); wf4 is the forward layout as e2m1 nibbles
// [T][Cout][Cin/2] for the MX-FP4 forward.
__global__ __launch_bounds__(256) void weight_pack_tiled_kernel(const float* __restrict__ w,
                                                                uint16_t* __restrict__ wt,
                                                                uint16_t* __restrict__ wf,
                                                                uint8_t* __restrict__ wf4,
                                                                int T, int Cin, int Cout) {
  __shared__ uint16_t tile[64][64 + 8];  // [co][ci] +-1 bf16, padded rows
  const int t = blockIdx.x, ci0 = blockIdx.y * 64, co0 = blockIdx.z * 64;
  const int tid = threadIdx.x;
  // load: 64 co rows x 64 ci (fp32) = 1024 float4; 4 per thread
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int i = tid + j * 256;
    const int co = i / 16, c4 = (i % 16) * 4;
    const float4 v =
        *reinterpret_cast<const float4*>(w + ((long long)(co0 + co) * T + t) * Cin + ci0 + c4);
    tile[co][c4 + 0] = v.x >= 0.f ? 0x3F80 : 0xBF80;
    tile[co][c4 + 1] = v.y >= 0.f ? 0x3F80 : 0xBF80;
    tile[co][c4 + 2] = v.z >= 0.f ? 0x3F80 : 0xBF80;
    tile[co][c4 + 3] = v.w >= 0.f ? 0x3F80 : 0xBF80;
  }
  __syncthreads();
  // wf[t][co][ci]: 64 rows x 128 B = 512 uint4; 2 per thread
  if (wf) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int i = tid + j * 256;
      const int co = i / 8, c8 = (i % 8) * 8;
      uint32_t u[4];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        u[k] = (uint32_t)tile[co][c8 + 2 * k] | ((uint32_t)tile[co][c8 + 2 * k + 1] << 16);
      *reinterpret_cast<uint4*>(wf + ((long long)t * Cout + co0 + co) * Cin + ci0 + c8) =
          make_uint4(u[0], u[1], u[2], u[3]);
    }
  }
  // wf4[t][co][ci/2]: 64 rows x 32 B = 128 uint4
  if (wf4 && tid < 128) {
    const int co = tid >> 1, hf = tid & 1;
    uint32_t u[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      uint32_t nb = 0;
#pragma unroll
      for (int e = 0; e < 8; ++e)
        nb |= ((tile[co][hf * 32 + 8 * k + e] & 0x8000u) ? 0xAu : 0x2u) << (4 * e);
      u[k] = nb;
    }
    *reinterpret_cast<uint4*>(wf4 + (((long long)t * Cout + co0 + co) * Cin + ci0) / 2 +
                              hf * 16) = make_uint4(u[0], u[1], u[2], u[3]);
  }
  // wt[t][ci][co]: transposed read of the tile
  if (wt) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int i = tid + j * 256;
      const int ci = i / 8, o8 = (i % 8) * 8;
      uint32_t u[4];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        u[k] = (uint32_t)tile[o8 + 2 * k][ci] | ((uint32_t)tile[o8 + 2 * k + 1][ci] << 16);
      *reinterpret_cast<uint4*>(wt + ((long long)t * Cin + ci0 + ci) * Cout + co0 + o8) =
          make_uint4(u[0], u[1], u[2], u[3]);
    }
  }
}

// --------------------------------------------------------------------------
// XNOR-popcount implicit-GEMM forward
// --------------------------------------------------------------------------
struct ConvGeom {
  int B, H, W, Ho, Wo, Cout, kh, kw, stride, pad_t, pad_l;
  long long P;  // B*Ho*Wo
};

// TPS taps per K-stage (KS = TPS*CW words staged at once): few, large stages
// amortise the barrier and global-load latency when Cin is small.
template <int CW>
struct StageCfg {
  static constexpr int TPS = (CW <= 2) ? 9 : (16 / CW > 0 ? 16 / CW : 1);
  static constexpr int KS = TPS * CW;
};

template <int CW>
__global__ __launch_bounds__(NT, 3) void bconv_fwd_kernel(const uint32_t* __restrict__ xbits,
                                                       const uint32_t* __restrict__ wbits,
                                                       const int* __restrict__ wpop,
                                                       int16_t* __restrict__ y,
                                                       unsigned long long* __restrict__ stats,
                                                       ConvGeom g, int pad_ones, int relu) {
  constexpr int TPS = StageCfg<CW>::TPS;
  constexpr int KS = StageCfg<CW>::KS;
  constexpr int A_WORDS = BM * KS;
  constexpr int A_PER = (A_WORDS + NT - 1) / NT;
  constexpr int B_WORDS = BN * KS;
  constexpr int B_PER = (B_WORDS + NT - 1) / NT;

  __shared__ uint32_t As[KS][BM];
  __shared__ uint32_t Bs[KS][BN];
  __shared__ int pix_b[BM], pix_h[BM], pix_w[BM];
  __shared__ int red1[4][BN];
  __shared__ long long red2[4][BN];

  const int tid = threadIdx.x;
  const int tn = tid & 15;  // 4 channels each
  const int tm = tid >> 4;  // 8 pixels each
  const long long m0 = (long long)blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int T = g.kh * g.kw;
  const int nstages = (T + TPS - 1) / TPS;

  if (tid < BM) {
    const long long m = m0 + tid;
    if (m < g.P) {
      const int wo = (int)(m % g.Wo);
      const long long r = m / g.Wo;
      pix_b[tid] = (int)(r / g.Ho);
      pix_h[tid] = (int)(r % g.Ho) * g.stride - g.pad_t;
      pix_w[tid] = wo * g.stride - g.pad_l;
    } else {
      pix_b[tid] = -1;
      pix_h[tid] = pix_w[tid] = 0;
    }
  }
  __syncthreads();

  // Loader mapping: word i of a stage tile -> (pixel = i % BM, k = i / BM), so
  // each thread always loads the same pixel (its coordinates stay in 3
  // registers) and consecutive lanes write consecutive LDS words.
  static_assert(NT % BM == 0 && NT % BN == 0, "loader mapping");
  uint32_t ra[A_PER], rb[B_PER];
  const uint32_t pad_word = pad_ones ? 0xFFFFFFFFu : 0u;
  const int my_pix = tid % BM;
  const int my_b = pix_b[my_pix], my_h = pix_h[my_pix], my_w = pix_w[my_pix];
  const int my_n = tid % BN;
  auto load_stage = [&](int s) {
    const int t0 = s * TPS;
#pragma unroll
    for (int j = 0; j < A_PER; ++j) {
      const int k = tid / BM + j * (NT / BM);
      uint32_t v = 0;
      const int t = t0 + k / CW;
      if (k < KS && my_b >= 0 && t < T) {
        const int hi = my_h + t / g.kw, wi = my_w + t % g.kw;
        v = (hi >= 0 && hi < g.H && wi >= 0 && wi < g.W)
                ? xbits[(((long long)my_b * g.H + hi) * g.W + wi) * CW + (k % CW)]
                : pad_word;
      }
      ra[j] = v;
    }
#pragma unroll
    for (int j = 0; j < B_PER; ++j) {
      const int k = tid / BN + j * (NT / BN);
      const int t = t0 + k / CW;
      uint32_t v = 0;
      if (k < KS && n0 + my_n < g.Cout && t < T)
        v = wbits[((long long)(n0 + my_n) * T + t) * CW + (k % CW)];
      rb[j] = v;
    }
  };
  auto store_stage = [&]() {
#pragma unroll
    for (int j = 0; j < A_PER; ++j) {
      const int k = tid / BM + j * (NT / BM);
      if (k < KS) As[k][my_pix] = ra[j];
    }
#pragma unroll
    for (int j = 0; j < B_PER; ++j) {
      const int k = tid / BN + j * (NT / BN);
      if (k < KS) Bs[k][my_n] = rb[j];
    }
  };

  int acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = 0;

  load_stage(0);
  for (int s = 0; s < nstages; ++s) {
    if (s) __syncthreads();  // previous stage fully consumed
    store_stage();
    __syncthreads();
    if (s + 1 < nstages) load_stage(s + 1);  // prefetch under the compute
    const int kwords = min(TPS, T - s * TPS) * CW;
    for (int k = 0; k < kwords; ++k) {
      const uint4 a0 = *reinterpret_cast<const uint4*>(&As[k][tm * 8]);
      const uint4 a1 = *reinterpret_cast<const uint4*>(&As[k][tm * 8 + 4]);
      const uint4 bq = *reinterpret_cast<const uint4*>(&Bs[k][tn * 4]);
      const uint32_t a[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
      const uint32_t b[4] = {bq.x, bq.y, bq.z, bq.w};
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] += __popc(a[i] ^ b[j]);
    }
  }

  // ---- epilogue: padding correction, ReLU, int16 store, BN statistics ----
  int s1[4] = {0, 0, 0, 0};
  long long s2[4] = {0, 0, 0, 0};
  const int nbase = n0 + tn * 4;
  const int full = 32 * CW * T;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int pix = tm * 8 + i;
    const long long m = m0 + pix;
    if (m >= g.P) continue;
    int corr[4] = {0, 0, 0, 0};
    int kmax = full;
    if (!pad_ones) {
      const int hi0 = pix_h[pix], wi0 = pix_w[pix];
      // Fast path: interior pixel, every tap valid.
      if (hi0 < 0 || wi0 < 0 || hi0 + g.kh > g.H || wi0 + g.kw > g.W) {
        int nvalid = 0;
        for (int t = 0; t < T; ++t) {
          const int hi = hi0 + t / g.kw, wi = wi0 + t % g.kw;
          if (hi >= 0 && hi < g.H && wi >= 0 && wi < g.W) {
            ++nvalid;
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
              corr[j] += (nbase + j < g.Cout) ? wpop[(nbase + j) * T + t] : 0;
          }
        }
        kmax = 32 * CW * nvalid;
      }
    }
    int16_t out[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int v = kmax - 2 * acc[i][j] + 2 * corr[j];
      if (relu) v = v > 0 ? v : 0;
      out[j] = (int16_t)v;
      s1[j] += v;
      s2[j] += (long long)v * v;
    }
    if (nbase + 3 < g.Cout) {
      uint2 pk;
      pk.x = (uint32_t)(uint16_t)out[0] | ((uint32_t)(uint16_t)out[1] << 16);
      pk.y = (uint32_t)(uint16_t)out[2] | ((uint32_t)(uint16_t)out[3] << 16);
      *reinterpret_cast<uint2*>(y + m * g.Cout + nbase) = pk;
    } else {
      for (int j = 0; j < 4; ++j)
        if (nbase + j < g.Cout) y[m * g.Cout + nbase + j] = out[j];
    }
  }
  // Statistics: reduce over the 16 threads sharing `tn` (lanes tn+16q of a
  // wave via shuffles, then the 4 waves through LDS), one atomic per channel.
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    s1[j] += __shfl_xor(s1[j], 16, 64);
    s1[j] += __shfl_xor(s1[j], 32, 64);
    s2[j] += __shfl_xor(s2[j], 16, 64);
    s2[j] += __shfl_xor(s2[j], 32, 64);
  }
  const int wave = tid >> 6, lane = tid & 63;
  if (lane < 16) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      red1[wave][lane * 4 + j] = s1[j];
      red2[wave][lane * 4 + j] = s2[j];
    }
  }
  __syncthreads();
  if (tid < BN && n0 + tid < g.Cout) {
    long long a = 0, b = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      a += red1[w][tid];
      b += red2[w][tid];
    }
    atomicAdd(stats + n0 + tid, (unsigned long long)a);
    atomicAdd(stats + g.Cout + n0 + tid, (unsigned long long)b);
  }
}

// --------------------------------------------------------------------------
// Bits -> bf16 ±1 (for library GEMM operands), optional +1 padding handled
// by the caller.
// --------------------------------------------------------------------------
__global__ __launch_bounds__(256) void unpack_sign_kernel(const uint32_t* __restrict__ bits,
                                                          uint16_t* __restrict__ out,
                                                          long long nwords) {
  for (long long w = blockIdx.x * (long long)blockDim.x + threadIdx.x; w < nwords;
       w += (long long)gridDim.x * blockDim.x) {
    const uint32_t b = bits[w];
    uint4* dst = reinterpret_cast<uint4*>(out + 32 * w);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint32_t v[4];
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const int i = q * 8 + h * 2;
        const uint32_t lo = ((b >> i) & 1) ? 0x3F80u : 0xBF80u;
        const uint32_t hi = ((b >> (i + 1)) & 1) ? 0x3F80u : 0xBF80u;
        v[h] = lo | (hi << 16);
      }
      dst[q] = make_uint4(v[0], v[1], v[2], v[3]);
    }
  }
}

int grid_for(long long work, int per_block = 256, int cap = 16384) {
  long long b = (work + per_block - 1) / per_block;
  if (b > cap) b = cap;
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace

// xs: bf16 +-1 image (optional), xs4: e2m1 +-1 image [.][C/2] (optional).
ZK_EXPORT int zk_sign_pack(const void* x, void* bits, void* mask, void* xs, void* xs4,
                           long long nwords, float clip, hipStream_t stream) {
  hipLaunchKernelGGL(sign_pack_kernel, dim3(grid_for(nwords)), dim3(256), 0, stream,
                     (const uint16_t*)x, (uint32_t*)bits, (uint32_t*)mask, (uint16_t*)xs,
                     (uint4*)xs4, nwords, clip);
  ZK_CHECK_LAUNCH();
  return 0;
}

// wf4 (e2m1 forward layout) needs the tiled path: no bit outputs, Cin and
// Cout multiples of 64.
ZK_EXPORT int zk_weight_pack(const void* w, void* wbits, void* wpop, void* wt, void* wf,
                             void* wf4, int Cout, int T, int Cin, hipStream_t stream) {
  if (Cin % 32) return (int)hipErrorInvalidValue;
  const bool tiled = !wbits && !wpop && Cin % 64 == 0 && Cout % 64 == 0;
  if (wf4 && !tiled) return (int)hipErrorInvalidValue;
  if (tiled) {
    hipLaunchKernelGGL(weight_pack_tiled_kernel, dim3(T, Cin / 64, Cout / 64), dim3(256), 0,
                       stream, (const float*)w, (uint16_t*)wt, (uint16_t*)wf, (uint8_t*)wf4, T,
                       Cin, Cout);
    ZK_CHECK_LAUNCH();
    return 0;
  }
  const long long nwords = (long long)Cout * T * (Cin / 32);
  if (wpop) hipMemsetAsync(wpop, 0, sizeof(int) * (size_t)Cout * T, stream);
  hipLaunchKernelGGL(weight_pack_kernel, dim3((unsigned)((nwords + 255) / 256)), dim3(256), 0,
                     stream, (const float*)w, (uint32_t*)wbits, (int*)wpop, (uint16_t*)wt,
                     (uint16_t*)wf, nwords, Cin / 32, T, Cout);
  ZK_CHECK_LAUNCH();
  return 0;
}

ZK_EXPORT int zk_unpack_sign(const void* bits, void* out, long long nwords, hipStream_t stream) {
  hipLaunchKernelGGL(unpack_sign_kernel, dim3(grid_for(nwords)), dim3(256), 0, stream,
                     (const uint32_t*)bits, (uint16_t*)out, nwords);
  ZK_CHECK_LAUNCH();
  return 0;
}

// stats must be zeroed by the caller ([2][Cout] int64).
ZK_EXPORT int zk_bconv_fwd(const void* xbits, const void* wbits, const void* wpop, void* y,
                           void* stats, int B, int H, int W, int Cin, int Cout, int kh, int kw,
                           int stride, int pad_t, int pad_l, int Ho, int Wo, int pad_ones,
                           int relu, hipStream_t stream) {
  if (Cin % 32 || kh * kw > 9) return (int)hipErrorInvalidValue;
  ConvGeom g{B, H, W, Ho, Wo, Cout, kh, kw, stride, pad_t, pad_l, (long long)B * Ho * Wo};
  dim3 grid((unsigned)((g.P + BM - 1) / BM), (unsigned)((Cout + BN - 1) / BN));
  const int CW = Cin / 32;
#define ZK_BCONV_CASE(cw)                                                                   \
  case cw:                                                                                  \
    hipLaunchKernelGGL(bconv_fwd_kernel<cw>, grid, dim3(NT), 0, stream,                      \
                       (const uint32_t*)xbits, (const uint32_t*)wbits, (const int*)wpop,     \
                       (int16_t*)y, (unsigned long long*)stats, g, pad_ones, relu);          \
    break;
  switch (CW) {
    ZK_BCONV_CASE(1)
    ZK_BCONV_CASE(2)
    ZK_BCONV_CASE(4)
    ZK_BCONV_CASE(8)
    ZK_BCONV_CASE(16)
    ZK_BCONV_CASE(32)
    default:
      return (int)hipErrorInvalidValue;
  }
#undef ZK_BCONV_CASE
  ZK_CHECK_LAUNCH();
  return 0;
}
