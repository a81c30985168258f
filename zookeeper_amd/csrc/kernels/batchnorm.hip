// BatchNorm pieces fused around the binary convolution (gfx950).
//
// Training-mode BN over NHWC [P][C] tensors (P = B*H*W):
//   forward   stats come exact (int64 sums of the int16 conv output, from the
//             conv epilogue) -> bn_finalize (per-channel scale/shift, running
//             statistics update with Bessel's correction, saved mean/rstd)
//             -> bn_apply: out = scale[c]*y + shift[c] (+ residual), bf16.
//   backward  bn_bwd_reduce: sum(g), sum(g*yhat) per channel
//             -> bn_bwd_dx: dy = gamma*rstd*(g - mean(g) - yhat*mean(g*yhat))
//                (times 1{y>0} when a ReLU sits between conv and BN)
//             -> optional STE + residual: dx = dgrad * 1{|x|<=clip} + dres.
// All kernels are HBM-bound; every thread moves 16 B per tensor per access
// (8 channels), vectorised, with grid-stride loops.
#include "../common.h"

namespace {

// Consumers re-zero the accumulators they read (stats / sums), so callers can
// keep one persistent zeroed buffer per layer instead of a fill per step.
// stats: [stripes][2][C] exact int64 copies (the conv epilogues spread their
// atomics over them).  A group of 32 lanes owns one channel: lane k sums
// copies k, k+32, ... and the group reduces with cross-lane shuffles.
__global__ __launch_bounds__(256) void bn_finalize_kernel(
    unsigned long long* __restrict__ stats, int C, int stripes, double P,
    const float* __restrict__ gamma, const float* __restrict__ beta, float eps, float momentum,
    float* __restrict__ running_mean, float* __restrict__ running_var, float* __restrict__ scale,
    float* __restrict__ shift, float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  const int k = threadIdx.x & 31;
  const int c = blockIdx.x * 8 + (threadIdx.x >> 5);
  if (c >= C) return;  // uniform over the 32-lane group
  long long t1 = 0, t2 = 0;
  for (int j = k; j < stripes; j += 32) {
    t1 += (long long)stats[(2LL * j) * C + c];
    t2 += (long long)stats[(2LL * j + 1) * C + c];
    stats[(2LL * j) * C + c] = 0;
    stats[(2LL * j + 1) * C + c] = 0;
  }
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) {
    t1 += __shfl_xor(t1, o, 32);
    t2 += __shfl_xor(t2, o, 32);
  }
  if (k != 0) return;
  const double s1 = (double)t1;
  const double s2 = (double)t2;
  const double mean = s1 / P;
  double var = s2 / P - mean * mean;
  if (var < 0) var = 0;
  const float rstd = (float)(1.0 / sqrt(var + (double)eps));
  const float g = gamma ? gamma[c] : 1.f;
  const float b = beta ? beta[c] : 0.f;
  scale[c] = g * rstd;
  shift[c] = b - (float)mean * g * rstd;
  mean_out[c] = (float)mean;
  rstd_out[c] = rstd;
  if (running_mean) {
    const double unbiased = P > 1 ? var * P / (P - 1) : var;
    // Keras convention: moving = momentum * moving + (1 - momentum) * batch.
    running_mean[c] = momentum * running_mean[c] + (1.f - momentum) * (float)mean;
    running_var[c] = momentum * running_var[c] + (1.f - momentum) * (float)unbiased;
  }
}

// The BN apply of one 8-channel chunk: scale*y + shift (+ the residual
// chunk rv when has_res), packed as stored (bf16).
__device__ __forceinline__ uint4 bn_apply_values(const uint4& yv, const uint4& rv, bool has_res,
                                                 const float (&sc)[8], const float (&sh)[8]) {
  const int16_t* yy = reinterpret_cast<const int16_t*>(&yv);
  float o[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) o[k] = sc[k] * (float)yy[k] + sh[k];
  if (has_res) {
    const uint32_t rr[4] = {rv.x, rv.y, rv.z, rv.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      o[2 * k] += zk::bf16_to_f32((uint16_t)(rr[k] & 0xffff));
      o[2 * k + 1] += zk::bf16_to_f32((uint16_t)(rr[k] >> 16));
    }
  }
  return make_uint4(zk::pack_bf16x2(o[0], o[1]), zk::pack_bf16x2(o[2], o[3]),
                    zk::pack_bf16x2(o[4], o[5]), zk::pack_bf16x2(o[6], o[7]));
}

// Store chunk i of the BN output and the next binary layer's input
// quantisation from the stored bf16 values (bf16 sign image, STE mask bits,
// e2m1 sign image; each optional).
__device__ __forceinline__ void bn_apply_store(long long i, const uint4& ov,
                                               uint16_t* __restrict__ out,
                                               uint16_t* __restrict__ sx,
                                               uint8_t* __restrict__ smask, float clip,
                                               uint32_t* __restrict__ sx4) {
  reinterpret_cast<uint4*>(out)[i] = ov;
  if (sx || sx4) {
    // the NEXT binary block's input quantisation, from the stored bf16
    // values: sign image (bf16 +-1 for the weight gradient, e2m1 nibbles
    // for the MX-FP4 forward) and STE mask bits (|x| <= clip)
    const uint32_t ow[4] = {ov.x, ov.y, ov.z, ov.w};
    uint32_t sw[4];
    uint32_t mk = 0, n4 = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float lo = zk::bf16_to_f32((uint16_t)(ow[k] & 0xffff));
      const float hi = zk::bf16_to_f32((uint16_t)(ow[k] >> 16));
      sw[k] = (lo >= 0.f ? 0x3F80u : 0xBF80u) | ((hi >= 0.f ? 0x3F80u : 0xBF80u) << 16);
      mk |= (uint32_t)(fabsf(lo) <= clip) << (2 * k);
      mk |= (uint32_t)(fabsf(hi) <= clip) << (2 * k + 1);
      n4 |= (zk::fp4_sign(lo) | (zk::fp4_sign(hi) << 4)) << (8 * k);
    }
    if (sx) reinterpret_cast<uint4*>(sx)[i] = make_uint4(sw[0], sw[1], sw[2], sw[3]);
    if (smask) smask[i] = (uint8_t)mk;  // byte i = channels 8i..8i+7 of the packed mask words
    if (sx4) sx4[i] = n4;               // 8 channels = 4 bytes of the [P][C/2] e2m1 image
  }
}

// y int16 [P][C] -> out bf16 = scale*y + shift (+ residual bf16).
// Each thread owns one group of 8 channels (coefficients in registers) and
// walks rows; CG = C/8 threads cover a row.
template <int CG>
__global__ __launch_bounds__(256) void bn_apply_kernel(const int16_t* __restrict__ y,
                                                       const float* __restrict__ scale,
                                                       const float* __restrict__ shift,
                                                       const uint16_t* __restrict__ res,
                                                       uint16_t* __restrict__ out,
                                                       long long P,
                                                       uint16_t* __restrict__ sx = nullptr,
                                                       uint8_t* __restrict__ smask = nullptr,
                                                       float clip = 1.f,
                                                       uint32_t* __restrict__ sx4 = nullptr) {
  constexpr int C = CG * 8;
  constexpr int RB = 256 / CG;
  const int cg = threadIdx.x % CG;
  float sc[8], sh[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    sc[k] = scale[cg * 8 + k];
    sh[k] = shift[cg * 8 + k];
  }
  for (long long r = (long long)blockIdx.x * RB + threadIdx.x / CG; r < P;
       r += (long long)gridDim.x * RB) {
    const long long i = (r * C) / 8 + cg;
    const uint4 yv = reinterpret_cast<const uint4*>(y)[i];
    const uint4 rv = res ? reinterpret_cast<const uint4*>(res)[i] : make_uint4(0, 0, 0, 0);
    bn_apply_store(i, bn_apply_values(yv, rv, res != nullptr, sc, sh), out, sx, smask, clip,
                   sx4);
  }
}

// bn_apply_kernel over 2x2 pixel quads of an even [B][H][W] image, plus the
// 2x2/2 average pool of the stored output (a downsampling shortcut's input):
// pooled [B][H/2][W/2][C] bf16, summed in avgpool2_fwd_kernel's order
// ((h, w), (h, w+1), (h+1, w), (h+1, w+1)) from the stored bf16 values, so it
// equals that kernel's result bit for bit.
template <int CG>
__global__ __launch_bounds__(256) void bn_apply_pool_kernel(
    const int16_t* __restrict__ y, const float* __restrict__ scale,
    const float* __restrict__ shift, const uint16_t* __restrict__ res,
    uint16_t* __restrict__ out, int B, int H, int W, uint16_t* __restrict__ sx,
    uint8_t* __restrict__ smask, float clip, uint32_t* __restrict__ sx4,
    uint16_t* __restrict__ pooled) {
  constexpr int QB = 256 / CG;  // quads per block iteration
  const int cg = threadIdx.x % CG;
  const int Ho = H / 2, Wo = W / 2;
  float sc[8], sh[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    sc[k] = scale[cg * 8 + k];
    sh[k] = shift[cg * 8 + k];
  }
  const long long nq = (long long)B * Ho * Wo;
  for (long long q = (long long)blockIdx.x * QB + threadIdx.x / CG; q < nq;
       q += (long long)gridDim.x * QB) {
    const int wo = (int)(q % Wo);
    const long long t = q / Wo;
    const int ho = (int)(t % Ho);
    const int b = (int)(t / Ho);
    // the quad's loads all issued before the first store
    long long ci[4];
    uint4 yv[4], rv[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      ci[d] = (((long long)b * H + 2 * ho + (d >> 1)) * W + 2 * wo + (d & 1)) * CG + cg;
      yv[d] = reinterpret_cast<const uint4*>(y)[ci[d]];
    }
#pragma unroll
    for (int d = 0; d < 4; ++d)
      rv[d] = res ? reinterpret_cast<const uint4*>(res)[ci[d]] : make_uint4(0, 0, 0, 0);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const uint4 ov = bn_apply_values(yv[d], rv[d], res != nullptr, sc, sh);
      bn_apply_store(ci[d], ov, out, sx, smask, clip, sx4);
      const uint32_t ow[4] = {ov.x, ov.y, ov.z, ov.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        acc[2 * k] += zk::bf16_to_f32((uint16_t)(ow[k] & 0xffff));
        acc[2 * k + 1] += zk::bf16_to_f32((uint16_t)(ow[k] >> 16));
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] *= 0.25f;
    reinterpret_cast<uint4*>(pooled)[q * CG + cg] =
        make_uint4(zk::pack_bf16x2(acc[0], acc[1]), zk::pack_bf16x2(acc[2], acc[3]),
                   zk::pack_bf16x2(acc[4], acc[5]), zk::pack_bf16x2(acc[6], acc[7]));
  }
}

// sums[0][c] += sum g ; sums[1][c] += sum g*yhat  (g bf16, y int16)
template <int CG>  // channel groups of 8 per row = C / 8
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(const uint16_t* __restrict__ g,
                                                            const int16_t* __restrict__ y,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ rstd,
                                                            float* __restrict__ sums,
                                                            long long P, int stripes) {
  constexpr int C = CG * 8;
  constexpr int RB = 256 / CG;  // rows per block iteration
  const int cg = threadIdx.x % CG;
  const int r0 = threadIdx.x / CG;
  float mu[8], rs[8], sg[8], sgy[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    mu[k] = mean[cg * 8 + k];
    rs[k] = rstd[cg * 8 + k];
    sg[k] = 0.f;
    sgy[k] = 0.f;
  }
  // UR rows per thread in flight per iteration (loads first, then math):
  // one 16-B load pair per iteration left HBM latency-bound (~3.7 TB/s)
  constexpr int UR = 4;
  const long long rstep = (long long)gridDim.x * RB;
  for (long long r = (long long)blockIdx.x * RB + r0; r < P; r += UR * rstep) {
    uint4 gv[UR], yv[UR];
#pragma unroll
    for (int u = 0; u < UR; ++u) {
      const long long ru = r + u * rstep;
      gv[u] = make_uint4(0, 0, 0, 0);
      yv[u] = make_uint4(0, 0, 0, 0);
      if (ru < P) {
        const long long off = ru * C + cg * 8;
        gv[u] = *reinterpret_cast<const uint4*>(g + off);
        yv[u] = *reinterpret_cast<const uint4*>(y + off);
      }
    }
#pragma unroll
    for (int u = 0; u < UR; ++u) {
      // rows past P loaded zeros: g = 0 adds nothing to either sum
      const uint32_t gg[4] = {gv[u].x, gv[u].y, gv[u].z, gv[u].w};
      const int16_t* yy = reinterpret_cast<const int16_t*>(&yv[u]);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float gk = zk::bf16_to_f32((uint16_t)(gg[k >> 1] >> (16 * (k & 1))));
        sg[k] += gk;
        sgy[k] += gk * ((float)yy[k] - mu[k]) * rs[k];
      }
    }
  }
  __shared__ float red[2][256][9];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    red[0][threadIdx.x][k] = sg[k];
    red[1][threadIdx.x][k] = sgy[k];
  }
  __syncthreads();
  // copies in channel-major layout [2][C][stripes]: copy j of channel c's
  // statistic s at (s*C + c)*stripes + j (bn_bwd_coef reads a channel's
  // copies as contiguous float4s).  One copy per block (stripes >= blocks,
  // the default): plain stores, summed in a fixed order by bn_bwd_coef.
  const int copy = (int)(blockIdx.x % stripes);
  const bool own = stripes >= (int)gridDim.x;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const int gcg = c / 8, k = c % 8;
    float a = 0.f, b = 0.f;
    for (int rr = 0; rr < RB; ++rr) {
      a += red[0][rr * CG + gcg][k];
      b += red[1][rr * CG + gcg][k];
    }
    float* o0 = sums + (long long)c * stripes + copy;
    float* o1 = sums + (long long)(C + c) * stripes + copy;
    if (own) {
      *o0 = a;
      *o1 = b;
    } else {
      atomicAdd(o0, a);
      atomicAdd(o1, b);
    }
  }
}

// dy = k1[c]*g + k0[c] - k3[c]*y   [times 1{y>0} if relu], with the folded
// coefficients from bn_bwd_coef: k1 = gamma*rstd, k3 = k1*rstd*mean(g*yhat),
// k0 = k3*mean - k1*mean(g).
template <int CG>
__global__ __launch_bounds__(256) void bn_bwd_dx_kernel(const uint16_t* __restrict__ g,
                                                        const int16_t* __restrict__ y,
                                                        const float* __restrict__ coef,
                                                        uint16_t* __restrict__ dy, long long P,
                                                        int relu) {
  constexpr int C = CG * 8;
  constexpr int RB = 256 / CG;
  const int cg = threadIdx.x % CG;
  float k1[8], k0[8], k3[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int c = cg * 8 + k;
    k1[k] = coef[c];
    k0[k] = coef[C + c];
    k3[k] = coef[2 * C + c];
  }
  for (long long r = (long long)blockIdx.x * RB + threadIdx.x / CG; r < P;
       r += (long long)gridDim.x * RB) {
    const long long i = (r * C) / 8 + cg;
    const uint4 gv = reinterpret_cast<const uint4*>(g)[i];
    const uint4 yv = reinterpret_cast<const uint4*>(y)[i];
    const uint32_t gg[4] = {gv.x, gv.y, gv.z, gv.w};
    const int16_t* yy = reinterpret_cast<const int16_t*>(&yv);
    float o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float gk = zk::bf16_to_f32((uint16_t)(gg[k >> 1] >> (16 * (k & 1))));
      float v = k1[k] * gk + k0[k] - k3[k] * (float)yy[k];
      if (relu && yy[k] <= 0) v = 0.f;
      o[k] = v;
    }
    reinterpret_cast<uint4*>(dy)[i] =
        make_uint4(zk::pack_bf16x2(o[0], o[1]), zk::pack_bf16x2(o[2], o[3]),
                   zk::pack_bf16x2(o[4], o[5]), zk::pack_bf16x2(o[6], o[7]));
  }
}

// Per-channel backward coefficients from the reductions (one tiny launch
// instead of a chain of framework ops), plus gamma/beta gradients
// accumulated straight into the parameters' gradient buffers:
//   sums = channel-major copies [2][C][stride] of (sum g, sum g*yhat): the
//   first `stripes` copies of a channel are contiguous, read as float4s by
//   32 lanes (4 per lane at 512 copies) and summed in a fixed order (lane
//   partials, then a butterfly), then re-zeroed;
//   coef = [k1, k0, k3];  dgamma += sum g*yhat,  dbeta += sum g.
// A group of 32 lanes owns one channel.  (The [stripe][2][C] layout this
// replaced made each lane walk its copies 2C floats apart, 16 dependent
// loads per lane at 512 copies: ~90 us per call on a busy chip.)
__device__ __forceinline__ float coef_row_sum(float* __restrict__ row, int stripes, int k) {
  float acc = 0.f;
  const int n4 = (reinterpret_cast<uintptr_t>(row) & 15) ? 0 : stripes >> 2;
  float4* r4 = reinterpret_cast<float4*>(row);
#pragma unroll 4
  for (int j = k; j < n4; j += 32) {
    const float4 q = r4[j];
    acc += (q.x + q.y) + (q.z + q.w);
    r4[j] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  for (int j = n4 * 4 + k; j < stripes; j += 32) {
    acc += row[j];
    row[j] = 0.f;
  }
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 32);
  return acc;
}

__global__ __launch_bounds__(256) void bn_bwd_coef_kernel(float* __restrict__ sums,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ rstd,
                                                          const float* __restrict__ gamma,
                                                          double P, int C, int stripes,
                                                          int stride,
                                                          float* __restrict__ coef,
                                                          float* __restrict__ dgamma,
                                                          float* __restrict__ dbeta) {
  const int k = threadIdx.x & 31;
  const int c = blockIdx.x * 8 + (threadIdx.x >> 5);
  if (c >= C) return;  // uniform over the 32-lane group
  const float sg = coef_row_sum(sums + (long long)c * stride, stripes, k);
  const float sgy = coef_row_sum(sums + (long long)(C + c) * stride, stripes, k);
  if (k != 0) return;
  const float rs = rstd[c];
  const float k1 = (gamma ? gamma[c] : 1.f) * rs;
  const float k3 = k1 * rs * (float)(sgy / P);
  coef[c] = k1;
  coef[C + c] = k3 * mean[c] - k1 * (float)(sg / P);
  coef[2 * C + c] = k3;
  if (dgamma) dgamma[c] += sgy;
  if (dbeta) dbeta[c] += sg;
}

// dx = dgrad * bit(mask) (+ dres), all [P][C]; mask packed [P][C/32]
__global__ __launch_bounds__(256) void ste_combine_kernel(const uint16_t* __restrict__ dgrad,
                                                          const uint32_t* __restrict__ mask,
                                                          const uint16_t* __restrict__ dres,
                                                          uint16_t* __restrict__ dx,
                                                          long long n8) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n8;
       i += (long long)gridDim.x * blockDim.x) {
    const uint32_t mw = mask[i >> 2];  // 8 channels = one quarter of a word
    const int sh = (int)(i & 3) * 8;
    const uint4 dv = reinterpret_cast<const uint4*>(dgrad)[i];
    uint32_t d[4] = {dv.x, dv.y, dv.z, dv.w};
    uint32_t r[4] = {0, 0, 0, 0};
    if (dres) {
      const uint4 rv = reinterpret_cast<const uint4*>(dres)[i];
      r[0] = rv.x; r[1] = rv.y; r[2] = rv.z; r[3] = rv.w;
    }
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float lo = ((mw >> (sh + 2 * k)) & 1) ? zk::bf16_to_f32((uint16_t)(d[k] & 0xffff)) : 0.f;
      float hi = ((mw >> (sh + 2 * k + 1)) & 1) ? zk::bf16_to_f32((uint16_t)(d[k] >> 16)) : 0.f;
      if (dres) {
        lo += zk::bf16_to_f32((uint16_t)(r[k] & 0xffff));
        hi += zk::bf16_to_f32((uint16_t)(r[k] >> 16));
      }
      o[k] = zk::pack_bf16x2(lo, hi);
    }
    reinterpret_cast<uint4*>(dx)[i] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

int grid_for(long long work, int cap = 4096) {
  long long b = (work + 255) / 256;
  if (b > cap) b = cap;
  return b < 1 ? 1 : (int)b;
}

}  // namespace

// stats: [stripes][2][C] int64 (sum, sum of squares), re-zeroed here.
ZK_EXPORT int zk_bn_finalize(const void* stats, int C, int stripes, double P, const void* gamma,
                             const void* beta, float eps, float momentum, void* running_mean,
                             void* running_var, void* scale, void* shift, void* mean,
                             void* rstd, hipStream_t stream) {
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 7) / 8), dim3(256), 0, stream,
                     (unsigned long long*)stats, C, stripes < 1 ? 1 : stripes, P,
                     (const float*)gamma,
                     (const float*)beta, eps, momentum, (float*)running_mean,
                     (float*)running_var, (float*)scale, (float*)shift, (float*)mean,
                     (float*)rstd);
  ZK_CHECK_LAUNCH();
  return 0;
}

#define ZK_CG_SWITCH(C, MACRO) \
  switch ((C) / 8) {            \
    MACRO(4)                    \
    MACRO(8)                    \
    MACRO(16)                   \
    MACRO(32)                   \
    MACRO(64)                   \
    default:                    \
      return (int)hipErrorInvalidValue; \
  }

// Up to 65536 blocks (a few rows per thread): the apply / dx kernels ran
// 12-16 % faster than with a 4096-block grid-stride walk at every E18 stage
// (tools/bn_lab.py, profiles/r6/bn_grid.md).
static int rows_grid(long long P, int C) {
  const long long rb = 256 / (C / 8);
  long long b = (P + rb - 1) / rb;
  if (b > 65536) b = 65536;
  return b < 1 ? 1 : (int)b;
}

ZK_EXPORT int zk_bn_apply(const void* y, const void* scale, const void* shift, const void* res,
                          void* out, long long P, int C, hipStream_t stream) {
  if (C % 32) return (int)hipErrorInvalidValue;
#define ZK_APPLY_CASE(cg)                                                                   \
  case cg:                                                                                  \
    hipLaunchKernelGGL(bn_apply_kernel<cg>, dim3(rows_grid(P, C)), dim3(256), 0, stream,    \
                       (const int16_t*)y, (const float*)scale, (const float*)shift,         \
                       (const uint16_t*)res, (uint16_t*)out, P);                            \
    break;
  ZK_CG_SWITCH(C, ZK_APPLY_CASE)
#undef ZK_APPLY_CASE
  ZK_CHECK_LAUNCH();
  return 0;
}

// zk_bn_apply + the next binary layer's input quantisation (sign image sx
// bf16 +-1, STE mask bits |out| <= clip and the e2m1 sign image sx4, packed
// like zk_sign_pack's; each optional).
ZK_EXPORT int zk_bn_apply_sign(const void* y, const void* scale, const void* shift,
                               const void* res, void* out, void* sx, void* mask, void* sx4,
                               float clip, long long P, int C, hipStream_t stream) {
  if (C % 32) return (int)hipErrorInvalidValue;
#define ZK_APPLY_CASE(cg)                                                                   \
  case cg:                                                                                  \
    hipLaunchKernelGGL(bn_apply_kernel<cg>, dim3(rows_grid(P, C)), dim3(256), 0, stream,    \
                       (const int16_t*)y, (const float*)scale, (const float*)shift,         \
                       (const uint16_t*)res, (uint16_t*)out, P, (uint16_t*)sx,              \
                       (uint8_t*)mask, clip, (uint32_t*)sx4);                               \
    break;
  ZK_CG_SWITCH(C, ZK_APPLY_CASE)
#undef ZK_APPLY_CASE
  ZK_CHECK_LAUNCH();
  return 0;
}

// zk_bn_apply_sign over an even [B][H][W] image, plus pooled = the 2x2/2
// average pool of out (bit-identical to zk_avgpool2 of it): the stage
// transition's shortcut input without a pass over out.
ZK_EXPORT int zk_bn_apply_sign_pool(const void* y, const void* scale, const void* shift,
                                    const void* res, void* out, void* sx, void* mask, void* sx4,
                                    float clip, void* pooled, int B, int H, int W, int C,
                                    hipStream_t stream) {
  if (C % 32 || H % 2 || W % 2 || !pooled || B < 1) return (int)hipErrorInvalidValue;
  const long long nq = (long long)B * (H / 2) * (W / 2);
#define ZK_APPLY_POOL_CASE(cg)                                                              \
  case cg: {                                                                                \
    long long blocks = (nq + 256 / cg - 1) / (256 / cg);                                    \
    if (blocks > 65536) blocks = 65536; /* as rows_grid: 5-7 % faster than 4096 */           \
    hipLaunchKernelGGL(bn_apply_pool_kernel<cg>, dim3((int)blocks), dim3(256), 0, stream,   \
                       (const int16_t*)y, (const float*)scale, (const float*)shift,         \
                       (const uint16_t*)res, (uint16_t*)out, B, H, W, (uint16_t*)sx,        \
                       (uint8_t*)mask, clip, (uint32_t*)sx4, (uint16_t*)pooled);            \
    break;                                                                                  \
  }
  ZK_CG_SWITCH(C, ZK_APPLY_POOL_CASE)
#undef ZK_APPLY_POOL_CASE
  ZK_CHECK_LAUNCH();
  return 0;
}

// sums: [2][C][stripes] fp32 channel-major copies (block b writes / adds
// into copy b % stripes).
ZK_EXPORT int zk_bn_bwd_reduce_blocks() { return 512; }

namespace {
int bn_bwd_reduce_launch(const void* g, const void* y, const void* mean, const void* rstd,
                         void* sums, long long P, int C, int stripes, hipStream_t stream) {
  if (stripes < 1) stripes = 1;
  // 512 blocks x 4 rows in flight per thread: enough bytes in flight for
  // HBM, few enough per-block atomics into the 2*C sums.  stripes >= 512:
  // every block owns a copy (no atomics: bit-reproducible).
  const int blocks = 512;
#define ZK_RED_CASE(cg)                                                                   \
  case cg:                                                                                \
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<cg>, dim3(blocks), dim3(256), 0, stream,      \
                       (const uint16_t*)g, (const int16_t*)y, (const float*)mean,         \
                       (const float*)rstd, (float*)sums, P, stripes);                     \
    break;
  switch (C / 8) {
    ZK_RED_CASE(4)
    ZK_RED_CASE(8)
    ZK_RED_CASE(16)
    ZK_RED_CASE(32)
    ZK_RED_CASE(64)
    default:
      return (int)hipErrorInvalidValue;
  }
#undef ZK_RED_CASE
  ZK_CHECK_LAUNCH();
  return 0;
}
}  // namespace

ZK_EXPORT int zk_bn_bwd_reduce(const void* g, const void* y, const void* mean, const void* rstd,
                               void* sums, long long P, int C, int stripes, hipStream_t stream) {
  return bn_bwd_reduce_launch(g, y, mean, rstd, sums, P, C, stripes, stream);
}

ZK_EXPORT int zk_bn_bwd_dx(const void* g, const void* y, const void* coef, void* dy, long long P,
                           int C, int relu, hipStream_t stream) {
  if (C % 32) return (int)hipErrorInvalidValue;
#define ZK_DX_CASE(cg)                                                                      \
  case cg:                                                                                  \
    hipLaunchKernelGGL(bn_bwd_dx_kernel<cg>, dim3(rows_grid(P, C)), dim3(256), 0, stream,   \
                       (const uint16_t*)g, (const int16_t*)y, (const float*)coef,           \
                       (uint16_t*)dy, P, relu);                                             \
    break;
  ZK_CG_SWITCH(C, ZK_DX_CASE)
#undef ZK_DX_CASE
  ZK_CHECK_LAUNCH();
  return 0;
}

// sums: channel-major copies [2][C][stride] (stride >= stripes; the first
// `stripes` copies of each row are summed in a fixed order and re-zeroed).
ZK_EXPORT int zk_bn_bwd_coef(const void* sums, const void* mean, const void* rstd,
                             const void* gamma, double P, int C, int stripes, int stride,
                             void* coef, void* dgamma, void* dbeta, hipStream_t stream) {
  if (stripes < 1) stripes = 1;
  if (stride < stripes) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(bn_bwd_coef_kernel, dim3((C + 7) / 8), dim3(256), 0, stream, (float*)sums,
                     (const float*)mean, (const float*)rstd, (const float*)gamma, P, C,
                     stripes, stride, (float*)coef, (float*)dgamma, (float*)dbeta);
  ZK_CHECK_LAUNCH();
  return 0;
}

ZK_EXPORT int zk_ste_combine(const void* dgrad, const void* mask, const void* dres, void* dx,
                             long long n_elems, hipStream_t stream) {
  if (n_elems % 32) return (int)hipErrorInvalidValue;
  const long long n8 = n_elems / 8;
  hipLaunchKernelGGL(ste_combine_kernel, dim3(grid_for(n8)), dim3(256), 0, stream,
                     (const uint16_t*)dgrad, (const uint32_t*)mask, (const uint16_t*)dres,
                     (uint16_t*)dx, n8);
  ZK_CHECK_LAUNCH();
  return 0;
}
