// BatchNorm (+ReLU) on bf16 NHWC activations and NHWC pooling, gfx950.
//
// Used for the float parts of the binary networks (stem, downsample
// shortcuts, transitions) and for the float ResNet: everything here is
// HBM-bound, 16 B per thread per access, channel-group-per-thread layout so
// per-channel coefficients stay in registers.
//
//   bn_stats_bf16     sum x, sum x^2 per channel (fp32 per thread, fp64 atomics)
//   bn_finalize_f64   scale/shift/mean/rstd + running statistics (Keras momentum)
//   bn_apply_bf16     y = scale*x + shift (+ReLU)
//   bn_bwd_reduce_bf16  sum g', sum g'*xhat   (g' = g * 1{y>0} when ReLU fused)
//   bn_bwd_dx_bf16    dx = k1*g' - k2 - k3*(x - mean)
//   maxpool_fwd/bwd   k x k / stride, TF 'same' (-inf) padding, argmax tap saved
//   avgpool2_fwd/bwd  2x2 / 2 'valid'
#include "../common.h"

namespace {

__device__ __forceinline__ void load8_bf16(const uint16_t* p, float (&v)[8]) {
  const uint4 q = *reinterpret_cast<const uint4*>(p);
  const uint32_t u[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[2 * k] = zk::bf16_to_f32((uint16_t)(u[k] & 0xffff));
    v[2 * k + 1] = zk::bf16_to_f32((uint16_t)(u[k] >> 16));
  }
}

__device__ __forceinline__ void unpack8_bf16(const uint4& q, float (&v)[8]) {
  const uint32_t u[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[2 * k] = zk::bf16_to_f32((uint16_t)(u[k] & 0xffff));
    v[2 * k + 1] = zk::bf16_to_f32((uint16_t)(u[k] >> 16));
  }
}

__device__ __forceinline__ void store8_bf16(uint16_t* p, const float (&v)[8]) {
  *reinterpret_cast<uint4*>(p) =
      make_uint4(zk::pack_bf16x2(v[0], v[1]), zk::pack_bf16x2(v[2], v[3]),
                 zk::pack_bf16x2(v[4], v[5]), zk::pack_bf16x2(v[6], v[7]));
}

// PARTS: per-block partial sums [block][2][C] with plain stores (summed in a
// fixed order by bn_finalize_f64_kernel: run-to-run deterministic) instead of
// fp64 atomics into one [2][C] row.
template <int CG, bool PARTS = false>
__global__ __launch_bounds__(256) void bn_stats_bf16_kernel(const uint16_t* __restrict__ x,
                                                            double* __restrict__ sums,
                                                            long long P) {
  constexpr int C = CG * 8;
  constexpr int RB = 256 / CG;
  const int cg = threadIdx.x % CG;
  float s1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  constexpr int UR = 4;  // rows in flight per thread (loads first, then math)
  const long long rstep = (long long)gridDim.x * RB;
  for (long long r = (long long)blockIdx.x * RB + threadIdx.x / CG; r < P; r += UR * rstep) {
    uint4 q[UR];
#pragma unroll
    for (int u = 0; u < UR; ++u) {
      const long long ru = r + u * rstep;
      q[u] = ru < P ? *reinterpret_cast<const uint4*>(x + ru * C + cg * 8)
                    : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < UR; ++u) {
      const uint32_t w4[4] = {q[u].x, q[u].y, q[u].z, q[u].w};
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float v = zk::bf16_to_f32((uint16_t)(w4[k >> 1] >> (16 * (k & 1))));
        s1[k] += v;
        s2[k] += v * v;
      }
    }
  }
  __shared__ float red[2][256][9];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    red[0][threadIdx.x][k] = s1[k];
    red[1][threadIdx.x][k] = s2[k];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    double a = 0, b = 0;
    for (int rr = 0; rr < RB; ++rr) {
      a += red[0][rr * CG + c / 8][c % 8];
      b += red[1][rr * CG + c / 8][c % 8];
    }
    if (PARTS) {
      sums[(2LL * blockIdx.x) * C + c] = a;
      sums[(2LL * blockIdx.x + 1) * C + c] = b;
    } else {
      atomicAdd(sums + c, a);
      atomicAdd(sums + C + c, b);
    }
  }
}

// sums: [nparts][2][C] (nparts = 1: the atomically accumulated row, re-zeroed
// here for the next use; > 1: per-block partials summed in a fixed order).
// A group of 32 lanes owns one channel: lane k sums parts k, k + 32, ... and
// the group reduces with cross-lane shuffles (one thread per channel walking
// all parts ran ~12 us per call at nparts = 512, 52 calls per ResNet-50 step,
// profiles/r6/bn_grid.md).
__global__ __launch_bounds__(256) void bn_finalize_f64_kernel(
    double* __restrict__ sums, int C, double P, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, float momentum, float* __restrict__ rmean,
    float* __restrict__ rvar, float* __restrict__ coef, int nparts, int rezero) {
  const int k = threadIdx.x & 31;
  const int c = blockIdx.x * 8 + (threadIdx.x >> 5);
  if (c >= C) return;  // uniform over the 32-lane group
  const bool zero = nparts == 1 || rezero;  // re-zeroed for the next use (persistent buffer)
  double s1 = 0.0, s2 = 0.0;
  for (int j = k; j < nparts; j += 32) {
    s1 += sums[(2LL * j) * C + c];
    s2 += sums[(2LL * j + 1) * C + c];
    if (zero) {
      sums[(2LL * j) * C + c] = 0.0;
      sums[(2LL * j + 1) * C + c] = 0.0;
    }
  }
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) {
    s1 += __shfl_xor(s1, o, 32);
    s2 += __shfl_xor(s2, o, 32);
  }
  if (k != 0) return;
  const double mean = s1 / P;
  double var = s2 / P - mean * mean;
  if (var < 0) var = 0;
  const float rstd = (float)(1.0 / sqrt(var + (double)eps));
  const float g = gamma ? gamma[c] : 1.f;
  const float b = beta ? beta[c] : 0.f;
  coef[c] = g * rstd;                          // scale
  coef[C + c] = b - (float)mean * g * rstd;    // shift
  coef[2 * C + c] = (float)mean;
  coef[3 * C + c] = rstd;
  if (rmean) {
    const double unbiased = P > 1 ? var * P / (P - 1) : var;
    rmean[c] = momentum * rmean[c] + (1.f - momentum) * (float)mean;
    rvar[c] = momentum * rvar[c] + (1.f - momentum) * (float)unbiased;
  }
}

// BN pre-activation sc * x + sh + r: one expression shared by the forward
// apply and the backward kernels that recompute the ReLU mask from x (same
// contraction, so the recomputed bf16 output, and its sign, are bit-identical
// to the stored one).
__device__ __forceinline__ float bn_pre(float sc, float x, float sh, float r) {
  return sc * x + sh + r;
}

// ReLU mask of the stored output bf16(max(v, 0)) from v: bf16(v) > 0.
__device__ __forceinline__ bool relu_live(float v) {
  return (int16_t)zk::f32_to_bf16(v) > 0;
}

template <int CG>
__global__ __launch_bounds__(256) void bn_apply_bf16_kernel(const uint16_t* __restrict__ x,
                                                            const float* __restrict__ coef,
                                                            uint16_t* __restrict__ y, long long P,
                                                            int relu,
                                                            uint16_t* __restrict__ sx = nullptr,
                                                            uint8_t* __restrict__ smask = nullptr,
                                                            float clip = 1.f,
                                                            uint32_t* __restrict__ sx4 = nullptr,
                                                            const uint16_t* __restrict__ res = nullptr,
                                                            uint8_t* __restrict__ omask = nullptr) {
  constexpr int C = CG * 8;
  constexpr int RB = 256 / CG;
  const int cg = threadIdx.x % CG;
  float sc[8], sh[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    sc[k] = coef[cg * 8 + k];
    sh[k] = coef[C + cg * 8 + k];
  }
  for (long long r = (long long)blockIdx.x * RB + threadIdx.x / CG; r < P;
       r += (long long)gridDim.x * RB) {
    float v[8];
    load8_bf16(x + r * C + cg * 8, v);
    float rv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (res) load8_bf16(res + r * C + cg * 8, rv);  // residual added before the ReLU
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      v[k] = bn_pre(sc[k], v[k], sh[k], rv[k]);
      if (relu) v[k] = fmaxf(v[k], 0.f);
    }
    const uint32_t ow[4] = {zk::pack_bf16x2(v[0], v[1]), zk::pack_bf16x2(v[2], v[3]),
                            zk::pack_bf16x2(v[4], v[5]), zk::pack_bf16x2(v[6], v[7])};
    *reinterpret_cast<uint4*>(y + r * C + cg * 8) = make_uint4(ow[0], ow[1], ow[2], ow[3]);
    if (omask) {
      // the ReLU mask of the stored output (bit k: y[8 cg + k] > 0), the
      // backward's instead of re-reading y: 1 bit per element, not 16
      uint32_t mk = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        mk |= (uint32_t)((int16_t)(ow[k] & 0xffff) > 0) << (2 * k);
        mk |= (uint32_t)((int16_t)(ow[k] >> 16) > 0) << (2 * k + 1);
      }
      omask[r * CG + cg] = (uint8_t)mk;
    }
    if (sx || sx4) {
      // next binary layer's input quantisation from the stored bf16 values
      // (same layout as batchnorm.hip's bn_apply_kernel / zk_sign_pack)
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
      if (sx)
        *reinterpret_cast<uint4*>(sx + r * C + cg * 8) = make_uint4(sw[0], sw[1], sw[2], sw[3]);
      if (smask) smask[r * CG + cg] = (uint8_t)mk;
      if (sx4) sx4[r * CG + cg] = n4;
    }
  }
}

constexpr int kBnBwdParts = 512;  // copy capacity of the PARTS reduce (red_grid <= it)

// PARTS: per-block partial sums with plain stores, channel-major [2][C][512]
// (summed in a fixed order by zk_bn_bwd_coef with stripes = blocks, stride =
// 512: run-to-run deterministic) instead of fp32 atomics into one [2][C] row.
// RC: BN + ReLU without a stored output: the ReLU mask is recomputed from x
// and the forward coefficients (relu_live(bn_pre(...))), saving a read of y.
// m (otherwise): the ReLU mask bits of the output (bn_apply's omask: a
// residual was added before the ReLU, so x alone does not give it), or null.
template <int CG, bool PARTS = false, bool RC = false>
__global__ __launch_bounds__(256) void bn_bwd_reduce_bf16_kernel(
    const uint16_t* __restrict__ g, const uint16_t* __restrict__ x,
    const uint8_t* __restrict__ m, const float* __restrict__ coef, float* __restrict__ sums,
    long long P) {
  constexpr int C = CG * 8;
  constexpr int RB = 256 / CG;
  const int cg = threadIdx.x % CG;
  float mu[8], rs[8], sg[8], sgx[8], fa[8], fs[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    mu[k] = coef[2 * C + cg * 8 + k];
    rs[k] = coef[3 * C + cg * 8 + k];
    fa[k] = RC ? coef[cg * 8 + k] : 0.f;
    fs[k] = RC ? coef[C + cg * 8 + k] : 0.f;
    sg[k] = sgx[k] = 0.f;
  }
  constexpr int UR = 4;  // rows in flight per thread (loads first, then math)
  const long long rstep = (long long)gridDim.x * RB;
  for (long long r = (long long)blockIdx.x * RB + threadIdx.x / CG; r < P; r += UR * rstep) {
    uint4 gq[UR], xq[UR];
    uint32_t mq[UR];
#pragma unroll
    for (int u = 0; u < UR; ++u) {
      const long long ru = r + u * rstep;
      const bool in = ru < P;
      const long long off = ru * C + cg * 8;
      gq[u] = in ? *reinterpret_cast<const uint4*>(g + off) : make_uint4(0, 0, 0, 0);
      xq[u] = in ? *reinterpret_cast<const uint4*>(x + off) : make_uint4(0, 0, 0, 0);
      // fused ReLU: gradient only where the output was positive
      mq[u] = (!RC && in && m) ? m[ru * CG + cg] : 0xFFu;
    }
#pragma unroll
    for (int u = 0; u < UR; ++u) {
      const uint32_t g4[4] = {gq[u].x, gq[u].y, gq[u].z, gq[u].w};
      const uint32_t x4[4] = {xq[u].x, xq[u].y, xq[u].z, xq[u].w};
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int sh = 16 * (k & 1);
        float gk = zk::bf16_to_f32((uint16_t)(g4[k >> 1] >> sh));
        const float xk = zk::bf16_to_f32((uint16_t)(x4[k >> 1] >> sh));
        if (RC) {
          if (!relu_live(bn_pre(fa[k], xk, fs[k], 0.f))) gk = 0.f;
        } else if (!((mq[u] >> k) & 1u)) {
          gk = 0.f;
        }
        sg[k] += gk;
        sgx[k] += gk * (xk - mu[k]) * rs[k];
      }
    }
  }
  __shared__ float red[2][256][9];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    red[0][threadIdx.x][k] = sg[k];
    red[1][threadIdx.x][k] = sgx[k];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float a = 0.f, b = 0.f;
    for (int rr = 0; rr < RB; ++rr) {
      a += red[0][rr * CG + c / 8][c % 8];
      b += red[1][rr * CG + c / 8][c % 8];
    }
    if (PARTS) {  // channel-major copies [2][C][kBnBwdParts] (zk_bn_bwd_coef)
      sums[(long long)c * kBnBwdParts + blockIdx.x] = a;
      sums[(long long)(C + c) * kBnBwdParts + blockIdx.x] = b;
    } else {
      atomicAdd(sums + c, a);
      atomicAdd(sums + C + c, b);
    }
  }
}

// bcoef: [k1, k0, k3] x C with dx = k1*g' + k0 - k3*x
// fcoef (forward coefficients, scale / shift rows): BN + ReLU with the mask
// recomputed from x instead of read from y (see bn_bwd_reduce_bf16_kernel).
// m: the output's ReLU mask bits (see bn_bwd_reduce_bf16_kernel), or null.
template <int CG>
__global__ __launch_bounds__(256) void bn_bwd_dx_bf16_kernel(
    const uint16_t* __restrict__ g, const uint16_t* __restrict__ x,
    const uint8_t* __restrict__ m, const float* __restrict__ bcoef, uint16_t* __restrict__ dx,
    long long P, uint16_t* __restrict__ dres = nullptr, const float* __restrict__ fcoef = nullptr) {
  constexpr int C = CG * 8;
  constexpr int RB = 256 / CG;
  const int cg = threadIdx.x % CG;
  float k1[8], k0[8], k3[8], fa[8], fs[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    k1[k] = bcoef[cg * 8 + k];
    k0[k] = bcoef[C + cg * 8 + k];
    k3[k] = bcoef[2 * C + cg * 8 + k];
    fa[k] = fcoef ? fcoef[cg * 8 + k] : 0.f;
    fs[k] = fcoef ? fcoef[C + cg * 8 + k] : 0.f;
  }
  for (long long r = (long long)blockIdx.x * RB + threadIdx.x / CG; r < P;
       r += (long long)gridDim.x * RB) {
    float gv[8], xv[8], o[8];
    load8_bf16(g + r * C + cg * 8, gv);
    load8_bf16(x + r * C + cg * 8, xv);
    if (m) {
      const uint32_t b = m[r * CG + cg];
#pragma unroll
      for (int k = 0; k < 8; ++k) gv[k] = (b >> k) & 1u ? gv[k] : 0.f;
    } else if (fcoef) {
#pragma unroll
      for (int k = 0; k < 8; ++k)
        gv[k] = relu_live(bn_pre(fa[k], xv[k], fs[k], 0.f)) ? gv[k] : 0.f;
    }
    // gradient of a residual added before the ReLU: the masked output gradient
    if (dres) store8_bf16(dres + r * C + cg * 8, gv);
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = k1[k] * gv[k] + k0[k] - k3[k] * xv[k];
    store8_bf16(dx + r * C + cg * 8, o);
  }
}

// ---------------------------------------------------------------------------
// Max pooling (NHWC bf16), window k, stride s, TF padding (pt, pl) with -inf.
// One thread = 8 channels of one output pixel; argmax tap (uint8) saved.
// relu: relu(max(window)) == max(0, window) -- the running max starts at 0
// with the tap sentinel 255 (k*k <= 255 taps never reach it), so an output
// clipped to 0 passes no gradient, as ReLU's backward (x <= 0 -> 0) does.
// ---------------------------------------------------------------------------
// KT > 0: the window size at compile time -- every tap of the window is
// loaded before the first comparison (a runtime-k loop issued one 16-B load
// per comparison and waited on it); the comparisons keep the (dh, dw) order,
// so the argmax taps are the same.  KT = 0: k at run time.
template <int KT>
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const uint16_t* __restrict__ x,
                                                          uint16_t* __restrict__ y,
                                                          uint8_t* __restrict__ arg, int B,
                                                          int H, int W, int C, int Ho, int Wo,
                                                          int k_rt, int s, int pt, int pl,
                                                          int relu) {
  const int k = KT > 0 ? KT : k_rt;
  const int CG = C / 8;
  const long long total = (long long)B * Ho * Wo * CG;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int cg = (int)(i % CG);
    const long long pix = i / CG;
    const int wo = (int)(pix % Wo);
    const int ho = (int)((pix / Wo) % Ho);
    const int b = (int)(pix / ((long long)Wo * Ho));
    float best[8];
    uint8_t bi[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      best[q] = relu ? 0.f : -INFINITY;
      bi[q] = relu ? 255 : 0;
    }
    auto take = [&](const uint4& raw, int t) {
      float v[8];
      unpack8_bf16(raw, v);
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (v[q] > best[q]) {
          best[q] = v[q];
          bi[q] = (uint8_t)t;
        }
    };
    if constexpr (KT > 0) {
      uint4 tv[KT * KT];
      bool ok[KT * KT];
#pragma unroll
      for (int t = 0; t < KT * KT; ++t) {
        const int hi = ho * s - pt + t / KT, wi = wo * s - pl + t % KT;
        ok[t] = hi >= 0 && hi < H && wi >= 0 && wi < W;
        tv[t] = ok[t] ? *reinterpret_cast<const uint4*>(
                            x + (((long long)b * H + hi) * W + wi) * C + cg * 8)
                      : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int t = 0; t < KT * KT; ++t)
        if (ok[t]) take(tv[t], t);
    } else {
      for (int dh = 0; dh < k; ++dh) {
        const int hi = ho * s - pt + dh;
        if (hi < 0 || hi >= H) continue;
        for (int dw = 0; dw < k; ++dw) {
          const int wi = wo * s - pl + dw;
          if (wi < 0 || wi >= W) continue;
          take(*reinterpret_cast<const uint4*>(x + (((long long)b * H + hi) * W + wi) * C +
                                               cg * 8),
               dh * k + dw);
        }
      }
    }
    store8_bf16(y + pix * C + cg * 8, best);
    uint2 packed;
    packed.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((uint32_t)bi[3] << 24);
    packed.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((uint32_t)bi[7] << 24);
    *reinterpret_cast<uint2*>(arg + pix * C + cg * 8) = packed;
  }
}

// Gather form (deterministic, no atomics): each input pixel sums the
// gradients of the output windows whose argmax it was.
// KT, ST > 0: window and stride at compile time -- the (at most
// ceil(k/s)^2) candidate outputs' dy / argmax chunks are all loaded before the
// first is added, in the same (ho, wo) order as the runtime loops, so the sums
// are bit-identical.  KT = 0: k and s at run time.
template <int KT, int ST>
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const uint16_t* __restrict__ dy,
                                                          const uint8_t* __restrict__ arg,
                                                          uint16_t* __restrict__ dx, int B,
                                                          int H, int W, int C, int Ho, int Wo,
                                                          int k_rt, int s_rt, int pt, int pl) {
  const int k = KT > 0 ? KT : k_rt, s = KT > 0 ? ST : s_rt;
  const int CG = C / 8;
  const long long total = (long long)B * H * W * CG;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int cg = (int)(i % CG);
    const long long pix = i / CG;
    const int wi = (int)(pix % W);
    const int hi = (int)((pix / W) % H);
    const int b = (int)(pix / ((long long)W * H));
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // outputs whose window covers (hi, wi): ho*s - pt <= hi <= ho*s - pt + k - 1
    const int ho_lo = max(0, (hi + pt - k + s) / s), ho_hi = min(Ho - 1, (hi + pt) / s);
    const int wo_lo = max(0, (wi + pl - k + s) / s), wo_hi = min(Wo - 1, (wi + pl) / s);
    auto add = [&](const uint4& gq, const uint2& a, int tap) {
      const uint8_t* ab = reinterpret_cast<const uint8_t*>(&a);
      float g[8];
      unpack8_bf16(gq, g);
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (ab[q] == (uint8_t)tap) acc[q] += g[q];
    };
    if constexpr (KT > 0) {
      constexpr int N = (KT + ST - 1) / ST;  // candidates per dimension
      uint4 gq[N * N];
      uint2 aq[N * N];
      int tap[N * N];
#pragma unroll
      for (int t = 0; t < N * N; ++t) {
        const int ho = ho_lo + t / N, wo = wo_lo + t % N;
        const int dh = hi - (ho * ST - pt), dw = wi - (wo * ST - pl);
        const bool ok = ho <= ho_hi && wo <= wo_hi && dh >= 0 && dh < KT && dw >= 0 && dw < KT;
        tap[t] = ok ? dh * KT + dw : -1;
        const long long o = (((long long)b * Ho + ho) * Wo + wo) * C + cg * 8;
        gq[t] = ok ? *reinterpret_cast<const uint4*>(dy + o) : make_uint4(0, 0, 0, 0);
        aq[t] = ok ? *reinterpret_cast<const uint2*>(arg + o) : make_uint2(0, 0);
      }
#pragma unroll
      for (int t = 0; t < N * N; ++t)
        if (tap[t] >= 0) add(gq[t], aq[t], tap[t]);
    } else {
      for (int ho = ho_lo; ho <= ho_hi; ++ho) {
        const int dh = hi - (ho * s - pt);
        if (dh < 0 || dh >= k) continue;
        for (int wo = wo_lo; wo <= wo_hi; ++wo) {
          const int dw = wi - (wo * s - pl);
          if (dw < 0 || dw >= k) continue;
          const long long o = (((long long)b * Ho + ho) * Wo + wo) * C + cg * 8;
          add(*reinterpret_cast<const uint4*>(dy + o), *reinterpret_cast<const uint2*>(arg + o),
              dh * k + dw);
        }
      }
    }
    store8_bf16(dx + pix * C + cg * 8, acc);
  }
}

// 2x2 / stride 2 'valid' average pooling.
__global__ __launch_bounds__(256) void avgpool2_fwd_kernel(const uint16_t* __restrict__ x,
                                                           uint16_t* __restrict__ y, int B,
                                                           int H, int W, int C, int Ho, int Wo) {
  const int CG = C / 8;
  const long long total = (long long)B * Ho * Wo * CG;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int cg = (int)(i % CG);
    const long long pix = i / CG;
    const int wo = (int)(pix % Wo);
    const int ho = (int)((pix / Wo) % Ho);
    const int b = (int)(pix / ((long long)Wo * Ho));
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      float v[8];
      load8_bf16(x + (((long long)b * H + 2 * ho + (d >> 1)) * W + 2 * wo + (d & 1)) * C + cg * 8,
                 v);
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += v[q];
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] *= 0.25f;
    store8_bf16(y + pix * C + cg * 8, acc);
  }
}

// add (optional, [B][H][W][C]): x's other gradient (a residual block's main
// path, ops.binary_block's hand-off) summed in the same pass.
__global__ __launch_bounds__(256) void avgpool2_bwd_kernel(const uint16_t* __restrict__ dy,
                                                           uint16_t* __restrict__ dx, int B,
                                                           int H, int W, int C, int Ho, int Wo,
                                                           const uint16_t* __restrict__ add) {
  const int CG = C / 8;
  const long long total = (long long)B * H * W * CG;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int cg = (int)(i % CG);
    const long long pix = i / CG;
    const int wi = (int)(pix % W);
    const int hi = (int)((pix / W) % H);
    const int b = (int)(pix / ((long long)W * H));
    float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if ((hi >> 1) < Ho && (wi >> 1) < Wo) {
      load8_bf16(dy + (((long long)b * Ho + (hi >> 1)) * Wo + (wi >> 1)) * C + cg * 8, v);
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] *= 0.25f;
    }
    if (add) {
      float a[8];
      load8_bf16(add + pix * C + cg * 8, a);
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] += a[q];
    }
    store8_bf16(dx + pix * C + cg * 8, v);
  }
}

// Per-tile BN-backward partials [tiles][2][C] (a GEMM epilogue's rows,
// zk_igemm_dgrad_bsums) -> the channel-major copies [2][C][kBnBwdParts] that
// zk_bn_bwd_coef sums: copy b = rows b, b + kBnBwdParts, ... in that order
// (fixed: bit-reproducible), each row read once and re-zeroed.  A block owns
// TR_C consecutive values of the 2C and TR_B consecutive copies, one (value,
// copy) per thread; a thread's rows are loaded TR_U at a time (independent
// loads) and added in row order.  The block's [TR_C][TR_B] tile goes through
// LDS so that every output row is written as TR_B contiguous floats.  (One
// block per copy with a thread per value wrote each float 2 KB from its
// neighbour: ~21 us per call at ResNet-50 shapes, profiles/r6/bn_grid.md.)
constexpr int TR_C = 16, TR_B = 16, TR_U = 8;
__global__ __launch_bounds__(256) void bn_bwd_tiles_reduce_kernel(float* __restrict__ rows,
                                                                  int tiles, int C,
                                                                  float* __restrict__ out) {
  __shared__ float tile[TR_C][TR_B + 1];
  const int c0 = blockIdx.x * TR_C, b0 = blockIdx.y * TR_B;
  const int cl = threadIdx.x % TR_C, bl = threadIdx.x / TR_C;
  const int c = c0 + cl, b = b0 + bl;
  float t = 0.f;
  if (c < 2 * C) {
    for (int r = b; r < tiles; r += TR_U * kBnBwdParts) {
      float v[TR_U];
#pragma unroll
      for (int u = 0; u < TR_U; ++u) {
        const int ru = r + u * kBnBwdParts;
        v[u] = ru < tiles ? rows[(long long)ru * 2 * C + c] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < TR_U; ++u) {
        const int ru = r + u * kBnBwdParts;
        if (ru < tiles) {
          t += v[u];
          rows[(long long)ru * 2 * C + c] = 0.f;
        }
      }
    }
  }
  tile[cl][bl] = t;
  __syncthreads();
  const int cc = threadIdx.x / TR_B, bb = threadIdx.x % TR_B;
  if (c0 + cc < 2 * C) out[(long long)(c0 + cc) * kBnBwdParts + b0 + bb] = tile[cc][bb];
}

int rows_grid(long long P, int C, long long cap = 2048) {
  const long long rb = 256 / (C / 8);
  long long b = (P + rb - 1) / rb;
  if (b > cap) b = cap;
  return b < 1 ? 1 : (int)b;
}

// The apply kernels take up to 65536 blocks (a few rows per thread: 5-9 %
// faster at the large ResNet-50 shapes); for the dx kernels larger grids were
// up to 3x slower at every shape with C >= 128 (tools/bn_lab.py,
// profiles/r6/bn_grid.md).
int apply_grid(long long P, int C) { return rows_grid(P, C, 65536); }
// The dx kernels: 1024 blocks with the stored ReLU mask (or none), 512 with
// the mask recomputed from x (RC) -- 10-30 % faster than 2048 at most
// ResNet-50 shapes, and larger grids were slower still (profiles/r6/bn_grid.md).
int dx_grid(long long P, int C) { return rows_grid(P, C, 1024); }
int dx_rc_grid(long long P, int C) { return rows_grid(P, C, 512); }

// reductions: fewer blocks (each with 4 rows in flight per thread) so the
// per-block atomics into the 2*C accumulators do not serialise
int red_grid(long long P, int C) {
  const int b = rows_grid(P, C);
  return b > 512 ? 512 : b;
}

int flat_grid(long long work) {
  long long b = (work + 255) / 256;
  if (b > 16384) b = 16384;
  return b < 1 ? 1 : (int)b;
}

}  // namespace

#define ZK_CG_CASES(C, BODY) \
  switch ((C) / 8) {         \
    BODY(1)                  \
    BODY(2)                  \
    BODY(4)                  \
    BODY(8)                  \
    BODY(16)                 \
    BODY(32)                 \
    BODY(64)                 \
    BODY(128)                \
    BODY(256)                \
    default:                 \
      return (int)hipErrorInvalidValue; \
  }

// sums: [2][C] fp64, zeroed by the caller.
ZK_EXPORT int zk_bn_stats_bf16(const void* x, void* sums, long long P, int C, hipStream_t st) {
  if (C % 8) return (int)hipErrorInvalidValue;
#define CASE(cg)                                                                           \
  case cg:                                                                                 \
    hipLaunchKernelGGL(bn_stats_bf16_kernel<cg>, dim3(red_grid(P, C)), dim3(256), 0, st,   \
                       (const uint16_t*)x, (double*)sums, P);                              \
    break;
  ZK_CG_CASES(C, CASE)
#undef CASE
  ZK_CHECK_LAUNCH();
  return 0;
}

// coef out: [4][C] = scale, shift, mean, rstd
ZK_EXPORT int zk_bn_finalize_f64(const void* sums, int C, double P, const void* gamma,
                                 const void* beta, float eps, float momentum, void* rmean,
                                 void* rvar, void* coef, hipStream_t st) {
  hipLaunchKernelGGL(bn_finalize_f64_kernel, dim3((C + 7) / 8), dim3(256), 0, st,
                     (double*)sums, C, P, (const float*)gamma, (const float*)beta, eps,
                     momentum, (float*)rmean, (float*)rvar, (float*)coef, 1, 0);
  ZK_CHECK_LAUNCH();
  return 0;
}

// Deterministic forms (the Runtime's deterministic mode): per-block partials
// [zk_bn_bwd_parts_max()][2][C] fp64 with plain stores, summed in block order
// by zk_bn_finalize_f64_parts.
ZK_EXPORT int zk_bn_stats_bf16_parts(const void* x, void* parts, long long P, int C,
                                     int* nparts, hipStream_t st) {
  if (C % 8) return (int)hipErrorInvalidValue;
  const int grid = red_grid(P, C);
  if (nparts) *nparts = grid;
#define CASE(cg)                                                                           \
  case cg:                                                                                 \
    hipLaunchKernelGGL((bn_stats_bf16_kernel<cg, true>), dim3(grid), dim3(256), 0, st,     \
                       (const uint16_t*)x, (double*)parts, P);                             \
    break;
  ZK_CG_CASES(C, CASE)
#undef CASE
  ZK_CHECK_LAUNCH();
  return 0;
}

ZK_EXPORT int zk_bn_finalize_f64_parts(const void* parts, int nparts, int C, double P,
                                       const void* gamma, const void* beta, float eps,
                                       float momentum, void* rmean, void* rvar, void* coef,
                                       hipStream_t st) {
  hipLaunchKernelGGL(bn_finalize_f64_kernel, dim3((C + 7) / 8), dim3(256), 0, st,
                     (double*)parts, C, P, (const float*)gamma, (const float*)beta, eps,
                     momentum, (float*)rmean, (float*)rvar, (float*)coef, nparts < 1 ? 1 : nparts, 0);
  ZK_CHECK_LAUNCH();
  return 0;
}

// zk_bn_finalize_f64_parts over striped accumulators that are re-zeroed after
// reading (the persistent [stripes][2][C] buffer the float forward GEMM's
// epilogue adds its statistics into: zk_igemm_dgrad_fstats).
ZK_EXPORT int zk_bn_finalize_f64_stripes(void* parts, int nparts, int C, double P,
                                         const void* gamma, const void* beta, float eps,
                                         float momentum, void* rmean, void* rvar, void* coef,
                                         hipStream_t st) {
  hipLaunchKernelGGL(bn_finalize_f64_kernel, dim3((C + 7) / 8), dim3(256), 0, st,
                     (double*)parts, C, P, (const float*)gamma, (const float*)beta, eps,
                     momentum, (float*)rmean, (float*)rvar, (float*)coef, nparts < 1 ? 1 : nparts,
                     1);
  ZK_CHECK_LAUNCH();
  return 0;
}

ZK_EXPORT int zk_bn_bwd_reduce_relu_bf16_parts(const void* g, const void* x, const void* coef,
                                               void* parts, long long P, int C, int* nparts,
                                               hipStream_t st) {
  if (C % 8) return (int)hipErrorInvalidValue;
  const int grid = red_grid(P, C);
  if (nparts) *nparts = grid;
#define CASE(cg)                                                                         \
  case cg:                                                                               \
    hipLaunchKernelGGL((bn_bwd_reduce_bf16_kernel<cg, true, true>), dim3(grid), dim3(256), \
                       0, st, (const uint16_t*)g, (const uint16_t*)x, nullptr,           \
                       (const float*)coef, (float*)parts, P);                            \
    break;
  ZK_CG_CASES(C, CASE)
#undef CASE
  ZK_CHECK_LAUNCH();
  return 0;
}

ZK_EXPORT int zk_bn_apply_bf16(const void* x, const void* coef, void* y, long long P, int C,
                               int relu, hipStream_t st) {
  if (C % 8) return (int)hipErrorInvalidValue;
#define CASE(cg)                                                                           \
  case cg:                                                                                 \
    hipLaunchKernelGGL(bn_apply_bf16_kernel<cg>, dim3(apply_grid(P, C)), dim3(256), 0, st,  \
                       (const uint16_t*)x, (const float*)coef, (uint16_t*)y, P, relu);     \
    break;
  ZK_CG_CASES(C, CASE)
#undef CASE
  ZK_CHECK_LAUNCH();
  return 0;
}

// zk_bn_apply_bf16 + the next binary layer's sign image (bf16 +-1) and STE
// mask bits (|y| <= clip), packed like zk_sign_pack's.
ZK_EXPORT int zk_bn_apply_bf16_sign(const void* x, const void* coef, void* y, void* sx,
                                    void* mask, void* sx4, float clip, long long P, int C,
                                    int relu, hipStream_t st) {
  if (C % 32) return (int)hipErrorInvalidValue;
#define CASE(cg)                                                                           \
  case cg:                                                                                 \
    hipLaunchKernelGGL(bn_apply_bf16_kernel<cg>, dim3(apply_grid(P, C)), dim3(256), 0, st,  \
                       (const uint16_t*)x, (const float*)coef, (uint16_t*)y, P, relu,      \
                       (uint16_t*)sx, (uint8_t*)mask, clip, (uint32_t*)sx4);               \
    break;
  ZK_CG_CASES(C, CASE)
#undef CASE
  ZK_CHECK_LAUNCH();
  return 0;
}

// m: the output's ReLU mask bits (zk_bn_apply_res_bf16's omask), or null.
ZK_EXPORT int zk_bn_bwd_reduce_bf16(const void* g, const void* x, const void* m,
                                    const void* coef, void* sums, long long P, int C,
                                    hipStream_t st) {
  if (C % 8) return (int)hipErrorInvalidValue;
#define CASE(cg)                                                                              \
  case cg:                                                                                    \
    hipLaunchKernelGGL(bn_bwd_reduce_bf16_kernel<cg>, dim3(red_grid(P, C)), dim3(256), 0, st, \
                       (const uint16_t*)g, (const uint16_t*)x, (const uint8_t*)m,             \
                       (const float*)coef, (float*)sums, P);                                  \
    break;
  ZK_CG_CASES(C, CASE)
#undef CASE
  ZK_CHECK_LAUNCH();
  return 0;
}

// Deterministic form: parts [2][C][zk_bn_bwd_parts_max()] (channel-major)
// receives one copy per block (*nparts of them); pass parts, *nparts and
// zk_bn_bwd_parts_max() as sums / stripes / stride to zk_bn_bwd_coef.
ZK_EXPORT int zk_bn_bwd_parts_max() { return kBnBwdParts; }

// rows [tiles][2][C] (re-zeroed) -> parts [2][C][zk_bn_bwd_parts_max()]: every
// copy written; pass parts, zk_bn_bwd_parts_max() (stripes and stride) to
// zk_bn_bwd_coef.
ZK_EXPORT int zk_bn_bwd_tiles_reduce(void* rows, int tiles, int C, void* parts, hipStream_t st) {
  if (tiles < 1 || C < 1) return (int)hipErrorInvalidValue;
  static_assert(kBnBwdParts % TR_B == 0, "copies tile by TR_B");
  hipLaunchKernelGGL(bn_bwd_tiles_reduce_kernel, dim3((2 * C + TR_C - 1) / TR_C, kBnBwdParts / TR_B),
                     dim3(256), 0, st, (float*)rows, tiles, C, (float*)parts);
  ZK_CHECK_LAUNCH();
  return 0;
}

ZK_EXPORT int zk_bn_bwd_reduce_bf16_parts(const void* g, const void* x, const void* m,
                                          const void* coef, void* parts, long long P, int C,
                                          int* nparts, hipStream_t st) {
  if (C % 8) return (int)hipErrorInvalidValue;
  const int grid = red_grid(P, C);
  if (nparts) *nparts = grid;
#define CASE(cg)                                                                           \
  case cg:                                                                                 \
    hipLaunchKernelGGL((bn_bwd_reduce_bf16_kernel<cg, true>), dim3(grid), dim3(256), 0, st, \
                       (const uint16_t*)g, (const uint16_t*)x, (const uint8_t*)m,          \
                       (const float*)coef, (float*)parts, P);                              \
    break;
  ZK_CG_CASES(C, CASE)
#undef CASE
  ZK_CHECK_LAUNCH();
  return 0;
}

ZK_EXPORT int zk_bn_bwd_dx_bf16(const void* g, const void* x, const void* m, const void* bcoef,
                                void* dx, long long P, int C, hipStream_t st) {
  if (C % 8) return (int)hipErrorInvalidValue;
#define CASE(cg)                                                                             \
  case cg:                                                                                   \
    hipLaunchKernelGGL(bn_bwd_dx_bf16_kernel<cg>, dim3(dx_grid(P, C)), dim3(256), 0, st,     \
                       (const uint16_t*)g, (const uint16_t*)x, (const uint8_t*)m,            \
                       (const float*)bcoef, (uint16_t*)dx, P);                               \
    break;
  ZK_CG_CASES(C, CASE)
#undef CASE
  ZK_CHECK_LAUNCH();
  return 0;
}

// BN + ReLU backward without the stored output: the ReLU mask is recomputed
// from x and the forward coefficients coef [4][C] (scale, shift, mean, rstd).
ZK_EXPORT int zk_bn_bwd_reduce_relu_bf16(const void* g, const void* x, const void* coef,
                                         void* sums, long long P, int C, hipStream_t st) {
  if (C % 8) return (int)hipErrorInvalidValue;
#define CASE(cg)                                                                         \
  case cg:                                                                               \
    hipLaunchKernelGGL((bn_bwd_reduce_bf16_kernel<cg, false, true>), dim3(red_grid(P, C)), \
                       dim3(256), 0, st, (const uint16_t*)g, (const uint16_t*)x, nullptr, \
                       (const float*)coef, (float*)sums, P);                             \
    break;
  ZK_CG_CASES(C, CASE)
#undef CASE
  ZK_CHECK_LAUNCH();
  return 0;
}

ZK_EXPORT int zk_bn_bwd_dx_relu_bf16(const void* g, const void* x, const void* coef,
                                     const void* bcoef, void* dx, long long P, int C,
                                     hipStream_t st) {
  if (C % 8) return (int)hipErrorInvalidValue;
#define CASE(cg)                                                                             \
  case cg:                                                                                   \
    hipLaunchKernelGGL(bn_bwd_dx_bf16_kernel<cg>, dim3(dx_rc_grid(P, C)), dim3(256), 0, st,  \
                       (const uint16_t*)g, (const uint16_t*)x, nullptr, (const float*)bcoef, \
                       (uint16_t*)dx, P, nullptr, (const float*)coef);                       \
    break;
  ZK_CG_CASES(C, CASE)
#undef CASE
  ZK_CHECK_LAUNCH();
  return 0;
}

// y = act(scale * x + shift + res): BN apply with a residual added before
// the optional ReLU (a ResNet bottleneck's tail: relu(bn3(conv3) + shortcut)).
// omask (optional): the ReLU mask bits of y, [P][C/8] bytes, for the backward.
ZK_EXPORT int zk_bn_apply_res_bf16(const void* x, const void* coef, const void* res, void* y,
                                   void* omask, long long P, int C, int relu, hipStream_t st) {
  if (C % 8) return (int)hipErrorInvalidValue;
#define CASE(cg)                                                                           \
  case cg:                                                                                 \
    hipLaunchKernelGGL(bn_apply_bf16_kernel<cg>, dim3(apply_grid(P, C)), dim3(256), 0, st,  \
                       (const uint16_t*)x, (const float*)coef, (uint16_t*)y, P, relu,      \
                       nullptr, nullptr, 1.f, nullptr, (const uint16_t*)res,               \
                       (uint8_t*)omask);                                                   \
    break;
  ZK_CG_CASES(C, CASE)
#undef CASE
  ZK_CHECK_LAUNCH();
  return 0;
}

// zk_bn_bwd_dx_bf16 + the residual's gradient (the ReLU-masked output
// gradient) written to dres in the same pass; m: the ReLU mask bits or null.
ZK_EXPORT int zk_bn_bwd_dx_res_bf16(const void* g, const void* x, const void* m,
                                    const void* bcoef, void* dx, void* dres, long long P, int C,
                                    hipStream_t st) {
  if (C % 8) return (int)hipErrorInvalidValue;
#define CASE(cg)                                                                             \
  case cg:                                                                                   \
    hipLaunchKernelGGL(bn_bwd_dx_bf16_kernel<cg>, dim3(dx_grid(P, C)), dim3(256), 0, st,     \
                       (const uint16_t*)g, (const uint16_t*)x, (const uint8_t*)m,            \
                       (const float*)bcoef, (uint16_t*)dx, P, (uint16_t*)dres);              \
    break;
  ZK_CG_CASES(C, CASE)
#undef CASE
  ZK_CHECK_LAUNCH();
  return 0;
}

// relu != 0: y = relu(maxpool(x)) in the same pass (QuickNet transitions).
ZK_EXPORT int zk_maxpool_fwd(const void* x, void* y, void* arg, int B, int H, int W, int C,
                             int Ho, int Wo, int k, int s, int pt, int pl, int relu,
                             hipStream_t st) {
  if (C % 8 || k * k > 255) return (int)hipErrorInvalidValue;
  const long long work = (long long)B * Ho * Wo * (C / 8);
  // window size at compile time for the shipped models' pools (QuickNet 2x2,
  // ResNet 3x3): 8-10 % faster at batch 1024, profiles/r6/maxpool.md
  auto kern = k == 2 ? maxpool_fwd_kernel<2> : k == 3 ? maxpool_fwd_kernel<3>
                                                      : maxpool_fwd_kernel<0>;
  hipLaunchKernelGGL(kern, dim3(flat_grid(work)), dim3(256), 0, st, (const uint16_t*)x,
                     (uint16_t*)y, (uint8_t*)arg, B, H, W, C, Ho, Wo, k, s, pt, pl, relu);
  ZK_CHECK_LAUNCH();
  return 0;
}

ZK_EXPORT int zk_maxpool_bwd(const void* dy, const void* arg, void* dx, int B, int H, int W,
                             int C, int Ho, int Wo, int k, int s, int pt, int pl,
                             hipStream_t st) {
  if (C % 8) return (int)hipErrorInvalidValue;
  const long long work = (long long)B * H * W * (C / 8);
  // QuickNet's 2x2/1 and ResNet's 3x3/2 at compile time: 15-20 % faster at
  // batch 1024 (profiles/r6/maxpool.md)
  auto kern = (k == 2 && s == 1) ? maxpool_bwd_kernel<2, 1>
              : (k == 3 && s == 2) ? maxpool_bwd_kernel<3, 2>
                                   : maxpool_bwd_kernel<0, 0>;
  hipLaunchKernelGGL(kern, dim3(flat_grid(work)), dim3(256), 0, st, (const uint16_t*)dy,
                     (const uint8_t*)arg, (uint16_t*)dx, B, H, W, C, Ho, Wo, k, s, pt, pl);
  ZK_CHECK_LAUNCH();
  return 0;
}

ZK_EXPORT int zk_avgpool2_fwd(const void* x, void* y, int B, int H, int W, int C, int Ho,
                              int Wo, hipStream_t st) {
  if (C % 8) return (int)hipErrorInvalidValue;
  const long long work = (long long)B * Ho * Wo * (C / 8);
  hipLaunchKernelGGL(avgpool2_fwd_kernel, dim3(flat_grid(work)), dim3(256), 0, st,
                     (const uint16_t*)x, (uint16_t*)y, B, H, W, C, Ho, Wo);
  ZK_CHECK_LAUNCH();
  return 0;
}

ZK_EXPORT int zk_avgpool2_bwd(const void* dy, void* dx, int B, int H, int W, int C, int Ho,
                              int Wo, hipStream_t st) {
  if (C % 8) return (int)hipErrorInvalidValue;
  const long long work = (long long)B * H * W * (C / 8);
  hipLaunchKernelGGL(avgpool2_bwd_kernel, dim3(flat_grid(work)), dim3(256), 0, st,
                     (const uint16_t*)dy, (uint16_t*)dx, B, H, W, C, Ho, Wo, nullptr);
  ZK_CHECK_LAUNCH();
  return 0;
}

// zk_avgpool2_bwd + add ([B][H][W][C] bf16, the input's other gradient):
// dx = upsample(dy) / 4 + add, one rounding.
ZK_EXPORT int zk_avgpool2_bwd_add(const void* dy, const void* add, void* dx, int B, int H, int W,
                                  int C, int Ho, int Wo, hipStream_t st) {
  if (C % 8 || !add) return (int)hipErrorInvalidValue;
  const long long work = (long long)B * H * W * (C / 8);
  hipLaunchKernelGGL(avgpool2_bwd_kernel, dim3(flat_grid(work)), dim3(256), 0, st,
                     (const uint16_t*)dy, (uint16_t*)dx, B, H, W, C, Ho, Wo,
                     (const uint16_t*)add);
  ZK_CHECK_LAUNCH();
  return 0;
}
