// Classifier head of the ImageNet models: (ReLU) -> global average pool ->
// dense layer, forward and backward, on native kernels (replaces x.mean +
// F.linear, i.e. a torch reduction and hipBLASLt GEMMs -- the last library
// kernels of the binary ResNet / QuickNet / ResNet-50 steps).
//
//   pooled[b][c] = mean_hw act(x[b][hw][c])              gap_fwd (fp32 out)
//   logits       = pooled . W^T + bias                   sgemm (fp32 MFMA)
//   dW += dlogits^T . pooled, dbias += colsum(dlogits)   sgemm (accumulate, colsum fused)
//   dpooled      = dlogits . W                           sgemm
//   dx[b][hw][c] = act'(x) * dpooled[b][c] / HW          gap_bwd (bf16 out)
//
// The GEMMs keep the reference's fp32 dense layer (Keras Dense in fp32,
// examples/larq_experiment.py:95-101 / the model zoo's float classifier) on
// v_mfma_f32_16x16x4_f32: exact fp32 products (one rounding per product, a
// k-ordered fmaf chain -- cdna_hip_programming.md §3 'FP32-input MFMA'), so
// the numerics match an fp32 library GEMM up to summation order.
#include "../common.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// pooled[b][c] = mean over the HW rows of act(x); x bf16 [B][HW][C], out
// fp32 (head) or bf16 (GlobalAvgPool).  One block per (image, 2048-channel
// slice); a thread owns 8 channels (one 16-B load per row).
template <bool OUT_BF16>
__global__ __launch_bounds__(256) void gap_fwd_kernel(const uint16_t* __restrict__ x,
                                                      void* __restrict__ out, int HW, int C,
                                                      int relu) {
  const int b = blockIdx.x;
  const int c8 = blockIdx.y * 256 + threadIdx.x;  // 8-channel group
  if (c8 * 8 >= C) return;
  const uint16_t* xb = x + (long long)b * HW * C + c8 * 8;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int r = 0; r < HW; ++r) {
    const uint4 v = *reinterpret_cast<const uint4*>(xb + (long long)r * C);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float f = zk::bf16_to_f32((uint16_t)(w[k >> 1] >> (16 * (k & 1))));
      if (relu) f = fmaxf(f, 0.f);
      s[k] += f;
    }
  }
  const float inv = 1.f / (float)HW;
  if (OUT_BF16) {
    uint16_t* o = (uint16_t*)out + (long long)b * C + c8 * 8;
    *reinterpret_cast<uint4*>(o) =
        make_uint4(zk::pack_bf16x2(s[0] * inv, s[1] * inv), zk::pack_bf16x2(s[2] * inv, s[3] * inv),
                   zk::pack_bf16x2(s[4] * inv, s[5] * inv), zk::pack_bf16x2(s[6] * inv, s[7] * inv));
  } else {
    float* o = (float*)out + (long long)b * C + c8 * 8;
    *reinterpret_cast<float4*>(o) = make_float4(s[0] * inv, s[1] * inv, s[2] * inv, s[3] * inv);
    *reinterpret_cast<float4*>(o + 4) = make_float4(s[4] * inv, s[5] * inv, s[6] * inv, s[7] * inv);
  }
}

// dx[b][hw][c] = act'(x) * dp[b][c] / HW (bf16).  Grid-stride over
// (row, 8-channel group) pairs.
__global__ __launch_bounds__(256) void gap_bwd_kernel(const float* __restrict__ dp,
                                                      const uint16_t* __restrict__ x,
                                                      uint16_t* __restrict__ dx, int B, int HW,
                                                      int C, int relu) {
  const long long groups = (long long)B * HW * (C / 8);
  const float inv = 1.f / (float)HW;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < groups;
       i += (long long)gridDim.x * blockDim.x) {
    const long long row = i / (C / 8);
    const int c8 = (int)(i - row * (C / 8));
    const int b = (int)(row / HW);
    const float4 d0 = *reinterpret_cast<const float4*>(dp + (long long)b * C + c8 * 8);
    const float4 d1 = *reinterpret_cast<const float4*>(dp + (long long)b * C + c8 * 8 + 4);
    const float d[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
    uint32_t w[4] = {0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u};
    if (relu) {
      const uint4 v = *reinterpret_cast<const uint4*>(x + row * C + c8 * 8);
      w[0] = v.x;
      w[1] = v.y;
      w[2] = v.z;
      w[3] = v.w;
    }
    float o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float xv = zk::bf16_to_f32((uint16_t)(w[k >> 1] >> (16 * (k & 1))));
      o[k] = (xv > 0.f) ? d[k] * inv : 0.f;
    }
    *reinterpret_cast<uint4*>(dx + row * C + c8 * 8) =
        make_uint4(zk::pack_bf16x2(o[0], o[1]), zk::pack_bf16x2(o[2], o[3]),
                   zk::pack_bf16x2(o[4], o[5]), zk::pack_bf16x2(o[6], o[7]));
  }
}

// C[m][n] (=|+=) sum_k A(m, k) * B(k, n) (+ bias[n]), all fp32 with strides:
// A(m, k) = A[m*sam + k*sak], B(k, n) = B[k*sbk + n*sbn], C row stride scm.
// Either stride of each operand may be the unit one (the head's three GEMMs
// read W, pooled and dlogits both ways).  32x32 tiles so even the 512x1000
// forward launches 512 blocks (2-4 per CU hide the latency a 1-block-per-CU
// grid cannot); K-steps of 32 staged through double-buffered LDS images
// [k][m] / [k][n] (row stride 48 floats: the f32-MFMA fragment reads of the
// two 16-lane k rows of a 32-lane half land in disjoint bank halves), the
// next step's global loads issued before the current step's MFMAs.  Each of
// the 4 waves owns one 16x16 block, two accumulators (even/odd k) to break the
// MFMA dependency chain.  colsum (optional, blocks of the first column tile):
// colsum[m] += sum_k A(m, k) -- the bias gradient rides on the dW GEMM.
constexpr int SG_T = 32, SG_LD = 48;

__device__ __forceinline__ void sg_load(const float* __restrict__ P, long long s_mn,
                                        long long s_k, int mn0, int k0, int MN, int K, int tid,
                                        float (&v)[4], bool& kfast) {
  // one float4 of the 32x32 tile per thread, vectorised along the unit stride
  kfast = (s_k == 1);
  int mn, k;
  if (kfast) {
    mn = tid >> 3;
    k = (tid & 7) * 4;
  } else {
    k = tid >> 3;
    mn = (tid & 7) * 4;
  }
  const int gm = mn0 + mn, gk = k0 + k;
  const long long base = (long long)gm * s_mn + (long long)gk * s_k;
  const bool full = kfast ? (gm < MN && gk + 3 < K) : (gk < K && gm + 3 < MN);
  if (full && ((base & 3) == 0)) {
    const float4 f = *reinterpret_cast<const float4*>(P + base);
    v[0] = f.x;
    v[1] = f.y;
    v[2] = f.z;
    v[3] = f.w;
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m2 = kfast ? gm : gm + i, k2 = kfast ? gk + i : gk;
      v[i] = (m2 < MN && k2 < K) ? P[(long long)m2 * s_mn + (long long)k2 * s_k] : 0.f;
    }
  }
}

__device__ __forceinline__ void sg_store(float* S, const float (&v)[4], bool kfast, int tid) {
  if (kfast) {
    const int mn = tid >> 3, k = (tid & 7) * 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) S[(k + i) * SG_LD + mn] = v[i];
  } else {
    const int k = tid >> 3, mn = (tid & 7) * 4;
    *reinterpret_cast<float4*>(S + k * SG_LD + mn) = make_float4(v[0], v[1], v[2], v[3]);
  }
}

template <bool ACC>
__global__ __launch_bounds__(256) void sgemm_kernel(const float* __restrict__ A, long long sam,
                                                    long long sak, const float* __restrict__ B,
                                                    long long sbk, long long sbn,
                                                    float* __restrict__ C, long long scm, int M,
                                                    int N, int K, const float* __restrict__ bias,
                                                    float* __restrict__ colsum) {
  __shared__ __attribute__((aligned(16))) float As[2][SG_T * SG_LD];
  __shared__ __attribute__((aligned(16))) float Bs[2][SG_T * SG_LD];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.y * SG_T, n0 = blockIdx.x * SG_T;
  const bool do_colsum = colsum != nullptr && blockIdx.x == 0;
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  float cs = 0.f;
  float va[4], vb[4];
  bool ka, kb;
  sg_load(A, sam, sak, m0, 0, M, K, tid, va, ka);
  sg_load(B, sbn, sbk, n0, 0, N, K, tid, vb, kb);
  sg_store(As[0], va, ka, tid);
  sg_store(Bs[0], vb, kb, tid);
  __syncthreads();
  const int nk = (K + SG_T - 1) / SG_T;
  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    const bool more = t + 1 < nk;
    if (more) {
      sg_load(A, sam, sak, m0, (t + 1) * SG_T, M, K, tid, va, ka);
      sg_load(B, sbn, sbk, n0, (t + 1) * SG_T, N, K, tid, vb, kb);
    }
    const float* as = As[cur];
    const float* bs = Bs[cur];
#pragma unroll
    for (int kk = 0; kk < SG_T / 4; kk += 2) {
      const int r0 = kk * 4 + (lane >> 4), r1 = r0 + 4;
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(as[r0 * SG_LD + wm * 16 + (lane & 15)],
                                                  bs[r0 * SG_LD + wn * 16 + (lane & 15)], acc0,
                                                  0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(as[r1 * SG_LD + wm * 16 + (lane & 15)],
                                                  bs[r1 * SG_LD + wn * 16 + (lane & 15)], acc1,
                                                  0, 0, 0);
    }
    if (do_colsum && tid < SG_T) {
#pragma unroll 8
      for (int k = 0; k < SG_T; ++k) cs += as[k * SG_LD + tid];
    }
    if (more) {
      sg_store(As[cur ^ 1], va, ka, tid);
      sg_store(Bs[cur ^ 1], vb, kb, tid);
    }
    __syncthreads();
  }
  if (do_colsum && tid < SG_T && m0 + tid < M) colsum[m0 + tid] += cs;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m = m0 + wm * 16 + 4 * (lane >> 4) + r;
    const int n = n0 + wn * 16 + (lane & 15);
    if (m < M && n < N) {
      float v = acc0[r] + acc1[r];
      if (bias) v += bias[n];
      float* cp = C + (long long)m * scm + n;
      *cp = ACC ? *cp + v : v;
    }
  }
}

int gap_fwd(const void* x, void* out, int B, int HW, int C, int relu, bool bf16,
            hipStream_t st) {
  if (C % 8 || B <= 0 || HW <= 0) return (int)hipErrorInvalidValue;
  const dim3 grid(B, (C / 8 + 255) / 256);
  if (bf16)
    hipLaunchKernelGGL(gap_fwd_kernel<true>, grid, dim3(256), 0, st, (const uint16_t*)x, out, HW,
                       C, relu);
  else
    hipLaunchKernelGGL(gap_fwd_kernel<false>, grid, dim3(256), 0, st, (const uint16_t*)x, out, HW,
                       C, relu);
  ZK_CHECK_LAUNCH();
  return 0;
}

int gap_bwd(const float* dp, const void* x, void* dx, int B, int HW, int C, int relu,
            hipStream_t st) {
  if (C % 8 || B <= 0 || HW <= 0) return (int)hipErrorInvalidValue;
  const long long groups = (long long)B * HW * (C / 8);
  long long grid = (groups + 255) / 256;
  if (grid > 8192) grid = 8192;
  hipLaunchKernelGGL(gap_bwd_kernel, dim3((unsigned)grid), dim3(256), 0, st, dp,
                     (const uint16_t*)x, (uint16_t*)dx, B, HW, C, relu);
  ZK_CHECK_LAUNCH();
  return 0;
}

int sgemm(const float* A, long long sam, long long sak, const float* B, long long sbk,
          long long sbn, float* C, long long scm, int M, int N, int K, const float* bias, bool acc,
          float* colsum, hipStream_t st) {
  const dim3 grid((N + SG_T - 1) / SG_T, (M + SG_T - 1) / SG_T);
  if (acc)
    hipLaunchKernelGGL(sgemm_kernel<true>, grid, dim3(256), 0, st, A, sam, sak, B, sbk, sbn, C,
                       scm, M, N, K, bias, colsum);
  else
    hipLaunchKernelGGL(sgemm_kernel<false>, grid, dim3(256), 0, st, A, sam, sak, B, sbk, sbn, C,
                       scm, M, N, K, bias, colsum);
  ZK_CHECK_LAUNCH();
  return 0;
}

}  // namespace

// Forward: x bf16 [B][HW][C] (C % 8 == 0), W fp32 [N][C],
// bias fp32 [N] (optional) -> pooled fp32 [B][C], logits fp32 [B][N].
ZK_EXPORT int zk_head_fwd(const void* x, const void* w, const void* bias, void* pooled,
                          void* logits, int B, int HW, int C, int N, int relu, hipStream_t st) {
  const int rc = gap_fwd(x, pooled, B, HW, C, relu, false, st);
  if (rc) return rc;
  // logits[b][n] = sum_c pooled[b][c] * W[n][c] + bias[n]
  return sgemm((const float*)pooled, C, 1, (const float*)w, 1, C, (float*)logits, N, B, N, C,
               (const float*)bias, false, nullptr, st);
}

// Backward: dlogits fp32 [B][N] -> dW fp32 [N][C] +=, dbias [N] += (optional,
// needs dw),
// dx bf16 [B][HW][C]; dpooled fp32 [B][C] is scratch.
ZK_EXPORT int zk_head_bwd(const void* dlogits, const void* x, const void* w, const void* pooled,
                          void* dw, void* dbias, void* dpooled, void* dx, int B, int HW, int C,
                          int N, int relu, hipStream_t st) {
  if (C % 8 || B <= 0 || HW <= 0) return (int)hipErrorInvalidValue;
  const float* dl = (const float*)dlogits;
  int rc;
  if (dw) {
    // dW[n][c] += sum_b dl[b][n] * pooled[b][c]; dbias[n] += sum_b dl[b][n] in the same pass
    rc = sgemm(dl, 1, N, (const float*)pooled, C, 1, (float*)dw, C, N, C, B, nullptr, true,
               (float*)dbias, st);
    if (rc) return rc;
  } else if (dbias) {
    return (int)hipErrorInvalidValue;  // the bias gradient rides on the dW GEMM
  }
  if (dx) {
    // dpooled[b][c] = sum_n dl[b][n] * W[n][c]
    rc = sgemm(dl, N, 1, (const float*)w, C, 1, (float*)dpooled, C, B, C, N, nullptr, false,
               nullptr, st);
    if (rc) return rc;
    return gap_bwd((const float*)dpooled, x, dx, B, HW, C, relu, st);
  }
  return 0;
}

// GlobalAvgPool alone: x bf16 [B][HW][C] -> out [B][C] (bf16 if out_bf16,
// else fp32); backward from an fp32 dout.
ZK_EXPORT int zk_gap_fwd(const void* x, void* out, int B, int HW, int C, int relu, int out_bf16,
                         hipStream_t st) {
  return gap_fwd(x, out, B, HW, C, relu, out_bf16 != 0, st);
}

ZK_EXPORT int zk_gap_bwd(const void* dout, const void* x, void* dx, int B, int HW, int C,
                         int relu, hipStream_t st) {
  return gap_bwd((const float*)dout, x, dx, B, HW, C, relu, st);
}
