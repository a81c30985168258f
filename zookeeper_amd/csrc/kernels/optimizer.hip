// Fused optimizer step over the flat parameter buffer.
//
// One launch updates every parameter: Adam/AdamW or SGD(+Nesterov) momentum,
// the data-parallel 1/world averaging folded into `grad_scale`, decoupled
// (Adam) or L2 (SGD) weight decay on parameters flagged `decay`, and the
// Larq `weight_clip` constraint (clamp to [-clip, clip]) on parameters with
// clip > 0 — all in the same pass (p, g, m, v each read once, p/m/v written
// once: 28 B/element for Adam).
//
// Work is described by a chunk table (int64 x4 per chunk: offset, numel,
// clip bits (f32), decay flag), each chunk lying inside one parameter and at
// most `chunk` elements long; one workgroup per chunk, float4 accesses
// (every parameter starts 256-B aligned in the flat buffer).
#include "../common.h"

namespace {

struct AdamArgs {
  float lr, b1, b2, eps, wd, bc1, bc2, grad_scale;
};

__device__ __forceinline__ float clampc(float x, float c) {
  return c > 0.f ? fminf(fmaxf(x, -c), c) : x;
}

__global__ __launch_bounds__(256) void adam_chunks(float* __restrict__ p,
                                                   const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   const long long* __restrict__ chunks,
                                                   AdamArgs a) {
  const long long* c = chunks + 4 * blockIdx.x;
  const long long off = c[0];
  const int n = (int)c[1];
  const float clip = __int_as_float((int)c[2]);
  const float wd = c[3] ? a.wd : 0.f;
  const float step = a.lr;
  const float inv_bc1 = 1.f / a.bc1;
  const float inv_sqrt_bc2 = rsqrtf(a.bc2);
  const int n4 = n >> 2;
  float4* p4 = reinterpret_cast<float4*>(p + off);
  const float4* g4 = reinterpret_cast<const float4*>(g + off);
  float4* m4 = reinterpret_cast<float4*>(m + off);
  float4* v4 = reinterpret_cast<float4*>(v + off);
  for (int i = threadIdx.x; i < n4; i += blockDim.x) {
    float4 pp = p4[i], gg = g4[i], mm = m4[i], vv = v4[i];
    float* P = &pp.x; float* G = &gg.x; float* M = &mm.x; float* V = &vv.x;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float gk = G[k] * a.grad_scale;
      M[k] = a.b1 * M[k] + (1.f - a.b1) * gk;
      V[k] = a.b2 * V[k] + (1.f - a.b2) * gk * gk;
      const float upd = (M[k] * inv_bc1) / (sqrtf(V[k]) * inv_sqrt_bc2 + a.eps) + wd * P[k];
      P[k] = clampc(P[k] - step * upd, clip);
    }
    p4[i] = pp; m4[i] = mm; v4[i] = vv;
  }
  // Scalar tail (numel not a multiple of 4).
  for (int i = (n4 << 2) + threadIdx.x; i < n; i += blockDim.x) {
    const long long j = off + i;
    const float gk = g[j] * a.grad_scale;
    m[j] = a.b1 * m[j] + (1.f - a.b1) * gk;
    v[j] = a.b2 * v[j] + (1.f - a.b2) * gk * gk;
    const float upd = (m[j] * inv_bc1) / (sqrtf(v[j]) * inv_sqrt_bc2 + a.eps) + wd * p[j];
    p[j] = clampc(p[j] - step * upd, clip);
  }
}

struct SgdArgs {
  float lr, momentum, wd, grad_scale;
  int nesterov;
};

__global__ __launch_bounds__(256) void sgd_chunks(float* __restrict__ p,
                                                  const float* __restrict__ g,
                                                  float* __restrict__ m,
                                                  const long long* __restrict__ chunks,
                                                  SgdArgs a) {
  const long long* c = chunks + 4 * blockIdx.x;
  const long long off = c[0];
  const int n = (int)c[1];
  const float clip = __int_as_float((int)c[2]);
  const float wd = c[3] ? a.wd : 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const long long j = off + i;
    const float gk = g[j] * a.grad_scale + wd * p[j];
    const float mk = a.momentum * m[j] + gk;
    m[j] = mk;
    const float d = a.nesterov ? gk + a.momentum * mk : mk;
    p[j] = clampc(p[j] - a.lr * d, clip);
  }
}

}  // namespace

ZK_EXPORT int zk_adam_step(void* p, const void* g, void* m, void* v, const void* chunks,
                           int num_chunks, float lr, float b1, float b2, float eps, float wd,
                           float bc1, float bc2, float grad_scale, hipStream_t stream) {
  if (num_chunks <= 0) return 0;
  AdamArgs a{lr, b1, b2, eps, wd, bc1, bc2, grad_scale};
  hipLaunchKernelGGL(adam_chunks, dim3(num_chunks), dim3(256), 0, stream, (float*)p,
                     (const float*)g, (float*)m, (float*)v, (const long long*)chunks, a);
  ZK_CHECK_LAUNCH();
  return 0;
}

ZK_EXPORT int zk_sgd_step(void* p, const void* g, void* m, const void* chunks, int num_chunks,
                          float lr, float momentum, float wd, float grad_scale, int nesterov,
                          hipStream_t stream) {
  if (num_chunks <= 0) return 0;
  SgdArgs a{lr, momentum, wd, grad_scale, nesterov};
  hipLaunchKernelGGL(sgd_chunks, dim3(num_chunks), dim3(256), 0, stream, (float*)p,
                     (const float*)g, (float*)m, (const long long*)chunks, a);
  ZK_CHECK_LAUNCH();
  return 0;
}
