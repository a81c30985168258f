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
// clip bits (f32), flags), each chunk lying inside one parameter and at
// most `chunk` elements long; one workgroup per chunk, float4 accesses
// (every parameter starts 256-B aligned in the flat buffer).  flags: bit 0 =
// weight decay applies; bits 8.. = 1 + the parameter's row in the weight-image
// table (0: none).
//
// Weight images: the float convs' MFMA kernels read their weights as bf16 in
// GEMM layouts ([T][Cout][Cin] for the forward, [T][Cin][Cout] for the data
// gradient).  Instead of a cast / transpose launch per conv and pass
// (~140 framework copy kernels per ResNet-50 step), the optimizer writes
// the images of the parameters it has just updated, in the same pass.
// Image-table row (int64 x 8): flat offset of the parameter, Cout, Cin, KH,
// KW, flags (bit 0: physical OHWI layout, else OIHW; bit 1: forward image
// with flipped taps), forward-image pointer, data-gradient-image pointer
// (0: not kept).  zk_weight_images builds them from the current parameters
// (first use, or after the parameters changed outside the optimizer).
#include "../common.h"

namespace {

__device__ __forceinline__ void write_images(const long long* __restrict__ ent, long long e,
                                             float v) {
  const int Cout = (int)ent[1], Cin = (int)ent[2], KH = (int)ent[3], KW = (int)ent[4];
  const int fl = (int)ent[5];
  int co, ci, kh, kw;
  if (fl & 1) {  // OHWI
    ci = (int)(e % Cin);
    long long r = e / Cin;
    kw = (int)(r % KW);
    r /= KW;
    kh = (int)(r % KH);
    co = (int)(r / KH);
  } else {  // OIHW
    kw = (int)(e % KW);
    long long r = e / KW;
    kh = (int)(r % KH);
    r /= KH;
    ci = (int)(r % Cin);
    co = (int)(r / Cin);
  }
  const uint16_t b = zk::f32_to_bf16(v);
  uint16_t* A = reinterpret_cast<uint16_t*>(ent[6]);
  uint16_t* Bt = reinterpret_cast<uint16_t*>(ent[7]);
  if (A) {
    const int t = (fl & 2) ? (KH - 1 - kh) * KW + (KW - 1 - kw) : kh * KW + kw;
    A[((long long)t * Cout + co) * Cin + ci] = b;
  }
  if (Bt) Bt[((long long)(kh * KW + kw) * Cin + ci) * Cout + co] = b;
}

// Image-table row of a chunk (nullptr: none).
__device__ __forceinline__ const long long* chunk_images(const long long* c,
                                                         const long long* images) {
  const long long idx = (c[3] >> 8) - 1;
  return (images && idx >= 0) ? images + 8 * idx : nullptr;
}

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
                                                   const long long* __restrict__ images,
                                                   AdamArgs a) {
  const long long* c = chunks + 4 * blockIdx.x;
  const long long off = c[0];
  const int n = (int)c[1];
  const float clip = __int_as_float((int)c[2]);
  const float wd = (c[3] & 1) ? a.wd : 0.f;
  const long long* img = chunk_images(c, images);
  const long long e0 = img ? off - img[0] : 0;  // chunk start within the parameter
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
      if (img) write_images(img, e0 + 4 * i + k, P[k]);
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
    if (img) write_images(img, e0 + i, p[j]);
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
                                                  const long long* __restrict__ images,
                                                  SgdArgs a) {
  const long long* c = chunks + 4 * blockIdx.x;
  const long long off = c[0];
  const int n = (int)c[1];
  const float clip = __int_as_float((int)c[2]);
  const float wd = (c[3] & 1) ? a.wd : 0.f;
  const long long* img = chunk_images(c, images);
  const long long e0 = img ? off - img[0] : 0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const long long j = off + i;
    const float gk = g[j] * a.grad_scale + wd * p[j];
    const float mk = a.momentum * m[j] + gk;
    m[j] = mk;
    const float d = a.nesterov ? gk + a.momentum * mk : mk;
    const float pn = clampc(p[j] - a.lr * d, clip);
    p[j] = pn;
    if (img) write_images(img, e0 + i, pn);
  }
}

// Images of every table row from the current parameters: grid.y = row,
// grid.x strides over the row's elements.
__global__ __launch_bounds__(256) void weight_images_kernel(const float* __restrict__ flat,
                                                            const long long* __restrict__ images) {
  const long long* ent = images + 8 * blockIdx.y;
  const long long numel = ent[1] * ent[2] * ent[3] * ent[4];
  const float* src = flat + ent[0];
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < numel;
       e += (long long)gridDim.x * blockDim.x)
    write_images(ent, e, src[e]);
}

}  // namespace

ZK_EXPORT int zk_adam_step(void* p, const void* g, void* m, void* v, const void* chunks,
                           int num_chunks, float lr, float b1, float b2, float eps, float wd,
                           float bc1, float bc2, float grad_scale, const void* images,
                           hipStream_t stream) {
  if (num_chunks <= 0) return 0;
  AdamArgs a{lr, b1, b2, eps, wd, bc1, bc2, grad_scale};
  hipLaunchKernelGGL(adam_chunks, dim3(num_chunks), dim3(256), 0, stream, (float*)p,
                     (const float*)g, (float*)m, (float*)v, (const long long*)chunks,
                     (const long long*)images, a);
  ZK_CHECK_LAUNCH();
  return 0;
}

ZK_EXPORT int zk_sgd_step(void* p, const void* g, void* m, const void* chunks, int num_chunks,
                          float lr, float momentum, float wd, float grad_scale, int nesterov,
                          const void* images, hipStream_t stream) {
  if (num_chunks <= 0) return 0;
  SgdArgs a{lr, momentum, wd, grad_scale, nesterov};
  hipLaunchKernelGGL(sgd_chunks, dim3(num_chunks), dim3(256), 0, stream, (float*)p,
                     (const float*)g, (float*)m, (const long long*)chunks,
                     (const long long*)images, a);
  ZK_CHECK_LAUNCH();
  return 0;
}

// Zero `bytes` of device memory on `stream` (the per-step gradient-buffer
// clear: a runtime memset instead of a framework fill kernel).
ZK_EXPORT int zk_zero(void* p, long long bytes, hipStream_t stream) {
  if (bytes <= 0) return 0;
  return (int)hipMemsetAsync(p, 0, (size_t)bytes, stream);
}

// Weight images of `rows` image-table rows (see the top of this file) from
// the flat parameter buffer; max_numel = the largest row's element count.
ZK_EXPORT int zk_weight_images(const void* flat, const void* images, int rows,
                               long long max_numel, hipStream_t stream) {
  if (rows <= 0 || max_numel <= 0) return 0;
  long long bx = (max_numel + 255) / 256;
  if (bx > 1024) bx = 1024;
  hipLaunchKernelGGL(weight_images_kernel, dim3((unsigned)bx, (unsigned)rows), dim3(256), 0,
                     stream, (const float*)flat, (const long long*)images);
  ZK_CHECK_LAUNCH();
  return 0;
}
