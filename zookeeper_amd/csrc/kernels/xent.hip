// Fused softmax + sparse categorical cross-entropy (+ label smoothing) and
// top-1 correctness, forward and backward, one wave per row (fp32 logits).
// Replaces Keras' softmax activation + sparse_categorical_crossentropy +
// "accuracy" metric of the reference example (examples/larq_experiment.py:
// 101,117-118) with two launches per step.
//
//   forward   loss_sum += (1-eps)*(lse - x_y) + eps*(lse - mean_j x_j)
//             correct  += [argmax_j x_j == y]     (first maximum)
//             lse[row] saved for backward
//   backward  dx_j = g/B * (softmax_j - (1-eps)*[j == y] - eps/C)
#include "../common.h"

namespace {

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  return v;
}

__global__ __launch_bounds__(256) void xent_fwd_kernel(const float* __restrict__ x,
                                                       const long long* __restrict__ labels,
                                                       float* __restrict__ lse_out,
                                                       float* __restrict__ loss_sum,
                                                       int* __restrict__ correct, int B, int C,
                                                       float eps, float* __restrict__ row_loss) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const float* xr = x + (long long)row * C;
  float mx = -INFINITY;
  int arg = 0;
  float sum = 0.f;
  for (int j = lane; j < C; j += 64) {
    const float v = xr[j];
    if (v > mx) {
      mx = v;
      arg = j;
    }
    sum += v;
  }
  // row max and its first index
  float gmax = wave_max(mx);
  int cand = (mx == gmax) ? arg : 0x7fffffff;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) cand = min(cand, __shfl_xor(cand, off, 64));
  float se = 0.f;
  for (int j = lane; j < C; j += 64) se += __expf(xr[j] - gmax);
  se = zk::wave_sum(se);
  sum = zk::wave_sum(sum);
  if (lane == 0) {
    const long long y = labels[row];
    const float lse = gmax + __logf(se);
    lse_out[row] = lse;
    const float nll = lse - xr[y];
    const float smooth = lse - sum / (float)C;
    const float lr = (1.f - eps) * nll + eps * smooth;
    if (row_loss)
      row_loss[row] = lr;  // deterministic mode: summed in row order by xent_sum_kernel
    else
      atomicAdd(loss_sum, lr);
    if (cand == (int)y) atomicAdd(correct, 1);
  }
}

// loss_sum = sum of row_loss in a fixed order (one block: per-thread strided
// partial sums, then a fixed tree): bit-reproducible, unlike the atomics.
__global__ __launch_bounds__(256) void xent_sum_kernel(const float* __restrict__ row_loss,
                                                       float* __restrict__ loss_sum, int B) {
  __shared__ float red[256];
  float s = 0.f;
  for (int i = threadIdx.x; i < B; i += 256) s += row_loss[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) loss_sum[0] += red[0];
}

__global__ __launch_bounds__(256) void xent_bwd_kernel(const float* __restrict__ x,
                                                       const long long* __restrict__ labels,
                                                       const float* __restrict__ lse,
                                                       const float* __restrict__ gout,
                                                       float* __restrict__ dx, int B, int C,
                                                       float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const float scale = gout[0] / (float)B;
  const float l = lse[row];
  const long long y = labels[row];
  const float off = eps / (float)C;
  const float* xr = x + (long long)row * C;
  float* dr = dx + (long long)row * C;
  for (int j = lane; j < C; j += 64) {
    const float p = __expf(xr[j] - l);
    dr[j] = scale * (p - off - (j == y ? 1.f - eps : 0.f));
  }
}

// Mean loss and hit count out of the accumulators, which are re-zeroed for
// the next call (no framework fill / divide / cast kernels around the op).
__global__ void xent_finalize_kernel(float* __restrict__ acc, float* __restrict__ loss,
                                     long long* __restrict__ hits, int B) {
  if (threadIdx.x != 0) return;
  loss[0] = __fdiv_rn(acc[0], (float)B);
  hits[0] = (long long)__float_as_int(acc[1]);
  acc[0] = 0.f;
  acc[1] = 0.f;  // int 0 bits
}

}  // namespace

// acc = [loss_sum fp32, correct int32 bits] -> loss = loss_sum / B (fp32),
// hits (int64); acc re-zeroed.
ZK_EXPORT int zk_xent_finalize(void* acc, void* loss, void* hits, int B, hipStream_t st) {
  hipLaunchKernelGGL(xent_finalize_kernel, dim3(1), dim3(64), 0, st, (float*)acc, (float*)loss,
                     (long long*)hits, B);
  ZK_CHECK_LAUNCH();
  return 0;
}

// loss_sum (fp32) and correct (int32) are accumulated (zeroed by the caller).
// row_loss (optional, [B] fp32): per-row losses summed in a fixed order
// instead of fp32 atomics (the deterministic mode).
ZK_EXPORT int zk_xent_fwd(const float* x, const void* labels, float* lse, float* loss_sum,
                          int* correct, int B, int C, float eps, float* row_loss,
                          hipStream_t st) {
  hipLaunchKernelGGL(xent_fwd_kernel, dim3((B + 3) / 4), dim3(256), 0, st, x,
                     (const long long*)labels, lse, loss_sum, correct, B, C, eps, row_loss);
  if (row_loss)
    hipLaunchKernelGGL(xent_sum_kernel, dim3(1), dim3(256), 0, st, row_loss, loss_sum, B);
  ZK_CHECK_LAUNCH();
  return 0;
}

// gout: device scalar (upstream gradient of the mean loss).
ZK_EXPORT int zk_xent_bwd(const float* x, const void* labels, const float* lse,
                          const float* gout, float* dx, int B, int C, float eps, hipStream_t st) {
  hipLaunchKernelGGL(xent_bwd_kernel, dim3((B + 3) / 4), dim3(256), 0, st, x,
                     (const long long*)labels, lse, gout, dx, B, C, eps);
  ZK_CHECK_LAUNCH();
  return 0;
}
