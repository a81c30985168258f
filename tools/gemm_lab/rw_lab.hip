// Lab driver for the row-window conv3 dgrad (zookeeper_amd/csrc/kernels/conv3rw.hip):
// built once per ablation (-DRW_ABL=n, see the kernel), times the E18
// stage-1 shape (batch 1024, 56x56x64 -> 64) with hipEvents.
//   usage: rw_labN [batch] [reps]
#include "../../zookeeper_amd/csrc/kernels/conv3rw.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 1024, reps = argc > 2 ? atoi(argv[2]) : 20;
  const int H = 56, W = 56, C = 64;
  const size_t act = (size_t)B * H * W * C;
  uint16_t *dy, *wt, *dres, *dx;
  uint32_t* mask;
  if (hipMalloc(&dy, act * 2) || hipMalloc(&dres, act * 2) || hipMalloc(&dx, act * 2) ||
      hipMalloc(&wt, 9 * C * C * 2) || hipMalloc(&mask, (size_t)B * H * W * 2 * 4))
    return 1;
  std::vector<uint16_t> h(act);
  for (size_t i = 0; i < act; ++i) h[i] = (uint16_t)(0x3F00u + (i * 2654435761u >> 24) % 256);
  (void)hipMemcpy(dy, h.data(), act * 2, hipMemcpyHostToDevice);
  (void)hipMemcpy(dres, h.data(), act * 2, hipMemcpyHostToDevice);
  (void)hipMemcpy(wt, h.data(), 9 * C * C * 2, hipMemcpyHostToDevice);
  (void)hipMemset(mask, 0xff, (size_t)B * H * W * 8);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int w = 0; w < 3; ++w)
    if (zk_conv3rw_dgrad_impl(dy, wt, mask, dres, dx, B, H, W, C, C, false, 0)) return 2;
  (void)hipEventRecord(e0, 0);
  for (int r = 0; r < reps; ++r) zk_conv3rw_dgrad_impl(dy, wt, mask, dres, dx, B, H, W, C, C, false, 0);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double us = 1e3 * ms / reps, fl = 2.0 * B * H * W * C * 9.0 * C;
  printf("RW_ABL=%d B=%d: %.1f us/call, %.3f PF/s\n", RW_ABL, B, us, fl / us * 1e-9);
  return 0;
}
