// Phase profile of the persistent binary forward (bfwd.hip), built
// with the kernel's diagnostic stamps on:
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DZK_BFWD_STAMPS -I zookeeper_amd/csrc \
//         tools/bfwd_stamps.cpp -o tools/bfwd_stamps
//   ./tools/bfwd_stamps [batch] [hw] [store_y] [channels]
//
// Runs the E18 stage geometry (batch x hw x hw x channels, 64 or 128 -> the
// same) on random e2m1 signs and prints the kernel time and, per wave, the
// mean shader cycles of each
// phase of the tile loop: DMA wait, barrier, DMA issue + edge flags, MFMA
// issue, epilogue (statistics, staging, stores), statistics flush.
#include "kernels/bfwd.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

int main(int argc, char** argv) {
  const int B = argc > 1 ? std::atoi(argv[1]) : 1536;
  const int HW = argc > 2 ? std::atoi(argv[2]) : 56;
  const int store_y = argc > 3 ? std::atoi(argv[3]) : 1;
  const int C = argc > 4 ? std::atoi(argv[4]) : 64;
  const long long M = (long long)B * HW * HW;
  srand(1);
  auto sgn = [] { return (unsigned char)((rand() & 1) ? 0x2 : 0xA); };
  std::vector<unsigned char> hx(M * C / 2), hw(9 * C * C / 2);
  for (auto& v : hx) v = sgn() | (sgn() << 4);
  for (auto& v : hw) v = sgn() | (sgn() << 4);
  unsigned char *x4 = nullptr, *w4 = nullptr;
  short* y = nullptr;
  unsigned long long* stats = nullptr;
  CK(hipMalloc(&x4, hx.size()));
  CK(hipMalloc(&w4, hw.size()));
  CK(hipMalloc(&y, M * C * 2));
  CK(hipMalloc(&stats, 32 * 2 * C * 8));
  CK(hipMemcpy(x4, hx.data(), hx.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(w4, hw.data(), hw.size(), hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 10;
  float tot = 0.f;
  for (int r = 0; r < reps + 1; ++r) {
    CK(hipMemset(stats, 0, 32 * 2 * C * 8));
    CK(hipEventRecord(e0, 0));
    CK((hipError_t)zk_bfwd_fp4(x4, w4, store_y ? y : nullptr, stats, B, HW, HW, C, C, 0, 0, 32,
                               0));
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (r) tot += ms / reps;
  }
  static unsigned long long st[2048 * 8][6];
  CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(g_bf_stamps), sizeof(st)));
  const int nwb = C == 64 ? Bf64::NW : Bf128::NW;  // waves per block
  const int nblk = C == 64 ? Bf64::OCC * bf_cus() : Bf128::OCC * bf_cus();
  std::printf("batch %d, %dx%dx%d, y %s: %.1f us per call (mean of %d)\n", B, HW, HW, C,
              store_y ? "stored" : "not stored", tot * 1e3, reps);
  const char* names[6] = {"DMA wait", "barrier", "DMA issue + edges", "MFMA issue",
                          "epilogue + stores", "stats flush"};
  double sum = 0;
  double ph[6] = {0, 0, 0, 0, 0, 0};
  int nw = 0;
  for (int b = 0; b < nblk && b < 2048; ++b)
    for (int w = 0; w < nwb; ++w) {
      for (int k = 0; k < 6; ++k) ph[k] += st[b * nwb + w][k];
      ++nw;
    }
  for (int k = 0; k < 6; ++k) sum += ph[k] / nw;
  for (int k = 0; k < 6; ++k)
    std::printf("  %-20s %10.0f cycles per wave (%4.1f %%)\n", names[k], ph[k] / nw,
                100.0 * ph[k] / nw / sum);
  std::printf("  %-20s %10.0f cycles per wave\n", "total", sum);
  return 0;
}
