// Role balance of the two-role stem pipelines (stem_fused.hip F and B2).
// Built with the kernels' diagnostic stamps on:
//
//   hipcc --offload-arch=gfx950 -O3 -DZK_STEM_STAMPS -I zookeeper_amd/csrc \
//         tools/stem_stamps.cpp -o tools/stem_stamps
//   ./tools/stem_stamps [batch]
//
// Runs the E18 stem geometry (224x224x3 -> 112x112x64 -> 56x56x64) on
// synthetic inputs and prints, per role (waves 0-3 / 4-7), the mean shader
// cycles per block spent working and waiting at the interval barrier, plus
// the kernel times.
#include "kernels/stem_fused.hip"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                         \
    }                                                                       \
  } while (0)

static uint16_t bf16(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  return (uint16_t)((u + 0x7FFF + ((u >> 16) & 1)) >> 16);
}

template <typename T>
static T* upload(const std::vector<T>& h) {
  T* d = nullptr;
  CK(hipMalloc(&d, h.size() * sizeof(T)));
  CK(hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
  return d;
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? std::atoi(argv[1]) : 1536;
  const int Cin = 3, KW = 7, Ho = 112, Wo = 112, Hp = 229, Wp = 230, H2 = 56, W2 = 56;
  const int pt2 = 0, pl2 = 0;
  srand(1);
  auto rnd = [] { return (float)rand() / RAND_MAX * 2.f - 1.f; };
  std::vector<uint16_t> hxp((size_t)B * Hp * Wp * 4);
  for (size_t i = 0; i < hxp.size(); ++i) hxp[i] = (i % 4 == 3) ? 0 : bf16(rnd());
  std::vector<uint16_t> hws(7 * 64 * 32);
  for (auto& v : hws) v = bf16(0.1f * rnd());
  std::vector<float> hg(64), hc1(4 * 64), hb1(3 * 64);
  for (auto& v : hg) v = rnd();
  for (int c = 0; c < 64; ++c) {
    hc1[c] = rnd();
    hc1[64 + c] = 0.1f * rnd();
    hc1[128 + c] = 0.f;
    hc1[192 + c] = 1.f;
    hb1[c] = rnd();
    hb1[64 + c] = 0.01f * rnd();
    hb1[128 + c] = 0.01f * rnd();
  }
  const long long P2 = (long long)B * H2 * W2;
  std::vector<uint16_t> hdp((size_t)P2 * 64);
  for (auto& v : hdp) v = bf16(rnd());
  uint16_t* xp = upload(hxp);
  uint16_t* ws = upload(hws);
  float* gamma = upload(hg);
  float* coef1 = upload(hc1);
  float* bcoef1 = upload(hb1);
  uint16_t* dp = upload(hdp);
  uint16_t* ya = nullptr;
  uint8_t* arg = nullptr;
  CK(hipMalloc(&ya, P2 * 64 * 2));
  CK(hipMalloc(&arg, P2 * 64));
  const int nf = zk_stem_fused_blocks(1, B, Ho, Wo, H2, W2);
  const int nb = zk_stem_fused_blocks(0, B, Ho, Wo, H2, W2);
  float *part = nullptr, *slab = nullptr, *dw = nullptr;
  CK(hipMalloc(&part, (size_t)nf * 2 * 64 * 4));
  CK(hipMalloc(&slab, (size_t)(nb + zk_stem_fused_slab_extra()) * zk_stem_fused_slab_floats() * 4));
  CK(hipMalloc(&dw, 64 * 7 * KW * Cin * 4));
  CK(hipMemset(dw, 0, 64 * 7 * KW * Cin * 4));
  hipEvent_t e0, e1, e2;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&e2));
  float tf = 0.f, tb = 0.f;
  const int reps = 5;
  for (int r = 0; r < reps + 1; ++r) {
    int np = 0;
    CK(hipEventRecord(e0, 0));
    CK((hipError_t)zk_stem_fwd_fused(xp, ws, gamma, ya, arg, part, B, Cin, KW, Ho, Wo, Hp, Wp, H2,
                                     W2, pt2, pl2, &np, 0));
    CK(hipEventRecord(e1, 0));
    CK((hipError_t)zk_stem_bwd_fused(xp, ws, dp, arg, coef1, bcoef1, slab, dw, B, Cin, KW, Ho, Wo,
                                     Hp, Wp, H2, W2, pt2, pl2, 0));
    CK(hipEventRecord(e2, 0));
    CK(hipEventSynchronize(e2));
    float a, b;
    CK(hipEventElapsedTime(&a, e0, e1));
    CK(hipEventElapsedTime(&b, e1, e2));
    if (r) {
      tf += a / reps;
      tb += b / reps;
    }
  }
  static unsigned long long st[2][1024 * 8][3];
  CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(g_stem_stamps), sizeof(st)));
  std::printf("batch %d: F %.1f us, B2 (+reduce) %.1f us (mean of %d)\n", B, tf * 1e3, tb * 1e3,
              reps);
  const int nblk[2] = {nf, nb};
  const char* names[2] = {"F ", "B2"};
  const char* roles[2][2] = {{"pool  ", "matrix"}, {"route ", "matrix"}};
  for (int k = 0; k < 2; ++k)
    for (int role = 0; role < 2; ++role) {
      double work = 0, wait = 0, mem = 0;
      int n = 0;
      for (int b = 0; b < nblk[k] && b < 1024; ++b)
        for (int w = 4 * role; w < 4 * role + 4; ++w) {
          work += st[k][b * 8 + w][0];
          wait += st[k][b * 8 + w][1];
          mem += st[k][b * 8 + w][2];
          ++n;
        }
      std::printf("%s %s waves: work %.0f  own-memory wait %.0f  barrier wait %.0f cycles per "
                  "wave (last launch)\n", names[k], roles[k][role], work / n, mem / n, wait / n);
    }
  return 0;
}
