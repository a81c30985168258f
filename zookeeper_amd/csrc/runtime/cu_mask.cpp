// CU-masked HIP streams (host code): a stream whose kernels may only be
// dispatched to a chosen subset of the compute units (hipExtStreamCreateWithCUMask).
//
// Used for the weight-gradient side stream (ops/streams.py,
// runtime.wgrad_cu_share): the side-stream split-K GEMMs are off the
// critical path, and each of their blocks holds a whole CU (128 KB of LDS,
// 512 threads), so unrestricted they can occupy every CU while the
// data-gradient chain on the compute stream waits for a slot.  Restricted to
// a share of the CUs, they leave the rest to the critical path.
//
// The mask takes CUs evenly over the enumeration (CU i is in the set when
// floor((i + 1) * num / den) > floor(i * num / den)), so the share is spread
// over the XCDs whichever way the driver numbers them.
#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include <vector>

#define ZK_EXPORT extern "C" __attribute__((visibility("default")))

// *out = the new stream (hipStream_t) on `device`; returns a hipError_t.
// share_num / share_den in (0, 1]; *ncu_out (optional) = CUs in the mask.
ZK_EXPORT int zk_cu_masked_stream(int device, int share_num, int share_den, void** out,
                                  int* ncu_out) {
  if (!out || share_num <= 0 || share_den <= 0 || share_num > share_den)
    return (int)hipErrorInvalidValue;
  int prev = 0;
  hipError_t e = hipGetDevice(&prev);
  if (e != hipSuccess) return (int)e;
  if ((e = hipSetDevice(device)) != hipSuccess) return (int)e;
  int ncu = 0;
  e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device);
  if (e != hipSuccess || ncu <= 0) {
    (void)hipSetDevice(prev);
    return e != hipSuccess ? (int)e : (int)hipErrorInvalidValue;
  }
  std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
  int n = 0;
  for (int i = 0; i < ncu; ++i) {
    const long long a = (long long)i * share_num / share_den;
    const long long b = (long long)(i + 1) * share_num / share_den;
    if (b > a) {
      mask[i / 32] |= 1u << (i % 32);
      ++n;
    }
  }
  hipStream_t s = nullptr;
  e = hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data());
  (void)hipSetDevice(prev);
  if (e != hipSuccess) return (int)e;
  *out = (void*)s;
  if (ncu_out) *ncu_out = n;
  return 0;
}
