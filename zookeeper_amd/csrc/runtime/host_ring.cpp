// Host-side input pipeline helpers (no GPU code).
//
// zk_gather_rows: multi-threaded gather of whole rows (one example each) from
// a source array (e.g. a memory-mapped dataset) into a destination buffer —
// normally a pinned host slot that the loader then copies to the device with
// hipMemcpyAsync on a side stream.  Rows are split into contiguous ranges, one
// per worker thread; each worker memcpy's its rows.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

extern "C" __attribute__((visibility("default"))) int zk_gather_rows(
    const void* src, int64_t row_bytes, const int64_t* idx, int64_t n, void* dst,
    int threads) {
  if (!src || !dst || !idx || row_bytes <= 0 || n < 0) return 1;
  const char* s = static_cast<const char*>(src);
  char* d = static_cast<char*>(dst);
  auto work = [&](int64_t lo, int64_t hi) {
    for (int64_t i = lo; i < hi; ++i) memcpy(d + i * row_bytes, s + idx[i] * row_bytes, row_bytes);
  };
  const int64_t bytes = n * row_bytes;
  int t = std::max(1, std::min<int>(threads, (int)std::min<int64_t>(n, 64)));
  if (bytes < (4 << 20)) t = 1;  // small batches: threads cost more than they save
  if (t == 1) {
    work(0, n);
    return 0;
  }
  std::vector<std::thread> pool;
  pool.reserve(t);
  const int64_t per = (n + t - 1) / t;
  for (int k = 0; k < t; ++k) {
    const int64_t lo = k * per, hi = std::min(n, lo + per);
    if (lo >= hi) break;
    pool.emplace_back(work, lo, hi);
  }
  for (auto& th : pool) th.join();
  return 0;
}
