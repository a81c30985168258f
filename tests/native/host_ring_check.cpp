// Driver for zk_gather_rows (zookeeper_amd/csrc/runtime/host_ring.cpp) under
// the host sanitizers (tests/test_native_sanitizers.py builds it with
// -fsanitize=address,undefined and with -fsanitize=thread): single- and
// multi-threaded gathers, every row checked, plus the argument checks.
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <vector>

extern "C" int zk_gather_rows(const void* src, int64_t row_bytes, const int64_t* idx, int64_t n,
                              void* dst, int threads);

static int check(int64_t rows, int64_t row_bytes, int64_t n, int threads) {
  std::vector<uint8_t> src((size_t)(rows * row_bytes));
  for (size_t i = 0; i < src.size(); ++i) src[i] = (uint8_t)(i * 2654435761u >> 13);
  std::vector<int64_t> idx((size_t)(n > 0 ? n : 1));  // valid pointer for n == 0
  for (int64_t i = 0; i < n; ++i) idx[(size_t)i] = (i * 7919 + 13) % rows;
  std::vector<uint8_t> dst((size_t)((n > 0 ? n : 1) * row_bytes), 0xCD);
  if (zk_gather_rows(src.data(), row_bytes, idx.data(), n, dst.data(), threads) != 0) return 1;
  for (int64_t i = 0; i < n; ++i)
    if (memcmp(dst.data() + i * row_bytes, src.data() + idx[(size_t)i] * row_bytes,
               (size_t)row_bytes) != 0) {
      fprintf(stderr, "row %lld mismatch (rows %lld, bytes %lld, threads %d)\n", (long long)i,
              (long long)rows, (long long)row_bytes, threads);
      return 1;
    }
  return 0;
}

int main() {
  int bad = 0;
  bad |= check(100, 3 * 32 * 32, 64, 1);        // small: single-threaded path
  bad |= check(100, 3 * 32 * 32, 64, 8);        // small batch keeps one thread
  bad |= check(512, 3 * 64 * 64, 384, 8);       // >= 4 MiB: worker threads
  bad |= check(300, 150528, 37, 5);             // ImageNet rows, uneven split
  bad |= check(10, 1, 0, 4);                    // empty gather
  // argument checks
  int64_t i0 = 0;
  uint8_t b = 0;
  bad |= zk_gather_rows(nullptr, 1, &i0, 1, &b, 1) != 1;
  bad |= zk_gather_rows(&b, 0, &i0, 1, &b, 1) != 1;
  bad |= zk_gather_rows(&b, 1, nullptr, 1, &b, 1) != 1;
  if (bad) {
    fprintf(stderr, "host_ring_check: FAILED\n");
    return 1;
  }
  printf("host_ring_check: ok\n");
  return 0;
}
