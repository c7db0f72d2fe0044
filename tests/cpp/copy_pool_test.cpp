// The host copy pool (slime_amd/csrc/host_copy.cpp) under concurrent callers,
// CPU only: every caller's bytes land exactly, whatever the interleaving of
// jobs, sizes below and above the serial threshold, and pool sizes.
#include <atomic>
#include <cstdio>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "host_copy.hpp"

int main() {
  std::atomic<int> bad{0};
  const int kThreads = 8;
  std::vector<std::thread> th;
  for (int t = 0; t < kThreads; ++t) {
    th.emplace_back([t, &bad] {
      std::mt19937_64 rng(1000 + t);
      for (int it = 0; it < 60; ++it) {
        const size_t nitems = 1 + rng() % 5;
        std::vector<std::vector<unsigned char>> src(nitems), dst(nitems);
        std::vector<slime::CopyItem> items;
        for (size_t i = 0; i < nitems; ++i) {
          const size_t n = (rng() % 3 == 0) ? rng() % 4096 : (rng() % (6u << 20));
          src[i].resize(n);
          for (size_t b = 0; b < n; b += 8) src[i][b] = (unsigned char)rng();
          dst[i].assign(n + 64, 0xEE);
          items.push_back({dst[i].data() + (rng() % 64), src[i].data(), n});
        }
        slime::parallel_copy(items.data(), items.size());
        for (size_t i = 0; i < nitems; ++i) {
          const unsigned char* d = (const unsigned char*)items[i].dst;
          if (memcmp(d, src[i].data(), src[i].size()) != 0) ++bad;
          const size_t off = d - dst[i].data();
          for (size_t b = 0; b < off; ++b)
            if (dst[i][b] != 0xEE) ++bad;  // nothing written before the range
          for (size_t b = off + src[i].size(); b < dst[i].size(); ++b)
            if (dst[i][b] != 0xEE) ++bad;  // nor after it
        }
      }
    });
  }
  for (auto& x : th) x.join();
  printf("copy pool: %d threads besides callers, %d mismatches\n", slime::copy_pool_threads(), bad.load());
  return bad.load() == 0 ? 0 : 1;
}
