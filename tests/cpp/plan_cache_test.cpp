// CPU test of the host entry points' recovery-plan cache (slime_amd/csrc/plan_cache.hpp):
// the product's LruCache over the product's host matrix code (rs_matrix.cpp),
// with a stand-in for the device table whose allocation count is tracked.
//
//   - 10,000 distinct survivor sets of a 20/40 code (RecoverData's inversion,
//     internal/rs/vector.go:69-77): the live plan count never exceeds the cap
//     and every evicted plan's table is released;
//   - 8 threads sharing the cache with a small cap: a plan a caller holds stays
//     intact while other threads evict it, and is released once let go;
//   - a failed build (singular survivor set, matrix.go:68) caches nothing;
//   - builds run outside the cache lock: 8 threads missing 8 different keys
//     with a 50 ms build finish in about 50 ms, not 400; 8 threads missing
//     the SAME key share one build;
//   - evicted values are released outside the lock (the deleter checks);
//   - a build that throws wakes its waiters and caches nothing.
// Usage: plan_cache_test   (exit 0 = pass)
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <new>
#include <cstdlib>
#include <random>
#include <set>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "gfp_host.hpp"
#include "plan_cache.hpp"
#include "rs_matrix.hpp"

using namespace slime;

static std::atomic<long> g_tables{0};  // stand-in device tables alive

struct FakePlan {
  std::vector<uint32_t> coeff;  // need x need inverse (RecoverData's matrix)
  std::vector<int> have;
  FakePlan() { g_tables.fetch_add(1); }
  ~FakePlan() { g_tables.fetch_sub(1); }
};

using Key = std::tuple<int, char, int, int, std::vector<int>>;

static int build(const Key& key, FakePlan** out) {
  const int need = std::get<2>(key);
  const std::vector<int>& have = std::get<4>(key);
  Matrix hv((size_t)need, (size_t)need), inv;
  std::vector<uint32_t> row;
  for (int i = 0; i < need; ++i) {
    if (code_row(need, have[i], &row) != Status::Ok) return 9;
    std::copy(row.begin(), row.end(), hv.v.begin() + (size_t)i * need);
  }
  if (Status st = invert(hv, &inv); st != Status::Ok) return (int)st;
  auto* p = new FakePlan;
  p->coeff = inv.v;
  p->have = have;
  *out = p;
  return 0;
}

static void del(FakePlan* p) { delete p; }

#define CHECK(cond)                                                     \
  do {                                                                  \
    if (!(cond)) {                                                      \
      std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond);       \
      std::exit(1);                                                     \
    }                                                                   \
  } while (0)

static std::vector<int> random_set(std::mt19937_64& rng, int need, int total) {
  std::vector<int> all(total);
  for (int i = 0; i < total; ++i) all[i] = i;
  std::shuffle(all.begin(), all.end(), rng);
  std::vector<int> have(all.begin(), all.begin() + need);
  std::sort(have.begin(), have.end());  // the caller's order (multi_store.go:218-235)
  return have;
}

// inv * code rows == I, exactly: the cached plan is the real inverse.
static bool is_inverse(const FakePlan& p, int need) {
  std::vector<uint32_t> row;
  for (int i = 0; i < need; ++i)
    for (int j = 0; j < need; ++j) {
      uint64_t acc = 0;
      for (int t = 0; t < need; ++t) {
        code_row(need, p.have[t], &row);
        acc = (acc + (uint64_t)p.coeff[(size_t)i * need + t] * row[j] % kP) % kP;
      }
      if (acc != (i == j ? 1u : 0u)) return false;
    }
  return true;
}

int main() {
  const int need = 20, total = 40;
  {  // 10,000 distinct survivor sets, cap 256
    LruCache<Key, FakePlan> cache(256);
    std::mt19937_64 rng(2040);
    std::set<std::vector<int>> seen;
    size_t max_live = 0;
    while (seen.size() < 10000) {
      std::vector<int> have = random_set(rng, need, total);
      if (!seen.insert(have).second) continue;
      std::shared_ptr<FakePlan> p;
      CHECK(cache.get(Key{0, 'R', need, 0, have}, &p, build, del) == 0);
      CHECK(p->have == have);
      max_live = std::max(max_live, cache.size());
    }
    CHECK(max_live == 256 && cache.size() == 256);
    CHECK(cache.misses() == 10000 && cache.evictions() == 10000 - 256);
    CHECK(g_tables.load() == 256);  // every evicted table released
    // An evicted set is rebuilt on demand into a correct inverse.
    std::shared_ptr<FakePlan> p;
    const std::vector<int> last = *seen.begin();
    CHECK(cache.get(Key{0, 'R', need, 0, last}, &p, build, del) == 0);
    CHECK(is_inverse(*p, need));
    cache.set_capacity(8);
    CHECK(cache.size() == 8 && g_tables.load() == 8);
    p.reset();
    cache.clear();
    CHECK(g_tables.load() == 0);
    std::printf("ok   TestPlanCacheBounded (10000 distinct 20/40 survivor sets, cap 256)\n");
  }
  {  // a singular set (duplicate index) fails and caches nothing
    LruCache<Key, FakePlan> cache(4);
    std::shared_ptr<FakePlan> p;
    std::vector<int> dup(need);
    for (int i = 0; i < need; ++i) dup[i] = i;
    dup[1] = 0;
    CHECK(cache.get(Key{0, 'R', need, 0, dup}, &p, build, del) == (int)Status::SingularNonzero);
    CHECK(!p && cache.size() == 0 && g_tables.load() == 0);
    std::printf("ok   TestPlanCacheFailedBuild\n");
  }
  {  // concurrent callers, cap 16: held plans outlive their eviction
    LruCache<Key, FakePlan> cache(16);
    std::atomic<int> bad{0};
    std::vector<std::thread> ts;
    for (int t = 0; t < 8; ++t)
      ts.emplace_back([&, t] {
        std::mt19937_64 rng(100 + t);
        for (int it = 0; it < 400; ++it) {
          const std::vector<int> have = random_set(rng, 8, 16);
          std::shared_ptr<FakePlan> p;
          if (cache.get(Key{t % 2, 'R', 8, 0, have}, &p, build, del) != 0) {
            ++bad;
            continue;
          }
          std::this_thread::yield();  // others evict meanwhile
          if (p->have != have || !is_inverse(*p, 8)) ++bad;
        }
      });
    for (auto& th : ts) th.join();
    CHECK(bad.load() == 0);
    CHECK(cache.size() <= 16 && g_tables.load() == (long)cache.size());
    std::printf("ok   TestPlanCacheConcurrent (8 threads, cap 16)\n");
  }
  {  // slow builds of different keys overlap; the builder never holds the lock
    LruCache<Key, FakePlan> cache(64);
    std::atomic<int> builds{0}, locked_builds{0};
    auto slow = [&](const Key& key, FakePlan** out) {
      if (cache.held_by_this_thread()) ++locked_builds;
      ++builds;
      std::this_thread::sleep_for(std::chrono::milliseconds(50));
      return build(key, out);
    };
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> ts;
    for (int t = 0; t < 8; ++t)
      ts.emplace_back([&, t] {
        std::vector<int> have(8);
        for (int i = 0; i < 8; ++i) have[i] = i + (i >= t ? 1 : 0);  // 8 distinct survivor sets of 8/9
        std::shared_ptr<FakePlan> p;
        CHECK(cache.get(Key{t, 'R', 8, 0, have}, &p, slow, del) == 0 && p->have == have);
      });
    for (auto& th : ts) th.join();
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    CHECK(builds.load() == 8 && locked_builds.load() == 0);
    CHECK(ms < 200.0);  // serialised builds would take >= 400 ms
    std::printf("ok   TestPlanCacheBuildsOutsideLock (8 x 50 ms builds in %.0f ms)\n", ms);
  }
  {  // one key, 8 concurrent callers: one build, one shared value
    LruCache<Key, FakePlan> cache(4);
    std::atomic<int> builds{0};
    auto slow = [&](const Key& key, FakePlan** out) {
      ++builds;
      std::this_thread::sleep_for(std::chrono::milliseconds(30));
      return build(key, out);
    };
    std::vector<int> have = {0, 1, 2, 3, 4, 5, 6, 8};
    std::vector<std::shared_ptr<FakePlan>> got(8);
    std::vector<std::thread> ts;
    for (int t = 0; t < 8; ++t)
      ts.emplace_back([&, t] { CHECK(cache.get(Key{0, 'R', 8, 0, have}, &got[t], slow, del) == 0); });
    for (auto& th : ts) th.join();
    CHECK(builds.load() == 1);
    for (int t = 1; t < 8; ++t) CHECK(got[t] == got[0]);
    // waiters on a failed build fail too (each retrying as the builder)
    std::vector<int> dup = {0, 0, 2, 3, 4, 5, 6, 7};
    std::atomic<int> fails{0};
    ts.clear();
    for (int t = 0; t < 4; ++t)
      ts.emplace_back([&] {
        std::shared_ptr<FakePlan> p;
        if (cache.get(Key{0, 'R', 8, 0, dup}, &p, slow, del) == (int)Status::SingularNonzero && !p) ++fails;
      });
    for (auto& th : ts) th.join();
    CHECK(fails.load() == 4 && cache.size() == 1);
    std::printf("ok   TestPlanCacheSharedBuild (8 callers, 1 build; failed builds cache nothing)\n");
  }
  {  // eviction releases values after the lock is dropped
    LruCache<Key, FakePlan> cache(2);
    std::atomic<int> deleted{0}, locked{0};
    auto checked_del = [&](FakePlan* p) {
      if (cache.held_by_this_thread()) ++locked;
      ++deleted;
      delete p;
    };
    std::mt19937_64 rng(7);
    std::set<std::vector<int>> seen;
    while (seen.size() < 50) {
      const std::vector<int> have = random_set(rng, 6, 12);
      if (!seen.insert(have).second) continue;
      std::shared_ptr<FakePlan> p;
      CHECK(cache.get(Key{0, 'R', 6, 0, have}, &p, build, checked_del) == 0);
    }
    cache.set_capacity(1);
    cache.clear();
    CHECK(deleted.load() == 50 && locked.load() == 0 && g_tables.load() == 0);
    std::printf("ok   TestPlanCacheReleaseOutsideLock (50 evictions, no deleter under the lock)\n");
  }
  {  // a build that throws (bad_alloc in a host table): waiters wake, nothing cached, key usable again
    LruCache<Key, FakePlan> cache(4);
    std::atomic<int> calls{0}, threw{0};
    auto throwing = [&](const Key& key, FakePlan** out) -> int {
      if (calls.fetch_add(1) < 3) {
        std::this_thread::sleep_for(std::chrono::milliseconds(30));
        throw std::bad_alloc();
      }
      return build(key, out);
    };
    std::vector<int> have = {0, 1, 2, 3, 4, 5, 6, 9};
    std::vector<std::thread> ts;
    for (int t = 0; t < 6; ++t)
      ts.emplace_back([&] {
        std::shared_ptr<FakePlan> p;
        const int rc = cache.get(Key{0, 'R', 8, 0, have}, &p, throwing, del);
        if (rc == LruCache<Key, FakePlan>::kBuildThrew && !p) ++threw;
        else CHECK(rc == 0 && p && p->have == have);
      });
    for (auto& th : ts) th.join();  // a waiter left blocked forever would hang here
    CHECK(threw.load() >= 1 && threw.load() <= 3);
    std::shared_ptr<FakePlan> p;
    CHECK(cache.get(Key{0, 'R', 8, 0, have}, &p, throwing, del) == 0 && is_inverse(*p, 8));
    std::printf("ok   TestPlanCacheBuildThrows (%d of 6 callers saw the exception, none blocked)\n", threw.load());
  }
  std::printf("7/7 passed\n");
  return 0;
}
