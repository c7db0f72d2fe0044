// Persistent host copy pool (host_copy.hpp).
#include "host_copy.hpp"

#include <emmintrin.h>
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

namespace slime {
namespace {

// Work pieces of 64..512 KiB, about four per thread (a fixed 512 KiB left
// most of the pool idle on a window's ~1 MiB of outputs).
constexpr size_t kPieceMax = 512u << 10, kPieceMin = 64u << 10;
// Copies below 2 MiB stay on the caller: a wake-up costs more than it saves
// there (1 MiB host calls ran 10-20% slower with a 512 KiB threshold,
// profiles/r04/s18_serialab).
constexpr size_t kSerialBelow = 2u << 20;
size_t serial_below() { return kSerialBelow; }
// After a job a worker spins this long for the next one before it sleeps.
// A host call posts one job per window (8-16 MiB, a fraction of a ms of
// copying); a worker that went to sleep between windows can take longer to
// wake than the caller needs to copy the whole window alone.  That is what
// the slow runs of the object entry points were: the same rate as with no
// workers at all (10 / 7 GiB/s against 28 / 24, tools/host_diag.py,
// profiles/r02/s8_hostdiag).
constexpr std::chrono::microseconds kSpin{3000};

struct Job {
  void (*fn)(const void* ctx, size_t piece) = nullptr;
  const void* ctx = nullptr;
  size_t n = 0;
  std::atomic<size_t> next{0};
  size_t done = 0;  // guarded by Pool::mu
  int active = 0;   // workers holding a pointer to this job (guarded)
};

// Streaming (non-temporal) copy: the staged rows are written once and not
// read again by this core, so bypassing the cache saves the read-for-ownership
// of every destination line.
void stream_copy(void* dst, const void* src, size_t n) {
  char* d = (char*)dst;
  const char* s = (const char*)src;
  const size_t head = (16 - ((uintptr_t)d & 15)) & 15;
  if (n < 256 || head > n) {
    memcpy(d, s, n);
    return;
  }
  memcpy(d, s, head);
  d += head, s += head, n -= head;
  size_t i = 0;
  for (; i + 64 <= n; i += 64) {
    const __m128i a = _mm_loadu_si128((const __m128i*)(s + i));
    const __m128i b = _mm_loadu_si128((const __m128i*)(s + i + 16));
    const __m128i c = _mm_loadu_si128((const __m128i*)(s + i + 32));
    const __m128i e = _mm_loadu_si128((const __m128i*)(s + i + 48));
    _mm_stream_si128((__m128i*)(d + i), a);
    _mm_stream_si128((__m128i*)(d + i + 16), b);
    _mm_stream_si128((__m128i*)(d + i + 32), c);
    _mm_stream_si128((__m128i*)(d + i + 48), e);
  }
  memcpy(d + i, s + i, n - i);
  _mm_sfence();
}

void copy_piece(const CopyItem& it) { stream_copy(it.dst, it.src, it.bytes); }

size_t drain(Job* j) {
  size_t did = 0;
  for (size_t i; (i = j->next.fetch_add(1, std::memory_order_relaxed)) < j->n; ++did) j->fn(j->ctx, i);
  return did;
}

// Jobs of several callers at once (concurrent host calls of a proxy, main.go:107-109):
// each caller posts its job and drains it itself; workers help the oldest
// job that still has unclaimed pieces.
class Pool {
 public:
  explicit Pool(int nthreads) {
    for (int t = 0; t < nthreads; ++t) th_.emplace_back([this] { worker(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_.store(true);
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int threads() const { return (int)th_.size(); }

  void run(size_t n, void (*fn)(const void*, size_t), const void* ctx) {
    if (th_.empty() || n == 1) {
      for (size_t i = 0; i < n; ++i) fn(ctx, i);
      return;
    }
    Job j;
    j.fn = fn;
    j.ctx = ctx;
    j.n = n;
    {
      std::lock_guard<std::mutex> lk(mu_);
      jobs_.push_back(&j);
      posted_.fetch_add(1, std::memory_order_release);
    }
    cv_.notify_all();
    const size_t did = drain(&j);
    std::unique_lock<std::mutex> lk(mu_);
    auto it = std::find(jobs_.begin(), jobs_.end(), &j);
    if (it != jobs_.end()) jobs_.erase(it);
    j.done += did;
    done_cv_.wait(lk, [&] { return j.done == j.n && j.active == 0; });
  }

 private:
  // First queued job with pieces left; drops exhausted ones.  Needs mu_.
  Job* pick() {
    while (!jobs_.empty()) {
      Job* j = jobs_.front();
      if (j->next.load(std::memory_order_relaxed) < j->n) return j;
      jobs_.pop_front();
    }
    return nullptr;
  }

  void worker() {
    uint64_t seen = 0;
    for (;;) {
      // Hot wait: poll the job counter (pool state only, never a job) for kSpin.
      const auto deadline = std::chrono::steady_clock::now() + kSpin;
      bool timed_out = false;
      for (uint32_t it = 1; posted_.load(std::memory_order_acquire) == seen && !stop_.load(std::memory_order_relaxed);
           ++it) {
        _mm_pause();
        if ((it & 255) == 0 && std::chrono::steady_clock::now() > deadline) {
          timed_out = true;
          break;
        }
      }
      std::unique_lock<std::mutex> lk(mu_);
      Job* j = pick();
      if (!timed_out && !j && !stop_.load()) {  // a job came and went while this worker spun up: keep spinning
        seen = posted_.load(std::memory_order_relaxed);
        continue;
      }
      cv_.wait(lk, [&] { return stop_.load() || (j = pick()) != nullptr; });
      if (stop_.load()) return;
      seen = posted_.load(std::memory_order_relaxed);
      ++j->active;
      lk.unlock();
      const size_t did = drain(j);
      lk.lock();
      j->done += did;
      --j->active;
      if (j->done == j->n && j->active == 0) done_cv_.notify_all();
    }
  }

  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  std::deque<Job*> jobs_;            // posted jobs, oldest first (guarded by mu_)
  std::atomic<uint64_t> posted_{0};  // jobs posted so far (the spinners' signal)
  std::atomic<bool> stop_{false};
  std::vector<std::thread> th_;
};

int usable_cpus_uncached() {
  cpu_set_t set;
  int n = sched_getaffinity(0, sizeof(set), &set) == 0 ? CPU_COUNT(&set) : 1;
  if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char quota[32] = {0};
    long period = 0;
    if (fscanf(f, "%31s %ld", quota, &period) == 2 && strcmp(quota, "max") != 0 && period > 0) {
      const long q = (atol(quota) + period - 1) / period;
      if (q > 0 && q < n) n = (int)q;
    }
    fclose(f);
  }
  return n < 1 ? 1 : n;
}

// Workers beside the calling thread (env SLIME_RS_COPY_THREADS, 0..64).
// Default: half the usable CPUs, 1..8.  On the 16-CPU share of the GPU box
// 8 workers ran the host codec's MapFromGF 1.3-1.6x faster than 4
// (profiles/r04/s7_hostab); more CPUs than that are left to the caller's
// own concurrency (a storage server runs many calls at once).
int env_threads() {
  const char* s = getenv("SLIME_RS_COPY_THREADS");
  if (!s || !*s) return std::min(8, std::max(1, usable_cpus_uncached() / 2));
  const int v = atoi(s);
  return v < 0 ? 0 : (v > 64 ? 64 : v);
}

Pool& pool() {
  static Pool* p = new Pool(env_threads());  // intentionally leaked: workers outlive static destructors
  return *p;
}

}  // namespace

int copy_pool_threads() { return pool().threads(); }

// A container's share of a large host sees every CPU in its mask but may
// run only its quota.
int usable_cpus() {
  static const int n = usable_cpus_uncached();
  return n;
}

void parallel_pieces(size_t n, void (*fn)(const void* ctx, size_t piece), const void* ctx) {
  if (n) pool().run(n, fn, ctx);
}

void parallel_copy(const CopyItem* items, size_t n) {
  size_t total = 0;
  for (size_t i = 0; i < n; ++i) total += items[i].bytes;
  if (total < serial_below()) {
    for (size_t i = 0; i < n; ++i)
      if (items[i].bytes) memcpy(items[i].dst, items[i].src, items[i].bytes);
    return;
  }
  const size_t piece = std::min(kPieceMax, std::max(kPieceMin, total / (4 * (size_t)(copy_pool_threads() + 1))));
  std::vector<CopyItem> pieces;
  pieces.reserve(total / piece + n);
  for (size_t i = 0; i < n; ++i) {
    char* d = (char*)items[i].dst;
    const char* s = (const char*)items[i].src;
    for (size_t off = 0; off < items[i].bytes; off += piece)
      pieces.push_back({d + off, s + off, std::min(piece, items[i].bytes - off)});
  }
  parallel_pieces(
      pieces.size(), [](const void* ctx, size_t i) { copy_piece(((const CopyItem*)ctx)[i]); }, pieces.data());
}

}  // namespace slime
