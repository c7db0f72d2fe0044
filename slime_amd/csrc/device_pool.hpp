// Routing of host calls to devices (host-only; no HIP): which GPU a host
// entry point runs on, and the per-device free lists of the resources it
// reuses.  rs_capi.cpp instantiates these over the visible HIP devices;
// tests/cpp/device_pool_test.cpp drives the same code on the CPU with a fixed
// device count.
//
// The reference's callers are concurrent -- up to `parallel-requests` HTTP
// goroutines (main.go:107-109) plus scrubbers (multi.go:54-58) -- and objects
// are independent, so a call that names no device takes the
// allowed GPU with the fewest calls in flight (ties: round robin), spreading
// concurrent callers over the node with no data-path exchange.  A device named
// by the call (*_ex) or by the calling thread (slime_rs_select_device) is
// always honoured.  The allowed set is every visible device unless
// SLIME_RS_DEVICES lists some (e.g. "3" for a rank that owns GPU 3).
#pragma once
#include <stdint.h>
#include <stdlib.h>

#include <atomic>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <string>
#include <vector>

namespace slime {

constexpr int kAnyDevice = -1;

struct DevicePool {
  static constexpr int kMax = 64;
  std::atomic<int> inflight[kMax] = {};
  std::atomic<uint64_t> calls[kMax] = {};
  std::atomic<uint64_t> next{0};

  // Allowed devices among n visible: the SLIME_RS_DEVICES list (ordinals
  // below n, in order, duplicates dropped) or 0..n-1.  Empty if n == 0.
  static std::vector<int> allowed(int n, const char* spec) {
    std::vector<int> out;
    if (spec && *spec) {
      std::string s(spec);
      size_t i = 0;
      while (i < s.size()) {
        size_t j = s.find(',', i);
        if (j == std::string::npos) j = s.size();
        const std::string tok = s.substr(i, j - i);
        char* end = nullptr;
        const long v = strtol(tok.c_str(), &end, 10);
        if (!tok.empty() && end && *end == '\0' && v >= 0 && v < n && v < kMax) {
          bool dup = false;
          for (int d : out) dup |= d == (int)v;
          if (!dup) out.push_back((int)v);
        }
        i = j + 1;
      }
      if (!out.empty()) return out;
    }
    for (int d = 0; d < n && d < kMax; ++d) out.push_back(d);
    return out;
  }

  // The allowed device with the fewest calls in flight; ties go round robin.
  int pick(const std::vector<int>& devs) {
    const int n = (int)devs.size();
    const int start = (int)(next.fetch_add(1, std::memory_order_relaxed) % (uint64_t)n);
    int best = devs[start];
    for (int i = 1; i < n; ++i) {
      const int d = devs[(start + i) % n];
      if (inflight[d].load(std::memory_order_relaxed) < inflight[best].load(std::memory_order_relaxed)) best = d;
    }
    return best;
  }
};

// The device of one host call, held for the call's life: the call's explicit
// device, else the thread's selected device, else the pool's pick among
// `devs`.  The caller validates an explicit device first.
struct PoolLease {
  DevicePool* pool = nullptr;
  int device = -1;
  bool counted = false;
  void take(DevicePool& p, int call_device, int thread_device, const std::vector<int>& devs) {
    pool = &p;
    int want = call_device;
    if (want == kAnyDevice) want = thread_device;
    device = want != kAnyDevice ? want : p.pick(devs);
    if (device >= 0 && device < DevicePool::kMax) {
      counted = true;
      p.inflight[device].fetch_add(1, std::memory_order_relaxed);
      p.calls[device].fetch_add(1, std::memory_order_relaxed);
    }
  }
  // The call no longer counts as in flight on its device (idempotent; the
  // destructor calls it too).
  void release() {
    if (counted) pool->inflight[device].fetch_sub(1, std::memory_order_relaxed);
    counted = false;
  }
  ~PoolLease() { release(); }
};

// Per-device free list of reusable per-call resources (T has an int `device`
// member): most recently released first, so a caller's next call gets the
// resource its last call sized instead of cycling through every one a burst
// of concurrent calls once created.  take() returns nullptr when the device
// has none free (the caller creates one).
template <class T>
class PerDeviceFreeList {
 public:
  T* take(int device) {
    std::lock_guard<std::mutex> lk(mu_);
    for (size_t i = free_.size(); i-- > 0;) {
      if (free_[i]->device == device) {
        T* t = free_[i];
        free_.erase(free_.begin() + (long)i);
        return t;
      }
    }
    return nullptr;
  }
  void give(T* t) {
    std::lock_guard<std::mutex> lk(mu_);
    free_.push_back(t);
  }
  size_t size() const {
    std::lock_guard<std::mutex> lk(mu_);
    return free_.size();
  }

 private:
  mutable std::mutex mu_;
  std::vector<T*> free_;
};

// A fixed number of slots handed out in arrival order (rs_capi.cpp uses one
// for the process's concurrent host calls): enter() takes a free slot when
// nobody waits, else sleeps until leave() hands it the slot of a finishing
// caller -- a freed slot goes straight to the oldest waiter.
class HostCallSlots {
 public:
  explicit HostCallSlots(int n) : free_(n) {}
  void enter() {
    std::unique_lock<std::mutex> lk(mu_);
    if (free_ > 0 && waiting_.empty()) {
      --free_;
      return;
    }
    Waiter w;
    waiting_.push_back(&w);
    w.cv.wait(lk, [&] { return w.granted; });
  }
  size_t waiting() const {  // callers asleep in enter() (tests)
    std::lock_guard<std::mutex> lk(mu_);
    return waiting_.size();
  }
  void leave() {
    std::lock_guard<std::mutex> lk(mu_);
    if (waiting_.empty()) {
      ++free_;
      return;
    }
    Waiter* w = waiting_.front();  // the slot passes to the oldest waiter
    waiting_.pop_front();
    w->granted = true;
    w->cv.notify_one();  // under the lock: w lives on its waiter's stack until it sees `granted`
  }

 private:
  struct Waiter {
    std::condition_variable cv;
    bool granted = false;
  };
  mutable std::mutex mu_;
  std::deque<Waiter*> waiting_;
  int free_;
};

}  // namespace slime
