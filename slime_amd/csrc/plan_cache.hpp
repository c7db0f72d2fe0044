// Bounded, thread-safe LRU of shared values: the recovery-plan cache of the
// host entry points (reference: the matrices RecoverData
// inverts per call, internal/rs/vector.go:69-77, and the unbounded memo of
// ParityMatrixCached, internal/rs/matrixcache.go:7-29).
//
// A device plan is keyed by (device, kind, shape, survivor set).  The
// reference's maximum code (100 shards) has C(100,50) survivor sets, so the
// cache must forget: past `capacity` entries the least recently used one is
// dropped.  Values are shared_ptrs: a caller that got a plan keeps it alive
// until its own call returns, so an entry evicted by another thread is freed
// (its device table released by the value's deleter) only after the last
// in-flight user lets go.  Host-only header; tests/cpp/plan_cache_test.cpp
// drives it on the CPU.
// Locking (reference: matrixcache.go:7-29 builds outside its read lock): the
// cache's mutex guards only the index and the LRU order.  A miss inserts a
// pending slot and builds the value OUTSIDE the lock -- a device plan's build
// is a hipMalloc plus a synchronous table upload -- while later callers of the
// same key wait on that slot alone, and callers of other keys (other devices,
// other survivor sets) go on.  Evicted values are released after the lock is
// dropped, so a deleter that frees device memory (hipFree synchronises the
// device) never stalls the other callers.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <atomic>
#include <condition_variable>
#include <list>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <utility>
#include <vector>

namespace slime {

template <class Key, class Val>
class LruCache {
 public:
  explicit LruCache(size_t capacity) : cap_(capacity ? capacity : 1) {}

  // Status get() returns when make() threw (e.g. std::bad_alloc from a host
  // table): the build counts as failed, like a nonzero status.
  static constexpr int kBuildThrew = -2;

  // The value for `key`: cached, or built by make(key, &raw) (status int, 0 =
  // ok, ownership of raw passes to the cache with `del` as its deleter).  On
  // a failed build -- a nonzero status or an exception (kBuildThrew) --
  // nothing is cached, every caller waiting on that build is woken, and the
  // failure is returned; the waiters then build it themselves.
  template <class Make, class Del>
  int get(const Key& key, std::shared_ptr<Val>* out, Make&& make, Del del) {
    for (;;) {
      std::shared_ptr<Slot> slot;
      bool build = false;
      std::vector<std::shared_ptr<Slot>> dropped;  // released after the lock
      {
        Guard lk(this);
        auto it = index_.find(key);
        if (it != index_.end()) {
          order_.splice(order_.begin(), order_, it->second);  // most recent first
          ++hits_;
          slot = it->second->second;
        } else {
          ++misses_;
          slot = std::make_shared<Slot>();
          order_.emplace_front(key, slot);
          index_[key] = order_.begin();
          build = true;
          trim(&dropped);
        }
      }
      dropped.clear();
      if (build) {
        Val* raw = nullptr;
        int rc;
        try {
          rc = make(key, &raw);
        } catch (...) {
          rc = kBuildThrew;
          raw = nullptr;
        }
        std::shared_ptr<Val> v;
        if (rc == 0) {
          try {
            v = std::shared_ptr<Val>(raw, del);  // on bad_alloc the constructor calls del(raw)
          } catch (...) {
            rc = kBuildThrew;
          }
        }
        {
          std::lock_guard<std::mutex> sl(slot->mu);
          slot->value = v;
          slot->rc = rc;
          slot->ready = true;
        }
        slot->cv.notify_all();
        if (rc) {  // forget the failed slot (unless evicted or replaced meanwhile)
          std::shared_ptr<Slot> gone;
          Guard lk(this);
          auto it = index_.find(key);
          if (it != index_.end() && it->second->second == slot) {
            gone = std::move(it->second->second);
            order_.erase(it->second);
            index_.erase(it);
          }
          lk.unlock();
          return rc;
        }
        *out = std::move(v);
        return 0;
      }
      std::unique_lock<std::mutex> sl(slot->mu);
      slot->cv.wait(sl, [&] { return slot->ready; });
      if (slot->rc == 0) {
        *out = slot->value;
        return 0;
      }
      // The build this caller waited on failed: try again as the builder.
    }
  }

  void set_capacity(size_t cap) {
    std::vector<std::shared_ptr<Slot>> dropped;
    Guard lk(this);
    cap_ = cap ? cap : 1;
    trim(&dropped);
    lk.unlock();
  }
  size_t capacity() const {
    Guard lk(this);
    return cap_;
  }
  size_t size() const {
    Guard lk(this);
    return index_.size();
  }
  uint64_t evictions() const {
    Guard lk(this);
    return evictions_;
  }
  uint64_t hits() const {
    Guard lk(this);
    return hits_;
  }
  uint64_t misses() const {
    Guard lk(this);
    return misses_;
  }
  void clear() {
    std::list<Entry> old;
    Guard lk(this);
    old.swap(order_);
    index_.clear();
    lk.unlock();  // values die with `old`, outside the lock
  }
  // Whether the calling thread holds the cache's lock (tests: deleters and
  // builders must run without it).
  bool held_by_this_thread() const { return owner_.load() == std::this_thread::get_id(); }

 private:
  struct Slot {
    std::mutex mu;
    std::condition_variable cv;
    bool ready = false;
    int rc = 0;
    std::shared_ptr<Val> value;
  };
  using Entry = std::pair<Key, std::shared_ptr<Slot>>;

  // The cache lock, recording its owner (held_by_this_thread).
  class Guard {
   public:
    explicit Guard(const LruCache* c) : c_(c) {
      c_->mu_.lock();
      c_->owner_.store(std::this_thread::get_id());
      locked_ = true;
    }
    void unlock() {
      if (!locked_) return;
      c_->owner_.store(std::thread::id());
      c_->mu_.unlock();
      locked_ = false;
    }
    ~Guard() { unlock(); }

   private:
    const LruCache* c_;
    bool locked_ = false;
  };

  void trim(std::vector<std::shared_ptr<Slot>>* dropped) {  // mu_ held
    while (index_.size() > cap_) {
      index_.erase(order_.back().first);
      dropped->push_back(std::move(order_.back().second));  // dies after the unlock unless a caller holds it
      order_.pop_back();
      ++evictions_;
    }
  }

  mutable std::mutex mu_;
  mutable std::atomic<std::thread::id> owner_{};
  size_t cap_;
  std::list<Entry> order_;
  std::map<Key, typename std::list<Entry>::iterator> index_;
  uint64_t hits_ = 0, misses_ = 0, evictions_ = 0;
};

}  // namespace slime
