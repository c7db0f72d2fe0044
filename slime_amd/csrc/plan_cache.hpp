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
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <list>
#include <map>
#include <memory>
#include <mutex>
#include <utility>

namespace slime {

template <class Key, class Val>
class LruCache {
 public:
  explicit LruCache(size_t capacity) : cap_(capacity ? capacity : 1) {}

  // The value for `key`: cached, or built by make(key, &raw) (status int, 0 =
  // ok, ownership of raw passes to the cache with `del` as its deleter).  On
  // a failed build nothing is cached and make's status is returned.
  template <class Make, class Del>
  int get(const Key& key, std::shared_ptr<Val>* out, Make&& make, Del del) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = index_.find(key);
    if (it != index_.end()) {
      order_.splice(order_.begin(), order_, it->second);  // most recent first
      ++hits_;
      *out = it->second->second;
      return 0;
    }
    ++misses_;
    Val* raw = nullptr;
    if (int rc = make(key, &raw)) return rc;
    std::shared_ptr<Val> v(raw, del);
    order_.emplace_front(key, v);
    index_[key] = order_.begin();
    trim();
    *out = std::move(v);
    return 0;
  }

  void set_capacity(size_t cap) {
    std::lock_guard<std::mutex> lk(mu_);
    cap_ = cap ? cap : 1;
    trim();
  }
  size_t capacity() const {
    std::lock_guard<std::mutex> lk(mu_);
    return cap_;
  }
  size_t size() const {
    std::lock_guard<std::mutex> lk(mu_);
    return index_.size();
  }
  uint64_t evictions() const {
    std::lock_guard<std::mutex> lk(mu_);
    return evictions_;
  }
  uint64_t hits() const {
    std::lock_guard<std::mutex> lk(mu_);
    return hits_;
  }
  uint64_t misses() const {
    std::lock_guard<std::mutex> lk(mu_);
    return misses_;
  }
  void clear() {
    std::lock_guard<std::mutex> lk(mu_);
    order_.clear();
    index_.clear();
  }

 private:
  void trim() {  // mu_ held
    while (index_.size() > cap_) {
      index_.erase(order_.back().first);
      order_.pop_back();  // the value dies here unless a caller still holds it
      ++evictions_;
    }
  }

  using Entry = std::pair<Key, std::shared_ptr<Val>>;
  mutable std::mutex mu_;
  size_t cap_;
  std::list<Entry> order_;
  std::map<Key, typename std::list<Entry>::iterator> index_;
  uint64_t hits_ = 0, misses_ = 0, evictions_ = 0;
};

}  // namespace slime
