// Chunk and object digests (digest.hpp): SHA-256 with the x86 SHA extensions
// or a portable loop, FNV-1a-64, and the digest thread pool.
#include "digest.hpp"
#include "host_copy.hpp"

#include <cpuid.h>
#include <immintrin.h>
#include <sched.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

namespace slime {

struct DigestTask {
  std::function<void(size_t)> fn;
  size_t n = 0;
  std::atomic<size_t> next{0};
  size_t done = 0;  // guarded by the pool's mutex
};

namespace {

// FIPS 180-4 §4.2.2 and §5.3.3 (derived here with exact integer roots of the
// first 64 primes; checked by the NIST vectors in tests/test_digest.py).
alignas(16) const uint32_t kK[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2,
};
const uint32_t kH0[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                         0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};

inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
inline uint32_t load_be32(const uint8_t* p) {
  return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
}

void blocks_portable(uint32_t h[8], const uint8_t* p, size_t nb) {
  for (; nb; --nb, p += 64) {
    uint32_t w[64];
    for (int i = 0; i < 16; ++i) w[i] = load_be32(p + 4 * i);
    for (int i = 16; i < 64; ++i) {
      const uint32_t s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
      const uint32_t s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
      w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int i = 0; i < 64; ++i) {
      const uint32_t t1 = hh + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) + kK[i] + w[i];
      const uint32_t t2 = (rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
      hh = g, g = f, f = e, e = d + t1, d = c, c = b, b = a, a = t1 + t2;
    }
    h[0] += a, h[1] += b, h[2] += c, h[3] += d, h[4] += e, h[5] += f, h[6] += g, h[7] += hh;
  }
}

// SHA extensions: the state lives as (A,B,E,F) and (C,D,G,H); each
// sha256rnds2 does two rounds, msg1/msg2 extend the schedule four words at a time.
__attribute__((target("sha,sse4.1,ssse3"))) void blocks_shani(uint32_t h[8], const uint8_t* p, size_t nb) {
  const __m128i bswap = _mm_set_epi64x(0x0c0d0e0f08090a0bll, 0x0405060700010203ll);
  __m128i t = _mm_shuffle_epi32(_mm_loadu_si128((const __m128i*)&h[0]), 0xB1);  // C D A B
  __m128i s1 = _mm_shuffle_epi32(_mm_loadu_si128((const __m128i*)&h[4]), 0x1B); // H G F E
  __m128i s0 = _mm_alignr_epi8(t, s1, 8);                                        // A B E F
  s1 = _mm_blend_epi16(s1, t, 0xF0);                                             // C D G H
  for (; nb; --nb, p += 64) {
    const __m128i save0 = s0, save1 = s1;
    __m128i m[4];
#pragma GCC unroll 16
    for (int g = 0; g < 16; ++g) {
      __m128i& w = m[g & 3];
      if (g < 4) {
        w = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(p + 16 * g)), bswap);
      } else {
        // W[t..t+3] from groups g-4 (w), g-3, g-2, g-1
        const __m128i x = _mm_add_epi32(_mm_sha256msg1_epu32(w, m[(g + 1) & 3]),
                                        _mm_alignr_epi8(m[(g + 3) & 3], m[(g + 2) & 3], 4));
        w = _mm_sha256msg2_epu32(x, m[(g + 3) & 3]);
      }
      __m128i k = _mm_add_epi32(w, _mm_load_si128((const __m128i*)&kK[4 * g]));
      s1 = _mm_sha256rnds2_epu32(s1, s0, k);
      s0 = _mm_sha256rnds2_epu32(s0, s1, _mm_shuffle_epi32(k, 0x0E));
    }
    s0 = _mm_add_epi32(s0, save0);
    s1 = _mm_add_epi32(s1, save1);
  }
  t = _mm_shuffle_epi32(s0, 0x1B);                                   // F E B A
  s1 = _mm_shuffle_epi32(s1, 0xB1);                                  // D C H G
  _mm_storeu_si128((__m128i*)&h[0], _mm_blend_epi16(t, s1, 0xF0));   // A B C D
  _mm_storeu_si128((__m128i*)&h[4], _mm_alignr_epi8(s1, t, 8));      // E F G H
}

bool detect_sha() {
  unsigned a, b, c, d;
  if (!__get_cpuid(1, &a, &b, &c, &d)) return false;
  const bool sse = (c >> 19 & 1) && (c >> 9 & 1);  // SSE4.1, SSSE3
  if (!__get_cpuid_count(7, 0, &a, &b, &c, &d)) return false;
  const char* e = getenv("SLIME_RS_SHA_NI");  // "0": force the portable loop (tests)
  return sse && (b >> 29 & 1) && !(e && e[0] == '0');
}

void blocks(uint32_t h[8], const uint8_t* p, size_t nb) {
  static const bool ni = detect_sha();
  if (ni)
    blocks_shani(h, p, nb);
  else
    blocks_portable(h, p, nb);
}

// ---- digest pool ---------------------------------------------------------------

class Pool {
 public:
  explicit Pool(int nthreads) {
    for (int i = 0; i < nthreads; ++i) th_.emplace_back([this] { worker(); });
  }
  int threads() const { return (int)th_.size(); }

  // Queue t for the workers; the caller goes on with other work.
  void start(DigestTask* t) {
    if (th_.empty() || t->n == 0) return;
    {
      std::lock_guard<std::mutex> lk(mu_);
      jobs_.push_back(t);
    }
    cv_.notify_all();
  }
  // Claim what is left of t on this thread, then wait for the workers' part.
  void wait(DigestTask* t) {
    size_t did = 0;
    for (size_t i; (i = t->next.fetch_add(1)) < t->n; ++did) t->fn(i);
    std::unique_lock<std::mutex> lk(mu_);
    auto it = std::find(jobs_.begin(), jobs_.end(), t);
    if (it != jobs_.end()) jobs_.erase(it);
    t->done += did;
    done_cv_.wait(lk, [&] { return t->done == t->n; });
  }

 private:
  void worker() {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [&] { return !jobs_.empty(); });
      DigestTask* t = jobs_.front();
      const size_t i = t->next.fetch_add(1);
      if (i >= t->n) {  // every index claimed: the job leaves the queue
        jobs_.pop_front();
        continue;
      }
      lk.unlock();
      t->fn(i);
      lk.lock();
      if (++t->done == t->n) done_cv_.notify_all();
    }
  }

  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  std::deque<DigestTask*> jobs_;  // jobs with indices left to claim
  std::vector<std::thread> th_;
};

int default_threads() {
  const char* s = getenv("SLIME_RS_DIGEST_THREADS");
  if (s && *s) return std::max(0, std::min(atoi(s), 256));
  return std::max(0, std::min(usable_cpus(), 16) - 1);
}

Pool& pool() {
  static Pool* p = new Pool(default_threads());  // leaked: workers outlive static destructors
  return *p;
}

}  // namespace

Sha256::Sha256() { memcpy(h_, kH0, sizeof(h_)); }

void Sha256::update(const void* data, size_t n) {
  const uint8_t* p = (const uint8_t*)data;
  total_ += n;
  if (buffered_) {
    const size_t take = std::min(n, 64 - buffered_);
    memcpy(buf_ + buffered_, p, take);
    buffered_ += take, p += take, n -= take;
    if (buffered_ < 64) return;
    blocks(h_, buf_, 1);
    buffered_ = 0;
  }
  if (n >= 64) {
    blocks(h_, p, n / 64);
    p += n & ~(size_t)63;
    n &= 63;
  }
  memcpy(buf_, p, n);
  buffered_ = n;
}

void Sha256::final(uint8_t out[32]) {
  const uint64_t bits = total_ * 8;
  uint8_t pad[72] = {0x80};
  const size_t padlen = (buffered_ < 56 ? 56 : 120) - buffered_;
  for (int i = 0; i < 8; ++i) pad[padlen + i] = (uint8_t)(bits >> (56 - 8 * i));
  update(pad, padlen + 8);
  for (int i = 0; i < 8; ++i)
    for (int j = 0; j < 4; ++j) out[4 * i + j] = (uint8_t)(h_[i] >> (24 - 8 * j));
}

bool sha_extensions() {
  static const bool ni = detect_sha();
  return ni;
}

uint64_t fnv1a64(uint64_t h, const void* data, size_t n) {
  const uint8_t* p = (const uint8_t*)data;
  constexpr uint64_t prime = 0x100000001b3ull;
  for (size_t i = 0; i < n; ++i) h = (h ^ p[i]) * prime;
  return h;
}

void digest_parallel(size_t n, const std::function<void(size_t)>& fn) {
  DigestJob job(n, fn);
  job.wait();
}

DigestJob::DigestJob(size_t n, std::function<void(size_t)> fn) : task_(new DigestTask) {
  task_->fn = std::move(fn);
  task_->n = n;
  pool().start(task_.get());
}

void DigestJob::wait() {
  if (task_ && !waited_) pool().wait(task_.get());
  waited_ = true;
}

DigestJob::~DigestJob() { wait(); }

int digest_threads() { return pool().threads(); }

// ---- writeChunks digests ---------------------------------------------------------

namespace {
constexpr uint64_t kSegment = 1u << 20;  // parity bytes hashed per hold of the buffers

void be64(uint64_t v, uint8_t* out) {
  for (int i = 0; i < 8; ++i) out[i] = (uint8_t)(v >> (56 - 8 * i));
}
}  // namespace

WriteChunkDigests::WriteChunkDigests(const uint8_t* data, uint64_t size, int need, int total, uint64_t chunk,
                                     uint8_t* const* chunks, uint8_t* sha_out, uint8_t* hdr_out)
    : data_(data), size_(size), chunk_(chunk), need_(need), chunks_(chunks), sha_out_(sha_out),
      hdr_out_(hdr_out) {
  job_.reset(new DigestJob((size_t)total, [this](size_t i) { run(i); }));
}

WriteChunkDigests::~WriteChunkDigests() {
  abort();
  finish();
}

void WriteChunkDigests::parity_ready(uint64_t bytes) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    ready_ = bytes < chunk_ ? bytes : chunk_;
  }
  cv_.notify_all();
}

void WriteChunkDigests::parity_rewrite() {
  std::unique_lock<std::mutex> lk(mu_);
  ++epoch_;
  ready_ = 0;
  cv_.notify_all();
  cv_.wait(lk, [&] { return readers_ == 0; });
}

void WriteChunkDigests::finalize(uint32_t mapping) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    mapping_ = mapping;
    final_ = true;
  }
  cv_.notify_all();
}

void WriteChunkDigests::abort() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    aborted_ = true;
  }
  cv_.notify_all();
}

void WriteChunkDigests::finish() {
  if (job_) job_->wait();
}

void WriteChunkDigests::run(size_t i) {
  uint8_t* sha = sha_out_ + 32 * i;
  uint8_t* hdr = hdr_out_ ? hdr_out_ + 8 * i : nullptr;
  if ((int)i < need_)
    data_chunk((int)i, sha, hdr);
  else
    parity_chunk((int)i, sha, hdr);
}

// Bytes of data chunk j past the object's own: zeros to the end of the
// object's last word, then BE(m) words (map.go:103-113 of splitVector's zero
// symbols, multi_store.go:279-296).
void WriteChunkDigests::tail(int j, uint32_t m, const std::function<void(const uint8_t*, size_t)>& sink) const {
  const uint64_t lo = (uint64_t)j * chunk_, hi = lo + chunk_;
  const uint64_t body = size_ > lo ? std::min(size_, hi) - lo : 0;
  const uint64_t word_end = (size_ + 3) & ~(uint64_t)3;
  const uint64_t zero_end = word_end > lo ? std::min(word_end, hi) - lo : 0;
  if (zero_end > body) {
    static const uint8_t zeros[4] = {0, 0, 0, 0};
    sink(zeros, zero_end - body);
  }
  uint64_t left = chunk_ - std::max(body, zero_end);
  if (!left) return;
  uint8_t pat[4096];
  for (int b = 0; b < 4096; b += 4)
    pat[b] = (uint8_t)(m >> 24), pat[b + 1] = (uint8_t)(m >> 16), pat[b + 2] = (uint8_t)(m >> 8), pat[b + 3] = (uint8_t)m;
  for (; left; left -= std::min<uint64_t>(left, sizeof(pat))) sink(pat, std::min<uint64_t>(left, sizeof(pat)));
}

void WriteChunkDigests::data_chunk(int j, uint8_t* sha_out, uint8_t* hdr) {
  const uint64_t lo = (uint64_t)j * chunk_;
  const uint64_t body = size_ > lo ? std::min(size_, lo + chunk_) - lo : 0;
  Sha256 sha;
  if (body) sha.update(data_ + lo, body);
  uint32_t m;
  {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return final_ || aborted_; });
    if (aborted_) return;
    m = mapping_;
  }
  tail(j, m, [&](const uint8_t* p, size_t n) { sha.update(p, n); });
  sha.final(sha_out);
  if (hdr) {
    uint64_t h = fnv1a64(kFnv64Offset, sha_out, 32);
    if (body) h = fnv1a64(h, data_ + lo, body);
    tail(j, m, [&](const uint8_t* p, size_t n) { h = fnv1a64(h, p, n); });
    be64(h, hdr);
  }
}

void WriteChunkDigests::parity_chunk(int i, uint8_t* sha_out, uint8_t* hdr) {
  const uint8_t* buf = chunks_[i];
  Sha256 sha;
  uint64_t done = 0;
  std::unique_lock<std::mutex> lk(mu_);
  uint64_t epoch = epoch_;
  for (;;) {
    cv_.wait(lk, [&] { return aborted_ || epoch_ != epoch || ready_ > done || (final_ && done == chunk_); });
    if (aborted_) return;
    if (epoch_ != epoch) {  // rewritten: start over
      sha = Sha256();
      done = 0;
      epoch = epoch_;
      continue;
    }
    if (ready_ <= done) break;  // final and complete
    const uint64_t hi = std::min(ready_, done + kSegment);
    ++readers_;
    lk.unlock();
    sha.update(buf + done, hi - done);
    lk.lock();
    if (--readers_ == 0) cv_.notify_all();
    if (epoch_ == epoch) done = hi;
  }
  lk.unlock();
  sha.final(sha_out);
  if (hdr) be64(fnv1a64(fnv1a64(kFnv64Offset, sha_out, 32), buf, chunk_), hdr);
}

}  // namespace slime
