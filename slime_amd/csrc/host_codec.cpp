// Host byte<->symbol codec (host_codec.hpp).
#include "host_codec.hpp"

#include <immintrin.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>

#include <algorithm>
#include <atomic>

#include "host_copy.hpp"

namespace slime {
namespace {

constexpr uint32_t kP = 4294967291u;          // gf.MaxVal (map.go:7)
constexpr uint64_t kPieceWords = 128u << 10;  // 512 KiB of words per piece
constexpr uint64_t kSerialWords = 256u << 10; // up to 1 MiB of words: the caller alone

bool use_avx2() {
  static const bool on = [] {
    const char* e = getenv("SLIME_RS_CODEC_ISA");
    if (e && strcmp(e, "scalar") == 0) return false;
    return (bool)__builtin_cpu_supports("avx2");
  }();
  return on;
}

inline uint32_t be32(const uint8_t* p) {
  uint32_t w;
  memcpy(&w, p, 4);
  return __builtin_bswap32(w);
}

// ---- one piece of each pass: scalar and AVX2 forms ------------------------------

// out[i] = BE32(in + 4i) ^ n for nw whole words; returns the running maxima of
// the words (mx0) and of the words ^ 1<<31 (mx1) when track is set.
void pack_scalar(const uint8_t* in, uint64_t nw, uint32_t n, uint32_t* out, bool track, uint32_t* mx0,
                 uint32_t* mx1) {
  uint32_t a = *mx0, b = *mx1;
  for (uint64_t i = 0; i < nw; ++i) {
    const uint32_t w = be32(in + 4 * i);
    if (track) {
      a = std::max(a, w);
      b = std::max(b, w ^ 0x80000000u);
    }
    out[i] = w ^ n;
  }
  *mx0 = a, *mx1 = b;
}

__attribute__((target("avx2"))) inline __m256i bswap_mask() {
  return _mm256_setr_epi8(3, 2, 1, 0, 7, 6, 5, 4, 11, 10, 9, 8, 15, 14, 13, 12, 3, 2, 1, 0, 7, 6, 5, 4, 11, 10, 9,
                          8, 15, 14, 13, 12);
}

__attribute__((target("avx2"))) uint32_t hmax(__m256i v) {
  alignas(32) uint32_t t[8];
  _mm256_store_si256((__m256i*)t, v);
  return *std::max_element(t, t + 8);
}

__attribute__((target("avx2"))) void pack_avx2(const uint8_t* in, uint64_t nw, uint32_t n, uint32_t* out,
                                               bool track, uint32_t* mx0, uint32_t* mx1) {
  const __m256i sh = bswap_mask(), vn = _mm256_set1_epi32((int)n), top = _mm256_set1_epi32((int)0x80000000u);
  __m256i a = _mm256_set1_epi32((int)*mx0), b = _mm256_set1_epi32((int)*mx1);
  uint64_t i = 0;
  if (track) {
    for (; i + 16 <= nw; i += 16) {
      const __m256i w0 = _mm256_shuffle_epi8(_mm256_loadu_si256((const __m256i*)(in + 4 * i)), sh);
      const __m256i w1 = _mm256_shuffle_epi8(_mm256_loadu_si256((const __m256i*)(in + 4 * i + 32)), sh);
      a = _mm256_max_epu32(a, _mm256_max_epu32(w0, w1));
      b = _mm256_max_epu32(b, _mm256_max_epu32(_mm256_xor_si256(w0, top), _mm256_xor_si256(w1, top)));
      _mm256_storeu_si256((__m256i*)(out + i), _mm256_xor_si256(w0, vn));
      _mm256_storeu_si256((__m256i*)(out + i + 8), _mm256_xor_si256(w1, vn));
    }
  } else {
    for (; i + 16 <= nw; i += 16) {
      const __m256i w0 = _mm256_shuffle_epi8(_mm256_loadu_si256((const __m256i*)(in + 4 * i)), sh);
      const __m256i w1 = _mm256_shuffle_epi8(_mm256_loadu_si256((const __m256i*)(in + 4 * i + 32)), sh);
      _mm256_storeu_si256((__m256i*)(out + i), _mm256_xor_si256(w0, vn));
      _mm256_storeu_si256((__m256i*)(out + i + 8), _mm256_xor_si256(w1, vn));
    }
  }
  uint32_t ra = hmax(a), rb = hmax(b);
  pack_scalar(in + 4 * i, nw - i, n, out + i, track, &ra, &rb);
  *mx0 = ra, *mx1 = rb;
}

void unpack_scalar(const uint32_t* in, uint64_t count, uint32_t n, uint8_t* out) {
  for (uint64_t i = 0; i < count; ++i) {
    const uint32_t w = __builtin_bswap32(in[i] ^ n);
    memcpy(out + 4 * i, &w, 4);
  }
}

__attribute__((target("avx2"))) void unpack_avx2(const uint32_t* in, uint64_t count, uint32_t n, uint8_t* out) {
  const __m256i sh = bswap_mask(), vn = _mm256_set1_epi32((int)n);
  uint64_t i = 0;
  for (; i + 16 <= count; i += 16) {
    const __m256i w0 = _mm256_xor_si256(_mm256_loadu_si256((const __m256i*)(in + i)), vn);
    const __m256i w1 = _mm256_xor_si256(_mm256_loadu_si256((const __m256i*)(in + i + 8)), vn);
    _mm256_storeu_si256((__m256i*)(out + 4 * i), _mm256_shuffle_epi8(w0, sh));
    _mm256_storeu_si256((__m256i*)(out + 4 * i + 32), _mm256_shuffle_epi8(w1, sh));
  }
  unpack_scalar(in + i, count - i, n, out + 4 * i);
}

void xor_scalar(uint32_t* w, uint64_t count, uint32_t n) {
  for (uint64_t i = 0; i < count; ++i) w[i] ^= n;
}

__attribute__((target("avx2"))) void xor_avx2(uint32_t* w, uint64_t count, uint32_t n) {
  const __m256i vn = _mm256_set1_epi32((int)n);
  uint64_t i = 0;
  for (; i + 8 <= count; i += 8)
    _mm256_storeu_si256((__m256i*)(w + i), _mm256_xor_si256(_mm256_loadu_si256((const __m256i*)(w + i)), vn));
  xor_scalar(w + i, count - i, n);
}

// max over w[i] ^ n (>= p: the mapping does not fit)
uint32_t xmax_scalar(const uint32_t* w, uint64_t count, uint32_t n) {
  uint32_t m = 0;
  for (uint64_t i = 0; i < count; ++i) m = std::max(m, w[i] ^ n);
  return m;
}

__attribute__((target("avx2"))) uint32_t xmax_avx2(const uint32_t* w, uint64_t count, uint32_t n) {
  const __m256i vn = _mm256_set1_epi32((int)n);
  __m256i m = _mm256_setzero_si256();
  uint64_t i = 0;
  for (; i + 8 <= count; i += 8)
    m = _mm256_max_epu32(m, _mm256_xor_si256(_mm256_loadu_si256((const __m256i*)(w + i)), vn));
  return std::max(hmax(m), xmax_scalar(w + i, count - i, n));
}

void mod_scalar(const uint32_t* in, uint64_t count, uint32_t* out) {
  for (uint64_t i = 0; i < count; ++i) out[i] = in[i] >= kP ? in[i] - kP : in[i];
}

__attribute__((target("avx2"))) void mod_avx2(const uint32_t* in, uint64_t count, uint32_t* out) {
  const __m256i p = _mm256_set1_epi32((int)kP);
  uint64_t i = 0;
  for (; i + 8 <= count; i += 8) {
    const __m256i w = _mm256_loadu_si256((const __m256i*)(in + i));
    const __m256i ge = _mm256_cmpeq_epi32(_mm256_max_epu32(w, p), w);  // w >= p
    _mm256_storeu_si256((__m256i*)(out + i), _mm256_sub_epi32(w, _mm256_and_si256(ge, p)));
  }
  mod_scalar(in + i, count - i, out + i);
}

// Output buffers of the Go API are fresh (Go's make, a Python bytearray or
// numpy array): their first touch is this pass, one 4 KiB page fault at a
// time.  With env SLIME_RS_CODEC_HUGEPAGE=1, ranges of at least 4 MiB are
// advised to fault as 2 MiB pages (transparent huge pages in "madvise" mode)
// before the pass writes them -- a hint on the 2 MiB-aligned interior only.
// Off by default: the buffers belong to the caller (under cgo, the Go heap,
// whose huge-page advice the Go runtime manages itself) and the advice would
// outlive the call.
void advise_huge(void* p, uint64_t bytes) {
  static const bool on = [] {
    const char* e = getenv("SLIME_RS_CODEC_HUGEPAGE");
    return e && e[0] == '1';
  }();
  constexpr uintptr_t kHuge = 2u << 20;
  if (!on || bytes < (4u << 20)) return;
  const uintptr_t lo = ((uintptr_t)p + kHuge - 1) & ~(kHuge - 1), hi = ((uintptr_t)p + bytes) & ~(kHuge - 1);
  if (hi > lo) (void)madvise((void*)lo, hi - lo, MADV_HUGEPAGE);
}

// ---- splitting a pass into pieces ----------------------------------------------

uint64_t pieces_of(uint64_t words) { return words <= kSerialWords ? 1 : (words + kPieceWords - 1) / kPieceWords; }

template <class F>
void run_pieces(uint64_t words, F&& f) {
  const uint64_t np = pieces_of(words);
  struct Ctx {
    F* f;
    uint64_t words, per;
  } ctx{&f, words, np == 1 ? words : kPieceWords};
  parallel_pieces(
      np,
      [](const void* c, size_t i) {
        const Ctx* x = (const Ctx*)c;
        const uint64_t w0 = (uint64_t)i * x->per;
        (*x->f)(w0, std::min(x->per, x->words - w0));
      },
      &ctx);
}

}  // namespace

const char* host_codec_isa() { return use_avx2() ? "avx2" : "scalar"; }

void host_pack(const uint8_t* in, uint64_t len, uint32_t n, uint32_t* out, uint32_t* flags) {
  const uint64_t whole = len / 4;
  const bool track = flags != nullptr;
  advise_huge(out, 4 * ((len + 3) / 4));
  std::atomic<uint32_t> m0{0}, m1{0};
  run_pieces(whole, [&](uint64_t w0, uint64_t nw) {
    uint32_t a = 0, b = 0;
    if (use_avx2())
      pack_avx2(in + 4 * w0, nw, n, out + w0, track, &a, &b);
    else
      pack_scalar(in + 4 * w0, nw, n, out + w0, track, &a, &b);
    if (track) {
      for (uint32_t cur = m0.load(); a > cur && !m0.compare_exchange_weak(cur, a);) {
      }
      for (uint32_t cur = m1.load(); b > cur && !m1.compare_exchange_weak(cur, b);) {
      }
    }
  });
  uint32_t a = m0.load(), b = m1.load();
  if (len % 4) {  // map.go:28-33: the trailing bytes fill the high positions of a last word
    uint32_t w = 0;
    for (uint64_t i = 0; i < len % 4; ++i) w |= (uint32_t)in[4 * whole + i] << ((3 - i) * 8);
    a = std::max(a, w);
    b = std::max(b, w ^ 0x80000000u);
    out[whole] = w ^ n;
  }
  if (track) *flags |= (a >= kP ? 1u : 0u) | (b >= kP ? 2u : 0u);
}

void host_unpack(const uint32_t* in, uint64_t count, uint32_t n, uint8_t* out) {
  advise_huge(out, 4 * count);
  run_pieces(count, [&](uint64_t w0, uint64_t nw) {
    if (use_avx2())
      unpack_avx2(in + w0, nw, n, out + 4 * w0);
    else
      unpack_scalar(in + w0, nw, n, out + 4 * w0);
  });
}

void host_xor(uint32_t* w, uint64_t count, uint32_t n) {
  run_pieces(count, [&](uint64_t w0, uint64_t nw) {
    if (use_avx2())
      xor_avx2(w + w0, nw, n);
    else
      xor_scalar(w + w0, nw, n);
  });
}

bool host_mapping_fits(const uint32_t* w, uint64_t count, uint32_t n) {
  std::atomic<bool> bad{false};
  run_pieces(count, [&](uint64_t w0, uint64_t nw) {
    if (bad.load(std::memory_order_relaxed)) return;  // another piece already refuted n
    const uint32_t m = use_avx2() ? xmax_avx2(w + w0, nw, n) : xmax_scalar(w + w0, nw, n);
    if (m >= kP) bad.store(true, std::memory_order_relaxed);
  });
  return !bad.load();
}

void host_mod_p(const uint32_t* in, uint64_t count, uint32_t* out) {
  if (in != out) advise_huge(out, 4 * count);
  run_pieces(count, [&](uint64_t w0, uint64_t nw) {
    if (use_avx2())
      mod_avx2(in + w0, nw, out + w0);
    else
      mod_scalar(in + w0, nw, out + w0);
  });
}

}  // namespace slime
