// CPU emulation of the matrix-core redo list's counter protocol
// (slime_amd/csrc/redo_list.hpp, rs_bytes_mfma.hip mfma_redo_list_kernel):
// waves of 64 lanes, each step OR-ing kSwitchedBit into the counter word when
// any lane saw a switched object and drawing list offsets with one atomicAdd
// per wave, exactly as the kernel's loop body does.
//
//   - fixed interleavings: a wave draws before any bit is set, a wave sets the
//     bit and then draws, a wave draws after another set it (its raw draw
//     carries bit 31): every entry lands at its masked offset, none twice;
//   - 8 real threads x random batches: the list holds exactly the needed
//     entries, redo_count() recovers their number and redo_switched() says
//     whether any object switched; raw draws with bit 31 set were seen, so
//     the masking was exercised;
//   - redo_list_fits() refuses nobj x units >= 2^31 and the degenerate
//     operands, and accepts everything below.
// Usage: redo_list_test   (exit 0 = pass)
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <thread>
#include <vector>

#include "redo_list.hpp"

using namespace slime::bytes;

#define CHECK(cond)                                               \
  do {                                                            \
    if (!(cond)) {                                                \
      std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      std::exit(1);                                               \
    }                                                             \
  } while (0)

namespace {

struct Batch {
  uint32_t nobj, units;
  std::vector<uint32_t> mapping, status;
  std::vector<uint8_t> record;  // 0 = encoded with mapping 0, 1 = with 1<<31, 2 = not interior
  bool need(uint64_t e) const {
    const uint32_t o = (uint32_t)(e / units);
    return mapping[o] != 0 && status[o] == 0 && record[e] == 0;
  }
  bool sw(uint64_t e) const {
    const uint32_t o = (uint32_t)(e / units);
    return mapping[o] != 0 && status[o] == 0;
  }
};

Batch make_batch(std::mt19937_64& rng, uint32_t nobj, uint32_t units, int switched_pct) {
  Batch b{nobj, units, std::vector<uint32_t>(nobj), std::vector<uint32_t>(nobj),
          std::vector<uint8_t>((size_t)nobj * units)};
  for (uint32_t o = 0; o < nobj; ++o) {
    const int r = (int)(rng() % 100);
    b.mapping[o] = r < switched_pct ? 0x80000000u : (r < switched_pct + 3 ? 0x1234567u : 0u);
    b.status[o] = (b.mapping[o] == 0x1234567u) ? 1u : 0u;  // a resolved fallback: not a switch
  }
  for (auto& v : b.record) v = (uint8_t)(rng() % 3);
  return b;
}

// One step of one wave over entries [base, base + 64): the kernel's loop body.
// Returns the raw value the wave's atomicAdd returned (or 0 if it drew none).
uint32_t wave_step(const Batch& b, uint64_t base, std::atomic<uint32_t>& count, std::vector<uint32_t>& list,
                   std::vector<std::atomic<int>>& hits, bool* drew) {
  const uint64_t total = (uint64_t)b.nobj * b.units;
  uint64_t swm = 0, mask = 0;
  for (int lane = 0; lane < 64; ++lane) {
    const uint64_t e = base + lane;
    if (e < total && b.sw(e)) swm |= 1ull << lane;
    if (e < total && b.need(e)) mask |= 1ull << lane;
  }
  if (swm) count.fetch_or(kSwitchedBit);
  *drew = false;
  if (!mask) return 0;
  const uint32_t raw = count.fetch_add((uint32_t)__builtin_popcountll(mask));
  const uint32_t at = redo_offset(raw);
  for (int lane = 0; lane < 64; ++lane)
    if (mask >> lane & 1) {
      const uint32_t slot = at + (uint32_t)__builtin_popcountll(mask & ((1ull << lane) - 1));
      CHECK(slot < list.size());
      list[slot] = (uint32_t)(base + lane);
      hits[slot].fetch_add(1);
    }
  *drew = true;
  return raw;
}

void check_list(const Batch& b, uint32_t word, const std::vector<uint32_t>& list,
                const std::vector<std::atomic<int>>& hits) {
  const uint64_t total = (uint64_t)b.nobj * b.units;
  uint64_t want = 0;
  bool any_sw = false;
  for (uint64_t e = 0; e < total; ++e) want += b.need(e), any_sw |= b.sw(e);
  CHECK(redo_count(word) == want);
  CHECK(redo_switched(word) == any_sw);
  std::vector<uint8_t> seen(total, 0);
  for (uint32_t i = 0; i < redo_count(word); ++i) {
    CHECK(hits[i].load() == 1);
    CHECK(list[i] < total && b.need(list[i]) && !seen[list[i]]);
    seen[list[i]] = 1;
  }
  for (size_t i = redo_count(word); i < hits.size(); ++i) CHECK(hits[i].load() == 0);
}

void test_fixed_orders() {
  // Three waves of one step each over 3 x 64 entries, all objects switched,
  // record 0 everywhere: every lane needs a redo.
  std::mt19937_64 rng(1);
  Batch b = make_batch(rng, 3, 64, 100);
  for (auto& v : b.record) v = 0;
  const int orders[6][3] = {{0, 1, 2}, {0, 2, 1}, {1, 0, 2}, {1, 2, 0}, {2, 0, 1}, {2, 1, 0}};
  int carried = 0;
  for (const auto& ord : orders) {
    std::atomic<uint32_t> count{0};
    std::vector<uint32_t> list(3 * 64, 0xFFFFFFFFu);
    std::vector<std::atomic<int>> hits(list.size());
    for (int w : ord) {
      bool drew = false;
      const uint32_t raw = wave_step(b, (uint64_t)w * 64, count, list, hits, &drew);
      CHECK(drew);
      carried += (raw & kSwitchedBit) != 0;  // every wave sets the bit before drawing
    }
    check_list(b, count.load(), list, hits);
  }
  CHECK(carried == 18);
  // A wave drawing before any wave set the bit: objects 0 (not switched, a
  // resolved fallback with record 0 entries) then 1 (switched).
  Batch c = make_batch(rng, 2, 64, 0);
  for (auto& v : c.record) v = 0;
  c.mapping[1] = 0x80000000u, c.status[1] = 0;
  std::atomic<uint32_t> count{0};
  std::vector<uint32_t> list(128, 0xFFFFFFFFu);
  std::vector<std::atomic<int>> hits(list.size());
  bool drew = false;
  CHECK(wave_step(c, 0, count, list, hits, &drew) == 0 && !drew && count.load() == 0);
  const uint32_t raw = wave_step(c, 64, count, list, hits, &drew);
  CHECK(drew && raw == kSwitchedBit && redo_offset(raw) == 0);
  check_list(c, count.load(), list, hits);
  std::printf("ok   TestRedoListFixedOrders\n");
}

void test_concurrent() {
  std::mt19937_64 rng(0x5113E);
  uint64_t carried = 0, batches = 0;
  for (int it = 0; it < 60; ++it) {
    const uint32_t nobj = 1 + (uint32_t)(rng() % 300), units = 1 + (uint32_t)(rng() % 90);
    const Batch b = make_batch(rng, nobj, units, (int)(rng() % 60));
    const uint64_t total = (uint64_t)nobj * units;
    std::atomic<uint32_t> count{0};
    std::vector<uint32_t> list(total + 64, 0xFFFFFFFFu);
    std::vector<std::atomic<int>> hits(list.size());
    std::atomic<uint64_t> carried_here{0};
    const int nthreads = 8;  // waves: thread t takes steps base = (t + i * nthreads) * 64, as the grid-stride loop
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t)
      th.emplace_back([&, t] {
        for (uint64_t base = (uint64_t)t * 64; base < total; base += (uint64_t)nthreads * 64) {
          bool drew = false;
          const uint32_t raw = wave_step(b, base, count, list, hits, &drew);
          if (drew && (raw & kSwitchedBit)) carried_here.fetch_add(1);
        }
      });
    for (auto& x : th) x.join();
    check_list(b, count.load(), list, hits);
    carried += carried_here.load();
    ++batches;
  }
  CHECK(carried > 100);  // draws that carried bit 31 and were masked
  std::printf("ok   TestRedoListConcurrent (%llu batches, %llu draws carried the flag bit)\n",
              (unsigned long long)batches, (unsigned long long)carried);
}

void test_fits() {
  CHECK(redo_list_fits(1, 1));
  CHECK(redo_list_fits(1, kSwitchedBit - 1));
  CHECK(!redo_list_fits(1, kSwitchedBit));
  CHECK(redo_list_fits(65536, 32767));   // 2^31 - 65536
  CHECK(!redo_list_fits(65536, 32768));  // exactly 2^31
  CHECK(!redo_list_fits(1ull << 32, 1));
  CHECK(!redo_list_fits(3, 1ull << 32));
  CHECK(!redo_list_fits(0xFFFFFFFFull, 0xFFFFFFFFull));
  // The entries of every batch that fits stay below the flag bit, so a draw
  // carrying it never changes the masked offset of a valid entry.
  for (uint64_t n : {1ull, 7ull, 4096ull, 1ull << 20})
    for (uint64_t u : {1ull, 3ull, 2047ull}) {
      if (!redo_list_fits(n, u)) continue;
      const uint32_t last = (uint32_t)(n * u - 1);
      CHECK(redo_offset(last | kSwitchedBit) == last);
    }
  std::printf("ok   TestRedoListFits\n");
}

}  // namespace

int main() {
  test_fixed_orders();
  test_concurrent();
  test_fits();
  return 0;
}
