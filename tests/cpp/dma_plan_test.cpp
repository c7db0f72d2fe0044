// CPU test of the host pipeline's copy planning (slime_amd/csrc/dma_plan.hpp),
// the commands dma_spans (host_pipeline.cpp) hands to hipMemcpy2DAsync,
// hipMemcpyAsync and the blit kernel:
//
//   - the window layouts the entry points build (host_apply's rows at the
//     device row stride, packed 64-byte-rounded in the stage; write_chunks'
//     flag word ahead of the data rows) plan to the expected commands, and
//     their last byte lands exactly at the end of the last span;
//   - a plan is faithful: replaying its commands byte by byte over a model of
//     both buffers copies every span's bytes to its place and touches nothing
//     else (random span lists, both directions, blit and copy-engine sizes);
//   - first_out_of_bounds() flags a plan exactly when some span reaches past
//     either buffer, including by one byte, and when a pitched extent
//     overflows 64 bits.
// Usage: dma_plan_test   (exit 0 = pass)
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "dma_plan.hpp"

using namespace slime;

#define CHECK(cond)                                               \
  do {                                                            \
    if (!(cond)) {                                                \
      std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      std::exit(1);                                               \
    }                                                             \
  } while (0)

namespace {

uint64_t round64(uint64_t n) { return (n + 63) & ~63ull; }

// The end of the furthest span on each side: what a correct plan may reach.
void span_ends(const std::vector<Span>& sp, const std::vector<size_t>& off, uint64_t* dev_end, uint64_t* pin_end) {
  *dev_end = *pin_end = 0;
  for (size_t i = 0; i < sp.size(); ++i) {
    if (!sp[i].bytes) continue;
    *dev_end = std::max<uint64_t>(*dev_end, sp[i].dev_off + sp[i].bytes);
    *pin_end = std::max<uint64_t>(*pin_end, off[i] + sp[i].bytes);
  }
}

// Byte-level replay: dev/pin hold distinct tags; h2d copies pin -> dev.
// Returns false if any command touches a byte outside the model.
bool replay(const DmaPlan& p, std::vector<uint32_t>& dev, std::vector<uint32_t>& pin, bool h2d) {
  for (const DmaCopy& c : p.copies)
    for (uint64_t r = 0; r < c.rows; ++r)
      for (uint64_t b = 0; b < c.width; ++b) {
        const uint64_t d = c.dev_off + r * c.dev_pitch + b, q = c.pin_off + r * c.pin_pitch + b;
        if (d >= dev.size() || q >= pin.size()) return false;
        if (h2d)
          dev[d] = pin[q];
        else
          pin[q] = dev[d];
      }
  return true;
}

void test_host_apply_layout() {
  // host_apply at need 4, one parity row, 64 MiB object: cl = 417792 columns,
  // rows at rs * 4 bytes on the device, packed in the stage.
  const uint64_t nin = 4, cl = 417792, rs = cl, stage_dev = (nin + 1) * rs * 4;
  for (uint64_t nc : {cl, (uint64_t)16384, (uint64_t)4096, (uint64_t)1}) {
    for (int s = 0; s < 3; ++s) {
      std::vector<Span> in;
      std::vector<size_t> off;
      size_t o = 0;
      for (uint64_t j = 0; j < nin; ++j) {
        in.push_back({nullptr, s * stage_dev + j * rs * 4, nc * 4});
        off.push_back(o);
        o = round64(o + nc * 4);
      }
      const DmaPlan p = plan_dma(in, off, true);
      uint64_t dend, pend;
      span_ends(in, off, &dend, &pend);
      CHECK(first_out_of_bounds(p, dend, pend) == -1);
      CHECK(first_out_of_bounds(p, dend - 1, pend) >= 0);
      CHECK(first_out_of_bounds(p, dend, pend - 1) >= 0);
      if (nin * nc * 4 > kBlitUpBytes) {  // copy engines: one pitched copy over the 4 rows
        CHECK(!p.blit && p.copies.size() == 1 && p.copies[0].rows == nin);
        CHECK(p.copies[0].dev_pitch == rs * 4 && p.copies[0].pin_pitch == round64(nc * 4));
      } else {
        CHECK(p.blit);
      }
    }
  }
  std::printf("ok   TestHostApplyLayout\n");
}

void test_write_chunks_layout() {
  // write_chunks' one-window form: the 8-byte flag word at the end of the
  // slot, then the data rows (the last one short), packed in the stage.
  const uint64_t chunk = 1 << 20, need = 8, stride = 12 * chunk;
  std::vector<Span> in{{nullptr, stride, 8}};
  std::vector<size_t> off{0};
  size_t o = 64;
  for (uint64_t j = 0; j < need; ++j) {
    const uint64_t bytes = j + 1 < need ? chunk : chunk - 13;
    in.push_back({nullptr, j * chunk, bytes});
    off.push_back(o);
    o = round64(o + bytes);
  }
  for (bool h2d : {true, false}) {
    const DmaPlan p = plan_dma(in, off, h2d);
    uint64_t dend, pend;
    span_ends(in, off, &dend, &pend);
    CHECK(first_out_of_bounds(p, stride + 16, pend) == -1);
    CHECK(first_out_of_bounds(p, stride + 7, pend) >= 0);
    CHECK(first_out_of_bounds(p, stride + 16, pend - 1) >= 0);
  }
  std::printf("ok   TestWriteChunksLayout\n");
}

void test_faithful_random() {
  std::mt19937_64 rng(0x5113E);
  int plans = 0, pitched = 0, blits = 0;
  for (int it = 0; it < 3000; ++it) {
    const bool h2d = rng() & 1;
    // Small buffers keep the byte-level model cheap; the blit limits are
    // scaled down with them so both forms are drawn.
    const uint64_t unit = 64, blit = (rng() & 1) ? 0 : 1024;
    const int n = 1 + (int)(rng() % 9);
    const bool equal = rng() & 1;  // equal rows at fixed strides (pitched candidates)
    const uint64_t w0 = unit * (1 + rng() % 4) - (rng() % 3 == 0 ? rng() % 13 : 0);
    const uint64_t dstride = w0 + (rng() % 3) * 64 * (rng() % 2), pstride = round64(w0) + (rng() % 2) * 64;
    std::vector<Span> sp;
    std::vector<size_t> off;
    uint64_t d = rng() % 256, q = 0;
    for (int i = 0; i < n; ++i) {
      const uint64_t w = equal ? w0 : unit * (rng() % 3) + rng() % 97;
      sp.push_back({nullptr, d, w});
      off.push_back(q);
      if (equal) {
        d += dstride, q += pstride;
      } else {
        d += w + (rng() % 2) * (rng() % 200);
        q += (rng() % 2) ? w : round64(w);
      }
    }
    const DmaPlan p = plan_dma(sp, off, h2d, blit, blit);
    uint64_t dend, pend;
    span_ends(sp, off, &dend, &pend);
    CHECK(first_out_of_bounds(p, dend, pend) == -1);
    if (dend) CHECK(first_out_of_bounds(p, dend - 1, pend) >= 0);
    if (pend) CHECK(first_out_of_bounds(p, dend, pend - 1) >= 0);
    // Replay against a model with a guard region past each end.
    std::vector<uint32_t> dev(dend + 64), pin(pend + 64);
    for (size_t i = 0; i < dev.size(); ++i) dev[i] = 0x10000000u + (uint32_t)i;
    for (size_t i = 0; i < pin.size(); ++i) pin[i] = 0x20000000u + (uint32_t)i;
    std::vector<uint32_t> want_dev = dev, want_pin = pin;
    for (size_t i = 0; i < sp.size(); ++i)
      for (uint64_t b = 0; b < sp[i].bytes; ++b)
        if (h2d)
          want_dev[sp[i].dev_off + b] = want_pin[off[i] + b];
        else
          want_pin[off[i] + b] = want_dev[sp[i].dev_off + b];
    CHECK(replay(p, dev, pin, h2d));
    CHECK(dev == want_dev && pin == want_pin);
    ++plans;
    blits += p.blit;
    for (const DmaCopy& c : p.copies) pitched += c.rows > 1;
  }
  CHECK(plans == 3000 && pitched > 300 && blits > 300);
  std::printf("ok   TestPlanFaithful (%d plans, %d pitched copies, %d blit lists)\n", plans, pitched, blits);
}

void test_overflow() {
  DmaPlan p;
  DmaCopy c;
  c.dev_off = 0, c.pin_off = 0, c.width = 16, c.rows = 3, c.dev_pitch = UINT64_MAX / 2, c.pin_pitch = 64;
  p.copies.push_back(c);
  CHECK(first_out_of_bounds(p, UINT64_MAX - 1, UINT64_MAX - 1) == 0);
  CHECK(copy_end(UINT64_MAX - 4, 1, 0, 8) == UINT64_MAX);
  CHECK(copy_end(100, 1, 12345, 8) == 108);
  CHECK(copy_end(100, 4, 1000, 8) == 3108);
  std::printf("ok   TestExtentOverflow\n");
}

}  // namespace

int main() {
  test_host_apply_layout();
  test_write_chunks_layout();
  test_faithful_random();
  test_overflow();
  return 0;
}
