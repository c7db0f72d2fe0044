// The copy commands one window of the host pipeline issues between the
// pinned stage and the device layout (dma_spans, host_pipeline.cpp), planned
// apart from the HIP calls that run them so that every command's full extent
// -- the last byte a pitched copy touches, not just its first row -- can be
// checked against the two buffers before anything is enqueued.  Pure host
// code: tests/cpp/dma_plan_test.cpp runs it on the CPU.
#pragma once
#include <stdint.h>

#include <vector>

namespace slime {

// A host range and its device offset.
struct Span {
  uint8_t* host;
  uint64_t dev_off;
  uint64_t bytes;
};

// One copy: `rows` rows of `width` bytes, row r at dev_off + r * dev_pitch on
// the device and pin_off + r * pin_pitch in the pinned stage (rows == 1: a
// linear copy, pitches unused).
struct DmaCopy {
  uint64_t dev_off = 0, pin_off = 0, width = 0, rows = 1, dev_pitch = 0, pin_pitch = 0;
};

struct DmaPlan {
  bool blit = false;  // one copy kernel over the list (host_blit.hip); every copy linear
  std::vector<DmaCopy> copies;
};

// Windows moving at most this many bytes one way go as one copy kernel over
// the mapped pinned ring instead of copy-engine transfers (host_blit.hip):
// uploads up to 4 MiB (a kernel reading host memory is latency-bound, so
// larger uploads keep the copy engines: a 64 MiB CreateParity ran 1.88 ms
// instead of 1.41 with kernel uploads), downloads of every window size (the
// kernel's writes are posted and run beside the copy engines' uploads --
// fused reconstruct +4-7%, write_chunks +3-10%, profiles/r04/s19-s20).
constexpr uint64_t kBlitUpBytes = 4u << 20;
constexpr uint64_t kBlitDownBytes = 64u << 20;

// Spans one by one, merging neighbours contiguous on both sides.  Runs of
// equal-length spans at constant device and pinned strides (a window's rows:
// one per chunk) go as one pitched copy: per-span copies reach the copy
// engine as separate commands ~10 us apart, and one pitched copy took the
// fused reconstruct from 22 to 27 GiB/s and write_chunks from 32 to 36
// (profiles/r04/s24_rctrace, s25_dma2d).  The blit limits are parameters
// only so the CPU test can reach every form with small buffers.
inline DmaPlan plan_dma(const std::vector<Span>& sp, const std::vector<size_t>& off, bool h2d,
                        uint64_t blit_up = kBlitUpBytes, uint64_t blit_down = kBlitDownBytes) {
  DmaPlan p;
  uint64_t total = 0;
  for (const Span& s : sp) total += s.bytes;
  if (total && total <= (h2d ? blit_up : blit_down)) {
    p.blit = true;
    for (size_t i = 0; i < sp.size();) {
      size_t j = i + 1;
      uint64_t bytes = sp[i].bytes;
      while (j < sp.size() && sp[j].dev_off == sp[i].dev_off + bytes && off[j] == off[i] + bytes) bytes += sp[j++].bytes;
      DmaCopy c;
      c.dev_off = sp[i].dev_off, c.pin_off = off[i], c.width = bytes;
      p.copies.push_back(c);
      i = j;
    }
    return p;
  }
  for (size_t i = 0; i < sp.size();) {
    size_t j = i + 1;
    const uint64_t bytes = sp[i].bytes;
    const int64_t dd = j < sp.size() ? (int64_t)sp[j].dev_off - (int64_t)sp[i].dev_off : 0;
    const int64_t dp = j < sp.size() ? (int64_t)off[j] - (int64_t)off[i] : 0;
    if (dd >= (int64_t)bytes && dp >= (int64_t)bytes)
      while (j < sp.size() && sp[j].bytes == bytes && (int64_t)sp[j].dev_off - (int64_t)sp[j - 1].dev_off == dd &&
             (int64_t)off[j] - (int64_t)off[j - 1] == dp)
        ++j;
    DmaCopy c;
    c.dev_off = sp[i].dev_off, c.pin_off = off[i];
    if (j - i >= 2) {
      c.width = bytes, c.rows = j - i, c.dev_pitch = (uint64_t)dd, c.pin_pitch = (uint64_t)dp;
    } else {  // a run of spans contiguous on both sides as one copy
      uint64_t run = bytes;
      for (j = i + 1; j < sp.size() && sp[j].dev_off == sp[i].dev_off + run && off[j] == off[i] + run; ++j)
        run += sp[j].bytes;
      c.width = run;
    }
    p.copies.push_back(c);
    i = j;
  }
  return p;
}

// One past the last byte a copy touches on one side, or UINT64_MAX if that
// does not fit in 64 bits.
inline uint64_t copy_end(uint64_t start, uint64_t rows, uint64_t pitch, uint64_t width) {
  uint64_t span = 0, end = 0;
  if (rows > 1 && __builtin_mul_overflow(rows - 1, pitch, &span)) return UINT64_MAX;
  if (__builtin_add_overflow(start, span, &end) || __builtin_add_overflow(end, width, &end)) return UINT64_MAX;
  return end;
}

// Index of the first copy that reaches past dev_cap bytes of the device
// buffer or pin_cap bytes of the pinned stage, or -1 if every copy fits
// (a copy of zero bytes touches nothing, wherever it points).
inline long first_out_of_bounds(const DmaPlan& p, uint64_t dev_cap, uint64_t pin_cap) {
  for (size_t i = 0; i < p.copies.size(); ++i) {
    const DmaCopy& c = p.copies[i];
    if (c.width && (copy_end(c.dev_off, c.rows, c.dev_pitch, c.width) > dev_cap ||
                    copy_end(c.pin_off, c.rows, c.pin_pitch, c.width) > pin_cap))
      return (long)i;
  }
  return -1;
}

}  // namespace slime
