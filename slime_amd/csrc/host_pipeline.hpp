// The host <-> device pipeline behind every host-memory entry point (the Go
// API's rows, the codec's device placement, writeChunks / reconstruct):
// per-call workspaces on each device and the windowed, pinned 3-stage ring.
// Not part of the public C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <vector>

#include "capi_internal.hpp"
#include "dma_plan.hpp"
#include "host_copy.hpp"

namespace slime {

// Pipeline depth: stages in flight per call.
constexpr int kHostStages = 3;
// In + out bytes one stage moves for the Go-API rows.
constexpr size_t kStageBytes = 8u << 20;
// Bytes one window of the object entry points moves (smaller windows measured
// slower, profiles/r04/s31).
constexpr size_t kObjWindowBytes = 16u << 20;

inline size_t round16(size_t n) { return (n + 15) & ~(size_t)15; }
inline size_t round64(size_t n) { return (n + 63) & ~(size_t)63; }

// One caller's device buffer, pinned ring and streams on one device.
struct Workspace {
  int device = -1;
  hipStream_t stream = nullptr;
  uint8_t* dbuf = nullptr;
  size_t dcap = 0;
  hipStream_t sst[kHostStages] = {};  // one stream per pipeline stage
  hipEvent_t sev[kHostStages] = {};   // stage's D2H done
  hipEvent_t cev = nullptr;           // compute stream reached a point (staged_d2h, fence_stages)
  uint8_t* pin = nullptr;             // pinned staging, kHostStages x (in rows | out rows)
  size_t pcap = 0;
  int reserve(size_t bytes);         // device buffer of at least `bytes`
  int reserve_pinned(size_t bytes);  // pinned ring of at least `bytes`
  int ensure_stages();
  // Every stage stream waits for the work queued on `stream` so far (a
  // call's setup: zeroed flags, the mapping) -- ordering on the device, no
  // host round trip.
  int fence_stages(int nstages);
};

// Waits for `ev` (recorded on a workspace stream) without holding a CPU:
// polls it for a few microseconds -- a small call's kernel and copies finish
// inside that -- then sleeps in hipEventSynchronize (the workspace's events
// are created with hipEventBlockingSync).  The runtime's default wait spins
// for the whole wait: 25 concurrent 64 MiB callers on a 16-CPU share ran
// 21 GiB/s spinning, 32 with blocking waits (profiles/r05/s5_sched).
int wait_event(hipEvent_t ev);
// Everything queued on ws->stream so far, waited for as wait_event does.
int sync_ws(Workspace* ws);

// A workspace on `device` from its free list (most recently released first),
// or a new one.
int acquire_ws(int device, Workspace** out);
void release_ws(Workspace* ws);
struct WsLease {
  Workspace* ws = nullptr;
  ~WsLease() {
    if (ws) release_ws(ws);
  }
};
// Waits for everything the workspace queued (error paths).
void drain_stages(Workspace* ws);

// dev -> host spans after everything queued on ws->stream so far, through
// the pinned stages; returns when the host copies are complete.
int staged_d2h(Workspace* ws, const uint8_t* dev, const Span* sp, size_t n);

// DMA spans between the device layout at `dev` (dev_cap bytes) and the
// pinned stage `pin` (pin_cap bytes; span i at offset off[i]) as plan_dma
// (dma_plan.hpp) cuts them: one copy kernel when the window is small,
// pitched copies for runs of equal rows, else one copy per run of contiguous
// spans.  A copy reaching past either buffer is refused before anything is
// enqueued (SLIME_RS_ERR_INVALID_ARG).
int dma_spans(uint8_t* dev, uint64_t dev_cap, uint8_t* pin, uint64_t pin_cap, const std::vector<Span>& sp,
              const std::vector<size_t>& off, bool h2d, hipStream_t st);

// Inputs (bytes) up to which a one-window call runs its kernel on the mapped
// pinned stage itself (env SLIME_RS_DIRECT_KIB, default 16384; 0 = never).
uint64_t direct_max_bytes();
// Pinned stage of a direct call: at least this much, as the device buffer
// (Workspace::reserve), so the kernel finds the same room past the layout.
constexpr size_t kDirectPinned = 1u << 20;

// Process-wide split of host-pipeline time (slime_rs_host_stats), microseconds.
struct HostStats {
  std::atomic<uint64_t> calls{0}, windows{0}, copy_in_us{0}, enqueue_us{0}, wait_us{0}, copy_out_us{0}, total_us{0};
};
extern HostStats g_host_stats;
void record_host_stats(uint64_t windows, double t_in, double t_enq, double t_wait, double t_out, double t_total);

// ---- windowed pipeline ---------------------------------------------------------
//
// A host call is cut into column windows.  Window c runs on stage s = c % S:
// its input spans are memcpy'd (copy pool) into stage s's pinned buffer and
// DMA'd on stage stream s, then the window's launch, then the DMA of its
// output spans back into the same pinned buffer.  The outputs reach the
// caller when stage s is needed again (or at the end), so the host copies of
// one window overlap the DMA and kernels of the others, and the H2D of one
// window overlaps the D2H of another.  Windows may also carry host-to-host
// copies (write_chunks' data-chunk bodies), done once the window is queued,
// while its upload and kernel run.
struct Window {
  uint64_t index = 0;  // window number c
  std::vector<Span> in, out;
  std::vector<CopyItem> host;
  std::vector<size_t> in_off, out_off;  // offsets in the stage's pinned buffer
};

// io(c, s, Window&) fills window c's spans; launch(c, s, stream, base)
// enqueues its kernels over the window's device layout at `base` (dev, or
// the pinned stage in a direct call); landed(c) runs once window c's outputs
// are in the caller's buffers (windows land in order).  direct_bytes: the
// size of one window's device layout when the caller's kernels may run on
// the pinned stage (direct_max_bytes), else 0.
template <class Io, class Launch, class Landed>
int run_windows(Workspace* ws, uint8_t* dev, uint64_t n, size_t stage_bytes, Io&& io, Launch&& launch,
                Landed&& landed, size_t direct_bytes = 0) {
  if (n == 0) return 0;
  using clk = std::chrono::steady_clock;
  auto ms_since = [](clk::time_point t) { return std::chrono::duration<double, std::milli>(clk::now() - t).count(); };
  const auto t_start = clk::now();
  double t_in = 0, t_wait = 0, t_out = 0, t_enq = 0;
  const int S = (int)std::min<uint64_t>(kHostStages, n);
  const bool may_direct = n == 1 && direct_bytes && direct_bytes <= 8 * direct_max_bytes();
  if (int rc = ws->reserve_pinned(may_direct ? std::max(std::max(stage_bytes, direct_bytes), kDirectPinned)
                                             : stage_bytes * S))
    return rc;
  if (int rc = ws->ensure_stages()) return rc;
  // `dev` lies in the workspace's device buffer (every caller passes
  // ws->dbuf); its copies are bounded by what is left of that buffer.
  if (dev < ws->dbuf || dev > ws->dbuf + ws->dcap) return fail(Status::InvalidArg, "window layout outside the workspace");
  const uint64_t dev_cap = (uint64_t)(ws->dbuf + ws->dcap - dev);
  std::vector<Window> win(S);
  std::vector<CopyItem> items;
  auto pin_of = [&](int s) { return ws->pin + (size_t)s * stage_bytes; };
  auto wait_stage = [&](int s) -> int {
    const auto t0 = clk::now();
    if (int rc = wait_event(ws->sev[s])) return rc;
    t_wait += ms_since(t0);
    return 0;
  };
  auto add_out_items = [&](int s) {  // stage s's landed outputs -> the caller's buffers
    const Window& w = win[s];
    for (size_t i = 0; i < w.out.size(); ++i) items.push_back({w.out[i].host, pin_of(s) + w.out_off[i], w.out[i].bytes});
  };
  auto land = [&](int s) -> int {
    if (int rc = wait_stage(s)) return rc;
    const auto t0 = clk::now();
    items.clear();
    add_out_items(s);
    parallel_copy(items.data(), items.size());
    t_out += ms_since(t0);
    landed(win[s].index);
    return 0;
  };
  auto body = [&]() -> int {
    for (uint64_t c = 0; c < n; ++c) {
      const int s = (int)(c % S);
      // Window c reuses stage s of window c - S: once that window's DMA is
      // done, its outputs leave the pinned stage in the same pool job as
      // window c's inputs arrive (two regions of the stage: c's inputs end
      // where c - S's did or earlier, and its outputs follow its inputs).
      Window& w = win[s];
      items.clear();
      bool prev = false;
      uint64_t prev_index = 0;
      size_t prev_out_start = 0;
      if (c >= (uint64_t)S) {
        if (int rc = wait_stage(s)) return rc;
        prev = true;
        prev_index = w.index;
        prev_out_start = w.out.empty() ? stage_bytes : w.out_off[0];
        add_out_items(s);
      }
      const size_t nprev = items.size();
      w.index = c;
      w.in.clear(), w.out.clear(), w.host.clear();
      io(c, s, w);
      uint8_t* const pin = pin_of(s);
      // Direct: every span inside the layout, inputs within the limit; the
      // stage then holds each span at its device offset.
      bool direct = may_direct;
      if (direct) {
        uint64_t in_bytes = 0;
        for (const Span& x : w.in) in_bytes += x.bytes, direct &= x.dev_off + x.bytes <= direct_bytes;
        for (const Span& x : w.out) direct &= x.dev_off + x.bytes <= direct_bytes;
        direct &= in_bytes <= direct_max_bytes();
      }
      size_t off = 0;
      w.in_off.resize(w.in.size());
      for (size_t i = 0; i < w.in.size(); ++i) {
        w.in_off[i] = direct ? w.in[i].dev_off : off;
        items.push_back({pin + w.in_off[i], w.in[i].host, w.in[i].bytes});
        off = round64(off + w.in[i].bytes);
      }
      const size_t in_end = off;
      w.out_off.resize(w.out.size());
      for (size_t i = 0; i < w.out.size(); ++i) {
        w.out_off[i] = direct ? w.out[i].dev_off : off;
        off = round64(off + w.out[i].bytes);
      }
      if (!direct && off > stage_bytes) return fail(Status::InvalidArg, "window larger than its pinned stage");
      auto t0 = clk::now();
      if (prev && in_end > prev_out_start) {  // the regions would overlap: outputs first, then inputs
        parallel_copy(items.data(), nprev);
        parallel_copy(items.data() + nprev, items.size() - nprev);
      } else {
        parallel_copy(items.data(), items.size());
      }
      t_in += ms_since(t0);
      if (prev) landed(prev_index);
      t0 = clk::now();
      hipStream_t st = ws->sst[s];
      if (direct) {  // the kernel on the stage: no copies across PCIe besides its own accesses
        if (int rc = launch(c, s, st, pin)) return rc;
      } else {
        if (int rc = dma_spans(dev, dev_cap, pin, stage_bytes, w.in, w.in_off, true, st)) return rc;
        if (int rc = launch(c, s, st, dev)) return rc;
        if (int rc = dma_spans(dev, dev_cap, pin, stage_bytes, w.out, w.out_off, false, st)) return rc;
      }
      HIP_TRY(hipEventRecord(ws->sev[s], st));
      t_enq += ms_since(t0);
      // Host-to-host copies (write_chunks' data-chunk bodies) are not needed
      // on the device: they run while the window's upload and kernel do.
      if (!w.host.empty()) {
        t0 = clk::now();
        parallel_copy(w.host.data(), w.host.size());
        t_in += ms_since(t0);
      }
    }
    for (uint64_t c = n > (uint64_t)S ? n - S : 0; c < n; ++c)
      if (int rc = land((int)(c % S))) return rc;
    return 0;
  };
  const int rc = body();
  if (rc) drain_stages(ws);
  record_host_stats(n, t_in, t_enq, t_wait, t_out, ms_since(t_start));
  return rc;
}

template <class Io, class Launch>
int run_windows(Workspace* ws, uint8_t* dev, uint64_t n, size_t stage_bytes, Io&& io, Launch&& launch) {
  return run_windows(ws, dev, n, stage_bytes, io, launch, [](uint64_t) {});
}

// Columns per window so that one window moves about `stage` bytes over
// `rows` rows of 4-byte symbols; a multiple of 4096 (16 KiB per row), or the
// whole length in one window.
inline uint64_t window_cols(uint64_t L, uint64_t rows, size_t stage) {
  const uint64_t cl = std::max<uint64_t>(stage / (rows * 4), 4096) & ~4095ull;
  return cl >= L ? L : cl;
}

// out[i][0:L] = sum_j coeff[i][j] * in[j][0:L] for a plan whose inputs are
// 0..k-1 and outputs 0..rows-1 (host memory on both sides), through the
// staged ring.
int host_apply(const slime_rs_plan* plan, const uint32_t* const* in, uint32_t* const* out, uint64_t L);

}  // namespace slime
