// Per-call workspaces and the pinned windowed pipeline (host_pipeline.hpp)
// behind the host-memory entry points, and the Go-API rows' staged apply.
#include "host_pipeline.hpp"

#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <stdlib.h>

#include <algorithm>
#include <chrono>
#include <memory>

namespace slime {

int Workspace::reserve(size_t bytes) {
  if (bytes <= dcap) return 0;
  DeviceScope ds(device);
  if (stream) (void)hipStreamSynchronize(stream);
  for (hipStream_t st : sst)
    if (st) (void)hipStreamSynchronize(st);
  if (dbuf) (void)hipFree(dbuf);
  dbuf = nullptr;
  dcap = 0;
  // Headroom: a host call's workspace serves calls of other shapes next
  // (write_chunks needs total x chunk, reconstruct 2 x need x chunk), and
  // every regrowth is a device-synchronising hipFree plus a fresh hipMalloc
  // whose freed predecessor the driver wipes while other DMA runs.
  const size_t want = std::max<size_t>(bytes + bytes / 2, 1u << 20);
  HIP_TRY(hipMalloc((void**)&dbuf, want));
  dcap = want;
  return 0;
}

int Workspace::reserve_pinned(size_t bytes) {
  if (bytes <= pcap) return 0;
  DeviceScope ds(device);
  for (hipStream_t st : sst)
    if (st) (void)hipStreamSynchronize(st);
  if (pin) (void)hipHostFree(pin);
  pin = nullptr;
  pcap = 0;
  const size_t want = bytes + bytes / 4;  // headroom, as reserve()
  HIP_TRY(hipHostMalloc((void**)&pin, want, hipHostMallocDefault));
  pcap = want;
  return 0;
}

int Workspace::ensure_stages() {
  if (sst[0]) return 0;
  DeviceScope ds(device);
  for (int i = 0; i < kHostStages; ++i) {
    HIP_TRY(hipStreamCreateWithFlags(&sst[i], hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&sev[i], hipEventDisableTiming | hipEventBlockingSync));
  }
  HIP_TRY(hipEventCreateWithFlags(&cev, hipEventDisableTiming | hipEventBlockingSync));
  return 0;
}

// Polling window of wait_event: the kernel of a 4 KiB call finishes ~10 us
// after its launch; a sleeping wait costs a wake-up on top of that.
constexpr std::chrono::microseconds kPollWindow{30};

int wait_event(hipEvent_t ev) {
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t i = 0;; ++i) {
    const hipError_t q = hipEventQuery(ev);
    if (q == hipSuccess) return 0;
    if (q != hipErrorNotReady) return fail_hip(q, "hipEventQuery");
    if ((i & 7) == 7 && std::chrono::steady_clock::now() - t0 > kPollWindow) break;
    for (int k = 0; k < 64; ++k) _mm_pause();
  }
  HIP_TRY(hipEventSynchronize(ev));
  return 0;
}

int sync_ws(Workspace* ws) {
  if (int rc = ws->ensure_stages()) return rc;
  HIP_TRY(hipEventRecord(ws->cev, ws->stream));
  return wait_event(ws->cev);
}

int Workspace::fence_stages(int nstages) {
  if (int rc = ensure_stages()) return rc;
  HIP_TRY(hipEventRecord(cev, stream));
  for (int s = 0; s < nstages && s < kHostStages; ++s) HIP_TRY(hipStreamWaitEvent(sst[s], cev, 0));
  return 0;
}

namespace {
PerDeviceFreeList<Workspace> g_ws_free;  // most recently released first (device_pool.hpp)
}  // namespace

int acquire_ws(int device, Workspace** out) {
  if (Workspace* ws = g_ws_free.take(device)) {
    *out = ws;
    return 0;
  }
  auto ws = std::make_unique<Workspace>();
  ws->device = device;
  DeviceScope ds(device);
  HIP_TRY(hipStreamCreateWithFlags(&ws->stream, hipStreamNonBlocking));
  *out = ws.release();
  return 0;
}

void release_ws(Workspace* ws) { g_ws_free.give(ws); }

void drain_stages(Workspace* ws) {
  if (ws->stream) (void)hipStreamSynchronize(ws->stream);
  for (hipStream_t st : ws->sst)
    if (st) (void)hipStreamSynchronize(st);
}

namespace {
// Spans are cut into pieces of at most kStageBytes; piece p goes through
// pinned stage p % S, so the host memcpy of one piece overlaps the DMA of the
// previous ones.
std::vector<Span> pieces_of(const Span* sp, size_t n) {
  std::vector<Span> out;
  for (size_t i = 0; i < n; ++i)
    for (uint64_t off = 0; off < sp[i].bytes; off += kStageBytes)
      out.push_back({sp[i].host + off, sp[i].dev_off + off, std::min<uint64_t>(kStageBytes, sp[i].bytes - off)});
  return out;
}
}  // namespace

int staged_d2h(Workspace* ws, const uint8_t* dev, const Span* sp, size_t n) {
  if (int rc = ws->reserve_pinned(kStageBytes * kHostStages)) return rc;
  if (int rc = ws->ensure_stages()) return rc;
  const std::vector<Span> pcs = pieces_of(sp, n);
  for (const Span& x : pcs)  // every download inside the device buffer (each piece fits its stage by construction)
    if (dev < ws->dbuf || copy_end((uint64_t)(dev - ws->dbuf) + x.dev_off, 1, 0, x.bytes) > ws->dcap)
      return fail(Status::InvalidArg, "download outside the workspace");
  const int S = kHostStages;
  HIP_TRY(hipEventRecord(ws->cev, ws->stream));
  for (int s = 0; s < S; ++s) HIP_TRY(hipStreamWaitEvent(ws->sst[s], ws->cev, 0));
  auto land = [&](size_t p) -> int {
    const int s = (int)(p % S);
    if (int rc = wait_event(ws->sev[s])) return rc;
    const CopyItem it{pcs[p].host, ws->pin + (size_t)s * kStageBytes, pcs[p].bytes};
    parallel_copy(&it, 1);
    return 0;
  };
  for (size_t p = 0; p < pcs.size(); ++p) {
    const int s = (int)(p % S);
    if (p >= (size_t)S)
      if (int rc = land(p - S)) return rc;
    HIP_TRY(hipMemcpyAsync(ws->pin + (size_t)s * kStageBytes, dev + pcs[p].dev_off, pcs[p].bytes,
                           hipMemcpyDeviceToHost, ws->sst[s]));
    HIP_TRY(hipEventRecord(ws->sev[s], ws->sst[s]));
  }
  for (size_t p = pcs.size() > (size_t)S ? pcs.size() - S : 0; p < pcs.size(); ++p)
    if (int rc = land(p)) return rc;
  return 0;
}

int dma_spans(uint8_t* dev, uint64_t dev_cap, uint8_t* pin, uint64_t pin_cap, const std::vector<Span>& sp,
              const std::vector<size_t>& off, bool h2d, hipStream_t st) {
  const DmaPlan p = plan_dma(sp, off, h2d);
  if (first_out_of_bounds(p, dev_cap, pin_cap) >= 0)
    return fail(Status::InvalidArg, h2d ? "window upload outside its buffers" : "window download outside its buffers");
  if (p.blit) {
    std::vector<BlitSpan> bl;
    bl.reserve(p.copies.size());
    for (const DmaCopy& c : p.copies)
      if (h2d)
        bl.push_back({dev + c.dev_off, pin + c.pin_off, c.width});
      else
        bl.push_back({pin + c.pin_off, dev + c.dev_off, c.width});
    HIP_TRY(launch_blit(bl.data(), (int)bl.size(), st));
    return 0;
  }
  for (const DmaCopy& c : p.copies) {
    if (!c.width) continue;
    if (c.rows >= 2) {
      if (h2d)
        HIP_TRY(hipMemcpy2DAsync(dev + c.dev_off, c.dev_pitch, pin + c.pin_off, c.pin_pitch, c.width, c.rows,
                                 hipMemcpyHostToDevice, st));
      else
        HIP_TRY(hipMemcpy2DAsync(pin + c.pin_off, c.pin_pitch, dev + c.dev_off, c.dev_pitch, c.width, c.rows,
                                 hipMemcpyDeviceToHost, st));
    } else if (h2d) {
      HIP_TRY(hipMemcpyAsync(dev + c.dev_off, pin + c.pin_off, c.width, hipMemcpyHostToDevice, st));
    } else {
      HIP_TRY(hipMemcpyAsync(pin + c.pin_off, dev + c.dev_off, c.width, hipMemcpyDeviceToHost, st));
    }
  }
  return 0;
}

// A one-window call whose inputs total at most this many bytes runs its
// kernel on the mapped pinned stage itself ("direct"): the stage holds the
// window in the device layout, the kernel reads its inputs and writes its
// outputs across PCIe, and the two copy kernels around it -- each a dispatch
// and a PCIe round trip, most of a 4 KiB call -- do not run.  One window has
// no upload/compute overlap to lose, and the static grid of a one-object
// launch (queue_spread) keeps enough loads in flight across the link: 4 KiB
// write_chunks 23 -> 20 us, 1 MiB 80 -> 67-80, 8 MiB 392-402 -> 363-366
// (profiles/r04/s44-s45, s52_directab2, s53_directab3; the 1 MiB gain varies
// by box).  Env SLIME_RS_DIRECT_KIB, default 16384 (every one-window call);
// 0 = never (the tests run both).
uint64_t direct_max_bytes() {
  static const uint64_t v = [] {
    const char* e = getenv("SLIME_RS_DIRECT_KIB");
    const long long kib = e ? atoll(e) : 16384;
    return kib > 0 ? (uint64_t)kib << 10 : 0ull;
  }();
  return v;
}

HostStats g_host_stats;

void record_host_stats(uint64_t windows, double t_in, double t_enq, double t_wait, double t_out, double t_total) {
  auto us = [](double ms) { return (uint64_t)(ms * 1e3 + 0.5); };
  g_host_stats.calls.fetch_add(1, std::memory_order_relaxed);
  g_host_stats.windows.fetch_add(windows, std::memory_order_relaxed);
  g_host_stats.copy_in_us.fetch_add(us(t_in), std::memory_order_relaxed);
  g_host_stats.enqueue_us.fetch_add(us(t_enq), std::memory_order_relaxed);
  g_host_stats.wait_us.fetch_add(us(t_wait), std::memory_order_relaxed);
  g_host_stats.copy_out_us.fetch_add(us(t_out), std::memory_order_relaxed);
  g_host_stats.total_us.fetch_add(us(t_total), std::memory_order_relaxed);
}

// The Go-API rows (CreateParity, RecoverData): column windows of ~8 MiB
// through the staged ring, the caller's rows pageable.  A pinned-registration
// mode and a one-shot pageable mode were measured and removed (MEASUREMENTS.md
// round 1, profiles/r01/host_pipe*).
int host_apply(const slime_rs_plan* plan, const uint32_t* const* in, uint32_t* const* out, uint64_t L) {
  WsLease lease;
  if (int rc = acquire_ws(plan->device, &lease.ws)) return rc;
  Workspace* ws = lease.ws;
  DeviceScope ds(plan->device);
  const uint64_t nin = plan->k, nout = plan->rows;
  const uint64_t cl = window_cols(L, nin + nout, kStageBytes);
  const uint64_t n = (L + cl - 1) / cl;
  const uint64_t rs = (cl + 63) & ~63ull;  // device row stride: 256 B aligned rows (line-aligned streams)
  const size_t stage_dev = (size_t)(nin + nout) * rs * 4;
  if (int rc = ws->reserve(stage_dev * std::min<uint64_t>(kHostStages, n))) return rc;
  uint8_t* const dev = ws->dbuf;
  return run_windows(
      ws, dev, n, (size_t)(nin + nout) * round64(rs * 4),
      [&](uint64_t c, int s, Window& w) {
        const uint64_t c0 = c * cl, nc = std::min(cl, L - c0);
        const uint64_t base = (uint64_t)s * stage_dev;
        for (uint64_t j = 0; j < nin; ++j) w.in.push_back({(uint8_t*)(in[j] + c0), base + j * rs * 4, nc * 4});
        for (uint64_t i = 0; i < nout; ++i) w.out.push_back({(uint8_t*)(out[i] + c0), base + (nin + i) * rs * 4, nc * 4});
      },
      [&](uint64_t c, int s, hipStream_t st, uint8_t* base) -> int {
        const uint64_t nc = std::min(cl, L - c * cl);
        const uint32_t* di = (const uint32_t*)(base + (size_t)s * stage_dev);
        return execute(plan, di, 0, rs, (uint32_t*)di + nin * rs, 0, rs, nc, 1, st);
      },
      [](uint64_t) {}, stage_dev);
}

}  // namespace slime
