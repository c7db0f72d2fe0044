// C-ABI of the MI355X Reed-Solomon shard codec (include/slime_rs.h).
//
// Go-API entry points mirror internal/rs and internal/rs/gf: same argument
// meaning, same validation order, and the reference's panic text through
// slime_rs_status_string().  All data-path work runs on the GPU through the
// kernels in rs_apply.hip / gf_codec.hip; with no device the compute entry
// points fail with SLIME_RS_ERR_NO_DEVICE (there is no CPU fallback).
#include "slime_rs.h"

#include <hip/hip_runtime.h>
#include <ctype.h>
#include <sched.h>
#include <stdio.h>
#include <string.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <tuple>
#include <vector>

#include "capi_common.hpp"
#include "device_pool.hpp"
#include "digest.hpp"
#include "gfp_host.hpp"
#include "host_codec.hpp"
#include "host_copy.hpp"
#include "kernels.hpp"
#include "mfma_table.hpp"
#include "plan_cache.hpp"
#include "rs_matrix.hpp"

struct slime_rs_plan {
  int device = 0;
  // Set by the first launch; slime_rs_plan_set_outputs refuses afterwards
  // (its table rewrite is not ordered against launches in flight).
  std::atomic<bool> executed{false};
  uint32_t rows = 0, k = 0;
  uint32_t out_max = 0;         // highest destination shard index
  std::vector<uint32_t> in_idx_host;  // input shard indices (host copy, bounds checks)
  std::vector<uint32_t> coeff;  // rows x k, host copy
  uint32_t* table = nullptr;    // device: coeff (rows x coeff_stride(k)) | in_idx (k) | out_idx (rows)
  const uint32_t* d_coeff = nullptr;
  const uint32_t* d_in_idx = nullptr;
  const uint32_t* d_out_idx = nullptr;
  const uint8_t* d_mfma = nullptr;     // device: matrix-core digit table (mfma_table.hpp), or null
  const uint8_t* d_mfma_be = nullptr;  // the same for big-endian chunk words (the byte path)
  uint32_t in_max = 0;              // highest input shard index
};

namespace slime {
namespace {
thread_local std::string t_error;
// Device of the calling thread's host entry points after
// slime_rs_select_device (-1: not selected, the device pool picks).
thread_local int t_device = -1;
// The per-call context of the *_ex entry points (explicit device, detail
// buffer), active for the duration of that one call on this thread.
thread_local const slime_rs_call_t* t_call = nullptr;
std::atomic<int64_t> g_tables_live{0};  // device plan tables allocated and not yet freed
}  // namespace

// capi_common.hpp
int fail(Status st, std::string detail) {
  t_error = std::move(detail);
  return (int)st;
}
int fail_hip(hipError_t e, const char* what) {
  return fail(Status::Hip, std::string(what) + ": " + hipGetErrorString(e));
}

int visible_devices() {
  static const int n = [] {
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    return c;
  }();
  return n;
}

int check_device(int dev) {
  const int n = visible_devices();
  if (n == 0)
    return fail(Status::NoDevice, "no HIP device visible: slime_rs data-path calls need an MI355X (gfx950) GPU");
  if (dev < 0 || dev >= n) return fail(Status::InvalidArg, "device ordinal " + std::to_string(dev) + " out of range");
  return 0;
}

namespace {
// ---- device pool (host entry points) -------------------------------------------
// Routing policy and its CPU test: device_pool.hpp.  Each device has its own
// workspaces and plans (plan keys and workspaces carry the device).
DevicePool g_pool;

const std::vector<int>& pool_devices() {
  static const std::vector<int> devs = DevicePool::allowed(visible_devices(), getenv("SLIME_RS_DEVICES"));
  return devs;
}

// The device of one host call: the *_ex call's explicit device, else the
// thread's selected device, else the pool's pick.  Holds the pool slot for
// the life of the call.
struct DeviceLease {
  PoolLease lease;
  int device = -1;
  int acquire() {
    const int call = t_call ? t_call->device : SLIME_RS_ANY_DEVICE;
    const int thread = t_call ? SLIME_RS_ANY_DEVICE : t_device;
    const int want = call != SLIME_RS_ANY_DEVICE ? call : thread;
    if (int rc = check_device(want != SLIME_RS_ANY_DEVICE ? want : 0)) return rc;
    lease.take(g_pool, call, thread, pool_devices());
    device = lease.device;
    return 0;
  }
};

// ---- plans -----------------------------------------------------------------

int build_plan(int device, uint32_t rows, uint32_t k, const uint32_t* coeff, const std::vector<uint32_t>& in_idx,
               const std::vector<uint32_t>& out_idx, slime_rs_plan** out) {
  if (int rc = check_device(device)) return rc;
  auto plan = std::make_unique<slime_rs_plan>();
  plan->device = device;
  plan->rows = rows;
  plan->k = k;
  plan->coeff.assign(coeff, coeff + (size_t)rows * k);
  plan->out_max = out_idx.empty() ? 0 : *std::max_element(out_idx.begin(), out_idx.end());
  plan->in_idx_host = in_idx;
  const uint32_t cs = coeff_stride(k);
  const size_t ncoef = (size_t)rows * cs;
  const size_t n_in = (k + 3) & ~3u, n_out = (rows + 3) & ~3u;
  // Wide codes also get the matrix-core kernel's digit table (rs_apply_mfma.hip),
  // 16-byte aligned after the index arrays.
  const size_t n_head = (ncoef + n_in + n_out + 3) & ~(size_t)3;
  std::vector<uint8_t> mt, mtb;
  if (k >= 17 && mfma::supported(rows, k)) {
    mt = mfma::build_table(coeff, rows, k, false);
    mtb = mfma::build_table(coeff, rows, k, true);
  }
  std::vector<uint32_t> host(n_head + (mt.size() + mtb.size()) / 4, 0u);
  for (uint32_t i = 0; i < rows; ++i)
    for (uint32_t j = 0; j < k; ++j) host[(size_t)i * cs + j] = coeff[(size_t)i * k + j] % kP;
  std::copy(in_idx.begin(), in_idx.end(), host.begin() + ncoef);
  std::copy(out_idx.begin(), out_idx.end(), host.begin() + ncoef + n_in);
  if (!mt.empty()) {
    memcpy(host.data() + n_head, mt.data(), mt.size());
    memcpy(host.data() + n_head + mt.size() / 4, mtb.data(), mtb.size());
  }
  plan->in_max = in_idx.empty() ? 0 : *std::max_element(in_idx.begin(), in_idx.end());
  DeviceScope ds(device);
  void* p = nullptr;
  HIP_TRY(hipMalloc(&p, host.size() * sizeof(uint32_t)));
  if (hipMemcpy(p, host.data(), host.size() * sizeof(uint32_t), hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipFree(p);
    return fail(Status::Hip, "plan table upload failed");
  }
  plan->table = (uint32_t*)p;
  g_tables_live.fetch_add(1, std::memory_order_relaxed);
  // The device's first ticket-counter sets, created here (never inside a
  // capture) so that a launch of this plan captured into a graph finds them.
  if (hipError_t e = warm_ticket_pool(device)) {
    (void)hipFree(p);
    g_tables_live.fetch_sub(1, std::memory_order_relaxed);
    return fail_hip(e, "ticket counter sets");
  }
  plan->d_coeff = plan->table;
  plan->d_in_idx = plan->table + ncoef;
  plan->d_out_idx = plan->table + ncoef + n_in;
  if (!mt.empty()) {
    plan->d_mfma = reinterpret_cast<const uint8_t*>(plan->table + n_head);
    plan->d_mfma_be = reinterpret_cast<const uint8_t*>(plan->table + n_head + mt.size() / 4);
  }
  *out = plan.release();
  return 0;
}

void destroy_plan(slime_rs_plan* plan) {
  if (!plan) return;
  if (plan->table) {
    DeviceScope ds(plan->device);
    (void)hipFree(plan->table);
    g_tables_live.fetch_sub(1, std::memory_order_relaxed);
  }
  delete plan;
}

bool aligned4(const void* p) { return ((uintptr_t)p & 3u) == 0; }

int execute(const slime_rs_plan* plan, const uint32_t* src, uint64_t src_obj, uint64_t src_shard, uint32_t* dst,
            uint64_t dst_obj, uint64_t dst_shard, uint64_t L, uint64_t nobj, hipStream_t stream) {
  if (nobj > 0xFFFFFFFFull) return fail(Status::InvalidArg, "nobj exceeds 2^32-1");
  ApplyLaunch a;
  a.in = src;
  a.out = dst;
  a.in_obj_stride = src_obj;
  a.in_shard_stride = src_shard;
  a.out_obj_stride = dst_obj;
  a.out_shard_stride = dst_shard;
  a.coeff = plan->d_coeff;
  a.in_idx = plan->d_in_idx;
  a.out_idx = plan->d_out_idx;
  a.ncols = L;
  a.nobj = (uint32_t)nobj;
  a.rows = plan->rows;
  a.k = plan->k;
  // The 16-byte-per-lane kernel needs only 4-byte alignment: gfx9+ runs with
  // unaligned memory access enabled (SH_MEM_CONFIG alignment_mode =
  // UNALIGNED), so dwordx4 loads/stores of shards whose stride is not a
  // multiple of 4 symbols (e.g. 10/14 on 1 GiB objects: L = 26843546) stay
  // vectorised.  16-byte aligned layouts are faster; pad strides where the
  // layout is yours to choose.
  a.vec_ok = aligned4(src) && aligned4(dst);
  a.mfma = plan->d_mfma;
  a.in_max = plan->in_max;
  a.out_max = plan->out_max;
  const_cast<slime_rs_plan*>(plan)->executed.store(true, std::memory_order_relaxed);
  DeviceScope ds(plan->device);
  HIP_TRY(launch_apply(a, stream));
  return 0;
}

// Plans the host entry points reuse, keyed by (device, kind, shape, indices):
// a bounded LRU (plan_cache.hpp).  Env SLIME_RS_PLAN_CACHE sets the capacity
// (default 256 plans: at 20/40 a recovery plan's table is about 4 KiB).
using PlanKey = std::tuple<int, char, int, int, std::vector<int>>;
using PlanRef = std::shared_ptr<slime_rs_plan>;
// Never destroyed: freeing device tables from a static destructor would run
// after the HIP runtime may have shut down.
LruCache<PlanKey, slime_rs_plan>& plans() {
  static auto* c = new LruCache<PlanKey, slime_rs_plan>([] {
    const char* e = getenv("SLIME_RS_PLAN_CACHE");
    const long long v = e ? atoll(e) : 0;
    return v > 0 ? (size_t)v : (size_t)256;
  }());
  return *c;
}

int cached_plan(const PlanKey& key, PlanRef* out, int (*make)(const PlanKey&, slime_rs_plan**)) {
  const int rc = plans().get(key, out, make, destroy_plan);
  if (rc == LruCache<PlanKey, slime_rs_plan>::kBuildThrew)
    return fail(Status::Hip, "plan build failed: host allocation (exception in the plan builder)");
  return rc;
}

// ---- per-call device workspaces (host entry points) ----------------------------

// NUMA placement of a host page, the GPU and the calling CPU (diagnostics:
// SLIME_RS_PIPE_TRACE).  -1 where unknown.
struct NumaInfo {
  int page_node = -1, gpu_node = -1, cpu = -1, cpu_node = -1;
};

int sysfs_int(const std::string& path) {
  FILE* f = fopen(path.c_str(), "r");
  if (!f) return -1;
  int v = -1;
  if (fscanf(f, "%d", &v) != 1) v = -1;
  fclose(f);
  return v;
}

NumaInfo numa_info(int device, const void* page) {
  NumaInfo ni;
  int node = -1;
  // get_mempolicy(MPOL_F_NODE | MPOL_F_ADDR): the node backing `page`
  if (syscall(SYS_get_mempolicy, &node, nullptr, 0, page, 3) == 0) ni.page_node = node;
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof(bus), device) == hipSuccess) {
    std::string id(bus);
    for (auto& ch : id) ch = (char)tolower(ch);
    ni.gpu_node = sysfs_int("/sys/bus/pci/devices/" + id + "/numa_node");
  }
  ni.cpu = sched_getcpu();
  if (ni.cpu >= 0)
    for (int n = 0; n < 64; ++n) {
      const std::string d = "/sys/devices/system/node/node" + std::to_string(n) + "/cpu" + std::to_string(ni.cpu);
      if (access(d.c_str(), F_OK) == 0) {
        ni.cpu_node = n;
        break;
      }
    }
  return ni;
}

// Host pipeline depth: stages in flight per call (env SLIME_RS_HOST_STAGES,
// 2..Workspace::kMaxStages, read once; default 3).
int host_stages() {
  static const int s = [] {
    const char* e = getenv("SLIME_RS_HOST_STAGES");
    const int v = e ? atoi(e) : 3;
    return v < 2 ? 2 : v > 6 ? 6 : v;
  }();
  return s;
}

struct Workspace {
  static constexpr int kMaxStages = 6;
  int device = -1;
  hipStream_t stream = nullptr;
  uint8_t* dbuf = nullptr;
  size_t dcap = 0;
  hipStream_t sst[kMaxStages] = {};  // one stream per pipeline stage
  hipEvent_t sev[kMaxStages] = {};   // stage's D2H done
  static constexpr int kParts = 4;
  hipEvent_t pev[kMaxStages][kParts] = {};  // a part of the stage's D2H done (run_windows)
  hipEvent_t cev = nullptr;          // compute stream reached a point (staged_d2h)
  uint8_t* pin = nullptr;            // pinned staging, host_stages() x (in rows | out rows)
  size_t pcap = 0;
  int reserve(size_t bytes) {
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
    size_t want = std::max<size_t>(bytes + bytes / 2, 1u << 20);
    HIP_TRY(hipMalloc((void**)&dbuf, want));
    dcap = want;
    return 0;
  }
  int reserve_pinned(size_t bytes) {
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
    if (getenv("SLIME_RS_PIPE_TRACE")) {
      const NumaInfo ni = numa_info(device, pin);
      fprintf(stderr, "slime_rs pinned %zu MiB: page node %d, gpu node %d, cpu %d (node %d)\n", bytes >> 20,
              ni.page_node, ni.gpu_node, ni.cpu, ni.cpu_node);
    }
    return 0;
  }
  int ensure_stages() {
    if (sst[0]) return 0;
    DeviceScope ds(device);
    for (int i = 0; i < kMaxStages; ++i) {
      HIP_TRY(hipStreamCreateWithFlags(&sst[i], hipStreamNonBlocking));
      HIP_TRY(hipEventCreateWithFlags(&sev[i], hipEventDisableTiming));
      for (int p = 0; p < kParts; ++p) HIP_TRY(hipEventCreateWithFlags(&pev[i][p], hipEventDisableTiming));
    }
    HIP_TRY(hipEventCreateWithFlags(&cev, hipEventDisableTiming));
    return 0;
  }
  // Every stage stream waits for the work queued on `stream` so far (a
  // call's setup: zeroed flags, the mapping) -- ordering on the device, no
  // host round trip.
  int fence_stages(int nstages) {
    if (int rc = ensure_stages()) return rc;
    HIP_TRY(hipEventRecord(cev, stream));
    for (int s = 0; s < nstages && s < kMaxStages; ++s) HIP_TRY(hipStreamWaitEvent(sst[s], cev, 0));
    return 0;
  }
};

PerDeviceFreeList<Workspace> g_ws_free;  // most recently released first (device_pool.hpp)

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

struct WsLease {
  Workspace* ws = nullptr;
  ~WsLease() {
    if (ws) release_ws(ws);
  }
};

size_t round16(size_t n) { return (n + 15) & ~(size_t)15; }

// ---- host <-> device pipeline for the Go-API entry points ----------------------
//
// Column-chunked and host_stages() deep: chunk c's H2D / kernel / D2H run on stage
// stream c % S while the host thread copies chunk c-S's results out of pinned
// memory and chunk c's inputs into it (host_copy.cpp spreads those memcpys
// over a small pool).  The caller's buffers stay pageable; only the staging
// ring is pinned, so nothing is registered per call.

constexpr size_t kStageBytes = 8u << 20;      // in + out bytes one stage moves (Go-API rows)
// Bytes one window of the object entry points moves (env
// SLIME_RS_OBJ_WINDOW_MIB, 1..256, read once; default 16).
size_t obj_window_bytes() {
  static const size_t b = [] {
    const char* e = getenv("SLIME_RS_OBJ_WINDOW_MIB");
    const long v = e ? atol(e) : 16;
    return (size_t)(v < 1 ? 1 : v > 256 ? 256 : v) << 20;
  }();
  return b;
}

enum class HostPipe : int { Staged = 0, Register = 1, Direct = 2 };

std::atomic<int> g_host_pipe{[] {
  const char* e = getenv("SLIME_RS_HOST_PIPE");
  if (e && strcmp(e, "direct") == 0) return (int)HostPipe::Direct;      // one-shot pageable copies
  if (e && strcmp(e, "register") == 0) return (int)HostPipe::Register;  // pin caller rows per call
  return (int)HostPipe::Staged;
}()};

HostPipe host_pipe_mode() { return (HostPipe)g_host_pipe.load(std::memory_order_relaxed); }

int host_apply_direct(Workspace* ws, const slime_rs_plan* plan, const uint32_t* const* in, uint32_t* const* out,
                      uint64_t L) {
  const size_t shard = (L + 63) & ~(size_t)63;  // every shard on a 256 B boundary (line-aligned streams)
  if (int rc = ws->reserve(shard * 4 * ((size_t)plan->k + plan->rows))) return rc;
  uint32_t* d_in = (uint32_t*)ws->dbuf;
  uint32_t* d_out = d_in + shard * plan->k;
  for (uint32_t j = 0; j < plan->k; ++j)
    HIP_TRY(hipMemcpyAsync(d_in + shard * j, in[j], L * 4, hipMemcpyHostToDevice, ws->stream));
  if (int rc = execute(plan, d_in, 0, shard, d_out, 0, shard, L, 1, ws->stream)) return rc;
  for (uint32_t i = 0; i < plan->rows; ++i)
    HIP_TRY(hipMemcpyAsync(out[i], d_out + shard * i, L * 4, hipMemcpyDeviceToHost, ws->stream));
  HIP_TRY(hipStreamSynchronize(ws->stream));
  return 0;
}

// ---- staged whole-buffer transfers (object entry points) -------------------------
//
// A span is a host range and its device offset.  Spans are cut into pieces
// of at most kStageBytes; piece p goes through pinned stage p % S, so the host
// memcpy of one piece overlaps the DMA of the previous ones.

struct Span {
  uint8_t* host;
  uint64_t dev_off;
  uint64_t bytes;
};

std::vector<Span> pieces_of(const Span* sp, size_t n) {
  std::vector<Span> out;
  for (size_t i = 0; i < n; ++i)
    for (uint64_t off = 0; off < sp[i].bytes; off += kStageBytes)
      out.push_back({sp[i].host + off, sp[i].dev_off + off, std::min<uint64_t>(kStageBytes, sp[i].bytes - off)});
  return out;
}

int stage_ring(Workspace* ws) {
  if (int rc = ws->reserve_pinned(kStageBytes * host_stages())) return rc;
  return ws->ensure_stages();
}

// dev -> host spans after everything queued on ws->stream so far; returns
// when the host copies are complete.
int staged_d2h(Workspace* ws, const uint8_t* dev, const Span* sp, size_t n) {
  if (int rc = stage_ring(ws)) return rc;
  const std::vector<Span> pcs = pieces_of(sp, n);
  const int S = host_stages();
  HIP_TRY(hipEventRecord(ws->cev, ws->stream));
  for (int s = 0; s < S; ++s) HIP_TRY(hipStreamWaitEvent(ws->sst[s], ws->cev, 0));
  auto land = [&](size_t p) -> int {
    const int s = (int)(p % S);
    HIP_TRY(hipEventSynchronize(ws->sev[s]));
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

void drain_stages(Workspace* ws) {
  if (ws->stream) (void)hipStreamSynchronize(ws->stream);
  for (hipStream_t st : ws->sst)
    if (st) (void)hipStreamSynchronize(st);
}

// ---- windowed pipeline ------------------------------------------------------------
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
  std::vector<size_t> part_end;         // out spans [part_end[p-1], part_end[p]) are D2H part p
};

// A one-window call's download of at least this many bytes goes as up to
// Workspace::kParts parts, each with its own event, so the host copies part
// p out of the ring while part p+1 still crosses PCIe (8 MiB reconstruct
// 496-522 -> 453-486 us, profiles/r04/s34_parts; env SLIME_RS_D2H_PARTS:
// parts, 1 = one download).
int d2h_parts() {
  static const int p = [] {
    const char* e = getenv("SLIME_RS_D2H_PARTS");
    const int v = e ? atoi(e) : 4;
    return v < 1 ? 1 : v > 4 ? 4 : v;
  }();
  return p;
}
constexpr uint64_t kPartedD2H = 8u << 20;

size_t round64(size_t n) { return (n + 63) & ~(size_t)63; }

// DMA spans one by one, merging neighbours contiguous on both sides.
// Runs of equal-length spans at constant device and pinned strides (a
// window's rows: one per chunk) go as one pitched copy (env SLIME_RS_DMA_2D=0:
// a copy per span).  Per-span copies reach the copy engine as separate
// commands ~10 us apart: a 64 MiB reconstruct's eight 1 MiB uploads per
// window ran back to back with those gaps, and one pitched copy took the
// fused reconstruct from 22 to 27 GiB/s and write_chunks from 32 to 36
// (profiles/r04/s24_rctrace, s25_dma2d).
bool dma_2d() {
  static const bool on = [] {
    const char* e = getenv("SLIME_RS_DMA_2D");
    return !(e && e[0] == '0');
  }();
  return on;
}

// Windows moving at most this many bytes one way go as one copy kernel over
// the mapped pinned ring instead of copy-engine transfers (host_blit.hip):
// uploads up to 4 MiB (env SLIME_RS_BLIT_KIB; a kernel reading host memory
// is latency-bound, so larger uploads keep the copy engines: a 64 MiB
// CreateParity ran 1.88 ms instead of 1.41 with kernel uploads), downloads
// of every window size (env SLIME_RS_BLIT_D2H_KIB, default 64 MiB: the
// kernel's writes are posted and run beside the copy engines' uploads --
// fused reconstruct +4-7%, write_chunks +3-10%, profiles/r04/s19-s20).  0 =
// always the copy engines.
uint64_t env_kib(const char* name, long long dflt) {
  const char* e = getenv(name);
  const long long v = e ? atoll(e) : dflt;
  return v > 0 ? (uint64_t)v << 10 : 0ull;
}
uint64_t blit_max_bytes(bool h2d) {
  static const uint64_t up = env_kib("SLIME_RS_BLIT_KIB", 4096);
  static const uint64_t down = env_kib("SLIME_RS_BLIT_D2H_KIB", 65536);
  return h2d ? up : down;
}

int dma_spans(uint8_t* dev, uint8_t* pin, const std::vector<Span>& sp, const std::vector<size_t>& off, bool h2d,
              hipStream_t st) {
  uint64_t total = 0;
  for (const Span& s : sp) total += s.bytes;
  if (total && total <= blit_max_bytes(h2d)) {
    std::vector<BlitSpan> bl;
    bl.reserve(sp.size());
    for (size_t i = 0; i < sp.size();) {  // neighbours contiguous on both sides merge, as below
      size_t j = i + 1, bytes = sp[i].bytes;
      while (j < sp.size() && sp[j].dev_off == sp[i].dev_off + bytes && off[j] == off[i] + bytes) bytes += sp[j++].bytes;
      if (h2d)
        bl.push_back({dev + sp[i].dev_off, pin + off[i], bytes});
      else
        bl.push_back({pin + off[i], dev + sp[i].dev_off, bytes});
      i = j;
    }
    HIP_TRY(launch_blit(bl.data(), (int)bl.size(), st));
    return 0;
  }
  if (dma_2d() && sp.size() >= 2) {
    for (size_t i = 0; i < sp.size();) {
      size_t j = i + 1;
      const uint64_t bytes = sp[i].bytes;
      const int64_t dd = j < sp.size() ? (int64_t)sp[j].dev_off - (int64_t)sp[i].dev_off : 0;
      const int64_t dp = j < sp.size() ? (int64_t)off[j] - (int64_t)off[i] : 0;
      if (dd >= (int64_t)bytes && dp >= (int64_t)bytes)
        while (j < sp.size() && sp[j].bytes == bytes && (int64_t)sp[j].dev_off - (int64_t)sp[j - 1].dev_off == dd &&
               (int64_t)off[j] - (int64_t)off[j - 1] == dp)
          ++j;
      if (j - i >= 2) {
        if (h2d)
          HIP_TRY(hipMemcpy2DAsync(dev + sp[i].dev_off, (size_t)dd, pin + off[i], (size_t)dp, bytes, j - i,
                                   hipMemcpyHostToDevice, st));
        else
          HIP_TRY(hipMemcpy2DAsync(pin + off[i], (size_t)dp, dev + sp[i].dev_off, (size_t)dd, bytes, j - i,
                                   hipMemcpyDeviceToHost, st));
      } else {
        j = i + 1;
        if (h2d)
          HIP_TRY(hipMemcpyAsync(dev + sp[i].dev_off, pin + off[i], bytes, hipMemcpyHostToDevice, st));
        else
          HIP_TRY(hipMemcpyAsync(pin + off[i], dev + sp[i].dev_off, bytes, hipMemcpyDeviceToHost, st));
      }
      i = j;
    }
    return 0;
  }
  for (size_t i = 0; i < sp.size();) {
    size_t j = i + 1, bytes = sp[i].bytes;
    while (j < sp.size() && sp[j].dev_off == sp[i].dev_off + bytes && off[j] == off[i] + bytes) bytes += sp[j++].bytes;
    if (h2d)
      HIP_TRY(hipMemcpyAsync(dev + sp[i].dev_off, pin + off[i], bytes, hipMemcpyHostToDevice, st));
    else
      HIP_TRY(hipMemcpyAsync(pin + off[i], dev + sp[i].dev_off, bytes, hipMemcpyDeviceToHost, st));
    i = j;
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
// 0 = never.
uint64_t direct_max_bytes() {
  static const uint64_t v = env_kib("SLIME_RS_DIRECT_KIB", 16384);
  return v;
}
// Pinned stage of a direct call: at least this much, as the device buffer
// (Workspace::reserve), so the kernel finds the same room past the layout.
constexpr size_t kDirectPinned = 1u << 20;

// Process-wide split of host-pipeline time (slime_rs_host_stats): where the
// host entry points spend their wall time, in microseconds.
struct HostStats {
  std::atomic<uint64_t> calls{0}, windows{0}, copy_in_us{0}, enqueue_us{0}, wait_us{0}, copy_out_us{0}, total_us{0};
};
HostStats g_host_stats;

// io(c, s, Window&) fills window c's spans; launch(c, s, stream, base)
// enqueues its kernels over the window's device layout at `base` (dev, or
// the pinned stage in a direct call); landed(c) runs once window c's outputs
// are in the caller's buffers (windows land in order).  direct_bytes: the
// size of one window's device layout when the caller's kernels may run on
// the pinned stage (direct_max_bytes), else 0.  SLIME_RS_PIPE_TRACE=1 prints
// each call's split of host time to stderr.
template <class Io, class Launch, class Landed>
int run_windows(const char* what, Workspace* ws, uint8_t* dev, uint64_t n, size_t stage_bytes, Io&& io,
                Launch&& launch, Landed&& landed, size_t direct_bytes = 0) {
  if (n == 0) return 0;
  static const bool trace = getenv("SLIME_RS_PIPE_TRACE") != nullptr;
  using clk = std::chrono::steady_clock;
  auto ms_since = [](clk::time_point t) { return std::chrono::duration<double, std::milli>(clk::now() - t).count(); };
  const auto t_start = clk::now();
  double t_in = 0, t_wait = 0, t_out = 0, t_enq = 0, t_h2d = 0, t_launch = 0;
  const int S = (int)std::min<uint64_t>(host_stages(), n);
  const bool may_direct = n == 1 && direct_bytes && direct_bytes <= 8 * direct_max_bytes();
  if (int rc = ws->reserve_pinned(may_direct ? std::max(std::max(stage_bytes, direct_bytes), kDirectPinned)
                                             : stage_bytes * S))
    return rc;
  if (int rc = ws->ensure_stages()) return rc;
  std::vector<Window> win(S);
  std::vector<CopyItem> items;
  auto pin_of = [&](int s) { return ws->pin + (size_t)s * stage_bytes; };
  auto wait_stage = [&](int s) -> int {
    const auto t0 = clk::now();
    HIP_TRY(hipEventSynchronize(ws->sev[s]));
    t_wait += ms_since(t0);
    return 0;
  };
  auto add_out_items = [&](int s) {  // stage s's landed outputs -> the caller's buffers
    const Window& w = win[s];
    for (size_t i = 0; i < w.out.size(); ++i) items.push_back({w.out[i].host, pin_of(s) + w.out_off[i], w.out[i].bytes});
  };
  auto land = [&](int s) -> int {
    const Window& w = win[s];
    if (w.part_end.size() > 1) {  // part by part, as each part's download completes
      size_t i0 = 0;
      for (size_t p = 0; p < w.part_end.size(); ++p) {
        auto t0 = clk::now();
        HIP_TRY(hipEventSynchronize(ws->pev[s][p]));
        t_wait += ms_since(t0);
        t0 = clk::now();
        items.clear();
        for (size_t i = i0; i < w.part_end[p]; ++i)
          items.push_back({w.out[i].host, pin_of(s) + w.out_off[i], w.out[i].bytes});
        parallel_copy(items.data(), items.size());
        t_out += ms_since(t0);
        i0 = w.part_end[p];
      }
      if (int rc = wait_stage(s)) return rc;  // the stage's own event, recorded after the last part
      landed(w.index);
      return 0;
    }
    if (int rc = wait_stage(s)) return rc;
    const auto t0 = clk::now();
    items.clear();
    add_out_items(s);
    parallel_copy(items.data(), items.size());
    t_out += ms_since(t0);
    landed(w.index);
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
        HIP_TRY(hipEventRecord(ws->sev[s], st));
        w.part_end.clear();
        const double e = ms_since(t0);
        t_enq += e;
        t_launch += e;
        if (!w.host.empty()) {
          t0 = clk::now();
          parallel_copy(w.host.data(), w.host.size());
          t_in += ms_since(t0);
        }
        continue;
      }
      if (int rc = dma_spans(dev, pin, w.in, w.in_off, true, st)) return rc;
      const double a = ms_since(t0);
      if (int rc = launch(c, s, st, dev)) return rc;
      const double b = ms_since(t0);
      uint64_t out_bytes = 0;
      for (const Span& o : w.out) out_bytes += o.bytes;
      // Only a call of one window lands every window alone; in longer calls
      // the parts measured no better (64 MiB reconstruct 26.2 vs 27.8 GiB/s).
      const size_t parts = n == 1 && out_bytes >= kPartedD2H ? std::min<size_t>(d2h_parts(), w.out.size()) : 1;
      w.part_end.clear();
      if (parts > 1) {
        std::vector<Span> psp;
        std::vector<size_t> poff;
        for (size_t p = 0, r0 = 0; p < parts; ++p) {
          const size_t r1 = w.out.size() * (p + 1) / parts;
          psp.assign(w.out.begin() + r0, w.out.begin() + r1);
          poff.assign(w.out_off.begin() + r0, w.out_off.begin() + r1);
          if (int rc = dma_spans(dev, pin, psp, poff, false, st)) return rc;
          HIP_TRY(hipEventRecord(ws->pev[s][p], st));
          w.part_end.push_back(r1);
          r0 = r1;
        }
      } else if (int rc = dma_spans(dev, pin, w.out, w.out_off, false, st)) {
        return rc;
      }
      HIP_TRY(hipEventRecord(ws->sev[s], st));
      t_enq += ms_since(t0);
      t_h2d += a;
      t_launch += b - a;
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
  const double t_total = ms_since(t_start);
  auto us = [](double ms) { return (uint64_t)(ms * 1e3 + 0.5); };
  g_host_stats.calls.fetch_add(1, std::memory_order_relaxed);
  g_host_stats.windows.fetch_add(n, std::memory_order_relaxed);
  g_host_stats.copy_in_us.fetch_add(us(t_in), std::memory_order_relaxed);
  g_host_stats.enqueue_us.fetch_add(us(t_enq), std::memory_order_relaxed);
  g_host_stats.wait_us.fetch_add(us(t_wait), std::memory_order_relaxed);
  g_host_stats.copy_out_us.fetch_add(us(t_out), std::memory_order_relaxed);
  g_host_stats.total_us.fetch_add(us(t_total), std::memory_order_relaxed);
  if (trace)
    fprintf(stderr,
            "slime_rs %s windows=%llu copy_in=%.3f enqueue=%.3f (h2d %.3f launch %.3f d2h %.3f) wait=%.3f "
            "copy_out=%.3f total=%.3f ms\n",
            what, (unsigned long long)n, t_in, t_enq, t_h2d, t_launch, t_enq - t_h2d - t_launch, t_wait, t_out,
            t_total);
  return rc;
}

template <class Io, class Launch>
int run_windows(const char* what, Workspace* ws, uint8_t* dev, uint64_t n, size_t stage_bytes, Io&& io,
                Launch&& launch) {
  return run_windows(what, ws, dev, n, stage_bytes, io, launch, [](uint64_t) {});
}

// Columns per window so that one window moves about `stage` bytes over
// `rows` rows of 4-byte symbols; a multiple of 4096 (16 KiB per row), or the
// whole length in one window.
uint64_t window_cols(uint64_t L, uint64_t rows, size_t stage) {
  const uint64_t cl = std::max<uint64_t>(stage / (rows * 4), 4096) & ~4095ull;
  return cl >= L ? L : cl;
}

int host_apply_staged(Workspace* ws, const slime_rs_plan* plan, const uint32_t* const* in, uint32_t* const* out,
                      uint64_t L) {
  const uint64_t nin = plan->k, nout = plan->rows;
  const uint64_t cl = window_cols(L, nin + nout, kStageBytes);
  const uint64_t n = (L + cl - 1) / cl;
  const uint64_t rs = (cl + 63) & ~63ull;  // device row stride: 256 B aligned rows (line-aligned streams)
  const size_t stage_dev = (size_t)(nin + nout) * rs * 4;
  if (int rc = ws->reserve(stage_dev * std::min<uint64_t>(host_stages(), n))) return rc;
  uint8_t* const dev = ws->dbuf;
  return run_windows(
      "rows", ws, dev, n, (size_t)(nin + nout) * round64(rs * 4),
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

// Register mode: page-lock the caller's rows for the duration of the call
// and DMA straight from / to them (no host memcpy at all).  Returns -1 when
// registration is refused (read-only or already-registered pages) so the
// caller can stage instead.
int host_apply_registered(Workspace* ws, const slime_rs_plan* plan, const uint32_t* const* in, uint32_t* const* out,
                          uint64_t L) {
  const uint64_t nin = plan->k, nout = plan->rows;
  std::vector<void*> reg;
  reg.reserve(nin + nout);
  auto unregister = [&] {
    for (void* p : reg) (void)hipHostUnregister(p);
  };
  auto pin_row = [&](const void* p) -> bool {
    if (hipHostRegister(const_cast<void*>(p), L * 4, hipHostRegisterDefault) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    reg.push_back(const_cast<void*>(p));
    return true;
  };
  for (uint64_t j = 0; j < nin; ++j)
    if (!pin_row(in[j])) return unregister(), -1;
  for (uint64_t i = 0; i < nout; ++i)
    if (!pin_row(out[i])) return unregister(), -1;
  uint64_t cl = std::max<uint64_t>(4 * kStageBytes / ((nin + nout) * 4), 4096) & ~4095ull;
  if (cl >= L) cl = (L + 63) & ~63ull;  // row stride: 256 B aligned
  const uint64_t nch = (L + cl - 1) / cl;
  const int S = (int)std::min<uint64_t>(host_stages(), nch);
  const size_t stage_words = (size_t)(nin + nout) * cl;
  int rc = ws->reserve(stage_words * 4 * S);
  if (!rc) rc = ws->ensure_stages();
  auto body = [&]() -> int {
    uint32_t* const dev = (uint32_t*)ws->dbuf;
    for (uint64_t c = 0; c < nch; ++c) {
      const int s = (int)(c % S);
      const uint64_t c0 = c * cl, n = std::min(cl, L - c0);
      uint32_t* di = dev + s * stage_words;
      hipStream_t st = ws->sst[s];
      for (uint64_t j = 0; j < nin; ++j)
        HIP_TRY(hipMemcpyAsync(di + j * cl, in[j] + c0, n * 4, hipMemcpyHostToDevice, st));
      if (int e = execute(plan, di, 0, cl, di + nin * cl, 0, cl, n, 1, st)) return e;
      for (uint64_t i = 0; i < nout; ++i)
        HIP_TRY(hipMemcpyAsync(out[i] + c0, di + (nin + i) * cl, n * 4, hipMemcpyDeviceToHost, st));
    }
    return 0;
  };
  if (!rc) rc = body();
  for (int s = 0; s < S; ++s)
    if (ws->sst[s] && hipStreamSynchronize(ws->sst[s]) != hipSuccess && !rc) rc = fail_hip(hipGetLastError(), "stage sync");
  unregister();
  return rc;
}


// out[i][0:L] = sum_j coeff[i][j] * in[j][0:L] for a plan whose inputs are
// 0..k-1 and outputs 0..rows-1 (host memory on both sides).
int host_apply(const slime_rs_plan* plan, const uint32_t* const* in, uint32_t* const* out, uint64_t L) {
  WsLease lease;
  if (int rc = acquire_ws(plan->device, &lease.ws)) return rc;
  DeviceScope ds(plan->device);
  switch (host_pipe_mode()) {
    case HostPipe::Direct:
      return host_apply_direct(lease.ws, plan, in, out, L);
    case HostPipe::Register:
      if (int rc = host_apply_registered(lease.ws, plan, in, out, L); rc != -1) return rc;
      [[fallthrough]];
    case HostPipe::Staged:
    default:
      return host_apply_staged(lease.ws, plan, in, out, L);
  }
}

// ---- MapToGF fallback candidates (the reference's rand.Uint32() stream) ------

std::mutex g_rng_mu;
std::mt19937_64 g_rng{std::random_device{}()};

const char* status_text(int st) {
  switch (st) {
    case 0: return "ok";
    case 1: return "CreateParity called on data chunks of varying length";
    case 2: return "RecoverData: len(chunks) != len(indices)";
    case 3: return "RecoverData: len(chunks) == 0";
    case 4: return "RecoverData: No indices given";
    case 5: return "Couldn't ensure nonzero m[i][i]";
    case 6: return "Couldn't ensure one m[i][i]";
    case 7: return "Couldn't ensure zero m[i][j]";
    case 8: return "runtime error: index out of range";
    case 9: return "invalid argument";
    case 10: return "no HIP device";
    case 11: return "HIP runtime error";
    case 12: return "no mapping value found";
    case 13: return "bad checksum after reconstruction";
    default: return "unknown status";
  }
}

int status_of(Status st, const char* what) {
  if (st == Status::Ok) return 0;
  return fail(st, std::string(what) + ": " + status_text((int)st));
}

}  // namespace
}  // namespace slime

using namespace slime;

extern "C" {

const char* slime_rs_status_string(int status) { return status_text(status); }
const char* slime_rs_last_error(void) { return t_error.c_str(); }
const char* slime_rs_version(void) { return "slime_rs 0.1 (gfx950, GF(2^32-5))"; }
int slime_rs_device_count(void) { return visible_devices(); }

int slime_rs_host_pipeline(int mode) {
  if (mode < 0) return g_host_pipe.load();
  if (mode > 2) return fail(Status::InvalidArg, "host_pipeline: mode must be 0 (staged), 1 (register) or 2 (direct)");
  g_host_pipe.store(mode);
  return 0;
}

int slime_rs_kernel_pipeline(int mode) {
  if (mode < 0) return pipelined_kernels() ? 1 : 0;
  if (mode > 1) return fail(Status::InvalidArg, "kernel_pipeline: mode must be 0 or 1");
  set_pipelined_kernels(mode == 1);
  return 0;
}

int slime_rs_kernel_schedule(int mode) {
  if (mode < 0) return queue_mode();
  if (mode > 2)
    return fail(Status::InvalidArg,
                "kernel_schedule: mode must be 0 (static), 1 (dynamic outside graph captures) or 2 (dynamic also "
                "in captures)");
  set_queue_mode(mode);
  return 0;
}

int slime_rs_kernel_matrix_cores(int mode) {
  if (mode < 0) return matrix_core_mode();
  if (mode > 1) return fail(Status::InvalidArg, "kernel_matrix_cores: mode must be 0 (VALU) or 1 (matrix cores)");
  set_matrix_core_mode(mode);
  return 0;
}

int slime_rs_ticket_sets(int device, uint64_t* sets, uint64_t* held) {
  if (!sets || !held) return fail(Status::InvalidArg, "ticket_sets: null output");
  if (int rc = check_device(device)) return rc;
  ticket_pool_stats(device, sets, held);
  return 0;
}

int slime_rs_schedule_counts(int device, uint64_t* dynamic, uint64_t* fallback) {
  if (!dynamic || !fallback) return fail(Status::InvalidArg, "schedule_counts: null output");
  if (int rc = check_device(device)) return rc;
  schedule_counts(device, dynamic, fallback);
  return 0;
}

int slime_rs_selected_device(void) { return t_device; }

int slime_rs_select_device(int device) {
  if (device != SLIME_RS_ANY_DEVICE)
    if (int rc = check_device(device)) return rc;
  t_device = device;
  return 0;
}

// ---- gf scalars / host matrices -------------------------------------------------

uint32_t slime_gf_max_val(void) { return kP; }
uint32_t slime_gf_minverse(uint32_t in) { return gf_minverse(in); }
uint32_t slime_gf_raise(uint32_t x, uint32_t n) { return gf_raise(x, n); }

void slime_gf_seed(uint64_t seed) {
  std::lock_guard<std::mutex> lk(g_rng_mu);
  g_rng.seed(seed);
}

int slime_rs_vandermonde_matrix(int d, int p, uint32_t* out) {
  if (d < 0 || p < 0 || (!out && d > 0)) return fail(Status::InvalidArg, "vandermonde: bad shape");
  const Matrix m = vandermonde(d, p);
  if (!m.v.empty()) memcpy(out, m.v.data(), m.v.size() * sizeof(uint32_t));
  return 0;
}

int slime_rs_parity_matrix(int d, int p, uint32_t* out) {
  if (d <= 0 || p < 0 || !out) return fail(Status::InvalidArg, "parity_matrix: bad shape");
  Matrix m;
  if (Status st = parity_matrix(d, p, &m); st != Status::Ok) return status_of(st, "ParityMatrix");
  memcpy(out, m.v.data(), m.v.size() * sizeof(uint32_t));
  return 0;
}

int slime_rs_parity_matrix_cached(int d, int p, const uint32_t** out) {
  if (d <= 0 || p < 0 || !out) return fail(Status::InvalidArg, "parity_matrix_cached: bad shape");
  const Matrix* m = nullptr;
  if (Status st = parity_matrix_cached(d, p, &m); st != Status::Ok) return status_of(st, "ParityMatrixCached");
  *out = m->v.data();
  return 0;
}

int slime_rs_solve_sub_identity(uint32_t* m, int rows, int cols) {
  if (rows <= 0 || cols <= 0 || rows < cols || !m) return fail(Status::InvalidArg, "solveSubIdentity: bad shape");
  Matrix w((size_t)rows, (size_t)cols);
  memcpy(w.v.data(), m, w.v.size() * sizeof(uint32_t));
  const Status st = reduce_cols(w);
  memcpy(m, w.v.data(), w.v.size() * sizeof(uint32_t));  // partial progress is visible, as in Go
  return status_of(st, "solveSubIdentity");
}

int slime_rs_invert_matrix(const uint32_t* m, int d, uint32_t* inv) {
  if (d <= 0 || !m || !inv) return fail(Status::InvalidArg, "invertMatrix: bad shape");
  Matrix a((size_t)d, (size_t)d), r;
  memcpy(a.v.data(), m, a.v.size() * sizeof(uint32_t));
  if (Status st = invert(a, &r); st != Status::Ok) return status_of(st, "invertMatrix");
  memcpy(inv, r.v.data(), r.v.size() * sizeof(uint32_t));
  return 0;
}

// ---- plans (device-resident batch API) ------------------------------------------

int slime_rs_plan_matrix(int device, const uint32_t* coeff, int rows, int k, const int* in_shards,
                         slime_rs_plan_t* plan) {
  if (!plan || !coeff || !in_shards || rows <= 0 || k <= 0) return fail(Status::InvalidArg, "plan_matrix: bad args");
  std::vector<uint32_t> in_idx(k), out_idx(rows);
  for (int j = 0; j < k; ++j) {
    if (in_shards[j] < 0) return fail(Status::InvalidArg, "plan_matrix: negative shard index");
    in_idx[j] = (uint32_t)in_shards[j];
  }
  for (int i = 0; i < rows; ++i) out_idx[i] = (uint32_t)i;
  return build_plan(device, (uint32_t)rows, (uint32_t)k, coeff, in_idx, out_idx, plan);
}

int slime_rs_plan_encode(int device, int need, int total, slime_rs_plan_t* plan) {
  if (!plan || need <= 0 || total <= need) return fail(Status::InvalidArg, "plan_encode: need 0 < need < total");
  const Matrix* m = nullptr;
  if (Status st = parity_matrix_cached(need, total - need, &m); st != Status::Ok)
    return status_of(st, "ParityMatrix");
  std::vector<int> in(need);
  for (int j = 0; j < need; ++j) in[j] = j;
  return slime_rs_plan_matrix(device, m->row(need), total - need, need, in.data(), plan);
}

int slime_rs_plan_reconstruct(int device, int need, int total, const int* have, const int* want, int nwant,
                              slime_rs_plan_t* plan) {
  if (!plan || !have || !want || need <= 0 || total < need || nwant <= 0)
    return fail(Status::InvalidArg, "plan_reconstruct: bad args");
  for (int i = 0; i < need; ++i)
    if (have[i] < 0 || have[i] >= total) return fail(Status::IndexRange, "plan_reconstruct: have index out of range");
  for (int i = 0; i < nwant; ++i)
    if (want[i] < 0 || want[i] >= total) return fail(Status::IndexRange, "plan_reconstruct: want index out of range");
  // inv maps the survivors to the data rows (RecoverData, vector.go:69-80).
  Matrix hv((size_t)need, (size_t)need), inv;
  std::vector<uint32_t> row;
  for (int i = 0; i < need; ++i) {
    if (Status st = code_row(need, have[i], &row); st != Status::Ok) return status_of(st, "ParityMatrix");
    std::copy(row.begin(), row.end(), hv.v.begin() + (size_t)i * need);
  }
  if (Status st = invert(hv, &inv); st != Status::Ok) return status_of(st, "invertMatrix");
  // Target row t: data row t of inv, or (parity) code_row(t) * inv.
  std::vector<uint32_t> coeff((size_t)nwant * need);
  for (int w = 0; w < nwant; ++w) {
    const int t = want[w];
    if (t < need) {
      std::copy(inv.row(t), inv.row(t) + need, coeff.begin() + (size_t)w * need);
      continue;
    }
    if (Status st = code_row(need, t, &row); st != Status::Ok) return status_of(st, "ParityMatrix");
    for (int q = 0; q < need; ++q) {
      uint64_t acc = 0;
      for (int j = 0; j < need; ++j) acc = (acc + mulmod(row[j], inv.at(j, q))) % kP;
      coeff[(size_t)w * need + q] = (uint32_t)acc;
    }
  }
  return slime_rs_plan_matrix(device, coeff.data(), nwant, need, have, plan);
}

int slime_rs_plan_execute(slime_rs_plan_t plan, const uint32_t* src, slime_rs_layout_t src_layout, uint32_t* dst,
                          slime_rs_layout_t dst_layout, uint64_t L, uint64_t nobj, void* stream) {
  if (!plan) return fail(Status::InvalidArg, "plan_execute: null plan");
  if (L == 0 || nobj == 0) return 0;
  if (!src || !dst) return fail(Status::InvalidArg, "plan_execute: null buffer");
  return execute(plan, src, src_layout.obj_stride, src_layout.shard_stride, dst, dst_layout.obj_stride,
                 dst_layout.shard_stride, L, nobj, (hipStream_t)stream);
}

int slime_rs_plan_set_outputs(slime_rs_plan_t plan, const int* out_shards) {
  if (!plan || !out_shards) return fail(Status::InvalidArg, "plan_set_outputs: bad args");
  // The table rewrite below is a synchronous copy that nothing orders against
  // launches of this plan still in flight on other streams: only before the
  // plan's first launch.
  if (plan->executed.load(std::memory_order_relaxed))
    return fail(Status::InvalidArg, "plan_set_outputs: plan already launched; build a new plan for other outputs");
  std::vector<uint32_t> idx(plan->rows);
  for (uint32_t i = 0; i < plan->rows; ++i) {
    if (out_shards[i] < 0) return fail(Status::InvalidArg, "plan_set_outputs: negative shard index");
    idx[i] = (uint32_t)out_shards[i];
  }
  DeviceScope ds(plan->device);
  HIP_TRY(hipMemcpy(const_cast<uint32_t*>(plan->d_out_idx), idx.data(), idx.size() * sizeof(uint32_t),
                    hipMemcpyHostToDevice));
  plan->out_max = *std::max_element(idx.begin(), idx.end());
  return 0;
}

int slime_rs_plan_shape(slime_rs_plan_t plan, int* rows, int* k) {
  if (!plan) return fail(Status::InvalidArg, "plan_shape: null plan");
  if (rows) *rows = (int)plan->rows;
  if (k) *k = (int)plan->k;
  return 0;
}

int slime_rs_plan_coefficients(slime_rs_plan_t plan, uint32_t* out) {
  if (!plan || !out) return fail(Status::InvalidArg, "plan_coefficients: bad args");
  memcpy(out, plan->coeff.data(), plan->coeff.size() * sizeof(uint32_t));
  return 0;
}

int slime_rs_plan_destroy(slime_rs_plan_t plan) {
  destroy_plan(plan);
  return 0;
}

// ---- fused byte-domain object pipeline ------------------------------------------------

static uint64_t slot_L(uint64_t S, uint32_t need) { return ((S + 3) / 4 + need - 1) / need; }

// Chunk stride of a slot layout: 0 selects the wire layout (4L, the object's
// bytes contiguous); otherwise >= 4L and a multiple of 4.
static int resolve_cstride(uint64_t L, uint64_t* cstride, const char* what) {
  if (*cstride == 0) *cstride = 4 * L;
  if (*cstride < 4 * L || *cstride % 4)
    return fail(Status::InvalidArg, std::string(what) + ": chunk_stride below 4L or not a multiple of 4");
  return 0;
}

static int check_slots(const slime_rs_plan* plan, const uint8_t* slots, uint64_t slot_stride, uint64_t cstride,
                       uint32_t first_out, const char* what) {
  if (!plan || !slots) return fail(Status::InvalidArg, std::string(what) + ": null plan or slots");
  if (plan->k == 0) return fail(Status::InvalidArg, std::string(what) + ": empty plan");
  uint64_t hi = first_out + plan->out_max;
  for (uint32_t j = 0; j < plan->k; ++j) hi = std::max<uint64_t>(hi, plan->in_idx_host[j]);
  if ((hi + 1) * cstride > slot_stride)
    return fail(Status::InvalidArg, std::string(what) + ": slot_stride smaller than the chunks it must hold");
  return 0;
}

static BytesLaunch bytes_launch(const slime_rs_plan* plan, uint8_t* slots, uint64_t slot_stride, uint64_t cstride,
                                uint64_t L, uint64_t S, uint64_t nobj, int phase, uint32_t* flags,
                                const uint32_t* mapping) {
  const_cast<slime_rs_plan*>(plan)->executed.store(true, std::memory_order_relaxed);
  BytesLaunch a;
  a.slots = slots;
  a.slot_stride = slot_stride;
  a.cstride = cstride;
  a.L = L;
  a.S = S;
  a.nobj = (uint32_t)nobj;
  a.rows = plan->rows;
  a.k = plan->k;
  a.phase = phase;
  a.coeff = plan->d_coeff;
  a.in_idx = plan->d_in_idx;
  a.out_idx = plan->d_out_idx;
  a.flags = flags;
  a.mapping = mapping;
  a.mfma = plan->d_mfma_be;
  a.in_max = plan->in_max;
  a.out_max = plan->out_max;
  return a;
}

// Device scratch for asynchronous launch sequences (the encode's
// mid-object-switch record and redo list): per device, buffers handed to one
// sequence at a time and returned behind an event recorded after its last
// launch, so a buffer is reused only once that sequence has finished --
// whatever stream ran it.  Inside a graph capture no buffer is handed out
// (the caller runs without scratch).
}  // extern "C"
namespace {
struct ScratchBuf {
  uint8_t* p = nullptr;
  uint64_t bytes = 0;
  hipEvent_t ev = nullptr;
};
struct ScratchPool {
  std::mutex mu;
  std::vector<ScratchBuf> bufs;  // free when ev has completed
};
ScratchPool& scratch_pool(int dev) {
  static std::mutex mu;
  static auto* pools = new std::map<int, ScratchPool>();  // never destroyed (see plans())
  std::lock_guard<std::mutex> lock(mu);
  return (*pools)[dev];
}
bool stream_capturing(hipStream_t s) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &st) != hipSuccess) {
    (void)hipGetLastError();
    return true;
  }
  return st != hipStreamCaptureStatusNone;
}
struct ScratchLease {
  int dev = -1;
  hipStream_t stream = nullptr;
  ScratchBuf buf;
  bool held = false;
  // A free buffer of >= bytes on `dev` (current device), or none (ok = false,
  // no error) inside a capture.
  int take(int device, uint64_t bytes, hipStream_t s) {
    dev = device;
    stream = s;
    if (bytes == 0 || stream_capturing(s)) return 0;
    ScratchPool& sp = scratch_pool(dev);
    std::lock_guard<std::mutex> lock(sp.mu);
    for (size_t i = 0; i < sp.bufs.size(); ++i) {
      if (sp.bufs[i].bytes < bytes) continue;
      const hipError_t q = hipEventQuery(sp.bufs[i].ev);
      if (q == hipErrorNotReady) continue;
      if (q != hipSuccess) (void)hipGetLastError();
      buf = sp.bufs[i];
      sp.bufs.erase(sp.bufs.begin() + (long)i);
      held = true;
      return 0;
    }
    const uint64_t want = std::max<uint64_t>(bytes + bytes / 4, 1u << 20);
    HIP_TRY(hipMalloc((void**)&buf.p, want));
    buf.bytes = want;
    if (hipError_t e = hipEventCreateWithFlags(&buf.ev, hipEventDisableTiming)) {
      (void)hipFree(buf.p);
      return fail_hip(e, "scratch event");
    }
    held = true;
    return 0;
  }
  uint8_t* ptr() const { return held ? buf.p : nullptr; }
  // Back to the pool behind an event on `s` (after the sequence's last launch).
  void release(hipStream_t s) {
    if (!held) return;
    held = false;
    if (hipEventRecord(buf.ev, s) != hipSuccess) {
      (void)hipGetLastError();
      (void)hipStreamSynchronize(s);  // cannot observe the release: wait for it here
    }
    ScratchPool& sp = scratch_pool(dev);
    std::lock_guard<std::mutex> lock(sp.mu);
    sp.bufs.push_back(buf);
  }
  ~ScratchLease() {
    if (held) release(stream);  // error paths: behind whatever the sequence queued
  }
};
}  // namespace
extern "C" {

extern "C" int slime_rs_encode_objects_chunked(slime_rs_plan_t plan, uint8_t* slots, uint64_t slot_stride,
                                               uint64_t chunk_stride, uint64_t object_size, uint64_t nobj,
                                               uint32_t* mapping, uint32_t* status, void* stream) {
  if (nobj == 0) return 0;
  if (nobj > 0xFFFFFFFFull) return fail(Status::InvalidArg, "encode_objects: nobj exceeds 2^32-1");
  if (!mapping || !status) return fail(Status::InvalidArg, "encode_objects: null mapping/status");
  const uint64_t L = slot_L(object_size, plan ? plan->k : 1);
  if (int rc = resolve_cstride(L, &chunk_stride, "encode_objects")) return rc;
  // parity row i goes to chunk need + out_idx[i]
  if (int rc = check_slots(plan, slots, slot_stride, chunk_stride, plan ? plan->k : 0, "encode_objects")) return rc;
  hipStream_t s = (hipStream_t)stream;
  DeviceScope ds(plan->device);
  HIP_TRY(hipMemsetAsync(status, 0, nobj * sizeof(uint32_t), s));
  HIP_TRY(hipMemsetAsync(mapping, 0, nobj * sizeof(uint32_t), s));
  if (L == 0) return 0;
  // Phase 0 with the mid-object mapping switch where the dynamic schedule
  // runs (a scratch record of each unit's mapping), so phase 1 redoes only
  // the units encoded before an object's first word >= p was seen.
  BytesLaunch a0 = bytes_launch(plan, slots, slot_stride, chunk_stride, L, object_size, nobj, 0, status, mapping);
  ScratchLease sc;
  if (int rc = sc.take(plan->device, encode_switch_bytes(a0, s), s)) return rc;
  SwitchRecord sw;
  a0.scratch = sc.ptr();
  a0.sw = &sw;
  HIP_TRY(launch_encode_bytes(a0, s));
  HIP_TRY(launch_select_mapping(mapping, status, (uint32_t)nobj, s));
  BytesLaunch a1 = bytes_launch(plan, slots, slot_stride, chunk_stride, L, object_size, nobj, 1, status, mapping);
  if (sw.switched) {
    a1.scratch = sc.ptr();
    a1.sw = &sw;
  }
  HIP_TRY(launch_encode_bytes(a1, s));
  sc.release(s);
  return 0;
}

extern "C" int slime_rs_encode_objects(slime_rs_plan_t plan, uint8_t* slots, uint64_t slot_stride,
                                       uint64_t object_size, uint64_t nobj, uint32_t* mapping, uint32_t* status,
                                       void* stream) {
  return slime_rs_encode_objects_chunked(plan, slots, slot_stride, 0, object_size, nobj, mapping, status, stream);
}

extern "C" int slime_rs_resolve_fallbacks_chunked(slime_rs_plan_t plan, uint8_t* slots, uint64_t slot_stride,
                                                  uint64_t chunk_stride, uint64_t object_size, uint64_t nobj,
                                                  uint32_t* mapping, uint32_t* status, void* stream, int* resolved) {
  if (resolved) *resolved = 0;
  if (nobj == 0) return 0;
  if (!mapping || !status) return fail(Status::InvalidArg, "resolve_fallbacks: null mapping/status");
  const uint64_t L = slot_L(object_size, plan ? plan->k : 1);
  if (int rc = resolve_cstride(L, &chunk_stride, "resolve_fallbacks")) return rc;
  if (int rc = check_slots(plan, slots, slot_stride, chunk_stride, plan ? plan->k : 0, "resolve_fallbacks")) return rc;
  hipStream_t s = (hipStream_t)stream;
  DeviceScope ds(plan->device);
  std::vector<uint32_t> st(nobj);
  HIP_TRY(hipMemcpyAsync(st.data(), status, nobj * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  const uint64_t nw = (object_size + 3) / 4;
  constexpr uint32_t kCand = 64;
  WsLease lease;
  bool have_ws = false;
  for (uint64_t o = 0; o < nobj; ++o) {
    if (st[o] != 1) continue;
    if (!have_ws) {
      if (int rc = acquire_ws(plan->device, &lease.ws)) return rc;
      if (int rc = lease.ws->reserve(round16(nw * 4) + 2 * kCand * 4)) return rc;
      have_ws = true;
    }
    uint32_t* d_words = (uint32_t*)lease.ws->dbuf;
    uint32_t* d_cand = (uint32_t*)(lease.ws->dbuf + round16(nw * 4));
    uint32_t* d_bad = d_cand + kCand;
    uint8_t* slot = slots + o * slot_stride;
    // the object's words, chunk by chunk (object byte i is in chunk i / 4L)
    for (uint64_t j = 0; j * 4 * L < object_size; ++j)
      HIP_TRY(launch_map_pack(slot + j * chunk_stride, std::min<uint64_t>(4 * L, object_size - j * 4 * L), 0,
                              d_words + j * L, nullptr, s));
    uint32_t m = 0;
    bool found = false;
    for (int round = 0; round < (1 << 16) && !found; ++round) {
      uint32_t cand[kCand], bad[kCand];
      {
        std::lock_guard<std::mutex> lk(g_rng_mu);
        for (uint32_t c = 0; c < kCand; ++c) cand[c] = (uint32_t)(g_rng() >> 32);
      }
      HIP_TRY(hipMemcpyAsync(d_cand, cand, sizeof(cand), hipMemcpyHostToDevice, s));
      HIP_TRY(hipMemsetAsync(d_bad, 0, sizeof(bad), s));
      HIP_TRY(launch_mapping_probe(d_words, nw, d_cand, kCand, d_bad, s));
      HIP_TRY(hipMemcpyAsync(bad, d_bad, sizeof(bad), hipMemcpyDeviceToHost, s));
      HIP_TRY(hipStreamSynchronize(s));
      for (uint32_t c = 0; c < kCand && !found; ++c)
        if (!bad[c] && cand[c] != 0) {
          m = cand[c];
          found = true;
        }
    }
    if (!found) return status_of(Status::MappingFallback, "resolve_fallbacks");
    const uint32_t zero = 0;
    HIP_TRY(hipMemcpyAsync(mapping + o, &m, 4, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(status + o, &zero, 4, hipMemcpyHostToDevice, s));
    HIP_TRY(launch_encode_bytes(
        bytes_launch(plan, slot, slot_stride, chunk_stride, L, object_size, 1, 1, status + o, mapping + o), s));
    HIP_TRY(hipStreamSynchronize(s));  // m and zero live on this frame
    if (resolved) ++*resolved;
  }
  return 0;
}

extern "C" int slime_rs_resolve_fallbacks(slime_rs_plan_t plan, uint8_t* slots, uint64_t slot_stride,
                                          uint64_t object_size, uint64_t nobj, uint32_t* mapping, uint32_t* status,
                                          void* stream, int* resolved) {
  return slime_rs_resolve_fallbacks_chunked(plan, slots, slot_stride, 0, object_size, nobj, mapping, status, stream,
                                            resolved);
}

extern "C" int slime_rs_decode_objects_chunked(slime_rs_plan_t plan, uint8_t* slots, uint64_t slot_stride,
                                               uint64_t chunk_stride, uint64_t L, uint64_t nobj,
                                               const uint32_t* mapping, void* stream) {
  if (nobj == 0 || L == 0) return 0;
  if (nobj > 0xFFFFFFFFull) return fail(Status::InvalidArg, "decode_objects: nobj exceeds 2^32-1");
  if (!mapping) return fail(Status::InvalidArg, "decode_objects: null mapping");
  if (int rc = resolve_cstride(L, &chunk_stride, "decode_objects")) return rc;
  if (int rc = check_slots(plan, slots, slot_stride, chunk_stride, 0, "decode_objects")) return rc;
  DeviceScope ds(plan->device);
  HIP_TRY(launch_decode_bytes(bytes_launch(plan, slots, slot_stride, chunk_stride, L, 0, nobj, 0, nullptr, mapping),
                              (hipStream_t)stream));
  return 0;
}

extern "C" int slime_rs_decode_objects(slime_rs_plan_t plan, uint8_t* slots, uint64_t slot_stride, uint64_t L,
                                       uint64_t nobj, const uint32_t* mapping, void* stream) {
  return slime_rs_decode_objects_chunked(plan, slots, slot_stride, 0, L, nobj, mapping, stream);
}

// ---- device codec / fill ------------------------------------------------------------

int slime_gf_pack_device(int device, const uint8_t* bytes, uint64_t len, uint32_t mapping, uint32_t* words,
                         uint32_t* flags, void* stream) {
  if (len == 0) return 0;
  if (!bytes || !words) return fail(Status::InvalidArg, "pack_device: null buffer");
  if (int rc = check_device(device)) return rc;
  DeviceScope ds(device);
  HIP_TRY(launch_map_pack(bytes, len, mapping, words, flags, (hipStream_t)stream));
  return 0;
}

int slime_gf_unpack_device(int device, const uint32_t* words, uint64_t count, uint32_t mapping, uint8_t* bytes,
                           void* stream) {
  if (count == 0) return 0;
  if (!bytes || !words) return fail(Status::InvalidArg, "unpack_device: null buffer");
  if (int rc = check_device(device)) return rc;
  DeviceScope ds(device);
  HIP_TRY(launch_map_unpack(words, count, mapping, bytes, (hipStream_t)stream));
  return 0;
}

int slime_rs_fill_symbols(int device, uint32_t* dst, uint64_t count, uint64_t seed, void* stream) {
  if (count == 0) return 0;
  if (!dst) return fail(Status::InvalidArg, "fill_symbols: null buffer");
  if (int rc = check_device(device)) return rc;
  DeviceScope ds(device);
  HIP_TRY(launch_fill_symbols(dst, count, seed, (hipStream_t)stream));
  return 0;
}

// ---- Go-API data entry points (host memory) ------------------------------------------

static int make_rows_plan(const PlanKey& key, slime_rs_plan** out) {
  // kind 'P': code rows key.indices[...] of a need = key.k code, inputs 0..need-1.
  const int dev = std::get<0>(key), need = std::get<2>(key);
  const std::vector<int>& rows = std::get<4>(key);
  std::vector<uint32_t> coeff;
  std::vector<uint32_t> row;
  for (int r : rows) {
    if (Status st = code_row(need, r, &row); st != Status::Ok) return status_of(st, "ParityMatrix");
    coeff.insert(coeff.end(), row.begin(), row.end());
  }
  std::vector<int> in(need);
  for (int j = 0; j < need; ++j) in[j] = j;
  return slime_rs_plan_matrix(dev, coeff.data(), (int)rows.size(), need, in.data(), out);
}

static int run_rows(int need, const std::vector<int>& rows, const uint32_t* const* data, uint64_t L,
                    uint32_t* const* out) {
  DeviceLease dl;
  if (int rc = dl.acquire()) return rc;
  PlanRef plan;
  if (int rc = cached_plan(PlanKey{dl.device, 'P', need, 0, rows}, &plan, make_rows_plan)) return rc;
  return host_apply(plan.get(), data, out, L);
}

int slime_rs_create_parity(const uint32_t* const* data, const uint64_t* lens, int ndata, int index, uint32_t* out) {
  if (ndata < 0 || (ndata > 0 && (!data || !lens))) return fail(Status::InvalidArg, "CreateParity: bad args");
  for (int i = 1; i < ndata; ++i)
    if (lens[i] != lens[0]) return status_of(Status::VaryingLength, "CreateParity");
  if (ndata == 0) return fail(Status::IndexRange, "runtime error: index out of range [0] with length 0");
  if (index < 0) return fail(Status::IndexRange, "runtime error: index out of range [" + std::to_string(index) + "]");
  std::vector<uint32_t> row;
  if (Status st = code_row(ndata, index, &row); st != Status::Ok) return status_of(st, "ParityMatrixCached");
  const uint64_t L = lens[0];
  if (L == 0) return 0;
  if (!out) return fail(Status::InvalidArg, "CreateParity: null out");
  for (int j = 0; j < ndata; ++j)
    if (!data[j]) return fail(Status::InvalidArg, "CreateParity: null data chunk");
  return run_rows(ndata, std::vector<int>{index}, data, L, &out);
}

int slime_rs_create_parities(const uint32_t* const* data, const uint64_t* lens, int ndata, int total,
                             uint32_t* const* out) {
  if (ndata <= 0 || total < ndata || !data || !lens) return fail(Status::InvalidArg, "CreateParities: bad args");
  for (int i = 1; i < ndata; ++i)
    if (lens[i] != lens[0]) return status_of(Status::VaryingLength, "CreateParity");
  if (total == ndata || lens[0] == 0) return 0;
  if (!out) return fail(Status::InvalidArg, "CreateParities: null out");
  for (int j = 0; j < ndata; ++j)
    if (!data[j]) return fail(Status::InvalidArg, "CreateParities: null data chunk");
  for (int i = 0; i < total - ndata; ++i)
    if (!out[i]) return fail(Status::InvalidArg, "CreateParities: null out row");
  std::vector<int> rows;
  for (int r = ndata; r < total; ++r) rows.push_back(r);
  return run_rows(ndata, rows, data, lens[0], out);
}

// The inverse rows `want` of the survivors' code rows (vector.go:69-77), as
// a plan over the staged chunks at inputs 0..need-1, outputs 0..|want|-1.
static int make_inverse_rows_plan(int dev, int need, const std::vector<int>& have, const std::vector<int>& want,
                                  slime_rs_plan** out) {
  const int total = std::max(need, *std::max_element(have.begin(), have.end()) + 1);
  slime_rs_plan* tmp = nullptr;
  if (int rc = slime_rs_plan_reconstruct(dev, need, total, have.data(), want.data(), (int)want.size(), &tmp))
    return rc;
  std::vector<int> pos(need);
  for (int q = 0; q < need; ++q) pos[q] = q;
  slime_rs_plan* staged = nullptr;
  const int rc = slime_rs_plan_matrix(dev, tmp->coeff.data(), (int)want.size(), need, pos.data(), &staged);
  destroy_plan(tmp);
  if (rc) return rc;
  *out = staged;
  return 0;
}

static int make_recover_plan(const PlanKey& key, slime_rs_plan** out) {
  // kind 'O': all need data rows of the inverse (the fused object path
  // rebuilds whole objects on the device).
  const int need = std::get<2>(key);
  std::vector<int> want(need);
  for (int t = 0; t < need; ++t) want[t] = t;
  return make_inverse_rows_plan(std::get<0>(key), need, std::get<4>(key), want, out);
}

// Data rows of `need` absent from the survivors `have`: the only rows of
// RecoverData's inverse that are not unit rows (vector.go:77-85).
static std::vector<int> erased_rows(int need, const int* have) {
  std::vector<int> e;
  for (int t = 0; t < need; ++t)
    if (std::find(have, have + need, t) == have + need) e.push_back(t);
  return e;
}

static int make_erased_rows_plan(const PlanKey& key, slime_rs_plan** out) {
  // kind 'R': the erased data rows only.
  const int need = std::get<2>(key);
  const std::vector<int>& have = std::get<4>(key);
  return make_inverse_rows_plan(std::get<0>(key), need, have, erased_rows(need, have.data()), out);
}

// RecoverData's index checks (vector.go:65-77): no non-negative index ->
// "No indices given"; a negative index -> Go's index-out-of-range; duplicate
// or otherwise dependent rows -> invertMatrix's panic.
static int check_survivors(int need, const int* indices) {
  int max_index = -1;
  for (int i = 0; i < need; ++i) max_index = std::max(max_index, indices[i]);
  if (max_index == -1) return status_of(Status::NoIndices, "RecoverData");
  for (int i = 0; i < need; ++i)
    if (indices[i] < 0)
      return fail(Status::IndexRange, "runtime error: index out of range [" + std::to_string(indices[i]) + "]");
  Matrix hv((size_t)need, (size_t)need), inv;
  std::vector<uint32_t> row;
  for (int i = 0; i < need; ++i) {
    if (Status st = code_row(need, indices[i], &row); st != Status::Ok) return status_of(st, "ParityMatrixCached");
    std::copy(row.begin(), row.end(), hv.v.begin() + (size_t)i * need);
  }
  if (Status st = invert(hv, &inv); st != Status::Ok) return status_of(st, "RecoverData");
  return 0;
}

int slime_rs_recover_data(const uint32_t* const* chunks, const uint64_t* lens, int nchunks, const int* indices,
                          int nindices, uint32_t* const* out) {
  if (nchunks < 0 || nindices < 0) return fail(Status::InvalidArg, "RecoverData: negative count");
  if (nchunks != nindices) return status_of(Status::LenMismatch, "RecoverData");
  if (nchunks == 0) return status_of(Status::Empty, "RecoverData");
  if (!chunks || !lens || !indices) return fail(Status::InvalidArg, "RecoverData: bad args");
  if (int rc = check_survivors(nchunks, indices)) return rc;
  const int need = nchunks;
  const uint64_t L = lens[0];
  for (int i = 1; i < need; ++i)
    if (lens[i] < L)
      return fail(Status::IndexRange, "runtime error: index out of range [" + std::to_string(lens[i]) +
                                          "] with length " + std::to_string(lens[i]));
  if (L == 0) return 0;
  if (!out) return fail(Status::InvalidArg, "RecoverData: null out");
  for (int i = 0; i < need; ++i)
    if (!chunks[i] || !out[i]) return fail(Status::InvalidArg, "RecoverData: null buffer");

  // vector.go:77-85 applies the whole inverse, but the inverse row of a data
  // shard that survived is a unit row: its output is that chunk mod p, a
  // host pass over memory the caller already holds.  Only the erased data
  // rows cross to the device (need chunks in, the erased rows back).
  const std::vector<int> erased = erased_rows(need, indices);
  auto unit_rows = [&] {
    for (int q = 0; q < need; ++q)
      if (indices[q] < need) host_mod_p(chunks[q], L, out[indices[q]]);
  };
  if (erased.empty()) {
    unit_rows();
    return 0;
  }
  DeviceLease dl;
  if (int rc = dl.acquire()) return rc;
  std::vector<int> have(indices, indices + nindices);
  PlanRef plan;
  if (int rc = cached_plan(PlanKey{dl.device, 'R', need, 0, have}, &plan, make_erased_rows_plan)) return rc;
  std::vector<uint32_t*> rows;
  for (int t : erased) rows.push_back(out[t]);
  // The unit rows run after the pipeline, not beside it on a side thread:
  // that form measured no faster (fresh-page faults of both compete,
  // MEASUREMENTS.md round 4, profiles/r04/s7_hostab).
  if (int rc = host_apply(plan.get(), chunks, rows.data(), L)) return rc;
  unit_rows();
  return 0;
}

// ---- object entry points (host memory): writeChunks / reconstruct ------------------

static int make_encode_plan(const PlanKey& key, slime_rs_plan** out) {
  return slime_rs_plan_encode(std::get<0>(key), std::get<2>(key), std::get<3>(key), out);
}

static int make_object_recover_plan(const PlanKey& key, slime_rs_plan** out) {
  // All need data rows of the inverse, inputs = staged survivors 0..need-1,
  // outputs = chunk positions need..2need-1 (the rebuilt object, in order).
  if (int rc = make_recover_plan(key, out)) return rc;
  const int need = std::get<2>(key);
  std::vector<int> pos(need);
  for (int t = 0; t < need; ++t) pos[t] = need + t;
  if (int rc = slime_rs_plan_set_outputs(*out, pos.data())) {
    destroy_plan(*out);
    *out = nullptr;
    return rc;
  }
  return 0;
}

uint64_t slime_rs_chunk_size(uint64_t size, int need) { return need > 0 ? 4 * slot_L(size, (uint32_t)need) : 0; }

// writeChunks of a code with no parity (need == total; checkConfig admits it,
// multi_config.go:36, and the reference's own tests run 1-of-1 stores,
// multi_test.go:179,257): only MapToGF's mapping depends on the data, so it
// is chosen on the device (pick_mapping) and the chunks are then written on
// the host.  Chunk j = MapFromGF(m, part j): the object's own bytes (the
// mapping cancels, map.go:15-33,103-113), zero low bytes in the object's
// partial last word, then splitVector's zero padding symbols, which
// serialise as BE(m) (multi_store.go:279-296).
static int pick_mapping(hipStream_t st, const uint8_t* d_bytes, uint64_t len, uint32_t* d_words,
                        uint32_t* d_scratch, uint32_t* mapping);

// Data chunk j's bytes past the object (its tail): zero low bytes of the
// object's partial last word, then splitVector's zero symbols serialised under
// mapping m as BE(m) (map.go:28-33,103-113; multi_store.go:279-296).  They
// depend only on m and the object's length, so the host writes them.
static void write_data_tails(uint64_t size, int need, uint64_t chunk, uint8_t* const* chunks, uint32_t m) {
  const uint8_t pad[4] = {(uint8_t)(m >> 24), (uint8_t)(m >> 16), (uint8_t)(m >> 8), (uint8_t)m};
  const uint64_t word_end = 4 * ((size + 3) / 4);  // end of the object's last (possibly partial) word
  for (int j = 0; j < need; ++j) {
    const uint64_t lo = (uint64_t)j * chunk, hi = lo + chunk;
    uint8_t* c = chunks[j];
    const uint64_t body = size > lo ? std::min(size, hi) - lo : 0;
    const uint64_t zero_end = word_end > lo ? std::min(word_end, hi) - lo : 0;
    if (zero_end > body) memset(c + body, 0, zero_end - body);
    for (uint64_t o = std::max(body, zero_end); o < chunk; o += 4) memcpy(c + o, pad, 4);
  }
}

static int write_data_chunks(int dev, const uint8_t* data, uint64_t size, int need, uint8_t* const* chunks,
                             uint32_t* mapping) {
  const uint64_t L = slot_L(size, (uint32_t)need), chunk = 4 * L, nw = (size + 3) / 4;
  WsLease lease;
  if (int rc = acquire_ws(dev, &lease.ws)) return rc;
  Workspace* ws = lease.ws;
  DeviceScope ds(dev);
  const size_t bbytes = round16(size), wbytes = round16(nw * 4);
  if (int rc = ws->reserve(bbytes + wbytes + 4 * (4 + 2 * 64))) return rc;
  uint8_t* d_bytes = ws->dbuf;
  uint32_t* d_words = (uint32_t*)(ws->dbuf + bbytes);
  HIP_TRY(hipMemcpyAsync(d_bytes, data, size, hipMemcpyHostToDevice, ws->stream));
  uint32_t m = 0;
  if (int rc = pick_mapping(ws->stream, d_bytes, size, d_words, (uint32_t*)(ws->dbuf + bbytes + wbytes), &m))
    return rc;
  for (int j = 0; j < need; ++j) {
    const uint64_t lo = (uint64_t)j * chunk;
    const uint64_t body = size > lo ? std::min(size, lo + chunk) - lo : 0;
    if (body && chunks[j] != data + lo) memcpy(chunks[j], data + lo, body);  // an aliased chunk is already the object's bytes
  }
  write_data_tails(size, need, chunk, chunks, m);
  *mapping = m;
  return 0;
}

static int write_chunks_check(const uint8_t* data, uint64_t size, int need, int total, uint8_t* const* chunks,
                              uint32_t* mapping) {
  if (!mapping) return fail(Status::InvalidArg, "write_chunks: null mapping");
  *mapping = 0;
  if (need < 1 || total < need) return fail(Status::InvalidArg, "write_chunks: need must be >= 1 and total >= need");
  if (slot_L(size, (uint32_t)need) == 0) return 0;
  if (!data || !chunks) return fail(Status::InvalidArg, "write_chunks: null buffer");
  for (int i = 0; i < total; ++i)
    if (!chunks[i]) return fail(Status::InvalidArg, "write_chunks: null chunk buffer");
  // Zero-copy data chunks: chunk j < need may BE the object's bytes
  // data + j*chunk when it lies wholly inside the object (its bytes are
  // final as they are: MapFromGF(m, MapToGF(x)) = x, map.go:15-33,103-113).
  // Any other overlap between a chunk buffer and the object is refused.
  const uint64_t chunk = 4 * slot_L(size, (uint32_t)need);
  const uintptr_t d0 = (uintptr_t)data, d1 = d0 + size;
  for (int i = 0; i < total; ++i) {
    const uintptr_t c0 = (uintptr_t)chunks[i], c1 = c0 + chunk;
    if (c1 <= d0 || c0 >= d1) continue;
    if (i < need && c0 == d0 + (uint64_t)i * chunk && (uint64_t)(i + 1) * chunk <= size) continue;
    return fail(Status::InvalidArg, "write_chunks: chunk buffer overlaps the object (only data chunk j may alias "
                                    "data + j*chunk_size, when it lies wholly inside the object)");
  }
  return 0;
}

// writeChunks' device pass; dg (optional) hashes the chunks as they become
// final (WriteChunkDigests): it hears of every parity window that lands, of
// a parity rewrite, and of the final mapping.  Arguments already checked.
static int write_chunks_impl(const uint8_t* data, uint64_t size, int need, int total, uint8_t* const* chunks,
                             uint32_t* mapping, WriteChunkDigests* dg) {
  const uint64_t L = slot_L(size, (uint32_t)need);
  if (L == 0) {  // MapToGF(empty) = (0, []): every chunk is empty
    if (dg) dg->finalize(0);
    return 0;
  }
  DeviceLease dl;
  if (int rc = dl.acquire()) return rc;
  const int dev = dl.device;
  if (total == need) {
    const int rc = write_data_chunks(dev, data, size, need, chunks, mapping);
    if (dg && !rc) dg->finalize(*mapping);
    return rc;
  }
  PlanRef plan_ref;
  if (int rc = cached_plan(PlanKey{dev, 'E', need, total, {}}, &plan_ref, make_encode_plan)) return rc;
  slime_rs_plan* const plan = plan_ref.get();
  WsLease lease;
  if (int rc = acquire_ws(dev, &lease.ws)) return rc;
  Workspace* ws = lease.ws;
  DeviceScope ds(dev);
  const uint64_t chunk = 4 * L, stride = (uint64_t)total * chunk;
  if (int rc = ws->reserve(round16(stride) + 16)) return rc;
  uint8_t* const slot = ws->dbuf;
  uint32_t* const d_map = (uint32_t*)(ws->dbuf + round16(stride));
  uint32_t* const d_status = d_map + 1;
  // Speculative pass (mapping 0) window by window: object bytes in, parity
  // out, MapToGF's flags accumulating on device; the data-chunk bodies below
  // the object's last word are the caller's own bytes (MapFromGF(m,
  // MapToGF(x)) = x, map.go:15-33,103-113) and are placed on the host with
  // each window's inputs.  The device computes every byte that depends on m.
  const int r = total - need;
  const uint64_t cl = window_cols(L, (uint64_t)total, obj_window_bytes());
  const uint64_t nwin = (L + cl - 1) / cl;
  // One window (objects up to about the window size): MapToGF's flags come
  // back with the parity, so a mapping-0 object costs one host round trip
  // in all.
  const bool one = nwin == 1;
  uint32_t ms[2] = {0, 0};
  static const uint32_t kZero[2] = {0, 0};
  bool ran_direct = false;
  auto rebase = [&](uint8_t* base, uint32_t* p) { return (uint32_t*)(base + ((uint8_t*)p - slot)); };
  auto pass = [&](size_t direct_bytes) -> int {
    return run_windows(
            "write_chunks", ws, slot, nwin, (size_t)total * round64(cl * 4) + 128,
            [&](uint64_t c, int, Window& w) {
              const uint64_t c0 = c * cl, nc = std::min(cl, L - c0);
              if (one)  // the flags zeroed by the window's own upload, ahead of its kernel
                w.in.push_back({(uint8_t*)kZero, (uint64_t)((uint8_t*)d_map - slot), sizeof(kZero)});
              for (int j = 0; j < need; ++j) {
                const uint64_t lo = (uint64_t)j * chunk + 4 * c0, hi = std::min(size, lo + 4 * nc);
                if (lo >= hi) continue;
                w.in.push_back({const_cast<uint8_t*>(data) + lo, lo, hi - lo});
                if (chunks[j] + 4 * c0 != data + lo) w.host.push_back({chunks[j] + 4 * c0, data + lo, hi - lo});
              }
              for (int i = 0; i < r; ++i)
                w.out.push_back({chunks[need + i] + 4 * c0, (uint64_t)(need + i) * chunk + 4 * c0, 4 * nc});
              if (one) w.out.push_back({(uint8_t*)ms, (uint64_t)((uint8_t*)d_map - slot), sizeof(ms)});
            },
            [&](uint64_t c, int, hipStream_t st, uint8_t* base) -> int {
              ran_direct = base != slot;
              BytesLaunch a =
                  bytes_launch(plan, base, stride, 0, L, size, 1, 0, rebase(base, d_status), rebase(base, d_map));
              a.col0 = c * cl;
              a.ncols = std::min(cl, L - a.col0);
              HIP_TRY(launch_encode_bytes(a, st));
              return 0;
            },
            [&](uint64_t c) {
              if (dg && !(ran_direct && (ms[1] & 1u))) dg->parity_ready(4 * std::min(L, (c + 1) * cl));
            },
            direct_bytes);
  };
  auto body = [&]() -> int {
    if (!one) {  // the flags start at zero for every window's kernel
      HIP_TRY(hipMemsetAsync(d_map, 0, 8, ws->stream));
      if (int rc = ws->fence_stages((int)std::min<uint64_t>(host_stages(), nwin))) return rc;
    }
    if (int rc = pass(one ? round16(stride) + 8 : 0)) return rc;
    // A direct pass (the kernel on the pinned stage) left nothing on the
    // device; an object that is not mapping 0 -- a word >= p, odds ~5 in 2^32
    // a word -- runs the window again through the device buffer, which the
    // choice of mapping and the re-encode below read.
    if (ran_direct && (ms[1] & 1u)) {
      ran_direct = false;
      if (int rc = pass(0)) return rc;
    }
    // One window: ms came back with the parity, ms[1] holding MapToGF's
    // flags (bit 0: a word >= p).  With bit 0 clear the mapping is 0 and
    // nothing else runs; otherwise -- and after several windows -- the
    // device chooses (select_mapping) as the 1<<31 re-encode and the
    // fallback expect.
    if (!one || (ms[1] & 1u)) {  // every window has landed: the flags are complete
      HIP_TRY(launch_select_mapping(d_map, d_status, 1, ws->stream));
      HIP_TRY(hipMemcpyAsync(ms, d_map, sizeof(ms), hipMemcpyDeviceToHost, ws->stream));
      HIP_TRY(hipStreamSynchronize(ws->stream));
    } else {
      ms[0] = ms[1] = 0;
    }
    const bool redo = ms[0] != 0 || ms[1] != 0;
    if (dg) {
      if (redo)
        dg->parity_rewrite();  // parity chunks are written again below
      else
        dg->finalize(0);
    }
    if (ms[1] != 0) {  // MapToGF's random fallback (map.go:64-66): resolved and re-encoded on device
      if (int rc = slime_rs_resolve_fallbacks(plan, slot, stride, size, 1, d_map, d_status, ws->stream, nullptr))
        return rc;
      HIP_TRY(hipMemcpyAsync(ms, d_map, sizeof(ms), hipMemcpyDeviceToHost, ws->stream));
      HIP_TRY(hipStreamSynchronize(ws->stream));
    } else if (ms[0] != 0) {  // mapping 1<<31: re-encode the whole object (map.go:47-62)
      HIP_TRY(launch_encode_bytes(bytes_launch(plan, slot, stride, 0, L, size, 1, 1, d_status, d_map), ws->stream));
    }
    // The data-chunk tails (partial word, splitVector padding) on the host,
    // and every parity chunk again from the device if the mapping was not 0.
    write_data_tails(size, need, chunk, chunks, ms[0]);
    if (redo) {
      std::vector<Span> out;
      for (int i = need; i < total; ++i) out.push_back({chunks[i], (uint64_t)i * chunk, chunk});
      if (int rc = staged_d2h(ws, slot, out.data(), out.size())) return rc;
    }
    *mapping = ms[0];
    if (dg && redo) {
      dg->parity_ready(chunk);
      dg->finalize(ms[0]);
    }
    return 0;
  };
  const int rc = body();
  if (rc) drain_stages(ws);
  return rc;
}

int slime_rs_write_chunks(const uint8_t* data, uint64_t size, int need, int total, uint8_t* const* chunks,
                          uint32_t* mapping) {
  if (int rc = write_chunks_check(data, size, need, total, chunks, mapping)) return rc;
  return write_chunks_impl(data, size, need, total, chunks, mapping, nullptr);
}

int slime_rs_write_chunks_digest(const uint8_t* data, uint64_t size, int need, int total, uint8_t* const* chunks,
                                 uint32_t* mapping, uint8_t* sha, uint8_t* hdr) {
  if (int rc = write_chunks_check(data, size, need, total, chunks, mapping)) return rc;
  if (!sha) return fail(Status::InvalidArg, "write_chunks_digest: null sha output");
  const uint64_t chunk = 4 * slot_L(size, (uint32_t)need);
  WriteChunkDigests dg(data, size, need, total, chunk, chunks, sha, hdr);
  const int rc = write_chunks_impl(data, size, need, total, chunks, mapping, &dg);
  if (rc) dg.abort();
  dg.finish();
  return rc;
}

int slime_rs_reconstruct(const uint8_t* const* chunks, const int* indices, int need, uint64_t chunk_bytes,
                         uint32_t mapping, uint64_t size, uint8_t* out) {
  if (need < 0) return fail(Status::InvalidArg, "reconstruct: negative count");
  if (need == 0) return status_of(Status::Empty, "RecoverData");
  if (!chunks || !indices) return fail(Status::InvalidArg, "reconstruct: bad args");
  if (int rc = check_survivors(need, indices)) return rc;
  if (size && !out) return fail(Status::InvalidArg, "reconstruct: null out");
  if (chunk_bytes % 4) {
    // Chunks of a length no writer produces (truncated or corrupt stored
    // chunks).  MapToGFWith packs a partial last word with zero low bytes
    // (map.go:16-33,74-98), so each survivor is its bytes zero-padded to
    // 4*ceil(chunk_bytes/4), and each recovered data row is that long too
    // (RecoverData, vector.go:80-85; MapFromGF, map.go:103-113).  Rare and
    // never on the fast path: stage padded copies and run the normal path.
    const uint64_t padded = (chunk_bytes + 3) & ~(uint64_t)3;
    std::vector<std::vector<uint8_t>> copy((size_t)need, std::vector<uint8_t>(padded, 0));
    std::vector<const uint8_t*> ptrs((size_t)need);
    for (int q = 0; q < need; ++q) {
      if (!chunks[q]) return fail(Status::InvalidArg, "reconstruct: null chunk");
      memcpy(copy[q].data(), chunks[q], chunk_bytes);
      ptrs[q] = copy[q].data();
    }
    return slime_rs_reconstruct(ptrs.data(), indices, need, padded, mapping, size, out);
  }
  const uint64_t L = chunk_bytes / 4, body_bytes = (uint64_t)need * chunk_bytes, got = std::min(size, body_bytes);
  // data[:f.Size] of a make([]byte, 0, Size+16) buffer (multi_store.go:203,241):
  // bytes past the recovered ones are the zeroed capacity.
  if (size > got) memset(out + got, 0, size - got);
  if (got == 0) return 0;
  for (int q = 0; q < need; ++q)
    if (!chunks[q]) return fail(Status::InvalidArg, "reconstruct: null chunk");
  DeviceLease dl;
  if (int rc = dl.acquire()) return rc;
  const int dev = dl.device;
  std::vector<int> have(indices, indices + need);
  PlanRef plan_ref;
  if (int rc = cached_plan(PlanKey{dev, 'O', need, 0, have}, &plan_ref, make_object_recover_plan)) return rc;
  slime_rs_plan* const plan = plan_ref.get();
  WsLease lease;
  if (int rc = acquire_ws(dev, &lease.ws)) return rc;
  Workspace* ws = lease.ws;
  DeviceScope ds(dev);
  const uint64_t stride = 2 * body_bytes;
  if (int rc = ws->reserve(round16(stride) + 16)) return rc;
  uint8_t* const slot = ws->dbuf;
  uint32_t* const d_map = (uint32_t*)(ws->dbuf + round16(stride));
  // Window by window: survivors' columns in, all need data rows decoded,
  // the object's bytes of those columns out.
  const uint64_t cl = window_cols(L, 2 * (uint64_t)need, obj_window_bytes());
  const uint64_t nwin = (L + cl - 1) / cl;
  // The mapping goes up with every window's inputs (the same word each time:
  // each window's kernel reads it behind its own upload).
  const uint32_t map_word = mapping;
  auto body = [&]() -> int {
    return run_windows(
        "reconstruct", ws, slot, nwin, (size_t)2 * need * round64(cl * 4) + 64,
        [&](uint64_t c, int, Window& w) {
          const uint64_t c0 = c * cl, nc = std::min(cl, L - c0);
          w.in.push_back({(uint8_t*)&map_word, (uint64_t)((uint8_t*)d_map - slot), 4});
          for (int q = 0; q < need; ++q)
            w.in.push_back({const_cast<uint8_t*>(chunks[q]) + 4 * c0, (uint64_t)q * chunk_bytes + 4 * c0, 4 * nc});
          for (int t = 0; t < need; ++t) {
            const uint64_t o = (uint64_t)t * chunk_bytes + 4 * c0;
            if (o < got) w.out.push_back({out + o, body_bytes + o, std::min(4 * nc, got - o)});
          }
        },
        [&](uint64_t c, int, hipStream_t st, uint8_t* base) -> int {
          BytesLaunch a =
              bytes_launch(plan, base, stride, 0, L, 0, 1, 0, nullptr, (uint32_t*)(base + ((uint8_t*)d_map - slot)));
          a.col0 = c * cl;
          a.ncols = std::min(cl, L - a.col0);
          HIP_TRY(launch_decode_bytes(a, st));
          return 0;
        },
        [](uint64_t) {}, round16(stride) + 4);
  };
  const int rc = body();
  if (rc) drain_stages(ws);
  return rc;
}

// ---- gf codec (host memory) -----------------------------------------------------------
//
// Where the Go API's codec calls run (slime_gf_codec_placement): on the host
// cores, in place on the caller's buffers (host_codec.cpp, default), or
// through the device codec and the pinned ring (the round-3 form, kept as the
// measured alternative and exercised by the GPU tests).

static std::atomic<int> g_codec_device{[] {
  const char* e = getenv("SLIME_RS_CODEC");
  return e && strcmp(e, "device") == 0 ? 1 : 0;
}()};

static bool codec_on_device() { return g_codec_device.load(std::memory_order_relaxed) != 0; }

int slime_gf_codec_info(const char** isa, int* threads) {
  if (isa) *isa = host_codec_isa();
  if (threads) *threads = copy_pool_threads() + 1;
  return 0;
}

int slime_gf_codec_placement(int mode) {
  if (mode < 0) return g_codec_device.load();
  if (mode > 1) return fail(Status::InvalidArg, "codec placement: 0 = host, 1 = device");
  g_codec_device.store(mode);
  return 0;
}


static int codec_setup(uint64_t bytes_needed, Workspace** wsp, WsLease& lease, DeviceLease& dl) {
  if (int rc = dl.acquire()) return rc;
  if (int rc = acquire_ws(dl.device, &lease.ws)) return rc;
  *wsp = lease.ws;
  return (*wsp)->reserve(bytes_needed);
}

// The codec's host entry points stream through the same pinned 3-stage ring
// as the object entry points (run_windows): the caller's buffers stay
// pageable, each window's H2D / kernel / D2H overlaps the host copies of the
// others, and fresh (never touched) output pages are faulted in by the
// ring's host copy instead of by a DMA (the direct pageable copy of round 1
// fell to 0.5 GiB/s into fresh pages, DESIGN.md "End-to-end").
constexpr uint64_t kCodecWindowBytes = 8u << 20;  // largest window: input bytes (+ as many out)

// Input bytes per codec window: at least 4 windows per call when the input
// allows (so H2D, kernel and D2H of one call overlap across the ring's 3
// stages: an 8 MiB chunk in one window runs them back to back), between
// 512 KiB and 8 MiB, a multiple of 64 KiB.
static uint64_t codec_window(uint64_t len) {
  const uint64_t quarter = ((len / 4) + 65535) & ~(uint64_t)65535;
  return std::min<uint64_t>(kCodecWindowBytes, std::max<uint64_t>(512u << 10, quarter));
}

// Bytes -> words windows of MapToGF(With): window c packs input bytes
// [c*W, c*W + W) into words [c*W/4, ...) on the device (mapping n, flags
// OR-reduced if given) and streams the words back to `out`.
static int pack_windows(Workspace* ws, const uint8_t* in, uint64_t len, uint32_t n, uint32_t* out,
                        uint8_t* d_bytes, uint32_t* d_words, uint32_t* d_flags) {
  const uint64_t W = codec_window(len), nwin = (len + W - 1) / W;
  uint8_t* const base = ws->dbuf;
  return run_windows(
      "codec_pack", ws, base, nwin, 2 * W,
      [&](uint64_t c, int, Window& w) {
        const uint64_t b0 = c * W, nb = std::min(W, len - b0);
        w.in.push_back({const_cast<uint8_t*>(in) + b0, (uint64_t)(d_bytes - base) + b0, nb});
        w.out.push_back({(uint8_t*)out + b0, (uint64_t)((uint8_t*)d_words - base) + b0, 4 * ((nb + 3) / 4)});
      },
      [&](uint64_t c, int, hipStream_t st, uint8_t*) -> int {
        const uint64_t b0 = c * W, nb = std::min(W, len - b0);
        HIP_TRY(launch_map_pack(d_bytes + b0, nb, n, d_words + b0 / 4, d_flags, st));
        return 0;
      });
}

static int map_to_gf_with_device(const uint8_t* in, uint64_t len, uint32_t n, uint32_t* out) {
  const uint64_t nw = (len + 3) / 4;
  WsLease lease;
  Workspace* ws = nullptr;
  const size_t bbytes = round16(len);
  DeviceLease dl;
  if (int rc = codec_setup(bbytes + round16(nw * 4), &ws, lease, dl)) return rc;
  DeviceScope ds(ws->device);
  const int rc = pack_windows(ws, in, len, n, out, ws->dbuf, (uint32_t*)(ws->dbuf + bbytes), nullptr);
  if (rc) drain_stages(ws);
  return rc;
}

int slime_gf_map_to_gf_with(const uint8_t* in, uint64_t len, uint32_t n, uint32_t* out) {
  const uint64_t nw = (len + 3) / 4;
  if (nw == 0) return 0;
  if (!in || !out) return fail(Status::InvalidArg, "MapToGFWith: null buffer");
  if (codec_on_device()) return map_to_gf_with_device(in, len, n, out);
  host_pack(in, len, n, out, nullptr);
  return 0;
}

// gf.MapToGF's choice of mapping (map.go:35-66) from the two flags already
// OR-reduced into d_scratch[0] while packing the nw words at d_words with
// mapping 0: 0, else 1<<31, else the first fitting value of the library's
// random candidate stream (64 per device probe pass).  d_scratch holds
// 4 + 2*64 words.
static int choose_mapping(hipStream_t st, const uint32_t* d_words, uint64_t nw, uint32_t* d_scratch,
                          uint32_t* mapping) {
  constexpr uint32_t kCand = 64;
  uint32_t* d_flags = d_scratch;
  uint32_t* d_cand = d_flags + 4;
  uint32_t* d_bad = d_cand + kCand;
  uint32_t flags = 0;
  HIP_TRY(hipMemcpyAsync(&flags, d_flags, 4, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  *mapping = 0;
  if (!(flags & 1u)) return 0;
  if (!(flags & 2u)) {
    *mapping = 1u << 31;  // map.go:47: try just switching the high bit first
    return 0;
  }
  for (int round = 0; round < (1 << 16); ++round) {  // map.go:64-66
    uint32_t cand[kCand], bad[kCand];
    {
      std::lock_guard<std::mutex> lk(g_rng_mu);
      for (uint32_t c = 0; c < kCand; ++c) cand[c] = (uint32_t)(g_rng() >> 32);
    }
    HIP_TRY(hipMemcpyAsync(d_cand, cand, sizeof(cand), hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemsetAsync(d_bad, 0, sizeof(bad), st));
    HIP_TRY(launch_mapping_probe(d_words, nw, d_cand, kCand, d_bad, st));
    HIP_TRY(hipMemcpyAsync(bad, d_bad, sizeof(bad), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    for (uint32_t c = 0; c < kCand; ++c)
      if (!bad[c]) {
        *mapping = cand[c];
        return 0;
      }
  }
  return status_of(Status::MappingFallback, "MapToGF");
}

// pack (mapping 0, flags) + choose_mapping for `len` bytes already on the device.
static int pick_mapping(hipStream_t st, const uint8_t* d_bytes, uint64_t len, uint32_t* d_words,
                        uint32_t* d_scratch, uint32_t* mapping) {
  HIP_TRY(hipMemsetAsync(d_scratch, 0, 4, st));
  HIP_TRY(launch_map_pack(d_bytes, len, 0, d_words, d_scratch, st));
  return choose_mapping(st, d_words, (len + 3) / 4, d_scratch, mapping);
}

static int map_to_gf_device(const uint8_t* in, uint64_t len, uint32_t* mapping, uint32_t* out) {
  const uint64_t nw = (len + 3) / 4;
  WsLease lease;
  Workspace* ws = nullptr;
  const size_t bbytes = round16(len), wbytes = round16(nw * 4);
  DeviceLease dl;
  if (int rc = codec_setup(bbytes + wbytes + 4 * (4 + 2 * 64), &ws, lease, dl)) return rc;
  DeviceScope ds(ws->device);
  uint8_t* d_bytes = ws->dbuf;
  uint32_t* d_words = (uint32_t*)(ws->dbuf + bbytes);
  uint32_t* d_scratch = (uint32_t*)(ws->dbuf + bbytes + wbytes);
  auto body = [&]() -> int {
    // Speculative mapping 0 (map.go:35-45): the words stream back while the
    // flags of every window accumulate on the device; 1<<31 (map.go:47-62,
    // about 2% of uniform 64 MiB bodies) or the random fallback (:64-66)
    // re-map the words on the device and send them again.
    HIP_TRY(hipMemsetAsync(d_scratch, 0, 4, ws->stream));
    HIP_TRY(hipStreamSynchronize(ws->stream));
    if (int rc = pack_windows(ws, in, len, 0, out, d_bytes, d_words, d_scratch)) return rc;
    uint32_t m = 0;
    if (int rc = choose_mapping(ws->stream, d_words, nw, d_scratch, &m)) return rc;
    if (m) {
      HIP_TRY(launch_xor_words(d_words, nw, m, ws->stream));
      const Span sp{(uint8_t*)out, (uint64_t)((uint8_t*)d_words - ws->dbuf), nw * 4};
      if (int rc = staged_d2h(ws, ws->dbuf, &sp, 1)) return rc;
    }
    *mapping = m;
    return 0;
  };
  const int rc = body();
  if (rc) drain_stages(ws);
  return rc;
}

// MapToGF on host memory, in place on the caller's buffers (map.go:15-67):
// one pass packs the words (mapping 0) and notes whether 0 and 1<<31 fit;
// a mapping other than 0 is then XORed in by a second pass.  The random
// fallback (:64-66) probes candidates of the library's stream in order, the
// first that fits wins (the device form's rule: choose_mapping).
static int map_to_gf_host(const uint8_t* in, uint64_t len, uint32_t* mapping, uint32_t* out) {
  const uint64_t nw = (len + 3) / 4;
  uint32_t flags = 0, m = 0;
  host_pack(in, len, 0, out, &flags);
  if (flags & 1u) {
    if (!(flags & 2u)) {
      m = 1u << 31;  // map.go:47
    } else {
      bool found = false;
      for (uint32_t tries = 0; tries < (1u << 22) && !found; ++tries) {
        uint32_t cand;
        {
          std::lock_guard<std::mutex> lk(g_rng_mu);
          cand = (uint32_t)(g_rng() >> 32);
        }
        if (host_mapping_fits(out, nw, cand)) m = cand, found = true;
      }
      if (!found) return status_of(Status::MappingFallback, "MapToGF");
    }
    host_xor(out, nw, m);
  }
  *mapping = m;
  return 0;
}

int slime_gf_map_to_gf(const uint8_t* in, uint64_t len, uint32_t* mapping, uint32_t* out) {
  if (!mapping) return fail(Status::InvalidArg, "MapToGF: null mapping");
  const uint64_t nw = (len + 3) / 4;
  *mapping = 0;
  if (nw == 0) return 0;
  if (!in || !out) return fail(Status::InvalidArg, "MapToGF: null buffer");
  return codec_on_device() ? map_to_gf_device(in, len, mapping, out) : map_to_gf_host(in, len, mapping, out);
}

static int map_from_gf_device(uint32_t n, const uint32_t* in, uint64_t count, uint8_t* out) {
  WsLease lease;
  Workspace* ws = nullptr;
  const size_t wbytes = round16(count * 4);
  DeviceLease dl;
  if (int rc = codec_setup(2 * wbytes, &ws, lease, dl)) return rc;
  DeviceScope ds(ws->device);
  uint32_t* d_words = (uint32_t*)ws->dbuf;
  uint8_t* d_bytes = ws->dbuf + wbytes;
  const uint64_t W = codec_window(4 * count) / 4, nwin = (count + W - 1) / W;  // words per window
  const int rc = run_windows(
      "codec_unpack", ws, ws->dbuf, nwin, 2 * kCodecWindowBytes,
      [&](uint64_t c, int, Window& w) {
        const uint64_t w0 = c * W, nwd = std::min(W, count - w0);
        w.in.push_back({(uint8_t*)(in + w0), 4 * w0, 4 * nwd});
        w.out.push_back({out + 4 * w0, wbytes + 4 * w0, 4 * nwd});
      },
      [&](uint64_t c, int, hipStream_t st, uint8_t*) -> int {
        const uint64_t w0 = c * W, nwd = std::min(W, count - w0);
        HIP_TRY(launch_map_unpack(d_words + w0, nwd, n, d_bytes + 4 * w0, st));
        return 0;
      });
  if (rc) drain_stages(ws);
  return rc;
}

int slime_gf_map_from_gf(uint32_t n, const uint32_t* in, uint64_t count, uint8_t* out) {
  if (count == 0) return 0;
  if (!in || !out) return fail(Status::InvalidArg, "MapFromGF: null buffer");
  if (codec_on_device()) return map_from_gf_device(n, in, count, out);
  host_unpack(in, count, n, out);
  return 0;
}

// ---- per-call context entry points (cgo) ------------------------------------------
//
// A goroutine can move to another OS thread between two cgo calls, so the
// shim must not read thread-local state in a second call: each *_ex entry
// point takes the device explicitly and returns the failure detail of THIS
// call in the caller's buffer.

namespace {
struct CallScope {
  const slime_rs_call_t* prev;
  const slime_rs_call_t* call;
  explicit CallScope(const slime_rs_call_t* c) : prev(t_call), call(c) {
    t_call = c;
    t_error.clear();
  }
  int done(int rc) {
    if (call && call->detail && call->detail_cap) {
      const std::string& d = rc ? t_error : std::string();
      const size_t n = std::min(d.size(), call->detail_cap - 1);
      memcpy(call->detail, d.data(), n);
      call->detail[n] = 0;
    }
    t_call = prev;
    return rc;
  }
};
int bad_call(const slime_rs_call_t* call) {
  if (!call) return fail(Status::InvalidArg, "null call context");
  if (call->device != SLIME_RS_ANY_DEVICE && call->device < 0)
    return fail(Status::InvalidArg, "call context: device must be >= 0 or SLIME_RS_ANY_DEVICE");
  return 0;
}
}  // namespace

#define SLIME_EX(call, expr)                      \
  do {                                            \
    CallScope cs_(call);                          \
    if (int rc_ = bad_call(call)) return cs_.done(rc_); \
    return cs_.done(expr);                        \
  } while (0)

int slime_rs_create_parity_ex(const slime_rs_call_t* call, const uint32_t* const* data, const uint64_t* lens,
                              int ndata, int index, uint32_t* out) {
  SLIME_EX(call, slime_rs_create_parity(data, lens, ndata, index, out));
}

int slime_rs_create_parities_ex(const slime_rs_call_t* call, const uint32_t* const* data, const uint64_t* lens,
                                int ndata, int total, uint32_t* const* out) {
  SLIME_EX(call, slime_rs_create_parities(data, lens, ndata, total, out));
}

int slime_rs_recover_data_ex(const slime_rs_call_t* call, const uint32_t* const* chunks, const uint64_t* lens,
                             int nchunks, const int* indices, int nindices, uint32_t* const* out) {
  SLIME_EX(call, slime_rs_recover_data(chunks, lens, nchunks, indices, nindices, out));
}

int slime_rs_write_chunks_ex(const slime_rs_call_t* call, const uint8_t* data, uint64_t size, int need, int total,
                             uint8_t* const* chunks, uint32_t* mapping) {
  SLIME_EX(call, slime_rs_write_chunks(data, size, need, total, chunks, mapping));
}

int slime_rs_reconstruct_ex(const slime_rs_call_t* call, const uint8_t* const* chunks, const int* indices, int need,
                            uint64_t chunk_bytes, uint32_t mapping, uint64_t size, uint8_t* out) {
  SLIME_EX(call, slime_rs_reconstruct(chunks, indices, need, chunk_bytes, mapping, size, out));
}

int slime_gf_map_to_gf_ex(const slime_rs_call_t* call, const uint8_t* in, uint64_t len, uint32_t* mapping,
                          uint32_t* out) {
  SLIME_EX(call, slime_gf_map_to_gf(in, len, mapping, out));
}

int slime_gf_map_to_gf_with_ex(const slime_rs_call_t* call, const uint8_t* in, uint64_t len, uint32_t n,
                               uint32_t* out) {
  SLIME_EX(call, slime_gf_map_to_gf_with(in, len, n, out));
}

int slime_gf_map_from_gf_ex(const slime_rs_call_t* call, uint32_t n, const uint32_t* in, uint64_t count,
                            uint8_t* out) {
  SLIME_EX(call, slime_gf_map_from_gf(n, in, count, out));
}

int slime_rs_parity_matrix_ex(const slime_rs_call_t* call, int d, int p, uint32_t* out) {
  SLIME_EX(call, slime_rs_parity_matrix(d, p, out));
}

int slime_rs_vandermonde_matrix_ex(const slime_rs_call_t* call, int d, int p, uint32_t* out) {
  SLIME_EX(call, slime_rs_vandermonde_matrix(d, p, out));
}

int slime_rs_solve_sub_identity_ex(const slime_rs_call_t* call, uint32_t* m, int rows, int cols) {
  SLIME_EX(call, slime_rs_solve_sub_identity(m, rows, cols));
}

int slime_rs_invert_matrix_ex(const slime_rs_call_t* call, const uint32_t* m, int d, uint32_t* inv) {
  SLIME_EX(call, slime_rs_invert_matrix(m, d, inv));
}

// ---- plan cache / device pool introspection ---------------------------------------

int slime_rs_plan_cache_stats(slime_rs_cache_stats_t* st) {
  if (!st) return fail(Status::InvalidArg, "plan_cache_stats: null");
  LruCache<PlanKey, slime_rs_plan>& c = plans();
  st->live = c.size();
  st->capacity = c.capacity();
  st->hits = c.hits();
  st->misses = c.misses();
  st->evictions = c.evictions();
  st->device_tables = (uint64_t)std::max<int64_t>(0, g_tables_live.load());
  return 0;
}

int slime_rs_plan_cache_capacity(uint64_t capacity) {
  if (capacity == 0) return fail(Status::InvalidArg, "plan_cache_capacity: must be >= 1");
  plans().set_capacity((size_t)capacity);
  return 0;
}

int slime_rs_host_stats(slime_rs_host_stats_t* st, int reset) {
  if (!st) return fail(Status::InvalidArg, "host_stats: null");
  auto take = [&](std::atomic<uint64_t>& a) { return reset ? a.exchange(0) : a.load(); };
  st->calls = take(g_host_stats.calls);
  st->windows = take(g_host_stats.windows);
  st->copy_in_us = take(g_host_stats.copy_in_us);
  st->enqueue_us = take(g_host_stats.enqueue_us);
  st->wait_us = take(g_host_stats.wait_us);
  st->copy_out_us = take(g_host_stats.copy_out_us);
  st->total_us = take(g_host_stats.total_us);
  return 0;
}

int slime_rs_pool_calls(int device, uint64_t* calls, int* inflight) {
  if (device < 0 || device >= DevicePool::kMax) return fail(Status::InvalidArg, "pool_calls: device out of range");
  if (calls) *calls = g_pool.calls[device].load();
  if (inflight) *inflight = g_pool.inflight[device].load();
  return 0;
}

// ---- chunk and object digests (host; digest.hpp) ------------------------------

int slime_rs_sha256(const uint8_t* data, uint64_t len, uint8_t* out) {
  if (!out || (len && !data)) return fail(Status::InvalidArg, "sha256: null buffer");
  Sha256 h;
  if (len) h.update(data, len);
  h.final(out);
  return 0;
}

int slime_rs_chunk_digests(const uint8_t* const* chunks, const uint64_t* lens, uint32_t n, uint8_t* sha,
                           uint8_t* hdr) {
  if (n == 0) return 0;
  if (!chunks || !lens || !sha) return fail(Status::InvalidArg, "chunk_digests: null argument");
  for (uint32_t i = 0; i < n; ++i)
    if (lens[i] && !chunks[i]) return fail(Status::InvalidArg, "chunk_digests: null chunk");
  digest_parallel(n, [&](size_t i) {
    Sha256 h;
    if (lens[i]) h.update(chunks[i], lens[i]);
    h.final(sha + 32 * i);
    if (hdr) {
      const uint64_t f = fnv1a64(fnv1a64(kFnv64Offset, sha + 32 * i, 32), chunks[i], lens[i]);
      for (int b = 0; b < 8; ++b) hdr[8 * i + b] = (uint8_t)(f >> (56 - 8 * b));
    }
  });
  return 0;
}

int slime_rs_reconstruct_verify(const uint8_t* const* chunks, const int* indices, int need, uint64_t chunk_bytes,
                                uint32_t mapping, uint64_t size, uint8_t* out, const uint8_t* want_sha) {
  if (!want_sha) return fail(Status::InvalidArg, "reconstruct_verify: null sha");
  if (int rc = slime_rs_reconstruct(chunks, indices, need, chunk_bytes, mapping, size, out)) return rc;
  uint8_t have[32];
  Sha256 h;
  if (size) h.update(out, size);
  h.final(have);
  if (memcmp(have, want_sha, 32) != 0) return status_of(Status::BadHash, "reconstruct");
  return 0;
}

int slime_rs_digest_info(int* sha_extensions_used, int* threads) {
  if (sha_extensions_used) *sha_extensions_used = sha_extensions() ? 1 : 0;
  if (threads) *threads = digest_threads();
  return 0;
}

int slime_rs_write_chunks_digest_ex(const slime_rs_call_t* call, const uint8_t* data, uint64_t size, int need,
                                    int total, uint8_t* const* chunks, uint32_t* mapping, uint8_t* sha,
                                    uint8_t* hdr) {
  SLIME_EX(call, slime_rs_write_chunks_digest(data, size, need, total, chunks, mapping, sha, hdr));
}

int slime_rs_reconstruct_verify_ex(const slime_rs_call_t* call, const uint8_t* const* chunks, const int* indices,
                                   int need, uint64_t chunk_bytes, uint32_t mapping, uint64_t size, uint8_t* out,
                                   const uint8_t* want_sha) {
  SLIME_EX(call, slime_rs_reconstruct_verify(chunks, indices, need, chunk_bytes, mapping, size, out, want_sha));
}

#undef SLIME_EX

}  // extern "C"
