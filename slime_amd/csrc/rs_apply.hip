// GF(2^32-5) shard-matrix apply for CDNA4 (gfx950): the data path of slime's
// internal/rs (applyMatrix, internal/rs/vector.go:90-102), used for both
// parity generation (CreateParity, vector.go:18-41 — all parity rows in ONE
// pass instead of one pass per row as multi_store.go:528-531 does) and
// reconstruction (RecoverData, vector.go:50-88 — only the erased rows).
//
// Shape of the work: every output symbol column b is independent; a lane owns
// 4 consecutive columns of one object, loads them from each of the k input
// shards with one 16-byte load per shard (coalesced: a wave reads 1 KiB of
// each shard stripe per load instruction), keeps the k x 4 symbols in VGPRs
// and produces every output row from them.  Coefficients are wave-uniform and
// come in through scalar loads into SGPRs (no LDS: the matrix is at most
// 100x100 words and uniform across the wave).  No cross-lane reduction is
// needed: the sum over j is in-register.  Arithmetic: exact 96-bit
// accumulate + one fold (gfp.hpp), bit-identical to the reference's
// per-term `%`.  The kernel is HBM-bound (its VALU ceiling is ~3.5x the HBM
// rate, tools/ubench.py), so launch geometry is chosen for DRAM efficiency.
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include <atomic>
#include <deque>
#include <functional>
#include <map>
#include <mutex>
#include <utility>
#include <vector>

#include "kernels.hpp"
#include "rs_apply_kernel.hpp"

namespace slime {

// Column segments per object (rs_apply_kernel): enough that the batch has
// about 256 independent object segments in flight -- 128 x 256 MiB objects
// reach 6.1 TB/s unsegmented, 32 x 64 MiB objects need 8 segments each to get
// from 5.08 to 5.54 TB/s (profiles/r01/segs/) -- and at least 1024 vectors
// (4 U=4 tiles) per segment.
uint32_t object_segments(uint32_t nobj, uint64_t ncols) {
  const uint64_t want = (256 + nobj - 1) / nobj;
  const uint64_t max_s = (ncols >> 2) / 1024 ? (ncols >> 2) / 1024 : 1;
  return (uint32_t)(want < max_s ? want : max_s);
}
namespace {

using apply::kBlock;
using apply::rs_apply_kernel;

// Non-pipelined vectorised kernel (the fallback for shards >= 4 GiB and
// slime_rs_kernel_pipeline(0); tools/apply_variants.py sweep, DESIGN.md "Tuning"): each wave streams U KiB of every shard per step with
// non-temporal loads and stores (read-once/write-once streams).  U = 4 up to
// k = 10 (<= 192 VGPRs, 2 waves/SIMD at the 512-block grid), U = 2 beyond so
// the k x U x 16 B of symbols stay in registers without dropping below that.
template <int K>
constexpr int unroll_for() {
  return K <= 10 ? 4 : 2;
}
constexpr bool kNtLoads = true;
constexpr bool kNtStores = true;

}  // namespace

namespace {

// Launch geometry: `target` resident 256-lane blocks over the batch's object
// segments (grid.y, at most 65535 at a time).  The block budget is 512, and
// 256 for 9 <= k <= 12 (U = 4 at k = 9, 10 holds 36-40 KiB of symbols per
// wave; fewer, fatter waves measured +5..18% at 10/14 and +2% at 12/16 on
// 1 GiB objects, profiles/r01/gridk/).
template <int K>
constexpr uint64_t default_blocks() {
  return K >= 9 && K <= 12 ? 256 : 512;
}

template <int K, bool VEC>
hipError_t launch_k(const ApplyLaunch& a, hipStream_t stream) {
  constexpr int U = unroll_for<K>();
  const uint64_t per_block = VEC && K > 0 ? 4ull * kBlock * U : (uint64_t)kBlock;
  const uint32_t nseg = VEC && K > 0 ? object_segments(a.nobj, a.ncols) : 1u;
  const uint64_t nwork = (uint64_t)a.nobj * nseg;
  const uint64_t gy = nwork < 65535 ? nwork : 65535;
  const uint64_t target = default_blocks<K>();
  uint64_t gx = (target + gy - 1) / gy;
  const uint64_t need = (a.ncols / nseg + per_block - 1) / per_block;
  if (gx > need) gx = need;
  if (gx < 1) gx = 1;
  hipLaunchKernelGGL((rs_apply_kernel<K, VEC, U, kNtLoads, kNtStores>), dim3((uint32_t)gx, (uint32_t)gy),
                     dim3(kBlock), 0, stream, a.in, a.out, a.in_obj_stride, a.in_shard_stride, a.out_obj_stride,
                     a.out_shard_stride, a.coeff, a.in_idx, a.out_idx, a.ncols, a.nobj, a.rows, a.k, nseg);
  return hipGetLastError();
}

// Software-pipelined product kernel (rs_apply_pipe_kernel): each wave keeps
// its next tile's loads in flight while it computes the current one, so
// fewer, fatter waves keep HBM busy.  In-process A/B against the
// non-pipelined kernel on fast-placement boxes (profiles/r01/pipe/, HBM GB/s,
// best product geometry -> pipelined): 4/6 C2 5480 -> 5557, 6/9 5431 -> 5643,
// 8/12 C3 6075 -> 6177, 10/14 C5 5530 -> 5595, 12/16 5041 -> 5225,
// 16/20 5172 -> 5317.  pipe_unroll<K>() 16-byte units per lane per tile (two
// register sets of K x U x 16 B; K = 12 at U = 3 spills into AGPRs, which
// measured fine), pipe_blocks<K>() 256-lane blocks.
template <int K>
constexpr int pipe_unroll() {
  return K == 1 ? 4 : K == 2 ? 2 : K <= 4 ? 1 : K <= 12 ? 3 : 1;
}
template <int K>
constexpr uint64_t pipe_blocks() {
  return K <= 12 ? 256 : 1024;
}

template <int K>
hipError_t launch_pipe(const ApplyLaunch& a, hipStream_t stream) {
  constexpr int U = pipe_unroll<K>();
  const uint64_t per_block = 4ull * kBlock * U;
  const uint32_t nseg = object_segments(a.nobj, a.ncols);
  const uint64_t nwork = (uint64_t)a.nobj * nseg;
  const uint64_t gy = nwork < 65535 ? nwork : 65535;
  const uint64_t target = pipe_blocks<K>();
  uint64_t gx = (target + gy - 1) / gy;
  const uint64_t need = (a.ncols / nseg + per_block - 1) / per_block;
  if (gx > need) gx = need;
  if (gx < 1) gx = 1;
  hipLaunchKernelGGL((apply::rs_apply_pipe_kernel<K, U, kNtLoads, kNtStores>), dim3((uint32_t)gx, (uint32_t)gy),
                     dim3(kBlock), 0, stream, a.in, a.out, a.in_obj_stride, a.in_shard_stride, a.out_obj_stride,
                     a.out_shard_stride, a.coeff, a.in_idx, a.out_idx, a.ncols, a.nobj, a.rows, a.k, nseg);
  return hipGetLastError();
}

// Dynamic schedule (rs_apply_queue_kernel): tickets instead of a fixed share
// per wave, so the XCDs that stream faster take more of the batch (the static
// walk left 3.4% of C3's wave-time idle behind the four slower XCDs; the
// dynamic one 0.1%, profiles/r02/s41_queue4/).  In-process A/B against the
// static kernel's best geometry: C3 encode 8.568 -> 8.295 ms, decode 8.441 ->
// 8.239 on a fast-placement allocation and 9.79 -> 9.33 on a slow one
// (s39_queue3/, s41_queue4/); 16/20 3.737 -> 3.600, C2 (4/6) 0.586 -> 0.575
// (s42_queuek/).  Geometry: 256 blocks (one per CU) for every k; U = 4 up to
// k = 4, 3 up to 12, 1 above; a unit is C tiles with C x U about 6 (C = 2 at
// U = 3), dealt over kQueueCounters ticket counters.  At k <= 4 a unit is
// three tiles: the narrow codes' tiles are short (24 KiB a wave at 4/6), and
// fewer draws per byte ran 4/6 at 32 objects +0.4 to +1.2% and slime's default
// 3/5 +1.1 to +2.0% on the stamped twin (64 objects +0 to +0.8%; four and six
// tiles no better; profiles/r06/s30_c2unit/).
constexpr uint64_t kQueueBlocks = 256;
template <int K>
constexpr int queue_unroll() {
  return K <= 4 ? 4 : K <= 12 ? 3 : 1;
}
template <int K>
constexpr int queue_unit_tiles() {
  return K <= 4 ? 3 : queue_unroll<K>() >= 3 ? 2 : 6 / queue_unroll<K>();
}

template <int K>
hipError_t launch_queue(const ApplyLaunch& a, hipStream_t stream, bool* launched) {
  constexpr int U = queue_unroll<K>();
  constexpr int C = queue_unit_tiles<K>();
  *launched = false;
  const uint32_t spread = queue_spread(a.nobj, a.ncols, U, C, (uint32_t)(a.k + a.rows));
  if (!spread) return hipSuccess;
  const uint64_t blocks = queue_blocks(kQueueBlocks, queue_units(a.nobj, a.ncols, U, C, spread));
  return with_tickets(
      stream,
      [&](uint32_t* set) {
        hipLaunchKernelGGL((apply::rs_apply_queue_kernel<K, U, C, kQueueCounters, kNtLoads, kNtStores>),
                           dim3((uint32_t)blocks), dim3(kBlock), 0, stream, a.in, a.out, a.in_obj_stride,
                           a.in_shard_stride, a.out_obj_stride, a.out_shard_stride, a.coeff, a.in_idx, a.out_idx,
                           a.ncols, a.nobj, a.rows, a.k, set, nullptr, spread);
        return hipGetLastError();
      },
      launched);
}

}  // namespace

// ---- ticket-counter sets -------------------------------------------------------
// A queue launch resets its own set before it ends (TicketWalk::finish), so
// a set is reusable as soon as the launch that held it has finished -- on any
// stream.  Per device: a pool of sets, each with an event recorded after the
// launch that last took it; a set is free when that event has completed.
// Nothing trusts the identity of the launch stream: hipStreamPerThread, the
// per-thread null stream, and a stream destroyed while its last launch runs
// (its handle then reused by hipStreamCreate) are all safe.
//
// When every set is held (more launches queued than sets), a launch takes
// the set of the latest launch queued under its own stream handle and makes
// its stream wait for that launch's event first: on a true in-order stream
// the wait is already implied by stream order, and under a shared or reused
// handle it orders the two launches.  So a deep queue on one stream runs on a
// fixed number of sets.  Other streams' launches get new sets (up to
// kMaxSets, then they too wait for the oldest holder).
//
// Inside a graph capture the default schedule (mode 1) launches the static
// kernels: a set is bound to the captured kernel node, so two execs of one
// graph (instantiated twice, or cloned) replayed at the same time would draw
// tickets from one set and skip each other's units.  Mode 2 captures the
// dynamic kernels too (one exec of a graph at a time): such a launch keeps
// its set for the graph's life -- every replay leaves it zero for the next --
// and a HIP user object retained by the graph gives the set back to the pool
// when the graph and its execs are destroyed.  Captured launches never wait
// on events from outside the capture and never create slabs: with no free
// set they take the static kernel.  Sets come in slabs of kSlabSets, zeroed
// when created.
namespace {
constexpr uint32_t kSetWords = apply::ticket_set_words(kQueueCounters);
constexpr int kSlabSets = 64;
constexpr uint64_t kMaxSets = 1024;
struct TicketSet {
  uint32_t* p = nullptr;
  hipEvent_t ev = nullptr;
  hipStream_t last = nullptr;  // stream handle of the launch that last took it
};
struct TicketPool {
  std::mutex mu;
  std::vector<TicketSet> free_sets;  // zero, no launch holds them
  std::deque<TicketSet> busy;        // held by a launch, in launch order
  uint64_t sets = 0, graph_held = 0, lost = 0;
  uint64_t dynamic = 0, fallback = 0;  // launches on a set / sent to the static kernel
  // Sets of destroyed graphs, handed back by a user-object destructor that
  // may run on a runtime thread at any time: its own lock, never held across
  // a HIP call, so it cannot wait on `mu`.
  std::mutex ret_mu;
  std::vector<TicketSet> returned;

  void give_back(const TicketSet& s) {  // from a graph's user-object destructor
    std::lock_guard<std::mutex> lk(ret_mu);
    returned.push_back(s);
  }
  void drain_returned() {  // mu held
    std::lock_guard<std::mutex> lk(ret_mu);
    for (const TicketSet& s : returned) free_sets.push_back(s);
    graph_held -= std::min<uint64_t>(graph_held, returned.size());
    returned.clear();
  }
  hipError_t grow() {  // mu held; not inside a capture
    void* p = nullptr;
    const size_t bytes = (size_t)kSlabSets * kSetWords * sizeof(uint32_t);
    if (hipError_t e = hipMalloc(&p, bytes)) return e;
    // Zeroed on a private non-blocking stream and waited for there only: the
    // zeroes are in memory before any stream can launch on a set of this
    // slab, and neither torch's default stream nor a capture in progress on
    // another thread is synchronised (a legacy null-stream sync would be).
    hipStream_t z = nullptr;
    hipError_t e = hipStreamCreateWithFlags(&z, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMemsetAsync(p, 0, bytes, z);
    if (e == hipSuccess) e = hipStreamSynchronize(z);
    if (z) (void)hipStreamDestroy(z);
    if (e != hipSuccess) {
      (void)hipFree(p);
      return e;
    }
    for (int i = 0; i < kSlabSets; ++i) {
      TicketSet s;
      s.p = (uint32_t*)p + (size_t)i * kSetWords;
      if ((e = hipEventCreateWithFlags(&s.ev, hipEventDisableTiming)) != hipSuccess) return e;  // slab stays partly used
      free_sets.push_back(s);
      ++sets;
    }
    return hipSuccess;
  }
  void reclaim() {  // mu held: every set whose launch has finished goes back
    drain_returned();
    for (auto it = busy.begin(); it != busy.end();) {
      const hipError_t q = hipEventQuery(it->ev);
      if (q == hipSuccess) {
        free_sets.push_back(*it);
        it = busy.erase(it);
      } else {
        if (q != hipErrorNotReady) (void)hipGetLastError();
        ++it;
      }
    }
  }
  // Hand `stream` the busy set at `it` once its holder is done (see above).
  bool take_busy(std::deque<TicketSet>::iterator it, hipStream_t stream, TicketSet* out, hipError_t* err) {
    if ((*err = hipStreamWaitEvent(stream, it->ev, 0)) != hipSuccess) return false;
    *out = *it;
    busy.erase(it);
    return true;
  }
  // A set for a launch on `stream`.  false: none to be had (*err says why,
  // hipSuccess for a capture with no free set).
  bool take(hipStream_t stream, bool cap, TicketSet* out, hipError_t* err) {
    *err = hipSuccess;
    if (free_sets.empty()) reclaim();
    if (free_sets.empty() && !cap) {
      for (auto it = busy.rbegin(); it != busy.rend(); ++it)
        if (it->last == stream) return take_busy(std::next(it).base(), stream, out, err);
      if (sets < kMaxSets) {
        if ((*err = grow()) != hipSuccess) return false;
      } else if (!busy.empty()) {
        return take_busy(busy.begin(), stream, out, err);
      }
    }
    if (free_sets.empty()) return false;
    *out = free_sets.back();
    free_sets.pop_back();
    return true;
  }
};
// A captured launch's set, owned by the graph under capture: the destructor
// of a user object the graph retains returns it to the pool.
struct GraphSet {
  TicketPool* pool;
  TicketSet set;
};
void graph_set_release(void* p) {
  GraphSet* g = (GraphSet*)p;
  if (g->pool) g->pool->give_back(g->set);
  delete g;
}
// Ties `set` to the graph `stream` is capturing into; false if HIP refused.
bool bind_to_graph(TicketPool& tp, const TicketSet& set, hipStream_t stream) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  unsigned long long id = 0;
  hipGraph_t graph = nullptr;
  if (hipStreamGetCaptureInfo_v2(stream, &st, &id, &graph, nullptr, nullptr) != hipSuccess || !graph ||
      st != hipStreamCaptureStatusActive) {
    (void)hipGetLastError();
    return false;
  }
  GraphSet* g = new GraphSet{&tp, set};
  hipUserObject_t obj = nullptr;
  if (hipUserObjectCreate(&obj, g, graph_set_release, 1, hipUserObjectNoDestructorSync) != hipSuccess) {
    (void)hipGetLastError();
    delete g;
    return false;
  }
  if (hipGraphRetainUserObject(graph, obj, 1, hipGraphUserObjectMove) != hipSuccess) {
    // The graph did not take the reference: keep the set (the object's
    // destructor must not hand it back while the graph may replay it), and
    // drop our reference so the object and `g` are freed.
    (void)hipGetLastError();
    g->pool = nullptr;
    (void)hipUserObjectRelease(obj, 1);
    (void)hipGetLastError();
    return false;
  }
  return true;
}
TicketPool& ticket_pool(int dev) {
  static std::mutex mu;
  static auto* pools = new std::map<int, TicketPool>();  // never destroyed (see plan cache)
  std::lock_guard<std::mutex> lock(mu);
  return (*pools)[dev];  // std::map: the entry's address is stable
}
bool capturing(hipStream_t stream) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &st) != hipSuccess) {
    (void)hipGetLastError();
    return true;  // unknown: behave as inside a capture (no slab creation, no event)
  }
  return st != hipStreamCaptureStatusNone;
}
}  // namespace

hipError_t warm_ticket_pool(int device) {
  TicketPool& tp = ticket_pool(device);
  std::lock_guard<std::mutex> lock(tp.mu);
  return tp.sets ? hipSuccess : tp.grow();
}

void ticket_pool_stats(int device, uint64_t* sets, uint64_t* held) {
  TicketPool& tp = ticket_pool(device);
  std::lock_guard<std::mutex> lock(tp.mu);
  tp.reclaim();
  *sets = tp.sets;
  *held = tp.busy.size() + tp.graph_held + tp.lost;
}

void schedule_counts(int device, uint64_t* dynamic, uint64_t* fallback) {
  TicketPool& tp = ticket_pool(device);
  std::lock_guard<std::mutex> lock(tp.mu);
  *dynamic = tp.dynamic;
  *fallback = tp.fallback;
}

hipError_t with_tickets(hipStream_t stream, const std::function<hipError_t(uint32_t*)>& launch, bool* launched) {
  *launched = false;
  int dev = 0;
  if (hipError_t e = hipGetDevice(&dev)) return e;
  const bool cap = capturing(stream);
  TicketPool& tp = ticket_pool(dev);
  // The pool's lock is held across the launch: a set handed over behind an
  // event wait must see its event re-recorded before anyone else looks.
  std::lock_guard<std::mutex> lock(tp.mu);
  TicketSet set;
  hipError_t e;
  if (cap && queue_mode() != 2) return hipSuccess;  // the static kernel inside captures (see above)
  if (!tp.take(stream, cap, &set, &e)) {  // hipSuccess + !launched: static kernel
    if (e == hipSuccess) ++tp.fallback;
    return e;
  }
  e = launch(set.p);
  if (e != hipSuccess) {  // never started: the set is zero again once its holder (if any) is done
    tp.busy.push_back(set);
    return e;
  }
  *launched = true;
  ++tp.dynamic;
  if (cap) {
    ++tp.graph_held;  // the graph owns it from now on; its user object gives it back
    if (!bind_to_graph(tp, set, stream)) {
      --tp.graph_held;
      ++tp.lost;  // held for the life of the process
    }
    return hipSuccess;
  }
  if (const hipError_t r = hipEventRecord(set.ev, stream)) {
    // Without the event the set's release cannot be observed: wait for the
    // launch here, then the set is free (zero) again.
    (void)hipGetLastError();
    if (hipStreamSynchronize(stream) == hipSuccess) {
      tp.free_sets.push_back(set);
    } else {
      (void)hipGetLastError();
      ++tp.lost;
    }
    return r;
  }
  set.last = stream;
  tp.busy.push_back(set);
  return hipSuccess;
}

// Kernel form (process-wide): the software-pipelined kernels (default) or
// the non-pipelined forms that shards/chunks of 4 GiB and more always take;
// slime_rs_kernel_pipeline() switches it (the parity tests cover both forms
// in one process).
static std::atomic<int> g_pipelined{1};
bool pipelined_kernels() { return g_pipelined.load(std::memory_order_relaxed) != 0; }
// Work schedule of the pipelined kernels (process-wide): 1 = dynamic outside
// graph captures, static inside (default); 2 = dynamic in captures too; 0 =
// static shares.  slime_rs_kernel_schedule() switches it.
static std::atomic<int> g_queue_mode{1};
int queue_mode() { return g_queue_mode.load(std::memory_order_relaxed); }
bool queue_allowed(hipStream_t s) {
  const int m = queue_mode();
  return m == 2 || (m == 1 && !capturing(s));
}
void set_queue_mode(int m) { g_queue_mode.store(m, std::memory_order_relaxed); }
void set_pipelined_kernels(bool on) { g_pipelined.store(on ? 1 : 0, std::memory_order_relaxed); }
static std::atomic<int> g_switch_bits{0};
int switch_bits_mode() { return g_switch_bits.load(std::memory_order_relaxed); }
void set_switch_bits_mode(int m) { g_switch_bits.store(m, std::memory_order_relaxed); }

namespace {
// The pipelined kernel addresses a shard with 32-bit byte offsets: it needs
// ncols * 4 < 2^32 (shards under 4 GiB -- objects under 4 GiB x need).
// Larger shards take rs_apply_kernel.
bool pipe_ok(const ApplyLaunch& a) { return pipelined_kernels() && a.ncols < (1ull << 30); }

template <int K>
hipError_t dispatch_vec(const ApplyLaunch& a, hipStream_t s) {
  if (!a.vec_ok) return launch_k<K, false>(a, s);
  if (!pipe_ok(a)) return launch_k<K, true>(a, s);
  if (queue_allowed(s)) {
    bool launched = false;
    const hipError_t e = launch_queue<K>(a, s, &launched);
    if (launched || e != hipSuccess) return e;
  }
  return launch_pipe<K>(a, s);
}

// k > 16: rs_apply_wide_kernel -- all inputs in registers with 8-row blocks
// up to k = 32, 16-shard chunks with 16-row blocks above.
template <int KC, int RB>
hipError_t launch_wide_k(const ApplyLaunch& a, hipStream_t stream) {
  const uint64_t per_block = 4ull * kBlock;
  const uint32_t nseg = object_segments(a.nobj, a.ncols);
  const uint64_t nwork = (uint64_t)a.nobj * nseg;
  const uint64_t gy = nwork < 65535 ? nwork : 65535;
  const uint64_t target = 512;
  uint64_t gx = (target + gy - 1) / gy;
  const uint64_t need = (a.ncols / nseg + per_block - 1) / per_block;
  if (gx > need) gx = need;
  if (gx < 1) gx = 1;
  hipLaunchKernelGGL((apply::rs_apply_wide_kernel<KC, RB, kNtLoads, kNtStores>), dim3((uint32_t)gx, (uint32_t)gy),
                     dim3(kBlock), 0, stream, a.in, a.out, a.in_obj_stride, a.in_shard_stride, a.out_obj_stride,
                     a.out_shard_stride, a.coeff, a.in_idx, a.out_idx, a.ncols, a.nobj, a.rows, a.k, nseg);
  return hipGetLastError();
}

// Pipelined wide form (rs_apply_wide_pipe_kernel): a stream of 16-shard
// chunk loads, one in flight while the previous one's math runs; row blocks
// of 8 rows, 16 for codes with more than 8 output rows.  Block budget 256 up
// to k = 32, 1024 above (profiles/r01/widepipe/: 20/24 4460 GB/s vs 4405 for
// the chunked kernel, 32/40 4975 vs 4909, 64/80 3415 vs 3188).
template <int RB>
hipError_t launch_wide_pipe(const ApplyLaunch& a, hipStream_t stream) {
  const uint64_t per_block = 4ull * kBlock;
  const uint32_t nseg = object_segments(a.nobj, a.ncols);
  const uint64_t nwork = (uint64_t)a.nobj * nseg;
  const uint64_t gy = nwork < 65535 ? nwork : 65535;
  const uint64_t target = a.k <= 32 ? 256 : 1024;
  uint64_t gx = (target + gy - 1) / gy;
  const uint64_t need = (a.ncols / nseg + per_block - 1) / per_block;
  if (gx > need) gx = need;
  if (gx < 1) gx = 1;
  hipLaunchKernelGGL((apply::rs_apply_wide_pipe_kernel<RB, kNtLoads, kNtStores>), dim3((uint32_t)gx, (uint32_t)gy),
                     dim3(kBlock), 0, stream, a.in, a.out, a.in_obj_stride, a.in_shard_stride, a.out_obj_stride,
                     a.out_shard_stride, a.coeff, a.in_idx, a.out_idx, a.ncols, a.nobj, a.rows, a.k, nseg);
  return hipGetLastError();
}

hipError_t launch_wide(const ApplyLaunch& a, hipStream_t stream) {
  if (pipe_ok(a) && a.k <= 32) return launch_pipe_k32(a, stream);
  if (pipe_ok(a)) return a.rows <= 8 ? launch_wide_pipe<8>(a, stream) : launch_wide_pipe<16>(a, stream);
  return a.k <= 32 ? launch_wide_k<32, 8>(a, stream) : launch_wide_k<16, 16>(a, stream);
}

}  // namespace

hipError_t launch_apply(const ApplyLaunch& a, hipStream_t s) {
  (void)hipGetLastError();  // report only this launch's error, not one left on the thread
  if (a.nobj == 0 || a.ncols == 0 || a.rows == 0) return hipSuccess;
  if (mfma_eligible(a)) return launch_apply_mfma(a, s);  // wide codes on the matrix cores
  switch (a.k) {
    case 1: return dispatch_vec<1>(a, s);
    case 2: return dispatch_vec<2>(a, s);
    case 3: return dispatch_vec<3>(a, s);
    case 4: return dispatch_vec<4>(a, s);
    case 5: return dispatch_vec<5>(a, s);
    case 6: return dispatch_vec<6>(a, s);
    case 7: return dispatch_vec<7>(a, s);
    case 8: return dispatch_vec<8>(a, s);
    case 9: return dispatch_vec<9>(a, s);
    case 10: return dispatch_vec<10>(a, s);
    case 11: return dispatch_vec<11>(a, s);
    case 12: return dispatch_vec<12>(a, s);
    case 13: return dispatch_vec<13>(a, s);
    case 14: return dispatch_vec<14>(a, s);
    case 15: return dispatch_vec<15>(a, s);
    case 16: return dispatch_vec<16>(a, s);
    default: return a.vec_ok ? launch_wide(a, s) : launch_k<0, false>(a, s);
  }
}

}  // namespace slime
