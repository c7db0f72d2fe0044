// C-ABI of the MI355X Reed-Solomon shard codec (include/slime_rs.h): thread
// state and failure details, device routing of host calls, plans and the
// device-resident batch API, the host-only matrices and gf scalars, the *_ex
// forms the cgo shim binds, and introspection.  The host-memory entry points
// live in go_api.cpp (the Go API's rows and codec) and object_calls.cpp
// (writeChunks / reconstruct), over the pipeline of host_pipeline.cpp.
//
// Go-API entry points mirror internal/rs and internal/rs/gf: same argument
// meaning, same validation order, and the reference's panic text through
// slime_rs_status_string().  All data-path work runs on the GPU; with no
// device the compute entry points fail with SLIME_RS_ERR_NO_DEVICE (there is
// no CPU fallback).
#include "slime_rs.h"

#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <tuple>
#include <vector>

#include "capi_internal.hpp"
#include "device_pool.hpp"
#include "digest.hpp"
#include "gfp_host.hpp"
#include "host_copy.hpp"
#include "host_pipeline.hpp"
#include "kernels.hpp"
#include "mfma_table.hpp"
#include "plan_cache.hpp"
#include "rs_matrix.hpp"

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
}  // namespace

const slime_rs_call_t* active_call() { return t_call; }
int selected_device() { return t_device; }

// Admission of host calls.  A host call keeps CPUs busy (its host copies,
// the launches, the waits' polling, the copy pool's help), so more calls at
// once than the process has CPUs only time-slice them -- and under a cgroup
// CPU quota the whole process is throttled for the rest of the quota period
// once it overdraws: 25 concurrent 1 MiB callers on a 16-CPU share ran 17.5
// GiB/s with a 36 ms p99 against 26.8 GiB/s and 0.8 ms at 16 callers
// (profiles/r05/s3_refactor, s5_sched).  Callers beyond the slots sleep
// until one frees; a Go proxy's goroutines (main.go:107-109) wait there
// instead of on the CPU.  Slots pass in arrival order (a freed slot goes
// straight to the oldest waiter): with a plain condition variable a caller
// could lose the race for a freed slot again and again -- 64 MiB requests
// waited up to 1.8 s behind others that took 15 ms (profiles/r05/s6_slots).
namespace {
HostCallSlots& host_slots() {
  static auto* s = new HostCallSlots(host_call_slots());  // never destroyed (callers may outlive statics)
  return *s;
}
}  // namespace

int host_call_slots() {
  static const int n = std::max(4, usable_cpus() / 2);
  return n;
}

int DeviceLease::acquire() {
  const int call = t_call ? t_call->device : SLIME_RS_ANY_DEVICE;
  const int thread = t_call ? SLIME_RS_ANY_DEVICE : t_device;
  const int want = call != SLIME_RS_ANY_DEVICE ? call : thread;
  if (int rc = check_device(want != SLIME_RS_ANY_DEVICE ? want : 0)) return rc;
  host_slots().enter();
  slot_ = true;
  lease.take(g_pool, call, thread, pool_devices());
  device = lease.device;
  return 0;
}

DeviceLease::~DeviceLease() {
  // Out of the device's in-flight count first, then the host-call slot: the
  // waiter the slot wakes routes by in-flight counts that no longer include
  // this finished call.
  lease.release();
  if (slot_) host_slots().leave();
}

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
  plan->in_seq = true;
  for (uint32_t j = 0; j < in_idx.size(); ++j) plan->in_seq = plan->in_seq && in_idx[j] == j;
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

static bool aligned4(const void* p) { return ((uintptr_t)p & 3u) == 0; }

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
  a.in_seq = plan->in_seq;
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

// The host entry points' plan cache (PlanKey: device, kind, need, total,
// indices): a bounded LRU (plan_cache.hpp).  Env SLIME_RS_PLAN_CACHE sets the
// capacity (default 256 plans: at 20/40 a recovery plan's table is about 4 KiB).
// Never destroyed: freeing device tables from a static destructor would run
// after the HIP runtime may have shut down.
static LruCache<PlanKey, slime_rs_plan>& plans() {
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

// ---- MapToGF fallback candidates (the reference's rand.Uint32() stream) ------

namespace {
std::mutex g_rng_mu;
std::mt19937_64 g_rng{std::random_device{}()};
}  // namespace

void draw_candidates(uint32_t* cand, uint32_t n) {
  std::lock_guard<std::mutex> lk(g_rng_mu);
  for (uint32_t c = 0; c < n; ++c) cand[c] = (uint32_t)(g_rng() >> 32);
}

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

}  // namespace slime

using namespace slime;

extern "C" {
const char* slime_rs_status_string(int status) { return status_text(status); }
const char* slime_rs_last_error(void) { return t_error.c_str(); }
const char* slime_rs_version(void) { return "slime_rs 0.1 (gfx950, GF(2^32-5))"; }
int slime_rs_device_count(void) { return visible_devices(); }

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

int slime_rs_switch_bits(int mode) {
  if (mode < 0) return switch_bits_mode();
  if (mode > 2)
    return fail(Status::InvalidArg,
                "switch_bits: mode must be 0 (by object size), 1 (always correct) or 2 (always re-encode)");
  set_switch_bits_mode(mode);
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

}  // extern "C"
BytesLaunch slime::bytes_launch(const slime_rs_plan* plan, uint8_t* slots, uint64_t slot_stride, uint64_t cstride,
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
extern "C" {

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
  uint64_t bytes() const { return held ? buf.bytes : 0; }
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

extern "C" int slime_rs_encode_objects_phased(slime_rs_plan_t plan, uint8_t* slots, uint64_t slot_stride,
                                              uint64_t chunk_stride, uint64_t object_size, uint64_t nobj,
                                              uint32_t* mapping, uint32_t* status, void* stream, void* phase_event) {
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
  a0.scratch_bytes = sc.bytes();
  a0.sw = &sw;
  HIP_TRY(launch_encode_bytes(a0, s));
  HIP_TRY(launch_select_mapping(mapping, status, (uint32_t)nobj, s));
  if (phase_event) HIP_TRY(hipEventRecord((hipEvent_t)phase_event, s));
  BytesLaunch a1 = bytes_launch(plan, slots, slot_stride, chunk_stride, L, object_size, nobj, 1, status, mapping);
  if (sw.switched) {
    a1.scratch = sc.ptr();
    a1.scratch_bytes = sc.bytes();
    a1.sw = &sw;
  }
  HIP_TRY(launch_encode_bytes(a1, s));
  sc.release(s);
  return 0;
}

extern "C" int slime_rs_encode_objects_chunked(slime_rs_plan_t plan, uint8_t* slots, uint64_t slot_stride,
                                               uint64_t chunk_stride, uint64_t object_size, uint64_t nobj,
                                               uint32_t* mapping, uint32_t* status, void* stream) {
  return slime_rs_encode_objects_phased(plan, slots, slot_stride, chunk_stride, object_size, nobj, mapping, status,
                                        stream, nullptr);
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
  constexpr uint32_t kCand = kMapCandidates;
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
      draw_candidates(cand, kCand);
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

int slime_rs_host_call_slots(void) { return host_call_slots(); }

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
