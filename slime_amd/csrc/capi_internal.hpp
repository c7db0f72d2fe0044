// Internal interface between the translation units of the C-ABI
// (include/slime_rs.h):
//   rs_capi.cpp        thread state, device routing, plans, the device-resident
//                      batch API, matrices/scalars, introspection, *_ex forms
//   host_pipeline.cpp  per-call workspaces and the pinned windowed pipeline
//                      (host_pipeline.hpp) behind every host-memory entry point
//   go_api.cpp         CreateParity / CreateParities / RecoverData and the
//                      MapToGF codec over host memory (the Go API's rows)
//   object_calls.cpp   writeChunks / reconstruct of whole objects (fused)
// Not part of the public C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <memory>
#include <string>
#include <tuple>
#include <vector>

#include "capi_common.hpp"
#include "device_pool.hpp"
#include "kernels.hpp"
#include "plan_cache.hpp"
#include "slime_rs.h"

// A compiled coefficient matrix on one device (slime_rs_plan_t).
struct slime_rs_plan {
  int device = 0;
  // Set by the first launch; slime_rs_plan_set_outputs refuses afterwards
  // (its table rewrite is not ordered against launches in flight).
  std::atomic<bool> executed{false};
  uint32_t rows = 0, k = 0;
  uint32_t out_max = 0;               // highest destination shard index
  std::vector<uint32_t> in_idx_host;  // input shard indices (host copy, bounds checks)
  std::vector<uint32_t> coeff;        // rows x k, host copy
  uint32_t* table = nullptr;          // device: coeff (rows x coeff_stride(k)) | in_idx (k) | out_idx (rows)
  const uint32_t* d_coeff = nullptr;
  const uint32_t* d_in_idx = nullptr;
  const uint32_t* d_out_idx = nullptr;
  const uint8_t* d_mfma = nullptr;     // device: matrix-core digit table (mfma_table.hpp), or null
  const uint8_t* d_mfma_be = nullptr;  // the same for big-endian chunk words (the byte path)
  uint32_t in_max = 0;                 // highest input shard index
  bool in_seq = false;                 // in_idx is 0..k-1 (encode plans)
};

namespace slime {

// ---- thread state (rs_capi.cpp) ----------------------------------------------
// The *_ex call active on this thread (explicit device, detail buffer), or null.
const slime_rs_call_t* active_call();
// The thread's slime_rs_select_device choice (SLIME_RS_ANY_DEVICE if none).
int selected_device();
// The reference's panic text (codes 1..8) or a short description.
const char* status_text(int st);
// fail() with "<what>: <status_text>" as the detail; 0 for Status::Ok.
int status_of(Status st, const char* what);

// ---- device routing (rs_capi.cpp) -------------------------------------------------
// The device of one host call: the *_ex call's explicit device, else the
// thread's selected device, else the device pool's pick (device_pool.hpp).
// Holds the pool slot for the life of the call, and one of the process's
// host-call slots (host_call_slots()): callers beyond them wait, asleep, for
// a slot before a device is picked.
struct DeviceLease {
  PoolLease lease;
  int device = -1;
  int acquire();
  ~DeviceLease();
  DeviceLease() = default;
  DeviceLease(const DeviceLease&) = delete;
  DeviceLease& operator=(const DeviceLease&) = delete;

 private:
  bool slot_ = false;
};
// Host calls that may run at once in this process: half the usable CPUs
// (affinity mask capped by the cgroup quota), at least 4.
int host_call_slots();

// ---- plans (rs_capi.cpp) ------------------------------------------------------------
int build_plan(int device, uint32_t rows, uint32_t k, const uint32_t* coeff, const std::vector<uint32_t>& in_idx,
               const std::vector<uint32_t>& out_idx, slime_rs_plan** out);
void destroy_plan(slime_rs_plan* plan);
int execute(const slime_rs_plan* plan, const uint32_t* src, uint64_t src_obj, uint64_t src_shard, uint32_t* dst,
            uint64_t dst_obj, uint64_t dst_shard, uint64_t L, uint64_t nobj, hipStream_t stream);
// Plans the host entry points reuse, keyed by (device, kind, need, total,
// indices): a bounded LRU (plan_cache.hpp; env SLIME_RS_PLAN_CACHE).
using PlanKey = std::tuple<int, char, int, int, std::vector<int>>;
using PlanRef = std::shared_ptr<slime_rs_plan>;
int cached_plan(const PlanKey& key, PlanRef* out, int (*make)(const PlanKey&, slime_rs_plan**));

// ---- byte path helpers (rs_capi.cpp) -----------------------------------------------
// perVector = ceil(ceil(S/4)/need) (multi_store.go:272).
inline uint64_t slot_L(uint64_t S, uint32_t need) { return ((S + 3) / 4 + need - 1) / need; }
BytesLaunch bytes_launch(const slime_rs_plan* plan, uint8_t* slots, uint64_t slot_stride, uint64_t cstride,
                         uint64_t L, uint64_t S, uint64_t nobj, int phase, uint32_t* flags, const uint32_t* mapping);

// ---- MapToGF fallback candidates (rs_capi.cpp) --------------------------------------
// The next n values of the library's random candidate stream (the
// reference's rand.Uint32(), map.go:64-66; slime_gf_seed).  Every placement
// draws kMapCandidates at a time and takes the first that fits, so a seeded
// stream gives the same mapping on the host and on the device.
constexpr uint32_t kMapCandidates = 64;
void draw_candidates(uint32_t* out, uint32_t n);

// ---- shared by go_api.cpp and object_calls.cpp ------------------------------------
// RecoverData's index checks (vector.go:65-77).
int check_survivors(int need, const int* indices);
// The survivors' inverse rows `want` as a plan over staged inputs 0..need-1.
int make_inverse_rows_plan(int dev, int need, const std::vector<int>& have, const std::vector<int>& want,
                           slime_rs_plan** out);
// gf.MapToGF's choice of mapping from the flags already OR-reduced into
// d_scratch[0] while packing nw words at d_words with mapping 0 (go_api.cpp);
// pick_mapping packs `len` device bytes first.  d_scratch: 4 + 2 *
// kMapCandidates words.
int choose_mapping(hipStream_t st, const uint32_t* d_words, uint64_t nw, uint32_t* d_scratch, uint32_t* mapping);
int pick_mapping(hipStream_t st, const uint8_t* d_bytes, uint64_t len, uint32_t* d_words, uint32_t* d_scratch,
                 uint32_t* mapping);

}  // namespace slime
