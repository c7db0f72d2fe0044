// Device batch buffers of the C-ABI (include/slime_rs.h: slime_rs_device_alloc,
// _alloc_info, _free).  A buffer is `n` physical chunks (hipMemCreate) mapped
// in order into one reserved virtual range, or (a probed alternative) one
// hipMalloc; a registry maps each base to its buffer for _free and _info.
// The physical placement of a large buffer decides whether the kernels run
// in the slow mode (DESIGN.md "Placement modes"), so large buffers are
// probed once created and re-placed when slow.
#include "slime_rs.h"

#include <hip/hip_runtime.h>
#include <stdlib.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "capi_common.hpp"
#include "gfp_host.hpp"
#include "kernels.hpp"

namespace slime {
namespace {
struct DevBuffer {
  int device = 0;
  uint64_t bytes = 0, chunk = 0;  // chunk 0: hipMalloc
  std::vector<hipMemGenericAllocationHandle_t> handles;
  slime_rs_alloc_info_t info = {};
};
std::mutex g_vmm_mu;
std::map<void*, DevBuffer>& dev_buffers() {
  static auto* m = new std::map<void*, DevBuffer>();
  return *m;
}
uint64_t vmm_chunk_bytes() {
  static const uint64_t c = [] {
    const char* e = getenv("SLIME_RS_VMM_CHUNK_MIB");
    const long long v = e ? atoll(e) : 0;
    return (uint64_t)(v > 0 ? v : 2) << 20;
  }();
  return c;
}
double env_double(const char* name, double dflt) {
  const char* e = getenv(name);
  return e && *e ? atof(e) : dflt;
}
// Unmaps and releases the first `mapped` / `created` chunks, frees the range.
void vmm_unwind(void* va, uint64_t bytes, uint64_t chunk, const std::vector<hipMemGenericAllocationHandle_t>& h,
                size_t created, size_t mapped) {
  for (size_t i = 0; i < mapped; ++i) (void)hipMemUnmap((char*)va + i * chunk, chunk);
  for (size_t i = 0; i < created; ++i) (void)hipMemRelease(h[i]);
  (void)hipMemAddressFree(va, bytes);
}
void release_buffer(void* va, const DevBuffer& b) {
  if (b.chunk == 0)
    (void)hipFree(va);
  else
    vmm_unwind(va, b.bytes, b.chunk, b.handles, b.handles.size(), b.handles.size());
}

// `bytes` as physical chunks of `chunk` bytes mapped in order (chunk 0:
// hipMalloc).  The current device is `device`.
int map_buffer(int device, uint64_t bytes, uint64_t chunk, void** va_out, DevBuffer* out) {
  out->device = device;
  if (chunk == 0) {
    void* p = nullptr;
    HIP_TRY(hipMalloc(&p, bytes));
    out->bytes = bytes;
    out->chunk = 0;
    *va_out = p;
    return 0;
  }
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = device;
  size_t gran = 0;
  HIP_TRY(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum));
  if (gran && chunk % gran) chunk = (chunk + gran - 1) / gran * gran;
  const uint64_t total = (bytes + chunk - 1) / chunk * chunk;
  const size_t n = (size_t)(total / chunk);
  void* va = nullptr;
  HIP_TRY(hipMemAddressReserve(&va, total, chunk, nullptr, 0));
  std::vector<hipMemGenericAllocationHandle_t> h(n);
  for (size_t i = 0; i < n; ++i) {
    if (hipError_t e = hipMemCreate(&h[i], chunk, &prop, 0)) {
      vmm_unwind(va, total, chunk, h, i, i);
      return fail(Status::Hip, std::string("device_alloc: hipMemCreate: ") + hipGetErrorString(e));
    }
    if (hipError_t e = hipMemMap((char*)va + i * chunk, chunk, 0, h[i], 0)) {
      vmm_unwind(va, total, chunk, h, i + 1, i);
      return fail(Status::Hip, std::string("device_alloc: hipMemMap: ") + hipGetErrorString(e));
    }
  }
  hipMemAccessDesc acc = {};
  acc.location = prop.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  if (hipError_t e = hipMemSetAccess(va, total, &acc, 1)) {
    vmm_unwind(va, total, chunk, h, n, n);
    return fail(Status::Hip, std::string("device_alloc: hipMemSetAccess: ") + hipGetErrorString(e));
  }
  out->bytes = total;
  out->chunk = chunk;
  out->handles = std::move(h);
  *va_out = va;
  return 0;
}

// The placement probe: the product apply kernel's C3-shaped walk (8 data
// shards in, 4 parity shards out, 128 objects) over the whole fresh buffer,
// one warm launch and two timed ones on a private stream; GB/s of
// algorithmic traffic of the faster timed launch (0: not measurable).  The
// slow placement mode follows a buffer's physical memory for its whole life
// and shows up in exactly this many-stream read/write mix (DESIGN.md
// "Placement modes"); the buffer's contents are garbage either way.
double placement_probe(int device, uint8_t* va, uint64_t bytes) {
  constexpr uint32_t kNeed = 8, kTotal = 12, kRows = kTotal - kNeed, kObj = 128;
  // The coefficient / index table goes in the buffer's last 4 KiB, past the
  // objects: no allocation (a hipMalloc / hipFree pair synchronises the
  // device, and is not allowed while another thread captures a graph).
  constexpr uint64_t kTableRoom = 4096;
  if (bytes < 2 * kTableRoom) return 0;
  const uint64_t L = ((bytes - kTableRoom) / 4 / kTotal / kObj) & ~(uint64_t)63;
  if (L < 65536) return 0;
  std::vector<uint32_t> table(kRows * 16 + 16, 0);
  for (uint32_t i = 0; i < kRows; ++i)
    for (uint32_t j = 0; j < kNeed; ++j) table[i * 16 + j] = 0x9E3779B9u * (i * kNeed + j + 1) % kP;
  for (uint32_t j = 0; j < kNeed; ++j) table[kRows * 16 + j] = j;
  for (uint32_t i = 0; i < kRows; ++i) table[kRows * 16 + 8 + i] = kNeed + i;
  uint32_t* const d = (uint32_t*)(va + bytes - kTableRoom);
  hipStream_t s = nullptr;
  hipEvent_t ev[3] = {};
  double best = 0;
  // Everything on a private non-blocking stream, waited for there only: no
  // other stream (torch's, or a capture in progress on another thread) is
  // synchronised, and nothing is allocated or freed.
  const bool made = hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess;
  bool ok = made && hipMemcpyAsync(d, table.data(), table.size() * 4, hipMemcpyHostToDevice, s) == hipSuccess;
  for (auto& e : ev) ok = ok && hipEventCreate(&e) == hipSuccess;
  if (ok) {
    ApplyLaunch a;
    a.in = (const uint32_t*)va;
    a.out = (uint32_t*)va;
    a.in_obj_stride = a.out_obj_stride = kTotal * L;
    a.in_shard_stride = a.out_shard_stride = L;
    a.coeff = d;
    a.in_idx = d + kRows * 16;
    a.out_idx = d + kRows * 16 + 8;
    a.ncols = L;
    a.nobj = kObj;
    a.rows = kRows;
    a.k = kNeed;
    a.vec_ok = true;
    ok = launch_apply(a, s) == hipSuccess && hipEventRecord(ev[0], s) == hipSuccess &&
         launch_apply(a, s) == hipSuccess && hipEventRecord(ev[1], s) == hipSuccess &&
         launch_apply(a, s) == hipSuccess && hipEventRecord(ev[2], s) == hipSuccess &&
         hipStreamSynchronize(s) == hipSuccess;
    float ms[2] = {0, 0};
    if (ok && hipEventElapsedTime(&ms[0], ev[0], ev[1]) == hipSuccess &&
        hipEventElapsedTime(&ms[1], ev[1], ev[2]) == hipSuccess) {
      const double t = std::min(ms[0], ms[1]) * 1e-3;
      if (t > 0) best = (double)kObj * 4.0 * L * kTotal / t / 1e9;
    }
  }
  if (!ok) (void)hipGetLastError();
  if (made) (void)hipStreamSynchronize(s);  // the table upload reads `table`: done before it goes
  for (auto& e : ev)
    if (e) (void)hipEventDestroy(e);
  if (s) (void)hipStreamDestroy(s);
  return best;
}
}  // namespace
}  // namespace slime

using namespace slime;

extern "C" {

// Placement: a buffer of at least SLIME_RS_PLACEMENT_PROBE_GIB (default 16)
// is probed once created (placement_probe).  Below SLIME_RS_PLACEMENT_MIN_GBS
// (default 6350, the top of the rates seen: so in practice always) the library
// tries the other placements -- 1 GiB chunks, then one hipMalloc -- while
// still holding the first, while the device has room for both, and keeps the
// fastest.  Fast placements differ by ~3% among themselves (C3 frac 0.761 to
// 0.783 at one threshold of 6100, profiles/r06/s34_placement_aim).
int slime_rs_device_alloc(int device, uint64_t bytes, void** ptr) {
  if (!ptr || bytes == 0) return fail(Status::InvalidArg, "device_alloc: null ptr or zero bytes");
  *ptr = nullptr;
  if (int rc = check_device(device)) return rc;
  DeviceScope ds(device);
  void* va = nullptr;
  DevBuffer best;
  if (int rc = map_buffer(device, bytes, vmm_chunk_bytes(), &va, &best)) return rc;
  const double probe_gib = env_double("SLIME_RS_PLACEMENT_PROBE_GIB", 16.0);
  slime_rs_alloc_info_t& info = best.info;
  info.kind = 0;
  info.chunk_bytes = best.chunk;
  if (probe_gib > 0 && (double)bytes >= probe_gib * (1ull << 30)) {
    const double want = slime_rs_placement_threshold();
    double best_gbs = placement_probe(device, (uint8_t*)va, bytes);
    info.probe_gbs[0] = best_gbs;
    info.probe_chunk[0] = best.chunk;
    info.probes = 1;
    const uint64_t alts[2] = {1ull << 30, 0};  // 1 GiB chunks, then hipMalloc
    for (uint64_t alt : alts) {
      if (best_gbs <= 0 || best_gbs >= want || alt == best.chunk) continue;
      size_t free_b = 0, total_b = 0;
      if (hipMemGetInfo(&free_b, &total_b) != hipSuccess || free_b < bytes + (2ull << 30)) break;
      void* va2 = nullptr;
      DevBuffer cand;
      if (map_buffer(device, bytes, alt, &va2, &cand) != 0) {
        (void)hipGetLastError();
        break;
      }
      const double gbs = placement_probe(device, (uint8_t*)va2, bytes);
      const int idx = info.probes++;
      info.probe_gbs[idx] = gbs;
      info.probe_chunk[idx] = alt;
      if (gbs > best_gbs) {  // keep the new placement, release the old one
        release_buffer(va, best);
        const slime_rs_alloc_info_t keep = info;
        best = std::move(cand);
        best.info = keep;
        best.info.chosen = idx;
        best.info.kind = alt ? 0 : 1;
        best.info.chunk_bytes = alt;
        va = va2;
        best_gbs = gbs;
      } else {
        release_buffer(va2, cand);
      }
    }
  }
  {
    std::lock_guard<std::mutex> lock(g_vmm_mu);
    dev_buffers()[va] = std::move(best);
  }
  *ptr = va;
  return 0;
}

double slime_rs_placement_threshold(void) { return env_double("SLIME_RS_PLACEMENT_MIN_GBS", 6350.0); }

// The allocator's probe over a caller's range.  The range must lie inside one
// device allocation (hipMalloc, or a slime_rs_device_alloc buffer): the probe
// kernel writes to all of it.
int slime_rs_probe_placement(void* ptr, uint64_t bytes, int device, double* gbs) {
  if (!ptr || !gbs) return fail(Status::InvalidArg, "probe_placement: null ptr or output");
  *gbs = 0;
  if (((uintptr_t)ptr & 3u) != 0) return fail(Status::InvalidArg, "probe_placement: ptr not 4-byte aligned");
  if (int rc = check_device(device)) return rc;
  DeviceScope ds(device);
  const uintptr_t p0 = (uintptr_t)ptr, p1 = p0 + bytes;
  bool inside = false;
  {
    std::lock_guard<std::mutex> lock(g_vmm_mu);
    for (const auto& kv : dev_buffers()) {
      const uintptr_t b0 = (uintptr_t)kv.first, b1 = b0 + kv.second.bytes;
      if (p0 >= b0 && p1 <= b1) {
        if (kv.second.device != device) return fail(Status::InvalidArg, "probe_placement: buffer is on another device");
        inside = true;
        break;
      }
    }
  }
  if (!inside) {
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    if (hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)ptr) != hipSuccess) {
      (void)hipGetLastError();
      return fail(Status::InvalidArg, "probe_placement: not a device allocation");
    }
    hipPointerAttribute_t attr = {};
    if (hipPointerGetAttributes(&attr, ptr) != hipSuccess || attr.type != hipMemoryTypeDevice ||
        attr.device != device) {
      (void)hipGetLastError();
      return fail(Status::InvalidArg, "probe_placement: not device memory of this device");
    }
    if (p0 < (uintptr_t)base || p1 > (uintptr_t)base + size)
      return fail(Status::InvalidArg, "probe_placement: range exceeds its allocation");
  }
  *gbs = placement_probe(device, (uint8_t*)ptr, bytes);  // synchronises its own stream only
  return 0;
}

int slime_rs_device_alloc_info(const void* ptr, slime_rs_alloc_info_t* info) {
  if (!info) return fail(Status::InvalidArg, "device_alloc_info: null info");
  std::lock_guard<std::mutex> lock(g_vmm_mu);
  auto it = dev_buffers().find(const_cast<void*>(ptr));
  if (it == dev_buffers().end()) return fail(Status::InvalidArg, "device_alloc_info: not a slime_rs_device_alloc base");
  *info = it->second.info;
  return 0;
}

int slime_rs_device_free(void* ptr) {
  DevBuffer b;
  {
    std::lock_guard<std::mutex> lock(g_vmm_mu);
    auto it = dev_buffers().find(ptr);
    if (it == dev_buffers().end()) return fail(Status::InvalidArg, "device_free: not a slime_rs_device_alloc base");
    b = std::move(it->second);
    dev_buffers().erase(it);
  }
  DeviceScope ds(b.device);
  // Work still queued on any stream may touch the range (a tensor dropped right
  // after an asynchronous launch): wait for the device before unmapping.
  const hipError_t e = hipDeviceSynchronize();
  release_buffer(ptr, b);
  if (e != hipSuccess) return fail(Status::Hip, std::string("device_free: hipDeviceSynchronize: ") + hipGetErrorString(e));
  return 0;
}

}  // extern "C"
