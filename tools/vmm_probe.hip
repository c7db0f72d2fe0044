// Does the physical placement of a batch buffer decide the "slow placement"
// mode of the apply kernel?  One process times the product encode (C3: 8/12,
// 128 x 256 MiB objects) on batch buffers that differ only in how their
// physical memory is laid out behind the same kind of virtual range:
//   malloc  - hipMalloc (what the bench uses);
//   vmm-id  - HIP virtual memory: physical chunks of `chunk` bytes mapped in order;
//   vmm-rnd - the same chunks mapped in a random permutation.
// Rounds interleave the buffers, so drift cannot bias one of them.
// Tools only:  make tools/vmm_probe && tools/vmm_probe <kinds> <trials>
//   kinds: comma list of malloc | vmm-id:<chunk MiB> | vmm-rnd:<chunk MiB>, e.g. malloc,vmm-rnd:2,vmm-id:1024
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <random>
#include <string>
#include <vector>

#include "slime_rs.h"

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));       \
      exit(2);                                                                                 \
    }                                                                                          \
  } while (0)

struct Buf {
  std::string kind;
  uint32_t* p = nullptr;
  size_t bytes = 0;
  std::vector<hipMemGenericAllocationHandle_t> handles;
  size_t chunk = 0;
};

static Buf make_malloc(size_t bytes) {
  Buf b;
  b.kind = "malloc";
  b.bytes = bytes;
  CK(hipMalloc(&b.p, bytes));
  return b;
}

static Buf make_vmm(size_t bytes, size_t chunk, bool shuffle, uint64_t seed) {
  Buf b;
  b.kind = shuffle ? "vmm-rnd" : "vmm-id";
  b.bytes = bytes;
  b.chunk = chunk;
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  void* va = nullptr;
  CK(hipMemAddressReserve(&va, bytes, chunk, nullptr, 0));
  const size_t n = bytes / chunk;
  std::vector<size_t> slot(n);
  for (size_t i = 0; i < n; ++i) slot[i] = i;
  if (shuffle) std::shuffle(slot.begin(), slot.end(), std::mt19937_64(seed));
  b.handles.resize(n);
  for (size_t i = 0; i < n; ++i) {
    CK(hipMemCreate(&b.handles[i], chunk, &prop, 0));
    CK(hipMemMap((char*)va + slot[i] * chunk, chunk, 0, b.handles[i], 0));
  }
  hipMemAccessDesc acc = {};
  acc.location = prop.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  CK(hipMemSetAccess(va, bytes, &acc, 1));
  b.p = (uint32_t*)va;
  return b;
}

static void free_buf(Buf& b) {
  if (b.kind == "malloc") {
    CK(hipFree(b.p));
  } else {
    CK(hipMemUnmap(b.p, b.bytes));
    for (auto h : b.handles) CK(hipMemRelease(h));
    CK(hipMemAddressFree(b.p, b.bytes));
  }
  b.p = nullptr;
}

int main(int argc, char** argv) {
  const std::string kinds = argc > 1 ? argv[1] : "malloc,vmm-id:1024,vmm-rnd:2,malloc";
  const int trials = argc > 2 ? atoi(argv[2]) : 2;
  const uint64_t need = 8, total = 12, nobj = 128, L = 8388608;
  const size_t bytes = nobj * total * L * 4;
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  size_t gmin = 0, grec = 0;
  CK(hipMemGetAllocationGranularity(&gmin, &prop, hipMemAllocationGranularityMinimum));
  CK(hipMemGetAllocationGranularity(&grec, &prop, hipMemAllocationGranularityRecommended));
  printf("{\"granularity_min\": %zu, \"granularity_recommended\": %zu, \"kinds\": \"%s\"}\n", gmin, grec,
         kinds.c_str());
  fflush(stdout);
  std::vector<std::pair<std::string, size_t>> spec;  // kind, chunk bytes
  for (size_t a = 0; a < kinds.size();) {
    size_t b = kinds.find(',', a);
    if (b == std::string::npos) b = kinds.size();
    const std::string k = kinds.substr(a, b - a);
    const size_t c = k.find(':');
    const size_t chunk = c == std::string::npos ? 0 : (size_t)atoll(k.c_str() + c + 1) << 20;
    if (chunk % gmin || bytes % (chunk ? chunk : 1)) {
      fprintf(stderr, "bad chunk in %s\n", k.c_str());
      return 2;
    }
    spec.push_back({k.substr(0, c), chunk});
    a = b + 1;
  }
  slime_rs_plan_t plan;
  if (slime_rs_plan_encode(0, need, total, &plan) != 0) return 3;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const slime_rs_layout_t lay{total * L, L};
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int t = 0; t < trials; ++t) {
    std::vector<Buf> bufs;
    for (auto& k : spec)
      bufs.push_back(k.first == "malloc" ? make_malloc(bytes) : make_vmm(bytes, k.second, k.first == "vmm-rnd", 1234 + t));
    for (auto& x : bufs)
      if (slime_rs_fill_symbols(0, x.p, bytes / 4, 7 + t, s) != 0) return 4;
    CK(hipStreamSynchronize(s));
    std::vector<std::vector<float>> ms(bufs.size());
    for (int r = 0; r < 6; ++r)
      for (size_t i = 0; i < bufs.size(); ++i) {
        CK(hipEventRecord(a, s));
        if (slime_rs_plan_execute(plan, bufs[i].p, lay, bufs[i].p + need * L, lay, L, nobj, s) != 0) return 5;
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float v = 0;
        CK(hipEventElapsedTime(&v, a, b));
        if (r) ms[i].push_back(v);
      }
    for (size_t i = 0; i < bufs.size(); ++i) {
      std::sort(ms[i].begin(), ms[i].end());
      printf("{\"trial\": %d, \"buffer\": %zu, \"kind\": \"%s\", \"chunk\": %zu, \"encode_ms_median\": %.4f, "
             "\"encode_ms_min\": %.4f, \"va\": \"%p\"}\n",
             t, i, bufs[i].kind.c_str(), bufs[i].chunk, ms[i][ms[i].size() / 2], ms[i][0], (void*)bufs[i].p);
    }
    fflush(stdout);
    for (auto& x : bufs) free_buf(x);
  }
  slime_rs_plan_destroy(plan);
  return 0;
}
