// Small host<->device transfers of the host pipeline as one kernel over a
// span list (kernels.hpp, BlitSpan).  The pinned staging ring is mapped into
// the device's address space, so a kernel reads it (H2D) or writes it (D2H)
// across PCIe directly.  For a window of a few MiB this beats the copy
// engine: an SDMA transfer costs ~15-20 us of latency per direction, which
// was most of a 64 KiB host call (69 us of write_chunks: 40 us with
// kernel copies, profiles/r04/s10_lat4), and one launch replaces the
// window's several hipMemcpyAsync calls.  Larger windows keep the copy
// engines (rs_capi.cpp, dma_spans).
#include <hip/hip_runtime.h>

#include "kernels.hpp"

namespace slime {
namespace {

constexpr int kBlock = 256;

// Span i covers flat byte range [start[i], start[i] + bytes) of a launch;
// start[i] is 16-aligned (spans padded to 16 bytes in the flat numbering), so
// a lane's 16-byte step never straddles two spans.
struct BlitArgs {
  BlitSpan s[kBlitSpans];
  uint64_t start[kBlitSpans + 1];
  int n;
};

__global__ __launch_bounds__(kBlock) void blit_kernel(BlitArgs a) {
  const uint64_t total = a.start[a.n];
  const uint64_t step = (uint64_t)gridDim.x * kBlock * 16;
  for (uint64_t off = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) * 16; off < total; off += step) {
    int i = 0;
    while (a.start[i + 1] <= off) ++i;
    const BlitSpan& s = a.s[i];
    const uint64_t o = off - a.start[i];
    if (o >= s.bytes) continue;  // the span's padding
    const uint64_t n = s.bytes - o < 16 ? s.bytes - o : 16;
    uint8_t* d = (uint8_t*)s.dst + o;
    const uint8_t* r = (const uint8_t*)s.src + o;
    const uintptr_t al = (uintptr_t)d | (uintptr_t)r;
    if (n == 16 && (al & 15) == 0) {
      *(uint4*)d = *(const uint4*)r;
    } else if ((al & 3) == 0) {
      uint64_t k = 0;
      for (; k + 4 <= n; k += 4) *(uint32_t*)(d + k) = *(const uint32_t*)(r + k);
      for (; k < n; ++k) d[k] = r[k];
    } else {
      for (uint64_t k = 0; k < n; ++k) d[k] = r[k];
    }
  }
}

}  // namespace

hipError_t launch_blit(const BlitSpan* spans, int n, hipStream_t stream) {
  for (int b = 0; b < n; b += kBlitSpans) {
    BlitArgs a;
    a.n = n - b < kBlitSpans ? n - b : kBlitSpans;
    uint64_t off = 0;
    for (int i = 0; i < a.n; ++i) {
      a.s[i] = spans[b + i];
      a.start[i] = off;
      off += (spans[b + i].bytes + 15) & ~15ull;
    }
    a.start[a.n] = off;
    if (off == 0) continue;
    // One 16-byte step per lane where the list allows (4 KiB a block, up to
    // 1024 blocks): a step across PCIe is a round trip of microseconds, so
    // the copy is latency-bound unless all of it is in flight at once.
    uint64_t blocks = (off + 4095) >> 12;
    if (blocks > 1024) blocks = 1024;
    hipLaunchKernelGGL(blit_kernel, dim3((uint32_t)blocks), dim3(kBlock), 0, stream, a);
    if (hipError_t e = hipGetLastError()) return e;
  }
  return hipSuccess;
}

}  // namespace slime
