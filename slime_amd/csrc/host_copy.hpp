// Parallel host memcpy (and other byte passes split into pieces) for the pinned staging pipeline of the Go-API entry
// points (rs_capi.cpp).  A single host thread copies at ~10-20 GB/s, below
// what one PCIe/xGMI host link moves; the staging copies are split into
// pieces and run on a small persistent pool so the host side keeps pace with
// the DMA engines.
#pragma once
#include <stddef.h>

namespace slime {

struct CopyItem {
  void* dst;
  const void* src;
  size_t bytes;
};

// Copy every item (non-overlapping ranges).  Large items are split into
// pieces spread over the pool; the caller works too.  Concurrent callers are
// safe and share the pool: each drains its own job, workers help the oldest.
void parallel_copy(const CopyItem* items, size_t n);

// Run fn(ctx, 0..n-1) on the same pool (the host codec's pieces, host_codec.cpp):
// the caller drains pieces too and returns when every piece has run.
void parallel_pieces(size_t n, void (*fn)(const void* ctx, size_t piece), const void* ctx);

// Threads the pool runs besides the caller (env SLIME_RS_COPY_THREADS, default 4).
int copy_pool_threads();

// CPUs this process may run on: its affinity mask capped by the cgroup
// CPU quota (cpu.max), at least 1.
int usable_cpus();

}  // namespace slime
