// 17 <= need <= 32: the software-pipelined k-template byte kernels
// (encode_bytes_pipe_kernel / decode_bytes_pipe_kernel, rs_bytes_kernel.hpp)
// instantiated for wide codes, as the apply kernel does in rs_apply_k32.hip:
// every data chunk's tile in registers at once instead of the wide kernels'
// 16-chunk item stream.  One 16-byte unit per lane per tile (the encode keeps
// MapToGF's flags and the edge path beside its two register sets), 256 blocks.
#include <hip/hip_runtime.h>

#include "kernels.hpp"
#include "rs_bytes_kernel.hpp"
#include "rs_bytes_launch.hpp"

namespace slime {
namespace {

constexpr uint64_t kBlocks = 256;
// Dynamic schedule (queue kernels, rs_bytes_kernel.hpp) unless switched off
// (slime_rs_kernel_schedule): units of C = 6 one-unit tiles, as the apply
// kernel's k32 queue form.  In-process A/B (tools/bytes_ab.py,
// profiles/r02/s68_bytesk32/): 20/24 encode 2.585 -> 2.464 ms, decode 2.279 ->
// 2.180; 32/40 decode 1.905 -> 1.906 but encode 2.623 -> 2.785 (the queue
// encode holds 484 registers at need 32), so the encode takes it up to need 24.
constexpr int kQueueTiles = 6;
constexpr int kQueueEncodeMaxK = 24;

template <int K>
hipError_t enc_k32(const BytesLaunch& a, hipStream_t s) {
  const uint64_t ncols = a.ncols ? a.ncols : a.L;
  if constexpr (K <= kQueueEncodeMaxK) {
    if (a.phase == 1 && a.scratch) return bytes::launch_redo<K, 1, kQueueTiles>(a, ncols, s);
    if (a.phase == 0) {
      bool launched = false;
      const hipError_t e = bytes::launch_encode_queue<K, 1, kQueueTiles>(a, ncols, s, &launched);
      if (launched || e != hipSuccess) return e;
    }
  }
  if (a.phase == 0) {
    const uint32_t nseg = object_segments(a.nobj, ncols);
    hipLaunchKernelGGL((bytes::encode_bytes_pipe_kernel<K, 1, 0>),
                       bytes_grid(ncols, (uint64_t)a.nobj * nseg, nseg, kBlocks, 1), dim3(apply::kBlock), 0, s,
                       a.slots, a.slot_stride, a.L, chunk_stride(a), a.col0, ncols, a.S, a.nobj, a.rows, a.coeff, a.out_idx, a.flags,
                       a.mapping, nseg);
  } else {
    hipLaunchKernelGGL((bytes::encode_bytes_pipe_kernel<K, 1, 1>), bytes_grid(ncols, 1, 1, kBlocks, 1),
                       dim3(apply::kBlock), 0, s, a.slots, a.slot_stride, a.L, chunk_stride(a), a.col0, ncols, a.S, a.nobj, a.rows,
                       a.coeff, a.out_idx, a.flags, a.mapping, 1u);
  }
  return hipGetLastError();
}

template <int K>
uint64_t enc_switch_bytes(const BytesLaunch& a, hipStream_t s) {
  if constexpr (K <= kQueueEncodeMaxK)
    return bytes::switch_layout<K, 1, kQueueTiles>(a, a.ncols ? a.ncols : a.L, s).bytes;
  return 0;
}

template <int K>
hipError_t dec_k32(const BytesLaunch& a, hipStream_t s) {
  const uint64_t ncols = a.ncols ? a.ncols : a.L;
  const uint32_t spread = queue_allowed(s) ? queue_spread(a.nobj, ncols, 1, kQueueTiles) : 0;
  if (spread) {
    bool launched = false;
    const hipError_t e = with_tickets(
        s,
        [&](uint32_t* set) {
          hipLaunchKernelGGL((bytes::decode_bytes_queue_kernel<K, 1, kQueueTiles, kQueueCounters>),
                             dim3((uint32_t)queue_blocks(kBlocks, queue_units(a.nobj, ncols, 1, kQueueTiles, spread))),
                             dim3(apply::kBlock), 0, s, a.slots, a.slot_stride, a.L, chunk_stride(a), a.col0,
                             ncols, a.nobj, a.rows, a.coeff, a.in_idx, a.out_idx, a.mapping, set, spread);
          return hipGetLastError();
        },
        &launched);
    if (launched || e != hipSuccess) return e;
  }
  const uint32_t nseg = object_segments(a.nobj, ncols);
  hipLaunchKernelGGL((bytes::decode_bytes_pipe_kernel<K, 1>),
                     bytes_grid(ncols, (uint64_t)a.nobj * nseg, nseg, kBlocks, 1), dim3(apply::kBlock), 0, s,
                     a.slots, a.slot_stride, a.L, chunk_stride(a), a.col0, ncols, a.nobj, a.rows, a.coeff, a.in_idx, a.out_idx,
                     a.mapping, nseg);
  return hipGetLastError();
}

#define SLIME_K32_SWITCH(fn)                 \
  switch (a.k) {                             \
    case 17: return fn<17>(a, s);            \
    case 18: return fn<18>(a, s);            \
    case 19: return fn<19>(a, s);            \
    case 20: return fn<20>(a, s);            \
    case 21: return fn<21>(a, s);            \
    case 22: return fn<22>(a, s);            \
    case 23: return fn<23>(a, s);            \
    case 24: return fn<24>(a, s);            \
    case 25: return fn<25>(a, s);            \
    case 26: return fn<26>(a, s);            \
    case 27: return fn<27>(a, s);            \
    case 28: return fn<28>(a, s);            \
    case 29: return fn<29>(a, s);            \
    case 30: return fn<30>(a, s);            \
    case 31: return fn<31>(a, s);            \
    case 32: return fn<32>(a, s);            \
    default: return hipErrorInvalidValue;    \
  }

}  // namespace

hipError_t launch_encode_bytes_k32(const BytesLaunch& a, hipStream_t s) { SLIME_K32_SWITCH(enc_k32) }
uint64_t encode_switch_bytes_k32(const BytesLaunch& a, hipStream_t s) { SLIME_K32_SWITCH(enc_switch_bytes) }
hipError_t launch_decode_bytes_k32(const BytesLaunch& a, hipStream_t s) { SLIME_K32_SWITCH(dec_k32) }

}  // namespace slime
