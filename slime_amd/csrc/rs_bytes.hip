// Fused byte-domain encode/decode launchers (kernels: rs_bytes_kernel.hpp).
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include <algorithm>

#include "kernels.hpp"
#include "rs_bytes_kernel.hpp"
#include "rs_bytes_launch.hpp"

namespace slime {
namespace bytes {
// flags -> MapToGF's choice (map.go:35-62): 0 if no word >= p, else 1<<31 if
// that fits, else the random fallback: status 1, resolved on the host.
// `status` holds the flags on entry (in place: each lane owns one object).
__global__ void select_mapping_kernel(uint32_t* __restrict__ mapping, uint32_t* __restrict__ status, uint32_t nobj) {
  const uint32_t o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= nobj) return;
  const uint32_t f = status[o];
  const bool zero_ok = !(f & 1u), high_ok = !(f & 2u);
  mapping[o] = zero_ok ? 0u : (high_ok ? 0x80000000u : 0u);
  status[o] = (!zero_ok && !high_ok) ? 1u : 0u;
}
}  // namespace bytes

namespace {

using apply::kBlock;
using bytes::decode_bytes_kernel;
using bytes::encode_bytes_kernel;
using bytes::select_mapping_kernel;

template <int K>
constexpr int bytes_unroll() {
  return K <= 8 ? 4 : (K <= 12 ? 2 : 1);
}

// `target` resident blocks (default 512) over `work` object segments of about
// ncols/nseg columns, U units of 4 columns per lane per step.
dim3 grid_for(uint64_t ncols, uint64_t work, uint32_t nseg, uint64_t target = 512, int U = 1) {
  return bytes_grid(ncols, work, nseg, target, U);
}

// Software-pipelined forms (rs_bytes_kernel.hpp), the product for need <= 16
// when a chunk is under 4 GiB (32-bit offsets) and the kernel form is
// pipelined (slime_rs_kernel_pipeline, rs_apply.hip).  Geometry as the
// pipelined apply kernel.
template <int K>
constexpr int pipe_unroll() {
  return K == 1 ? 4 : K == 2 ? 2 : K <= 4 ? 1 : K <= 12 ? 3 : 1;
}
template <int K>
constexpr uint64_t pipe_blocks() {
  return K <= 12 ? 256 : 1024;
}
bool pipe_ok(const BytesLaunch& a) { return pipelined_kernels() && a.L < (1ull << 30); }

// The encode keeps its flags and the edge-tile path live beside the two
// register sets: U = 2 up to need 8, 1 above (no spills to scratch).
template <int K>
constexpr int enc_pipe_unroll() {
  return K <= 8 ? 2 : 1;
}

// Dynamic schedule (rs_bytes_kernel.hpp queue kernels, as the apply kernels in
// rs_apply.hip): 256 blocks, units of C tiles with C x U about 6, unless the
// schedule was switched to static (slime_rs_kernel_schedule) or the batch has
// too many units for 32-bit tickets (queue_spread, kernels.hpp).
constexpr uint64_t kQueueBlocks = 256;
template <int U>
constexpr int queue_tiles() {
  return U >= 3 ? 2 : 6 / U;
}

}  // namespace


namespace {

template <int K>
hipError_t enc_pipe(const BytesLaunch& a, hipStream_t s) {
  constexpr int U = enc_pipe_unroll<K>();
  constexpr int C = queue_tiles<U>();
  const uint64_t ncols = a.ncols ? a.ncols : a.L;
  if (a.phase == 1 && a.scratch) return bytes::launch_redo<K, U, C>(a, ncols, s);
  if (a.phase == 0) {
    bool launched = false;
    const hipError_t e = bytes::launch_encode_queue<K, U, C>(a, ncols, s, &launched);
    if (launched || e != hipSuccess) return e;
    const uint32_t nseg = object_segments(a.nobj, ncols);
    hipLaunchKernelGGL((bytes::encode_bytes_pipe_kernel<K, U, 0>),
                       grid_for(ncols, (uint64_t)a.nobj * nseg, nseg, pipe_blocks<K>(), U), dim3(kBlock), 0, s,
                       a.slots, a.slot_stride, a.L, chunk_stride(a), a.col0, ncols, a.S, a.nobj, a.rows, a.coeff, a.out_idx, a.flags,
                       a.mapping, nseg);
  } else {
    hipLaunchKernelGGL((bytes::encode_bytes_pipe_kernel<K, U, 1>), grid_for(ncols, 1, 1, pipe_blocks<K>(), U),
                       dim3(kBlock), 0, s, a.slots, a.slot_stride, a.L, chunk_stride(a), a.col0, ncols, a.S, a.nobj, a.rows, a.coeff,
                       a.out_idx, a.flags, a.mapping, 1u);
  }
  return hipGetLastError();
}

template <int K>
uint64_t enc_switch_bytes(const BytesLaunch& a, hipStream_t s) {
  if (!pipe_ok(a)) return 0;
  constexpr int U = enc_pipe_unroll<K>();
  return bytes::switch_layout<K, U, queue_tiles<U>()>(a, a.ncols ? a.ncols : a.L, s).bytes;
}

template <int K>
constexpr int dec_queue_unroll() {
  return K <= 4 ? 4 : K <= 12 ? 3 : 1;
}

template <int K>
hipError_t dec_pipe(const BytesLaunch& a, hipStream_t s) {
  constexpr int U = pipe_unroll<K>();
  const uint64_t ncols = a.ncols ? a.ncols : a.L;
  constexpr int QU = dec_queue_unroll<K>();
  const uint32_t spread = queue_allowed(s) ? queue_spread(a.nobj, ncols, QU, queue_tiles<QU>()) : 0;
  if (spread) {
    bool launched = false;
    const hipError_t e = with_tickets(
        s,
        [&](uint32_t* set) {
          hipLaunchKernelGGL((bytes::decode_bytes_queue_kernel<K, QU, queue_tiles<QU>(), kQueueCounters>),
                             dim3((uint32_t)queue_blocks(kQueueBlocks, queue_units(a.nobj, ncols, QU, queue_tiles<QU>(), spread))),
                             dim3(kBlock), 0, s, a.slots, a.slot_stride, a.L, chunk_stride(a), a.col0,
                             ncols, a.nobj, a.rows, a.coeff, a.in_idx, a.out_idx, a.mapping, set, spread);
          return hipGetLastError();
        },
        &launched);
    if (launched || e != hipSuccess) return e;
  }
  const uint32_t nseg = object_segments(a.nobj, ncols);
  hipLaunchKernelGGL((bytes::decode_bytes_pipe_kernel<K, U>),
                     grid_for(ncols, (uint64_t)a.nobj * nseg, nseg, pipe_blocks<K>(), U), dim3(kBlock), 0, s, a.slots,
                     a.slot_stride, a.L, chunk_stride(a), a.col0, ncols, a.nobj, a.rows, a.coeff, a.in_idx, a.out_idx, a.mapping, nseg);
  return hipGetLastError();
}

template <int K>
hipError_t enc_k(const BytesLaunch& a, hipStream_t s) {
  if (pipe_ok(a)) return enc_pipe<K>(a, s);
  constexpr int U = bytes_unroll<K>();
  // Phase 0 streams every object at once; phase 1 re-encodes the few objects
  // MapToGF maps with 1<<31 (~7.5% of 256 MiB random objects), so the whole
  // grid sweeps them one after another instead of 512/nobj blocks each.
  const uint64_t ncols = a.ncols ? a.ncols : a.L;
  if (a.phase == 0) {
    const uint32_t nseg = object_segments(a.nobj, ncols);
    hipLaunchKernelGGL((encode_bytes_kernel<K, U, 0>), grid_for(ncols, (uint64_t)a.nobj * nseg, nseg), dim3(kBlock),
                       0, s, a.slots, a.slot_stride, a.L, chunk_stride(a), a.col0, ncols, a.S, a.nobj, a.rows, a.coeff, a.out_idx,
                       a.flags, a.mapping, nseg);
  } else {
    hipLaunchKernelGGL((encode_bytes_kernel<K, U, 1>), grid_for(ncols, 1, 1), dim3(kBlock), 0, s, a.slots,
                       a.slot_stride, a.L, chunk_stride(a), a.col0, ncols, a.S, a.nobj, a.rows, a.coeff, a.out_idx, a.flags,
                       a.mapping, 1u);
  }
  return hipGetLastError();
}

template <int K>
hipError_t dec_k(const BytesLaunch& a, hipStream_t s) {
  if (pipe_ok(a)) return dec_pipe<K>(a, s);
  constexpr int U = bytes_unroll<K>();
  const uint64_t ncols = a.ncols ? a.ncols : a.L;
  const uint32_t nseg = object_segments(a.nobj, ncols);
  hipLaunchKernelGGL((decode_bytes_kernel<K, U>), grid_for(ncols, (uint64_t)a.nobj * nseg, nseg), dim3(kBlock), 0, s,
                     a.slots, a.slot_stride, a.L, chunk_stride(a), a.col0, ncols, a.nobj, a.rows, a.coeff, a.in_idx, a.out_idx,
                     a.mapping, nseg);
  return hipGetLastError();
}

// need > 16: the chunked byte kernels (rs_bytes_kernel.hpp, "wide k"):
// every input in registers up to need = 32, 16-chunk steps above.
constexpr int kWideRows = 8;

// Pipelined wide encode (rs_bytes_kernel.hpp): one wave per SIMD (256
// blocks; the kernel holds its flags and edge path beside two register sets).
template <int RB>
hipError_t enc_wide_pipe(const BytesLaunch& a, hipStream_t s) {
  const uint64_t ncols = a.ncols ? a.ncols : a.L;
  const uint64_t blocks = 256;
  if (a.phase == 0) {
    const uint32_t nseg = object_segments(a.nobj, ncols);
    hipLaunchKernelGGL((bytes::encode_bytes_wide_pipe_kernel<RB, 0>),
                       grid_for(ncols, (uint64_t)a.nobj * nseg, nseg, blocks, 1), dim3(kBlock), 0, s, a.slots,
                       a.slot_stride, a.L, chunk_stride(a), a.col0, ncols, a.S, a.nobj, a.rows, a.k, a.coeff, a.out_idx, a.flags,
                       a.mapping, nseg);
  } else {
    hipLaunchKernelGGL((bytes::encode_bytes_wide_pipe_kernel<RB, 1>), grid_for(ncols, 1, 1, blocks, 1), dim3(kBlock),
                       0, s, a.slots, a.slot_stride, a.L, chunk_stride(a), a.col0, ncols, a.S, a.nobj, a.rows, a.k, a.coeff, a.out_idx,
                       a.flags, a.mapping, 1u);
  }
  return hipGetLastError();
}

template <int KC>
hipError_t enc_wide_k(const BytesLaunch& a, hipStream_t s) {
  const uint64_t ncols = a.ncols ? a.ncols : a.L;
  if (a.phase == 0) {
    const uint32_t nseg = object_segments(a.nobj, ncols);
    hipLaunchKernelGGL((bytes::encode_bytes_wide_kernel<KC, kWideRows, 0>),
                       grid_for(ncols, (uint64_t)a.nobj * nseg, nseg), dim3(kBlock), 0, s, a.slots, a.slot_stride,
                       a.L, chunk_stride(a), a.col0, ncols, a.S, a.nobj, a.rows, a.k, a.coeff, a.out_idx, a.flags, a.mapping, nseg);
  } else {
    hipLaunchKernelGGL((bytes::encode_bytes_wide_kernel<KC, kWideRows, 1>), grid_for(ncols, 1, 1), dim3(kBlock), 0,
                       s, a.slots, a.slot_stride, a.L, chunk_stride(a), a.col0, ncols, a.S, a.nobj, a.rows, a.k, a.coeff, a.out_idx,
                       a.flags, a.mapping, 1u);
  }
  return hipGetLastError();
}

// Pipelined wide decode (rs_bytes_kernel.hpp): 8-row blocks, 16 for more
// than 8 rebuilt chunks; block budget as the wide apply kernel.
template <int RB>
hipError_t dec_wide_pipe(const BytesLaunch& a, hipStream_t s) {
  const uint64_t ncols = a.ncols ? a.ncols : a.L;
  const uint32_t nseg = object_segments(a.nobj, ncols);
  hipLaunchKernelGGL((bytes::decode_bytes_wide_pipe_kernel<RB>),
                     grid_for(ncols, (uint64_t)a.nobj * nseg, nseg, a.k <= 32 ? 256 : 1024, 1), dim3(kBlock), 0, s,
                     a.slots, a.slot_stride, a.L, chunk_stride(a), a.col0, ncols, a.nobj, a.rows, a.k, a.coeff, a.in_idx, a.out_idx,
                     a.mapping, nseg);
  return hipGetLastError();
}

template <int KC>
hipError_t dec_wide_k(const BytesLaunch& a, hipStream_t s) {
  const uint64_t ncols = a.ncols ? a.ncols : a.L;
  const uint32_t nseg = object_segments(a.nobj, ncols);
  hipLaunchKernelGGL((bytes::decode_bytes_wide_kernel<KC, kWideRows>), grid_for(ncols, (uint64_t)a.nobj * nseg, nseg),
                     dim3(kBlock), 0, s, a.slots, a.slot_stride, a.L, chunk_stride(a), a.col0, ncols, a.nobj, a.rows, a.k, a.coeff,
                     a.in_idx, a.out_idx, a.mapping, nseg);
  return hipGetLastError();
}

hipError_t enc_wide(const BytesLaunch& a, hipStream_t s) {
  if (bytes_mfma_eligible(a, true)) return launch_encode_bytes_mfma(a, s);
  if (pipe_ok(a) && a.k <= 32) return launch_encode_bytes_k32(a, s);
  if (pipe_ok(a)) return a.rows <= 8 ? enc_wide_pipe<8>(a, s) : enc_wide_pipe<16>(a, s);
  return a.k <= 32 ? enc_wide_k<32>(a, s) : enc_wide_k<16>(a, s);
}
hipError_t dec_wide(const BytesLaunch& a, hipStream_t s) {
  if (bytes_mfma_eligible(a, false)) return launch_decode_bytes_mfma(a, s);
  if (pipe_ok(a) && a.k <= 32) return launch_decode_bytes_k32(a, s);
  if (pipe_ok(a)) return a.rows <= 8 ? dec_wide_pipe<8>(a, s) : dec_wide_pipe<16>(a, s);
  return a.k <= 32 ? dec_wide_k<32>(a, s) : dec_wide_k<16>(a, s);
}

#define SLIME_K_SWITCH(fn)               \
  switch (a.k) {                         \
    case 1: return fn##_k<1>(a, s);      \
    case 2: return fn##_k<2>(a, s);      \
    case 3: return fn##_k<3>(a, s);      \
    case 4: return fn##_k<4>(a, s);      \
    case 5: return fn##_k<5>(a, s);      \
    case 6: return fn##_k<6>(a, s);      \
    case 7: return fn##_k<7>(a, s);      \
    case 8: return fn##_k<8>(a, s);      \
    case 9: return fn##_k<9>(a, s);      \
    case 10: return fn##_k<10>(a, s);    \
    case 11: return fn##_k<11>(a, s);    \
    case 12: return fn##_k<12>(a, s);    \
    case 13: return fn##_k<13>(a, s);    \
    case 14: return fn##_k<14>(a, s);    \
    case 15: return fn##_k<15>(a, s);    \
    case 16: return fn##_k<16>(a, s);    \
    default: return fn##_wide(a, s);     \
  }

}  // namespace

uint64_t encode_switch_bytes(const BytesLaunch& a, hipStream_t s) {
  if (a.nobj == 0 || a.L == 0 || a.phase != 0) return 0;
  switch (a.k) {
    case 1: return enc_switch_bytes<1>(a, s);
    case 2: return enc_switch_bytes<2>(a, s);
    case 3: return enc_switch_bytes<3>(a, s);
    case 4: return enc_switch_bytes<4>(a, s);
    case 5: return enc_switch_bytes<5>(a, s);
    case 6: return enc_switch_bytes<6>(a, s);
    case 7: return enc_switch_bytes<7>(a, s);
    case 8: return enc_switch_bytes<8>(a, s);
    case 9: return enc_switch_bytes<9>(a, s);
    case 10: return enc_switch_bytes<10>(a, s);
    case 11: return enc_switch_bytes<11>(a, s);
    case 12: return enc_switch_bytes<12>(a, s);
    case 13: return enc_switch_bytes<13>(a, s);
    case 14: return enc_switch_bytes<14>(a, s);
    case 15: return enc_switch_bytes<15>(a, s);
    case 16: return enc_switch_bytes<16>(a, s);
    default:
      if (bytes_mfma_eligible(a, true)) return encode_switch_bytes_mfma(a);
      return a.k <= 32 && pipe_ok(a) ? encode_switch_bytes_k32(a, s) : 0;
  }
}

hipError_t launch_encode_bytes(const BytesLaunch& a, hipStream_t s) {
  (void)hipGetLastError();  // report only this launch's error, not one left on the thread
  if (a.nobj == 0 || a.L == 0) return hipSuccess;
  if (a.col0 % 4 || a.col0 + a.ncols > a.L) return hipErrorInvalidValue;
  SLIME_K_SWITCH(enc)
}

hipError_t launch_decode_bytes(const BytesLaunch& a, hipStream_t s) {
  (void)hipGetLastError();  // report only this launch's error, not one left on the thread
  if (a.nobj == 0 || a.L == 0 || a.rows == 0) return hipSuccess;
  if (a.col0 % 4 || a.col0 + a.ncols > a.L) return hipErrorInvalidValue;
  SLIME_K_SWITCH(dec)
}

hipError_t launch_select_mapping(uint32_t* mapping, uint32_t* status, uint32_t nobj, hipStream_t s) {
  (void)hipGetLastError();  // report only this launch's error, not one left on the thread
  if (nobj == 0) return hipSuccess;
  hipLaunchKernelGGL(select_mapping_kernel, dim3((nobj + 255) / 256), dim3(256), 0, s, mapping, status, nobj);
  return hipGetLastError();
}

#undef SLIME_K_SWITCH

}  // namespace slime
