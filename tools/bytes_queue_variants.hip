// Unroll / unit-size variants of the fused byte encode's first pass
// (bytes::encode_bytes_queue_kernel, rs_bytes_kernel.hpp) at need 8 and 10,
// launched directly on a caller-owned ticket set (the kernel leaves it zero).
// Tools only: tools/bytes_queue_variants.py drives it.
#include <hip/hip_runtime.h>

#include "rs_bytes_launch.hpp"

using namespace slime;

namespace {
template <int K, int U, int C>
int launch(uint8_t* slots, uint64_t stride, uint64_t cstride, uint64_t L, uint64_t S, uint32_t nobj, uint32_t rows,
           const uint32_t* coeff, const uint32_t* out_idx, uint32_t* flags, uint32_t* ticket, uint32_t blocks,
           uint8_t* record, hipStream_t s) {
  const uint32_t spread = queue_spread(nobj, L, U, C);
  if (!spread) return -2;
  const uint32_t units = apply::walk_units<C>(bytes::encode_interior_tiles(S, L, 0, L, K, U), spread);
  hipLaunchKernelGGL((bytes::encode_bytes_queue_kernel<K, U, C, kQueueCounters>), dim3(blocks), dim3(apply::kBlock),
                     0, s, slots, stride, L, cstride, (uint64_t)0, L, S, nobj, rows, coeff, out_idx, flags, ticket,
                     spread, record, record ? units : 0u);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
}  // namespace

// record: the mid-object switch's per-unit record (>= nobj x units bytes) or
// null (mapping 0 throughout, as the capture form runs).
// variant: 0 <8,2,3> (product), 1 <8,3,2>, 2 <8,4,2>, 3 <10,1,6> (product), 4 <10,2,3>, 5 <10,3,2>, 6 <8,1,6>,
// 7 <4,2,3> (product), 8 <4,4,2>, 9 <4,3,2>
extern "C" int bqv_encode(int variant, uint8_t* slots, uint64_t stride, uint64_t cstride, uint64_t L, uint64_t S,
                          uint32_t nobj, uint32_t rows, const uint32_t* coeff, const uint32_t* out_idx,
                          uint32_t* flags, uint32_t* ticket, uint32_t blocks, uint8_t* record,
                          void* stream) {
  hipStream_t s = (hipStream_t)stream;
  switch (variant) {
    case 0: return launch<8, 2, 3>(slots, stride, cstride, L, S, nobj, rows, coeff, out_idx, flags, ticket, blocks, record, s);
    case 1: return launch<8, 3, 2>(slots, stride, cstride, L, S, nobj, rows, coeff, out_idx, flags, ticket, blocks, record, s);
    case 2: return launch<8, 4, 2>(slots, stride, cstride, L, S, nobj, rows, coeff, out_idx, flags, ticket, blocks, record, s);
    case 3: return launch<10, 1, 6>(slots, stride, cstride, L, S, nobj, rows, coeff, out_idx, flags, ticket, blocks, record, s);
    case 4: return launch<10, 2, 3>(slots, stride, cstride, L, S, nobj, rows, coeff, out_idx, flags, ticket, blocks, record, s);
    case 5: return launch<10, 3, 2>(slots, stride, cstride, L, S, nobj, rows, coeff, out_idx, flags, ticket, blocks, record, s);
    case 6: return launch<8, 1, 6>(slots, stride, cstride, L, S, nobj, rows, coeff, out_idx, flags, ticket, blocks, record, s);
    case 7: return launch<4, 2, 3>(slots, stride, cstride, L, S, nobj, rows, coeff, out_idx, flags, ticket, blocks, record, s);
    case 8: return launch<4, 4, 2>(slots, stride, cstride, L, S, nobj, rows, coeff, out_idx, flags, ticket, blocks, record, s);
    case 9: return launch<4, 3, 2>(slots, stride, cstride, L, S, nobj, rows, coeff, out_idx, flags, ticket, blocks, record, s);
    default: return -3;
  }
}

// Second pass after a switched first pass (record from bqv_encode): the redo
// list and the redo kernel, the latter on `blocks` blocks.  count: 1 word,
// zeroed here; list: nobj x units words.
template <int K, int U, int C>
int redo(uint8_t* slots, uint64_t stride, uint64_t cstride, uint64_t L, uint64_t S, uint32_t nobj, uint32_t rows,
         const uint32_t* coeff, const uint32_t* out_idx, const uint32_t* mapping, const uint32_t* status,
         const uint8_t* record, uint32_t* list, uint32_t* count, uint32_t blocks, hipStream_t s) {
  const uint32_t spread = queue_spread(nobj, L, U, C);
  if (!spread) return -2;
  const uint32_t nint = bytes::encode_interior_tiles(S, L, 0, L, K, U);
  const uint32_t units = apply::walk_units<C>(nint, spread);
  if (hipMemsetAsync(count, 0, 4, s) != hipSuccess) return -1;
  hipLaunchKernelGGL(bytes::redo_list_kernel<C>, dim3(1024), dim3(apply::kBlock), 0, s, record, mapping, status, nobj,
                     units, nint, list, count);
  hipLaunchKernelGGL((bytes::encode_bytes_redo_kernel<K, U, C>), dim3(blocks), dim3(apply::kBlock), 0, s, slots,
                     stride, L, cstride, (uint64_t)0, L, S, nobj, rows, coeff, out_idx, status, mapping, list, count,
                     units);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int bqv_redo(int variant, uint8_t* slots, uint64_t stride, uint64_t cstride, uint64_t L, uint64_t S,
                        uint32_t nobj, uint32_t rows, const uint32_t* coeff, const uint32_t* out_idx,
                        const uint32_t* mapping, const uint32_t* status, const uint8_t* record, uint32_t* list,
                        uint32_t* count, uint32_t blocks, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  switch (variant) {
    case 0: return redo<8, 2, 3>(slots, stride, cstride, L, S, nobj, rows, coeff, out_idx, mapping, status, record, list, count, blocks, s);
    case 3: return redo<10, 1, 6>(slots, stride, cstride, L, S, nobj, rows, coeff, out_idx, mapping, status, record, list, count, blocks, s);
    default: return -3;
  }
}

extern "C" int bqv_ticket_words() { return (int)apply::ticket_set_words(kQueueCounters); }
