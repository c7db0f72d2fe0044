// A/B harness (tools only) of the fused byte encode's second pass at need <=
// 10 on the ticket walk: the product kernels (rs_bytes_kernel.hpp) launched
// as rs_bytes_launch.hpp launches them, with the first pass storing no top
// bits (then the re-encode of the listed units), or storing them per tile
// (TopBits, layout 1) for encode_bytes_fix_kernel.  tools/topbits_fix.py
// drives it and checks every variant's chunks against the re-encode's.  (A
// per-unit layout, commit 34ad9c0, measured the same and was removed.)
#include <hip/hip_runtime.h>

#include "rs_bytes_launch.hpp"

using namespace slime;
using namespace slime::bytes;

namespace {

struct Geo {
  uint32_t spread, nint, units;
};

template <int K, int U, int C>
Geo geo(uint64_t S, uint64_t L, uint32_t nobj) {
  Geo g;
  g.spread = queue_spread(nobj, L, U, C);
  g.nint = encode_interior_tiles(S, L, 0, L, K, U);
  g.units = apply::walk_units<C>(g.nint, g.spread);
  return g;
}

template <int K, int U, int C>
int pass0(int layout, uint8_t* slots, uint64_t stride, uint64_t cstride, uint64_t L, uint64_t S, uint32_t nobj,
          uint32_t rows, const uint32_t* coeff, const uint32_t* out_idx, uint32_t* flags, uint32_t* ticket,
          uint32_t blocks, uint8_t* record, uint8_t* bits, hipStream_t s) {
  const Geo g = geo<K, U, C>(S, L, nobj);
  if (!g.spread) return -2;
  const dim3 grid(blocks), block(apply::kBlock);
  if (layout == 0)
    hipLaunchKernelGGL((encode_bytes_queue_kernel<K, U, C, kQueueCounters>), grid, block, 0, s, slots, stride, L,
                       cstride, (uint64_t)0, L, S, nobj, rows, coeff, out_idx, flags, ticket, g.spread, record, g.units);
  else
    hipLaunchKernelGGL((encode_bytes_queue_bits_kernel<K, U, C, kQueueCounters>), grid, block, 0, s, slots, stride, L,
                       cstride, (uint64_t)0, L, S, nobj, rows, coeff, out_idx, flags, ticket, g.spread, record, g.units,
                       bits);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// count: 2 words (the list count, then a zero word for the edge-only redo).
template <int K, int U, int C>
int second(int layout, uint8_t* slots, uint64_t stride, uint64_t cstride, uint64_t L, uint64_t S, uint32_t nobj,
           uint32_t rows, const uint32_t* coeff, const uint32_t* out_idx, const uint32_t* mapping,
           const uint32_t* status, const uint8_t* record, const uint8_t* bits, uint32_t* list, uint32_t* count,
           uint32_t blocks, hipStream_t s) {
  const Geo g = geo<K, U, C>(S, L, nobj);
  if (!g.spread) return -2;
  if (hipMemsetAsync(count, 0, 8, s) != hipSuccess) return -1;
  hipLaunchKernelGGL(redo_list_kernel<C>, dim3(1024), dim3(apply::kBlock), 0, s, record, mapping, status, nobj, g.units,
                     g.nint, list, count);
  const uint32_t* n = count;
  if (layout) {
    hipLaunchKernelGGL((encode_bytes_fix_kernel<K, U, C>), dim3(blocks), dim3(apply::kBlock), 0, s, slots, stride,
                       cstride, (uint64_t)0, rows, coeff, out_idx, mapping, bits, list, count, g.units, g.nint);
    n = count + 1;
  }
  hipLaunchKernelGGL((encode_bytes_redo_kernel<K, U, C>), dim3(blocks), dim3(apply::kBlock), 0, s, slots, stride, L,
                     cstride, (uint64_t)0, L, S, nobj, rows, coeff, out_idx, status, mapping, list, n, g.units);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
}  // namespace

// shape 0: K = 8 (U 2, C 3, the product's C3 form); 1: K = 10 (U 1, C 6, C5's)
extern "C" int tbf_pass0(int shape, int layout, uint8_t* slots, uint64_t stride, uint64_t cstride, uint64_t L,
                         uint64_t S, uint32_t nobj, uint32_t rows, const uint32_t* coeff, const uint32_t* out_idx,
                         uint32_t* flags, uint32_t* ticket, uint32_t blocks, uint8_t* record, uint8_t* bits,
                         void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (shape == 0) return pass0<8, 2, 3>(layout, slots, stride, cstride, L, S, nobj, rows, coeff, out_idx, flags, ticket, blocks, record, bits, s);
  if (shape == 1) return pass0<10, 1, 6>(layout, slots, stride, cstride, L, S, nobj, rows, coeff, out_idx, flags, ticket, blocks, record, bits, s);
  return -3;
}

extern "C" int tbf_second(int shape, int layout, uint8_t* slots, uint64_t stride, uint64_t cstride, uint64_t L,
                          uint64_t S, uint32_t nobj, uint32_t rows, const uint32_t* coeff, const uint32_t* out_idx,
                          const uint32_t* mapping, const uint32_t* status, const uint8_t* record, const uint8_t* bits,
                          uint32_t* list, uint32_t* count, uint32_t blocks, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (shape == 0) return second<8, 2, 3>(layout, slots, stride, cstride, L, S, nobj, rows, coeff, out_idx, mapping, status, record, bits, list, count, blocks, s);
  if (shape == 1) return second<10, 1, 6>(layout, slots, stride, cstride, L, S, nobj, rows, coeff, out_idx, mapping, status, record, bits, list, count, blocks, s);
  return -3;
}

// Bytes of the top-bit buffer and units per object.
extern "C" uint64_t tbf_bits_bytes(int shape, uint64_t S, uint64_t L, uint32_t nobj) {
  if (shape == 0) return (uint64_t)nobj * geo<8, 2, 3>(S, L, nobj).nint * TopBits<8, 2>::kTileBytes;
  if (shape == 1) return (uint64_t)nobj * geo<10, 1, 6>(S, L, nobj).nint * TopBits<10, 1>::kTileBytes;
  return 0;
}
extern "C" uint32_t tbf_units(int shape, uint64_t S, uint64_t L, uint32_t nobj) {
  if (shape == 0) return geo<8, 2, 3>(S, L, nobj).units;
  if (shape == 1) return geo<10, 1, 6>(S, L, nobj).units;
  return 0;
}
extern "C" int tbf_ticket_words() { return (int)apply::ticket_set_words(kQueueCounters); }
