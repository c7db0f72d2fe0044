// Host launch templates of the fused byte encode's mid-object mapping switch
// (kernels: rs_bytes_kernel.hpp encode_bytes_queue_kernel, redo_list_kernel,
// encode_bytes_redo_kernel), shared by rs_bytes.hip (need <= 16) and
// rs_bytes_k32.hip (17 <= need <= 24).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>

#include "kernels.hpp"
#include "rs_bytes_kernel.hpp"

namespace slime {
// Mid-object switch scratch (BytesLaunch::scratch): the redo count, the redo
// list (nobj x units words) and the per-unit mapping record (nobj x units
// bytes) of a phase 0 on the ticket walk with C-tile units of U vectors.
namespace bytes {
// With top bits (switch_bits_wanted): the planes of every object's interior
// tiles follow, 256 B-aligned (TopBits<K, U>::kTileBytes a tile).  Word 1 of
// the header stays zero: the edge-only redo reads it as its list count.
struct SwitchLayout {
  uint32_t spread = 0, nint = 0, units = 0;
  uint64_t bytes = 0;
  uint64_t bits_off = 0;  // 0: no top bits
  uint32_t* count(uint8_t* p) const { return reinterpret_cast<uint32_t*>(p); }
  uint32_t* zero(uint8_t* p) const { return reinterpret_cast<uint32_t*>(p) + 1; }
  uint32_t* list(uint8_t* p) const { return reinterpret_cast<uint32_t*>(p + 256); }
  uint8_t* record(uint8_t* p, uint32_t nobj) const { return p + 256 + 4ull * nobj * units; }
  uint8_t* bits(uint8_t* p) const { return bits_off ? p + bits_off : nullptr; }
};

// Objects of at least this many bytes take the top-bit correction under
// switch_bits_mode() 0.  A word of uniform bytes is >= p with probability
// 5/2^32, so 1 GiB objects switch 27% of the time and redo, on the bench
// data, 16-20% of the encode time; storing the bits costs the first pass
// K/8 bytes a column (+2.6% at 10/14), and the correction moves 4r + K/8
// bytes a redone column instead of 4(K + r): at 10/14 the second pass ran
// 0.235 against 0.389 ms on the same list, at 8/12 with 256 MiB objects (7.5%
// switch, redo 3.5%) the sum lost 1.2% (profiles/r06/s21_topbits/).
constexpr uint64_t kTopBitsMinObject = 1ull << 30;
template <int K>
bool switch_bits_wanted(const BytesLaunch& a) {
  if (K > kTopBitsMaxK) return false;
  const int mode = switch_bits_mode();
  return mode == 1 || (mode == 0 && a.S >= kTopBitsMinObject);
}

inline uint64_t bits_offset(uint32_t nobj, uint32_t units) { return (256 + 5ull * nobj * units + 255) & ~255ull; }

template <int K, int U, int C>
SwitchLayout switch_layout(const BytesLaunch& a, uint64_t ncols, hipStream_t s) {
  SwitchLayout l;
  if (!queue_allowed(s)) return l;
  l.spread = queue_spread(a.nobj, ncols, U, C);
  if (!l.spread) return l;
  l.nint = encode_interior_tiles(a.S, a.L, a.col0, ncols, K, U);
  l.units = apply::walk_units<C>(l.nint, l.spread);
  l.bytes = 256 + 5ull * a.nobj * l.units;
  if (switch_bits_wanted<K>(a) && l.nint) {
    l.bits_off = bits_offset(a.nobj, l.units);
    l.bytes = l.bits_off + (uint64_t)a.nobj * l.nint * TopBits<K, U>::kTileBytes;
  }
  return l;
}

// Grid of the first pass and of the redo: two blocks per CU for the need <=
// 16 forms, whose registers allow two waves per SIMD (at most 250 VGPRs, no
// AGPRs: -Rpass-analysis=kernel-resource-usage), when the batch has at least
// 64 units per wave at that grid; else one.  The second wave per SIMD covers
// the first's unit-start latency (flags read, ticket draw, list entry): 512
// blocks measured 1-4% faster than 256 for the first pass at C3 and C5 (341 /
// 136 units per wave) and 3-4% for the redo, but 3.5% slower at C2 (43 units
// per wave) (profiles/r03/s8_bqv/, s14_redob/, s17_bqv_c2/).  A compile-time
// rule rather than an occupancy query: the first launch may be inside a graph
// capture.
constexpr uint64_t kTwoBlockMinUnits = 64ull * 512 * apply::kWaves;
template <int K>
uint32_t switch_grid(uint64_t batch_units) {
  return K <= 16 && batch_units >= kTwoBlockMinUnits ? 512u : 256u;
}

// Phase 1 after a switched phase 0: build the redo list, then re-encode the
// listed units plus the edge tiles and column tails of the objects mapped
// with 1<<31.
template <int K, int U, int C>
hipError_t launch_redo(const BytesLaunch& a, uint64_t ncols, hipStream_t s) {
  if (!a.sw || !a.sw->switched || !a.sw->spread) return hipErrorInvalidValue;  // phase 0 did not switch
  SwitchLayout l;  // phase 0's layout, as it ran
  l.spread = a.sw->spread;
  l.nint = a.sw->nint;
  l.units = a.sw->units;
  uint32_t* count = l.count(a.scratch);
  // count and the zero word beside it
  if (hipError_t e = hipMemsetAsync(count, 0, 2 * sizeof(uint32_t), s)) return e;
  const uint64_t batch_units = (uint64_t)a.nobj * l.units;
  const uint64_t lblocks = std::min<uint64_t>(1024, (batch_units + apply::kBlock - 1) / apply::kBlock);
  hipLaunchKernelGGL(redo_list_kernel<C>, dim3((uint32_t)std::max<uint64_t>(lblocks, 1)), dim3(apply::kBlock), 0, s,
                     l.record(a.scratch, a.nobj), a.mapping, a.flags, a.nobj, l.units, l.nint, l.list(a.scratch),
                     count);
  if (hipError_t e = hipGetLastError()) return e;
  if constexpr (K <= kTopBitsMaxK) {
    if (a.sw->bits) {
      // The listed units corrected from phase 0's top bits; the redo kernel
      // then walks an empty list (the zero word) and rewrites only the edge
      // tiles and column tails of the objects mapped with 1<<31.
      hipLaunchKernelGGL((encode_bytes_fix_kernel<K, U, C>), dim3(switch_grid<K>(batch_units)), dim3(apply::kBlock), 0,
                         s, a.slots, a.slot_stride, chunk_stride(a), a.col0, a.rows, a.coeff, a.out_idx, a.mapping,
                         a.scratch + bits_offset(a.nobj, l.units), l.list(a.scratch), count, l.units, l.nint);
      if (hipError_t e = hipGetLastError()) return e;
      count = l.zero(a.scratch);
    }
  }
  hipLaunchKernelGGL((encode_bytes_redo_kernel<K, U, C>), dim3(switch_grid<K>(batch_units)), dim3(apply::kBlock),
                     0, s, a.slots, a.slot_stride, a.L, chunk_stride(a), a.col0, ncols, a.S, a.nobj, a.rows, a.coeff,
                     a.out_idx, a.flags, a.mapping, l.list(a.scratch), count, l.units);
  return hipGetLastError();
}

// Phase 0 on the ticket walk (the mid-object switch when a.scratch is given).
// *launched = false when the batch has too many units for 32-bit tickets or
// no counter set could be had (the caller takes the static kernel).
template <int K, int U, int C>
hipError_t launch_encode_queue(const BytesLaunch& a, uint64_t ncols, hipStream_t s, bool* launched) {
  *launched = false;
  SwitchLayout l = switch_layout<K, U, C>(a, ncols, s);
  if (!l.spread) return hipSuccess;
  // The caller sized the scratch by encode_switch_bytes; the top-bit choice
  // reads process-wide state (switch_bits_mode) that may have changed since,
  // so the layout is checked against the bytes actually held: without room
  // for the bits the switch runs without them, without room for the record
  // the second pass re-encodes whole objects.
  if (a.scratch && l.bytes > a.scratch_bytes && l.bits_off) {
    l.bytes = 256 + 5ull * a.nobj * l.units;
    l.bits_off = 0;
  }
  const bool fits = a.scratch && l.bytes <= a.scratch_bytes;
  uint8_t* record = fits ? l.record(a.scratch, a.nobj) : nullptr;
  uint8_t* bits = fits ? l.bits(a.scratch) : nullptr;
  const dim3 grid((uint32_t)queue_blocks(switch_grid<K>((uint64_t)a.nobj * l.units), (uint64_t)a.nobj * l.units));
  const hipError_t e = with_tickets(
      s,
      [&](uint32_t* set) {
        if constexpr (K <= kTopBitsMaxK) {
          if (bits) {
            hipLaunchKernelGGL((encode_bytes_queue_bits_kernel<K, U, C, kQueueCounters>), grid, dim3(apply::kBlock), 0,
                               s, a.slots, a.slot_stride, a.L, chunk_stride(a), a.col0, ncols, a.S, a.nobj, a.rows,
                               a.coeff, a.out_idx, a.flags, set, l.spread, record, l.units, bits);
            return hipGetLastError();
          }
        }
        hipLaunchKernelGGL((encode_bytes_queue_kernel<K, U, C, kQueueCounters>), grid, dim3(apply::kBlock), 0, s,
                           a.slots, a.slot_stride, a.L, chunk_stride(a), a.col0, ncols, a.S, a.nobj, a.rows, a.coeff,
                           a.out_idx, a.flags, set, l.spread, record, l.units);
        return hipGetLastError();
      },
      launched);
  if (*launched && record && a.sw) {
    a.sw->switched = true;
    a.sw->bits = bits != nullptr;
    a.sw->spread = l.spread;
    a.sw->nint = l.nint;
    a.sw->units = l.units;
  }
  return e;
}
}  // namespace bytes

}  // namespace slime
