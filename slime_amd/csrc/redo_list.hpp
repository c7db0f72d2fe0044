// The counter word of the matrix-core redo list (rs_bytes_mfma.hip,
// mfma_redo_list_kernel / encode_bytes_mfma_redo_kernel): its low 31 bits
// count the list's entries, drawn by atomicAdd as offsets into the list, and
// bit 31 (kSwitchedBit) is OR-ed in by any wave that saw a switched object,
// so the redo skips its edge pass when none did.  Offsets drawn after some
// wave set the bit carry it: every drawn value goes through redo_offset().
// That is exact only while the count stays below 2^31 -- redo_list_fits()
// is the host's guard before it hands a launch the switch scratch (a batch
// that does not fit re-encodes whole switched objects instead).  The same
// functions run on the CPU in tests/cpp/redo_list_test.cpp.  No other
// counter word in the kernels carries a flag bit (the walk tickets, the
// apply kernel's done counter and the VALU redo count are plain counts; the
// MapToGF flags are their own words).
#pragma once
#include <stdint.h>

#ifndef __HIP__
#ifndef __host__
#define __host__
#define __device__
#define __forceinline__ inline
#endif
#endif

namespace slime {
namespace bytes {

constexpr uint32_t kSwitchedBit = 0x80000000u;

// List offset of a value atomicAdd returned from the counter word.
__host__ __device__ __forceinline__ uint32_t redo_offset(uint32_t drawn) { return drawn & ~kSwitchedBit; }
// Entries listed, and whether any object switched, from the final word.
__host__ __device__ __forceinline__ uint32_t redo_count(uint32_t word) { return word & ~kSwitchedBit; }
__host__ __device__ __forceinline__ bool redo_switched(uint32_t word) { return (word & kSwitchedBit) != 0; }

// A batch of nobj objects x units interior tiles has at most nobj * units
// entries: below 2^31 the count never reaches the flag bit.
__host__ __device__ __forceinline__ bool redo_list_fits(uint64_t nobj, uint64_t units) {
  return nobj < (1ull << 32) && units < (1ull << 32) && nobj * units < (uint64_t)kSwitchedBit;
}

}  // namespace bytes
}  // namespace slime
