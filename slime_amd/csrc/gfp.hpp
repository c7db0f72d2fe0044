// GF(p), p = 2^32 - 5: the field of slime's internal/rs (internal/rs/doc.go:1-2,
// internal/rs/gf/map.go:7). Device arithmetic for CDNA4 (gfx950) plus the
// host-side scalar helpers the matrix code uses.
//
// Data-path identity (the reference's own TODO, internal/rs/vector.go:91-92):
//   2^32 = 5 (mod p),  2^64 = 25 (mod p).
// A dot product sum_j c_j * x_j is accumulated EXACTLY as a 96-bit integer
// (64-bit running sum `lo` + a 32-bit wrap counter `hi`), then folded once.
// Modular arithmetic is exact, so the result equals the reference's
// per-term `((x*c)%p + o)%p` (vector.go:97) bit for bit, for any uint32
// inputs (including non-canonical x >= p, which the reference also accepts).
#pragma once
#include <stdint.h>

#include "gfp_host.hpp"

namespace slime {

#if defined(__HIP_DEVICE_COMPILE__)
// lo += x * c, hi += carry-out.  One v_mad_u64_u32 (whose carry-out lands in
// an SGPR pair) and one v_addc_co_u32 that adds that carry to the counter.
// Plain C++ makes hipcc emit mad + 64-bit add + v_cmp_lt_u64 + cndmask
// (4 VALU ops); this is 2.  `c` is wave-uniform (a code coefficient), so it
// rides in an SGPR operand.  Non-volatile asm: the compiler may schedule it.
__device__ __forceinline__ void mac(uint64_t& lo, uint32_t& hi, uint32_t x, uint32_t c) {
  uint64_t carry;
  asm("v_mad_u64_u32 %0, %2, %3, %4, %0\n\t"
      "v_addc_co_u32_e64 %1, %2, %1, 0, %2"
      : "+v"(lo), "+v"(hi), "=&s"(carry)
      : "v"(x), "s"(c));
}

// Four independent columns against one coefficient in ONE asm statement:
// four mads (carry-outs into four SGPR pairs) then four addcs.  hipcc pads one
// wait state after every `;;#ASMEND` before a VALU that touches the outputs
// (cdna_hip_programming.md §5.7 item 2), so batching four MACs per statement
// amortises that pad, and the mad->addc distance of 4 instructions hides the
// mad's latency within the wave.  VALU carry-out -> VALU carry-in needs no
// manual wait state (the same pairing hipcc emits unpadded for 64-bit adds).
__device__ __forceinline__ void mac4(uint64_t& l0, uint64_t& l1, uint64_t& l2, uint64_t& l3, uint32_t& h0,
                                     uint32_t& h1, uint32_t& h2, uint32_t& h3, uint32_t x0, uint32_t x1,
                                     uint32_t x2, uint32_t x3, uint32_t c) {
  uint64_t c0, c1, c2, c3;
  asm("v_mad_u64_u32 %0, %8, %12, %16, %0\n\t"
      "v_mad_u64_u32 %1, %9, %13, %16, %1\n\t"
      "v_mad_u64_u32 %2, %10, %14, %16, %2\n\t"
      "v_mad_u64_u32 %3, %11, %15, %16, %3\n\t"
      "v_addc_co_u32_e64 %4, %8, %4, 0, %8\n\t"
      "v_addc_co_u32_e64 %5, %9, %5, 0, %9\n\t"
      "v_addc_co_u32_e64 %6, %10, %6, 0, %10\n\t"
      "v_addc_co_u32_e64 %7, %11, %7, 0, %11"
      : "+v"(l0), "+v"(l1), "+v"(l2), "+v"(l3), "+v"(h0), "+v"(h1), "+v"(h2), "+v"(h3), "=&s"(c0), "=&s"(c1),
        "=&s"(c2), "=&s"(c3)
      : "v"(x0), "v"(x1), "v"(x2), "v"(x3), "s"(c));
}
#else
// Host compilation pass of a .hip file parses device functions but never
// emits or runs them; these declarations only keep that pass well-formed.
__device__ void mac(uint64_t& lo, uint32_t& hi, uint32_t x, uint32_t c);
__device__ void mac4(uint64_t&, uint64_t&, uint64_t&, uint64_t&, uint32_t&, uint32_t&, uint32_t&, uint32_t&,
                     uint32_t, uint32_t, uint32_t, uint32_t, uint32_t);
#endif

// Fold V = hi*2^64 + lo (hi small: at most one wrap per term) to [0, p).
//   V = 25*hi + 5*m + l        (m:l = lo)          < 6*2^32 + 25*hi
//     = 5*th + tl              (th:tl = t)         < 2^32 + 30 + ...
//     = ul + 5*uh              (uh <= 1; if uh==1 then ul < 40)
// then one conditional subtract of p gives the canonical residue.
__host__ __device__ __forceinline__ uint32_t fold96(uint64_t lo, uint32_t hi) {
  const uint32_t l = (uint32_t)lo, m = (uint32_t)(lo >> 32);
  const uint64_t t = (uint64_t)m * 5u + (uint64_t)l + (uint64_t)hi * 25u;
  const uint64_t u = (t >> 32) * 5u + (uint32_t)t;
  const uint32_t w = (uint32_t)u + (uint32_t)(u >> 32) * 5u;
  return w >= kP ? w - kP : w;
}

// Canonical residue of a single (possibly non-canonical) symbol: x mod p.
__host__ __device__ __forceinline__ uint32_t canon(uint32_t x) { return x >= kP ? x - kP : x; }

}  // namespace slime
