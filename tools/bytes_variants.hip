// Tuning harness for the fused byte-domain kernels (rs_bytes_kernel.hpp):
// K = 8 variants of the speculative encode pass.  Tools only: make bytesvar.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rs_bytes_kernel.hpp"

using namespace slime::bytes;
using slime::apply::kBlock;

namespace {
template <int U, bool FAST, bool FLAGS>
void enc(uint8_t* slots, uint64_t stride, uint64_t L, uint64_t S, uint32_t nobj, uint32_t rows, const uint32_t* coeff,
         const uint32_t* oi, uint32_t* flags, const uint32_t* mapping, uint32_t gx, uint32_t gy, hipStream_t s) {
  hipLaunchKernelGGL((encode_bytes_kernel<8, U, 0, FAST, FLAGS>), dim3(gx, gy), dim3(kBlock), 0, s, slots, stride, L,
                     4 * L, (uint64_t)0, L, S, nobj, rows, coeff, oi, flags, mapping, 1u);
}
}  // namespace

extern "C" int bv_encode(int v, uint8_t* slots, uint64_t stride, uint64_t L, uint64_t S, uint32_t nobj,
                         uint32_t rows, const uint32_t* coeff, const uint32_t* oi, uint32_t* flags,
                         const uint32_t* mapping, uint32_t gx, uint32_t gy, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  switch (v) {
    case 0: enc<4, true, true>(slots, stride, L, S, nobj, rows, coeff, oi, flags, mapping, gx, gy, s); break;
    case 1: enc<4, true, false>(slots, stride, L, S, nobj, rows, coeff, oi, flags, mapping, gx, gy, s); break;
    case 2: enc<4, false, true>(slots, stride, L, S, nobj, rows, coeff, oi, flags, mapping, gx, gy, s); break;
    case 3: enc<2, true, true>(slots, stride, L, S, nobj, rows, coeff, oi, flags, mapping, gx, gy, s); break;
    case 4: enc<1, true, true>(slots, stride, L, S, nobj, rows, coeff, oi, flags, mapping, gx, gy, s); break;
    case 5: enc<2, true, false>(slots, stride, L, S, nobj, rows, coeff, oi, flags, mapping, gx, gy, s); break;
    case 6: enc<1, true, false>(slots, stride, L, S, nobj, rows, coeff, oi, flags, mapping, gx, gy, s); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
