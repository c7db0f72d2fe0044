// Tuning harness: variants of the product apply kernel template
// (slime_amd/csrc/rs_apply_kernel.hpp) for A/B timing in one process.
// Built into tools/libapplyvar.so by `make applyvar`; tools only.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rs_apply_kernel.hpp"

using namespace slime::apply;

namespace {
template <int K, int U, bool NTL, bool NTS, bool ROT = false>
void go(const uint32_t* in, uint32_t* out, uint64_t io, uint64_t is, uint64_t oo, uint64_t os, const uint32_t* coeff,
        const uint32_t* ii, const uint32_t* oi, uint64_t ncols, uint32_t nobj, uint32_t rows, uint32_t gx, uint32_t gy,
        hipStream_t s, uint32_t nseg) {
  hipLaunchKernelGGL((rs_apply_kernel<K, true, U, NTL, NTS, ROT>), dim3(gx, gy), dim3(kBlock), 0, s, in, out, io, is, oo,
                     os, coeff, ii, oi, ncols, nobj, rows, (uint32_t)K, nseg);
}
template <int K, int U, bool NTL, bool NTS, int MODE = 0>
void gp(const uint32_t* in, uint32_t* out, uint64_t io, uint64_t is, uint64_t oo, uint64_t os, const uint32_t* coeff,
        const uint32_t* ii, const uint32_t* oi, uint64_t ncols, uint32_t nobj, uint32_t rows, uint32_t gx, uint32_t gy,
        hipStream_t s, uint32_t nseg) {
  hipLaunchKernelGGL((rs_apply_pipe_kernel<K, U, NTL, NTS, MODE>), dim3(gx, gy), dim3(kBlock), 0, s, in, out, io, is, oo, os,
                     coeff, ii, oi, ncols, nobj, rows, (uint32_t)K, nseg);
}
}  // namespace

extern "C" int av_launch(int variant, int k, const uint32_t* in, uint32_t* out, uint64_t io, uint64_t is,
                         uint64_t oo, uint64_t os, const uint32_t* coeff, const uint32_t* ii, const uint32_t* oi,
                         uint64_t ncols, uint32_t nobj, uint32_t rows, uint32_t gx, uint32_t gy, void* stream,
                         uint32_t nseg) {
  hipStream_t s = (hipStream_t)stream;
#define V2(id, U, NTL, NTS, ROT)                                                                            \
  case id:                                                                                                 \
    if (k == 8) go<8, U, NTL, NTS, ROT>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, gx, gy, s, nseg);     \
    else if (k == 10) go<10, U, NTL, NTS, ROT>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, gx, gy, s, nseg); \
    else if (k == 4) go<4, U, NTL, NTS, ROT>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, gx, gy, s, nseg);   \
    else if (k == 6) go<6, U, NTL, NTS, ROT>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, gx, gy, s, nseg);   \
    else if (k == 12) go<12, U, NTL, NTS, ROT>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, gx, gy, s, nseg); \
    else if (k == 16) go<16, U, NTL, NTS, ROT>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, gx, gy, s, nseg); \
    else if (k == 4) gp<4, U, true, true>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, gx, gy, s, nseg);   \
    else if (k == 6) gp<6, U, true, true>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, gx, gy, s, nseg);   \
    else if (k == 12) gp<12, U, true, true>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, gx, gy, s, nseg); \
    else if (k == 16) gp<16, U, true, true>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, gx, gy, s, nseg); \
    else return -2;                                                                                        \
    break;
#define V(id, U, NTL, NTS) V2(id, U, NTL, NTS, false)
#define P(id, U)                                                                                            \
  case id:                                                                                                 \
    if (k == 8) gp<8, U, true, true>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, gx, gy, s, nseg);     \
    else if (k == 10) gp<10, U, true, true>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, gx, gy, s, nseg); \
    else if (k == 4) gp<4, U, true, true>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, gx, gy, s, nseg);   \
    else if (k == 6) gp<6, U, true, true>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, gx, gy, s, nseg);   \
    else if (k == 12) gp<12, U, true, true>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, gx, gy, s, nseg); \
    else if (k == 16) gp<16, U, true, true>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, gx, gy, s, nseg); \
    else return -2;                                                                                        \
    break;
  switch (variant) {
    V(0, 1, true, false)
    V(1, 1, false, false)
    V(2, 1, true, true)
    V(3, 1, false, true)
    V(4, 2, true, false)
    V(5, 2, false, false)
    V(6, 2, true, true)
    V(7, 2, false, true)
    V(8, 4, true, true)
    V(9, 4, true, false)
    V(10, 3, true, true)
    V2(11, 4, true, true, true)
    V2(12, 2, true, true, true)
    P(13, 1)
    P(14, 2)
    P(15, 3)
    // XOR stand-in math (wrong results by design): how much does the field math cost?
    case 16:
      if (k == 8) gp<8, 3, true, true, 1>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, gx, gy, s, nseg);
      else if (k == 10) gp<10, 3, true, true, 1>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, gx, gy, s, nseg);
      else return -2;
      break;
    case 18:  // read-only probe (U3): the loads of the product walk, no stores
      if (k == 8) gp<8, 3, true, true, 2>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, gx, gy, s, nseg);
      else if (k == 10) gp<10, 3, true, true, 2>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, gx, gy, s, nseg);
      else return -2;
      break;
    case 19:  // write-only probe (U3): the stores of the product walk, no loads
      if (k == 8) gp<8, 3, true, true, 3>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, gx, gy, s, nseg);
      else if (k == 10) gp<10, 3, true, true, 3>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, gx, gy, s, nseg);
      else return -2;
      break;
    case 20:  // pipelined, 4 KiB per wave per stream per tile (AGPR-backed register sets)
      if (k == 8) gp<8, 4, true, true>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, gx, gy, s, nseg);
      else if (k == 10) gp<10, 4, true, true>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, gx, gy, s, nseg);
      else return -2;
      break;
    case 21:  // product math, XCD-grouped work order
      if (k == 8) gp<8, 3, true, true, 4>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, gx, gy, s, nseg);
      else if (k == 10) gp<10, 3, true, true, 4>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, gx, gy, s, nseg);
      else return -2;
      break;
    case 17:
      if (k == 8) gp<8, 2, true, true, 1>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, gx, gy, s, nseg);
      else if (k == 10) gp<10, 2, true, true, 1>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, gx, gy, s, nseg);
      else return -2;
      break;
    default:
      return -1;
  }
#undef V
#undef P
#undef V2
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
