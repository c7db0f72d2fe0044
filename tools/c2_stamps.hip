// Stamped twin of the product's dynamic-schedule apply launch (rs_apply.hip
// launch_queue): the same kernel template, geometry, spread and block count,
// instantiated with STAMP = 2 (rs_apply_kernel.hpp), so each wave records
// {start, first loads issued, tiles 4 / 16 / 64 entered, last stores issued,
// stores retired, exit counted, XCD | tiles | last-out}.  tools/c2_stamps.py splits a launch's
// fixed cost with it.  Tools only.
#include <hip/hip_runtime.h>

#include "kernels.hpp"
#include "rs_apply_kernel.hpp"

using namespace slime;
using namespace slime::apply;

namespace {
template <int K, int U, int C>
int launch(const uint32_t* in, uint32_t* out, uint64_t io, uint64_t is, uint64_t oo, uint64_t os,
           const uint32_t* coeff, const uint32_t* ii, const uint32_t* oi, uint64_t ncols, uint32_t nobj, uint32_t rows,
           hipStream_t s, uint32_t* ticket, uint64_t* stamps, uint32_t* nwaves, uint32_t spread_override,
           uint32_t blocks_override) {
  const uint32_t spread = spread_override ? spread_override : queue_spread(nobj, ncols, U, C, K + rows);
  if (!spread) return -2;
  const uint64_t blocks = blocks_override ? blocks_override : queue_blocks(256, queue_units(nobj, ncols, U, C, spread));
  *nwaves = (uint32_t)blocks * kWaves;
  if (!stamps) return 0;  // the caller sizes the stamp buffer first
  hipLaunchKernelGGL((rs_apply_queue_kernel<K, U, C, kQueueCounters, true, true, 1, 2>), dim3((uint32_t)blocks),
                     dim3(kBlock), 0, s, in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, (uint32_t)K, ticket,
                     stamps, spread);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
}  // namespace

// k = 3 (slime's default 3/5: U 4, C 3), 4 (C2: U 4, C 3), 8 (C3: U 3, C 2), 10 (C5: U 3, C 2),
// 12 (U 3, C 2) or 16 (U 1, C 6): the product's queue geometry (rs_apply.hip queue_unroll /
// queue_unit_tiles).
// ticket: a zeroed counter set of kQueueCounters + 1 lines of 64 words (each
// launch leaves it zero).  stamps: 9 words per wave, or null to get the wave
// count only (*nwaves).  spread / blocks: 0 = the product's rule, else that
// many segments per object / blocks (A/B of the geometry).
extern "C" int cs_launch(int k, const uint32_t* in, uint32_t* out, uint64_t io, uint64_t is, uint64_t oo, uint64_t os,
                         const uint32_t* coeff, const uint32_t* ii, const uint32_t* oi, uint64_t ncols, uint32_t nobj,
                         uint32_t rows, void* stream, void* ticket, void* stamps, uint32_t* nwaves, uint32_t spread,
                         uint32_t blocks) {
  hipStream_t s = (hipStream_t)stream;
  if (k == 3)
    return launch<3, 4, 3>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, s, (uint32_t*)ticket,
                           (uint64_t*)stamps, nwaves, spread, blocks);
  if (k == 4)
    return launch<4, 4, 3>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, s, (uint32_t*)ticket,
                           (uint64_t*)stamps, nwaves, spread, blocks);
  // 8/12 and 10/14 unit variants: 1308 U 3 C 3, 1408 U 3 C 4, 1508 U 2 C 3, 1310 U 3 C 3
  if (k == 1308)
    return launch<8, 3, 3>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, s, (uint32_t*)ticket,
                           (uint64_t*)stamps, nwaves, spread, blocks);
  if (k == 1408)
    return launch<8, 3, 4>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, s, (uint32_t*)ticket,
                           (uint64_t*)stamps, nwaves, spread, blocks);
  if (k == 1508)
    return launch<8, 2, 3>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, s, (uint32_t*)ticket,
                           (uint64_t*)stamps, nwaves, spread, blocks);
  if (k == 1310)
    return launch<10, 3, 3>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, s, (uint32_t*)ticket,
                            (uint64_t*)stamps, nwaves, spread, blocks);
  // the round-6 s30 product form, units of two tiles: 1104 (4/6), 1203 (3/5)
  if (k == 1104)
    return launch<4, 4, 2>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, s, (uint32_t*)ticket,
                           (uint64_t*)stamps, nwaves, spread, blocks);
  if (k == 1203)
    return launch<3, 4, 2>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, s, (uint32_t*)ticket,
                           (uint64_t*)stamps, nwaves, spread, blocks);
  // 4/6 unroll / unit variants (k code 100 * variant + 4): U 2 C 3, U 3 C 2, U 1 C 6, U 6 C 1, U 4 C 1, U 4 C 3,
  // U 4 C 4, U 4 C 6; 3/5: 903 U 4 C 3, 1003 U 4 C 4
  if (k == 104)
    return launch<4, 2, 3>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, s, (uint32_t*)ticket,
                           (uint64_t*)stamps, nwaves, spread, blocks);
  if (k == 204)
    return launch<4, 3, 2>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, s, (uint32_t*)ticket,
                           (uint64_t*)stamps, nwaves, spread, blocks);
  if (k == 304)
    return launch<4, 1, 6>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, s, (uint32_t*)ticket,
                           (uint64_t*)stamps, nwaves, spread, blocks);
  if (k == 404)
    return launch<4, 6, 1>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, s, (uint32_t*)ticket,
                           (uint64_t*)stamps, nwaves, spread, blocks);
  if (k == 504)
    return launch<4, 4, 1>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, s, (uint32_t*)ticket,
                           (uint64_t*)stamps, nwaves, spread, blocks);
  if (k == 604)
    return launch<4, 4, 3>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, s, (uint32_t*)ticket,
                           (uint64_t*)stamps, nwaves, spread, blocks);
  if (k == 704)
    return launch<4, 4, 4>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, s, (uint32_t*)ticket,
                           (uint64_t*)stamps, nwaves, spread, blocks);
  if (k == 804)
    return launch<4, 4, 6>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, s, (uint32_t*)ticket,
                           (uint64_t*)stamps, nwaves, spread, blocks);
  if (k == 903)  // 3/5 (slime's default) with units of 3 tiles
    return launch<3, 4, 3>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, s, (uint32_t*)ticket,
                           (uint64_t*)stamps, nwaves, spread, blocks);
  if (k == 1003)
    return launch<3, 4, 4>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, s, (uint32_t*)ticket,
                           (uint64_t*)stamps, nwaves, spread, blocks);
  if (k == 12)
    return launch<12, 3, 2>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, s, (uint32_t*)ticket,
                            (uint64_t*)stamps, nwaves, spread, blocks);
  if (k == 16)
    return launch<16, 1, 6>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, s, (uint32_t*)ticket,
                            (uint64_t*)stamps, nwaves, spread, blocks);
  if (k == 10)
    return launch<10, 3, 2>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, s, (uint32_t*)ticket,
                            (uint64_t*)stamps, nwaves, spread, blocks);
  if (k == 8)
    return launch<8, 3, 2>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, s, (uint32_t*)ticket,
                           (uint64_t*)stamps, nwaves, spread, blocks);
  return -1;
}
