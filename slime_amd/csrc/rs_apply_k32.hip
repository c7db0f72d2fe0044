// 17 <= k <= 32: the software-pipelined k-template apply kernel
// (rs_apply_pipe_kernel, rs_apply_kernel.hpp) instantiated for wide codes, in
// its own translation unit so the product build compiles it in parallel.
//
// For these k the wide kernel's 16-shard chunk stream (rs_apply_wide_pipe_kernel)
// is bound by its item stream, not by the field math: its XOR stand-in runs
// 20/24 at the same speed (profiles/r02/s16_widemath/).  Holding all k input
// vectors of a tile in registers (two sets, AGPR-backed where needed) and
// reading each coefficient row as ceil(k/16) s_load_dwordx16 runs, in-process
// against the wide kernel (profiles/r02/s18_pipek/, HBM GB/s, best geometry
// of each): 20/24 encode 5117 vs 4829, decode 5403 vs 4986; 24/28 4925 vs
// 4754; 32/40 5639 vs 5287.  U = 2 (2 KiB per shard per tile) up to k = 24,
// U = 1 above (register budget); 256 blocks.
#include <hip/hip_runtime.h>

#include "kernels.hpp"
#include "rs_apply_kernel.hpp"

namespace slime {
namespace {

// Dynamic schedule (rs_apply_queue_kernel, as for k <= 16 in rs_apply.hip):
// a unit is C = 6 / U tiles.
template <int K>
hipError_t launch_k32_queue(const ApplyLaunch& a, hipStream_t stream, bool* launched) {
  constexpr int U = K <= 24 ? 2 : 1;
  constexpr int C = 6 / U;
  *launched = false;
  const uint32_t spread = queue_spread(a.nobj, a.ncols, U, C, (uint32_t)(a.k + a.rows));
  if (!spread) return hipSuccess;
  const uint64_t blocks = queue_blocks(256, queue_units(a.nobj, a.ncols, U, C, spread));
  return with_tickets(
      stream,
      [&](uint32_t* set) {
        hipLaunchKernelGGL((apply::rs_apply_queue_kernel<K, U, C, kQueueCounters, true, true>),
                           dim3((uint32_t)blocks), dim3(apply::kBlock), 0, stream, a.in, a.out, a.in_obj_stride,
                           a.in_shard_stride, a.out_obj_stride, a.out_shard_stride, a.coeff, a.in_idx, a.out_idx,
                           a.ncols, a.nobj, a.rows, a.k, set, nullptr, spread);
        return hipGetLastError();
      },
      launched);
}

template <int K>
hipError_t launch_k32(const ApplyLaunch& a, hipStream_t stream) {
  if (queue_allowed(stream)) {
    bool launched = false;
    const hipError_t e = launch_k32_queue<K>(a, stream, &launched);
    if (launched || e != hipSuccess) return e;
  }
  constexpr int U = K <= 24 ? 2 : 1;
  constexpr uint64_t kBlocks = 256;
  const uint64_t per_block = 4ull * apply::kBlock * U;
  const uint32_t nseg = object_segments(a.nobj, a.ncols);
  const uint64_t nwork = (uint64_t)a.nobj * nseg;
  const uint64_t gy = nwork < 65535 ? nwork : 65535;
  uint64_t gx = (kBlocks + gy - 1) / gy;
  const uint64_t need = (a.ncols / nseg + per_block - 1) / per_block;
  if (gx > need) gx = need;
  if (gx < 1) gx = 1;
  hipLaunchKernelGGL((apply::rs_apply_pipe_kernel<K, U, true, true>), dim3((uint32_t)gx, (uint32_t)gy),
                     dim3(apply::kBlock), 0, stream, a.in, a.out, a.in_obj_stride, a.in_shard_stride,
                     a.out_obj_stride, a.out_shard_stride, a.coeff, a.in_idx, a.out_idx, a.ncols, a.nobj, a.rows,
                     a.k, nseg);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_pipe_k32(const ApplyLaunch& a, hipStream_t s) {
  switch (a.k) {
    case 17: return launch_k32<17>(a, s);
    case 18: return launch_k32<18>(a, s);
    case 19: return launch_k32<19>(a, s);
    case 20: return launch_k32<20>(a, s);
    case 21: return launch_k32<21>(a, s);
    case 22: return launch_k32<22>(a, s);
    case 23: return launch_k32<23>(a, s);
    case 24: return launch_k32<24>(a, s);
    case 25: return launch_k32<25>(a, s);
    case 26: return launch_k32<26>(a, s);
    case 27: return launch_k32<27>(a, s);
    case 28: return launch_k32<28>(a, s);
    case 29: return launch_k32<29>(a, s);
    case 30: return launch_k32<30>(a, s);
    case 31: return launch_k32<31>(a, s);
    case 32: return launch_k32<32>(a, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace slime
