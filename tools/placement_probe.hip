// Placement-mode probe (tools only): the apply kernel's exact stripe walk
// (objects on blockIdx.y, 4-KiB-per-stripe tiles per wave, nt loads/stores)
// with the field math replaced by XOR, for any mix of NR read stripes and NW
// write stripes per object.  Timing the mixes on a fast-mode and a slow-mode
// buffer tells which traffic the slow mode slows down.
// Built into tools/libplaceprobe.so by `make placeprobe`.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {
constexpr int B = 256, W = B / 64, U = 4;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int NR, int NW>
__global__ __launch_bounds__(B) void stripes(uint32_t* __restrict__ base, uint64_t obj_stride, uint64_t shard,
                                             uint64_t ncols, uint32_t nobj, uint32_t rd0, uint32_t wr0,
                                             uint32_t* __restrict__ sink) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * W + (threadIdx.x >> 6);
  const uint64_t nwaves = (uint64_t)gridDim.x * W;
  const uint64_t nvec = ncols >> 2, ntiles = (nvec + 64 * U - 1) / (64 * U);
  u32x4 acc = {0, 0, 0, 0};
  for (uint32_t obj = blockIdx.y; obj < nobj; obj += gridDim.y) {
    uint32_t* const ob = base + (uint64_t)obj * obj_stride;
    for (uint64_t t = wave; t < ntiles; t += nwaves) {
      const uint64_t g0 = t * (64 * U) + lane;
      u32x4 x[U];
#pragma unroll
      for (int u = 0; u < U; ++u) x[u] = u32x4{(uint32_t)t, lane, 1u, 2u};
#pragma unroll
      for (int j = 0; j < NR; ++j)
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (g0 + 64 * u < nvec)
            x[u] ^= __builtin_nontemporal_load(
                reinterpret_cast<const u32x4*>(ob + (uint64_t)(rd0 + j) * shard + ((g0 + 64 * u) << 2)));
#pragma unroll
      for (int i = 0; i < NW; ++i)
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (g0 + 64 * u < nvec)
            __builtin_nontemporal_store(x[u] + (uint32_t)i,
                                        reinterpret_cast<u32x4*>(ob + (uint64_t)(wr0 + i) * shard + ((g0 + 64 * u) << 2)));
      if constexpr (NW == 0) {
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= x[u];
      }
    }
  }
  if constexpr (NW == 0) sink[(uint64_t)blockIdx.y * gridDim.x * B + (uint64_t)blockIdx.x * B + threadIdx.x] =
      acc.x ^ acc.y ^ acc.z ^ acc.w;
}
}  // namespace

// mix: 0 = read 12, 1 = read 8, 2 = write 4, 3 = read 8 + write 4 (the encode's
// traffic), 4 = read 4, 5 = write 12.  Returns 0, or -1 for an unknown mix.
extern "C" int pp_launch(int mix, uint32_t* base, uint64_t obj_stride, uint64_t shard, uint64_t ncols, uint32_t nobj,
                         uint32_t gx, uint32_t gy, uint32_t* sink, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const dim3 g(gx, gy), b(B);
  switch (mix) {
    case 0: hipLaunchKernelGGL((stripes<12, 0>), g, b, 0, s, base, obj_stride, shard, ncols, nobj, 0u, 0u, sink); break;
    case 1: hipLaunchKernelGGL((stripes<8, 0>), g, b, 0, s, base, obj_stride, shard, ncols, nobj, 0u, 0u, sink); break;
    case 2: hipLaunchKernelGGL((stripes<0, 4>), g, b, 0, s, base, obj_stride, shard, ncols, nobj, 0u, 8u, sink); break;
    case 3: hipLaunchKernelGGL((stripes<8, 4>), g, b, 0, s, base, obj_stride, shard, ncols, nobj, 0u, 8u, sink); break;
    case 4: hipLaunchKernelGGL((stripes<4, 0>), g, b, 0, s, base, obj_stride, shard, ncols, nobj, 8u, 0u, sink); break;
    case 5: hipLaunchKernelGGL((stripes<0, 12>), g, b, 0, s, base, obj_stride, shard, ncols, nobj, 0u, 0u, sink); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
