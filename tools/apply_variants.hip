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
// ---- time-phased walk (read/write turnaround experiment, round 2) ----------
// Every wave of the chip reads only inside the first `rwin` ticks of each
// `period` ticks of the 100 MHz s_memrealtime clock and writes only after
// them, so the DRAM sees chip-wide read bursts and write bursts instead of a
// 2:1 mix at every instant.  Per period a wave loads T tiles of U KiB per
// shard (T register sets), computes all R output rows into registers, waits
// for the write window and stores them.  R = 4 rows (C3 encode / C4 decode).
__device__ __forceinline__ void wait_phase(uint32_t period, uint32_t lo, uint32_t hi) {
  for (;;) {
    const uint32_t t = (uint32_t)__builtin_amdgcn_s_memrealtime() % period;
    if (t >= lo && t < hi) return;
    __builtin_amdgcn_s_sleep(2);
  }
}

template <int K, int U, int R>
__global__ __launch_bounds__(kBlock) void phased_kernel(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                        uint64_t in_obj_stride, uint64_t in_shard,
                                                        uint64_t out_obj_stride, uint64_t out_shard,
                                                        const uint32_t* __restrict__ coeff,
                                                        const uint32_t* __restrict__ in_idx,
                                                        const uint32_t* __restrict__ out_idx, uint64_t ncols,
                                                        uint32_t nobj, uint32_t nseg, uint32_t period, uint32_t rwin) {
  const uint32_t nvec = (uint32_t)(ncols >> 2);
  const uint32_t seg_vec = segment_vectors(nvec, nseg);
  const uint64_t nwork = (uint64_t)nobj * nseg;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = blockIdx.x * kWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nwaves = gridDim.x * kWaves;
  for (uint64_t wi = blockIdx.y; wi < nwork; wi += gridDim.y) {
    const uint64_t obj = wi / nseg;
    const uint32_t seg = (uint32_t)(wi % nseg);
    const uint32_t* __restrict__ ib = in + obj * in_obj_stride;
    uint32_t* __restrict__ ob = out + obj * out_obj_stride;
    const uint32_t* sb[K];
#pragma unroll
    for (int j = 0; j < K; ++j) sb[j] = ib + (uint64_t)in_idx[j] * in_shard;
    const uint32_t v0 = seg * seg_vec < nvec ? seg * seg_vec : nvec;
    const uint32_t v1 = nvec - v0 > seg_vec ? v0 + seg_vec : nvec;
    const uint32_t ntiles = (v1 - v0 + 64 * U - 1) / (64 * U);
    for (uint32_t step = wave; step < ntiles; step += nwaves) {
      const uint32_t g0 = v0 + step * (64 * U) + lane;
      uint4 x[U][K];
      wait_phase(period, 0, rwin);
      load_tile<K, U, true>(x, sb, g0, v1);
      uint4 y[R][U];
#pragma unroll
      for (int i = 0; i < R; ++i) {
        const u32x16 c = *reinterpret_cast<const u32x16*>(coeff + (uint64_t)i * kCoeffStride);
#pragma unroll
        for (int u = 0; u < U; ++u) y[i][u] = dot4<K>(x[u], c);
      }
      wait_phase(period, rwin, period);
#pragma unroll
      for (int i = 0; i < R; ++i) {
        char* const orow = reinterpret_cast<char*>(ob + (uint64_t)out_idx[i] * out_shard);
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (g0 + 64 * u < v1) st16<true>(reinterpret_cast<uint32_t*>(orow + ((g0 + 64 * u) << 4)), y[i][u]);
      }
    }
  }
}
// ---- LDS-staged write bursts (round 2) --------------------------------------
// The product's software pipeline, but a wave parks each tile's R x U output
// vectors in LDS and stores T tiles' worth as one burst every T tiles, so the
// wave's store stream reaches the memory system in runs of T x R x U KiB.
template <int K, int U, int R, int T>
__global__ __launch_bounds__(kBlock) void burst_kernel(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                       uint64_t in_obj_stride, uint64_t in_shard,
                                                       uint64_t out_obj_stride, uint64_t out_shard,
                                                       const uint32_t* __restrict__ coeff,
                                                       const uint32_t* __restrict__ in_idx,
                                                       const uint32_t* __restrict__ out_idx, uint64_t ncols,
                                                       uint32_t nobj, uint32_t nseg) {
  __shared__ uint4 stage[kWaves][T][R][U][64];
  const uint32_t nvec = (uint32_t)(ncols >> 2);
  const uint32_t seg_vec = segment_vectors(nvec, nseg);
  const uint64_t nwork = (uint64_t)nobj * nseg;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t wave = blockIdx.x * kWaves + wv;
  const uint32_t nwaves = gridDim.x * kWaves;
  for (uint64_t wi = blockIdx.y; wi < nwork; wi += gridDim.y) {
    const uint64_t obj = wi / nseg;
    const uint32_t seg = (uint32_t)(wi % nseg);
    const uint32_t* __restrict__ ib = in + obj * in_obj_stride;
    uint32_t* __restrict__ ob = out + obj * out_obj_stride;
    const uint32_t* sb[K];
#pragma unroll
    for (int j = 0; j < K; ++j) sb[j] = ib + (uint64_t)in_idx[j] * in_shard;
    const uint32_t v0 = seg * seg_vec < nvec ? seg * seg_vec : nvec;
    const uint32_t v1 = nvec - v0 > seg_vec ? v0 + seg_vec : nvec;
    const uint32_t ntiles = (v1 - v0 + 64 * U - 1) / (64 * U);
    uint4 xa[U][K];
    uint32_t step = wave, slot = 0, first = wave;
    auto flush = [&](uint32_t nslots) {
      for (uint32_t t = 0; t < nslots; ++t) {
        const uint32_t g0 = v0 + (first + t * nwaves) * (64 * U) + lane;
#pragma unroll
        for (int i = 0; i < R; ++i) {
          char* const orow = reinterpret_cast<char*>(ob + (uint64_t)out_idx[i] * out_shard);
#pragma unroll
          for (int u = 0; u < U; ++u)
            if (g0 + 64 * u < v1) st16<true>(reinterpret_cast<uint32_t*>(orow + ((g0 + 64 * u) << 4)), stage[wv][t][i][u][lane]);
        }
      }
    };
    if (step < ntiles) load_tile<K, U, true>(xa, sb, v0 + step * (64 * U) + lane, v1);
    while (step < ntiles) {
      const uint32_t next = step + nwaves;
      uint4 xb[U][K];
      load_tile<K, U, true>(xb, sb, v0 + (next < ntiles ? next : step) * (64 * U) + lane, v1);
#pragma unroll
      for (int i = 0; i < R; ++i) {
        const u32x16 c = *reinterpret_cast<const u32x16*>(coeff + (uint64_t)i * kCoeffStride);
#pragma unroll
        for (int u = 0; u < U; ++u) stage[wv][slot][i][u][lane] = dot4<K>(xa[u], c);
      }
      if (++slot == T || next >= ntiles) {
        flush(slot);
        slot = 0;
        first = next;
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < K; ++j) xa[u][j] = xb[u][j];
      step = next;
    }
  }
}
// The product's software pipeline with every output row of a tile computed
// into registers first and the tile's R x U stores issued back to back
// (the product interleaves each row's stores with the next row's math).
template <int K, int U, int R>
__global__ __launch_bounds__(kBlock) void batched_kernel(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                         uint64_t in_obj_stride, uint64_t in_shard,
                                                         uint64_t out_obj_stride, uint64_t out_shard,
                                                         const uint32_t* __restrict__ coeff,
                                                         const uint32_t* __restrict__ in_idx,
                                                         const uint32_t* __restrict__ out_idx, uint64_t ncols,
                                                         uint32_t nobj, uint32_t nseg) {
  const uint32_t nvec = (uint32_t)(ncols >> 2);
  const uint32_t seg_vec = segment_vectors(nvec, nseg);
  const uint64_t nwork = (uint64_t)nobj * nseg;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = blockIdx.x * kWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nwaves = gridDim.x * kWaves;
  for (uint64_t wi = blockIdx.y; wi < nwork; wi += gridDim.y) {
    const uint64_t obj = wi / nseg;
    const uint32_t seg = (uint32_t)(wi % nseg);
    const uint32_t* __restrict__ ib = in + obj * in_obj_stride;
    uint32_t* __restrict__ ob = out + obj * out_obj_stride;
    const uint32_t* sb[K];
#pragma unroll
    for (int j = 0; j < K; ++j) sb[j] = ib + (uint64_t)in_idx[j] * in_shard;
    const uint32_t v0 = seg * seg_vec < nvec ? seg * seg_vec : nvec;
    const uint32_t v1 = nvec - v0 > seg_vec ? v0 + seg_vec : nvec;
    const uint32_t ntiles = (v1 - v0 + 64 * U - 1) / (64 * U);
    auto tile = [&](const uint4(&x)[U][K], uint32_t g0) {
      uint4 y[R][U];
#pragma unroll
      for (int i = 0; i < R; ++i) {
        const u32x16 c = *reinterpret_cast<const u32x16*>(coeff + (uint64_t)i * kCoeffStride);
#pragma unroll
        for (int u = 0; u < U; ++u) y[i][u] = dot4<K>(x[u], c);
      }
#pragma unroll
      for (int i = 0; i < R; ++i) {
        char* const orow = reinterpret_cast<char*>(ob + (uint64_t)out_idx[i] * out_shard);
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (g0 + 64 * u < v1) st16<true>(reinterpret_cast<uint32_t*>(orow + ((g0 + 64 * u) << 4)), y[i][u]);
      }
    };
    uint4 xa[U][K], xb[U][K];
    uint32_t step = wave;
    if (step < ntiles) load_tile<K, U, true>(xa, sb, v0 + step * (64 * U) + lane, v1);
    while (step < ntiles) {
      uint32_t next = step + nwaves;
      load_tile<K, U, true>(xb, sb, v0 + (next < ntiles ? next : step) * (64 * U) + lane, v1);
      tile(xa, v0 + step * (64 * U) + lane);
      step = next;
      if (step >= ntiles) break;
      next = step + nwaves;
      load_tile<K, U, true>(xa, sb, v0 + (next < ntiles ? next : step) * (64 * U) + lane, v1);
      tile(xb, v0 + step * (64 * U) + lane);
      step = next;
    }
  }
}
// The product's pipelined walk (rs_apply_pipe_kernel<K,U,true,true>) with a
// per-wave record of when it started, when it issued its last store, which
// XCD it ran on and how many tiles it walked: is the launch's tail (waves
// idle while others finish) worth a dynamic schedule?
struct WaveStamp {
  uint64_t t0, t1;
  uint32_t xcc, tiles;
};
__device__ __forceinline__ uint32_t xcc_id() {
  uint32_t v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 0xF;
}
template <int K, int U>
__global__ __launch_bounds__(kBlock) void timed_kernel(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                       uint64_t in_obj_stride, uint64_t in_shard,
                                                       uint64_t out_obj_stride, uint64_t out_shard,
                                                       const uint32_t* __restrict__ coeff,
                                                       const uint32_t* __restrict__ in_idx,
                                                       const uint32_t* __restrict__ out_idx, uint64_t ncols,
                                                       uint32_t nobj, uint32_t rows, uint32_t nseg,
                                                       WaveStamp* __restrict__ stamps) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const uint32_t nvec = (uint32_t)(ncols >> 2);
  const uint32_t seg_vec = segment_vectors(nvec, nseg);
  const uint64_t nwork = (uint64_t)nobj * nseg;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = blockIdx.x * kWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nwaves = gridDim.x * kWaves;
  uint32_t walked = 0;
  for (uint64_t wi = blockIdx.y; wi < nwork; wi += gridDim.y) {
    const uint64_t obj = wi / nseg;
    const uint32_t seg = (uint32_t)(wi % nseg);
    const uint32_t* __restrict__ ib = in + obj * in_obj_stride;
    uint32_t* __restrict__ ob = out + obj * out_obj_stride;
    const uint32_t* sb[K];
#pragma unroll
    for (int j = 0; j < K; ++j) sb[j] = ib + (uint64_t)in_idx[j] * in_shard;
    const uint32_t v0 = seg * seg_vec < nvec ? seg * seg_vec : nvec;
    const uint32_t v1 = nvec - v0 > seg_vec ? v0 + seg_vec : nvec;
    const uint32_t ntiles = (v1 - v0 + 64 * U - 1) / (64 * U);
    uint4 xa[U][K], xb[U][K];
    uint32_t step = wave;
    if (step < ntiles) load_tile<K, U, true>(xa, sb, v0 + step * (64 * U) + lane, v1);
    while (step < ntiles) {
      uint32_t next = step + nwaves;
      load_tile<K, U, true>(xb, sb, v0 + (next < ntiles ? next : step) * (64 * U) + lane, v1);
      store_tile<K, U, true>(xa, ob, coeff, out_idx, out_shard, rows, v0 + step * (64 * U) + lane, v1);
      ++walked;
      step = next;
      if (step >= ntiles) break;
      next = step + nwaves;
      load_tile<K, U, true>(xa, sb, v0 + (next < ntiles ? next : step) * (64 * U) + lane, v1);
      store_tile<K, U, true>(xb, ob, coeff, out_idx, out_shard, rows, v0 + step * (64 * U) + lane, v1);
      ++walked;
      step = next;
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0) {
    const uint32_t w = (blockIdx.y * gridDim.x + blockIdx.x) * kWaves + (threadIdx.x >> 6);
    WaveStamp st;
    st.t0 = t0;
    st.t1 = t1;
    st.xcc = xcc_id();
    st.tiles = walked;
    stamps[w] = st;
  }
}
}  // namespace

// Product walk with per-wave stamps (k = 8, U = 3); stamps: gx*gy*4 records.
extern "C" int av_launch_timed(const uint32_t* in, uint32_t* out, uint64_t io, uint64_t is, uint64_t oo, uint64_t os,
                               const uint32_t* coeff, const uint32_t* ii, const uint32_t* oi, uint64_t ncols,
                               uint32_t nobj, uint32_t rows, uint32_t gx, uint32_t gy, void* stream, uint32_t nseg,
                               void* stamps) {
  hipLaunchKernelGGL((timed_kernel<8, 3>), dim3(gx, gy), dim3(kBlock), 0, (hipStream_t)stream, in, out, io, is, oo, os,
                     coeff, ii, oi, ncols, nobj, rows, nseg, (WaveStamp*)stamps);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

// Dynamic-schedule walk (rs_apply_queue_kernel<K, 3, C, NC, .., TB, STAMP>), k = 8 or 10.
// C argument = C + 100 * NC + 10000 * TB + 100000 * U (TB = tickets per atomic, 1 when 0; U = 3 when 0);
// tickets: a counter set of NC + 1 lines (64 words each), zero at launch (each launch leaves it zero);
// stamps (3 words per wave) recorded when non-null.
extern "C" int av_launch_queue(int C, int k, const uint32_t* in, uint32_t* out, uint64_t io, uint64_t is, uint64_t oo,
                               uint64_t os, const uint32_t* coeff, const uint32_t* ii, const uint32_t* oi,
                               uint64_t ncols, uint32_t nobj, uint32_t rows, uint32_t blocks, void* stream,
                               void* ticket, void* stamps, uint32_t spread) {
  hipStream_t s = (hipStream_t)stream;
  uint32_t* t = (uint32_t*)ticket;
  if ((C / 10000) % 10 == 0) C += 10000;  // TB defaults to 1
#define QU(KK, UU, CC, NN, TT)                                                                                   \
  if (k == KK && C == CC + 100 * NN + 10000 * TT + 100000 * (UU == 3 ? 0 : UU)) {                              \
    if (stamps)                                                                                                 \
      hipLaunchKernelGGL((rs_apply_queue_kernel<KK, UU, CC, NN, true, true, TT, true>), dim3(blocks), dim3(kBlock), \
                         0, s, in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, (uint32_t)KK, t,    \
                         (uint64_t*)stamps, spread);                                                            \
    else                                                                                                        \
      hipLaunchKernelGGL((rs_apply_queue_kernel<KK, UU, CC, NN, true, true, TT, false>), dim3(blocks), dim3(kBlock), \
                         0, s, in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, (uint32_t)KK, t,    \
                         nullptr, spread);                                                                      \
    return hipGetLastError() == hipSuccess ? 0 : -3;                                                            \
  }
#define Q(KK, CC, NN, TT) QU(KK, 3, CC, NN, TT)
  // C + 100 NC + 10000 TB + 1000000: on-demand (SYNC) ticket fetch
#define QS(KK, UU, CC, NN, TT)                                                                                   \
  if (k == KK && C == CC + 100 * NN + 10000 * TT + 100000 * (UU == 3 ? 0 : UU) + 1000000) {                    \
    hipLaunchKernelGGL((rs_apply_queue_kernel<KK, UU, CC, NN, true, true, TT, false, true>), dim3(blocks),        \
                       dim3(kBlock), 0, s, in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, (uint32_t)KK, \
                       t, nullptr, spread);                                                                  \
    return hipGetLastError() == hipSuccess ? 0 : -3;                                                            \
  }
  QS(8, 3, 2, 8, 1) QS(8, 3, 2, 8, 2) QS(8, 3, 2, 8, 4) QS(8, 3, 2, 8, 8) QS(8, 3, 4, 8, 2)
  QS(4, 4, 2, 8, 2) QS(4, 4, 2, 8, 4) QS(4, 4, 2, 8, 8)
  // C + 100 NC + 10000000 * (1 + 2 * !NTL + !NTS): load/store cache policy (nt = non-temporal)
#define QN(KK, CC, NN, LL, SS)                                                                                   \
  if (k == KK && C == CC + 100 * NN + 10000 + 10000000 * (1 + 2 * !LL + !SS)) {                                  \
    hipLaunchKernelGGL((rs_apply_queue_kernel<KK, 3, CC, NN, LL, SS>), dim3(blocks), dim3(kBlock), 0, s, in, out, io, \
                       is, oo, os, coeff, ii, oi, ncols, nobj, rows, (uint32_t)KK, t, nullptr, spread);       \
    return hipGetLastError() == hipSuccess ? 0 : -3;                                                            \
  }
  QN(8, 2, 8, true, false) QN(8, 2, 8, false, true) QN(8, 2, 8, false, false)
#undef QN
  Q(8, 4, 1, 1) Q(8, 1, 8, 1) Q(8, 2, 8, 1) Q(8, 4, 8, 1) Q(8, 8, 8, 1) Q(10, 2, 8, 1) Q(10, 4, 8, 1)
  Q(8, 2, 8, 2) Q(8, 2, 8, 4) Q(8, 1, 8, 4) Q(8, 1, 8, 8)
  // k = 4 (C2): U = 3, 2, 1; round 3: U = 5, 6, 8 (more bytes in flight per wave)
  Q(4, 2, 8, 1) Q(4, 4, 8, 1) QU(4, 2, 3, 8, 1) QU(4, 1, 6, 8, 1) QU(4, 1, 12, 8, 1) QU(4, 4, 2, 8, 1)
  QU(4, 5, 1, 8, 1) QU(4, 6, 1, 8, 1) QU(4, 6, 2, 8, 1) QU(4, 8, 1, 8, 1) QU(4, 4, 1, 8, 1)
  // k = 8: U = 4, 2
  QU(8, 4, 2, 8, 1) QU(8, 4, 1, 8, 1) QU(8, 2, 3, 8, 1) QU(8, 2, 2, 8, 1) Q(8, 3, 8, 1)
  // k = 10 (C5): U = 2, 1 (no AGPRs: the U = 3 form holds 256 VGPRs + 14 AGPRs)
  QU(10, 2, 3, 8, 1) QU(10, 2, 2, 8, 1) QU(10, 1, 6, 8, 1)
  // k = 16: U = 1, 2
  QU(16, 1, 6, 8, 1) QU(16, 1, 12, 8, 1) QU(16, 2, 3, 8, 1)
#undef Q
#undef QU
#undef QS
  return -2;
}

extern "C" int av_launch_batched(int U, const uint32_t* in, uint32_t* out, uint64_t io, uint64_t is, uint64_t oo,
                                 uint64_t os, const uint32_t* coeff, const uint32_t* ii, const uint32_t* oi,
                                 uint64_t ncols, uint32_t nobj, uint32_t gx, uint32_t gy, void* stream,
                                 uint32_t nseg) {
  hipStream_t s = (hipStream_t)stream;
  if (U == 2)
    hipLaunchKernelGGL((batched_kernel<8, 2, 4>), dim3(gx, gy), dim3(kBlock), 0, s, in, out, io, is, oo, os, coeff, ii,
                       oi, ncols, nobj, nseg);
  else if (U == 3)
    hipLaunchKernelGGL((batched_kernel<8, 3, 4>), dim3(gx, gy), dim3(kBlock), 0, s, in, out, io, is, oo, os, coeff, ii,
                       oi, ncols, nobj, nseg);
  else
    return -2;
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

extern "C" int av_launch_burst(int T, const uint32_t* in, uint32_t* out, uint64_t io, uint64_t is, uint64_t oo,
                               uint64_t os, const uint32_t* coeff, const uint32_t* ii, const uint32_t* oi,
                               uint64_t ncols, uint32_t nobj, uint32_t gx, uint32_t gy, void* stream, uint32_t nseg) {
  hipStream_t s = (hipStream_t)stream;
  if (T == 1)
    hipLaunchKernelGGL((burst_kernel<8, 3, 4, 1>), dim3(gx, gy), dim3(kBlock), 0, s, in, out, io, is, oo, os, coeff, ii,
                       oi, ncols, nobj, nseg);
  else if (T == 2)
    hipLaunchKernelGGL((burst_kernel<8, 3, 4, 2>), dim3(gx, gy), dim3(kBlock), 0, s, in, out, io, is, oo, os, coeff, ii,
                       oi, ncols, nobj, nseg);
  else if (T == 3)
    hipLaunchKernelGGL((burst_kernel<8, 3, 4, 3>), dim3(gx, gy), dim3(kBlock), 0, s, in, out, io, is, oo, os, coeff, ii,
                       oi, ncols, nobj, nseg);
  else
    return -2;
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

// Wide-k pipelined kernel (the product's rs_apply_wide_pipe_kernel) with the
// field math or the XOR stand-in: how much of a wide launch is VALU?
extern "C" int av_launch_wide(int math, const uint32_t* in, uint32_t* out, uint64_t io, uint64_t is, uint64_t oo,
                              uint64_t os, const uint32_t* coeff, const uint32_t* ii, const uint32_t* oi,
                              uint64_t ncols, uint32_t nobj, uint32_t rows, uint32_t k, uint32_t gx, uint32_t gy,
                              void* stream, uint32_t nseg) {
  hipStream_t s = (hipStream_t)stream;
  const dim3 g(gx, gy), b(kBlock);
#define W(RB, M) \
  hipLaunchKernelGGL((rs_apply_wide_pipe_kernel<RB, true, true, M>), g, b, 0, s, in, out, io, is, oo, os, coeff, ii, oi, \
                     ncols, nobj, rows, k, nseg)
  if (rows <= 8) {
    if (math) W(8, true); else W(8, false);
  } else {
    if (math) W(16, true); else W(16, false);
  }
#undef W
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

// The k <= 16 pipelined kernel instantiated for wider k (coefficient rows of
// ceil(K/16) x 16 words): a candidate for 17 <= k <= 32 instead of the wide kernel.
extern "C" int av_launch_pipek(int K, int U, const uint32_t* in, uint32_t* out, uint64_t io, uint64_t is,
                               uint64_t oo, uint64_t os, const uint32_t* coeff, const uint32_t* ii, const uint32_t* oi,
                               uint64_t ncols, uint32_t nobj, uint32_t rows, uint32_t gx, uint32_t gy, void* stream,
                               uint32_t nseg) {
  hipStream_t s = (hipStream_t)stream;
#define PK(KK, UU)                                                                                               \
  if (K == KK && U == UU) {                                                                                      \
    gp<KK, UU, true, true>(in, out, io, is, oo, os, coeff, ii, oi, ncols, nobj, rows, gx, gy, s, nseg);          \
    return hipGetLastError() == hipSuccess ? 0 : -3;                                                            \
  }
  PK(20, 1) PK(20, 2) PK(24, 1) PK(24, 2) PK(28, 1) PK(32, 1) PK(40, 1) PK(48, 1)
#undef PK
  return -2;
}

// Phased walk launch (k = 8, 4 rows): U in {3, 6}.
extern "C" int av_launch_phased(int U, const uint32_t* in, uint32_t* out, uint64_t io, uint64_t is, uint64_t oo,
                                uint64_t os, const uint32_t* coeff, const uint32_t* ii, const uint32_t* oi,
                                uint64_t ncols, uint32_t nobj, uint32_t gx, uint32_t gy, void* stream, uint32_t nseg,
                                uint32_t period, uint32_t rwin) {
  hipStream_t s = (hipStream_t)stream;
  if (period == 0 || rwin == 0 || rwin >= period) return -4;
  if (U == 3)
    hipLaunchKernelGGL((phased_kernel<8, 3, 4>), dim3(gx, gy), dim3(kBlock), 0, s, in, out, io, is, oo, os, coeff, ii,
                       oi, ncols, nobj, nseg, period, rwin);
  else if (U == 6)
    hipLaunchKernelGGL((phased_kernel<8, 6, 4>), dim3(gx, gy), dim3(kBlock), 0, s, in, out, io, is, oo, os, coeff, ii,
                       oi, ncols, nobj, nseg, period, rwin);
  else
    return -2;
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

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
