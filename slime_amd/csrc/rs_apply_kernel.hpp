// The GF(2^32-5) shard-matrix apply kernel template (device code), shared by
// the product instantiations (rs_apply.hip) and the tuning harness
// (tools/apply_variants.hip).  See rs_apply.hip for the design notes.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gfp.hpp"

namespace slime {
namespace apply {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;
// Device coefficient tables: rows padded to a multiple of 16 words (64 B), so
// a row (k <= 16) or a 16-coefficient chunk of one (wide k) arrives in one
// s_load_dwordx16.  kCoeffStride is the row stride of the k <= 16 kernels.
constexpr int kCoeffStride = 16;
__host__ __device__ constexpr uint32_t wide_coeff_stride(uint32_t k) { return (k + 15u) & ~15u; }

// 16-byte vectors per column segment: an even split rounded UP to a whole
// 1 KiB of every stream (64 vectors), so every segment -- and with it every
// wave's tile -- starts on the same 1 KiB grid as its shard base.  An odd
// split (e.g. 10/14 on 1 GiB objects: 6710886 vectors / 8 = 838861) puts
// every 1 KiB access of the launch across a cache-line boundary: 10/14 ran
// at 5.5 TB/s against 6.1 for the same kernel on line-aligned segments
// (profiles/r01/segalign/).  Trailing segments may come out empty.
template <typename T>
__host__ __device__ __forceinline__ T segment_vectors(T nvec, uint32_t nseg) {
  return ((nvec + nseg - 1) / nseg + 63) & ~(T)63;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));

template <bool NT>
__device__ __forceinline__ uint4 ld16(const uint32_t* p) {
  u32x4 v;
  if constexpr (NT)
    v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  else
    v = *reinterpret_cast<const u32x4*>(p);
  return make_uint4(v.x, v.y, v.z, v.w);
}

template <bool NT>
__device__ __forceinline__ void st16(uint32_t* p, uint4 r) {
  const u32x4 v = {r.x, r.y, r.z, r.w};
  if constexpr (NT)
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
  else
    *reinterpret_cast<u32x4*>(p) = v;
}

// Coefficient row of a compile-time-K kernel: ceil(K/16) s_load_dwordx16 of
// a row padded to a multiple of 16 words (the plan table's row stride,
// coeff_stride(k)); K <= 16 is one load at stride kCoeffStride.
template <int K>
struct CoeffRow {
  static constexpr int kVecs = (K + 15) / 16;
  static constexpr int kStride = kVecs * 16;
  u32x16 v[kVecs];
  __device__ __forceinline__ uint32_t operator[](int j) const { return v[j >> 4][j & 15]; }
};
template <int K>
__device__ __forceinline__ CoeffRow<K> load_coeff_row(const uint32_t* __restrict__ coeff, uint32_t i) {
  CoeffRow<K> r;
#pragma unroll
  for (int q = 0; q < CoeffRow<K>::kVecs; ++q)
    r.v[q] = *reinterpret_cast<const u32x16*>(coeff + (uint64_t)i * CoeffRow<K>::kStride + 16 * q);
  return r;
}

// One output word of a wide column, sum_j c[j] x(j) over k inputs: the
// loads sixteen at a time, all issued before the first product (indices past
// k re-read input k-1 and multiply by zero), so a lane waits one memory
// latency per sixteen inputs -- one load per product left a lane's rows x k
// loads in a serial chain, ~0.5 us each (0.15 ms of a 4-row, 80-input tail).
template <class X>
__device__ __forceinline__ uint32_t wide_dot(const uint32_t* __restrict__ c, uint32_t k, X x) {
  uint64_t lo = 0;
  uint32_t hi = 0;
  for (uint32_t j0 = 0; j0 < k; j0 += 16) {
    uint32_t v[16], w[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const uint32_t jj = j0 + j < k ? j0 + j : k - 1;
      v[j] = x(jj);
      w[j] = j0 + j < k ? c[jj] : 0u;
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) mac(lo, hi, v[j], w[j]);
  }
  return fold96(lo, hi);
}

// Output row i of column b of a wide (generic k) column.
__device__ __forceinline__ void apply_cell(const uint32_t* __restrict__ ib, uint32_t* __restrict__ ob,
                                           const uint32_t* __restrict__ coeff, const uint32_t* __restrict__ in_idx,
                                           uint64_t in_shard, const uint32_t* __restrict__ out_idx,
                                           uint64_t out_shard, uint32_t k, uint32_t i, uint64_t b) {
  ob[(uint64_t)out_idx[i] * out_shard + b] = wide_dot(coeff + (uint64_t)i * wide_coeff_stride(k), k, [&](uint32_t j) {
    return ib[(uint64_t)in_idx[j] * in_shard + b];
  });
}

// One column per lane (tails, unaligned layouts, generic k).
template <int K>
__device__ __forceinline__ void apply_column(const uint32_t* __restrict__ ib, uint32_t* __restrict__ ob,
                                             const uint32_t* __restrict__ coeff,
                                             const uint32_t* __restrict__ in_idx, uint64_t in_shard,
                                             const uint32_t* __restrict__ out_idx, uint64_t out_shard,
                                             uint32_t rows, uint32_t k, uint64_t b) {
  if constexpr (K > 0) {
    uint32_t x[K];
#pragma unroll
    for (int j = 0; j < K; ++j) x[j] = ib[(uint64_t)in_idx[j] * in_shard + b];
    for (uint32_t i = 0; i < rows; ++i) {
      const CoeffRow<K> c = load_coeff_row<K>(coeff, i);
      uint64_t lo = 0;
      uint32_t hi = 0;
#pragma unroll
      for (int j = 0; j < K; ++j) mac(lo, hi, x[j], c[j]);
      ob[(uint64_t)out_idx[i] * out_shard + b] = fold96(lo, hi);
    }
  } else {
    for (uint32_t i = 0; i < rows; ++i) apply_cell(ib, ob, coeff, in_idx, in_shard, out_idx, out_shard, k, i, b);
  }
}

// One output row over 4 columns (C: a u32x16 for K <= 16, or a CoeffRow<K>).
template <int K, class C>
__device__ __forceinline__ uint4 dot4(const uint4 (&x)[K], const C& c) {
  uint64_t lo0 = 0, lo1 = 0, lo2 = 0, lo3 = 0;
  uint32_t hi0 = 0, hi1 = 0, hi2 = 0, hi3 = 0;
#pragma unroll
  for (int j = 0; j < K; ++j) mac4(lo0, lo1, lo2, lo3, hi0, hi1, hi2, hi3, x[j].x, x[j].y, x[j].z, x[j].w, c[j]);
  return make_uint4(fold96(lo0, hi0), fold96(lo1, hi1), fold96(lo2, hi2), fold96(lo3, hi3));
}

// Accumulate one output row over 4 columns and store it.
template <int K, bool NTS>
__device__ __forceinline__ void row4(const uint4 (&x)[K], const u32x16& c, uint32_t* dst) {
  uint64_t lo0 = 0, lo1 = 0, lo2 = 0, lo3 = 0;
  uint32_t hi0 = 0, hi1 = 0, hi2 = 0, hi3 = 0;
#pragma unroll
  for (int j = 0; j < K; ++j) mac4(lo0, lo1, lo2, lo3, hi0, hi1, hi2, hi3, x[j].x, x[j].y, x[j].z, x[j].w, c[j]);
  uint4 r;
  r.x = fold96(lo0, hi0);
  r.y = fold96(lo1, hi1);
  r.z = fold96(lo2, hi2);
  r.w = fold96(lo3, hi3);
  st16<NTS>(dst, r);
}

// K > 0: compile-time number of input shards (1..16), 4 columns (16 B) per
// lane per unit; a wave owns U*64 consecutive 16-byte units (U*1 KiB of every
// shard stripe) per step, so each load instruction is a fully coalesced 1 KiB
// and the wave streams U KiB contiguous per shard.  K == 0: generic k.
// Objects: blockIdx.y strides over objects, so gridDim.y bounds how many
// objects (x shards) are streamed concurrently.
// Segments: each object's columns are cut into `nseg` contiguous segments
// that are scheduled like separate objects (blockIdx.y strides over
// object x segment), so a batch of few objects still keeps many independent
// stripe streams in flight; nseg = 1 is the plain per-object walk.
//
// ROT: each object walks its column tiles starting at a per-object rotation
// (a bijection of [0, ntiles)), so the ~k x objects-in-flight concurrent
// streams, whose shard bases share their low address bits when shards are
// large powers of two, do not all hit the same DRAM channels/banks in step.
template <int K, bool VEC, int U, bool NTL, bool NTS, bool ROT = false>
__global__ __launch_bounds__(kBlock) void rs_apply_kernel(
    const uint32_t* __restrict__ in, uint32_t* __restrict__ out, uint64_t in_obj_stride, uint64_t in_shard,
    uint64_t out_obj_stride, uint64_t out_shard, const uint32_t* __restrict__ coeff,
    const uint32_t* __restrict__ in_idx, const uint32_t* __restrict__ out_idx, uint64_t ncols, uint32_t nobj,
    uint32_t rows, uint32_t k, uint32_t nseg) {
  const uint64_t tid = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const uint64_t nthr = (uint64_t)gridDim.x * kBlock;
  const uint64_t nvec = VEC && K > 0 ? ncols >> 2 : 0;
  const uint64_t seg_vec = segment_vectors(nvec, nseg);  // 16-byte vectors per segment
  const uint64_t nwork = (uint64_t)nobj * nseg;
  for (uint64_t wi = blockIdx.y; wi < nwork; wi += gridDim.y) {
    const uint64_t obj = wi / nseg, seg = wi % nseg;
    const uint32_t* __restrict__ ib = in + obj * in_obj_stride;
    uint32_t* __restrict__ ob = out + obj * out_obj_stride;
    if constexpr (VEC && K > 0) {
      uint64_t ioff[K];
#pragma unroll
      for (int j = 0; j < K; ++j) ioff[j] = (uint64_t)in_idx[j] * in_shard;
      // This segment's vectors [v0, v1).
      const uint64_t v0 = seg * seg_vec < nvec ? seg * seg_vec : nvec;
      const uint64_t v1 = v0 + seg_vec < nvec ? v0 + seg_vec : nvec;
      const uint32_t lane = threadIdx.x & 63;
      const uint64_t wave = (uint64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
      const uint64_t nwaves = (uint64_t)gridDim.x * kWaves;
      const uint64_t ntiles = (v1 - v0 + 64 * U - 1) / (64 * U);
      const uint64_t rot = ROT && ntiles ? ((uint64_t)wi * 0x9E3779B97F4A7C15ull >> 20) % ntiles : 0;
      for (uint64_t step = wave; step < ntiles; step += nwaves) {
        uint64_t t = step + rot;
        if (t >= ntiles) t -= ntiles;
        const uint64_t g0 = v0 + t * (64 * U) + lane;
        uint4 x[U][K];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint64_t b = (g0 + 64 * u) << 2;
          if (g0 + 64 * u < v1) {
#pragma unroll
            for (int j = 0; j < K; ++j) x[u][j] = ld16<NTL>(ib + ioff[j] + b);
          }
        }
        for (uint32_t i = 0; i < rows; ++i) {
          // One 64-byte row -> one s_load_dwordx16 (SGPRs).
          const u32x16 c = *reinterpret_cast<const u32x16*>(coeff + (uint64_t)i * kCoeffStride);
          uint32_t* const orow = ob + (uint64_t)out_idx[i] * out_shard;
#pragma unroll
          for (int u = 0; u < U; ++u)
            if (g0 + 64 * u < v1) row4<K, NTS>(x[u], c, orow + ((g0 + 64 * u) << 2));
        }
      }
    }
    // Columns past the last whole vector (all columns for the one-column
    // kernels), one per lane, by the object's last segment.
    if (seg == nseg - 1)
      for (uint64_t b = (nvec << 2) + tid; b < ncols; b += nthr)
        apply_column<K>(ib, ob, coeff, in_idx, in_shard, out_idx, out_shard, rows, k, b);
  }
}

// Software-pipelined form of the vectorised rs_apply_kernel: a wave issues
// the loads of its NEXT tile before it computes and stores the current one,
// so its own loads stay in flight through the math (two register sets of
// U x K x 16 B, alternating; no copies).  Same tiles, same segments, same
// results as rs_apply_kernel<K, true, U, ...>.
// Loads are unconditional (lanes past the segment end re-read its last
// vector), so the waitcnt pass sees a fixed count of loads per tile and can
// wait for one register set while the other is still in flight.
// Addressing: a shard is < 4 GiB (L < 2^30 symbols, checked by the host),
// so every access is a wave-uniform 64-bit shard base (SGPRs) plus a 32-bit
// per-lane byte offset -- the saddr form of global_load/store, one VGPR per
// address instead of a 64-bit VGPR pair built by two VALU ops.
template <bool NT>
__device__ __forceinline__ uint4 ld16_at(const uint32_t* base, uint32_t byte_off) {
  return ld16<NT>(reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(base) + byte_off));
}

// Loads are unconditional (lanes past the segment end re-read its last
// vector), so the waitcnt pass sees a fixed count of loads per tile and can
// wait for one register set while the other is still in flight.
template <int K, int U, bool NTL, bool LOAD = true>
__device__ __forceinline__ void load_tile(uint4 (&x)[U][K], const uint32_t* const (&sb)[K], uint32_t g0, uint32_t v1) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t g = g0 + 64 * u < v1 ? g0 + 64 * u : v1 - 1;
#pragma unroll
    for (int j = 0; j < K; ++j)
      if constexpr (LOAD)
        x[u][j] = ld16_at<NTL>(sb[j], g << 4);
      else
        x[u][j] = make_uint4(g, g + j, g ^ j, g * 3u + j);  // write-only probe
  }
}

// One output row of a tile: math outside the store branch, so every
// register set is consumed on every path.
// XOR stand-in for dot4 (one full-rate op per term instead of mad + addc):
// WRONG results, used only by the tuning harness (MODE != 0) to measure
// how much of the pipelined kernel's time the field math costs.
template <int K, class C>
__device__ __forceinline__ uint4 xor4(const uint4 (&x)[K], const C& c) {
  uint4 r = make_uint4(c[0], c[1], c[2], c[3]);
#pragma unroll
  for (int j = 0; j < K; ++j) {
    r.x ^= x[j].x + c[j];
    r.y ^= x[j].y + c[j];
    r.z ^= x[j].z + c[j];
    r.w ^= x[j].w + c[j];
  }
  return r;
}

template <int K, int U, bool NTS, int MODE = 0>
__device__ __forceinline__ void tile_row(const uint4 (&x)[U][K], uint32_t* __restrict__ ob,
                                         const uint32_t* __restrict__ coeff, const uint32_t* __restrict__ out_idx,
                                         uint64_t out_shard, uint32_t i, uint32_t g0, uint32_t v1) {
  const CoeffRow<K> c = load_coeff_row<K>(coeff, i);
  char* const orow = reinterpret_cast<char*>(ob + (uint64_t)out_idx[i] * out_shard);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    uint4 r;
    if constexpr (MODE == 0 || MODE == 4)
      r = dot4<K>(x[u], c);
    else
      r = xor4<K>(x[u], c);
    if constexpr (MODE == 2)  // read-only probe: a store that (for random data) never happens
      if (r.x != r.y || r.y != r.z || r.z != r.w) continue;
    if (g0 + 64 * u < v1) st16<NTS>(reinterpret_cast<uint32_t*>(orow + ((g0 + 64 * u) << 4)), r);
  }
}

// Row 0 is peeled (rows >= 1 always): it reads every symbol of the tile, so
// the waitcnt pass resolves the tile's loads there, with per-load counts that
// leave the other register set in flight, and the runtime row loop after it
// has nothing left to wait for.
template <int K, int U, bool NTS, int MODE = 0>
__device__ __forceinline__ void store_tile(const uint4 (&x)[U][K], uint32_t* __restrict__ ob,
                                           const uint32_t* __restrict__ coeff, const uint32_t* __restrict__ out_idx,
                                           uint64_t out_shard, uint32_t rows, uint32_t g0, uint32_t v1) {
  tile_row<K, U, NTS, MODE>(x, ob, coeff, out_idx, out_shard, 0, g0, v1);
  for (uint32_t i = 1; i < rows; ++i) tile_row<K, U, NTS, MODE>(x, ob, coeff, out_idx, out_shard, i, g0, v1);
}

// MODE (tuning harness only; the product is MODE 0, the field math):
//   1 swaps the field math for xor4, 2 also drops the stores (read-only),
//   3 keeps xor4 and the stores but drops the loads (write-only),
//   4 is the product math with an XCD-grouped work order (blocks are dispatched
//     round-robin over the 8 XCDs; 4 gives XCD x the contiguous work items
//     [x*gy/8, (x+1)*gy/8) instead of every 8th one).
template <int K, int U, bool NTL, bool NTS, int MODE = 0>
__global__ __launch_bounds__(kBlock) void rs_apply_pipe_kernel(
    const uint32_t* __restrict__ in, uint32_t* __restrict__ out, uint64_t in_obj_stride, uint64_t in_shard,
    uint64_t out_obj_stride, uint64_t out_shard, const uint32_t* __restrict__ coeff,
    const uint32_t* __restrict__ in_idx, const uint32_t* __restrict__ out_idx, uint64_t ncols, uint32_t nobj,
    uint32_t rows, uint32_t k, uint32_t nseg) {
  static_assert(K > 0, "compile-time k only");
  const uint64_t tid = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const uint64_t nthr = (uint64_t)gridDim.x * kBlock;
  // Vector indices within a shard are 32-bit (host guarantees L < 2^30).
  const uint32_t nvec = (uint32_t)(ncols >> 2);
  const uint32_t seg_vec = segment_vectors(nvec, nseg);
  const uint64_t nwork = (uint64_t)nobj * nseg;
  const uint32_t lane = threadIdx.x & 63;
  // Wave-uniform (readfirstlane) 32-bit tile counters: the tile loop is a
  // scalar loop with scalar compares.
  const uint32_t wave = blockIdx.x * kWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nwaves = gridDim.x * kWaves;
  uint32_t by = blockIdx.y;
  if constexpr (MODE == 4)
    if (gridDim.x == 1 && gridDim.y % 8 == 0) by = (blockIdx.y % 8) * (gridDim.y / 8) + blockIdx.y / 8;
  for (uint64_t wi = by; wi < nwork; wi += gridDim.y) {
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
    if (step < ntiles) load_tile<K, U, NTL, MODE != 3>(xa, sb, v0 + step * (64 * U) + lane, v1);
    // The last prefetch of a wave (past ntiles) re-reads its current tile.
    while (step < ntiles) {
      uint32_t next = step + nwaves;
      load_tile<K, U, NTL, MODE != 3>(xb, sb, v0 + (next < ntiles ? next : step) * (64 * U) + lane, v1);
      store_tile<K, U, NTS, MODE>(xa, ob, coeff, out_idx, out_shard, rows, v0 + step * (64 * U) + lane, v1);
      step = next;
      if (step >= ntiles) break;
      next = step + nwaves;
      load_tile<K, U, NTL, MODE != 3>(xa, sb, v0 + (next < ntiles ? next : step) * (64 * U) + lane, v1);
      store_tile<K, U, NTS, MODE>(xb, ob, coeff, out_idx, out_shard, rows, v0 + step * (64 * U) + lane, v1);
      step = next;
    }
    if (seg == nseg - 1)
      for (uint64_t b = ((uint64_t)nvec << 2) + tid; b < ncols; b += nthr)
        apply_column<K>(ib, ob, coeff, in_idx, in_shard, out_idx, out_shard, rows, k, b);
  }
}

// ---- dynamic schedule -------------------------------------------------------
// rs_apply_pipe_kernel hands every wave a fixed share of the batch.  The eight
// XCDs do not stream at the same rate (C3 on one box: waves on the odd XCDs
// finished 4% after those on the even ones, so 3.3% of the launch's wave-time
// was idle tail; tools/apply_variants.py --timed, profiles/r02/s36_tail/).
// Here waves take work from ticket counters instead, so fast XCDs take more.
//
// Units: an object's tiles are cut into groups of 4*C consecutive tiles; unit
// = (group, sub) walks tiles grp*4C + sub + 4i, i < C.  The waves that take
// four consecutive tickets sweep one 4C-tile window of one object together --
// as a block's four waves do in the static walk.  Ticket-order group g
// belongs to object g % nobj, so the groups running at any moment spread over
// all objects; within an object, its q-th group in ticket order sits at
// segment q % S, position q / S (S = `spread` segments of B groups), so a
// batch of few objects also keeps its windows spread over each object, as
// the static walk's column segments do.
//
// Tickets: one device-scope counter serialises at ~12 ns per atomic (C = 1:
// 1.4M tickets took 16.6 ms at C3), so the groups are dealt over NC counters
// (partition p owns groups g = p (mod NC)), each on its own 256-byte line.  A
// wave draws from its XCD's partition and, once that is exhausted, from the
// next ones in turn; a wave is done when all NC have run dry.  The ticket for
// a wave's next unit is requested when it enters a unit and read one unit
// later, so its latency is hidden (the compiler still waits vmcnt(0) before
// reading it: atomics and loads share the counter).
//
// A launch leaves its counter set as it found it, zero: every wave bumps the
// set's exit counter once it has found every partition dry (its last draw
// has returned by then), and the wave that brings it to the launch's wave
// count -- no draw can follow -- zeroes the NC counters and the exit counter.
// So a set needs no host-side reset between launches: the host hands each
// launch a set no unfinished launch holds (rs_apply.hip, TicketPool), and a
// set captured into a graph is reset by every replay itself.
constexpr uint32_t kTicketStride = 64;  // words between counters
// Words of one counter set of NC partitions: NC draw counters, then the exit
// counter, each on its own 256-byte line.
__host__ __device__ constexpr uint32_t ticket_set_words(int nc) { return (uint32_t)(nc + 1) * kTicketStride; }

__device__ __forceinline__ uint32_t hw_xcc_id() {
  uint32_t v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 0xF;
}

// A wave's walk over the units of a launch (device state, wave-uniform):
// the current unit (object obj, tiles tb + 4i for i < cnt) and the ticket
// bookkeeping.  Shared by the apply and byte queue kernels.  TB tickets per
// atomic (tuning harness; the product uses 1).
// SYNC: fetch a ticket only when it is needed (the wave waits for the atomic
// there) instead of one unit ahead.  With a ticket pending across tiles, the
// compiler waits vmcnt(0) before every tile's loads (an atomic and loads share
// the counter), draining the wave's pipeline each tile; fetched on demand,
// only the tiles that start a ticket batch pay the atomic's round trip.
template <int C, int NC, int TB = 1, bool SYNC = false>
struct TicketWalk {
  uint32_t* ticket;
  uint32_t spread, seg_groups;  // S segments of B groups per object
  uint32_t ngrp_all, nobj, ntiles, lane;
  uint32_t p, dry = 0;                           // partition, partitions found dry
  uint32_t obj = 0, tb = 0, cnt = 0, i = 0;      // current unit
  uint32_t pend = 0, bl = 0, bn = 0;             // pending atomic; rest of the ticket batch
  bool live = true;

  // ntiles: tiles per object; the launch's units cover nobj objects.  The
  // host guarantees nobj * spread * B * 4 < 2^32 (B = ceil(groups / spread)).
  __device__ __forceinline__ TicketWalk(uint32_t* t, uint32_t nobj_, uint32_t ntiles_, uint32_t lane_,
                                        uint32_t spread_ = 1)
      : ticket(t),
        spread(spread_ ? spread_ : 1),
        seg_groups(((ntiles_ + 4 * C - 1) / (4 * C) + spread - 1) / spread),
        ngrp_all(nobj_ * spread * seg_groups),
        nobj(nobj_),
        ntiles(ntiles_),
        lane(lane_) {
    p = hw_xcc_id() % NC;
    if (!skip_empty()) return;
    if (!SYNC) request();
    next_unit();
  }
  // Partitions with no units at all (a launch of fewer than NC groups: a
  // host call on a small object) are passed over without a draw -- each draw
  // is a memory-side atomic round trip of about a microsecond, and a wave
  // that asked all NC counters spent most of such a launch on them.
  // Partition p holds units iff p < ngrp_all, so the empty ones are the tail
  // p..NC-1: counted dry at once, the walk goes on at partition 0.  false:
  // every partition is dry (live cleared).
  __device__ __forceinline__ bool skip_empty() {
    if (p < ngrp_all) return true;
    dry += NC - p;
    p = 0;
    if (ngrp_all == 0 || dry >= NC) {
      live = false;
      return false;
    }
    return true;
  }
  __device__ __forceinline__ void request() {
    pend = 0;
    if (lane == 0) pend = atomicAdd(ticket + p * kTicketStride, (uint32_t)TB);
  }
  // Enter the unit of the pending ticket (or of later ones: exhausted
  // partitions and empty sub-units are skipped) and request the next ticket.
  __device__ __forceinline__ void next_unit() {
    for (;;) {
      uint32_t l;
      bool fresh = true;
      if (TB > 1 && bn) {
        l = bl++;
        --bn;
        fresh = false;
      } else {
        if (SYNC) request();
        l = __builtin_amdgcn_readlane(pend, 0);  // lane 0 drew it, whatever the exec mask
        bl = l + 1;
        bn = TB - 1;
      }
      const uint32_t units = 4 * ((ngrp_all + NC - 1 - p) / NC);
      if (l >= units) {
        if (++dry >= NC) {
          live = false;
          return;
        }
        p = p + 1 == NC ? 0 : p + 1;
        bn = 0;
        if (!skip_empty()) return;
        if (fresh && !SYNC) request();  // else the batch's successor is already pending
        continue;
      }
      if (fresh && !SYNC) request();
      const uint32_t g = (l >> 2) * NC + p;
      obj = g % nobj;
      const uint32_t q = g / nobj;
      tb = ((q % spread) * seg_groups + q / spread) * (4 * C) + (l & 3);
      i = 0;
      cnt = tb < ntiles ? (ntiles - tb + 3) / 4 : 0;
      if (cnt > C) cnt = C;
      if (cnt) return;
    }
  }
  __device__ __forceinline__ uint32_t tile() const { return tb + 4 * i; }
  // The current unit's index within its object (group * 4 + sub; see
  // unit_tile_base) and whether the current tile is the unit's first.
  __device__ __forceinline__ uint32_t unit() const { return (tb / (4 * C)) * 4 + tb % (4 * C); }
  __device__ __forceinline__ bool unit_start() const { return i == 0; }
  // Step to the next tile (the next unit's first after the last of this one).
  __device__ __forceinline__ void advance() {
    if (++i >= cnt) next_unit();
  }
  // Once per wave, after the walk ended (live == false): count the wave out;
  // the launch's last wave returns the set to zero (see kTicketStride).
  // Zeroed with atomics, which execute at the memory side like the draws.
  __device__ __forceinline__ void finish() { (void)finish_last(); }
  // finish(), telling lane 0 of the launch's last wave out (stamped harness).
  __device__ __forceinline__ bool finish_last() {
    bool last = false;
    if (lane == 0) {
      uint32_t* const done = ticket + NC * kTicketStride;
      if (atomicAdd(done, 1u) == gridDim.x * gridDim.y * (blockDim.x >> 6) - 1) {
        last = true;
#pragma unroll
        for (int q = 0; q < NC; ++q) atomicExch(ticket + q * kTicketStride, 0u);
        atomicExch(done, 0u);
      }
    }
    return last;
  }
};

// First tile of unit u (group u / 4, sub u % 4) of a C-tile-unit walk, and
// the units of an object of `ntiles` tiles walked with `spread` segments
// (TicketWalk's numbering: every (group, sub) pair, empty ones included).
template <int C>
__host__ __device__ __forceinline__ uint32_t unit_tile_base(uint32_t u) {
  return (u / 4) * (4 * C) + u % 4;
}
template <int C>
__host__ __device__ inline uint32_t walk_units(uint32_t ntiles, uint32_t spread) {
  const uint32_t s = spread ? spread : 1;
  const uint32_t groups = (ntiles + 4 * C - 1) / (4 * C);
  return s * ((groups + s - 1) / s) * 4;
}

// A static walk over a device-built list of units (entries obj * units +
// unit, `*count` of them): wave w takes entries w, w + nwaves, ...  Same
// interface as TicketWalk, for kernels that redo a chosen subset of a
// TicketWalk launch's units.
template <int C>
struct ListWalk {
  const uint32_t* list;
  uint32_t n, e, step, units, ntiles;
  uint32_t obj = 0, tb = 0, cnt = 0, i = 0;
  bool live = true;
  __device__ __forceinline__ ListWalk(const uint32_t* list_, uint32_t n_, uint32_t first, uint32_t step_,
                                      uint32_t units_, uint32_t ntiles_)
      : list(list_), n(n_), e(first - step_), step(step_), units(units_), ntiles(ntiles_) {
    next_unit();
  }
  __device__ __forceinline__ void next_unit() {
    for (;;) {
      e += step;
      if (e >= n) {
        live = false;
        return;
      }
      const uint32_t v = list[e];
      obj = v / units;
      tb = unit_tile_base<C>(v % units);
      i = 0;
      cnt = tb < ntiles ? (ntiles - tb + 3) / 4 : 0;
      if (cnt > C) cnt = C;
      if (cnt) return;
    }
  }
  __device__ __forceinline__ uint32_t tile() const { return tb + 4 * i; }
  __device__ __forceinline__ void advance() {
    if (++i >= cnt) next_unit();
  }
};

// STAMP 2: the time a wave enters its 4th, 16th and 64th tile (0 if never).
__device__ __forceinline__ void stamp_milestone(uint32_t walked, uint64_t (&t_at)[3]) {
  if (walked == 4 || walked == 16 || walked == 64) t_at[walked == 4 ? 0 : walked == 16 ? 1 : 2] =
      __builtin_amdgcn_s_memrealtime();
}

// Tuning-harness knobs (the product uses TB = 1, STAMP = 0): TB tickets per
// atomic (a wave takes TB consecutive units at a time); STAMP 1 records per
// wave {start, end, XCD | tiles << 32} (s_memrealtime ticks, 100 MHz) into
// `stamps`; STAMP 2 records 8 words {start, first tile's loads issued, tile
// 4 entered, tile 16 entered, tile 64 entered, last tile's stores issued,
// those stores retired (s_waitcnt 0), exit counted (finish)} and a ninth,
// XCD | tiles << 32 | last-out flag << 63 -- the launch's fixed costs apart
// (tools/c2_stamps.py).
template <int K, int U, int C, int NC, bool NTL, bool NTS, int TB = 1, int STAMP = 0, bool SYNC = false>
__global__ __launch_bounds__(kBlock) void rs_apply_queue_kernel(
    const uint32_t* __restrict__ in, uint32_t* __restrict__ out, uint64_t in_obj_stride, uint64_t in_shard,
    uint64_t out_obj_stride, uint64_t out_shard, const uint32_t* __restrict__ coeff,
    const uint32_t* __restrict__ in_idx, const uint32_t* __restrict__ out_idx, uint64_t ncols, uint32_t nobj,
    uint32_t rows, uint32_t k, uint32_t* __restrict__ ticket, uint64_t* __restrict__ stamps, uint32_t spread) {
  static_assert(K > 0 && NC > 0 && NC <= 64 && TB >= 1, "compile-time k only");
  uint64_t t_start = 0, t_walk = 0, t_issued = 0, t_retired = 0, t_at[3] = {0, 0, 0};
  uint32_t walked = 0;
  if constexpr (STAMP > 0) t_start = __builtin_amdgcn_s_memrealtime();
  // Host guarantees: ncols < 2^30 (32-bit byte offsets), nobj * 4 * groups < 2^32.
  const uint32_t nvec = (uint32_t)(ncols >> 2);
  const uint32_t ntiles = (nvec + 64 * U - 1) / (64 * U);
  const uint32_t lane = threadIdx.x & 63;
  uint64_t ioff[K];
#pragma unroll
  for (int j = 0; j < K; ++j) ioff[j] = (uint64_t)in_idx[j] * in_shard;
  TicketWalk<C, NC, TB, SYNC> w(ticket, nobj, ntiles, lane, spread);
  auto load = [&](uint4(&x)[U][K], uint32_t o, uint32_t t) {
    const uint32_t* base = in + (uint64_t)o * in_obj_stride;
    const uint32_t* sb[K];
#pragma unroll
    for (int j = 0; j < K; ++j) sb[j] = base + ioff[j];
    load_tile<K, U, NTL>(x, sb, t * (64 * U) + lane, nvec);
  };
  auto store = [&](const uint4(&x)[U][K], uint32_t o, uint32_t t) {
    store_tile<K, U, NTS>(x, out + (uint64_t)o * out_obj_stride, coeff, out_idx, out_shard, rows, t * (64 * U) + lane,
                          nvec);
  };
  if (w.live) {
    uint4 xa[U][K], xb[U][K];
    load(xa, w.obj, w.tile());
    if constexpr (STAMP > 1) t_walk = __builtin_amdgcn_s_memrealtime();
    for (;;) {
      uint32_t co = w.obj, ct = w.tile();
      if constexpr (STAMP > 0) ++walked;
      if constexpr (STAMP > 1) stamp_milestone(walked, t_at);
      w.advance();
      // Past the last unit the prefetch re-reads the current tile (unconditional loads, see load_tile).
      load(xb, w.live ? w.obj : co, w.live ? w.tile() : ct);
      store(xa, co, ct);
      if (!w.live) break;
      co = w.obj;
      ct = w.tile();
      if constexpr (STAMP > 0) ++walked;
      if constexpr (STAMP > 1) stamp_milestone(walked, t_at);
      w.advance();
      load(xa, w.live ? w.obj : co, w.live ? w.tile() : ct);
      store(xb, co, ct);
      if (!w.live) break;
    }
  }
  if constexpr (STAMP > 1) {
    t_issued = __builtin_amdgcn_s_memrealtime();
    __builtin_amdgcn_s_waitcnt(0);  // every load and store of the walk retired
    t_retired = __builtin_amdgcn_s_memrealtime();
  }
  bool last_out = false;
  if constexpr (STAMP > 1) {
    last_out = w.finish_last();
  } else {
    w.finish();
  }
  if constexpr (STAMP == 1) {
    const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
      uint64_t* r = stamps + 3 * ((uint64_t)blockIdx.x * kWaves + (threadIdx.x >> 6));
      r[0] = t_start;
      r[1] = t_end;
      r[2] = hw_xcc_id() | ((uint64_t)walked << 32);
    }
  }
  if constexpr (STAMP > 1) {
    __builtin_amdgcn_s_waitcnt(0);  // the exit count (and, last out, the counter reset) retired
    const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
      uint64_t* r = stamps + 9 * ((uint64_t)blockIdx.x * kWaves + (threadIdx.x >> 6));
      r[0] = t_start;
      r[1] = t_walk ? t_walk : t_start;
      r[2] = t_at[0];
      r[3] = t_at[1];
      r[4] = t_at[2];
      r[5] = t_issued;
      r[6] = t_retired;
      r[7] = t_end;
      r[8] = hw_xcc_id() | ((uint64_t)walked << 32) | ((uint64_t)last_out << 63);
    }
  }
  // Columns past the last whole vector of each object, one per lane.
  const uint32_t tailc = (uint32_t)(ncols - ((uint64_t)nvec << 2));
  if (tailc) {
    const uint64_t tid = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    const uint64_t nthr = (uint64_t)gridDim.x * kBlock;
    for (uint64_t t = tid; t < (uint64_t)nobj * tailc; t += nthr) {
      const uint64_t o = t / tailc;
      apply_column<K>(in + o * in_obj_stride, out + o * out_obj_stride, coeff, in_idx, in_shard, out_idx, out_shard,
                      rows, k, ((uint64_t)nvec << 2) + t % tailc);
    }
  }
}

// ---- wide k, software-pipelined ------------------------------------------
// A wave's work is a stream of items (tile, row block rb, input chunk jc):
// one 64-vector tile per step, row blocks of RB rows, chunks of 16 input
// shards.  Each item loads 16 vectors (shard indices past k are clamped to
// k-1; their coefficients are zero in the plan table) and MACs them into the
// row block's RB running residues (canonical 32-bit, one fold per chunk);
// the last chunk of a row block stores it.  The next item's 16 loads are
// issued before the current item's math (two register sets), so a wave
// always has a chunk in flight.  Row 0 of a block always exists and
// consumes every loaded register unconditionally (waitcnt, see
// rs_apply_pipe_kernel).
struct WideItem {
  uint32_t tile, rb, jc;  // tile: the wave's step index (< ntiles when valid)
};
__device__ __forceinline__ void wide_next(WideItem& it, uint32_t nch, uint32_t nrb, uint32_t nwaves) {
  if (++it.jc == nch) {
    it.jc = 0;
    if (++it.rb == nrb) {
      it.rb = 0;
      it.tile += nwaves;
    }
  }
}

// 16 input vectors of chunk jc at vector g (clamped to the segment).
template <bool NTL>
__device__ __forceinline__ void wide_load16(uint4 (&x)[16], const uint32_t* __restrict__ ib,
                                            const uint32_t* __restrict__ in_idx, uint64_t in_shard, uint32_t k,
                                            uint32_t jc, uint32_t g, uint32_t v1) {
  const uint32_t gc = g < v1 ? g : v1 - 1;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint32_t s = jc * 16 + j < k ? jc * 16 + j : k - 1;
    // An opaque wave-uniform shard base (readfirstlane), so the compiler
    // keeps it in SGPRs as the saddr operand instead of folding the lane
    // offset into a 64-bit VGPR address per load.
    const uint64_t base = (uint64_t)(ib + (uint64_t)in_idx[s] * in_shard);
    // (readfirstlane returns int: widen through uint32_t, no sign extension)
    const uint64_t ub = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(base >> 32)) << 32) |
                        (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)base);
    typedef const __attribute__((address_space(1))) u32x4 global_u32x4;
    const global_u32x4* gp = reinterpret_cast<const global_u32x4*>(ub + (uint64_t)(gc << 4));
    const u32x4 v = NTL ? __builtin_nontemporal_load(gp) : *gp;
    x[j] = make_uint4(v.x, v.y, v.z, v.w);
  }
}

// acc = (acc + sum_j c[j] * x[j]) mod p, exact, one fold.  MATH = false is
// the tuning harness's XOR stand-in (wrong results by design; see xor4).
template <bool MATH = true>
__device__ __forceinline__ void wide_mac16(const uint4 (&x)[16], const uint32_t* __restrict__ crow, uint4& acc) {
  const u32x16 c = *reinterpret_cast<const u32x16*>(crow);
  if constexpr (!MATH) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      acc.x ^= x[j].x + c[j];
      acc.y ^= x[j].y + c[j];
      acc.z ^= x[j].z + c[j];
      acc.w ^= x[j].w + c[j];
    }
    return;
  }
  uint64_t lo0 = acc.x, lo1 = acc.y, lo2 = acc.z, lo3 = acc.w;
  uint32_t hi0 = 0, hi1 = 0, hi2 = 0, hi3 = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) mac4(lo0, lo1, lo2, lo3, hi0, hi1, hi2, hi3, x[j].x, x[j].y, x[j].z, x[j].w, c[j]);
  acc = make_uint4(fold96(lo0, hi0), fold96(lo1, hi1), fold96(lo2, hi2), fold96(lo3, hi3));
}

// One item's math (and the row block's stores after its last chunk).
template <int RB, bool NTS, bool MATH = true>
__device__ __forceinline__ void wide_item(const uint4 (&x)[16], uint4 (&acc)[RB], const WideItem& it, uint32_t nch,
                                          uint32_t rows, uint32_t cs, const uint32_t* __restrict__ coeff,
                                          const uint32_t* __restrict__ out_idx, uint32_t* __restrict__ ob,
                                          uint64_t out_shard, uint32_t g, uint32_t v1) {
  if (it.jc == 0) {
#pragma unroll
    for (int i = 0; i < RB; ++i) acc[i] = make_uint4(0, 0, 0, 0);
  }
  const uint32_t r0 = it.rb * RB;
  const uint32_t* const c0 = coeff + (uint64_t)r0 * cs + it.jc * 16;
  wide_mac16<MATH>(x, c0, acc[0]);
#pragma unroll
  for (int i = 1; i < RB; ++i)
    if (r0 + i < rows) wide_mac16<MATH>(x, c0 + (uint64_t)i * cs, acc[i]);
  if (it.jc == nch - 1 && g < v1) {
#pragma unroll
    for (int i = 0; i < RB; ++i)
      if (r0 + i < rows)
        st16<NTS>(reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(ob + (uint64_t)out_idx[r0 + i] * out_shard) +
                                              ((uint64_t)g << 4)),
                  acc[i]);
  }
}

template <int RB, bool NTL, bool NTS, bool MATH = true>
__global__ __launch_bounds__(kBlock) void rs_apply_wide_pipe_kernel(
    const uint32_t* __restrict__ in, uint32_t* __restrict__ out, uint64_t in_obj_stride, uint64_t in_shard,
    uint64_t out_obj_stride, uint64_t out_shard, const uint32_t* __restrict__ coeff,
    const uint32_t* __restrict__ in_idx, const uint32_t* __restrict__ out_idx, uint64_t ncols, uint32_t nobj,
    uint32_t rows, uint32_t k, uint32_t nseg) {
  const uint32_t cs = wide_coeff_stride(k);
  const uint32_t nch = (k + 15) / 16, nrb = (rows + RB - 1) / RB;
  const uint64_t tid = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const uint64_t nthr = (uint64_t)gridDim.x * kBlock;
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
    const uint32_t v0 = seg * seg_vec < nvec ? seg * seg_vec : nvec;
    const uint32_t v1 = nvec - v0 > seg_vec ? v0 + seg_vec : nvec;
    const uint32_t ntiles = (v1 - v0 + 63) / 64;
    uint4 xa[16], xb[16], acc[RB];
    WideItem it{wave, 0, 0};
    if (it.tile < ntiles) wide_load16<NTL>(xa, ib, in_idx, in_shard, k, it.jc, v0 + it.tile * 64 + lane, v1);
    while (it.tile < ntiles) {
      WideItem nx = it;
      wide_next(nx, nch, nrb, nwaves);
      const WideItem& ld = nx.tile < ntiles ? nx : it;
      wide_load16<NTL>(xb, ib, in_idx, in_shard, k, ld.jc, v0 + ld.tile * 64 + lane, v1);
      wide_item<RB, NTS, MATH>(xa, acc, it, nch, rows, cs, coeff, out_idx, ob, out_shard, v0 + it.tile * 64 + lane, v1);
      it = nx;
      if (it.tile >= ntiles) break;
      nx = it;
      wide_next(nx, nch, nrb, nwaves);
      const WideItem& ld2 = nx.tile < ntiles ? nx : it;
      wide_load16<NTL>(xa, ib, in_idx, in_shard, k, ld2.jc, v0 + ld2.tile * 64 + lane, v1);
      wide_item<RB, NTS, MATH>(xb, acc, it, nch, rows, cs, coeff, out_idx, ob, out_shard, v0 + it.tile * 64 + lane, v1);
      it = nx;
    }
    if (seg == nseg - 1)
      for (uint64_t b = ((uint64_t)nvec << 2) + tid; b < ncols; b += nthr)
        apply_column<0>(ib, ob, coeff, in_idx, in_shard, out_idx, out_shard, rows, k, b);
  }
}

// Wide k (k > 16, up to the reference's 100 shards): the same 4-columns-per-
// lane streaming as rs_apply_kernel, with the inputs taken in chunks of 16
// shards and the outputs in blocks of up to RB rows.  Per row and column the
// running value is a canonical 32-bit residue: each chunk's 16 products are
// accumulated exactly on top of it (96-bit, gfp.hpp) and folded once, so a
// block of RB rows costs 4 VGPRs per row instead of 12.  Inputs are read once
// per row block: once in all for rows <= RB.
//
// KC (16 or 32) is the chunk width: KC = 32 holds all inputs of a k <= 32
// code in registers at once (one HBM round trip per step), KC = 16 keeps the
// register budget for 16-row blocks at larger k.
template <int KC, int RB, bool NTL, bool NTS>
__global__ __launch_bounds__(kBlock) void rs_apply_wide_kernel(
    const uint32_t* __restrict__ in, uint32_t* __restrict__ out, uint64_t in_obj_stride, uint64_t in_shard,
    uint64_t out_obj_stride, uint64_t out_shard, const uint32_t* __restrict__ coeff,
    const uint32_t* __restrict__ in_idx, const uint32_t* __restrict__ out_idx, uint64_t ncols, uint32_t nobj,
    uint32_t rows, uint32_t k, uint32_t nseg) {
  static_assert(KC % 16 == 0, "chunks are whole 16-coefficient loads");
  const uint32_t cs = wide_coeff_stride(k);
  const uint64_t tid = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const uint64_t nthr = (uint64_t)gridDim.x * kBlock;
  const uint64_t nvec = ncols >> 2;
  const uint64_t seg_vec = segment_vectors(nvec, nseg);
  const uint64_t nwork = (uint64_t)nobj * nseg;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  const uint64_t nwaves = (uint64_t)gridDim.x * kWaves;
  for (uint64_t wi = blockIdx.y; wi < nwork; wi += gridDim.y) {
    const uint64_t obj = wi / nseg, seg = wi % nseg;
    const uint32_t* __restrict__ ib = in + obj * in_obj_stride;
    uint32_t* __restrict__ ob = out + obj * out_obj_stride;
    const uint64_t v0 = seg * seg_vec < nvec ? seg * seg_vec : nvec;
    const uint64_t v1 = v0 + seg_vec < nvec ? v0 + seg_vec : nvec;
    for (uint64_t g = v0 + wave * 64 + lane; g - lane < v1; g += nwaves * 64) {
      const bool valid = g < v1;
      const uint64_t b = g << 2;
      for (uint32_t r0 = 0; r0 < rows; r0 += RB) {
        uint32_t acc[RB][4];
#pragma unroll
        for (int i = 0; i < RB; ++i) acc[i][0] = acc[i][1] = acc[i][2] = acc[i][3] = 0;
        for (uint32_t j0 = 0; j0 < k; j0 += KC) {
          uint4 x[KC];
#pragma unroll
          for (int j = 0; j < KC; ++j)
            x[j] = valid && j0 + j < k ? ld16<NTL>(ib + (uint64_t)in_idx[j0 + j] * in_shard + b) : make_uint4(0, 0, 0, 0);
#pragma unroll
          for (int i = 0; i < RB; ++i) {
            if (r0 + i < rows) {
              // Padding coefficients past k are zero (plan table), so the
              // whole chunk runs unconditionally.
              uint64_t lo0 = acc[i][0], lo1 = acc[i][1], lo2 = acc[i][2], lo3 = acc[i][3];
              uint32_t hi0 = 0, hi1 = 0, hi2 = 0, hi3 = 0;
#pragma unroll
              for (int h = 0; h < KC; h += 16) {
                if (j0 + h < k) {
                  const u32x16 c = *reinterpret_cast<const u32x16*>(coeff + (uint64_t)(r0 + i) * cs + j0 + h);
#pragma unroll
                  for (int j = 0; j < 16; ++j)
                    mac4(lo0, lo1, lo2, lo3, hi0, hi1, hi2, hi3, x[h + j].x, x[h + j].y, x[h + j].z, x[h + j].w,
                         c[j]);
                }
              }
              acc[i][0] = fold96(lo0, hi0);
              acc[i][1] = fold96(lo1, hi1);
              acc[i][2] = fold96(lo2, hi2);
              acc[i][3] = fold96(lo3, hi3);
            }
          }
        }
        if (valid) {
#pragma unroll
          for (int i = 0; i < RB; ++i)
            if (r0 + i < rows)
              st16<NTS>(ob + (uint64_t)out_idx[r0 + i] * out_shard + b,
                        make_uint4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]));
        }
      }
    }
    if (seg == nseg - 1)
      for (uint64_t b = (nvec << 2) + tid; b < ncols; b += nthr)
        apply_column<0>(ib, ob, coeff, in_idx, in_shard, out_idx, out_shard, rows, k, b);
  }
}

}  // namespace apply
}  // namespace slime
