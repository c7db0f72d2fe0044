// Matrix-core form of the GF(2^32-5) shard-matrix apply (applyMatrix,
// internal/rs/vector.go:90-102) for wide codes: the exact int8-limb identity
// of mfma_table.hpp evaluated with v_mfma_i32_16x16x64_i8.
//
// Why: the VALU kernels spend 2 instructions per multiply-accumulate (exact
// 96-bit MAC, gfp.hpp), so at 64/80 a column costs 2048 lane-ops and the
// kernel is VALU-bound at 0.43 of the HBM roofline.  Here the k x rows
// products of a column are MFMA work (16 shards x 4 bytes x 16 (row, digit)
// pairs per instruction, about 14% of the matrix cores at the HBM rate) and
// the VALU does one XOR per loaded word plus an in-lane recombination and
// fold per output symbol.
//
// Wave tile: 64 consecutive columns of one object segment.  Lane l (group
// g = l >> 4, n = l & 15) loads 16 B (columns 4n..4n+3 of the tile) of the
// shards 16q + 4g + jj, jj = 0..3, for every K step q: one load instruction
// reads 256 contiguous bytes of each of 4 shards.  Component c of those four
// vectors, XORed with 0x80808080, is the lane's B fragment of N tile c (its
// column 4n + c), so an N tile is the columns = c (mod 4) and the D fragment
// of (M tile m, N tile c) gives the lane output row 4m + g, column 4n + c.
// After the four N tiles the lane holds 16 B of one output row: one store
// instruction writes 256 contiguous bytes of each of 4 rows.  A fragments
// (the plan's digit table) and the row constants sit in LDS for the block.
// Addressing: a wave-uniform 64-bit object base plus 32-bit per-lane byte
// offsets (the launcher checks that every object spans under 4 GiB).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mfma_table.hpp"
#include "rs_apply_kernel.hpp"

namespace slime {
namespace apply {

typedef int32_t i32x4 __attribute__((ext_vector_type(4)));

// Dynamic LDS bytes of a launch: A fragments, row constants, output offsets.
__host__ __device__ constexpr uint32_t mfma_lds_bytes(uint32_t mt, uint32_t ks) {
  return mt * ks * mfma::kFragBytes + mt * 4 * (8 + 4);
}

#if defined(__HIP_DEVICE_COMPILE__)
// R + d0 + 2^8 d1 + 2^16 d2 + 2^24 d3 as a 64-bit integer (R carries the
// offset that keeps it positive): four v_mad_i64_i32, the constants in SGPRs
// (gfx9 VOP3 takes no literals).
__device__ __forceinline__ uint64_t mfma_recombine(const i32x4& d, uint64_t R) {
  uint64_t v = R, cc;
  asm("v_mad_i64_i32 %0, %1, %2, 1, %0" : "+v"(v), "=s"(cc) : "v"(d[0]));
  asm("v_mad_i64_i32 %0, %1, %2, %3, %0" : "+v"(v), "=s"(cc) : "v"(d[1]), "s"(256));
  asm("v_mad_i64_i32 %0, %1, %2, %3, %0" : "+v"(v), "=s"(cc) : "v"(d[2]), "s"(65536));
  asm("v_mad_i64_i32 %0, %1, %2, %3, %0" : "+v"(v), "=s"(cc) : "v"(d[3]), "s"(16777216));
  return v;
}
#else
__device__ uint64_t mfma_recombine(const i32x4& d, uint64_t R);
#endif

// Waves per SIMD the kernel is compiled for (registers permitting): two up
// to four K steps (k <= 64; the refill form then fits 256 VGPRs with the
// accumulators in VGPRs), one above (k <= 112 holds up to 112 data VGPRs).
__host__ __device__ constexpr int mfma_waves(int ks, int mode) { return ks <= (mode == 1 ? 2 : 4) ? 2 : 1; }

template <int KS, bool NTL>
__device__ __forceinline__ void mfma_load_tile(uint4 (&x)[KS][4], const char* __restrict__ ib,
                                               const uint32_t (&soff)[KS][4], uint32_t colb, uint32_t lim) {
#pragma unroll
  for (int q = 0; q < KS; ++q)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj)
      x[q][jj] = ld16<NTL>(reinterpret_cast<const uint32_t*>(ib + (uint32_t)(soff[q][jj] + colb)));
  (void)lim;
}

// One row block (M tiles mb..mb+3) of a tile: the MFMAs over every K step,
// then the recombination, fold and store of the lane's output vector (byte
// offset colb; only if `store`).  REFILL: after K step q's B fragments are
// built, x[q] is reloaded with the next tile's vectors (byte offset colbn), so
// the next tile streams in one K step at a time behind the math and the wave
// holds one tile of data registers instead of two.
template <int KS, bool NTL, bool NTS, bool REFILL>
__device__ __forceinline__ void mfma_rows(uint4 (&x)[KS][4], const char* __restrict__ ib,
                                          const uint32_t (&soff)[KS][4], uint32_t colbn,
                                          const i32x4* __restrict__ lfrag, const uint64_t* __restrict__ lrowc,
                                          const uint32_t* __restrict__ loff, uint32_t mb, uint32_t MT, uint32_t rows,
                                          uint32_t lane, uint32_t g, char* __restrict__ ob, uint32_t colb, bool store) {
  i32x4 acc[4][4];
#pragma unroll
  for (int q = 0; q < KS; ++q) {
    // B fragments of K step q: b[c] = the lane's four shards at column
    // 4n+c, each byte XOR 0x80 (u - 128 as int8).
    i32x4 b[4];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      b[0][jj] = (int)(x[q][jj].x ^ 0x80808080u);
      b[1][jj] = (int)(x[q][jj].y ^ 0x80808080u);
      b[2][jj] = (int)(x[q][jj].z ^ 0x80808080u);
      b[3][jj] = (int)(x[q][jj].w ^ 0x80808080u);
    }
    if constexpr (REFILL) {
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
        x[q][jj] = ld16<NTL>(reinterpret_cast<const uint32_t*>(ib + (uint32_t)(soff[q][jj] + colbn)));
    }
#pragma unroll
    for (int mm = 0; mm < 4; ++mm) {
      if (mb + mm < MT) {
        const i32x4 a = lfrag[((mb + mm) * KS + q) * 64 + lane];
#pragma unroll
        for (int c = 0; c < 4; ++c)
          acc[mm][c] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b[c], q == 0 ? i32x4{0, 0, 0, 0} : acc[mm][c], 0, 0, 0);
      }
    }
    // Keep step q's refill loads in step q: scheduled all at the top they
    // would double the live data registers (and halve the occupancy).
    if constexpr (REFILL) __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int mm = 0; mm < 4; ++mm) {
    const uint32_t i = 4 * (mb + mm) + g;
    if (mb + mm < MT && i < rows && store) {
      const uint64_t R = lrowc[i];
      uint32_t r[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        r[c] = fold96(mfma_recombine(acc[mm][c], R), 0);
      }
      st16<NTS>(reinterpret_cast<uint32_t*>(ob + (uint32_t)(loff[i] + colb)), make_uint4(r[0], r[1], r[2], r[3]));
    }
  }
}

// One tile: every row block; with REFILL the last one reloads x with the
// next tile.
template <int KS, bool NTL, bool NTS, bool REFILL>
__device__ __forceinline__ void mfma_tile(uint4 (&x)[KS][4], const char* __restrict__ ib,
                                          const uint32_t (&soff)[KS][4], uint32_t colbn,
                                          const i32x4* __restrict__ lfrag, const uint64_t* __restrict__ lrowc,
                                          const uint32_t* __restrict__ loff, uint32_t MT, uint32_t rows, uint32_t lane,
                                          uint32_t g, char* __restrict__ ob, uint32_t colb, bool store) {
  uint32_t mb = 0;
  for (; mb + 4 < MT; mb += 4)
    mfma_rows<KS, NTL, NTS, false>(x, ib, soff, colbn, lfrag, lrowc, loff, mb, MT, rows, lane, g, ob, colb, store);
  mfma_rows<KS, NTL, NTS, REFILL>(x, ib, soff, colbn, lfrag, lrowc, loff, mb, MT, rows, lane, g, ob, colb, store);
}

// table: the plan's mfma table (mfma_table.hpp layout); coeff: the plan's
// coefficient rows (column tails).  MODE 0: load a tile, compute it; 1: two
// tile buffers, the next tile's loads issued before the current tile's math;
// 2: one tile buffer refilled K step by K step behind the math (mfma_rows).
template <int KS, bool NTL, bool NTS, int MODE>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(mfma_waves(KS, MODE)))) void rs_apply_mfma_kernel(
    const uint32_t* __restrict__ in, uint32_t* __restrict__ out, uint64_t in_obj_stride, uint64_t in_shard,
    uint64_t out_obj_stride, uint64_t out_shard, const uint8_t* __restrict__ table, const uint32_t* __restrict__ coeff,
    const uint32_t* __restrict__ in_idx, const uint32_t* __restrict__ out_idx, uint64_t ncols, uint32_t nobj,
    uint32_t rows, uint32_t k, uint32_t nseg) {
  extern __shared__ i32x4 lds[];
  const uint32_t MT = (rows + 3) / 4;
  const uint32_t nfrag = MT * KS * 64;
  {
    const i32x4* gfrag = reinterpret_cast<const i32x4*>(table);
    for (uint32_t f = threadIdx.x; f < nfrag; f += kBlock) lds[f] = gfrag[f];
  }
  uint64_t* lrowc = reinterpret_cast<uint64_t*>(lds + nfrag);
  uint32_t* loff = reinterpret_cast<uint32_t*>(lrowc + MT * 4);
  {
    const uint64_t* growc = reinterpret_cast<const uint64_t*>(table + (size_t)nfrag * 16);
    for (uint32_t i = threadIdx.x; i < MT * 4; i += kBlock) {
      lrowc[i] = i < rows ? growc[i] : 0;
      loff[i] = i < rows ? (uint32_t)(out_idx[i] * out_shard * 4) : 0;
    }
  }
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, g = lane >> 4, n = lane & 15;
  uint32_t soff[KS][4];
#pragma unroll
  for (int q = 0; q < KS; ++q)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const uint32_t j = 16 * q + 4 * g + jj;
      // Shards past k: their digits are zero, so any real shard will do --
      // in_idx[k-1], whose lines the lanes of shard k-1 fetch anyway.
      soff[q][jj] = (uint32_t)(in_idx[j < k ? j : k - 1] * in_shard * 4);
    }
  const uint64_t tid = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const uint64_t nthr = (uint64_t)gridDim.x * kBlock;
  const uint32_t nvec = (uint32_t)(ncols >> 2);
  const uint32_t seg_vec = segment_vectors(nvec, nseg);
  const uint64_t nwork = (uint64_t)nobj * nseg;
  const uint32_t wave = blockIdx.x * kWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nwaves = gridDim.x * kWaves;
  for (uint64_t wi = blockIdx.y; wi < nwork; wi += gridDim.y) {
    const uint64_t obj = wi / nseg;
    const uint32_t seg = (uint32_t)(wi % nseg);
    const char* __restrict__ ib = reinterpret_cast<const char*>(in + obj * in_obj_stride);
    char* __restrict__ ob = reinterpret_cast<char*>(out + obj * out_obj_stride);
    const uint32_t v0 = seg * seg_vec < nvec ? seg * seg_vec : nvec;
    const uint32_t v1 = nvec - v0 > seg_vec ? v0 + seg_vec : nvec;
    const uint32_t ntiles = (v1 - v0 + 15) / 16;
    auto colb_of = [&](uint32_t tile) {
      const uint32_t v = v0 + tile * 16 + n;
      return (v < v1 ? v : v1 - 1) << 4;
    };
    if constexpr (MODE == 1) {
      uint4 xa[KS][4], xb[KS][4];
      uint32_t t = wave;
      if (t < ntiles) mfma_load_tile<KS, NTL>(xa, ib, soff, colb_of(t), 0);
      while (t < ntiles) {
        const uint32_t t1 = t + nwaves;
        mfma_load_tile<KS, NTL>(xb, ib, soff, colb_of(t1 < ntiles ? t1 : t), 0);
        mfma_tile<KS, NTL, NTS, false>(xa, ib, soff, 0, lds, lrowc, loff, MT, rows, lane, g, ob, colb_of(t),
                                       v0 + t * 16 + n < v1);
        t = t1;
        if (t >= ntiles) break;
        const uint32_t t2 = t + nwaves;
        mfma_load_tile<KS, NTL>(xa, ib, soff, colb_of(t2 < ntiles ? t2 : t), 0);
        mfma_tile<KS, NTL, NTS, false>(xb, ib, soff, 0, lds, lrowc, loff, MT, rows, lane, g, ob, colb_of(t),
                                       v0 + t * 16 + n < v1);
        t = t2;
      }
    } else if constexpr (MODE == 2) {
      uint4 x[KS][4];
      uint32_t t = wave;
      if (t < ntiles) mfma_load_tile<KS, NTL>(x, ib, soff, colb_of(t), 0);
      while (t < ntiles) {
        const uint32_t tn = t + nwaves;
        if (tn < ntiles)
          mfma_tile<KS, NTL, NTS, true>(x, ib, soff, colb_of(tn), lds, lrowc, loff, MT, rows, lane, g, ob, colb_of(t),
                                        v0 + t * 16 + n < v1);
        else
          mfma_tile<KS, NTL, NTS, false>(x, ib, soff, 0, lds, lrowc, loff, MT, rows, lane, g, ob, colb_of(t),
                                         v0 + t * 16 + n < v1);
        t = tn;
      }
    } else {
      for (uint32_t t = wave; t < ntiles; t += nwaves) {
        uint4 x[KS][4];
        mfma_load_tile<KS, NTL>(x, ib, soff, colb_of(t), 0);
        mfma_tile<KS, NTL, NTS, false>(x, ib, soff, 0, lds, lrowc, loff, MT, rows, lane, g, ob, colb_of(t),
                                       v0 + t * 16 + n < v1);
      }
    }
    if (seg == nseg - 1)
      for (uint64_t b = ((uint64_t)nvec << 2) + tid; b < ncols; b += nthr)
        apply_column<0>(reinterpret_cast<const uint32_t*>(ib), reinterpret_cast<uint32_t*>(ob), coeff, in_idx,
                        in_shard, out_idx, out_shard, rows, k, b);
  }
}

}  // namespace apply
}  // namespace slime
