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

template <int KS, bool NTL>
__device__ __forceinline__ void mfma_load_tile(uint4 (&x)[KS][4], const char* __restrict__ ib,
                                               const uint32_t (&soff)[KS][4], uint32_t colb, uint32_t lim) {
#pragma unroll
  for (int q = 0; q < KS; ++q)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj)
      x[q][jj] = soff[q][jj] != 0xFFFFFFFFu
                     ? ld16<NTL>(reinterpret_cast<const uint32_t*>(ib + (uint32_t)(soff[q][jj] + colb)))
                     : make_uint4(0, 0, 0, 0);
  (void)lim;
}

// One tile's math and stores: x holds the raw words, lane's output column
// vector at byte offset colb (store only if `store`).
template <int KS, bool NTS>
__device__ __forceinline__ void mfma_tile(const uint4 (&x)[KS][4], const i32x4* __restrict__ lfrag,
                                          const uint64_t* __restrict__ lrowc, const uint32_t* __restrict__ loff,
                                          uint32_t MT, uint32_t rows, uint32_t lane, uint32_t g, char* __restrict__ ob,
                                          uint32_t colb, bool store) {
  for (uint32_t mb = 0; mb < MT; mb += 4) {
    i32x4 acc[4][4];
#pragma unroll
    for (int mm = 0; mm < 4; ++mm)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[mm][c] = i32x4{0, 0, 0, 0};
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
#pragma unroll
      for (int mm = 0; mm < 4; ++mm) {
        if (mb + mm < MT) {
          const i32x4 a = lfrag[((mb + mm) * KS + q) * 64 + lane];
#pragma unroll
          for (int c = 0; c < 4; ++c) acc[mm][c] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b[c], acc[mm][c], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int mm = 0; mm < 4; ++mm) {
      const uint32_t i = 4 * (mb + mm) + g;
      if (mb + mm < MT && i < rows && store) {
        const uint64_t R = lrowc[i];
        uint32_t r[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const i32x4 d = acc[mm][c];
          const int64_t v = (int64_t)d[0] + ((int64_t)d[1] << 8) + ((int64_t)d[2] << 16) + ((int64_t)d[3] << 24);
          r[c] = fold96(R + (uint64_t)v, 0);
        }
        st16<NTS>(reinterpret_cast<uint32_t*>(ob + (uint32_t)(loff[i] + colb)), make_uint4(r[0], r[1], r[2], r[3]));
      }
    }
  }
}

// table: the plan's mfma table (mfma_table.hpp layout); coeff: the plan's
// coefficient rows (column tails); PIPE: the next tile's loads are issued
// before the current tile's math.
template <int KS, bool NTL, bool NTS, bool PIPE>
__global__ __launch_bounds__(kBlock) void rs_apply_mfma_kernel(
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
      soff[q][jj] = j < k ? (uint32_t)(in_idx[j] * in_shard * 4) : 0xFFFFFFFFu;
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
    if constexpr (PIPE) {
      uint4 xa[KS][4], xb[KS][4];
      uint32_t t = wave;
      auto colb_of = [&](uint32_t tile) {
        const uint32_t v = v0 + tile * 16 + n;
        return (v < v1 ? v : v1 - 1) << 4;
      };
      if (t < ntiles) mfma_load_tile<KS, NTL>(xa, ib, soff, colb_of(t), 0);
      while (t < ntiles) {
        const uint32_t t1 = t + nwaves;
        mfma_load_tile<KS, NTL>(xb, ib, soff, colb_of(t1 < ntiles ? t1 : t), 0);
        mfma_tile<KS, NTS>(xa, lds, lrowc, loff, MT, rows, lane, g, ob, colb_of(t), v0 + t * 16 + n < v1);
        t = t1;
        if (t >= ntiles) break;
        const uint32_t t2 = t + nwaves;
        mfma_load_tile<KS, NTL>(xa, ib, soff, colb_of(t2 < ntiles ? t2 : t), 0);
        mfma_tile<KS, NTS>(xb, lds, lrowc, loff, MT, rows, lane, g, ob, colb_of(t), v0 + t * 16 + n < v1);
        t = t2;
      }
    } else {
      for (uint32_t t = wave; t < ntiles; t += nwaves) {
        const uint32_t v = v0 + t * 16 + n;
        const uint32_t colb = (v < v1 ? v : v1 - 1) << 4;
        uint4 x[KS][4];
        mfma_load_tile<KS, NTL>(x, ib, soff, colb, 0);
        mfma_tile<KS, NTS>(x, lds, lrowc, loff, MT, rows, lane, g, ob, colb, v < v1);
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
