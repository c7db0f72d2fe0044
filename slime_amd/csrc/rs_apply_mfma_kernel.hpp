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
// Wave tile: 16 W consecutive columns of one object segment (W = 4; the
// byte encodes above k = 80 use 2, mfma_width).  Lane l (group g = l >> 4,
// n = l & 15) loads 4W bytes (columns nW..nW+W-1 of the tile) of the shards
// 16q + 4g + jj, jj = 0..3, for every K step q: one load instruction reads
// 64W contiguous bytes of each of 4 shards.  Component c of those four
// vectors, XORed with 0x80808080, is the lane's B fragment of N tile c (its
// column nW + c), so an N tile is the columns = c (mod W) and the D fragment
// of (M tile m, N tile c) gives the lane output row 4m + g, column nW + c.
// After the W N tiles the lane holds 4W bytes of one output row: one store
// instruction writes 64W contiguous bytes of each of 4 rows.  A fragments
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
// Four outputs' recombinations in one statement, interleaved digit by digit
// (four independent multiply-add chains back to back instead of one chain at
// a time, and one wait-state pad per statement instead of one per mad).
__device__ __forceinline__ void mfma_recombine4(const i32x4& d0, const i32x4& d1, const i32x4& d2, const i32x4& d3,
                                                uint64_t R, uint64_t (&v)[4]) {
  v[0] = v[1] = v[2] = v[3] = R;
  asm("v_mad_i64_i32 %0, vcc, %4, 1, %0\n\t"
      "v_mad_i64_i32 %1, vcc, %5, 1, %1\n\t"
      "v_mad_i64_i32 %2, vcc, %6, 1, %2\n\t"
      "v_mad_i64_i32 %3, vcc, %7, 1, %3\n\t"
      "v_mad_i64_i32 %0, vcc, %8, %20, %0\n\t"
      "v_mad_i64_i32 %1, vcc, %9, %20, %1\n\t"
      "v_mad_i64_i32 %2, vcc, %10, %20, %2\n\t"
      "v_mad_i64_i32 %3, vcc, %11, %20, %3\n\t"
      "v_mad_i64_i32 %0, vcc, %12, %21, %0\n\t"
      "v_mad_i64_i32 %1, vcc, %13, %21, %1\n\t"
      "v_mad_i64_i32 %2, vcc, %14, %21, %2\n\t"
      "v_mad_i64_i32 %3, vcc, %15, %21, %3\n\t"
      "v_mad_i64_i32 %0, vcc, %16, %22, %0\n\t"
      "v_mad_i64_i32 %1, vcc, %17, %22, %1\n\t"
      "v_mad_i64_i32 %2, vcc, %18, %22, %2\n\t"
      "v_mad_i64_i32 %3, vcc, %19, %22, %3"
      : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3])
      : "v"(d0[0]), "v"(d1[0]), "v"(d2[0]), "v"(d3[0]), "v"(d0[1]), "v"(d1[1]), "v"(d2[1]), "v"(d3[1]), "v"(d0[2]),
        "v"(d1[2]), "v"(d2[2]), "v"(d3[2]), "v"(d0[3]), "v"(d1[3]), "v"(d2[3]), "v"(d3[3]), "s"(256), "s"(65536),
        "s"(16777216)
      : "vcc");
}
#else
__device__ uint64_t mfma_recombine(const i32x4& d, uint64_t R);
__device__ void mfma_recombine4(const i32x4&, const i32x4&, const i32x4&, const i32x4&, uint64_t, uint64_t (&)[4]);
#endif

// Columns per lane of a tile: 4 at every K step count (16-byte loads; the
// byte encodes keep 2 above five K steps, rs_bytes_mfma.hip enc_width).
__host__ __device__ constexpr int mfma_width(int ks) { return ks <= 7 ? 4 : 2; }
// Waves per SIMD the matrix-core kernels are compiled for: two, and one from
// five K steps on, where four-column tiles' data (80-112 VGPRs) and
// accumulators (64) in one pass do not fit two -- one pass at one wave per
// SIMD beat two column passes at two (the refill then overlaps only the
// second pass) and two-column tiles: 80/100 encode 0.643 vs 0.618 / 0.625
// (tools/wide_variants, profiles/r05/s12_widevar/); 96/100, 90/100 and
// 100/116 encode and repair 2-7% faster than on two-column tiles
// (profiles/r05/s21_ks67/).
constexpr int kMfmaWaves = 2;
__host__ __device__ constexpr int mfma_waves(int ks, int w) { return ks >= 5 && w == 4 ? 1 : kMfmaWaves; }
// Column passes per K loop (mfma_rows): 2 where four-column tiles need their
// accumulators halved to fit two waves per SIMD.
__host__ __device__ constexpr int mfma_halves_at(int ks, int w, int waves) {
  return ks > 4 && w == 4 && waves == 2 ? 2 : 1;
}
__host__ __device__ constexpr int mfma_halves(int ks, int w) { return mfma_halves_at(ks, w, mfma_waves(ks, w)); }

template <int W>
using vec_t = uint32_t __attribute__((ext_vector_type(W)));

template <int W, bool NT>
__device__ __forceinline__ vec_t<W> ldw(const char* p) {
  if constexpr (NT)
    return __builtin_nontemporal_load(reinterpret_cast<const vec_t<W>*>(p));
  else
    return *reinterpret_cast<const vec_t<W>*>(p);
}
template <int W, bool NT>
__device__ __forceinline__ void stw(char* p, vec_t<W> v) {
  if constexpr (NT)
    __builtin_nontemporal_store(v, reinterpret_cast<vec_t<W>*>(p));
  else
    *reinterpret_cast<vec_t<W>*>(p) = v;
}

// A lane's input byte offsets (from the object's base) for shard 16q + 4g + jj
// of K step q.  General (decode: in_idx names the survivors): one per step and
// shard.  Uniform (in_idx null, shards in order: the encodes): steps before the
// last read step 0's shards 16q further on, so a step's address is a
// wave-uniform base (ib + q * step, scalar registers) plus step 0's four
// per-lane offsets; the last step keeps its own (shards past k read shard
// k-1, see mfma_prologue).
template <int KS, bool UNI>
struct ShardOffs {
  uint32_t o[KS][4];
  __device__ __forceinline__ void init(const uint32_t* __restrict__ in_idx, uint64_t in_unit, uint32_t k, uint32_t g) {
#pragma unroll
    for (int q = 0; q < KS; ++q)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const uint32_t j = 16 * q + 4 * g + jj;
        const uint32_t jc = j < k ? j : k - 1;
        o[q][jj] = (uint32_t)((in_idx ? in_idx[jc] : jc) * in_unit);
      }
  }
  __device__ __forceinline__ const char* at(const char* ib, int q, int jj, uint32_t colb) const {
    return ib + (uint32_t)(o[q][jj] + colb);
  }
};
template <int KS>
struct ShardOffs<KS, true> {
  uint32_t o0[4], ol[4];
  uint64_t step;  // 16 shards, in bytes
  __device__ __forceinline__ void init(const uint32_t* __restrict__, uint64_t in_unit, uint32_t k, uint32_t g) {
    step = 16 * in_unit;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const uint32_t j = 16 * (KS - 1) + 4 * g + jj;
      o0[jj] = (uint32_t)((4 * g + jj) * in_unit);
      ol[jj] = (uint32_t)((j < k ? j : k - 1) * in_unit);
    }
  }
  __device__ __forceinline__ const char* at(const char* ib, int q, int jj, uint32_t colb) const {
    if (q == KS - 1) return ib + (uint32_t)(ol[jj] + colb);
    return (ib + (uint64_t)q * step) + (uint32_t)(o0[jj] + colb);
  }
};

template <int KS, int W, bool NTL, class SO>
__device__ __forceinline__ void mfma_load_tile(vec_t<W> (&x)[KS][4], const char* __restrict__ ib, const SO& so,
                                               uint32_t colb) {
#pragma unroll
  for (int q = 0; q < KS; ++q)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) x[q][jj] = ldw<W, NTL>(so.at(ib, q, jj, colb));
}

// Hook run on every loaded vector of a tile before its B fragments are
// built (the byte encode folds MapToGF's flags there); the symbol path's is
// empty.
struct NoPre {
  template <class V>
  __device__ __forceinline__ void operator()(const V&) {}
};

// Per-launch word transforms: B fragments are (word ^ xin) as int8 bytes
// (xin = 0x80808080 for symbols: u - 128), outputs are stored as r ^ xout,
// byte-swapped when BSWAP (the byte path's big-endian chunk words).
struct MfmaIO {
  uint32_t xin, xout;
};

// One row block (M tiles mb..mb+3) of a tile: the MFMAs over every K step,
// then the recombination, fold and store of the lane's output vector (byte
// offset colb; only if `store`).  REFILL: after K step q's B fragments are
// built, x[q] is reloaded with the next tile's vectors (object base ibn, byte
// offset colbn), so
// the next tile streams in one K step at a time behind the math and the wave
// holds one tile of data registers instead of two.
template <int KS, int W, bool NTL, bool NTS, bool REFILL, bool BSWAP, class Pre, class SO,
          int NH = mfma_halves(KS, W)>
__device__ __forceinline__ void mfma_rows(vec_t<W> (&x)[KS][4], const char* __restrict__ ibn, const SO& so,
                                          uint32_t colbn,
                                          const i32x4* __restrict__ lfrag, const uint64_t* __restrict__ lrowc,
                                          const uint32_t* __restrict__ loff, uint32_t mb, uint32_t MT, uint32_t rows,
                                          uint32_t lane, uint32_t g, char* __restrict__ ob, uint32_t colb, bool store,
                                          MfmaIO io, Pre& pre) {
  // NH passes over the K steps, each for W / NH of the lane's columns (its
  // accumulators and B fragments shrink by NH; the A fragments are read NH
  // times from LDS); the results wait in `out` for one W-wide store per row.
  constexpr int CW = W / NH;
  uint32_t out[4][W];
#pragma unroll
  for (int h = 0; h < NH; ++h) {
    i32x4 acc[4][CW];
#pragma unroll
    for (int q = 0; q < KS; ++q) {
      // B fragments of K step q: b[c] = the lane's four shards at column nW + h CW + c.
      i32x4 b[CW];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        if (h == 0) pre(x[q][jj]);
#pragma unroll
        for (int c = 0; c < CW; ++c) b[c][jj] = (int)(x[q][jj][h * CW + c] ^ io.xin);
      }
      // (Refilling each pass's columns right after that pass -- half-width
      // loads -- ran 0.36 of peak against 0.62: profiles/r05/s12_widevar/.)
      if constexpr (REFILL) {
        if (h == NH - 1) {
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) x[q][jj] = ldw<W, NTL>(so.at(ibn, q, jj, colbn));
        }
      }
#pragma unroll
      for (int mm = 0; mm < 4; ++mm) {
        if (mb + mm < MT) {
          const i32x4 a = lfrag[((mb + mm) * KS + q) * 64 + lane];
#pragma unroll
          for (int c = 0; c < CW; ++c)
            acc[mm][c] =
                __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b[c], q == 0 ? i32x4{0, 0, 0, 0} : acc[mm][c], 0, 0, 0);
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
        if constexpr (CW == 4 && !BSWAP) {  // (the byte kernels' extra state leaves no room for it)
          uint64_t rv[4];
          mfma_recombine4(acc[mm][0], acc[mm][1], acc[mm][2], acc[mm][3], R, rv);
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const uint32_t v = fold96(rv[c], 0) ^ io.xout;
            out[mm][h * CW + c] = BSWAP ? __builtin_bswap32(v) : v;
          }
        } else {
#pragma unroll
          for (int c = 0; c < CW; ++c) {
            const uint32_t v = fold96(mfma_recombine(acc[mm][c], R), 0) ^ io.xout;
            out[mm][h * CW + c] = BSWAP ? __builtin_bswap32(v) : v;
          }
        }
      }
    }
  }
#pragma unroll
  for (int mm = 0; mm < 4; ++mm) {
    const uint32_t i = 4 * (mb + mm) + g;
    if (mb + mm < MT && i < rows && store) {
      vec_t<W> r;
#pragma unroll
      for (int c = 0; c < W; ++c) r[c] = out[mm][c];
      stw<W, NTS>(ob + (uint32_t)(loff[i] + colb), r);
    }
  }
}

// One tile: every row block, the first (a full block of four M tiles) last:
// with REFILL it reloads x with the next tile (object base ibn, byte offset
// colbn), behind the most matrix work (rows 17-20: one M tile in the other).
template <int KS, int W, bool NTL, bool NTS, bool REFILL, bool BSWAP, class Pre, class SO,
          int NH = mfma_halves(KS, W)>
__device__ __forceinline__ void mfma_tile(vec_t<W> (&x)[KS][4], const char* __restrict__ ibn, const SO& so,
                                          uint32_t colbn,
                                          const i32x4* __restrict__ lfrag, const uint64_t* __restrict__ lrowc,
                                          const uint32_t* __restrict__ loff, uint32_t MT, uint32_t rows, uint32_t lane,
                                          uint32_t g, char* __restrict__ ob, uint32_t colb, bool store, MfmaIO io,
                                          Pre& pre) {
  for (uint32_t mb = (MT - 1) & ~3u; mb > 0; mb -= 4)
    mfma_rows<KS, W, NTL, NTS, false, BSWAP, Pre, SO, NH>(x, ibn, so, colbn, lfrag, lrowc, loff, mb, MT, rows, lane, g,
                                                          ob, colb, store, io, pre);
  mfma_rows<KS, W, NTL, NTS, REFILL, BSWAP, Pre, SO, NH>(x, ibn, so, colbn, lfrag, lrowc, loff, 0, MT, rows, lane, g,
                                                         ob, colb, store, io, pre);
}

// The tile walk of one wave over columns [c0, c1) of one object (c0, c1
// multiples of W): tiles t = wave, wave + nwaves, ..., one tile buffer
// refilled K step by K step behind the math (mfma_rows).  The refill beat two
// tile buffers and no prefetch at every K step count (profiles/r03/
// s33_mfma_queue_bytes/, s35_mfma_bytes/), which were removed.
template <int KS, int W, bool NTL, bool NTS, bool BSWAP, class Pre, class SO, int NH = mfma_halves(KS, W)>
__device__ __forceinline__ void mfma_walk(const char* __restrict__ ib, char* __restrict__ ob, const SO& so,
                                          const i32x4* __restrict__ lfrag,
                                          const uint64_t* __restrict__ lrowc, const uint32_t* __restrict__ loff,
                                          uint32_t MT, uint32_t rows, uint32_t lane, uint32_t g, uint32_t n,
                                          uint32_t c0, uint32_t c1, uint32_t wave, uint32_t nwaves, MfmaIO io,
                                          Pre& pre) {
  constexpr uint32_t TC = 16 * W;
  const uint32_t ntiles = (c1 - c0 + TC - 1) / TC;
  auto col_of = [&](uint32_t tile) { return c0 + tile * TC + n * W; };
  auto colb_of = [&](uint32_t tile) {
    const uint32_t c = col_of(tile);
    return (c < c1 ? c : c1 - W) << 2;
  };
  vec_t<W> x[KS][4];
  uint32_t t = wave;
  if (t < ntiles) mfma_load_tile<KS, W, NTL>(x, ib, so, colb_of(t));
  while (t < ntiles) {
    const uint32_t tn = t + nwaves;
    if (tn < ntiles)
      mfma_tile<KS, W, NTL, NTS, true, BSWAP, Pre, SO, NH>(x, ib, so, colb_of(tn), lfrag, lrowc, loff, MT, rows, lane,
                                                          g, ob, colb_of(t), col_of(t) < c1, io, pre);
    else
      mfma_tile<KS, W, NTL, NTS, false, BSWAP, Pre, SO, NH>(x, ib, so, 0, lfrag, lrowc, loff, MT, rows, lane, g, ob,
                                                           colb_of(t), col_of(t) < c1, io, pre);
    t = tn;
  }
}

// The tile walk over short objects: tiles of every object numbered object by
// object (tpo a object, the last partial as in mfma_walk), walked by every
// wave of the grid (wave, wave + nwaves, ...), the refill streaming the next
// tile in across object boundaries.  Objects of a few tiles otherwise leave
// most of a block's waves idle (one work item per block) and restart the
// refill per object.
// io_of(obj): the object's word mapping (MfmaIO; the byte path's BSWAP
// chunks carry one mapping an object).
template <int KS, int W, bool NTL, bool NTS, bool BSWAP, class SO, class IOF>
__device__ __forceinline__ void mfma_flat_walk(const char* __restrict__ in, char* __restrict__ out,
                                               uint64_t in_obj_bytes, uint64_t out_obj_bytes, const SO& so,
                                               const i32x4* __restrict__ lfrag, const uint64_t* __restrict__ lrowc,
                                               const uint32_t* __restrict__ loff, uint32_t MT, uint32_t rows,
                                               uint32_t lane, uint32_t g, uint32_t n, uint32_t c1, uint32_t tpo,
                                               uint64_t ntiles, uint64_t wave, uint64_t nwaves, IOF io_of) {
  constexpr uint32_t TC = 16 * W;
  NoPre pre;
  auto col_of = [&](uint64_t f) { return (uint32_t)(f % tpo) * TC + n * W; };
  auto colb_of = [&](uint64_t f) {
    const uint32_t c = col_of(f);
    return (c < c1 ? c : c1 - W) << 2;
  };
  auto in_of = [&](uint64_t f) { return in + (f / tpo) * in_obj_bytes; };
  vec_t<W> x[KS][4];
  uint64_t t = wave;
  if (t < ntiles) mfma_load_tile<KS, W, NTL>(x, in_of(t), so, colb_of(t));
  while (t < ntiles) {
    const uint64_t tn = t + nwaves;
    const uint64_t obj = t / tpo;
    char* const ob = out + obj * out_obj_bytes;
    const MfmaIO io = io_of(obj);
    if (tn < ntiles)
      mfma_tile<KS, W, NTL, NTS, true, BSWAP, NoPre, SO>(x, in_of(tn), so, colb_of(tn), lfrag, lrowc, loff, MT, rows,
                                                         lane, g, ob, colb_of(t), col_of(t) < c1, io, pre);
    else
      mfma_tile<KS, W, NTL, NTS, false, BSWAP, NoPre, SO>(x, nullptr, so, 0, lfrag, lrowc, loff, MT, rows, lane, g,
                                                          ob, colb_of(t), col_of(t) < c1, io, pre);
    t = tn;
  }
}

// Block prologue: the plan's A fragments and row constants into LDS, the
// output rows' byte offsets (out_idx[i] * out_unit), and each lane's input
// byte offsets (in_idx[j] * in_unit, in_idx null: j; shards past k read shard in_idx[k-1],
// whose digits are zero -- lines the lanes of shard k-1 fetch anyway).
template <class SO>
__device__ __forceinline__ void mfma_prologue(i32x4* lds, const uint8_t* __restrict__ table,
                                              const uint32_t* __restrict__ in_idx,
                                              const uint32_t* __restrict__ out_idx, uint64_t in_unit,
                                              uint64_t out_unit, uint32_t MT, uint32_t KS, uint32_t rows, uint32_t k,
                                              uint32_t g, uint64_t** lrowc, uint32_t** loff, SO& so) {
  const uint32_t nfrag = MT * KS * 64;
  const i32x4* gfrag = reinterpret_cast<const i32x4*>(table);
  for (uint32_t f = threadIdx.x; f < nfrag; f += kBlock) lds[f] = gfrag[f];
  *lrowc = reinterpret_cast<uint64_t*>(lds + nfrag);
  *loff = reinterpret_cast<uint32_t*>(*lrowc + MT * 4);
  const uint64_t* growc = reinterpret_cast<const uint64_t*>(table + (size_t)nfrag * 16);
  for (uint32_t i = threadIdx.x; i < MT * 4; i += kBlock) {
    (*lrowc)[i] = i < rows ? growc[i] : 0;
    (*loff)[i] = i < rows ? (uint32_t)(out_idx[i] * out_unit) : 0;
  }
  so.init(in_idx, in_unit, k, g);
  __syncthreads();
}

// table: the plan's mfma table (mfma_table.hpp layout); coeff: the plan's
// coefficient rows (column tails).
// UNI: in_idx is 0..k-1 (ShardOffs<KS, true>: scalar step bases, 8 offset registers instead of 4 KS).
template <int KS, bool NTL, bool NTS, bool UNI>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(mfma_waves(KS, mfma_width(KS))))) void
rs_apply_mfma_kernel(
    const uint32_t* __restrict__ in, uint32_t* __restrict__ out, uint64_t in_obj_stride, uint64_t in_shard,
    uint64_t out_obj_stride, uint64_t out_shard, const uint8_t* __restrict__ table, const uint32_t* __restrict__ coeff,
    const uint32_t* __restrict__ in_idx, const uint32_t* __restrict__ out_idx, uint64_t ncols, uint32_t nobj,
    uint32_t rows, uint32_t k, uint32_t nseg, uint32_t flat) {
  constexpr int W = mfma_width(KS);
  extern __shared__ i32x4 lds[];
  const uint32_t MT = (rows + 3) / 4;
  const uint32_t lane = threadIdx.x & 63, g = lane >> 4, n = lane & 15;
  uint64_t* lrowc;
  uint32_t* loff;
  ShardOffs<KS, UNI> so;
  mfma_prologue(lds, table, in_idx, out_idx, in_shard * 4, out_shard * 4, MT, KS, rows, k, g, &lrowc, &loff, so);
  const uint64_t tid = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const uint64_t nthr = (uint64_t)gridDim.x * kBlock;
  const uint32_t nvec = (uint32_t)(ncols >> 2);
  const uint32_t seg_vec = segment_vectors(nvec, nseg);
  const uint64_t nwork = (uint64_t)nobj * nseg;
  const uint32_t wave = blockIdx.x * kWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nwaves = gridDim.x * kWaves;
  NoPre nopre;
  if (flat) {  // short objects (a 1D grid, nseg 1): one walk over every object's tiles, then the column tails
    constexpr uint32_t TC = 16 * W;
    const uint32_t c1 = 4 * nvec, tpo = (c1 + TC - 1) / TC;
    if (tpo)
      mfma_flat_walk<KS, W, NTL, NTS, false>(reinterpret_cast<const char*>(in), reinterpret_cast<char*>(out),
                                             in_obj_stride * 4, out_obj_stride * 4, so, lds, lrowc, loff, MT, rows,
                                             lane, g, n, c1, tpo, (uint64_t)nobj * tpo, wave, nwaves,
                                             [](uint64_t) { return MfmaIO{0x80808080u, 0u}; });
    // Tails as (object, row, column) cells, one per lane.
    const uint32_t tailc = (uint32_t)(ncols - c1);
    for (uint64_t i = tid; tailc && i < (uint64_t)nobj * rows * tailc; i += nthr) {
      const uint64_t or_ = i / tailc, obj = or_ / rows;
      apply_cell(in + obj * in_obj_stride, out + obj * out_obj_stride, coeff, in_idx, in_shard, out_idx, out_shard, k,
                 (uint32_t)(or_ % rows), c1 + i % tailc);
    }
    return;
  }
  for (uint64_t wi = blockIdx.y; wi < nwork; wi += gridDim.y) {
    const uint64_t obj = wi / nseg;
    const uint32_t seg = (uint32_t)(wi % nseg);
    const char* __restrict__ ib = reinterpret_cast<const char*>(in + obj * in_obj_stride);
    char* __restrict__ ob = reinterpret_cast<char*>(out + obj * out_obj_stride);
    const uint32_t v0 = seg * seg_vec < nvec ? seg * seg_vec : nvec;
    const uint32_t v1 = nvec - v0 > seg_vec ? v0 + seg_vec : nvec;
    if (v1 > v0)
      mfma_walk<KS, W, NTL, NTS, false>(ib, ob, so, lds, lrowc, loff, MT, rows, lane, g, n, 4 * v0, 4 * v1, wave,
                                        nwaves, MfmaIO{0x80808080u, 0u}, nopre);
    const uint32_t tailc = (uint32_t)(ncols - 4 * (uint64_t)nvec);  // (row, column) cells, one per lane
    if (seg == nseg - 1)
      for (uint64_t i = tid; tailc && i < (uint64_t)rows * tailc; i += nthr)
        apply_cell(reinterpret_cast<const uint32_t*>(ib), reinterpret_cast<uint32_t*>(ob), coeff, in_idx, in_shard,
                   out_idx, out_shard, k, (uint32_t)(i / tailc), 4 * (uint64_t)nvec + i % tailc);
  }
}

}  // namespace apply
}  // namespace slime
