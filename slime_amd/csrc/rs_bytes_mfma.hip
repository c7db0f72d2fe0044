// Matrix-core form of the fused byte-domain encode and decode for wide codes
// (bytes_mfma_eligible: need >= 33, or from need 17 (decode) / 25 (encode) when
// need x rows >= 128): writeChunks' MapToGF -> splitVector -> CreateParity ->
// MapFromGF (internal/store/multi/multi_store.go:526-557) and reconstruct's
// MapToGFWith -> RecoverData -> MapFromGF (multi_store.go:185-242), on the
// int8-limb product of rs_apply_mfma_kernel.hpp.
//
// Chunk bytes hold big-endian symbols: a chunk word loaded little-endian is
// w = bswap(x ^ m), so the plan's byte-order digit table (mfma_table.hpp,
// big_endian: register byte b weighs 2^(8(3-b))) takes (w ^ bswap(m)) directly
// -- with the signed-byte shift, B fragments are w ^ (0x80808080 ^ bswap(m))
// -- and results are stored as bswap(r ^ m).  No per-word byte swap on the
// data path; the encode's MapToGF flags take bswap(w) of every data word.
// Tiles whose every data word is a whole object word (the bulk) run on the
// matrix cores; the encode's edge columns (splitVector padding, the partial
// last word, the data-chunk tails MapFromGF writes, the vectors short of a
// whole tile) run as (object, row, column) items spread over the grid
// (spread_edges), or -- for windows too small to hold them in the last
// segment -- the VALU step of the wide byte kernels (encode_wide_step,
// rs_bytes_kernel.hpp); the repair's column tails run per lane.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "kernels.hpp"
#include "rs_apply_mfma_kernel.hpp"
#include "rs_bytes_kernel.hpp"
#include "rs_bytes_launch.hpp"
#include "redo_list.hpp"

namespace slime {
namespace bytes {

using apply::i32x4;
using apply::MfmaIO;

// MapToGF's flags over every loaded data word (encode, speculative pass) in
// two registers: the unsigned maximum of the words (bit0: >= p) and their
// signed maximum (the unsigned maximum of word ^ 1<<31; bit1: >= p) --
// a byte swap (v_perm_b32) per word and one v_max3 of each kind per two
// words, as one asm chain per pair.
// Written in C, the compiler batched the byte swaps of a K step ahead of its
// MFMAs and the refill form spilled 56 VGPRs at four K steps (64/80); the
// chain keeps one temporary live, and the refill form fits two waves per
// SIMD at every K step count (247 VGPRs at four, -Rpass-analysis).
struct FlagPre {
  uint32_t umax = 0;
  int32_t smax = INT32_MIN;
  template <class V>
  __device__ __forceinline__ void operator()(const V& v) {
    constexpr int W = sizeof(V) / sizeof(uint32_t);
    static_assert(W % 2 == 0, "pairs of words");
#pragma unroll
    for (int c = 0; c < W; c += 2) {  // two words per v_max3: 2 VALU ops per word
      uint32_t t0, t1;
      const uint32_t w0 = v[c], w1 = v[c + 1];
      asm volatile(
          "v_perm_b32 %0, %4, %4, %6\n\t"
          "v_perm_b32 %1, %5, %5, %6\n\t"
          "v_max3_u32 %2, %2, %0, %1\n\t"
          "v_max3_i32 %3, %3, %0, %1"
          : "=&v"(t0), "=&v"(t1), "+v"(umax), "+v"(smax)
          : "v"(w0), "v"(w1), "s"(0x00010203u));
    }
  }
  __device__ __forceinline__ uint32_t bits() const {
    return (umax >= kP ? 1u : 0u) | (((uint32_t)smax ^ 0x80000000u) >= kP ? 2u : 0u);
  }
};

// Mid-object mapping switch on the matrix cores (phase 0 with a scratch
// record): the refill walk of one segment's interior tiles [c0, c1) of object
// obj, but each tile takes its mapping from flags[obj] as phase 0 found it so
// far -- 1<<31 once some word >= p has been seen (map.go:35-62) -- and lane 0
// records it (rec[t], one byte per tile, 2 = "no interior tile" before the
// pass).  The flags word for tile t+1 is loaded while tile t computes; the
// wave's own flag bits are published after every tile.  Phase 1 then redoes
// only the tiles an object mapped with 1<<31 encoded with 0 (the tiles before
// its first word >= p), not the whole object.  A stale flags read only delays
// the switch: the record says what each tile wrote.
__device__ __forceinline__ uint32_t flags_now(const uint32_t* f) {
  return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <int KS, int W, int NH, class SO>
__device__ __forceinline__ void mfma_switch_walk(const char* __restrict__ ib, char* __restrict__ ob, const SO& so,
                                                 const i32x4* __restrict__ lfrag, const uint64_t* __restrict__ lrowc,
                                                 const uint32_t* __restrict__ loff,
                                                 uint32_t MT, uint32_t rows, uint32_t lane, uint32_t g, uint32_t n,
                                                 uint32_t c0, uint32_t c1, uint32_t wave, uint32_t nwaves,
                                                 uint32_t* __restrict__ fobj, uint8_t* __restrict__ rec, FlagPre& pre,
                                                 uint32_t& sent) {
  constexpr uint32_t TC = 16 * W;
  const uint32_t ntiles = (c1 - c0) / TC;  // interior: whole tiles only
  auto colb_of = [&](uint32_t t) { return (c0 + t * TC + n * W) << 2; };
  uint32_t t = wave;
  if (t >= ntiles) return;
  apply::vec_t<W> x[KS][4];
  apply::mfma_load_tile<KS, W, true>(x, ib, so, colb_of(t));
  uint32_t f = flags_now(fobj);
  while (t < ntiles) {
    const uint32_t tn = t + nwaves;
    // lane 0's load: the lane that records the mapping this tile used
    const uint32_t m = (__builtin_amdgcn_readlane(f, 0) & 1u) ? 0x80000000u : 0u;
    if (lane == 0) rec[t] = m ? 1 : 0;
    if (tn < ntiles) f = flags_now(fobj);  // tile tn's mapping, in flight during tile t
    const MfmaIO io{0x80808080u ^ be(m), m};
    if (tn < ntiles)
      apply::mfma_tile<KS, W, true, true, true, true, FlagPre, SO, NH>(x, ib, so, colb_of(tn), lfrag, lrowc, loff, MT,
                                                                       rows, lane, g, ob, colb_of(t), true, io, pre);
    else
      apply::mfma_tile<KS, W, true, true, false, true, FlagPre, SO, NH>(x, ib, so, 0, lfrag, lrowc, loff, MT, rows,
                                                                        lane, g, ob, colb_of(t), true, io, pre);
    const uint32_t fb = pre.bits();
    const uint32_t wf = (__ballot(fb & 1u) ? 1u : 0u) | (__ballot(fb & 2u) ? 2u : 0u);
    if (wf & ~sent) {
      if (lane == 0) atomicOr(fobj, wf);
      sent |= wf;
    }
    t = tn;
  }
}

// Phase 0 over short objects (one segment each, nint interior tiles an
// object): one walk over every object's interior tiles across the grid, the
// refill crossing objects (as apply::mfma_flat_walk), each tile encoded with
// its object's mapping as phase 0 has found it so far when `record` (the
// mid-object switch: one record byte per tile, as mfma_switch_walk) or with 0,
// and its flag bits published after the tile.  A block per object left most
// of its waves idle and restarted the refill per object.
template <int KS, int W, int NH, class SO>
__device__ __forceinline__ void mfma_flat_phase0(uint8_t* __restrict__ slots, uint64_t slot_stride, uint64_t col0,
                                                 uint64_t chunk, uint32_t k, const SO& so,
                                                 const i32x4* __restrict__ lfrag, const uint64_t* __restrict__ lrowc,
                                                 const uint32_t* __restrict__ loff, uint32_t MT, uint32_t rows,
                                                 uint32_t lane, uint32_t g, uint32_t n, uint32_t nint, uint64_t ntiles,
                                                 uint32_t wave, uint32_t nwaves, uint32_t* __restrict__ flags,
                                                 uint8_t* __restrict__ record, uint32_t units) {
  constexpr uint32_t TC = 16 * W;
  auto colb_of = [&](uint64_t f) { return (uint32_t)(((f % nint) * TC + n * W) << 2); };
  auto base_of = [&](uint64_t o) { return slots + o * slot_stride + 4 * col0; };
  uint64_t t = wave;
  if (t >= ntiles) return;
  apply::vec_t<W> x[KS][4];
  apply::mfma_load_tile<KS, W, true>(x, reinterpret_cast<const char*>(base_of(t / nint)), so, colb_of(t));
  uint32_t f = record ? flags_now(flags + t / nint) : 0u;
  while (t < ntiles) {
    const uint64_t tn = t + nwaves;
    const uint64_t obj = t / nint;
    const uint32_t m = (__builtin_amdgcn_readlane(f, 0) & 1u) ? 0x80000000u : 0u;
    if (record) {
      if (lane == 0) record[obj * units + t % nint] = m ? 1 : 0;
      if (tn < ntiles) f = flags_now(flags + tn / nint);  // tile tn's mapping, in flight during tile t
    }
    const MfmaIO io{0x80808080u ^ be(m), m};
    char* const ob = reinterpret_cast<char*>(base_of(obj) + (uint64_t)k * chunk);
    FlagPre pre;
    if (tn < ntiles)
      apply::mfma_tile<KS, W, true, true, true, true, FlagPre, SO, NH>(
          x, reinterpret_cast<const char*>(base_of(tn / nint)), so, colb_of(tn), lfrag, lrowc, loff, MT, rows, lane, g,
          ob, colb_of(t), true, io, pre);
    else
      apply::mfma_tile<KS, W, true, true, false, true, FlagPre, SO, NH>(x, nullptr, so, 0, lfrag, lrowc, loff, MT, rows,
                                                                        lane, g, ob, colb_of(t), true, io, pre);
    const uint32_t fb = pre.bits();
    const uint32_t wf = (__ballot(fb & 1u) ? 1u : 0u) | (__ballot(fb & 2u) ? 2u : 0u);
    if (wf && lane == 0) atomicOr(flags + obj, wf);
    t = tn;
  }
}

// The edge steps of one segment (vectors [e0, u1)), one vector per lane: the
// windows whose edges spread_edges does not take, and the whole-object
// re-encode.
template <bool F>
__device__ __forceinline__ uint32_t encode_edges(uint8_t* slot, uint8_t* par, uint64_t chunk, uint64_t L, uint64_t col0,
                                              ObjWords ow, uint64_t first_tail_word, uint32_t m, uint32_t rows,
                                              uint32_t k, uint32_t cs, const uint32_t* __restrict__ coeff,
                                              const uint32_t* __restrict__ out_idx, uint64_t e0, uint64_t nvec,
                                              uint64_t u1, uint64_t seg_v1, uint32_t lane, uint32_t wave,
                                              uint32_t nwaves) {
  Flags fl;
  for (uint64_t gv = e0 + (uint64_t)wave * 64 + lane; gv - lane < u1; gv += (uint64_t)nwaves * 64)
    encode_wide_step<16, 8, F>(slot, par, chunk, L, col0, ow, first_tail_word, m, rows, k, cs, coeff, out_idx, gv, nvec,
                               u1, seg_v1, lane, fl);
  return F ? fl.bits() : 0u;
}

// The edge columns of an encode window, [4 e0, ncols): from the end of the
// last whole matrix-core tile below the object's last word in chunk k-1 to the
// window's last column.  The last data chunk is short by fewer than k words
// (L = ceil(ceil(S/4)/k)), so the edges sit in the last segment (`spread`;
// segments are whole tiles) unless the window is tiny -- then the segments'
// own edge steps run.  The same columns for every object of a launch.
struct EdgeSpan {
  uint64_t e0;
  bool spread;
};
template <uint32_t TCV>
__device__ __forceinline__ EdgeSpan edge_span(uint64_t S, uint64_t L, uint64_t col0, uint32_t k, uint64_t nvec,
                                              uint32_t nseg) {
  const Segment last = segment_of(nseg - 1, nseg, nvec);
  uint64_t end_max = interior_vectors(S, L, col0, k);
  if (end_max > last.v1) end_max = last.v1;
  EdgeSpan s;
  s.spread = end_max >= last.v0;
  s.e0 = last.v0 + (end_max > last.v0 ? (end_max - last.v0) / TCV * TCV : 0);
  return s;
}

// Edge columns [b0, ncols) of every object `take` selects, spread over the
// whole grid: a wave takes 64 consecutive columns of one object and sixteen of
// its rows (object and rows uniform, so the coefficients are scalar loads),
// a lane one column: the k data chunks' symbols (splitVector padding, the
// partial last word) loaded sixteen at a time, summed into the sixteen rows
// (eight or four reloaded the symbols more often and ran 15-25% slower at
// 80/100, profiles/r05/s42_rb/),
// stored with MapFromGF's mapping; the first row block also writes the
// data-chunk tails and (F) folds MapToGF's flags into flags[obj].  Replaces a
// single wave's serial VALU edge step per object, and then one lane per (row,
// column) that loaded and unpacked every symbol once per row: batches of short
// objects are mostly edge (80/100 at 16 KiB: all 52 columns), and that ran
// 345 us for 16 MiB of objects.  Row blocks of one column may read a tail word
// before or after the first rewrote it: the rewrite is its packed value
// (padding words read as zero either way), so every read agrees.
template <bool F, class Take>
__device__ __forceinline__ void spread_edges(uint8_t* __restrict__ slots, uint64_t slot_stride, uint64_t L,
                                             uint64_t chunk, uint64_t col0, uint64_t ncols, const ObjWords& ow,
                                             uint32_t nobj, uint32_t rows, uint32_t k, uint32_t cs,
                                             const uint32_t* __restrict__ coeff, const uint32_t* __restrict__ out_idx,
                                             uint64_t b0, uint32_t* __restrict__ flags, Take take) {
  if (b0 >= ncols) return;
  constexpr uint32_t RB = 16;
  const uint64_t ncb = (ncols - b0 + 63) / 64, nrb = (rows + RB - 1) / RB;
  const uint64_t per = nrb * ncb, total = per * nobj;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t gw = ((uint64_t)blockIdx.y * gridDim.x + blockIdx.x) * kWaves +
                      __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t gn = (uint64_t)gridDim.x * gridDim.y * kWaves;
  for (uint64_t u = gw; u < total; u += gn) {
    const uint32_t o = (uint32_t)(u / per);
    const uint64_t rem = u % per;
    const uint32_t r0 = (uint32_t)(rem / ncb) * RB;
    const uint64_t bl = b0 + (rem % ncb) * 64 + lane;
    const bool act = bl < ncols;
    const uint64_t b = act ? bl : ncols - 1;  // idle lanes re-read the last column, store nothing
    uint32_t m;
    if (!take(o, m)) continue;
    uint8_t* const slot = slots + (uint64_t)o * slot_stride + 4 * col0;
    Flags fl;
    uint64_t lo[RB];
    uint32_t hi[RB];
#pragma unroll
    for (uint32_t rr = 0; rr < RB; ++rr) lo[rr] = 0, hi[rr] = 0;
    for (uint32_t j0 = 0; j0 < k; j0 += 16) {
      uint32_t x[16][4];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        x[j][0] = 0;
        if (j0 + j < k) load_data_symbol<false, F>(slot, chunk, L, col0, j0 + j, b, 1, ow, m, x[j], &fl);
      }
      if (r0 == 0 && act)
#pragma unroll
        for (int j = 0; j < 16; ++j)
          if (j0 + j < k) fix_data_tail_one(slot, chunk, L, col0, j0 + j, b, 1, ow, m, x[j]);
#pragma unroll
      for (uint32_t rr = 0; rr < RB; ++rr) {
        if (r0 + rr >= rows) break;
        const uint32_t* const crow = coeff + (uint64_t)(r0 + rr) * cs + j0;  // cs: rows padded to 16
#pragma unroll
        for (int j = 0; j < 16; ++j) mac(lo[rr], hi[rr], x[j][0], crow[j]);
      }
    }
    if (act)
#pragma unroll
      for (uint32_t rr = 0; rr < RB; ++rr) {
        if (r0 + rr >= rows) break;
        *reinterpret_cast<uint32_t*>(slot + ((uint64_t)k + out_idx[r0 + rr]) * chunk + 4 * b) =
            be(fold96(lo[rr], hi[rr]) ^ m);
      }
    if constexpr (F) {
      const uint32_t bits = r0 == 0 ? fl.bits() : 0u;
      if (bits) atomicOr(&flags[o], bits);
    }
  }
}

// MODE 0: speculative pass (mapping 0, MapToGF flags into flags[obj]);
// MODE 1: re-encode of the objects select_mapping gave mapping != 0 (status 0).
// The encodes' tiles: four columns a lane up to five K steps, two above (six
// and seven K steps on four columns spill at two waves per SIMD, and phase 0
// stays at two: at five K steps in two column passes -- one pass at one wave
// ran its flag folding and mapping switch 3-14% slower,
// profiles/r05/s14_onewave/).  Phase 0, its redo and the whole-object
// re-encode share the width (the redo walks phase 0's tiles); the redo and
// the re-encode run at the other matrix-core kernels' waves (mfma_waves).
constexpr int enc_width(int ks) { return ks <= 5 ? 4 : 2; }
template <int KS, int MODE>
constexpr int enc_waves() { return MODE == 0 ? apply::kMfmaWaves : apply::mfma_waves(KS, enc_width(KS)); }
template <int KS, int MODE>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(enc_waves<KS, MODE>()))) void
encode_bytes_mfma_kernel(uint8_t* __restrict__ slots, uint64_t slot_stride, uint64_t L, uint64_t chunk, uint64_t col0,
                         uint64_t ncols, uint64_t S, uint32_t nobj, uint32_t rows, uint32_t k,
                         const uint8_t* __restrict__ table, const uint32_t* __restrict__ coeff,
                         const uint32_t* __restrict__ out_idx, uint32_t* __restrict__ flags,
                         const uint32_t* __restrict__ mapping, uint32_t nseg, uint8_t* __restrict__ record,
                         uint32_t units, uint32_t flat0) {
  constexpr int W = enc_width(KS);
  constexpr int NH = apply::mfma_halves_at(KS, W, enc_waves<KS, MODE>());
  constexpr uint32_t TCV = 4 * W;  // tile width in 16-byte vectors
  constexpr bool F = MODE == 0;
  extern __shared__ i32x4 lds[];
  const uint32_t MT = (rows + 3) / 4;
  const uint32_t lane = threadIdx.x & 63, lg = lane >> 4, ln = lane & 15;
  uint64_t* lrowc;
  uint32_t* loff;
  apply::ShardOffs<KS, true> so;  // data chunks in order
  apply::mfma_prologue(lds, table, nullptr, out_idx, chunk, chunk, MT, KS, rows, k, lg, &lrowc, &loff, so);
  const uint32_t cs = apply::wide_coeff_stride(k);
  const ObjWords ow{(S + 3) / 4, S % 4 ? 0xFFFFFFFFu << (8 * (4 - S % 4)) : 0xFFFFFFFFu};
  const uint64_t first_tail_word = ow.nw ? ow.nw - 1 : 0;
  const uint32_t wave = blockIdx.x * kWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nwaves = gridDim.x * kWaves;
  const uint64_t nvec = ncols >> 2;
  // Phase 0: every object's edge columns first, spread over the grid (their
  // flags published before the tile walks start).
  bool edges_done = false;
  if constexpr (F) {
    const EdgeSpan es = edge_span<TCV>(S, L, col0, k, nvec, nseg);
    if (es.spread) {
      spread_edges<true>(slots, slot_stride, L, chunk, col0, ncols, ow, nobj, rows, k, cs, coeff, out_idx, 4 * es.e0,
                         flags, [](uint32_t, uint32_t& m) {
                           m = 0;
                           return true;
                         });
      edges_done = true;
    }
    if (flat0) {  // short objects (a 1D grid, nseg 1, edges spread): the flat interior walk, then done
      uint64_t end_max = interior_vectors(S, L, col0, k);
      if (end_max > nvec) end_max = nvec;
      const uint32_t nint = (uint32_t)(end_max / TCV);
      if (nint)
        mfma_flat_phase0<KS, W, NH>(slots, slot_stride, col0, chunk, k, so, lds, lrowc, loff, MT, rows, lane, lg, ln,
                                    nint, (uint64_t)nobj * nint, wave, nwaves, flags, record, units);
      return;
    }
  }
  // Re-encode of up to 64 objects (one segment each): one flat tile walk over
  // the interior tiles of every object select_mapping gave 1<<31, so the grid
  // streams them back to back (the refill crosses objects) instead of
  // restarting its walk per object; then their edge steps.
  bool flat = false;
  if constexpr (MODE == 1) {
    if (nobj <= 64 && nseg == 1) {
      flat = true;
      const uint32_t mlane = lane < nobj ? mapping[lane] : 0u;  // object `lane`'s mapping, read once
      const bool selm = lane < nobj && mlane != 0 && flags[lane] == 0;
      const uint64_t sel = __ballot(selm);
      const uint32_t count = (uint32_t)__popcll(sel);
      uint64_t end_max = interior_vectors(S, L, col0, k);
      if (end_max > nvec) end_max = nvec;
      const uint32_t nint = (uint32_t)(end_max / TCV);
      auto nth = [&](uint32_t i) {  // object of the i-th selected slot
        uint64_t b = sel;
        for (uint32_t q = 0; q < i; ++q) b &= b - 1;
        return (uint32_t)__builtin_ctzll(b);
      };
      auto slot_of = [&](uint32_t o) { return slots + (uint64_t)o * slot_stride + 4 * col0; };
      // The flat tile space f < T (object nth(f / nint), tile f % nint) is cut
      // into G contiguous streams walked by 8 waves each, as the speculative
      // pass's segments are: all waves on one window of one object streamed
      // at 2.3 TB/s (profiles/r03/s35_mfma_bytes/).
      const uint32_t T = count * nint;
      const uint32_t G = nwaves / 8 ? nwaves / 8 : 1;
      const uint32_t len = (T + G - 1) / G;
      auto flat = [&](uint32_t t) { return (t % G) * len + t / G; };  // < T for every visited t
      auto colb_of = [&](uint32_t f) { return ((f % nint) * (16 * W) + ln * W) << 2; };
      auto next = [&](uint32_t t) {  // the wave's next visited index (or >= G * len)
        for (t += nwaves; t < G * len && flat(t) >= T; t += nwaves) {
        }
        return t;
      };
      apply::NoPre pre;
      uint32_t t = wave;
      if (t < G * len && flat(t) >= T) t = next(t);
      apply::vec_t<W> x[KS][4];
      if (t < G * len)
        apply::mfma_load_tile<KS, W, true>(x, reinterpret_cast<const char*>(slot_of(nth(flat(t) / nint))), so,
                                           colb_of(flat(t)));
      while (t < G * len) {
        const uint32_t tn = next(t);
        const uint32_t f = flat(t);
        const uint32_t o = nth(f / nint);
        const uint32_t mo = __builtin_amdgcn_readlane(mlane, o);  // no memory round trip per tile
        const MfmaIO io{0x80808080u ^ be(mo), mo};
        char* const ob = reinterpret_cast<char*>(slot_of(o) + (uint64_t)k * chunk);
        if (tn < G * len) {
          const uint32_t fn = flat(tn);
          apply::mfma_tile<KS, W, true, true, true, true>(x, reinterpret_cast<const char*>(slot_of(nth(fn / nint))),
                                                          so, colb_of(fn), lds, lrowc, loff, MT, rows, lane, lg, ob,
                                                          colb_of(f), true, io, pre);
        } else {
          apply::mfma_tile<KS, W, true, true, false, true>(x, nullptr, so, 0, lds, lrowc, loff, MT, rows, lane, lg,
                                                           ob, colb_of(f), true, io, pre);
        }
        t = tn;
      }
      // Edge steps: object i's on waves offset by i * nwaves / count, so the
      // objects' (serial, VALU) edge steps run side by side.
      for (uint32_t i = 0; i < count; ++i) {
        const uint32_t o = nth(i);
        uint8_t* const slot = slot_of(o);
        const uint32_t wrel = (wave + nwaves - (uint32_t)((uint64_t)i * nwaves / count)) % nwaves;
        (void)encode_edges<false>(slot, slot + (uint64_t)k * chunk, chunk, L, col0, ow, first_tail_word,
                                  __builtin_amdgcn_readlane(mlane, o), rows, k, cs, coeff, out_idx,
                                  (uint64_t)nint * TCV, nvec, nvec + (ncols & 3), nvec, lane, wrel, nwaves);
      }
    }
  }
  for (uint64_t wi = blockIdx.y; wi < (uint64_t)nobj * nseg; wi += gridDim.y) {
    const Segment sg = segment_of(wi, nseg, nvec);
    const uint32_t obj = sg.obj;
    const uint32_t v0 = (uint32_t)sg.v0, v1 = (uint32_t)sg.v1;
    const uint64_t u1 = sg.last ? nvec + (ncols & 3) : sg.v1;
    uint32_t m = 0;
    if constexpr (MODE == 1) {
      if (flat) break;  // the flat walk below did every object
      m = mapping[obj];
      if (m == 0 || flags[obj] != 0) continue;  // uniform per block
    }
    uint8_t* const slot = slots + (uint64_t)obj * slot_stride + 4 * col0;  // window base
    uint8_t* const par = slot + (uint64_t)k * chunk;
    // Interior tiles: whole tiles of the segment whose columns are below the
    // object's last word in the last data chunk (k-1), hence in every chunk.
    uint64_t end_max = interior_vectors(S, L, col0, k);
    if (end_max > v1) end_max = v1;
    const uint32_t nint = end_max > v0 ? (uint32_t)((end_max - v0) / TCV) : 0u;
    const MfmaIO io{0x80808080u ^ be(m), m};
    uint32_t fbits = 0;
    if (nint) {
      if constexpr (F) {
        FlagPre pre;
        if (record) {  // the mid-object switch (mfma_switch_walk)
          uint32_t sent = 0;
          mfma_switch_walk<KS, W, NH>(reinterpret_cast<const char*>(slot), reinterpret_cast<char*>(par), so, lds, lrowc,
                                  loff, MT, rows, lane, lg, ln, 4 * v0, 4 * (v0 + nint * TCV), wave, nwaves,
                                  flags + obj, record + (uint64_t)obj * units + v0 / TCV, pre, sent);
        } else {
          apply::mfma_walk<KS, W, true, true, true, FlagPre, apply::ShardOffs<KS, true>, NH>(
              reinterpret_cast<const char*>(slot), reinterpret_cast<char*>(par), so, lds, lrowc, loff, MT, rows, lane,
              lg, ln, 4 * v0, 4 * (v0 + nint * TCV), wave, nwaves, io, pre);
        }
        fbits = pre.bits();
      } else {
        apply::NoPre pre;
        apply::mfma_walk<KS, W, true, true, true, apply::NoPre, apply::ShardOffs<KS, true>, NH>(
            reinterpret_cast<const char*>(slot), reinterpret_cast<char*>(par), so, lds, lrowc, loff, MT, rows, lane, lg,
            ln, 4 * v0, 4 * (v0 + nint * TCV), wave, nwaves, io, pre);
      }
    }
    // Edge tiles and tail columns (VALU step, with the data-chunk tail fix).
    const uint64_t e0 = (uint64_t)v0 + (uint64_t)nint * TCV;
    if (e0 < u1 && !edges_done)
      fbits |= encode_edges<F>(slot, par, chunk, L, col0, ow, first_tail_word, m, rows, k, cs, coeff, out_idx, e0, nvec,
                               u1, sg.v1, lane, wave, nwaves);
    if constexpr (F) {
      const uint64_t a1 = __ballot(fbits & 1u), a2 = __ballot(fbits & 2u);
      const uint32_t wf = (a1 ? 1u : 0u) | (a2 ? 2u : 0u);
      if (wf && lane == 0) atomicOr(&flags[obj], wf);
    }
  }
}

// The redo list of a switched matrix-core phase 0: every interior tile of an
// object whose mapping came out 1<<31 (status 0) that phase 0 encoded with
// mapping 0 (record 0; 1 = encoded with 1<<31, 2 = not an interior tile), as
// entries obj * units + tile; *count (zero on entry) receives their number,
// or'd with kSwitchedBit when any object switched (units >= 1: every object
// has entries), so the redo skips its edge pass outright when none did.  The
// word's protocol and its bound are redo_list.hpp's (the host launches this
// only when redo_list_fits(nobj, units)).
__global__ __launch_bounds__(kBlock) void mfma_redo_list_kernel(const uint8_t* __restrict__ record,
                                                                const uint32_t* __restrict__ mapping,
                                                                const uint32_t* __restrict__ status, uint32_t nobj,
                                                                uint32_t units, uint32_t* __restrict__ list,
                                                                uint32_t* __restrict__ count) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  const uint64_t nwaves = (uint64_t)gridDim.x * kWaves;
  const uint64_t total = (uint64_t)nobj * units;
  for (uint64_t base = wave * 64; base < total; base += nwaves * 64) {
    const uint64_t e = base + lane;
    bool sw = false, need = false;
    if (e < total) {
      const uint32_t o = (uint32_t)(e / units);
      sw = mapping[o] != 0 && status[o] == 0;
      need = sw && record[e] == 0;
    }
    if (__ballot(sw) && lane == 0) atomicOr(count, kSwitchedBit);
    const uint64_t mask = __ballot(need);
    if (!mask) continue;
    uint32_t at = 0;
    if (lane == 0) at = atomicAdd(count, (uint32_t)__popcll(mask));
    at = redo_offset(__builtin_amdgcn_readlane(at, 0));  // lane 0 drew it, whatever the exec mask
    if (need) list[at + (uint32_t)__popcll(mask & ((1ull << lane) - 1))] = (uint32_t)e;
  }
}

// Phase 1 after a switched matrix-core phase 0: the listed interior tiles
// re-encoded with their object's mapping (one refill walk over the list, the
// next entry's data streaming in behind the current one's math, across
// objects), then every edge range of the objects mapped with 1<<31, segment
// by segment as phase 0 cut them (phase 0 writes edges with mapping 0).
// The redo at five K steps: four-column tiles in one pass at one wave per
// SIMD (80/100 encode both passes 2.236 vs 2.267 ms at two waves and two
// column passes, profiles/r05/s15_redowaves/).
constexpr int redo_waves(int ks) { return apply::mfma_waves(ks, enc_width(ks)); }
template <int KS>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(redo_waves(KS)))) void
encode_bytes_mfma_redo_kernel(uint8_t* __restrict__ slots, uint64_t slot_stride, uint64_t L, uint64_t chunk,
                              uint64_t col0, uint64_t ncols, uint64_t S, uint32_t nobj, uint32_t rows, uint32_t k,
                              const uint8_t* __restrict__ table, const uint32_t* __restrict__ coeff,
                              const uint32_t* __restrict__ out_idx, const uint32_t* __restrict__ status,
                              const uint32_t* __restrict__ mapping, uint32_t nseg, const uint32_t* __restrict__ list,
                              const uint32_t* __restrict__ count, uint32_t units) {
  constexpr int W = enc_width(KS);
  constexpr int NH = apply::mfma_halves_at(KS, W, redo_waves(KS));
  constexpr uint32_t TCV = 4 * W;
  extern __shared__ i32x4 lds[];
  const uint32_t MT = (rows + 3) / 4;
  const uint32_t lane = threadIdx.x & 63, lg = lane >> 4, ln = lane & 15;
  uint64_t* lrowc;
  uint32_t* loff;
  apply::ShardOffs<KS, true> so;
  apply::mfma_prologue(lds, table, nullptr, out_idx, chunk, chunk, MT, KS, rows, k, lg, &lrowc, &loff, so);
  const uint32_t cs = apply::wide_coeff_stride(k);
  const ObjWords ow{(S + 3) / 4, S % 4 ? 0xFFFFFFFFu << (8 * (4 - S % 4)) : 0xFFFFFFFFu};
  const uint64_t first_tail_word = ow.nw ? ow.nw - 1 : 0;
  const uint32_t wave = blockIdx.x * kWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nwaves = gridDim.x * kWaves;
  const uint64_t nvec = ncols >> 2;
  auto slot_of = [&](uint32_t o) { return slots + (uint64_t)o * slot_stride + 4 * col0; };
  auto colb_of = [&](uint32_t e) { return ((e % units) * (16 * W) + ln * W) << 2; };
  // The switched objects' edge columns first, spread over the grid (phase 0
  // wrote them with mapping 0).
  const EdgeSpan es = edge_span<TCV>(S, L, col0, k, nvec, nseg);
  const uint32_t listed = *count;
  if (!redo_switched(listed)) return;  // no object switched: nothing to redo
  if (es.spread)
    spread_edges<false>(slots, slot_stride, L, chunk, col0, ncols, ow, nobj, rows, k, cs, coeff, out_idx, 4 * es.e0,
                        nullptr, [&](uint32_t o, uint32_t& m) {
                          m = mapping[o];
                          return m != 0 && status[o] == 0;
                        });
  const uint32_t n = redo_count(listed);
  // The list (ascending tiles of each object, roughly) is cut into G
  // contiguous streams of 8 waves each, as the re-encode's flat walk: all
  // waves on one window of one object streamed at 2.3 TB/s
  // (profiles/r03/s35_mfma_bytes/).  Entry i of stream s is list[s*len + i];
  // wave (s, r) takes i = r, r + 8, ...  The list word and the mapping of the
  // entry after next are loaded one entry ahead, so the refill's addresses
  // never wait on a dependent load.
  const uint32_t G = nwaves / 8 ? nwaves / 8 : 1;
  const uint32_t len = (n + G - 1) / G;
  const uint32_t sid = wave / 8 < G ? wave / 8 : G - 1, r8 = wave % 8;
  const uint32_t lo = sid * len, hi = std::min(n, lo + len);
  apply::NoPre pre;
  uint32_t i = lo + r8;
  if (wave / 8 < G && i < hi) {
    apply::vec_t<W> x[KS][4];
    uint32_t e = list[i];
    uint32_t mo = mapping[e / units];
    uint32_t en = i + 8 < hi ? list[i + 8] : e;
    uint32_t mn = i + 8 < hi ? mapping[en / units] : mo;
    apply::mfma_load_tile<KS, W, true>(x, reinterpret_cast<const char*>(slot_of(e / units)), so, colb_of(e));
    while (i < hi) {
      const uint32_t in_ = i + 8;
      // entry in_ + 8's list word and mapping, in flight during this tile
      const uint32_t enn = in_ + 8 < hi ? list[in_ + 8] : en;
      const uint32_t o = e / units;
      const uint32_t m = __builtin_amdgcn_readfirstlane(mo);
      const MfmaIO io{0x80808080u ^ be(m), m};
      char* const ob = reinterpret_cast<char*>(slot_of(o) + (uint64_t)k * chunk);
      if (in_ < hi)
        apply::mfma_tile<KS, W, true, true, true, true, apply::NoPre, apply::ShardOffs<KS, true>, NH>(
            x, reinterpret_cast<const char*>(slot_of(en / units)), so,
                                                        colb_of(en), lds, lrowc, loff, MT, rows, lane, lg, ob,
                                                        colb_of(e), true, io, pre);
      else
        apply::mfma_tile<KS, W, true, true, false, true, apply::NoPre, apply::ShardOffs<KS, true>, NH>(
            x, nullptr, so, 0, lds, lrowc, loff, MT, rows, lane, lg, ob,
                                                         colb_of(e), true, io, pre);
      const uint32_t mnn = in_ + 8 < hi ? mapping[enn / units] : mn;
      i = in_;
      e = en;
      mo = mn;
      en = enn;
      mn = mnn;
    }
  }
  // Edge ranges of the switched objects, per phase-0 segment (none when the
  // objects fill their chunks exactly).  The switched objects are found 64 at
  // a time with one ballot (a serial scan of every object's mapping and status
  // put two dependent loads per object in front of every wave); object i's
  // ranges start on waves offset by i * nwaves / count so they run side by side.
  if (es.spread) return;
  const uint64_t iv = interior_vectors(S, L, col0, k);
  uint32_t nsel = 0;
  for (uint32_t ob = 0; ob < nobj; ob += 64) {
    const uint32_t ol = ob + lane;
    nsel += (uint32_t)__popcll(__ballot(ol < nobj && mapping[ol] != 0 && status[ol] == 0));
  }
  uint32_t si = 0;
  for (uint32_t ob = 0; ob < nobj && nsel; ob += 64) {
    const uint32_t ol = ob + lane;
    const uint32_t ml = ol < nobj ? mapping[ol] : 0u;
    uint64_t sel = __ballot(ol < nobj && ml != 0 && status[ol] == 0);
    for (; sel; sel &= sel - 1, ++si) {
      const uint32_t b = (uint32_t)__builtin_ctzll(sel);
      const uint32_t o = ob + b;
      const uint32_t m = __builtin_amdgcn_readlane(ml, b);
      uint8_t* const slot = slot_of(o);
      const uint32_t wrel = (wave + nwaves - (uint32_t)((uint64_t)si * nwaves / nsel)) % nwaves;
      for (uint32_t seg = 0; seg < nseg; ++seg) {
        const Segment sg = segment_of((uint64_t)o * nseg + seg, nseg, nvec);
        const uint64_t u1 = sg.last ? nvec + (ncols & 3) : sg.v1;
        const uint64_t end_max = iv < sg.v1 ? iv : sg.v1;
        const uint32_t nint = end_max > sg.v0 ? (uint32_t)((end_max - sg.v0) / TCV) : 0u;
        const uint64_t e0 = sg.v0 + (uint64_t)nint * TCV;
        if (e0 < u1)
          (void)encode_edges<false>(slot, slot + (uint64_t)k * chunk, chunk, L, col0, ow, first_tail_word, m, rows, k,
                                    cs, coeff, out_idx, e0, nvec, u1, sg.v1, lane, wrel, nwaves);
      }
    }
  }
}

// Decode: survivors in_idx -> rebuilt chunks out_idx of the same slot.
template <int KS>
__global__ __launch_bounds__(kBlock)
__attribute__((amdgpu_waves_per_eu(apply::mfma_waves(KS, apply::mfma_width(KS))))) void
decode_bytes_mfma_kernel(uint8_t* __restrict__ slots, uint64_t slot_stride, uint64_t L, uint64_t chunk, uint64_t col0,
                         uint64_t ncols, uint32_t nobj, uint32_t rows, uint32_t k, const uint8_t* __restrict__ table,
                         const uint32_t* __restrict__ coeff, const uint32_t* __restrict__ in_idx,
                         const uint32_t* __restrict__ out_idx, const uint32_t* __restrict__ mapping, uint32_t nseg,
                         uint32_t flat) {
  constexpr int W = apply::mfma_width(KS);
  extern __shared__ i32x4 lds[];
  const uint32_t MT = (rows + 3) / 4;
  const uint32_t lane = threadIdx.x & 63, lg = lane >> 4, ln = lane & 15;
  uint64_t* lrowc;
  uint32_t* loff;
  apply::ShardOffs<KS, false> so;  // survivors in_idx
  apply::mfma_prologue(lds, table, in_idx, out_idx, chunk, chunk, MT, KS, rows, k, lg, &lrowc, &loff, so);
  const uint32_t cs = apply::wide_coeff_stride(k);
  const uint32_t wave = blockIdx.x * kWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nwaves = gridDim.x * kWaves;
  const uint64_t nvec = ncols >> 2;
  (void)L;
  apply::NoPre pre;
  // Row i of tail column b (columns past the last whole vector), one per lane.
  auto tail_cell = [&](uint8_t* slot, uint32_t m, uint32_t i, uint64_t b) {
    const uint32_t v = apply::wide_dot(coeff + (uint64_t)i * cs, k, [&](uint32_t j) {
      return be(*reinterpret_cast<const uint32_t*>(slot + (uint64_t)in_idx[j] * chunk + 4 * b)) ^ m;
    });
    *reinterpret_cast<uint32_t*>(slot + (uint64_t)out_idx[i] * chunk + 4 * b) = be(v ^ m);
  };
  if (flat) {  // short chunks (a 1D grid, nseg 1): one walk over every object's tiles, then the column tails
    constexpr uint32_t TC = 16 * W;
    const uint32_t c1 = 4 * (uint32_t)nvec, tpo = (c1 + TC - 1) / TC;
    uint8_t* const base = slots + 4 * col0;
    if (tpo)
      apply::mfma_flat_walk<KS, W, true, true, true>(
          reinterpret_cast<const char*>(base), reinterpret_cast<char*>(base), slot_stride, slot_stride, so, lds, lrowc,
          loff, MT, rows, lane, lg, ln, c1, tpo, (uint64_t)nobj * tpo, wave, nwaves, [&](uint64_t o) {
            const uint32_t m = mapping[o];
            return MfmaIO{0x80808080u ^ be(m), m};
          });
    const uint32_t tailc = (uint32_t)(ncols - c1);
    const uint64_t tid = (uint64_t)wave * 64 + lane, nthr = (uint64_t)nwaves * 64;
    for (uint64_t i = tid; tailc && i < (uint64_t)nobj * rows * tailc; i += nthr) {
      const uint64_t or_ = i / tailc, o = or_ / rows;
      tail_cell(base + o * slot_stride, mapping[o], (uint32_t)(or_ % rows), c1 + i % tailc);
    }
    return;
  }
  for (uint64_t wi = blockIdx.y; wi < (uint64_t)nobj * nseg; wi += gridDim.y) {
    const Segment sg = segment_of(wi, nseg, nvec);
    const uint32_t m = mapping[sg.obj];
    uint8_t* const slot = slots + (uint64_t)sg.obj * slot_stride + 4 * col0;  // window base
    if (sg.v1 > sg.v0)
      apply::mfma_walk<KS, W, true, true, true>(reinterpret_cast<const char*>(slot), reinterpret_cast<char*>(slot), so,
                                                lds, lrowc, loff, MT, rows, lane, lg, ln, 4 * (uint32_t)sg.v0,
                                                4 * (uint32_t)sg.v1, wave, nwaves, MfmaIO{0x80808080u ^ be(m), m}, pre);
    const uint32_t tailc = (uint32_t)(ncols - (nvec << 2));
    for (uint64_t i = (uint64_t)wave * 64 + lane; sg.last && tailc && i < (uint64_t)rows * tailc;
         i += (uint64_t)nwaves * 64)
      tail_cell(slot, m, (uint32_t)(i / tailc), (nvec << 2) + i % tailc);
  }
}

}  // namespace bytes

namespace {

using apply::kBlock;

// Interior tiles per object the switch record covers (one byte each).
template <int KS>
uint32_t switch_units(const BytesLaunch& a) {
  constexpr uint64_t TCV = 4 * bytes::enc_width(KS);
  const uint64_t nvec = (a.ncols ? a.ncols : a.L) >> 2;
  return (uint32_t)((nvec + TCV - 1) / TCV);
}

template <int KS>
hipError_t enc_ks(const BytesLaunch& a, hipStream_t s) {
  const uint64_t ncols = a.ncols ? a.ncols : a.L;
  const uint32_t lds = apply::mfma_lds_bytes(mfma::mtiles(a.rows), KS);
  const uint64_t blocks = 256ull * bytes::enc_waves<KS, 0>();  // resident blocks
  const uint64_t blocks1 = 256ull * bytes::enc_waves<KS, 1>();
  const uint64_t rblocks = 256ull * bytes::redo_waves(KS);
  if (a.phase == 0) {
    const uint32_t nseg = object_segments(a.nobj, ncols);
    // The mid-object switch runs when the caller handed scratch for its
    // record (never inside a graph capture).
    uint8_t* record = nullptr;
    uint32_t units = 0;
    if (a.scratch && a.sw && bytes::redo_list_fits(a.nobj, switch_units<KS>(a))) {
      units = switch_units<KS>(a);
      bytes::SwitchLayout l;
      l.units = units;
      record = l.record(a.scratch, a.nobj);
      if (hipError_t e = hipMemsetAsync(record, 2, (uint64_t)a.nobj * units, s)) return e;
    }
    // Batches of short objects (one segment, at most four interior tiles an
    // object: the apply path's rule at two waves per SIMD) walk flat.
    constexpr uint64_t TCV = 4 * bytes::enc_width(KS);
    const uint64_t nint = std::min<uint64_t>(bytes::interior_vectors(a.S, a.L, a.col0, a.k), ncols >> 2) / TCV;
    const bool flat = a.nobj > 1 && nseg == 1 && nint <= 4;
    const dim3 grid = flat ? dim3((uint32_t)blocks) : bytes_grid(ncols, (uint64_t)a.nobj * nseg, nseg, blocks, 1);
    hipLaunchKernelGGL((bytes::encode_bytes_mfma_kernel<KS, 0>), grid, dim3(kBlock), lds, s, a.slots, a.slot_stride,
                       a.L, chunk_stride(a), a.col0, ncols, a.S, a.nobj, a.rows, a.k, a.mfma, a.coeff, a.out_idx,
                       a.flags, a.mapping, nseg, record, units, flat ? 1u : 0u);
    if (hipError_t e = hipGetLastError()) return e;
    if (record) {
      a.sw->switched = true;
      a.sw->units = units;
      a.sw->nseg = nseg;
    }
    return hipSuccess;
  }
  if (a.scratch && a.sw && a.sw->switched && a.sw->units) {
    // Phase 1 after the switch: the list of tiles to redo, then the redo.
    bytes::SwitchLayout l;
    l.units = a.sw->units;
    uint32_t* count = l.count(a.scratch);
    if (hipError_t e = hipMemsetAsync(count, 0, sizeof(uint32_t), s)) return e;
    const uint64_t total = (uint64_t)a.nobj * l.units;
    const uint64_t lblocks = std::min<uint64_t>(1024, (total + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(bytes::mfma_redo_list_kernel, dim3((uint32_t)std::max<uint64_t>(lblocks, 1)), dim3(kBlock), 0, s,
                       l.record(a.scratch, a.nobj), a.mapping, a.flags, a.nobj, l.units, l.list(a.scratch), count);
    if (hipError_t e = hipGetLastError()) return e;
    hipLaunchKernelGGL((bytes::encode_bytes_mfma_redo_kernel<KS>), dim3((uint32_t)rblocks), dim3(kBlock), lds, s,
                       a.slots, a.slot_stride, a.L, chunk_stride(a), a.col0, ncols, a.S, a.nobj, a.rows, a.k, a.mfma,
                       a.coeff, a.out_idx, a.flags, a.mapping, a.sw->nseg, l.list(a.scratch), count, l.units);
    return hipGetLastError();
  }
  hipLaunchKernelGGL((bytes::encode_bytes_mfma_kernel<KS, 1>), bytes_grid(ncols, 1, 1, blocks1, 1), dim3(kBlock), lds,
                     s, a.slots, a.slot_stride, a.L, chunk_stride(a), a.col0, ncols, a.S, a.nobj, a.rows, a.k, a.mfma,
                     a.coeff, a.out_idx, a.flags, a.mapping, 1u, nullptr, 0u, 0u);
  return hipGetLastError();
}

template <int KS>
hipError_t dec_ks(const BytesLaunch& a, hipStream_t s) {
  const uint64_t ncols = a.ncols ? a.ncols : a.L;
  const uint32_t lds = apply::mfma_lds_bytes(mfma::mtiles(a.rows), KS);
  const uint64_t blocks = 256ull * apply::mfma_waves(KS, apply::mfma_width(KS));
  // Batches of short chunks: the flat walk (the apply path's rule, rs_apply_mfma.hip).
  const uint64_t flat_tiles = apply::mfma_waves(KS, apply::mfma_width(KS)) == 1 ? 32 : 4;
  const uint64_t tc = 16ull * apply::mfma_width(KS);
  const uint64_t tpo = ((ncols >> 2) * 4 + tc - 1) / tc;
  if (a.nobj > 1 && tpo <= flat_tiles) {
    const uint64_t nb = (tpo * a.nobj + apply::kWaves - 1) / apply::kWaves;
    const uint64_t gx = nb < 1 ? 1 : nb < blocks ? nb : blocks;
    hipLaunchKernelGGL((bytes::decode_bytes_mfma_kernel<KS>), dim3((uint32_t)gx), dim3(kBlock), lds, s, a.slots,
                       a.slot_stride, a.L, chunk_stride(a), a.col0, ncols, a.nobj, a.rows, a.k, a.mfma, a.coeff,
                       a.in_idx, a.out_idx, a.mapping, 1u, 1u);
    return hipGetLastError();
  }
  const uint32_t nseg = object_segments(a.nobj, ncols);
  hipLaunchKernelGGL((bytes::decode_bytes_mfma_kernel<KS>),
                     bytes_grid(ncols, (uint64_t)a.nobj * nseg, nseg, blocks, 1), dim3(kBlock), lds, s, a.slots,
                     a.slot_stride, a.L, chunk_stride(a), a.col0, ncols, a.nobj, a.rows, a.k, a.mfma, a.coeff,
                     a.in_idx, a.out_idx, a.mapping, nseg, 0u);
  return hipGetLastError();
}

}  // namespace

// Scratch of the matrix-core mid-object switch (bytes::SwitchLayout: count,
// redo list, one record byte per interior tile).
uint64_t encode_switch_bytes_mfma(const BytesLaunch& a) {
  if (a.phase != 0 || a.nobj == 0) return 0;
  uint32_t units = 0;
  switch (mfma::ksteps(a.k)) {
    case 2: units = switch_units<2>(a); break;
    case 3: units = switch_units<3>(a); break;
    case 4: units = switch_units<4>(a); break;
    case 5: units = switch_units<5>(a); break;
    case 6: units = switch_units<6>(a); break;
    case 7: units = switch_units<7>(a); break;
    default: return 0;
  }
  // No switch scratch when the list could reach the counter's flag bit: the
  // batch then re-encodes its switched objects whole (redo_list.hpp).
  if (!units || !bytes::redo_list_fits(a.nobj, units)) return 0;
  return 256 + 5ull * a.nobj * units;
}

bool bytes_mfma_eligible(const BytesLaunch& a, bool encode) {
  if (!a.mfma || !matrix_core_mode() || a.k < 17 || !mfma_wanted(a.k, a.rows) || !mfma::supported(a.rows, a.k))
    return false;
  // need 17..24 encodes on the VALU queue kernel, whose mid-object switch
  // redoes only part of a 1<<31 object.
  if (encode && a.k < 25) return false;
  if (!pipelined_kernels()) return false;  // kernel_pipeline(0): the non-pipelined VALU forms
  const uint64_t ncols = a.ncols ? a.ncols : a.L;
  // 32-bit byte offsets from the window base: every chunk the launch reads
  // or writes, plus the window's columns.
  // (Encode writes parity chunk k + out_idx[i]; decode reads in_idx and
  // writes out_idx: k + out_max bounds both.)
  const uint64_t hi_chunk = (uint64_t)a.k + a.out_max > a.in_max ? (uint64_t)a.k + a.out_max : a.in_max;
  return (hi_chunk + 1) * chunk_stride(a) + 4 * ncols < (1ull << 32);
}

hipError_t launch_encode_bytes_mfma(const BytesLaunch& a, hipStream_t s) {
  switch (mfma::ksteps(a.k)) {
    case 2: return enc_ks<2>(a, s);
    case 3: return enc_ks<3>(a, s);
    case 4: return enc_ks<4>(a, s);
    case 5: return enc_ks<5>(a, s);
    case 6: return enc_ks<6>(a, s);
    case 7: return enc_ks<7>(a, s);
    default: return hipErrorInvalidValue;  // 17 <= k <= 112 (bytes_mfma_eligible)
  }
}

hipError_t launch_decode_bytes_mfma(const BytesLaunch& a, hipStream_t s) {
  switch (mfma::ksteps(a.k)) {
    case 2: return dec_ks<2>(a, s);
    case 3: return dec_ks<3>(a, s);
    case 4: return dec_ks<4>(a, s);
    case 5: return dec_ks<5>(a, s);
    case 6: return dec_ks<6>(a, s);
    case 7: return dec_ks<7>(a, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace slime
