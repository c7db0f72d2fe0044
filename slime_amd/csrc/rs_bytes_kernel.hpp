// Fused byte-domain encode/decode kernels (device code) for CDNA4, shared by
// rs_bytes.hip (product) and tools/bytes_variants.hip (tuning): slime's writeChunks and
// reconstruct data paths (internal/store/multi/multi_store.go:516-557 and
// :215-242) on device, without materialising the symbol domain.
//
// Object slot layout (bytes): slot o starts at base + o*slot_stride; chunk c
// of object o is the 4L bytes at slot + c*chunk, L = ceil(ceil(S/4)/need)
// (splitVector, multi_store.go:272), chunk >= 4L the chunk stride (every
// kernel takes it).  With chunk = 4L (the wire layout) the object's S bytes
// occupy the start of its slot, so data chunk j IS bytes [4jL, 4(j+1)L) of
// the slot once the encoder has written the tail past S with what MapFromGF
// produces there; with a larger stride (chunks on the 256 B line grid) object
// byte i lives in chunk i / 4L at offset i % 4L.
//
// Encode (one object, mapping m chosen as gf.MapToGF does, map.go:15-67):
//   word w < nw = ceil(S/4): packed = BE(bytes[4w..4w+3]) (a partial last
//   word keeps its high bytes, low bytes zero, map.go:25-32); symbol =
//   packed ^ m.  Words nw..kL-1 are splitVector's zero padding (symbol 0,
//   NOT xor-ed).  Chunk word = BE(symbol ^ m) (MapFromGF, map.go:103-113):
//   parity chunks from the code rows, data-chunk tail = BE(packed) for the
//   partial word and BE(m) for padding words.
//   Speculative: pass 0 assumes m = 0 and reduces the two MapToGF flag bits
//   per object; a tiny kernel turns flags into m (0, 1<<31, or "fallback");
//   pass 1 re-encodes only objects whose m != 0 (other blocks exit at once).
// Decode: symbol = BE(chunk word) ^ m for the survivors, rebuilt chunk word =
//   BE(symbol ^ m) (MapToGFWith + RecoverData + MapFromGF).
#pragma once
#include <hip/hip_runtime.h>

#include "gfp.hpp"
#include "rs_apply_kernel.hpp"

namespace slime {
namespace bytes {

using apply::kBlock;
using apply::kCoeffStride;
using apply::kWaves;
using apply::u32x16;
using apply::u32x4;

__device__ __forceinline__ uint32_t be(uint32_t w) { return __builtin_bswap32(w); }

__device__ __forceinline__ uint32_t flag_bits(uint32_t w) {
  return (w >= kP ? 1u : 0u) | ((w ^ 0x80000000u) >= kP ? 2u : 0u);
}

struct ObjWords {
  uint64_t nw;        // ceil(S/4): words carrying object bytes
  uint32_t tailmask;  // mask of the valid high bytes of word nw-1 (0xFFFFFFFF if S%4 == 0)
};

// Symbol-domain word w of an object from the slot bytes loaded as `raw`.
// Returns the packed (pre-mapping) word; *pad says "splitVector padding".
__device__ __forceinline__ uint32_t packed_word(uint32_t raw, uint64_t w, const ObjWords& ow, bool* pad) {
  *pad = w >= ow.nw;
  const uint32_t p = be(raw);
  return *pad ? 0u : (w + 1 == ow.nw ? p & ow.tailmask : p);
}

template <int K>
__device__ __forceinline__ void rows_out(const uint32_t (&x)[K][4], uint32_t rows, const uint32_t* __restrict__ coeff,
                                         const uint32_t* __restrict__ out_idx, uint8_t* out_slot, uint64_t chunk,
                                         uint64_t byte_off, uint32_t m, int ncol) {
  for (uint32_t i = 0; i < rows; ++i) {
    const apply::CoeffRow<K> c = apply::load_coeff_row<K>(coeff, i);
    uint64_t lo0 = 0, lo1 = 0, lo2 = 0, lo3 = 0;
    uint32_t hi0 = 0, hi1 = 0, hi2 = 0, hi3 = 0;
#pragma unroll
    for (int j = 0; j < K; ++j) mac4(lo0, lo1, lo2, lo3, hi0, hi1, hi2, hi3, x[j][0], x[j][1], x[j][2], x[j][3], c[j]);
    uint8_t* dst = out_slot + (uint64_t)out_idx[i] * chunk + byte_off;
    if (ncol == 4) {
      const u32x4 v = {be(fold96(lo0, hi0) ^ m), be(fold96(lo1, hi1) ^ m), be(fold96(lo2, hi2) ^ m),
                       be(fold96(lo3, hi3) ^ m)};
      __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(dst));
    } else {
      reinterpret_cast<uint32_t*>(dst)[0] = be(fold96(lo0, hi0) ^ m);
    }
  }
}

// All output rows for U units of 4 columns: rows outer (one s_load_dwordx16
// of coefficients per row), units inner, so the units' independent MAC chains
// interleave.  valid_units: units [0, n) are inside the chunk.
template <int K, int U>
__device__ __forceinline__ void rows_out_units(const uint32_t (&x)[U][K][4], int n, uint32_t rows,
                                               const uint32_t* __restrict__ coeff,
                                               const uint32_t* __restrict__ out_idx, uint8_t* out_slot,
                                               uint64_t chunk, uint64_t g0, uint32_t m) {
  for (uint32_t i = 0; i < rows; ++i) {
    const apply::CoeffRow<K> c = apply::load_coeff_row<K>(coeff, i);
    uint8_t* const orow = out_slot + (uint64_t)out_idx[i] * chunk;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (u >= n) break;
      uint64_t lo0 = 0, lo1 = 0, lo2 = 0, lo3 = 0;
      uint32_t hi0 = 0, hi1 = 0, hi2 = 0, hi3 = 0;
#pragma unroll
      for (int j = 0; j < K; ++j)
        mac4(lo0, lo1, lo2, lo3, hi0, hi1, hi2, hi3, x[u][j][0], x[u][j][1], x[u][j][2], x[u][j][3], c[j]);
      const u32x4 v = {be(fold96(lo0, hi0) ^ m), be(fold96(lo1, hi1) ^ m), be(fold96(lo2, hi2) ^ m),
                       be(fold96(lo3, hi3) ^ m)};
      __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(orow + (((g0 + 64 * u) << 2) << 2)));
    }
  }
}

// MapToGF's two flag bits (map.go:35-62) as running maxima:
// bit0 <=> max(word) >= p, bit1 <=> max(word ^ 1<<31) >= p.  One accumulator
// pair per column lane c keeps four independent max chains instead of one
// serial chain through every word of a step.
struct Flags {
  uint32_t a[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0};
  __device__ __forceinline__ void add(int c, uint32_t w) {
    a[c] = a[c] > w ? a[c] : w;
    const uint32_t h = w ^ 0x80000000u;
    b[c] = b[c] > h ? b[c] : h;
  }
  __device__ __forceinline__ uint32_t bits() const {
    uint32_t ma = 0, mb = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      ma = ma > a[c] ? ma : a[c];
      mb = mb > b[c] ? mb : b[c];
    }
    return (ma >= kP ? 1u : 0u) | (mb >= kP ? 2u : 0u);
  }
};

// Load data chunk j's words of window columns [b, b+ncol) as symbols
// (mapping m, splitVector padding), folding the packed words into MapToGF's
// flags.  `slot` points at the window (object slot + 4*col0); the object word
// index of chunk j, window column b is j*L + col0 + b.
// INTERIOR: every word of the unit is a full object word (the bulk of every
// object) -- no padding/partial-word checks.
template <bool INTERIOR, bool FLAGS>
__device__ __forceinline__ void load_data_symbol(const uint8_t* slot, uint64_t chunk, uint64_t L, uint64_t col0,
                                                 uint32_t j, uint64_t b, int ncol, const ObjWords& ow, uint32_t m,
                                                 uint32_t (&x)[4], Flags* fl) {
  const uint8_t* src = slot + (uint64_t)j * chunk + 4 * b;
  uint32_t raw[4] = {0, 0, 0, 0};
  if (ncol == 4) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src));
    raw[0] = v.x, raw[1] = v.y, raw[2] = v.z, raw[3] = v.w;
  } else {
    raw[0] = *reinterpret_cast<const uint32_t*>(src);
  }
  if constexpr (INTERIOR) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const uint32_t p = be(raw[c]);
      if (FLAGS) fl->add(c, p);
      x[c] = p ^ m;
    }
  } else {
    const uint64_t w0 = (uint64_t)j * L + col0 + b;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      bool pad;
      const uint32_t p = packed_word(raw[c], w0 + c, ow, &pad);
      if (FLAGS && !pad && c < ncol) fl->add(c, p);
      x[c] = pad ? 0u : p ^ m;
    }
  }
}

template <int K, bool INTERIOR, bool FLAGS>
__device__ __forceinline__ void load_data_symbols(const uint8_t* slot, uint64_t chunk, uint64_t L, uint64_t col0,
                                                  uint64_t b, int ncol, const ObjWords& ow, uint32_t m,
                                                  uint32_t (&x)[K][4], Flags* fl) {
#pragma unroll
  for (int j = 0; j < K; ++j) load_data_symbol<INTERIOR, FLAGS>(slot, chunk, L, col0, j, b, ncol, ow, m, x[j], fl);
}

// Data chunk j's bytes from the last object word on (only units that reach
// it): BE(packed) for the partial word, BE(m) for splitVector padding words.
__device__ __forceinline__ void fix_data_tail_one(uint8_t* slot, uint64_t chunk, uint64_t L, uint64_t col0,
                                                  uint32_t j, uint64_t b, int ncol, const ObjWords& ow, uint32_t m,
                                                  const uint32_t (&x)[4]) {
  const uint64_t w0 = (uint64_t)j * L + col0 + b;
  if (w0 + ncol < ow.nw) return;
  uint32_t fix[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) fix[c] = be(w0 + c >= ow.nw ? m : x[c] ^ m);
  uint8_t* d = slot + (uint64_t)j * chunk + 4 * b;
  if (ncol == 4) {
    const u32x4 v = {fix[0], fix[1], fix[2], fix[3]};
    *reinterpret_cast<u32x4*>(d) = v;
  } else {
    *reinterpret_cast<uint32_t*>(d) = fix[0];
  }
}

template <int K>
__device__ __forceinline__ void fix_data_tail(uint8_t* slot, uint64_t chunk, uint64_t L, uint64_t col0, uint64_t b,
                                              int ncol, const ObjWords& ow, uint32_t m, const uint32_t (&x)[K][4]) {
#pragma unroll
  for (int j = 0; j < K; ++j) fix_data_tail_one(slot, chunk, L, col0, j, b, ncol, ow, m, x[j]);
}

// Work item wi of a launch = (object, column segment): each object's window
// is cut into nseg contiguous segments of whole vectors, scheduled like
// separate objects on blockIdx.y (rs_apply_kernel does the same), so a
// small batch keeps many independent chunk streams in flight.  The columns
// past the last whole vector belong to the object's last segment.
struct Segment {
  uint32_t obj;
  bool last;
  uint64_t v0, v1;  // vectors [v0, v1) of the window
};
__device__ __forceinline__ Segment segment_of(uint64_t wi, uint32_t nseg, uint64_t nvec) {
  const uint64_t per = apply::segment_vectors(nvec, nseg);
  const uint32_t seg = (uint32_t)(wi % nseg);
  Segment g;
  g.obj = (uint32_t)(wi / nseg);
  g.last = seg == nseg - 1;
  g.v0 = (uint64_t)seg * per < nvec ? (uint64_t)seg * per : nvec;
  g.v1 = g.v0 + per < nvec ? g.v0 + per : nvec;
  return g;
}

// Interior vectors of an encode window: vectors v (from the window's column
// 0) whose four words in the last data chunk (k-1) -- hence in every data
// chunk -- are whole object words, so no splitVector padding, partial last
// word or data-chunk tail is involved: lim + 4v + 3 < whole, with whole = nw
// (S a multiple of 4) or nw - 1 (the last word partial).  Objects whose size
// fills every chunk exactly (256 MiB at 8/12 and 64/80) are all interior.
__host__ __device__ inline uint64_t interior_vectors(uint64_t S, uint64_t L, uint64_t col0, uint32_t k) {
  const uint64_t nw = (S + 3) / 4;
  const uint64_t whole = S % 4 ? nw - 1 : nw;
  const uint64_t lim = (uint64_t)(k - 1) * L + col0;
  return whole > lim ? (whole - lim) / 4 : 0;
}

// MODE 0: speculative encode with m = 0, OR-ing MapToGF's flag bits into
//         flags[obj] (the caller's status array, zeroed first).
// MODE 1: re-encode objects with mapping[obj] != 0 and status[obj] == 0.
// Lanes own 4 columns (16 B per chunk) per unit; a wave issues the loads of
// U units (U KiB of every data chunk) before any math or store; columns past
// the last multiple of 4 go one per lane.
// Column window: columns [col0, col0 + ncols) of every chunk (col0 a
// multiple of 4; the whole object is col0 = 0, ncols = L).  Chunks stay 4L
// bytes apart; the host pipeline streams an object window by window.
template <int K, int U, int MODE, bool FAST = true, bool FLAGS_ON = true>
__global__ __launch_bounds__(kBlock) void encode_bytes_kernel(
    uint8_t* __restrict__ slots, uint64_t slot_stride, uint64_t L, uint64_t chunk, uint64_t col0, uint64_t ncols, uint64_t S,
    uint32_t nobj, uint32_t rows, const uint32_t* __restrict__ coeff, const uint32_t* __restrict__ out_idx,
    uint32_t* __restrict__ flags, const uint32_t* __restrict__ mapping, uint32_t nseg) {
  const ObjWords ow{(S + 3) / 4, S % 4 ? 0xFFFFFFFFu << (8 * (4 - S % 4)) : 0xFFFFFFFFu};
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  const uint64_t nwaves = (uint64_t)gridDim.x * kWaves;
  const uint64_t nvec = ncols >> 2;
  // Units whose columns reach the object's last word (or padding) need the
  // data-chunk tail fix; every other unit skips that branch.
  const uint64_t first_tail_word = ow.nw ? ow.nw - 1 : 0;
  for (uint64_t wi = blockIdx.y; wi < (uint64_t)nobj * nseg; wi += gridDim.y) {
    const Segment sg = segment_of(wi, nseg, nvec);
    const uint32_t obj = sg.obj;
    const uint64_t ntiles = (sg.v1 - sg.v0 + 64 * U - 1) / (64 * U);
    uint32_t m = 0;
    if constexpr (MODE == 1) {
      m = mapping[obj];
      if (m == 0 || flags[obj] != 0) continue;  // nothing to redo / random fallback pending (uniform per block)
    }
    uint8_t* const slot = slots + (uint64_t)obj * slot_stride + 4 * col0;  // window base
    uint8_t* const par = slot + (uint64_t)K * chunk;  // parity chunk i at par + out_idx[i]*chunk
    constexpr bool F = MODE == 0 && FLAGS_ON;
    Flags fl;
    for (uint64_t step = wave; step < ntiles; step += nwaves) {
      const uint64_t g0 = sg.v0 + step * (64 * U) + lane;
      // Interior step: the highest word the wave's units touch (last data
      // chunk, last unit) is below the object's last word: no checks needed.
      const uint64_t top = (uint64_t)(K - 1) * L + col0 + ((sg.v0 + step * (64 * U) + 64 * U) << 2);
      uint32_t x[U][K][4];
      if (FAST && top < first_tail_word && sg.v0 + (step + 1) * (64 * U) <= sg.v1) {
#pragma unroll
        for (int u = 0; u < U; ++u)
          load_data_symbols<K, true, F>(slot, chunk, L, col0, (g0 + 64 * u) << 2, 4, ow, m, x[u], &fl);
        rows_out_units<K, U>(x, U, rows, coeff, out_idx, par, chunk, g0, m);
        continue;
      }
      // Edge step: units past the chunk end are skipped; units reaching the
      // object's last word also rewrite the data-chunk tail.  Units inside
      // the chunk always form a prefix [0, n) of the step's units.
      int n = 0;
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (g0 + 64 * u < sg.v1) {
          load_data_symbols<K, false, F>(slot, chunk, L, col0, (g0 + 64 * u) << 2, 4, ow, m, x[u], &fl);
          n = u + 1;
        }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (u >= n) break;
        const uint64_t b = (g0 + 64 * u) << 2;
        if ((uint64_t)(K - 1) * L + col0 + b + 4 > first_tail_word)
          fix_data_tail<K>(slot, chunk, L, col0, b, 4, ow, m, x[u]);
      }
      rows_out_units<K, U>(x, n, rows, coeff, out_idx, par, chunk, g0, m);
    }
    for (uint64_t b = (nvec << 2) + wave * 64 + lane; sg.last && b < ncols; b += nwaves * 64) {
      uint32_t x[K][4];
      load_data_symbols<K, false, F>(slot, chunk, L, col0, b, 1, ow, m, x, &fl);
      fix_data_tail<K>(slot, chunk, L, col0, b, 1, ow, m, x);
      rows_out<K>(x, rows, coeff, out_idx, par, chunk, 4 * b, m, 1);
    }
    if constexpr (F) {
      const uint32_t f = fl.bits();
      const uint64_t a1 = __ballot(f & 1u), a2 = __ballot(f & 2u);
      const uint32_t wf = (a1 ? 1u : 0u) | (a2 ? 2u : 0u);
      if (wf && lane == 0) atomicOr(&flags[obj], wf);
    }
  }
}


// Decode: rebuild `rows` chunks (out_idx slots) from need survivors (in_idx).
template <int K>
__device__ __forceinline__ void load_chunk_symbols(const uint8_t* slot, const uint64_t (&ioff)[K], uint64_t b,
                                                   int ncol, uint32_t m, uint32_t (&x)[K][4]) {
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const uint8_t* src = slot + ioff[j] + 4 * b;
    if (ncol == 4) {
      const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src));
      x[j][0] = be(v.x) ^ m, x[j][1] = be(v.y) ^ m, x[j][2] = be(v.z) ^ m, x[j][3] = be(v.w) ^ m;
    } else {
      x[j][0] = be(*reinterpret_cast<const uint32_t*>(src)) ^ m;
      x[j][1] = x[j][2] = x[j][3] = 0;
    }
  }
}

// Column window [col0, col0 + ncols) as in encode_bytes_kernel.
template <int K, int U>
__global__ __launch_bounds__(kBlock) void decode_bytes_kernel(uint8_t* __restrict__ slots, uint64_t slot_stride,
                                                              uint64_t L, uint64_t chunk, uint64_t col0, uint64_t ncols,
                                                              uint32_t nobj, uint32_t rows,
                                                              const uint32_t* __restrict__ coeff,
                                                              const uint32_t* __restrict__ in_idx,
                                                              const uint32_t* __restrict__ out_idx,
                                                              const uint32_t* __restrict__ mapping, uint32_t nseg) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  const uint64_t nwaves = (uint64_t)gridDim.x * kWaves;
  const uint64_t nvec = ncols >> 2;
  for (uint64_t wi = blockIdx.y; wi < (uint64_t)nobj * nseg; wi += gridDim.y) {
    const Segment sg = segment_of(wi, nseg, nvec);
    const uint32_t obj = sg.obj;
    const uint64_t ntiles = (sg.v1 - sg.v0 + 64 * U - 1) / (64 * U);
    const uint32_t m = mapping[obj];
    uint8_t* const slot = slots + (uint64_t)obj * slot_stride + 4 * col0;  // window base
    uint64_t ioff[K];
#pragma unroll
    for (int j = 0; j < K; ++j) ioff[j] = (uint64_t)in_idx[j] * chunk;
    for (uint64_t step = wave; step < ntiles; step += nwaves) {
      const uint64_t g0 = sg.v0 + step * (64 * U) + lane;
      uint32_t x[U][K][4];
      int n = 0;
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (g0 + 64 * u < sg.v1) {
          load_chunk_symbols<K>(slot, ioff, (g0 + 64 * u) << 2, 4, m, x[u]);
          n = u + 1;
        }
      rows_out_units<K, U>(x, n, rows, coeff, out_idx, slot, chunk, g0, m);
    }
    for (uint64_t b = (nvec << 2) + wave * 64 + lane; sg.last && b < ncols; b += nwaves * 64) {
      uint32_t x[K][4];
      load_chunk_symbols<K>(slot, ioff, b, 1, m, x);
      rows_out<K>(x, rows, coeff, out_idx, slot, chunk, 4 * b, m, 1);
    }
  }
}

// ---- software-pipelined forms (need <= 16, chunks < 4 GiB) -----------------
// The byte kernels above with rs_apply_pipe_kernel's pipeline: a wave issues
// the raw 16-byte loads of its next tile before it transforms, computes and
// stores the current one (two register sets of K x U raw vectors).  Loads
// are unconditional (lanes past the segment end re-read its last vector:
// flags are running maxima, so the repeats change nothing), and the raw ->
// symbol transform reads every loaded register before any row math, so the
// waitcnt pass resolves a tile's loads there and leaves the other set in
// flight.  Addresses are wave-uniform chunk bases plus 32-bit byte offsets
// (chunk = 4L < 4 GiB, checked by the host).
template <int K, int U>
__device__ __forceinline__ void load_raw_tile(uint4 (&r)[U][K], const uint8_t* const (&cb)[K], uint32_t g0,
                                              uint32_t v1) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t g = g0 + 64 * u < v1 ? g0 + 64 * u : v1 - 1;
#pragma unroll
    for (int j = 0; j < K; ++j) r[u][j] = apply::ld16_at<true>(reinterpret_cast<const uint32_t*>(cb[j]), g << 4);
  }
}

// Rows of a tile from its symbols (columns as 4-vectors), BE(symbol ^ m)
// stored into chunk out_idx[i] of the window at `base`, for the lanes whose
// unit lies inside the segment.
template <int K, int U>
__device__ __forceinline__ void rows_tile(const uint4 (&x)[U][K], uint32_t rows, const uint32_t* __restrict__ coeff,
                                          const uint32_t* __restrict__ out_idx, uint8_t* base, uint64_t chunk,
                                          uint32_t g0, uint32_t v1, uint32_t m) {
  for (uint32_t i = 0; i < rows; ++i) {
    const apply::CoeffRow<K> c = apply::load_coeff_row<K>(coeff, i);
    uint8_t* const orow = base + (uint64_t)out_idx[i] * chunk;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint4 r = apply::dot4<K>(x[u], c);
      const u32x4 v = {be(r.x ^ m), be(r.y ^ m), be(r.z ^ m), be(r.w ^ m)};
      if (g0 + 64 * u < v1) __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(orow + ((g0 + 64 * u) << 4)));
    }
  }
}

template <int K, int U>
__global__ __launch_bounds__(kBlock) void decode_bytes_pipe_kernel(
    uint8_t* __restrict__ slots, uint64_t slot_stride, uint64_t L, uint64_t chunk, uint64_t col0, uint64_t ncols, uint32_t nobj,
    uint32_t rows, const uint32_t* __restrict__ coeff, const uint32_t* __restrict__ in_idx,
    const uint32_t* __restrict__ out_idx, const uint32_t* __restrict__ mapping, uint32_t nseg) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = blockIdx.x * kWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nwaves = gridDim.x * kWaves;
  const uint64_t nvec = ncols >> 2;
  for (uint64_t wi = blockIdx.y; wi < (uint64_t)nobj * nseg; wi += gridDim.y) {
    const Segment sg = segment_of(wi, nseg, nvec);
    const uint32_t v0 = (uint32_t)sg.v0, v1 = (uint32_t)sg.v1;
    const uint32_t ntiles = (v1 - v0 + 64 * U - 1) / (64 * U);
    const uint32_t m = mapping[sg.obj];
    uint8_t* const slot = slots + (uint64_t)sg.obj * slot_stride + 4 * col0;  // window base
    const uint8_t* cb[K];
#pragma unroll
    for (int j = 0; j < K; ++j) cb[j] = slot + (uint64_t)in_idx[j] * chunk;
    uint4 ra[U][K], rb[U][K];
    uint32_t step = wave;
    if (step < ntiles) load_raw_tile<K, U>(ra, cb, v0 + step * (64 * U) + lane, v1);
    while (step < ntiles) {
      uint32_t next = step + nwaves;
      load_raw_tile<K, U>(rb, cb, v0 + (next < ntiles ? next : step) * (64 * U) + lane, v1);
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < K; ++j)
          ra[u][j] = make_uint4(be(ra[u][j].x) ^ m, be(ra[u][j].y) ^ m, be(ra[u][j].z) ^ m, be(ra[u][j].w) ^ m);
      rows_tile<K, U>(ra, rows, coeff, out_idx, slot, chunk, v0 + step * (64 * U) + lane, v1, m);
      step = next;
      if (step >= ntiles) break;
      next = step + nwaves;
      load_raw_tile<K, U>(ra, cb, v0 + (next < ntiles ? next : step) * (64 * U) + lane, v1);
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < K; ++j)
          rb[u][j] = make_uint4(be(rb[u][j].x) ^ m, be(rb[u][j].y) ^ m, be(rb[u][j].z) ^ m, be(rb[u][j].w) ^ m);
      rows_tile<K, U>(rb, rows, coeff, out_idx, slot, chunk, v0 + step * (64 * U) + lane, v1, m);
      step = next;
    }
    uint64_t ioff[K];
#pragma unroll
    for (int j = 0; j < K; ++j) ioff[j] = (uint64_t)in_idx[j] * chunk;
    for (uint64_t b = (nvec << 2) + (uint64_t)wave * 64 + lane; sg.last && b < ncols; b += (uint64_t)nwaves * 64) {
      uint32_t x[K][4];
      load_chunk_symbols<K>(slot, ioff, b, 1, m, x);
      rows_out<K>(x, rows, coeff, out_idx, slot, chunk, 4 * b, m, 1);
    }
  }
}

// Interior tile of the encode: raw data-chunk vectors -> symbols (mapping
// m, MapToGF flags; no padding or partial word), then every parity row.
template <int K, int U, bool F>
__device__ __forceinline__ void encode_interior_tile(uint4 (&r)[U][K], uint8_t* par, uint64_t chunk, uint32_t m,
                                                     uint32_t rows, const uint32_t* __restrict__ coeff,
                                                     const uint32_t* __restrict__ out_idx, uint32_t g0, uint32_t v1,
                                                     Flags& fl) {
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int j = 0; j < K; ++j) {
      uint32_t w[4] = {r[u][j].x, r[u][j].y, r[u][j].z, r[u][j].w};
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const uint32_t p = be(w[c]);
        if (F) fl.add(c, p);
        w[c] = p ^ m;
      }
      r[u][j] = make_uint4(w[0], w[1], w[2], w[3]);
    }
  rows_tile<K, U>(r, rows, coeff, out_idx, par, chunk, g0, v1, m);
}

// MODE as in encode_bytes_kernel.  A segment's tiles split into an interior
// prefix -- whole tiles whose highest word (last data chunk, last unit) is
// below the object's last word: the pipelined loop -- and the few edge tiles
// after it (padding, the partial last word, the segment's partial last
// tile), which take encode_bytes_kernel's edge step without the pipeline.
template <int K, int U, int MODE>
__global__ __launch_bounds__(kBlock) void encode_bytes_pipe_kernel(
    uint8_t* __restrict__ slots, uint64_t slot_stride, uint64_t L, uint64_t chunk, uint64_t col0, uint64_t ncols, uint64_t S,
    uint32_t nobj, uint32_t rows, const uint32_t* __restrict__ coeff, const uint32_t* __restrict__ out_idx,
    uint32_t* __restrict__ flags, const uint32_t* __restrict__ mapping, uint32_t nseg) {
  const ObjWords ow{(S + 3) / 4, S % 4 ? 0xFFFFFFFFu << (8 * (4 - S % 4)) : 0xFFFFFFFFu};
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = blockIdx.x * kWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nwaves = gridDim.x * kWaves;
  const uint64_t nvec = ncols >> 2;
  const uint64_t first_tail_word = ow.nw ? ow.nw - 1 : 0;
  constexpr bool F = MODE == 0;
  for (uint64_t wi = blockIdx.y; wi < (uint64_t)nobj * nseg; wi += gridDim.y) {
    const Segment sg = segment_of(wi, nseg, nvec);
    const uint32_t obj = sg.obj;
    const uint32_t v0 = (uint32_t)sg.v0, v1 = (uint32_t)sg.v1;
    const uint32_t ntiles = (v1 - v0 + 64 * U - 1) / (64 * U);
    uint32_t m = 0;
    if constexpr (MODE == 1) {
      m = mapping[obj];
      if (m == 0 || flags[obj] != 0) continue;  // uniform per block
    }
    uint8_t* const slot = slots + (uint64_t)obj * slot_stride + 4 * col0;  // window base
    uint8_t* const par = slot + (uint64_t)K * chunk;
    // Interior tiles st < nint: end = v0 + (st+1)*64U <= v1 and
    // (K-1)L + col0 + 4*end < first_tail_word.
    uint64_t end_max = interior_vectors(S, L, col0, K);
    if (end_max > v1) end_max = v1;
    const uint32_t nint = end_max > v0 ? (uint32_t)((end_max - v0) / (64 * U)) : 0u;
    const uint8_t* cb[K];
#pragma unroll
    for (int j = 0; j < K; ++j) cb[j] = slot + (uint64_t)j * chunk;
    Flags fl;
    uint4 ra[U][K], rb[U][K];
    uint32_t step = wave;
    if (step < nint) load_raw_tile<K, U>(ra, cb, v0 + step * (64 * U) + lane, v1);
    while (step < nint) {
      uint32_t next = step + nwaves;
      load_raw_tile<K, U>(rb, cb, v0 + (next < nint ? next : step) * (64 * U) + lane, v1);
      encode_interior_tile<K, U, F>(ra, par, chunk, m, rows, coeff, out_idx, v0 + step * (64 * U) + lane, v1, fl);
      step = next;
      if (step >= nint) break;
      next = step + nwaves;
      load_raw_tile<K, U>(ra, cb, v0 + (next < nint ? next : step) * (64 * U) + lane, v1);
      encode_interior_tile<K, U, F>(rb, par, chunk, m, rows, coeff, out_idx, v0 + step * (64 * U) + lane, v1, fl);
      step = next;
    }
    // Edge tiles (encode_bytes_kernel's edge step).
    for (uint32_t st = nint + wave; st < ntiles; st += nwaves) {
      const uint64_t g0 = (uint64_t)v0 + (uint64_t)st * (64 * U) + lane;
      uint32_t x[U][K][4];
      int n = 0;
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (g0 + 64 * u < v1) {
          load_data_symbols<K, false, F>(slot, chunk, L, col0, (g0 + 64 * u) << 2, 4, ow, m, x[u], &fl);
          n = u + 1;
        }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (u >= n) break;
        const uint64_t b = (g0 + 64 * u) << 2;
        if ((uint64_t)(K - 1) * L + col0 + b + 4 > first_tail_word)
          fix_data_tail<K>(slot, chunk, L, col0, b, 4, ow, m, x[u]);
      }
      rows_out_units<K, U>(x, n, rows, coeff, out_idx, par, chunk, g0, m);
    }
    for (uint64_t b = (nvec << 2) + (uint64_t)wave * 64 + lane; sg.last && b < ncols; b += (uint64_t)nwaves * 64) {
      uint32_t x[K][4];
      load_data_symbols<K, false, F>(slot, chunk, L, col0, b, 1, ow, m, x, &fl);
      fix_data_tail<K>(slot, chunk, L, col0, b, 1, ow, m, x);
      rows_out<K>(x, rows, coeff, out_idx, par, chunk, 4 * b, m, 1);
    }
    if constexpr (F) {
      const uint32_t f = fl.bits();
      const uint64_t a1 = __ballot(f & 1u), a2 = __ballot(f & 2u);
      const uint32_t wf = (a1 ? 1u : 0u) | (a2 ? 2u : 0u);
      if (wf && lane == 0) atomicOr(&flags[obj], wf);
    }
  }
}

// ---- dynamic schedule (need <= 16, chunks < 4 GiB): the product forms -------
// The pipelined byte kernels above with rs_apply_queue_kernel's ticket walk
// (apply::TicketWalk: units of C tiles drawn from NC counters, zero at launch,
// each launch zeroing `zero_next`), so the faster XCDs take more of the
// batch.  Every object of a launch has the same window, so a unit is any
// object's tiles and the schedule spans the whole batch.
template <int K, int U, int C, int NC>
__global__ __launch_bounds__(kBlock) void decode_bytes_queue_kernel(
    uint8_t* __restrict__ slots, uint64_t slot_stride, uint64_t L, uint64_t chunk, uint64_t col0, uint64_t ncols, uint32_t nobj,
    uint32_t rows, const uint32_t* __restrict__ coeff, const uint32_t* __restrict__ in_idx,
    const uint32_t* __restrict__ out_idx, const uint32_t* __restrict__ mapping, uint32_t* __restrict__ ticket,
    uint32_t spread) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t nvec = (uint32_t)(ncols >> 2);
  const uint32_t ntiles = (nvec + 64 * U - 1) / (64 * U);
  uint64_t ioff[K];
#pragma unroll
  for (int j = 0; j < K; ++j) ioff[j] = (uint64_t)in_idx[j] * chunk;
  auto window = [&](uint32_t o) { return slots + (uint64_t)o * slot_stride + 4 * col0; };
  auto load = [&](uint4(&r)[U][K], uint32_t o, uint32_t t) {
    const uint8_t* cb[K];
#pragma unroll
    for (int j = 0; j < K; ++j) cb[j] = window(o) + ioff[j];
    load_raw_tile<K, U>(r, cb, t * (64 * U) + lane, nvec);
  };
  // The tile's mapping is read when its loads are issued, so it is in SGPRs by the math.
  auto compute = [&](const uint4(&r)[U][K], uint32_t o, uint32_t t, uint32_t m) {
    uint4 x[U][K];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < K; ++j)
        x[u][j] = make_uint4(be(r[u][j].x) ^ m, be(r[u][j].y) ^ m, be(r[u][j].z) ^ m, be(r[u][j].w) ^ m);
    rows_tile<K, U>(x, rows, coeff, out_idx, window(o), chunk, t * (64 * U) + lane, nvec, m);
  };
  apply::TicketWalk<C, NC> w(ticket, nobj, ntiles, lane, spread);
  if (w.live) {
    uint4 ra[U][K], rb[U][K];
    uint32_t ma = mapping[w.obj], mb = 0;
    load(ra, w.obj, w.tile());
    for (;;) {
      uint32_t co = w.obj, ct = w.tile();
      w.advance();
      mb = mapping[w.live ? w.obj : co];
      load(rb, w.live ? w.obj : co, w.live ? w.tile() : ct);
      compute(ra, co, ct, ma);
      if (!w.live) break;
      co = w.obj;
      ct = w.tile();
      w.advance();
      ma = mapping[w.live ? w.obj : co];
      load(ra, w.live ? w.obj : co, w.live ? w.tile() : ct);
      compute(rb, co, ct, mb);
      if (!w.live) break;
    }
  }
  w.finish();
  // Columns past the last whole vector of each object, one per lane.
  const uint32_t tailc = (uint32_t)(ncols - ((uint64_t)nvec << 2));
  const uint64_t tid = (uint64_t)blockIdx.x * kBlock + threadIdx.x, nthr = (uint64_t)gridDim.x * kBlock;
  for (uint64_t t = tid; tailc && t < (uint64_t)nobj * tailc; t += nthr) {
    const uint32_t o = (uint32_t)(t / tailc);
    const uint64_t b = ((uint64_t)nvec << 2) + t % tailc;
    const uint32_t m = mapping[o];
    uint32_t x[K][4];
    load_chunk_symbols<K>(window(o), ioff, b, 1, m, x);
    rows_out<K>(x, rows, coeff, out_idx, window(o), chunk, 4 * b, m, 1);
  }
}

// Interior tiles of an encode window (encode_bytes_pipe_kernel's pipelined
// prefix, the same count for every object): tiles t with (t+1)*64U <= nvec
// of interior vectors.  Host and device compute it alike (the redo list
// needs the count).
__host__ __device__ inline uint32_t encode_interior_tiles(uint64_t S, uint64_t L, uint64_t col0, uint64_t ncols, int K,
                                                          int U) {
  uint64_t end_max = interior_vectors(S, L, col0, (uint32_t)K);
  const uint64_t nvec = ncols >> 2;
  if (end_max > nvec) end_max = nvec;
  return (uint32_t)(end_max / (64 * (uint64_t)U));
}

// Top bits of a mapping-0 tile, for the second pass's parity correction
// (encode_bytes_fix_kernel): a lane's string holds, for vector u and column
// c, the K top bits of its column as one K-bit field at bit (u*4 + c)*K (bit
// j of the field = bit 31 of chunk j's packed word = bit 7 of the raw
// little-endian load), so the correction reads a column's field as one table
// index.  Planes of 32 bits per lane (plane q at tile + 256 q,
// lane-contiguous), the last plane only as wide as the bits left: K/8 bytes
// per column.
template <int K, int U>
struct TopBits {
  static constexpr int kBits = K * U * 4;
  static constexpr int kWords = (kBits + 31) / 32;
  static constexpr int kLastBits = kBits - 32 * (kWords - 1);
  static constexpr int kLastBytes = kLastBits <= 8 ? 1 : kLastBits <= 16 ? 2 : 4;
  static constexpr uint64_t kTileBytes = 64ull * (4 * (kWords - 1) + kLastBytes);
};
// Widest code the correction takes: its table holds 2^K entries per row.
constexpr int kTopBitsMaxK = 10;

template <int K, int U>
__device__ __forceinline__ void store_top_bits(const uint4 (&r)[U][K], uint8_t* __restrict__ tile, uint32_t lane) {
  using T = TopBits<K, U>;
  uint32_t w[T::kWords];
#pragma unroll
  for (int q = 0; q < T::kWords; ++q) w[q] = 0;
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const uint32_t t[4] = {(r[u][j].x >> 7) & 1u, (r[u][j].y >> 7) & 1u, (r[u][j].z >> 7) & 1u,
                             (r[u][j].w >> 7) & 1u};
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int b = (u * 4 + c) * K + j;
        w[b >> 5] |= t[c] << (b & 31);
      }
    }
#pragma unroll
  for (int q = 0; q + 1 < T::kWords; ++q)
    __builtin_nontemporal_store(w[q], reinterpret_cast<uint32_t*>(tile + 256 * q) + lane);
  uint8_t* const last = tile + 256 * (T::kWords - 1);
  if constexpr (T::kLastBytes == 1)
    last[lane] = (uint8_t)w[T::kWords - 1];
  else if constexpr (T::kLastBytes == 2)
    reinterpret_cast<uint16_t*>(last)[lane] = (uint16_t)w[T::kWords - 1];
  else
    __builtin_nontemporal_store(w[T::kWords - 1], reinterpret_cast<uint32_t*>(last) + lane);
}

template <int K, int U>
__device__ __forceinline__ void load_top_bits(const uint8_t* __restrict__ tile, uint32_t lane,
                                              uint32_t (&w)[TopBits<K, U>::kWords]) {
  using T = TopBits<K, U>;
#pragma unroll
  for (int q = 0; q + 1 < T::kWords; ++q) w[q] = reinterpret_cast<const uint32_t*>(tile + 256 * q)[lane];
  const uint8_t* const last = tile + 256 * (T::kWords - 1);
  if constexpr (T::kLastBytes == 1)
    w[T::kWords - 1] = last[lane];
  else if constexpr (T::kLastBytes == 2)
    w[T::kWords - 1] = reinterpret_cast<const uint16_t*>(last)[lane];
  else
    w[T::kWords - 1] = reinterpret_cast<const uint32_t*>(last)[lane];
}

// The K-bit field of vector u, column c from a lane's loaded planes.
template <int K, int U>
__device__ __forceinline__ uint32_t top_field(const uint32_t (&w)[TopBits<K, U>::kWords], int u, int c) {
  const int b = (u * 4 + c) * K, q = b >> 5;
  uint64_t v = w[q];
  if (q + 1 < TopBits<K, U>::kWords) v |= (uint64_t)w[q + 1] << 32;
  return (uint32_t)(v >> (b & 31)) & ((1u << K) - 1);
}

// MODE 0 (speculative) encode on the ticket walk: the interior tiles are
// dealt as units; the few edge tiles and column tails of every object follow,
// spread over all waves (mapping 0).  MapToGF's flags (map.go:35-62) are OR-ed
// into flags[obj] as soon as a tile shows a new bit.
//
// Mid-object switch (record != nullptr): a wave entering a unit reads its
// object's flags; once some word >= p has been seen, the object cannot keep
// mapping 0, so the unit is encoded with 1<<31 straight away, and
// record[obj * units + unit] says which mapping it used.  Phase 1
// (encode_bytes_redo_kernel) then redoes only the units whose mapping differs
// from the one the object ends with -- the units encoded before the first
// word >= p was seen -- instead of the whole object.  A stale flag read only
// delays the switch: the record always tells what the unit wrote.
//
// BITS (encode_bytes_queue_bits_kernel): every interior tile encoded with
// mapping 0 also stores its top bits (TopBits) at bits + (obj * nint + tile)
// * kTileBytes, so phase 1 corrects the listed units' parity
// (encode_bytes_fix_kernel) instead of re-encoding them.  Kept per tile:
// buffering a unit's bits in registers and storing them as whole lines at the
// unit's end cost the first pass the same (+2.4% vs +2.2% at 10/14,
// profiles/r06/s22_layout/).
template <int K, int U, int C, int NC, bool BITS>
__device__ __forceinline__ void encode_queue_body(
    uint8_t* __restrict__ slots, uint64_t slot_stride, uint64_t L, uint64_t chunk, uint64_t col0, uint64_t ncols, uint64_t S,
    uint32_t nobj, uint32_t rows, const uint32_t* __restrict__ coeff, const uint32_t* __restrict__ out_idx,
    uint32_t* __restrict__ flags, uint32_t* __restrict__ ticket, uint32_t spread, uint8_t* __restrict__ record,
    uint32_t units, uint8_t* __restrict__ bits) {
  const ObjWords ow{(S + 3) / 4, S % 4 ? 0xFFFFFFFFu << (8 * (4 - S % 4)) : 0xFFFFFFFFu};
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = blockIdx.x * kWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nwaves = gridDim.x * kWaves;
  const uint32_t nvec = (uint32_t)(ncols >> 2);
  const uint32_t ntiles = (nvec + 64 * U - 1) / (64 * U);
  const uint64_t first_tail_word = ow.nw ? ow.nw - 1 : 0;
  const uint32_t nint = encode_interior_tiles(S, L, col0, ncols, K, U);
  const bool sw = record != nullptr;
  auto window = [&](uint32_t o) { return slots + (uint64_t)o * slot_stride + 4 * col0; };
  auto load = [&](uint4(&r)[U][K], uint32_t o, uint32_t t) {
    const uint8_t* cb[K];
#pragma unroll
    for (int j = 0; j < K; ++j) cb[j] = window(o) + (uint64_t)j * chunk;
    load_raw_tile<K, U>(r, cb, t * (64 * U) + lane, nvec);
  };
  // The mapping a unit of object o starts with: 1<<31 once bit 0 is set.
  // Every lane loads the word (one request); the value stays in a VGPR and
  // is waited for only when the unit's first tile is computed.
  auto unit_mapping = [&](uint32_t o) -> uint32_t {
    const uint32_t f = __hip_atomic_load(flags + o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return (f & 1u) ? 0x80000000u : 0u;
  };
  Flags fl;
  uint32_t fobj = 0xFFFFFFFFu, sent = 0;  // the object fl belongs to, bits already OR-ed into flags[fobj]
  auto publish = [&] {  // OR the wave's new flag bits into flags[fobj] (wave-uniform)
    const uint32_t f = fl.bits();
    const uint32_t wf = (__ballot(f & 1u) ? 1u : 0u) | (__ballot(f & 2u) ? 2u : 0u);
    if (wf & ~sent) {
      if (lane == 0) atomicOr(&flags[fobj], wf);
      sent |= wf;
    }
  };
  auto compute = [&](uint4(&r)[U][K], uint32_t o, uint32_t t, uint32_t m, bool first, uint32_t unit) {
    if (o != fobj) {
      fl = Flags();
      fobj = o;
      sent = 0;
    }
    if (sw && first && lane == 0) record[(uint64_t)o * units + unit] = m ? 1 : 0;
    if constexpr (BITS)
      if (m == 0) store_top_bits<K, U>(r, bits + ((uint64_t)o * nint + t) * TopBits<K, U>::kTileBytes, lane);
    encode_interior_tile<K, U, true>(r, window(o) + (uint64_t)K * chunk, chunk, m, rows, coeff, out_idx,
                                     t * (64 * U) + lane, nvec, fl);
    publish();
  };
  {
    apply::TicketWalk<C, NC> w(ticket, nobj, nint, lane, spread);
    if (w.live) {
      uint4 ra[U][K], rb[U][K];
      uint32_t ma = sw ? unit_mapping(w.obj) : 0u, mb = 0;
      uint32_t ua = w.unit(), ub = 0;
      bool fa = true, fb = false;
      load(ra, w.obj, w.tile());
      for (;;) {
        uint32_t co = w.obj, ct = w.tile();
        w.advance();
        fb = w.live && w.unit_start();
        mb = sw && fb ? unit_mapping(w.obj) : ma;
        ub = w.unit();
        load(rb, w.live ? w.obj : co, w.live ? w.tile() : ct);
        compute(ra, co, ct, ma, fa, ua);
        if (!w.live) break;
        co = w.obj;
        ct = w.tile();
        w.advance();
        fa = w.live && w.unit_start();
        ma = sw && fa ? unit_mapping(w.obj) : mb;
        ua = w.unit();
        load(ra, w.live ? w.obj : co, w.live ? w.tile() : ct);
        compute(rb, co, ct, mb, fb, ub);
        if (!w.live) break;
      }
    }
    w.finish();
  }
  // Edge tiles [nint, ntiles) of every object (encode_bytes_kernel's edge step).
  const uint32_t nedge = ntiles - nint;
  for (uint64_t e = wave; e < (uint64_t)nobj * nedge; e += nwaves) {
    const uint32_t o = (uint32_t)(e / nedge);
    if (o != fobj) {
      fl = Flags();
      fobj = o;
      sent = 0;
    }
    uint8_t* const slot = window(o);
    const uint64_t g0 = (uint64_t)(nint + (uint32_t)(e % nedge)) * (64 * U) + lane;
    uint32_t x[U][K][4];
    int n = 0;
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (g0 + 64 * u < nvec) {
        load_data_symbols<K, false, true>(slot, chunk, L, col0, (g0 + 64 * u) << 2, 4, ow, 0u, x[u], &fl);
        n = u + 1;
      }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (u >= n) break;
      const uint64_t b = (g0 + 64 * u) << 2;
      if ((uint64_t)(K - 1) * L + col0 + b + 4 > first_tail_word) fix_data_tail<K>(slot, chunk, L, col0, b, 4, ow, 0u, x[u]);
    }
    rows_out_units<K, U>(x, n, rows, coeff, out_idx, slot + (uint64_t)K * chunk, chunk, g0, 0u);
    publish();
  }
  // Columns past the last whole vector of each object, one per lane.
  const uint32_t tailc = (uint32_t)(ncols - ((uint64_t)nvec << 2));
  const uint64_t tid = (uint64_t)blockIdx.x * kBlock + threadIdx.x, nthr = (uint64_t)gridDim.x * kBlock;
  for (uint64_t t = tid; tailc && t < (uint64_t)nobj * tailc; t += nthr) {
    const uint32_t o = (uint32_t)(t / tailc);
    uint8_t* const slot = window(o);
    const uint64_t b = ((uint64_t)nvec << 2) + t % tailc;
    uint32_t x[K][4];
    Flags f1;
    load_data_symbols<K, false, true>(slot, chunk, L, col0, b, 1, ow, 0u, x, &f1);
    fix_data_tail<K>(slot, chunk, L, col0, b, 1, ow, 0u, x);
    rows_out<K>(x, rows, coeff, out_idx, slot + (uint64_t)K * chunk, chunk, 4 * b, 0u, 1);
    const uint32_t f = f1.bits();
    if (f) atomicOr(&flags[o], f);  // per lane: tails are a handful of columns per object
  }
}

template <int K, int U, int C, int NC>
__global__ __launch_bounds__(kBlock) void encode_bytes_queue_kernel(
    uint8_t* __restrict__ slots, uint64_t slot_stride, uint64_t L, uint64_t chunk, uint64_t col0, uint64_t ncols, uint64_t S,
    uint32_t nobj, uint32_t rows, const uint32_t* __restrict__ coeff, const uint32_t* __restrict__ out_idx,
    uint32_t* __restrict__ flags, uint32_t* __restrict__ ticket, uint32_t spread, uint8_t* __restrict__ record,
    uint32_t units) {
  encode_queue_body<K, U, C, NC, false>(slots, slot_stride, L, chunk, col0, ncols, S, nobj, rows, coeff, out_idx, flags,
                                        ticket, spread, record, units, nullptr);
}
// The same with the top-bit store (record != nullptr, K <= kTopBitsMaxK).
template <int K, int U, int C, int NC>
__global__ __launch_bounds__(kBlock) void encode_bytes_queue_bits_kernel(
    uint8_t* __restrict__ slots, uint64_t slot_stride, uint64_t L, uint64_t chunk, uint64_t col0, uint64_t ncols, uint64_t S,
    uint32_t nobj, uint32_t rows, const uint32_t* __restrict__ coeff, const uint32_t* __restrict__ out_idx,
    uint32_t* __restrict__ flags, uint32_t* __restrict__ ticket, uint32_t spread, uint8_t* __restrict__ record,
    uint32_t units, uint8_t* __restrict__ bits) {
  encode_queue_body<K, U, C, NC, true>(slots, slot_stride, L, chunk, col0, ncols, S, nobj, rows, coeff, out_idx, flags,
                                       ticket, spread, record, units, bits);
}

// The redo list of a switched phase 0: every interior unit of an object whose
// mapping came out 1<<31 (status 0) that phase 0 encoded with mapping 0,
// as entries obj * units + unit, appended in any order; *count (zero on
// entry) receives their number.
template <int C>
__global__ __launch_bounds__(kBlock) void redo_list_kernel(const uint8_t* __restrict__ record,
                                                           const uint32_t* __restrict__ mapping,
                                                           const uint32_t* __restrict__ status, uint32_t nobj,
                                                           uint32_t units, uint32_t nint, uint32_t* __restrict__ list,
                                                           uint32_t* __restrict__ count) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  const uint64_t nwaves = (uint64_t)gridDim.x * kWaves;
  const uint64_t total = (uint64_t)nobj * units;
  for (uint64_t base = wave * 64; base < total; base += nwaves * 64) {
    const uint64_t e = base + lane;
    bool need = false;
    if (e < total) {
      const uint32_t o = (uint32_t)(e / units), u = (uint32_t)(e % units);
      need = mapping[o] != 0 && status[o] == 0 && apply::unit_tile_base<C>(u) < nint && record[e] == 0;
    }
    const uint64_t mask = __ballot(need);
    if (!mask) continue;
    uint32_t at = 0;
    if (lane == 0) at = atomicAdd(count, (uint32_t)__popcll(mask));
    at = __builtin_amdgcn_readlane(at, 0);  // lane 0 drew it, whatever the exec mask
    if (need) list[at + (uint32_t)__popcll(mask & ((1ull << lane) - 1))] = (uint32_t)e;
  }
}

// Phase 1 after a switched phase 0: re-encode with the object's mapping the
// listed interior units (redo_list_kernel), then every edge tile and column
// tail of the objects mapped with 1<<31 (phase 0 wrote those with mapping 0).
// The interior walk is the queue kernel's pipeline over a static share of the
// list.
template <int K, int U, int C>
__global__ __launch_bounds__(kBlock) void encode_bytes_redo_kernel(
    uint8_t* __restrict__ slots, uint64_t slot_stride, uint64_t L, uint64_t chunk, uint64_t col0, uint64_t ncols, uint64_t S,
    uint32_t nobj, uint32_t rows, const uint32_t* __restrict__ coeff, const uint32_t* __restrict__ out_idx,
    const uint32_t* __restrict__ status, const uint32_t* __restrict__ mapping, const uint32_t* __restrict__ list,
    const uint32_t* __restrict__ count, uint32_t units) {
  const ObjWords ow{(S + 3) / 4, S % 4 ? 0xFFFFFFFFu << (8 * (4 - S % 4)) : 0xFFFFFFFFu};
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = blockIdx.x * kWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nwaves = gridDim.x * kWaves;
  const uint32_t nvec = (uint32_t)(ncols >> 2);
  const uint32_t ntiles = (nvec + 64 * U - 1) / (64 * U);
  const uint64_t first_tail_word = ow.nw ? ow.nw - 1 : 0;
  const uint32_t nint = encode_interior_tiles(S, L, col0, ncols, K, U);
  auto window = [&](uint32_t o) { return slots + (uint64_t)o * slot_stride + 4 * col0; };
  auto load = [&](uint4(&r)[U][K], uint32_t o, uint32_t t) {
    const uint8_t* cb[K];
#pragma unroll
    for (int j = 0; j < K; ++j) cb[j] = window(o) + (uint64_t)j * chunk;
    load_raw_tile<K, U>(r, cb, t * (64 * U) + lane, nvec);
  };
  Flags unused;
  auto compute = [&](uint4(&r)[U][K], uint32_t o, uint32_t t) {
    encode_interior_tile<K, U, false>(r, window(o) + (uint64_t)K * chunk, chunk, mapping[o], rows, coeff, out_idx,
                                      t * (64 * U) + lane, nvec, unused);
  };
  apply::ListWalk<C> w(list, *count, wave, nwaves, units, nint);
  if (w.live) {
    uint4 ra[U][K], rb[U][K];
    load(ra, w.obj, w.tile());
    for (;;) {
      uint32_t co = w.obj, ct = w.tile();
      w.advance();
      load(rb, w.live ? w.obj : co, w.live ? w.tile() : ct);
      compute(ra, co, ct);
      if (!w.live) break;
      co = w.obj;
      ct = w.tile();
      w.advance();
      load(ra, w.live ? w.obj : co, w.live ? w.tile() : ct);
      compute(rb, co, ct);
      if (!w.live) break;
    }
  }
  // Edge tiles and column tails of the objects mapped with 1<<31.
  const uint32_t nedge = ntiles - nint;
  for (uint64_t e = wave; e < (uint64_t)nobj * nedge; e += nwaves) {
    const uint32_t o = (uint32_t)(e / nedge);
    const uint32_t m = mapping[o];
    if (m == 0 || status[o] != 0) continue;  // wave-uniform
    uint8_t* const slot = window(o);
    const uint64_t g0 = (uint64_t)(nint + (uint32_t)(e % nedge)) * (64 * U) + lane;
    uint32_t x[U][K][4];
    int n = 0;
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (g0 + 64 * u < nvec) {
        load_data_symbols<K, false, false>(slot, chunk, L, col0, (g0 + 64 * u) << 2, 4, ow, m, x[u], nullptr);
        n = u + 1;
      }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (u >= n) break;
      const uint64_t b = (g0 + 64 * u) << 2;
      if ((uint64_t)(K - 1) * L + col0 + b + 4 > first_tail_word) fix_data_tail<K>(slot, chunk, L, col0, b, 4, ow, m, x[u]);
    }
    rows_out_units<K, U>(x, n, rows, coeff, out_idx, slot + (uint64_t)K * chunk, chunk, g0, m);
  }
  const uint32_t tailc = (uint32_t)(ncols - ((uint64_t)nvec << 2));
  const uint64_t tid = (uint64_t)blockIdx.x * kBlock + threadIdx.x, nthr = (uint64_t)gridDim.x * kBlock;
  for (uint64_t t = tid; tailc && t < (uint64_t)nobj * tailc; t += nthr) {
    const uint32_t o = (uint32_t)(t / tailc);
    const uint32_t m = mapping[o];
    if (m == 0 || status[o] != 0) continue;
    uint8_t* const slot = window(o);
    const uint64_t b = ((uint64_t)nvec << 2) + t % tailc;
    uint32_t x[K][4];
    load_data_symbols<K, false, false>(slot, chunk, L, col0, b, 1, ow, m, x, nullptr);
    fix_data_tail<K>(slot, chunk, L, col0, b, 1, ow, m, x);
    rows_out<K>(x, rows, coeff, out_idx, slot + (uint64_t)K * chunk, chunk, 4 * b, m, 1);
  }
}

// Phase 1 after a phase 0 that stored its top bits: the listed interior units
// (redo_list_kernel) are corrected in place instead of re-encoded.  Under
// 1<<31 an interior symbol is x ^ 2^31 = x + 2^31 - 2^32 b = x + 2^31 - 5 b
// (mod p), b = bit 31 of the packed word x, so parity row i becomes
//   parity0 + 2^31 sum_j c_ij - 5 sum_j c_ij b_j   (mod p),
// and the data chunks of an interior unit are the object's own bytes under
// either mapping (MapFromGF(m, x ^ m) = x).  Each block first builds, for
// four rows at a time, T_i[f] = that correction for every K-bit field f of
// top bits (LDS), so a column costs one lookup per row.  A wave then takes
// whole units (static share of the list): every tile's bit planes and four
// parity rows loaded at once, corrected, stored back.  Per column 4r + K/8
// bytes read and 4r written instead of the re-encode's 4K and 4r.  Edge tiles
// and column tails stay with encode_bytes_redo_kernel.
template <int K, int U, int C>
__global__ __launch_bounds__(kBlock) void encode_bytes_fix_kernel(
    uint8_t* __restrict__ slots, uint64_t slot_stride, uint64_t chunk, uint64_t col0, uint32_t rows,
    const uint32_t* __restrict__ coeff, const uint32_t* __restrict__ out_idx, const uint32_t* __restrict__ mapping,
    const uint8_t* __restrict__ bits, const uint32_t* __restrict__ list, const uint32_t* __restrict__ count,
    uint32_t units, uint32_t nint) {
  static_assert(K <= kTopBitsMaxK, "the correction table holds 2^K entries per row");
  constexpr int KW = TopBits<K, U>::kWords;
  constexpr uint32_t NF = 1u << K;
  __shared__ uint32_t table[4][NF];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = blockIdx.x * kWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nwaves = gridDim.x * kWaves;
  const uint32_t n = *count;
  for (uint32_t i0 = 0; i0 < rows; i0 += 4) {
    for (uint32_t x = threadIdx.x; x < 4 * NF; x += kBlock) {
      const uint32_t ii = x / NF, f = x % NF;
      if (i0 + ii >= rows) continue;
      const uint32_t* const c = coeff + (uint64_t)(i0 + ii) * kCoeffStride;  // reduced mod p by the plan
      uint64_t csum = 0;
      uint32_t acc = 0;
      for (int j = 0; j < K; ++j) {
        csum += c[j];
        if ((f >> j) & 1u) {
          const uint32_t t5 = fold96(5ull * c[j], 0);
          const uint32_t d = t5 ? kP - t5 : 0u;  // -5 c_ij mod p
          const uint64_t s2 = (uint64_t)acc + d;
          acc = (uint32_t)(s2 >= kP ? s2 - kP : s2);
        }
      }
      const uint64_t s2 = (uint64_t)acc + fold96((uint64_t)fold96(csum, 0) << 31, 0);  // + 2^31 sum_j c_ij
      table[ii][f] = (uint32_t)(s2 >= kP ? s2 - kP : s2);
    }
    __syncthreads();
    for (uint32_t e = wave; e < n; e += nwaves) {
      const uint32_t v = list[e];
      const uint32_t o = v / units, tb = apply::unit_tile_base<C>(v % units);
      uint32_t cnt = tb < nint ? (nint - tb + 3) / 4 : 0;
      if (cnt > C) cnt = C;
      const uint32_t m = mapping[o];
      uint8_t* const par = slots + (uint64_t)o * slot_stride + 4 * col0 + (uint64_t)K * chunk;
      uint32_t tbits[C][KW];
      uint4 pv[C][4][U];
#pragma unroll
      for (int i = 0; i < C; ++i)
        if ((uint32_t)i < cnt) {
          load_top_bits<K, U>(bits + ((uint64_t)o * nint + tb + 4 * i) * TopBits<K, U>::kTileBytes, lane, tbits[i]);
#pragma unroll
          for (int ii = 0; ii < 4; ++ii)
#pragma unroll
            for (int u = 0; u < U; ++u)
              if (i0 + ii < rows)
                pv[i][ii][u] = apply::ld16_at<false>(
                    reinterpret_cast<const uint32_t*>(par + (uint64_t)out_idx[i0 + ii] * chunk),
                    ((tb + 4 * i) * (64 * U) + 64 * u + lane) << 4);
        }
#pragma unroll
      for (int i = 0; i < C; ++i) {
        if ((uint32_t)i >= cnt) break;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          uint32_t f[4];
#pragma unroll
          for (int c = 0; c < 4; ++c) f[c] = top_field<K, U>(tbits[i], u, c);
#pragma unroll
          for (int ii = 0; ii < 4; ++ii) {
            if (i0 + ii >= rows) break;
            const uint4 pw = pv[i][ii][u];
            const uint32_t w[4] = {pw.x, pw.y, pw.z, pw.w};
            uint32_t y[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) {  // phase 0 stored BE(parity0), parity0 < p; entries < p
              const uint64_t s2 = (uint64_t)be(w[c]) + table[ii][f[c]];
              y[c] = be((uint32_t)(s2 >= kP ? s2 - kP : s2) ^ m);
            }
            const u32x4 out = {y[0], y[1], y[2], y[3]};
            uint8_t* const orow = par + (uint64_t)out_idx[i0 + ii] * chunk;
            __builtin_nontemporal_store(
                out, reinterpret_cast<u32x4*>(orow + (uint32_t)(((tb + 4 * i) * (64 * U) + 64 * u + lane) << 4)));
          }
        }
      }
    }
    __syncthreads();  // the table is rebuilt for the next four rows
  }
}

// ---- wide k (need > 16): the byte kernels in 16-chunk form ------------------
// Same column walk as rs_apply_wide_kernel (4 columns per lane, one unit per
// step), with the byte<->symbol transforms of the kernels above: inputs in
// chunks of 16 data chunks, outputs in blocks of RB rows, a canonical 32-bit
// running residue per row and column.

// One chunk of KC inputs (KC a multiple of 16; coefficients past k are zero
// in the plan table) applied on top of a row's running residues, exactly,
// with one fold.  `crow` points at the row's coefficients for the chunk.
template <int KC>
__device__ __forceinline__ void wide_mac_chunk(const uint32_t (&x)[KC][4], const uint32_t* __restrict__ crow,
                                               uint32_t j0, uint32_t k, uint32_t (&acc)[4]) {
  uint64_t lo0 = acc[0], lo1 = acc[1], lo2 = acc[2], lo3 = acc[3];
  uint32_t hi0 = 0, hi1 = 0, hi2 = 0, hi3 = 0;
#pragma unroll
  for (int h = 0; h < KC; h += 16) {
    if (j0 + h < k) {
      const u32x16 c = *reinterpret_cast<const u32x16*>(crow + h);
#pragma unroll
      for (int j = 0; j < 16; ++j)
        mac4(lo0, lo1, lo2, lo3, hi0, hi1, hi2, hi3, x[h + j][0], x[h + j][1], x[h + j][2], x[h + j][3], c[j]);
    }
  }
  acc[0] = fold96(lo0, hi0);
  acc[1] = fold96(lo1, hi1);
  acc[2] = fold96(lo2, hi2);
  acc[3] = fold96(lo3, hi3);
}

// MODE as in encode_bytes_kernel.  Column tails (past the last whole vector
// of the window) go one column per lane with ncol = 1.
// KC = 32 holds every input of a need <= 32 code in registers at once.
// One lane-unit step of the chunked wide encode at unit g (a whole vector,
// or a tail column past the window's last whole vector): every row block and
// input chunk, with the data-chunk tail fix on edge steps.
template <int KC, int RB, bool F>
__device__ __forceinline__ void encode_wide_step(uint8_t* slot, uint8_t* par, uint64_t chunk, uint64_t L,
                                                 uint64_t col0, const ObjWords& ow, uint64_t first_tail_word,
                                                 uint32_t m, uint32_t rows, uint32_t k, uint32_t cs,
                                                 const uint32_t* __restrict__ coeff,
                                                 const uint32_t* __restrict__ out_idx, uint64_t g, uint64_t nvec,
                                                 uint64_t u1, uint64_t seg_v1, uint32_t lane, Flags& fl) {
  const bool valid = g < u1;
  const bool vec = g < nvec;
  const int ncol = vec ? 4 : 1;
  const uint64_t b = vec ? g << 2 : (nvec << 2) + (g - nvec);
  // Interior step (wave-uniform): every data word the step touches is a
  // whole object word, below the object's last word.
  const uint64_t gw = g - lane;
  const bool interior = gw + 64 <= seg_v1 && (uint64_t)(k - 1) * L + col0 + ((gw + 64) << 2) < first_tail_word;
  for (uint32_t r0 = 0; r0 < rows; r0 += RB) {
    uint32_t acc[RB][4];
#pragma unroll
    for (int i = 0; i < RB; ++i) acc[i][0] = acc[i][1] = acc[i][2] = acc[i][3] = 0;
    for (uint32_t j0 = 0; j0 < k; j0 += KC) {
      uint32_t x[KC][4];
#pragma unroll
      for (int j = 0; j < KC; ++j) {
        x[j][0] = x[j][1] = x[j][2] = x[j][3] = 0;
        if (valid && j0 + j < k) {
          if (interior) {
            if (F && r0 == 0)
              load_data_symbol<true, true>(slot, chunk, L, col0, j0 + j, b, 4, ow, m, x[j], &fl);
            else
              load_data_symbol<true, false>(slot, chunk, L, col0, j0 + j, b, 4, ow, m, x[j], nullptr);
          } else {
            if (F && r0 == 0)
              load_data_symbol<false, true>(slot, chunk, L, col0, j0 + j, b, ncol, ow, m, x[j], &fl);
            else
              load_data_symbol<false, false>(slot, chunk, L, col0, j0 + j, b, ncol, ow, m, x[j], nullptr);
            if (r0 == 0) fix_data_tail_one(slot, chunk, L, col0, j0 + j, b, ncol, ow, m, x[j]);
          }
        }
      }
#pragma unroll
      for (int i = 0; i < RB; ++i)
        if (r0 + i < rows) wide_mac_chunk<KC>(x, coeff + (uint64_t)(r0 + i) * cs + j0, j0, k, acc[i]);
    }
    if (valid) {
#pragma unroll
      for (int i = 0; i < RB; ++i) {
        if (r0 + i < rows) {
          uint8_t* dst = par + (uint64_t)out_idx[r0 + i] * chunk + 4 * b;
          if (vec) {
            const u32x4 v = {be(acc[i][0] ^ m), be(acc[i][1] ^ m), be(acc[i][2] ^ m), be(acc[i][3] ^ m)};
            __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(dst));
          } else {
            *reinterpret_cast<uint32_t*>(dst) = be(acc[i][0] ^ m);
          }
        }
      }
    }
  }
}

template <int KC, int RB, int MODE>
__global__ __launch_bounds__(kBlock) void encode_bytes_wide_kernel(
    uint8_t* __restrict__ slots, uint64_t slot_stride, uint64_t L, uint64_t chunk, uint64_t col0, uint64_t ncols, uint64_t S,
    uint32_t nobj, uint32_t rows, uint32_t k, const uint32_t* __restrict__ coeff,
    const uint32_t* __restrict__ out_idx, uint32_t* __restrict__ flags, const uint32_t* __restrict__ mapping,
    uint32_t nseg) {
  const uint32_t cs = apply::wide_coeff_stride(k);
  const ObjWords ow{(S + 3) / 4, S % 4 ? 0xFFFFFFFFu << (8 * (4 - S % 4)) : 0xFFFFFFFFu};
  const uint64_t first_tail_word = ow.nw ? ow.nw - 1 : 0;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  const uint64_t nwaves = (uint64_t)gridDim.x * kWaves;
  const uint64_t nvec = ncols >> 2;
  constexpr bool F = MODE == 0;
  for (uint64_t wi = blockIdx.y; wi < (uint64_t)nobj * nseg; wi += gridDim.y) {
    const Segment sg = segment_of(wi, nseg, nvec);
    const uint32_t obj = sg.obj;
    // Units: the segment's whole vectors, then (last segment) one per tail column.
    const uint64_t u1 = sg.last ? nvec + (ncols & 3) : sg.v1;
    uint32_t m = 0;
    if constexpr (MODE == 1) {
      m = mapping[obj];
      if (m == 0 || flags[obj] != 0) continue;
    }
    uint8_t* const slot = slots + (uint64_t)obj * slot_stride + 4 * col0;
    uint8_t* const par = slot + (uint64_t)k * chunk;
    Flags fl;
    for (uint64_t g = sg.v0 + wave * 64 + lane; g - lane < u1; g += nwaves * 64)
      encode_wide_step<KC, RB, F>(slot, par, chunk, L, col0, ow, first_tail_word, m, rows, k, cs, coeff, out_idx, g,
                                  nvec, u1, sg.v1, lane, fl);
    if constexpr (F) {
      const uint32_t f = fl.bits();
      const uint64_t a1 = __ballot(f & 1u), a2 = __ballot(f & 2u);
      const uint32_t wf = (a1 ? 1u : 0u) | (a2 ? 2u : 0u);
      if (wf && lane == 0) atomicOr(&flags[obj], wf);
    }
  }
}

template <int KC, int RB>
__global__ __launch_bounds__(kBlock) void decode_bytes_wide_kernel(
    uint8_t* __restrict__ slots, uint64_t slot_stride, uint64_t L, uint64_t chunk, uint64_t col0, uint64_t ncols, uint32_t nobj,
    uint32_t rows, uint32_t k, const uint32_t* __restrict__ coeff, const uint32_t* __restrict__ in_idx,
    const uint32_t* __restrict__ out_idx, const uint32_t* __restrict__ mapping, uint32_t nseg) {
  const uint32_t cs = apply::wide_coeff_stride(k);
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  const uint64_t nwaves = (uint64_t)gridDim.x * kWaves;
  const uint64_t nvec = ncols >> 2;
  for (uint64_t wi = blockIdx.y; wi < (uint64_t)nobj * nseg; wi += gridDim.y) {
    const Segment sg = segment_of(wi, nseg, nvec);
    const uint32_t obj = sg.obj;
    const uint64_t u1 = sg.last ? nvec + (ncols & 3) : sg.v1;
    const uint32_t m = mapping[obj];
    uint8_t* const slot = slots + (uint64_t)obj * slot_stride + 4 * col0;
    for (uint64_t g = sg.v0 + wave * 64 + lane; g - lane < u1; g += nwaves * 64) {
      const bool valid = g < u1;
      const bool vec = g < nvec;
      const uint64_t b = vec ? g << 2 : (nvec << 2) + (g - nvec);
      for (uint32_t r0 = 0; r0 < rows; r0 += RB) {
        uint32_t acc[RB][4];
#pragma unroll
        for (int i = 0; i < RB; ++i) acc[i][0] = acc[i][1] = acc[i][2] = acc[i][3] = 0;
        for (uint32_t j0 = 0; j0 < k; j0 += KC) {
          uint32_t x[KC][4];
#pragma unroll
          for (int j = 0; j < KC; ++j) {
            x[j][0] = x[j][1] = x[j][2] = x[j][3] = 0;
            if (valid && j0 + j < k) {
              const uint8_t* src = slot + (uint64_t)in_idx[j0 + j] * chunk + 4 * b;
              if (vec) {
                const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src));
                x[j][0] = be(v.x) ^ m, x[j][1] = be(v.y) ^ m, x[j][2] = be(v.z) ^ m, x[j][3] = be(v.w) ^ m;
              } else {
                x[j][0] = be(*reinterpret_cast<const uint32_t*>(src)) ^ m;
              }
            }
          }
#pragma unroll
          for (int i = 0; i < RB; ++i)
            if (r0 + i < rows) wide_mac_chunk<KC>(x, coeff + (uint64_t)(r0 + i) * cs + j0, j0, k, acc[i]);
        }
        if (valid) {
#pragma unroll
          for (int i = 0; i < RB; ++i) {
            if (r0 + i < rows) {
              uint8_t* dst = slot + (uint64_t)out_idx[r0 + i] * chunk + 4 * b;
              if (vec) {
                const u32x4 v = {be(acc[i][0] ^ m), be(acc[i][1] ^ m), be(acc[i][2] ^ m), be(acc[i][3] ^ m)};
                __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(dst));
              } else {
                *reinterpret_cast<uint32_t*>(dst) = be(acc[i][0] ^ m);
              }
            }
          }
        }
      }
    }
  }
}

// Pipelined wide encode (need > 16, chunks < 4 GiB).  The interior tiles of
// a segment (whole 64-vector tiles below the object's last word, a prefix)
// run as rs_apply_wide_pipe_kernel's item stream over data-chunk bytes: the
// transform (BE, MapToGF flags on the first row block, ^ m) reads every
// loaded register before the math.  The segment's remaining units (edge
// tiles, tail columns) take encode_wide_step.  MODE as in encode_bytes_kernel.
template <int RB, int MODE>
__global__ __launch_bounds__(kBlock) void encode_bytes_wide_pipe_kernel(
    uint8_t* __restrict__ slots, uint64_t slot_stride, uint64_t L, uint64_t chunk, uint64_t col0, uint64_t ncols, uint64_t S,
    uint32_t nobj, uint32_t rows, uint32_t k, const uint32_t* __restrict__ coeff,
    const uint32_t* __restrict__ out_idx, uint32_t* __restrict__ flags, const uint32_t* __restrict__ mapping,
    uint32_t nseg) {
  using apply::WideItem;
  const uint32_t cs = apply::wide_coeff_stride(k);
  const uint32_t nch = (k + 15) / 16, nrb = (rows + RB - 1) / RB;
  const ObjWords ow{(S + 3) / 4, S % 4 ? 0xFFFFFFFFu << (8 * (4 - S % 4)) : 0xFFFFFFFFu};
  const uint64_t first_tail_word = ow.nw ? ow.nw - 1 : 0;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = blockIdx.x * kWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nwaves = gridDim.x * kWaves;
  const uint64_t nvec = ncols >> 2;
  constexpr bool F = MODE == 0;
  for (uint64_t wi = blockIdx.y; wi < (uint64_t)nobj * nseg; wi += gridDim.y) {
    const Segment sg = segment_of(wi, nseg, nvec);
    const uint32_t obj = sg.obj;
    const uint32_t v0 = (uint32_t)sg.v0, v1 = (uint32_t)sg.v1;
    const uint64_t u1 = sg.last ? nvec + (ncols & 3) : sg.v1;
    uint32_t m = 0;
    if constexpr (MODE == 1) {
      m = mapping[obj];
      if (m == 0 || flags[obj] != 0) continue;  // uniform per block
    }
    uint8_t* const slot = slots + (uint64_t)obj * slot_stride + 4 * col0;  // window base
    uint8_t* const par = slot + (uint64_t)k * chunk;
    // Interior tiles t < nint: end = v0 + 64(t+1) <= v1 and
    // (k-1)L + col0 + 4*end < first_tail_word.
    uint64_t end_max = interior_vectors(S, L, col0, k);
    if (end_max > v1) end_max = v1;
    const uint32_t nint = end_max > v0 ? (uint32_t)((end_max - v0) / 64) : 0u;
    Flags fl;
    auto load = [&](uint4 (&x)[16], const WideItem& it) {
      const uint32_t g = v0 + it.tile * 64 + lane;  // interior: always inside the segment
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const uint32_t s = it.jc * 16 + j < k ? it.jc * 16 + j : k - 1;
        const uint64_t base = (uint64_t)(slot + (uint64_t)s * chunk);
        const uint64_t ub = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(base >> 32)) << 32) |
                            (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)base);
        typedef const __attribute__((address_space(1))) u32x4 global_u32x4;
        const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const global_u32x4*>(ub + (uint64_t)(g << 4)));
        x[j] = make_uint4(v.x, v.y, v.z, v.w);
      }
    };
    uint4 acc[RB];
    auto item = [&](uint4 (&x)[16], const WideItem& it) {
      // Indices past k repeat chunk k-1 (real object words; flags are maxima).
      const bool add_flags = F && it.rb == 0;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        uint32_t w[4] = {be(x[j].x), be(x[j].y), be(x[j].z), be(x[j].w)};
        if (add_flags) {
#pragma unroll
          for (int c = 0; c < 4; ++c) fl.add(c, w[c]);
        }
        x[j] = make_uint4(w[0] ^ m, w[1] ^ m, w[2] ^ m, w[3] ^ m);
      }
      if (it.jc == 0) {
#pragma unroll
        for (int i = 0; i < RB; ++i) acc[i] = make_uint4(0, 0, 0, 0);
      }
      const uint32_t r0 = it.rb * RB;
      const uint32_t* const c0 = coeff + (uint64_t)r0 * cs + it.jc * 16;
      apply::wide_mac16(x, c0, acc[0]);
#pragma unroll
      for (int i = 1; i < RB; ++i)
        if (r0 + i < rows) apply::wide_mac16(x, c0 + (uint64_t)i * cs, acc[i]);
      if (it.jc == nch - 1) {
        const uint32_t g = v0 + it.tile * 64 + lane;
#pragma unroll
        for (int i = 0; i < RB; ++i)
          if (r0 + i < rows) {
            const u32x4 v = {be(acc[i].x ^ m), be(acc[i].y ^ m), be(acc[i].z ^ m), be(acc[i].w ^ m)};
            __builtin_nontemporal_store(
                v, reinterpret_cast<u32x4*>(par + (uint64_t)out_idx[r0 + i] * chunk + ((uint64_t)g << 4)));
          }
      }
    };
    uint4 xa[16], xb[16];
    WideItem it{wave, 0, 0};
    if (it.tile < nint) load(xa, it);
    while (it.tile < nint) {
      WideItem nx = it;
      apply::wide_next(nx, nch, nrb, nwaves);
      load(xb, nx.tile < nint ? nx : it);
      item(xa, it);
      it = nx;
      if (it.tile >= nint) break;
      nx = it;
      apply::wide_next(nx, nch, nrb, nwaves);
      load(xa, nx.tile < nint ? nx : it);
      item(xb, it);
      it = nx;
    }
    // Edge tiles and tail columns.
    for (uint64_t g = (uint64_t)v0 + (uint64_t)nint * 64 + (uint64_t)wave * 64 + lane; g - lane < u1;
         g += (uint64_t)nwaves * 64)
      encode_wide_step<16, RB, F>(slot, par, chunk, L, col0, ow, first_tail_word, m, rows, k, cs, coeff, out_idx, g,
                                  nvec, u1, sg.v1, lane, fl);
    if constexpr (F) {
      const uint32_t f = fl.bits();
      const uint64_t a1 = __ballot(f & 1u), a2 = __ballot(f & 2u);
      const uint32_t wf = (a1 ? 1u : 0u) | (a2 ? 2u : 0u);
      if (wf && lane == 0) atomicOr(&flags[obj], wf);
    }
  }
}

// Pipelined wide decode (need > 16, chunks < 4 GiB): rs_apply_wide_pipe_kernel's
// item stream over chunk bytes.  Items load 16 raw survivor vectors (indices
// past k clamped to k-1, zero coefficients); the transform BE(word) ^ m
// reads every loaded register before the math; the last chunk of a row
// block stores BE(residue ^ m).
template <int RB>
__global__ __launch_bounds__(kBlock) void decode_bytes_wide_pipe_kernel(
    uint8_t* __restrict__ slots, uint64_t slot_stride, uint64_t L, uint64_t chunk, uint64_t col0, uint64_t ncols, uint32_t nobj,
    uint32_t rows, uint32_t k, const uint32_t* __restrict__ coeff, const uint32_t* __restrict__ in_idx,
    const uint32_t* __restrict__ out_idx, const uint32_t* __restrict__ mapping, uint32_t nseg) {
  using apply::WideItem;
  const uint32_t cs = apply::wide_coeff_stride(k);
  const uint32_t nch = (k + 15) / 16, nrb = (rows + RB - 1) / RB;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = blockIdx.x * kWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nwaves = gridDim.x * kWaves;
  const uint64_t nvec = ncols >> 2;
  for (uint64_t wi = blockIdx.y; wi < (uint64_t)nobj * nseg; wi += gridDim.y) {
    const Segment sg = segment_of(wi, nseg, nvec);
    const uint32_t v0 = (uint32_t)sg.v0, v1 = (uint32_t)sg.v1;
    const uint32_t ntiles = (v1 - v0 + 63) / 64;
    const uint32_t m = mapping[sg.obj];
    uint8_t* const slot = slots + (uint64_t)sg.obj * slot_stride + 4 * col0;  // window base
    auto load = [&](uint4 (&x)[16], const WideItem& it) {
      const uint32_t g = v0 + it.tile * 64 + lane;
      const uint32_t gc = g < v1 ? g : v1 - 1;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const uint32_t s = it.jc * 16 + j < k ? it.jc * 16 + j : k - 1;
        const uint64_t base = (uint64_t)(slot + (uint64_t)in_idx[s] * chunk);
        const uint64_t ub = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(base >> 32)) << 32) |
                            (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)base);
        typedef const __attribute__((address_space(1))) u32x4 global_u32x4;
        const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const global_u32x4*>(ub + (uint64_t)(gc << 4)));
        x[j] = make_uint4(v.x, v.y, v.z, v.w);
      }
    };
    uint4 acc[RB];
    auto item = [&](uint4 (&x)[16], const WideItem& it) {
#pragma unroll
      for (int j = 0; j < 16; ++j) x[j] = make_uint4(be(x[j].x) ^ m, be(x[j].y) ^ m, be(x[j].z) ^ m, be(x[j].w) ^ m);
      if (it.jc == 0) {
#pragma unroll
        for (int i = 0; i < RB; ++i) acc[i] = make_uint4(0, 0, 0, 0);
      }
      const uint32_t r0 = it.rb * RB;
      const uint32_t* const c0 = coeff + (uint64_t)r0 * cs + it.jc * 16;
      apply::wide_mac16(x, c0, acc[0]);
#pragma unroll
      for (int i = 1; i < RB; ++i)
        if (r0 + i < rows) apply::wide_mac16(x, c0 + (uint64_t)i * cs, acc[i]);
      const uint32_t g = v0 + it.tile * 64 + lane;
      if (it.jc == nch - 1 && g < v1) {
#pragma unroll
        for (int i = 0; i < RB; ++i)
          if (r0 + i < rows) {
            const u32x4 v = {be(acc[i].x ^ m), be(acc[i].y ^ m), be(acc[i].z ^ m), be(acc[i].w ^ m)};
            __builtin_nontemporal_store(
                v, reinterpret_cast<u32x4*>(slot + (uint64_t)out_idx[r0 + i] * chunk + ((uint64_t)g << 4)));
          }
      }
    };
    uint4 xa[16], xb[16];
    WideItem it{wave, 0, 0};
    if (it.tile < ntiles) load(xa, it);
    while (it.tile < ntiles) {
      WideItem nx = it;
      apply::wide_next(nx, nch, nrb, nwaves);
      load(xb, nx.tile < ntiles ? nx : it);
      item(xa, it);
      it = nx;
      if (it.tile >= ntiles) break;
      nx = it;
      apply::wide_next(nx, nch, nrb, nwaves);
      load(xa, nx.tile < ntiles ? nx : it);
      item(xb, it);
      it = nx;
    }
    // Columns past the last whole vector of the window, one per lane.
    for (uint64_t b = (nvec << 2) + (uint64_t)wave * 64 + lane; sg.last && b < ncols; b += (uint64_t)nwaves * 64) {
      for (uint32_t i = 0; i < rows; ++i) {
        const uint32_t* crow = coeff + (uint64_t)i * cs;
        uint64_t lo = 0;
        uint32_t hi = 0;
        for (uint32_t j = 0; j < k; ++j)
          mac(lo, hi, be(*reinterpret_cast<const uint32_t*>(slot + (uint64_t)in_idx[j] * chunk + 4 * b)) ^ m, crow[j]);
        *reinterpret_cast<uint32_t*>(slot + (uint64_t)out_idx[i] * chunk + 4 * b) = be(fold96(lo, hi) ^ m);
      }
    }
  }
}

}  // namespace bytes
}  // namespace slime
