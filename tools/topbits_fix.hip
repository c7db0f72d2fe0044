// Experiment (tools only): the byte encode's second pass as a parity
// correction from stored top bits instead of a re-encode, at need <= 16 on
// the ticket walk (tools/topbits_fix.py drives it).
//
// A switched object's units encoded with mapping 0 hold parity0 = sum_j c_ij
// x_j; under 1<<31 every interior symbol is x ^ 2^31 = x + 2^31 - 2^32 b =
// x + 2^31 - 5 b (mod p), b = bit 31 of x, so
//   parity' = parity0 + 2^31 sum_j c_ij - 5 sum_j c_ij b_j   (mod p)
// needs the k top bits of a column, not its k data words.  First pass: the
// product's encode_bytes_queue_kernel (rs_bytes_kernel.hpp) plus a store of
// each mapping-0 tile's top bits (bit planes, lane-contiguous).  Second pass:
// the product's redo list, then per listed unit all C tiles' bits and
// parity rows loaded at once, corrected and stored back -- 4r + k/8 bytes read
// and 4r written per column instead of the re-encode's 4k + 4r.  Edge tiles
// keep the product's redo (not timed here: the same in both forms).
//
// Round 3 built a first form (commit 148f5a8: one tile and four rows of loads
// in flight per wave, 0.762 ms against the re-encode's 0.807 at C5) and
// removed it; this form keeps a whole unit's loads in flight.
#include <hip/hip_runtime.h>

#include "rs_bytes_launch.hpp"

using namespace slime;
using namespace slime::bytes;

namespace {

// Top bits of a first-pass tile: a lane's string holds, for vector u and
// column c, the K top bits of its column as one K-bit field at bit
// (u*4 + c)*K (bit j of the field = bit 31 of chunk j's packed word = bit 7
// of the raw little-endian load), so the second pass reads a column's field
// as one index.  Planes of 32 bits per lane (plane q at tile + 256 q),
// lane-contiguous, the last plane only as wide as the bits left.
template <int K, int U>
struct TopBits {
  static constexpr int kBits = K * U * 4;
  static constexpr int kWords = (kBits + 31) / 32;
  static constexpr int kLastBits = kBits - 32 * (kWords - 1);
  static constexpr int kLastBytes = kLastBits <= 8 ? 1 : kLastBits <= 16 ? 2 : 4;
  static constexpr uint64_t kTileBytes = 64ull * (4 * (kWords - 1) + kLastBytes);
};

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
      const uint32_t t[4] = {(r[u][j].x >> 7) & 1u, (r[u][j].y >> 7) & 1u, (r[u][j].z >> 7) & 1u, (r[u][j].w >> 7) & 1u};
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int b = (u * 4 + c) * K + j;
        w[b >> 5] |= t[c] << (b & 31);
      }
    }
#pragma unroll
  for (int q = 0; q + 1 < T::kWords; ++q) __builtin_nontemporal_store(w[q], reinterpret_cast<uint32_t*>(tile + 256 * q) + lane);
  uint8_t* const last = tile + 256 * (T::kWords - 1);
  if constexpr (T::kLastBytes == 1)
    last[lane] = (uint8_t)w[T::kWords - 1];
  else if constexpr (T::kLastBytes == 2)
    reinterpret_cast<uint16_t*>(last)[lane] = (uint16_t)w[T::kWords - 1];
  else
    __builtin_nontemporal_store(w[T::kWords - 1], reinterpret_cast<uint32_t*>(last) + lane);
}

// The K-bit field of vector u, column c from a lane's loaded planes.
template <int K, int U>
__device__ __forceinline__ uint32_t top_field(const uint32_t (&w)[TopBits<K, U>::kWords], int u, int c) {
  const int b = (u * 4 + c) * K, q = b >> 5;
  uint64_t v = w[q];
  if (q + 1 < TopBits<K, U>::kWords) v |= (uint64_t)w[q + 1] << 32;
  return (uint32_t)(v >> (b & 31)) & ((1u << K) - 1);
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

// encode_bytes_queue_kernel's interior walk (rs_bytes_kernel.hpp) with the
// top-bit store; BITS = false is the product's interior walk, for the A/B.
// Edge tiles and column tails are left out of both (the same work in both).
template <int K, int U, int C, int NC, bool BITS>
__global__ __launch_bounds__(kBlock) void pass0_kernel(uint8_t* __restrict__ slots, uint64_t slot_stride, uint64_t chunk,
                                                       uint64_t ncols, uint32_t nobj, uint32_t rows,
                                                       const uint32_t* __restrict__ coeff,
                                                       const uint32_t* __restrict__ out_idx, uint32_t* __restrict__ flags,
                                                       uint32_t* __restrict__ ticket, uint32_t spread,
                                                       uint8_t* __restrict__ record, uint32_t units, uint32_t nint,
                                                       uint8_t* __restrict__ bits) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t nvec = (uint32_t)(ncols >> 2);
  auto window = [&](uint32_t o) { return slots + (uint64_t)o * slot_stride; };
  auto load = [&](uint4(&r)[U][K], uint32_t o, uint32_t t) {
    const uint8_t* cb[K];
#pragma unroll
    for (int j = 0; j < K; ++j) cb[j] = window(o) + (uint64_t)j * chunk;
    load_raw_tile<K, U>(r, cb, t * (64 * U) + lane, nvec);
  };
  auto unit_mapping = [&](uint32_t o) -> uint32_t {
    const uint32_t f = __hip_atomic_load(flags + o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return (f & 1u) ? 0x80000000u : 0u;
  };
  Flags fl;
  uint32_t fobj = 0xFFFFFFFFu, sent = 0;
  auto publish = [&] {
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
    if (first && lane == 0) record[(uint64_t)o * units + unit] = m ? 1 : 0;
    if (BITS && m == 0) store_top_bits<K, U>(r, bits + ((uint64_t)o * nint + t) * TopBits<K, U>::kTileBytes, lane);
    encode_interior_tile<K, U, true>(r, window(o) + (uint64_t)K * chunk, chunk, m, rows, coeff, out_idx,
                                     t * (64 * U) + lane, nvec, fl);
    publish();
  };
  apply::TicketWalk<C, NC> w(ticket, nobj, nint, lane, spread);
  if (w.live) {
    uint4 ra[U][K], rb[U][K];
    uint32_t ma = unit_mapping(w.obj), mb = 0;
    uint32_t ua = w.unit(), ub = 0;
    bool fa = true, fb = false;
    load(ra, w.obj, w.tile());
    for (;;) {
      uint32_t co = w.obj, ct = w.tile();
      w.advance();
      fb = w.live && w.unit_start();
      mb = fb ? unit_mapping(w.obj) : ma;
      ub = w.unit();
      load(rb, w.live ? w.obj : co, w.live ? w.tile() : ct);
      compute(ra, co, ct, ma, fa, ua);
      if (!w.live) break;
      co = w.obj;
      ct = w.tile();
      w.advance();
      fa = w.live && w.unit_start();
      ma = fa ? unit_mapping(w.obj) : mb;
      ua = w.unit();
      load(ra, w.live ? w.obj : co, w.live ? w.tile() : ct);
      compute(rb, co, ct, mb, fb, ub);
      if (!w.live) break;
    }
  }
  w.finish();
}

// The correction of the listed units (redo_list_kernel's list).  Each block
// first builds, per parity row i, the table T_i[f] = 2^31 sum_j c_ij - 5
// sum_{j in f} c_ij (mod p) over the 2^K top-bit fields f (LDS), so a
// column's correction is one lookup per row.  Every tile of a unit is loaded
// at once (its bit planes and four parity rows), then corrected and stored;
// rows in blocks of four.
template <int K, int U, int C>
__global__ __launch_bounds__(kBlock) void fix_kernel(uint8_t* __restrict__ slots, uint64_t slot_stride, uint64_t chunk,
                                                     uint32_t rows, const uint32_t* __restrict__ dtab,
                                                     const uint32_t* __restrict__ out_idx,
                                                     const uint32_t* __restrict__ mapping,
                                                     const uint8_t* __restrict__ bits, const uint32_t* __restrict__ list,
                                                     const uint32_t* __restrict__ count, uint32_t units, uint32_t nint) {
  constexpr int KW = TopBits<K, U>::kWords;
  constexpr uint32_t NF = 1u << K;
  __shared__ uint32_t table[4][NF];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = blockIdx.x * kWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nwaves = gridDim.x * kWaves;
  const uint32_t n = *count;
  for (uint32_t i0 = 0; i0 < rows; i0 += 4) {
    // dtab row i: d[j] = -5 c_ij mod p (j < K), d[15] = 2^31 sum_j c_ij mod p (host-built, fix_table)
    for (uint32_t x = threadIdx.x; x < 4 * NF; x += kBlock) {
      const uint32_t ii = x / NF, f = x % NF;
      if (i0 + ii >= rows) continue;
      const uint32_t* d = dtab + 16 * (i0 + ii);
      uint64_t acc = d[15];
      for (int j = 0; j < K; ++j)
        if ((f >> j) & 1u) acc += d[j];
      table[ii][f] = (uint32_t)(acc % kP);
    }
    __syncthreads();
    for (uint32_t e = wave; e < n; e += nwaves) {
      const uint32_t v = list[e];
      const uint32_t o = v / units, tb = apply::unit_tile_base<C>(v % units);
      uint32_t cnt = tb < nint ? (nint - tb + 3) / 4 : 0;
      if (cnt > C) cnt = C;
      const uint32_t m = mapping[o];
      uint8_t* const par = slots + (uint64_t)o * slot_stride + (uint64_t)K * chunk;
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
            for (int c = 0; c < 4; ++c) {
              const uint64_t s2 = (uint64_t)be(w[c]) + table[ii][f[c]];  // parity0 < p (canonical), entry < p
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

// The product's redo kernel restricted to its interior walk, for the A/B.
template <int K, int U, int C>
__global__ __launch_bounds__(kBlock) void redo_interior_kernel(uint8_t* __restrict__ slots, uint64_t slot_stride,
                                                               uint64_t chunk, uint64_t ncols, uint32_t rows,
                                                               const uint32_t* __restrict__ coeff,
                                                               const uint32_t* __restrict__ out_idx,
                                                               const uint32_t* __restrict__ mapping,
                                                               const uint32_t* __restrict__ list,
                                                               const uint32_t* __restrict__ count, uint32_t units,
                                                               uint32_t nint) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = blockIdx.x * kWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nwaves = gridDim.x * kWaves;
  const uint32_t nvec = (uint32_t)(ncols >> 2);
  auto window = [&](uint32_t o) { return slots + (uint64_t)o * slot_stride; };
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
}

struct Geo {
  uint32_t spread, nint, units;
};

template <int K, int U, int C>
Geo geo(uint64_t S, uint64_t L, uint32_t nobj) {
  Geo g;
  g.spread = queue_spread(nobj, L, U, C);
  g.nint = encode_interior_tiles(S, L, 0, L, K, U);
  g.units = apply::walk_units<C>(g.nint, g.spread);
  return g;
}

template <int K, int U, int C>
int pass0(int bits_on, uint8_t* slots, uint64_t stride, uint64_t cstride, uint64_t L, uint64_t S, uint32_t nobj,
          uint32_t rows, const uint32_t* coeff, const uint32_t* out_idx, uint32_t* flags, uint32_t* ticket,
          uint32_t blocks, uint8_t* record, uint8_t* bits, hipStream_t s) {
  const Geo g = geo<K, U, C>(S, L, nobj);
  if (!g.spread) return -2;
  if (bits_on)
    hipLaunchKernelGGL((pass0_kernel<K, U, C, kQueueCounters, true>), dim3(blocks), dim3(kBlock), 0, s, slots, stride,
                       cstride, L, nobj, rows, coeff, out_idx, flags, ticket, g.spread, record, g.units, g.nint, bits);
  else
    hipLaunchKernelGGL((pass0_kernel<K, U, C, kQueueCounters, false>), dim3(blocks), dim3(kBlock), 0, s, slots, stride,
                       cstride, L, nobj, rows, coeff, out_idx, flags, ticket, g.spread, record, g.units, g.nint, bits);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

template <int K, int U, int C>
int second(int fix, uint8_t* slots, uint64_t stride, uint64_t cstride, uint64_t L, uint64_t S, uint32_t nobj,
           uint32_t rows, const uint32_t* coeff, const uint32_t* dtab, const uint32_t* out_idx, const uint32_t* mapping,
           const uint32_t* status, const uint8_t* record, const uint8_t* bits, uint32_t* list, uint32_t* count,
           uint32_t blocks, hipStream_t s) {
  const Geo g = geo<K, U, C>(S, L, nobj);
  if (!g.spread) return -2;
  if (hipMemsetAsync(count, 0, 4, s) != hipSuccess) return -1;
  hipLaunchKernelGGL(redo_list_kernel<C>, dim3(1024), dim3(kBlock), 0, s, record, mapping, status, nobj, g.units,
                     g.nint, list, count);
  if (fix)
    hipLaunchKernelGGL((fix_kernel<K, U, C>), dim3(blocks), dim3(kBlock), 0, s, slots, stride, cstride, rows, dtab,
                       out_idx, mapping, bits, list, count, g.units, g.nint);
  else
    hipLaunchKernelGGL((redo_interior_kernel<K, U, C>), dim3(blocks), dim3(kBlock), 0, s, slots, stride, cstride, L,
                       rows, coeff, out_idx, mapping, list, count, g.units, g.nint);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
}  // namespace

// shape 0: K = 8 (U 2, C 3, the product's C3 form); 1: K = 10 (U 1, C 6, C5's)
extern "C" int tbf_pass0(int shape, int bits_on, uint8_t* slots, uint64_t stride, uint64_t cstride, uint64_t L,
                         uint64_t S, uint32_t nobj, uint32_t rows, const uint32_t* coeff, const uint32_t* out_idx,
                         uint32_t* flags, uint32_t* ticket, uint32_t blocks, uint8_t* record, uint8_t* bits,
                         void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (shape == 0) return pass0<8, 2, 3>(bits_on, slots, stride, cstride, L, S, nobj, rows, coeff, out_idx, flags, ticket, blocks, record, bits, s);
  if (shape == 1) return pass0<10, 1, 6>(bits_on, slots, stride, cstride, L, S, nobj, rows, coeff, out_idx, flags, ticket, blocks, record, bits, s);
  return -3;
}

extern "C" int tbf_second(int shape, int fix, uint8_t* slots, uint64_t stride, uint64_t cstride, uint64_t L,
                          uint64_t S, uint32_t nobj, uint32_t rows, const uint32_t* coeff, const uint32_t* dtab,
                          const uint32_t* out_idx,
                          const uint32_t* mapping, const uint32_t* status, const uint8_t* record, const uint8_t* bits,
                          uint32_t* list, uint32_t* count, uint32_t blocks, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (shape == 0) return second<8, 2, 3>(fix, slots, stride, cstride, L, S, nobj, rows, coeff, dtab, out_idx, mapping, status, record, bits, list, count, blocks, s);
  if (shape == 1) return second<10, 1, 6>(fix, slots, stride, cstride, L, S, nobj, rows, coeff, dtab, out_idx, mapping, status, record, bits, list, count, blocks, s);
  return -3;
}

// Bytes of the top-bit buffer and of the record (units per object) for a shape.
extern "C" uint64_t tbf_bits_bytes(int shape, uint64_t S, uint64_t L, uint32_t nobj) {
  if (shape == 0) return (uint64_t)nobj * geo<8, 2, 3>(S, L, nobj).nint * TopBits<8, 2>::kTileBytes;
  if (shape == 1) return (uint64_t)nobj * geo<10, 1, 6>(S, L, nobj).nint * TopBits<10, 1>::kTileBytes;
  return 0;
}
extern "C" uint32_t tbf_units(int shape, uint64_t S, uint64_t L, uint32_t nobj) {
  if (shape == 0) return geo<8, 2, 3>(S, L, nobj).units;
  if (shape == 1) return geo<10, 1, 6>(S, L, nobj).units;
  return 0;
}
extern "C" int tbf_ticket_words() { return (int)apply::ticket_set_words(kQueueCounters); }
