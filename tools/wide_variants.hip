// Variant harness for the matrix-core apply at five K steps (65 <= k <= 80,
// uniform input offsets: the encodes), tools only: the product kernel's walk
// (rs_apply_mfma_kernel.hpp) instantiated at other tile widths, column passes
// and waves per SIMD, and a 32x32x32 form (8 output rows per B fragment),
// launched on caller buffers so that tools/wide_variants.py times them in
// interleaved rounds in one process (profiles/r05/s12_widevar/, s28_m32/,
// s29_m32w1/; every variant is checked bit-exact against variant 0).
//
//   make widevar && python tools/wide_variants.py --need 80 --total 100
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "mfma_table.hpp"
#include "rs_apply_mfma_kernel.hpp"

using namespace slime;
using namespace slime::apply;

namespace {

// ---- 32x32x32 form: M = 8 output rows x 4 digits, K = 8 shards x 4 bytes ----
// v_mfma_i32_32x32x32_i8: lane l (r = l & 31, h = l >> 5) supplies A[row r][k =
// 16h + t] and B[k = 16h + t][col r]; D: col r, rows (reg & 3) + 8 (reg >> 2) +
// 4h -- register group i = reg >> 2 holds the four digits of output row
// 2i + h of the M tile.  One B fragment (a column's 8 shards) serves 8 output
// rows instead of 4.
namespace m32 {
typedef int32_t i32x16 __attribute__((ext_vector_type(16)));
constexpr uint32_t kShards = 8, kRows = 8;
inline uint32_t ksteps(uint32_t k) { return (k + kShards - 1) / kShards; }
inline uint32_t mtiles(uint32_t rows) { return (rows + kRows - 1) / kRows; }

// Uniform input offsets: shard 8q + 4h + jj; the last step clamps past k.
template <int KS>
struct Offs {
  uint32_t o0[4], ol[4];
  uint64_t step;
  __device__ __forceinline__ void init(uint64_t in_unit, uint32_t k, uint32_t h) {
    step = kShards * in_unit;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const uint32_t j = kShards * (KS - 1) + 4 * h + jj;
      o0[jj] = (uint32_t)((4 * h + jj) * in_unit);
      ol[jj] = (uint32_t)((j < k ? j : k - 1) * in_unit);
    }
  }
  __device__ __forceinline__ const char* at(const char* ib, int q, int jj, uint32_t colb) const {
    if (q == KS - 1) return ib + (uint32_t)(ol[jj] + colb);
    return (ib + (uint64_t)q * step) + (uint32_t)(o0[jj] + colb);
  }
};

template <int KS, int W, int MT, bool REFILL>
__device__ __forceinline__ void tile(vec_t<W> (&x)[KS][4], const char* __restrict__ ib, const Offs<KS>& so,
                                     uint32_t colbn, const i32x4* __restrict__ lfrag,
                                     const uint64_t* __restrict__ lrowc, const uint32_t* __restrict__ loff,
                                     uint32_t rows, uint32_t lane, uint32_t h, char* __restrict__ ob, uint32_t colb,
                                     bool store, uint32_t xin) {
  i32x16 acc[MT][W];
#pragma unroll
  for (int q = 0; q < KS; ++q) {
    i32x4 b[W];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj)
#pragma unroll
      for (int w = 0; w < W; ++w) b[w][jj] = (int)(x[q][jj][w] ^ xin);
    if constexpr (REFILL) {
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) x[q][jj] = ldw<W, true>(so.at(ib, q, jj, colbn));
    }
#pragma unroll
    for (int mm = 0; mm < MT; ++mm) {
      const i32x4 a = lfrag[(mm * KS + q) * 64 + lane];
#pragma unroll
      for (int w = 0; w < W; ++w)
        acc[mm][w] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b[w], q == 0 ? i32x16{} : acc[mm][w], 0, 0, 0);
    }
    if constexpr (REFILL) __builtin_amdgcn_sched_barrier(0);
  }
  if (!store) return;
#pragma unroll
  for (int mm = 0; mm < MT; ++mm)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t row = kRows * mm + 2 * i + h;
      if (row < rows) {
        const uint64_t R = lrowc[row];
        vec_t<W> r;
#pragma unroll
        for (int w = 0; w < W; ++w) {
          const i32x4 d = {acc[mm][w][4 * i], acc[mm][w][4 * i + 1], acc[mm][w][4 * i + 2], acc[mm][w][4 * i + 3]};
          r[w] = fold96(mfma_recombine(d, R), 0);
        }
        stw<W, true>(ob + (uint32_t)(loff[row] + colb), r);
      }
    }
}

template <int KS, int W, int MT, int WAVES>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WAVES, WAVES))) void kernel(
    const uint32_t* __restrict__ in, uint32_t* __restrict__ out, uint64_t in_obj_stride, uint64_t in_shard,
    uint64_t out_obj_stride, uint64_t out_shard, const uint8_t* __restrict__ table,
    const uint32_t* __restrict__ out_idx, uint64_t ncols, uint32_t nobj, uint32_t rows, uint32_t k, uint32_t nseg) {
  extern __shared__ i32x4 lds[];
  const uint32_t lane = threadIdx.x & 63, h = lane >> 5, r32 = lane & 31;
  const uint32_t nfrag = MT * KS * 64;
  const i32x4* gfrag = reinterpret_cast<const i32x4*>(table);
  for (uint32_t f = threadIdx.x; f < nfrag; f += kBlock) lds[f] = gfrag[f];
  uint64_t* lrowc = reinterpret_cast<uint64_t*>(lds + nfrag);
  uint32_t* loff = reinterpret_cast<uint32_t*>(lrowc + MT * kRows);
  const uint64_t* growc = reinterpret_cast<const uint64_t*>(table + (size_t)nfrag * 16);
  for (uint32_t i = threadIdx.x; i < MT * kRows; i += kBlock) {
    lrowc[i] = i < rows ? growc[i] : 0;
    loff[i] = i < rows ? (uint32_t)(out_idx[i] * out_shard * 4) : 0;
  }
  Offs<KS> so;
  so.init(in_shard * 4, k, h);
  __syncthreads();
  const uint32_t nvec = (uint32_t)(ncols >> 2);
  const uint32_t seg_vec = segment_vectors(nvec, nseg);
  const uint64_t nwork = (uint64_t)nobj * nseg;
  const uint32_t wave = blockIdx.x * kWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nwaves = gridDim.x * kWaves;
  constexpr uint32_t TC = 32 * W;
  for (uint64_t wi = blockIdx.y; wi < nwork; wi += gridDim.y) {
    const uint64_t obj = wi / nseg;
    const uint32_t seg = (uint32_t)(wi % nseg);
    const char* __restrict__ ib = reinterpret_cast<const char*>(in + obj * in_obj_stride);
    char* __restrict__ ob = reinterpret_cast<char*>(out + obj * out_obj_stride);
    const uint32_t v0 = seg * seg_vec < nvec ? seg * seg_vec : nvec;
    const uint32_t v1 = nvec - v0 > seg_vec ? v0 + seg_vec : nvec;
    const uint32_t c0 = 4 * v0, c1 = 4 * v1;  // whole tiles (the harness's ncols is a multiple of 64 * W)
    const uint32_t ntiles = (c1 - c0) / TC;
    auto colb_of = [&](uint32_t t) { return (c0 + t * TC + r32 * W) << 2; };
    vec_t<W> x[KS][4];
    uint32_t t = wave;
    if (t < ntiles) {
#pragma unroll
      for (int q = 0; q < KS; ++q)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) x[q][jj] = ldw<W, true>(so.at(ib, q, jj, colb_of(t)));
    }
    while (t < ntiles) {
      const uint32_t tn = t + nwaves;
      if (tn < ntiles)
        tile<KS, W, MT, true>(x, ib, so, colb_of(tn), lds, lrowc, loff, rows, lane, h, ob, colb_of(t), true,
                              0x80808080u);
      else
        tile<KS, W, MT, false>(x, ib, so, 0, lds, lrowc, loff, rows, lane, h, ob, colb_of(t), true, 0x80808080u);
      t = tn;
    }
  }
}

template <int KS, int W, int MT, int WAVES>
hipError_t launch(const uint32_t* in, uint32_t* out, uint64_t in_obj, uint64_t in_shard, uint64_t out_obj,
                  uint64_t out_shard, const uint8_t* table, const uint32_t* out_idx, uint64_t ncols, uint32_t nobj,
                  uint32_t rows, uint32_t k, hipStream_t s) {
  const uint32_t lds = MT * KS * 1024 + MT * kRows * 12;
  const uint64_t want = (256 + nobj - 1) / nobj, max_s = (ncols >> 2) / 1024 ? (ncols >> 2) / 1024 : 1;
  const uint32_t nseg = (uint32_t)(want < max_s ? want : max_s);
  const uint64_t nwork = (uint64_t)nobj * nseg;
  const uint64_t gy = nwork < 65535 ? nwork : 65535;
  uint64_t gx = (256ull * WAVES + gy - 1) / gy;
  if (gx < 1) gx = 1;
  hipLaunchKernelGGL((kernel<KS, W, MT, WAVES>), dim3((uint32_t)gx, (uint32_t)gy), dim3(kBlock), lds, s, in, out,
                     in_obj, in_shard, out_obj, out_shard, table, out_idx, ncols, nobj, rows, k, nseg);
  return hipGetLastError();
}

// The 32x32 table: A fragments [mtiles][ksteps][64][16 B] (lane l: output row
// 8m + ((l & 31) >> 2), digit (l & 31) & 3, shards 8q + 4(l >> 5) + t/4, byte
// t & 3), then the row constants (mfma_table.hpp's identity).
std::vector<uint8_t> build(const uint32_t* coeff, uint32_t rows, uint32_t k) {
  const uint32_t MT = mtiles(rows), KS = ksteps(k);
  std::vector<uint8_t> t((size_t)MT * KS * 1024 + (size_t)MT * kRows * 8, 0);
  int8_t* frag = reinterpret_cast<int8_t*>(t.data());
  for (uint32_t m = 0; m < MT; ++m)
    for (uint32_t q = 0; q < KS; ++q)
      for (uint32_t l = 0; l < 64; ++l) {
        const uint32_t rr = l & 31, i = kRows * m + (rr >> 2), e = rr & 3, h = l >> 5;
        int8_t* o = frag + (((size_t)m * KS + q) * 64 + l) * 16;
        if (i >= rows) continue;
        for (uint32_t tt = 0; tt < 16; ++tt) {
          const uint32_t j = kShards * q + 4 * h + (tt >> 2), b = tt & 3;
          if (j >= k) continue;
          uint32_t w = coeff[(size_t)i * k + j] % kP;
          for (uint32_t z = 0; z < b; ++z) w = mulmod(w, 256);
          int8_t d[4];
          mfma::digits(w, d);
          o[tt] = d[e];
        }
      }
  uint64_t* rowc = reinterpret_cast<uint64_t*>(t.data() + (size_t)MT * KS * 1024);
  const uint32_t half = (uint32_t)((128ull * 0x01010101ull) % kP);
  for (uint32_t i = 0; i < rows; ++i) {
    uint32_t sum = 0;
    for (uint32_t j = 0; j < k; ++j) sum = addmod(sum, coeff[(size_t)i * k + j] % kP);
    rowc[i] = (uint64_t)mulmod(half, sum) + mfma::kOffset;
  }
  return t;
}
}  // namespace m32

// ---- column-block interleaved layout (research: is the wide-code rate the
// DRAM side of k concurrent shard streams?) ----
// Block t of the buffer holds 64 columns of every shard: [total shards][64
// symbols], 256 B per shard, so one wave tile reads one contiguous
// total x 256 B region instead of k far-apart rows.  Same math as the
// product's walk (mfma_tile, four-column tiles); the parity rows land in
// their 256 B slots of the same block.
template <int KS, int WAVES>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WAVES, WAVES))) void ilv_kernel(
    const uint32_t* __restrict__ in, const uint8_t* __restrict__ table, const uint32_t* __restrict__ out_idx,
    uint64_t nblocks, uint32_t total, uint32_t rows, uint32_t k) {
  extern __shared__ i32x4 lds[];
  const uint32_t MT = (rows + 3) / 4;
  const uint32_t lane = threadIdx.x & 63, g = lane >> 4, n = lane & 15;
  uint64_t* lrowc;
  uint32_t* loff;
  ShardOffs<KS, true> so;
  mfma_prologue(lds, table, nullptr, out_idx, 256, 256, MT, KS, rows, k, g, &lrowc, &loff, so);
  const uint64_t gw = (uint64_t)blockIdx.x * kWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t gn = (uint64_t)gridDim.x * kWaves;
  const uint64_t bstride = (uint64_t)total * 256;  // bytes per block
  const char* base = reinterpret_cast<const char*>(in);
  const uint32_t colb = n * 16;  // the lane's four columns in each 256 B shard slot
  NoPre nopre;
  vec_t<4> x[KS][4];
  uint64_t t = gw;
  if (t < nblocks) mfma_load_tile<KS, 4, true>(x, base + t * bstride, so, colb);
  while (t < nblocks) {
    const uint64_t tn = t + gn;
    char* ob = const_cast<char*>(base + t * bstride);
    if (tn < nblocks)
      mfma_tile<KS, 4, true, true, true, false, NoPre, ShardOffs<KS, true>, 1>(
          x, base + tn * bstride, so, colb, lds, lrowc, loff, MT, rows, lane, g, ob, colb, true,
          MfmaIO{0x80808080u, 0u}, nopre);
    else
      mfma_tile<KS, 4, true, true, false, false, NoPre, ShardOffs<KS, true>, 1>(
          x, nullptr, so, 0, lds, lrowc, loff, MT, rows, lane, g, ob, colb, true, MfmaIO{0x80808080u, 0u}, nopre);
    t = tn;
  }
}

template <int KS, int W, int NH, int WAVES>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WAVES, WAVES))) void wv_kernel(
    const uint32_t* __restrict__ in, uint32_t* __restrict__ out, uint64_t in_obj_stride, uint64_t in_shard,
    uint64_t out_obj_stride, uint64_t out_shard, const uint8_t* __restrict__ table,
    const uint32_t* __restrict__ out_idx, uint64_t ncols, uint32_t nobj, uint32_t rows, uint32_t k, uint32_t nseg) {
  extern __shared__ i32x4 lds[];
  const uint32_t MT = (rows + 3) / 4;
  const uint32_t lane = threadIdx.x & 63, g = lane >> 4, n = lane & 15;
  uint64_t* lrowc;
  uint32_t* loff;
  ShardOffs<KS, true> so;
  mfma_prologue(lds, table, nullptr, out_idx, in_shard * 4, out_shard * 4, MT, KS, rows, k, g, &lrowc, &loff, so);
  const uint32_t nvec = (uint32_t)(ncols >> 2);
  const uint32_t seg_vec = segment_vectors(nvec, nseg);
  const uint64_t nwork = (uint64_t)nobj * nseg;
  const uint32_t wave = blockIdx.x * kWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nwaves = gridDim.x * kWaves;
  NoPre nopre;
  for (uint64_t wi = blockIdx.y; wi < nwork; wi += gridDim.y) {
    const uint64_t obj = wi / nseg;
    const uint32_t seg = (uint32_t)(wi % nseg);
    const char* __restrict__ ib = reinterpret_cast<const char*>(in + obj * in_obj_stride);
    char* __restrict__ ob = reinterpret_cast<char*>(out + obj * out_obj_stride);
    const uint32_t v0 = seg * seg_vec < nvec ? seg * seg_vec : nvec;
    const uint32_t v1 = nvec - v0 > seg_vec ? v0 + seg_vec : nvec;
    if (v1 > v0)
      mfma_walk<KS, W, true, true, false, NoPre, ShardOffs<KS, true>, NH>(
          ib, ob, so, lds, lrowc, loff, MT, rows, lane, g, n, 4 * v0, 4 * v1, wave, nwaves, MfmaIO{0x80808080u, 0u},
          nopre);
  }
}

template <int KS, int W, int NH, int WAVES>
hipError_t launch(const uint32_t* in, uint32_t* out, uint64_t in_obj, uint64_t in_shard, uint64_t out_obj,
                  uint64_t out_shard, const uint8_t* table, const uint32_t* out_idx, uint64_t ncols, uint32_t nobj,
                  uint32_t rows, uint32_t k, hipStream_t s) {
  const uint32_t lds = mfma_lds_bytes(mfma::mtiles(rows), KS);
  // object_segments (rs_apply.hip): about 256 object segments in flight
  const uint64_t want = (256 + nobj - 1) / nobj, max_s = (ncols >> 2) / 1024 ? (ncols >> 2) / 1024 : 1;
  const uint32_t nseg = (uint32_t)(want < max_s ? want : max_s);
  const uint64_t nwork = (uint64_t)nobj * nseg;
  const uint64_t gy = nwork < 65535 ? nwork : 65535;
  uint64_t gx = (256ull * WAVES + gy - 1) / gy;
  if (gx < 1) gx = 1;
  hipLaunchKernelGGL((wv_kernel<KS, W, NH, WAVES>), dim3((uint32_t)gx, (uint32_t)gy), dim3(kBlock), lds, s, in,
                     out, in_obj, in_shard, out_obj, out_shard, table, out_idx, ncols, nobj, rows, k, nseg);
  return hipGetLastError();
}

}  // namespace

extern "C" {

// Variant names, one per id (nullptr past the last).
const char* wv_name(int v) {
  // (split refills -- each column pass's half reloaded right after it -- ran 0.36 of peak: removed)
  static const char* names[] = {"W4 NH2 2w", "W2 NH1 2w", "W4 NH1 1w (product)", "W4 NH1 2w (spills)",
                                "32x32 W2 2w", "32x32 W2 1w", "32x32 W1 2w", "32x32 W1 3w",
                                "interleaved 256 B blocks W4 1w (timing only)"};
  return v >= 0 && v < (int)(sizeof(names) / sizeof(names[0])) ? names[v] : nullptr;
}

// Host-side digit table of coeff (rows x k) into dst (capacity cap); its size.
// Variants from 4 on take the 32x32 table.
uint64_t wv_table(int v, const uint32_t* coeff, uint32_t rows, uint32_t k, uint8_t* dst, uint64_t cap) {
  const std::vector<uint8_t> t = v >= 4 ? m32::build(coeff, rows, k) : mfma::build_table(coeff, rows, k, false);
  if (dst && cap >= t.size()) memcpy(dst, t.data(), t.size());
  return t.size();
}

int wv_launch(int v, const uint32_t* in, uint32_t* out, uint64_t in_obj, uint64_t in_shard, uint64_t out_obj,
              uint64_t out_shard, const uint8_t* table, const uint32_t* out_idx, uint64_t ncols, uint32_t nobj,
              uint32_t rows, uint32_t k, hipStream_t s) {
  if (rows > 32 || (ncols & 127)) return (int)hipErrorInvalidValue;
  if (v == 8) {  // the same buffer as 64-column blocks of every shard (ncols x nobj columns)
    if (mfma::ksteps(k) != 5 || in_shard != ncols) return (int)hipErrorInvalidValue;
    const uint32_t total = (uint32_t)(in_obj / in_shard);
    const uint64_t nblocks = (uint64_t)nobj * ncols / 64;
    const uint32_t lds = mfma_lds_bytes(mfma::mtiles(rows), 5);
    hipLaunchKernelGGL((ilv_kernel<5, 1>), dim3(256), dim3(kBlock), lds, s, in, table, out_idx, nblocks, total, rows,
                       k);
    return (int)hipGetLastError();
  }
  if (v >= 4) {  // 32x32x32: k 73..80 (ten K steps of 8 shards), rows 17..24 (three M tiles of 8)
    if (m32::ksteps(k) != 10 || m32::mtiles(rows) != 3) return (int)hipErrorInvalidValue;
#define W32(W, WV_) \
  m32::launch<10, W, 3, WV_>(in, out, in_obj, in_shard, out_obj, out_shard, table, out_idx, ncols, nobj, rows, k, s)
    switch (v) {
      case 4: return (int)W32(2, 2);
      case 5: return (int)W32(2, 1);
      case 6: return (int)W32(1, 2);
      case 7: return (int)W32(1, 3);
      default: return (int)hipErrorInvalidValue;
    }
#undef W32
  }
  if (mfma::ksteps(k) != 5) return (int)hipErrorInvalidValue;
#define WV(W, NH, WV_) \
  launch<5, W, NH, WV_>(in, out, in_obj, in_shard, out_obj, out_shard, table, out_idx, ncols, nobj, rows, k, s)
  switch (v) {
    case 0: return (int)WV(4, 2, 2);
    case 1: return (int)WV(2, 1, 2);
    case 2: return (int)WV(4, 1, 1);
    case 3: return (int)WV(4, 1, 2);
    default: return (int)hipErrorInvalidValue;
  }
#undef WV
}

}  // extern "C"
