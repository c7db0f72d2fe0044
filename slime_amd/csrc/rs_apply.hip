// GF(2^32-5) shard-matrix apply for CDNA4 (gfx950): the data path of slime's
// internal/rs (applyMatrix, internal/rs/vector.go:90-102), used for both
// parity generation (CreateParity, vector.go:18-41 — all parity rows in ONE
// pass instead of one pass per row as multi_store.go:528-531 does) and
// reconstruction (RecoverData, vector.go:50-88 — only the erased rows).
//
// Shape of the work: every output symbol column b is independent; a lane owns
// 4 consecutive columns of one object, loads them from each of the k input
// shards with one 16-byte load per shard (coalesced: a wave reads 1 KiB of
// each shard stripe), keeps the k x 4 symbols in VGPRs and produces every
// output row from them.  Coefficients are wave-uniform and come in through
// scalar loads into SGPRs (no LDS: the matrix is at most 100x100 words and
// uniform across the wave).  No cross-lane reduction is needed: the sum over
// j is in-register.  Arithmetic: exact 96-bit accumulate + one fold
// (gfp.hpp), bit-identical to the reference's per-term `%`.
#include <hip/hip_runtime.h>

#include "gfp.hpp"
#include "kernels.hpp"

namespace slime {
namespace {

constexpr int kBlock = 256;
constexpr int kMaxTemplK = 16;
// Device coefficient tables: rows padded to 16 words (64 B) for k <= 16 so a
// row arrives in one s_load_dwordx16; row stride k for the generic kernel.
constexpr int kCoeffStride = 16;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ uint4 ld16(const uint32_t* p) {
  const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st16(uint32_t* p, uint4 v) { *reinterpret_cast<uint4*>(p) = v; }

// Tail columns (ncols % 4 of them per object, or all columns when a layout is
// not 16-byte aligned): one column per lane.
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
      const u32x16 c = *reinterpret_cast<const u32x16*>(coeff + (uint64_t)i * kCoeffStride);
      uint64_t lo = 0;
      uint32_t hi = 0;
#pragma unroll
      for (int j = 0; j < K; ++j) mac(lo, hi, x[j], c[j]);
      ob[(uint64_t)out_idx[i] * out_shard + b] = fold96(lo, hi);
    }
  } else {
    for (uint32_t i = 0; i < rows; ++i) {
      const uint32_t* c = coeff + (uint64_t)i * k;
      uint64_t lo = 0;
      uint32_t hi = 0;
      for (uint32_t j = 0; j < k; ++j) mac(lo, hi, ib[(uint64_t)in_idx[j] * in_shard + b], c[j]);
      ob[(uint64_t)out_idx[i] * out_shard + b] = fold96(lo, hi);
    }
  }
}

// K > 0: compile-time number of input shards (1..16), vectorised 4 columns
// per lane.  K == 0: generic (any k up to 100), one column per lane.
template <int K, bool VEC>
__global__ __launch_bounds__(kBlock) void rs_apply_kernel(
    const uint32_t* __restrict__ in, uint32_t* __restrict__ out, uint64_t in_obj_stride, uint64_t in_shard,
    uint64_t out_obj_stride, uint64_t out_shard, const uint32_t* __restrict__ coeff,
    const uint32_t* __restrict__ in_idx, const uint32_t* __restrict__ out_idx, uint64_t ncols, uint32_t nobj,
    uint32_t rows, uint32_t k) {
  const uint64_t tid = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const uint64_t nthr = (uint64_t)gridDim.x * kBlock;
  for (uint32_t obj = blockIdx.y; obj < nobj; obj += gridDim.y) {
    const uint32_t* __restrict__ ib = in + (uint64_t)obj * in_obj_stride;
    uint32_t* __restrict__ ob = out + (uint64_t)obj * out_obj_stride;
    uint64_t done = 0;
    if constexpr (VEC && K > 0) {
      uint64_t ioff[K];
#pragma unroll
      for (int j = 0; j < K; ++j) ioff[j] = (uint64_t)in_idx[j] * in_shard;
      const uint64_t nvec = ncols >> 2;
      for (uint64_t g = tid; g < nvec; g += nthr) {
        const uint64_t b = g << 2;
        uint4 x[K];
#pragma unroll
        for (int j = 0; j < K; ++j) x[j] = ld16(ib + ioff[j] + b);
        for (uint32_t i = 0; i < rows; ++i) {
          // One 64-byte row -> one s_load_dwordx16 (SGPRs).
          const u32x16 c = *reinterpret_cast<const u32x16*>(coeff + (uint64_t)i * kCoeffStride);
          uint64_t lo0 = 0, lo1 = 0, lo2 = 0, lo3 = 0;
          uint32_t hi0 = 0, hi1 = 0, hi2 = 0, hi3 = 0;
#pragma unroll
          for (int j = 0; j < K; ++j)
            mac4(lo0, lo1, lo2, lo3, hi0, hi1, hi2, hi3, x[j].x, x[j].y, x[j].z, x[j].w, c[j]);
          uint4 r;
          r.x = fold96(lo0, hi0);
          r.y = fold96(lo1, hi1);
          r.z = fold96(lo2, hi2);
          r.w = fold96(lo3, hi3);
          st16(ob + (uint64_t)out_idx[i] * out_shard + b, r);
        }
      }
      done = nvec << 2;
    }
    for (uint64_t b = done + tid; b < ncols; b += nthr) apply_column<K>(ib, ob, coeff, in_idx, in_shard, out_idx, out_shard, rows, k, b);
  }
}

template <int K, bool VEC>
hipError_t launch_k(const ApplyLaunch& a, hipStream_t stream) {
  const uint64_t per_lane = VEC && K > 0 ? 4 : 1;
  const uint64_t units = (a.ncols + per_lane - 1) / per_lane;
  const uint32_t gy = a.nobj < 65535u ? a.nobj : 65535u;
  // ~8 resident 256-lane blocks per CU on 256 CUs; spread across objects.
  const uint64_t target = 2048;
  uint64_t gx = (target + gy - 1) / gy;
  const uint64_t need = (units + kBlock - 1) / kBlock;
  if (gx > need) gx = need;
  if (gx < 1) gx = 1;
  hipLaunchKernelGGL((rs_apply_kernel<K, VEC>), dim3((uint32_t)gx, gy), dim3(kBlock), 0, stream, a.in, a.out,
                     a.in_obj_stride, a.in_shard_stride, a.out_obj_stride, a.out_shard_stride, a.coeff, a.in_idx,
                     a.out_idx, a.ncols, a.nobj, a.rows, a.k);
  return hipGetLastError();
}

template <int K>
hipError_t dispatch_vec(const ApplyLaunch& a, hipStream_t s) {
  return a.vec_ok ? launch_k<K, true>(a, s) : launch_k<K, false>(a, s);
}

__global__ __launch_bounds__(kBlock) void canon_copy_kernel(const uint32_t* __restrict__ in,
                                                            uint32_t* __restrict__ out, uint64_t n) {
  const uint64_t nthr = (uint64_t)gridDim.x * kBlock;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += nthr) out[i] = canon(in[i]);
}

}  // namespace

hipError_t launch_apply(const ApplyLaunch& a, hipStream_t s) {
  if (a.nobj == 0 || a.ncols == 0 || a.rows == 0) return hipSuccess;
  switch (a.k) {
    case 1: return dispatch_vec<1>(a, s);
    case 2: return dispatch_vec<2>(a, s);
    case 3: return dispatch_vec<3>(a, s);
    case 4: return dispatch_vec<4>(a, s);
    case 5: return dispatch_vec<5>(a, s);
    case 6: return dispatch_vec<6>(a, s);
    case 7: return dispatch_vec<7>(a, s);
    case 8: return dispatch_vec<8>(a, s);
    case 9: return dispatch_vec<9>(a, s);
    case 10: return dispatch_vec<10>(a, s);
    case 11: return dispatch_vec<11>(a, s);
    case 12: return dispatch_vec<12>(a, s);
    case 13: return dispatch_vec<13>(a, s);
    case 14: return dispatch_vec<14>(a, s);
    case 15: return dispatch_vec<15>(a, s);
    case 16: return dispatch_vec<16>(a, s);
    default: return launch_k<0, false>(a, s);
  }
}

hipError_t launch_canon_copy(const uint32_t* in, uint32_t* out, uint64_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  uint64_t blocks = (n + kBlock - 1) / kBlock;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(canon_copy_kernel, dim3((uint32_t)blocks), dim3(kBlock), 0, s, in, out, n);
  return hipGetLastError();
}

static_assert(kMaxTemplK == 16, "dispatch table covers k = 1..16");

}  // namespace slime
