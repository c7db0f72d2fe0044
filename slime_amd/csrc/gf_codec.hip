// Byte <-> symbol codec of slime's internal/rs/gf (map.go) on CDNA4, plus the
// synthetic-symbol generator used by the benchmark.
//
//   pack   (MapToGF / MapToGFWith, map.go:15-33, :74-98): big-endian 4-byte
//          words, trailing 1-3 bytes in the HIGH bytes of a last word with
//          zero low bytes, XOR with the mapping value.  Also reduces the two
//          bits MapToGF's mapping choice needs (map.go:35-62).
//   probe  (MapToGF fallback, map.go:64-66): tests up to 64 candidate mapping
//          values in one pass over the words.
//   unpack (MapFromGF, map.go:103-113): words XOR mapping -> big-endian bytes.
//
// All byte-bound streaming work: one lane handles 16 bytes (4 words) per
// step with 16-byte accesses when the pointers allow it, grid-stride.
#include <hip/hip_runtime.h>

#include "gfp.hpp"
#include "kernels.hpp"

namespace slime {
namespace {

constexpr int kBlock = 256;

__device__ __forceinline__ uint32_t bswap(uint32_t w) { return __builtin_bswap32(w); }

__device__ __forceinline__ uint32_t flag_bits(uint32_t w) {
  // bit0: w >= p  (MapToGF can't use mapping 0);  bit1: (w ^ 1<<31) >= p.
  return (w >= kP ? 1u : 0u) | ((w ^ 0x80000000u) >= kP ? 2u : 0u);
}

__device__ __forceinline__ void flush_flags(uint32_t f, uint32_t* flags) {
  // One atomic per wave that saw anything.
  const uint64_t any1 = __ballot(f & 1u);
  const uint64_t any2 = __ballot(f & 2u);
  const uint32_t wf = (any1 ? 1u : 0u) | (any2 ? 2u : 0u);
  if (wf && (threadIdx.x & 63) == 0) atomicOr(flags, wf);
}

uint64_t grid_for(uint64_t units) {
  uint64_t blocks = (units + kBlock - 1) / kBlock;
  if (blocks > 8192) blocks = 8192;
  return blocks ? blocks : 1;
}

// Aligned fast path: bytes 16-byte aligned, whole 16-byte groups.
__global__ __launch_bounds__(kBlock) void pack16_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                        uint64_t ngroups, uint32_t mapping, uint32_t* flags) {
  uint32_t f = 0;
  const uint64_t nthr = (uint64_t)gridDim.x * kBlock;
  for (uint64_t g = (uint64_t)blockIdx.x * kBlock + threadIdx.x; g < ngroups; g += nthr) {
    uint4 v = src[g];
    v.x = bswap(v.x);
    v.y = bswap(v.y);
    v.z = bswap(v.z);
    v.w = bswap(v.w);
    f |= flag_bits(v.x) | flag_bits(v.y) | flag_bits(v.z) | flag_bits(v.w);
    v.x ^= mapping;
    v.y ^= mapping;
    v.z ^= mapping;
    v.w ^= mapping;
    dst[g] = v;
  }
  if (flags) flush_flags(f, flags);
}

// General path: word i from bytes [4i, 4i+4) with byte loads (any alignment,
// partial last word).  Covers [w0, nwords).
__global__ __launch_bounds__(kBlock) void pack_any_kernel(const uint8_t* __restrict__ src, uint64_t len,
                                                          uint64_t w0, uint64_t nwords, uint32_t* __restrict__ dst,
                                                          uint32_t mapping, uint32_t* flags) {
  uint32_t f = 0;
  const uint64_t nthr = (uint64_t)gridDim.x * kBlock;
  for (uint64_t i = w0 + (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < nwords; i += nthr) {
    uint32_t w = 0;
    const uint64_t b = i * 4;
#pragma unroll
    for (int t = 0; t < 4; ++t)
      if (b + t < len) w |= (uint32_t)src[b + t] << (8 * (3 - t));
    f |= flag_bits(w);
    dst[i] = w ^ mapping;
  }
  if (flags) flush_flags(f, flags);
}

__global__ __launch_bounds__(kBlock) void xor_kernel(uint32_t* __restrict__ w, uint64_t n, uint32_t m) {
  const uint64_t nthr = (uint64_t)gridDim.x * kBlock;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += nthr) w[i] ^= m;
}

__global__ __launch_bounds__(kBlock) void probe_kernel(const uint32_t* __restrict__ w, uint64_t n,
                                                       const uint32_t* __restrict__ cand, uint32_t ncand,
                                                       uint32_t* __restrict__ bad) {
  // bad_mask bit c set <=> some word ^ cand[c] >= p, i.e. word ^ cand[c] in
  // {0xFFFFFFFB..0xFFFFFFFF}, i.e. (word ^ cand[c]) > 0xFFFFFFFA.
  uint64_t bad_mask = 0;
  const uint64_t nthr = (uint64_t)gridDim.x * kBlock;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += nthr) {
    const uint32_t x = w[i];
    for (uint32_t c = 0; c < ncand; ++c)
      if ((x ^ cand[c]) >= kP) bad_mask |= 1ull << c;
  }
  for (uint32_t c = 0; c < ncand; ++c)
    if (__ballot((bad_mask >> c) & 1ull) && (threadIdx.x & 63) == 0) atomicOr(&bad[c], 1u);
}

__global__ __launch_bounds__(kBlock) void unpack16_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                          uint64_t ngroups, uint32_t mapping) {
  const uint64_t nthr = (uint64_t)gridDim.x * kBlock;
  for (uint64_t g = (uint64_t)blockIdx.x * kBlock + threadIdx.x; g < ngroups; g += nthr) {
    uint4 v = src[g];
    v.x = bswap(v.x ^ mapping);
    v.y = bswap(v.y ^ mapping);
    v.z = bswap(v.z ^ mapping);
    v.w = bswap(v.w ^ mapping);
    dst[g] = v;
  }
}

__global__ __launch_bounds__(kBlock) void unpack_any_kernel(const uint32_t* __restrict__ src, uint64_t w0,
                                                            uint64_t n, uint32_t mapping, uint8_t* __restrict__ dst) {
  const uint64_t nthr = (uint64_t)gridDim.x * kBlock;
  for (uint64_t i = w0 + (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += nthr) {
    const uint32_t w = src[i] ^ mapping;
    dst[4 * i] = (uint8_t)(w >> 24);
    dst[4 * i + 1] = (uint8_t)(w >> 16);
    dst[4 * i + 2] = (uint8_t)(w >> 8);
    dst[4 * i + 3] = (uint8_t)w;
  }
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(kBlock) void fill_kernel(uint32_t* __restrict__ dst, uint64_t n, uint64_t seed) {
  const uint64_t nthr = (uint64_t)gridDim.x * kBlock;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += nthr) {
    const uint32_t w = (uint32_t)(splitmix64(seed ^ (i * 0xD1B54A32D192ED03ull)) >> 32);
    dst[i] = canon(w);
  }
}

}  // namespace

hipError_t launch_map_pack(const uint8_t* bytes, uint64_t len, uint32_t mapping, uint32_t* words_out,
                           uint32_t* flags, hipStream_t s) {
  (void)hipGetLastError();  // report only this launch's error, not one left on the thread
  const uint64_t nwords = (len + 3) / 4;
  if (nwords == 0) return hipSuccess;
  uint64_t done_words = 0;
  const bool aligned = (((uintptr_t)bytes | (uintptr_t)words_out) & 15u) == 0;
  if (aligned && len >= 16) {
    const uint64_t ngroups = len / 16;
    hipLaunchKernelGGL(pack16_kernel, dim3((uint32_t)grid_for(ngroups)), dim3(kBlock), 0, s,
                       reinterpret_cast<const uint4*>(bytes), reinterpret_cast<uint4*>(words_out), ngroups, mapping,
                       flags);
    done_words = ngroups * 4;
  }
  if (done_words < nwords)
    hipLaunchKernelGGL(pack_any_kernel, dim3((uint32_t)grid_for(nwords - done_words)), dim3(kBlock), 0, s, bytes,
                       len, done_words, nwords, words_out, mapping, flags);
  return hipGetLastError();
}

hipError_t launch_xor_words(uint32_t* words, uint64_t n, uint32_t mapping, hipStream_t s) {
  (void)hipGetLastError();  // report only this launch's error, not one left on the thread
  if (n == 0 || mapping == 0) return hipSuccess;
  hipLaunchKernelGGL(xor_kernel, dim3((uint32_t)grid_for(n)), dim3(kBlock), 0, s, words, n, mapping);
  return hipGetLastError();
}

hipError_t launch_mapping_probe(const uint32_t* words, uint64_t n, const uint32_t* cand, uint32_t ncand,
                                uint32_t* bad, hipStream_t s) {
  (void)hipGetLastError();  // report only this launch's error, not one left on the thread
  if (n == 0 || ncand == 0) return hipSuccess;
  if (ncand > 64) return hipErrorInvalidValue;
  hipLaunchKernelGGL(probe_kernel, dim3((uint32_t)grid_for(n)), dim3(kBlock), 0, s, words, n, cand, ncand, bad);
  return hipGetLastError();
}

hipError_t launch_map_unpack(const uint32_t* words, uint64_t n, uint32_t mapping, uint8_t* bytes_out, hipStream_t s) {
  (void)hipGetLastError();  // report only this launch's error, not one left on the thread
  if (n == 0) return hipSuccess;
  uint64_t done = 0;
  const bool aligned = (((uintptr_t)words | (uintptr_t)bytes_out) & 15u) == 0;
  if (aligned && n >= 4) {
    const uint64_t ngroups = n / 4;
    hipLaunchKernelGGL(unpack16_kernel, dim3((uint32_t)grid_for(ngroups)), dim3(kBlock), 0, s,
                       reinterpret_cast<const uint4*>(words), reinterpret_cast<uint4*>(bytes_out), ngroups, mapping);
    done = ngroups * 4;
  }
  if (done < n)
    hipLaunchKernelGGL(unpack_any_kernel, dim3((uint32_t)grid_for(n - done)), dim3(kBlock), 0, s, words, done, n,
                       mapping, bytes_out);
  return hipGetLastError();
}

hipError_t launch_fill_symbols(uint32_t* dst, uint64_t n, uint64_t seed, hipStream_t s) {
  (void)hipGetLastError();  // report only this launch's error, not one left on the thread
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(fill_kernel, dim3((uint32_t)grid_for(n)), dim3(kBlock), 0, s, dst, n, seed);
  return hipGetLastError();
}

}  // namespace slime
