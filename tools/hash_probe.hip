// Throughput probe for §8(f3): chunk/object hashes on the GPU (tools only).
//   sha256_msgs  SHA-256 (FIPS 180-4) of nmsg messages of nbytes each (nbytes a
//                multiple of 64), one lane per message -- the hash is a
//                sequential chain per message, so lanes = messages.
//   fnv1a64_msgs FNV-1a-64 of each message (storedir key-file checksum,
//                internal/store/storedir/directory.go:25-28,549), one lane per message.
// Built into tools/libhashprobe.so by `make hashprobe`; driven by tools/hash_probe.py.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {
constexpr int B = 64;  // one wave per block: spreads few messages over many CUs

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

#define K256                                                                                                   \
  0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,      \
      0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,  \
      0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,  \
      0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,  \
      0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,  \
      0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,  \
      0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,  \
      0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u

__device__ __forceinline__ void compress(uint32_t st[8], uint32_t w[16]) {
  constexpr uint32_t k[64] = {K256};
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    if (i >= 16) {
      const uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
      const uint32_t s0 = rotr(w15, 7) ^ rotr(w15, 18) ^ (w15 >> 3);
      const uint32_t s1 = rotr(w2, 17) ^ rotr(w2, 19) ^ (w2 >> 10);
      w[i & 15] += s0 + w[(i - 7) & 15] + s1;
    }
    const uint32_t t1 = h + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) + k[i] + w[i & 15];
    const uint32_t t2 = (rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    h = g, g = f, f = e, e = d + t1, d = c, c = b, b = a, a = t1 + t2;
  }
  st[0] += a, st[1] += b, st[2] += c, st[3] += d, st[4] += e, st[5] += f, st[6] += g, st[7] += h;
}

__global__ __launch_bounds__(B) void sha256_msgs(const uint8_t* __restrict__ in, uint64_t nbytes, uint32_t nmsg,
                                                 uint32_t* __restrict__ digest) {
  const uint32_t m = blockIdx.x * B + threadIdx.x;
  if (m >= nmsg) return;
  const uint4* p = reinterpret_cast<const uint4*>(in + (uint64_t)m * nbytes);
  uint32_t st[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                    0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  uint32_t w[16];
  for (uint64_t blk = 0; blk < nbytes / 64; ++blk) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint4 v = p[blk * 4 + q];
      w[4 * q + 0] = __builtin_bswap32(v.x);
      w[4 * q + 1] = __builtin_bswap32(v.y);
      w[4 * q + 2] = __builtin_bswap32(v.z);
      w[4 * q + 3] = __builtin_bswap32(v.w);
    }
    compress(st, w);
  }
  // padding block (nbytes % 64 == 0): 0x80, zeros, 64-bit big-endian bit length
#pragma unroll
  for (int i = 0; i < 16; ++i) w[i] = 0;
  w[0] = 0x80000000u;
  const uint64_t bits = nbytes * 8;
  w[14] = (uint32_t)(bits >> 32);
  w[15] = (uint32_t)bits;
  compress(st, w);
#pragma unroll
  for (int i = 0; i < 8; ++i) digest[(uint64_t)m * 8 + i] = st[i];
}

__global__ __launch_bounds__(B) void fnv1a64_msgs(const uint8_t* __restrict__ in, uint64_t nbytes, uint32_t nmsg,
                                                  uint64_t* __restrict__ out) {
  const uint32_t m = blockIdx.x * B + threadIdx.x;
  if (m >= nmsg) return;
  const uint4* p = reinterpret_cast<const uint4*>(in + (uint64_t)m * nbytes);
  uint64_t h = 0xcbf29ce484222325ull;
  for (uint64_t i = 0; i < nbytes / 16; ++i) {
    const uint4 v = p[i];
    const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        h ^= (wd[q] >> (8 * b)) & 0xFF;
        h *= 0x100000001b3ull;
      }
  }
  out[m] = h;
}

float timed(void (*launch)(const void*, uint64_t, uint32_t, void*), const void* in, uint64_t nbytes, uint32_t nmsg,
            void* out, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  launch(in, nbytes, nmsg, out);  // warm
  (void)hipEventRecord(a, nullptr);
  for (int r = 0; r < reps; ++r) launch(in, nbytes, nmsg, out);
  (void)hipEventRecord(b, nullptr);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  return ms / reps;
}

void launch_sha(const void* in, uint64_t nbytes, uint32_t nmsg, void* out) {
  hipLaunchKernelGGL(sha256_msgs, dim3((nmsg + B - 1) / B), dim3(B), 0, nullptr, (const uint8_t*)in, nbytes, nmsg,
                     (uint32_t*)out);
}
void launch_fnv(const void* in, uint64_t nbytes, uint32_t nmsg, void* out) {
  hipLaunchKernelGGL(fnv1a64_msgs, dim3((nmsg + B - 1) / B), dim3(B), 0, nullptr, (const uint8_t*)in, nbytes, nmsg,
                     (uint64_t*)out);
}
}  // namespace

extern "C" {
// Average ms per launch over `reps` launches (after one warm-up), or -1 on a bad shape.
float hp_sha256(const void* in, uint64_t nbytes, uint32_t nmsg, void* digest, int reps) {
  if (nbytes % 64 || nmsg == 0) return -1.f;
  return timed(launch_sha, in, nbytes, nmsg, digest, reps);
}
float hp_fnv1a64(const void* in, uint64_t nbytes, uint32_t nmsg, void* out, int reps) {
  if (nbytes % 16 || nmsg == 0) return -1.f;
  return timed(launch_fnv, in, nbytes, nmsg, out, reps);
}
}
