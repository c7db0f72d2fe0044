// CPU emulation of the matrix-core apply kernel's arithmetic (rs_apply_mfma.hip)
// on the table mfma_table.hpp builds: every D fragment value is recomputed from
// the A fragment images and the B fragments the kernel assembles (XOR 0x80 per
// byte, int8), recombined and folded exactly as the kernel does, and compared
// with sum_j c_ij x_j mod p (applyMatrix, internal/rs/vector.go:90-102).
// Exit status 0 = all cases bit-exact.
#include <stdio.h>
#include <stdlib.h>

#include <random>
#include <vector>

// gfp.hpp is HIP code; its host fold96 compiles as plain C++ with these.
#define __host__
#define __device__
#define __forceinline__ inline
#include "gfp.hpp"
#include "mfma_table.hpp"

using namespace slime;

static uint32_t bswap32(uint32_t v) {
  return (v >> 24) | ((v >> 8) & 0xFF00u) | ((v << 8) & 0xFF0000u) | (v << 24);
}

// One column: x[j] = the register word of shard j (symbol, or bswap of one).
static bool check_case(uint32_t rows, uint32_t k, bool be, std::mt19937_64& rng, int ncols) {
  std::vector<uint32_t> c((size_t)rows * k);
  const uint32_t edge[] = {0u, 1u, kP - 1, 2139062143u, 2139062144u, 2155905147u, 0x80000000u, 256u, 255u};
  for (auto& v : c) v = (rng() % 4 == 0) ? edge[rng() % 9] : (uint32_t)(rng() % kP);
  const std::vector<uint8_t> tab = mfma::build_table(c.data(), rows, k, be);
  const int8_t* frag = reinterpret_cast<const int8_t*>(tab.data());
  const uint64_t* rowc = reinterpret_cast<const uint64_t*>(tab.data() + mfma::frag_bytes(rows, k));
  const uint32_t KS = mfma::ksteps(k);
  const uint32_t xedge[] = {0u, 1u, kP - 1, kP, kP + 4, 0xFFFFFFFFu, 0x7FFFFFFFu, 0x80000000u, 0x80808080u};
  for (int col = 0; col < ncols; ++col) {
    std::vector<uint32_t> w(k);  // register words
    for (auto& v : w) v = (rng() % 5 == 0) ? xedge[rng() % 9] : (uint32_t)rng();
    for (uint32_t i = 0; i < rows; ++i) {
      const uint32_t m = i / 4, il = i % 4;
      int32_t D[4] = {0, 0, 0, 0};
      for (uint32_t e = 0; e < 4; ++e)
        for (uint32_t q = 0; q < KS; ++q)
          for (uint32_t g = 0; g < 4; ++g) {
            const uint32_t lane = 16 * g + 4 * il + e;  // A row rho = 4 il + e, lane group g
            const int8_t* a = frag + (((size_t)m * KS + q) * 64 + lane) * 16;
            for (uint32_t t = 0; t < 16; ++t) {
              const uint32_t j = 16 * q + 4 * g + (t >> 2), b = t & 3;
              const uint32_t word = j < k ? w[j] : 0u;  // the kernel loads nothing past k: zero
              const int8_t s = (int8_t)(uint8_t)(((word >> (8 * b)) & 0xFF) ^ 0x80);
              D[e] += (int32_t)a[t] * (int32_t)s;
            }
          }
      const int64_t v = (int64_t)D[0] + ((int64_t)D[1] << 8) + ((int64_t)D[2] << 16) + ((int64_t)D[3] << 24);
      const uint32_t got = fold96(rowc[i] + (uint64_t)v, 0);
      uint64_t want = 0;
      for (uint32_t j = 0; j < k; ++j) {
        const uint32_t x = be ? bswap32(w[j]) : w[j];
        want = (want + (uint64_t)(c[(size_t)i * k + j] % kP) * (x % kP)) % kP;
      }
      if (got != (uint32_t)want) {
        fprintf(stderr, "MISMATCH rows=%u k=%u be=%d col=%d row=%u: got %u want %llu\n", rows, k, (int)be, col, i,
                got, (unsigned long long)want);
        return false;
      }
    }
  }
  return true;
}

int main() {
  std::mt19937_64 rng(20261017);
  // digits(): every representative reassembles, at the window edges too.
  const uint32_t probe[] = {0u, 1u, 127u, 128u, 2139062143u, 2139062144u, kP - 1, kP - 2155905152u + 0u};
  for (uint32_t v : probe) {
    int8_t d[4];
    mfma::digits(v % kP, d);
    const int64_t r = d[0] + 256ll * d[1] + 65536ll * d[2] + 16777216ll * d[3];
    if (((r % (int64_t)kP) + kP) % kP != v % kP) {
      fprintf(stderr, "digits(%u) wrong\n", v);
      return 1;
    }
  }
  int n = 0;
  const uint32_t ks[] = {1, 3, 16, 17, 32, 33, 48, 64, 80, 99, 112};
  const uint32_t rs[] = {1, 2, 3, 4, 5, 8, 16, 17, 20, 32};
  for (uint32_t k : ks)
    for (uint32_t r : rs)
      for (int be = 0; be < 2; ++be) {
        if (!mfma::supported(r, k)) continue;
        if (!check_case(r, k, be != 0, rng, 24)) return 1;
        ++n;
      }
  if (mfma::supported(33, 16) || mfma::supported(4, 113)) {
    fprintf(stderr, "supported() bounds wrong\n");
    return 1;
  }
  printf("mfma table: %d cases bit-exact\n", n);
  return 0;
}
