// Host side of the matrix-core apply kernel (rs_apply_mfma.hip): the exact
// int8-limb form of one applyMatrix (internal/rs/vector.go:90-102) and the
// per-plan table the kernel reads.  Plain C++ (no HIP types), so the CPU test
// (tests/cpp/mfma_table_test.cpp) emulates the kernel's arithmetic on it.
//
// The identity.  A symbol x (any uint32) is four bytes u_b (register byte b,
// weight 2^(8 a(b)), a(b) = b for symbols, 3 - b for big-endian chunk bytes);
// as signed int8, s_b = u_b - 128 (one XOR with 0x80 per byte).  A coefficient
// product c * 2^(8a) mod p has a representative in [-128*M, 127*M],
// M = 0x01010101 (that window is p + 4 wide), i.e. four balanced base-256
// digits g_e in [-128, 127].  Then, exactly over the integers,
//
//   sum_j c_ij x_j  ==  R_i + sum_e 2^(8e) D_ie       (mod p)
//   D_ie = sum_{j,b} g_e(c_ij 2^(8 a(b))) * s_jb       (|D| <= k * 2^16)
//   R_i  = 128 M * sum_j c_ij                          (mod p, a row constant)
//
// D is an int8 x int8 -> int32 matrix product with K = (shard, byte) pairs:
// one v_mfma_i32_16x16x64_i8 takes 16 shards x 4 bytes of K.  The M rows of a
// 16-row tile are (output row, digit) pairs, rho = 4 i_local + e, so the D
// fragment a lane receives (rows 4(lane>>4) + r, r = 0..3) is the four digits
// of ONE output row and column: the recombination R + D0 + 2^8 D1 + 2^16 D2 +
// 2^24 D3 is in-lane, then one fold.  |sum| < 2^47 for k <= 112, so the table
// stores R_i + p * 2^16 (keeps the 64-bit sum positive).
//
// Fragment order (the kernel's contract): A fragment (M tile m, K step q,
// lane l) is 16 int8, byte t = digit e = (l & 15) & 3 of output row
// i = 4m + ((l & 15) >> 2) against shard j = 16q + 4(l >> 4) + (t >> 2), register
// byte b = t & 3.  The B fragment a lane (group g = l >> 4, column n = l & 15)
// builds is the four words of shards 16q + 4g + 0..3 at its column, so byte t
// of B is (shard 16q + 4g + (t >> 2), byte t & 3): the same K slot.  The MFMA
// may order K slots however it likes internally; A and B share the order.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <vector>

#include "gfp_host.hpp"

namespace slime {
namespace mfma {

constexpr uint32_t kShardsPerStep = 16;  // 16 shards x 4 bytes = K 64
constexpr uint32_t kRowsPerTile = 4;     // 4 output rows x 4 digits = M 16
constexpr uint32_t kMaxSteps = 7;        // k <= 112 (reference codes: total <= 100)
constexpr uint32_t kMaxRows = 32;        // 8 M tiles in LDS
constexpr uint32_t kFragBytes = 64 * 16;  // one A fragment image (64 lanes x 16 B)
constexpr uint64_t kOffset = (uint64_t)kP << 16;  // added to R: keeps R + sum(D) > 0

inline uint32_t ksteps(uint32_t k) { return (k + kShardsPerStep - 1) / kShardsPerStep; }
inline uint32_t mtiles(uint32_t rows) { return (rows + kRowsPerTile - 1) / kRowsPerTile; }
inline bool supported(uint32_t rows, uint32_t k) {
  return k >= 1 && rows >= 1 && ksteps(k) <= kMaxSteps && rows <= kMaxRows;
}
// Table: A fragments [mtiles][ksteps][64 lanes][16 B], then row constants
// uint64 [mtiles * 4].  Sizes in bytes.
inline size_t frag_bytes(uint32_t rows, uint32_t k) { return (size_t)mtiles(rows) * ksteps(k) * kFragBytes; }
inline size_t table_bytes(uint32_t rows, uint32_t k) {
  return frag_bytes(rows, k) + (size_t)mtiles(rows) * kRowsPerTile * sizeof(uint64_t);
}

// Balanced base-256 digits of v (any residue in [0, p)): the representative
// r = v or v - p that lies in [-128 M, 127 M], r = sum_e d[e] 256^e.
inline void digits(uint32_t v, int8_t d[4]) {
  const int64_t M = 0x01010101;
  int64_t r = (int64_t)v <= 127 * M ? (int64_t)v : (int64_t)v - (int64_t)kP;
  for (int e = 0; e < 4; ++e) {
    int64_t q = ((r % 256) + 256) % 256;  // r mod 256 in [0, 256)
    if (q >= 128) q -= 256;
    d[e] = (int8_t)q;
    r = (r - q) / 256;
  }
}

// coeff: rows x k canonical-or-not residues, row-major.  big_endian: register
// byte b of a symbol carries weight 2^(8(3-b)) (chunk bytes loaded as words).
inline std::vector<uint8_t> build_table(const uint32_t* coeff, uint32_t rows, uint32_t k, bool big_endian) {
  const uint32_t MT = mtiles(rows), KS = ksteps(k);
  std::vector<uint8_t> t(table_bytes(rows, k), 0);
  int8_t* frag = reinterpret_cast<int8_t*>(t.data());
  for (uint32_t m = 0; m < MT; ++m)
    for (uint32_t q = 0; q < KS; ++q)
      for (uint32_t l = 0; l < 64; ++l) {
        const uint32_t rho = l & 15, i = 4 * m + (rho >> 2), e = rho & 3, g = l >> 4;
        int8_t* out = frag + (((size_t)m * KS + q) * 64 + l) * 16;
        if (i >= rows) continue;
        for (uint32_t tt = 0; tt < 16; ++tt) {
          const uint32_t j = 16 * q + 4 * g + (tt >> 2), b = tt & 3;
          if (j >= k) continue;
          const uint32_t a = big_endian ? 3 - b : b;
          uint32_t w = coeff[(size_t)i * k + j] % kP;
          for (uint32_t s = 0; s < a; ++s) w = mulmod(w, 256);
          int8_t d[4];
          digits(w, d);
          out[tt] = d[e];
        }
      }
  uint64_t* rowc = reinterpret_cast<uint64_t*>(t.data() + frag_bytes(rows, k));
  const uint32_t half = (uint32_t)((128ull * 0x01010101ull) % kP);
  for (uint32_t i = 0; i < rows; ++i) {
    uint32_t s = 0;
    for (uint32_t j = 0; j < k; ++j) s = addmod(s, coeff[(size_t)i * k + j] % kP);
    rowc[i] = (uint64_t)mulmod(half, s) + kOffset;
  }
  return t;
}

}  // namespace mfma
}  // namespace slime
