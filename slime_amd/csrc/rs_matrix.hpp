// Host-side GF(2^32-5) code matrices (see rs_matrix.cpp for reference citations).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <vector>

namespace slime {

enum class Status : int {
  Ok = 0,
  VaryingLength = 1,
  LenMismatch = 2,
  Empty = 3,
  NoIndices = 4,
  SingularNonzero = 5,
  SingularOne = 6,
  SingularZero = 7,
  IndexRange = 8,
  InvalidArg = 9,
  NoDevice = 10,
  Hip = 11,
  MappingFallback = 12,
  BadHash = 13,
};

struct Matrix {
  size_t rows = 0, cols = 0;
  std::vector<uint32_t> v;
  Matrix() = default;
  Matrix(size_t r, size_t c) : rows(r), cols(c), v(r * c, 0u) {}
  uint32_t& at(size_t r, size_t c) { return v[r * cols + c]; }
  uint32_t at(size_t r, size_t c) const { return v[r * cols + c]; }
  const uint32_t* row(size_t r) const { return v.data() + r * cols; }
};

uint32_t gf_pow(uint32_t x, uint64_t e);
uint32_t gf_minverse(uint32_t in);
uint32_t gf_raise(uint32_t x, uint32_t n);

Matrix vandermonde(int d, int p);
Status reduce_cols(Matrix& m);
Status parity_matrix(int d, int p, Matrix* out);
Status parity_matrix_cached(int d, int p, const Matrix** out);
Status invert(const Matrix& m, Matrix* inv);
Status code_row(int need, int index, std::vector<uint32_t>* row);

}  // namespace slime
