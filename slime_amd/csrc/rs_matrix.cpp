// Host-side code-matrix construction for the GF(2^32-5) Reed-Solomon code of
// slime's internal/rs.  These are tiny (<= 200 x 100) and computed once per
// shape, then cached; the data path never runs here.
//
//   vandermonde   internal/rs/matrix.go:8-22
//   reduce_cols   internal/rs/matrix.go:35-97   (solveSubIdentity)
//   parity        internal/rs/matrix.go:27-31   (ParityMatrix)
//   inverse       internal/rs/matrix.go:112-121 (invertMatrix)
//   cache         internal/rs/matrixcache.go:7-29
//   minverse/pow  internal/rs/gf/gf.go:5-60
//
// Exact modular arithmetic makes the systematic matrix V * V_top^-1 and every
// inverse unique, so the values match the reference bit for bit.  The column
// elimination keeps the reference's pivot rule so singular inputs fail with
// the same condition (and hence the same panic text) as the reference.
#include "rs_matrix.hpp"

#include <map>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <utility>

#include "gfp_host.hpp"

namespace slime {

uint32_t gf_pow(uint32_t x, uint64_t e) {
  uint64_t base = x % kP, acc = 1;
  while (e) {
    if (e & 1) acc = (acc * base) % kP;
    base = (base * base) % kP;
    e >>= 1;
  }
  return (uint32_t)acc;
}

// gf.MInverse: the reference's fixed chain computes in^(2^32 - 7) = in^(p-2).
uint32_t gf_minverse(uint32_t in) { return gf_pow(in, (uint64_t)kP - 2); }

// gf.Raise: x^n with Raise(x, 0) = 1 for every x (including 0).
uint32_t gf_raise(uint32_t x, uint32_t n) { return n == 0 ? 1u : gf_pow(x, n); }

Matrix vandermonde(int d, int p) {
  Matrix m((size_t)(d + p), (size_t)d);
  for (int j = 0; j < d; ++j) {
    // Row i holds (j+1)^i: walk powers instead of recomputing each one.
    uint64_t v = 1;
    for (int i = 0; i < d + p; ++i) {
      m.at(i, j) = (uint32_t)v;
      v = (v * (uint64_t)(j + 1)) % kP;
    }
  }
  return m;
}

Status reduce_cols(Matrix& m) {
  const size_t cols = m.cols, rows = m.rows;
  for (size_t i = 0; i < cols; ++i) {
    if (m.at(i, i) == 0) {
      // Pivot: the first column to the right with a nonzero entry in row i.
      for (size_t j = i + 1; j < cols; ++j) {
        if (m.at(i, j) != 0) {
          for (size_t r = 0; r < rows; ++r) std::swap(m.at(r, i), m.at(r, j));
          break;
        }
      }
      if (m.at(i, i) == 0) return Status::SingularNonzero;
    }
    if (m.at(i, i) != 1) {
      const uint32_t s = gf_minverse(m.at(i, i));
      for (size_t r = 0; r < rows; ++r) m.at(r, i) = mulmod(m.at(r, i), s);
      if (m.at(i, i) != 1) return Status::SingularOne;
    }
    for (size_t j = 0; j < cols; ++j) {
      if (j == i || m.at(i, j) == 0) continue;
      const uint32_t f = kP - m.at(i, j);  // column j += f * column i
      for (size_t r = 0; r < rows; ++r) m.at(r, j) = addmod(m.at(r, j), mulmod(m.at(r, i), f));
      if (m.at(i, j) != 0) return Status::SingularZero;
    }
  }
  return Status::Ok;
}

Status parity_matrix(int d, int p, Matrix* out) {
  Matrix m = vandermonde(d, p);
  const Status st = reduce_cols(m);
  if (st == Status::Ok) *out = std::move(m);
  return st;
}

Status invert(const Matrix& m, Matrix* inv) {
  const size_t d = m.cols;
  Matrix aug(m.rows + d, d);
  for (size_t r = 0; r < m.rows; ++r)
    for (size_t c = 0; c < d; ++c) aug.at(r, c) = m.at(r, c);
  for (size_t i = 0; i < d; ++i) aug.at(m.rows + i, i) = 1;
  const Status st = reduce_cols(aug);
  if (st != Status::Ok) return st;
  Matrix res(d, d);
  for (size_t r = 0; r < d; ++r)
    for (size_t c = 0; c < d; ++c) res.at(r, c) = aug.at(aug.rows - d + r, c);
  *inv = std::move(res);
  return Status::Ok;
}

namespace {
std::shared_mutex g_cache_mu;
std::map<std::pair<int, int>, std::unique_ptr<const Matrix>> g_cache;
}  // namespace

Status parity_matrix_cached(int d, int p, const Matrix** out) {
  const auto key = std::make_pair(d, p);
  {
    std::shared_lock<std::shared_mutex> rd(g_cache_mu);
    auto it = g_cache.find(key);
    if (it != g_cache.end()) {
      *out = it->second.get();
      return Status::Ok;
    }
  }
  Matrix m;
  const Status st = parity_matrix(d, p, &m);
  if (st != Status::Ok) return st;
  std::unique_lock<std::shared_mutex> wr(g_cache_mu);
  auto& slot = g_cache[key];
  if (!slot) slot = std::make_unique<const Matrix>(std::move(m));
  *out = slot.get();
  return Status::Ok;
}

// Code row `index` of the (need, total) systematic code.  Rows do not depend
// on how many parity rows the matrix was built with (the reference builds
// ParityMatrixCached(len(data), p) per call; every such matrix agrees on the
// rows it has), so one (need, index-need+1) matrix serves every caller.
Status code_row(int need, int index, std::vector<uint32_t>* row) {
  const int p = index >= need ? index - need + 1 : 0;
  const Matrix* m = nullptr;
  const Status st = parity_matrix_cached(need, p, &m);
  if (st != Status::Ok) return st;
  row->assign(m->row(index), m->row(index) + need);
  return Status::Ok;
}

}  // namespace slime
