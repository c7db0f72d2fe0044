// slime_rs.hpp — C++ host mirror of encryptio/slime's Go packages
// internal/rs and internal/rs/gf over the C-ABI in slime_rs.h.
//
// The reference is compiled Go; with no Go toolchain in this image the
// testable host side above the C-ABI is this header (the cgo shim in go/ is
// the maintainer's drop-in).  Same names, argument meaning and error
// behaviour as the reference:
//   Go []uint32 / [][]uint32  ->  slime::rs::Vector / slime::rs::Matrix
//   Go []byte                 ->  std::vector<uint8_t>
//   Go panic(msg)             ->  throw slime::Panic (what() = the reference's text)
// Header-only; link with -lslime_rs.
#ifndef SLIME_RS_HPP
#define SLIME_RS_HPP

#include <array>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "slime_rs.h"

namespace slime {

// Where the reference panics (status 1..8): what() is the reference's panic
// message, or Go's runtime "index out of range" text for status 8.
struct Panic : std::runtime_error {
  int status;
  Panic(int st, const std::string& msg) : std::runtime_error(msg), status(st) {}
};

// Any other failure of the library: no device, HIP error, misuse.
struct NativeError : std::runtime_error {
  int status;
  NativeError(int st, const std::string& msg) : std::runtime_error(msg), status(st) {}
};

// Device of the data-path calls below (process-wide; SLIME_RS_ANY_DEVICE,
// the default, lets the library's device pool pick per call).
inline int& Device() {
  static int d = SLIME_RS_ANY_DEVICE;
  return d;
}

namespace detail {
// One call's context: the device goes in, that call's failure detail comes
// back (the *_ex entry points), so no thread-local state is read afterwards.
struct Call {
  char buf[512] = {0};
  slime_rs_call_t c{Device(), buf, sizeof(buf)};
  Call() = default;
  Call(const Call&) = delete;  // c points into this object's buffer
  Call& operator=(const Call&) = delete;
  const slime_rs_call_t* ptr() const { return &c; }
  void check(int rc) const {
    if (rc == SLIME_RS_OK) return;
    const std::string last = buf;
    if (rc >= SLIME_RS_ERR_VARYING_LENGTH && rc <= SLIME_RS_ERR_INDEX_RANGE) {
      std::string msg = slime_rs_status_string(rc);
      if (rc == SLIME_RS_ERR_INDEX_RANGE && !last.empty()) msg = last;
      throw Panic(rc, msg);
    }
    throw NativeError(rc, std::string("slime_rs error ") + std::to_string(rc) + ": " + last);
  }
};
}  // namespace detail

namespace gf {

// gf.MaxVal (internal/rs/gf/map.go:7)
constexpr uint32_t MaxVal = SLIME_GF_MAXVAL;

// gf.MInverse (internal/rs/gf/gf.go:5), gf.Raise (gf.go:46)
inline uint32_t MInverse(uint32_t in) { return slime_gf_minverse(in); }
inline uint32_t Raise(uint32_t x, uint32_t n) { return slime_gf_raise(x, n); }

// gf.MapToGF (internal/rs/gf/map.go:15): (mapping, words).
inline std::pair<uint32_t, std::vector<uint32_t>> MapToGF(const std::vector<uint8_t>& in) {
  std::vector<uint32_t> out((in.size() + 3) / 4);
  uint32_t mapping = 0;
  slime::detail::Call k;
  k.check(slime_gf_map_to_gf_ex(k.ptr(), in.empty() ? nullptr : in.data(), in.size(), &mapping,
                                   out.empty() ? nullptr : out.data()));
  return {mapping, std::move(out)};
}

// gf.MapToGFWith (internal/rs/gf/map.go:74)
inline std::vector<uint32_t> MapToGFWith(const std::vector<uint8_t>& in, uint32_t n) {
  std::vector<uint32_t> out((in.size() + 3) / 4);
  slime::detail::Call k;
  k.check(slime_gf_map_to_gf_with_ex(k.ptr(), in.empty() ? nullptr : in.data(), in.size(), n,
                                        out.empty() ? nullptr : out.data()));
  return out;
}

// gf.MapFromGF (internal/rs/gf/map.go:103)
inline std::vector<uint8_t> MapFromGF(uint32_t inn, const std::vector<uint32_t>& inv) {
  std::vector<uint8_t> out(4 * inv.size());
  slime::detail::Call k;
  k.check(slime_gf_map_from_gf_ex(k.ptr(), inn, inv.empty() ? nullptr : inv.data(), inv.size(),
                                     out.empty() ? nullptr : out.data()));
  return out;
}

}  // namespace gf

namespace rs {

using Vector = std::vector<uint32_t>;
using Matrix = std::vector<Vector>;

namespace detail {
inline Matrix rows_of(const uint32_t* flat, int rows, int cols) {
  Matrix m((size_t)rows, Vector((size_t)cols));
  for (int i = 0; i < rows; ++i)
    for (int j = 0; j < cols; ++j) m[i][j] = flat[(size_t)i * cols + j];
  return m;
}
inline Vector flat_of(const Matrix& m) {
  Vector f;
  for (const Vector& r : m) f.insert(f.end(), r.begin(), r.end());
  return f;
}
struct Rows {  // pointer + length arrays for the C-ABI (C never keeps them)
  std::vector<const uint32_t*> ptrs;
  std::vector<uint64_t> lens;
  explicit Rows(const Matrix& m) {
    for (const Vector& r : m) {
      ptrs.push_back(r.data());
      lens.push_back(r.size());
    }
  }
};
}  // namespace detail

// vandermondeMatrix (internal/rs/matrix.go:8): (d+p) x d, m[i][j] = (j+1)^i.
inline Matrix vandermondeMatrix(int d, int p) {
  Vector f((size_t)(d + p) * (size_t)(d > 0 ? d : 0));
  slime::detail::Call k;
  k.check(slime_rs_vandermonde_matrix_ex(k.ptr(), d, p, f.data()));
  return detail::rows_of(f.data(), d + p, d);
}

// ParityMatrix (internal/rs/matrix.go:27): systematic (d+p) x d code matrix.
inline Matrix ParityMatrix(int d, int p) {
  Vector f((size_t)(d + p) * (size_t)(d > 0 ? d : 0));
  slime::detail::Call k;
  k.check(slime_rs_parity_matrix_ex(k.ptr(), d, p, f.data()));
  return detail::rows_of(f.data(), d + p, d);
}

// ParityMatrixCached (internal/rs/matrixcache.go:11): one shared, read-only
// matrix per (d, p) for the life of the process.
inline const Matrix& ParityMatrixCached(int d, int p) {
  static std::mutex mu;
  static std::map<std::pair<int, int>, std::unique_ptr<Matrix>> cache;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find({d, p});
  if (it != cache.end()) return *it->second;
  const uint32_t* flat = nullptr;
  slime::detail::Call().check(slime_rs_parity_matrix_cached(d, p, &flat));
  auto m = std::make_unique<Matrix>(detail::rows_of(flat, d + p, d));
  const Matrix& ref = *m;
  cache.emplace(std::make_pair(d, p), std::move(m));
  return ref;
}

// solveSubIdentity (internal/rs/matrix.go:35), in place.
inline void solveSubIdentity(Matrix& m) {
  if (m.empty()) return;
  Vector f = detail::flat_of(m);
  slime::detail::Call k;
  k.check(slime_rs_solve_sub_identity_ex(k.ptr(), f.data(), (int)m.size(), (int)m[0].size()));
  m = detail::rows_of(f.data(), (int)m.size(), (int)m[0].size());
}

// cloneMatrix (internal/rs/matrix.go:99)
inline Matrix cloneMatrix(const Matrix& m) { return m; }

// invertMatrix (internal/rs/matrix.go:112): inverse of a d x d matrix.
inline Matrix invertMatrix(const Matrix& m) {
  const int d = (int)m.size();
  Vector f = detail::flat_of(m), inv((size_t)d * d);
  slime::detail::Call k;
  k.check(slime_rs_invert_matrix_ex(k.ptr(), f.data(), d, inv.data()));
  return detail::rows_of(inv.data(), d, d);
}

// CreateParity (internal/rs/vector.go:18): code row `index` of `data`,
// computed on the GPU.  Like Go, `out` is reused when its capacity holds
// len(data[0]) symbols, and the slice actually used is returned.
inline Vector CreateParity(const Matrix& data, int index, Vector out = {}) {
  detail::Rows rows(data);
  const size_t L = data.empty() ? 0 : data[0].size();
  bool same = !data.empty();
  for (const Vector& r : data) same = same && r.size() == L;
  if (same) {
    if (out.capacity() < L) out = Vector();
    out.resize(L);
  }
  slime::detail::Call k;
  k.check(slime_rs_create_parity_ex(k.ptr(), rows.ptrs.data(), rows.lens.data(), (int)data.size(), index,
                                              same ? out.data() : nullptr));
  return out;
}

// All total-len(data) parity rows in one GPU pass (the batched form of the
// caller's loop, multi_store.go:528-531).  Additive: no reference counterpart.
inline Matrix CreateParities(const Matrix& data, int total) {
  detail::Rows rows(data);
  const size_t L = data.empty() ? 0 : data[0].size();
  const int r = total - (int)data.size();
  Matrix out(r > 0 ? (size_t)r : 0, Vector(L));
  std::vector<uint32_t*> optrs;
  for (Vector& o : out) optrs.push_back(o.data());
  slime::detail::Call k;
  k.check(slime_rs_create_parities_ex(k.ptr(), rows.ptrs.data(), rows.lens.data(), (int)data.size(), total,
                                                optrs.empty() ? nullptr : optrs.data()));
  return out;
}

// RecoverData (internal/rs/vector.go:50): every data row from any len(chunks)
// code rows with the given indices.
inline Matrix RecoverData(const Matrix& chunks, const std::vector<int>& indices) {
  detail::Rows rows(chunks);
  const size_t L = chunks.empty() ? 0 : chunks[0].size();
  Matrix out(chunks.size(), Vector(L));
  std::vector<uint32_t*> optrs;
  for (Vector& o : out) optrs.push_back(o.data());
  slime::detail::Call k;
  k.check(slime_rs_recover_data_ex(k.ptr(), rows.ptrs.data(), rows.lens.data(), (int)chunks.size(),
                                             indices.empty() ? nullptr : indices.data(), (int)indices.size(),
                                             optrs.empty() ? nullptr : optrs.data()));
  return out;
}

// The data path of Multi.writeChunks (multi_store.go:526-531, :554) in one
// fused device pass: (MappingValue, chunk bytes).  Additive.
inline std::pair<uint32_t, std::vector<std::vector<uint8_t>>> WriteChunks(const std::vector<uint8_t>& data,
                                                                         int need, int total) {
  const uint64_t cb = slime_rs_chunk_size(data.size(), need);
  std::vector<std::vector<uint8_t>> chunks(total > 0 ? (size_t)total : 0, std::vector<uint8_t>(cb));
  std::vector<uint8_t*> ptrs;
  for (auto& c : chunks) ptrs.push_back(c.data());
  uint32_t mapping = 0;
  slime::detail::Call k;
  k.check(slime_rs_write_chunks_ex(k.ptr(), data.empty() ? nullptr : data.data(), data.size(), need, total,
                                             ptrs.empty() ? nullptr : ptrs.data(), &mapping));
  return {mapping, std::move(chunks)};
}

// The slow path of Multi.reconstruct (multi_store.go:215-241): the object's
// `size` bytes from `need` chunks and their indices.  Additive.
inline std::vector<uint8_t> ReconstructObject(const std::vector<std::vector<uint8_t>>& chunks,
                                              const std::vector<int>& indices, uint32_t mapping, uint64_t size) {
  std::vector<const uint8_t*> ptrs;
  for (const auto& c : chunks) ptrs.push_back(c.data());
  std::vector<uint8_t> out(size);
  slime::detail::Call k;
  k.check(slime_rs_reconstruct_ex(k.ptr(), ptrs.empty() ? nullptr : ptrs.data(),
                                            indices.empty() ? nullptr : indices.data(), (int)chunks.size(),
                                            chunks.empty() ? 0 : chunks[0].size(), mapping, size,
                                            out.empty() ? nullptr : out.data()));
  return out;
}

// WriteChunks plus each chunk's SHA-256 (store.DataV per chunk,
// multi_store.go:554-556), hashed while the device pipeline runs.  Additive.
struct WrittenChunks {
  uint32_t mapping = 0;
  std::vector<std::vector<uint8_t>> chunks;
  std::vector<std::array<uint8_t, 32>> sha256;
};
inline WrittenChunks WriteChunksDigest(const std::vector<uint8_t>& data, int need, int total) {
  WrittenChunks w;
  const uint64_t cb = slime_rs_chunk_size(data.size(), need);
  w.chunks.assign(total > 0 ? (size_t)total : 0, std::vector<uint8_t>(cb));
  w.sha256.resize(w.chunks.size());
  std::vector<uint8_t*> ptrs;
  for (auto& c : w.chunks) ptrs.push_back(c.data());
  std::vector<uint8_t> sha(32 * (w.chunks.size() + 1));
  slime::detail::Call k;
  k.check(slime_rs_write_chunks_digest_ex(k.ptr(), data.empty() ? nullptr : data.data(), data.size(), need, total,
                                          ptrs.empty() ? nullptr : ptrs.data(), &w.mapping, sha.data(), nullptr));
  for (size_t i = 0; i < w.chunks.size(); ++i) std::copy(sha.begin() + 32 * i, sha.begin() + 32 * i + 32, w.sha256[i].begin());
  return w;
}

// ReconstructObject followed by reconstruct's verify (multi_store.go:244-249):
// false (ErrBadHash) when the rebuilt object's SHA-256 is not `sha256`.
inline bool ReconstructObjectVerified(const std::vector<std::vector<uint8_t>>& chunks, const std::vector<int>& indices,
                                      uint32_t mapping, uint64_t size, const std::array<uint8_t, 32>& sha256,
                                      std::vector<uint8_t>* out) {
  std::vector<const uint8_t*> ptrs;
  for (const auto& c : chunks) ptrs.push_back(c.data());
  out->assign(size, 0);
  slime::detail::Call k;
  const int rc = slime_rs_reconstruct_verify_ex(k.ptr(), ptrs.empty() ? nullptr : ptrs.data(),
                                                indices.empty() ? nullptr : indices.data(), (int)chunks.size(),
                                                chunks.empty() ? 0 : chunks[0].size(), mapping, size,
                                                out->empty() ? nullptr : out->data(), sha256.data());
  if (rc == SLIME_RS_ERR_BAD_HASH) return false;
  k.check(rc);
  return true;
}

}  // namespace rs
}  // namespace slime

#endif  // SLIME_RS_HPP
