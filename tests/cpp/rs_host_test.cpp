// C++ parity tests for the host mirror of internal/rs and internal/rs/gf
// (include/slime_rs.hpp) -- the reference's own test suite restated against
// the C++ API, with the reference's known answers read from the committed
// fixtures (tests/golden/reference_kats.json, vectors.json):
//   internal/rs/matrix_test.go:8-55     Vandermonde KATs
//   internal/rs/matrix_test.go:57-115   ParityMatrix KATs
//   internal/rs/matrix_test.go:117-168  every d-row subset of ParityMatrix(d,p) invertible
//   internal/rs/vector_test.go:24-63    CreateParity KAT
//   internal/rs/vector_test.go:65-113   random encode / erase / RecoverData round trips
//   internal/rs/gf/gf_test.go:8-26      MInverse(v)*v == 1, MInverse == Raise(v, p-2)
//   internal/rs/gf/map_test.go:9-105    MapToGF byte packing, mapping and tricky cases
// Usage: rs_host_test <golden dir> [cpu|gpu|all]
//   cpu: host-only tests (matrices, scalars, validation panics) -- no device
//   gpu: data-path tests through the HIP kernels (needs an MI355X)
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <map>
#include <random>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "slime_rs.hpp"

using slime::rs::Matrix;
using slime::rs::Vector;
namespace gf = slime::gf;
namespace rs = slime::rs;

// ---------------------------------------------------------------- tiny JSON
struct Json {
  enum Kind { Null, Num, Str, Arr, Obj } kind = Null;
  double num = 0;
  std::string str;
  std::vector<Json> arr;
  std::map<std::string, Json> obj;
  const Json& operator[](const std::string& k) const { return obj.at(k); }
  uint64_t u() const { return (uint64_t)num; }
  Vector vec() const {
    Vector v;
    for (const Json& x : arr) v.push_back((uint32_t)x.u());
    return v;
  }
  Matrix mat() const {
    Matrix m;
    for (const Json& r : arr) m.push_back(r.vec());
    return m;
  }
  std::vector<uint8_t> bytes() const {
    std::vector<uint8_t> b;
    for (const Json& x : arr) b.push_back((uint8_t)x.u());
    return b;
  }
  std::vector<int> ints() const {
    std::vector<int> v;
    for (const Json& x : arr) v.push_back((int)x.u());
    return v;
  }
};

// Objects, arrays, strings, numbers: what the fixtures hold.
struct JsonParser {
  const std::string& s;
  size_t i = 0;
  explicit JsonParser(const std::string& text) : s(text) {}
  void ws() {
    while (i < s.size() && (s[i] == ' ' || s[i] == '\n' || s[i] == '\r' || s[i] == '\t')) ++i;
  }
  Json value() {
    ws();
    Json j;
    if (s[i] == '{') {
      j.kind = Json::Obj;
      ++i;
      ws();
      if (s[i] == '}') return ++i, j;
      for (;;) {
        std::string k = value().str;
        ws();
        ++i;  // ':'
        j.obj[k] = value();
        ws();
        if (s[i++] == '}') return j;
      }
    }
    if (s[i] == '[') {
      j.kind = Json::Arr;
      ++i;
      ws();
      if (s[i] == ']') return ++i, j;
      for (;;) {
        j.arr.push_back(value());
        ws();
        if (s[i++] == ']') return j;
      }
    }
    if (s[i] == '"') {
      j.kind = Json::Str;
      ++i;
      while (s[i] != '"') {
        if (s[i] == '\\') ++i;
        j.str += s[i++];
      }
      ++i;
      return j;
    }
    if (s.compare(i, 4, "null") == 0) return i += 4, j;
    size_t end = i;
    while (end < s.size() && std::string("+-0123456789.eE").find(s[end]) != std::string::npos) ++end;
    j.kind = Json::Num;
    j.num = std::stod(s.substr(i, end - i));
    i = end;
    return j;
  }
};

Json load_json(const std::string& path) {
  std::ifstream f(path);
  if (!f) throw std::runtime_error("cannot open " + path);
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string text = ss.str();
  JsonParser p(text);
  return p.value();
}

// ---------------------------------------------------------------- harness
struct Failure : std::runtime_error {
  using std::runtime_error::runtime_error;
};
#define EXPECT(cond)                                                                               \
  do {                                                                                             \
    if (!(cond)) throw Failure(std::string(__FILE__ ":") + std::to_string(__LINE__) + ": " #cond); \
  } while (0)

template <class F>
std::string panic_text(F&& f) {
  try {
    f();
  } catch (const slime::Panic& p) {
    return p.what();
  }
  return "<no panic>";
}

struct Test {
  const char* name;
  bool gpu;
  void (*fn)();
};
std::vector<Test>& registry() {
  static std::vector<Test> t;
  return t;
}
struct Reg {
  Reg(const char* n, bool g, void (*f)()) { registry().push_back({n, g, f}); }
};
#define TEST_CPU(name)                       \
  void name();                               \
  static Reg reg_##name(#name, false, name); \
  void name()
#define TEST_GPU(name)                      \
  void name();                              \
  static Reg reg_##name(#name, true, name); \
  void name()

std::string g_golden;
const Json& kats() {
  static const Json j = load_json(g_golden + "/reference_kats.json");
  return j;
}
const Json& vectors() {
  static const Json j = load_json(g_golden + "/vectors.json");
  return j;
}

constexpr uint64_t P = gf::MaxVal;

// ---------------------------------------------------------------- host-only
TEST_CPU(TestVandermonde) {  // matrix_test.go:8-55
  for (const Json& c : kats()["vandermonde"].arr)
    EXPECT(rs::vandermondeMatrix((int)c["d"].u(), (int)c["p"].u()) == c["m"].mat());
}

TEST_CPU(TestParityMatrix) {  // matrix_test.go:57-115
  for (const Json& c : kats()["parity_matrix"].arr) {
    const int d = (int)c["d"].u(), p = (int)c["p"].u();
    const Matrix want = c["m"].mat();
    const Matrix got = rs::ParityMatrix(d, p);
    // Fixtures hold either the whole matrix or its bottom rows.
    EXPECT(got.size() >= want.size());
    EXPECT(Matrix(got.end() - (long)want.size(), got.end()) == want);
    EXPECT(rs::ParityMatrixCached(d, p) == got);
    EXPECT(&rs::ParityMatrixCached(d, p) == &rs::ParityMatrixCached(d, p));  // shared
  }
  for (const Json& c : vectors()["parity_matrices"].arr) {
    const int need = (int)c["need"].u(), total = (int)c["total"].u();
    EXPECT(rs::ParityMatrix(need, total - need) == c["m"].mat());
  }
}

TEST_CPU(TestParityMatrixInvertible) {  // matrix_test.go:117-168
  for (int d = 1; d <= 6; ++d)
    for (int p = 0; p <= 6; ++p) {
      const Matrix m = rs::ParityMatrix(d, p);
      std::vector<int> pick(d);
      for (int i = 0; i < d; ++i) pick[i] = i;
      for (;;) {
        Matrix have;
        for (int r : pick) have.push_back(m[r]);
        const Matrix inv = rs::invertMatrix(have);
        for (int i = 0; i < d; ++i)  // inv * have == I, exactly
          for (int j = 0; j < d; ++j) {
            uint64_t acc = 0;
            for (int t = 0; t < d; ++t) acc = (acc + (uint64_t)inv[i][t] * have[t][j] % P) % P;
            EXPECT(acc == (i == j ? 1u : 0u));
          }
        int i = d - 1;  // next d-subset of [0, d+p) in lexicographic order
        while (i >= 0 && pick[i] == p + i) --i;
        if (i < 0) break;
        ++pick[i];
        for (int k = i + 1; k < d; ++k) pick[k] = pick[k - 1] + 1;
      }
    }
}

TEST_CPU(TestInverses) {  // golden inverses (vectors.json)
  for (const Json& c : vectors()["inverses"].arr) {
    const int need = (int)c["need"].u(), total = (int)c["total"].u();
    const Matrix m = rs::ParityMatrix(need, total - need);
    Matrix have;
    for (int r : c["have"].ints()) have.push_back(m[r]);
    EXPECT(rs::invertMatrix(have) == c["inv"].mat());
  }
}

TEST_CPU(TestSolveSubIdentityAndClone) {
  Matrix m = rs::vandermondeMatrix(4, 3);
  const Matrix c = rs::cloneMatrix(m);
  rs::solveSubIdentity(m);
  EXPECT(m == rs::ParityMatrix(4, 3));
  EXPECT(c == rs::vandermondeMatrix(4, 3));  // the clone is independent
}

TEST_CPU(TestSingularPanics) {  // matrix.go:68, reached through duplicate rows
  const Matrix m = rs::ParityMatrix(3, 2);
  EXPECT(panic_text([&] { rs::invertMatrix({m[0], m[0], m[1]}); }) == "Couldn't ensure nonzero m[i][i]");
}

TEST_CPU(TestMInverse) {  // gf_test.go:8-26
  std::mt19937_64 rng(1);
  for (int n = 0; n < 1000; ++n) {
    uint32_t v = 0;
    while (v == 0 || v >= gf::MaxVal) v = (uint32_t)rng();
    const uint32_t inv = gf::MInverse(v);
    EXPECT((uint64_t)v * inv % P == 1);
    EXPECT(inv == gf::Raise(v, gf::MaxVal - 2));
  }
  EXPECT(gf::Raise(0, 0) == 1);
}

TEST_CPU(TestValidationPanics) {  // vector.go:19-23, :51-57 -- reached before any device work
  EXPECT(panic_text([] { rs::CreateParity({{1, 2, 3}, {1, 2}}, 2); }) ==
         "CreateParity called on data chunks of varying length");
  EXPECT(panic_text([] { rs::RecoverData({{1, 2}}, {0, 1}); }) == "RecoverData: len(chunks) != len(indices)");
  EXPECT(panic_text([] { rs::RecoverData({}, {}); }) == "RecoverData: len(chunks) == 0");
}

// The cgo contract: each *_ex call returns its own
// failure detail, whatever other threads fail with meanwhile, so a goroutine
// that changes OS threads between calls still panics with its own text
// (vector.go:18-88's panics, concurrent callers as at main.go:107-109).
TEST_CPU(TestCallDetailPerCall) {
  std::atomic<int> bad{0};
  std::vector<std::thread> ts;
  ts.emplace_back([&] {  // CreateParity index -k: Go's index-out-of-range text (code 8)
    const uint32_t x[2] = {1, 2};
    const uint32_t* d[2] = {x, x};
    const uint64_t lens[2] = {2, 2};
    for (int it = 0; it < 3000; ++it) {
      char buf[256];
      slime_rs_call_t c{SLIME_RS_ANY_DEVICE, buf, sizeof(buf)};
      const int index = -(1 + it % 7);
      const int rc = slime_rs_create_parity_ex(&c, d, lens, 2, index, nullptr);
      if (rc != SLIME_RS_ERR_INDEX_RANGE ||
          std::string(buf) != "runtime error: index out of range [" + std::to_string(index) + "]")
        ++bad;
    }
  });
  ts.emplace_back([&] {  // RecoverData with a short chunk: a different code-8 text per call
    const uint32_t x[3] = {1, 2, 3};
    const uint32_t* d[2] = {x, x};
    const int idx[2] = {0, 1};
    for (int it = 0; it < 3000; ++it) {
      char buf[256];
      slime_rs_call_t c{SLIME_RS_ANY_DEVICE, buf, sizeof(buf)};
      const uint64_t short_len = (uint64_t)(it % 3);
      const uint64_t lens[2] = {3, short_len};
      const int rc = slime_rs_recover_data_ex(&c, d, lens, 2, idx, 2, nullptr);
      const std::string want = "runtime error: index out of range [" + std::to_string(short_len) + "] with length " +
                               std::to_string(short_len);
      if (rc != SLIME_RS_ERR_INDEX_RANGE || std::string(buf) != want) ++bad;
    }
  });
  ts.emplace_back([&] {  // varying lengths: code 1, its own detail
    const uint32_t x[3] = {1, 2, 3};
    const uint32_t* d[2] = {x, x};
    const uint64_t lens[2] = {3, 2};
    for (int it = 0; it < 3000; ++it) {
      char buf[256];
      slime_rs_call_t c{SLIME_RS_ANY_DEVICE, buf, sizeof(buf)};
      const int rc = slime_rs_create_parity_ex(&c, d, lens, 2, 2, nullptr);
      if (rc != SLIME_RS_ERR_VARYING_LENGTH || std::string(buf).find("varying length") == std::string::npos) ++bad;
    }
  });
  ts.emplace_back([&] {  // successes report an empty detail
    std::vector<uint32_t> m(12 * 8);
    for (int it = 0; it < 3000; ++it) {
      char buf[256] = "stale";
      slime_rs_call_t c{SLIME_RS_ANY_DEVICE, buf, sizeof(buf)};
      if (slime_rs_parity_matrix_ex(&c, 8, 4, m.data()) != SLIME_RS_OK || buf[0] != 0) ++bad;
    }
  });
  for (auto& t : ts) t.join();
  EXPECT(bad.load() == 0);
  // A detail longer than the caller's buffer is truncated, still NUL-terminated.
  char tiny[8];
  slime_rs_call_t c{SLIME_RS_ANY_DEVICE, tiny, sizeof(tiny)};
  const uint32_t x[1] = {1};
  const uint32_t* d[1] = {x};
  const uint64_t lens[1] = {1};
  EXPECT(slime_rs_create_parity_ex(&c, d, lens, 1, -5, nullptr) == SLIME_RS_ERR_INDEX_RANGE);
  EXPECT(std::string(tiny) == "runtime");
  // A bad context is refused before anything runs.
  slime_rs_call_t neg{-7, tiny, sizeof(tiny)};
  EXPECT(slime_rs_parity_matrix_ex(&neg, 4, 2, nullptr) == SLIME_RS_ERR_INVALID_ARG);
}

// checkConfig admits need == total (multi_config.go:36; the reference's own
// multi-store tests run 1-of-1, multi_test.go:179,257): writeChunks must not
// reject it.  total < need is a caller error.
TEST_CPU(TestWriteChunksConfigChecks) {
  const std::vector<uint8_t> obj(1000, 7);
  std::vector<std::vector<uint8_t>> chunks(3, std::vector<uint8_t>(slime_rs_chunk_size(obj.size(), 3)));
  std::vector<uint8_t*> ptrs;
  for (auto& ch : chunks) ptrs.push_back(ch.data());
  uint32_t m = 0;
  char buf[256];
  slime_rs_call_t c{SLIME_RS_ANY_DEVICE, buf, sizeof(buf)};
  const int rc = slime_rs_write_chunks_ex(&c, obj.data(), obj.size(), 3, 3, ptrs.data(), &m);
  EXPECT(rc == SLIME_RS_OK || rc == SLIME_RS_ERR_NO_DEVICE);  // never INVALID_ARG
  EXPECT(slime_rs_write_chunks_ex(&c, obj.data(), obj.size(), 3, 2, ptrs.data(), &m) == SLIME_RS_ERR_INVALID_ARG);
}

// ---------------------------------------------------------------- data path
TEST_GPU(TestWriteChunksNoParity) {  // need == total: chunks are MapFromGF(m, splitVector parts)
  std::mt19937_64 rng(11);
  for (int need : {1, 3}) {
    for (size_t size : {(size_t)1, (size_t)5, (size_t)4099, (size_t)100003}) {
      for (int force_high : {0, 1}) {
        std::vector<uint8_t> obj(size);
        for (uint8_t& b : obj) b = (uint8_t)rng();
        if (force_high && size >= 4) obj[0] = obj[1] = obj[2] = obj[3] = 0xFF;  // a word >= p: mapping != 0
        const auto [m, chunks] = rs::WriteChunks(obj, need, need);
        const auto [m_ref, words] = gf::MapToGF(obj);
        EXPECT(m == m_ref);
        EXPECT(force_high == 0 || size < 4 || m != 0);
        const size_t L = chunks[0].size() / 4;
        Matrix parts((size_t)need, Vector(L, 0));
        for (size_t w = 0; w < words.size(); ++w) parts[w / L][w % L] = words[w];
        for (int i = 0; i < need; ++i) EXPECT(gf::MapFromGF(m, parts[i]) == chunks[i]);
      }
    }
  }
}

TEST_GPU(TestDevicePool) {  // calls without a pinned device go through the pool (one GPU here)
  const int n = slime_rs_device_count();
  EXPECT(n >= 1);
  std::vector<uint64_t> before(n);
  for (int d = 0; d < n; ++d) EXPECT(slime_rs_pool_calls(d, &before[d], nullptr) == SLIME_RS_OK);
  for (int i = 0; i < 10; ++i) EXPECT(rs::CreateParity({{0, 0, 0}, {1, 2, 3}}, 2) == Vector({3, 6, 9}));
  uint64_t routed = 0;
  for (int d = 0; d < n; ++d) {
    uint64_t now = 0;
    int inflight = -1;
    EXPECT(slime_rs_pool_calls(d, &now, &inflight) == SLIME_RS_OK);
    EXPECT(inflight == 0);
    routed += now - before[d];
  }
  EXPECT(routed == 10);
}

// Chunk digests computed beside the device pipeline equal the digests of the
// finished chunks, for the three mapping outcomes (0, 1<<31: parity chunks
// rewritten after the speculative pass, random fallback); the verified
// reconstruct accepts the object's own SHA-256 and rejects any other.
TEST_GPU(TestWriteChunksDigest) {
  std::mt19937_64 rng(29);
  for (size_t size : {(size_t)5, (size_t)100003, (size_t)(3u << 20) + 11}) {
    for (int kind : {0, 1, 2}) {
      if (kind == 2 && size < 8) continue;
      std::vector<uint8_t> obj(size);
      for (uint8_t& b : obj) b = (uint8_t)rng();
      if (kind == 1) obj[0] = obj[1] = obj[2] = obj[3] = 0xFF;
      if (kind == 2) {
        const uint8_t tricky[8] = {0xFF, 0xFF, 0xFF, 0xFF, 0x7F, 0xFF, 0xFF, 0xFF};
        std::copy(tricky, tricky + 8, obj.begin());
      }
      const rs::WrittenChunks w = rs::WriteChunksDigest(obj, 4, 7);
      EXPECT(kind != 1 || w.mapping == 1u << 31);
      EXPECT(kind != 2 || (w.mapping != 0 && w.mapping != 1u << 31));
      const auto [m, chunks] = rs::WriteChunks(obj, 4, 7);
      EXPECT(kind == 2 || m == w.mapping);  // the fallback draw is random per call
      std::vector<const uint8_t*> ptrs;
      std::vector<uint64_t> lens;
      for (const auto& c : w.chunks) ptrs.push_back(c.data()), lens.push_back(c.size());
      std::vector<uint8_t> sha(32 * w.chunks.size());
      EXPECT(slime_rs_chunk_digests(ptrs.data(), lens.data(), (uint32_t)ptrs.size(), sha.data(), nullptr) == 0);
      for (size_t i = 0; i < w.chunks.size(); ++i)
        EXPECT(std::equal(w.sha256[i].begin(), w.sha256[i].end(), sha.begin() + 32 * i));
      std::array<uint8_t, 32> want;
      EXPECT(slime_rs_sha256(obj.data(), obj.size(), want.data()) == 0);
      const std::vector<int> have = {1, 3, 4, 6};
      std::vector<std::vector<uint8_t>> surv;
      for (int i : have) surv.push_back(w.chunks[i]);
      std::vector<uint8_t> out;
      EXPECT(rs::ReconstructObjectVerified(surv, have, w.mapping, size, want, &out) && out == obj);
      want[7] ^= 1;
      EXPECT(!rs::ReconstructObjectVerified(surv, have, w.mapping, size, want, &out));
    }
  }
}

TEST_GPU(TestCreateParity) {  // vector_test.go:24-63
  for (const Json& c : kats()["create_parity"].arr)
    EXPECT(rs::CreateParity(c["data"].mat(), (int)c["index"].u()) == c["out"].vec());
  // Like Go, `out` is reused when its capacity holds the row.
  Vector buf;
  buf.reserve(64);
  const uint32_t* before = buf.data();
  const Vector got = rs::CreateParity({{0, 0, 0}, {1, 2, 3}}, 2, std::move(buf));
  EXPECT(got == Vector({3, 6, 9}) && got.data() == before);
}

TEST_GPU(TestGoldenEncodeDecode) {
  for (const Json& c : vectors()["encode"].arr) {
    const Matrix data = c["data"].mat(), parity = c["parity"].mat();
    const int need = (int)c["need"].u(), total = (int)c["total"].u();
    for (int i = 0; i < total - need; ++i) EXPECT(rs::CreateParity(data, need + i) == parity[i]);
    EXPECT(rs::CreateParities(data, total) == parity);
  }
  for (const Json& c : vectors()["decode"].arr)
    EXPECT(rs::RecoverData(c["chunks"].mat(), c["have"].ints()) == c["data"].mat());
}

TEST_GPU(TestRecovery) {  // vector_test.go:65-113
  std::mt19937_64 rng(65);
  for (int round = 0; round < 12; ++round)
    for (int L = 1; L < 10; ++L) {
      const int nd = 1 + (int)(rng() % 19), npar = (int)(rng() % 20);
      Matrix data((size_t)nd, Vector((size_t)L));
      for (Vector& r : data)
        for (uint32_t& x : r) x = (uint32_t)(rng() % P);
      Matrix code = data;
      for (int j = 0; j < npar; ++j) code.push_back(rs::CreateParity(data, nd + j));
      std::vector<int> all(nd + npar);
      for (int i = 0; i < nd + npar; ++i) all[i] = i;
      std::shuffle(all.begin(), all.end(), rng);
      const std::vector<int> have(all.begin(), all.begin() + nd);
      Matrix chunks;
      for (int i : have) chunks.push_back(code[i]);
      EXPECT(rs::RecoverData(chunks, have) == data);
    }
}

TEST_GPU(TestMapTrivial) {  // map_test.go:9-76
  for (const Json& c : kats()["map_trivial"].arr) {
    const std::vector<uint8_t> in = c["in"].bytes();
    const auto [n, v] = gf::MapToGF(in);
    EXPECT(n == (uint32_t)c["n"].u() && v == c["v"].vec());
    std::vector<uint8_t> back = gf::MapFromGF(n, v);
    back.resize(in.size());
    EXPECT(back == in);
    EXPECT(gf::MapToGFWith(in, n) == v);
  }
}

TEST_GPU(TestMapTricky) {  // map_test.go:78-105 (the last case needs the random fallback)
  slime_gf_seed(99);
  for (const Json& c : kats()["map_tricky"].arr) {
    const std::vector<uint8_t> in = c.bytes();
    const auto [n, v] = gf::MapToGF(in);
    for (uint32_t w : v) EXPECT(w < gf::MaxVal);
    std::vector<uint8_t> back = gf::MapFromGF(n, v);
    back.resize(in.size());
    EXPECT(back == in);
  }
}

TEST_GPU(TestWriteChunksRoundTrip) {  // fused object entry points vs the [][]uint32 API
  std::mt19937_64 rng(7);
  for (int need : {2, 4, 8, 10, 20}) {
    const int total = need + 4;
    std::vector<uint8_t> obj(100003);
    for (uint8_t& b : obj) b = (uint8_t)rng();
    const auto [m, chunks] = rs::WriteChunks(obj, need, total);
    // The reference's framing: MapToGF, splitVector, CreateParity, MapFromGF.
    const auto [m_ref, words] = gf::MapToGF(obj);
    EXPECT(m == m_ref);
    const size_t L = chunks[0].size() / 4;
    Matrix parts((size_t)need, Vector(L, 0));
    for (size_t w = 0; w < words.size(); ++w) parts[w / L][w % L] = words[w];
    for (int i = 0; i < total; ++i) {
      const Vector row = i < need ? parts[i] : rs::CreateParity(parts, i);
      EXPECT(gf::MapFromGF(m, row) == chunks[i]);
    }
    std::vector<int> have;
    std::vector<std::vector<uint8_t>> surv;
    for (int i = total - need; i < total; ++i) have.push_back(i), surv.push_back(chunks[i]);
    EXPECT(rs::ReconstructObject(surv, have, m, obj.size()) == obj);
  }
}

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s <golden dir> [cpu|gpu|all]\n", argv[0]);
    return 2;
  }
  g_golden = argv[1];
  const std::string which = argc > 2 ? argv[2] : "all";
  int failed = 0, ran = 0;
  for (const Test& t : registry()) {
    if ((which == "cpu" && t.gpu) || (which == "gpu" && !t.gpu)) continue;
    ++ran;
    try {
      t.fn();
      std::printf("ok   %s\n", t.name);
    } catch (const std::exception& e) {
      ++failed;
      std::printf("FAIL %s: %s\n", t.name, e.what());
    }
  }
  std::printf("%d/%d passed\n", ran - failed, ran);
  return failed ? 1 : 0;
}
