// Proxy-level load on the host entry points, the way one slime proxy drives
// them: `threads` concurrent requests (main.go:107-109, --parallel-requests,
// default 25), each a PUT (Multi.writeChunks, multi_store.go:516-557) followed
// by a GET of the same object (Multi.reconstruct's slow path,
// multi_store.go:185-252), every call through the *_ex forms the cgo shim
// binds with device = SLIME_RS_ANY_DEVICE, so the library's device pool
// spreads the calls over every GPU it may use (SLIME_RS_DEVICES).  Built by
// `make` into tools/libproxy_load.so; bench.py's host_path.pooled leg calls
// proxy_load() through ctypes (no Python between the calls: goroutines do
// not take a GIL).
//
// pattern 0 (fused): slime_rs_write_chunks_ex + slime_rs_reconstruct_ex, the
//   data chunks that lie wholly inside the object aliasing it as the shim's
//   WriteChunks passes them (go/internal/rs/rs.go chunkBuffers: no copy).
// pattern 1 (unchanged caller, multi_store.go as it is):
//   PUT = MapToGF (:526) + splitVector (:527, in place) + r x CreateParity
//         (:528-531) + a MapFromGF per chunk (:554);
//   GET = MapToGFWith per survivor (:224) + RecoverData (:237) + MapFromGF
//         per data row into one buffer truncated to Size (:238-241).
// Within a request the calls run one after another (the reference runs the
// per-chunk MapFromGF calls on goroutines; here 25 requests already keep the
// codec pool and the GPUs busy).  Buffers are allocated once per thread and
// reused (Go's heap recycles its spans; fresh-page faults are measured by
// bench.py's unchanged_caller leg).
//
// Verified: every thread's first and last GET returns its object's bytes,
// its chunks after the last PUT hash the same as after the first, and (pattern
// 1) equal the fused path's chunks for that object.
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <memory>
#include <thread>
#include <vector>

#include "crash_report.hpp"
#include "slime_rs.h"

namespace {

using Clock = std::chrono::steady_clock;

uint64_t hash_bytes(const uint8_t* p, size_t n) {  // FNV-1a over 8-byte words (a fingerprint, not a digest)
  uint64_t h = 1469598103934665603ull;
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t w;
    memcpy(&w, p + i, 8);
    h = (h ^ w) * 1099511628211ull;
  }
  for (; i < n; ++i) h = (h ^ p[i]) * 1099511628211ull;
  return h;
}

void fill_random(uint8_t* p, size_t n, uint64_t seed) {  // splitmix64 stream
  uint64_t x = seed;
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t z = (x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    memcpy(p + i, &z, 8);
  }
  for (; i < n; ++i) p[i] = (uint8_t)(x >> (8 * (i & 7)));
}

struct Request {
  int need, total;
  std::vector<int> have;
  uint64_t S, cb, L;
  std::vector<uint8_t> data, out;
  std::vector<std::vector<uint8_t>> chunks;
  std::vector<uint8_t*> cptr;
  std::vector<const uint8_t*> surv;
  // unchanged caller's symbol buffers
  std::vector<uint32_t> words;
  std::vector<std::vector<uint32_t>> par, sym, rec;
  std::vector<const uint32_t*> parts, symp;
  std::vector<uint32_t*> recp;
  std::vector<uint64_t> lens;
  uint32_t mapping = 0;
  uint64_t calls = 0;
  std::vector<double> put_ms, get_ms;

  Request(int need_, int total_, const int* have_, uint64_t S_, uint64_t seed, int pattern)
      : need(need_), total(total_), have(have_, have_ + need_), S(S_) {
    cb = slime_rs_chunk_size(S, need);
    L = cb / 4;
    data.resize(S);
    fill_random(data.data(), S, seed);
    out.assign((size_t)need * cb + 16, 0);
    chunks.assign(total, std::vector<uint8_t>(cb));
    // The shim's WriteChunks (go/internal/rs/rs.go, chunkBuffers): a data
    // chunk that lies wholly inside the object is a subslice of it, so the
    // library never copies it; the unchanged caller's chunks are MapFromGF's
    // fresh outputs.
    for (int i = 0; i < total; ++i)
      cptr.push_back(pattern == 0 && i < need && (uint64_t)(i + 1) * cb <= S ? data.data() + (uint64_t)i * cb
                                                                             : chunks[i].data());
    for (int q = 0; q < need; ++q) surv.push_back(cptr[have[q]]);
    if (pattern == 1) {
      words.assign((size_t)need * L, 0u);  // splitVector's zero padding stays zero
      for (int j = 0; j < need; ++j) parts.push_back(words.data() + (size_t)j * L);
      par.assign(total - need, std::vector<uint32_t>(L));
      sym.assign(need, std::vector<uint32_t>(L));
      rec.assign(need, std::vector<uint32_t>(L));
      for (auto& s : sym) symp.push_back(s.data());
      for (auto& r : rec) recp.push_back(r.data());
      lens.assign(need, L);
    }
  }

  int put(const slime_rs_call_t* c, int pattern) {
    if (pattern == 0) {
      ++calls;
      return slime_rs_write_chunks_ex(c, data.data(), S, need, total, cptr.data(), &mapping);
    }
    if (int rc = slime_gf_map_to_gf_ex(c, data.data(), S, &mapping, words.data())) return rc;
    for (int i = 0; i < total - need; ++i)
      if (int rc = slime_rs_create_parity_ex(c, parts.data(), lens.data(), need, need + i, par[i].data())) return rc;
    for (int i = 0; i < total; ++i) {
      const uint32_t* row = i < need ? parts[i] : par[i - need].data();
      if (int rc = slime_gf_map_from_gf_ex(c, mapping, row, L, cptr[i])) return rc;
    }
    calls += 1 + (total - need) + total;
    return 0;
  }

  int get(const slime_rs_call_t* c, int pattern) {
    if (pattern == 0) {
      ++calls;
      return slime_rs_reconstruct_ex(c, surv.data(), have.data(), need, cb, mapping, S, out.data());
    }
    for (int q = 0; q < need; ++q)
      if (int rc = slime_gf_map_to_gf_with_ex(c, surv[q], cb, mapping, sym[q].data())) return rc;
    if (int rc = slime_rs_recover_data_ex(c, symp.data(), lens.data(), need, have.data(), need, recp.data()))
      return rc;
    for (int t = 0; t < need; ++t)
      if (int rc = slime_gf_map_from_gf_ex(c, mapping, recp[t], L, out.data() + (size_t)t * cb)) return rc;
    calls += need + 1 + need;
    return 0;
  }

  uint64_t chunk_hash() const {
    uint64_t h = 0;
    for (uint8_t* c : cptr) h = h * 31 + hash_bytes(c, cb);
    return h;
  }
  bool got_object() const { return memcmp(out.data(), data.data(), S) == 0; }
};

double pct(std::vector<double> v, double q) {
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  return v[std::min(v.size() - 1, (size_t)(q * (v.size() - 1) + 0.5))];
}

}  // namespace

// out[0] requests (PUT + GET pairs) completed   out[1] wall seconds of the timed loop
// out[2] verified (1/0)                        out[3] C-ABI calls made in the timed loop
// out[4..5] PUT p50 / p99 ms                   out[6..7] GET p50 / p99 ms
// out[8] failed calls                          out[9] setup + warm-up seconds
// Returns 0, or the first nonzero status a call returned.
extern "C" int proxy_load(int threads, uint64_t object_bytes, int need, int total, const int* have, int pattern,
                          double seconds, uint64_t seed, double* out) {
  if (threads < 1 || need < 1 || total < need || !have || !out || (pattern != 0 && pattern != 1)) return 9;
  // A fault in any thread prints a resolved report first (crash_report.hpp;
  // PROXY_LOAD_CRASH_REPORT=0 turns it off).
  const char* cr = getenv("PROXY_LOAD_CRASH_REPORT");
  const bool report = !cr || atoi(cr) != 0;
  if (report) crash_report::install();
  struct Uninstall {
    bool on;
    ~Uninstall() {
      if (on) crash_report::uninstall();
    }
  } uninstall_at_exit{report};
  const auto t_setup = Clock::now();
  std::vector<std::unique_ptr<Request>> reqs(threads);
  {
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t)
      th.emplace_back([&, t] { reqs[t].reset(new Request(need, total, have, object_bytes, seed + 7919 * t, pattern)); });
    for (auto& x : th) x.join();
  }
  slime_rs_call_t call{SLIME_RS_ANY_DEVICE, nullptr, 0};
  std::atomic<int> first_rc{0};
  std::atomic<uint64_t> failed{0};
  auto note = [&](int rc) {
    if (rc) {
      failed.fetch_add(1);
      int z = 0;
      first_rc.compare_exchange_strong(z, rc);
    }
  };
  // Warm-up, all threads at once: each concurrent caller gets its workspace on
  // every device it lands on; also the reference chunks of each object.
  std::vector<uint64_t> h0(threads);
  std::vector<uint8_t> ok(threads, 1);
  {
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t)
      th.emplace_back([&, t] {
        Request& r = *reqs[t];
        for (int i = 0; i < 2; ++i) {
          note(r.put(&call, pattern));
          note(r.get(&call, pattern));
        }
        h0[t] = r.chunk_hash();
        if (pattern == 1) {  // the unchanged caller's chunks equal the fused entry point's
          std::vector<std::vector<uint8_t>> keep = r.chunks;
          note(slime_rs_write_chunks_ex(&call, r.data.data(), r.S, need, total, r.cptr.data(), &r.mapping));
          if (r.chunk_hash() != h0[t]) ok[t] = 0;
          r.chunks = keep;
        }
        ok[t] &= r.got_object();
        std::fill(r.out.begin(), r.out.end(), 0);
        r.calls = 0;
      });
    for (auto& x : th) x.join();
  }
  const double warm_s = std::chrono::duration<double>(Clock::now() - t_setup).count();
  std::atomic<int> ready{0};
  std::atomic<bool> go{false};
  Clock::time_point start, deadline;
  std::vector<Clock::time_point> done(threads);
  std::vector<uint64_t> nreq(threads, 0);
  {
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t)
      th.emplace_back([&, t] {
        Request& r = *reqs[t];
        ready.fetch_add(1);
        while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
        bool first = true;
        for (;;) {
          const auto a = Clock::now();
          note(r.put(&call, pattern));
          const auto b = Clock::now();
          note(r.get(&call, pattern));
          const auto c = Clock::now();
          r.put_ms.push_back(std::chrono::duration<double, std::milli>(b - a).count());
          r.get_ms.push_back(std::chrono::duration<double, std::milli>(c - b).count());
          if (first) {
            ok[t] &= r.got_object();
            first = false;
          }
          ++nreq[t];
          if (c >= deadline) break;
        }
        done[t] = Clock::now();
        ok[t] &= r.got_object() && r.chunk_hash() == h0[t];
      });
    while (ready.load() < threads) std::this_thread::yield();
    start = Clock::now();
    deadline = start + std::chrono::duration_cast<Clock::duration>(std::chrono::duration<double>(seconds));
    go.store(true, std::memory_order_release);
    for (auto& x : th) x.join();
  }
  const auto end = *std::max_element(done.begin(), done.end());
  std::vector<double> put, get;
  uint64_t calls = 0, n = 0;
  for (int t = 0; t < threads; ++t) {
    put.insert(put.end(), reqs[t]->put_ms.begin(), reqs[t]->put_ms.end());
    get.insert(get.end(), reqs[t]->get_ms.begin(), reqs[t]->get_ms.end());
    calls += reqs[t]->calls;
    n += nreq[t];
  }
  out[0] = (double)n;
  out[1] = std::chrono::duration<double>(end - start).count();
  out[2] = failed.load() == 0 && std::all_of(ok.begin(), ok.end(), [](uint8_t v) { return v != 0; }) ? 1.0 : 0.0;
  out[3] = (double)calls;
  out[4] = pct(put, 0.5);
  out[5] = pct(put, 0.99);
  out[6] = pct(get, 0.5);
  out[7] = pct(get, 0.99);
  out[8] = (double)failed.load();
  out[9] = warm_s;
  return first_rc.load();
}

// Test hook of the crash report (tests/test_host.py): installs it, then
// writes past the end of a mapping into a PROT_NONE page as a runaway memcpy
// would.  The process then dies of SIGSEGV after the report.
extern "C" void proxy_load_fault_selftest(void) {
  crash_report::install();
  const long pg = sysconf(_SC_PAGESIZE);
  uint8_t* p = (uint8_t*)mmap(nullptr, 2 * pg, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (p == MAP_FAILED) return;
  mprotect(p + pg, pg, PROT_NONE);
  static uint8_t src[1 << 16];
  volatile size_t n = 2 * (size_t)pg;
  memcpy(p, src, n);
}
