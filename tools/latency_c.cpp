// Per-call latency of the host entry points through the C-ABI alone (what the
// Go shim's cgo calls see; no Python), tools only.  8/12, erased {0,1,2,3}.
// Prints one JSON line: per object size, median / p90 microseconds of
// slime_rs_write_chunks, slime_rs_reconstruct, slime_rs_create_parity (one
// row) and slime_rs_recover_data, and whether reconstruct returned the object.
// With a second argument T: T threads each issue write_chunks / reconstruct
// on their own 4 KiB and 64 KiB objects, and the line reports calls/s (the
// concurrency of a proxy's small requests, without Python's GIL).
// Build: make tools/latency_c   Run: tools/latency_c [reps] [T]
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <functional>
#include <random>
#include <thread>
#include <vector>

#include "slime_rs.h"

namespace {

struct Stat {
  double p50, p90;
};

Stat timed(int reps, const std::function<int()>& fn) {
  if (fn()) exit(1);
  std::vector<double> t;
  for (int i = 0; i < reps; ++i) {
    const auto a = std::chrono::steady_clock::now();
    if (fn()) exit(1);
    t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count());
  }
  std::sort(t.begin(), t.end());
  return {t[t.size() / 2], t[t.size() * 9 / 10]};
}

}  // namespace

// T threads x reps calls of each kind on their own objects: calls per second.
void concurrency(int reps, int T) {
  const int need = 8, total = 12;
  const int have[8] = {4, 5, 6, 7, 8, 9, 10, 11};
  printf("{\"threads\": %d, \"reps\": %d, \"calls_per_s\": [", T, reps);
  const uint64_t sizes[] = {4096, 65536};
  for (size_t si = 0; si < 2; ++si) {
    const uint64_t S = sizes[si], cb = slime_rs_chunk_size(S, need);
    struct Obj {
      std::vector<uint8_t> data, out;
      std::vector<std::vector<uint8_t>> chunks;
      uint32_t m = 0;
    };
    std::vector<Obj> objs(T);
    std::mt19937_64 rng(si + 1);
    for (auto& o : objs) {
      o.data.resize(S);
      for (auto& b : o.data) b = (uint8_t)rng();
      o.out.resize(S);
      o.chunks.assign(total, std::vector<uint8_t>(cb));
    }
    for (int kind = 0; kind < 2; ++kind) {
      std::atomic<bool> ok{true};
      auto work = [&](int t) {
        Obj& o = objs[t];
        std::vector<uint8_t*> cp(total);
        for (int i = 0; i < total; ++i) cp[i] = o.chunks[i].data();
        std::vector<const uint8_t*> surv(need);
        for (int q = 0; q < need; ++q) surv[q] = o.chunks[have[q]].data();
        for (int r = 0; r < reps; ++r) {
          const int rc = kind == 0 ? slime_rs_write_chunks(o.data.data(), S, need, total, cp.data(), &o.m)
                                   : slime_rs_reconstruct(surv.data(), have, need, cb, o.m, S, o.out.data());
          if (rc) ok.store(false);
        }
      };
      if (kind == 0 || kind == 1)  // warm (the process's first calls load kernels); reconstruct reads these chunks
        for (int t = 0; t < T; ++t) {  // chunks and mapping from a first write
          std::vector<uint8_t*> cp(total);
          for (int i = 0; i < total; ++i) cp[i] = objs[t].chunks[i].data();
          if (slime_rs_write_chunks(objs[t].data.data(), S, need, total, cp.data(), &objs[t].m)) exit(1);
        }
      // One untimed round with all T threads first: each concurrent caller
      // gets its own workspace (streams, pinned ring) on its first call.
      double s = 0;
      for (int round = 0; round < 2; ++round) {
        const auto a = std::chrono::steady_clock::now();
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t) th.emplace_back(work, t);
        for (auto& x : th) x.join();
        s = std::chrono::duration<double>(std::chrono::steady_clock::now() - a).count();
      }
      if (kind == 1)
        for (auto& o : objs)
          if (memcmp(o.out.data(), o.data.data(), S) != 0) ok.store(false);
      printf("%s{\"object_bytes\": %llu, \"call\": \"%s\", \"per_s\": %.0f, \"ok\": %s}", si || kind ? ", " : "",
             (unsigned long long)S, kind ? "reconstruct" : "write_chunks", T * reps / s, ok.load() ? "true" : "false");
    }
  }
  printf("]}\n");
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 200;
  if (argc > 2) {
    concurrency(reps, atoi(argv[2]));
    return 0;
  }
  const int need = 8, total = 12;
  const int have[8] = {4, 5, 6, 7, 8, 9, 10, 11};  // erased {0,1,2,3}
  std::mt19937_64 rng(0x1A7);
  printf("{\"reps\": %d, \"sizes\": [", reps);
  const uint64_t sizes[] = {4096, 65536, 1 << 20, 8 << 20};
  for (size_t si = 0; si < sizeof(sizes) / sizeof(sizes[0]); ++si) {
    const uint64_t S = sizes[si];
    std::vector<uint8_t> data(S);
    for (auto& b : data) b = (uint8_t)rng();
    const uint64_t cb = slime_rs_chunk_size(S, need), L = cb / 4;
    std::vector<std::vector<uint8_t>> chunks(total, std::vector<uint8_t>(cb));
    std::vector<uint8_t*> cp(total);
    for (int i = 0; i < total; ++i) cp[i] = chunks[i].data();
    uint32_t m = 0;
    const Stat w = timed(reps, [&] { return slime_rs_write_chunks(data.data(), S, need, total, cp.data(), &m); });
    std::vector<const uint8_t*> surv(need);
    for (int q = 0; q < need; ++q) surv[q] = chunks[have[q]].data();
    std::vector<uint8_t> out(S);
    const Stat r = timed(reps, [&] { return slime_rs_reconstruct(surv.data(), have, need, cb, m, S, out.data()); });
    const bool ok = memcmp(out.data(), data.data(), S) == 0;
    // Symbol rows: the chunks' words as they stand (any uint32 is valid input).
    std::vector<const uint32_t*> rows(need);
    std::vector<uint64_t> lens(need, L);
    for (int j = 0; j < need; ++j) rows[j] = (const uint32_t*)chunks[j].data();
    std::vector<uint32_t> par(L);
    const Stat c = timed(reps, [&] { return slime_rs_create_parity(rows.data(), lens.data(), need, need, par.data()); });
    std::vector<const uint32_t*> srows(need);
    for (int q = 0; q < need; ++q) srows[q] = (const uint32_t*)chunks[have[q]].data();
    std::vector<std::vector<uint32_t>> rec(need, std::vector<uint32_t>(L));
    std::vector<uint32_t*> rp(need);
    for (int t = 0; t < need; ++t) rp[t] = rec[t].data();
    const Stat d = timed(reps, [&] { return slime_rs_recover_data(srows.data(), lens.data(), need, have, need, rp.data()); });
    printf("%s{\"object_bytes\": %llu, \"write_chunks\": [%.1f, %.1f], \"reconstruct\": [%.1f, %.1f], "
           "\"create_parity_one_row\": [%.1f, %.1f], \"recover_data\": [%.1f, %.1f], \"verified\": %s}",
           si ? ", " : "", (unsigned long long)S, w.p50, w.p90, r.p50, r.p90, c.p50, c.p90, d.p50, d.p90,
           ok ? "true" : "false");
  }
  printf("], \"unit\": \"us [p50, p90]\"}\n");
  return 0;
}
