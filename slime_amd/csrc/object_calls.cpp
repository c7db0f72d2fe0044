// Whole-object entry points over host memory (include/slime_rs.h, "Object
// entry points"): Multi.writeChunks' data path (MapToGF -> splitVector ->
// CreateParity x r -> MapFromGF per chunk, multi_store.go:526-557) and
// Multi.reconstruct's slow path (MapToGFWith -> RecoverData -> MapFromGF,
// multi_store.go:215-241), each one fused device pass through the pinned
// windowed pipeline (host_pipeline.hpp), plus their digest forms.
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "capi_internal.hpp"
#include "digest.hpp"
#include "host_pipeline.hpp"

namespace slime {
namespace {

int make_encode_plan(const PlanKey& key, slime_rs_plan** out) {
  return slime_rs_plan_encode(std::get<0>(key), std::get<2>(key), std::get<3>(key), out);
}

int make_object_recover_plan(const PlanKey& key, slime_rs_plan** out) {
  // kind 'O': all need data rows of the inverse (the object is rebuilt whole
  // on the device), inputs = staged survivors 0..need-1, outputs = chunk
  // positions need..2need-1 (the rebuilt object, in order).
  const int need = std::get<2>(key);
  std::vector<int> want(need);
  for (int t = 0; t < need; ++t) want[t] = t;
  if (int rc = make_inverse_rows_plan(std::get<0>(key), need, std::get<4>(key), want, out)) return rc;
  std::vector<int> pos(need);
  for (int t = 0; t < need; ++t) pos[t] = need + t;
  if (int rc = slime_rs_plan_set_outputs(*out, pos.data())) {
    destroy_plan(*out);
    *out = nullptr;
    return rc;
  }
  return 0;
}

// Data chunk j's bytes past the object (its tail): zero low bytes of the
// object's partial last word, then splitVector's zero symbols serialised under
// mapping m as BE(m) (map.go:28-33,103-113; multi_store.go:279-296).  They
// depend only on m and the object's length, so the host writes them.
void write_data_tails(uint64_t size, int need, uint64_t chunk, uint8_t* const* chunks, uint32_t m) {
  const uint8_t pad[4] = {(uint8_t)(m >> 24), (uint8_t)(m >> 16), (uint8_t)(m >> 8), (uint8_t)m};
  const uint64_t word_end = 4 * ((size + 3) / 4);  // end of the object's last (possibly partial) word
  for (int j = 0; j < need; ++j) {
    const uint64_t lo = (uint64_t)j * chunk, hi = lo + chunk;
    uint8_t* c = chunks[j];
    const uint64_t body = size > lo ? std::min(size, hi) - lo : 0;
    const uint64_t zero_end = word_end > lo ? std::min(word_end, hi) - lo : 0;
    if (zero_end > body) memset(c + body, 0, zero_end - body);
    for (uint64_t o = std::max(body, zero_end); o < chunk; o += 4) memcpy(c + o, pad, 4);
  }
}

// writeChunks of a code with no parity (need == total; checkConfig admits it,
// multi_config.go:36, and the reference's own tests run 1-of-1 stores,
// multi_test.go:179,257): only MapToGF's mapping depends on the data, so it
// is chosen on the device (pick_mapping) and the chunks are then written on
// the host.  Chunk j = MapFromGF(m, part j): the object's own bytes (the
// mapping cancels, map.go:15-33,103-113), zero low bytes in the object's
// partial last word, then splitVector's zero padding symbols, which
// serialise as BE(m) (multi_store.go:279-296).
int write_data_chunks(int dev, const uint8_t* data, uint64_t size, int need, uint8_t* const* chunks, uint32_t* mapping) {
  const uint64_t L = slot_L(size, (uint32_t)need), chunk = 4 * L, nw = (size + 3) / 4;
  WsLease lease;
  if (int rc = acquire_ws(dev, &lease.ws)) return rc;
  Workspace* ws = lease.ws;
  DeviceScope ds(dev);
  const size_t bbytes = round16(size), wbytes = round16(nw * 4);
  if (int rc = ws->reserve(bbytes + wbytes + 4 * (4 + 2 * kMapCandidates))) return rc;
  uint8_t* d_bytes = ws->dbuf;
  uint32_t* d_words = (uint32_t*)(ws->dbuf + bbytes);
  HIP_TRY(hipMemcpyAsync(d_bytes, data, size, hipMemcpyHostToDevice, ws->stream));
  uint32_t m = 0;
  if (int rc = pick_mapping(ws->stream, d_bytes, size, d_words, (uint32_t*)(ws->dbuf + bbytes + wbytes), &m))
    return rc;
  for (int j = 0; j < need; ++j) {
    const uint64_t lo = (uint64_t)j * chunk;
    const uint64_t body = size > lo ? std::min(size, lo + chunk) - lo : 0;
    if (body && chunks[j] != data + lo) memcpy(chunks[j], data + lo, body);  // an aliased chunk is already the object's bytes
  }
  write_data_tails(size, need, chunk, chunks, m);
  *mapping = m;
  return 0;
}

int write_chunks_check(const uint8_t* data, uint64_t size, int need, int total, uint8_t* const* chunks,
                       uint32_t* mapping) {
  if (!mapping) return fail(Status::InvalidArg, "write_chunks: null mapping");
  *mapping = 0;
  if (need < 1 || total < need) return fail(Status::InvalidArg, "write_chunks: need must be >= 1 and total >= need");
  if (slot_L(size, (uint32_t)need) == 0) return 0;
  if (!data || !chunks) return fail(Status::InvalidArg, "write_chunks: null buffer");
  for (int i = 0; i < total; ++i)
    if (!chunks[i]) return fail(Status::InvalidArg, "write_chunks: null chunk buffer");
  // Zero-copy data chunks: chunk j < need may BE the object's bytes
  // data + j*chunk when it lies wholly inside the object (its bytes are
  // final as they are: MapFromGF(m, MapToGF(x)) = x, map.go:15-33,103-113).
  // Any other overlap between a chunk buffer and the object is refused.
  const uint64_t chunk = 4 * slot_L(size, (uint32_t)need);
  const uintptr_t d0 = (uintptr_t)data, d1 = d0 + size;
  for (int i = 0; i < total; ++i) {
    const uintptr_t c0 = (uintptr_t)chunks[i], c1 = c0 + chunk;
    if (c1 <= d0 || c0 >= d1) continue;
    if (i < need && c0 == d0 + (uint64_t)i * chunk && (uint64_t)(i + 1) * chunk <= size) continue;
    return fail(Status::InvalidArg, "write_chunks: chunk buffer overlaps the object (only data chunk j may alias "
                                    "data + j*chunk_size, when it lies wholly inside the object)");
  }
  return 0;
}

// writeChunks' device pass; dg (optional) hashes the chunks as they become
// final (WriteChunkDigests): it hears of every parity window that lands, of
// a parity rewrite, and of the final mapping.  Arguments already checked.
int write_chunks_impl(const uint8_t* data, uint64_t size, int need, int total, uint8_t* const* chunks,
                      uint32_t* mapping, WriteChunkDigests* dg) {
  const uint64_t L = slot_L(size, (uint32_t)need);
  if (L == 0) {  // MapToGF(empty) = (0, []): every chunk is empty
    if (dg) dg->finalize(0);
    return 0;
  }
  DeviceLease dl;
  if (int rc = dl.acquire()) return rc;
  const int dev = dl.device;
  if (total == need) {
    const int rc = write_data_chunks(dev, data, size, need, chunks, mapping);
    if (dg && !rc) dg->finalize(*mapping);
    return rc;
  }
  PlanRef plan_ref;
  if (int rc = cached_plan(PlanKey{dev, 'E', need, total, {}}, &plan_ref, make_encode_plan)) return rc;
  slime_rs_plan* const plan = plan_ref.get();
  WsLease lease;
  if (int rc = acquire_ws(dev, &lease.ws)) return rc;
  Workspace* ws = lease.ws;
  DeviceScope ds(dev);
  const uint64_t chunk = 4 * L, stride = (uint64_t)total * chunk;
  if (int rc = ws->reserve(round16(stride) + 16)) return rc;
  uint8_t* const slot = ws->dbuf;
  uint32_t* const d_map = (uint32_t*)(ws->dbuf + round16(stride));
  uint32_t* const d_status = d_map + 1;
  // Speculative pass (mapping 0) window by window: object bytes in, parity
  // out, MapToGF's flags accumulating on device; the data-chunk bodies below
  // the object's last word are the caller's own bytes (MapFromGF(m,
  // MapToGF(x)) = x, map.go:15-33,103-113) and are placed on the host with
  // each window's inputs.  The device computes every byte that depends on m.
  const int r = total - need;
  const uint64_t cl = window_cols(L, (uint64_t)total, kObjWindowBytes);
  const uint64_t nwin = (L + cl - 1) / cl;
  // One window (objects up to about the window size): MapToGF's flags come
  // back with the parity, so a mapping-0 object costs one host round trip
  // in all.
  const bool one = nwin == 1;
  uint32_t ms[2] = {0, 0};
  static const uint32_t kZero[2] = {0, 0};
  bool ran_direct = false;
  auto rebase = [&](uint8_t* base, uint32_t* p) { return (uint32_t*)(base + ((uint8_t*)p - slot)); };
  auto pass = [&](size_t direct_bytes) -> int {
    return run_windows(
        ws, slot, nwin, (size_t)total * round64(cl * 4) + 128,
        [&](uint64_t c, int, Window& w) {
          const uint64_t c0 = c * cl, nc = std::min(cl, L - c0);
          if (one)  // the flags zeroed by the window's own upload, ahead of its kernel
            w.in.push_back({(uint8_t*)kZero, (uint64_t)((uint8_t*)d_map - slot), sizeof(kZero)});
          for (int j = 0; j < need; ++j) {
            const uint64_t lo = (uint64_t)j * chunk + 4 * c0, hi = std::min(size, lo + 4 * nc);
            if (lo >= hi) continue;
            w.in.push_back({const_cast<uint8_t*>(data) + lo, lo, hi - lo});
            if (chunks[j] + 4 * c0 != data + lo) w.host.push_back({chunks[j] + 4 * c0, data + lo, hi - lo});
          }
          for (int i = 0; i < r; ++i)
            w.out.push_back({chunks[need + i] + 4 * c0, (uint64_t)(need + i) * chunk + 4 * c0, 4 * nc});
          if (one) w.out.push_back({(uint8_t*)ms, (uint64_t)((uint8_t*)d_map - slot), sizeof(ms)});
        },
        [&](uint64_t c, int, hipStream_t st, uint8_t* base) -> int {
          ran_direct = base != slot;
          BytesLaunch a = bytes_launch(plan, base, stride, 0, L, size, 1, 0, rebase(base, d_status), rebase(base, d_map));
          a.col0 = c * cl;
          a.ncols = std::min(cl, L - a.col0);
          HIP_TRY(launch_encode_bytes(a, st));
          return 0;
        },
        [&](uint64_t c) {
          if (dg && !(ran_direct && (ms[1] & 1u))) dg->parity_ready(4 * std::min(L, (c + 1) * cl));
        },
        direct_bytes);
  };
  auto body = [&]() -> int {
    if (!one) {  // the flags start at zero for every window's kernel
      HIP_TRY(hipMemsetAsync(d_map, 0, 8, ws->stream));
      if (int rc = ws->fence_stages((int)std::min<uint64_t>(kHostStages, nwin))) return rc;
    }
    if (int rc = pass(one ? round16(stride) + 8 : 0)) return rc;
    // A direct pass (the kernel on the pinned stage) left nothing on the
    // device; an object that is not mapping 0 -- a word >= p, odds ~5 in 2^32
    // a word -- runs the window again through the device buffer, which the
    // choice of mapping and the re-encode below read.
    if (ran_direct && (ms[1] & 1u)) {
      ran_direct = false;
      if (int rc = pass(0)) return rc;
    }
    // One window: ms came back with the parity, ms[1] holding MapToGF's
    // flags (bit 0: a word >= p).  With bit 0 clear the mapping is 0 and
    // nothing else runs; otherwise -- and after several windows -- the
    // device chooses (select_mapping) as the 1<<31 re-encode and the
    // fallback expect.
    if (!one || (ms[1] & 1u)) {  // every window has landed: the flags are complete
      HIP_TRY(launch_select_mapping(d_map, d_status, 1, ws->stream));
      HIP_TRY(hipMemcpyAsync(ms, d_map, sizeof(ms), hipMemcpyDeviceToHost, ws->stream));
      if (int rc = sync_ws(ws)) return rc;
    } else {
      ms[0] = ms[1] = 0;
    }
    const bool redo = ms[0] != 0 || ms[1] != 0;
    if (dg) {
      if (redo)
        dg->parity_rewrite();  // parity chunks are written again below
      else
        dg->finalize(0);
    }
    if (ms[1] != 0) {  // MapToGF's random fallback (map.go:64-66): resolved and re-encoded on device
      if (int rc = slime_rs_resolve_fallbacks(plan, slot, stride, size, 1, d_map, d_status, ws->stream, nullptr))
        return rc;
      HIP_TRY(hipMemcpyAsync(ms, d_map, sizeof(ms), hipMemcpyDeviceToHost, ws->stream));
      if (int rc = sync_ws(ws)) return rc;
    } else if (ms[0] != 0) {  // mapping 1<<31: re-encode the whole object (map.go:47-62)
      HIP_TRY(launch_encode_bytes(bytes_launch(plan, slot, stride, 0, L, size, 1, 1, d_status, d_map), ws->stream));
    }
    // The data-chunk tails (partial word, splitVector padding) on the host,
    // and every parity chunk again from the device if the mapping was not 0.
    write_data_tails(size, need, chunk, chunks, ms[0]);
    if (redo) {
      std::vector<Span> out;
      for (int i = need; i < total; ++i) out.push_back({chunks[i], (uint64_t)i * chunk, chunk});
      if (int rc = staged_d2h(ws, slot, out.data(), out.size())) return rc;
    }
    *mapping = ms[0];
    if (dg && redo) {
      dg->parity_ready(chunk);
      dg->finalize(ms[0]);
    }
    return 0;
  };
  const int rc = body();
  if (rc) drain_stages(ws);
  return rc;
}

}  // namespace
}  // namespace slime

using namespace slime;

extern "C" {

uint64_t slime_rs_chunk_size(uint64_t size, int need) { return need > 0 ? 4 * slot_L(size, (uint32_t)need) : 0; }

int slime_rs_write_chunks(const uint8_t* data, uint64_t size, int need, int total, uint8_t* const* chunks,
                          uint32_t* mapping) {
  if (int rc = write_chunks_check(data, size, need, total, chunks, mapping)) return rc;
  return write_chunks_impl(data, size, need, total, chunks, mapping, nullptr);
}

int slime_rs_write_chunks_digest(const uint8_t* data, uint64_t size, int need, int total, uint8_t* const* chunks,
                                 uint32_t* mapping, uint8_t* sha, uint8_t* hdr) {
  if (int rc = write_chunks_check(data, size, need, total, chunks, mapping)) return rc;
  if (!sha) return fail(Status::InvalidArg, "write_chunks_digest: null sha output");
  const uint64_t chunk = 4 * slot_L(size, (uint32_t)need);
  WriteChunkDigests dg(data, size, need, total, chunk, chunks, sha, hdr);
  const int rc = write_chunks_impl(data, size, need, total, chunks, mapping, &dg);
  if (rc) dg.abort();
  dg.finish();
  return rc;
}

int slime_rs_reconstruct(const uint8_t* const* chunks, const int* indices, int need, uint64_t chunk_bytes,
                         uint32_t mapping, uint64_t size, uint8_t* out) {
  if (need < 0) return fail(Status::InvalidArg, "reconstruct: negative count");
  if (need == 0) return status_of(Status::Empty, "RecoverData");
  if (!chunks || !indices) return fail(Status::InvalidArg, "reconstruct: bad args");
  if (int rc = check_survivors(need, indices)) return rc;
  if (size && !out) return fail(Status::InvalidArg, "reconstruct: null out");
  if (chunk_bytes % 4) {
    // Chunks of a length no writer produces (truncated or corrupt stored
    // chunks).  MapToGFWith packs a partial last word with zero low bytes
    // (map.go:16-33,74-98), so each survivor is its bytes zero-padded to
    // 4*ceil(chunk_bytes/4), and each recovered data row is that long too
    // (RecoverData, vector.go:80-85; MapFromGF, map.go:103-113).  Rare and
    // never on the fast path: stage padded copies and run the normal path.
    const uint64_t padded = (chunk_bytes + 3) & ~(uint64_t)3;
    std::vector<std::vector<uint8_t>> copy((size_t)need, std::vector<uint8_t>(padded, 0));
    std::vector<const uint8_t*> ptrs((size_t)need);
    for (int q = 0; q < need; ++q) {
      if (!chunks[q]) return fail(Status::InvalidArg, "reconstruct: null chunk");
      memcpy(copy[q].data(), chunks[q], chunk_bytes);
      ptrs[q] = copy[q].data();
    }
    return slime_rs_reconstruct(ptrs.data(), indices, need, padded, mapping, size, out);
  }
  const uint64_t L = chunk_bytes / 4, body_bytes = (uint64_t)need * chunk_bytes, got = std::min(size, body_bytes);
  // data[:f.Size] of a make([]byte, 0, Size+16) buffer (multi_store.go:203,241):
  // bytes past the recovered ones are the zeroed capacity.
  if (size > got) memset(out + got, 0, size - got);
  if (got == 0) return 0;
  for (int q = 0; q < need; ++q)
    if (!chunks[q]) return fail(Status::InvalidArg, "reconstruct: null chunk");
  DeviceLease dl;
  if (int rc = dl.acquire()) return rc;
  const int dev = dl.device;
  std::vector<int> have(indices, indices + need);
  PlanRef plan_ref;
  if (int rc = cached_plan(PlanKey{dev, 'O', need, 0, have}, &plan_ref, make_object_recover_plan)) return rc;
  slime_rs_plan* const plan = plan_ref.get();
  WsLease lease;
  if (int rc = acquire_ws(dev, &lease.ws)) return rc;
  Workspace* ws = lease.ws;
  DeviceScope ds(dev);
  const uint64_t stride = 2 * body_bytes;
  if (int rc = ws->reserve(round16(stride) + 16)) return rc;
  uint8_t* const slot = ws->dbuf;
  uint32_t* const d_map = (uint32_t*)(ws->dbuf + round16(stride));
  // Window by window: survivors' columns in, all need data rows decoded,
  // the object's bytes of those columns out.
  const uint64_t cl = window_cols(L, 2 * (uint64_t)need, kObjWindowBytes);
  const uint64_t nwin = (L + cl - 1) / cl;
  // The mapping goes up with every window's inputs (the same word each time:
  // each window's kernel reads it behind its own upload).
  const uint32_t map_word = mapping;
  const int rc = run_windows(
      ws, slot, nwin, (size_t)2 * need * round64(cl * 4) + 64,
      [&](uint64_t c, int, Window& w) {
        const uint64_t c0 = c * cl, nc = std::min(cl, L - c0);
        w.in.push_back({(uint8_t*)&map_word, (uint64_t)((uint8_t*)d_map - slot), 4});
        for (int q = 0; q < need; ++q)
          w.in.push_back({const_cast<uint8_t*>(chunks[q]) + 4 * c0, (uint64_t)q * chunk_bytes + 4 * c0, 4 * nc});
        for (int t = 0; t < need; ++t) {
          const uint64_t o = (uint64_t)t * chunk_bytes + 4 * c0;
          if (o < got) w.out.push_back({out + o, body_bytes + o, std::min(4 * nc, got - o)});
        }
      },
      [&](uint64_t c, int, hipStream_t st, uint8_t* base) -> int {
        BytesLaunch a =
            bytes_launch(plan, base, stride, 0, L, 0, 1, 0, nullptr, (uint32_t*)(base + ((uint8_t*)d_map - slot)));
        a.col0 = c * cl;
        a.ncols = std::min(cl, L - a.col0);
        HIP_TRY(launch_decode_bytes(a, st));
        return 0;
      },
      [](uint64_t) {}, round16(stride) + 4);
  if (rc) drain_stages(ws);
  return rc;
}

int slime_rs_reconstruct_verify(const uint8_t* const* chunks, const int* indices, int need, uint64_t chunk_bytes,
                                uint32_t mapping, uint64_t size, uint8_t* out, const uint8_t* want_sha) {
  if (!want_sha) return fail(Status::InvalidArg, "reconstruct_verify: null sha");
  if (int rc = slime_rs_reconstruct(chunks, indices, need, chunk_bytes, mapping, size, out)) return rc;
  uint8_t have[32];
  Sha256 h;
  if (size) h.update(out, size);
  h.final(have);
  if (memcmp(have, want_sha, 32) != 0) return status_of(Status::BadHash, "reconstruct");
  return 0;
}

}  // extern "C"
