// The Go API's data entry points over host memory (include/slime_rs.h,
// "internal/rs: Go-API data entry points" and the gf codec): CreateParity /
// CreateParities / RecoverData through the staged pipeline to the GPU
// (host_pipeline.hpp), and MapToGF / MapToGFWith / MapFromGF on the host
// cores (host_codec.cpp) or through the device codec.
// Reference: internal/rs/vector.go:18-102, internal/rs/gf/map.go:15-113.
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <string>
#include <vector>

#include "capi_internal.hpp"
#include "gfp_host.hpp"
#include "host_codec.hpp"
#include "host_copy.hpp"
#include "host_pipeline.hpp"
#include "rs_matrix.hpp"

namespace slime {

// ---- plans of the Go-API rows ---------------------------------------------------------

namespace {

int make_rows_plan(const PlanKey& key, slime_rs_plan** out) {
  // kind 'P': code rows key.indices[...] of a need = key.k code, inputs 0..need-1.
  const int dev = std::get<0>(key), need = std::get<2>(key);
  const std::vector<int>& rows = std::get<4>(key);
  std::vector<uint32_t> coeff;
  std::vector<uint32_t> row;
  for (int r : rows) {
    if (Status st = code_row(need, r, &row); st != Status::Ok) return status_of(st, "ParityMatrix");
    coeff.insert(coeff.end(), row.begin(), row.end());
  }
  std::vector<int> in(need);
  for (int j = 0; j < need; ++j) in[j] = j;
  return slime_rs_plan_matrix(dev, coeff.data(), (int)rows.size(), need, in.data(), out);
}

int run_rows(int need, const std::vector<int>& rows, const uint32_t* const* data, uint64_t L, uint32_t* const* out) {
  DeviceLease dl;
  if (int rc = dl.acquire()) return rc;
  PlanRef plan;
  if (int rc = cached_plan(PlanKey{dl.device, 'P', need, 0, rows}, &plan, make_rows_plan)) return rc;
  return host_apply(plan.get(), data, out, L);
}

// Data rows of `need` absent from the survivors `have`: the only rows of
// RecoverData's inverse that are not unit rows (vector.go:77-85).
std::vector<int> erased_rows(int need, const int* have) {
  std::vector<int> e;
  for (int t = 0; t < need; ++t)
    if (std::find(have, have + need, t) == have + need) e.push_back(t);
  return e;
}

int make_erased_rows_plan(const PlanKey& key, slime_rs_plan** out) {
  // kind 'R': the erased data rows only.
  const int need = std::get<2>(key);
  const std::vector<int>& have = std::get<4>(key);
  return make_inverse_rows_plan(std::get<0>(key), need, have, erased_rows(need, have.data()), out);
}

bool overlaps(const void* a, uint64_t an, const void* b, uint64_t bn) {
  const uintptr_t a0 = (uintptr_t)a, b0 = (uintptr_t)b;
  return a0 < b0 + bn && b0 < a0 + an;
}

}  // namespace

int make_inverse_rows_plan(int dev, int need, const std::vector<int>& have, const std::vector<int>& want,
                           slime_rs_plan** out) {
  const int total = std::max(need, *std::max_element(have.begin(), have.end()) + 1);
  slime_rs_plan* tmp = nullptr;
  if (int rc = slime_rs_plan_reconstruct(dev, need, total, have.data(), want.data(), (int)want.size(), &tmp))
    return rc;
  std::vector<int> pos(need);
  for (int q = 0; q < need; ++q) pos[q] = q;
  slime_rs_plan* staged = nullptr;
  const int rc = slime_rs_plan_matrix(dev, tmp->coeff.data(), (int)want.size(), need, pos.data(), &staged);
  destroy_plan(tmp);
  if (rc) return rc;
  *out = staged;
  return 0;
}

// RecoverData's index checks (vector.go:65-77): no non-negative index ->
// "No indices given"; a negative index -> Go's index-out-of-range; duplicate
// or otherwise dependent rows -> invertMatrix's panic.
int check_survivors(int need, const int* indices) {
  int max_index = -1;
  for (int i = 0; i < need; ++i) max_index = std::max(max_index, indices[i]);
  if (max_index == -1) return status_of(Status::NoIndices, "RecoverData");
  for (int i = 0; i < need; ++i)
    if (indices[i] < 0)
      return fail(Status::IndexRange, "runtime error: index out of range [" + std::to_string(indices[i]) + "]");
  Matrix hv((size_t)need, (size_t)need), inv;
  std::vector<uint32_t> row;
  for (int i = 0; i < need; ++i) {
    if (Status st = code_row(need, indices[i], &row); st != Status::Ok) return status_of(st, "ParityMatrixCached");
    std::copy(row.begin(), row.end(), hv.v.begin() + (size_t)i * need);
  }
  if (Status st = invert(hv, &inv); st != Status::Ok) return status_of(st, "RecoverData");
  return 0;
}

// ---- the device codec's mapping choice ----------------------------------------------

int choose_mapping(hipStream_t st, const uint32_t* d_words, uint64_t nw, uint32_t* d_scratch, uint32_t* mapping) {
  constexpr uint32_t kCand = kMapCandidates;
  uint32_t* d_flags = d_scratch;
  uint32_t* d_cand = d_flags + 4;
  uint32_t* d_bad = d_cand + kCand;
  uint32_t flags = 0;
  HIP_TRY(hipMemcpyAsync(&flags, d_flags, 4, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  *mapping = 0;
  if (!(flags & 1u)) return 0;
  if (!(flags & 2u)) {
    *mapping = 1u << 31;  // map.go:47: try just switching the high bit first
    return 0;
  }
  for (int round = 0; round < (1 << 16); ++round) {  // map.go:64-66
    uint32_t cand[kCand], bad[kCand];
    draw_candidates(cand, kCand);
    HIP_TRY(hipMemcpyAsync(d_cand, cand, sizeof(cand), hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemsetAsync(d_bad, 0, sizeof(bad), st));
    HIP_TRY(launch_mapping_probe(d_words, nw, d_cand, kCand, d_bad, st));
    HIP_TRY(hipMemcpyAsync(bad, d_bad, sizeof(bad), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    for (uint32_t c = 0; c < kCand; ++c)
      if (!bad[c]) {
        *mapping = cand[c];
        return 0;
      }
  }
  return status_of(Status::MappingFallback, "MapToGF");
}

int pick_mapping(hipStream_t st, const uint8_t* d_bytes, uint64_t len, uint32_t* d_words, uint32_t* d_scratch,
                 uint32_t* mapping) {
  HIP_TRY(hipMemsetAsync(d_scratch, 0, 4, st));
  HIP_TRY(launch_map_pack(d_bytes, len, 0, d_words, d_scratch, st));
  return choose_mapping(st, d_words, (len + 3) / 4, d_scratch, mapping);
}

// ---- the codec over host memory, placed on the GPU ----------------------------------
//
// slime_gf_codec_placement(1): the codec calls stream through the same pinned
// 3-stage ring as the object entry points (run_windows), the caller's
// buffers pageable (the round-3 form, kept as the measured alternative and
// exercised by the GPU tests).

namespace {

std::atomic<int> g_codec_device{0};

bool codec_on_device() { return g_codec_device.load(std::memory_order_relaxed) != 0; }

int codec_setup(uint64_t bytes_needed, Workspace** wsp, WsLease& lease, DeviceLease& dl) {
  if (int rc = dl.acquire()) return rc;
  if (int rc = acquire_ws(dl.device, &lease.ws)) return rc;
  *wsp = lease.ws;
  return (*wsp)->reserve(bytes_needed);
}

constexpr uint64_t kCodecWindowBytes = 8u << 20;  // largest window: input bytes (+ as many out)

// Input bytes per codec window: at least 4 windows per call when the input
// allows (so H2D, kernel and D2H of one call overlap across the ring's 3
// stages), between 512 KiB and 8 MiB, a multiple of 64 KiB.
uint64_t codec_window(uint64_t len) {
  const uint64_t quarter = ((len / 4) + 65535) & ~(uint64_t)65535;
  return std::min<uint64_t>(kCodecWindowBytes, std::max<uint64_t>(512u << 10, quarter));
}

// Bytes -> words windows of MapToGF(With): window c packs input bytes
// [c*W, c*W + W) into words [c*W/4, ...) on the device (mapping n, flags
// OR-reduced if given) and streams the words back to `out`.
int pack_windows(Workspace* ws, const uint8_t* in, uint64_t len, uint32_t n, uint32_t* out, uint8_t* d_bytes,
                 uint32_t* d_words, uint32_t* d_flags) {
  const uint64_t W = codec_window(len), nwin = (len + W - 1) / W;
  uint8_t* const base = ws->dbuf;
  return run_windows(
      ws, base, nwin, 2 * W,
      [&](uint64_t c, int, Window& w) {
        const uint64_t b0 = c * W, nb = std::min(W, len - b0);
        w.in.push_back({const_cast<uint8_t*>(in) + b0, (uint64_t)(d_bytes - base) + b0, nb});
        w.out.push_back({(uint8_t*)out + b0, (uint64_t)((uint8_t*)d_words - base) + b0, 4 * ((nb + 3) / 4)});
      },
      [&](uint64_t c, int, hipStream_t st, uint8_t*) -> int {
        const uint64_t b0 = c * W, nb = std::min(W, len - b0);
        HIP_TRY(launch_map_pack(d_bytes + b0, nb, n, d_words + b0 / 4, d_flags, st));
        return 0;
      });
}

int map_to_gf_with_device(const uint8_t* in, uint64_t len, uint32_t n, uint32_t* out) {
  const uint64_t nw = (len + 3) / 4;
  WsLease lease;
  Workspace* ws = nullptr;
  const size_t bbytes = round16(len);
  DeviceLease dl;
  if (int rc = codec_setup(bbytes + round16(nw * 4), &ws, lease, dl)) return rc;
  DeviceScope ds(ws->device);
  const int rc = pack_windows(ws, in, len, n, out, ws->dbuf, (uint32_t*)(ws->dbuf + bbytes), nullptr);
  if (rc) drain_stages(ws);
  return rc;
}

int map_to_gf_device(const uint8_t* in, uint64_t len, uint32_t* mapping, uint32_t* out) {
  const uint64_t nw = (len + 3) / 4;
  WsLease lease;
  Workspace* ws = nullptr;
  const size_t bbytes = round16(len), wbytes = round16(nw * 4);
  DeviceLease dl;
  if (int rc = codec_setup(bbytes + wbytes + 4 * (4 + 2 * kMapCandidates), &ws, lease, dl)) return rc;
  DeviceScope ds(ws->device);
  uint8_t* d_bytes = ws->dbuf;
  uint32_t* d_words = (uint32_t*)(ws->dbuf + bbytes);
  uint32_t* d_scratch = (uint32_t*)(ws->dbuf + bbytes + wbytes);
  auto body = [&]() -> int {
    // Speculative mapping 0 (map.go:35-45): the words stream back while the
    // flags of every window accumulate on the device; 1<<31 (map.go:47-62,
    // about 2% of uniform 64 MiB bodies) or the random fallback (:64-66)
    // re-map the words on the device and send them again.
    HIP_TRY(hipMemsetAsync(d_scratch, 0, 4, ws->stream));
    HIP_TRY(hipStreamSynchronize(ws->stream));
    if (int rc = pack_windows(ws, in, len, 0, out, d_bytes, d_words, d_scratch)) return rc;
    uint32_t m = 0;
    if (int rc = choose_mapping(ws->stream, d_words, nw, d_scratch, &m)) return rc;
    if (m) {
      HIP_TRY(launch_xor_words(d_words, nw, m, ws->stream));
      const Span sp{(uint8_t*)out, (uint64_t)((uint8_t*)d_words - ws->dbuf), nw * 4};
      if (int rc = staged_d2h(ws, ws->dbuf, &sp, 1)) return rc;
    }
    *mapping = m;
    return 0;
  };
  const int rc = body();
  if (rc) drain_stages(ws);
  return rc;
}

// MapToGF on host memory, in place on the caller's buffers (map.go:15-67):
// one pass packs the words (mapping 0) and notes whether 0 and 1<<31 fit;
// a mapping other than 0 is then XORed in by a second pass.  The random
// fallback (:64-66) draws kMapCandidates candidates at a time from the
// library's stream and takes the first that fits -- the device form's rule
// (choose_mapping), so both placements consume the stream alike.
int map_to_gf_host(const uint8_t* in, uint64_t len, uint32_t* mapping, uint32_t* out) {
  const uint64_t nw = (len + 3) / 4;
  uint32_t flags = 0, m = 0;
  host_pack(in, len, 0, out, &flags);
  if (flags & 1u) {
    if (!(flags & 2u)) {
      m = 1u << 31;  // map.go:47
    } else {
      bool found = false;
      for (int round = 0; round < (1 << 16) && !found; ++round) {
        uint32_t cand[kMapCandidates];
        draw_candidates(cand, kMapCandidates);
        for (uint32_t c = 0; c < kMapCandidates && !found; ++c)
          if (host_mapping_fits(out, nw, cand[c])) m = cand[c], found = true;
      }
      if (!found) return status_of(Status::MappingFallback, "MapToGF");
    }
    host_xor(out, nw, m);
  }
  *mapping = m;
  return 0;
}

int map_from_gf_device(uint32_t n, const uint32_t* in, uint64_t count, uint8_t* out) {
  WsLease lease;
  Workspace* ws = nullptr;
  const size_t wbytes = round16(count * 4);
  DeviceLease dl;
  if (int rc = codec_setup(2 * wbytes, &ws, lease, dl)) return rc;
  DeviceScope ds(ws->device);
  uint32_t* d_words = (uint32_t*)ws->dbuf;
  uint8_t* d_bytes = ws->dbuf + wbytes;
  const uint64_t W = codec_window(4 * count) / 4, nwin = (count + W - 1) / W;  // words per window
  const int rc = run_windows(
      ws, ws->dbuf, nwin, 2 * kCodecWindowBytes,
      [&](uint64_t c, int, Window& w) {
        const uint64_t w0 = c * W, nwd = std::min(W, count - w0);
        w.in.push_back({(uint8_t*)(in + w0), 4 * w0, 4 * nwd});
        w.out.push_back({out + 4 * w0, wbytes + 4 * w0, 4 * nwd});
      },
      [&](uint64_t c, int, hipStream_t st, uint8_t*) -> int {
        const uint64_t w0 = c * W, nwd = std::min(W, count - w0);
        HIP_TRY(launch_map_unpack(d_words + w0, nwd, n, d_bytes + 4 * w0, st));
        return 0;
      });
  if (rc) drain_stages(ws);
  return rc;
}

}  // namespace
}  // namespace slime

using namespace slime;

extern "C" {

int slime_rs_create_parity(const uint32_t* const* data, const uint64_t* lens, int ndata, int index, uint32_t* out) {
  if (ndata < 0 || (ndata > 0 && (!data || !lens))) return fail(Status::InvalidArg, "CreateParity: bad args");
  for (int i = 1; i < ndata; ++i)
    if (lens[i] != lens[0]) return status_of(Status::VaryingLength, "CreateParity");
  if (ndata == 0) return fail(Status::IndexRange, "runtime error: index out of range [0] with length 0");
  if (index < 0) return fail(Status::IndexRange, "runtime error: index out of range [" + std::to_string(index) + "]");
  std::vector<uint32_t> row;
  if (Status st = code_row(ndata, index, &row); st != Status::Ok) return status_of(st, "ParityMatrixCached");
  const uint64_t L = lens[0];
  if (L == 0) return 0;
  if (!out) return fail(Status::InvalidArg, "CreateParity: null out");
  for (int j = 0; j < ndata; ++j)
    if (!data[j]) return fail(Status::InvalidArg, "CreateParity: null data chunk");
  return run_rows(ndata, std::vector<int>{index}, data, L, &out);
}

int slime_rs_create_parities(const uint32_t* const* data, const uint64_t* lens, int ndata, int total,
                             uint32_t* const* out) {
  if (ndata <= 0 || total < ndata || !data || !lens) return fail(Status::InvalidArg, "CreateParities: bad args");
  for (int i = 1; i < ndata; ++i)
    if (lens[i] != lens[0]) return status_of(Status::VaryingLength, "CreateParity");
  if (total == ndata || lens[0] == 0) return 0;
  if (!out) return fail(Status::InvalidArg, "CreateParities: null out");
  for (int j = 0; j < ndata; ++j)
    if (!data[j]) return fail(Status::InvalidArg, "CreateParities: null data chunk");
  for (int i = 0; i < total - ndata; ++i)
    if (!out[i]) return fail(Status::InvalidArg, "CreateParities: null out row");
  std::vector<int> rows;
  for (int r = ndata; r < total; ++r) rows.push_back(r);
  return run_rows(ndata, rows, data, lens[0], out);
}

int slime_rs_recover_data(const uint32_t* const* chunks, const uint64_t* lens, int nchunks, const int* indices,
                          int nindices, uint32_t* const* out) {
  if (nchunks < 0 || nindices < 0) return fail(Status::InvalidArg, "RecoverData: negative count");
  if (nchunks != nindices) return status_of(Status::LenMismatch, "RecoverData");
  if (nchunks == 0) return status_of(Status::Empty, "RecoverData");
  if (!chunks || !lens || !indices) return fail(Status::InvalidArg, "RecoverData: bad args");
  if (int rc = check_survivors(nchunks, indices)) return rc;
  const int need = nchunks;
  const uint64_t L = lens[0];
  for (int i = 1; i < need; ++i)
    if (lens[i] < L)
      return fail(Status::IndexRange, "runtime error: index out of range [" + std::to_string(lens[i]) +
                                          "] with length " + std::to_string(lens[i]));
  if (L == 0) return 0;
  if (!out) return fail(Status::InvalidArg, "RecoverData: null out");
  for (int i = 0; i < need; ++i)
    if (!chunks[i] || !out[i]) return fail(Status::InvalidArg, "RecoverData: null buffer");

  // A caller repairing in place may pass output rows that overlap survivor
  // chunks (Go's RecoverData returns fresh rows, so the shim never does).
  // The erased rows are written before the unit rows below read their
  // chunks: such survivors are read from copies taken first.  (A unit row
  // written over its own chunk is safe: it reads each word before writing it.)
  std::vector<std::vector<uint32_t>> saved;
  std::vector<const uint32_t*> in(chunks, chunks + need);
  for (int q = 0; q < need; ++q) {
    bool hit = false;
    for (int t = 0; t < need && !hit; ++t)
      hit = !(indices[q] == t && out[t] == chunks[q]) && overlaps(out[t], 4 * L, chunks[q], 4 * L);
    if (hit) {
      saved.emplace_back(chunks[q], chunks[q] + L);
      in[q] = saved.back().data();
    }
  }

  // vector.go:77-85 applies the whole inverse, but the inverse row of a data
  // shard that survived is a unit row: its output is that chunk mod p, a
  // host pass over memory the caller already holds.  Only the erased data
  // rows cross to the device (need chunks in, the erased rows back).
  const std::vector<int> erased = erased_rows(need, indices);
  auto unit_rows = [&] {
    for (int q = 0; q < need; ++q)
      if (indices[q] < need) host_mod_p(in[q], L, out[indices[q]]);
  };
  if (erased.empty()) {
    unit_rows();
    return 0;
  }
  DeviceLease dl;
  if (int rc = dl.acquire()) return rc;
  std::vector<int> have(indices, indices + nindices);
  PlanRef plan;
  if (int rc = cached_plan(PlanKey{dl.device, 'R', need, 0, have}, &plan, make_erased_rows_plan)) return rc;
  std::vector<uint32_t*> rows;
  for (int t : erased) rows.push_back(out[t]);
  // The unit rows run after the pipeline, not beside it on a side thread:
  // that form measured no faster (fresh-page faults of both compete,
  // MEASUREMENTS.md round 4, profiles/r04/s7_hostab).
  if (int rc = host_apply(plan.get(), in.data(), rows.data(), L)) return rc;
  unit_rows();
  return 0;
}

// ---- gf codec (host memory) -----------------------------------------------------------

int slime_gf_codec_info(const char** isa, int* threads) {
  if (isa) *isa = host_codec_isa();
  if (threads) *threads = copy_pool_threads() + 1;
  return 0;
}

int slime_gf_codec_placement(int mode) {
  if (mode < 0) return g_codec_device.load();
  if (mode > 1) return fail(Status::InvalidArg, "codec placement: 0 = host, 1 = device");
  g_codec_device.store(mode);
  return 0;
}

int slime_gf_map_to_gf_with(const uint8_t* in, uint64_t len, uint32_t n, uint32_t* out) {
  const uint64_t nw = (len + 3) / 4;
  if (nw == 0) return 0;
  if (!in || !out) return fail(Status::InvalidArg, "MapToGFWith: null buffer");
  if (codec_on_device()) return map_to_gf_with_device(in, len, n, out);
  host_pack(in, len, n, out, nullptr);
  return 0;
}

int slime_gf_map_to_gf(const uint8_t* in, uint64_t len, uint32_t* mapping, uint32_t* out) {
  if (!mapping) return fail(Status::InvalidArg, "MapToGF: null mapping");
  const uint64_t nw = (len + 3) / 4;
  *mapping = 0;
  if (nw == 0) return 0;
  if (!in || !out) return fail(Status::InvalidArg, "MapToGF: null buffer");
  return codec_on_device() ? map_to_gf_device(in, len, mapping, out) : map_to_gf_host(in, len, mapping, out);
}

int slime_gf_map_from_gf(uint32_t n, const uint32_t* in, uint64_t count, uint8_t* out) {
  if (count == 0) return 0;
  if (!in || !out) return fail(Status::InvalidArg, "MapFromGF: null buffer");
  if (codec_on_device()) return map_from_gf_device(n, in, count, out);
  host_unpack(in, count, n, out);
  return 0;
}

}  // extern "C"
