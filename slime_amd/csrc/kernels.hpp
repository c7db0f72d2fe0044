// Internal launcher interface between the host library (rs_capi.cpp) and the
// HIP kernels (rs_apply.hip, gf_codec.hip). Not part of the public C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <stdlib.h>

#include <functional>

namespace slime {

// One matrix application over a batch of objects:
//   out[o*out_obj + out_idx[i]*out_shard + b]
//       = sum_j coeff[i][j] * in[o*in_obj + in_idx[j]*in_shard + b]   (mod p)
// for o < nobj, i < rows, b < ncols.  Strides are in uint32 elements.
// coeff / in_idx / out_idx are DEVICE pointers (a plan's tables).
struct ApplyLaunch {
  const uint32_t* in;
  uint32_t* out;
  uint64_t in_obj_stride;
  uint64_t in_shard_stride;
  uint64_t out_obj_stride;
  uint64_t out_shard_stride;
  const uint32_t* coeff;    // rows x coeff_stride(k), row-major, canonical residues
  const uint32_t* in_idx;   // k input shard indices
  const uint32_t* out_idx;  // rows output shard indices
  uint64_t ncols;
  uint32_t nobj;
  uint32_t rows;
  uint32_t k;
  bool vec_ok;              // 16-byte units per lane (needs 4-byte aligned bases; see rs_capi.cpp)
  // Matrix-core form (rs_apply_mfma.hip): the plan's digit table
  // (mfma_table.hpp, device) or null, and the highest input / output shard
  // index (the kernel's 32-bit offsets need every object under 4 GiB).
  const uint8_t* mfma = nullptr;
  uint32_t in_max = 0, out_max = 0;
  bool in_seq = false;  // in_idx is 0..k-1 (encode plans): uniform input offsets
};

// Matrix-core apply kernel: whether this launch can take it (table present,
// mode on, mfma_wanted, shape and spans supported), and the launch.
// Process-wide mode, on by default: slime_rs_kernel_matrix_cores() switches it.
bool mfma_eligible(const ApplyLaunch& a);
hipError_t launch_apply_mfma(const ApplyLaunch& a, hipStream_t stream);
int matrix_core_mode();
void set_matrix_core_mode(int m);
// The product rule (rs_apply_mfma.hip): k >= 33, or 17 <= k <= 32 with
// k * rows >= 128 multiply-accumulates per column.
bool mfma_wanted(uint32_t k, uint32_t rows);

// Row stride (words) of a device coefficient table: k rounded up to 16 words,
// so every 16-coefficient chunk of a row is one aligned s_load_dwordx16.
inline uint32_t coeff_stride(uint32_t k) { return (k + 15u) & ~15u; }

hipError_t launch_apply(const ApplyLaunch& a, hipStream_t stream);

// 17 <= k <= 32, 16-byte-aligned-capable layouts, shards under 4 GiB: the
// pipelined k-template kernel instantiated for wide k (rs_apply_k32.hip).
hipError_t launch_pipe_k32(const ApplyLaunch& a, hipStream_t stream);

// Kernel form for shards/chunks under 4 GiB: software-pipelined (default) or
// not (the form larger ones always take).  Process-wide; see rs_apply.hip.
bool pipelined_kernels();
void set_pipelined_kernels(bool on);
// Work schedule of the pipelined kernels: 1 dynamic (ticket counters) outside
// graph captures and static inside (default), 2 dynamic in captures too, 0
// static shares.  Process-wide; see rs_apply.hip.
int queue_mode();
void set_queue_mode(int m);
// Second pass of the fused byte encode at need <= 10 on the ticket walk:
// 0 = correct the switched units' parity from top bits phase 0 stored when
// objects are >= 1 GiB (where uniform bytes switch in more than a quarter of
// the objects), else re-encode them (default); 1 = always correct; 2 =
// always re-encode.  Process-wide; see rs_bytes_launch.hpp.
int switch_bits_mode();
void set_switch_bits_mode(int m);
// Whether a launch on `s` may take the dynamic schedule under the mode (a
// captured launch replays on the set it was captured with: mode 2 only).
bool queue_allowed(hipStream_t s);
// Ticket counters of the dynamic-schedule kernels (rs_apply_queue_kernel):
// kQueueCounters draw counters + an exit counter per set (zero whenever no
// launch holds the set).  Takes a set that no unfinished launch holds from
// the current device's pool and calls launch(set); the set goes back to the
// pool behind an event recorded on `stream` after the launch, or stays with
// the graph when `stream` is capturing.  *launched = false (and hipSuccess)
// when no set could be had -- a capture with the pool exhausted; the caller
// then takes the static kernel.  Returns launch's result.
constexpr int kQueueCounters = 8;
hipError_t with_tickets(hipStream_t stream, const std::function<hipError_t(uint32_t*)>& launch, bool* launched);
// Creates the current device's first counter sets outside any capture (plan
// creation calls it), so a captured launch finds the pool ready.
hipError_t warm_ticket_pool(int device);
// Sets allocated / held by launches in flight or graphs, for `device` (tests).
void ticket_pool_stats(int device, uint64_t* sets, uint64_t* held);
// Launches on `device` that took a counter set (dynamic) / asked with_tickets
// for one and were sent to the static kernel (no set to be had).
void schedule_counts(int device, uint64_t* dynamic, uint64_t* fallback);

// Column segments per object for a launch over nobj objects of ncols
// columns (the apply and byte kernels cut each object into this many
// contiguous segments scheduled like separate objects).
uint32_t object_segments(uint32_t nobj, uint64_t ncols);

// Walk units of a queue launch over nobj objects of ncols columns (4 columns
// a lane, 64 U lanes a tile, C tiles a unit, `spread` segments an object:
// TicketWalk's numbering, empty units included).
inline uint64_t queue_units(uint32_t nobj, uint64_t ncols, int U, int C, uint32_t spread) {
  const uint64_t ntiles = ((ncols >> 2) + 64ull * U - 1) / (64ull * U);
  const uint64_t groups = (ntiles + 4ull * C - 1) / (4ull * C), s = spread ? spread : 1;
  return (uint64_t)nobj * s * ((groups + s - 1) / s) * 4;
}

// Blocks of a queue launch with `units` walk units: the full grid, or one
// wave per unit (4 waves a block) when there are fewer.  Every wave of a
// queue launch draws from the counters and counts itself out with
// memory-side atomics (TicketWalk::finish): a full grid over the few units
// of a host call on a small object spent ~20 us there, against ~2 us of
// work (profiles/r04/s8_lat*).  Edge tiles and column tails are strided over
// whatever grid runs, so any grid is correct.
inline uint64_t queue_blocks(uint64_t full, uint64_t units) {
  const uint64_t want = (units + 3) / 4;
  return want < 1 ? 1 : want < full ? want : full;
}

// Segments per object of a dynamic-schedule launch (TicketWalk `spread`,
// rs_apply_kernel.hpp): about 64 segments over the batch, ceil(64 / nobj),
// capped at the object's groups of 4*C tiles of U 16-byte vectors per lane
// (in-process sweeps, profiles/r02/s61_spread/, s62_spread2/: best S = 1 at
// 64 and 128 objects, 2 at C2's 32, 4 at C5's 16; more segments cost up to 4%).
// `streams` = k + rows of an apply launch (0: not given, the byte kernels):
// an apply launch over six streams an object (4/6) takes about 256 segments,
// one per wave group in flight -- C2's 32 objects at S = 8 ran +1.0 to +2.8%
// and 64 objects at S = 4 +1.3 to +2.1% on four boxes, where 8/12 and 10/14
// gained nothing consistent from more (profiles/r06/s5_spread/,
// s6_spread2/), and slime's default 3/5 lost up to 3% at S = 8 on a slow
// allocation and was level on a fast one (s13_spread35/): it keeps the 64
// (tools/c2_stamps.py).
// 0 when the launch has too many units for 32-bit tickets, or at most one
// block's (below): the caller takes the static kernel.
inline uint32_t queue_spread(uint32_t nobj, uint64_t ncols, int U, int C, uint32_t streams = 0) {
  const uint64_t ntiles = ((ncols >> 2) + 64ull * U - 1) / (64ull * U);
  const uint64_t groups = (ntiles + 4ull * C - 1) / (4ull * C);
  const uint64_t target = streams == 6 ? 256 : 64;
  uint64_t S = (target + (uint64_t)nobj - 1) / (nobj ? nobj : 1);
  if (S > groups) S = groups ? groups : 1;
  const uint64_t B = (groups + S - 1) / S;
  const uint64_t units = (uint64_t)nobj * S * B * 4;
  if (units >= (1ull << 32)) return 0;
  // A launch of at most one block's units takes the static kernels: the
  // dynamic schedule has nothing to balance there, and its set hand-out and
  // ticket atomics are most of such a launch (env SLIME_RS_TINY_UNITS,
  // default 4; 0 = off).  So does a launch over ONE object of at most 1024
  // units -- a host call's window, up to about 16 MiB: one block or less per
  // CU, and the static grid's waves load their tiles at once where the
  // queue's fewer waves walk them (1 MiB write_chunks 94-113 -> 82-92 us,
  // reconstruct 122-150 -> 110-125, 8 MiB 3-5% faster, 64 MiB fused write and
  // reconstruct equal or better: profiles/r04/s50_tinyab2, s51_tinyab3; env
  // SLIME_RS_ONE_OBJECT_UNITS, default 1024; 0 = off).  Batches of several
  // objects keep the queue from 5 units up.
  static const uint64_t tiny = [] {
    const char* e = getenv("SLIME_RS_TINY_UNITS");
    const long long v = e ? atoll(e) : 4;
    return v > 0 ? (uint64_t)v : 0ull;
  }();
  static const uint64_t one_object = [] {
    const char* e = getenv("SLIME_RS_ONE_OBJECT_UNITS");
    const long long v = e ? atoll(e) : 1024;
    return v > 0 ? (uint64_t)v : 0ull;
  }();
  if (units <= tiny || (nobj == 1 && units <= one_object)) return 0;
  return (uint32_t)S;
}

// --- fused byte-domain encode/decode over object slots (rs_bytes.hip) --------
// Slot o at slots + o*slot_stride bytes; chunk c at slot + c*cstride (4L by default).  coeff /
// in_idx / out_idx are a plan's device tables.  Encode: phase 0 = speculative
// (mapping 0, OR MapToGF flag bits into flags[obj]); select_mapping turns the
// flags into mapping[] and a fallback status in place; phase 1 re-encodes the
// objects with mapping != 0 and status == 0.  Decode uses mapping[obj].
// What phase 0 of the fused encode did (BytesLaunch::sw): whether it ran the
// mid-object-switching kernel, and the unit layout it ran with -- phase 1
// redoes units by this record, never by re-deriving it from process-wide
// state that another thread may have changed in between.
struct SwitchRecord {
  bool switched = false;
  bool bits = false;  // phase 0 stored its mapping-0 tiles' top bits (switch_bits_mode)
  uint32_t spread = 0, nint = 0, units = 0;
  uint32_t nseg = 0;  // matrix-core form: the column segments per object phase 0 ran with
};
struct BytesLaunch {
  uint8_t* slots;
  uint64_t slot_stride;
  uint64_t L;
  uint64_t S;  // object size in bytes (encode)
  uint32_t nobj, rows, k;
  int phase;
  const uint32_t* coeff;
  const uint32_t* in_idx;
  const uint32_t* out_idx;
  uint32_t* flags;  // encode: the caller's status array (flags, then fallback status)
  const uint32_t* mapping;
  uint64_t col0 = 0;   // column window [col0, col0 + ncols) of every chunk; col0 % 4 == 0
  uint64_t ncols = 0;  // 0: the whole chunk (L columns)
  // Mid-object mapping switch (encode_bytes_queue_kernel): device scratch of
  // encode_switch_bytes(a) bytes, or null.  Phase 0 with scratch records each
  // unit's mapping there and fills *sw (switched + its unit layout) when it
  // ran the switching kernel; phase 1 given the same scratch and record (only
  // if sw->switched) redoes just the units that used the wrong mapping.
  // Null: phase 1 re-encodes whole objects.
  uint8_t* scratch = nullptr;
  uint64_t scratch_bytes = 0;  // bytes at scratch: a layout that needs more runs without the record
  SwitchRecord* sw = nullptr;
  uint64_t cstride = 0;  // bytes between a slot's chunks (0: 4L, the wire layout)
  // Matrix-core form (rs_bytes_mfma.hip): the plan's byte-order digit table
  // or null, and the highest input / output chunk index.
  const uint8_t* mfma = nullptr;
  uint32_t in_max = 0, out_max = 0;
};
inline uint64_t chunk_stride(const BytesLaunch& a) { return a.cstride ? a.cstride : 4 * a.L; }
hipError_t launch_encode_bytes(const BytesLaunch& a, hipStream_t stream);
// Scratch bytes the mid-object switch needs for this launch; 0 when its
// phase 0 would not run the switching (dynamic-schedule) kernel.
uint64_t encode_switch_bytes(const BytesLaunch& a, hipStream_t stream);
uint64_t encode_switch_bytes_k32(const BytesLaunch& a, hipStream_t stream);
uint64_t encode_switch_bytes_mfma(const BytesLaunch& a);
// 17 <= need <= 32 through the pipelined k-template byte kernels (rs_bytes_k32.hip).
hipError_t launch_encode_bytes_k32(const BytesLaunch& a, hipStream_t stream);
hipError_t launch_decode_bytes_k32(const BytesLaunch& a, hipStream_t stream);

// Byte-kernel grid: about `target` resident 256-lane blocks over `work` object
// segments of ncols/nseg columns, U 16-byte units per lane per step.
inline dim3 bytes_grid(uint64_t ncols, uint64_t work, uint32_t nseg, uint64_t target = 512, int U = 1) {
  uint64_t gy = work < 65535u ? work : 65535u;
  if (gy < 1) gy = 1;
  uint64_t gx = (target + gy - 1) / gy;
  const uint64_t need = (ncols / nseg + 4ull * 256 * U - 1) / (4ull * 256 * U);
  if (gx > need) gx = need;
  if (gx < 1) gx = 1;
  return dim3((uint32_t)gx, (uint32_t)gy);
}
hipError_t launch_decode_bytes(const BytesLaunch& a, hipStream_t stream);
// Wide codes on the matrix cores (rs_bytes_mfma.hip): eligibility (table,
// mode, mfma_wanted -- for the encode only from need 25, below which the VALU
// queue encode's mid-object switch wins -- shape, chunk offsets under 4 GiB)
// and the launches.
bool bytes_mfma_eligible(const BytesLaunch& a, bool encode);
hipError_t launch_encode_bytes_mfma(const BytesLaunch& a, hipStream_t stream);
hipError_t launch_decode_bytes_mfma(const BytesLaunch& a, hipStream_t stream);
hipError_t launch_select_mapping(uint32_t* mapping, uint32_t* status, uint32_t nobj, hipStream_t stream);

// --- small host<->device transfers as one kernel (host_blit.hip) ----------
// dst/src: device addresses (device memory, or pinned host memory mapped
// into the device's address space); any alignment.
struct BlitSpan {
  void* dst;
  const void* src;
  uint64_t bytes;
};
constexpr int kBlitSpans = 32;  // spans per launch (larger lists take several)
hipError_t launch_blit(const BlitSpan* spans, int n, hipStream_t stream);

// --- byte <-> symbol codec (internal/rs/gf/map.go) -------------------------
// Pack len bytes big-endian into ceil(len/4) words (zero low bytes in a partial
// last word), XOR with `mapping`; words_out must hold ceil(len/4) words.
// Also OR-reduces two flags into *flags (device): bit0 = some packed word >= p,
// bit1 = some (word ^ 1<<31) >= p.  Pass flags == nullptr to skip.
hipError_t launch_map_pack(const uint8_t* bytes, uint64_t len, uint32_t mapping, uint32_t* words_out,
                           uint32_t* flags, hipStream_t stream);
// In-place XOR of n words with a mapping value.
hipError_t launch_xor_words(uint32_t* words, uint64_t n, uint32_t mapping, hipStream_t stream);
// For each of ncand candidate mappings, set bad[c] = 1 if some word ^ cand[c] >= p.
hipError_t launch_mapping_probe(const uint32_t* words, uint64_t n, const uint32_t* cand, uint32_t ncand,
                                uint32_t* bad, hipStream_t stream);
// Unpack n words (XOR mapping) to 4n big-endian bytes.
hipError_t launch_map_unpack(const uint32_t* words, uint64_t n, uint32_t mapping, uint8_t* bytes_out,
                             hipStream_t stream);

// Synthetic symbols for benchmarks/tests: word g = splitmix64-derived value
// reduced into [0, p), a pure function of (seed, g).
hipError_t launch_fill_symbols(uint32_t* dst, uint64_t n, uint64_t seed, hipStream_t stream);

}  // namespace slime
