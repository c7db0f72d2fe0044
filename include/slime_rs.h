/*
 * slime_rs.h — C-ABI of the MI355X-native Reed-Solomon shard codec that
 * replaces encryptio/slime's internal/rs and internal/rs/gf (Go) behind their
 * unchanged Go API.  Field: GF(p), p = 2^32 - 5, 32-bit symbols
 * (internal/rs/doc.go:1-2, internal/rs/gf/map.go:7).
 *
 * Two layers:
 *   1. Go-API entry points (host memory in, host memory out).  Each one is
 *      what the cgo shim of the corresponding Go function binds (see
 *      INTEGRATION.md).  They validate exactly like the reference and return
 *      a status code; slime_rs_status_string() gives the reference's panic
 *      text, which the shim re-raises with panic().
 *   2. Device-resident batch API (new, additive): plans + layouts over
 *      objects already in HBM, launched on a caller-supplied hipStream_t.
 *      This is the hot path the benchmark measures.
 *
 * Every compute entry point runs on the GPU (HIP kernels for gfx950). There is
 * no CPU fallback: without a usable device they return SLIME_RS_ERR_NO_DEVICE.
 * Host-only entry points (matrix construction, gf scalars) need no device.
 * All functions are thread-safe.
 */
#ifndef SLIME_RS_H
#define SLIME_RS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes --------------------------------------------------------
 * Codes 1..8 correspond one-to-one to the reference's panics; the strings
 * returned by slime_rs_status_string() are the reference's exact messages. */
enum slime_rs_status {
  SLIME_RS_OK = 0,
  SLIME_RS_ERR_VARYING_LENGTH = 1, /* "CreateParity called on data chunks of varying length" vector.go:21 */
  SLIME_RS_ERR_LEN_MISMATCH = 2,   /* "RecoverData: len(chunks) != len(indices)"            vector.go:52 */
  SLIME_RS_ERR_EMPTY = 3,          /* "RecoverData: len(chunks) == 0"                       vector.go:56 */
  SLIME_RS_ERR_NO_INDICES = 4,     /* "RecoverData: No indices given"                       vector.go:66 */
  SLIME_RS_ERR_SINGULAR_NONZERO = 5, /* "Couldn't ensure nonzero m[i][i]"                   matrix.go:68 */
  SLIME_RS_ERR_SINGULAR_ONE = 6,   /* "Couldn't ensure one m[i][i]"                         matrix.go:77 */
  SLIME_RS_ERR_SINGULAR_ZERO = 7,  /* "Couldn't ensure zero m[i][j]"                        matrix.go:92 */
  SLIME_RS_ERR_INDEX_RANGE = 8,    /* Go runtime "index out of range" panic                  */
  SLIME_RS_ERR_INVALID_ARG = 9,    /* C-ABI misuse (null pointer, bad shape)                  */
  SLIME_RS_ERR_NO_DEVICE = 10,     /* no usable HIP device: compute calls fail loudly         */
  SLIME_RS_ERR_HIP = 11,           /* HIP runtime error (detail in slime_rs_last_error())     */
  SLIME_RS_ERR_MAPPING_FALLBACK = 12, /* no candidate mapping fits (only with a bounded search) */
  SLIME_RS_ERR_BAD_HASH = 13       /* "bad checksum after reconstruction" (ErrBadHash) multi_store.go:26,244-249 */
};

/* Reference panic message (codes 1..8) or a short description. Static storage. */
const char *slime_rs_status_string(int status);
/* Detail of the last failure on the calling thread ("" if none).  Meaningful
 * only on the thread that made the failing call, before its next call: the
 * *_ex forms return the detail of the call itself instead. */
const char *slime_rs_last_error(void);
/* Library version string. */
const char *slime_rs_version(void);
/* Number of visible HIP devices (0 without a GPU; never fails). */
int slime_rs_device_count(void);

/* Device of a host-memory entry point (CreateParity ... reconstruct, the
 * MapToGF codec).  SLIME_RS_ANY_DEVICE: the library's device pool picks the
 * visible GPU with the fewest calls in flight (ties round-robin), so
 * concurrent callers spread over every GPU of the node (objects are
 * independent: no data exchange between GPUs). */
#define SLIME_RS_ANY_DEVICE (-1)
/* Pin the calling OS thread's host entry points to `device`
 * (SLIME_RS_ANY_DEVICE, the default, returns them to the pool).  Thread-local:
 * callers whose threads migrate between calls (Go) use the *_ex forms. */
int slime_rs_select_device(int device);
/* The calling thread's selection (SLIME_RS_ANY_DEVICE if none): lets a scope
 * that selects a device restore the one it found. */
int slime_rs_selected_device(void);

/* Per-call context of the *_ex entry points, for callers that must not depend
 * on thread-local state between calls (cgo: a goroutine may run consecutive
 * C calls on different OS threads, and concurrent goroutines share threads).
 * Replaces, for these callers, slime_rs_select_device and
 * slime_rs_last_error. */
typedef struct slime_rs_call {
  int device;        /* device ordinal, or SLIME_RS_ANY_DEVICE (the pool picks) */
  char *detail;      /* optional: receives this call's failure detail, NUL-terminated ("" on success) */
  size_t detail_cap; /* bytes at detail (0: no detail wanted) */
} slime_rs_call_t;
/* Kernel form for shards/chunks under 4 GiB (process-wide): 1 =
 * software-pipelined kernels (default), 0 = the non-pipelined forms that
 * larger shards always take.  mode < 0 queries.  Results are identical; the
 * parity tests run both. */
int slime_rs_kernel_pipeline(int mode);
/* Work schedule of the pipelined kernels for k <= 32 (process-wide): 1 =
 * dynamic, waves take units
 * of work from ticket counters, except inside a graph capture, where the
 * static kernels are captured (default); 2 = dynamic inside captures too --
 * the captured launch keeps a counter set for the graph's life (returned to
 * the library when the graph and its execs are destroyed), so a graph holding
 * one must not be replayed by two execs at the same time; 0 = static shares
 * per wave.  mode < 0 queries.  Results are identical; the parity tests run
 * every mode. */
int slime_rs_kernel_schedule(int mode);
/* Wide codes (k >= 33, or 17 <= k <= 32 with k x rows >= 128; up to 32 output
 * rows and k <= 112) on the matrix cores (process-wide): 1 = the exact
 * int8-limb kernel on v_mfma_i32_16x16x64_i8 (default), 0 = the VALU kernels.
 * mode < 0 queries.  Results are identical; the parity tests run both. */
int slime_rs_kernel_matrix_cores(int mode);
/* Second pass of the fused byte encode (writeChunks on device) for need <= 10
 * (process-wide).  The first pass assumes MapToGF's mapping 0; the units it
 * encoded before an object's first word >= p must be redone with 1<<31.
 * 0 = by object size (default): objects of 1 GiB and more (uniform bytes
 * switch in 27% of them) have the first pass also store each mapping-0
 * column's need top bits (need/8 bytes a column of device scratch), and the
 * second pass corrects those units' parity from the bits and the parity
 * itself instead of re-reading the data; smaller objects re-encode the units.
 * 1 = always correct, 2 = always re-encode.  mode < 0 queries.  Results are
 * identical; the parity tests run every mode. */
int slime_rs_switch_bits(int mode);

/* ==== internal/rs/gf ===================================================== */

/* gf.MaxVal = 1<<32 - 5  (internal/rs/gf/map.go:7) */
#define SLIME_GF_MAXVAL 4294967291u
uint32_t slime_gf_max_val(void);
/* gf.MInverse (internal/rs/gf/gf.go:5): in^(p-2) mod p. Host-only. */
uint32_t slime_gf_minverse(uint32_t in);
/* gf.Raise (internal/rs/gf/gf.go:46): x^n mod p, Raise(x,0) = 1. Host-only. */
uint32_t slime_gf_raise(uint32_t x, uint32_t n);

/* gf.MapToGF (internal/rs/gf/map.go:15).  out must hold (len+3)/4 words.
 * Mapping 0 if every big-endian word is < p, else 1<<31 if that fits, else
 * the first fitting value from the library's random candidate stream (the
 * reference draws rand.Uint32(); see slime_gf_seed).  Host memory: runs on
 * the host cores where the bytes are (slime_gf_codec_placement). */
int slime_gf_map_to_gf(const uint8_t *in, uint64_t len, uint32_t *mapping, uint32_t *out);
/* gf.MapToGFWith (internal/rs/gf/map.go:74). out holds (len+3)/4 words. */
int slime_gf_map_to_gf_with(const uint8_t *in, uint64_t len, uint32_t n, uint32_t *out);
/* gf.MapFromGF (internal/rs/gf/map.go:103). out holds 4*count bytes. */
int slime_gf_map_from_gf(uint32_t n, const uint32_t *in, uint64_t count, uint8_t *out);
/* Where the three host-memory codec calls above run (process-wide): 0 = on
 * the host cores, in
 * place on the caller's buffers (AVX2 passes split over the library's copy
 * pool; default -- the codec is a byte swap, an XOR and a compare, and the
 * bytes are in host memory); 1 = through the GPU codec kernels and the pinned
 * staging ring (two PCIe crossings per call).  Device-resident buffers and
 * the fused object entry points always use the GPU codec.  mode < 0 queries.
 * Results are identical; the parity tests run both. */
int slime_gf_codec_placement(int mode);
/* The host codec's instruction set ("avx2" or "scalar"; env
 * SLIME_RS_CODEC_ISA=scalar forces the portable form) and the threads its
 * passes use (the library's copy pool plus the calling thread). */
int slime_gf_codec_info(const char **isa, int *threads);
/* Seed the MapToGF fallback candidate stream (default: std::random_device,
 * like the reference's crypto-seeded math/rand, main.go:128-136). */
void slime_gf_seed(uint64_t seed);

/* ==== internal/rs: matrices (host-only, exact) =========================== */

/* vandermondeMatrix (internal/rs/matrix.go:8): out is (d+p) x d row-major. */
int slime_rs_vandermonde_matrix(int d, int p, uint32_t *out);
/* ParityMatrix (internal/rs/matrix.go:27): out is (d+p) x d row-major. */
int slime_rs_parity_matrix(int d, int p, uint32_t *out);
/* ParityMatrixCached (internal/rs/matrixcache.go:11): *out points at a shared,
 * read-only (d+p) x d matrix that lives for the life of the process. */
int slime_rs_parity_matrix_cached(int d, int p, const uint32_t **out);
/* solveSubIdentity (internal/rs/matrix.go:35), in place on rows x cols. */
int slime_rs_solve_sub_identity(uint32_t *m, int rows, int cols);
/* invertMatrix (internal/rs/matrix.go:112): inv = m^-1, both d x d. */
int slime_rs_invert_matrix(const uint32_t *m, int d, uint32_t *inv);

/* ==== internal/rs: Go-API data entry points (host memory, GPU compute) ===== */

/* CreateParity (internal/rs/vector.go:18).  data[i] points at lens[i] words;
 * out receives lens[0] words (the shim handles Go's `out` reuse rule). */
int slime_rs_create_parity(const uint32_t *const *data, const uint64_t *lens, int ndata, int index,
                           uint32_t *out);
/* All total-ndata parity rows in one pass (the batched form of the
 * reference's per-row loop, multi_store.go:528-531): out[i] receives row
 * ndata+i, each lens[0] words. */
int slime_rs_create_parities(const uint32_t *const *data, const uint64_t *lens, int ndata, int total,
                             uint32_t *const *out);
/* RecoverData (internal/rs/vector.go:50).  chunks[i] has lens[i] words and
 * code-row index indices[i]; out[0..nchunks-1] each receive lens[0] words of
 * data rows 0..nchunks-1.  Only the erased data rows (those not among
 * indices) are computed on the GPU; a surviving data row's inverse row is a
 * unit row, so its output is that chunk mod p, written on the host.  Output
 * rows may overlap the chunks (an in-place repair): survivors an output
 * overlaps are read from copies taken first. */
int slime_rs_recover_data(const uint32_t *const *chunks, const uint64_t *lens, int nchunks, const int *indices,
                          int nindices, uint32_t *const *out);

/* ==== device-resident batch API (hot path) =============================== */

/* Symbol layout of a batch of objects in device memory: shard s of object o
 * starts at base + o*obj_stride + s*shard_stride (uint32 elements). */
typedef struct slime_rs_layout {
  uint64_t obj_stride;
  uint64_t shard_stride;
} slime_rs_layout_t;

typedef struct slime_rs_plan *slime_rs_plan_t;

/* Encode: inputs = src shards 0..need-1, outputs = parity rows need..total-1
 * written to dst shards 0..total-need-1. */
int slime_rs_plan_encode(int device, int need, int total, slime_rs_plan_t *plan);
/* Reconstruct: inputs = src shards have[0..need-1] (code-row indices of the
 * survivors, any order, distinct), outputs = code rows want[0..nwant-1]
 * (data rows < need, or parity rows) written to dst shards 0..nwant-1.
 * Bit-identical to RecoverData (+CreateParity for parity targets). */
int slime_rs_plan_reconstruct(int device, int need, int total, const int *have, const int *want, int nwant,
                              slime_rs_plan_t *plan);
/* Arbitrary rows x k coefficient matrix (host, row-major) applied to src
 * shards in_shards[0..k-1], written to dst shards 0..rows-1. */
int slime_rs_plan_matrix(int device, const uint32_t *coeff, int rows, int k, const int *in_shards,
                         slime_rs_plan_t *plan);
/* Launch the plan over nobj objects of L symbols per shard.  src and dst are
 * device pointers on the plan's device; stream is a hipStream_t (NULL = the
 * null stream).  Asynchronous; capturable into a hipGraph. */
int slime_rs_plan_execute(slime_rs_plan_t plan, const uint32_t *src, slime_rs_layout_t src_layout, uint32_t *dst,
                          slime_rs_layout_t dst_layout, uint64_t L, uint64_t nobj, void *stream);
/* Write output row i to dst shard out_shards[i] instead of shard i (e.g. a
 * repair that writes rebuilt shards back into their erased slots of the
 * source layout, which is also the faster placement on MI355X: DESIGN.md).
 * Only before the plan's first launch (SLIME_RS_ERR_INVALID_ARG after it:
 * launches in flight read the table). */
int slime_rs_plan_set_outputs(slime_rs_plan_t plan, const int *out_shards);
/* Shape of a plan: rows written and inputs read per column. */
int slime_rs_plan_shape(slime_rs_plan_t plan, int *rows, int *k);
/* Host copy of the plan's coefficient rows (rows x k, row-major). */
int slime_rs_plan_coefficients(slime_rs_plan_t plan, uint32_t *out);
int slime_rs_plan_destroy(slime_rs_plan_t plan);

/* ==== fused byte-domain object pipeline (writeChunks / reconstruct on device) ====
 * Object slots: object o's slot starts at slots + o*slot_stride bytes and holds
 * its `total` chunks of 4L bytes (chunk c at slot + c*4L, L = ceil(ceil(S/4)/need),
 * multi_store.go:272).  The object's S bytes are the first S bytes of its slot,
 * so the data chunks are in place: after encoding, chunk c of the slot is
 * exactly MapFromGF(mapping, part c) (multi_store.go:526-554).  Any need (k > 16
 * runs the 16-chunk byte kernels). */

/* Encode nobj objects of S bytes: mapping[o] receives gf.MapToGF's choice
 * (map.go:35-62) and status[o] = 1 marks an object that needs MapToGF's random
 * fallback (map.go:64-66; its chunks are not final until
 * slime_rs_resolve_fallbacks).  mapping/status are device arrays of nobj
 * words.  Speculative single pass (mapping 0) plus a re-encode pass only for
 * objects whose mapping is 1<<31.  Asynchronous. */
int slime_rs_encode_objects(slime_rs_plan_t encode_plan, uint8_t *slots, uint64_t slot_stride, uint64_t object_size,
                            uint64_t nobj, uint32_t *mapping, uint32_t *status, void *stream);
/* Synchronous: for each object with status 1, draw random mapping candidates
 * (64 per device pass) until one fits, store it in mapping[o], clear status[o]
 * and re-encode the object.  *resolved (optional) = objects fixed. */
int slime_rs_resolve_fallbacks(slime_rs_plan_t encode_plan, uint8_t *slots, uint64_t slot_stride,
                               uint64_t object_size, uint64_t nobj, uint32_t *mapping, uint32_t *status, void *stream,
                               int *resolved);
/* Rebuild chunks from `need` surviving chunks of each slot: a reconstruct plan
 * whose inputs are the survivors' chunk indices and whose outputs
 * (slime_rs_plan_set_outputs) are the chunk slots to write.  mapping[o] is the
 * object's mapping value (meta.File.MappingValue).  Asynchronous. */
int slime_rs_decode_objects(slime_rs_plan_t reconstruct_plan, uint8_t *slots, uint64_t slot_stride, uint64_t L,
                            uint64_t nobj, const uint32_t *mapping, void *stream);
/* The same three over a slot layout whose chunks are chunk_stride bytes apart
 * (chunk c at slot + c*chunk_stride; chunk_stride >= 4L, a multiple of 4; 0
 * selects 4L, the forms above).  Object byte i then lives in chunk i / 4L at
 * offset i % 4L: the device-resident layout the caller fills chunk by chunk
 * (e.g. 256 B-aligned chunk_stride, every chunk on a line boundary). */
int slime_rs_encode_objects_chunked(slime_rs_plan_t encode_plan, uint8_t *slots, uint64_t slot_stride,
                                    uint64_t chunk_stride, uint64_t object_size, uint64_t nobj, uint32_t *mapping,
                                    uint32_t *status, void *stream);
int slime_rs_resolve_fallbacks_chunked(slime_rs_plan_t encode_plan, uint8_t *slots, uint64_t slot_stride,
                                       uint64_t chunk_stride, uint64_t object_size, uint64_t nobj, uint32_t *mapping,
                                       uint32_t *status, void *stream, int *resolved);
int slime_rs_decode_objects_chunked(slime_rs_plan_t reconstruct_plan, uint8_t *slots, uint64_t slot_stride,
                                    uint64_t chunk_stride, uint64_t L, uint64_t nobj, const uint32_t *mapping,
                                    void *stream);
/* encode_objects_chunked that also records the hipEvent_t `phase_event` (may be
 * null) on `stream` between its two passes: after the speculative pass and the
 * mapping selection, before the re-encode of the objects mapped with 1<<31 --
 * so a caller can time the re-encode's share of the call.  A call with nothing
 * to encode (nobj or the object size 0) records nothing. */
int slime_rs_encode_objects_phased(slime_rs_plan_t encode_plan, uint8_t *slots, uint64_t slot_stride,
                                   uint64_t chunk_stride, uint64_t object_size, uint64_t nobj, uint32_t *mapping,
                                   uint32_t *status, void *stream, void *phase_event);

/* ---- Object entry points over host memory (the callers' data paths) ----
 *
 * Byte length of every chunk of a `size`-byte object split `need` ways:
 * 4 * ceil(ceil(size/4) / need)  (splitVector, multi_store.go:271-278). */
uint64_t slime_rs_chunk_size(uint64_t size, int need);

/* The data path of Multi.writeChunks (multi_store.go:526-531 and :554):
 *   mapping, all := gf.MapToGF(data); parts := splitVector(all, need);
 *   parity i := rs.CreateParity(parts, need+i, nil); chunk i := gf.MapFromGF(mapping, part i)
 * in one device pass (fused byte kernels) with pinned, overlapped transfers.
 * chunks[0..total-1] each receive slime_rs_chunk_size(size, need) bytes;
 * *mapping receives MappingValue.  The random-mapping fallback draws from the
 * library's stream (slime_gf_seed).  need >= 1 and total >= need (total ==
 * need: a store without parity, multi_config.go:36); size 0 gives mapping 0
 * and empty chunks.  Zero-copy data chunks: chunks[j] (j < need) may be
 * data + j*chunk_size when that chunk lies wholly inside the object; its bytes
 * are then already final and are not copied.  Any other overlap between a
 * chunk buffer and data is refused (SLIME_RS_ERR_INVALID_ARG).  Synchronous;
 * thread-safe. */
int slime_rs_write_chunks(const uint8_t *data, uint64_t size, int need, int total, uint8_t *const *chunks,
                          uint32_t *mapping);

/* The slow path of Multi.reconstruct (multi_store.go:215-241): the first
 * `need` available chunks (chunk_bytes each; a length that is not a multiple
 * of 4 is zero-padded to whole words as MapToGFWith does) with their
 * chunk indices, and the file's MappingValue -> the object's `size` bytes in
 * out:  chunk := MapToGFWith(data, mapping); RecoverData(chunks, indices);
 * MapFromGF each data row; data[:size].  Same panics as RecoverData for bad
 * indices.  Bytes past need*chunk_bytes are zero, as
 * in the reference's data[:Size] of a zeroed buffer.  Synchronous. */
int slime_rs_reconstruct(const uint8_t *const *chunks, const int *indices, int need, uint64_t chunk_bytes,
                         uint32_t mapping, uint64_t size, uint8_t *out);

/* Device codec (internal/rs/gf/map.go) over device buffers, asynchronous on
 * `stream`.  pack: words[i] = BE(bytes[4i..4i+3]) ^ mapping (zero low bytes
 * in a partial last word); if flags != NULL it is OR-ed with bit0 = some
 * unmapped word >= p, bit1 = some (word ^ 1<<31) >= p  (MapToGF's choice).
 * unpack: bytes = BE(words[i] ^ mapping). */
int slime_gf_pack_device(int device, const uint8_t *bytes, uint64_t len, uint32_t mapping, uint32_t *words,
                         uint32_t *flags, void *stream);
int slime_gf_unpack_device(int device, const uint32_t *words, uint64_t count, uint32_t mapping, uint8_t *bytes,
                           void *stream);

/* Device batch buffers (MI355X; no reference counterpart: the Go path works in
 * host memory).  A hipMalloc'd batch of tens of GiB lands, allocation by
 * allocation, in one of two physical placements, and the apply kernels stream
 * about 13% slower from the bad one (DESIGN.md "Placement modes").  This allocator
 * builds the buffer from physical chunks (HIP virtual memory: hipMemCreate,
 * mapped in order into one reserved virtual range): 2 MiB-chunk buffers landed
 * in the slow placement in 1 of 58 trials, hipMalloc'd ones in 36 of 98
 * (DESIGN.md "the allocator changes the odds").  `bytes` is
 * rounded up to the chunk size (env SLIME_RS_VMM_CHUNK_MIB, default 2 MiB);
 * *ptr receives a base usable by every device entry point.  Synchronous.
 * Returns 0, SLIME_RS_ERR_INVALID_ARG, SLIME_RS_ERR_NO_DEVICE or
 * SLIME_RS_ERR_HIP (out of memory). */
int slime_rs_device_alloc(int device, uint64_t bytes, void **ptr);
/* How a slime_rs_device_alloc buffer was placed.  Buffers of at least
 * SLIME_RS_PLACEMENT_PROBE_GIB GiB (default 16; 0 disables) are probed when
 * created: the apply kernel's C3-shaped read/write walk over the whole buffer
 * (GB/s of algorithmic traffic).  Below SLIME_RS_PLACEMENT_MIN_GBS (default
 * 6350, the top of the rates seen, so in practice always) the allocator tries
 * up to two other placements (1 GiB chunks, then one hipMalloc), holding the
 * first meanwhile, and keeps the fastest (DESIGN.md "Placement"). */
typedef struct slime_rs_alloc_info {
  int kind;                /* kept placement: 0 = physical chunks mapped into one range, 1 = hipMalloc */
  int probes;              /* placements probed (0: buffer too small, not probed) */
  int chosen;              /* index into probe_* of the kept placement */
  uint64_t chunk_bytes;    /* kept placement's chunk size (0 for hipMalloc) */
  double probe_gbs[4];     /* each probed placement's rate */
  uint64_t probe_chunk[4]; /* each probed placement's chunk size (0: hipMalloc) */
} slime_rs_alloc_info_t;
int slime_rs_device_alloc_info(const void *ptr, slime_rs_alloc_info_t *info);
/* The same placement probe over a caller's own device range [ptr, ptr+bytes)
 * on `device` (e.g. a hipMalloc'd or torch batch buffer): *gbs = GB/s of
 * algorithmic traffic of the C3-shaped read/write walk, 0 when the range is
 * too small to measure (under ~400 MB).  The physical placement of a large
 * buffer fixes, for its whole life, whether the kernels stream in the fast
 * mode (~6.0-6.4 TB/s at C3) or the slow one (~5.3-5.7): a buffer that
 * probes in the slow mode is worth re-allocating, or allocating with
 * slime_rs_device_alloc, which probes and re-places by itself.
 * OVERWRITES the range: probe a buffer before filling it.  The range must lie
 * inside one device allocation on `device` (else SLIME_RS_ERR_INVALID_ARG).
 * Synchronous. */
int slime_rs_probe_placement(void *ptr, uint64_t bytes, int device, double *gbs);
/* The allocator's re-placement threshold, GB/s (env SLIME_RS_PLACEMENT_MIN_GBS,
 * default 6350: a first placement below it is re-placed, keeping the fastest
 * of up to three; 6350 is about the C3 apply kernel at 8.2 ms). */
double slime_rs_placement_threshold(void);
/* Frees a buffer from slime_rs_device_alloc (its base).  Waits for the device
 * first (hipDeviceSynchronize), so work still queued on it cannot fault.
 * Returns SLIME_RS_ERR_INVALID_ARG for other pointers. */
int slime_rs_device_free(void *ptr);

/* Deterministic synthetic symbols (benchmarks/tests): word g of the buffer is
 * a pure function of (seed, g), uniform over [0, p). Asynchronous. */
int slime_rs_fill_symbols(int device, uint32_t *dst, uint64_t count, uint64_t seed, void *stream);

/* ==== *_ex forms: the entry points above with a per-call context ==========
 * Same arguments and results as the plain forms; `call` gives the device and
 * receives this call's failure detail (see slime_rs_call_t).  These are what
 * the cgo shim binds. */
int slime_rs_create_parity_ex(const slime_rs_call_t *call, const uint32_t *const *data, const uint64_t *lens,
                              int ndata, int index, uint32_t *out);                       /* vector.go:18 */
int slime_rs_create_parities_ex(const slime_rs_call_t *call, const uint32_t *const *data, const uint64_t *lens,
                                int ndata, int total, uint32_t *const *out);              /* multi_store.go:528-531 */
int slime_rs_recover_data_ex(const slime_rs_call_t *call, const uint32_t *const *chunks, const uint64_t *lens,
                             int nchunks, const int *indices, int nindices, uint32_t *const *out); /* vector.go:50 */
int slime_rs_write_chunks_ex(const slime_rs_call_t *call, const uint8_t *data, uint64_t size, int need, int total,
                             uint8_t *const *chunks, uint32_t *mapping);                  /* multi_store.go:526-554 */
int slime_rs_reconstruct_ex(const slime_rs_call_t *call, const uint8_t *const *chunks, const int *indices, int need,
                            uint64_t chunk_bytes, uint32_t mapping, uint64_t size, uint8_t *out); /* :215-241 */
int slime_gf_map_to_gf_ex(const slime_rs_call_t *call, const uint8_t *in, uint64_t len, uint32_t *mapping,
                          uint32_t *out);                                                 /* map.go:15 */
int slime_gf_map_to_gf_with_ex(const slime_rs_call_t *call, const uint8_t *in, uint64_t len, uint32_t n,
                               uint32_t *out);                                            /* map.go:74 */
int slime_gf_map_from_gf_ex(const slime_rs_call_t *call, uint32_t n, const uint32_t *in, uint64_t count,
                            uint8_t *out);                                                /* map.go:103 */
int slime_rs_parity_matrix_ex(const slime_rs_call_t *call, int d, int p, uint32_t *out);  /* matrix.go:27 */
int slime_rs_vandermonde_matrix_ex(const slime_rs_call_t *call, int d, int p, uint32_t *out); /* matrix.go:8 */
int slime_rs_solve_sub_identity_ex(const slime_rs_call_t *call, uint32_t *m, int rows, int cols); /* matrix.go:35 */
int slime_rs_invert_matrix_ex(const slime_rs_call_t *call, const uint32_t *m, int d, uint32_t *inv); /* matrix.go:112 */

/* ==== plan cache and device pool (host entry points) =====================
 * Host entry points keep their device plans (coefficient tables; recovery
 * plans keyed by survivor set, reference: vector.go:69-77) in one bounded LRU
 * per process (default 256 plans, env SLIME_RS_PLAN_CACHE).  An evicted plan
 * releases its device table once no call in flight still uses it. */
typedef struct slime_rs_cache_stats {
  uint64_t live;          /* plans cached now (<= capacity) */
  uint64_t capacity;
  uint64_t hits, misses, evictions;
  uint64_t device_tables; /* plan tables allocated on devices and not yet freed (all plans, cached or not) */
} slime_rs_cache_stats_t;
int slime_rs_plan_cache_stats(slime_rs_cache_stats_t *stats);
/* Set the cache capacity (>= 1); shrinking evicts at once. */
int slime_rs_plan_cache_capacity(uint64_t capacity);
/* Where the host entry points' windowed pipeline spends its wall time (all
 * threads, since the start or the last reset; microseconds): copy_in = host
 * copies into pinned staging, enqueue = DMA/kernel launches, wait = waiting
 * for a stage's transfers and kernels (device and link side), copy_out = host
 * copies out of pinned staging.  reset != 0 zeroes the counters after reading. */
typedef struct slime_rs_host_stats {
  uint64_t calls, windows;
  uint64_t copy_in_us, enqueue_us, wait_us, copy_out_us, total_us;
} slime_rs_host_stats_t;
int slime_rs_host_stats(slime_rs_host_stats_t *stats, int reset);
/* Host calls the device pool has routed to `device` so far and calls in flight there. */
int slime_rs_pool_calls(int device, uint64_t *calls, int *inflight);
/* Host calls (the data entry points over host memory) that run at once in
 * this process: half its usable CPUs (affinity mask capped by the cgroup CPU
 * quota), at least 4.  Further callers wait, asleep, for a slot -- more calls
 * than CPUs only time-slice, and a process over its CPU quota is throttled
 * as a whole. */
int slime_rs_host_call_slots(void);
/* Ticket-counter sets of the dynamic-schedule kernels on `device`: *sets
 * allocated so far, *held by launches not yet known to have finished plus
 * those owned by captured graphs.  A set is reused by any stream once its
 * launch has finished (each launch leaves its set zero; DESIGN.md "Dynamic
 * schedule"). */
int slime_rs_ticket_sets(int device, uint64_t *sets, uint64_t *held);
/* Launches on `device` since start that ran the dynamic schedule on a counter
 * set, and that asked for one and were sent to the static kernels instead
 * (no set to be had) -- diagnostics and tests.  Launches the mode itself
 * keeps on the static kernels (mode 0, captures under mode 1) count in
 * neither. */
int slime_rs_schedule_counts(int device, uint64_t *dynamic, uint64_t *fallback);

/* ==== chunk and object digests ======================
 * Host computations on the library's digest threads (DESIGN.md "Chunk
 * digests"): SHA-256 and FNV-1a are sequential per message, so one x86 core
 * with the SHA extensions outruns a GPU lane ~100x; what the library adds is
 * hashing writeChunks' chunks while its device pipeline still runs. */

/* SHA-256 of len bytes (sha256.Sum256 as store.DataV uses it,
 * internal/store/store.go:104-110, and reconstruct's verify, multi_store.go:244). */
int slime_rs_sha256(const uint8_t *data, uint64_t len, uint8_t *out /* 32 bytes */);

/* For each of n chunks (lens[i] bytes): sha[32i..] = SHA-256 of the chunk
 * (store.DataV per chunk, multi_store.go:554-556) and, if hdr != NULL,
 * hdr[8i..] = the chunk file's header hash: FNV-1a-64 over SHA-256 ‖ chunk,
 * big-endian as hash.Sum appends it (storedir/directory.go:25-28,548-553).
 * Chunks are hashed in parallel, one per digest thread. */
int slime_rs_chunk_digests(const uint8_t *const *chunks, const uint64_t *lens, uint32_t n, uint8_t *sha,
                           uint8_t *hdr);

/* slime_rs_write_chunks plus every chunk's digests as slime_rs_chunk_digests
 * gives them (sha: total x 32 bytes; hdr optional, total x 8), computed while
 * the device pipeline runs: data chunks are hashed from `data` at once and
 * finished when the mapping is known, parity chunks as their windows land in
 * the caller's buffers.  Replaces writeChunks' per-chunk goroutines'
 * MapFromGF + store.DataV (multi_store.go:552-557). */
int slime_rs_write_chunks_digest(const uint8_t *data, uint64_t size, int need, int total, uint8_t *const *chunks,
                                 uint32_t *mapping, uint8_t *sha, uint8_t *hdr);

/* slime_rs_reconstruct, then the object's SHA-256 against want_sha (the
 * file's SHA256, multi_store.go:244-249): SLIME_RS_ERR_BAD_HASH on mismatch
 * (out holds the rebuilt bytes either way). */
int slime_rs_reconstruct_verify(const uint8_t *const *chunks, const int *indices, int need, uint64_t chunk_bytes,
                                uint32_t mapping, uint64_t size, uint8_t *out, const uint8_t *want_sha);

/* Whether SHA-256 runs on the CPU's SHA extensions, and the digest threads
 * besides the caller (env SLIME_RS_DIGEST_THREADS). */
int slime_rs_digest_info(int *sha_extensions, int *threads);

int slime_rs_write_chunks_digest_ex(const slime_rs_call_t *call, const uint8_t *data, uint64_t size, int need,
                                    int total, uint8_t *const *chunks, uint32_t *mapping, uint8_t *sha,
                                    uint8_t *hdr);
int slime_rs_reconstruct_verify_ex(const slime_rs_call_t *call, const uint8_t *const *chunks, const int *indices,
                                   int need, uint64_t chunk_bytes, uint32_t mapping, uint64_t size, uint8_t *out,
                                   const uint8_t *want_sha);

#ifdef __cplusplus
}
#endif
#endif /* SLIME_RS_H */
