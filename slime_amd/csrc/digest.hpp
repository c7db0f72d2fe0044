// Chunk and object digests of slime's store path:
// SHA-256 per chunk (store.DataV, internal/store/store.go:104-110, called per
// chunk by writeChunks at multi_store.go:554-556), SHA-256 per object
// (reconstruct's verify, multi_store.go:244-249) and the chunk file's
// FNV-1a-64 header over SHA-256 ‖ data (storedir/directory.go:25-28,548-553).
//
// These are host computations by design (DESIGN.md "Chunk digests"): SHA-256
// and FNV-1a are sequential per message, a GPU lane hashes one message at
// ~20 MB/s against ~2 GB/s for one x86 core with the SHA extensions, and a
// writeChunks call has `total` messages.  What the library adds is running
// them beside the device pipeline instead of after it.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>

namespace slime {

// Incremental SHA-256 (FIPS 180-4); the x86 SHA extensions when present.
class Sha256 {
 public:
  Sha256();
  void update(const void* data, size_t n);
  void final(uint8_t out[32]);

 private:
  uint32_t h_[8];
  uint8_t buf_[64];
  size_t buffered_ = 0;
  uint64_t total_ = 0;
};

// True when this CPU runs SHA-256 on its SHA extensions (else a portable loop).
bool sha_extensions();

// FNV-1a 64 (Go's hash/fnv New64a): h ^= byte; h *= 1099511628211, from h.
constexpr uint64_t kFnv64Offset = 0xcbf29ce484222325ull;
uint64_t fnv1a64(uint64_t h, const void* data, size_t n);

// Run fn(i) for every i in [0, n) on the digest pool, the caller included;
// returns when all have run.
void digest_parallel(size_t n, const std::function<void(size_t)>& fn);

struct DigestTask;
// fn(0..n-1) started on the digest pool at construction; wait() (or the
// destructor) claims what no worker has taken yet on the calling thread and
// returns when every index has run.  Tasks may block on work the caller does
// meanwhile (pipeline progress), as long as that work never waits for them.
class DigestJob {
 public:
  DigestJob(size_t n, std::function<void(size_t)> fn);
  ~DigestJob();
  void wait();
  DigestJob(const DigestJob&) = delete;
  DigestJob& operator=(const DigestJob&) = delete;

 private:
  std::unique_ptr<DigestTask> task_;
  bool waited_ = false;
};

// Digests of writeChunks' chunks (multi_store.go:554-556, storedir
// directory.go:548-553) computed while the device pipeline is still
// producing them.  Chunk j < need is the object's bytes [j*chunk, ...) up to
// `size`, zero bytes to the end of the object's last word, then BE(mapping)
// words (splitVector's padding through MapFromGF): its hash starts at once
// from `data` and finishes when the mapping is known.  Parity chunks are read
// from their buffers as the pipeline reports them final, front to back.
// sha_out: total x 32 bytes; hdr_out (optional): total x 8 bytes, the chunk
// file's FNV-1a-64 of SHA-256 ‖ chunk, big-endian.
class WriteChunkDigests {
 public:
  WriteChunkDigests(const uint8_t* data, uint64_t size, int need, int total, uint64_t chunk, uint8_t* const* chunks,
                    uint8_t* sha_out, uint8_t* hdr_out);
  ~WriteChunkDigests();  // abort() unless finish() ran
  // Parity chunks' bytes [0, bytes) are in their buffers (a later rewrite()
  // may still replace them).
  void parity_ready(uint64_t bytes);
  // Parity buffers are about to be rewritten: returns once no hasher reads
  // them; hashers start those chunks over from the next parity_ready().
  void parity_rewrite();
  // The mapping is final, and so are the parity bytes reported so far.
  void finalize(uint32_t mapping);
  void abort();  // the pipeline failed: hashers stop
  void finish(); // wait for every digest

 private:
  void run(size_t i);
  void data_chunk(int j, uint8_t* sha, uint8_t* hdr);
  void parity_chunk(int i, uint8_t* sha, uint8_t* hdr);
  void tail(int j, uint32_t m, const std::function<void(const uint8_t*, size_t)>& sink) const;

  const uint8_t* data_;
  uint64_t size_, chunk_;
  int need_;
  uint8_t* const* chunks_;
  uint8_t *sha_out_, *hdr_out_;
  std::mutex mu_;
  std::condition_variable cv_;
  uint64_t ready_ = 0, epoch_ = 0;
  int readers_ = 0;
  bool final_ = false, aborted_ = false;
  uint32_t mapping_ = 0;
  std::unique_ptr<DigestJob> job_;
};

// Threads of the digest pool besides the caller (env SLIME_RS_DIGEST_THREADS;
// default min(usable CPUs, 16) - 1).
int digest_threads();

}  // namespace slime
