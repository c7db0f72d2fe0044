// The byte<->symbol codec of internal/rs/gf (map.go) over HOST memory.
//
// gf.MapToGF / MapToGFWith / MapFromGF are byte swaps, an XOR and a compare
// against p: the Go API's host-memory calls run them where the bytes already
// are, on the host copy pool (host_copy.hpp), instead of shipping every byte
// over PCIe and back.  The device codec (gf_codec.hip, rs_bytes_kernel.hpp)
// stays the codec of device-resident buffers and of the fused object passes.
// AVX2 where the CPU has it, scalar otherwise; pieces of 512 KiB of words run
// in parallel.  CPU-testable: tests/cpp/host_codec_test.cpp.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace slime {

// MapToGF's word packing (map.go:16-33) of `len` bytes into (len+3)/4 words,
// XOR n (map.go:94-96): out[i] = BE32(in[4i..4i+3]) ^ n, a partial last word
// with its bytes in the high positions and zero low bytes.  With flags
// non-null (n must be 0): *flags |= 1 if some word is >= p (mapping 0 does
// not fit, map.go:35-45), |= 2 if some word ^ (1<<31) is >= p (map.go:47-56).
void host_pack(const uint8_t* in, uint64_t len, uint32_t n, uint32_t* out, uint32_t* flags);

// MapFromGF (map.go:103-113): out[4i..4i+3] = BE32(in[i] ^ n).
void host_unpack(const uint32_t* in, uint64_t count, uint32_t n, uint8_t* out);

// w[i] ^= n, in place (MapToGF's final XOR with the chosen mapping, map.go:57-60).
void host_xor(uint32_t* w, uint64_t count, uint32_t n);

// Whether every w[i] ^ n is < p (one probe of MapToGF's candidate loop, map.go:48-56).
bool host_mapping_fits(const uint32_t* w, uint64_t count, uint32_t n);

// out[i] = in[i] mod p: a RecoverData output row whose inverse row is a unit
// row (a surviving data shard: applyMatrix's ((x*1)%p + 0)%p, vector.go:97).
void host_mod_p(const uint32_t* in, uint64_t count, uint32_t* out);

// Which instruction set the codec runs ("avx2" or "scalar").
const char* host_codec_isa();

}  // namespace slime
