// Host-only scalar GF(2^32-5) helpers for code-matrix construction (plain C++,
// no HIP types).  The device data path lives in gfp.hpp.
#pragma once
#include <stdint.h>

namespace slime {

constexpr uint32_t kP = 4294967291u;  // gf.MaxVal, internal/rs/gf/map.go:7

inline uint32_t mulmod(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) % kP); }
inline uint32_t addmod(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a + b) % kP); }

}  // namespace slime
