// Internal helpers shared by the C-ABI translation units (rs_capi.cpp,
// device_alloc.cpp): the calling thread's failure detail behind the status
// codes of include/slime_rs.h, HIP error mapping and device checks.
#pragma once
#include <hip/hip_runtime.h>

#include <string>

#include "rs_matrix.hpp"  // Status

namespace slime {

// Record `detail` as the calling thread's failure detail (slime_rs_last_error,
// or the active *_ex call's buffer) and return the status code.
int fail(Status st, std::string detail);
int fail_hip(hipError_t e, const char* what);
// Visible HIP devices (counted once); check_device: 0, or NoDevice /
// InvalidArg with a detail.
int visible_devices();
int check_device(int dev);

// Switch the calling thread to `dev` for the scope, restoring its previous device.
struct DeviceScope {
  int prev = -1;
  explicit DeviceScope(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceScope() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

}  // namespace slime

#define HIP_TRY(expr)                                         \
  do {                                                        \
    const hipError_t e_ = (expr);                             \
    if (e_ != hipSuccess) return ::slime::fail_hip(e_, #expr); \
  } while (0)
