// Shared helpers for the HIP native module (gfx950 / MI355X only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdexcept>
#include <string>

#define HIP_CHECK(expr)                                                                 \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess)                                                               \
      throw std::runtime_error(std::string(#expr " failed: ") + hipGetErrorString(_e)); \
  } while (0)

namespace gs {
constexpr int kWave = 64;
constexpr int kXcds = 8;
constexpr int kCus = 256;
}  // namespace gs
