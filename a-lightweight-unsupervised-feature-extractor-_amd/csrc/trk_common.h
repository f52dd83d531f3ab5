// Shared helpers for the gfx950 tracker kernels (C-ABI error plumbing, bf16).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>

#include "../../include/trk_amd.h"

namespace trk {

void set_error(const char* fmt, ...);

// Report the first launch error of the preceding kernel; 0 if clean.
int check_launch(const char* what);

#define TRK_REQUIRE(cond, ...)            \
  do {                                    \
    if (!(cond)) {                        \
      ::trk::set_error(__VA_ARGS__);      \
      return TRK_EINVAL;                  \
    }                                     \
  } while (0)

// Round-to-nearest-even f32 -> bf16 (NaN stays NaN: MI355X_MICROARCH.md
// correctness table; hipcc lowers the plain conversion to v_cvt_pk_bf16_f32).
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  __hip_bfloat16 h = __float2bfloat16(f);
  return *reinterpret_cast<uint16_t*>(&h);
}

// two floats -> packed bf16 pair (a in the low half), round to nearest even: one
// v_cvt_pk_bf16_f32 (two f32_to_bf16 + shift/or compile to two conversions and a merge)
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack2_bf16(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_t{a, b}, bf16x2_t));
}

constexpr int kWave = 64;

inline bool aligned16_ptr(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// A diagnostics buffer set by a trk_*_set_prof call: bound to the device current at that call,
// and handed only to launches on that same device (get() is null elsewhere), so a stamp buffer
// never receives another device's writes.  The library's only process-wide device pointers.
struct DiagBuf {
  unsigned long long* p = nullptr;
  int dev = -1;
  void set(unsigned long long* q) {
    p = q;
    dev = -1;
    if (q && hipGetDevice(&dev) != hipSuccess) p = nullptr;
  }
  unsigned long long* get() const {
    int d = -1;
    return (p && hipGetDevice(&d) == hipSuccess && d == dev) ? p : nullptr;
  }
};

}  // namespace trk
