// Shared host/device helpers for libsesa (MI355X / gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <string>

#include "sesa.h"

namespace sesa {

// ---- error reporting: every C entry returns int (0 ok, <0 error) + thread-local message ----
void set_error(const char* fmt, ...);
void clear_error();

#define SESA_CHECK_HIP(expr)                                                        \
  do {                                                                               \
    hipError_t _e = (expr);                                                          \
    if (_e != hipSuccess) {                                                          \
      ::sesa::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #expr,                 \
                        hipGetErrorString(_e));                                      \
      return SESA_ERR_HIP;                                                           \
    }                                                                                \
  } while (0)

#define SESA_REQUIRE(cond, code, ...)                                               \
  do {                                                                               \
    if (!(cond)) {                                                                   \
      ::sesa::set_error(__VA_ARGS__);                                                \
      return (code);                                                                 \
    }                                                                                \
  } while (0)

// Launch-error check after a kernel launch (async errors surface at the next sync).
#define SESA_CHECK_LAUNCH() SESA_CHECK_HIP(hipGetLastError())

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ---- device helpers ----
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Exact (erf) GELU, torch.nn.GELU(approximate='none').
__device__ __forceinline__ float gelu_erf(float v) {
  return 0.5f * v * (1.0f + erff(v * 0.70710678118654752440f));
}

// Split an fp32 value into bf16 hi + bf16 lo (v ~= hi + lo to ~2^-17 relative).
__device__ __forceinline__ void split_bf16(float v, __bf16& hi, __bf16& lo) {
  hi = (__bf16)v;
  lo = (__bf16)(v - (float)hi);
}

}  // namespace sesa
