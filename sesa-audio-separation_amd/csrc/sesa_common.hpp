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
// Workgroup barrier that first retires this wave's own LDS operations.  __syncthreads() leaves the lgkmcnt wait to the
// memory legalizer, which omits it where its fence needs no cross-address-space ordering (LLVM takes LDS operations of
// all waves to execute in one global order), e.g. at the top of an LDS ping-pong FFT stage loop.  On MI355X that
// order did not hold with another kernel's waves on the CU: the BS-Roformer iSTFT read a previous stage's values for
// whole waves (512-sample runs of a frame) when another stream's forward ran beside it (tools/barrier_scan.py lists the
// barriers reachable with LDS writes in flight).
__device__ __forceinline__ void sesa_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
}

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Exact (erf) GELU, torch.nn.GELU(approximate='none'), branch-free:
//   Phi(v) = 1 - erfc(z)/2 (v >= 0) or erfc(z)/2 (v < 0), z = |v|/sqrt(2), with
//   erfc(z) = t * P4(t) * exp(-z^2), t = 1/(1 + p z)  (Abramowitz & Stegun 7.1.26, |erf error| < 1.5e-7).
// Max |error| vs the float64 GELU over [-12, 12] in float32 is 4.2e-7 -- the float32 resolution of the
// result there (the 9-term Chebyshev erfc form used before: 3.8e-7; ocml erff: 4.5e-7) and far below the
// 2^-17 hi/lo bf16 split that follows -- at ~14 VALU ops (5 fewer than that form; the TDF staging and the
// FF1 epilogue that use it are VALU-issue-bound).
__device__ __forceinline__ float gelu_erf(float v) {
  const float z = fabsf(v) * 0.70710678118654752440f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  float p = 1.061405429f;
  p = fmaf(p, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float e = p * t * __builtin_amdgcn_exp2f(-(z * z) * 1.4426950408889634f);  // erfc(z)
  const float phi = v >= 0.f ? fmaf(-0.5f, e, 1.0f) : 0.5f * e;
  return v * phi;
}

// gelu_erf on two values at once: the same sequence of fmas on float2, which gfx950 issues as
// packed v_pk_fma_f32 / v_pk_mul_f32 (half the VALU issue slots of the scalar form; the rcp / exp2
// stay per component).
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 gelu_erf2(f32x2 v) {
  const f32x2 z = __builtin_elementwise_abs(v) * 0.70710678118654752440f;
  const f32x2 d = __builtin_elementwise_fma(z, f32x2{0.3275911f, 0.3275911f}, f32x2{1.0f, 1.0f});
  const f32x2 t = {__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
  f32x2 p = {1.061405429f, 1.061405429f};
  p = __builtin_elementwise_fma(p, t, f32x2{-1.453152027f, -1.453152027f});
  p = __builtin_elementwise_fma(p, t, f32x2{1.421413741f, 1.421413741f});
  p = __builtin_elementwise_fma(p, t, f32x2{-0.284496736f, -0.284496736f});
  p = __builtin_elementwise_fma(p, t, f32x2{0.254829592f, 0.254829592f});
  const f32x2 a = (z * z) * -1.4426950408889634f;
  const f32x2 e = p * t * f32x2{__builtin_amdgcn_exp2f(a[0]), __builtin_amdgcn_exp2f(a[1])};
  const f32x2 one_minus = __builtin_elementwise_fma(e, f32x2{-0.5f, -0.5f}, f32x2{1.0f, 1.0f});
  const f32x2 half = e * 0.5f;
  const f32x2 phi = {v[0] >= 0.f ? one_minus[0] : half[0], v[1] >= 0.f ? one_minus[1] : half[1]};
  return v * phi;
}

// Split an fp32 value into bf16 hi + bf16 lo (v ~= hi + lo to ~2^-17 relative).
__device__ __forceinline__ void split_bf16(float v, __bf16& hi, __bf16& lo) {
  hi = (__bf16)v;
  lo = (__bf16)(v - (float)hi);
}

}  // namespace sesa
