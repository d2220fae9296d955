// 4096-point real FFT machinery shared by the n_fft = 4096 models (SCNet, HTDemucs): a 2048-point
// complex Stockham FFT in LDS (five radix-4 stages + one radix-2 stage, 256 threads) plus the
// per-device twiddle tables for the real split / merge.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <mutex>
#include <vector>

#include "sesa_common.hpp"

namespace sesa {

constexpr int kFft4096 = 4096;  // real transform length (n_fft)
constexpr int kFft2048 = 2048;  // complex transform length
constexpr int kFftThreads = 256;

struct Fft2048Tables {
  float2* tw = nullptr;   // exp(-2 pi i j / 2048), j < 2048
  float2* twN = nullptr;  // exp(-2 pi i k / 4096), k <= 2048
};

// Per-device tables, built once under a mutex (immutable afterwards).
inline int get_fft2048_tables(Fft2048Tables* out) {
  static std::mutex mu;
  static std::vector<Fft2048Tables> tabs;
  int dev = 0;
  SESA_CHECK_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(mu);
  if ((int)tabs.size() <= dev) tabs.resize(dev + 1);
  Fft2048Tables& t = tabs[dev];
  if (!t.tw) {
    std::vector<float2> a(kFft2048), b(kFft2048 + 1);
    for (int j = 0; j < kFft2048; ++j) {
      const double ang = -2.0 * M_PI * j / kFft2048;
      a[j] = make_float2((float)cos(ang), (float)sin(ang));
    }
    for (int k = 0; k <= kFft2048; ++k) {
      const double ang = -2.0 * M_PI * k / kFft4096;
      b[k] = make_float2((float)cos(ang), (float)sin(ang));
    }
    SESA_CHECK_HIP(hipMalloc(&t.tw, kFft2048 * sizeof(float2)));
    SESA_CHECK_HIP(hipMalloc(&t.twN, (kFft2048 + 1) * sizeof(float2)));
    SESA_CHECK_HIP(hipMemcpy(t.tw, a.data(), kFft2048 * sizeof(float2), hipMemcpyHostToDevice));
    SESA_CHECK_HIP(hipMemcpy(t.twN, b.data(), (kFft2048 + 1) * sizeof(float2), hipMemcpyHostToDevice));
  }
  *out = t;
  return SESA_OK;
}

__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
// complex add / sub as explicit two-lane vectors: one v_pk_add_f32 each, both halves in place (no op_sel).  libsesa
// is built without the SLP vectorizer (its packed complex arithmetic used half-swapping op_sel forms, which are wrong
// beside MFMA work on gfx950: tools/isa_guard.py); these lane-parallel forms are the safe part of that packing.
__device__ __forceinline__ float2 cadd(float2 a, float2 b) {
  const f32x2 r = f32x2{a.x, a.y} + f32x2{b.x, b.y};
  return make_float2(r[0], r[1]);
}
__device__ __forceinline__ float2 csub(float2 a, float2 b) {
  const f32x2 r = f32x2{a.x, a.y} - f32x2{b.x, b.y};
  return make_float2(r[0], r[1]);
}
__device__ __forceinline__ float2 cconj(float2 a) { return make_float2(a.x, -a.y); }

// 2048-point Stockham FFT in LDS (x -> returned buffer, y is scratch); 256 threads.
template <bool INV>
__device__ float2* fft2048(float2* x, float2* y, const float2* __restrict__ tw) {
  int n = kFft2048, s = 1;
#pragma unroll 1
  for (int stage = 0; stage < 5; ++stage) {
    const int m = n >> 2;
    sesa_sync();
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int bfly = threadIdx.x + r * kFftThreads;  // 512 butterflies per stage
      const int q = bfly & (s - 1);
      const int p = bfly >> __builtin_ctz(s);
      const float2 a = x[q + s * p], b = x[q + s * (p + m)], c = x[q + s * (p + 2 * m)], d = x[q + s * (p + 3 * m)];
      float2 w1 = tw[p * s], w2 = tw[2 * p * s], w3 = tw[3 * p * s];
      if (INV) { w1 = cconj(w1); w2 = cconj(w2); w3 = cconj(w3); }
      const float2 apc = cadd(a, c), amc = csub(a, c), bpd = cadd(b, d), bmd = csub(b, d);
      const float2 jbmd = INV ? make_float2(-bmd.y, bmd.x) : make_float2(bmd.y, -bmd.x);
      y[q + s * (4 * p + 0)] = cadd(apc, bpd);
      y[q + s * (4 * p + 1)] = cmul(w1, cadd(amc, jbmd));
      y[q + s * (4 * p + 2)] = cmul(w2, csub(apc, bpd));
      y[q + s * (4 * p + 3)] = cmul(w3, csub(amc, jbmd));
    }
    float2* t = x; x = y; y = t;
    n = m;
    s <<= 2;
  }
  sesa_sync();  // n = 2, s = 1024: final radix-2 stage, unit twiddles
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int q = threadIdx.x + r * kFftThreads;
    const float2 a = x[q], b = x[q + 1024];
    y[q] = cadd(a, b);
    y[q + 1024] = csub(a, b);
  }
  sesa_sync();
  return y;
}

// Real split after a 2048-point complex FFT of the even/odd-interleaved 4096 real samples:
// returns bin k (0..2048) of the 4096-point real transform.
__device__ __forceinline__ float2 rfft_bin(const float2* Z, const float2* __restrict__ twN, int k) {
  const float2 zk = Z[k & (kFft2048 - 1)];
  const float2 zm = cconj(Z[(kFft2048 - k) & (kFft2048 - 1)]);
  const float2 E = make_float2(0.5f * (zk.x + zm.x), 0.5f * (zk.y + zm.y));
  const float2 D = csub(zk, zm);
  const float2 O = make_float2(0.5f * D.y, -0.5f * D.x);
  return cadd(E, cmul(twN[k], O));
}

// Inverse of rfft_bin: packs the half spectrum X[0..2048] (LDS) into the 2048-point complex
// sequence whose inverse FFT yields the even/odd-interleaved real samples; entry k < 2048.
__device__ __forceinline__ float2 irfft_pack(const float2* X, const float2* __restrict__ twN, int k) {
  const float2 xk = X[k];
  const float2 xm = cconj(X[kFft2048 - k]);
  const float2 E = make_float2(0.5f * (xk.x + xm.x), 0.5f * (xk.y + xm.y));
  const float2 D = csub(xk, xm);
  const float2 O = cmul(make_float2(0.5f * D.x, 0.5f * D.y), cconj(twN[k]));
  return make_float2(E.x - O.y, E.y + O.x);
}

}  // namespace sesa
