// Round 6 diagnostic (tools/fft_stress.py agg:<name>): synthetic side-stream workloads, each isolating one property of
// the MDX23C kernels that disturbed a concurrent STFT (tools/fft_stress.py, SESA_DEBUG_ONLY): MFMA-heavy loops, fp64 /
// fp32 no-return global atomics, LDS traffic with barriers.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/aggressors.hip -o tools/_canary/libaggressors.so
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__global__ void __launch_bounds__(256, 2) agg_mfma(float* out, int iters) {
  f32x16 acc = {};
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = (__bf16)(0.001f * (threadIdx.x + i));
    b[i] = (__bf16)(0.002f * (blockIdx.x + i));
  }
  for (int it = 0; it < iters; ++it) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
  float s = 0.f;
  for (int r = 0; r < 16; ++r) s += acc[r];
  if (s == 12345.678f) out[threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) agg_atomic64(double* st, int n_slots, int iters) {
  for (int it = 0; it < iters; ++it) {
    const int k = (blockIdx.x * 7 + it * 13 + threadIdx.x) % n_slots;
    atomicAdd(st + k, 1.0);
  }
}

__global__ void __launch_bounds__(256) agg_atomic32(float* st, int n_slots, int iters) {
  for (int it = 0; it < iters; ++it) {
    const int k = (blockIdx.x * 7 + it * 13 + threadIdx.x) % n_slots;
    atomicAdd(st + k, 1.f);
  }
}

__global__ void __launch_bounds__(256, 2) agg_lds(float* out, int iters) {
  __shared__ float buf[17408];   // 68 KiB
  float v = threadIdx.x;
  for (int it = 0; it < iters; ++it) {
    for (int i = threadIdx.x; i < 17408; i += 256) buf[i] = v + i;
    __syncthreads();
    v += buf[(threadIdx.x * 67 + it) % 17408];
    __syncthreads();
  }
  if (v == 12345.678f) out[threadIdx.x] = v;
}

// the tap_gemm epilogue's shape: stores, then an LDS reduction of fp64 sums, then fp64 atomics
__global__ void __launch_bounds__(256, 2) agg_epilogue(float* out, double* st, int n_slots, int iters) {
  __shared__ double red[4 * 128 * 2];
  for (int it = 0; it < iters; ++it) {
    double s = threadIdx.x + it;
    s += __shfl_xor(s, 32);
    red[threadIdx.x * 2] = s;
    __syncthreads();
    if (threadIdx.x < 128) atomicAdd(st + (blockIdx.x * 128 + threadIdx.x + it) % n_slots, red[threadIdx.x * 2 + 256]);
    __syncthreads();
    out[((int64_t)blockIdx.x * 256 + threadIdx.x + it * 997) % (1 << 22)] = (float)s;
  }
}
// ---- victims: deterministic kernels whose output is compared bit for bit with an idle-device run ----
typedef float f32x2 __attribute__((ext_vector_type(2)));

// packed f32 FMA chain (v_pk_fma_f32), registers only
__global__ void __launch_bounds__(256) vic_pk(float* out, int iters) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  f32x2 a = {1e-3f * (t & 1023), 2e-3f * (t & 511)}, b = {1.0001f, 0.9999f}, c = {1e-4f, -1e-4f};
  for (int it = 0; it < iters; ++it) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
  out[2 * t] = a[0];
  out[2 * t + 1] = a[1];
}

// the packed forms the compiler emits in the FFT: v_pk_add_f32 with neg modifiers, v_pk_mul_f32, v_pk_mov_b32 op_sel
__global__ void __launch_bounds__(256) vic_pkmix(float* out, int iters) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  f32x2 a = {1e-3f * (t & 1023), 2e-3f * (t & 511)}, b = {1.0001f, 0.9999f}, c = {1e-4f, -1e-4f}, d = {0.5f, 0.25f};
  for (int it = 0; it < iters; ++it) {
    asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(a) : "v"(b));
    asm volatile("v_pk_add_f32 %0, %0, %1 neg_lo:[0,1] neg_hi:[0,1]" : "+v"(a) : "v"(c));
    asm volatile("v_pk_mov_b32 %0, %1, %0 op_sel:[1,0]" : "+v"(d) : "v"(a));
    asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a) : "v"(d));
  }
  out[2 * t] = a[0];
  out[2 * t + 1] = a[1] + d[0];
}

// a packed-f32 result stored by the very next instruction (ds_write_b64 / global_store_dwordx2, no wait state between):
// the LDS / memory copy is compared with the register value; mode 0 v_pk_mul_f32, 1 v_pk_add_f32, 2 v_pk_fma_f32,
// 3 two scalar v_mul_f32 (control), 4 v_pk_mul_f32 + s_nop 0, 5 v_pk_mul_f32 -> global_store_dwordx2
__global__ void __launch_bounds__(256) vic_pkst(float* out, int iters, int mode) {
  __shared__ f32x2 buf[256];
  const int t = blockIdx.x * 256 + threadIdx.x;
  f32x2 a = {1.0f + 1e-3f * (t & 1023), 2.0f - 1e-3f * (t & 511)}, b = {1.0001f, 0.9999f};
  const uint32_t addr = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) f32x2*)&buf[threadIdx.x];
  f32x2* gdst = reinterpret_cast<f32x2*>(out) + (int64_t)gridDim.x * 256 + t;
  uint32_t bad = 0;
  for (int it = 0; it < iters; ++it) {
    f32x2 r;
    if (mode == 0) asm volatile("v_pk_mul_f32 %0, %1, %2\n\tds_write_b64 %3, %0" : "=&v"(r) : "v"(a), "v"(b), "v"(addr) : "memory");
    else if (mode == 1) asm volatile("v_pk_add_f32 %0, %1, %2\n\tds_write_b64 %3, %0" : "=&v"(r) : "v"(a), "v"(b), "v"(addr) : "memory");
    else if (mode == 2) asm volatile("v_pk_fma_f32 %0, %1, %2, %1\n\tds_write_b64 %3, %0" : "=&v"(r) : "v"(a), "v"(b), "v"(addr) : "memory");
    else if (mode == 3) {
      float r0, r1;
      asm volatile("v_mul_f32 %0, %1, %2" : "=v"(r0) : "v"(a[0]), "v"(b[0]));
      asm volatile("v_mul_f32 %0, %1, %2" : "=v"(r1) : "v"(a[1]), "v"(b[1]));
      r = f32x2{r0, r1};
    }
    else if (mode == 4) asm volatile("v_pk_mul_f32 %0, %1, %2\n\ts_nop 0\n\tds_write_b64 %3, %0" : "=&v"(r) : "v"(a), "v"(b), "v"(addr) : "memory");
    else asm volatile("v_pk_mul_f32 %0, %1, %2\n\tglobal_store_dwordx2 %3, %0, off" : "=&v"(r) : "v"(a), "v"(b), "v"(gdst) : "memory");
    if (mode == 3) buf[threadIdx.x] = r;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    const f32x2 m = mode == 5 ? *(volatile f32x2*)gdst : buf[threadIdx.x];
    bad += (m[0] != r[0]) | (m[1] != r[1]);
    a = r * 0.5f + a * 0.5f + f32x2{1e-3f, -1e-3f};
  }
  out[t] = __uint_as_float(bad);
}

// one packed form of the compiler's FFT code per mode, in a dependent chain (tools/victim_stress.py form<k>)
template <int MODE>
__global__ void __launch_bounds__(256) vic_form(float* out, int iters, float sv0, float sv1) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  f32x2 x = {1.0f + 1e-3f * (t & 1023), 1.0f - 1e-3f * (t & 511)}, y = {1.0001f, 0.9999f}, z = {1e-5f, -2e-5f};
  const f32x2 sp = {sv0, sv1};   // kernel-argument values: SGPR pair
  for (int it = 0; it < iters; ++it) {
    if constexpr (MODE == 0) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(x) : "v"(z));
    if constexpr (MODE == 1) asm volatile("v_pk_add_f32 %0, %0, %1 neg_lo:[0,1] neg_hi:[0,1]" : "+v"(x) : "v"(z));
    if constexpr (MODE == 2) asm volatile("v_pk_add_f32 %0, %0, %1 op_sel:[0,1] op_sel_hi:[0,1]" : "+v"(x) : "v"(z));
    if constexpr (MODE == 3) asm volatile("v_pk_mul_f32 %0, %0, %1 op_sel:[0,1] op_sel_hi:[1,0]" : "+v"(x) : "v"(y));
    if constexpr (MODE == 4) asm volatile("v_pk_fma_f32 %0, %0, %1, %2 neg_lo:[0,0,1] neg_hi:[0,0,1]" : "+v"(x) : "v"(y), "v"(z));
    if constexpr (MODE == 5) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(x) : "s"(sp));
    if constexpr (MODE == 6) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x) : "s"(sp), "v"(z));
    if constexpr (MODE == 7) asm volatile("v_pk_mov_b32 %0, %0, %1 op_sel:[1,0]" : "+v"(x) : "v"(y));
    if constexpr (MODE == 8) asm volatile("v_pk_fma_f32 %0, %0, 0.5, %1 op_sel_hi:[1,0,1]" : "+v"(x) : "v"(y));
    if constexpr (MODE == 7) x = x * 1.0001f;
  }
  out[2 * t] = x[0];
  out[2 * t + 1] = x[1];
}

// scalar f32 FMA chain (v_fma_f32), registers only
__global__ void __launch_bounds__(256) vic_fma(float* out, int iters) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  float a = 1e-3f * (t & 1023), a2 = 2e-3f * (t & 511);
  const float b = 1.0001f, b2 = 0.9999f, c = 1e-4f, c2 = -1e-4f;
  for (int it = 0; it < iters; ++it) {
    asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
    asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a2) : "v"(b2), "v"(c2));
  }
  out[2 * t] = a;
  out[2 * t + 1] = a2;
}

// LDS round trips with barriers (4 waves), plain integer data
__global__ void __launch_bounds__(256) vic_lds(float* out, int iters) {
  __shared__ uint32_t buf[8704];   // 34 KiB
  uint32_t v = blockIdx.x * 256 + threadIdx.x;
  for (int it = 0; it < iters; ++it) {
    for (int i = threadIdx.x; i < 8704; i += 256) buf[i] = v * 2654435761u + i;
    __syncthreads();
    v ^= buf[(threadIdx.x * 131 + it * 7) % 8704];
    __syncthreads();
  }
  out[blockIdx.x * 256 + threadIdx.x] = __uint_as_float(v & 0x3fffffffu);
}
}  // namespace

extern "C" int vic_launch(int which, int blocks, int iters, void* out, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  switch (which) {
    case 0: hipLaunchKernelGGL(vic_pk, dim3(blocks), dim3(256), 0, st, (float*)out, iters); break;
    case 1: hipLaunchKernelGGL(vic_fma, dim3(blocks), dim3(256), 0, st, (float*)out, iters); break;
    case 2: hipLaunchKernelGGL(vic_lds, dim3(blocks), dim3(256), 0, st, (float*)out, iters); break;
    case 3: hipLaunchKernelGGL(vic_pkmix, dim3(blocks), dim3(256), 0, st, (float*)out, iters); break;
#define VF(K) case 20 + K: hipLaunchKernelGGL(vic_form<K>, dim3(blocks), dim3(256), 0, st, (float*)out, iters, 1.0001f, 0.9999f); break;
    VF(0) VF(1) VF(2) VF(3) VF(4) VF(5) VF(6) VF(7) VF(8)
#undef VF
    case 10: case 11: case 12: case 13: case 14: case 15:
      hipLaunchKernelGGL(vic_pkst, dim3(blocks), dim3(256), 0, st, (float*)out, iters, which - 10); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int agg_launch(int which, int blocks, int iters, void* fbuf, void* dbuf, int n_slots, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  switch (which) {
    case 0: hipLaunchKernelGGL(agg_mfma, dim3(blocks), dim3(256), 0, st, (float*)fbuf, iters); break;
    case 1: hipLaunchKernelGGL(agg_atomic64, dim3(blocks), dim3(256), 0, st, (double*)dbuf, n_slots, iters); break;
    case 2: hipLaunchKernelGGL(agg_atomic32, dim3(blocks), dim3(256), 0, st, (float*)fbuf, n_slots, iters); break;
    case 3: hipLaunchKernelGGL(agg_lds, dim3(blocks), dim3(256), 0, st, (float*)fbuf, iters); break;
    case 4: hipLaunchKernelGGL(agg_epilogue, dim3(blocks), dim3(256), 0, st, (float*)fbuf, (double*)dbuf, n_slots, iters); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
