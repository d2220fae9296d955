// ds_read_b64_tr_b16 operands feeding v_mfma_f32_32x32x16_bf16 (diagnostic): V[key][d] = key, P^T one-hot
// (query column q selects key q): O^T[d][q] must be q for every d.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short v4s __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
__device__ __forceinline__ int swz(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }
__global__ void k(float* out) {
  __shared__ __attribute__((aligned(16))) char V[64 * 128];
  for (int e = threadIdx.x; e < 64 * 64; e += 64) {
    const int key = e / 64, d = e % 64;
    *reinterpret_cast<__bf16*>(V + swz(key, d >> 3) + ((d & 7) << 1)) = (__bf16)(float)key;
  }
  __syncthreads();
  const int lane = threadIdx.x, l32 = lane & 31, hl = lane >> 5;
  const int tg = lane >> 4, ti = lane & 15, tr_q = ti >> 2, tp = ti & 3, th = tg >> 1;
  f32x16 o = {};
  const int qcol = l32;   // this lane's query column (keys 0..31 only: block rb = 0)
  for (int ks = 0; ks < 2; ++ks) {
    const int db = 0;
    const int d = db * 32 + 16 * (tg & 1) + 4 * tp;
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    bf16x4 t2[2];
    for (int r = 0; r < 2; ++r) {
      const int key = 32 * (ks >> 1) + 16 * (ks & 1) + 8 * r + 4 * th + tr_q;
      t2[r] = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
          (__attribute__((address_space(3))) bf16x4*)(V + swz(key, d >> 3) + ((d & 7) << 1)));
    }
    const bf16x8 f = __builtin_shufflevector(t2[0], t2[1], 0, 1, 2, 3, 4, 5, 6, 7);
    bf16x8 p;
    for (int j = 0; j < 8; ++j) {
      const int key = 16 * ks + 8 * (j >> 2) + 4 * hl + (j & 3);
      p[j] = (__bf16)(key == qcol ? 1.f : 0.f);
    }
    o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f, p, o, 0, 0, 0);
  }
  for (int r = 0; r < 16; ++r) {
    const int drow = 8 * (r >> 2) + 4 * hl + (r & 3);
    out[drow * 32 + l32] = o[r];
  }
}
int main() {
  float* d;
  (void)hipMalloc(&d, 32 * 32 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  float h[32 * 32];
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int dd = 0; dd < 32; ++dd)
    for (int q = 0; q < 32; ++q)
      if (h[dd * 32 + q] != (float)q) {
        if (bad < 10) printf("d %d q %d: got %g\n", dd, q, h[dd * 32 + q]);
        ++bad;
      }
  printf("bad %d of 1024\n", bad);
  return 0;
}
