// Probe of the attention kernel's transposed V^T fragment reads (diagnostic): the swizzled
// [64 key][64 d] image holds 64*key + d; every lane checks the 8 elements of each (ks, db) fragment
// against the key / d the MFMA operand maps require.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short v4s __attribute__((ext_vector_type(4)));
__device__ __forceinline__ int swz(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }
__global__ void k(int* bad, int* first) {
  __shared__ __attribute__((aligned(16))) char smem[4 * 64 * 128];
  char* V = smem + 2 * 64 * 128;      // as attn_kernel: V behind the K images, a generic pointer
  for (int e = threadIdx.x; e < 64 * 64; e += blockDim.x) {
    const int key = e / 64, d = e % 64;
    *reinterpret_cast<short*>(V + swz(key, d >> 3) + ((d & 7) << 1)) = (short)(64 * key + d);
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, l32 = lane & 31, hl = lane >> 5;
  const int tg = lane >> 4, ti = lane & 15, tr_q = ti >> 2, tp = ti & 3, th = tg >> 1;
  int nbad = 0;
  for (int ks = 0; ks < 4; ++ks)
    for (int db = 0; db < 2; ++db) {
      const int d = db * 32 + 16 * (tg & 1) + 4 * tp;
      short f[8];
      for (int r = 0; r < 2; ++r) {
        const int key = 32 * (ks >> 1) + 16 * (ks & 1) + 8 * r + 4 * th + tr_q;
        const v4s t = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) v4s*)(V + swz(key, d >> 3) + ((d & 7) << 1)));
        for (int q = 0; q < 4; ++q) f[4 * r + q] = t[q];
      }
      for (int j = 0; j < 8; ++j) {
        const int key = 16 * ks + 8 * (j >> 2) + 4 * hl + (j & 3), dd = db * 32 + l32;
        if (f[j] != (short)(64 * key + dd)) {
          if (atomicAdd(first, 1) < 8) printf("lane %d ks %d db %d j %d: got key %d d %d, want key %d d %d\n", lane, ks, db, j, f[j] / 64, f[j] % 64, key, dd);
          ++nbad;
        }
      }
    }
  atomicAdd(bad, nbad);
}
int main() {
  int* d;
  (void)hipMalloc(&d, 8);
  (void)hipMemset(d, 0, 8);
  hipLaunchKernelGGL(k, dim3(1), dim3(256), 0, 0, d, d + 1);
  int h[2];
  (void)hipMemcpy(h, d, 8, hipMemcpyDeviceToHost);
  printf("bad elements: %d of %d\n", h[0], 4 * 64 * 64);
  return 0;
}
