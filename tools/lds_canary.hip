// Round 6 diagnostic (tools/lds_canary.py): an LDS canary.  Each workgroup of lds_canary_kernel fills its dynamic LDS
// with a known pattern, then re-reads it for a while; any word that changes was written by someone else -- a
// co-resident workgroup of another kernel writing outside its own LDS allocation.  The first changed words (LDS byte
// offset, value seen, value expected) are appended to a device log.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/lds_canary.hip -o tools/_canary/liblds_canary.so
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {
__device__ __forceinline__ uint32_t pattern(uint32_t i) { return 0xC0DE0000u ^ (i * 2654435761u); }

__global__ void __launch_bounds__(256) lds_canary_kernel(int words, int rounds, uint32_t* log, int log_cap,
                                                         unsigned long long* hits) {
  extern __shared__ uint32_t buf[];
  for (int i = threadIdx.x; i < words; i += 256) buf[i] = pattern(i);
  __syncthreads();
  for (int r = 0; r < rounds; ++r) {
    __builtin_amdgcn_s_sleep(16);
    for (int i = threadIdx.x; i < words; i += 256) {
      const uint32_t v = buf[i];
      if (v != pattern(i)) {
        const unsigned long long k = atomicAdd(hits, 1ull);
        if (k < (unsigned long long)log_cap) {
          log[4 * k + 0] = (uint32_t)i * 4;      // LDS byte offset within this workgroup's allocation
          log[4 * k + 1] = v;
          log[4 * k + 2] = blockIdx.x;
          log[4 * k + 3] = (uint32_t)r;
        }
        buf[i] = pattern(i);                     // re-arm
      }
    }
  }
}
}  // namespace

extern "C" int lds_canary_launch(int blocks, int lds_bytes, int rounds, void* log, int log_cap, void* hits,
                                 void* stream) {
  hipLaunchKernelGGL(lds_canary_kernel, dim3(blocks), dim3(256), lds_bytes, (hipStream_t)stream, lds_bytes / 4, rounds,
                     (uint32_t*)log, log_cap, (unsigned long long*)hits);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
