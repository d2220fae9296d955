// Standalone timing of the MDX23C TFC 3x3 convolution (conv3x3_db_kernel) on the vocals config's
// level shapes (diagnostic, not product).  Compiles sesa_tapgemm.hip into this translation unit so
// kernel variants / ablations can be launched directly; median of 10 HIP-event-timed launches.
//   ./tools/conv_bench [batch=57]
#include "../sesa-audio-separation_amd/csrc/sesa_tapgemm.hip"

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <vector>

namespace sesa {
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vfprintf(stderr, fmt, ap);
  va_end(ap);
  fputc('\n', stderr);
}
void clear_error() {}
}  // namespace sesa

using namespace sesa;

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

__global__ void fill_bf16(uint16_t* p, int64_t n, uint32_t seed, float scale) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 15;
    x *= 2246822519u;
    x ^= x >> 13;
    const float v = scale * ((float)(x & 0xffff) / 32768.f - 1.f);
    p[i] = __builtin_bit_cast(uint16_t, (__bf16)v);
  }
}

template <class F>
float time_ms(F&& launch, int reps = 10) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  launch();
  launch();
  std::vector<float> ts;
  for (int i = 0; i < reps; ++i) {
    CK(hipEventRecord(e0, 0));
    launch();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float t;
    CK(hipEventElapsedTime(&t, e0, e1));
    ts.push_back(t);
  }
  std::sort(ts.begin(), ts.end());
  return ts[ts.size() / 2];
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 57;
  printf("batch %d\n%-5s %-26s %9s %9s\n", B, "level", "variant", "ms", "TF/s(alg)");
  for (int lvl = 0; lvl < 4; ++lvl) {
    const int C = 128 * (lvl + 1), T = 256 >> lvl, F = 1024 >> lvl;
    const int64_t n_act = (int64_t)B * T * F * C;
    uint16_t *hi, *lo, *w;
    float* out;
    double* stats;
    const int nblk = C / 64, nch = C / kConvBK;
    const int64_t w_elems = (int64_t)nblk * nch * 2 * 9 * 64 * 16;
    CK(hipMalloc(&hi, n_act * 2));
    CK(hipMalloc(&lo, n_act * 2));
    CK(hipMalloc(&w, w_elems * 2));
    CK(hipMalloc(&out, n_act * 4));
    CK(hipMalloc(&stats, (size_t)B * C * 2 * 8));
    hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, hi, n_act, 1u, 1.f);
    hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, lo, n_act, 2u, 1.f / 256);
    hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, w, w_elems, 3u, 0.03f);
    CK(hipDeviceSynchronize());
    ConvArgs a{};
    a.in.src[0].mode = SRC_PRE;
    a.in.src[0].hi = hi;
    a.in.src[0].lo = lo;
    a.in.src[0].C = C;
    a.in.C_split = C;
    a.in.C_in = C;
    a.out.ptr = out;
    a.out.stats = stats;
    a.out.C_out = C;
    a.w = w;
    a.T_in = a.T_out = T;
    a.F_in = a.F_out = F;
    a.n_cols = C;
    a.n_chunks = nch;
    const double flop = 2.0 * B * T * F * (double)C * C * 9;
    const dim3 grid((unsigned)(((T + 15) / 16) * (F / kTF) * ((C + 63) / 64)), 1u, (unsigned)B);
    auto rep = [&](const char* v, float ms) { printf("L%-4d %-26s %9.3f %9.1f\n", lvl, v, ms, flop / ms * 1e-9); };
    rep("conv3x3_db (launch_conv)", time_ms([&] {
          CK(hipMemsetAsync(stats, 0, (size_t)B * C * 16, 0));
          launch_conv(CONV3X3, 64, 1, a, B, 0);
        }));
    rep("no statistics", time_ms([&] { hipLaunchKernelGGL((conv3x3_db_kernel<true, false, 1>), grid, dim3(512), 0, 0, a); }));
    rep("no epilogue", time_ms([&] { hipLaunchKernelGGL((conv3x3_db_kernel<true, false, 2>), grid, dim3(512), 0, 0, a); }));
    CK(hipFree(hi));
    CK(hipFree(lo));
    CK(hipFree(w));
    CK(hipFree(out));
    CK(hipFree(stats));
  }
  return 0;
}
