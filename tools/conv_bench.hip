// Standalone timing of the MDX23C TFC 3x3 convolution (conv3x3_db_kernel) on the vocals config's
// level shapes (diagnostic, not product).  Compiles sesa_tapgemm.hip into this translation unit so
// kernel variants / ablations can be launched directly; median of 10 HIP-event-timed launches.
//   ./tools/conv_bench [batch=57] [tdf]
#include "../sesa-audio-separation_amd/csrc/sesa_tapgemm.hip"

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <vector>

namespace sesa {
namespace {
// kernel variants launched only from this file's lambdas: instantiated here so their host stubs are emitted
template __global__ void conv3x3_db_kernel<true, true, 0, false, 1, true, 2, 2, false>(ConvArgs);
template __global__ void conv3x3_db_kernel<true, true, 0, false, 1, true, 1, 1, false>(ConvArgs);
template __global__ void conv3x3_db_kernel<true, true, 0, false, 1, true, 1, 2, false>(ConvArgs);
template __global__ void conv3x3_db_kernel<true, true, 0, false, 1, true, 1, 1, true>(ConvArgs);
template __global__ void conv3x3_db_kernel<true, true, 0, false, 1, true, 0, 2, true>(ConvArgs);
template __global__ void conv3x3_db_kernel<true, true, 0, false, 0, false, 0, 2, true>(ConvArgs);
}  // namespace
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

__global__ void max_diff(const float* a, const float* b, int64_t n, unsigned int* out) {
  float d = 0.f, m = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    d = fmaxf(d, fabsf(a[i] - b[i]));
    m = fmaxf(m, fabsf(b[i]));
  }
  atomicMax(out, __float_as_uint(d));
  atomicMax(out + 1, __float_as_uint(m));
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
  const bool only_tdf = argc > 2 && strcmp(argv[2], "tdf") == 0;  // ./tools/conv_bench 57 tdf
  const bool only_act = argc > 2 && strcmp(argv[2], "act") == 0;  // ./tools/conv_bench 57 act
  const bool only_wino = argc > 2 && strcmp(argv[2], "wino") == 0;  // ./tools/conv_bench 57 wino
  const bool only_f16 = argc > 2 && strcmp(argv[2], "f16") == 0;    // ./tools/conv_bench 57 f16
  const bool only_mdma = argc > 2 && strcmp(argv[2], "mdma") == 0;  // ./tools/conv_bench 57 mdma
  const bool only_sci = argc > 2 && strcmp(argv[2], "sci") == 0;    // ./tools/conv_bench 57 sci
  if (only_sci) {
    // fp16 MI4 MDMA TFC conv with the fused shortcut: per-wave DMA ring after the main loop (SCR = 2, the default) vs
    // interleaved with the main loop (SCR = 3); same operands, different fp32 summation order
    for (int lvl = 0; lvl < 4; ++lvl)
      for (int dec = 0; dec < 2; ++dec) {
        const int C = 128 * (lvl + 1), Cx = dec ? 2 * C : C, T = 256 >> lvl, F = 1024 >> lvl;
        const int64_t n_act = (int64_t)B * T * F * C, n_x = (int64_t)B * T * F * Cx;
        float *x, *out, *out2;
        uint16_t *hi, *w;
        double* stats;
        const int nblk = C / 64, nch = C / kConvBK, xch = Cx / kConvBK;
        const int64_t w_elems = (int64_t)nblk * (nch * 9 * 64 * 32 + xch * 64 * 32);
        CK(hipMalloc(&x, n_x * 4));
        CK(hipMalloc(&hi, n_act * 2));
        CK(hipMalloc(&w, w_elems * 2));
        CK(hipMalloc(&out, n_act * 4));
        CK(hipMalloc(&out2, n_act * 4));
        CK(hipMalloc(&stats, (size_t)B * C * 2 * 8));
        hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint16_t*>(x), n_x * 2, 4u, 1.f);
        hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, hi, n_act, 1u, 1.f);
        hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, w, w_elems, 3u, 0.03f);
        CK(hipDeviceSynchronize());
        ConvArgs a{};
        a.in.src[0] = Src{nullptr, nullptr, nullptr, C, SRC_PRE, hi, nullptr};
        a.in.src[1] = a.in.src[0];
        a.in.C_split = a.in.C_in = C;
        a.out.ptr = out;
        a.out.stats = stats;
        a.out.C_out = C;
        a.w = w;
        a.T_in = a.T_out = T;
        a.F_in = a.F_out = F;
        a.n_cols = C;
        a.n_chunks = nch;
        a.xin.src[0] = Src{x, nullptr, nullptr, Cx, SRC_RAW, nullptr, nullptr};
        a.xin.src[1] = a.xin.src[0];
        a.xin.C_split = a.xin.C_in = Cx;
        a.x_chunks = xch;
        const double flop_x = 2.0 * B * T * F * (double)C * C * 9 + 2.0 * B * T * F * (double)C * Cx;
        const dim3 g32((unsigned)(((T + 31) / 32) * (F / kTF) * ((C + 63) / 64)), 1u, (unsigned)B);
        auto rep = [&](const char* v, float ms, double fl) {
          printf("L%d%s %-34s %9.3f %9.1f\n", lvl, dec ? "dec" : "enc", v, ms, fl / ms * 1e-9);
        };
        rep("ring shortcut (SCR 2)", time_ms([&] {
              hipLaunchKernelGGL((conv3x3_db_kernel<true, true, 0, false, 1, true, 2, 2, false, 1>), g32, dim3(512), 0, 0, a);
            }), flop_x);
        rep("interleaved shortcut (SCR 3)", time_ms([&] {
              hipLaunchKernelGGL((conv3x3_db_kernel<true, true, 0, false, 1, true, 3, 2, false, 1>), g32, dim3(512), 0, 0, a);
            }), flop_x);
        unsigned int* dm;
        CK(hipMalloc(&dm, 8));
        CK(hipMemset(dm, 0, 8));
        ConvArgs q = a;
        q.out.ptr = out2;
        hipLaunchKernelGGL((conv3x3_db_kernel<true, true, 0, false, 1, true, 2, 2, false, 1>), g32, dim3(512), 0, 0, a);
        hipLaunchKernelGGL((conv3x3_db_kernel<true, true, 0, false, 1, true, 3, 2, false, 1>), g32, dim3(512), 0, 0, q);
        hipLaunchKernelGGL(max_diff, dim3(2048), dim3(256), 0, 0, out, out2, n_act, dm);
        unsigned int hh[2];
        CK(hipMemcpy(hh, dm, 8, hipMemcpyDeviceToHost));
        float d, mm;
        memcpy(&d, &hh[0], 4);
        memcpy(&mm, &hh[1], 4);
        printf("L%d%s SCR 3 vs SCR 2: max|diff| %.3e max|out| %.3e rel %.2e %s\n", lvl, dec ? "dec" : "enc", d, mm,
               d / mm, d / mm < 1e-5f ? "OK" : "MISMATCH");
        CK(hipFree(dm));
        CK(hipFree(x));
        CK(hipFree(hi));
        CK(hipFree(w));
        CK(hipFree(out));
        CK(hipFree(out2));
        CK(hipFree(stats));
      }
    return 0;
  }
  if (only_mdma) {
    // fp16 MI4 TFC conv: register-staged main chunks vs LDS-DMA staged (MDMA), without and with the per-wave DMA ring
    // shortcut; outputs must be bit-identical (same operands, same MFMA order)
    for (int lvl = 0; lvl < 4; ++lvl)
      for (int dec = 0; dec < 2; ++dec) {
        const int C = 128 * (lvl + 1), Cx = dec ? 2 * C : C, T = 256 >> lvl, F = 1024 >> lvl;
        const int64_t n_act = (int64_t)B * T * F * C, n_x = (int64_t)B * T * F * Cx;
        float *x, *out, *out2;
        uint16_t *hi, *w;
        double* stats;
        const int nblk = C / 64, nch = C / kConvBK, xch = Cx / kConvBK;
        const int64_t w_elems = (int64_t)nblk * (nch * 9 * 64 * 32 + xch * 64 * 32);
        CK(hipMalloc(&x, n_x * 4));
        CK(hipMalloc(&hi, n_act * 2));
        CK(hipMalloc(&w, w_elems * 2));
        CK(hipMalloc(&out, n_act * 4));
        CK(hipMalloc(&out2, n_act * 4));
        CK(hipMalloc(&stats, (size_t)B * C * 2 * 8));
        hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint16_t*>(x), n_x * 2, 4u, 1.f);
        hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, hi, n_act, 1u, 1.f);
        hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, w, w_elems, 3u, 0.03f);
        CK(hipDeviceSynchronize());
        ConvArgs a{};
        a.in.src[0] = Src{nullptr, nullptr, nullptr, C, SRC_PRE, hi, nullptr};
        a.in.src[1] = a.in.src[0];
        a.in.C_split = a.in.C_in = C;
        a.out.ptr = out;
        a.out.stats = stats;
        a.out.C_out = C;
        a.w = w;
        a.T_in = a.T_out = T;
        a.F_in = a.F_out = F;
        a.n_cols = C;
        a.n_chunks = nch;
        ConvArgs ax = a;
        ax.xin.src[0] = Src{x, nullptr, nullptr, Cx, SRC_RAW, nullptr, nullptr};
        ax.xin.src[1] = ax.xin.src[0];
        ax.xin.C_split = ax.xin.C_in = Cx;
        ax.x_chunks = xch;
        const double flop = 2.0 * B * T * F * (double)C * C * 9, flop_x = flop + 2.0 * B * T * F * (double)C * Cx;
        const dim3 g32((unsigned)(((T + 31) / 32) * (F / kTF) * ((C + 63) / 64)), 1u, (unsigned)B);
        auto rep = [&](const char* v, float ms, double fl) {
          printf("L%d%s %-34s %9.3f %9.1f\n", lvl, dec ? "dec" : "enc", v, ms, fl / ms * 1e-9);
        };
        rep("mi4 no shortcut (regs)", time_ms([&] {
              hipLaunchKernelGGL((conv3x3_db_kernel<true, false, 0, false, 1, true>), g32, dim3(512), 0, 0, a);
            }), flop);
        rep("mi4 no shortcut (MDMA)", time_ms([&] {
              hipLaunchKernelGGL((conv3x3_db_kernel<true, false, 0, false, 1, true, 0, 2, false, 1>), g32, dim3(512), 0, 0, a);
            }), flop);
        rep("mi4 + ring shortcut (regs)", time_ms([&] {
              hipLaunchKernelGGL((conv3x3_db_kernel<true, true, 0, false, 1, true, 2>), g32, dim3(512), 0, 0, ax);
            }), flop_x);
        rep("mi4 + ring shortcut (MDMA)", time_ms([&] {
              hipLaunchKernelGGL((conv3x3_db_kernel<true, true, 0, false, 1, true, 2, 2, false, 1>), g32, dim3(512), 0, 0, ax);
            }), flop_x);
        unsigned int* dm;
        CK(hipMalloc(&dm, 8));
        for (int v = 0; v < 2; ++v) {
          CK(hipMemset(dm, 0, 8));
          ConvArgs p = v ? ax : a, q = p;
          q.out.ptr = out2;
          if (v) {
            hipLaunchKernelGGL((conv3x3_db_kernel<true, true, 0, false, 1, true, 2>), g32, dim3(512), 0, 0, p);
            hipLaunchKernelGGL((conv3x3_db_kernel<true, true, 0, false, 1, true, 2, 2, false, 1>), g32, dim3(512), 0, 0, q);
          } else {
            hipLaunchKernelGGL((conv3x3_db_kernel<true, false, 0, false, 1, true>), g32, dim3(512), 0, 0, p);
            hipLaunchKernelGGL((conv3x3_db_kernel<true, false, 0, false, 1, true, 0, 2, false, 1>), g32, dim3(512), 0, 0, q);
          }
          hipLaunchKernelGGL(max_diff, dim3(2048), dim3(256), 0, 0, out, out2, n_act, dm);
          unsigned int hh[2];
          CK(hipMemcpy(hh, dm, 8, hipMemcpyDeviceToHost));
          float d, mm;
          memcpy(&d, &hh[0], 4);
          memcpy(&mm, &hh[1], 4);
          printf("L%d%s MDMA vs regs (%s): max|diff| %.3e max|out| %.3e %s\n", lvl, dec ? "dec" : "enc",
                 v ? "ring shortcut" : "no shortcut", d, mm, d == 0.f ? "IDENTICAL" : "MISMATCH");
        }
        CK(hipFree(dm));
        CK(hipFree(x));
        CK(hipFree(hi));
        CK(hipFree(w));
        CK(hipFree(out));
        CK(hipFree(out2));
        CK(hipFree(stats));
      }
    return 0;
  }
  if (only_f16) {
    // fp16 MI4 TFC conv (SESA_PREC_F16 / fp16mix '1' levels) with the fused bf16x3 1x1 shortcut: LDS-staged
    // shortcut phase vs the register-direct one (SCR, SCD chunks in flight); agreement must be bit-exact.
    // Encoder conv2 shapes (C_in = C_out = C, shortcut over C raw channels) and decoder conv2 (shortcut
    // over 2C raw channels).
    for (int lvl = 0; lvl < 4; ++lvl)
      for (int dec = 0; dec < 2; ++dec) {
        const int C = 128 * (lvl + 1), Cx = dec ? 2 * C : C, T = 256 >> lvl, F = 1024 >> lvl;
        const int64_t n_act = (int64_t)B * T * F * C, n_x = (int64_t)B * T * F * Cx;
        float *x, *out, *out2;
        uint16_t *hi, *w;
        double* stats;
        const int nblk = C / 64, nch = C / kConvBK, xch = Cx / kConvBK;
        const int64_t w_elems = (int64_t)nblk * (nch * 9 * 64 * 32 + xch * 64 * 32);
        CK(hipMalloc(&x, n_x * 4));
        CK(hipMalloc(&hi, n_act * 2));
        CK(hipMalloc(&w, w_elems * 2));
        CK(hipMalloc(&out, n_act * 4));
        CK(hipMalloc(&out2, n_act * 4));
        CK(hipMalloc(&stats, (size_t)B * C * 2 * 8));
        hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint16_t*>(x), n_x * 2, 4u, 1.f);
        hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, hi, n_act, 1u, 1.f);
        hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, w, w_elems, 3u, 0.03f);
        CK(hipDeviceSynchronize());
        ConvArgs a{};
        a.in.src[0] = Src{nullptr, nullptr, nullptr, C, SRC_PRE, hi, nullptr};
        a.in.src[1] = a.in.src[0];
        a.in.C_split = a.in.C_in = C;
        a.out.ptr = out;
        a.out.stats = stats;
        a.out.C_out = C;
        a.w = w;
        a.T_in = a.T_out = T;
        a.F_in = a.F_out = F;
        a.n_cols = C;
        a.n_chunks = nch;
        ConvArgs ax = a;
        ax.xin.src[0] = Src{x, nullptr, nullptr, Cx, SRC_RAW, nullptr, nullptr};
        ax.xin.src[1] = ax.xin.src[0];
        ax.xin.C_split = ax.xin.C_in = Cx;
        ax.x_chunks = xch;
        const double flop = 2.0 * B * T * F * (double)C * C * 9, flop_x = flop + 2.0 * B * T * F * (double)C * Cx;
        const dim3 g32((unsigned)(((T + 31) / 32) * (F / kTF) * ((C + 63) / 64)), 1u, (unsigned)B);
        auto rep = [&](const char* v, float ms, double fl) {
          printf("L%d%s %-34s %9.3f %9.1f\n", lvl, dec ? "dec" : "enc", v, ms, fl / ms * 1e-9);
        };
        rep("mi4 no shortcut", time_ms([&] {
              hipLaunchKernelGGL((conv3x3_db_kernel<true, false, 0, false, 1, true>), g32, dim3(512), 0, 0, a);
            }), flop);
        rep("mi4 + shortcut (LDS)", time_ms([&] {
              hipLaunchKernelGGL((conv3x3_db_kernel<true, true, 0, false, 1, true>), g32, dim3(512), 0, 0, ax);
            }), flop_x);
        rep("mi4 + shortcut (regs, 2 in flight)", time_ms([&] {
              hipLaunchKernelGGL((conv3x3_db_kernel<true, true, 0, false, 1, true, 1, 2>), g32, dim3(512), 0, 0, ax);
            }), flop_x);
        rep("mi4 + shortcut (regs, 1 in flight)", time_ms([&] {
              hipLaunchKernelGGL((conv3x3_db_kernel<true, true, 0, false, 1, true, 1, 1>), g32, dim3(512), 0, 0, ax);
            }), flop_x);
        rep("mi4 + shortcut (per-wave DMA ring)", time_ms([&] {
              hipLaunchKernelGGL((conv3x3_db_kernel<true, true, 0, false, 1, true, 2>), g32, dim3(512), 0, 0, ax);
            }), flop_x);
        rep("mi4 + shortcut (LDS, split order)", time_ms([&] {
              hipLaunchKernelGGL((conv3x3_db_kernel<true, true, 0, false, 1, true, false, 2, true>), g32, dim3(512), 0, 0, ax);
            }), flop_x);
        rep("mi4 + shortcut (regs 1, split order)", time_ms([&] {
              hipLaunchKernelGGL((conv3x3_db_kernel<true, true, 0, false, 1, true, 1, 1, true>), g32, dim3(512), 0, 0, ax);
            }), flop_x);
        {  // bf16x3 16-row tile (the parity precision, fp16mix '3' levels): hi / lo planes
          uint16_t* lo;
          CK(hipMalloc(&lo, n_act * 2));
          hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, lo, n_act, 2u, 1.f / 256);
          ConvArgs b3 = ax;
          b3.in.src[0].lo = lo;
          b3.in.src[1] = b3.in.src[0];
          const dim3 g16((unsigned)(((T + 15) / 16) * (F / kTF) * ((C + 63) / 64)), 1u, (unsigned)B);
          rep("bf16x3 + shortcut", time_ms([&] {
                hipLaunchKernelGGL((conv3x3_db_kernel<true, true, 0, false, 0, false>), g16, dim3(512), 0, 0, b3);
              }), flop_x);
          rep("bf16x3 + shortcut (split order)", time_ms([&] {
                hipLaunchKernelGGL((conv3x3_db_kernel<true, true, 0, false, 0, false, false, 2, true>), g16, dim3(512), 0, 0,
                                   b3);
              }), flop_x);
          CK(hipFree(lo));
        }
        unsigned int* dm;
        CK(hipMalloc(&dm, 8));
        CK(hipMemset(dm, 0, 8));
        ConvArgs ax2 = ax;
        ax2.out.ptr = out2;
        hipLaunchKernelGGL((conv3x3_db_kernel<true, true, 0, false, 1, true>), g32, dim3(512), 0, 0, ax);
        hipLaunchKernelGGL((conv3x3_db_kernel<true, true, 0, false, 1, true, 2>), g32, dim3(512), 0, 0, ax2);
        hipLaunchKernelGGL(max_diff, dim3(2048), dim3(256), 0, 0, out, out2, n_act, dm);
        unsigned int hh[2];
        CK(hipMemcpy(hh, dm, 8, hipMemcpyDeviceToHost));
        float d, m;
        memcpy(&d, &hh[0], 4);
        memcpy(&m, &hh[1], 4);
        printf("L%d%s DMA-ring shortcut vs LDS-staged: max|diff| %.3e max|out| %.3e %s\n", lvl, dec ? "dec" : "enc", d, m,
               d == 0.f ? "IDENTICAL" : d <= 1e-5f * m ? "OK (summation order)" : "MISMATCH");
        CK(hipFree(dm));
        CK(hipFree(x));
        CK(hipFree(hi));
        CK(hipFree(w));
        CK(hipFree(out));
        CK(hipFree(out2));
        CK(hipFree(stats));
      }
    return 0;
  }
  if (only_wino) {
    // Winograd F(2, 3) conv3x3_wino_kernel (SRC_ACT32 input) vs the direct conv3x3_db_kernel (act_split
    // planes) on the level shapes; random operands (timing only -- parity is tests/test_gpu_parity.py)
    for (int lvl = 0; lvl < 4; ++lvl) {
      const int C = 128 * (lvl + 1), T = 256 >> lvl, F = 1024 >> lvl;
      const int64_t n_act = (int64_t)B * T * F * C;
      float *x, *out;
      uint16_t *hi, *lo, *w, *ww;
      double* stats;
      const int nblk = C / 64, nch = C / kConvBK;
      const int64_t w_elems = (int64_t)nblk * nch * 2 * 9 * 64 * 16;
      const int64_t ww_elems = (int64_t)nblk * (nch * 2 * kWinoMainImg + nch * kWinoShortImg);
      CK(hipMalloc(&x, n_act * 4));
      CK(hipMalloc(&hi, n_act * 2));
      CK(hipMalloc(&lo, n_act * 2));
      CK(hipMalloc(&w, w_elems * 2));
      CK(hipMalloc(&ww, ww_elems * 2));
      CK(hipMalloc(&out, n_act * 4));
      CK(hipMalloc(&stats, (size_t)B * C * 2 * 8));
      hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint16_t*>(x), n_act * 2, 4u, 1.f);
      hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, hi, n_act, 1u, 1.f);
      hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, lo, n_act, 2u, 1.f / 256);
      hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, w, w_elems, 3u, 0.03f);
      hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, ww, ww_elems, 5u, 0.03f);
      CK(hipDeviceSynchronize());
      ConvArgs a{};
      a.in.src[0] = Src{nullptr, nullptr, nullptr, C, SRC_PRE, hi, lo};
      a.in.src[1] = a.in.src[0];
      a.in.C_split = a.in.C_in = C;
      a.out.ptr = out;
      a.out.stats = stats;
      a.out.C_out = C;
      a.w = w;
      a.T_in = a.T_out = T;
      a.F_in = a.F_out = F;
      a.n_cols = C;
      a.n_chunks = nch;
      ConvArgs aw = a;
      aw.in.src[0] = Src{x, nullptr, nullptr, C, SRC_ACT32, nullptr, nullptr};
      aw.in.src[1] = aw.in.src[0];
      aw.w = ww;
      ConvArgs ax = aw;  // + fused 1x1 shortcut over a raw C-channel input
      ax.xin.src[0] = Src{x, nullptr, nullptr, C, SRC_RAW, nullptr, nullptr};
      ax.xin.src[1] = ax.xin.src[0];
      ax.xin.C_split = ax.xin.C_in = C;
      ax.x_chunks = nch;
      ConvArgs adx = a;
      adx.xin = ax.xin;
      adx.x_chunks = nch;
      const double flop = 2.0 * B * T * F * (double)C * C * 9;
      const dim3 grid((unsigned)(((T + 15) / 16) * (F / kTF) * ((C + 63) / 64)), 1u, (unsigned)B);
      auto rep = [&](const char* v, float ms) { printf("L%-4d %-26s %9.3f %9.1f\n", lvl, v, ms, flop / ms * 1e-9); };
      rep("db", time_ms([&] { hipLaunchKernelGGL((conv3x3_db_kernel<true, false, 0>), grid, dim3(512), 0, 0, a); }));
      rep("wino", time_ms([&] { hipLaunchKernelGGL((conv3x3_wino_kernel<true, false, 0>), grid, dim3(512), 0, 0, aw); }));
      rep("wino sliced staging", time_ms([&] { hipLaunchKernelGGL((conv3x3_wino_kernel<true, false, 0, false, 0, true>), grid, dim3(512), 0, 0, aw); }));
      rep("wino frdb", time_ms([&] { hipLaunchKernelGGL((conv3x3_wino_kernel<true, false, 0, true>), grid, dim3(512), 0, 0, aw); }));
      rep("wino abl1 no V writes", time_ms([&] { hipLaunchKernelGGL((conv3x3_wino_kernel<true, false, 0, false, 1>), grid, dim3(512), 0, 0, aw); }));
      rep("wino abl4 no rows 16/17", time_ms([&] { hipLaunchKernelGGL((conv3x3_wino_kernel<true, false, 0, false, 4>), grid, dim3(512), 0, 0, aw); }));
      rep("wino abl2 no W DMA", time_ms([&] { hipLaunchKernelGGL((conv3x3_wino_kernel<true, false, 0, false, 2>), grid, dim3(512), 0, 0, aw); }));
      rep("wino abl3 no staging", time_ms([&] { hipLaunchKernelGGL((conv3x3_wino_kernel<true, false, 0, false, 3>), grid, dim3(512), 0, 0, aw); }));
      rep("wino abl3 no stg/epi", time_ms([&] { hipLaunchKernelGGL((conv3x3_wino_kernel<true, false, 2, false, 3>), grid, dim3(512), 0, 0, aw); }));
      rep("wino no epilogue",
          time_ms([&] { hipLaunchKernelGGL((conv3x3_wino_kernel<true, false, 2>), grid, dim3(512), 0, 0, aw); }));
      rep("db + shortcut", time_ms([&] { hipLaunchKernelGGL((conv3x3_db_kernel<true, true, 0>), grid, dim3(512), 0, 0, adx); }));
      rep("wino + shortcut",
          time_ms([&] { hipLaunchKernelGGL((conv3x3_wino_kernel<true, true, 0>), grid, dim3(512), 0, 0, ax); }));
      CK(hipFree(x));
      CK(hipFree(hi));
      CK(hipFree(lo));
      CK(hipFree(w));
      CK(hipFree(ww));
      CK(hipFree(out));
      CK(hipFree(stats));
    }
    return 0;
  }
  if (only_act) {
    // act_split + pre-activated conv3x3_db_kernel vs conv3x3_db_kernel<ACT> (norm + GELU + split fused
    // into the staging) on the level shapes; cat: two channel-concatenated sources (decoder tfc1)
    for (int lvl = 0; lvl < 4; ++lvl)
      for (int cat = 0; cat < 2; ++cat) {
        const int Co = 128 * (lvl + 1), C = cat ? 2 * Co : Co, T = 256 >> lvl, F = 1024 >> lvl;
        const int64_t n_act = (int64_t)B * T * F * C, n_out = (int64_t)B * T * F * Co;
        float *x, *out, *out2;
        uint16_t *hi, *lo, *w;
        double *st_x, *st_o;
        const int nblk = Co / 64, nch = C / kConvBK;
        const int64_t w_elems = (int64_t)nblk * nch * 2 * 9 * 64 * 16;
        CK(hipMalloc(&x, n_act * 4));
        CK(hipMalloc(&hi, n_act * 2));
        CK(hipMalloc(&lo, n_act * 2));
        CK(hipMalloc(&w, w_elems * 2));
        CK(hipMalloc(&out, n_out * 4));
        CK(hipMalloc(&out2, n_out * 4));
        CK(hipMalloc(&st_x, (size_t)B * C * 16));
        CK(hipMalloc(&st_o, (size_t)B * Co * 16));
        hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint16_t*>(x), n_act * 2, 4u, 1.f);
        hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, w, w_elems, 3u, 0.03f);
        std::vector<double> sth((size_t)B * C * 2);
        for (size_t i = 0; i < sth.size(); i += 2) { sth[i] = 0.1 * (double)T * F; sth[i + 1] = 0.8 * (double)T * F; }
        CK(hipMemcpy(st_x, sth.data(), sth.size() * 8, hipMemcpyHostToDevice));
        GemmIn gin{};
        const int c0 = cat ? Co : C;
        gin.src[0] = Src{x, st_x, nullptr, c0, SRC_NORM_GELU, nullptr, nullptr};
        gin.src[1] = cat ? Src{x + (int64_t)B * T * F * c0, st_x + (size_t)B * c0 * 2, nullptr, C - c0, SRC_NORM_GELU,
                               nullptr, nullptr}
                         : gin.src[0];
        gin.C_split = c0;
        gin.C_in = C;
        gin.inv_count = 1.0 / ((double)T * F);
        ConvArgs a{};
        a.out.ptr = out;
        a.out.stats = st_o;
        a.out.C_out = Co;
        a.w = w;
        a.T_in = a.T_out = T;
        a.F_in = a.F_out = F;
        a.n_cols = Co;
        a.n_chunks = nch;
        ConvArgs ap = a;     // pre-activated operands from act_split
        ap.in = GemmIn{};
        ap.in.src[0] = Src{nullptr, nullptr, nullptr, C, SRC_PRE, hi, lo};
        ap.in.src[1] = ap.in.src[0];
        ap.in.C_split = C;
        ap.in.C_in = C;
        ConvArgs af = a;     // fused
        af.in = gin;
        af.out.ptr = out2;
        const double flop = 2.0 * B * T * F * (double)Co * C * 9;
        const dim3 grid((unsigned)(((T + 15) / 16) * (F / kTF) * ((Co + 63) / 64)), 1u, (unsigned)B);
        const float ms_split = time_ms([&] { launch_act_split(gin, (int64_t)T * F, B, hi, lo, 0); });
        const float ms_pre = time_ms([&] { hipLaunchKernelGGL((conv3x3_db_kernel<true, false, 0, false>), grid, dim3(512), 0, 0, ap); });
        const float ms_act = time_ms([&] { hipLaunchKernelGGL((conv3x3_db_kernel<true, false, 0, true>), grid, dim3(512), 0, 0, af); });
        unsigned int* dm;
        CK(hipMalloc(&dm, 8));
        CK(hipMemset(dm, 0, 8));
        launch_act_split(gin, (int64_t)T * F, B, hi, lo, 0);
        hipLaunchKernelGGL((conv3x3_db_kernel<true, false, 0, false>), grid, dim3(512), 0, 0, ap);
        hipLaunchKernelGGL((conv3x3_db_kernel<true, false, 0, true>), grid, dim3(512), 0, 0, af);
        hipLaunchKernelGGL(max_diff, dim3(2048), dim3(256), 0, 0, out, out2, n_out, dm);
        unsigned int hh[2];
        CK(hipMemcpy(hh, dm, 8, hipMemcpyDeviceToHost));
        float d, m;
        memcpy(&d, &hh[0], 4);
        memcpy(&m, &hh[1], 4);
        printf("L%d%s C_in %4d: act_split %7.3f + db %7.3f = %7.3f ms | fused %7.3f ms (%6.1f TF/s) | max|diff| "
               "%.2e (max|out| %.2e) %s\n", lvl, cat ? " cat" : "    ", C, ms_split, ms_pre, ms_split + ms_pre, ms_act,
               flop / ms_act * 1e-9, d, m, d == 0.f ? "IDENTICAL" : "DIFFERENT");
        CK(hipFree(dm));
        CK(hipFree(x));
        CK(hipFree(hi));
        CK(hipFree(lo));
        CK(hipFree(w));
        CK(hipFree(out));
        CK(hipFree(out2));
        CK(hipFree(st_x));
        CK(hipFree(st_o));
      }
    return 0;
  }
  for (int lvl = 0; lvl < (only_tdf ? 0 : 4); ++lvl) {
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
    const int n_work = (int)grid.x * B;
    int n_cu = 0;
    CK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0));
    const dim3 pgrid((unsigned)std::min(n_work, n_cu));
    rep("conv3x3 (launch_conv)", time_ms([&] {
          CK(hipMemsetAsync(stats, 0, (size_t)B * C * 16, 0));
          launch_conv(CONV3X3, 64, 1, a, B, 0);
        }));
    rep("m16", time_ms([&] {
          CK(hipMemsetAsync(stats, 0, (size_t)B * C * 16, 0));
          hipLaunchKernelGGL((conv3x3_m16_kernel<true, false, 0>), pgrid, dim3(512), 0, 0, a, n_work);
        }));
    rep("m16 no statistics",
        time_ms([&] { hipLaunchKernelGGL((conv3x3_m16_kernel<true, false, 1>), pgrid, dim3(512), 0, 0, a, n_work); }));
    rep("m16 no epilogue",
        time_ms([&] { hipLaunchKernelGGL((conv3x3_m16_kernel<true, false, 2>), pgrid, dim3(512), 0, 0, a, n_work); }));
    rep("db (round 1)", time_ms([&] { hipLaunchKernelGGL((conv3x3_db_kernel<true, false, 0>), grid, dim3(512), 0, 0, a); }));
    {  // agreement: m16 vs db on the same operands (both bf16x3, fp32 accumulate; summation order differs)
      float* out2;
      unsigned int* dm;
      CK(hipMalloc(&out2, n_act * 4));
      CK(hipMalloc(&dm, 8));
      CK(hipMemset(dm, 0, 8));
      hipLaunchKernelGGL((conv3x3_m16_kernel<true, false, 0>), pgrid, dim3(512), 0, 0, a, n_work);
      ConvArgs a2 = a;
      a2.out.ptr = out2;
      hipLaunchKernelGGL((conv3x3_db_kernel<true, false, 0>), grid, dim3(512), 0, 0, a2);
      hipLaunchKernelGGL(max_diff, dim3(2048), dim3(256), 0, 0, out, out2, n_act, dm);
      unsigned int h[2];
      CK(hipMemcpy(h, dm, 8, hipMemcpyDeviceToHost));
      float d, m;
      memcpy(&d, &h[0], 4);
      memcpy(&m, &h[1], 4);
      printf("L%-4d m16 vs db: max|diff| %.3e  max|out| %.3e  %s\n", lvl, d, m, d <= 1e-4f * m ? "OK" : "MISMATCH");
      CK(hipFree(out2));
      CK(hipFree(dm));
    }
    CK(hipFree(hi));
    CK(hipFree(lo));
    CK(hipFree(w));
    CK(hipFree(out));
    CK(hipFree(stats));
  }
  // TDF Linears (first: NHWC -> tiled U, second: U -> NHWC + residual) on the level shapes
  for (int lvl = 0; lvl < 3; ++lvl) {
    const int C = 128 * (lvl + 1), T = 256 >> lvl, F = 1024 >> lvl, Fb = F / 4;
    const int64_t n_act = (int64_t)B * T * F * C;
    const int64_t n_u = tdf_u_floats((int64_t)B * T * C, Fb);
    float *x, *h, *u;
    double *st_x, *st_u, *st_o;
    uint16_t *w1, *w2;
    const int64_t w1n = (int64_t)((Fb + tdf_block_rows(Fb) - 1) / tdf_block_rows(Fb)) * ((F + 31) / 32) * 2 *
                        tdf_block_rows(Fb) * 32;
    const int64_t w2n = (int64_t)((F + tdf_block_rows(F) - 1) / tdf_block_rows(F)) * ((Fb + 31) / 32) * 2 *
                        tdf_block_rows(F) * 32;
    CK(hipMalloc(&x, n_act * 4));
    CK(hipMalloc(&h, n_act * 4));
    CK(hipMalloc(&u, n_u * 4));
    CK(hipMalloc(&st_x, (size_t)B * C * 16));
    CK(hipMalloc(&st_u, (size_t)B * C * 16));
    CK(hipMalloc(&st_o, (size_t)B * C * 16));
    CK(hipMalloc(&w1, w1n * 2));
    CK(hipMalloc(&w2, w2n * 2));
    hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint16_t*>(x), n_act * 2, 4u, 1.f);
    hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint16_t*>(u), n_u * 2, 5u, 1.f);
    hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, w1, w1n, 6u, 0.03f);
    hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, w2, w2n, 7u, 0.05f);
    std::vector<double> sth((size_t)B * C * 2);
    for (size_t i = 0; i < sth.size(); i += 2) { sth[i] = 0.0; sth[i + 1] = (double)T * F; }
    CK(hipMemcpy(st_x, sth.data(), sth.size() * 8, hipMemcpyHostToDevice));
    for (size_t i = 0; i < sth.size(); i += 2) sth[i + 1] = (double)T * Fb;
    CK(hipMemcpy(st_u, sth.data(), sth.size() * 8, hipMemcpyHostToDevice));
    const double flop = 2.0 * B * T * (double)F * Fb * C;
    auto mk = [&](const float* in, const double* st, int K, int M, float* out, const float* res, const uint16_t* w,
                  double inv) {
      TdfArgs t{};
      t.in.src[0] = Src{in, st, nullptr, C, SRC_NORM_GELU, nullptr, nullptr};
      t.in.src[1] = t.in.src[0];
      t.in.C_split = C;
      t.in.C_in = C;
      t.in.inv_count = inv;
      t.out = GemmOut{out, res, st_o, C, 0};
      t.w = w;
      t.T = T;
      t.K = K;
      t.M = M;
      t.n_chunks = (K + 31) / 32;
      return t;
    };
    const TdfArgs t1 = mk(x, st_x, F, Fb, u, nullptr, w1, 1.0 / ((double)T * F));
    const TdfArgs t2 = mk(u, st_u, Fb, F, h, x, w2, 1.0 / ((double)T * Fb));
    const double b1 = (double)n_act * 4 + (double)B * T * C * Fb * 4, b2 = (double)n_act * 8 + (double)B * T * C * Fb * 4;
    uint16_t* up;
    CK(hipMalloc(&up, n_u * 4));
    TdfArgs t2p = t2;
    t2p.u_planes = up;
    const float ms1 = time_ms([&] { launch_tdf(1, t1, B, 0, 0); });
    const float ms2 = time_ms([&] { launch_tdf(1, t2, B, 0, 1); });
    const float ms2p = time_ms([&] { launch_tdf(1, t2p, B, 0, 1); });
    {  // agreement of the two second-Linear paths
      float* h2;
      unsigned int* dm;
      CK(hipMalloc(&h2, n_act * 4));
      CK(hipMalloc(&dm, 8));
      CK(hipMemset(dm, 0, 8));
      TdfArgs ta = t2, tb = t2p;
      tb.out.ptr = h2;
      launch_tdf(1, ta, B, 0, 1);
      launch_tdf(1, tb, B, 0, 1);
      hipLaunchKernelGGL(max_diff, dim3(2048), dim3(256), 0, 0, h, h2, n_act, dm);
      unsigned int hh[2];
      CK(hipMemcpy(hh, dm, 8, hipMemcpyDeviceToHost));
      float d, m;
      memcpy(&d, &hh[0], 4);
      memcpy(&m, &hh[1], 4);
      printf("L%-4d tdf2 pre-split vs in-kernel: max|diff| %.3e max|out| %.3e %s\n", lvl, d, m,
             d <= 1e-5f * m ? "OK" : "MISMATCH");
      CK(hipFree(h2));
      CK(hipFree(dm));
    }
    CK(hipFree(up));
    printf("L%-4d tdf1 (F %d -> %d)          %9.3f %9.1f  HBM-alg %.0f GB/s\n", lvl, F, Fb, ms1, flop / ms1 * 1e-9,
           b1 / ms1 * 1e-6);
    printf("L%-4d tdf2 (%d -> %d, +res)     %9.3f %9.1f  HBM-alg %.0f GB/s\n", lvl, Fb, F, ms2, flop / ms2 * 1e-9,
           b2 / ms2 * 1e-6);
    printf("L%-4d tdf2 pre-split U (+split) %9.3f %9.1f  HBM-alg %.0f GB/s\n", lvl, ms2p, flop / ms2p * 1e-9,
           b2 / ms2p * 1e-6);
    CK(hipFree(x));
    CK(hipFree(h));
    CK(hipFree(u));
    CK(hipFree(st_x));
    CK(hipFree(st_u));
    CK(hipFree(st_o));
    CK(hipFree(w1));
    CK(hipFree(w2));
  }
  return 0;
}
