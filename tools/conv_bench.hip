// Micro-benchmark of the MDX23C contraction kernels at the vocals-config shapes (diagnostic).
// Build:  hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I sesa-audio-separation_amd/csrc \
//           tools/conv_bench.hip sesa-audio-separation_amd/csrc/sesa_tapgemm.hip \
//           sesa-audio-separation_amd/csrc/sesa_capi.cpp -o /tmp/conv_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "sesa_common.hpp"
#include "sesa_tapgemm.hpp"

using namespace sesa;

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);           \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

template <class T>
T* dalloc(size_t n, float fill_scale = 0.f) {
  T* p;
  CK(hipMalloc(&p, n * sizeof(T)));
  CK(hipMemset(p, 0, n * sizeof(T)));
  if (fill_scale != 0.f) {
    std::vector<T> h(n);
    for (size_t i = 0; i < n; ++i) h[i] = (T)(fill_scale * ((rand() / (float)RAND_MAX) - 0.5f));
    CK(hipMemcpy(p, h.data(), n * sizeof(T), hipMemcpyHostToDevice));
  }
  return p;
}

// random bf16 bit patterns in +-0.05 (non-zero operands: zero MFMA operands raise the clock)
uint16_t* dalloc_bf16(size_t n) {
  std::vector<uint16_t> h(n);
  for (size_t i = 0; i < n; ++i) {
    float f = 0.1f * ((rand() / (float)RAND_MAX) - 0.5f);
    uint32_t u;
    memcpy(&u, &f, 4);
    h[i] = (uint16_t)(u >> 16);
  }
  uint16_t* p;
  CK(hipMalloc(&p, n * 2));
  CK(hipMemcpy(p, h.data(), n * 2, hipMemcpyHostToDevice));
  return p;
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 16;
  const int x3 = argc > 2 ? atoi(argv[2]) : 1;
  const bool nostats = argc > 3 && atoi(argv[3]) == 1;  // ablation: no norm-statistics atomics
  struct Shape { int T, F, Cin, Cout, kind; };
  Shape shapes[] = {{256, 1024, 128, 128, CONV3X3}, {128, 512, 256, 256, CONV3X3}, {64, 256, 384, 384, CONV3X3},
                    {32, 128, 512, 512, CONV3X3}, {16, 64, 640, 640, CONV3X3},  {256, 1024, 128, 128, CONV1X1},
                    {256, 1024, 256, 128, CONV1X1}, {128, 512, 128, 256, CONV2X2S2}, {128, 512, 256, 128, DECONV2X2S2},
                    {256, 1024, 128, 128, 100 + CONV3X3}};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const bool only_tdf = getenv("ONLY_TDF") != nullptr;
  const bool only_conv = getenv("ONLY_CONV") != nullptr;
  for (auto& s0 : shapes) {
    if (only_tdf) break;
    Shape s = s0;
    const bool xtra = s.kind >= 100;  // conv3x3 with the block input fused as a 1x1 shortcut (extra K)
    if (xtra) s.kind -= 100;
    const bool ups = s.kind == DECONV2X2S2;
    const int taps = s.kind == CONV3X3 ? 9 : (s.kind == CONV2X2S2 ? 4 : 1);
    const int Tin = s.T, Fin = s.F;
    const int Tout = s.kind == CONV2X2S2 ? s.T / 2 : s.T, Fout = s.kind == CONV2X2S2 ? s.F / 2 : s.F;
    const int ncols = ups ? 4 * s.Cout : s.Cout;
    const int bn = 64;
    size_t in_n = (size_t)B * Tin * Fin * s.Cin;
    size_t out_n = (size_t)B * Tout * Fout * s.Cout * (ups ? 4 : 1);
    float* x = dalloc<float>(in_n, 2.f);
    float* y = dalloc<float>(out_n);
    double* st_in = dalloc<double>((size_t)B * s.Cin * 2);
    double* st_out = dalloc<double>((size_t)B * s.Cout * 2);
    std::vector<double> hs((size_t)B * s.Cin * 2);
    for (size_t i = 0; i < hs.size(); i += 2) { hs[i] = 0.0; hs[i + 1] = (double)Tin * Fin * 0.33; }
    CK(hipMemcpy(st_in, hs.data(), hs.size() * 8, hipMemcpyHostToDevice));
    float* gam = dalloc<float>(s.Cin, 1.f);
    float* bet = dalloc<float>(s.Cin, 0.2f);
    size_t wn = (size_t)((ncols + bn - 1) / bn) * ((s.Cin / 16) * 2 * taps * bn * 16 + (xtra ? (s.Cin / 16) * 2 * bn * 16 : 0));
    uint16_t* w = dalloc_bf16(wn);
    const bool pre = s.kind != CONV1X1;
    uint16_t* xh = pre ? dalloc_bf16(in_n) : nullptr;
    uint16_t* xl = pre ? dalloc_bf16(in_n) : nullptr;
    ConvArgs a{};
    a.in.src[0] = pre ? Src{x, st_in, nullptr, s.Cin, SRC_PRE, xh, xl} : Src{x, st_in, nullptr, s.Cin, SRC_NORM_GELU};
    a.in.src[1] = a.in.src[0];
    a.in.C_split = s.Cin;
    a.in.C_in = s.Cin;
    a.in.gamma = gam;
    a.in.beta = bet;
    a.in.inv_count = 1.0 / ((double)Tin * Fin);
    a.out = GemmOut{y, nullptr, nostats ? nullptr : st_out, s.Cout, 0};
    a.w = w;
    a.T_in = Tin;
    a.F_in = Fin;
    a.T_out = ups ? Tin : Tout;
    a.F_out = ups ? Fin : Fout;
    a.n_cols = ncols;
    a.n_chunks = s.Cin / 16;
    if (xtra) {
      a.xin = a.in;
      a.xin.src[0] = Src{x, nullptr, nullptr, s.Cin, SRC_RAW};
      a.xin.src[1] = a.xin.src[0];
      a.x_chunks = s.Cin / 16;
    }
    for (int it = 0; it < 2; ++it)
      if (launch_conv(s.kind, bn, x3, a, B, 0)) { printf("launch failed: %s\n", sesa_last_error()); return 1; }
    CK(hipDeviceSynchronize());
    const int iters = 5;
    CK(hipEventRecord(e0, 0));
    for (int it = 0; it < iters; ++it) launch_conv(s.kind, bn, x3, a, B, 0);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= iters;
    const double flop = 2.0 * B * (double)(ups ? Tin * Fin : Tout * Fout) * ncols * (s.Cin * taps + (xtra ? s.Cin : 0));
    printf("kind %d%s T%4d F%5d Cin%4d Cout%4d B%2d x3=%d: %8.3f ms  %7.1f TF alg  (%.1f%% of %s peak)\n", s.kind, xtra ? "+sc" : "", s.T, s.F,
           s.Cin, s.Cout, B, x3, ms, flop / ms / 1e9, 100 * flop / ms / 1e9 / (x3 ? 833.3 : 2500.0),
           x3 ? "bf16x3" : "bf16");
    CK(hipFree(x)); CK(hipFree(y)); CK(hipFree(st_in)); CK(hipFree(st_out)); CK(hipFree(gam)); CK(hipFree(bet));
    CK(hipFree(w));
    if (pre) { CK(hipFree(xh)); CK(hipFree(xl)); }
  }
  if (!only_tdf) {  // act_split over a level-0 tensor
    const int64_t npos = 256 * 1024;
    const int C = 128;
    float* x = dalloc<float>((size_t)B * npos * C, 2.f);
    double* st_in = dalloc<double>((size_t)B * C * 2);
    std::vector<double> hs((size_t)B * C * 2);
    for (size_t i = 0; i < hs.size(); i += 2) { hs[i] = 0.0; hs[i + 1] = (double)npos * 0.33; }
    CK(hipMemcpy(st_in, hs.data(), hs.size() * 8, hipMemcpyHostToDevice));
    uint16_t *hi, *lo;
    CK(hipMalloc(&hi, (size_t)B * npos * C * 2));
    CK(hipMalloc(&lo, (size_t)B * npos * C * 2));
    GemmIn in{};
    in.src[0] = Src{x, st_in, nullptr, C, SRC_NORM_GELU};
    in.src[1] = in.src[0];
    in.C_split = C;
    in.C_in = C;
    in.inv_count = 1.0 / npos;
    launch_act_split(in, npos, B, hi, lo, 0);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int it = 0; it < 5; ++it) launch_act_split(in, npos, B, hi, lo, 0);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= 5;
    printf("act_split T 256 F 1024 C 128 B%2d: %8.3f ms  %7.1f GB/s (8 B/elem)\n", B, ms, 8.0 * B * npos * C / ms / 1e6);
    CK(hipFree(x)); CK(hipFree(st_in)); CK(hipFree(hi)); CK(hipFree(lo));
  }
  // TDF
  if (only_conv) return 0;
  struct TShape { int T, K, M, C; };
  TShape ts[] = {{256, 1024, 256, 128}, {256, 256, 1024, 128}, {128, 512, 128, 256}, {128, 128, 512, 256},
                 {32, 128, 32, 512}, {32, 32, 128, 512}, {8, 32, 8, 768}, {8, 8, 32, 768}};
  int tio[] = {0, 1, 0, 1, 0, 1, 0, 1};
  int ti = 0;
  for (auto& s : ts) {
    const int io = tio[ti++];
    size_t in_n = (size_t)tdf_u_floats((int64_t)B * s.T * s.C, s.K), out_n = (size_t)tdf_u_floats((int64_t)B * s.T * s.C, s.M);
    float* x = dalloc<float>(in_n, 2.f);
    float* y = dalloc<float>(out_n);
    double* st_in = dalloc<double>((size_t)B * s.C * 2);
    double* st_out = dalloc<double>((size_t)B * s.C * 2);
    const int BM = tdf_block_rows(s.M);
    size_t wn = (size_t)((s.M + BM - 1) / BM) * ((s.K + 31) / 32) * 2 * BM * 32;
    uint16_t* w = dalloc_bf16(wn);
    TdfArgs a{};
    a.in.src[0] = Src{x, st_in, nullptr, s.C, SRC_NORM_GELU};
    a.in.src[1] = a.in.src[0];
    a.in.C_split = s.C;
    a.in.C_in = s.C;
    a.in.inv_count = 1.0 / ((double)s.T * s.K);
    a.out = GemmOut{y, (io == 1 && !getenv("NORES")) ? y : nullptr, nostats ? nullptr : st_out, s.C, 0};  // lin2: in-place residual
    a.w = w;
    a.T = s.T;
    a.K = s.K;
    a.M = s.M;
    a.n_chunks = (s.K + 31) / 32;
    for (int it = 0; it < 2; ++it) launch_tdf(x3, a, B, 0, io);
    CK(hipDeviceSynchronize());
    const int iters = 5;
    CK(hipEventRecord(e0, 0));
    for (int it = 0; it < iters; ++it) launch_tdf(x3, a, B, 0, io);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= iters;
    const double flop = 2.0 * B * (double)s.T * s.M * s.K * s.C;
    printf("tdf%d T%4d K%5d M%5d C%4d B%2d x3=%d: %8.3f ms  %7.1f TF alg (%.1f%%)\n", io, s.T, s.K, s.M, s.C, B, x3, ms,
           flop / ms / 1e9, 100 * flop / ms / 1e9 / (x3 ? 833.3 : 2500.0));
    CK(hipFree(x)); CK(hipFree(y)); CK(hipFree(st_in)); CK(hipFree(st_out)); CK(hipFree(w));
  }
  return 0;
}
