// Standalone timing of the token-GEMM kernels on the BS-Roformer Linear shapes (diagnostic, not
// product): build with `make -C tools tokgemm_bench`, run on the GPU box.  Compiles
// sesa_tokgemm.hip into this translation unit so each kernel variant / ablation can be launched
// directly; times each with HIP events (median of 20) and cross-checks the variants' outputs.
#include "../sesa-audio-separation_amd/csrc/sesa_tokgemm.hip"

#include <algorithm>
#include <cstring>
#include <cstdarg>
#include <cstdio>
#include <random>
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

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

struct Shape {
  const char* name;
  int N, K, rope, rownorm, act, resid, split_out;
};

template <class F>
float time_ms(F&& launch, int reps = 20) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) launch();
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

// fp16 single-pass Linears (x3 == 2): the DEPTH-2 two-stage kernel vs the compact DEPTH-slot rings, with
// and without the epilogue; outputs of every ring depth must equal DEPTH 2 bit for bit.
template <int EP, int D>
void launch_f16(const TokGemmArgs& a, dim3 g) {
  hipLaunchKernelGGL((tok_gemm_glds_kernel<EP, true, D>), g, dim3(512), 0, 0, a);
}
// half tile: 256 x 128 per 256-thread workgroup, two workgroups per CU
template <int EP>
void launch_ht(const TokGemmArgs& a) {
  const dim3 g((unsigned)(((a.M + 255) / 256) * a.n_tiles_n));
  hipLaunchKernelGGL((tok_gemm_glds_kernel<EP, true, 3, true>), g, dim3(256), 0, 0, a);
}
template <int EP>
void f16_shape(const char* name, int M, int N, int K, TokGemmArgs a, dim3 g, size_t n_out, bool planes) {
  const double flop = 2.0 * M * (double)N * K;
  auto rep = [&](const char* v, float ms) { printf("%-4s %-28s %9.3f %9.1f\n", name, v, ms, flop / ms * 1e-9); };
  rep("f16 depth 2", time_ms([&] { launch_f16<EP, 2>(a, g); }));
  rep("f16 depth 3", time_ms([&] { launch_f16<EP, 3>(a, g); }));
  rep("f16 depth 4", time_ms([&] { launch_f16<EP, 4>(a, g); }));
  rep("f16 half tile (2 WG / CU)", time_ms([&] { launch_ht<EP>(a); }));
  rep("f16 half tile no epilogue", time_ms([&] { launch_ht<EP_F16 | EP_NONE>(a); }));
  rep("f16 depth 2 no epilogue", time_ms([&] { launch_f16<EP_F16 | EP_NONE, 2>(a, g); }));
  rep("f16 depth 4 no epilogue", time_ms([&] { launch_f16<EP_F16 | EP_NONE, 4>(a, g); }));
  if constexpr ((EP & EP_GELU) != 0)
    rep("f16 depth 4 no GELU", time_ms([&] { launch_f16<EP & ~EP_GELU, 4>(a, g); }));
  auto get = [&](auto launch) {
    std::vector<uint16_t> r(planes ? n_out : 2 * n_out);
    CK(hipMemset(planes ? (void*)a.out_hi : (void*)a.out, 0, planes ? n_out * 2 : n_out * 4));
    launch();
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(r.data(), planes ? (void*)a.out_hi : (void*)a.out, r.size() * 2, hipMemcpyDeviceToHost));
    return r;
  };
  const auto r2 = get([&] { launch_f16<EP, 2>(a, g); });
  const auto r3 = get([&] { launch_f16<EP, 3>(a, g); });
  const auto r4 = get([&] { launch_f16<EP, 4>(a, g); });
  const auto rh = get([&] { launch_ht<EP>(a); });
  printf("     depth 3 %s depth 2, depth 4 %s depth 2, half tile %s depth 2\n", r3 == r2 ? "IDENTICAL to" : "DIFFERS from",
         r4 == r2 ? "IDENTICAL to" : "DIFFERS from", rh == r2 ? "IDENTICAL to" : "DIFFERS from");
}

void run_f16(int M) {
  std::mt19937 rng(1);
  std::normal_distribution<float> nd(0.f, 1.f);
  const int Kmax = 2048, Nmax = 2048;
  std::vector<uint16_t> ha((size_t)M * Kmax);
  for (auto& v : ha) v = __builtin_bit_cast(uint16_t, (_Float16)nd(rng));
  uint16_t *a16, *ohi;
  float *out, *res;
  float2* rope;
  CK(hipMalloc(&a16, ha.size() * 2));
  CK(hipMemcpy(a16, ha.data(), ha.size() * 2, hipMemcpyHostToDevice));
  CK(hipMalloc(&out, (size_t)M * Nmax * 4));
  CK(hipMalloc(&res, (size_t)M * Nmax * 4));
  CK(hipMemset(res, 0, (size_t)M * Nmax * 4));
  CK(hipMalloc(&ohi, (size_t)M * Nmax * 2));
  {
    std::vector<float2> t(801 * 32);
    for (size_t i = 0; i < t.size(); ++i) t[i] = make_float2(cosf(0.01f * i), sinf(0.01f * i));
    CK(hipMalloc(&rope, t.size() * 8));
    CK(hipMemcpy(rope, t.data(), t.size() * 8, hipMemcpyHostToDevice));
  }
  printf("fp16 single pass, M=%d\n", M);
  const Shape shapes[] = {{"qkv", 1544, 512, 1, 1, TOK_ACT_NONE, 0, 0},
                          {"out", 512, 512, 0, 0, TOK_ACT_NONE, 1, 0},
                          {"ff1", 2048, 512, 0, 1, TOK_ACT_GELU, 0, 1},
                          {"ff2", 512, 2048, 0, 0, TOK_ACT_NONE, 1, 0}};
  for (const Shape& sh : shapes) {
    std::vector<uint16_t> blob;
    std::vector<float> bias;
    Gemm gm;
    gm.groups.push_back(pack_group(
        sh.N, sh.K, [&](int n, int k) { return 0.02f * (float)(((n * 131 + k * 71) % 97) - 48) / 48.f; }, true,
        [&](int n) { return 0.01f * (n % 7); }, blob, bias, true));
    uint16_t* w;
    float* b;
    CK(hipMalloc(&w, blob.size() * 2));
    CK(hipMemcpy(w, blob.data(), blob.size() * 2, hipMemcpyHostToDevice));
    CK(hipMalloc(&b, bias.size() * 4));
    CK(hipMemcpy(b, bias.data(), bias.size() * 4, hipMemcpyHostToDevice));
    upload_groups(gm);
    TokGemmArgs a{};
    a.w = w;
    a.bias = b;
    a.groups = gm.d_groups;
    a.n_groups = 1;
    a.n_tiles_n = gm.n_tiles_n;
    a.k8 = gm.k8;
    a.n4 = gm.n4;
    a.M = M;
    a.out = out;
    a.o_ld = sh.N;
    a.a_hi = a16;
    a.a_ld = sh.K;
    a.act = sh.act;
    a.dim_head = 64;
    if (sh.rope) {
      a.rope = rope;
      a.rope_cols = 1024;
      a.pos_F = 62;
      a.pos_T = 801;
      a.pos_time = 1;
    }
    if (sh.resid) a.residual = res;
    if (sh.split_out) {
      a.out_hi = ohi;
    }
    const dim3 g((unsigned)(((M + 255) / 256) * ((gm.n_tiles_n + 1) / 2)));
    const size_t n_out = (size_t)M * sh.N;
    if (sh.rope) f16_shape<EP_F16 | EP_ROPE>(sh.name, M, sh.N, sh.K, a, g, n_out, false);
    else if (sh.split_out) f16_shape<EP_F16 | EP_GELU | EP_SPLIT>(sh.name, M, sh.N, sh.K, a, g, n_out, true);
    else f16_shape<EP_F16 | EP_RES>(sh.name, M, sh.N, sh.K, a, g, n_out, false);
    CK(hipFree(w));
    CK(hipFree(b));
  }
  CK(hipFree(a16));
  CK(hipFree(out));
  CK(hipFree(res));
  CK(hipFree(ohi));
  CK(hipFree(rope));
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 198648;  // 4 chunks x 801 frames x 62 bands
  if (argc > 2 && !strcmp(argv[2], "f16")) {
    run_f16(M);
    return 0;
  }
  const bool small = argc > 2 && !strcmp(argv[2], "small");   // the parity tests' reduced BS-Roformer
  const Shape big_shapes[] = {{"qkv", 1544, 512, 1, 1, TOK_ACT_NONE, 0, 0},
                              {"out", 512, 512, 0, 0, TOK_ACT_NONE, 1, 0},
                              {"ff1", 2048, 512, 0, 1, TOK_ACT_GELU, 0, 1},
                              {"ff2", 512, 2048, 0, 0, TOK_ACT_NONE, 1, 0}};
  const Shape small_shapes[] = {{"qkv", 386, 128, 1, 1, TOK_ACT_NONE, 0, 0},
                                {"out", 128, 128, 0, 0, TOK_ACT_NONE, 1, 0},
                                {"ff1", 512, 128, 0, 1, TOK_ACT_GELU, 0, 1},
                                {"ff2", 128, 512, 0, 0, TOK_ACT_NONE, 1, 0}};
  const Shape* shapes = small ? small_shapes : big_shapes;
  std::mt19937 rng(0);
  std::normal_distribution<float> nd(0.f, 1.f);
  const int Kmax = 2048, Nmax = 2048;
  // A planes (random bf16 hi / lo of N(0,1) values), out, residual, rope table
  std::vector<uint16_t> hhi((size_t)M * Kmax), hlo((size_t)M * Kmax);
  for (size_t i = 0; i < hhi.size(); ++i) {
    const float v = nd(rng);
    hhi[i] = f2bf(v);
    hlo[i] = f2bf(v - bf2f(hhi[i]));
  }
  uint16_t *ahi, *alo, *ohi, *olo;
  float *out, *out2, *res, *rsc;
  float2* rope;
  CK(hipMalloc(&ahi, hhi.size() * 2));
  CK(hipMalloc(&alo, hlo.size() * 2));
  CK(hipMemcpy(ahi, hhi.data(), hhi.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(alo, hlo.data(), hlo.size() * 2, hipMemcpyHostToDevice));
  CK(hipMalloc(&out, (size_t)M * Nmax * 4));
  CK(hipMalloc(&out2, (size_t)M * Nmax * 4));
  CK(hipMalloc(&res, (size_t)M * Nmax * 4));
  CK(hipMemset(res, 0, (size_t)M * Nmax * 4));
  CK(hipMalloc(&ohi, (size_t)M * Nmax * 2));
  CK(hipMalloc(&olo, (size_t)M * Nmax * 2));
  CK(hipMalloc(&rsc, (size_t)M * 4));
  {
    std::vector<float> r(M, 1.0f);
    CK(hipMemcpy(rsc, r.data(), M * 4, hipMemcpyHostToDevice));
    std::vector<float2> t(801 * 32);
    for (auto& c : t) c = make_float2(0.8f, 0.6f);
    CK(hipMalloc(&rope, t.size() * 8));
    CK(hipMemcpy(rope, t.data(), t.size() * 8, hipMemcpyHostToDevice));
  }
  printf("M=%d\n%-4s %-28s %9s %9s\n", M, "gemm", "variant", "ms", "TF/s(alg)");
  for (int si = 0; si < 4; ++si) {
    const Shape& sh = shapes[si];
    std::vector<uint16_t> blob;
    std::vector<float> bias;
    Gemm gm;
    gm.groups.push_back(pack_group(
        sh.N, sh.K, [&](int n, int k) { return 0.02f * (float)(((n * 131 + k * 71) % 97) - 48) / 48.f; }, true,
        [&](int n) { return 0.01f * (n % 7); }, blob, bias));
    uint16_t* w;
    float* b;
    CK(hipMalloc(&w, blob.size() * 2));
    CK(hipMemcpy(w, blob.data(), blob.size() * 2, hipMemcpyHostToDevice));
    CK(hipMalloc(&b, bias.size() * 4));
    CK(hipMemcpy(b, bias.data(), bias.size() * 4, hipMemcpyHostToDevice));
    upload_groups(gm);
    TokGemmArgs a{};
    a.w = w;
    a.bias = b;
    a.groups = gm.d_groups;
    a.n_groups = 1;
    a.n_tiles_n = gm.n_tiles_n;
    a.k8 = gm.k8;
    a.M = M;
    a.out = out;
    a.o_ld = sh.N;
    a.a_hi = ahi;
    a.a_lo = alo;
    a.a_ld = sh.K;
    a.row_scale = rsc;
    a.rownorm = sh.rownorm;
    a.act = sh.act;
    a.dim_head = 64;
    if (sh.rope) {
      a.rope = rope;
      a.rope_cols = 1024;
      a.pos_F = 62;
      a.pos_T = 801;
      a.pos_time = 1;
    }
    if (sh.resid) a.residual = res;
    if (sh.split_out) {
      a.out_hi = ohi;
      a.out_lo = olo;
    }
    const double flop = 2.0 * M * (double)sh.N * sh.K;
    const dim3 gbig((unsigned)(((M + 255) / 256) * ((gm.n_tiles_n + 1) / 2)));
    const dim3 gv0((unsigned)(((M + 127) / 128) * gm.n_tiles_n));
    auto rep = [&](const char* v, float ms) { printf("%-4s %-28s %9.3f %9.1f\n", sh.name, v, ms, flop / ms * 1e-9); };
    TokGemmArgs a1 = a;
    a1.out = out2;
    a1.out_hi = nullptr;
    a1.out_lo = nullptr;
    a1.residual = nullptr;
    rep("v0 reg-staged 128x128", time_ms([&] { hipLaunchKernelGGL((tok_gemm_kernel<true, 256, 128, 2, 2, 2, false, false, true>), gv0, dim3(256), 0, 0, a); }));
    rep("glds 256x256 (launch_tok_gemm)", time_ms([&] { launch_tok_gemm(a, 1, 0); }));
    {
      setenv("SESA_TOKGEMM_M16", "1", 1);   // read once per process: time the M16 instantiation directly
      const int ep = (sh.rownorm ? EP_RS : 0) | (sh.rope ? EP_ROPE : 0) | (sh.act == TOK_ACT_GELU ? EP_GELU : 0) |
                     (sh.resid ? EP_RES : 0) | (sh.split_out ? EP_SPLIT : 0);
      auto l16 = [&] {
        switch (ep) {
          case EP_RS | EP_ROPE: hipLaunchKernelGGL((tok_gemm_glds_kernel<EP_RS | EP_ROPE, true>), gbig, dim3(512), 0, 0, a); break;
          case EP_RES: hipLaunchKernelGGL((tok_gemm_glds_kernel<EP_RES, true>), gbig, dim3(512), 0, 0, a); break;
          default: hipLaunchKernelGGL((tok_gemm_glds_kernel<EP_RS | EP_GELU | EP_SPLIT, true>), gbig, dim3(512), 0, 0, a);
        }
      };
      rep("glds 16x16x32", time_ms(l16));
      rep("glds 16x16x32 no epilogue", time_ms([&] { hipLaunchKernelGGL((tok_gemm_glds_kernel<EP_NONE, true>), gbig, dim3(512), 0, 0, a1); }));
      {  // plain epilogue (bias only): main-loop agreement
        TokGemmArgs p0 = a, p1 = a;
        p0.rope = p1.rope = nullptr;
        p0.rownorm = p1.rownorm = 0;
        p0.residual = p1.residual = nullptr;
        p0.out_hi = p1.out_hi = nullptr;
        p0.out_lo = p1.out_lo = nullptr;
        p0.act = p1.act = TOK_ACT_NONE;
        p1.out = out2;
        hipLaunchKernelGGL((tok_gemm_glds_kernel<0, true>), gbig, dim3(512), 0, 0, p0);
        hipLaunchKernelGGL((tok_gemm_glds_kernel<0, false>), gbig, dim3(512), 0, 0, p1);
        CK(hipDeviceSynchronize());
        std::vector<float> h1((size_t)M * sh.N), h2((size_t)M * sh.N);
        CK(hipMemcpy(h1.data(), out, h1.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(h2.data(), out2, h2.size() * 4, hipMemcpyDeviceToHost));
        double md = 0;
        size_t wq = 0;
        for (size_t q = 0; q < h1.size(); ++q)
          if (fabsf(h1[q] - h2[q]) > md) { md = fabsf(h1[q] - h2[q]); wq = q; }
        printf("     plain: max |m16 - 32x32| = %.3g at row %zu col %zu (%g vs %g)\n", md, wq / sh.N, wq % sh.N, h1[wq], h2[wq]);
      }
      // cross-check M16 vs 32x32 on the fp32 outputs
      if (!sh.split_out && !sh.resid) {
        TokGemmArgs a2 = a;
        a2.out = out2;
        l16();
        hipLaunchKernelGGL((tok_gemm_glds_kernel<EP_RS | EP_ROPE, false>), gbig, dim3(512), 0, 0, a2);
        CK(hipDeviceSynchronize());
        std::vector<float> h1((size_t)M * sh.N), h2((size_t)M * sh.N);
        CK(hipMemcpy(h1.data(), out, h1.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(h2.data(), out2, h2.size() * 4, hipMemcpyDeviceToHost));
        double md = 0;
        for (size_t q = 0; q < h1.size(); ++q) md = std::max(md, (double)fabsf(h1[q] - h2[q]));
        printf("     max |m16 - 32x32| = %.3g\n", md);
      }
    }
    rep("glds 256x256 raw store", time_ms([&] { hipLaunchKernelGGL((tok_gemm_glds_kernel<EP_RAW, false>), gbig, dim3(512), 0, 0, a1); }));
    rep("v0 bf16 (1 pass)", time_ms([&] { hipLaunchKernelGGL((tok_gemm_kernel<false, 256, 128, 2, 2, 2, false, false, true>), gv0, dim3(256), 0, 0, a); }));
    // cross-check v0 vs glds on the full epilogue (fp32 out, or hi + lo planes; residual = 1)
    {
      const size_t n_out = (size_t)M * sh.N;
      auto run_get = [&](bool glds) {
        CK(hipMemset(out, 0, n_out * 4));
        CK(hipMemset(ohi, 0, n_out * 2));
        CK(hipMemset(olo, 0, n_out * 2));
        if (sh.resid) {
          std::vector<float> one(n_out, 1.0f);
          CK(hipMemcpy(out, one.data(), n_out * 4, hipMemcpyHostToDevice));
          a.residual = out;
        }
        if (glds) launch_tok_gemm(a, 1, 0);
        else hipLaunchKernelGGL((tok_gemm_kernel<true, 256, 128, 2, 2, 2, false, false, true>), gv0, dim3(256), 0, 0, a);
        CK(hipDeviceSynchronize());
        a.residual = sh.resid ? res : nullptr;
        std::vector<float> r(n_out);
        if (sh.split_out) {
          std::vector<uint16_t> hh(n_out), ll(n_out);
          CK(hipMemcpy(hh.data(), ohi, n_out * 2, hipMemcpyDeviceToHost));
          CK(hipMemcpy(ll.data(), olo, n_out * 2, hipMemcpyDeviceToHost));
          for (size_t i = 0; i < n_out; ++i) r[i] = bf2f(hh[i]) + bf2f(ll[i]);
        } else {
          CK(hipMemcpy(r.data(), out, n_out * 4, hipMemcpyDeviceToHost));
        }
        return r;
      };
      const std::vector<float> r0 = run_get(false), r1 = run_get(true);
      double md = 0, mx = 0;
      size_t worst = 0;
      for (size_t i = 0; i < n_out; ++i) {
        const double e = fabs((double)r0[i] - r1[i]);
        if (e > md) { md = e; worst = i; }
        mx = std::max(mx, (double)fabsf(r0[i]));
      }
      printf("     max |v0 - glds| = %.3g (max |v0| %.3g) at row %zu col %zu\n", md, mx, worst / sh.N, worst % sh.N);
    }
    CK(hipFree(w));
    CK(hipFree(b));
  }
  CK(hipDeviceSynchronize());
  return 0;
}
