// attn_kernel vs a float64 CPU softmax(Q K^T / sqrt(d)) V on random data (diagnostic):
//   ./tools/attn_probe [L=100] [x3=1]
#include "../sesa-audio-separation_amd/csrc/sesa_tokgemm.hip"

#include <cmath>
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

int main(int argc, char** argv) {
  const int L = argc > 1 ? atoi(argv[1]) : 100, x3 = argc > 2 ? atoi(argv[2]) : 1;
  const bool onehot = argc > 3;   // Q_i = 100 e_i, K_j = e_j, V_j[d] = 64 j + d: O_i[d] ~ V_i[d] tells which key / d was read
  const int H = 2, S = 3, D = 64, ld = 3 * H * D;
  std::mt19937 rng(1);
  std::normal_distribution<float> nd(0.f, 1.f);
  std::vector<float> qkv((size_t)S * L * ld);
  for (auto& v : qkv) v = nd(rng);
  if (onehot)
    for (int s = 0; s < S; ++s)
      for (int i = 0; i < L; ++i)
        for (int h = 0; h < H; ++h)
          for (int e = 0; e < D; ++e) {
            float* r = &qkv[((size_t)s * L + i) * ld];
            r[h * D + e] = (e == i % D) ? 100.f : 0.f;
            r[H * D + h * D + e] = (e == i % D) ? 1.f : 0.f;
            r[2 * H * D + h * D + e] = (float)(64 * (i % 64) + e);
          }
  float *dq, *dout;
  (void)hipMalloc(&dq, qkv.size() * 4);
  (void)hipMalloc(&dout, (size_t)S * L * H * D * 4);
  (void)hipMemcpy(dq, qkv.data(), qkv.size() * 4, hipMemcpyHostToDevice);
  AttnArgs a{};
  a.qkv = dq;
  a.ld = ld;
  a.k_off = H * D;
  a.v_off = 2 * H * D;
  a.g_off = -1;
  a.out = dout;
  a.o_ld = H * D;
  a.L = L;
  a.n_seq = S;
  a.heads = H;
  a.sdiv = 1;
  a.smul_a = L;
  a.smul_b = 0;
  a.pstride = 1;
  a.dh = D;
  if (launch_attention(a, x3, 0)) return 1;
  (void)hipDeviceSynchronize();
  std::vector<float> got((size_t)S * L * H * D);
  (void)hipMemcpy(got.data(), dout, got.size() * 4, hipMemcpyDeviceToHost);
  double max_err = 0, max_ref = 0;
  std::vector<double> sc(L);
  for (int s = 0; s < S; ++s)
    for (int h = 0; h < H; ++h)
      for (int i = 0; i < L; ++i) {
        const float* q = &qkv[((size_t)s * L + i) * ld + h * D];
        double mx = -1e300;
        for (int j = 0; j < L; ++j) {
          const float* k = &qkv[((size_t)s * L + j) * ld + H * D + h * D];
          double d = 0;
          for (int e = 0; e < D; ++e) d += (double)q[e] * k[e];
          sc[j] = d / 8.0;
          mx = std::max(mx, sc[j]);
        }
        double sum = 0;
        for (int j = 0; j < L; ++j) sum += (sc[j] = std::exp(sc[j] - mx));
        for (int e = 0; e < D; ++e) {
          double o = 0;
          for (int j = 0; j < L; ++j) o += sc[j] * qkv[((size_t)s * L + j) * ld + 2 * H * D + h * D + e];
          o /= sum;
          const double g = got[((size_t)s * L + i) * H * D + h * D + e];
          max_err = std::max(max_err, std::fabs(g - o));
          max_ref = std::max(max_ref, std::fabs(o));
        }
      }
  printf("L %d x3 %d: max |err| %.3e (max |ref| %.3e)\n", L, x3, max_err, max_ref);
  if (onehot)
    for (int i = 0; i < 40; ++i) {
      printf("q %2d:", i);
      for (int e = 0; e < 8; ++e) {
        const float g = got[(size_t)i * H * D + e];
        printf(" (%d,%d)", (int)lrintf(g) / 64, (int)lrintf(g) % 64);
      }
      printf("\n");
    }
  return 0;
}
