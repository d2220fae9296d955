// STFT / iSTFT for the MDX23C front and back end (gfx950).
//
// Reference: models/mdx23c_tfc_tdf_v3.py:14-30 (torch.stft, center=True, reflect, periodic
// Hann, onesided, cropped to dim_f) and :32-44 (Nyquist zero pad + torch.istft, no length).
//
// One workgroup per (signal, frame).  The 8192-point real DFT is computed as a 4096-point
// complex FFT of the even/odd packed frame (z[m] = v[2m] + i v[2m+1]) -- radix-4 Stockham
// autosort, six stages, ping-ponged between two 32 KiB LDS images -- followed by the
// real-spectrum split X[k] = E[k] + W_N^k O[k].  The inverse runs the mirror image.
// Twiddles / window come from per-device tables computed once in double on the host.
//
// HBM roofline (per frame of one signal): STFT reads 8192*4 B (2x overlap re-read through
// L2: algorithmic 1024*4 B new) and writes dim_f*8 B; iSTFT reads dim_f*8 B, writes the
// windowed frame 8192*4 B to the OLA scratch, and the OLA kernel reads it back once.
#include <hip/hip_runtime.h>

#include <cmath>
#include <mutex>
#include <vector>

#include "sesa_common.hpp"
#include "sesa_internal.hpp"

namespace sesa {

namespace {

constexpr int kFFT = 4096;   // complex FFT length (n_fft / 2)
constexpr int kNFFT = 8192;  // supported n_fft
constexpr int kThreads = 256;

struct SpectralTables {
  float2* tw4096 = nullptr;  // exp(-2 pi i j / 4096), j < 4096
  float2* twN = nullptr;     // exp(-2 pi i k / 8192), k < 4096
  float* window = nullptr;   // periodic Hann(8192)
};

std::mutex g_tab_mu;
std::vector<SpectralTables> g_tabs;  // indexed by device ordinal

}  // namespace

int get_spectral_tables(const float2** tw4096, const float2** twN, const float** window) {
  int dev = 0;
  SESA_CHECK_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(g_tab_mu);
  if ((int)g_tabs.size() <= dev) g_tabs.resize(dev + 1);
  SpectralTables& t = g_tabs[dev];
  if (!t.tw4096) {
    std::vector<float2> a(kFFT), b(kFFT);
    std::vector<float> w(kNFFT);
    for (int j = 0; j < kFFT; ++j) {
      double ang = -2.0 * M_PI * (double)j / (double)kFFT;
      a[j] = make_float2((float)cos(ang), (float)sin(ang));
      double angN = -2.0 * M_PI * (double)j / (double)kNFFT;
      b[j] = make_float2((float)cos(angN), (float)sin(angN));
    }
    for (int n = 0; n < kNFFT; ++n) w[n] = (float)(0.5 - 0.5 * cos(2.0 * M_PI * (double)n / (double)kNFFT));
    float2 *da = nullptr, *db = nullptr;
    float* dw = nullptr;
    SESA_CHECK_HIP(hipMalloc(&da, kFFT * sizeof(float2)));
    SESA_CHECK_HIP(hipMalloc(&db, kFFT * sizeof(float2)));
    SESA_CHECK_HIP(hipMalloc(&dw, kNFFT * sizeof(float)));
    SESA_CHECK_HIP(hipMemcpy(da, a.data(), kFFT * sizeof(float2), hipMemcpyHostToDevice));
    SESA_CHECK_HIP(hipMemcpy(db, b.data(), kFFT * sizeof(float2), hipMemcpyHostToDevice));
    SESA_CHECK_HIP(hipMemcpy(dw, w.data(), kNFFT * sizeof(float), hipMemcpyHostToDevice));
    t.tw4096 = da;
    t.twN = db;
    t.window = dw;
  }
  *tw4096 = t.tw4096;
  *twN = t.twN;
  *window = t.window;
  return SESA_OK;
}

namespace {

__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cconj(float2 a) { return make_float2(a.x, -a.y); }

// 4096-point radix-16 Stockham FFT: 3 stages (16^3), one 16-point DFT per thread per stage, held in
// registers (a radix-4 x radix-4 decomposition), 4 barriers instead of 7.  The first two stages write
// a padded image (index i stored at i + i / 16: the stride-16 store pattern of a stage is then
// bank-conflict free); the last stage writes natural order into `out`.
// `in` holds natural order; `pad` and `out` are distinct buffers of kFFTPad float2.  INV: conjugated
// twiddles (un-normalised inverse).
constexpr int kFFTPad = kFFT + kFFT / 16;

template <bool INV>
__device__ __forceinline__ void dft4(float2& a0, float2& a1, float2& a2, float2& a3) {
  const float2 s02 = cadd(a0, a2), d02 = csub(a0, a2), s13 = cadd(a1, a3), d13 = csub(a1, a3);
  // forward: y1 = d02 - i d13, y3 = d02 + i d13; inverse: the conjugate rotation
  const float2 jd13 = INV ? make_float2(-d13.y, d13.x) : make_float2(d13.y, -d13.x);
  a0 = cadd(s02, s13);
  a2 = csub(s02, s13);
  a1 = cadd(d02, jd13);
  a3 = csub(d02, jd13);
}

// in-register 16-point DFT: v[r] (r = 4 r1 + r2) -> v[k1 + 4 k2] = X[k1 + 4 k2]
template <bool INV>
__device__ __forceinline__ void dft16(float2 (&v)[16]) {
  // omega_16^j, j = 0..9 (forward: exp(-2 pi i j / 16))
  constexpr float C1 = 0.92387953251128674f, S1 = 0.38268343236508978f, C2 = 0.70710678118654752f;
  const float sg = INV ? 1.f : -1.f;
  const float2 w16[10] = {make_float2(1.f, 0.f),       make_float2(C1, sg * S1),  make_float2(C2, sg * C2),
                          make_float2(S1, sg * C1),     make_float2(0.f, sg * 1.f), make_float2(-S1, sg * C1),
                          make_float2(-C2, sg * C2),    make_float2(-C1, sg * S1), make_float2(-1.f, 0.f),
                          make_float2(-C1, -sg * S1)};
  float2 b[16];
#pragma unroll
  for (int r2 = 0; r2 < 4; ++r2) {  // 4-point DFTs over r1 -> B[r2][k1]
    float2 a0 = v[r2], a1 = v[4 + r2], a2 = v[8 + r2], a3 = v[12 + r2];
    dft4<INV>(a0, a1, a2, a3);
    b[r2 * 4 + 0] = a0;
    b[r2 * 4 + 1] = r2 ? cmul(a1, w16[r2]) : a1;
    b[r2 * 4 + 2] = r2 ? cmul(a2, w16[2 * r2]) : a2;
    b[r2 * 4 + 3] = r2 ? cmul(a3, w16[3 * r2]) : a3;
  }
#pragma unroll
  for (int k1 = 0; k1 < 4; ++k1) {  // 4-point DFTs over r2 -> X[k1 + 4 k2]
    float2 a0 = b[k1], a1 = b[4 + k1], a2 = b[8 + k1], a3 = b[12 + k1];
    dft4<INV>(a0, a1, a2, a3);
    v[k1] = a0;
    v[k1 + 4] = a1;
    v[k1 + 8] = a2;
    v[k1 + 12] = a3;
  }
}

__device__ __forceinline__ int padi(int i) { return i + (i >> 4); }

// X: input, natural order (kFFT float2); Y: result, natural order.  Both kFFTPad float2 (X holds
// the padded stage-2 image in between).
template <bool INV>
__device__ void fft4096(float2* X, float2* Y, const float2* __restrict__ tw) {
  static_assert(kThreads == 256, "one 16-point butterfly per thread per stage");
  const int b = threadIdx.x;
  float2 v[16];
  // stage 1 (s = 1, p = b): X[b + 256 r] -> Y'[16 b + k] * tw[k b]
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = X[b + 256 * r];
  dft16<INV>(v);
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    float2 w = tw[k * b];
    if (INV) w = cconj(w);
    Y[padi(16 * b + k)] = k ? cmul(v[k], w) : v[k];
  }
  // stage 2 (s = 16, q = b & 15, p = b >> 4): Y'[q + 16 (p + 16 r)] -> X'[q + 16 (16 p + k)] * tw[16 k p]
  __syncthreads();
  const int q = b & 15, p = b >> 4;
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = Y[padi(q + 16 * (p + 16 * r))];
  dft16<INV>(v);
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    float2 w = tw[16 * k * p];
    if (INV) w = cconj(w);
    X[padi(q + 16 * (16 * p + k))] = k ? cmul(v[k], w) : v[k];
  }
  // stage 3 (s = 256, p = 0): X'[b + 256 r] -> Y[b + 256 k] (natural order, no twiddle)
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = X[padi(b + 256 * r)];
  dft16<INV>(v);
#pragma unroll
  for (int k = 0; k < 16; ++k) Y[b + 256 * k] = v[k];
  __syncthreads();
}

// Output layouts of the forward transform.
//  0: reference [n_sig][2][dim_f][frames]
//  1: MDX23C channels-last cac2cws image [b][frame][dim_f/nsub][2*2*nsub], sig = b*2 + s,
//     channel = (s*2 + r)*nsub + k/Fs, column = k % Fs (mdx23c_tfc_tdf_v3.py:191-196, :213).
__global__ void __launch_bounds__(kThreads)
stft_kernel(const float* __restrict__ x, int len, int hop, int frames, int dim_f, int layout, int nsub,
            const float2* __restrict__ tw, const float2* __restrict__ twN, const float* __restrict__ win,
            float* __restrict__ out) {
  __shared__ float2 bufA[kFFTPad];
  __shared__ float2 bufB[kFFTPad];
  const int t = blockIdx.x;
  const int sig = blockIdx.y;
  const float* xs = x + (int64_t)sig * len;
  const int64_t base = (int64_t)t * hop - kNFFT / 2;  // center=True
  for (int m = threadIdx.x; m < kFFT; m += kThreads) {
    float v[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int n = 2 * m + e;
      int64_t pos = base + n;
      if (pos < 0) pos = -pos;                    // reflect (torch.stft pad_mode='reflect')
      if (pos >= len) pos = 2 * (int64_t)(len - 1) - pos;
      v[e] = xs[pos] * win[n];
    }
    bufA[m] = make_float2(v[0], v[1]);
  }
  fft4096<false>(bufA, bufB, tw);
  const float2* Z = bufB;
  auto bin = [&](int k) {  // real-spectrum split X[k] = E[k] + W_N^k O[k]
    const float2 zk = Z[k & (kFFT - 1)];
    const float2 zm = cconj(Z[(kFFT - k) & (kFFT - 1)]);
    const float2 E = make_float2(0.5f * (zk.x + zm.x), 0.5f * (zk.y + zm.y));
    const float2 D = csub(zk, zm);                         // O = D / (2i) = (D.y, -D.x)/2
    const float2 O = make_float2(0.5f * D.y, -0.5f * D.x);
    return cadd(E, cmul(twN[k], O));
  };
  if (layout == 0) {
    float* o = out + ((int64_t)sig * 2) * dim_f * frames;
    for (int k = threadIdx.x; k < dim_f; k += kThreads) {
      const float2 X = bin(k);
      o[(int64_t)k * frames + t] = X.x;
      o[((int64_t)dim_f + k) * frames + t] = X.y;
    }
  } else {
    // one thread per column: this signal's 2 * nsub channels of the record are contiguous
    // ((s * 2 + r) * nsub + sub), written as 16-B stores when nsub == 4
    const int Fs = dim_f / nsub;
    const int b = sig >> 1, s = sig & 1;
    const int C = 4 * nsub;
    for (int col = threadIdx.x; col < Fs; col += kThreads) {
      float* o = out + (((int64_t)b * frames + t) * Fs + col) * C + s * 2 * nsub;
      if (nsub == 4) {
        float2 X[4];
#pragma unroll
        for (int sub = 0; sub < 4; ++sub) X[sub] = bin(sub * Fs + col);
        reinterpret_cast<float4*>(o)[0] = make_float4(X[0].x, X[1].x, X[2].x, X[3].x);
        reinterpret_cast<float4*>(o)[1] = make_float4(X[0].y, X[1].y, X[2].y, X[3].y);
      } else {
        for (int sub = 0; sub < nsub; ++sub) {
          const float2 X = bin(sub * Fs + col);
          o[sub] = X.x;
          o[nsub + sub] = X.y;
        }
      }
    }
  }
}

// Inverse: one workgroup per (signal, frame); writes the windowed frame x[n]*w[n] (n < 8192)
// to frame_ws[sig][frame][8192].
//  layout 0: spec is reference [n_sig][2][dim_f][frames]
//  layout 1: spec is the MDX23C final channels-last image [b][frame][Fs][C] with
//            sig = (b*ni + instr)*2 + s, channel = ((instr*2 + s)*2 + r)*nsub + k/Fs
//            (cws2cac + reshape, mdx23c_tfc_tdf_v3.py:198-203, :234-238, :35-41).
__global__ void __launch_bounds__(kThreads)
istft_frames_kernel(const float* __restrict__ spec, int frames, int dim_f, int layout, int nsub, int ni,
                    const float2* __restrict__ tw, const float2* __restrict__ twN, const float* __restrict__ win,
                    float* __restrict__ frame_ws) {
  __shared__ float2 bufA[kFFTPad];
  __shared__ float2 bufB[kFFTPad];
  float2* Xs = bufB;  // bins 0..4095; bin 4096 (Nyquist) is always the zero pad (dim_f <= 4096)
  const int t = blockIdx.x;
  const int sig = blockIdx.y;
  if (layout == 0) {
    const float* sp = spec + ((int64_t)sig * 2) * dim_f * frames;
    for (int k = threadIdx.x; k < kFFT; k += kThreads)
      Xs[k] = k < dim_f ? make_float2(sp[(int64_t)k * frames + t], sp[((int64_t)dim_f + k) * frames + t])
                        : make_float2(0.f, 0.f);
  } else {
    // one thread per column: the signal's 2 * nsub channels ((instr * 2 + s) * 2 + r) * nsub + sub are
    // contiguous in the record (16-B loads when nsub == 4)
    const int Fs = dim_f / nsub;
    const int s = sig & 1, bi = sig >> 1;
    const int b = bi / ni, instr = bi - b * ni;
    const int C = ni * 4 * nsub;
    for (int col = threadIdx.x; col < Fs; col += kThreads) {
      const float* sp = spec + (((int64_t)b * frames + t) * Fs + col) * C + (instr * 2 + s) * 2 * nsub;
      if (nsub == 4) {
        const float4 re = reinterpret_cast<const float4*>(sp)[0], im = reinterpret_cast<const float4*>(sp)[1];
        Xs[0 * Fs + col] = make_float2(re.x, im.x);
        Xs[1 * Fs + col] = make_float2(re.y, im.y);
        Xs[2 * Fs + col] = make_float2(re.z, im.z);
        Xs[3 * Fs + col] = make_float2(re.w, im.w);
      } else {
        for (int sub = 0; sub < nsub; ++sub) Xs[sub * Fs + col] = make_float2(sp[sub], sp[nsub + sub]);
      }
    }
    for (int k = dim_f + threadIdx.x; k < kFFT; k += kThreads) Xs[k] = make_float2(0.f, 0.f);
  }
  __syncthreads();
  if (threadIdx.x == 0) Xs[0].y = 0.f;  // C2R ignores the imaginary part of DC
  __syncthreads();
  for (int k = threadIdx.x; k < kFFT; k += kThreads) {
    const float2 xk = Xs[k];
    const float2 xm = k == 0 ? make_float2(0.f, 0.f) : cconj(Xs[kFFT - k]);
    const float2 E = make_float2(0.5f * (xk.x + xm.x), 0.5f * (xk.y + xm.y));
    const float2 w = cconj(twN[k]);                       // exp(+2 pi i k / N)
    const float2 D = csub(xk, xm);
    const float2 O = cmul(make_float2(0.5f * D.x, 0.5f * D.y), w);
    bufA[k] = make_float2(E.x - O.y, E.y + O.x);          // E + i O
  }
  fft4096<true>(bufA, bufB, tw);
  const float2* z = bufB;
  float* fw = frame_ws + ((int64_t)sig * frames + t) * kNFFT;
  const float scale = 1.0f / (float)kFFT;
  for (int m = threadIdx.x; m < kFFT; m += kThreads) {
    const float2 v = z[m];
    const float2 o = make_float2(v.x * scale * win[2 * m], v.y * scale * win[2 * m + 1]);
    reinterpret_cast<float2*>(fw)[m] = o;
  }
}

// Overlap-add of the windowed frames and division by the window envelope (torch.istft,
// center=True: output sample j is full-signal position j + n_fft/2).
__global__ void istft_ola_kernel(const float* __restrict__ frame_ws, int frames, int hop, int out_len,
                                 const float* __restrict__ win, float* __restrict__ out) {
  const int sig = blockIdx.y;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= out_len) return;
  const int n = j + kNFFT / 2;
  int t_lo = n - kNFFT + 1 <= 0 ? 0 : (n - kNFFT + hop) / hop;
  int t_hi = n / hop;
  if (t_hi > frames - 1) t_hi = frames - 1;
  const float* fw = frame_ws + (int64_t)sig * frames * kNFFT;
  float acc = 0.f, env = 0.f;
  for (int t = t_lo; t <= t_hi; ++t) {
    const int o = n - t * hop;
    acc += fw[(int64_t)t * kNFFT + o];
    const float w = win[o];
    env += w * w;
  }
  out[(int64_t)sig * out_len + j] = acc / env;
}

}  // namespace

int stft_launch(const float* x, int n_sig, int len, int hop, int dim_f, int layout, int nsub, float* out,
                hipStream_t st) {
  const float2 *tw, *twN;
  const float* win;
  int rc = get_spectral_tables(&tw, &twN, &win);
  if (rc) return rc;
  const int frames = 1 + len / hop;
  dim3 grid(frames, n_sig);
  hipLaunchKernelGGL(stft_kernel, grid, dim3(kThreads), 0, st, x, len, hop, frames, dim_f, layout, nsub, tw, twN,
                     win, out);
  SESA_CHECK_LAUNCH();
  return SESA_OK;
}

int istft_launch(const float* spec, int n_sig, int dim_f, int frames, int hop, int layout, int nsub, int ni,
                 float* out, float* frame_ws, hipStream_t st) {
  const float2 *tw, *twN;
  const float* win;
  int rc = get_spectral_tables(&tw, &twN, &win);
  if (rc) return rc;
  hipLaunchKernelGGL(istft_frames_kernel, dim3(frames, n_sig), dim3(kThreads), 0, st, spec, frames, dim_f, layout,
                     nsub, ni, tw, twN, win, frame_ws);
  SESA_CHECK_LAUNCH();
  const int out_len = hop * (frames - 1);
  hipLaunchKernelGGL(istft_ola_kernel, dim3((out_len + 255) / 256, n_sig), dim3(256), 0, st, frame_ws, frames, hop,
                     out_len, win, out);
  SESA_CHECK_LAUNCH();
  return SESA_OK;
}

}  // namespace sesa

using namespace sesa;

extern "C" int sesa_stft_f32(const float* x, int n_sig, int len, int n_fft, int hop, int dim_f, float* out,
                             void* stream) {
  clear_error();
  SESA_REQUIRE(x && out && n_sig > 0, SESA_ERR_INVALID, "sesa_stft_f32: null pointer or n_sig <= 0");
  SESA_REQUIRE(n_fft == kNFFT, SESA_ERR_INVALID, "sesa_stft_f32: only n_fft=8192 is supported (got %d)", n_fft);
  SESA_REQUIRE(hop > 0 && len % hop == 0 && len > n_fft / 2, SESA_ERR_INVALID,
               "sesa_stft_f32: need len %% hop == 0 and len > n_fft/2 (len=%d hop=%d)", len, hop);
  SESA_REQUIRE(dim_f > 0 && dim_f <= n_fft / 2 + 1, SESA_ERR_INVALID, "sesa_stft_f32: bad dim_f %d", dim_f);
  SESA_REQUIRE(dim_f <= kFFT, SESA_ERR_INVALID, "sesa_stft_f32: dim_f must be <= n_fft/2 (Nyquist not produced)");
  return stft_launch(x, n_sig, len, hop, dim_f, 0, 1, out, as_stream(stream));
}

extern "C" size_t sesa_istft_workspace_size(int n_sig, int frames, int n_fft) {
  return (size_t)n_sig * frames * n_fft * sizeof(float);
}

extern "C" int sesa_istft_f32(const float* spec, int n_sig, int dim_f, int frames, int n_fft, int hop, float* out,
                              void* frame_ws, void* stream) {
  clear_error();
  SESA_REQUIRE(spec && out && frame_ws && n_sig > 0, SESA_ERR_INVALID, "sesa_istft_f32: null pointer");
  SESA_REQUIRE(n_fft == kNFFT, SESA_ERR_INVALID, "sesa_istft_f32: only n_fft=8192 is supported (got %d)", n_fft);
  SESA_REQUIRE(frames >= 2 && hop > 0 && dim_f > 0 && dim_f <= kFFT, SESA_ERR_INVALID,
               "sesa_istft_f32: bad frames/hop/dim_f");
  return istft_launch(spec, n_sig, dim_f, frames, hop, 0, 1, 1, out, (float*)frame_ws, as_stream(stream));
}
