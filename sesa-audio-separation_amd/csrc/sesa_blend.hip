// Ensemble blend of separated stems (ensemble.py:172-407, AudioEnsembleEngine) on gfx950.
//
// Reference semantics, computed in float64 like the reference (soundfile reads float64; numpy /
// scipy compute in float64):
//  * waveform methods (process_waveform, :172-183): weighted mean (np.average with the float32-
//    normalised weights, :288-293: sum(w_i x_i) / sum(w_i)), median (mean of the two middle values
//    for an even count), max, min over files -- elementwise, so the buffer split is irrelevant.
//  * spectral methods (process_spectral, :185-256) per `buffer`-frame piece (:319-372), per channel:
//    scipy.signal.stft(nperseg = min(1024, len), noverlap = nperseg/2, periodic Hann, boundary
//    zeros, padded, scaling 'spectrum'), |Z| combined over files (max / min / median) with the
//    phase of file 0, scipy.signal.istft (OLA / sum w^2 where > 1e-10, boundary trimmed), cut to
//    the piece.  Pieces shorter than 256 samples fall back to avg_wave with the weights (:355-357).
//  One workgroup per (frame, channel, piece): the frame of every file is transformed in LDS
//  (radix-2 Stockham FFT for nperseg = 1024, direct DFT otherwise -- only a short last piece),
//  combined per bin, inverse-transformed and windowed into a frame scratch; a second kernel
//  overlap-adds.  HBM-bound: reads n_files x 4 B per sample (x2 frame overlap through L2),
//  writes 8 B per sample.
//  Up to kMaxFiles (64) files: max / min / mean reduce over the files in a loop; the medians keep one
//  value per file (waveform: a per-thread array; spectral: magnitudes in LDS for <= kLdsFiles files,
//  else in a global scratch after the frame images).  NaN propagates like numpy's max / min / median.
#include <hip/hip_runtime.h>

#include <cmath>
#include <mutex>
#include <vector>

#include "sesa_common.hpp"
#include "sesa_internal.hpp"

namespace sesa {
namespace {

constexpr int kMaxFiles = 64;
constexpr int kLdsFiles = 8;   // spectral median: magnitudes of up to 8 files in LDS
constexpr int kT = 256;
constexpr int kSeg = 1024;

struct Weights {
  double w[kMaxFiles];
  double sum;
  int has;
};

// numpy semantics: any NaN makes max / min / median NaN (fmax / fmin would drop it)
__device__ __forceinline__ double nmax(double a, double b) { return (a != a || b != b) ? a + b : fmax(a, b); }
__device__ __forceinline__ double nmin(double a, double b) { return (a != a || b != b) ? a + b : fmin(a, b); }

// median of v[0 .. n) with stride `st` (insertion sort in place; n <= kMaxFiles)
__device__ double median_of(double* v, int n, int st = 1) {
  for (int i = 0; i < n; ++i)
    if (v[i * st] != v[i * st]) return v[i * st];
  for (int i = 1; i < n; ++i) {
    const double x = v[i * st];
    int j = i - 1;
    while (j >= 0 && v[j * st] > x) {
      v[(j + 1) * st] = v[j * st];
      --j;
    }
    v[(j + 1) * st] = x;
  }
  return (n & 1) ? v[(n / 2) * st] : (v[(n / 2 - 1) * st] + v[(n / 2) * st]) * 0.5;
}

// out[ch][t] for t in [t0, t1): x [file][n_ch][L] fp32
__global__ void blend_wave_kernel(const float* __restrict__ x, int n_files, int n_ch, int64_t L, int64_t t0,
                                  int64_t t1, int method, Weights wt, double* __restrict__ out) {
  const int64_t span = t1 - t0;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= span * n_ch) return;
  const int ch = (int)(i / span);
  const int64_t t = t0 + (i - (int64_t)ch * span);
  auto val = [&](int f) { return (double)x[((int64_t)f * n_ch + ch) * L + t]; };
  double r;
  if (method == SESA_BLEND_AVG_WAVE) {
    double s = 0.0;
    if (wt.has) {
      for (int f = 0; f < n_files; ++f) s += val(f) * wt.w[f];
      r = s / wt.sum;
    } else {
      for (int f = 0; f < n_files; ++f) s += val(f);
      r = s / (double)n_files;
    }
  } else if (method == SESA_BLEND_MEDIAN_WAVE) {
    double v[kMaxFiles];
    for (int f = 0; f < n_files; ++f) v[f] = val(f);
    r = median_of(v, n_files);
  } else if (method == SESA_BLEND_MAX_WAVE) {
    r = val(0);
    for (int f = 1; f < n_files; ++f) r = nmax(r, val(f));
  } else {
    r = val(0);
    for (int f = 1; f < n_files; ++f) r = nmin(r, val(f));
  }
  out[(int64_t)ch * L + t] = r;
}

__device__ __forceinline__ double2 zc(double a, double b) { return make_double2(a, b); }

// In-place-by-pingpong radix-2 Stockham FFT of kSeg points (forward: sign = -1).
__device__ double2* fft1024d(double2* a, double2* b, const double2* __restrict__ tw, bool inverse) {
  int n = kSeg, s = 1;
  for (int stage = 0; stage < 10; ++stage) {
    const int m = n >> 1;
    __syncthreads();
    for (int bf = threadIdx.x; bf < kSeg / 2; bf += kT) {
      const int q = bf & (s - 1), p = bf >> __builtin_ctz(s);
      const double2 u = a[q + s * p], v = a[q + s * (p + m)];
      double2 w = tw[p * s];
      if (inverse) w.y = -w.y;
      const double2 d = zc(u.x - v.x, u.y - v.y);
      b[q + s * 2 * p] = zc(u.x + v.x, u.y + v.y);
      b[q + s * (2 * p + 1)] = zc(w.x * d.x - w.y * d.y, w.x * d.y + w.y * d.x);
    }
    double2* t = a; a = b; b = t;
    n = m;
    s <<= 1;
  }
  __syncthreads();
  return a;
}

struct Piece {
  int64_t pos, len;  // samples of the piece
  int N, nstep, nseg;
  double wsum;
};

// One workgroup per (frame, channel): files' frames -> spectra -> combined -> windowed inverse frame.
// mg_g: global magnitude scratch [n_files][nb] per (frame, channel) workgroup, used by the median
// when n_files > kLdsFiles.
__global__ void __launch_bounds__(kT) blend_fft_frames_kernel(const float* __restrict__ x, int n_files, int n_ch,
                                                              int64_t L, Piece pc, int method,
                                                              const double2* __restrict__ tw,
                                                              double* __restrict__ frames, double* __restrict__ mg_g) {
  __shared__ double2 bufA[kSeg];
  __shared__ double2 bufB[kSeg];
  __shared__ double2 Z0[kSeg / 2 + 1];                  // file 0's spectrum (its phase is kept)
  __shared__ double mg_l[kLdsFiles][kSeg / 2 + 1];      // magnitudes: median over <= kLdsFiles files,
                                                        // running max / min in row 0 otherwise
  __shared__ double win[kSeg];
  const int fr = blockIdx.x, ch = blockIdx.y;
  const int N = pc.N, half = N / 2, nb = N / 2 + 1;
  const bool med = method == SESA_BLEND_MEDIAN_FFT;
  const bool lds_med = med && n_files <= kLdsFiles;
  double* mgw = mg_g + ((int64_t)ch * pc.nseg + fr) * (int64_t)n_files * nb;
  for (int n = threadIdx.x; n < N; n += kT) win[n] = 0.5 - 0.5 * cospi(2.0 * n / N);
  __syncthreads();
  const int64_t start = (int64_t)fr * pc.nstep - half;  // piece coordinates of frame sample 0
  for (int f = 0; f < n_files; ++f) {
    const float* xs = x + ((int64_t)f * n_ch + ch) * L + pc.pos;
    for (int n = threadIdx.x; n < N; n += kT) {
      const int64_t t = start + n;
      const double v = (t >= 0 && t < pc.len) ? (double)xs[t] : 0.0;  // boundary zeros + padding
      bufA[n] = zc(v * win[n], 0.0);
    }
    const double2* y = nullptr;
    if (N == kSeg) {
      y = fft1024d(bufA, bufB, tw, false);
    } else {
      __syncthreads();
      for (int k = threadIdx.x; k < nb; k += kT) {  // direct DFT (short last piece only) into bufB
        double re = 0.0, im = 0.0;
        for (int n = 0; n < N; ++n) {
          const int64_t kn = ((int64_t)k * n) % N;
          double sn, cs;
          sincospi(2.0 * (double)kn / N, &sn, &cs);
          re += bufA[n].x * cs;
          im -= bufA[n].x * sn;
        }
        bufB[k] = zc(re, im);
      }
      y = bufB;
    }
    for (int k = threadIdx.x; k < nb; k += kT) {
      const double2 z = zc(y[k].x / pc.wsum, y[k].y / pc.wsum);
      const double m = hypot(z.x, z.y);
      if (f == 0) Z0[k] = z;
      if (lds_med) mg_l[f][k] = m;
      else if (med) mgw[(int64_t)f * nb + k] = m;
      else if (f == 0) mg_l[0][k] = m;
      else mg_l[0][k] = method == SESA_BLEND_MAX_FFT ? nmax(mg_l[0][k], m) : nmin(mg_l[0][k], m);
    }
    __syncthreads();
  }
  // combine magnitudes, phase of file 0 (np.abs / np.angle / exp(1j * angle))
  for (int k = threadIdx.x; k < nb; k += kT) {
    double c;
    if (lds_med) c = median_of(&mg_l[0][k], n_files, kSeg / 2 + 1);
    else if (med) c = median_of(mgw + k, n_files, nb);
    else c = mg_l[0][k];
    const double ang = atan2(Z0[k].y, Z0[k].x);
    double sn, cs;
    sincos(ang, &sn, &cs);
    Z0[k] = zc(c * cs, c * sn);  // (only this thread reads bin k)
  }
  __syncthreads();
  // irfft(n = N): Hermitian extension, imaginary parts of DC (and Nyquist, even N) ignored
  double* out = frames + ((int64_t)ch * pc.nseg + fr) * N;
  if (N == kSeg) {
    for (int k = threadIdx.x; k < N; k += kT) {
      double2 v;
      if (k == 0) v = zc(Z0[0].x, 0.0);
      else if (k == half) v = zc(Z0[half].x, 0.0);
      else if (k < half) v = Z0[k];
      else v = zc(Z0[N - k].x, -Z0[N - k].y);
      bufA[k] = v;
    }
    double2* y = fft1024d(bufA, bufB, tw, true);
    for (int n = threadIdx.x; n < N; n += kT) out[n] = y[n].x / N * pc.wsum * win[n];
  } else {
    for (int n = threadIdx.x; n < N; n += kT) {
      double acc = Z0[0].x;
      const int kmax = (N & 1) ? half : half - 1;
      for (int k = 1; k <= kmax; ++k) {
        const int64_t kn = ((int64_t)k * n) % N;
        double sn, cs;
        sincospi(2.0 * (double)kn / N, &sn, &cs);
        acc += 2.0 * (Z0[k].x * cs - Z0[k].y * sn);
      }
      if (!(N & 1)) acc += Z0[half].x * ((n & 1) ? -1.0 : 1.0);
      out[n] = acc / N * pc.wsum * win[n];
    }
  }
}

__global__ void blend_fft_ola_kernel(const double* __restrict__ frames, int n_ch, int64_t L, Piece pc,
                                     double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= pc.len * n_ch) return;
  const int ch = (int)(i / pc.len);
  const int64_t t = i - (int64_t)ch * pc.len;
  const int N = pc.N;
  const int64_t p = t + N / 2;  // padded coordinates (boundary trim)
  int64_t i_hi = p / pc.nstep;
  if (i_hi > pc.nseg - 1) i_hi = pc.nseg - 1;
  int64_t i_lo = p - N + 1 <= 0 ? 0 : (p - N + pc.nstep) / pc.nstep;
  double acc = 0.0, norm = 0.0;
  for (int64_t fr = i_lo; fr <= i_hi; ++fr) {
    const int64_t o = p - fr * pc.nstep;
    const double w = 0.5 - 0.5 * cospi(2.0 * (double)o / N);
    acc += frames[((int64_t)ch * pc.nseg + fr) * N + o];
    norm += w * w;
  }
  out[(int64_t)ch * L + pc.pos + t] = acc / (norm > 1e-10 ? norm : 1.0);
}

std::mutex g_tw_mu;
std::vector<double2*> g_tw;  // per device: exp(-2 pi i j / 1024), j < 512

int twiddles(const double2** tw, hipStream_t st) {
  int dev = 0;
  SESA_CHECK_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(g_tw_mu);
  if ((int)g_tw.size() <= dev) g_tw.resize(dev + 1, nullptr);
  if (!g_tw[dev]) {
    std::vector<double2> h(kSeg / 2);
    for (int j = 0; j < kSeg / 2; ++j) {
      const double a = -2.0 * M_PI * j / kSeg;
      h[j] = make_double2(cos(a), sin(a));
    }
    double2* d = nullptr;
    SESA_CHECK_HIP(hipMalloc(&d, h.size() * sizeof(double2)));
    // ordered before the caller's kernels on its stream; the host copy must outlive the transfer
    SESA_CHECK_HIP(hipMemcpyAsync(d, h.data(), h.size() * sizeof(double2), hipMemcpyHostToDevice, st));
    SESA_CHECK_HIP(hipStreamSynchronize(st));
    g_tw[dev] = d;
  }
  *tw = g_tw[dev];
  return SESA_OK;
}

Piece make_piece(int64_t pos, int64_t len) {
  Piece p{};
  p.pos = pos;
  p.len = len;
  p.N = (int)(len < kSeg ? len : kSeg);
  p.nstep = p.N - p.N / 2;
  const int64_t Lp = len + 2 * (p.N / 2);
  const int64_t nadd = ((-(Lp - p.N)) % p.nstep + p.nstep) % p.nstep % p.N;
  p.nseg = (int)((Lp + nadd - p.N) / p.nstep + 1);
  double s = 0.0;
  for (int n = 0; n < p.N; ++n) s += 0.5 - 0.5 * cos(2.0 * M_PI * n / p.N);
  p.wsum = s;
  return p;
}

Weights make_weights(const float* w, int n) {
  Weights wt{};
  if (!w) return wt;
  // np.float32 array .sum(): numpy's pairwise summation (sequential below 8 items, else 8 partial
  // sums combined as ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)), then the remainder)
  float sum = 0.f;
  if (n < 8) {
    for (int i = 0; i < n; ++i) sum += w[i];
  } else {
    float r[8];
    for (int j = 0; j < 8; ++j) r[j] = w[j];
    int i = 8;
    for (; i + 8 <= n; i += 8)
      for (int j = 0; j < 8; ++j) r[j] += w[i + j];
    sum = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) sum += w[i];
  }
  double dsum = 0.0;
  for (int i = 0; i < n; ++i) {
    const float wn = w[i] / sum;  // float32 normalisation (ensemble.py:289-290)
    wt.w[i] = (double)wn;
    dsum += (double)wn;
  }
  wt.sum = dsum;
  wt.has = 1;
  return wt;
}

// frame images (+ the spectral-median magnitude scratch when n_files > kLdsFiles)
size_t blend_workspace(int n_files, int n_ch, int64_t buffer) {
  const Piece p = make_piece(0, buffer);
  size_t b = (size_t)n_ch * p.nseg * p.N * sizeof(double) + 1024;
  if (n_files > kLdsFiles) b += (size_t)n_ch * p.nseg * n_files * (p.N / 2 + 1) * sizeof(double);
  return b;
}

}  // namespace
}  // namespace sesa

using namespace sesa;

extern "C" size_t sesa_blend_workspace_size(int n_ch, int64_t buffer) {
  return sesa::blend_workspace(sesa::kLdsFiles, n_ch, buffer);
}

extern "C" size_t sesa_blend_workspace_size_n(int n_files, int n_ch, int64_t buffer) {
  return sesa::blend_workspace(n_files, n_ch, buffer);
}

extern "C" int sesa_blend_f32(const float* x, int n_files, int n_ch, int64_t L, int64_t buffer, int method,
                              const float* weights, double* out, void* workspace, size_t workspace_bytes,
                              void* stream) {
  clear_error();
  SESA_REQUIRE(x && out && n_files >= 1 && n_files <= kMaxFiles && n_ch >= 1 && L >= 0 && buffer > 0,
               SESA_ERR_INVALID, "sesa_blend_f32: bad arguments (1 <= n_files <= %d)", kMaxFiles);
  SESA_REQUIRE(method >= SESA_BLEND_AVG_WAVE && method <= SESA_BLEND_MEDIAN_FFT, SESA_ERR_INVALID,
               "sesa_blend_f32: unknown method %d", method);
  hipStream_t st = as_stream(stream);
  const Weights wt = make_weights(weights, n_files);
  const bool fft = method >= SESA_BLEND_MAX_FFT;
  if (!fft) {
    if (L == 0) return SESA_OK;
    const int64_t n = L * n_ch;
    hipLaunchKernelGGL(blend_wave_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, x, n_files, n_ch, L,
                       (int64_t)0, L, method, wt, out);
    SESA_CHECK_LAUNCH();
    return SESA_OK;
  }
  SESA_REQUIRE(workspace && workspace_bytes >= blend_workspace(method == SESA_BLEND_MEDIAN_FFT ? n_files : 1, n_ch,
                                                               buffer),
               SESA_ERR_INVALID, "sesa_blend_f32: workspace too small (sesa_blend_workspace_size_n)");
  const double2* tw = nullptr;
  int rc = twiddles(&tw, st);
  if (rc) return rc;
  for (int64_t pos = 0; pos < L; pos += buffer) {
    const int64_t len = buffer < L - pos ? buffer : L - pos;
    if (len < 256) {  // process_spectral -> None -> avg_wave with the weights (:198-200, :355-357)
      hipLaunchKernelGGL(blend_wave_kernel, dim3((unsigned)((len * n_ch + 255) / 256)), dim3(256), 0, st, x, n_files,
                         n_ch, L, pos, pos + len, (int)SESA_BLEND_AVG_WAVE, wt, out);
      SESA_CHECK_LAUNCH();
      continue;
    }
    const Piece pc = make_piece(pos, len);
    double* frames = reinterpret_cast<double*>(workspace);
    double* mg = frames + (size_t)n_ch * pc.nseg * pc.N;
    hipLaunchKernelGGL(blend_fft_frames_kernel, dim3(pc.nseg, n_ch), dim3(kT), 0, st, x, n_files, n_ch, L, pc, method,
                       tw, frames, mg);
    SESA_CHECK_LAUNCH();
    hipLaunchKernelGGL(blend_fft_ola_kernel, dim3((unsigned)((len * n_ch + 255) / 256)), dim3(256), 0, st, frames,
                       n_ch, L, pc, out);
    SESA_CHECK_LAUNCH();
  }
  return SESA_OK;
}
