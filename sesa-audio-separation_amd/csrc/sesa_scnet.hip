// SCNet (sparse compression network): parameter registry, weight packing, spectral front / back
// end and the forward pass (gfx950).
//
// Reference: models/scnet/scnet.py:239-373 (SCNet; SDlayer :86-148, SUlayer :151-196, SDblock
// :199-236, ConvolutionModule :15-52, FusionLayer :55-83) and models/scnet/separation.py
// (DualPathRNN :37-86, FeatureConversion :6-34, SeparationNet :89-113).  Parameter names /
// shapes are the reference state_dict keys, so released checkpoints load by name.
//
// Data layout: every activation is channels-last fp32 [B][F][T][C] (F = frequency rows, T = STFT
// frames).  With F outermost, the SD layer's band outputs and the SU layer's trimmed band outputs
// are contiguous F ranges of one buffer (torch.cat over F is free), a ConvolutionModule row
// (b, f) is one contiguous [T][C] block, and the dual-path LSTMs read both of their sequence
// families -- (b, t) -> f and (b, f) -> t -- as strided token rows of the same buffer.
//
// Kernels (all fp32 FMA unless noted):
//   scn_stft_kernel         4096-point normalized rectangular-window STFT (2048-point complex
//                           radix-4/2 Stockham FFT in LDS + real split), virtual right zero pad
//   scn_sdconv_kernel       SD layer band conv (kernel k x 1, stride s x 1) into the band's F range
//   scn_cm_in_kernel        ConvolutionModule head, one workgroup per (b, f) row: GroupNorm(1, C)
//                           stats, normalise-on-load, conv1d k3 (weights in LDS), GLU
//   scn_cm_in_rb_kernel     the same, register-blocked (4 positions x 2 hidden units per thread): the default
//   scn_cm_out_kernel       ConvolutionModule tail per row: depthwise k3, GroupNorm(1, h), Swish,
//                           1x1 conv, residual (+ the SD block's GELU after the last layer)
//   tok_gemm (conv mode)    3x3 conv over (F, T) as an implicit GEMM, K = 9 taps x C (MFMA, bf16x3):
//                           globalconv, and FusionLayer with the skip added on load, the repeated
//                           input folded into the weights, GLU over interleaved column pairs
//   scn_conv3x3_kernel      the same convs in exact fp32 on the VALU (SESA_SCN_CONV3_VALU=1, A/B)
//   scn_convtr_kernel       SU layer transposed band conv with the symmetric trim
//   scn_gn_*                DualPathRNN GroupNorm(1, d) (fp64 statistics)
//   tok_gemm (MFMA)         LSTM input projections (both directions, b_ih + b_hh) and the
//                           Linear(2H -> d) + residual -- sesa_tokgemm.hip, bf16x3 in parity mode
//   scn_lstm_mfma_kernel    bi-LSTM recurrence on MFMA (bf16x3): one workgroup per (32 sequences,
//                           direction), a wave per 32 hidden units x 4 gates (lane-local cell
//                           update), h as the LDS A operand, W_hh fragments register-resident
//                           (H <= 128) or streamed (H = 256), c in registers
//   scn_lstm_kernel         fp32-FMA recurrence (A/B comparison path)
//   scn_rfft / scn_irfft    FeatureConversion as direct DFTs over T (norm="ortho")
//   scn_istft_*             normalized inverse (c2r by_root_n), OLA / envelope, trim and crop
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <map>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "sesa_common.hpp"
#include "sesa_internal.hpp"
#include "sesa_fft2048.hpp"
#include "sesa_tokgemm.hpp"

namespace sesa {
namespace {

constexpr int kSN = kFft4096;  // n_fft
constexpr int kSH = kFft2048;  // complex FFT length
constexpr int kST = kFftThreads;   // threads per workgroup
using ScnTables = Fft2048Tables;
inline int get_tables(ScnTables* out) { return get_fft2048_tables(out); }
__device__ __forceinline__ float sigm(float v) { return 1.0f / (1.0f + expf(-v)); }

// x [B][ach][chunk] (right zero-padded to Lpad virtually, scnet.py:330-333) -> spec [B][F0][T][2*ach],
// channel 2*s + (re, im) (scnet.py:343-348).  torch.stft: center, reflect, window = ones.
__global__ void __launch_bounds__(kST) scn_stft_kernel(const float* __restrict__ x, int ach, int chunk, int Lpad,
                                                       int hop, int T, float scale, ScnTables tb,
                                                       float* __restrict__ spec) {
  __shared__ float2 bufA[kSH];
  __shared__ float2 bufB[kSH];
  const int t = blockIdx.x;
  const int sig = blockIdx.y;
  const int b = sig / ach, s = sig - b * ach;
  const float* xs = x + (int64_t)sig * chunk;
  const int64_t base = (int64_t)t * hop - kSN / 2;
  for (int m = threadIdx.x; m < kSH; m += kST) {
    float v[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      int64_t pos = base + 2 * m + e;
      if (pos < 0) pos = -pos;
      if (pos >= Lpad) pos = 2 * (int64_t)(Lpad - 1) - pos;
      v[e] = pos < chunk ? xs[pos] : 0.f;
    }
    bufA[m] = make_float2(v[0], v[1]);
  }
  const float2* Z = fft2048<false>(bufA, bufB, tb.tw);
  const int C0 = 2 * ach;
  for (int k = threadIdx.x; k <= kSH; k += kST) {
    const float2 X = rfft_bin(Z, tb.twN, k);
    *reinterpret_cast<float2*>(spec + (((int64_t)b * (kSH + 1) + k) * T + t) * C0 + 2 * s) =
        make_float2(X.x * scale, X.y * scale);
  }
}

// spec -> frames [B*nsig][T][4096] (c2r with scale, window = ones; scnet.py:364-368).  spec is frame-major
// [B][T][F0][2 nsig] (fmajor: the MFMA band convs' output) or band-major [B][F0][T][2 nsig] (the VALU fallback).
// One workgroup per (item, frame, signal), signals fastest and the workgroups of one frame on one XCD (blockIdx
// remapped like tok_gemm's xcd_tile): a frame's signals share its 64-B bin lines in that XCD's L2.
__global__ void __launch_bounds__(kST) scn_istft_frames_kernel(const float* __restrict__ spec, int nsig, int T,
                                                               int fmajor, float scale, ScnTables tb,
                                                               float* __restrict__ fw) {
  __shared__ float2 bufA[kSH];
  __shared__ float2 bufB[kSH + 1];
  const int nb = gridDim.x, q8 = nb >> 3, r8 = nb & 7, x8 = blockIdx.x & 7;
  const int id = x8 * q8 + min(x8, r8) + (blockIdx.x >> 3);
  const int m = id % nsig, bt = id / nsig;
  const int b = bt / T, t = bt - b * T;
  const int sg = b * nsig + m;
  const int C = 2 * nsig;
  const int64_t ks = fmajor ? C : (int64_t)T * C;
  const float* sp = spec + (int64_t)b * (kSH + 1) * T * C + (fmajor ? (int64_t)t * (kSH + 1) * C : (int64_t)t * C) + 2 * m;
  for (int k = threadIdx.x; k <= kSH; k += kST) {
    float2 X = *reinterpret_cast<const float2*>(sp + k * ks);
    if (k == 0 || k == kSH) X.y = 0.f;  // C2R ignores the imaginary parts of DC and Nyquist
    bufB[k] = X;
  }
  __syncthreads();
  for (int k = threadIdx.x; k < kSH; k += kST) bufA[k] = irfft_pack(bufB, tb.twN, k);
  const float2* z = fft2048<true>(bufA, bufB, tb.tw);
  float2* o = reinterpret_cast<float2*>(fw + ((int64_t)sg * T + t) * kSN);
  for (int k = threadIdx.x; k < kSH; k += kST) {
    const float2 v = z[k];
    o[k] = make_float2(v.x * scale, v.y * scale);
  }
}

// overlap-add / sum(w^2) (rectangular window: the covering frame count), center trim, crop to chunk
__global__ void scn_istft_ola_kernel(const float* __restrict__ fw, int T, int hop, int chunk, float* __restrict__ out) {
  const int sg = blockIdx.y;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= chunk) return;
  const int n = j + kSN / 2;
  const int t_lo = n - kSN + 1 <= 0 ? 0 : (n - kSN + hop) / hop;
  const int t_hi = min(n / hop, T - 1);
  const float* f = fw + (int64_t)sg * T * kSN;
  float acc = 0.f, env = 0.f;
  for (int t = t_lo; t <= t_hi; ++t) {
    acc += f[(int64_t)t * kSN + (n - t * hop)];
    env += 1.f;
  }
  out[(int64_t)sg * chunk + j] = acc / env;
}

// ---- SD / SU band convolutions (scnet.py:114-148, :171-196) ---------------------------------
struct BandConv {
  int in_off, n_in, pad_left, stride, kern, n_out, out_off, dist;
};

// Y[b][out_off + fo][t][co] = bias + sum_{kk, ci} W[kk][ci][co] X[b][in_off + fo*s + kk - pad][t][ci]
// One thread = 4 consecutive output channels of one (b, fo, t): float4 weight loads, each input
// value feeds 4 FMAs (Cout % 4 == 0, checked at create).  `total` counts (position, channel quad).
__global__ void scn_sdconv_kernel(const float* __restrict__ X, int Fin, int T, int Cin, const float* __restrict__ W,
                                  const float* __restrict__ bias, BandConv bc, float* __restrict__ Y, int Fout,
                                  int Cout, int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int C4 = Cout >> 2;
  const int co = (int)(i % C4) * 4;
  int64_t r = i / C4;
  const int t = (int)(r % T);
  r /= T;
  const int fo = (int)(r % bc.n_out);
  const int64_t b = r / bc.n_out;
  float4 acc = *reinterpret_cast<const float4*>(bias + co);
  for (int kk = 0; kk < bc.kern; ++kk) {
    const int fi = fo * bc.stride + kk - bc.pad_left;
    if (fi < 0 || fi >= bc.n_in) continue;
    const float* xp = X + ((b * Fin + bc.in_off + fi) * T + t) * Cin;
    const float* wp = W + (int64_t)kk * Cin * Cout + co;
    for (int ci = 0; ci < Cin; ++ci) {
      const float xv = xp[ci];
      const float4 w = *reinterpret_cast<const float4*>(wp + (int64_t)ci * Cout);
      acc.x = fmaf(w.x, xv, acc.x);
      acc.y = fmaf(w.y, xv, acc.y);
      acc.z = fmaf(w.z, xv, acc.z);
      acc.w = fmaf(w.w, xv, acc.w);
    }
  }
  *reinterpret_cast<float4*>(Y + ((b * Fout + bc.out_off + fo) * T + t) * Cout + co) = acc;
}

// ConvTranspose2d (kern x 1, stride x 1) of the band rows, trimmed: out row fo <- full row fo + dist
// (same thread shape as scn_sdconv_kernel)
__global__ void scn_convtr_kernel(const float* __restrict__ X, int Fin, int T, int Cin, const float* __restrict__ W,
                                  const float* __restrict__ bias, BandConv bc, float* __restrict__ Y, int Fout,
                                  int Cout, int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int C4 = Cout >> 2;
  const int co = (int)(i % C4) * 4;
  int64_t r = i / C4;
  const int t = (int)(r % T);
  r /= T;
  const int fo = (int)(r % bc.n_out);
  const int64_t b = r / bc.n_out;
  const int fp = fo + bc.dist;
  float4 acc = *reinterpret_cast<const float4*>(bias + co);
  for (int kk = 0; kk < bc.kern; ++kk) {
    const int d = fp - kk;
    if (d < 0 || d % bc.stride) continue;
    const int fi = d / bc.stride;
    if (fi >= bc.n_in) continue;
    const float* xp = X + ((b * Fin + bc.in_off + fi) * T + t) * Cin;
    const float* wp = W + (int64_t)kk * Cin * Cout + co;
    for (int ci = 0; ci < Cin; ++ci) {
      const float xv = xp[ci];
      const float4 w = *reinterpret_cast<const float4*>(wp + (int64_t)ci * Cout);
      acc.x = fmaf(w.x, xv, acc.x);
      acc.y = fmaf(w.y, xv, acc.y);
      acc.z = fmaf(w.z, xv, acc.z);
      acc.w = fmaf(w.w, xv, acc.w);
    }
  }
  *reinterpret_cast<float4*>(Y + ((b * Fout + bc.out_off + fo) * T + t) * Cout + co) = acc;
}

// ---- ConvolutionModule (scnet.py:15-52), one workgroup per (b, f) row of [T][C] --------------
struct CmArgs {
  float* X;          // [B][F_all][T][C], rows f_off .. f_off + n_f of each item
  int F_all, f_off, n_f, T, C, h;
  const float *g1, *be1;   // GroupNorm(1, C) affine
  const float* W1;         // [C][3][2h]
  const float* b1;         // [2h]
  float* U;                // [B * n_f][T][h]
  const float *wdw, *bdw;  // [h][3], [h]
  const float *g2, *be2;   // GroupNorm(1, h) affine
  const float* W3;         // [h][C]
  const float* b3;         // [C]
  int gelu;                // SDblock F.gelu after the module's last layer (:229-234)
  const uint16_t* W1h;     // scn_cm_mfma_kernel: W1 as fp16 16x16x32 B fragments [3C / 32][h / 8][64][8]
  const uint16_t* W3h;     //   and W3 as [hp / 32][C / 16][64][8] (hp = h rounded up to 32, zero rows past h)
};

__device__ __forceinline__ void block_sum2(double& s, double& ss, double* red) {
  for (int o = 32; o >= 1; o >>= 1) {
    s += __shfl_xor(s, o);
    ss += __shfl_xor(ss, o);
  }
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) {
    red[2 * w] = s;
    red[2 * w + 1] = ss;
  }
  __syncthreads();
  s = 0;
  ss = 0;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) {
    s += red[2 * i];
    ss += red[2 * i + 1];
  }
}

__global__ void __launch_bounds__(kST) scn_cm_in_kernel(CmArgs a) {
  extern __shared__ __align__(16) float sm[];
  const int C = a.C, h = a.h, T = a.T;
  const int TT = 512 / h;
  float* Ws = sm;                                    // [C][3][2h]
  float* xs = Ws + 6 * h * C;                        // [TT + 2][C]
  double* red = reinterpret_cast<double*>(xs + (TT + 2) * C);
  const int row = blockIdx.x;
  const int64_t b = row / a.n_f;
  const int f = a.f_off + row % a.n_f;
  const float* xr = a.X + ((b * a.F_all + f) * T) * C;
  double s = 0, ss = 0;
  for (int i = threadIdx.x; i < T * C; i += kST) {
    const double v = xr[i];
    s += v;
    ss += v * v;
  }
  block_sum2(s, ss, red);
  const double n = (double)T * C;
  const double mu = s / n;
  const double var = fmax(ss / n - mu * mu, 0.0);
  const float mean = (float)mu, rstd = (float)(1.0 / sqrt(var + 1e-5));
  for (int i = threadIdx.x; i < 6 * h * C; i += kST) Ws[i] = a.W1[i];
  float* U = a.U + (int64_t)row * T * h;
  for (int t0 = 0; t0 < T; t0 += TT) {
    __syncthreads();
    for (int i = threadIdx.x; i < (TT + 2) * C; i += kST) {
      const int tl = i / C, c = i - tl * C;
      const int t = t0 - 1 + tl;
      xs[i] = (t >= 0 && t < T) ? (xr[(int64_t)t * C + c] - mean) * rstd * a.g1[c] + a.be1[c] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int q = threadIdx.x + r * kST;
      const int j = q % h, tl = q / h;
      const int t = t0 + tl;
      if (t >= T) continue;
      float ga = a.b1[j], gg = a.b1[j + h];
#pragma unroll
      for (int dt = 0; dt < 3; ++dt) {
        const float* xrow = xs + (tl + dt) * C;
        const float* w = Ws + dt * 2 * h + j;
        for (int c = 0; c < C; ++c) {
          const float xv = xrow[c];
          ga = fmaf(w[c * 6 * h], xv, ga);
          gg = fmaf(w[c * 6 * h + h], xv, gg);
        }
      }
      U[(int64_t)t * h + j] = ga * sigm(gg);
    }
  }
}

// scn_cm_in_rb_kernel: the same ConvolutionModule head (GroupNorm(1, C) stats, normalise-on-load, conv1d
// k3 C -> 2h, GLU), register-blocked: each thread owns CM_TB consecutive positions x CM_JB hidden units (both
// GLU halves: 2 CM_TB CM_JB accumulators), so per input channel c it reads CM_TB + 2 normalised inputs and 6
// CM_JB weights from LDS for 6 CM_TB CM_JB FMAs (2.7 FMAs per LDS read at 4 x 2, against 0.67 in
// scn_cm_in_kernel's one-output-per-thread loop, which is LDS-issue-bound).  Same fp32 arithmetic per
// output (the k3 taps and channels accumulate in the same order), so the outputs are identical to
// scn_cm_in_kernel's.  Tile: 256 threads x CM_TB x CM_JB / h positions.
constexpr int CM_TB = 4, CM_JB = 2;
__host__ __device__ constexpr int cm_rb_tt(int h) { return kST * CM_TB * CM_JB / h; }

__global__ void __launch_bounds__(kST) scn_cm_in_rb_kernel(CmArgs a) {
  extern __shared__ __align__(16) float sm[];
  const int C = a.C, h = a.h, T = a.T;
  const int TT = cm_rb_tt(h);
  float* Ws = sm;                                    // [C][3][2h]
  float* xs = Ws + 6 * h * C;                        // [TT + 2][C]
  double* red = reinterpret_cast<double*>(xs + (TT + 2) * C);
  const int row = blockIdx.x;
  const int64_t b = row / a.n_f;
  const int f = a.f_off + row % a.n_f;
  const float* xr = a.X + ((b * a.F_all + f) * T) * C;
  double s = 0, ss = 0;
  for (int i = threadIdx.x; i < T * C; i += kST) {
    const double v = xr[i];
    s += v;
    ss += v * v;
  }
  block_sum2(s, ss, red);
  const double n = (double)T * C;
  const double mu = s / n;
  const double var = fmax(ss / n - mu * mu, 0.0);
  const float mean = (float)mu, rstd = (float)(1.0 / sqrt(var + 1e-5));
  for (int i = threadIdx.x; i < 6 * h * C; i += kST) Ws[i] = a.W1[i];
  float* U = a.U + (int64_t)row * T * h;
  const int nj = h / CM_JB;
  const int jb = threadIdx.x % nj, tb = threadIdx.x / nj;   // lanes of one position block share its x reads
  const int j0 = jb * CM_JB;
  for (int t0 = 0; t0 < T; t0 += TT) {
    __syncthreads();
    for (int i = threadIdx.x; i < (TT + 2) * C; i += kST) {
      const int tl = i / C, c = i - tl * C;
      const int t = t0 - 1 + tl;
      xs[i] = (t >= 0 && t < T) ? (xr[(int64_t)t * C + c] - mean) * rstd * a.g1[c] + a.be1[c] : 0.f;
    }
    __syncthreads();
    float ga[CM_TB][CM_JB], gg[CM_TB][CM_JB];
#pragma unroll
    for (int r = 0; r < CM_TB; ++r)
#pragma unroll
      for (int q = 0; q < CM_JB; ++q) {
        ga[r][q] = a.b1[j0 + q];
        gg[r][q] = a.b1[j0 + q + h];
      }
    const int tl0 = tb * CM_TB;
    // tap-major over the same (dt, c) order as scn_cm_in_kernel
#pragma unroll
    for (int dt = 0; dt < 3; ++dt) {
      for (int c = 0; c < C; ++c) {
        float xv[CM_TB];
#pragma unroll
        for (int r = 0; r < CM_TB; ++r) xv[r] = xs[(tl0 + r + dt) * C + c];
        const float* w = Ws + c * 6 * h + dt * 2 * h + j0;
        float wa[CM_JB], wg[CM_JB];
#pragma unroll
        for (int q = 0; q < CM_JB; ++q) {
          wa[q] = w[q];
          wg[q] = w[q + h];
        }
#pragma unroll
        for (int r = 0; r < CM_TB; ++r)
#pragma unroll
          for (int q = 0; q < CM_JB; ++q) {
            ga[r][q] = fmaf(wa[q], xv[r], ga[r][q]);
            gg[r][q] = fmaf(wg[q], xv[r], gg[r][q]);
          }
      }
    }
#pragma unroll
    for (int r = 0; r < CM_TB; ++r) {
      const int t = t0 + tl0 + r;
      if (t >= T) continue;
#pragma unroll
      for (int q = 0; q < CM_JB; ++q) U[(int64_t)t * h + j0 + q] = ga[r][q] * sigm(gg[r][q]);
    }
  }
}

__global__ void __launch_bounds__(kST) scn_cm_out_kernel(CmArgs a) {
  extern __shared__ __align__(16) float sm[];
  const int C = a.C, h = a.h, T = a.T;
  float* Us = sm;              // [T][h]
  float* Vs = Us + T * h;      // [T][h]
  float* W3s = Vs + T * h;     // [h][C]
  double* red = reinterpret_cast<double*>(W3s + h * C + ((h * C) & 1));
  const int row = blockIdx.x;
  const int64_t b = row / a.n_f;
  const int f = a.f_off + row % a.n_f;
  float* xr = a.X + ((b * a.F_all + f) * T) * C;
  const float* U = a.U + (int64_t)row * T * h;
  for (int i = threadIdx.x; i < T * h; i += kST) Us[i] = U[i];
  for (int i = threadIdx.x; i < h * C; i += kST) W3s[i] = a.W3[i];
  __syncthreads();
  double s = 0, ss = 0;
  for (int i = threadIdx.x; i < T * h; i += kST) {
    const int t = i / h, j = i - t * h;
    float v = a.bdw[j];
    if (t > 0) v = fmaf(a.wdw[3 * j], Us[i - h], v);
    v = fmaf(a.wdw[3 * j + 1], Us[i], v);
    if (t < T - 1) v = fmaf(a.wdw[3 * j + 2], Us[i + h], v);
    Vs[i] = v;
    s += v;
    ss += (double)v * v;
  }
  block_sum2(s, ss, red);
  const double n = (double)T * h;
  const double mu = s / n;
  const double var = fmax(ss / n - mu * mu, 0.0);
  const float mean = (float)mu, rstd = (float)(1.0 / sqrt(var + 1e-5));
  for (int i = threadIdx.x; i < T * h; i += kST) {
    const int j = i % h;
    const float v = (Vs[i] - mean) * rstd * a.g2[j] + a.be2[j];
    Vs[i] = v * sigm(v);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < T * C; i += kST) {
    const int t = i / C, c = i - t * C;
    float acc = a.b3[c];
    const float* sv = Vs + t * h;
    for (int j = 0; j < h; ++j) acc = fmaf(W3s[j * C + c], sv[j], acc);
    float v = xr[i] + acc;
    if (a.gelu) v = gelu_erf(v);
    xr[i] = v;
  }
}

// ---- ConvolutionModule layer on MFMA (fp16mix), one workgroup per (b, f) row: both convolutions of
// scnet.py:35-43 as fp16 GEMMs (v_mfma_f32_16x16x32_f16, fp32 accumulation), the norms / GLU / depthwise / Swish /
// residual in fp32 around them, in ONE launch per layer (scn_cm_in_rb_kernel + scn_cm_out_kernel are two, and spend
// their time on LDS-bound VALU FMAs: 9-14 TF/s).
//   A: GroupNorm(1, C) statistics of the row (fp64 sums, as scn_cm_in_kernel); W1's fragments into LDS.
//   B: per slab of kCmTT positions, the normalised rows t0 - 1 .. t0 + kCmTT as fp16 in LDS (row stride C + 8).  The
//      k3 conv is a GEMM whose A row t is the three input rows t - 1, t, t + 1 (k = dt C + c); each wave takes 16
//      positions and every column tile.  Packed column tile i holds the GLU value columns 8i .. 8i + 7 (lanes 0-7)
//      and their gates (lanes 8-15), so the GLU is a lane swap in the epilogue; U [T + 2][h] fp32 stays in LDS
//      (zero end rows: the depthwise conv's padding).
//   C: depthwise k3 + GroupNorm(1, h) statistics (fp64), then Swish of the normalised values as fp16 V [T16][h]
//      into the dead phase-B region (zero rows past T; phase D zeroes the k past h).
//   D: the 1x1 conv h -> C as a GEMM over V (K = hp), + b3 + the residual x (+ the SDblock gelu), stored in place
//      (each element is read and written by the same lane).
constexpr int kCmTT = 64;
__host__ __device__ constexpr int cm_hp(int h) { return (h + 31) / 32 * 32; }
struct CmMfmaLds {
  int xs, w1, vh, w3, u, red, total;   // byte offsets of the regions, total bytes
};
__host__ __device__ inline CmMfmaLds cm_mfma_layout(int T, int C, int h) {
  CmMfmaLds l{};
  const int T16 = (T + 15) / 16 * 16, hp = cm_hp(h);
  const int xs_b = (kCmTT + 2) * (C + 8) * 2, w1_b = 3 * C * 2 * h * 2;
  const int vh_b = T16 * (h + 8) * 2, w3_b = hp * C * 2;
  const int r1 = max(xs_b + w1_b, vh_b + w3_b);
  l.xs = 0;
  l.w1 = xs_b;
  l.vh = 0;
  l.w3 = vh_b;
  l.u = (r1 + 15) / 16 * 16;
  l.red = l.u + ((T + 2) * h * 4 + 15) / 16 * 16;
  l.total = l.red + 16 * 8;
  return l;
}
typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 h16x4 __attribute__((ext_vector_type(4)));

template <int NT1>   // h / 8: column tiles of the k3 conv (GLU pairs)
__global__ void __launch_bounds__(kST) scn_cm_mfma_kernel(CmArgs a) {
  extern __shared__ __align__(16) char smc[];
  const int C = a.C, h = a.h, T = a.T;
  const int hp = cm_hp(h), T16 = (T + 15) / 16 * 16;
  const CmMfmaLds L = cm_mfma_layout(T, C, h);
  _Float16* xs = reinterpret_cast<_Float16*>(smc + L.xs);
  const u32x4* w1s = reinterpret_cast<const u32x4*>(smc + L.w1);
  _Float16* vh = reinterpret_cast<_Float16*>(smc + L.vh);
  const u32x4* w3s = reinterpret_cast<const u32x4*>(smc + L.w3);
  float* U = reinterpret_cast<float*>(smc + L.u);
  double* red = reinterpret_cast<double*>(smc + L.red);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int row = blockIdx.x;
  const int64_t b = row / a.n_f;
  const int f = a.f_off + row % a.n_f;
  float* xr = a.X + ((b * a.F_all + f) * T) * C;
  const f32x4* xr4 = reinterpret_cast<const f32x4*>(xr);
  const int SX = C + 8, SV = h + 8, C4 = C / 4;   // (h % 8 == 0: 16-B aligned V rows)
  const int K1 = 3 * C;

  // ---- A: GroupNorm(1, C) statistics; W1 fragments -> LDS; U's zero end rows ----
  {
    u32x4* d = reinterpret_cast<u32x4*>(smc + L.w1);
    const u32x4* s = reinterpret_cast<const u32x4*>(a.W1h);
    for (int i = tid; i < K1 * 2 * h / 8; i += kST) d[i] = s[i];
    for (int i = tid; i < h; i += kST) {
      U[i] = 0.f;
      U[(T + 1) * h + i] = 0.f;
    }
  }
  double s = 0, ss = 0;
#pragma unroll 4
  for (int i = tid; i < T * C4; i += kST) {
    const f32x4 v = xr4[i];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      s += v[q];
      ss += (double)v[q] * v[q];
    }
  }
  block_sum2(s, ss, red);
  float mean, rstd;
  {
    const double n = (double)T * C;
    const double mu = s / n;
    const double var = fmax(ss / n - mu * mu, 0.0);
    mean = (float)mu;
    rstd = (float)(1.0 / sqrt(var + 1e-5));
  }
  // this thread's channel quad when staging (kST % C4 == 0: host check)
  const int cq = tid % C4, c0 = cq * 4;
  float gs[4], gb[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    gs[q] = rstd * a.g1[c0 + q];
    gb[q] = a.be1[c0 + q];
  }
  // this lane's packed k3-conv columns: bias of the value column and of its gate
  const int col = lane & 15;
  float bias1[NT1];
#pragma unroll
  for (int nt = 0; nt < NT1; ++nt) bias1[nt] = a.b1[col < 8 ? 8 * nt + col : h + 8 * nt + col - 8];

  // ---- B: k3 conv C -> 2h + GLU, slab by slab ----
  for (int t0 = 0; t0 < T; t0 += kCmTT) {
    sesa_sync();   // (the previous slab's fragment reads are done; first slab: W1 and the stats are in place)
    for (int i = tid; i < (kCmTT + 2) * C4; i += kST) {
      const int rl = i / C4;
      const int t = t0 - 1 + rl;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (t >= 0 && t < T) {
        v = xr4[(int64_t)t * C4 + cq];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = (v[q] - mean) * gs[q] + gb[q];
      }
      h16x4 hv;
#pragma unroll
      for (int q = 0; q < 4; ++q) hv[q] = (_Float16)v[q];
      *reinterpret_cast<h16x4*>(xs + rl * SX + c0) = hv;
    }
    sesa_sync();
    const int tl0 = 16 * w;
    if (t0 + tl0 < T) {   // (wave-uniform)
      f32x4 acc[NT1];
#pragma unroll
      for (int nt = 0; nt < NT1; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int arow = tl0 + (lane & 15);
      for (int ks = 0; ks < K1 / 32; ++ks) {
        const int kb = 32 * ks + 8 * (lane >> 4);
        const int dt = kb / C, c = kb - dt * C;   // (C % 32 == 0: a lane's 8 k lie in one tap)
        const h16x8 av = *reinterpret_cast<const h16x8*>(xs + (arow + dt) * SX + c);
#pragma unroll
        for (int nt = 0; nt < NT1; ++nt) {
          const h16x8 bv = __builtin_bit_cast(h16x8, w1s[(ks * NT1 + nt) * 64 + lane]);
          acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av, bv, acc[nt], 0, 0, 0);
        }
      }
#pragma unroll
      for (int nt = 0; nt < NT1; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = acc[nt][r] + bias1[nt];
          const float g = __shfl_xor(v, 8);
          const int t = t0 + tl0 + (lane >> 4) * 4 + r;
          if (col < 8 && t < T) U[(t + 1) * h + 8 * nt + col] = v * sigm(g);
        }
    }
  }
  sesa_sync();   // U complete; the slab buffer and W1 are dead

  // ---- C: depthwise k3 + GroupNorm(1, h) statistics, then Swish(norm) as fp16 V; W3 fragments -> LDS ----
  {
    u32x4* d = reinterpret_cast<u32x4*>(smc + L.w3);
    const u32x4* s3 = reinterpret_cast<const u32x4*>(a.W3h);
    for (int i = tid; i < hp * C / 8; i += kST) d[i] = s3[i];
  }
  const int j = tid % h;              // (kST % h == 0: host check) this thread's hidden unit
  const float wd0 = a.wdw[3 * j], wd1 = a.wdw[3 * j + 1], wd2 = a.wdw[3 * j + 2], bd = a.bdw[j];
  s = 0;
  ss = 0;
  for (int t = tid / h; t < T; t += kST / h) {
    float v = bd;
    v = fmaf(wd0, U[t * h + j], v);
    v = fmaf(wd1, U[(t + 1) * h + j], v);
    v = fmaf(wd2, U[(t + 2) * h + j], v);
    s += v;
    ss += (double)v * v;
  }
  block_sum2(s, ss, red);
  {
    const double n = (double)T * h;
    const double mu = s / n;
    const double var = fmax(ss / n - mu * mu, 0.0);
    mean = (float)mu;
    rstd = (float)(1.0 / sqrt(var + 1e-5));
  }
  const float g2 = rstd * a.g2[j], be2 = a.be2[j];
  for (int t = tid / h; t < T16; t += kST / h) {
    float o = 0.f;
    if (t < T) {
      float v = bd;
      v = fmaf(wd0, U[t * h + j], v);
      v = fmaf(wd1, U[(t + 1) * h + j], v);
      v = fmaf(wd2, U[(t + 2) * h + j], v);
      v = (v - mean) * g2 + be2;
      o = v * sigm(v);
    }
    vh[t * SV + j] = (_Float16)o;
  }
  sesa_sync();

  // ---- D: 1x1 conv h -> C + b3 + residual (+ gelu), in place ----
  const int KS2 = hp / 32, NT2 = C / 16;
  for (int mt = w; mt < T16 / 16; mt += kST / 64) {
    h16x8 av[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      if (ks < KS2) {   // k past h: zero (V holds h columns; W3's rows past h are zero too)
        const int kb = 32 * ks + 8 * (lane >> 4);
        av[ks] = kb < h ? *reinterpret_cast<const h16x8*>(vh + (16 * mt + (lane & 15)) * SV + kb) : h16x8{};
      }
    for (int nt = 0; nt < NT2; ++nt) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        if (ks < KS2)
          acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[ks], __builtin_bit_cast(h16x8, w3s[(ks * NT2 + nt) * 64 + lane]),
                                                       acc, 0, 0, 0);
      const int c = 16 * nt + col;
      const float bias = a.b3[c];
      float res[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int t = 16 * mt + (lane >> 4) * 4 + r;
        res[r] = t < T ? xr[(int64_t)t * C + c] : 0.f;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int t = 16 * mt + (lane >> 4) * 4 + r;
        float v = res[r] + (acc[r] + bias);
        if (a.gelu) v = gelu_erf(v);
        if (t < T) xr[(int64_t)t * C + c] = v;
      }
    }
  }
}

// ---- ConvolutionModule for wide levels (SCNet-large / XL: C = 256, h = 64, or h not dividing 512),
// where a row's conv1d weight [C][3][2h] (393 KB at C = 256) or its [T][h] hidden planes exceed LDS.
// Same arithmetic as scn_cm_in_kernel / scn_cm_out_kernel, restaged:
//   in:  one workgroup per (b, f) row; GroupNorm(1, C) stats once per row, then per tile of kGenTT
//        positions the weight is walked in 16-channel slices ([16][3][2h] in LDS) with the normalised
//        [TT + 2][16] input slice beside it; each thread accumulates up to 8 (t, j) GLU pairs.
//   out: one workgroup per row; pass 1 recomputes the depthwise k3 conv from U (global, L2-resident)
//        for the GroupNorm(1, h) sums, pass 2 per tile of kGenTO positions: depthwise conv, GN, Swish
//        into LDS, then the 1x1 conv h -> C from the LDS-resident W3 [h][C], residual, optional GELU.
constexpr int kGenCC = 16;   // channels per weight slice
constexpr int kGenNQ = 8;    // (t, j) outputs per thread per tile
constexpr int kGenTO = 16;   // positions per output tile
inline int gen_tt(int h) { return kGenNQ * (kST / h); }
size_t cm_in_gen_lds(int h) { return (size_t)(kGenCC * 6 * h + (gen_tt(h) + 2) * kGenCC) * 4 + 16 * 8 + 16; }
size_t cm_out_gen_lds(int C, int h) { return (size_t)(kGenTO * h + h * C) * 4 + 16 * 8 + 16; }

__global__ void __launch_bounds__(kST) scn_cm_in_gen_kernel(CmArgs a) {
  extern __shared__ __align__(16) float sm[];
  const int C = a.C, h = a.h, T = a.T;
  const int G = kST / h;                        // thread groups; thread (g, j) owns unit j
  const int TT = kGenNQ * G;                    // positions per tile: tl = g + G * r, r < kGenNQ
  float* Ws = sm;                               // [16][3][2h]
  float* xs = Ws + kGenCC * 6 * h;              // [TT + 2][16]
  double* red = reinterpret_cast<double*>(xs + (TT + 2) * kGenCC + 2);
  const int row = blockIdx.x;
  const int64_t b = row / a.n_f;
  const int f = a.f_off + row % a.n_f;
  const float* xr = a.X + ((b * a.F_all + f) * T) * C;
  double s = 0, ss = 0;
  for (int i = threadIdx.x; i < T * C; i += kST) {
    const double v = xr[i];
    s += v;
    ss += v * v;
  }
  block_sum2(s, ss, red);
  const double n = (double)T * C;
  const double mu = s / n;
  const double var = fmax(ss / n - mu * mu, 0.0);
  const float mean = (float)mu, rstd = (float)(1.0 / sqrt(var + 1e-5));
  float* U = a.U + (int64_t)row * T * h;
  const int g = threadIdx.x / h, j = threadIdx.x - g * h;
  const bool active = g < G;
  for (int t0 = 0; t0 < T; t0 += TT) {
    float ga[kGenNQ], gg[kGenNQ];
#pragma unroll
    for (int r = 0; r < kGenNQ; ++r) {
      ga[r] = active ? a.b1[j] : 0.f;
      gg[r] = active ? a.b1[j + h] : 0.f;
    }
    for (int c0 = 0; c0 < C; c0 += kGenCC) {
      __syncthreads();
      for (int i = threadIdx.x; i < kGenCC * 6 * h; i += kST) {
        const int cl = i / (6 * h), e = i - cl * 6 * h;
        Ws[i] = c0 + cl < C ? a.W1[(int64_t)(c0 + cl) * 6 * h + e] : 0.f;
      }
      for (int i = threadIdx.x; i < (TT + 2) * kGenCC; i += kST) {
        const int tl = i / kGenCC, cl = i - tl * kGenCC;
        const int t = t0 - 1 + tl, c = c0 + cl;
        xs[i] = (t >= 0 && t < T && c < C) ? (xr[(int64_t)t * C + c] - mean) * rstd * a.g1[c] + a.be1[c] : 0.f;
      }
      __syncthreads();
      if (!active) continue;
#pragma unroll 1
      for (int dt = 0; dt < 3; ++dt) {
#pragma unroll 4
        for (int c = 0; c < kGenCC; ++c) {
          const float wa = Ws[(c * 3 + dt) * 2 * h + j], wg = Ws[(c * 3 + dt) * 2 * h + h + j];
#pragma unroll
          for (int r = 0; r < kGenNQ; ++r) {
            const float xv = xs[(g + G * r + dt) * kGenCC + c];
            ga[r] = fmaf(wa, xv, ga[r]);
            gg[r] = fmaf(wg, xv, gg[r]);
          }
        }
      }
    }
    if (active) {
#pragma unroll
      for (int r = 0; r < kGenNQ; ++r) {
        const int t = t0 + g + G * r;
        if (t < T) U[(int64_t)t * h + j] = ga[r] * sigm(gg[r]);
      }
    }
  }
}

__global__ void __launch_bounds__(kST) scn_cm_out_gen_kernel(CmArgs a) {
  extern __shared__ __align__(16) float sm[];
  const int C = a.C, h = a.h, T = a.T;
  float* W3s = sm;                 // [h][C]
  float* Vs = W3s + h * C;         // [kGenTO][h]
  double* red = reinterpret_cast<double*>(Vs + kGenTO * h + ((h * C + kGenTO * h) & 1));
  const int row = blockIdx.x;
  const int64_t b = row / a.n_f;
  const int f = a.f_off + row % a.n_f;
  float* xr = a.X + ((b * a.F_all + f) * T) * C;
  const float* U = a.U + (int64_t)row * T * h;
  for (int i = threadIdx.x; i < h * C; i += kST) W3s[i] = a.W3[i];
  auto dw = [&](int t, int j) {
    const int i = t * h + j;
    float v = a.bdw[j];
    if (t > 0) v = fmaf(a.wdw[3 * j], U[i - h], v);
    v = fmaf(a.wdw[3 * j + 1], U[i], v);
    if (t < T - 1) v = fmaf(a.wdw[3 * j + 2], U[i + h], v);
    return v;
  };
  double s = 0, ss = 0;
  for (int i = threadIdx.x; i < T * h; i += kST) {
    const int t = i / h, j = i - t * h;
    const float v = dw(t, j);
    s += v;
    ss += (double)v * v;
  }
  block_sum2(s, ss, red);
  const double n = (double)T * h;
  const double mu = s / n;
  const double var = fmax(ss / n - mu * mu, 0.0);
  const float mean = (float)mu, rstd = (float)(1.0 / sqrt(var + 1e-5));
  for (int t0 = 0; t0 < T; t0 += kGenTO) {
    const int nt = min(kGenTO, T - t0);
    __syncthreads();
    for (int i = threadIdx.x; i < nt * h; i += kST) {
      const int tl = i / h, j = i - tl * h;
      const float v = (dw(t0 + tl, j) - mean) * rstd * a.g2[j] + a.be2[j];
      Vs[i] = v * sigm(v);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nt * C; i += kST) {
      const int tl = i / C, c = i - tl * C;
      float acc = a.b3[c];
      const float* sv = Vs + tl * h;
      for (int j = 0; j < h; ++j) acc = fmaf(W3s[j * C + c], sv[j], acc);
      const int64_t o = (int64_t)(t0 + tl) * C + c;
      float v = xr[o] + acc;
      if (a.gelu) v = gelu_erf(v);
      xr[o] = v;
    }
  }
}

__global__ void scn_gelu_rows_kernel(float* X, int F_all, int f_off, int n_f, int64_t row_elems, int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int64_t row = i / row_elems, e = i - row * row_elems;
  const int64_t b = row / n_f;
  const int64_t f = f_off + row % n_f;
  float* p = X + (b * F_all + f) * row_elems + e;
  *p = gelu_erf(*p);
}

// ---- 3x3 convolution over (F, T), padding 1 (globalconv :215, FusionLayer :76) --------------
struct C3Args {
  const float* A;      // [B][F][T][Cin]
  const float* S;      // nullable, added to A on load (FusionLayer x += skip)
  int F, T, Cin;
  const float* W;      // [9][Cin][ncols]
  const float* bias;   // [ncols]
  int ncols;
  float* out;          // [B][F][T][c_store]
  int c_store;
  int glu;             // packed columns (a_2q, a_2q+1, g_2q, g_2q+1) -> out channels 2q, 2q+1
};
constexpr int kC3F = 4, kC3T = 32, kC3N = 64, kC3K = 16, kC3R = kC3T + 4;

__global__ void __launch_bounds__(kST) scn_conv3x3_kernel(C3Args a) {
  __shared__ __align__(16) float xs[kC3K][kC3F + 2][kC3R];
  __shared__ __align__(16) float ws[9][kC3K][kC3N];
  const int F = a.F, T = a.T, Cin = a.Cin;
  const int ntt = (T + kC3T - 1) / kC3T;
  const int t0 = (blockIdx.x % ntt) * kC3T, f0 = (blockIdx.x / ntt) * kC3F;
  const int n0 = blockIdx.y * kC3N;
  const int64_t b = blockIdx.z;
  const int cg = threadIdx.x & 15, pg = threadIdx.x >> 4;
  const int fl = pg >> 2, tg = pg & 3;
  float acc[8][4];
#pragma unroll
  for (int p = 0; p < 8; ++p)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[p][q] = 0.f;
  for (int ci0 = 0; ci0 < Cin; ci0 += kC3K) {
    __syncthreads();
    for (int i = threadIdx.x; i < kC3K * (kC3F + 2) * (kC3T + 2); i += kST) {
      const int ci = i & (kC3K - 1);
      const int r = i >> 4;
      const int tt = r % (kC3T + 2), fr = r / (kC3T + 2);
      const int f = f0 - 1 + fr, t = t0 - 1 + tt;
      float v = 0.f;
      if (f >= 0 && f < F && t >= 0 && t < T) {
        const int64_t idx = ((b * F + f) * T + t) * Cin + ci0 + ci;
        v = a.A[idx];
        if (a.S) v += a.S[idx];
      }
      xs[ci][fr][tt] = v;
    }
    for (int i = threadIdx.x; i < 9 * kC3K * kC3N; i += kST) {
      const int col = i & (kC3N - 1);
      const int r = i >> 6;
      const int ci = r & (kC3K - 1), tap = r >> 4;
      ws[tap][ci][col] = (n0 + col < a.ncols) ? a.W[((int64_t)tap * Cin + ci0 + ci) * a.ncols + n0 + col] : 0.f;
    }
    __syncthreads();
#pragma unroll 2
    for (int ci = 0; ci < kC3K; ++ci) {
#pragma unroll
      for (int df = 0; df < 3; ++df) {
        const float* xr = &xs[ci][fl + df][8 * tg];
        float xv[10];
        const float4 x0 = *reinterpret_cast<const float4*>(xr);
        const float4 x1 = *reinterpret_cast<const float4*>(xr + 4);
        const float2 x2 = *reinterpret_cast<const float2*>(xr + 8);
        xv[0] = x0.x; xv[1] = x0.y; xv[2] = x0.z; xv[3] = x0.w;
        xv[4] = x1.x; xv[5] = x1.y; xv[6] = x1.z; xv[7] = x1.w;
        xv[8] = x2.x; xv[9] = x2.y;
#pragma unroll
        for (int dt = 0; dt < 3; ++dt) {
          const float4 w = *reinterpret_cast<const float4*>(&ws[df * 3 + dt][ci][4 * cg]);
#pragma unroll
          for (int p = 0; p < 8; ++p) {
            const float xv_ = xv[p + dt];
            acc[p][0] = fmaf(xv_, w.x, acc[p][0]);
            acc[p][1] = fmaf(xv_, w.y, acc[p][1]);
            acc[p][2] = fmaf(xv_, w.z, acc[p][2]);
            acc[p][3] = fmaf(xv_, w.w, acc[p][3]);
          }
        }
      }
    }
  }
  const int f = f0 + fl;
  if (f >= F) return;
  const int col = n0 + 4 * cg;
  if (col >= a.ncols) return;
  float bv[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) bv[q] = col + q < a.ncols ? a.bias[col + q] : 0.f;
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int t = t0 + 8 * tg + p;
    if (t >= T) break;
    float* o = a.out + ((b * F + f) * T + t) * a.c_store;
    const float v0 = acc[p][0] + bv[0], v1 = acc[p][1] + bv[1], v2 = acc[p][2] + bv[2], v3 = acc[p][3] + bv[3];
    if (a.glu) {
      *reinterpret_cast<float2*>(o + col / 2) = make_float2(v0 * sigm(v2), v1 * sigm(v3));
    } else {
      o[col] = v0;
      if (col + 1 < a.ncols) o[col + 1] = v1;
      if (col + 2 < a.ncols) o[col + 2] = v2;
      if (col + 3 < a.ncols) o[col + 3] = v3;
    }
  }
}

// ---- DualPathRNN GroupNorm(1, d) over (C, F, T) per item (separation.py:66, :77) -------------
__global__ void scn_gn_stats_kernel(const float* __restrict__ X, int64_t n_item, double* __restrict__ stats) {
  __shared__ double red[2 * (kST / 64)];
  const int64_t b = blockIdx.y;
  const float* x = X + b * n_item;
  double s = 0, ss = 0;
  for (int64_t i = (int64_t)blockIdx.x * kST + threadIdx.x; i < n_item; i += (int64_t)gridDim.x * kST) {
    const double v = x[i];
    s += v;
    ss += v * v;
  }
  block_sum2(s, ss, red);
  if (threadIdx.x == 0) {
    atomicAdd(&stats[2 * b], s);
    atomicAdd(&stats[2 * b + 1], ss);
  }
}

__global__ void scn_gn_apply_kernel(const float* __restrict__ X, int64_t n_item, int C, const double* __restrict__ stats,
                                    const float* __restrict__ g, const float* __restrict__ be, float* __restrict__ Y,
                                    int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int64_t b = i / n_item;
  const int c = (int)(i % C);
  const double mu = stats[2 * b] / (double)n_item;
  const double var = fmax(stats[2 * b + 1] / (double)n_item - mu * mu, 0.0);
  const float mean = (float)mu, rstd = (float)(1.0 / sqrt(var + 1e-5));
  Y[i] = (X[i] - mean) * rstd * g[c] + be[c];
}
// the same as one fp16 plane (the fp16 input projection's A), four elements per thread (n_item % 4 == 0, C % 4 == 0)
__global__ void scn_gn_apply_f16_kernel(const float* __restrict__ X, int64_t n_item, int C, const double* __restrict__ stats,
                                        const float* __restrict__ g, const float* __restrict__ be, uint16_t* __restrict__ Y,
                                        int64_t total4) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total4) return;
  const int64_t e = 4 * i;
  const int64_t b = e / n_item;
  const int c = (int)(e % C);
  const double mu = stats[2 * b] / (double)n_item;
  const double var = fmax(stats[2 * b + 1] / (double)n_item - mu * mu, 0.0);
  const float mean = (float)mu, rstd = (float)(1.0 / sqrt(var + 1e-5));
  const f32x4 v = reinterpret_cast<const f32x4*>(X)[i];
  uint16_t o[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) o[q] = __builtin_bit_cast(uint16_t, (_Float16)((v[q] - mean) * rstd * g[c + q] + be[c + q]));
  *reinterpret_cast<uint2*>(Y + e) = make_uint2(o[0] | ((uint32_t)o[1] << 16), o[2] | ((uint32_t)o[3] << 16));
}

// ---- bi-LSTM recurrence (torch.nn.LSTM, batch_first, gate order i, f, g, o) -----------------
// token row of (sequence s, position p) = (s / sdiv) * smul_a + (s % sdiv) * smul_b + p * pstride
struct LstmArgs {
  const float* G;     // [rows][g_ld]: x W_ih^T + b_ih + b_hh, direction d at column d * 4H
  int64_t g_ld;
  float* HO;          // [rows][ho_ld]: h, direction d at column d * H
  int64_t ho_ld;
  const float* Wt;    // [2][H][4H]  (W_hh transposed, k-major)
  int H, L, n_seq, sdiv;
  int64_t smul_a, smul_b, pstride;
  // fp16mix chain (DpLayer::p16): the gates as the input projection's fp16 plane G16 (g_ld) with each direction's
  // columns gate-interleaved, 4 j + q = gate q of unit j (one 8-B load per row and lane), and h written as the output
  // Linear's fp16 A plane HO16 (ho_ld); null: G / HO in fp32, column q H + j
  const uint16_t* G16;
  uint16_t* HO16;
};
__device__ __forceinline__ float h2f(uint16_t v) { return (float)__builtin_bit_cast(_Float16, v); }

template <int ST>
__global__ void __launch_bounds__(kST) scn_lstm_kernel(LstmArgs a) {
  extern __shared__ __align__(16) float hs[];  // [2][S][H]
  const int H = a.H, H4 = 4 * H;
  const int ngrp = kST / H;
  const int S = ST * ngrp;
  const int j = threadIdx.x % H, sg = threadIdx.x / H;
  const int dir = blockIdx.y;
  const int seq0 = blockIdx.x * S + sg * ST;
  int64_t rowbase[ST];
  bool ok[ST];
  float c[ST];
#pragma unroll
  for (int u = 0; u < ST; ++u) {
    const int s = seq0 + u;
    ok[u] = s < a.n_seq;
    rowbase[u] = ok[u] ? (int64_t)(s / a.sdiv) * a.smul_a + (int64_t)(s % a.sdiv) * a.smul_b : 0;
    c[u] = 0.f;
    hs[(sg * ST + u) * H + j] = 0.f;
  }
  const float* W = a.Wt + (int64_t)dir * H * H4 + j;
  __syncthreads();
  for (int step = 0; step < a.L; ++step) {
    const int pos = dir ? a.L - 1 - step : step;
    const float* hc = hs + (step & 1) * S * H + sg * ST * H;
    float* hn = hs + ((step + 1) & 1) * S * H + sg * ST * H;
    float acc[ST][4];
#pragma unroll
    for (int u = 0; u < ST; ++u) {
      if (ok[u]) {
        const float* gp = a.G + (rowbase[u] + (int64_t)pos * a.pstride) * a.g_ld + dir * H4 + j;
#pragma unroll
        for (int g = 0; g < 4; ++g) acc[u][g] = gp[g * H];
      } else {
#pragma unroll
        for (int g = 0; g < 4; ++g) acc[u][g] = 0.f;
      }
    }
#pragma unroll 4
    for (int k = 0; k < H; ++k) {
      const float* wk = W + (int64_t)k * H4;
      const float w0 = wk[0], w1 = wk[H], w2 = wk[2 * H], w3 = wk[3 * H];
#pragma unroll
      for (int u = 0; u < ST; ++u) {
        const float hv = hc[u * H + k];
        acc[u][0] = fmaf(w0, hv, acc[u][0]);
        acc[u][1] = fmaf(w1, hv, acc[u][1]);
        acc[u][2] = fmaf(w2, hv, acc[u][2]);
        acc[u][3] = fmaf(w3, hv, acc[u][3]);
      }
    }
#pragma unroll
    for (int u = 0; u < ST; ++u) {
      const float ig = sigm(acc[u][0]), fg = sigm(acc[u][1]), gg = tanhf(acc[u][2]), og = sigm(acc[u][3]);
      c[u] = fg * c[u] + ig * gg;
      const float hv = og * tanhf(c[u]);
      hn[u * H + j] = hv;
      if (ok[u]) a.HO[(rowbase[u] + (int64_t)pos * a.pstride) * a.ho_ld + dir * H + j] = hv;
    }
    __syncthreads();
  }
}

// MFMA recurrence (bf16x3): one workgroup = 32 sequences of one direction, NW = H / 32 waves; wave w
// owns hidden units 32w .. 32w + 31 for all four gates, so the cell update is lane-local:
//   gates[32 seq][4H] = h[32][H] . W_hh^T  as v_mfma_f32_32x32x16_bf16 (h and W split hi/lo, 3 passes)
// h (bf16 hi/lo) lives in LDS as the A operand; W_hh's B fragments are pre-packed per lane
// ([dir][w][k-step][gate][hi, lo][64 lanes][8]) and streamed from L2 with a PF-deep register ring;
// the next step's input-projection gates are prefetched under the MFMAs.  c stays in registers.
// compact gate nonlinearities for the MFMA recurrence (abs. error ~1e-7, far below the bf16x3
// product error and the 1e-4 gate): one v_exp_f32 + one v_rcp_f32 each
__device__ __forceinline__ float sigm_f(float v) { return __builtin_amdgcn_rcpf(1.0f + __expf(-v)); }
__device__ __forceinline__ float tanh_f(float v) {
  const float t = __expf(-2.0f * fabsf(v));
  return copysignf((1.0f - t) * __builtin_amdgcn_rcpf(1.0f + t), v);
}

__device__ __forceinline__ f32x16 mfma_bf16(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 mfma_f16(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h16x8, a), __builtin_bit_cast(h16x8, b), c, 0, 0, 0);
}
// PS: MFMA passes of the recurrence product.  3: h and W_hh as bf16 hi + lo, three bf16 products (bf16x3).
// 2: h as one fp16 plane x W_hh as fp16 hi + lo (two fp16 products).  1: fp16 h x fp16 W_hh.  PS < 3 reads the
// fp16 fragment image (same layout, fp16 values) and keeps only the hi plane of h in LDS.
template <int PS>
__device__ __forceinline__ void lstm_mfma_step(const bf16x8& ah, const bf16x8& al, const bf16x8& bh, const bf16x8& bl,
                                               f32x16& acc) {
  if constexpr (PS == 3) {
    acc = mfma_bf16(al, bh, acc);
    acc = mfma_bf16(ah, bl, acc);
    acc = mfma_bf16(ah, bh, acc);
  } else if constexpr (PS == 2) {
    acc = mfma_f16(ah, bl, acc);
    acc = mfma_f16(ah, bh, acc);
  } else {
    acc = mfma_f16(ah, bh, acc);
  }
}
template <int PS>
__device__ __forceinline__ void lstm_store_h(float hv, uint16_t* hi, uint16_t* lo) {
  if constexpr (PS == 3) {
    __bf16 h, l;
    split_bf16(hv, h, l);
    *hi = __builtin_bit_cast(uint16_t, h);
    *lo = __builtin_bit_cast(uint16_t, l);
  } else {
    *hi = __builtin_bit_cast(uint16_t, (_Float16)hv);
  }
}

template <int NW, int PF, int PS = 3, bool G16 = false>
__global__ void __launch_bounds__(64 * NW) scn_lstm_mfma_kernel(LstmArgs a, const uint16_t* __restrict__ Wf) {
  static_assert(!G16 || PS < 3, "the fp16 gate plane feeds the fp16 recurrences");
  constexpr int H = 32 * NW, H4 = 4 * H, KS = H / 16, RS = H + 8;
  extern __shared__ __align__(16) uint16_t lsa[];
  uint16_t* Ahi = lsa;            // [32 seq][RS]
  uint16_t* Alo = lsa + 32 * RS;
  int64_t* rowb = reinterpret_cast<int64_t*>(lsa + 64 * RS);  // [32] token row of (seq, position 0); -1 = none
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int dir = blockIdx.y;
  const int s0 = blockIdx.x * 32;
  const int j = 32 * w + l32;
  float c[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) c[r] = 0.f;
  for (int i = threadIdx.x; i < 64 * RS; i += 64 * NW) lsa[i] = 0;  // h_0 = 0 (hi and lo)
  if (threadIdx.x < 32) {
    const int sq = s0 + threadIdx.x;
    rowb[threadIdx.x] = sq < a.n_seq ? (int64_t)(sq / a.sdiv) * a.smul_a + (int64_t)(sq % a.sdiv) * a.smul_b : -1;
  }
  // H <= 128: the compiler keeps the whole W_hh slice of a wave in registers across steps (<= 256,
  // one wave per SIMD); H = 160 .. 256 (two waves on a SIMD) streams it from L2 every step: `volatile`
  // stops that hoisting.
  constexpr bool STREAM = NW > 4;
  using WP = typename std::conditional<STREAM, const volatile bf16x8*, const bf16x8*>::type;
  WP wb = reinterpret_cast<WP>(Wf) + (int64_t)(dir * NW + w) * KS * 4 * 2 * 64 + lane;
  __syncthreads();
  for (int step = 0; step < a.L; ++step) {
    const int pos = dir ? a.L - 1 - step : step;
    // input-projection gates: issued now, added after the MFMAs (their latency hides under them);
    // the streamed-W variant (H = 256) loads them after the MFMAs (register budget of 2 waves/SIMD)
    // G16: the fp16 gate plane stays packed (8 B per row, 32 registers) until the cell update -- converting at the
    // load would make the MFMAs below wait for it
    float gv[G16 ? 1 : 4][16];
    uint2 graw[G16 ? 16 : 1];
    auto load_g = [&]() {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t rb = rowb[(r & 3) + 8 * (r >> 2) + 4 * hh];
        const int64_t go = rb >= 0 ? (rb + (int64_t)pos * a.pstride) * a.g_ld + dir * H4 : 0;
        if constexpr (G16) {
          graw[r] = rb >= 0 ? *reinterpret_cast<const uint2*>(a.G16 + go + 4 * j) : make_uint2(0u, 0u);
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) gv[G16 ? 0 : q][r] = rb >= 0 ? a.G[go + q * H + j] : 0.f;
        }
      }
    };
    if constexpr (!STREAM) load_g();
    f32x16 acc[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[q][r] = 0.f;
    bf16x8 bh[PF][4], bl[PF][4];
#pragma unroll
    for (int p = 0; p < PF; ++p)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        bh[p][q] = wb[((p * 4 + q) * 2 + 0) * 64];
        if constexpr (PS >= 2) bl[p][q] = wb[((p * 4 + q) * 2 + 1) * 64];
      }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int slot = ks % PF;
      const int ao = l32 * RS + 16 * ks + 8 * hh;
      const bf16x8 ah = *reinterpret_cast<const bf16x8*>(Ahi + ao);
      bf16x8 al{};
      if constexpr (PS == 3) al = *reinterpret_cast<const bf16x8*>(Alo + ao);
#pragma unroll
      for (int q = 0; q < 4; ++q) lstm_mfma_step<PS>(ah, al, bh[slot][q], bl[slot][q], acc[q]);
      if (ks + PF < KS) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          bh[slot][q] = wb[(((ks + PF) * 4 + q) * 2 + 0) * 64];
          if constexpr (PS >= 2) bl[slot][q] = wb[(((ks + PF) * 4 + q) * 2 + 1) * 64];
        }
      }
      if constexpr (STREAM) asm volatile("" ::: "memory");  // keep the prefetch depth at PF k-steps
    }
    if constexpr (STREAM) load_g();
    __syncthreads();  // every wave has read h_{t-1}
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int sl = (r & 3) + 8 * (r >> 2) + 4 * hh;
      float g4[4];
      if constexpr (G16) {
        const uint2 v = graw[r];
        g4[0] = h2f((uint16_t)v.x);
        g4[1] = h2f((uint16_t)(v.x >> 16));
        g4[2] = h2f((uint16_t)v.y);
        g4[3] = h2f((uint16_t)(v.y >> 16));
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) g4[q] = gv[G16 ? 0 : q][r];
      }
      const float ig = sigm_f(acc[0][r] + g4[0]), fg = sigm_f(acc[1][r] + g4[1]);
      const float gg = tanh_f(acc[2][r] + g4[2]), og = sigm_f(acc[3][r] + g4[3]);
      c[r] = fg * c[r] + ig * gg;
      const float hv = og * tanh_f(c[r]);
      lstm_store_h<PS>(hv, Ahi + sl * RS + j, Alo + sl * RS + j);
      const int64_t rb = rowb[sl];
      const int64_t ho = (rb + (int64_t)pos * a.pstride) * a.ho_ld + dir * H + j;
      if (a.HO16) {
        if (rb >= 0) a.HO16[ho] = __builtin_bit_cast(uint16_t, (_Float16)hv);
      } else {
        if (rb >= 0) a.HO[ho] = hv;
      }
    }
    __syncthreads();  // h_t visible
  }
}

// Wide recurrence (H = 288 .. 512, SCNet-large / XL odd dual-path layers: d = 2 dims[-1]): NW = H / 32
// waves (up to 1024 threads, 4 waves per SIMD, 128 registers each), the MFMA decomposition of
// scn_lstm_mfma_kernel.  The register budget is met by starting the accumulators from the
// input-projection gates (no separate gate registers) and streaming W_hh's B fragments through a
// one-k-step ring (4 gates x hi / lo = 32 registers): gate q of k-step ks + 1 is requested as soon as
// gate q of k-step ks has been consumed.
template <int NW, int PS = 3>
__global__ void __launch_bounds__(64 * NW, NW <= 8 ? 2 : 1) scn_lstm_mfma_wide_kernel(LstmArgs a,
                                                                                      const uint16_t* __restrict__ Wf) {
  constexpr int H = 32 * NW, H4 = 4 * H, KS = H / 16, RS = H + 8;
  extern __shared__ __align__(16) uint16_t lsa[];
  uint16_t* Ahi = lsa;            // [32 seq][RS]
  uint16_t* Alo = lsa + 32 * RS;
  int64_t* rowb = reinterpret_cast<int64_t*>(lsa + 64 * RS);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int dir = blockIdx.y;
  const int s0 = blockIdx.x * 32;
  const int j = 32 * w + l32;
  float c[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) c[r] = 0.f;
  for (int i = threadIdx.x; i < 64 * RS; i += 64 * NW) lsa[i] = 0;  // h_0 = 0 (hi and lo)
  if (threadIdx.x < 32) {
    const int sq = s0 + threadIdx.x;
    rowb[threadIdx.x] = sq < a.n_seq ? (int64_t)(sq / a.sdiv) * a.smul_a + (int64_t)(sq % a.sdiv) * a.smul_b : -1;
  }
  const volatile bf16x8* wb =
      reinterpret_cast<const volatile bf16x8*>(Wf) + (int64_t)(dir * NW + w) * KS * 4 * 2 * 64 + lane;
  __syncthreads();
  for (int step = 0; step < a.L; ++step) {
    const int pos = dir ? a.L - 1 - step : step;
    asm volatile("" ::: "memory");  // re-read rowb per step (no 32 hoisted row registers)
    f32x16 acc[4];
    // fp16 gate plane (PS < 3): one 8-B load per row, converted into the starting accumulators (no extra registers:
    // the kernel must stay within 128 VGPRs for two workgroups per CU at H = 256)
    const bool g16 = PS < 3 && a.G16 != nullptr;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t rb = rowb[(r & 3) + 8 * (r >> 2) + 4 * hh];
      const int64_t go = rb >= 0 ? (rb + (int64_t)pos * a.pstride) * a.g_ld + dir * H4 : 0;
      if (g16) {
        const uint2 v = rb >= 0 ? *reinterpret_cast<const uint2*>(a.G16 + go + 4 * j) : make_uint2(0u, 0u);
        acc[0][r] = h2f((uint16_t)v.x);
        acc[1][r] = h2f((uint16_t)(v.x >> 16));
        acc[2][r] = h2f((uint16_t)v.y);
        acc[3][r] = h2f((uint16_t)(v.y >> 16));
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q][r] = rb >= 0 ? a.G[go + q * H + j] : 0.f;
      }
    }
    bf16x8 bh[4], bl[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      bh[q] = wb[(q * 2 + 0) * 64];
      if constexpr (PS >= 2) bl[q] = wb[(q * 2 + 1) * 64];
    }
#pragma unroll 1
    for (int ks = 0; ks < KS; ++ks) {
      const int ao = l32 * RS + 16 * ks + 8 * hh;
      const bf16x8 ah = *reinterpret_cast<const bf16x8*>(Ahi + ao);
      bf16x8 al{};
      if constexpr (PS == 3) al = *reinterpret_cast<const bf16x8*>(Alo + ao);
      const int kn = ks + 1 < KS ? ks + 1 : ks;  // (the last k-step re-reads its own fragments: harmless)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        lstm_mfma_step<PS>(ah, al, bh[q], bl[q], acc[q]);
        bh[q] = wb[((kn * 4 + q) * 2 + 0) * 64];
        if constexpr (PS >= 2) bl[q] = wb[((kn * 4 + q) * 2 + 1) * 64];
      }
    }
    __syncthreads();  // every wave has read h_{t-1}
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int sl = (r & 3) + 8 * (r >> 2) + 4 * hh;
      const float ig = sigm_f(acc[0][r]), fg = sigm_f(acc[1][r]);
      const float gg = tanh_f(acc[2][r]), og = sigm_f(acc[3][r]);
      c[r] = fg * c[r] + ig * gg;
      const float hv = og * tanh_f(c[r]);
      lstm_store_h<PS>(hv, Ahi + sl * RS + j, Alo + sl * RS + j);
      const int64_t rb = rowb[sl];
      const int64_t ho = (rb + (int64_t)pos * a.pstride) * a.ho_ld + dir * H + j;
      if (a.HO16) {
        if (rb >= 0) a.HO16[ho] = __builtin_bit_cast(uint16_t, (_Float16)hv);
      } else {
        if (rb >= 0) a.HO[ho] = hv;
      }
    }
    __syncthreads();  // h_t visible
  }
}

// Smallest NW = H / 32 that takes scn_lstm_mfma_wide_kernel (SESA_LSTM_WIDE_MIN_NW, default 5: every H > 128).
// The register-resident kernel (NW <= 4) keeps W_hh in registers; its streamed form (NW 5..8) spills
// (170 VGPRs at H = 256), which the wide kernel's ring does not: same box, musdb18 SCNet 4-min track,
// LSTM class 180 -> 134 ms per step, 335.6x -> 359.1x real-time (profiles/r03_scnet_lstm_wide_{A,B,A2}.json).
int lstm_wide_min_nw() {
  static const int v = getenv("SESA_LSTM_WIDE_MIN_NW") ? atoi(getenv("SESA_LSTM_WIDE_MIN_NW")) : 5;
  return v;
}

size_t lstm_mfma_lds(int H) { return (size_t)64 * (H + 8) * 2 + 32 * 8; }

template <int NW, int PS = 3>
void launch_lstm_mfma_t(const LstmArgs& a, const uint16_t* Wf, hipStream_t st) {
  constexpr int PF = 2;
  const size_t lds = lstm_mfma_lds(32 * NW);
  dim3 grid((unsigned)((a.n_seq + 31) / 32), 2);
  if constexpr (NW <= 8) {
    if (NW < lstm_wide_min_nw()) {
      if constexpr (PS < 3) {
        if (a.G16) {
          hipLaunchKernelGGL((scn_lstm_mfma_kernel<NW, PF, PS, true>), grid, dim3(64 * NW), lds, st, a, Wf);
          return;
        }
      }
      hipLaunchKernelGGL((scn_lstm_mfma_kernel<NW, PF, PS>), grid, dim3(64 * NW), lds, st, a, Wf);
      return;
    }
  }
  hipLaunchKernelGGL((scn_lstm_mfma_wide_kernel<NW, PS>), grid, dim3(64 * NW), lds, st, a, Wf);
}
// the fp16 recurrence forms (PS 1 / 2) exist for H <= 256 (the musdb18 / base widths); wider layers run bf16x3
template <int PS>
bool launch_lstm_mfma_f16(const LstmArgs& a, const uint16_t* Wf, hipStream_t st) {
  switch (a.H / 32) {
    case 1: launch_lstm_mfma_t<1, PS>(a, Wf, st); return true;
    case 2: launch_lstm_mfma_t<2, PS>(a, Wf, st); return true;
    case 3: launch_lstm_mfma_t<3, PS>(a, Wf, st); return true;
    case 4: launch_lstm_mfma_t<4, PS>(a, Wf, st); return true;
    case 5: launch_lstm_mfma_t<5, PS>(a, Wf, st); return true;
    case 6: launch_lstm_mfma_t<6, PS>(a, Wf, st); return true;
    case 7: launch_lstm_mfma_t<7, PS>(a, Wf, st); return true;
    case 8: launch_lstm_mfma_t<8, PS>(a, Wf, st); return true;
    default: return false;
  }
}

// Raise the dynamic-LDS limit of the wide recurrence instances (> 64 KiB at H = 512); finalize time.
int lstm_mfma_prepare(int H) {
  if (lstm_mfma_lds(H) <= 64 * 1024) return SESA_OK;
  const void* fn = nullptr;
  switch (H / 32) {
#define SESA_WIDE(n) \
  case n: fn = (const void*)scn_lstm_mfma_wide_kernel<n>; break;
    SESA_WIDE(9) SESA_WIDE(10) SESA_WIDE(11) SESA_WIDE(12) SESA_WIDE(13) SESA_WIDE(14) SESA_WIDE(15) SESA_WIDE(16)
#undef SESA_WIDE
    default: return SESA_OK;
  }
  SESA_CHECK_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lstm_mfma_lds(H)));
  return SESA_OK;
}

// ps: 3 bf16x3 (Wf = the bf16 hi / lo image); 2 / 1: the fp16 forms (Wf = the fp16 hi / lo image), H <= 256
void launch_lstm_mfma(const LstmArgs& a, const uint16_t* Wf, int ps, hipStream_t st) {
  if (ps == 2 && launch_lstm_mfma_f16<2>(a, Wf, st)) return;
  if (ps == 1 && launch_lstm_mfma_f16<1>(a, Wf, st)) return;
  switch (a.H / 32) {
    case 1: launch_lstm_mfma_t<1>(a, Wf, st); break;
    case 2: launch_lstm_mfma_t<2>(a, Wf, st); break;
    case 3: launch_lstm_mfma_t<3>(a, Wf, st); break;
    case 4: launch_lstm_mfma_t<4>(a, Wf, st); break;
    case 5: launch_lstm_mfma_t<5>(a, Wf, st); break;
    case 6: launch_lstm_mfma_t<6>(a, Wf, st); break;
    case 7: launch_lstm_mfma_t<7>(a, Wf, st); break;
    case 8: launch_lstm_mfma_t<8>(a, Wf, st); break;
    case 9: launch_lstm_mfma_t<9>(a, Wf, st); break;
    case 10: launch_lstm_mfma_t<10>(a, Wf, st); break;
    case 11: launch_lstm_mfma_t<11>(a, Wf, st); break;
    case 12: launch_lstm_mfma_t<12>(a, Wf, st); break;
    case 13: launch_lstm_mfma_t<13>(a, Wf, st); break;
    case 14: launch_lstm_mfma_t<14>(a, Wf, st); break;
    case 15: launch_lstm_mfma_t<15>(a, Wf, st); break;
    default: launch_lstm_mfma_t<16>(a, Wf, st); break;
  }
}

// Launch-time choice of ST (sequences per thread; S = ST * 256 / H per workgroup): every
// workgroup re-reads all of W_hh^T (4 H^2 floats) from L2 per step, so small S multiplies L2
// traffic while large S serialises FMAs on few CUs.  Model per step: max(L2 bytes / 20 TB/s,
// resident-wave rounds x S * 4H * H FMA / (128 FMA/clk * 2.4 GHz)); pick the smallest.
void launch_lstm(const LstmArgs& a, hipStream_t st) {
  const int H = a.H;
  int best = 1;
  double best_t = 1e30;
  for (int ST = 1; ST <= 16; ST *= 2) {
    const int S = ST * (kST / H);
    const double n_wg = 2.0 * ((a.n_seq + S - 1) / S);
    const double l2 = n_wg * 16.0 * H * H / 20e12;
    const double comp = std::ceil(n_wg / 256.0) * (double)S * 4.0 * H * H / (128.0 * 2.4e9);
    const double t = std::max(l2, comp);
    if (t < best_t * 0.97) {
      best_t = t;
      best = ST;
    }
  }
  const int Sq = best * (kST / H);
  dim3 grid((unsigned)((a.n_seq + Sq - 1) / Sq), 2);
  const size_t lds = (size_t)2 * Sq * H * 4;
  switch (best) {
    case 16: hipLaunchKernelGGL(scn_lstm_kernel<16>, grid, dim3(kST), lds, st, a); break;
    case 8: hipLaunchKernelGGL(scn_lstm_kernel<8>, grid, dim3(kST), lds, st, a); break;
    case 4: hipLaunchKernelGGL(scn_lstm_kernel<4>, grid, dim3(kST), lds, st, a); break;
    case 2: hipLaunchKernelGGL(scn_lstm_kernel<2>, grid, dim3(kST), lds, st, a); break;
    default: hipLaunchKernelGGL(scn_lstm_kernel<1>, grid, dim3(kST), lds, st, a); break;
  }
}

// ---- FeatureConversion (separation.py:20-34): DFTs over T, norm = "ortho" -------------------
// rfft: X [R][T][C] -> Y [R][K][2C] (real | imag), K = T/2 + 1.  tw[m] = (cos, sin)(2 pi m / T).
__global__ void __launch_bounds__(kST) scn_rfft_kernel(const float* __restrict__ X, int T, int C,
                                                       const float2* __restrict__ tw, float scale,
                                                       float* __restrict__ Y) {
  __shared__ __align__(16) float xs[32][64];
  __shared__ float2 tws[1024];
  const int K = T / 2 + 1;
  const int64_t r = blockIdx.z;
  const int k0 = blockIdx.x * 32, c0 = blockIdx.y * 64;
  const int kq = threadIdx.x >> 5, cq = threadIdx.x & 31;
  for (int i = threadIdx.x; i < T; i += kST) tws[i] = tw[i];
  float are[4][2], aim[4][2];
  int idx[4], stp[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    stp[i] = (k0 + kq + 8 * i) % T;
    idx[i] = 0;
#pragma unroll
    for (int e = 0; e < 2; ++e) are[i][e] = aim[i][e] = 0.f;
  }
  const float* xr = X + r * T * C;
  for (int t0 = 0; t0 < T; t0 += 32) {
    __syncthreads();
    for (int i = threadIdx.x; i < 32 * 64; i += kST) {
      const int tt = i >> 6, cc = i & 63;
      const int t = t0 + tt, c = c0 + cc;
      xs[tt][cc] = (t < T && c < C) ? xr[(int64_t)t * C + c] : 0.f;
    }
    __syncthreads();
    const int nt = min(32, T - t0);
    for (int tt = 0; tt < nt; ++tt) {
      const float2 xv = *reinterpret_cast<const float2*>(&xs[tt][2 * cq]);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float2 w = tws[idx[i]];
        are[i][0] = fmaf(w.x, xv.x, are[i][0]);
        are[i][1] = fmaf(w.x, xv.y, are[i][1]);
        aim[i][0] = fmaf(-w.y, xv.x, aim[i][0]);
        aim[i][1] = fmaf(-w.y, xv.y, aim[i][1]);
        idx[i] += stp[i];
        if (idx[i] >= T) idx[i] -= T;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int k = k0 + kq + 8 * i;
    if (k >= K) continue;
    float* yr = Y + (r * K + k) * 2 * C;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int c = c0 + 2 * cq + e;
      if (c >= C) continue;
      yr[c] = are[i][e] * scale;
      yr[C + c] = aim[i][e] * scale;
    }
  }
}

// irfft: Y [R][K][2C] -> X [R][T][C], T = 2 (K - 1); imaginary parts of DC / Nyquist ignored.
__global__ void __launch_bounds__(kST) scn_irfft_kernel(const float* __restrict__ Y, int K, int C,
                                                        const float2* __restrict__ tw, float scale,
                                                        float* __restrict__ X) {
  __shared__ __align__(16) float ys[32][2][64];
  __shared__ float2 tws[1024];
  const int T = 2 * (K - 1);
  const int64_t r = blockIdx.z;
  const int t0 = blockIdx.x * 32, c0 = blockIdx.y * 64;
  const int tq = threadIdx.x >> 5, cq = threadIdx.x & 31;
  for (int i = threadIdx.x; i < T; i += kST) tws[i] = tw[i];
  float acc[4][2];
  int idx[4], stp[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    stp[i] = (t0 + tq + 8 * i) % T;
    idx[i] = 0;
    acc[i][0] = acc[i][1] = 0.f;
  }
  const float* yr = Y + r * K * 2 * C;
  for (int k0 = 0; k0 < K; k0 += 32) {
    __syncthreads();
    for (int i = threadIdx.x; i < 32 * 64; i += kST) {
      const int kk = i >> 6, cc = i & 63;
      const int k = k0 + kk, c = c0 + cc;
      float re = 0.f, im = 0.f;
      if (k < K && c < C) {
        const bool edge = k == 0 || k == K - 1;
        re = yr[(int64_t)k * 2 * C + c] * (edge ? 1.f : 2.f);
        im = edge ? 0.f : 2.f * yr[(int64_t)k * 2 * C + C + c];
      }
      ys[kk][0][cc] = re;
      ys[kk][1][cc] = im;
    }
    __syncthreads();
    const int nk = min(32, K - k0);
    for (int kk = 0; kk < nk; ++kk) {
      const float2 re = *reinterpret_cast<const float2*>(&ys[kk][0][2 * cq]);
      const float2 im = *reinterpret_cast<const float2*>(&ys[kk][1][2 * cq]);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float2 w = tws[idx[i]];
        acc[i][0] = fmaf(w.x, re.x, fmaf(-w.y, im.x, acc[i][0]));
        acc[i][1] = fmaf(w.x, re.y, fmaf(-w.y, im.y, acc[i][1]));
        idx[i] += stp[i];
        if (idx[i] >= T) idx[i] -= T;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int t = t0 + tq + 8 * i;
    if (t >= T) continue;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int c = c0 + 2 * cq + e;
      if (c < C) X[(r * T + t) * C + c] = acc[i][e] * scale;
    }
  }
}

// ---- FeatureConversion on the matrix cores (round 5) ------------------------------------------
// Both directions as one GEMM per sequence r:  out_r[m][n] = sum_k D[m][k] in_r[k][n].  D is constant per model
// (the ortho scale and the Hermitian weights folded in) and packed at finalize as bf16 hi / lo in MFMA A-fragment
// order, [MT][KS][hi, lo][64 lanes][8]: one 1 KiB contiguous load per fragment, L2-resident across the grid.
// in_r is staged once per workgroup into LDS as bf16 hi / lo with k contiguous (the B fragments); 3-pass bf16x3
// v_mfma_f32_32x32x16_bf16 (hi.hi + hi.lo + lo.hi), fp32 accumulation.
//   rfft : D [2K][T]; rows m < K -> real part of bin m, m >= K -> imaginary part of bin m - K
//          in_r[t][n] = X[r][t][n];                     out row m -> Y[r][m mod K][(m >= K) C + n]
//   irfft: D [T][2K]; cols k < K -> real part of bin k, k >= K -> imaginary part of bin k - K
//          in_r[k][n] = Y[r][k mod K][(k >= K) Ch + n];  out row t -> X[r][t][n]
struct DftArgs {
  const float* in;
  int64_t in_rs;           // floats per sequence
  int KK, Kh, ld, off2;    // k extent; rows k < Kh at k ld, rows k >= Kh at (k - Kh) ld + off2
  int N;                   // columns
  const uint16_t* D;       // packed matrix
  int MT, KS;              // 32-row tiles, 16-deep k steps (KP = 16 KS >= KK, zero padded)
  int Mtot, Mh, old, ooff2;
  int64_t out_rs;
  float* out;
};
constexpr int kDftWaves = 8;

__host__ __device__ constexpr size_t dft_lds_bytes(int nblk, int KS) {
  return (size_t)32 * nblk * (16 * KS + 8) * 2 * sizeof(uint16_t);
}

template <int NBLK>
__global__ void __launch_bounds__(64 * kDftWaves) scn_dft_mfma_kernel(DftArgs a) {
  constexpr int NB = 32 * NBLK, MPW = 4 / NBLK;  // wave tile: MPW M-tiles x NBLK N-tiles (64 accumulators)
  extern __shared__ __align__(16) uint16_t dls[];
  const int KP = 16 * a.KS, RS = KP + 8;  // RS * 2 B = 16 (mod 32) words: conflict-free ds_read_b128 rows
  uint16_t* Bh = dls;
  uint16_t* Bl = dls + NB * RS;
  const int64_t r = blockIdx.y;
  const int n0 = blockIdx.x * NB;
  const float* src = a.in + r * a.in_rs;
  // stage in_r[0, KP)[n0, n0 + NB) -> LDS (bf16 hi / lo, two k per 32-bit store); coalesced along n
  for (int i = threadIdx.x; i < NB * (KP / 2); i += 64 * kDftWaves) {
    const int n = i % NB, k = 2 * (i / NB), nn = n0 + n;
    float v[2] = {0.f, 0.f};
    if (nn < a.N) {
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int kk = k + e;
        if (kk < a.KK)
          v[e] = src[(kk < a.Kh ? (int64_t)kk * a.ld : (int64_t)(kk - a.Kh) * a.ld + a.off2) + nn];
      }
    }
    __bf16 h0, l0, h1, l1;
    split_bf16(v[0], h0, l0);
    split_bf16(v[1], h1, l1);
    const uint32_t ph = (uint32_t)__builtin_bit_cast(uint16_t, h0) | ((uint32_t)__builtin_bit_cast(uint16_t, h1) << 16);
    const uint32_t pl = (uint32_t)__builtin_bit_cast(uint16_t, l0) | ((uint32_t)__builtin_bit_cast(uint16_t, l1) << 16);
    *reinterpret_cast<uint32_t*>(Bh + n * RS + k) = ph;
    *reinterpret_cast<uint32_t*>(Bl + n * RS + k) = pl;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, l32 = lane & 31, hh = lane >> 5;
  const int ngroups = (a.MT + MPW - 1) / MPW;
  for (int g = w; g < ngroups; g += kDftWaves) {
    // tiles past MT re-read the last tile (valid memory); their rows are >= Mtot and never stored
    const bf16x8* dp[MPW];
#pragma unroll
    for (int i = 0; i < MPW; ++i)
      dp[i] = reinterpret_cast<const bf16x8*>(a.D) + (int64_t)min(g * MPW + i, a.MT - 1) * a.KS * 2 * 64 + lane;
    f32x16 acc[MPW][NBLK];
#pragma unroll
    for (int i = 0; i < MPW; ++i)
#pragma unroll
      for (int j = 0; j < NBLK; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
    bf16x8 ah[2][MPW], al[2][MPW];
#pragma unroll
    for (int i = 0; i < MPW; ++i) {
      ah[0][i] = dp[i][0];
      al[0][i] = dp[i][64];
    }
    const uint16_t* bh0 = Bh + l32 * RS + 8 * hh;
    const uint16_t* bl0 = Bl + l32 * RS + 8 * hh;
    auto step = [&](int ks, const bf16x8 (&h)[MPW], const bf16x8 (&l)[MPW]) {
      bf16x8 bh[NBLK], bl[NBLK];
#pragma unroll
      for (int j = 0; j < NBLK; ++j) {
        bh[j] = *reinterpret_cast<const bf16x8*>(bh0 + j * 32 * RS + 16 * ks);
        bl[j] = *reinterpret_cast<const bf16x8*>(bl0 + j * 32 * RS + 16 * ks);
      }
#pragma unroll
      for (int i = 0; i < MPW; ++i)
#pragma unroll
        for (int j = 0; j < NBLK; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(h[i], bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(h[i], bl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(l[i], bh[j], acc[i][j], 0, 0, 0);
        }
    };
    for (int ks = 0; ks < a.KS; ks += 2) {
      if (ks + 1 < a.KS) {
#pragma unroll
        for (int i = 0; i < MPW; ++i) {
          ah[1][i] = dp[i][((int64_t)(ks + 1) * 2) * 64];
          al[1][i] = dp[i][((int64_t)(ks + 1) * 2 + 1) * 64];
        }
      }
      step(ks, ah[0], al[0]);
      if (ks + 2 < a.KS) {
#pragma unroll
        for (int i = 0; i < MPW; ++i) {
          ah[0][i] = dp[i][((int64_t)(ks + 2) * 2) * 64];
          al[0][i] = dp[i][((int64_t)(ks + 2) * 2 + 1) * 64];
        }
      }
      if (ks + 1 < a.KS) step(ks + 1, ah[1], al[1]);
    }
    float* dst = a.out + r * a.out_rs;
#pragma unroll
    for (int i = 0; i < MPW; ++i)
#pragma unroll
      for (int j = 0; j < NBLK; ++j) {
        const int n = n0 + 32 * j + l32;
        if (n >= a.N) continue;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int mm = (g * MPW + i) * 32 + 8 * (e >> 2) + 4 * hh + (e & 3);
          if (mm >= a.Mtot) continue;
          dst[(mm < a.Mh ? (int64_t)mm * a.old : (int64_t)(mm - a.Mh) * a.old + a.ooff2) + n] = acc[i][j][e];
        }
      }
  }
}

// ---------------------------------------------------------------------------------------------
struct Param {
  std::string name;
  std::vector<int64_t> shape;
  int64_t numel = 0;
  std::vector<float> host;
  bool set = false;
};

struct CmLayer {  // float offsets into the packed fp32 blob
  int64_t g1, be1, w1, b1, wdw, bdw, g2, be2, w3, b3;
  int64_t w1h = -1, w3h = -1;   // uint16 offsets of scn_cm_mfma_kernel's fp16 fragments in the d_w blob (-1: none)
};

struct Level {
  int Fin, Fout, Cin, Cout, h, Cdec;  // Cdec: SU output channels
  bool cm_gen;                        // ConvolutionModule on the wide-level kernels (scn_cm_*_gen_kernel)
  BandConv sd[3], su[3];
  int64_t sd_w[3], sd_b[3], gc_w, gc_b, fu_w, fu_b, su_w[3], su_b[3];
  Gemm gc_gm, fu_gm;                  // globalconv / FusionLayer as implicit-GEMM convs (MFMA, bf16x3)
  // SD / SU band convs as implicit GEMMs in tok_gemm's sub-range conv form (sd_mm / su_mm: the band's geometry
  // has that form -- SU needs kern == stride (one tap, `stride` output phases) or stride 1 (flipped taps))
  bool sd_mm[3], su_mm[3];
  ConvGeo sd_geo[3], su_geo[3];
  Gemm sd_gm[3], su_gm[3];
  std::vector<CmLayer> cm[3];
};

struct DpLayer {
  int d, H;
  Gemm ih[2], lin[2];
  int64_t whh[2], gn_g[2], gn_b[2];
  int64_t whh_frag[2];  // uint16 offset of the MFMA B fragments (d_w blob)
  int64_t whh_frag16[2] = {-1, -1};  // the same as fp16 hi / lo (fp16mix, H <= 256: the PS < 3 recurrences)
  int p16 = 0;  // fp16mix plane chain (scn_p16_mode): 0 fp32 G / HO; 1 fp16 gate-interleaved G16; 2 G16 + fp16 HO16
};

}  // namespace
}  // namespace sesa

struct sesa_scnet {
  sesa_scnet_config cfg;
  std::vector<int> dims;
  int nl = 0, F0 = 0, T = 0, K = 0, Lpad = 0, padding = 0, nsig = 0;
  std::vector<sesa::Level> lv;
  std::vector<sesa::DpLayer> dp;
  std::vector<sesa::Param> params;
  std::map<std::string, int> by_name;
  float* d_f32 = nullptr;     // packed fp32 weights (convs, norms, W_hh^T)
  uint16_t* d_w = nullptr;    // token-GEMM bf16 hi/lo images
  float* d_bias = nullptr;
  float2* d_twT = nullptr;    // (cos, sin)(2 pi m / T)
  uint16_t* d_dft = nullptr;  // FeatureConversion DFT matrices, packed bf16 hi / lo ([0] rfft, [1] irfft)
  int dft_mt[2] = {0, 0}, dft_ks[2] = {0, 0};
  size_t dft_off[2] = {0, 0};
  bool finalized = false;
};

namespace sesa {
namespace {

void add_param(sesa_scnet* m, const std::string& name, std::vector<int64_t> shape) {
  Param p;
  p.name = name;
  p.shape = shape;
  p.numel = 1;
  for (auto s : shape) p.numel *= s;
  m->by_name[name] = (int)m->params.size();
  m->params.push_back(std::move(p));
}

const std::vector<float>& P(sesa_scnet* m, const std::string& name) { return m->params[m->by_name.at(name)].host; }

std::string S(int i) { return std::to_string(i); }

// SDlayer split points (scnet.py:117-122): ceil(Fr * SR_low), ceil(Fr * (SR_low + SR_mid)), in double
void splits(int Fr, const double* sr, int* s) {
  s[0] = 0;
  s[1] = (int)std::ceil(Fr * sr[0]);
  s[2] = (int)std::ceil(Fr * (sr[0] + sr[1]));
  s[3] = Fr;
}

struct Plan {
  size_t spec, skip[4], bufA, bufB, bufN, U, G, HO, stats, frames, total;
};

size_t al(size_t floats) { return (floats * 4 + 255) / 256 * 256; }

// Recurrence kernel choice (measured on MI355X, musdb18 config, 4-min track): bf16x3 MFMA for every
// H (325.7x real-time) beats MFMA for H <= 128 only (307.6x) and the fp32-FMA kernel (280.8x).
// SESA_LSTM_MFMA=0: fp32 everywhere; =1: MFMA for H <= 128 only (A/B comparisons).
// globalconv / FusionLayer 3x3 convs on the token GEMM's conv mode (MFMA, bf16x3); SESA_SCN_CONV3_VALU=1
// keeps the exact-fp32 VALU kernel (scn_conv3x3_kernel) for A/B.
bool scn_conv3_mfma() {
  static const bool v = !(getenv("SESA_SCN_CONV3_VALU") && std::string(getenv("SESA_SCN_CONV3_VALU")) == "1");
  return v;
}

// FeatureConversion DFTs on MFMA (scn_dft_mfma_kernel, bf16x3); SESA_SCN_DFT=0 keeps the fp32 VALU direct DFTs
// (scn_rfft_kernel / scn_irfft_kernel) for A/B.
// SESA_SCN_BAND_VALU=1: the SD / SU band convs on the fp32 VALU kernels (scn_sdconv_kernel / scn_convtr_kernel)
// instead of tok_gemm's conv mode (A/B runs)
bool scn_band_mfma() {
  static const bool v = !(getenv("SESA_SCN_BAND_VALU") && std::string(getenv("SESA_SCN_BAND_VALU")) == "1");
  return v;
}

// the fused MFMA ConvolutionModule layer (scn_cm_mfma_kernel) takes this geometry; SESA_SCN_CM_VALU=1: the VALU
// kernels in fp16mix too (A/B runs)
bool scn_cm_mfma_ok(int T, int C, int h) {
  return C % 32 == 0 && h % 8 == 0 && h <= 64 && kST % (C / 4) == 0 && kST % h == 0 &&
         cm_mfma_layout(T, C, h).total <= 160 * 1024;
}
bool scn_cm_mfma_env() {
  static const bool v = !(getenv("SESA_SCN_CM_VALU") && std::string(getenv("SESA_SCN_CM_VALU")) == "1");
  return v;
}
int launch_cm_mfma(const CmArgs& a, int rows, hipStream_t st) {
  const size_t lds = cm_mfma_layout(a.T, a.C, a.h).total;
  switch (a.h / 8) {
    case 1: hipLaunchKernelGGL(scn_cm_mfma_kernel<1>, dim3(rows), dim3(kST), lds, st, a); break;
    case 2: hipLaunchKernelGGL(scn_cm_mfma_kernel<2>, dim3(rows), dim3(kST), lds, st, a); break;
    case 4: hipLaunchKernelGGL(scn_cm_mfma_kernel<4>, dim3(rows), dim3(kST), lds, st, a); break;
    case 8: hipLaunchKernelGGL(scn_cm_mfma_kernel<8>, dim3(rows), dim3(kST), lds, st, a); break;
    default: SESA_REQUIRE(false, SESA_ERR_INVALID, "scnet: ConvolutionModule MFMA hidden size %d", a.h);
  }
  SESA_CHECK_LAUNCH();
  return SESA_OK;
}

// fp16mix LSTM recurrence passes (lstm_mfma_step): SESA_SCN_LSTM_PASSES = 1 (default: fp16 h x fp16 W_hh) | 2 | 3
// (bf16x3).  Same box, musdb18 4-min track: lstm class 121.6 / 114.6 / 59.6 ms per step at 3 / 2 / 1 passes, the
// full-chunk fixture's rms 1.6558e-5 / 1.6560e-5 / 1.6556e-5 (profiles/r06_scnet_lstm_ps*.json): the wide kernel
// streams W_hh's fragments from L2 every step, and one pass reads half of them (the hi image only)
int scn_lstm_passes() {
  static const int v = [] {
    const int p = getenv("SESA_SCN_LSTM_PASSES") ? atoi(getenv("SESA_SCN_LSTM_PASSES")) : 1;
    return p == 1 || p == 2 ? p : 3;
  }();
  return v;
}

// SESA_SCN_P16 = 0 | 1 | 2 (default 2): how much of the fp16mix dual-path chain runs in fp16 planes (DpLayer::p16)
int scn_p16_mode() {
  static const int v = getenv("SESA_SCN_P16") ? atoi(getenv("SESA_SCN_P16")) : 2;
  return v;
}

bool scn_dft_mfma() {
  static const bool v = !(getenv("SESA_SCN_DFT") && std::string(getenv("SESA_SCN_DFT")) == "0");
  return v;
}

// (The fp32 kernel needs 256 % H == 0; wider or odd widths always take the MFMA recurrence.)
bool lstm_mfma_on(int H) {
  static const int mode = getenv("SESA_LSTM_MFMA") ? atoi(getenv("SESA_LSTM_MFMA")) : 2;
  return mode == 2 || (mode == 1 && H <= 128) || H > 256 || kST % H != 0;
}

Plan plan(const sesa_scnet* m, int B) {
  Plan p{};
  size_t off = 0;
  const int64_t T = m->T;
  p.spec = off;
  off += al((size_t)B * m->F0 * T * m->dims[0]);
  size_t e = 0, u = 0;
  for (int i = 0; i < m->nl; ++i) {
    const Level& L = m->lv[i];
    p.skip[i] = off;
    off += al((size_t)B * L.Fout * T * L.Cout);
    e = std::max(e, (size_t)B * L.Fout * T * L.Cout);
    e = std::max(e, (size_t)B * L.Fin * T * L.Cdec);
    u = std::max(u, (size_t)B * L.Fout * T * L.h);
  }
  const int Fn = m->lv[m->nl - 1].Fout, d = m->dims[m->nl];
  e = std::max(e, (size_t)B * Fn * T * d);
  e = std::max(e, (size_t)B * Fn * m->K * 2 * d);
  size_t g = 0, ho = 0;
  for (const DpLayer& L : m->dp) {
    const size_t rows = (size_t)B * Fn * (L.d == d ? T : m->K);
    g = std::max(g, rows * 8 * L.H);
    ho = std::max(ho, rows * 2 * L.H);
  }
  p.bufA = off; off += al(e);
  p.bufB = off; off += al(e);
  p.bufN = off; off += al(e);
  p.U = off; off += al(u);
  p.G = off; off += al(g);
  p.HO = off; off += al(ho);
  p.stats = off; off += al((size_t)B * 4);
  p.frames = off; off += al((size_t)B * m->nsig * T * kSN);
  p.total = off;
  return p;
}

size_t cm_in_lds(int C, int h) { return (size_t)(6 * h * C + (512 / h + 2) * C) * 4 + 16 * 8 + 16; }
size_t cm_in_rb_lds(int C, int h) { return (size_t)(6 * h * C + (cm_rb_tt(h) + 2) * C) * 4 + 16 * 8 + 16; }
// SESA_SCN_CM_RB=0: the one-output-per-thread ConvolutionModule head (A/B of scn_cm_in_rb_kernel)
bool scn_cm_rb_on(int C, int h) {
  static const bool off = getenv("SESA_SCN_CM_RB") && std::string(getenv("SESA_SCN_CM_RB")) == "0";
  return !off && h % CM_JB == 0 && (kST * CM_TB * CM_JB) % h == 0 && cm_in_rb_lds(C, h) <= 160 * 1024;
}
size_t cm_out_lds(int T, int C, int h) { return (size_t)(2 * T * h + h * C + 1) * 4 + 16 * 8 + 16; }

double gemm_flops(const Gemm& gm, int64_t M) {
  double f = 0;
  for (auto& g : gm.groups) f += 2.0 * (double)M * g.N * g.K;
  return f;
}

}  // namespace
}  // namespace sesa

using namespace sesa;

extern "C" int sesa_scnet_create(const sesa_scnet_config* cfg, sesa_scnet** out) {
  clear_error();
  SESA_REQUIRE(cfg && out && cfg->dims && cfg->n_dims >= 2 && cfg->n_dims <= 5, SESA_ERR_INVALID,
               "sesa_scnet_create: bad arguments");
  const sesa_scnet_config& c = *cfg;
  SESA_REQUIRE(c.n_fft == kSN && c.win_size == kSN, SESA_ERR_INVALID, "scnet: only nfft = win_size = 4096");
  SESA_REQUIRE(c.hop_size > 0 && c.chunk_size > kSN / 2, SESA_ERR_INVALID, "scnet: bad hop_size / chunk_size");
  SESA_REQUIRE(c.audio_channels >= 1 && c.audio_channels <= 2 && c.n_sources >= 1, SESA_ERR_INVALID,
               "scnet: audio_channels 1 or 2, n_sources >= 1");
  SESA_REQUIRE(c.dims[0] == 2 * c.audio_channels, SESA_ERR_INVALID, "scnet: dims[0] must be 2 * audio_channels");
  SESA_REQUIRE(c.conv_kernel == 3, SESA_ERR_INVALID, "scnet: conv_kernel 3 only");
  SESA_REQUIRE(c.num_dplayer >= 0 && c.num_dplayer % 2 == 0 && c.expand >= 1, SESA_ERR_INVALID,
               "scnet: num_dplayer must be even (rfft/irfft pairs)");
  SESA_REQUIRE(c.precision == SESA_PREC_BF16X3 || c.precision == SESA_PREC_BF16 || c.precision == SESA_PREC_F16MIX,
               SESA_ERR_INVALID, "scnet: precision");
  sesa_scnet* m = new sesa_scnet();
  m->cfg = c;
  m->dims.assign(c.dims, c.dims + c.n_dims);
  m->cfg.dims = nullptr;
  m->nl = c.n_dims - 1;
  auto fail = [&](const char* msg, int v) {
    delete m;
    set_error("scnet: %s (%d)", msg, v);
    return SESA_ERR_INVALID;
  };
  const int hop = c.hop_size;
  int padding = hop - c.chunk_size % hop;
  if ((c.chunk_size + padding) / hop % 2 == 0) padding += hop;
  m->padding = padding;
  m->Lpad = c.chunk_size + padding;
  m->T = m->Lpad / hop + 1;
  m->K = m->T / 2 + 1;
  m->F0 = kSN / 2 + 1;
  m->nsig = c.n_sources * c.audio_channels;
  if (m->T % 2) return fail("odd frame count", m->T);
  if (m->T > 1024) return fail("more than 1024 STFT frames per chunk (DFT twiddle table)", m->T);
  // levels: SD geometry (scnet.py:114-148) and SU trims (:171-196)
  int Fr = m->F0;
  for (int i = 0; i < m->nl; ++i) {
    Level L{};
    L.Fin = Fr;
    L.Cin = m->dims[i];
    L.Cout = m->dims[i + 1];
    L.h = (int)(L.Cout / (double)c.compress);
    L.Cdec = i == 0 ? m->dims[0] * c.n_sources : m->dims[i];
    int sp[4];
    splits(Fr, c.band_sr, sp);
    int fo = 0;
    for (int b = 0; b < 3; ++b) {
      BandConv& bc = L.sd[b];
      bc.in_off = sp[b];
      bc.n_in = sp[b + 1] - sp[b];
      bc.stride = c.band_stride[b];
      bc.kern = c.band_kernel[b];
      if (bc.n_in <= 0 || bc.stride <= 0 || bc.kern <= 0) return fail("empty band", b);
      const int tot = bc.stride == 1 ? bc.kern - bc.stride : (bc.stride - bc.n_in % bc.stride) % bc.stride;
      bc.pad_left = tot / 2;
      bc.n_out = (bc.n_in + tot - bc.kern) / bc.stride + 1;
      if (bc.n_out <= 0) return fail("band shorter than its kernel", b);
      bc.out_off = fo;
      fo += bc.n_out;
      BandConv& su = L.su[b];
      su.in_off = bc.out_off;
      su.n_in = bc.n_out;
      su.stride = bc.stride;
      su.kern = bc.kern;
      const int full = (bc.n_out - 1) * bc.stride + bc.kern;
      if (full < bc.n_in) return fail("transposed band conv shorter than the band", b);
      su.dist = (full - bc.n_in) / 2;
      su.n_out = bc.n_in;
      su.out_off = bc.in_off;
    }
    L.Fout = fo;
    // band conv geometry on the (F, T) grid, taps along F; input / output bands are row sub-ranges of the level
    // tensors [B][F][T][C] (scnet.py:114-148 SD, :171-196 SU)
    for (int b = 0; b < 3; ++b) {
      const BandConv& bc = L.sd[b];
      ConvGeo& g = L.sd_geo[b];
      g = ConvGeo{};
      g.P1 = bc.n_out; g.P2 = m->T; g.Q1 = bc.n_in; g.Q2 = m->T; g.s1 = bc.stride; g.s2 = 1;
      g.Cin = L.Cin;
      g.n_taps = bc.kern;
      for (int kk = 0; kk < std::min(bc.kern, kMaxTaps); ++kk) g.d1[kk] = kk - bc.pad_left;
      g.phases = 1; g.O1 = bc.n_out;
      g.xq1 = L.Fin; g.x_row0 = bc.in_off; g.oq1 = L.Fout; g.o_row0 = bc.out_off;
      L.sd_mm[b] = bc.kern <= kMaxTaps && L.Cin % 4 == 0;
      const BandConv& su = L.su[b];
      ConvGeo& u = L.su_geo[b];
      u = ConvGeo{};
      u.P2 = m->T; u.Q1 = su.n_in; u.Q2 = m->T; u.s1 = 1; u.s2 = 1;
      u.Cin = L.Cout;
      u.O1 = su.n_out;
      u.xq1 = L.Fout; u.x_row0 = su.in_off; u.oq1 = L.Fin; u.o_row0 = su.out_off;
      u.o_fmajor = i == 0;   // the last decoder layer writes the iSTFT's frame-major spectrum [B][T][F0][2 nsig]
      if (su.kern == su.stride) {  // input row fi -> output rows fi s + r - dist, r < s: one tap, s phases
        u.P1 = su.n_in;
        u.n_taps = 1;
        u.phases = su.stride;
        u.opad = su.dist;
      } else {                     // stride 1: output row fo <- input rows fo + dist - kk (flipped taps)
        u.P1 = su.n_out;
        u.n_taps = su.kern;
        for (int kk = 0; kk < std::min(su.kern, kMaxTaps); ++kk) u.d1[kk] = su.dist - kk;
        u.phases = 1;
      }
      L.su_mm[b] = (su.kern == su.stride || (su.stride == 1 && su.kern <= kMaxTaps)) && L.Cout % 4 == 0;
    }
    if (L.h < 1) return fail("ConvolutionModule hidden size must be >= 1", L.h);
    if (L.Cout % 16 || L.Cdec % 4) return fail("dims must be multiples of 16 (decoder output channels of 4)", L.Cout);
    // the row-resident kernels where they fit (base / small configs), else the wide-level kernels
    L.cm_gen = (512 % L.h) != 0 || L.h > 64 || cm_in_lds(L.Cout, L.h) > 160 * 1024 ||
               cm_out_lds(m->T, L.Cout, L.h) > 160 * 1024;
    if (L.cm_gen && (L.h > kST || cm_in_gen_lds(L.h) > 160 * 1024 || cm_out_gen_lds(L.Cout, L.h) > 160 * 1024))
      return fail("ConvolutionModule too wide for LDS (1x1 weight [h][C] must fit)", L.Cout);
    m->lv.push_back(L);
    Fr = fo;
  }
  const int dlast = m->dims[m->nl];
  for (int i = 0; i < c.num_dplayer; ++i) {
    DpLayer L{};
    L.d = dlast * (i % 2 ? 2 : 1);
    L.H = L.d * c.expand;
    if (L.H % 32 || L.H < 32 || L.H > 512) return fail("LSTM hidden size must be a multiple of 32 in [32, 512]", L.H);
    m->dp.push_back(L);
  }
  // parameter registry, reference state_dict order (scnet.py:280-323)
  for (int i = 0; i < m->nl; ++i) {
    const Level& L = m->lv[i];
    const std::string p = "encoder." + S(i);
    for (int b = 0; b < 3; ++b) {
      add_param(m, p + ".SDlayer.convs." + S(b) + ".weight", {L.Cout, L.Cin, c.band_kernel[b], 1});
      add_param(m, p + ".SDlayer.convs." + S(b) + ".bias", {L.Cout});
    }
    for (int b = 0; b < 3; ++b)
      for (int l = 0; l < std::abs(c.conv_depths[b]); ++l) {
        const std::string q = p + ".conv_modules." + S(b) + ".layers." + S(l);
        add_param(m, q + ".0.weight", {L.Cout});
        add_param(m, q + ".0.bias", {L.Cout});
        add_param(m, q + ".1.weight", {2 * L.h, L.Cout, 3});
        add_param(m, q + ".1.bias", {2 * L.h});
        add_param(m, q + ".3.weight", {L.h, 1, 3});
        add_param(m, q + ".3.bias", {L.h});
        add_param(m, q + ".4.weight", {L.h});
        add_param(m, q + ".4.bias", {L.h});
        add_param(m, q + ".6.weight", {L.Cout, L.h, 1});
        add_param(m, q + ".6.bias", {L.Cout});
      }
    add_param(m, p + ".globalconv.weight", {L.Cout, L.Cout, 3, 3});
    add_param(m, p + ".globalconv.bias", {L.Cout});
  }
  for (int j = 0; j < m->nl; ++j) {
    const Level& L = m->lv[m->nl - 1 - j];
    const std::string p = "decoder." + S(j);
    add_param(m, p + ".0.conv.weight", {2 * L.Cout, 2 * L.Cout, 3, 3});
    add_param(m, p + ".0.conv.bias", {2 * L.Cout});
    for (int b = 0; b < 3; ++b) {
      add_param(m, p + ".1.convtrs." + S(b) + ".weight", {L.Cout, L.Cdec, c.band_kernel[b], 1});
      add_param(m, p + ".1.convtrs." + S(b) + ".bias", {L.Cdec});
    }
  }
  for (int i = 0; i < c.num_dplayer; ++i) {
    const DpLayer& L = m->dp[i];
    const std::string p = "separation_net.dp_modules." + S(i);
    for (int l = 0; l < 2; ++l)
      for (const char* sfx : {"", "_reverse"}) {
        const std::string q = p + ".lstm_layers." + S(l);
        add_param(m, q + ".weight_ih_l0" + sfx, {4 * L.H, L.d});
        add_param(m, q + ".weight_hh_l0" + sfx, {4 * L.H, L.H});
        add_param(m, q + ".bias_ih_l0" + sfx, {4 * L.H});
        add_param(m, q + ".bias_hh_l0" + sfx, {4 * L.H});
      }
    for (int l = 0; l < 2; ++l) {
      add_param(m, p + ".linear_layers." + S(l) + ".weight", {L.d, 2 * L.H});
      add_param(m, p + ".linear_layers." + S(l) + ".bias", {L.d});
    }
    for (int l = 0; l < 2; ++l) {
      add_param(m, p + ".norm_layers." + S(l) + ".weight", {L.d});
      add_param(m, p + ".norm_layers." + S(l) + ".bias", {L.d});
    }
  }
  *out = m;
  return SESA_OK;
}

extern "C" int sesa_scnet_num_params(const sesa_scnet* m) { return m ? (int)m->params.size() : 0; }

extern "C" int sesa_scnet_param_info(const sesa_scnet* m, int i, const char** name, int64_t* numel) {
  clear_error();
  SESA_REQUIRE(m && i >= 0 && i < (int)m->params.size(), SESA_ERR_INVALID, "scnet param_info: index out of range");
  if (name) *name = m->params[i].name.c_str();
  if (numel) *numel = m->params[i].numel;
  return SESA_OK;
}

extern "C" int sesa_scnet_set_param(sesa_scnet* m, const char* name, const float* host, int64_t numel) {
  clear_error();
  SESA_REQUIRE(m && name && host, SESA_ERR_INVALID, "scnet set_param: null argument");
  auto it = m->by_name.find(name);
  SESA_REQUIRE(it != m->by_name.end(), SESA_ERR_INVALID, "scnet set_param: unknown parameter '%s'", name);
  Param& p = m->params[it->second];
  SESA_REQUIRE(p.numel == numel, SESA_ERR_INVALID, "scnet set_param: '%s' expects %lld elements, got %lld", name,
               (long long)p.numel, (long long)numel);
  p.host.assign(host, host + numel);
  p.set = true;
  m->finalized = false;
  return SESA_OK;
}

extern "C" int sesa_scnet_finalize(sesa_scnet* m, void* stream) {
  clear_error();
  SESA_REQUIRE(m, SESA_ERR_INVALID, "scnet finalize: null model");
  for (auto& p : m->params)
    SESA_REQUIRE(p.set, SESA_ERR_STATE, "scnet finalize: parameter '%s' was never set", p.name.c_str());
  const sesa_scnet_config& c = m->cfg;
  std::vector<float> f32;
  auto put = [&](const std::vector<float>& v) {
    const int64_t o = (int64_t)f32.size();
    f32.insert(f32.end(), v.begin(), v.end());
    while (f32.size() % 4) f32.push_back(0.f);
    return o;
  };
  auto putp = [&](const std::string& n) { return put(P(m, n)); };
  for (int i = 0; i < m->nl; ++i) {
    Level& L = m->lv[i];
    const std::string p = "encoder." + S(i);
    for (int b = 0; b < 3; ++b) {  // [Cout][Cin][k][1] -> [k][Cin][Cout]
      const auto& W = P(m, p + ".SDlayer.convs." + S(b) + ".weight");
      const int k = L.sd[b].kern;
      std::vector<float> w((size_t)k * L.Cin * L.Cout);
      for (int co = 0; co < L.Cout; ++co)
        for (int ci = 0; ci < L.Cin; ++ci)
          for (int kk = 0; kk < k; ++kk) w[((size_t)kk * L.Cin + ci) * L.Cout + co] = W[((size_t)co * L.Cin + ci) * k + kk];
      L.sd_w[b] = put(w);
      L.sd_b[b] = putp(p + ".SDlayer.convs." + S(b) + ".bias");
      L.cm[b].clear();
      for (int l = 0; l < std::abs(c.conv_depths[b]); ++l) {
        const std::string q = p + ".conv_modules." + S(b) + ".layers." + S(l);
        CmLayer cl{};
        const int C = L.Cout, h = L.h;
        cl.g1 = putp(q + ".0.weight");
        cl.be1 = putp(q + ".0.bias");
        const auto& W1 = P(m, q + ".1.weight");  // [2h][C][3] -> [C][3][2h]
        std::vector<float> w1((size_t)6 * h * C);
        for (int o = 0; o < 2 * h; ++o)
          for (int ci = 0; ci < C; ++ci)
            for (int kk = 0; kk < 3; ++kk) w1[((size_t)ci * 3 + kk) * 2 * h + o] = W1[((size_t)o * C + ci) * 3 + kk];
        cl.w1 = put(w1);
        cl.b1 = putp(q + ".1.bias");
        cl.wdw = putp(q + ".3.weight");
        cl.bdw = putp(q + ".3.bias");
        cl.g2 = putp(q + ".4.weight");
        cl.be2 = putp(q + ".4.bias");
        const auto& W3 = P(m, q + ".6.weight");  // [C][h][1] -> [h][C]
        std::vector<float> w3((size_t)h * C);
        for (int co = 0; co < C; ++co)
          for (int j = 0; j < h; ++j) w3[(size_t)j * C + co] = W3[(size_t)co * h + j];
        cl.w3 = put(w3);
        cl.b3 = putp(q + ".6.bias");
        L.cm[b].push_back(cl);
      }
    }
    {  // globalconv [Cout][Cout][3][3] -> [9][Cin][Cout]
      const auto& W = P(m, p + ".globalconv.weight");
      const int C = L.Cout;
      std::vector<float> w((size_t)9 * C * C);
      for (int co = 0; co < C; ++co)
        for (int ci = 0; ci < C; ++ci)
          for (int tap = 0; tap < 9; ++tap) w[((size_t)tap * C + ci) * C + co] = W[((size_t)co * C + ci) * 9 + tap];
      L.gc_w = put(w);
      L.gc_b = putp(p + ".globalconv.bias");
    }
    const std::string dpfx = "decoder." + S(m->nl - 1 - i);
    {  // FusionLayer: repeat(1, 2) folded (W[:, ci] + W[:, ci + C]); GLU column interleave
      const auto& W = P(m, dpfx + ".0.conv.weight");
      const auto& Bv = P(m, dpfx + ".0.conv.bias");
      const int C = L.Cout, C2 = 2 * C;
      std::vector<float> w((size_t)9 * C * C2), bias(C2);
      auto src_col = [C](int col) { const int q = col >> 2, r = col & 3; return (r < 2 ? 0 : C) + 2 * q + (r & 1); };
      for (int col = 0; col < C2; ++col) {
        const int co = src_col(col);
        bias[col] = Bv[co];
        for (int ci = 0; ci < C; ++ci)
          for (int tap = 0; tap < 9; ++tap)
            w[((size_t)tap * C + ci) * C2 + col] =
                W[((size_t)co * C2 + ci) * 9 + tap] + W[((size_t)co * C2 + ci + C) * 9 + tap];
      }
      L.fu_w = put(w);
      L.fu_b = put(bias);
    }
    for (int b = 0; b < 3; ++b) {  // ConvTranspose2d [Cin][Cout][k][1] -> [k][Cin][Cout]
      const auto& W = P(m, dpfx + ".1.convtrs." + S(b) + ".weight");
      const int k = L.su[b].kern, Ci = L.Cout, Co = L.Cdec;
      std::vector<float> w((size_t)k * Ci * Co);
      for (int ci = 0; ci < Ci; ++ci)
        for (int co = 0; co < Co; ++co)
          for (int kk = 0; kk < k; ++kk) w[((size_t)kk * Ci + ci) * Co + co] = W[((size_t)ci * Co + co) * k + kk];
      L.su_w[b] = put(w);
      L.su_b[b] = putp(dpfx + ".1.convtrs." + S(b) + ".bias");
    }
  }
  std::vector<uint16_t> blob;
  std::vector<float> bias;
  // fp16mix: the token GEMMs (3x3 convs, LSTM input projections, dual-path Linears) as fp16 weight images for
  // the fp16 single-pass kernels; W_hh (the recurrence) stays bf16 hi / lo
  const bool f16w = m->cfg.precision == SESA_PREC_F16MIX;
  // globalconv / FusionLayer 3x3 convs for the token GEMM's conv mode: K = 9 taps x C (tap = 3 df + dt,
  // channel-minor); FusionLayer: repeat(1, 2) folded, GLU pairs interleaved (column 2j = a_j, 2j + 1 = gate_j)
  for (int i = 0; i < m->nl; ++i) {
    Level& L = m->lv[i];
    const int C = L.Cout;
    const auto& Wg = P(m, "encoder." + S(i) + ".globalconv.weight");  // [C][C][3][3]
    const auto& Bg = P(m, "encoder." + S(i) + ".globalconv.bias");
    TokGroup g = pack_group(
        C, 9 * C, [&](int n, int k) { const int tap = k / C, ci = k - tap * C; return Wg[((size_t)n * C + ci) * 9 + tap]; },
        true, [&](int n) { return Bg[n]; }, blob, bias, f16w);
    g.x_off = g.o_off = 0;
    L.gc_gm.groups = {g};
    const std::string dpfx = "decoder." + S(m->nl - 1 - i);
    const auto& Wf = P(m, dpfx + ".0.conv.weight");  // [2C][2C][3][3]
    const auto& Bf = P(m, dpfx + ".0.conv.bias");
    const int C2 = 2 * C;
    g = pack_group(
        C2, 9 * C,
        [&](int n, int k) {
          const int co = (n & 1) ? C + (n >> 1) : (n >> 1), tap = k / C, ci = k - tap * C;
          return Wf[((size_t)co * C2 + ci) * 9 + tap] + Wf[((size_t)co * C2 + ci + C) * 9 + tap];
        },
        true, [&](int n) { return Bf[(n & 1) ? C + (n >> 1) : (n >> 1)]; }, blob, bias, f16w);
    g.x_off = g.o_off = 0;
    L.fu_gm.groups = {g};
    // band convs: SD K = kern x Cin (tap-major); SU one tap with `stride` phases (column r Cdec + co = kernel row
    // r, output channel co), or stride 1 with K = kern x Cin
    for (int b = 0; b < 3; ++b) {
      const std::string sp = "encoder." + S(i) + ".SDlayer.convs." + S(b);
      const auto& Ws = P(m, sp + ".weight");  // [Cout][Cin][k][1]
      const auto& Bs = P(m, sp + ".bias");
      const int k = L.sd[b].kern, Ci = L.Cin;
      if (L.sd_mm[b]) {
        g = pack_group(
            L.Cout, k * Ci, [&](int n, int kx) { const int kk = kx / Ci, ci = kx - kk * Ci; return Ws[((size_t)n * Ci + ci) * k + kk]; },
            true, [&](int n) { return Bs[n]; }, blob, bias, f16w);
        g.x_off = g.o_off = 0;
        L.sd_gm[b].groups = {g};
      }
      const std::string up = dpfx + ".1.convtrs." + S(b);
      const auto& Wu = P(m, up + ".weight");  // [Cout][Cdec][k][1]
      const auto& Bu = P(m, up + ".bias");
      const int ku = L.su[b].kern, s = L.su[b].stride, Cu = L.Cout, Cd = L.Cdec;
      if (!L.su_mm[b]) continue;
      if (ku == s)
        g = pack_group(
            s * Cd, Cu, [&](int n, int ci) { const int r = n / Cd, co = n - r * Cd; return Wu[((size_t)ci * Cd + co) * ku + r]; },
            true, [&](int n) { return Bu[n % Cd]; }, blob, bias, f16w);
      else
        g = pack_group(
            Cd, ku * Cu, [&](int n, int kx) { const int kk = kx / Cu, ci = kx - kk * Cu; return Wu[((size_t)ci * Cd + n) * ku + kk]; },
            true, [&](int n) { return Bu[n]; }, blob, bias, f16w);
      g.x_off = g.o_off = 0;
      L.su_gm[b].groups = {g};
    }
    // ConvolutionModule layers as fp16 MFMA fragments (scn_cm_mfma_kernel): W1 [2h][C][3] -> [3C / 32][h / 8][64][8]
    // with k = dt C + c and column tile nt = value columns 8 nt .. 8 nt + 7, then their gates; W3 [C][h][1] ->
    // [hp / 32][C / 16][64][8], zero past h
    if (f16w && scn_cm_mfma_ok(m->T, L.Cout, L.h)) {
      const int h = L.h, NT1 = h / 8, hp = cm_hp(h);
      auto f16 = [](float v) { return __builtin_bit_cast(uint16_t, (_Float16)v); };
      for (int b = 0; b < 3; ++b)
        for (size_t l = 0; l < L.cm[b].size(); ++l) {
          const std::string q = "encoder." + S(i) + ".conv_modules." + S(b) + ".layers." + S((int)l);
          const auto& W1 = P(m, q + ".1.weight");
          const auto& W3 = P(m, q + ".6.weight");
          while (blob.size() % 8) blob.push_back(0);
          CmLayer& cl = L.cm[b][l];
          cl.w1h = (int64_t)blob.size();
          for (int ks = 0; ks < 3 * C / 32; ++ks)
            for (int nt = 0; nt < NT1; ++nt)
              for (int ln = 0; ln < 64; ++ln)
                for (int e = 0; e < 8; ++e) {
                  const int k = 32 * ks + 8 * (ln >> 4) + e, dt = k / C, c = k - dt * C, qc = ln & 15;
                  const int o = qc < 8 ? 8 * nt + qc : h + 8 * nt + qc - 8;
                  blob.push_back(f16(W1[((size_t)o * C + c) * 3 + dt]));
                }
          cl.w3h = (int64_t)blob.size();
          for (int ks = 0; ks < hp / 32; ++ks)
            for (int nt = 0; nt < C / 16; ++nt)
              for (int ln = 0; ln < 64; ++ln)
                for (int e = 0; e < 8; ++e) {
                  const int k = 32 * ks + 8 * (ln >> 4) + e, n = 16 * nt + (ln & 15);
                  blob.push_back(k < h ? f16(W3[(size_t)n * h + k]) : 0);
                }
        }
    }
  }
  for (int i = 0; i < (int)m->dp.size(); ++i) {
    DpLayer& L = m->dp[i];
    const std::string p = "separation_net.dp_modules." + S(i);
    const int H = L.H, d = L.d;
    for (int l = 0; l < 2; ++l) {
      const std::string q = p + ".lstm_layers." + S(l);
      const auto& Wf = P(m, q + ".weight_ih_l0");
      const auto& Wr = P(m, q + ".weight_ih_l0_reverse");
      const auto& bif = P(m, q + ".bias_ih_l0");
      const auto& bhf = P(m, q + ".bias_hh_l0");
      const auto& bir = P(m, q + ".bias_ih_l0_reverse");
      const auto& bhr = P(m, q + ".bias_hh_l0_reverse");
      // the fp16 chain's gate plane interleaves each direction's columns: packed column dir 4H + 4 j + q = gate q of
      // unit j (source row dir 4H + q H + j)
      L.p16 = f16w && H <= 256 && lstm_mfma_on(H) && scn_lstm_passes() < 3 ? scn_p16_mode() : 0;
      const bool ilv = L.p16 > 0;
      auto src_n = [&](int n) { const int dir = n / (4 * H), r = n - dir * 4 * H;
                                return ilv ? dir * 4 * H + (r & 3) * H + (r >> 2) : n; };
      TokGroup g = pack_group(
          8 * H, d,
          [&](int n, int k) { const int sn = src_n(n);
                              return sn < 4 * H ? Wf[(int64_t)sn * d + k] : Wr[(int64_t)(sn - 4 * H) * d + k]; }, true,
          [&](int n) { const int sn = src_n(n); return sn < 4 * H ? bif[sn] + bhf[sn] : bir[sn - 4 * H] + bhr[sn - 4 * H]; },
          blob, bias, f16w);
      g.x_off = g.o_off = 0;
      L.ih[l].groups = {g};
      const auto& Wl = P(m, p + ".linear_layers." + S(l) + ".weight");
      const auto& bl = P(m, p + ".linear_layers." + S(l) + ".bias");
      g = pack_group(d, 2 * H, [&](int n, int k) { return Wl[(int64_t)n * 2 * H + k]; }, true,
                     [&](int n) { return bl[n]; }, blob, bias, f16w);
      g.x_off = g.o_off = 0;
      L.lin[l].groups = {g};
      std::vector<float> wt((size_t)2 * H * 4 * H);  // W_hh [4H][H] -> [dir][k][4H]
      for (int dir = 0; dir < 2; ++dir) {
        const auto& Wh = P(m, q + (dir ? ".weight_hh_l0_reverse" : ".weight_hh_l0"));
        for (int n = 0; n < 4 * H; ++n)
          for (int k = 0; k < H; ++k) wt[((size_t)dir * H + k) * 4 * H + n] = Wh[(size_t)n * H + k];
      }
      L.whh[l] = put(wt);
      {  // B fragments of W_hh for scn_lstm_mfma_kernel: [dir][w][ks][gate][hi, lo][64 lanes][8]
        const int NW = H / 32, KS = H / 16;
        L.whh_frag[l] = (int64_t)blob.size();
        blob.resize(blob.size() + (size_t)2 * NW * KS * 4 * 2 * 64 * 8, 0);
        uint16_t* f = blob.data() + L.whh_frag[l];
        for (int dir = 0; dir < 2; ++dir) {
          const auto& Wh = P(m, q + (dir ? ".weight_hh_l0_reverse" : ".weight_hh_l0"));
          for (int w = 0; w < NW; ++w)
            for (int ks = 0; ks < KS; ++ks)
              for (int g4 = 0; g4 < 4; ++g4)
                for (int ln = 0; ln < 64; ++ln)
                  for (int e = 0; e < 8; ++e) {
                    const int n = g4 * H + 32 * w + (ln & 31);
                    const int k = 16 * ks + 8 * (ln >> 5) + e;
                    const float v = Wh[(size_t)n * H + k];
                    const uint16_t hb = f2bf(v);
                    const size_t base = ((((((size_t)dir * NW + w) * KS + ks) * 4 + g4) * 2) * 64 + ln) * 8 + e;
                    f[base] = hb;
                    f[base + 64 * 8] = f2bf(v - bf2f(hb));
                  }
        }
      }
      if (f16w && H <= 256) {  // the same fragments as fp16 hi / lo (lstm_mfma_step PS 1 / 2)
        const int NW = H / 32, KS = H / 16;
        while (blob.size() % 8) blob.push_back(0);
        L.whh_frag16[l] = (int64_t)blob.size();
        blob.resize(blob.size() + (size_t)2 * NW * KS * 4 * 2 * 64 * 8, 0);
        uint16_t* f = blob.data() + L.whh_frag16[l];
        for (int dir = 0; dir < 2; ++dir) {
          const auto& Wh = P(m, q + (dir ? ".weight_hh_l0_reverse" : ".weight_hh_l0"));
          for (int w = 0; w < NW; ++w)
            for (int ks = 0; ks < KS; ++ks)
              for (int g4 = 0; g4 < 4; ++g4)
                for (int ln = 0; ln < 64; ++ln)
                  for (int e = 0; e < 8; ++e) {
                    const float v = Wh[(size_t)(g4 * H + 32 * w + (ln & 31)) * H + 16 * ks + 8 * (ln >> 5) + e];
                    const _Float16 hh = (_Float16)v;
                    const size_t base = ((((((size_t)dir * NW + w) * KS + ks) * 4 + g4) * 2) * 64 + ln) * 8 + e;
                    f[base] = __builtin_bit_cast(uint16_t, hh);
                    f[base + 64 * 8] = __builtin_bit_cast(uint16_t, (_Float16)(v - (float)hh));
                  }
        }
      }
      L.gn_g[l] = putp(p + ".norm_layers." + S(l) + ".weight");
      L.gn_b[l] = putp(p + ".norm_layers." + S(l) + ".bias");
    }
  }
  std::vector<float2> twT(m->T);
  for (int i = 0; i < m->T; ++i) {
    const double ang = 2.0 * M_PI * i / m->T;
    twT[i] = make_float2((float)cos(ang), (float)sin(ang));
  }
  // FeatureConversion DFT matrices (separation.py:20-34, norm = "ortho"), built in double and split hi / lo in
  // A-fragment order: [MT][KS][hi, lo][64 lanes][8], lane -> row 32 mt + lane % 32, k 16 ks + 8 (lane / 32) + e.
  std::vector<uint16_t> dft;
  {
    const int T = m->T, K = m->K;
    const double s = 1.0 / std::sqrt((double)T);
    for (int dir = 0; dir < 2; ++dir) {
      const int M = dir == 0 ? 2 * K : T, KK = dir == 0 ? T : 2 * K;
      const int MT = (M + 31) / 32, KS = (KK + 15) / 16;
      auto val = [&](int row, int col) -> double {
        if (row >= M || col >= KK) return 0.0;
        if (dir == 0) {  // row = bin (re | im), col = frame
          const int k = row < K ? row : row - K;
          const double ang = 2.0 * M_PI * (double)(((int64_t)k * col) % T) / T;
          return row < K ? s * std::cos(ang) : -s * std::sin(ang);
        }
        const int k = col < K ? col : col - K;  // row = frame, col = bin (re | im)
        const bool edge = k == 0 || k == K - 1;
        const double ang = 2.0 * M_PI * (double)(((int64_t)k * row) % T) / T;
        if (col < K) return s * (edge ? 1.0 : 2.0) * std::cos(ang);
        return edge ? 0.0 : -2.0 * s * std::sin(ang);
      };
      m->dft_mt[dir] = MT;
      m->dft_ks[dir] = KS;
      m->dft_off[dir] = dft.size();
      dft.resize(dft.size() + (size_t)MT * KS * 2 * 64 * 8);
      uint16_t* o = dft.data() + m->dft_off[dir];
      for (int mt = 0; mt < MT; ++mt)
        for (int ks = 0; ks < KS; ++ks)
          for (int ln = 0; ln < 64; ++ln)
            for (int e = 0; e < 8; ++e) {
              const float v = (float)val(32 * mt + ln % 32, 16 * ks + 8 * (ln / 32) + e);
              const uint16_t hb = f2bf(v);
              const size_t base = ((((size_t)mt * KS + ks) * 2) * 64 + ln) * 8 + e;
              o[base] = hb;
              o[base + 64 * 8] = f2bf(v - bf2f(hb));
            }
    }
  }
  for (void* p : {(void*)m->d_f32, (void*)m->d_w, (void*)m->d_bias, (void*)m->d_twT, (void*)m->d_dft})
    if (p) (void)hipFree(p);
  m->d_dft = nullptr;
  m->d_f32 = nullptr;
  m->d_w = nullptr;
  m->d_bias = nullptr;
  m->d_twT = nullptr;
  SESA_REQUIRE(hipMalloc(&m->d_f32, std::max<size_t>(f32.size(), 1) * 4) == hipSuccess, SESA_ERR_NOMEM,
               "scnet finalize: hipMalloc weights");
  SESA_REQUIRE(hipMalloc(&m->d_w, std::max<size_t>(blob.size(), 1) * 2) == hipSuccess, SESA_ERR_NOMEM,
               "scnet finalize: hipMalloc gemm weights");
  SESA_REQUIRE(hipMalloc(&m->d_bias, std::max<size_t>(bias.size(), 1) * 4) == hipSuccess, SESA_ERR_NOMEM,
               "scnet finalize: hipMalloc bias");
  SESA_REQUIRE(hipMalloc(&m->d_twT, twT.size() * sizeof(float2)) == hipSuccess, SESA_ERR_NOMEM,
               "scnet finalize: hipMalloc twiddles");
  SESA_REQUIRE(hipMalloc(&m->d_dft, dft.size() * 2) == hipSuccess, SESA_ERR_NOMEM,
               "scnet finalize: hipMalloc DFT matrices");
  hipStream_t st = as_stream(stream);
  SESA_CHECK_HIP(hipMemcpyAsync(m->d_f32, f32.data(), f32.size() * 4, hipMemcpyHostToDevice, st));
  if (!blob.empty()) SESA_CHECK_HIP(hipMemcpyAsync(m->d_w, blob.data(), blob.size() * 2, hipMemcpyHostToDevice, st));
  if (!bias.empty()) SESA_CHECK_HIP(hipMemcpyAsync(m->d_bias, bias.data(), bias.size() * 4, hipMemcpyHostToDevice, st));
  SESA_CHECK_HIP(hipMemcpyAsync(m->d_twT, twT.data(), twT.size() * sizeof(float2), hipMemcpyHostToDevice, st));
  SESA_CHECK_HIP(hipMemcpyAsync(m->d_dft, dft.data(), dft.size() * 2, hipMemcpyHostToDevice, st));
  SESA_CHECK_HIP(hipStreamSynchronize(st));
  for (auto& L : m->dp) {
    const int rc = lstm_mfma_prepare(L.H);
    if (rc) return rc;
  }
  for (auto& L : m->lv) {
    int rc = upload_groups(L.gc_gm);
    if (!rc) rc = upload_groups(L.fu_gm);
    for (int b = 0; b < 3 && !rc; ++b) {
      if (L.sd_mm[b]) rc = upload_groups(L.sd_gm[b]);
      if (!rc && L.su_mm[b]) rc = upload_groups(L.su_gm[b]);
    }
    if (rc) return rc;
  }
  for (auto& L : m->dp)
    for (int l = 0; l < 2; ++l) {
      int rc = upload_groups(L.ih[l]);
      if (!rc) rc = upload_groups(L.lin[l]);
      if (rc) return rc;
    }
  SESA_CHECK_HIP(hipFuncSetAttribute((const void*)scn_cm_in_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     160 * 1024));
  SESA_CHECK_HIP(hipFuncSetAttribute((const void*)scn_cm_out_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     160 * 1024));
  SESA_CHECK_HIP(hipFuncSetAttribute((const void*)scn_cm_in_rb_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     160 * 1024));
  SESA_CHECK_HIP(hipFuncSetAttribute((const void*)scn_cm_in_gen_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     160 * 1024));
  SESA_CHECK_HIP(hipFuncSetAttribute((const void*)scn_cm_out_gen_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     160 * 1024));
  SESA_CHECK_HIP(hipFuncSetAttribute((const void*)scn_dft_mfma_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     160 * 1024));
  SESA_CHECK_HIP(hipFuncSetAttribute((const void*)scn_dft_mfma_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     160 * 1024));
  for (const void* k : {(const void*)scn_cm_mfma_kernel<1>, (const void*)scn_cm_mfma_kernel<2>,
                        (const void*)scn_cm_mfma_kernel<4>, (const void*)scn_cm_mfma_kernel<8>})
    SESA_CHECK_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  m->finalized = true;
  return SESA_OK;
}

extern "C" size_t sesa_scnet_workspace_size(const sesa_scnet* m, int batch) {
  if (!m || batch <= 0) return 0;
  return plan(m, batch).total;
}

extern "C" int sesa_scnet_forward(sesa_scnet* m, const float* x, int B, float* out, void* workspace,
                                  size_t workspace_bytes, void* stream) {
  clear_error();
  SESA_REQUIRE(m && x && out && workspace && B > 0, SESA_ERR_INVALID, "scnet forward: bad arguments");
  SESA_REQUIRE(m->finalized, SESA_ERR_STATE, "scnet forward: call sesa_scnet_finalize first");
  const Plan pl = plan(m, B);
  SESA_REQUIRE(workspace_bytes >= pl.total, SESA_ERR_INVALID, "scnet forward: workspace %zu < required %zu",
               workspace_bytes, pl.total);
  const sesa_scnet_config& c = m->cfg;
  hipStream_t st = as_stream(stream);
  char* ws = reinterpret_cast<char*>(workspace);
  auto F32 = [&](size_t off) { return reinterpret_cast<float*>(ws + off); };
  const float* Wb = m->d_f32;
  const int T = m->T, K = m->K, F0 = m->F0, ach = c.audio_channels;
  const bool f16mix = c.precision == SESA_PREC_F16MIX;
  // the VALU-recurrence fallback's / DFTs' passes: bf16x3 in fp16mix (the MFMA recurrence: scn_lstm_passes())
  const int x3 = c.precision == SESA_PREC_BF16X3 || f16mix ? 1 : 0;
  const int gx = f16mix ? 2 : x3;   // token GEMMs (3x3 convs, input projections, Linears): fp16 single pass
  ScnTables tb;
  int rc = get_tables(&tb);
  if (rc) return rc;
  auto blocks = [](int64_t n) { return dim3((unsigned)((n + kST - 1) / kST)); };
  // 3x3 conv over (F, T), padding 1, as an implicit GEMM (K = 9 taps x C): A = x (+ S on load), bias,
  // optional GLU over interleaved column pairs (FusionLayer)
  double conv3_bytes = 0;   // algorithmic bytes of the last conv3_gemm launch (profiling)
  auto conv3_gemm = [&](const Gemm& gm, const float* xin, const float* S, int F, int C, float* o, int o_ld, int glu) {
    TokGemmArgs a{};
    a.x = xin;
    a.x_ld = C;
    a.out = o;
    a.o_ld = o_ld;
    a.w = m->d_w;
    a.bias = m->d_bias;
    a.groups = gm.d_groups;
    a.n_groups = 1;
    a.n_tiles_n = gm.n_tiles_n;
    a.M = B * F * T;
    a.act = TOK_ACT_NONE;
    a.glu = glu;
    a.conv = 1;
    ConvGeo& g = a.geo;
    g.P1 = F; g.P2 = T; g.Q1 = F; g.Q2 = T; g.s1 = 1; g.s2 = 1;
    g.Cin = C;
    g.n_taps = 9;
    for (int t = 0; t < 9; ++t) {
      g.d1[t] = t / 3 - 1;
      g.d2[t] = t % 3 - 1;
    }
    g.x2 = S;
    g.phases = 1;
    if (gm.groups[0].N % 128 == 64) {  // 64-column tiles where a 128-column tile would be 75 % full
      a.bn64 = 1;
      a.n_tiles_n = (gm.groups[0].N + 63) / 64;
    }
    conv3_bytes = tok_gemm_bytes(a, gm, gx);
    return launch_tok_gemm(a, gx, st);
  };
  // one SD / SU band conv (sub-range conv form, geometry from create): x [B][xq1][T][Cin] -> o [B][oq1][T][o_ld];
  // adds its algorithmic flops / bytes to *fl / *by
  auto band_gemm = [&](const Gemm& gm, const ConvGeo& geo, const float* xin, float* o, int o_ld, double* fl,
                       double* by) {
    TokGemmArgs a{};
    a.x = xin;
    a.x_ld = geo.Cin;
    a.out = o;
    a.o_ld = o_ld;
    a.w = m->d_w;
    a.bias = m->d_bias;
    a.groups = gm.d_groups;
    a.n_groups = 1;
    a.M = B * geo.P1 * geo.P2;
    a.act = TOK_ACT_NONE;
    a.conv = 1;
    a.geo = geo;
    const int N = gm.groups[0].N;
    a.bn64 = N <= 64 || N % 128 == 64;   // narrow bands: 64-column tiles
    a.n_tiles_n = a.bn64 ? (N + 63) / 64 : gm.n_tiles_n;
    *fl += 2.0 * a.M * N * gm.groups[0].K;
    *by += tok_gemm_bytes(a, gm, gx);
    return launch_tok_gemm(a, gx, st);
  };

  // 1. STFT (scnet.py:335-348)
  float* spec = F32(pl.spec);
  {
    void* tok = profile_begin(st);
    hipLaunchKernelGGL(scn_stft_kernel, dim3(T, B * ach), dim3(kST), 0, st, x, ach, c.chunk_size, m->Lpad,
                       c.hop_size, T, c.normalized ? 1.0f / 64.0f : 1.0f, tb, spec);
    SESA_CHECK_LAUNCH();
    profile_end(tok, st, SESA_KCLASS_STFT, 4.0 * B * ach * ((double)c.chunk_size + (double)T * F0 * 2));
  }
  float* bufA = F32(pl.bufA);
  float* bufB = F32(pl.bufB);
  float* bufN = F32(pl.bufN);
  float* U = F32(pl.U);
  // 2. encoder (scnet.py:356-361)
  const float* cur = spec;
  for (int i = 0; i < m->nl; ++i) {
    const Level& L = m->lv[i];
    float* skip = F32(pl.skip[i]);
    void* tok = profile_begin(st);
    double fl = 0;
    // algorithmic bytes of the simt group: the level input read once and the band outputs written once, then
    // every ConvolutionModule layer reads and writes its rows once
    double by = 4.0 * B * T * ((double)L.Fin * L.Cin + (double)L.Fout * L.Cout);
    const bool sd_mfma = scn_band_mfma() && L.sd_mm[0] && L.sd_mm[1] && L.sd_mm[2];
    if (sd_mfma) {  // the three bands on MFMA, profiled as their own record
      double gfl = 0, gby = 0;
      for (int b = 0; b < 3 && !rc; ++b) rc = band_gemm(L.sd_gm[b], L.sd_geo[b], cur, skip, L.Cout, &gfl, &gby);
      if (rc) return rc;
      profile_end(tok, st, SESA_KCLASS_TOKGEMM, gfl, gby);
      tok = profile_begin(st);
      by = 0;
    }
    for (int b = 0; b < 3 && !sd_mfma; ++b) {
      const BandConv& bc = L.sd[b];
      const int64_t total = (int64_t)B * bc.n_out * T * (L.Cout / 4);
      hipLaunchKernelGGL(scn_sdconv_kernel, blocks(total), dim3(kST), 0, st, cur, L.Fin, T, L.Cin, Wb + L.sd_w[b],
                         Wb + L.sd_b[b], bc, skip, L.Fout, L.Cout, total);
      SESA_CHECK_LAUNCH();
      fl += 2.0 * total * 4 * L.Cin * bc.kern;
    }
    for (int b = 0; b < 3; ++b) {
      const BandConv& bc = L.sd[b];
      const int rows = B * bc.n_out;
      if (L.cm[b].empty()) {
        const int64_t total = (int64_t)rows * T * L.Cout;
        hipLaunchKernelGGL(scn_gelu_rows_kernel, blocks(total), dim3(kST), 0, st, skip, L.Fout, bc.out_off, bc.n_out,
                           (int64_t)T * L.Cout, total);
        SESA_CHECK_LAUNCH();
      }
      for (size_t l = 0; l < L.cm[b].size(); ++l) {
        const CmLayer& cl = L.cm[b][l];
        CmArgs a{};
        a.X = skip;
        a.F_all = L.Fout;
        a.f_off = bc.out_off;
        a.n_f = bc.n_out;
        a.T = T;
        a.C = L.Cout;
        a.h = L.h;
        a.g1 = Wb + cl.g1;
        a.be1 = Wb + cl.be1;
        a.W1 = Wb + cl.w1;
        a.b1 = Wb + cl.b1;
        a.U = U;
        a.wdw = Wb + cl.wdw;
        a.bdw = Wb + cl.bdw;
        a.g2 = Wb + cl.g2;
        a.be2 = Wb + cl.be2;
        a.W3 = Wb + cl.w3;
        a.b3 = Wb + cl.b3;
        a.gelu = l + 1 == L.cm[b].size();
        if (cl.w1h >= 0 && scn_cm_mfma_env()) {
          a.W1h = m->d_w + cl.w1h;
          a.W3h = m->d_w + cl.w3h;
          rc = launch_cm_mfma(a, rows, st);
          if (rc) return rc;
        } else if (L.cm_gen) {
          hipLaunchKernelGGL(scn_cm_in_gen_kernel, dim3(rows), dim3(kST), cm_in_gen_lds(L.h), st, a);
          SESA_CHECK_LAUNCH();
          hipLaunchKernelGGL(scn_cm_out_gen_kernel, dim3(rows), dim3(kST), cm_out_gen_lds(L.Cout, L.h), st, a);
          SESA_CHECK_LAUNCH();
        } else {
          if (scn_cm_rb_on(L.Cout, L.h))
            hipLaunchKernelGGL(scn_cm_in_rb_kernel, dim3(rows), dim3(kST), cm_in_rb_lds(L.Cout, L.h), st, a);
          else
            hipLaunchKernelGGL(scn_cm_in_kernel, dim3(rows), dim3(kST), cm_in_lds(L.Cout, L.h), st, a);
          SESA_CHECK_LAUNCH();
          hipLaunchKernelGGL(scn_cm_out_kernel, dim3(rows), dim3(kST), cm_out_lds(T, L.Cout, L.h), st, a);
          SESA_CHECK_LAUNCH();
        }
        fl += 2.0 * rows * T * (6.0 * L.h * L.Cout + 3.0 * L.h + (double)L.h * L.Cout);
        by += 8.0 * rows * T * L.Cout;
      }
    }
    if (scn_conv3_mfma()) {  // globalconv (3x3) -> bufA on the token GEMM's conv mode
      profile_end(tok, st, SESA_KCLASS_SIMT, fl, by);
      tok = profile_begin(st);
      rc = conv3_gemm(L.gc_gm, skip, nullptr, L.Fout, L.Cout, bufA, L.Cout, 0);
      if (rc) return rc;
      profile_end(tok, st, SESA_KCLASS_TOKGEMM, 2.0 * B * L.Fout * T * L.Cout * L.Cout * 9, conv3_bytes);
      cur = bufA;
      continue;
    }
    {  // globalconv (3x3) -> bufA
      C3Args a{};
      a.A = skip;
      a.F = L.Fout;
      a.T = T;
      a.Cin = L.Cout;
      a.W = Wb + L.gc_w;
      a.bias = Wb + L.gc_b;
      a.ncols = L.Cout;
      a.out = bufA;
      a.c_store = L.Cout;
      dim3 grid((unsigned)(((T + kC3T - 1) / kC3T) * ((L.Fout + kC3F - 1) / kC3F)), (unsigned)((L.Cout + kC3N - 1) / kC3N),
                (unsigned)B);
      hipLaunchKernelGGL(scn_conv3x3_kernel, grid, dim3(kST), 0, st, a);
      SESA_CHECK_LAUNCH();
      fl += 2.0 * B * L.Fout * T * L.Cout * L.Cout * 9;
      by += 8.0 * B * L.Fout * T * L.Cout;
    }
    profile_end(tok, st, SESA_KCLASS_SIMT, fl, by);
    cur = bufA;
  }
  // 3. separation net (separation.py:107-113): X in bufA, [B][Fn][T][d]
  const int Fn = m->lv[m->nl - 1].Fout;
  float* X = bufA;
  float* Y = bufB;
  float* G = F32(pl.G);
  float* HO = F32(pl.HO);
  double* stats = reinterpret_cast<double*>(ws + pl.stats);
  for (size_t i = 0; i < m->dp.size(); ++i) {
    const DpLayer& L = m->dp[i];
    const int Tc = (i % 2) ? K : T;  // frames (even layers) or rfft bins (odd layers)
    const int d = L.d, H = L.H;
    const int64_t rows = (int64_t)B * Fn * Tc;
    const int64_t n_item = (int64_t)Fn * Tc * d;
    SESA_REQUIRE(rows < (1ll << 31), SESA_ERR_INVALID, "scnet forward: batch too large");
    for (int path = 0; path < 2; ++path) {
      // GroupNorm(1, d) -> bufN
      void* tok = profile_begin(st);
      SESA_CHECK_HIP(hipMemsetAsync(stats, 0, (size_t)B * 2 * sizeof(double), st));
      const unsigned gb = (unsigned)std::min<int64_t>((n_item + kST * 8 - 1) / (kST * 8), 512);
      hipLaunchKernelGGL(scn_gn_stats_kernel, dim3(gb, B), dim3(kST), 0, st, X, n_item, stats);
      SESA_CHECK_LAUNCH();
      // fp16mix with the fp16 recurrence: the dual-path chain in fp16 planes -- GroupNorm -> fp16 A plane, input
      // projection -> fp16 gate plane (LDS-DMA kernel, split epilogue), recurrence -> fp16 h plane, Linear from it
      const int p16m = f16mix ? L.p16 : 0;
      const bool p16 = p16m > 0;
      uint16_t* N16 = reinterpret_cast<uint16_t*>(bufN);
      uint16_t* G16 = reinterpret_cast<uint16_t*>(G);
      uint16_t* HO16 = reinterpret_cast<uint16_t*>(HO);
      if (p16)
        hipLaunchKernelGGL(scn_gn_apply_f16_kernel, blocks(B * n_item / 4), dim3(kST), 0, st, X, n_item, d, stats,
                           Wb + L.gn_g[path], Wb + L.gn_b[path], N16, (int64_t)B * n_item / 4);
      else
        hipLaunchKernelGGL(scn_gn_apply_kernel, blocks(B * n_item), dim3(kST), 0, st, X, n_item, d, stats,
                           Wb + L.gn_g[path], Wb + L.gn_b[path], bufN, (int64_t)B * n_item);
      SESA_CHECK_LAUNCH();
      profile_end(tok, st, SESA_KCLASS_ACT, (p16 ? 10.0 : 12.0) * B * n_item);
      // input projection, both directions: G = XN W_ih^T + (b_ih + b_hh)
      {
        TokGemmArgs a{};
        a.x = bufN;
        a.x_ld = d;
        a.out = G;
        a.o_ld = 8 * H;
        if (p16) {
          a.a_hi = N16;
          a.a_ld = d;
          a.out = nullptr;
          a.out_hi = G16;
          a.k8 = L.ih[path].k8;
          a.n4 = L.ih[path].n4;
        }
        a.w = m->d_w;
        a.bias = m->d_bias;
        a.groups = L.ih[path].d_groups;
        a.n_groups = 1;
        a.n_tiles_n = L.ih[path].n_tiles_n;
        a.M = (int)rows;
        a.act = TOK_ACT_NONE;
        void* t0 = profile_begin(st);
        rc = launch_tok_gemm(a, gx, st);
        profile_end(t0, st, SESA_KCLASS_TOKGEMM, gemm_flops(L.ih[path], rows), tok_gemm_bytes(a, L.ih[path], gx));
        if (rc) return rc;
      }
      // recurrence: path 0 = frequency path, sequences (b, t) over f; path 1 = time path, (b, f) over t
      {
        LstmArgs a{};
        a.G = G;
        a.g_ld = 8 * H;
        a.HO = HO;
        a.ho_ld = 2 * H;
        a.Wt = Wb + L.whh[path];
        a.H = H;
        if (p16) a.G16 = G16;
        if (p16m == 2) a.HO16 = HO16;
        if (path == 0) {
          a.L = Fn;
          a.n_seq = B * Tc;
          a.sdiv = Tc;
          a.smul_a = (int64_t)Fn * Tc;
          a.smul_b = 1;
          a.pstride = Tc;
        } else {
          a.L = Tc;
          a.n_seq = B * Fn;
          a.sdiv = Fn;
          a.smul_a = (int64_t)Fn * Tc;
          a.smul_b = Tc;
          a.pstride = 1;
        }
        void* t0 = profile_begin(st);
        if (lstm_mfma_on(H)) {
          const int ps = L.whh_frag16[path] >= 0 ? scn_lstm_passes() : 3;
          launch_lstm_mfma(a, m->d_w + (ps < 3 ? L.whh_frag16[path] : L.whh_frag[path]), ps, st);
        }
        else launch_lstm(a, st);
        SESA_CHECK_LAUNCH();
        // bytes: the input-projection gates read once, the hidden outputs written once (W_hh stays on chip)
        profile_end(t0, st, SESA_KCLASS_LSTM, 2.0 * rows * 2 * 4 * H * (double)H,
                    rows * ((p16 ? 2.0 : 4.0) * 8.0 * H + (p16m == 2 ? 2.0 : 4.0) * 2.0 * H));
      }
      // Linear(2H -> d) + residual, in place
      {
        TokGemmArgs a{};
        a.x = HO;
        a.x_ld = 2 * H;
        a.out = X;
        a.o_ld = d;
        a.residual = X;
        if (p16m == 2) {
          a.a_hi = HO16;
          a.a_ld = 2 * H;
          a.k8 = L.lin[path].k8;
          a.n4 = L.lin[path].n4;
        }
        a.w = m->d_w;
        a.bias = m->d_bias;
        a.groups = L.lin[path].d_groups;
        a.n_groups = 1;
        a.n_tiles_n = L.lin[path].n_tiles_n;
        a.M = (int)rows;
        a.act = TOK_ACT_NONE;
        void* t0 = profile_begin(st);
        rc = launch_tok_gemm(a, gx, st);
        profile_end(t0, st, SESA_KCLASS_TOKGEMM, gemm_flops(L.lin[path], rows), tok_gemm_bytes(a, L.lin[path], gx));
        if (rc) return rc;
      }
    }
    // FeatureConversion
    void* tok = profile_begin(st);
    const float scale = (float)(1.0 / std::sqrt((double)T));
    // (the MFMA form stages a whole sequence's columns in LDS: past ~1270 frames even the one-block stage exceeds the
    // 160 KiB, so such long chunks keep the VALU DFTs)
    if (scn_dft_mfma() && dft_lds_bytes(1, m->dft_ks[i % 2]) <= 160 * 1024) {
      const int dir = i % 2, Ch = d / 2;
      DftArgs a{};
      a.in = X;
      a.D = m->d_dft + m->dft_off[dir];
      a.MT = m->dft_mt[dir];
      a.KS = m->dft_ks[dir];
      a.out = Y;
      if (dir == 0) {  // X [R][T][d] -> Y [R][K][2d]
        a.in_rs = (int64_t)T * d;
        a.KK = T, a.Kh = T, a.ld = d, a.off2 = 0, a.N = d;
        a.Mtot = 2 * K, a.Mh = K, a.old = 2 * d, a.ooff2 = d;
        a.out_rs = (int64_t)K * 2 * d;
      } else {         // Y [R][K][2 Ch] -> X [R][T][Ch]
        a.in_rs = (int64_t)K * 2 * Ch;
        a.KK = 2 * K, a.Kh = K, a.ld = 2 * Ch, a.off2 = Ch, a.N = Ch;
        a.Mtot = T, a.Mh = T, a.old = Ch, a.ooff2 = 0;
        a.out_rs = (int64_t)T * Ch;
      }
      SESA_REQUIRE(16 * a.KS >= a.KK && 32 * a.MT >= a.Mtot, SESA_ERR_INVALID, "scnet: DFT matrix geometry");
      const bool wide = dft_lds_bytes(2, a.KS) <= 160 * 1024;
      const int nb = wide ? 64 : 32;
      dim3 grid((unsigned)((a.N + nb - 1) / nb), (unsigned)(B * Fn));
      if (wide)
        hipLaunchKernelGGL(scn_dft_mfma_kernel<2>, grid, dim3(64 * kDftWaves), dft_lds_bytes(2, a.KS), st, a);
      else
        hipLaunchKernelGGL(scn_dft_mfma_kernel<1>, grid, dim3(64 * kDftWaves), dft_lds_bytes(1, a.KS), st, a);
      SESA_CHECK_LAUNCH();
      // flops: the dense GEMM the matrix cores run (one pass); bytes: activations read once, written once
      profile_end(tok, st, SESA_KCLASS_DFT, 2.0 * B * Fn * (double)a.Mtot * a.KK * a.N,
                  4.0 * B * Fn * ((double)a.KK * a.N + (double)a.Mtot * a.N));
      std::swap(X, Y);
      continue;
    }
    if (i % 2 == 0) {
      dim3 grid((unsigned)((K + 31) / 32), (unsigned)((d + 63) / 64), (unsigned)(B * Fn));
      hipLaunchKernelGGL(scn_rfft_kernel, grid, dim3(kST), 0, st, X, T, d, m->d_twT, scale, Y);
    } else {
      const int Ch = d / 2;
      dim3 grid((unsigned)((T + 31) / 32), (unsigned)((Ch + 63) / 64), (unsigned)(B * Fn));
      hipLaunchKernelGGL(scn_irfft_kernel, grid, dim3(kST), 0, st, X, K, Ch, m->d_twT, scale, Y);
    }
    SESA_CHECK_LAUNCH();
    // bytes: the layer's activations read once and the converted ones written once
    profile_end(tok, st, SESA_KCLASS_SIMT, 4.0 * B * Fn * (double)K * T * (i % 2 ? d / 2 : d),
                4.0 * B * Fn * ((double)T * d + (double)K * d));
    std::swap(X, Y);
  }
  // 4. decoder (scnet.py:363-366): X [B][F_{i+1}][T][C_{i+1}] -> [B][F_i][T][Cdec_i]
  for (int j = 0; j < m->nl; ++j) {
    const Level& L = m->lv[m->nl - 1 - j];
    void* tok = profile_begin(st);
    double fl = 0;
    // simt bytes: the band transposed convs read the fused level once and write the level output once
    double by = 4.0 * B * T * ((double)L.Fout * L.Cout + (double)L.Fin * L.Cdec);
    if (scn_conv3_mfma()) {  // FusionLayer: x + skip on load, 3x3 C -> 2C, GLU
      rc = conv3_gemm(L.fu_gm, X, F32(pl.skip[m->nl - 1 - j]), L.Fout, L.Cout, Y, L.Cout, 1);
      if (rc) return rc;
      profile_end(tok, st, SESA_KCLASS_TOKGEMM, 2.0 * B * L.Fout * T * 2.0 * L.Cout * L.Cout * 9, conv3_bytes);
      tok = profile_begin(st);
    } else {
    C3Args a{};
    a.A = X;
    a.S = F32(pl.skip[m->nl - 1 - j]);
    a.F = L.Fout;
    a.T = T;
    a.Cin = L.Cout;
    a.W = Wb + L.fu_w;
    a.bias = Wb + L.fu_b;
    a.ncols = 2 * L.Cout;
    a.out = Y;
    a.c_store = L.Cout;
    a.glu = 1;
    dim3 grid((unsigned)(((T + kC3T - 1) / kC3T) * ((L.Fout + kC3F - 1) / kC3F)), (unsigned)((2 * L.Cout + kC3N - 1) / kC3N),
              (unsigned)B);
    hipLaunchKernelGGL(scn_conv3x3_kernel, grid, dim3(kST), 0, st, a);
    SESA_CHECK_LAUNCH();
    fl = 2.0 * B * L.Fout * T * 2.0 * L.Cout * 2.0 * L.Cout * 9;
    by += 12.0 * B * L.Fout * T * L.Cout;
    }
    if (scn_band_mfma() && L.su_mm[0] && L.su_mm[1] && L.su_mm[2]) {  // the band transposed convs on MFMA
      if (!scn_conv3_mfma()) {
        profile_end(tok, st, SESA_KCLASS_SIMT, fl, by - 4.0 * B * T * ((double)L.Fout * L.Cout + (double)L.Fin * L.Cdec));
        tok = profile_begin(st);
      }
      double gfl = 0, gby = 0;
      for (int b = 0; b < 3 && !rc; ++b) rc = band_gemm(L.su_gm[b], L.su_geo[b], Y, X, L.Cdec, &gfl, &gby);
      if (rc) return rc;
      profile_end(tok, st, SESA_KCLASS_TOKGEMM, gfl, gby);
      continue;
    }
    for (int b = 0; b < 3; ++b) {
      const BandConv& bc = L.su[b];
      const int64_t total = (int64_t)B * bc.n_out * T * (L.Cdec / 4);
      hipLaunchKernelGGL(scn_convtr_kernel, blocks(total), dim3(kST), 0, st, Y, L.Fout, T, L.Cout, Wb + L.su_w[b],
                         Wb + L.su_b[b], bc, X, L.Fin, L.Cdec, total);
      SESA_CHECK_LAUNCH();
      fl += 2.0 * total * 4 * L.Cout * ((bc.kern + bc.stride - 1) / bc.stride);
    }
    profile_end(tok, st, SESA_KCLASS_SIMT, fl, by);
  }
  // 5. iSTFT (scnet.py:367-373)
  {
    void* tok = profile_begin(st);
    float* FR = F32(pl.frames);
    const float scale = c.normalized ? 2.0f / 64.0f : 2.0f / (float)kSN;
    const Level& L0 = m->lv[0];   // frame-major when the level-0 band transposed convs ran on MFMA
    const int fmajor = scn_band_mfma() && L0.su_mm[0] && L0.su_mm[1] && L0.su_mm[2] ? 1 : 0;
    hipLaunchKernelGGL(scn_istft_frames_kernel, dim3((unsigned)(T * B * m->nsig)), dim3(kST), 0, st, X, m->nsig, T,
                       fmajor, scale, tb, FR);
    SESA_CHECK_LAUNCH();
    hipLaunchKernelGGL(scn_istft_ola_kernel, dim3((c.chunk_size + kST - 1) / kST, B * m->nsig), dim3(kST), 0, st, FR, T,
                       c.hop_size, c.chunk_size, out);
    SESA_CHECK_LAUNCH();
    profile_end(tok, st, SESA_KCLASS_ISTFT, 4.0 * B * m->nsig * ((double)T * F0 * 2 + (double)c.chunk_size));
  }
  return SESA_OK;
}

extern "C" int sesa_scnet_destroy(sesa_scnet* m) {
  if (!m) return SESA_OK;
  for (void* p : {(void*)m->d_f32, (void*)m->d_w, (void*)m->d_bias, (void*)m->d_twT, (void*)m->d_dft})
    if (p) (void)hipFree(p);
  for (auto& L : m->dp)
    for (int l = 0; l < 2; ++l) {
      if (L.ih[l].d_groups) (void)hipFree(L.ih[l].d_groups);
      if (L.lin[l].d_groups) (void)hipFree(L.lin[l].d_groups);
    }
  for (auto& L : m->lv) {
    for (Gemm* g : {&L.gc_gm, &L.fu_gm})
      if (g->d_groups) (void)hipFree(g->d_groups);
    for (int b = 0; b < 3; ++b)
      for (Gemm* g : {&L.sd_gm[b], &L.su_gm[b]})
        if (g->d_groups) (void)hipFree(g->d_groups);
  }
  delete m;
  return SESA_OK;
}
