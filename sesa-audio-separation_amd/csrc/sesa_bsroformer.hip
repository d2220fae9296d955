// BS-Roformer (band-split RoPE transformer): parameter registry, weight packing, spectral front /
// back end and the forward pass (gfx950).
//
// Reference: models/bs_roformer/bs_roformer.py:327-587 (BSRoformer), :43-310 (RMSNorm,
// FeedForward, Attention, Transformer, BandSplit, MaskEstimator), attend.py:76-95 (SDPA).
// Parameter names / shapes are the reference state_dict keys (incl. the per-layer rotary
// `freqs`, whose values drive the rotary tables), so released checkpoints load by name.
//
// Data layout (all token-major fp32, tokens ordered (b, t, band) = 'b t f d'):
//   spec  [B*T][F*ch*2]      STFT features in the reference's '(f s) c' order (:495-497)
//   X     [B*T*nb][dim]      the residual stream; the time transformer's sequences are the strided
//                            views (b, band) -> t and the freq transformer's (b, t) -> band (:526-543),
//                            consumed in place by the attention kernel (no rearranges)
//   QKV   [tokens][3*inner + heads (pad 4)]  q | k | v | gate logits
//   mask  [stem][B*T][F*ch*2] GLU outputs concatenated over bands (:310)
// Forward per transformer layer: QKV+gates GEMM (RMSNorm + rotary fused) -> attention (gates
// fused) -> to_out GEMM (+x) -> FF1 GEMM (RMSNorm, bias, GELU) -> FF2 GEMM (bias, +x).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "sesa_common.hpp"
#include "sesa_internal.hpp"
#include "sesa_tokgemm.hpp"

namespace sesa {
namespace {

// ---------------------------------------------------------------------------------------------
// Spectral kernels for n_fft = 2048 (1024-point complex radix-4 Stockham + real split),
// torch.stft / torch.istft semantics: center=True, reflect pad, periodic Hann(win = n_fft),
// onesided 1025 bins incl. Nyquist, istft(length = chunk) = OLA / sum(w^2), trimmed.
constexpr int kN = 2048;
constexpr int kH = 1024;  // complex FFT length
constexpr int kFT = 256;  // threads

struct BsrTables {
  float2* tw = nullptr;   // exp(-2 pi i j / 1024), j < 1024
  float2* twN = nullptr;  // exp(-2 pi i k / 2048), k <= 1024
  float* win = nullptr;   // periodic Hann(2048)
};
std::mutex g_mu;
std::vector<BsrTables> g_tabs;

int get_tables(BsrTables* out) {
  int dev = 0;
  SESA_CHECK_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(g_mu);
  if ((int)g_tabs.size() <= dev) g_tabs.resize(dev + 1);
  BsrTables& t = g_tabs[dev];
  if (!t.tw) {
    std::vector<float2> a(kH), b(kH + 1);
    std::vector<float> w(kN);
    for (int j = 0; j < kH; ++j) {
      const double ang = -2.0 * M_PI * j / kH;
      a[j] = make_float2((float)cos(ang), (float)sin(ang));
    }
    for (int k = 0; k <= kH; ++k) {
      const double ang = -2.0 * M_PI * k / kN;
      b[k] = make_float2((float)cos(ang), (float)sin(ang));
    }
    for (int n = 0; n < kN; ++n) w[n] = (float)(0.5 - 0.5 * cos(2.0 * M_PI * n / kN));
    SESA_CHECK_HIP(hipMalloc(&t.tw, kH * sizeof(float2)));
    SESA_CHECK_HIP(hipMalloc(&t.twN, (kH + 1) * sizeof(float2)));
    SESA_CHECK_HIP(hipMalloc(&t.win, kN * sizeof(float)));
    SESA_CHECK_HIP(hipMemcpy(t.tw, a.data(), kH * sizeof(float2), hipMemcpyHostToDevice));
    SESA_CHECK_HIP(hipMemcpy(t.twN, b.data(), (kH + 1) * sizeof(float2), hipMemcpyHostToDevice));
    SESA_CHECK_HIP(hipMemcpy(t.win, w.data(), kN * sizeof(float), hipMemcpyHostToDevice));
  }
  *out = t;
  return SESA_OK;
}

__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cconj(float2 a) { return make_float2(a.x, -a.y); }

template <bool INV>
__device__ float2* fft1024(float2* x, float2* y, const float2* __restrict__ tw) {
  int n = kH, s = 1;
#pragma unroll 1
  for (int stage = 0; stage < 5; ++stage) {
    const int m = n >> 2;
    sesa_sync();
    const int bfly = threadIdx.x;  // 256 butterflies per stage
    const int q = bfly & (s - 1);
    const int p = bfly >> __builtin_ctz(s);
    float2 a = x[q + s * p], b = x[q + s * (p + m)], c = x[q + s * (p + 2 * m)], d = x[q + s * (p + 3 * m)];
    float2 w1 = tw[p * s], w2 = tw[2 * p * s], w3 = tw[3 * p * s];
    if (INV) { w1 = cconj(w1); w2 = cconj(w2); w3 = cconj(w3); }
    const float2 apc = cadd(a, c), amc = csub(a, c), bpd = cadd(b, d), bmd = csub(b, d);
    const float2 jbmd = INV ? make_float2(-bmd.y, bmd.x) : make_float2(bmd.y, -bmd.x);
    y[q + s * (4 * p + 0)] = cadd(apc, bpd);
    y[q + s * (4 * p + 1)] = cmul(w1, cadd(amc, jbmd));
    y[q + s * (4 * p + 2)] = cmul(w2, csub(apc, bpd));
    y[q + s * (4 * p + 3)] = cmul(w3, csub(amc, jbmd));
    float2* t = x; x = y; y = t;
    n = m;
    s <<= 2;
  }
  sesa_sync();
  return x;
}

// x [B][ch][len] -> spec [B][T][F][ch][2], F = 1025 (bs_roformer.py:485-497)
__global__ void __launch_bounds__(kFT) bsr_stft_kernel(const float* __restrict__ x, int ch, int len, int hop,
                                                       int frames, BsrTables tb, float* __restrict__ spec) {
  __shared__ float2 bufA[kH];
  __shared__ float2 bufB[kH];
  const int t = blockIdx.x;
  const int sig = blockIdx.y;  // b * ch + s
  const int b = sig / ch, s = sig - b * ch;
  const float* xs = x + (int64_t)sig * len;
  const int64_t base = (int64_t)t * hop - kN / 2;
  for (int m = threadIdx.x; m < kH; m += kFT) {
    float v[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int n = 2 * m + e;
      int64_t pos = base + n;
      if (pos < 0) pos = -pos;
      if (pos >= len) pos = 2 * (int64_t)(len - 1) - pos;
      v[e] = xs[pos] * tb.win[n];
    }
    bufA[m] = make_float2(v[0], v[1]);
  }
  float2* Z = fft1024<false>(bufA, bufB, tb.tw);
  float* o = spec + ((int64_t)b * frames + t) * (kH + 1) * ch * 2;
  for (int k = threadIdx.x; k <= kH; k += kFT) {
    const float2 zk = Z[k & (kH - 1)];
    const float2 zm = cconj(Z[(kH - k) & (kH - 1)]);
    const float2 E = make_float2(0.5f * (zk.x + zm.x), 0.5f * (zk.y + zm.y));
    const float2 D = csub(zk, zm);
    const float2 O = make_float2(0.5f * D.y, -0.5f * D.x);
    const float2 X = cadd(E, cmul(tb.twN[k], O));
    *reinterpret_cast<float2*>(o + ((int64_t)k * ch + s) * 2) = X;
  }
}

// (spec * mask) -> windowed inverse frames; sig = (b * stems + n) * ch + s  (:560-577)
__global__ void __launch_bounds__(kFT) bsr_istft_frames_kernel(const float* __restrict__ spec,
                                                                const float* __restrict__ mask, int ch, int stems,
                                                                int B, int frames, BsrTables tb,
                                                                float* __restrict__ frame_ws) {
  __shared__ float2 bufA[kH];
  __shared__ float2 bufB[kH + 1];
  const int t = blockIdx.x;
  const int sig = blockIdx.y;
  const int s = sig % ch, bn = sig / ch;
  const int n = bn % stems, b = bn / stems;
  const int64_t row = (int64_t)b * frames + t;
  const int64_t feat = (int64_t)(kH + 1) * ch * 2;
  const float* sp = spec + row * feat;
  const float* mk = mask + ((int64_t)n * B * frames + row) * feat;
  for (int k = threadIdx.x; k <= kH; k += kFT) {
    const float2 X = *reinterpret_cast<const float2*>(sp + ((int64_t)k * ch + s) * 2);
    const float2 Mk = *reinterpret_cast<const float2*>(mk + ((int64_t)k * ch + s) * 2);
    float2 Y = cmul(X, Mk);
    if (k == 0 || k == kH) Y.y = 0.f;  // C2R ignores the imaginary parts of DC and Nyquist
    bufB[k] = Y;
  }
  sesa_sync();
  for (int k = threadIdx.x; k < kH; k += kFT) {
    const float2 xk = bufB[k];
    const float2 xm = cconj(bufB[kH - k]);
    const float2 E = make_float2(0.5f * (xk.x + xm.x), 0.5f * (xk.y + xm.y));
    const float2 w = cconj(tb.twN[k]);
    const float2 D = csub(xk, xm);
    const float2 O = cmul(make_float2(0.5f * D.x, 0.5f * D.y), w);
    bufA[k] = make_float2(E.x - O.y, E.y + O.x);
  }
  sesa_sync();  // bufB is reused as the FFT ping-pong buffer
  float2* z = fft1024<true>(bufA, bufB, tb.tw);
  float* fw = frame_ws + ((int64_t)sig * frames + t) * kN;
  const float scale = 1.0f / (float)kH;
  for (int m = threadIdx.x; m < kH; m += kFT) {
    const float2 v = z[m];
    reinterpret_cast<float2*>(fw)[m] = make_float2(v.x * scale * tb.win[2 * m], v.y * scale * tb.win[2 * m + 1]);
  }
}

__global__ void bsr_istft_ola_kernel(const float* __restrict__ frame_ws, int frames, int hop, int out_len,
                                     const float* __restrict__ win, float* __restrict__ out) {
  const int sig = blockIdx.y;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= out_len) return;
  const int n = j + kN / 2;
  const int t_lo = n - kN + 1 <= 0 ? 0 : (n - kN + hop) / hop;
  int t_hi = n / hop;
  if (t_hi > frames - 1) t_hi = frames - 1;
  const float* fw = frame_ws + (int64_t)sig * frames * kN;
  float acc = 0.f, env = 0.f;
  for (int t = t_lo; t <= t_hi; ++t) {
    const int o = n - t * hop;
    acc += fw[(int64_t)t * kN + o];
    const float w = win[o];
    env += w * w;
  }
  out[(int64_t)sig * out_len + j] = acc / env;
}

// Mel-Band-Roformer helpers (mel_band_roformer.py:522-533, :218, :596-606).
// gather: xg[row][j] = spec[row][gidx[j]]
__global__ void mel_gather_kernel(const float* __restrict__ spec, int feat, const int* __restrict__ gidx, int G,
                                  int64_t rows, float* __restrict__ xg) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * G) return;
  const int64_t r = i / G;
  const int j = (int)(i - r * G);
  xg[i] = spec[r * feat + gidx[j]];
}

// in-place RMSNorm of token rows (Transformer.norm, norm_output=True): one wave per row
__global__ void rownorm_kernel(float* __restrict__ x, int64_t rows, int dim, const float* __restrict__ gamma) {
  const int64_t row = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  float* xr = x + row * dim;
  float ss = 0.f;
  for (int d = lane; d < dim; d += 64) ss += xr[d] * xr[d];
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) ss += __shfl_xor(ss, o);
  const float s = sqrtf((float)dim) / fmaxf(sqrtf(ss), 1e-12f);
  for (int d = lane; d < dim; d += 64) xr[d] = xr[d] * s * gamma[d];
}

// scatter-average: out[row][f] = sum_{j in inv(f)} mg[row][j] / max(|inv(f)|, 1e-8), j ascending
__global__ void mel_scatter_avg_kernel(const float* __restrict__ mg, int G, const int* __restrict__ inv_ptr,
                                       const int* __restrict__ inv_idx, int feat, int64_t rows,
                                       float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * feat) return;
  const int64_t r = i / feat;
  const int f = (int)(i - r * feat);
  const float* src = mg + r * G;
  float acc = 0.f;
  const int b = inv_ptr[f], e = inv_ptr[f + 1];
  for (int k = b; k < e; ++k) acc += src[inv_idx[k]];
  out[i] = acc / fmaxf((float)(e - b), 1e-8f);
}

// ---------------------------------------------------------------------------------------------
struct Param {
  std::string name;
  std::vector<int64_t> shape;
  int64_t numel = 0;
  std::vector<float> host;
  bool set = false;
};

struct Layer {         // one transformer layer (Attention + FeedForward)
  std::string prefix;  // layers.i.j.layers.l
  int time = 1;
  Gemm qkv, out, ff1, ff2;
  int64_t rope_off = 0;  // float2 offset into the rope blob
};

}  // namespace
}  // namespace sesa

struct sesa_bsr {
  sesa_bsr_config cfg;
  std::vector<int> fidx; // mel: gathered (f, s) rows
  std::vector<int> fpb;  // freqs per band
  std::vector<int> dims; // band input dims 2*f*ch
  std::vector<int> offs; // band feature offsets
  int nb = 0, F = 0, T = 0, inner = 0, ff = 0, hidden = 0, qkv_ld = 0, feat = 0;
  int gfeat = 0;          // band-split input width (= feat for BS; gathered width for mel)
  int n_lin = 0;          // Linear layers per mask MLP
  int* d_gidx = nullptr;  // mel: gathered feature -> spectrum feature
  int* d_inv_ptr = nullptr;  // mel: CSR spectrum feature -> gathered features (scatter-average)
  int* d_inv_idx = nullptr;
  float* d_affine = nullptr;                    // mel: per-Transformer output norm gammas
  std::map<std::string, int64_t> norm_off;      // "layers.i.j" -> float offset into d_affine
  std::vector<sesa::Param> params;
  std::map<std::string, int> by_name;
  std::vector<sesa::Layer> layers;
  sesa::Gemm band;
  std::vector<sesa::Gemm> mlp;  // per Linear layer of the mask MLPs, stems * nb groups each
  uint16_t* d_w = nullptr;
  float* d_bias = nullptr;
  float2* d_rope = nullptr;
  bool finalized = false;
};

namespace sesa {
namespace {

int add_param(sesa_bsr* m, const std::string& name, std::vector<int64_t> shape) {
  Param p;
  p.name = name;
  p.shape = shape;
  p.numel = 1;
  for (auto s : shape) p.numel *= s;
  m->by_name[name] = (int)m->params.size();
  m->params.push_back(std::move(p));
  return (int)m->params.size() - 1;
}

const std::vector<float>& P(sesa_bsr* m, const std::string& name) { return m->params[m->by_name.at(name)].host; }


}  // namespace
}  // namespace sesa

using namespace sesa;

extern "C" int sesa_bsr_create(const sesa_bsr_config* cfg, sesa_bsr** out) {
  clear_error();
  SESA_REQUIRE(cfg && out && cfg->freqs_per_bands && cfg->n_bands > 1, SESA_ERR_INVALID, "sesa_bsr_create: bad arguments");
  const sesa_bsr_config& c = *cfg;
  SESA_REQUIRE(c.n_fft == 2048 && c.win_length == 2048, SESA_ERR_INVALID, "bsr: only n_fft = win_length = 2048");
  SESA_REQUIRE(c.hop_length > 0 && c.chunk_size % c.hop_length == 0 && c.chunk_size > c.n_fft / 2, SESA_ERR_INVALID,
               "bsr: chunk_size must be a multiple of hop_length and > n_fft/2");
  SESA_REQUIRE(c.audio_channels == 1 || c.audio_channels == 2, SESA_ERR_INVALID, "bsr: audio_channels 1 or 2");
  SESA_REQUIRE(c.dim_head == 64, SESA_ERR_INVALID, "bsr: dim_head must be 64 (attention kernel)");
  SESA_REQUIRE(c.dim % 4 == 0 && c.heads >= 1 && c.depth >= 1 && c.num_stems >= 1, SESA_ERR_INVALID, "bsr: bad dims");
  SESA_REQUIRE(c.mask_estimator_depth >= 1 && c.mask_estimator_depth <= 4, SESA_ERR_INVALID,
               "bsr: mask_estimator_depth 1..4");
  SESA_REQUIRE(!c.mel || (c.freq_indices && c.n_freq_indices > 0), SESA_ERR_INVALID, "bsr: mel needs freq_indices");
  SESA_REQUIRE(c.mel || c.mask_estimator_depth >= 2, SESA_ERR_INVALID, "bsr: BS-Roformer mask MLP needs depth >= 2");
  SESA_REQUIRE(c.precision == SESA_PREC_BF16X3 || c.precision == SESA_PREC_BF16 || c.precision == SESA_PREC_F16,
               SESA_ERR_INVALID, "bsr: precision");
  sesa_bsr* m = new sesa_bsr();
  m->cfg = c;
  m->fpb.assign(c.freqs_per_bands, c.freqs_per_bands + c.n_bands);
  m->cfg.freqs_per_bands = nullptr;
  if (c.mel) m->fidx.assign(c.freq_indices, c.freq_indices + c.n_freq_indices);
  m->cfg.freq_indices = nullptr;
  m->n_lin = c.mel ? c.mask_estimator_depth + 1 : c.mask_estimator_depth;
  int sum = 0, off = 0;
  for (int f : m->fpb) {
    sum += f;
    m->dims.push_back(2 * f * c.audio_channels);
    m->offs.push_back(off);
    off += 2 * f * c.audio_channels;
  }
  if ((!c.mel && sum != c.n_fft / 2 + 1) || (c.mel && sum * c.audio_channels != c.n_freq_indices)) {
    delete m;
    set_error("bsr: freqs_per_bands sums to %d, expected %d", sum,
              c.mel ? c.n_freq_indices / c.audio_channels : c.n_fft / 2 + 1);
    return SESA_ERR_INVALID;
  }
  for (int v : m->fidx)
    if (v < 0 || v >= (c.n_fft / 2 + 1) * c.audio_channels) {
      delete m;
      set_error("bsr: freq_indices entry %d out of range", v);
      return SESA_ERR_INVALID;
    }
  m->nb = c.n_bands;
  m->F = c.n_fft / 2 + 1;
  m->T = c.chunk_size / c.hop_length + 1;
  m->inner = c.heads * c.dim_head;
  m->ff = c.dim * 4;
  m->hidden = c.dim * c.mlp_expansion_factor;
  m->qkv_ld = (3 * m->inner + c.heads + 3) / 4 * 4;
  m->feat = m->F * c.audio_channels * 2;
  m->gfeat = c.mel ? 2 * c.n_freq_indices : m->feat;
  const int dim = c.dim, inner = m->inner;
  for (int i = 0; i < c.depth; ++i)
    for (int j = 0; j < 2; ++j) {
      const int dep = j == 0 ? c.time_transformer_depth : c.freq_transformer_depth;
      for (int l = 0; l < dep; ++l) {
        const std::string p = "layers." + std::to_string(i) + "." + std::to_string(j) + ".layers." + std::to_string(l);
        add_param(m, p + ".0.rotary_embed.freqs", {c.dim_head / 2});
        add_param(m, p + ".0.norm.gamma", {dim});
        add_param(m, p + ".0.to_qkv.weight", {3 * inner, dim});
        add_param(m, p + ".0.to_gates.weight", {c.heads, dim});
        add_param(m, p + ".0.to_gates.bias", {c.heads});
        add_param(m, p + ".0.to_out.0.weight", {dim, inner});
        add_param(m, p + ".1.net.0.gamma", {dim});
        add_param(m, p + ".1.net.1.weight", {m->ff, dim});
        add_param(m, p + ".1.net.1.bias", {m->ff});
        add_param(m, p + ".1.net.4.weight", {dim, m->ff});
        add_param(m, p + ".1.net.4.bias", {dim});
        Layer L;
        L.prefix = p;
        L.time = j == 0;
        m->layers.push_back(L);
      }
      if (c.mel) add_param(m, "layers." + std::to_string(i) + "." + std::to_string(j) + ".norm.gamma", {dim});
    }
  if (!c.mel) add_param(m, "final_norm.gamma", {dim});
  for (int b = 0; b < m->nb; ++b) {
    const std::string p = "band_split.to_features." + std::to_string(b);
    add_param(m, p + ".0.gamma", {m->dims[b]});
    add_param(m, p + ".1.weight", {dim, m->dims[b]});
    add_param(m, p + ".1.bias", {dim});
  }
  for (int n = 0; n < c.num_stems; ++n)
    for (int b = 0; b < m->nb; ++b) {
      const std::string p = "mask_estimators." + std::to_string(n) + ".to_freqs." + std::to_string(b) + ".0";
      for (int li = 0; li < m->n_lin; ++li) {
        const int in = li == 0 ? dim : m->hidden;
        const int out = li == m->n_lin - 1 ? 2 * m->dims[b] : m->hidden;
        add_param(m, p + "." + std::to_string(2 * li) + ".weight", {out, in});
        add_param(m, p + "." + std::to_string(2 * li) + ".bias", {out});
      }
    }
  *out = m;
  return SESA_OK;
}

extern "C" int sesa_bsr_num_params(const sesa_bsr* m) { return m ? (int)m->params.size() : 0; }

extern "C" int sesa_bsr_param_info(const sesa_bsr* m, int i, const char** name, int64_t* numel) {
  clear_error();
  SESA_REQUIRE(m && i >= 0 && i < (int)m->params.size(), SESA_ERR_INVALID, "bsr param_info: index out of range");
  if (name) *name = m->params[i].name.c_str();
  if (numel) *numel = m->params[i].numel;
  return SESA_OK;
}

extern "C" int sesa_bsr_set_param(sesa_bsr* m, const char* name, const float* host, int64_t numel) {
  clear_error();
  SESA_REQUIRE(m && name && host, SESA_ERR_INVALID, "bsr set_param: null argument");
  auto it = m->by_name.find(name);
  SESA_REQUIRE(it != m->by_name.end(), SESA_ERR_INVALID, "bsr set_param: unknown parameter '%s'", name);
  Param& p = m->params[it->second];
  SESA_REQUIRE(p.numel == numel, SESA_ERR_INVALID, "bsr set_param: '%s' expects %lld elements, got %lld", name,
               (long long)p.numel, (long long)numel);
  p.host.assign(host, host + numel);
  p.set = true;
  m->finalized = false;
  return SESA_OK;
}

extern "C" int sesa_bsr_finalize(sesa_bsr* m, void* stream) {
  clear_error();
  SESA_REQUIRE(m, SESA_ERR_INVALID, "bsr finalize: null model");
  for (auto& p : m->params)
    SESA_REQUIRE(p.set, SESA_ERR_STATE, "bsr finalize: parameter '%s' was never set", p.name.c_str());
  const sesa_bsr_config& c = m->cfg;
  const int dim = c.dim, inner = m->inner;
  std::vector<uint16_t> blob;
  std::vector<float> bias;
  const bool f16p = c.precision == SESA_PREC_F16;  // QKV / out / FF1 / FF2 weight images in fp16 (one-pass Linears)
  std::vector<float2> rope;
  // band split: W' = W diag(gamma) (RMSNorm folded)
  m->band.groups.clear();
  for (int b = 0; b < m->nb; ++b) {
    const std::string p = "band_split.to_features." + std::to_string(b);
    const auto& W = P(m, p + ".1.weight");
    const auto& G = P(m, p + ".0.gamma");
    const auto& Bv = P(m, p + ".1.bias");
    const int K = m->dims[b];
    TokGroup g = pack_group(dim, K, [&](int n, int k) { return W[(int64_t)n * K + k] * G[k]; }, true,
                            [&](int n) { return Bv[n]; }, blob, bias);
    g.x_off = m->offs[b];
    g.o_off = (int64_t)b * dim;
    m->band.groups.push_back(g);
  }
  for (auto& L : m->layers) {
    const std::string& p = L.prefix;
    const auto& Wqkv = P(m, p + ".0.to_qkv.weight");
    const auto& Wg = P(m, p + ".0.to_gates.weight");
    const auto& bg = P(m, p + ".0.to_gates.bias");
    const auto& ga = P(m, p + ".0.norm.gamma");
    const int Nq = 3 * inner + c.heads;
    TokGroup g = pack_group(
        Nq, dim,
        [&](int n, int k) {
          return (n < 3 * inner ? Wqkv[(int64_t)n * dim + k] : Wg[(int64_t)(n - 3 * inner) * dim + k]) * ga[k];
        },
        true, [&](int n) { return n < 3 * inner ? 0.f : bg[n - 3 * inner]; }, blob, bias, f16p);
    g.x_off = 0;
    g.o_off = 0;
    L.qkv.groups = {g};
    const auto& Wo = P(m, p + ".0.to_out.0.weight");
    g = pack_group(dim, inner, [&](int n, int k) { return Wo[(int64_t)n * inner + k]; }, false, [](int) { return 0.f; },
                   blob, bias, f16p);
    g.x_off = g.o_off = 0;
    L.out.groups = {g};
    const auto& W1 = P(m, p + ".1.net.1.weight");
    const auto& b1 = P(m, p + ".1.net.1.bias");
    const auto& gf = P(m, p + ".1.net.0.gamma");
    g = pack_group(m->ff, dim, [&](int n, int k) { return W1[(int64_t)n * dim + k] * gf[k]; }, true,
                   [&](int n) { return b1[n]; }, blob, bias, f16p);
    g.x_off = g.o_off = 0;
    L.ff1.groups = {g};
    const auto& W2 = P(m, p + ".1.net.4.weight");
    const auto& b2 = P(m, p + ".1.net.4.bias");
    const int ffd = m->ff;
    g = pack_group(dim, ffd, [&](int n, int k) { return W2[(int64_t)n * ffd + k]; }, true, [&](int n) { return b2[n]; },
                   blob, bias, f16p);
    g.x_off = g.o_off = 0;
    L.ff2.groups = {g};
    // rotary table from this layer's freqs: angle = fp32(pos * freq) (the library's fp32 einsum)
    const auto& fr = P(m, p + ".0.rotary_embed.freqs");
    const int npos = L.time ? m->T : m->nb;
    L.rope_off = (int64_t)rope.size();
    for (int pos = 0; pos < npos; ++pos)
      for (int i = 0; i < c.dim_head / 2; ++i) {
        const float ang = (float)pos * fr[i];
        rope.push_back(make_float2((float)cos((double)ang), (float)sin((double)ang)));
      }
  }
  // mask estimators: (BS) final RMSNorm gamma folded into every band's first Linear; the last
  // Linear's rows interleaved (a_j, b_j) so the GLU pairs sit in adjacent columns
  const int hid = m->hidden;
  std::vector<float> ones(dim, 1.f);
  const std::vector<float>& gfin = c.mel ? ones : P(m, "final_norm.gamma");
  m->mlp.assign(m->n_lin, Gemm{});
  for (int n = 0; n < c.num_stems; ++n)
    for (int b = 0; b < m->nb; ++b) {
      const std::string p = "mask_estimators." + std::to_string(n) + ".to_freqs." + std::to_string(b) + ".0";
      const int din = m->dims[b];
      for (int li = 0; li < m->n_lin; ++li) {
        const auto& W = P(m, p + "." + std::to_string(2 * li) + ".weight");
        const auto& bv = P(m, p + "." + std::to_string(2 * li) + ".bias");
        const int K = li == 0 ? dim : hid;
        const bool last = li == m->n_lin - 1;
        TokGroup g;
        if (!last) {
          g = pack_group(hid, K, [&](int r, int k) { return W[(int64_t)r * K + k] * (li == 0 ? gfin[k] : 1.f); },
                         true, [&](int r) { return bv[r]; }, blob, bias);
          g.o_off = (int64_t)b * hid;
        } else {
          auto src_row = [din](int r) { return (r & 1) ? din + (r >> 1) : (r >> 1); };
          g = pack_group(2 * din, K, [&](int r, int k) { return W[(int64_t)src_row(r) * K + k]; }, true,
                         [&](int r) { return bv[src_row(r)]; }, blob, bias);
          g.o_off = m->offs[b];
        }
        g.x_off = (int64_t)b * (li == 0 ? dim : hid);
        m->mlp[li].groups.push_back(g);
      }
    }
  if (m->d_w) (void)hipFree(m->d_w);
  if (m->d_bias) (void)hipFree(m->d_bias);
  if (m->d_rope) (void)hipFree(m->d_rope);
  m->d_w = nullptr;
  m->d_bias = nullptr;
  m->d_rope = nullptr;
  SESA_REQUIRE(hipMalloc(&m->d_w, blob.size() * 2) == hipSuccess, SESA_ERR_NOMEM, "bsr finalize: hipMalloc weights");
  SESA_REQUIRE(hipMalloc(&m->d_bias, std::max<size_t>(bias.size(), 1) * 4) == hipSuccess, SESA_ERR_NOMEM,
               "bsr finalize: hipMalloc bias");
  SESA_REQUIRE(hipMalloc(&m->d_rope, std::max<size_t>(rope.size(), 1) * sizeof(float2)) == hipSuccess, SESA_ERR_NOMEM,
               "bsr finalize: hipMalloc rope");
  hipStream_t st = as_stream(stream);
  SESA_CHECK_HIP(hipMemcpyAsync(m->d_w, blob.data(), blob.size() * 2, hipMemcpyHostToDevice, st));
  if (!bias.empty()) SESA_CHECK_HIP(hipMemcpyAsync(m->d_bias, bias.data(), bias.size() * 4, hipMemcpyHostToDevice, st));
  if (!rope.empty())
    SESA_CHECK_HIP(hipMemcpyAsync(m->d_rope, rope.data(), rope.size() * sizeof(float2), hipMemcpyHostToDevice, st));
  SESA_CHECK_HIP(hipStreamSynchronize(st));
  int rc = upload_groups(m->band);
  for (auto& g : m->mlp)
    if (!rc) rc = upload_groups(g);
  if (!rc && c.mel) {
    std::vector<float> aff;
    m->norm_off.clear();
    for (int i = 0; i < c.depth; ++i)
      for (int j = 0; j < 2; ++j) {
        const std::string tp = "layers." + std::to_string(i) + "." + std::to_string(j);
        m->norm_off[tp] = (int64_t)aff.size();
        const auto& gm = P(m, tp + ".norm.gamma");
        aff.insert(aff.end(), gm.begin(), gm.end());
      }
    if (m->d_affine) (void)hipFree(m->d_affine);
    m->d_affine = nullptr;
    SESA_CHECK_HIP(hipMalloc(&m->d_affine, aff.size() * sizeof(float)));
    SESA_CHECK_HIP(hipMemcpy(m->d_affine, aff.data(), aff.size() * sizeof(float), hipMemcpyHostToDevice));
    // gathered feature j -> spectrum feature; CSR inverse for the scatter-average
    std::vector<int> gidx(m->gfeat);
    for (int p2 = 0; p2 < (int)m->fidx.size(); ++p2) {
      gidx[2 * p2] = 2 * m->fidx[p2];
      gidx[2 * p2 + 1] = 2 * m->fidx[p2] + 1;
    }
    std::vector<int> cnt(m->feat + 1, 0), ptr(m->feat + 1, 0), idx(m->gfeat);
    for (int j = 0; j < m->gfeat; ++j) cnt[gidx[j]]++;
    for (int f = 0; f < m->feat; ++f) ptr[f + 1] = ptr[f] + cnt[f];
    std::vector<int> fill(ptr.begin(), ptr.end() - 1);
    for (int j = 0; j < m->gfeat; ++j) idx[fill[gidx[j]]++] = j;  // ascending j per feature
    auto up = [&](int** d, const std::vector<int>& h) -> int {
      if (*d) (void)hipFree(*d);
      SESA_CHECK_HIP(hipMalloc(d, h.size() * sizeof(int)));
      SESA_CHECK_HIP(hipMemcpy(*d, h.data(), h.size() * sizeof(int), hipMemcpyHostToDevice));
      return SESA_OK;
    };
    rc = up(&m->d_gidx, gidx);
    if (!rc) rc = up(&m->d_inv_ptr, ptr);
    if (!rc) rc = up(&m->d_inv_idx, idx);
  }
  for (auto& L : m->layers) {
    if (!rc) rc = upload_groups(L.qkv);
    if (!rc) rc = upload_groups(L.out);
    if (!rc) rc = upload_groups(L.ff1);
    if (!rc) rc = upload_groups(L.ff2);
  }
  if (rc) return rc;
  BsrTables tb;
  rc = get_tables(&tb);
  if (rc) return rc;
  m->finalized = true;
  return SESA_OK;
}

namespace {

struct Plan {
  size_t spec, xg, x, xp, rsc, qkv, ao, h, h2, mask, maskg, frames, total;
};

Plan plan(const sesa_bsr* m, int B) {
  auto al = [](size_t n) { return (n * 4 + 255) & ~(size_t)255; };
  const int64_t tok = (int64_t)B * m->T * m->nb;
  Plan p{};
  size_t off = 0;
  p.spec = off; off += al((size_t)B * m->T * m->feat);
  p.xg = off; off += m->cfg.mel ? al((size_t)B * m->T * m->gfeat) : 0;
  p.x = off; off += al((size_t)tok * m->cfg.dim);
  p.xp = off; off += al((size_t)tok * m->cfg.dim);  // X as bf16 hi / lo planes (2 x 2 B per element)
  p.rsc = off; off += al((size_t)tok);               // RMSNorm row scales of X
  p.qkv = off; off += al((size_t)tok * m->qkv_ld);
  p.ao = off; off += al((size_t)tok * m->inner);
  p.h = off; off += al((size_t)tok * std::max(m->ff, m->hidden));
  p.h2 = off; off += m->n_lin >= 3 ? al((size_t)tok * m->hidden) : 0;
  p.mask = off; off += al((size_t)m->cfg.num_stems * B * m->T * m->feat);
  p.maskg = off; off += m->cfg.mel ? al((size_t)m->cfg.num_stems * B * m->T * m->gfeat) : 0;
  p.frames = off; off += al((size_t)B * m->cfg.num_stems * m->cfg.audio_channels * m->T * kN);
  p.total = off;
  return p;
}

TokGemmArgs gemm_args(const sesa_bsr* m, const Gemm& gm, const float* x, int64_t x_ld, float* out, int64_t o_ld,
                      int M) {
  TokGemmArgs a{};
  a.x = x;
  a.x_ld = x_ld;
  a.out = out;
  a.o_ld = o_ld;
  a.w = m->d_w;
  a.bias = m->d_bias;
  a.groups = gm.d_groups;
  a.n_groups = (int)gm.groups.size();
  a.n_tiles_n = gm.n_tiles_n;
  a.k8 = gm.k8;
  a.n4 = gm.n4;
  a.M = M;
  a.act = TOK_ACT_NONE;
  a.dim_head = m->cfg.dim_head;
  return a;
}

double gemm_flops(const Gemm& gm, int64_t M) {
  double f = 0;
  for (auto& g : gm.groups) f += 2.0 * (double)M * g.N * g.K;
  return f;
}

}  // namespace

extern "C" size_t sesa_bsr_workspace_size(const sesa_bsr* m, int batch) {
  if (!m || batch <= 0) return 0;
  return plan(m, batch).total;
}

extern "C" int sesa_bsr_forward(sesa_bsr* m, const float* x, int B, float* out, void* workspace,
                                size_t workspace_bytes, void* stream) {
  clear_error();
  SESA_REQUIRE(m && x && out && workspace && B > 0, SESA_ERR_INVALID, "bsr forward: bad arguments");
  SESA_REQUIRE(m->finalized, SESA_ERR_STATE, "bsr forward: call sesa_bsr_finalize first");
  const Plan pl = plan(m, B);
  SESA_REQUIRE(workspace_bytes >= pl.total, SESA_ERR_INVALID, "bsr forward: workspace %zu < required %zu",
               workspace_bytes, pl.total);
  const sesa_bsr_config& c = m->cfg;
  hipStream_t st = as_stream(stream);
  char* ws = reinterpret_cast<char*>(workspace);
  float* spec = reinterpret_cast<float*>(ws + pl.spec);
  float* X = reinterpret_cast<float*>(ws + pl.x);
  float* QKV = reinterpret_cast<float*>(ws + pl.qkv);
  float* AO = reinterpret_cast<float*>(ws + pl.ao);
  float* H = reinterpret_cast<float*>(ws + pl.h);
  float* MASK = reinterpret_cast<float*>(ws + pl.mask);
  float* FR = reinterpret_cast<float*>(ws + pl.frames);
  float* XG = reinterpret_cast<float*>(ws + pl.xg);
  float* H2 = reinterpret_cast<float*>(ws + pl.h2);
  float* MASKG = reinterpret_cast<float*>(ws + pl.maskg);
  // SESA_PREC_F16: the QKV / out-projection / FF1 / FF2 Linears one fp16 pass (fp16 A planes, fp16 weight
  // images; tok_gemm x3 = 2) and the attention's QK^T / PV one fp16 pass (attn_f16_kernel); band split and
  // mask MLPs bf16x3
  const bool f16 = c.precision == SESA_PREC_F16;
  const int x3 = c.precision == SESA_PREC_BF16 ? 0 : 1;
  const int ch = c.audio_channels, dim = c.dim;
  const int T = m->T, nb = m->nb;
  const int64_t Mtok = (int64_t)B * T * nb;
  SESA_REQUIRE(Mtok < (1ll << 31), SESA_ERR_INVALID, "bsr forward: batch too large");
  const int M = (int)Mtok;
  BsrTables tb;
  int rc = get_tables(&tb);
  if (rc) return rc;
  // (diagnostics: the input, then the whole workspace after every launch -- sesa_debug_trace_begin)
  debug_trace(st, SESA_KCLASS_STFT, x, (size_t)B * ch * c.chunk_size * 4);
  debug_trace_range(ws, pl.total);

  void* tok = profile_begin(st);
  hipLaunchKernelGGL(bsr_stft_kernel, dim3(T, B * ch), dim3(kFT), 0, st, x, ch, c.chunk_size, c.hop_length, T, tb, spec);
  SESA_CHECK_LAUNCH();
  profile_end(tok, st, SESA_KCLASS_STFT, 4.0 * B * ch * ((double)c.chunk_size + (double)T * m->F * 2));

  auto gemm = [&](const TokGemmArgs& a, const Gemm& gm, int64_t rows, bool h16 = false) {
    if (rc) return;
    void* t0 = profile_begin(st);
    rc = launch_tok_gemm(a, h16 ? 2 : x3, st);
    profile_end(t0, st, SESA_KCLASS_TOKGEMM, gemm_flops(gm, rows), tok_gemm_bytes(a, gm, h16 ? 2 : x3));
  };
  const int64_t rowsBT = (int64_t)B * T;
  const float* bs_in = spec;
  if (c.mel) {  // gather the overlapping mel bands' (f, s, c) features (mel_band_roformer.py:522-528)
    const int64_t n = rowsBT * m->gfeat;
    hipLaunchKernelGGL(mel_gather_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, spec, m->feat,
                       m->d_gidx, m->gfeat, rowsBT, XG);
    SESA_CHECK_LAUNCH();
    bs_in = XG;
  }
  // band split: rows (b, t), groups over bands -> X rows (b, t, band)
  {
    TokGemmArgs a = gemm_args(m, m->band, bs_in, m->gfeat, X, (int64_t)nb * dim, B * T);
    a.rownorm = 1;
    gemm(a, m->band, B * T);
  }
  // Transformer GEMM operands as bf16 planes, split once per producer (not once per N tile):
  // X -> XP (tok_split, + RMSNorm row scales), attention -> AO planes, FF1 epilogue -> H planes.
  uint16_t* XPhi = reinterpret_cast<uint16_t*>(ws + pl.xp);
  uint16_t* XPlo = x3 ? XPhi + Mtok * dim : nullptr;
  float* RSC = reinterpret_cast<float*>(ws + pl.rsc);
  uint16_t* AOhi = reinterpret_cast<uint16_t*>(AO);
  uint16_t* AOlo = x3 ? AOhi + Mtok * m->inner : nullptr;
  uint16_t* Hhi = reinterpret_cast<uint16_t*>(H);
  uint16_t* Hlo = x3 ? Hhi + Mtok * m->ff : nullptr;
  auto split_x = [&]() {
    if (rc) return;
    void* t0 = profile_begin(st);
    rc = f16 ? launch_tok_split_f16(X, dim, Mtok, dim, XPhi, dim, RSC, st)
             : launch_tok_split(X, dim, Mtok, dim, XPhi, XPlo, dim, RSC, st);
    profile_end(t0, st, SESA_KCLASS_ACT, (double)Mtok * dim * (x3 && !f16 ? 8.0 : 6.0) + 4.0 * Mtok);
  };
  auto pre = [&](TokGemmArgs& a, const uint16_t* hi, const uint16_t* lo, int64_t ld) {
    a.x = nullptr;
    a.a_hi = hi;
    a.a_lo = lo;
    a.a_ld = ld;
    a.row_scale = RSC;
  };
  // SESA_BSR_QKV_PLANES=1: q / k / v / gate logits as bf16 planes written by the QKV epilogue (the attention
  // then stages K / V by plain copies).  Off by default: measured same-box on the vocals 4-min track, the
  // fp32 QKV buffer is faster -- 115.3x vs 110.5x real-time, attention 356 vs 410 ms and token GEMMs 1597
  // vs 1634 ms per step, twice each (profiles/r03_bsr_qkv_planes_ab_*.json).
  static const bool qkv_planes = getenv("SESA_BSR_QKV_PLANES") && std::string(getenv("SESA_BSR_QKV_PLANES")) == "1";
  const bool qp = qkv_planes && !f16 && m->qkv_ld % 8 == 0 && c.dim_head % 8 == 0;
  uint16_t* QKVhi = reinterpret_cast<uint16_t*>(QKV);
  uint16_t* QKVlo = x3 ? QKVhi + (int64_t)M * m->qkv_ld : nullptr;
  // fp16: the QKV epilogue writes q / k / v / gate logits as one fp16 plane (the rounding the fp16 attention
  // applies on load, at half the bytes written and read); SESA_BSR_QKV16=0: fp32 rows (A/B)
  static const bool qkv16_on = !(getenv("SESA_BSR_QKV16") && std::string(getenv("SESA_BSR_QKV16")) == "0");
  const bool q16 = f16 && qkv16_on && m->qkv_ld % 4 == 0 && c.dim_head % 8 == 0 && m->inner % 4 == 0;
  for (size_t li = 0; li < m->layers.size(); ++li) {
    const Layer& L = m->layers[li];
    // attention: QKV + gates (RMSNorm, rotary on q/k)
    split_x();
    {
      TokGemmArgs a = gemm_args(m, L.qkv, X, dim, QKV, m->qkv_ld, M);
      pre(a, XPhi, f16 ? XPhi : XPlo, dim);  // (fp16: the kernel stages a second copy it does not read)
      a.rownorm = 1;
      a.rope = m->d_rope + L.rope_off;
      a.rope_cols = 2 * m->inner;
      a.pos_F = nb;
      a.pos_T = T;
      a.pos_time = L.time;
      if (qp) {
        a.out_hi = QKVhi;
        a.out_lo = QKVlo;
      }
      if (q16) a.out_hi = QKVhi;   // one fp16 plane (EP_F16 | EP_ROPE | EP_SPLIT)
      gemm(a, L.qkv, M, f16);
    }
    if (rc) return rc;
    {
      AttnArgs a{};
      a.qkv = QKV;
      a.ld = m->qkv_ld;
      a.k_off = m->inner;
      a.v_off = 2 * m->inner;
      a.g_off = 3 * m->inner;
      a.out = AO;
      a.out_hi = AOhi;
      a.out_lo = f16 ? nullptr : AOlo;
      a.out_f16 = f16;   // fp16: one fp16 plane, the fp16 out-projection's A
      a.o_ld = m->inner;
      if (qp) {
        a.qkv_hi = QKVhi;
        a.qkv_lo = QKVlo;
      }
      if (q16) a.qkv16 = QKVhi;
      a.heads = c.heads;
      if (L.time) {  // sequences (b, band) over t
        a.L = T;
        a.n_seq = B * nb;
        a.sdiv = nb;
        a.smul_a = (int64_t)T * nb;
        a.smul_b = 1;
        a.pstride = nb;
      } else {       // sequences (b, t) over bands
        a.L = nb;
        a.n_seq = B * T;
        a.sdiv = 1;
        a.smul_a = nb;
        a.smul_b = 0;
        a.pstride = 1;
      }
      void* t0 = profile_begin(st);
      rc = launch_attention(a, f16 ? 2 : x3, st);   // fp16: QK^T / PV on one fp16 pass
      profile_end(t0, st, SESA_KCLASS_ATTN, 4.0 * (double)a.n_seq * c.heads * (double)a.L * a.L * c.dim_head,
                  attention_bytes(a, f16 ? 2 : x3));
    }
    {
      TokGemmArgs a = gemm_args(m, L.out, AO, m->inner, X, dim, M);
      pre(a, AOhi, f16 ? AOhi : AOlo, m->inner);
      a.residual = X;
      gemm(a, L.out, M, f16);
    }
    split_x();
    {
      TokGemmArgs a = gemm_args(m, L.ff1, X, dim, H, m->ff, M);
      pre(a, XPhi, f16 ? XPhi : XPlo, dim);
      a.rownorm = 1;
      a.act = TOK_ACT_GELU;
      a.out_hi = Hhi;
      a.out_lo = f16 ? nullptr : Hlo;  // fp16: one plane
      gemm(a, L.ff1, M, f16);
    }
    {
      TokGemmArgs a = gemm_args(m, L.ff2, H, m->ff, X, dim, M);
      pre(a, Hhi, f16 ? Hhi : Hlo, m->ff);
      a.residual = X;
      gemm(a, L.ff2, M, f16);
    }
    if (rc) return rc;
    // Mel: Transformer.norm after the last layer of each (time / freq) transformer (:218, :226)
    const bool stack_end = li + 1 == m->layers.size() || m->layers[li + 1].time != L.time ||
                           m->layers[li + 1].prefix.substr(0, m->layers[li + 1].prefix.find(".layers.")) !=
                               L.prefix.substr(0, L.prefix.find(".layers."));
    if (c.mel && stack_end) {
      const std::string tp = L.prefix.substr(0, L.prefix.find(".layers."));
      hipLaunchKernelGGL(rownorm_kernel, dim3((unsigned)((Mtok + 3) / 4)), dim3(256), 0, st, X, Mtok, dim,
                         m->d_affine + m->norm_off.at(tp));
      SESA_CHECK_LAUNCH();
    }
  }
  // mask estimators, per stem: Linear (+Tanh) x (n_lin - 1), last Linear + GLU.  BS: final RMSNorm
  // folded into the first Linear (rownorm).  Mel: GLU outputs land in the gathered layout and are
  // scatter-averaged onto the spectrum features.
  for (int n = 0; n < c.num_stems && !rc; ++n) {
    const float* hin = X;
    int64_t hin_ld = (int64_t)nb * dim;
    float* hbuf[2] = {H, H2};
    for (int li = 0; li < m->n_lin && !rc; ++li) {
      const Gemm& G = m->mlp[li];
      Gemm gf;
      gf.groups.assign(G.groups.begin() + n * nb, G.groups.begin() + (n + 1) * nb);
      const bool last = li == m->n_lin - 1;
      float* o = last ? (c.mel ? MASKG + (int64_t)n * rowsBT * m->gfeat : MASK + (int64_t)n * rowsBT * m->feat)
                      : hbuf[li & 1];
      const int64_t o_ld = last ? (c.mel ? m->gfeat : m->feat) : (int64_t)nb * m->hidden;
      TokGemmArgs a = gemm_args(m, G, hin, hin_ld, o, o_ld, B * T);
      a.groups = G.d_groups + n * nb;
      a.n_groups = nb;
      if (li == 0 && !c.mel) a.rownorm = 1;
      if (last) a.glu = 1;
      else a.act = TOK_ACT_TANH;
      gemm(a, gf, B * T);
      hin = o;
      hin_ld = o_ld;
    }
    if (c.mel && !rc) {
      const int64_t nn = rowsBT * m->feat;
      hipLaunchKernelGGL(mel_scatter_avg_kernel, dim3((unsigned)((nn + 255) / 256)), dim3(256), 0, st,
                         MASKG + (int64_t)n * rowsBT * m->gfeat, m->gfeat, m->d_inv_ptr, m->d_inv_idx, m->feat, rowsBT,
                         MASK + (int64_t)n * rowsBT * m->feat);
      SESA_CHECK_LAUNCH();
    }
  }
  const int n_sig = B * c.num_stems * ch;
  tok = profile_begin(st);
  hipLaunchKernelGGL(bsr_istft_frames_kernel, dim3(T, n_sig), dim3(kFT), 0, st, spec, MASK, ch, c.num_stems, B, T, tb,
                     FR);
  SESA_CHECK_LAUNCH();
  hipLaunchKernelGGL(bsr_istft_ola_kernel, dim3((c.chunk_size + 255) / 256, n_sig), dim3(256), 0, st, FR, T,
                     c.hop_length, c.chunk_size, tb.win, out);
  SESA_CHECK_LAUNCH();
  profile_end(tok, st, SESA_KCLASS_ISTFT, 4.0 * n_sig * ((double)T * m->F * 4 + 2.0 * T * kN + c.chunk_size));
  debug_trace_range(nullptr, 0);
  debug_trace(st, SESA_KCLASS_ISTFT, out, (size_t)n_sig * c.chunk_size * 4);
  return SESA_OK;
}

extern "C" int sesa_bsr_destroy(sesa_bsr* m) {
  if (!m) return SESA_OK;
  if (m->d_w) (void)hipFree(m->d_w);
  if (m->d_bias) (void)hipFree(m->d_bias);
  if (m->d_rope) (void)hipFree(m->d_rope);
  auto fr = [](Gemm& g) {
    if (g.d_groups) (void)hipFree(g.d_groups);
  };
  fr(m->band);
  for (auto& g : m->mlp) fr(g);
  if (m->d_gidx) (void)hipFree(m->d_gidx);
  if (m->d_inv_ptr) (void)hipFree(m->d_inv_ptr);
  if (m->d_inv_idx) (void)hipFree(m->d_inv_idx);
  if (m->d_affine) (void)hipFree(m->d_affine);
  for (auto& L : m->layers) {
    fr(L.qkv);
    fr(L.out);
    fr(L.ff1);
    fr(L.ff2);
  }
  delete m;
  return SESA_OK;
}
