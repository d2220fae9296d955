// Chunker + windowed overlap-add on the device (gfx950).
//
// Reference: inference_pytorch.py:55-186 (demix_pytorch_optimized), identical to the generic
// mode of utils.py:330-477.  The reference keeps `result`/`counter` on the host and does a
// blocking D2H per chunk; here both stay resident in HBM for the whole track and the host only
// issues launches.  Summation order and fp32 rounding (multiply, then add; no FMA contraction)
// are kept so that, given identical model outputs, the stems are bit-identical to the reference.
//
// All three kernels are HBM-bound streaming kernels (grid-stride, 4-byte coalesced lanes):
//   gather:     reads 2*C*4 B, writes 2*C*4 B per chunk
//   accumulate: per covered sample reads y (n_out_ch*4 B per covering chunk) + RMW result/counter
//   finalize:   reads n_out_ch*4 + 4 B, writes n_out_ch*4 B per output sample
#include <hip/hip_runtime.h>

#include <cfloat>
#include <vector>

#include "sesa_common.hpp"
#include "sesa_internal.hpp"

namespace sesa {
namespace {

constexpr int kMaxChunks = 64;  // chunks per launch (one batch); the host splits larger plans

struct ChunkTable {
  int64_t start[kMaxChunks];
  int64_t seg[kMaxChunks];
};

// reflect index into [0, n) (torch/numpy 'reflect': edge not repeated)
__device__ __forceinline__ int64_t reflect_idx(int64_t p, int64_t n) {
  if (p < 0) p = -p;
  if (p >= n) p = 2 * (n - 1) - p;
  return p;
}

__global__ void chunk_gather_kernel(const float* __restrict__ mix, int n_ch, int64_t L, int64_t border,
                                    int64_t L_pad, ChunkTable tab, int n_chunks, int chunk,
                                    int tail_constant, float* __restrict__ out) {
  const int j = blockIdx.y;  // chunk
  const int64_t s = tab.start[j];
  const int64_t seg = tab.seg[j];  // valid length inside the padded mix (<= chunk)
  const bool reflect_tail = !tail_constant && seg > chunk / 2;  // demucs mode: always 'constant'
  for (int c = 0; c < n_ch; ++c) {
    const float* src = mix + (int64_t)c * L;
    float* dst = out + ((int64_t)j * n_ch + c) * chunk;
    for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < chunk; q += (int64_t)gridDim.x * blockDim.x) {
      int64_t qq = q;
      float v = 0.f;
      bool valid = true;
      if (q >= seg) {
        if (reflect_tail) qq = 2 * (seg - 1) - q;   // F.pad(part, (0, C-len), 'reflect')
        else valid = false;                          // 'constant' zeros
      }
      if (valid) {
        const int64_t p = s + qq;                    // padded coordinate
        const int64_t o = border > 0 ? reflect_idx(p - border, L) : p;
        v = src[o];
      }
      dst[q] = v;
    }
  }
}

__global__ void ola_accumulate_kernel(const float* __restrict__ y, int n_chunks, int n_out_ch, int chunk,
                                      ChunkTable tab, int64_t span_lo, int64_t span_len,
                                      const float* __restrict__ window, float* __restrict__ result,
                                      float* __restrict__ counter, int64_t L_pad) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < span_len;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t n = span_lo + i;
    float cnt = counter[n];
    for (int j = 0; j < n_chunks; ++j) {  // chunk order == reference loop order (:157)
      const int64_t off = n - tab.start[j];
      if (off < 0 || off >= tab.seg[j]) continue;
      const float w = window[off];
      cnt = __fadd_rn(cnt, w);
    }
    counter[n] = cnt;
    for (int c = 0; c < n_out_ch; ++c) {
      float r = result[(int64_t)c * L_pad + n];
      for (int j = 0; j < n_chunks; ++j) {
        const int64_t off = n - tab.start[j];
        if (off < 0 || off >= tab.seg[j]) continue;
        // the reference rounds y*w to fp32 before the += : keep the product out of an FMA
        float prod = y[((int64_t)j * n_out_ch + c) * chunk + off] * window[off];
        asm volatile("" : "+v"(prod));
        r = r + prod;
      }
      result[(int64_t)c * L_pad + n] = r;
    }
  }
}

__global__ void ola_finalize_kernel(const float* __restrict__ result, const float* __restrict__ counter,
                                    int n_out_ch, int64_t L_pad, int64_t border, int64_t L_out,
                                    float* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < L_out; i += (int64_t)gridDim.x * blockDim.x) {
    const float cnt = counter[border + i];
    for (int c = 0; c < n_out_ch; ++c) {
      float v = __fdiv_rn(result[(int64_t)c * L_pad + border + i], cnt);
      if (isnan(v)) v = 0.f;                       // np.nan_to_num(nan=0.0)
      else if (isinf(v)) v = v > 0 ? FLT_MAX : -FLT_MAX;
      out[(int64_t)c * L_out + i] = v;
    }
  }
}

int grid_for(int64_t n, int block) {
  int64_t g = (n + block - 1) / block;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace
}  // namespace sesa

using namespace sesa;

namespace {
int chunk_gather(const float* mix, int n_ch, int64_t L, int64_t border, const int64_t* starts, int n_chunks, int chunk,
                 int tail_constant, float* out, void* stream) {
  clear_error();
  SESA_REQUIRE(mix && out && starts && n_ch > 0 && L > 0 && chunk > 0, SESA_ERR_INVALID,
               "sesa_chunk_gather_f32: bad arguments");
  SESA_REQUIRE(border >= 0 && (border == 0 || L > border), SESA_ERR_INVALID,
               "sesa_chunk_gather_f32: reflect pad needs L > border");
  const int64_t L_pad = L + 2 * border;
  for (int base = 0; base < n_chunks; base += kMaxChunks) {
    const int n = n_chunks - base < kMaxChunks ? n_chunks - base : kMaxChunks;
    ChunkTable tab{};
    for (int j = 0; j < n; ++j) {
      const int64_t s = starts[base + j];
      SESA_REQUIRE(s >= 0 && s < L_pad, SESA_ERR_INVALID, "sesa_chunk_gather_f32: start %lld out of range",
                   (long long)s);
      tab.start[j] = s;
      tab.seg[j] = (L_pad - s) < chunk ? (L_pad - s) : chunk;
    }
    dim3 grid((unsigned)grid_for(chunk, 256), (unsigned)n);
    void* tok = profile_begin(as_stream(stream));
    hipLaunchKernelGGL(chunk_gather_kernel, grid, dim3(256), 0, as_stream(stream), mix, n_ch, L, border, L_pad, tab,
                       n, chunk, tail_constant, out + (int64_t)base * n_ch * chunk);
    SESA_CHECK_LAUNCH();
    profile_end(tok, as_stream(stream), SESA_KCLASS_OLA, 8.0 * n * n_ch * (double)chunk);  // read + write
  }
  return SESA_OK;
}
}  // namespace

extern "C" int sesa_chunk_gather_f32(const float* mix, int n_ch, int64_t L, int64_t border, const int64_t* starts,
                                     int n_chunks, int chunk, float* out, void* stream) {
  return chunk_gather(mix, n_ch, L, border, starts, n_chunks, chunk, 0, out, stream);
}

// utils.demix demucs mode (utils.py:371-380, :413-418): no border pad, every short tail zero-padded
extern "C" int sesa_chunk_gather_constant_f32(const float* mix, int n_ch, int64_t L, const int64_t* starts,
                                              int n_chunks, int chunk, float* out, void* stream) {
  return chunk_gather(mix, n_ch, L, 0, starts, n_chunks, chunk, 1, out, stream);
}

extern "C" int sesa_ola_accumulate_f32(const float* y, int n_chunks, int n_out_ch, int chunk, const int64_t* starts,
                                       const int64_t* seg_lens, const float* window, float* result, float* counter,
                                       int64_t L_pad, void* stream) {
  clear_error();
  // n_out_ch == 0 (y / result may be NULL): counter only -- the multi-GPU path recomputes the
  // deterministic counter locally instead of exchanging it
  SESA_REQUIRE(starts && seg_lens && window && counter && n_out_ch >= 0 && chunk > 0 &&
                   (n_out_ch == 0 || (y && result)),
               SESA_ERR_INVALID, "sesa_ola_accumulate_f32: bad arguments");
  // Launch in groups of kMaxChunks; groups are issued in order on one stream, so the per-sample
  // summation order stays the reference's chunk order.
  for (int base = 0; base < n_chunks; base += kMaxChunks) {
    const int n = n_chunks - base < kMaxChunks ? n_chunks - base : kMaxChunks;
    ChunkTable tab{};
    int64_t lo = INT64_MAX, hi = 0;
    for (int j = 0; j < n; ++j) {
      const int64_t s = starts[base + j], sl = seg_lens[base + j];
      SESA_REQUIRE(s >= 0 && sl > 0 && sl <= chunk && s + sl <= L_pad, SESA_ERR_INVALID,
                   "sesa_ola_accumulate_f32: chunk %d [%lld,+%lld) outside [0,%lld)", base + j, (long long)s,
                   (long long)sl, (long long)L_pad);
      tab.start[j] = s;
      tab.seg[j] = sl;
      lo = s < lo ? s : lo;
      hi = s + sl > hi ? s + sl : hi;
    }
    double seg_sum = 0;
    for (int j = 0; j < n; ++j) seg_sum += (double)tab.seg[j];
    void* tok = profile_begin(as_stream(stream));
    hipLaunchKernelGGL(ola_accumulate_kernel, dim3(grid_for(hi - lo, 256)), dim3(256), 0, as_stream(stream),
                       y ? y + (int64_t)base * n_out_ch * chunk : nullptr, n, n_out_ch, chunk, tab, lo, hi - lo, window, result,
                       counter, L_pad);
    SESA_CHECK_LAUNCH();
    // algorithmic bytes: y read once + result / counter span read and written once
    profile_end(tok, as_stream(stream), SESA_KCLASS_OLA, 4.0 * n_out_ch * seg_sum + 8.0 * (n_out_ch + 1) * (double)(hi - lo));
  }
  return SESA_OK;
}

extern "C" int sesa_ola_finalize_f32(const float* result, const float* counter, int n_out_ch, int64_t L_pad,
                                     int64_t border, float* out, void* stream) {
  clear_error();
  SESA_REQUIRE(n_out_ch > 0 && border >= 0 && L_pad >= 2 * border, SESA_ERR_INVALID,
               "sesa_ola_finalize_f32: bad arguments");
  const int64_t L_out = L_pad - 2 * border;
  if (L_out == 0) return SESA_OK;  // empty track (the reference returns empty stems)
  SESA_REQUIRE(result && counter && out, SESA_ERR_INVALID, "sesa_ola_finalize_f32: null pointer");
  void* tok = profile_begin(as_stream(stream));
  hipLaunchKernelGGL(ola_finalize_kernel, dim3(grid_for(L_out, 256)), dim3(256), 0, as_stream(stream), result,
                     counter, n_out_ch, L_pad, border, L_out, out);
  SESA_CHECK_LAUNCH();
  profile_end(tok, as_stream(stream), SESA_KCLASS_OLA, 4.0 * (double)L_out * (2 * n_out_ch + 1));
  return SESA_OK;
}
