// Argument blocks for the token-major contraction kernels of the transformer models
// (BS-Roformer, sesa_tokgemm.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstring>
#include <vector>

#include "sesa_common.hpp"

namespace sesa {

constexpr int kTokBM = 256;  // token rows per workgroup tile
constexpr int kTokBN = 128;  // output columns per workgroup tile (= packed weight row block)
constexpr int kTokBK = 32;   // K per staged chunk

enum TokAct : int { TOK_ACT_NONE = 0, TOK_ACT_GELU = 1, TOK_ACT_TANH = 2, TOK_ACT_RELU = 3 };

// One GEMM of a (possibly grouped) launch: out[m, o_off + n] = epi(sum_k x[m, x_off + k] W[n, k]).
struct TokGroup {
  int K, N;        // contraction length; output columns (GLU: pre-GLU columns, interleaved a/b)
  int64_t x_off;   // float offset of the group's A block inside a token row
  int64_t o_off;   // float offset of the group's output block inside an output row
  int64_t w_off;   // uint16 offset of the packed weight [ceil(N/128)][ceil(K/32)][hi,lo][128][32]
  int64_t b_off;   // float offset of the bias (< 0: none)
};

// Implicit-GEMM convolution addressing for tok_gemm (HTDemucs, sesa_htdemucs.hip).  Channels-last
// activations on a per-item 2-D grid: input element (b, i1, i2, c) at x[((b Q1 + i1) Q2 + i2) x_ld + c].
// GEMM row m = (b P1 + i1) P2 + i2 (an output position); K = n_taps * Cin with k = tap * Cin + c;
// tap t reads input position (i1 s1 + d1[t], i2 s2 + d2[t]) (zero outside the grid: conv padding).
// phases > 1: transposed-conv epilogue -- column n = r * (N / phases) + co is written to output row
// (b O1 + i1 phases + r - opad) P2 + i2 when 0 <= i1 phases + r - opad < O1 (1-D along axis 1).
// Sub-range form (SCNet's band convs, sesa_scnet.hip): xq1 > 0 -- the item's input grid is rows
// [x_row0, x_row0 + Q1) of a larger per-item grid of xq1 rows (base (b xq1 + x_row0) instead of b Q1; validity
// still against Q1); oq1 > 0 -- output row i1' (i1 itself, or the transposed row above) of item b lands at
// (b oq1 + o_row0 + i1') P2 + i2 (validity against O1, = P1 when phases == 1); with o_fmajor the output is
// axis-2-major instead, (b P2 + i2) oq1 + o_row0 + i1' (SCNet's last band convs write the frame-major spectrum the
// iSTFT reads).
constexpr int kMaxTaps = 16;
struct ConvGeo {
  int P1, P2, Q1, Q2, s1, s2;
  int Cin, n_taps;
  int d1[kMaxTaps], d2[kMaxTaps];
  const float* x2;            // nullable: A = x + x2 (same layout; the decoder's x + skip)
  int phases, O1, opad;
  int xq1, x_row0, oq1, o_row0;
  int o_fmajor;
};

struct TokGemmArgs {
  const float* x;
  int64_t x_ld;               // floats between consecutive token rows of x
  float* out;
  int64_t o_ld;
  const float* residual;      // nullable, out's layout (may alias out): added after the epilogue
  const uint16_t* w;
  const float* bias;
  const TokGroup* groups;     // device table [n_groups]
  int n_groups, n_tiles_n;    // n_tiles_n = max over groups of ceil(N / kTokBN)
  int M;                      // token rows
  int rownorm;                // RMSNorm over the group's K: scale sqrt(K) / max(||x||_2, 1e-12)
                              // (F.normalize * sqrt(dim); gamma is folded into W at pack time)
  int act;                    // TokAct
  int glu;                    // out col j = a_j * sigmoid(b_j), (a_j, b_j) = pre-GLU cols (2j, 2j+1)
  const float2* rope;         // rotary (cos, sin) table [n_pos][dim_head / 2], nullable
  int rope_cols;              // columns [0, rope_cols) are rotated (q and k)
  int dim_head;
  int pos_F, pos_T, pos_time; // rotary position of row m: pos_time ? (m / pos_F) % pos_T : m % pos_F
  int conv;                   // 1: A rows / output rows addressed through `geo` (implicit-GEMM conv)
  ConvGeo geo;
  // Pre-split A (not with conv): A[m, k] = a_hi + a_lo as bf16 planes [M][a_ld] (tok_split or a split
  // epilogue wrote them once), so the kernel stages them without per-N-tile fp32 -> hi/lo work.
  // a_lo may be null for one-pass bf16.  With rownorm the row scales come from row_scale[M].  On this
  // path every group's o_off % 4 == 0 (the residual is staged in 16-B pieces).
  const uint16_t* a_hi;
  const uint16_t* a_lo;
  int64_t a_ld;
  const float* row_scale;
  int k8;                     // every group's K % 8 == 0 (Gemm::k8): pre-split A may take the LDS-DMA kernel
  int n4;                     // every group's N % 4 == 0 and o_off % 4 == 0 (Gemm::n4): the LDS-DMA
                              // kernel's residual epilogue stages 16-B pieces and needs it
  // Split epilogue: write bf16 planes out_hi / out_lo [.][o_ld] instead of fp32 `out` (the result
  // only feeds another tok_gemm; no residual).  out_lo may be null (bf16).
  uint16_t* out_hi;
  uint16_t* out_lo;
  // conv mode: 64-column tiles (n_tiles_n then counts ceil(N / 64)) for narrow convolutions
  int bn64;
  // persistent launch (tok_gemm_glds_kernel<PERS>, set by launch_tok_gemm): tiles of the full grid, and the delay of
  // the second half of the workgroups in units of s_sleep(127)
  int pers_tiles;
  int stagger;
};

// Split fp32 rows into bf16 planes for tok_gemm's pre-split A: hi = bf16(x), lo = bf16(x - hi),
// row m of x (x_ld floats) -> row m of the planes (p_ld elements); K % 4 == 0.  row_scale (nullable)
// gets sqrt(K) / max(||x_m||_2, 1e-12) (the RMSNorm scale of rownorm).  lo null: hi only.
int launch_tok_split(const float* x, int64_t x_ld, int64_t M, int K, uint16_t* hi, uint16_t* lo, int64_t p_ld,
                     float* row_scale, hipStream_t st);
// the same rows as ONE fp16 plane (round to nearest even): A of the fp16 single-pass Linears (tok_gemm x3 = 2)
int launch_tok_split_f16(const float* x, int64_t x_ld, int64_t M, int K, uint16_t* hi, int64_t p_ld, float* row_scale,
                         hipStream_t st);

// Flash attention over strided sequences of a token-major qkv buffer.
// token(seq, p) = (seq / sdiv) * smul_a + (seq % sdiv) * smul_b + p * pstride
struct AttnArgs {
  const float* qkv;
  int64_t ld;                 // qkv row stride (floats)
  int k_off, v_off, g_off;    // column of k / v / gate logits (q at 0); head h adds h * dh (gates: + h);
                              // g_off < 0: no gate (plain SDPA)
  float* out;                 // [token][heads * dh]
  int64_t o_ld;
  int L, n_seq, heads;
  int sdiv;
  int64_t smul_a, smul_b, pstride;
  // cross attention (HTDemucs CrossTransformerEncoderLayer): keys / values from a second buffer
  const float* kv;            // nullable: k / v columns read from kv (else from qkv)
  int64_t kv_ld;
  int Lk;                     // keys per sequence (0: L)
  int64_t kv_smul;            // kv token of (seq, p) = seq * kv_smul + p (when kv != nullptr)
  int dh;                     // head dim, <= 64 and % 4 == 0 (0: 64); scale 1 / sqrt(dh)
  uint16_t* out_hi;           // nullable: write bf16 planes (o_ld) instead of fp32 `out` (pre-split A of
  uint16_t* out_lo;           //   the following to_out tok_gemm); out_lo may be null (bf16)
  // nullable: q / k / v / gate logits as the bf16 hi / lo planes the projection GEMM's split epilogue
  // wrote (same strides and column offsets as qkv / kv); the kernel then stages K / V with plain copies
  // (no fp32 -> hi / lo split per query block) and takes Q from the planes.  *_lo null for bf16.
  const uint16_t* qkv_hi;
  const uint16_t* qkv_lo;
  const uint16_t* kv_hi;
  const uint16_t* kv_lo;
  int out_f16;                // with out_hi: one fp16 plane (the fp16 kernel, x3 == 2; the fp16 out-projection's A)
  // nullable (fp16 kernel, self attention): q / k / v / gate logits as ONE fp16 plane written by the fp16 QKV
  // GEMM's split epilogue (same stride and column offsets as qkv): the values the kernel would round to fp16
  // itself, at half the bytes
  const uint16_t* qkv16;
  const uint16_t* kv16;       // nullable (cross attention with qkv16): k / v as one fp16 plane (kv's layout)
};


// ---- host-side weight packing shared by the token-GEMM users (sesa_bsroformer.hip, sesa_scnet.hip) ----
inline uint16_t f2bf(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7fc0;
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
inline float bf2f(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

struct Gemm {          // one packed (possibly grouped) GEMM
  std::vector<TokGroup> groups;
  TokGroup* d_groups = nullptr;
  int n_tiles_n = 0;
  int k8 = 0;          // every group's K % 8 == 0
  int n4 = 0;          // every group's N % 4 == 0 and o_off % 4 == 0
};

// Pack W[n][k] (row accessor) of an N x K GEMM for one group; returns the TokGroup with w_off/b_off set.
// f16: the image as fp16 hi = fp16(v), lo = fp16(v - hi) (the fp16 single-pass Linears read hi only).
template <class RowFn, class BiasFn>
TokGroup pack_group(int N, int K, RowFn row_val, bool has_bias, BiasFn bias_val, std::vector<uint16_t>& blob,
                    std::vector<float>& bias, bool f16 = false) {
  TokGroup g{};
  g.K = K;
  g.N = N;
  g.w_off = (int64_t)blob.size();
  const int nt = (N + kTokBN - 1) / kTokBN, nch = (K + kTokBK - 1) / kTokBK;
  const int64_t img = (int64_t)kTokBN * kTokBK;
  blob.resize(blob.size() + (size_t)nt * nch * 2 * img, 0);
  uint16_t* base = blob.data() + g.w_off;
  for (int t = 0; t < nt; ++t)
    for (int kc = 0; kc < nch; ++kc) {
      uint16_t* hi = base + ((int64_t)t * nch + kc) * 2 * img;
      uint16_t* lo = hi + img;
      for (int r = 0; r < kTokBN; ++r) {
        const int n = t * kTokBN + r;
        for (int kk = 0; kk < kTokBK; ++kk) {
          const int k = kc * kTokBK + kk;
          const float v = (n < N && k < K) ? row_val(n, k) : 0.f;
          const int64_t o = (int64_t)r * kTokBK + (((kk >> 3) ^ ((r >> 2) & 3)) << 3) + (kk & 7);
          if (f16) {
            const _Float16 hh = (_Float16)v;
            hi[o] = __builtin_bit_cast(uint16_t, hh);
            lo[o] = __builtin_bit_cast(uint16_t, (_Float16)(v - (float)hh));
            continue;
          }
          const uint16_t h = f2bf(v);
          hi[o] = h;
          lo[o] = f2bf(v - bf2f(h));
        }
      }
    }
  g.b_off = -1;
  if (has_bias) {
    g.b_off = (int64_t)bias.size();
    for (int n = 0; n < N; ++n) bias.push_back(bias_val(n));
    while (bias.size() % 4) bias.push_back(0.f);
  }
  return g;
}

inline int upload_groups(Gemm& gm) {
  if (gm.d_groups) (void)hipFree(gm.d_groups);
  SESA_CHECK_HIP(hipMalloc(&gm.d_groups, gm.groups.size() * sizeof(TokGroup)));
  SESA_CHECK_HIP(hipMemcpy(gm.d_groups, gm.groups.data(), gm.groups.size() * sizeof(TokGroup), hipMemcpyHostToDevice));
  gm.n_tiles_n = 0;
  gm.k8 = 1;
  gm.n4 = 1;
  for (auto& g : gm.groups) {
    gm.n_tiles_n = std::max(gm.n_tiles_n, (g.N + kTokBN - 1) / kTokBN);
    if (g.K % 8) gm.k8 = 0;
    if (g.N % 4 || g.o_off % 4) gm.n4 = 0;
  }
  return SESA_OK;
}

int launch_tok_gemm(const TokGemmArgs& a, int x3, hipStream_t st);
int launch_attention(const AttnArgs& a, int x3, hipStream_t st);

// ---- algorithmic HBM bytes (the roofline's HBM floor, sesa_profile_read2) ----
// One tok_gemm launch: A read once in the form the kernel reads it (fp32 rows 4 B; pre-split planes 2 B per plane
// read: fp16 / bf16 single pass one plane, bf16x3 hi + lo), conv mode the input grid once (+ the skip operand), the
// weight image once (bf16x3 hi + lo 4 B per coefficient, else 2 B), the output once (fp32 4 B, or the split
// epilogue's plane(s)) and the residual once.  x3: 0 bf16, 1 bf16x3, 2 fp16 (launch_tok_gemm's argument).
inline double tok_gemm_bytes(const TokGemmArgs& a, const Gemm& gm, int x3) {
  double k_sum = 0, n_out = 0, wcoef = 0;
  const int ng = a.n_groups > 0 ? a.n_groups : (int)gm.groups.size();
  for (int i = 0; i < ng && i < (int)gm.groups.size(); ++i) {
    const TokGroup& g = gm.groups[i];
    k_sum += g.K;
    n_out += a.glu ? g.N / 2 : g.N;
    wcoef += (double)g.N * g.K;
  }
  const double M = a.M;
  double in;
  if (a.conv) {
    const double items = M / ((double)a.geo.P1 * a.geo.P2);
    in = items * a.geo.Q1 * a.geo.Q2 * a.geo.Cin * 4.0 * (a.geo.x2 ? 2.0 : 1.0);
  } else if (a.a_hi) {
    in = M * k_sum * (a.a_lo && x3 == 1 ? 4.0 : 2.0);
  } else {
    in = M * k_sum * 4.0;
  }
  const double w = wcoef * (x3 == 1 ? 4.0 : 2.0);
  const double out = M * n_out * (a.out_hi ? (a.out_lo ? 4.0 : 2.0) : 4.0) + (a.residual ? M * n_out * 4.0 : 0.0);
  return in + w + out;
}

// One attention launch: Q, K, V (and the gate logits) read once in the form the kernel reads them (one fp16 plane
// 2 B, bf16 hi + lo planes 4 B, fp32 rows 4 B), the output written once (fp16 plane 2 B, bf16 planes 4 B, fp32 4 B).
inline double attention_bytes(const AttnArgs& a, int x3) {
  const double dh = a.dh > 0 ? a.dh : 64, heads = a.heads, L = a.L, Lk = a.Lk > 0 ? a.Lk : a.L, ns = a.n_seq;
  const double q_e = a.qkv16 ? 2.0 : a.qkv_hi ? (a.qkv_lo && x3 == 1 ? 4.0 : 2.0) : 4.0;
  const double kv_e = (a.kv ? a.kv16 : a.qkv16) ? 2.0 : (a.kv ? a.kv_hi : a.qkv_hi) ? (x3 == 1 ? 4.0 : 2.0) : 4.0;
  const double o_e = a.out_hi ? (a.out_f16 || x3 != 1 ? 2.0 : 4.0) : 4.0;
  return ns * heads * (L * dh * q_e + 2.0 * Lk * dh * kv_e + L * dh * o_e + (a.g_off >= 0 ? L * q_e : 0.0));
}

}  // namespace sesa
