// Argument blocks for the token-major contraction kernels of the transformer models
// (BS-Roformer, sesa_tokgemm.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace sesa {

constexpr int kTokBM = 256;  // token rows per workgroup tile
constexpr int kTokBN = 128;  // output columns per workgroup tile (= packed weight row block)
constexpr int kTokBK = 32;   // K per staged chunk

enum TokAct : int { TOK_ACT_NONE = 0, TOK_ACT_GELU = 1, TOK_ACT_TANH = 2 };

// One GEMM of a (possibly grouped) launch: out[m, o_off + n] = epi(sum_k x[m, x_off + k] W[n, k]).
struct TokGroup {
  int K, N;        // contraction length; output columns (GLU: pre-GLU columns, interleaved a/b)
  int64_t x_off;   // float offset of the group's A block inside a token row
  int64_t o_off;   // float offset of the group's output block inside an output row
  int64_t w_off;   // uint16 offset of the packed weight [ceil(N/128)][ceil(K/32)][hi,lo][128][32]
  int64_t b_off;   // float offset of the bias (< 0: none)
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
};

// Flash attention over strided sequences of a token-major qkv buffer.
// token(seq, p) = (seq / sdiv) * smul_a + (seq % sdiv) * smul_b + p * pstride
struct AttnArgs {
  const float* qkv;
  int64_t ld;                 // qkv row stride (floats)
  int k_off, v_off, g_off;    // column of k / v / gate logits (q at 0); head h adds h * 64 (gates: + h)
  float* out;                 // [token][heads * 64]
  int64_t o_ld;
  int L, n_seq, heads;
  int sdiv;
  int64_t smul_a, smul_b, pstride;
};

int launch_tok_gemm(const TokGemmArgs& a, int x3, hipStream_t st);
int launch_attention(const AttnArgs& a, int x3, hipStream_t st);

}  // namespace sesa
