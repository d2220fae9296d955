// Argument blocks for the MFMA contraction kernels of the MDX23C network (see sesa_tapgemm.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace sesa {

enum SrcMode : int {
  SRC_RAW = 0,        // x
  SRC_NORM_GELU = 1,  // GELU(InstanceNorm_affine(x))   (get_norm + get_act, mdx23c_tfc_tdf_v3.py:47-71)
  SRC_MUL = 2,        // x * mul                         (x * first_conv_out, :230)
  SRC_PRE = 3,        // pre-activated: bf16 hi/lo planes written by act_split (GELU(IN(x)) already applied)
  SRC_ACT32 = 4,      // pre-activated fp32 (launch_act_f32): the input of the Winograd 3x3 kernel
};

// One input source of a (possibly channel-concatenated) NHWC fp32 activation
// [B][T][F][C] -- torch.cat([a, b], 1) is expressed as two sources (:225, :232).
struct Src {
  const float* ptr;
  const double* stats;  // [B][C][2] (sum, sumsq) over T*F, for SRC_NORM_GELU
  const float* mul;     // same layout as ptr, for SRC_MUL
  int C;
  int mode;
  const uint16_t* hi;   // SRC_PRE: bf16 planes, NHWC like ptr
  const uint16_t* lo;
};

struct GemmIn {
  Src src[2];
  int C_split;          // channels [0, C_split) from src[0], the rest from src[1]
  int C_in;
  const float* gamma;   // InstanceNorm affine over the concatenated channels (nullable)
  const float* beta;
  double inv_count;     // 1 / (T_in * F_in)
};

struct GemmOut {
  float* ptr;                // NHWC [B][T_out][F_out][C_out]
  const float* residual;     // nullable, same layout (may alias ptr)
  double* stats;             // nullable, [B][C_out][2] accumulated with atomics
  int C_out;
  int gelu;                  // apply exact GELU to the stored value (final_conv[1], :185)
};

struct ConvArgs {
  GemmIn in;
  GemmOut out;
  const uint16_t* w;         // packed bf16 hi/lo weight image (host packing in sesa_mdx23c.hip)
  int T_in, F_in, T_out, F_out;
  int n_cols;                // GEMM N (C_out, or 4*C_out for the transposed 2x2 conv)
  int n_chunks;              // C_in / 16
  GemmIn xin;                // optional RAW extra input over the centre tap (fused 1x1 shortcut)
  int x_chunks;              // xin.C_in / 16 (0 = none)
};

struct TdfArgs {
  GemmIn in;
  GemmOut out;
  const uint16_t* w;         // packed [M/BM][K/32][BM][32] hi, lo (BM = tdf_block_rows(M))
  int T, K, M;               // F_in = K, F_out = M
  int n_chunks;              // ceil(K / 32)
  int batch;                 // set by launch_tdf
  uint16_t* u_planes;        // second Linear: scratch of tdf_u_floats(..) floats for the pre-split act(U)
                             // B images (nullable: the kernel then converts U itself)
};

// conv kinds
enum ConvKind : int { CONV3X3 = 0, CONV1X1 = 1, CONV2X2S2 = 2, DECONV2X2S2 = 3 };

int launch_conv(int kind, int bn, int x3, const ConvArgs& a, int batch, hipStream_t st);
// act_split: hi/lo[b][pos][c] = split_bf16(GELU(IN_affine(x))) for the (possibly two-source,
// channel-concatenated) input `in` of n_pos positions per batch item.
int launch_act_split(const GemmIn& in, int64_t n_pos, int batch, uint16_t* hi, uint16_t* lo, hipStream_t st,
                     uint16_t* raw_hi = nullptr, uint16_t* raw_lo = nullptr);
// act_f32: out[b][pos][c] = GELU(IN_affine(x)) as fp32 (the SRC_ACT32 input of the Winograd conv).
int launch_act_f32(const GemmIn& in, int64_t n_pos, int batch, float* out, hipStream_t st);
// GELU(InstanceNorm(x)) rounded to fp16 (one plane, NHWC): the A operand of the fp16 TFC 3x3 convs
int launch_act_f16(const GemmIn& in, int64_t n_pos, int batch, uint16_t* out, hipStream_t st);
// True when a same-size TFC 3x3 conv at T_out runs as Winograd F(2, 3) (conv3x3_wino_kernel): its weights
// are then packed by pack_conv_wino (sesa_mdx23c.hip) and its input is given as SRC_ACT32.
bool conv3x3_wino_selected(int T_out, int C_in, int C_out);
int set_conv3x3_wino(int mode);  // 0 off, 1 levels 1-3, 2 every T >= 32 level; returns the previous
// Winograd weight images (uint16 per stage): main stage = 2 points x 3 dy x 64 co x 16 ci, hi + lo;
// shortcut stage = 2 points x 64 x 16, hi + lo.
constexpr int kWinoMainImg = 2 * 6 * 64 * 16;
constexpr int kWinoShortImg = 2 * 2 * 64 * 16;
// True when launch_conv runs a 3x3 same-size conv on conv3x3_m16_kernel, whose fused 1x1 shortcut
// (C_shortcut > 0) must then be given as act_split raw planes (SRC_PRE) instead of a raw fp32 input.
bool conv3x3_m16_selected(int T_out, int C_in, int C_out, int C_shortcut);
// True when a same-size 3x3 conv at T_out with C_in normalised input channels runs conv3x3_db_kernel with
// the InstanceNorm + GELU + split fused into its staging: its input is then given as the raw fp32
// sources (SRC_NORM_GELU) instead of act_split planes.
bool conv3x3_fused_act_ok(int T_out, int C_in, int C_out);
int set_conv3x3_variant(int v);
bool tap_bn128_enabled();  // SESA_TAP_BN128=0 disables the 128-column down / up tiles (A/B)  // 0 = conv3x3_db_kernel, 1 = conv3x3_m16_kernel; returns the previous
int launch_tdf(int x3, const TdfArgs& a, int batch, hipStream_t st, int transposed_io);
int tdf_block_rows(int M);
bool tdf_dma_eligible(int C, int K, int M);
// floats of the tiled U^T buffer [n/128][ceil(M/32)][128][32] for n_cols = B*T*C columns
int64_t tdf_u_floats(int64_t n_cols, int M);  // BM chosen for a TDF Linear with M output rows (weights packed to match)

// Tile geometry shared by the host packer and the kernels.
constexpr int kTF = 32;       // output columns per tile (one MFMA 32-row block = one tile row)
constexpr int kConvBK = 16;   // input channels per K chunk of the tap GEMM
constexpr int kTdfBK = 32;    // TDF K (frequency) per chunk

}  // namespace sesa
