// Token-major MFMA contractions for the transformer models (BS-Roformer) on gfx950.
//
// tok_gemm_kernel -- Y[m, n] = epi( sum_k X[m, k] * W[n, k] ) for the Linear layers of
//   bs_roformer.py: BandSplit (:222-249, grouped over the 62 bands), Attention.to_qkv + to_gates
//   (:97-99, one GEMM, rotary applied to q/k in the epilogue, :111-113), to_out (:101-104, +
//   residual :214), FeedForward (:55-74, GELU / + residual :215), MaskEstimator MLPs (:277-310,
//   grouped, Tanh and GLU in the epilogues).  RMSNorm (:43-50) is fused: gamma is folded into W at
//   pack time and the row scale sqrt(K)/max(||x||, 1e-12) is applied in the epilogue.
//   Two staging paths: (a) fp32 A rows split to bf16 hi/lo per K chunk in registers and stored to
//   LDS (band split, mask MLPs, implicit-GEMM conv of HTDemucs, SCNet); (b) A pre-split once into
//   bf16 planes by its producer (tok_split / split epilogues) and copied to LDS by LDS-DMA
//   (tok_gemm_glds_kernel: the transformer Linear layers).  Weights arrive pre-split and
//   pre-swizzled; tiles are ordered XCD-major so the N tiles of an M tile share one L2.
//   Precision bf16x3 (hi*hi + hi*lo + lo*hi, fp32 accumulate) or bf16 (one pass).
// attn_kernel -- softmax(Q K^T / sqrt(64)) V per (sequence, head) (attend.py:76-95, SDPA), the
//   flash formulation with S^T = K Q^T so every query owns one lane column: row max / sum are
//   in-lane (+1 shuffle), the O^T accumulator rescale is a per-lane scalar, and P^T feeds the
//   P.V MFMA straight from registers (V^T staged in LDS with the matching key permutation).
//   Sigmoid gates (:117-118) are applied in the epilogue.  Sequences are strided views of the
//   token-major buffer, so the time/freq transformers (:526-543) need no transposes.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <type_traits>

#include "sesa_common.hpp"
#include "sesa_tokgemm.hpp"

namespace sesa {
namespace {

constexpr int kThreads = 256;

template <int I, int N>
struct Unroll {
  template <class F>
  __device__ __forceinline__ static void run(F&& f) {
    f(std::integral_constant<int, I>{});
    Unroll<I + 1, N>::run(f);
  }
};
template <int N>
struct Unroll<N, N> {
  template <class F>
  __device__ __forceinline__ static void run(F&&) {}
};

__device__ __forceinline__ f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ uint32_t pack2(__bf16 a, __bf16 b) {
  return (uint32_t)__builtin_bit_cast(uint16_t, a) | ((uint32_t)__builtin_bit_cast(uint16_t, b) << 16);
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }

// XCD-aware tile order: workgroups are dispatched round-robin over the 8 XCDs (each with its own
// L2), so block b runs on XCD b % 8.  Tile t = (XCD, b / 8) packed XCD-major keeps consecutive tiles
// -- the N tiles of one M tile, which share the A rows -- on one XCD's L2 instead of fetching the A
// rows once per XCD.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ int xcd_tile(int b, int nb) {
  const int q = nb >> 3, r = nb & 7, x = b & 7, i = b >> 3;
  return x * q + min(x, r) + i;
}

// ---------------------------------------------------------------------------------------------
// Register-staged kernel.  NT threads, tile BM tokens x 128 columns, waves of (32 MI) x (32 NI).
// DB = false (default, 256 threads, 2 WG / CU): single LDS stage, two barriers per 32-wide K chunk,
// the next chunk's global loads in flight under the MFMAs.  DB = true (512 threads, 1 WG / CU):
// two stages, one barrier per chunk.  The body is straight-line (clamped addresses, validity
// applied at store time).
// BN: output columns per tile, 128 (the packed weight row block) or 64 (one half of it, for the narrow
// implicit-GEMM convs of HTDemucs: N = 24 / 32 / 48 / 64 fill a 128-column tile to 19-50 %).
// F16 (X3 = false): the A operand rounded once to fp16 and the fp16 weight image (pack_group(..., f16)), one
// v_mfma_f32_32x32x16_f16 pass -- the implicit-GEMM convs of HTDemucs' fp16mix precision.
// PD (single-stage form): register sets for PD chunks, so chunk kc + PD is loading while chunk kc is staged and
// computed (PD = 1: the next chunk only -- its gather latency, not the MFMAs, bounded the narrow HTDemucs convs).
template <bool X3, int NT, int BM, int WN, int MI, int NI, bool DB, bool CONV, bool PRE, int BN = kTokBN,
          bool F16 = false, int PD = 1>
__global__ void __launch_bounds__(NT, DB ? 1 : 2) tok_gemm_kernel(TokGemmArgs a) {
  static_assert(!F16 || (!X3 && !PRE), "fp16: one pass on fp32 rows / conv gathers");
  static_assert(PD >= 1 && (PD == 1 || !DB), "register prefetch depth: single-stage form");
  constexpr int BK = kTokBK;
  static_assert(BN == kTokBN || BN == kTokBN / 2, "tile width");
  static_assert((NT / 64) == (BM / (32 * MI)) * WN && BN == WN * NI * 32, "tile");
  static_assert(!(PRE && CONV), "pre-split A is for token rows");
  constexpr int ROWB = BK * 2;                 // 64 B per image row (32 bf16)
  constexpr int A_BYTES = BM * ROWB;
  constexpr int W_BYTES = BN * ROWB;
  constexpr int STAGE = 2 * A_BYTES + 2 * W_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[(DB ? 2 : 1) * STAGE];
  __shared__ float rs[BM];
  __shared__ int orow_base[CONV ? BM : 1], orow_i1[CONV ? BM : 1];  // transposed-conv output rows
  __shared__ int tap_d1[CONV ? kMaxTaps : 1], tap_d2[CONV ? kMaxTaps : 1];   // CONV: tap offsets (LDS copy)

  const TokGroup g = a.groups[blockIdx.y];
  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  const int n_tiles = a.n_tiles_n;             // BN-column tiles (the caller counts them for this BN)
  const int n_tile = tile % n_tiles;
  const int m_tile = tile / n_tiles;
  const int n0 = n_tile * BN;
  if (n0 >= g.N) return;                       // this group has fewer column tiles
  const int m0 = m_tile * BM;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int l32 = lane & 31, h = lane >> 5;
  const int n_chunks = (g.K + BK - 1) / BK;

  f32x16 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // A staging: item (row, 4 k); thread covers rows (tid >> 3) + (NT / 8) i, k quad (tid & 7)
  constexpr int AI = BM * 8 / NT;
  constexpr int RS = NT / 8;
  const int arow0 = tid >> 3, akq = (tid & 7) * 4;
  f32x4 areg[PD][AI];
  f32x4 a2reg[PD][CONV ? AI : 1];
  uint2 ahreg[PD][PRE ? AI : 1], alreg[PD][PRE && X3 ? AI : 1];  // pre-split quads (4 bf16 each)
  float ss[AI];
  const float* xrow[AI];
  int64_t prow[PRE ? AI : 1];                             // plane element offset of the row
  bool rok[AI];
  // CONV: per-row input grid origin (b Q1, i1 s1, i2 s2), its input position index, and per-chunk validity
  int rb1[CONV ? AI : 1], ri1[CONV ? AI : 1], ri2[CONV ? AI : 1], rpos0[CONV ? AI : 1];
  bool aval[PD][CONV ? AI : 1];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    ss[i] = 0.f;
    const int m = m0 + arow0 + RS * i;
    rok[i] = m < a.M;
    if constexpr (PRE) prow[i] = (int64_t)(rok[i] ? m : a.M - 1) * a.a_ld + g.x_off;
    else xrow[i] = a.x + (int64_t)(rok[i] ? m : a.M - 1) * a.x_ld + g.x_off;
    if constexpr (CONV) {
      const int mm = rok[i] ? m : 0;
      const int i2 = mm % a.geo.P2, t = mm / a.geo.P2;
      const int i1 = t % a.geo.P1, b = t / a.geo.P1;
      rb1[i] = a.geo.xq1 ? b * a.geo.xq1 + a.geo.x_row0 : b * a.geo.Q1;
      ri1[i] = i1 * a.geo.s1;
      ri2[i] = i2 * a.geo.s2;
      rpos0[i] = (rb1[i] + ri1[i]) * a.geo.Q2 + ri2[i];   // input position of tap offset (0, 0)
      for (int s = 0; s < PD; ++s) aval[s][i] = false;
    }
  }
  bool kok[PD];
  // CONV: this thread's k quad as (tap, channel), advanced incrementally (no division per chunk); the tap
  // offsets come from an LDS copy of the geometry (a per-lane index into the kernel arguments is a memory
  // round trip per chunk)
  int k_cur = 0, tap_s = 0, c_s = 0;
  if constexpr (CONV) {
    for (int t = tid; t < a.geo.n_taps; t += NT) {
      tap_d1[t] = a.geo.d1[t];
      tap_d2[t] = a.geo.d2[t];
    }
    __syncthreads();
  }
  constexpr int W16 = (X3 ? 2 : 1) * W_BYTES / 16;
  constexpr int W_ITEMS = (W16 + NT - 1) / NT;
  u32x4 wreg[PD][W_ITEMS];
  // packed per 128-column block: [block][chunk][hi 128 x 32][lo 128 x 32]; a 64-column tile takes rows
  // 64 half .. 64 half + 63 of both planes (the row swizzle depends on row & 15 only, so it carries over)
  constexpr int IMG128 = kTokBN * BK;                       // uint16 per plane of a packed chunk image
  const uint16_t* wblk = a.w + g.w_off + (int64_t)(BN == kTokBN ? n_tile : n_tile >> 1) * n_chunks * (2 * IMG128) +
                         (BN == kTokBN ? 0 : (n_tile & 1) * (BN * BK));

  auto load_chunk = [&](auto S, int kc) {
    constexpr int s = decltype(S)::value;
    const uint16_t* wc = wblk + (int64_t)kc * (2 * IMG128);
    Unroll<0, W_ITEMS>::run([&](auto I) {
      const int e = min(tid + I * NT, W16 - 1);
      constexpr int PL16 = W_BYTES / 16;                    // u32x4 per plane of this tile
      const int pl = e >= PL16 ? 1 : 0, ee = e - pl * PL16;
      wreg[s][I] = reinterpret_cast<const u32x4*>(wc + pl * IMG128)[ee];
    });
    const int k = kc * BK + akq;
    kok[s] = k < g.K;  // K % 4 == 0 (host check): a quad is wholly in or out
    const int kc_ = kok[s] ? k : 0;
    if constexpr (CONV) {
      // Cin % 4 == 0 (host check): a quad lies inside one tap.  k advances monotonically (0, 32, 64, ... plus
      // clamped repeats of the last chunk)
      c_s += k - k_cur;
      k_cur = k;
      while (c_s >= a.geo.Cin) {
        c_s -= a.geo.Cin;
        ++tap_s;
      }
      const int tap = min(tap_s, a.geo.n_taps - 1), c = c_s;
      const int d1 = tap_d1[tap], d2 = tap_d2[tap];
      const int dpos = d1 * a.geo.Q2 + d2;
#pragma unroll
      for (int i = 0; i < AI; ++i) {
        const int j1 = ri1[i] + d1, j2 = ri2[i] + d2;
        aval[s][i] = rok[i] && kok[s] && (unsigned)j1 < (unsigned)a.geo.Q1 && (unsigned)j2 < (unsigned)a.geo.Q2;
        const int64_t off = aval[s][i] ? (int64_t)(rpos0[i] + dpos) * a.x_ld + g.x_off + c : 0;
        areg[s][i] = *reinterpret_cast<const f32x4*>(a.x + off);
        if (a.geo.x2) a2reg[s][i] = *reinterpret_cast<const f32x4*>(a.geo.x2 + off);
      }
    } else if constexpr (PRE) {
#pragma unroll
      for (int i = 0; i < AI; ++i) {
        ahreg[s][i] = *reinterpret_cast<const uint2*>(a.a_hi + prow[i] + kc_);
        if constexpr (X3) alreg[s][i] = *reinterpret_cast<const uint2*>(a.a_lo + prow[i] + kc_);
      }
    } else {
#pragma unroll
      for (int i = 0; i < AI; ++i) areg[s][i] = *reinterpret_cast<const f32x4*>(xrow[i] + kc_);
    }
  };
  // count: 1 when this store is a real chunk (0 for the clamped repeat past the end: no RMS sum)
  auto store_chunk = [&](auto S, char* stg, float count) {
    constexpr int s = decltype(S)::value;
    char* Ahi = stg;
    char* Alo = stg + A_BYTES;
    u32x4* d4 = reinterpret_cast<u32x4*>(stg + 2 * A_BYTES);
    Unroll<0, W_ITEMS>::run([&](auto I) {
      const int e = min(tid + I * NT, W16 - 1);  // duplicates write identical values
      d4[e] = wreg[s][I];
    });
    if constexpr (PRE) {
#pragma unroll
      for (int i = 0; i < AI; ++i) {
        const int row = arow0 + RS * i;
        const bool ok = rok[i] && kok[s];
        const int off = row * ROWB + ((((akq >> 3) ^ ((row >> 2) & 3))) << 4) + ((akq & 4) << 1);
        *reinterpret_cast<uint2*>(Ahi + off) = ok ? ahreg[s][i] : make_uint2(0u, 0u);
        if (X3) *reinterpret_cast<uint2*>(Alo + off) = ok ? alreg[s][i] : make_uint2(0u, 0u);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int row = arow0 + RS * i;
      bool ok = rok[i] && kok[s];
      if constexpr (CONV) ok = aval[s][i];
      __bf16 hi[4], lo[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float v = ok ? areg[s][i][q] : 0.f;
        if constexpr (CONV) {
          if (a.geo.x2 && ok) v += a2reg[s][i][q];
        }
        if constexpr (!CONV) ss[i] = fmaf(v * count, v, ss[i]);
        if constexpr (F16) areg[s][i][q] = v;   // (the fp16 pack below reads the final values)
        else split_bf16(v, hi[q], lo[q]);
      }
      const int off = row * ROWB + ((((akq >> 3) ^ ((row >> 2) & 3))) << 4) + ((akq & 4) << 1);
      if constexpr (F16) {
        const f32x4 v = areg[s][i];
        const uint32_t m = ok ? 0xffffffffu : 0u;
        const auto h2 = [](float x, float y) {
          return (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)x) |
                 ((uint32_t)__builtin_bit_cast(uint16_t, (_Float16)y) << 16);
        };
        *reinterpret_cast<uint2*>(Ahi + off) = make_uint2(h2(v[0], v[1]) & m, h2(v[2], v[3]) & m);
        continue;
      }
      *reinterpret_cast<uint2*>(Ahi + off) = make_uint2(pack2(hi[0], hi[1]), pack2(hi[2], hi[3]));
      if (X3) *reinterpret_cast<uint2*>(Alo + off) = make_uint2(pack2(lo[0], lo[1]), pack2(lo[2], lo[3]));
    }
  };
  auto kstep = [&](const char* stg, int ks) {
    const char* Ahi = stg;
    const char* Alo = stg + A_BYTES;
    const char* Whi = stg + 2 * A_BYTES;
    bf16x8 ah[MI], al[MI], bh[NI], bl[NI];
    const int q = ks * 2 + h;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int row = (wm * MI + i) * 32 + l32;
      const int off = row * ROWB + ((q ^ ((row >> 2) & 3)) << 4);
      ah[i] = *reinterpret_cast<const bf16x8*>(Ahi + off);
      if (X3) al[i] = *reinterpret_cast<const bf16x8*>(Alo + off);
    }
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int n = (wn * NI + j) * 32 + l32;
      const int off = n * ROWB + ((q ^ ((n >> 2) & 3)) << 4);
      bh[j] = *reinterpret_cast<const bf16x8*>(Whi + off);
      if (X3) bl[j] = *reinterpret_cast<const bf16x8*>(Whi + W_BYTES + off);
    }
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        if (X3) {
          acc[i][j] = mfma32(al[i], bh[j], acc[i][j]);
          acc[i][j] = mfma32(ah[i], bl[j], acc[i][j]);
        }
        if constexpr (F16)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, ah[i]),
                                                             __builtin_bit_cast(f16x8, bh[j]), acc[i][j], 0, 0, 0);
        else acc[i][j] = mfma32(ah[i], bh[j], acc[i][j]);
      }
  };

  using S0 = std::integral_constant<int, 0>;
  if constexpr (DB) {
    load_chunk(S0{}, 0);
    store_chunk(S0{}, smem, 1.f);
    load_chunk(S0{}, min(1, n_chunks - 1));
    __syncthreads();
    for (int kc = 0; kc < n_chunks; ++kc) {
      const char* cur = smem + (kc & 1) * STAGE;
      char* nxt = smem + ((kc + 1) & 1) * STAGE;
      kstep(cur, 0);
      store_chunk(S0{}, nxt, kc + 1 < n_chunks ? 1.f : 0.f);
      load_chunk(S0{}, min(kc + 2, n_chunks - 1));
      kstep(cur, 1);
      __syncthreads();
    }
  } else if constexpr (PD == 1) {
    // single stage, two barriers per chunk, register prefetch of the next chunk under the MFMAs;
    // two workgroups per CU overlap one's staging / epilogue with the other's MFMAs
    load_chunk(S0{}, 0);
    for (int kc = 0; kc < n_chunks; ++kc) {
      __syncthreads();
      store_chunk(S0{}, smem, 1.f);
      __syncthreads();
      load_chunk(S0{}, min(kc + 1, n_chunks - 1));
      kstep(smem, 0);
      kstep(smem, 1);
    }
  } else {
    // PD register sets: the loop is unrolled by PD so every set is addressed at compile time; chunk kc's set
    // is refilled with chunk kc + PD right after it is staged (past the end: clamped repeats, never staged)
    Unroll<0, PD>::run([&](auto S) { load_chunk(S, min((int)decltype(S)::value, n_chunks - 1)); });
    for (int kc0 = 0; kc0 < n_chunks; kc0 += PD) {
      Unroll<0, PD>::run([&](auto S) {
        const int kc = kc0 + decltype(S)::value;
        if (kc < n_chunks) {
          __syncthreads();
          store_chunk(S, smem, 1.f);
          __syncthreads();
          load_chunk(S, min(kc + PD, n_chunks - 1));
          kstep(smem, 0);
          kstep(smem, 1);
        }
      });
    }
  }

  // ---- RMSNorm row scales: 8 threads share a row ----
  if (PRE && a.rownorm) {
    for (int r = tid; r < BM; r += NT) rs[r] = a.row_scale[min(m0 + r, a.M - 1)];
    __syncthreads();
  } else if (a.rownorm) {
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      float v = ss[i];
      v += __shfl_xor(v, 1);
      v += __shfl_xor(v, 2);
      v += __shfl_xor(v, 4);
      if ((tid & 7) == 0) rs[arow0 + RS * i] = sqrtf((float)g.K) / fmaxf(sqrtf(v), 1e-12f);
    }
    __syncthreads();
  }

  // output rows through the table: transposed conv, or the sub-range form (phases == 1: n_ph = N, ph = 0)
  const bool tconv = CONV && (a.geo.phases > 1 || a.geo.oq1 > 0);
  if constexpr (CONV) {
    if (tconv) {
      for (int r = tid; r < BM; r += NT) {
        const int m = min(m0 + r, a.M - 1);
        const int i2 = m % a.geo.P2, t = m / a.geo.P2;
        const int i1 = t % a.geo.P1, b = t / a.geo.P1;
        orow_i1[r] = i1 * a.geo.phases - a.geo.opad;
        orow_base[r] = a.geo.o_fmajor ? (b * a.geo.P2 + i2) * a.geo.oq1 + a.geo.o_row0 + orow_i1[r]
                                      : ((a.geo.oq1 ? b * a.geo.oq1 + a.geo.o_row0 : b * a.geo.O1) + orow_i1[r]) * a.geo.P2 + i2;
      }
      __syncthreads();
    }
  }
  const int n_ph = tconv ? g.N / a.geo.phases : g.N;

  // ---- epilogue, one 32x32 block at a time (compile-time block indices: acc stays in VGPRs):
  // scale, bias, activation, rotary / GLU, then residual loads (all before any store: residual may
  // alias out), then stores ----
  Unroll<0, MI>::run([&](auto I) {
    constexpr int i = decltype(I)::value;
    Unroll<0, NI>::run([&](auto J) {
      constexpr int j = decltype(J)::value;
      const int n = n0 + (wn * NI + j) * 32 + l32;
      const bool n_ok = n < g.N;
      const float bias = (g.b_off >= 0 && n_ok) ? a.bias[g.b_off + n] : 0.f;
      const int d = n % a.dim_head;
      const bool rot = a.rope && n < a.rope_cols;
      f32x16 v = acc[i][j];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ml = (wm * MI + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        float x = v[r];
        if (a.rownorm) x *= rs[ml];
        x += bias;
        if (a.act == TOK_ACT_GELU) x = gelu_erf(x);
        else if (a.act == TOK_ACT_TANH) x = tanhf(x);
        else if (a.act == TOK_ACT_RELU) x = fmaxf(x, 0.f);
        const float partner = __shfl_xor(x, 1);  // column n ^ 1, same row
        if (rot) {
          const int m = m0 + ml;
          const int pos = a.pos_time ? (m / a.pos_F) % a.pos_T : m % a.pos_F;
          const float2 cs = a.rope[(int64_t)pos * (a.dim_head >> 1) + (d >> 1)];
          x = (d & 1) ? fmaf(x, cs.x, partner * cs.y) : fmaf(x, cs.x, -partner * cs.y);
        }
        if (a.glu) x = x * sigmoidf_(partner);  // valid on even columns (a_j); odd lanes discarded
        v[r] = x;
      }
      const int rb = m0 + (wm * MI + i) * 32 + 4 * h;
      // output row of tile row ml (identity unless transposed conv), validity, column
      const int ph = tconv ? n / n_ph : 0;
      const int ncol = tconv ? n - ph * n_ph : n;
      auto orow = [&](int r, bool& ok) -> int64_t {
        const int m = rb + (r & 3) + 8 * (r >> 2);
        ok = m < a.M;
        if (!tconv) return m;
        const int ml = m - m0;
        const int i1 = orow_i1[ml] + ph;
        ok = ok && i1 >= 0 && i1 < a.geo.O1;
        return (int64_t)orow_base[ml] + (int64_t)ph * (a.geo.o_fmajor ? 1 : a.geo.P2);
      };
      if (a.residual && n_ok) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          bool ok;
          const int64_t m = orow(r, ok);
          if (ok) v[r] += a.residual[m * a.o_ld + g.o_off + ncol];
        }
      }
      if (n_ok && !(a.glu && (n & 1))) {
        const int nc = a.glu ? n >> 1 : ncol;
        if (a.out_hi) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            bool ok;
            const int64_t m = orow(r, ok);
            __bf16 hi, lo;
            split_bf16(v[r], hi, lo);
            if (ok) {
              a.out_hi[m * a.o_ld + g.o_off + nc] = __builtin_bit_cast(uint16_t, hi);
              if (a.out_lo) a.out_lo[m * a.o_ld + g.o_off + nc] = __builtin_bit_cast(uint16_t, lo);
            }
          }
        } else {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            bool ok;
            const int64_t m = orow(r, ok);
            if (ok) a.out[m * a.o_ld + g.o_off + nc] = v[r];
          }
        }
      }
    });
  });
}

// ---------------------------------------------------------------------------------------------
// Pre-split A, LDS-DMA staging, big tile (bf16x3).  512 threads (8 waves: 2 along M x 4 along N,
// 128 x 64 each = 4 x 2 blocks of 32x32), tile 256 tokens x 256 columns (two packed 128-column
// weight tiles), K chunks of 32 in two 64 KiB LDS stages filled by global_load_lds_dwordx4 (1 KiB per
// wave-instruction, lane-linear destination; the A image's 16-B XOR swizzle goes on the per-lane
// SOURCE address, so fragment reads match tok_gemm_kernel's).  Per chunk and wave: 48 MFMAs on 12
// fragment reads per k-step (0.5 ds_read_b128 per MFMA vs 0.67 for 64x64 wave tiles); chunk kc + 1's
// DMA is issued at the top of iteration kc and retired by one counted wait + raw barrier at its end.
// All LDS in one array (a second __shared__ object can make hipcc wait vmcnt(0) before the fragment
// reads).
// The epilogue is specialised at compile time (EP flags) and has a guard-free body for full tiles:
// with runtime mode flags and per-element row / column guards it compiled to ~1.4k branches and
// cost more than the main loop.  Operands a 32x32 block would gather with a load -> wait round trip
// each are staged once into the freed LDS by LDS-DMA: the rotary (cos, sin) rows of the tile's tokens
// (64 KiB), the residual in two 128-row halves (128 KiB each).
enum : int { EP_RS = 1, EP_ROPE = 2, EP_GELU = 4, EP_RES = 8, EP_SPLIT = 16, EP_RAW = 32, EP_NONE = 64, EP_F16 = 128 };

__device__ __forceinline__ float dpp_xor1(float x) {  // lane ^ 1 (quad_perm [1, 0, 3, 2])
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0xB1, 0xF, 0xF, false));
}
__device__ __forceinline__ uint32_t dpp_xor1u(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false);
}

// EP: EP_RS (row scale) | EP_ROPE (rotary, dim_head 64) | EP_GELU | EP_RES (residual) | EP_SPLIT
// (bf16 planes out); bias always (per group).  EP_RAW / EP_NONE: ablations for tools/tokgemm_bench.hip.
// M16: v_mfma_f32_16x16x32_bf16 blocks (8 x 4 per wave, one k-step per 32-deep chunk) instead of
// 32x32x16 (4 x 2, two k-steps); same wave tile, accumulator count and LDS images.
// DEPTH > 2 (EP_F16 only): compact fp16 stages (A hi plane + the two 128-column hi images, 32 KiB)
// in a DEPTH-slot ring over the same LDS, DEPTH - 1 chunks in flight instead of one, one barrier per
// chunk (counted vmcnt waits); the epilogue is unchanged.
// HT (half tile; fp16 ring only): 256 threads, 256 tokens x 128 columns (4 waves of 128 x 64), a 24 KiB ring
// slot, two workgroups per CU -- one workgroup's epilogue runs beside the other's main loop instead of
// idling the MFMA pipe (the epilogues of the fp16 Linears cost as much as their main loops).
// PERS (HT ring only): persistent workgroups -- 2 per CU, each walks tiles wgi = blockIdx.x, + gridDim.x, ... of the
// a.pers_tiles the grid would have had -- and the second half of the grid (the second slot of every CU) starts a.stagger
// x 8128 cycles late, so the two co-resident workgroups run out of phase: one's VALU-bound epilogue (GELU / rotary /
// fp16 packing) beside the other's MFMA-bound main loop, where a one-tile-per-workgroup grid keeps them in lockstep.
template <int EP, bool M16 = false, int DEPTH = 2, bool HT = false, bool PERS = false>
__global__ void __launch_bounds__(HT ? 256 : 512, HT ? 2 : 1) tok_gemm_glds_kernel(TokGemmArgs a) {
  static_assert(!PERS || HT, "persistent: the half-tile fp16 ring");
  constexpr int NT = HT ? 256 : 512, BM = 256, BK = kTokBK, WN = HT ? 2 : 4;
  constexpr int NW = NT / 64;                              // waves
  constexpr int TN = HT ? 128 : 256;                       // tile columns
  constexpr int BLK = M16 ? 16 : 32;                       // MFMA block edge
  constexpr int MI = 128 / BLK, NI = 64 / BLK;             // blocks per 128 x 64 wave tile
  constexpr int RPB = BLK * BLK / 64;                      // accumulator registers per block
  using Acc = std::conditional_t<M16, f32x4, f32x16>;
  constexpr int ROWB = BK * 2;
  constexpr int A_BYTES = BM * ROWB;                       // 16 KiB per plane
  constexpr int A_REG = 2 * A_BYTES;
  constexpr int W_PLANE = kTokBN * ROWB;                   // 8 KiB: one packed 128-column image plane
  constexpr int W_IMG = 2 * W_PLANE;
  constexpr int STAGE = A_REG + 2 * W_IMG;                 // 64 KiB
  constexpr int A_PIECES = A_REG / 1024, W_PIECES = 2 * W_IMG / 1024, W_HALF = W_IMG / 1024;
  constexpr int PPW = (A_PIECES + W_PIECES) / (NT / 64);   // glds per wave per chunk (8)
  constexpr int APW = A_PIECES / (NT / 64);                 // of which A pieces (4)
  static_assert((A_PIECES + W_PIECES) % (NT / 64) == 0 && A_PIECES % (NT / 64) == 0, "piece split");
  static_assert(2 * STAGE >= 128 * 1024, "epilogue staging reuses the two stages");
  constexpr bool CMP = (EP & EP_F16) != 0 && DEPTH > 2;   // compact fp16 ring
  constexpr int SSZ = CMP ? A_BYTES + (HT ? 1 : 2) * W_PLANE : STAGE;  // bytes per ring slot
  static_assert(!HT || CMP, "half tile: the fp16 ring only");
  // LDS: the two bf16x3 stages, or (HT) the ring, at least the 64 KiB the epilogue staging takes
  constexpr int RING = HT ? (DEPTH * SSZ > 65536 ? DEPTH * SSZ : 65536) : 2 * STAGE;
  __shared__ __attribute__((aligned(16))) char smem[RING + 2 * BM * 4];
  float* rs = reinterpret_cast<float*>(smem + RING);
  int* rpos = reinterpret_cast<int*>(rs + BM);

  const int n_wg = PERS ? a.pers_tiles : (int)gridDim.x;
  if (PERS && blockIdx.x >= gridDim.x / 2)
    for (int i = 0; i < a.stagger; ++i) __builtin_amdgcn_s_sleep(127);
  for (int wgi = blockIdx.x; wgi < n_wg; wgi += (PERS ? (int)gridDim.x : n_wg)) {
  if (PERS) sesa_sync();   // the previous tile's epilogue is done with the LDS the ring and tables reuse
  const TokGroup g = a.groups[blockIdx.y];
  const int n_tiles2 = HT ? a.n_tiles_n : (a.n_tiles_n + 1) >> 1;   // TN-column tiles
  const int tile = xcd_tile(wgi, n_wg);
  const int n_tile2 = tile % n_tiles2;
  const int m_tile = tile / n_tiles2;
  const int n0 = n_tile2 * TN;
  if (n0 >= g.N) continue;
  const int m0 = m_tile * BM;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int l32 = lane & 31, h = lane >> 5;
  const int n_chunks = (g.K + BK - 1) / BK;
  static_assert(!CMP || DEPTH * SSZ <= RING, "ring fits the LDS");
  static_assert(DEPTH == 2 || ((EP & EP_F16) != 0 && M16), "deep ring: the fp16 16x16x32 kernel only");

  for (int r = tid; r < BM; r += NT) {                      // ordinary loads, before any DMA is in flight
    const int m = min(m0 + r, a.M - 1);
    if (EP & EP_RS) rs[r] = a.row_scale[m];
    if (EP & EP_ROPE) rpos[r] = a.pos_time ? (m / a.pos_F) % a.pos_T : m % a.pos_F;
  }

  // this lane's A pieces: piece p (per plane) covers tile rows 16 p .. 16 p + 15, 4 lanes a row
  constexpr int AP1 = A_BYTES / 1024 / NW;                  // pieces per plane per wave (2; HT 4)
  constexpr bool F16 = (EP & EP_F16) != 0;                  // fp16 A planes x fp16 weight images, one pass
  int64_t asrc[AP1];
  int aslot8[AP1];
#pragma unroll
  for (int i = 0; i < AP1; ++i) {
    const int row = 16 * (wave + NW * i) + (lane >> 2);
    asrc[i] = (int64_t)min(m0 + row, a.M - 1) * a.a_ld + g.x_off;
    aslot8[i] = 8 * ((lane & 3) ^ ((row >> 2) & 3));
  }
  const int64_t wimg = W_IMG / 2;                           // uint16 per packed chunk image (hi + lo)
  const uint16_t* wblk0 = a.w + g.w_off + (int64_t)((HT ? 1 : 2) * n_tile2) * n_chunks * wimg;
  // the second 128-column tile; past the group's last tile a harmless repeat (its columns are >= N)
  const uint16_t* wblk1 = n0 + kTokBN < g.N ? wblk0 + (int64_t)n_chunks * wimg : wblk0;

  // compact fp16 ring: per wave and chunk AP1 A pieces + WPW hi-image pieces (the lo planes are never read)
  constexpr int WPW = (HT ? 8 : 16) / NW;
  constexpr int PPC = AP1 + WPW;                            // DMA pieces per wave per chunk
  auto issue = [&](int kc, char* stg) {
    if constexpr (CMP) {
#pragma unroll
      for (int i = 0; i < AP1; ++i) {                       // A piece wave + NW i: tile rows 16 p .. 16 p + 15
        const int k = kc * BK + aslot8[i];
        const uint16_t* src = a.a_hi + asrc[i] + (k < g.K ? k : 0);
        __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(stg + (wave + NW * i) * 1024),
                                         16, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < WPW; ++i) {                       // hi piece q of the (one or two) 128-column images
        const int q = wave + NW * i, half = q >> 3, qq = q & 7;
        const uint16_t* src = (half ? wblk1 : wblk0) + (int64_t)kc * wimg + qq * 512 + lane * 8;
        __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(stg + A_BYTES + q * 1024), 16,
                                         0, 0);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      // EP_F16: the lo planes are never read -- skip their pieces (A plane 1; the odd W pieces of this
      // wave, q = wave + 8 (i - APW), are the lo halves of the two 128-column images)
      if (F16 && (i < APW ? i / AP1 == 1 : ((i - APW) & 1) == 1)) continue;
      if (i < APW) {                                        // A: plane i / AP1, piece wave + 8 (i % AP1)
        const int ii = i % AP1, plane = i / AP1;
        const int k = kc * BK + aslot8[ii];
        const int64_t off = asrc[ii] + (k < g.K ? k : 0);  // K % 8 == 0 (host check); W is zero past K
        const uint16_t* src = (plane ? a.a_lo : a.a_hi) + off;
        __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(stg + plane * A_BYTES +
                                                                                       (wave + 8 * ii) * 1024),
                                         16, 0, 0);
      } else {                                              // W piece q: image half q / W_HALF
        const int q = wave + 8 * (i - APW);
        const int half = q / W_HALF, qq = q - half * W_HALF;
        const uint16_t* src = (half ? wblk1 : wblk0) + (int64_t)kc * wimg + qq * 512 + lane * 8;
        __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(stg + A_REG + q * 1024), 16,
                                         0, 0);
      }
    }
  };

  Acc acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int r = 0; r < RPB; ++r) acc[i][j][r] = 0.f;

  // fragment row / 16-B chunk of this lane: 32x32x16 -> row l32, chunk 2 ks + h (two k-steps per
  // chunk); 16x16x32 -> row lane & 15, chunk lane >> 4 (one k-step)
  const int frow = M16 ? (lane & 15) : l32;
  struct Frags {
    bf16x8 ah[MI], al[MI], bh[NI], bl[NI];
  };
  auto read_frags = [&](Frags& f, const char* stg, int ks) {
    const int q = M16 ? (lane >> 4) : ks * 2 + h;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int row = (wm * MI + i) * BLK + frow;
      const int off = row * ROWB + ((q ^ ((row >> 2) & 3)) << 4);
      f.ah[i] = *reinterpret_cast<const bf16x8*>(stg + off);
      if constexpr (!F16) f.al[i] = *reinterpret_cast<const bf16x8*>(stg + A_BYTES + off);
    }
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int c = (wn * NI + j) * BLK + frow;             // 0..255
      const int r = c & (kTokBN - 1);
      const int off = (CMP ? A_BYTES + (c >> 7) * W_PLANE : A_REG + (c >> 7) * W_IMG) + r * ROWB +
                      ((q ^ ((r >> 2) & 3)) << 4);
      f.bh[j] = *reinterpret_cast<const bf16x8*>(stg + off);
      if constexpr (!F16) f.bl[j] = *reinterpret_cast<const bf16x8*>(stg + off + W_PLANE);
    }
  };
  // EP_F16: fp16 A planes x fp16 weight images, one pass
  auto mma = [&](const bf16x8& x, const bf16x8& y, Acc& c) {
    if constexpr (F16) {
      const f16x8 xh = __builtin_bit_cast(f16x8, x), yh = __builtin_bit_cast(f16x8, y);
      if constexpr (M16) c = __builtin_amdgcn_mfma_f32_16x16x32_f16(xh, yh, c, 0, 0, 0);
      else c = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, yh, c, 0, 0, 0);
    } else {
      if constexpr (M16) c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, y, c, 0, 0, 0);
      else c = mfma32(x, y, c);
    }
  };
  auto mfmas = [&](const Frags& f) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        if constexpr (!F16) {
          mma(f.al[i], f.bh[j], acc[i][j]);
          mma(f.ah[i], f.bl[j], acc[i][j]);
        }
        mma(f.ah[i], f.bh[j], acc[i][j]);
      }
  };

  sesa_sync();                                         // rs / rpos visible; no DMA in flight yet
  // waves whose 64 columns all lie past the group's N (the partial last tile, e.g. BS-Roformer's
  // 8 gate columns after q / k / v) skip their MFMAs (wave-uniform); they still issue their DMA pieces
  const bool busy = n0 + wn * 64 < g.N;
  if constexpr (CMP) {
    // PPC DMA pieces per wave per chunk: chunk kc has landed for this wave when at most
    // PPC min(DEPTH - 2, n_chunks - 1 - kc) of its pieces are still outstanding
    static_assert(DEPTH <= 4 && 2 * PPC <= 63, "counted waits");
#pragma unroll
    for (int s = 0; s < DEPTH - 1; ++s)
      if (s < n_chunks) issue(s, smem + s * SSZ);
    for (int kc = 0; kc < n_chunks; ++kc) {
      const int pend = min(DEPTH - 2, n_chunks - 1 - kc);
      if (pend >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PPC) : "memory");
      else if (pend == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPC) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      // every wave's pieces of chunk kc landed, and every wave's reads of slot (kc - 1) % DEPTH retired
      // (lgkmcnt(0) below) -- that slot takes chunk kc + DEPTH - 1
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (kc + DEPTH - 1 < n_chunks) issue(kc + DEPTH - 1, smem + ((kc + DEPTH - 1) % DEPTH) * SSZ);
      if (busy) {
        Frags f0;
        read_frags(f0, smem + (kc % DEPTH) * SSZ, 0);
        mfmas(f0);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();                          // the epilogue's LDS staging reuses the ring
    asm volatile("" ::: "memory");
  } else {
  issue(0, smem);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  for (int kc = 0; kc < n_chunks; ++kc) {
    char* cur = smem + (kc & 1) * STAGE;
    // chunk kc + 1 into the other stage: its last fragment reads (iteration kc - 1) were retired
    // by the lgkmcnt(0) before that iteration's barrier
    if (kc + 1 < n_chunks) issue(kc + 1, smem + ((kc + 1) & 1) * STAGE);
    if (!busy) {
    } else if constexpr (M16) {
      Frags f0;
      read_frags(f0, cur, 0);
      mfmas(f0);
    } else {
      Frags f0, f1;
      read_frags(f0, cur, 0);
      read_frags(f1, cur, 1);
      mfmas(f0);
      mfmas(f1);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  }

  if constexpr ((EP & EP_NONE) != 0) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) asm volatile("" ::"v"(acc[i][j]));
    continue;
  }

  // ---- epilogue ----
  // Lane / wave indices re-derived behind an optimisation barrier: every epilogue address then depends on a value the
  // compiler cannot hoist above the main loop (it used to compute ~128 per-element store addresses before the main
  // loop and spill them to scratch across it, profiles/r05_tokgemm_spills.txt)
  int etid = tid;
  asm volatile("" : "+v"(etid));
  const int elane = etid & 63, ewave = etid >> 6;
  const int ewm = ewave / WN, ewn = ewave % WN;
  const int el32 = elane & 31, eh = elane >> 5;
  const float* lres = reinterpret_cast<const float*>(smem);
  const float2* lrope = reinterpret_cast<const float2*>(smem);
  if constexpr ((EP & EP_ROPE) != 0) {
#pragma unroll
    for (int i = 0; i < 64 / NW; ++i) {                    // piece q: tile rows 4 q .. 4 q + 3 (256 B each)
      const int q = ewave + NW * i;
      const int row = 4 * q + (elane >> 4);
      const float2* src = a.rope + (int64_t)rpos[row] * 32 + (elane & 15) * 2;
      __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(smem + q * 1024), 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  const bool full = m0 + BM <= a.M && n0 + TN <= g.N;
  // fp16 split output staged through LDS (the ring is free after the main loop) and stored as full lines
  // (not beside the rotary table, which occupies the same LDS during the epilogue)
  const bool stage16 = (EP & EP_SPLIT) != 0 && (EP & EP_ROPE) == 0 && F16 && a.o_ld % 8 == 0 && g.o_off % 8 == 0;
  float bias[NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int n = n0 + (ewn * NI + j) * BLK + (M16 ? (elane & 15) : el32);
    bias[j] = (g.b_off >= 0 && n < g.N) ? a.bias[g.b_off + n] : 0.f;
  }
  // FULL-tile output bases (the tile's first row and column); per-element offsets are 32-bit (< 256 rows x o_ld)
  uint16_t* const out16_tile = (EP & EP_SPLIT) ? a.out_hi + (int64_t)m0 * a.o_ld + g.o_off + n0 : nullptr;
  float* const out32_tile = (EP & EP_SPLIT) ? nullptr : a.out + (int64_t)m0 * a.o_ld + g.o_off + n0;
  auto row_of = [&](int i, int r) -> int {
    return M16 ? (ewm * MI + i) * 16 + 4 * (elane >> 4) + r : (ewm * MI + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * eh;
  };
  // FULL-tile store addresses: one 64-bit tile base and a per-elane 32-bit part, so that (i, r) -- compile-time in the
  // unrolled block loops -- only adds a constant (row_of = lane_row + (ewm MI + i) BLK + const(r)).  Written as
  // 64-bit expressions per element, the compiler hoisted ~128 per-element addresses to the kernel start and spilled
  // them to scratch (profiles/r05_tokgemm_spills.txt: 32-56 VGPRs of scratch spills per epilogue variant).
  const int lane_row = M16 ? 4 * (elane >> 4) : 4 * eh;
  auto row_c = [&](int i, int r) -> int { return (ewm * MI + i) * BLK + (M16 ? r : (r & 3) + 8 * (r >> 2)); };
  // LDS stage image offset of (row_of(i, r), column nl): the 32-B group swizzle (row >> 2) & 3 is (elane >> 4) & 3 for
  // the 16x16 blocks and (2 (r >> 2) + eh) & 3 for the 32x32 ones
  auto stage_off = [&](int i, int r, int nl) -> int {
    const int sw = M16 ? ((elane >> 4) & 3) : ((2 * (r >> 2) + eh) & 3);
    return (row_c(i, r) + lane_row) * (2 * TN) + ((2 * nl) ^ (sw << 5));
  };
  // one MFMA block: FULL = no row / column guards; row of accumulator register r of block i
  auto block = [&](auto I, auto J, auto P, auto FULLT) {
    constexpr int i = decltype(I)::value, j = decltype(J)::value, p = decltype(P)::value;
    constexpr bool FULL = decltype(FULLT)::value;
    const int nl = (ewn * NI + j) * BLK + (M16 ? (elane & 15) : el32);
    const int n = n0 + nl;
    Acc v = acc[i][j];
    if constexpr ((EP & EP_RAW) == 0) {
      const int d = n & 63;
      const bool rot = n < a.rope_cols;
#pragma unroll
      for (int r = 0; r < RPB; ++r) {
        const int ml = row_of(i, r);
        float x = v[r];
        if constexpr ((EP & EP_RS) != 0) x *= rs[ml];
        v[r] = x + bias[j];
      }
      if constexpr ((EP & EP_GELU) != 0) {
        // two values per packed v_pk_fma_f32 sequence: this epilogue is VALU-issue-bound
#pragma unroll
        for (int r = 0; r < RPB; r += 2) {
          const f32x2 y = gelu_erf2(f32x2{v[r], v[r + 1]});
          v[r] = y[0];
          v[r + 1] = y[1];
        }
      }
#pragma unroll
      for (int r = 0; r < RPB; ++r) {
        const int ml = row_of(i, r);
        float x = v[r];
        if constexpr ((EP & EP_ROPE) != 0) {
          const float partner = dpp_xor1(x);
          const float2 cs = lrope[ml * 32 + (d >> 1)];
          const float y = (d & 1) ? fmaf(x, cs.x, partner * cs.y) : fmaf(x, cs.x, -partner * cs.y);
          x = rot ? y : x;
        }
        if constexpr ((EP & EP_RES) != 0) x += lres[(ml - p * 64 - ewm * 64) * TN + nl];
        v[r] = x;
      }
    }
    if constexpr ((EP & EP_SPLIT) != 0 && F16) {
      // one fp16 plane, two columns per 4-byte store by the even lanes
#pragma unroll
      for (int r = 0; r < RPB; ++r) {
        const int m = m0 + row_of(i, r);
        const uint32_t hb = __builtin_bit_cast(uint16_t, (_Float16)v[r]);
        const int64_t o = (int64_t)m * a.o_ld + g.o_off + n;
        const uint32_t hn = dpp_xor1u(hb);  // uniform control flow
        if (FULL && stage16) {
          // into the LDS tile image (row stride 2 TN bytes, 32-B groups XOR-permuted by (row >> 2) & 3: the
          // four row groups of one store land in different banks); written out in full lines below
          if (!(el32 & 1)) *reinterpret_cast<uint32_t*>(smem + stage_off(i, r, nl)) = hb | (hn << 16);
        } else if (FULL) {
          if (!(el32 & 1))
            *reinterpret_cast<uint32_t*>(out16_tile + ((row_c(i, r) + lane_row) * a.o_ld + nl)) = hb | (hn << 16);
        } else if (m < a.M && n < g.N) {
          a.out_hi[o] = (uint16_t)hb;
        }
      }
    } else if constexpr ((EP & EP_SPLIT) != 0) {
      // bf16 planes, two columns per 4-byte store: even lanes write the hi pair (n, n + 1), odd
      // lanes the lo pair (n - 1, n)
#pragma unroll
      for (int r = 0; r < RPB; ++r) {
        const int m = m0 + row_of(i, r);
        __bf16 hi, lo;
        split_bf16(v[r], hi, lo);
        const uint32_t hb = __builtin_bit_cast(uint16_t, hi), lb = __builtin_bit_cast(uint16_t, lo);
        const int64_t o = (int64_t)m * a.o_ld + g.o_off + n;
        // both exchanges in uniform control flow (a DPP read of a elane masked off by a branch yields 0)
        const uint32_t hn = dpp_xor1u(hb), ln = dpp_xor1u(lb);
        if (FULL) {
          const uint32_t pv = (el32 & 1) ? ln | (lb << 16) : hb | (hn << 16);
          uint16_t* dst = (el32 & 1) ? a.out_lo + o - 1 : a.out_hi + o;
          *reinterpret_cast<uint32_t*>(dst) = pv;
        } else if (m < a.M && n < g.N) {
          a.out_hi[o] = (uint16_t)hb;
          a.out_lo[o] = (uint16_t)lb;
        }
      }
    } else {
#pragma unroll
      for (int r = 0; r < RPB; ++r) {
        const int m = m0 + row_of(i, r);
        if (FULL) out32_tile[(row_c(i, r) + lane_row) * a.o_ld + nl] = v[r];
        else if (m < a.M && n < g.N) a.out[(int64_t)m * a.o_ld + g.o_off + n] = v[r];
      }
    }
  };
  auto run = [&](auto FULLT) {
    Unroll<0, 2>::run([&](auto P) {                        // row half p
      constexpr int p = decltype(P)::value;
      if constexpr ((EP & EP_RES) != 0) {
        if (p == 1) {                                      // every ewave is done with half 0
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_s_barrier();
          asm volatile("" ::: "memory");
        }
        // 128 local rows of TN fp32 (1 KiB piece = 1024 / (4 TN) rows); local row rl <-> tile row (half p of
        // each ewm)
        constexpr int RPP = 256 / TN, LPR = 64 / RPP;      // rows per piece, lanes per row
#pragma unroll
        for (int i = 0; i < 128 / RPP / NW; ++i) {
          const int pc = ewave + NW * i;
          const int rl = pc * RPP + elane / LPR;
          const int row = rl < 64 ? p * 64 + rl : 128 + p * 64 + (rl - 64);
          const int m = min(m0 + row, a.M - 1);
          int col = n0 + (elane % LPR) * 4;
          if (col + 4 > g.N) col = n0;                     // columns >= N are never used
          const float* src = a.residual + (int64_t)m * a.o_ld + g.o_off + col;
          __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(smem + pc * 1024), 16, 0,
                                           0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
      Unroll<p * (MI / 2), (p + 1) * (MI / 2)>::run([&](auto I) {   // the blocks of rows ewm 128 + p 64 ..
        Unroll<0, NI>::run([&](auto J) { block(I, J, P, FULLT); });
      });
    });
  };
  if (full) run(std::true_type{});
  else run(std::false_type{});
  if constexpr ((EP & EP_SPLIT) != 0 && F16) {
    if (full && stage16) {
      // the fp16 tile from LDS as full rows: 16 B per elane, 2 TN bytes contiguous per row
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      constexpr int C16 = 2 * TN / 16;                     // 16-B groups per row
#pragma unroll 4
      for (int it = 0; it < BM * C16 / NT; ++it) {
        const int e = etid + it * NT;
        const int row = e / C16, c16 = e % C16;
        const u32x4 v = *reinterpret_cast<const u32x4*>(smem + row * (2 * TN) + ((16 * c16) ^ (((row >> 2) & 3) << 5)));
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(a.out_hi + (int64_t)(m0 + row) * a.o_ld + g.o_off + n0 +
                                                                8 * c16));
      }
    }
  }
  }   // tiles
}

// ---------------------------------------------------------------------------------------------
// Flash attention, head dim 64, 4 waves x 32 queries per workgroup, 64-key blocks.
// LDS images per block (bf16 hi / lo): K [64 key][64 d] and V [64 key][64 d], 128-B rows with the
// 16-B chunk index XOR-swizzled by ((row >> 1) & 7) (conflict-free ds_read_b128 groups), both written
// with 8-byte stores.  The V^T A-fragments of O^T += V^T P^T are read with ds_read_b64_tr_b16 (a
// transposing read: 16 lanes get 16 d-columns of 4 key rows), and the key each k-slot needs is chosen
// in the read address, matching the S^T register layout of P^T:
//   k-slot 8 h + 4 r + q of k-step ks  <->  key 32 (ks >> 1) + 16 (ks & 1) + 8 r + 4 h + q.
constexpr int kHD = 64;
constexpr int kKB = 64;

__device__ __forceinline__ int swz(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }

template <bool X3, bool PRE = false>
__global__ void __launch_bounds__(kThreads, 2) attn_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[4 * kKB * kHD * 2];
  char* Khi = smem;
  char* Klo = smem + kKB * kHD * 2;
  char* Vhi = smem + 2 * kKB * kHD * 2;
  char* Vlo = smem + 3 * kKB * kHD * 2;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hl = lane >> 5;
  const int head = blockIdx.y;
  const int seq = blockIdx.z;
  const int64_t sbase = (int64_t)(seq / a.sdiv) * a.smul_a + (int64_t)(seq % a.sdiv) * a.smul_b;
  auto token = [&](int p) -> int64_t { return sbase + (int64_t)p * a.pstride; };
  // keys / values: the same sequence of qkv (self) or sequence `seq` of the kv buffer (cross)
  const float* kvb = a.kv ? a.kv : a.qkv;
  const int64_t kv_ld = a.kv ? a.kv_ld : a.ld;
  const int Lk = a.Lk > 0 ? a.Lk : a.L;
  auto ktoken = [&](int p) -> int64_t { return a.kv ? (int64_t)seq * a.kv_smul + p : token(p); };
  const int dh = a.dh > 0 ? a.dh : kHD;   // <= 64, % 4 == 0: dims >= dh are zero-padded
  const float qscale = dh == kHD ? 0.125f : 1.0f / sqrtf((float)dh);
  const int q_pos = blockIdx.x * 128 + wave * 32 + l32;  // this lane's query
  const bool q_ok = q_pos < a.L;

  // Q fragments (B operand of S^T = K Q^T): lane holds Q[q][16 ks + 8 hl + j] / sqrt(dh), split
  bf16x8 qh[4], ql[4];
  if constexpr (PRE) {
    // planes: hi + lo of q, then (q * qscale) split again -- for dh = 64 (qscale = 2^-3) exactly the
    // fp32 path's operands, since the split commutes with a power-of-two scale
    const int64_t qo = token(q_ok ? q_pos : 0) * a.ld + head * dh;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int d0 = 16 * ks + 8 * hl;
      uint4 hv = make_uint4(0u, 0u, 0u, 0u), lv = make_uint4(0u, 0u, 0u, 0u);
      if (q_ok && d0 < dh) {   // dh % 8 == 0 on this path (host check)
        hv = *reinterpret_cast<const uint4*>(a.qkv_hi + qo + d0);
        if (a.qkv_lo) lv = *reinterpret_cast<const uint4*>(a.qkv_lo + qo + d0);
      }
      const uint32_t hw[4] = {hv.x, hv.y, hv.z, hv.w}, lw[4] = {lv.x, lv.y, lv.z, lv.w};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float vh = __uint_as_float((j & 1) ? (hw[j >> 1] & 0xffff0000u) : (hw[j >> 1] << 16));
        const float vl = __uint_as_float((j & 1) ? (lw[j >> 1] & 0xffff0000u) : (lw[j >> 1] << 16));
        const float v = (vh + vl) * qscale;
        __bf16 hi, lo;
        split_bf16(v, hi, lo);
        qh[ks][j] = hi;
        ql[ks][j] = lo;
      }
    }
  } else {
    const float* qp = a.qkv + token(q_ok ? q_pos : 0) * a.ld + head * dh;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int d0 = 16 * ks + 8 * hl;
      const f32x4 v0 = q_ok && d0 < dh ? *reinterpret_cast<const f32x4*>(qp + d0) : f32x4{0.f, 0.f, 0.f, 0.f};
      const f32x4 v1 = q_ok && d0 + 4 < dh ? *reinterpret_cast<const f32x4*>(qp + d0 + 4) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float v = (j < 4 ? v0[j] : v1[j - 4]) * qscale;  // 1/sqrt(64) = 0.125 exactly
        __bf16 hi, lo;
        split_bf16(v, hi, lo);
        qh[ks][j] = hi;
        ql[ks][j] = lo;
      }
    }
  }

  f32x16 o[2];  // O^T [d = 32 db + row][q = lane column]
#pragma unroll
  for (int db = 0; db < 2; ++db)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[db][r] = 0.f;
  float m_run = -INFINITY, l_run = 0.f;

  // staging: 64 keys x 64 d of K and of V (fp32) = 2 x 1024 f32x4; 8 per thread.  PRE: the same
  // (key, 4-d quad) items as bf16 hi / lo pairs (8 B each), copied to LDS without a split
  f32x4 kreg[PRE ? 1 : 4], vreg[PRE ? 1 : 4];
  uint2 kh2[PRE ? 4 : 1], kl2[PRE ? 4 : 1], vh2[PRE ? 4 : 1], vl2[PRE ? 4 : 1];
  const uint16_t* kvh = a.kv ? a.kv_hi : a.qkv_hi;
  const uint16_t* kvl = a.kv ? a.kv_lo : a.qkv_lo;
  auto load_block = [&](int kb) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + i * kThreads;  // (key, 4-d quad): 64 keys x 16 quads
      const int key = e >> 4, dq = (e & 15) * 4;
      const int p = kb * kKB + key;
      const bool ok = p < Lk && dq < dh;
      const int64_t ro = ktoken(ok ? p : 0) * kv_ld + head * dh + (ok ? dq : 0);
      if constexpr (PRE) {
        const uint2 z = make_uint2(0u, 0u);
        kh2[i] = ok ? *reinterpret_cast<const uint2*>(kvh + ro + a.k_off) : z;
        vh2[i] = ok ? *reinterpret_cast<const uint2*>(kvh + ro + a.v_off) : z;
        if (X3) {
          kl2[i] = ok && kvl ? *reinterpret_cast<const uint2*>(kvl + ro + a.k_off) : z;
          vl2[i] = ok && kvl ? *reinterpret_cast<const uint2*>(kvl + ro + a.v_off) : z;
        }
      } else {
        const float* row = kvb + ro;
        kreg[i] = ok ? *reinterpret_cast<const f32x4*>(row + a.k_off) : f32x4{0.f, 0.f, 0.f, 0.f};
        vreg[i] = ok ? *reinterpret_cast<const f32x4*>(row + a.v_off) : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  };
  auto store_block = [&]() {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + i * kThreads;
      const int key = e >> 4, dq = (e & 15) * 4;
      const int off = swz(key, dq >> 3) + ((dq & 4) << 1);
      if constexpr (PRE) {
        *reinterpret_cast<uint2*>(Khi + off) = kh2[i];
        *reinterpret_cast<uint2*>(Vhi + off) = vh2[i];
        if (X3) {
          *reinterpret_cast<uint2*>(Klo + off) = kl2[i];
          *reinterpret_cast<uint2*>(Vlo + off) = vl2[i];
        }
        continue;
      }
      __bf16 hi[4], lo[4], vh[4], vl[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        split_bf16(kreg[i][q], hi[q], lo[q]);
        split_bf16(vreg[i][q], vh[q], vl[q]);
      }
      *reinterpret_cast<uint2*>(Khi + off) = make_uint2(pack2(hi[0], hi[1]), pack2(hi[2], hi[3]));
      *reinterpret_cast<uint2*>(Vhi + off) = make_uint2(pack2(vh[0], vh[1]), pack2(vh[2], vh[3]));
      if (X3) {
        *reinterpret_cast<uint2*>(Klo + off) = make_uint2(pack2(lo[0], lo[1]), pack2(lo[2], lo[3]));
        *reinterpret_cast<uint2*>(Vlo + off) = make_uint2(pack2(vl[0], vl[1]), pack2(vl[2], vl[3]));
      }
    }
  };
  // V^T fragment of k-step ks, d-block db (see the image comment): two transposing reads
  const int tg = lane >> 4, ti = lane & 15;
  const int tr_q = ti >> 2, tp = ti & 3, th = tg >> 1;
  auto vt_frag = [&](const char* V, int ks, int db) -> bf16x8 {
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    const int d = db * 32 + 16 * (tg & 1) + 4 * tp;
    const int key0 = 32 * (ks >> 1) + 16 * (ks & 1) + 4 * th + tr_q;
    // whole-vector assembly: element-wise short -> bf16 inserts miscompiled (every element became
    // element 0; tools/tr_probe2.hip)
    const bf16x4 t0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
        (__attribute__((address_space(3))) bf16x4*)(V + swz(key0, d >> 3) + ((d & 7) << 1)));
    const bf16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
        (__attribute__((address_space(3))) bf16x4*)(V + swz(key0 + 8, d >> 3) + ((d & 7) << 1)));
    return __builtin_shufflevector(t0, t1, 0, 1, 2, 3, 4, 5, 6, 7);
  };

  const int n_blocks = (Lk + kKB - 1) / kKB;
  load_block(0);
  for (int kb = 0; kb < n_blocks; ++kb) {
    __syncthreads();
    store_block();
    __syncthreads();
    if (kb + 1 < n_blocks) load_block(kb + 1);

    // S^T [key][q] for the block's 2 x 32 keys
    f32x16 s[2];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
#pragma unroll
      for (int r = 0; r < 16; ++r) s[rb][r] = 0.f;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int key = rb * 32 + l32;
        const int off = swz(key, 2 * ks + hl);
        const bf16x8 kh = *reinterpret_cast<const bf16x8*>(Khi + off);
        if (X3) {
          const bf16x8 kl = *reinterpret_cast<const bf16x8*>(Klo + off);
          s[rb] = mfma32(kl, qh[ks], s[rb]);
          s[rb] = mfma32(kh, ql[ks], s[rb]);
        }
        s[rb] = mfma32(kh, qh[ks], s[rb]);
      }
    }
    // online softmax (per lane = per query); keys past L are masked
    float bmax = -INFINITY;
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kb * kKB + rb * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
        if (key >= Lk) s[rb][r] = -INFINITY;
        bmax = fmaxf(bmax, s[rb][r]);
      }
    bmax = fmaxf(bmax, __shfl_xor(bmax, 32));
    const float m_new = fmaxf(m_run, bmax);
    const float alpha = __expf(m_run - m_new);
    float psum = 0.f;
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = __expf(s[rb][r] - m_new);
        s[rb][r] = p;
        psum += p;
      }
    psum += __shfl_xor(psum, 32);
    l_run = l_run * alpha + psum;
    m_run = m_new;
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[db][r] *= alpha;
    // O^T += V^T P^T: k-step ks covers keys 16 ks .. +15 = regs 8 (ks & 1) .. +7 of s[ks >> 1]
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      bf16x8 ph, pl;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float p = s[ks >> 1][8 * (ks & 1) + j];
        __bf16 hi, lo;
        split_bf16(p, hi, lo);
        ph[j] = hi;
        pl[j] = lo;
      }
#pragma unroll
      for (int db = 0; db < 2; ++db) {
        const bf16x8 vh = vt_frag(Vhi, ks, db);
        if (X3) {
          const bf16x8 vl = vt_frag(Vlo, ks, db);
          o[db] = mfma32(vl, ph, o[db]);
          o[db] = mfma32(vh, pl, o[db]);
        }
        o[db] = mfma32(vh, ph, o[db]);
      }
    }
  }

  if (!q_ok) return;
  const int64_t tq = token(q_pos);
  float glogit = 0.f;
  if (a.g_off >= 0) {
    if constexpr (PRE) {
      const int64_t go = tq * a.ld + a.g_off + head;
      glogit = __uint_as_float((uint32_t)a.qkv_hi[go] << 16) +
               (a.qkv_lo ? __uint_as_float((uint32_t)a.qkv_lo[go] << 16) : 0.f);
    } else {
      glogit = a.qkv[tq * a.ld + a.g_off + head];
    }
  }
  const float gate = a.g_off >= 0 ? sigmoidf_(glogit) : 1.f;
  const float scale = gate / l_run;
  const int64_t obase = tq * a.o_ld + head * dh;
#pragma unroll
  for (int db = 0; db < 2; ++db)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const int d = db * 32 + 8 * g4 + 4 * hl;
      if (d >= dh) continue;
      f32x4 v;
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = o[db][4 * g4 + q] * scale;
      if (a.out_hi) {
        __bf16 hi[4], lo[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) split_bf16(v[q], hi[q], lo[q]);
        *reinterpret_cast<uint2*>(a.out_hi + obase + d) = make_uint2(pack2(hi[0], hi[1]), pack2(hi[2], hi[3]));
        if (a.out_lo)
          *reinterpret_cast<uint2*>(a.out_lo + obase + d) = make_uint2(pack2(lo[0], lo[1]), pack2(lo[2], lo[3]));
      } else {
        *reinterpret_cast<f32x4*>(a.out + obase + d) = v;
      }
    }
}

// ---------------------------------------------------------------------------------------------
// attn_f16_kernel: the same flash attention (S^T = K Q^T, P^T from registers, V^T by transposing LDS
// reads, gates in the epilogue) with QK^T and PV on ONE v_mfma_f32_32x32x16_f16 pass each: q / sqrt(dh),
// k, v and the block's P = exp(s - m) rounded once to fp16, softmax statistics (m, l) and the O accumulator
// in fp32 (CPU emulation on the BS-Roformer vocals chunk: 3.0e-7 RMS, tests/emulation/emulate_bsr_attn16.py).
// The fp16 K / V images are half the bf16 hi + lo pair, so K / V are DOUBLE-BUFFERED in the same 32 KiB:
// block kb + 1 is converted and stored into the other stage under block kb's MFMAs, block kb + 2 loads
// into registers, one barrier per block (the bf16x3 kernel: single stage, two barriers).
// Output: fp32 rows, or (out_f16) one fp16 plane -- the A operand of the fp16 out-projection.
__device__ __forceinline__ f32x16 mfma32h_(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                0);
}
__device__ __forceinline__ uint32_t pack2h_(float a, float b) {
  return (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)a) | ((uint32_t)__builtin_bit_cast(uint16_t, (_Float16)b) << 16);
}

// NW: waves per workgroup (32 queries each): 4 (128 queries) for long sequences, 2 (64 queries) where L <= 64
// (BS-Roformer's band attention, L = 62: a 128-query tile would compute half of its MFMAs on padding).
// H16: q / k / v / gates from the fp16 plane a.qkv16 (the rounding the fp32 path does here, done by the QKV
// epilogue; the gate logit is the fp16-rounded one)
template <int NW, bool H16 = false>
__global__ void __launch_bounds__(NW * 64, 2) attn_f16_kernel(AttnArgs a) {
  constexpr int NTH = NW * 64, QB = NW * 32, NIT = kKB * 16 / NTH;   // staging items per thread
  constexpr int IMG = kKB * kHD * 2;                      // one fp16 [64 key][64 d] image
  __shared__ __attribute__((aligned(16))) char smem[4 * IMG];   // [stage][K, V]
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hl = lane >> 5;
  const int head = blockIdx.y;
  const int seq = blockIdx.z;
  const int64_t sbase = (int64_t)(seq / a.sdiv) * a.smul_a + (int64_t)(seq % a.sdiv) * a.smul_b;
  auto token = [&](int p) -> int64_t { return sbase + (int64_t)p * a.pstride; };
  const float* kvb = a.kv ? a.kv : a.qkv;
  const int64_t kv_ld = a.kv ? a.kv_ld : a.ld;
  const int Lk = a.Lk > 0 ? a.Lk : a.L;
  auto ktoken = [&](int p) -> int64_t { return a.kv ? (int64_t)seq * a.kv_smul + p : token(p); };
  const int dh = a.dh > 0 ? a.dh : kHD;
  const float qscale = dh == kHD ? 0.125f : 1.0f / sqrtf((float)dh);
  const int q_pos = blockIdx.x * QB + wave * 32 + l32;
  const bool q_ok = q_pos < a.L;

  bf16x8 qf[4];   // fp16 bits: Q[q][16 ks + 8 hl + j] / sqrt(dh)
  if constexpr (H16) {
    const uint16_t* qp = a.qkv16 + token(q_ok ? q_pos : 0) * a.ld + head * dh;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int d0 = 16 * ks + 8 * hl;
      u32x4 w = {0u, 0u, 0u, 0u};
      if (q_ok && d0 < dh) {
        const u32x4 raw = *reinterpret_cast<const u32x4*>(qp + d0);   // dh % 8 == 0 (host check)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float lo = (float)__builtin_bit_cast(_Float16, (uint16_t)(raw[e] & 0xffffu));
          const float hi = (float)__builtin_bit_cast(_Float16, (uint16_t)(raw[e] >> 16));
          w[e] = pack2h_(lo * qscale, hi * qscale);
        }
      }
      qf[ks] = __builtin_bit_cast(bf16x8, w);
    }
  } else {
    const float* qp = a.qkv + token(q_ok ? q_pos : 0) * a.ld + head * dh;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int d0 = 16 * ks + 8 * hl;
      const f32x4 v0 = q_ok && d0 < dh ? *reinterpret_cast<const f32x4*>(qp + d0) : f32x4{0.f, 0.f, 0.f, 0.f};
      const f32x4 v1 = q_ok && d0 + 4 < dh ? *reinterpret_cast<const f32x4*>(qp + d0 + 4) : f32x4{0.f, 0.f, 0.f, 0.f};
      const u32x4 w = {pack2h_(v0[0] * qscale, v0[1] * qscale), pack2h_(v0[2] * qscale, v0[3] * qscale),
                       pack2h_(v1[0] * qscale, v1[1] * qscale), pack2h_(v1[2] * qscale, v1[3] * qscale)};
      qf[ks] = __builtin_bit_cast(bf16x8, w);
    }
  }
  f32x16 o[2];
#pragma unroll
  for (int db = 0; db < 2; ++db)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[db][r] = 0.f;
  float m_run = -INFINITY, l_run = 0.f;

  f32x4 kreg[H16 ? 1 : NIT], vreg[H16 ? 1 : NIT];
  uint2 kreg16[H16 ? NIT : 1], vreg16[H16 ? NIT : 1];   // H16: 4 fp16 per item, stored as loaded
  auto load_block = [&](int kb) {
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      const int e = tid + i * NTH;
      const int key = e >> 4, dq = (e & 15) * 4;
      const int p = kb * kKB + key;
      const bool ok = p < Lk && dq < dh;
      if constexpr (H16) {
        const uint16_t* row = (a.kv16 ? a.kv16 + ktoken(ok ? p : 0) * kv_ld : a.qkv16 + token(ok ? p : 0) * a.ld) +
                              head * dh + (ok ? dq : 0);
        kreg16[i] = ok ? *reinterpret_cast<const uint2*>(row + a.k_off) : make_uint2(0u, 0u);
        vreg16[i] = ok ? *reinterpret_cast<const uint2*>(row + a.v_off) : make_uint2(0u, 0u);
      } else {
        const float* row = kvb + ktoken(ok ? p : 0) * kv_ld + head * dh + (ok ? dq : 0);
        kreg[i] = ok ? *reinterpret_cast<const f32x4*>(row + a.k_off) : f32x4{0.f, 0.f, 0.f, 0.f};
        vreg[i] = ok ? *reinterpret_cast<const f32x4*>(row + a.v_off) : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  };
  auto store_block = [&](char* stg) {
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      const int e = tid + i * NTH;
      const int key = e >> 4, dq = (e & 15) * 4;
      const int off = swz(key, dq >> 3) + ((dq & 4) << 1);
      if constexpr (H16) {
        *reinterpret_cast<uint2*>(stg + off) = kreg16[i];
        *reinterpret_cast<uint2*>(stg + IMG + off) = vreg16[i];
      } else {
        *reinterpret_cast<uint2*>(stg + off) =
            make_uint2(pack2h_(kreg[i][0], kreg[i][1]), pack2h_(kreg[i][2], kreg[i][3]));
        *reinterpret_cast<uint2*>(stg + IMG + off) =
            make_uint2(pack2h_(vreg[i][0], vreg[i][1]), pack2h_(vreg[i][2], vreg[i][3]));
      }
    }
  };
  const int tg = lane >> 4, ti = lane & 15;
  const int tr_q = ti >> 2, tp = ti & 3, th = tg >> 1;
  auto vt_frag = [&](const char* V, int ks, int db) -> bf16x8 {
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    const int d = db * 32 + 16 * (tg & 1) + 4 * tp;
    const int key0 = 32 * (ks >> 1) + 16 * (ks & 1) + 4 * th + tr_q;
    // a transposing 16-bit read is a pure data movement: the fp16 bits travel in a bf16 container
    const bf16x4 t0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
        (__attribute__((address_space(3))) bf16x4*)(V + swz(key0, d >> 3) + ((d & 7) << 1)));
    const bf16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
        (__attribute__((address_space(3))) bf16x4*)(V + swz(key0 + 8, d >> 3) + ((d & 7) << 1)));
    return __builtin_shufflevector(t0, t1, 0, 1, 2, 3, 4, 5, 6, 7);
  };

  const int n_blocks = (Lk + kKB - 1) / kKB;
  load_block(0);
  store_block(smem);
  if (n_blocks > 1) load_block(1);
  __syncthreads();
  for (int kb = 0; kb < n_blocks; ++kb) {
    const char* K = smem + (kb & 1) * 2 * IMG;
    const char* V = K + IMG;
    f32x16 s[2];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
#pragma unroll
      for (int r = 0; r < 16; ++r) s[rb][r] = 0.f;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(K + swz(rb * 32 + l32, 2 * ks + hl));
        s[rb] = mfma32h_(kf, qf[ks], s[rb]);
      }
    }
    // stage block kb + 1 (in registers since the previous iteration) into the other buffer -- every wave
    // finished reading it before the previous iteration's barrier -- then start loading block kb + 2
    if (kb + 1 < n_blocks) {
      store_block(smem + ((kb + 1) & 1) * 2 * IMG);
      if (kb + 2 < n_blocks) load_block(kb + 2);
    }
    // keys past Lk exist only in the last block (uniform branch: the full blocks skip 32 compare / selects)
    if ((kb + 1) * kKB > Lk) {
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = kb * kKB + rb * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
          if (key >= Lk) s[rb][r] = -INFINITY;
        }
    }
    float bmax = -INFINITY;
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int r = 0; r < 16; ++r) bmax = fmaxf(bmax, s[rb][r]);
    bmax = fmaxf(bmax, __shfl_xor(bmax, 32));
    // lazy rescale: the running max m (and with it O and l) moves only when a block's max exceeds it by more than
    // 8, so between rescales P = exp(s - m) <= e^8 ~ 2981 (well inside fp16) and most blocks skip the 32
    // multiplies of O; O / l is unchanged (P and l carry the same factor).  The two lanes of a query row hold the
    // same bmax and m, so they agree.
    constexpr float kLog2e = 1.4426950408889634f;
    if (bmax > m_run + 8.f) {
      const float alpha = __builtin_amdgcn_exp2f((m_run - bmax) * kLog2e);   // (0 on the first block)
      l_run *= alpha;
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[db][r] *= alpha;
      m_run = bmax;
    }
    // exp(x - m) as exp2(x log2e - m log2e): one fma per element feeding v_exp_f32 (exp2)
    const float ml = m_run * kLog2e;
    float psum = 0.f;
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = __builtin_amdgcn_exp2f(fmaf(s[rb][r], kLog2e, -ml));
        s[rb][r] = p;
        psum += p;
      }
    psum += __shfl_xor(psum, 32);
    l_run += psum;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int r0 = 8 * (ks & 1);
      const f32x16& sv = s[ks >> 1];
      const u32x4 w = {pack2h_(sv[r0], sv[r0 + 1]), pack2h_(sv[r0 + 2], sv[r0 + 3]), pack2h_(sv[r0 + 4], sv[r0 + 5]),
                       pack2h_(sv[r0 + 6], sv[r0 + 7])};
      const bf16x8 pf = __builtin_bit_cast(bf16x8, w);
#pragma unroll
      for (int db = 0; db < 2; ++db) o[db] = mfma32h_(vt_frag(V, ks, db), pf, o[db]);
    }
    __syncthreads();
  }

  if (!q_ok) return;
  const int64_t tq = token(q_pos);
  const float glogit = a.g_off < 0 ? 0.f
                       : H16 ? (float)__builtin_bit_cast(_Float16, a.qkv16[tq * a.ld + a.g_off + head])
                             : a.qkv[tq * a.ld + a.g_off + head];
  const float gate = a.g_off >= 0 ? sigmoidf_(glogit) : 1.f;
  const float scale = gate / l_run;
  const int64_t obase = tq * a.o_ld + head * dh;
#pragma unroll
  for (int db = 0; db < 2; ++db)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const int d = db * 32 + 8 * g4 + 4 * hl;
      if (d >= dh) continue;
      f32x4 v;
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = o[db][4 * g4 + q] * scale;
      if (a.out_hi && a.out_f16) {
        *reinterpret_cast<uint2*>(a.out_hi + obase + d) = make_uint2(pack2h_(v[0], v[1]), pack2h_(v[2], v[3]));
      } else if (a.out_hi) {
        __bf16 hi[4], lo[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) split_bf16(v[q], hi[q], lo[q]);
        *reinterpret_cast<uint2*>(a.out_hi + obase + d) = make_uint2(pack2(hi[0], hi[1]), pack2(hi[2], hi[3]));
        if (a.out_lo)
          *reinterpret_cast<uint2*>(a.out_lo + obase + d) = make_uint2(pack2(lo[0], lo[1]), pack2(lo[2], lo[3]));
      } else {
        *reinterpret_cast<f32x4*>(a.out + obase + d) = v;
      }
    }
}

// ---------------------------------------------------------------------------------------------
// attn_f16_band_kernel<HPW>: BS-Roformer's band attention (self attention over L <= 64 band tokens, dh = 64,
// q / k / v / gates from the fp16 plane, fp16 output plane), HPW heads of one sequence per workgroup: the
// sequence has a single key block, so the per-head work is one QK^T / PV block (16 MFMAs a wave) and the
// one-head-per-workgroup form spent its time on setup and exposed load latency (4 % MFMA-busy).  Here head h + 1's
// Q / K / V are loaded into registers under head h's MFMAs and staged into the other LDS buffer, one barrier
// per head.  Same arithmetic as attn_f16_kernel<2, true> on its single block (bit-identical output).
template <int HPW>
__global__ void __launch_bounds__(128, 2) attn_f16_band_kernel(AttnArgs a) {
  constexpr int NTH = 128, NIT = kKB * 16 / NTH;   // 8 staging items (4 fp16 of K and of V) per thread
  constexpr int IMG = kKB * kHD * 2;                // one fp16 [64 key][64 d] image
  __shared__ __attribute__((aligned(16))) char smem[4 * IMG];   // [buffer][K, V]
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hl = lane >> 5;
  const int head0 = blockIdx.y * HPW;
  const int seq = blockIdx.z;
  const int64_t sbase = (int64_t)(seq / a.sdiv) * a.smul_a + (int64_t)(seq % a.sdiv) * a.smul_b;
  auto token = [&](int p) -> int64_t { return sbase + (int64_t)p * a.pstride; };
  const int L = a.L;
  const int q_pos = wave * 32 + l32;
  const bool q_ok = q_pos < L;
  const uint16_t* qrow = a.qkv16 + token(q_ok ? q_pos : 0) * a.ld;

  u32x4 qraw[4];
  uint2 kr[NIT], vr[NIT];
  auto load = [&](int head) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
      qraw[ks] = q_ok ? *reinterpret_cast<const u32x4*>(qrow + head * kHD + 16 * ks + 8 * hl) : u32x4{0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      const int e = tid + i * NTH;
      const int key = e >> 4, dq = (e & 15) * 4;
      const bool ok = key < L;
      const uint16_t* row = a.qkv16 + token(ok ? key : 0) * a.ld + head * kHD + dq;
      kr[i] = ok ? *reinterpret_cast<const uint2*>(row + a.k_off) : make_uint2(0u, 0u);
      vr[i] = ok ? *reinterpret_cast<const uint2*>(row + a.v_off) : make_uint2(0u, 0u);
    }
  };
  auto store = [&](char* stg) {
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      const int e = tid + i * NTH;
      const int key = e >> 4, dq = (e & 15) * 4;
      const int off = swz(key, dq >> 3) + ((dq & 4) << 1);
      *reinterpret_cast<uint2*>(stg + off) = kr[i];
      *reinterpret_cast<uint2*>(stg + IMG + off) = vr[i];
    }
  };
  bf16x8 qf[4];   // Q / 8 (exact: dh = 64), fp16 bits
  auto q_convert = [&]() {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      u32x4 w;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float lo = (float)__builtin_bit_cast(_Float16, (uint16_t)(qraw[ks][e] & 0xffffu));
        const float hi = (float)__builtin_bit_cast(_Float16, (uint16_t)(qraw[ks][e] >> 16));
        w[e] = pack2h_(lo * 0.125f, hi * 0.125f);
      }
      qf[ks] = __builtin_bit_cast(bf16x8, w);
    }
  };
  const int tg = lane >> 4, ti = lane & 15;
  const int tr_q = ti >> 2, tp = ti & 3, th = tg >> 1;
  auto vt_frag = [&](const char* V, int ks, int db) -> bf16x8 {
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    const int d = db * 32 + 16 * (tg & 1) + 4 * tp;
    const int key0 = 32 * (ks >> 1) + 16 * (ks & 1) + 4 * th + tr_q;
    const bf16x4 t0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
        (__attribute__((address_space(3))) bf16x4*)(V + swz(key0, d >> 3) + ((d & 7) << 1)));
    const bf16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
        (__attribute__((address_space(3))) bf16x4*)(V + swz(key0 + 8, d >> 3) + ((d & 7) << 1)));
    return __builtin_shufflevector(t0, t1, 0, 1, 2, 3, 4, 5, 6, 7);
  };

  load(head0);
  store(smem);
  q_convert();
  __syncthreads();
  for (int hi_ = 0; hi_ < HPW; ++hi_) {
    const int head = head0 + hi_;
    const bf16x8 q0 = qf[0], q1 = qf[1], q2 = qf[2], q3 = qf[3];
    if (hi_ + 1 < HPW) load(head + 1);   // registers only: lands under this head's MFMAs
    const char* K = smem + (hi_ & 1) * 2 * IMG;
    const char* V = K + IMG;
    f32x16 s[2];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
#pragma unroll
      for (int r = 0; r < 16; ++r) s[rb][r] = 0.f;
      s[rb] = mfma32h_(*reinterpret_cast<const bf16x8*>(K + swz(rb * 32 + l32, 0 + hl)), q0, s[rb]);
      s[rb] = mfma32h_(*reinterpret_cast<const bf16x8*>(K + swz(rb * 32 + l32, 2 + hl)), q1, s[rb]);
      s[rb] = mfma32h_(*reinterpret_cast<const bf16x8*>(K + swz(rb * 32 + l32, 4 + hl)), q2, s[rb]);
      s[rb] = mfma32h_(*reinterpret_cast<const bf16x8*>(K + swz(rb * 32 + l32, 6 + hl)), q3, s[rb]);
    }
    if (L < kKB) {
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = rb * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
          if (key >= L) s[rb][r] = -INFINITY;
        }
    }
    float m = -INFINITY;
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int r = 0; r < 16; ++r) m = fmaxf(m, s[rb][r]);
    m = fmaxf(m, __shfl_xor(m, 32));
    constexpr float kLog2e = 1.4426950408889634f;
    const float ml = m * kLog2e;
    float l = 0.f;
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = __builtin_amdgcn_exp2f(fmaf(s[rb][r], kLog2e, -ml));
        s[rb][r] = p;
        l += p;
      }
    l += __shfl_xor(l, 32);
    f32x16 o[2];
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[db][r] = 0.f;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int r0 = 8 * (ks & 1);
      const f32x16& sv = s[ks >> 1];
      const u32x4 w = {pack2h_(sv[r0], sv[r0 + 1]), pack2h_(sv[r0 + 2], sv[r0 + 3]), pack2h_(sv[r0 + 4], sv[r0 + 5]),
                       pack2h_(sv[r0 + 6], sv[r0 + 7])};
      const bf16x8 pf = __builtin_bit_cast(bf16x8, w);
#pragma unroll
      for (int db = 0; db < 2; ++db) o[db] = mfma32h_(vt_frag(V, ks, db), pf, o[db]);
    }
    if (q_ok) {
      const int64_t tq = token(q_pos);
      const float gate =
          a.g_off >= 0 ? sigmoidf_((float)__builtin_bit_cast(_Float16, a.qkv16[tq * a.ld + a.g_off + head])) : 1.f;
      const float scale = gate / l;
      const int64_t obase = tq * a.o_ld + head * kHD;
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int d = db * 32 + 8 * g4 + 4 * hl;
          *reinterpret_cast<uint2*>(a.out_hi + obase + d) =
              make_uint2(pack2h_(o[db][4 * g4] * scale, o[db][4 * g4 + 1] * scale),
                         pack2h_(o[db][4 * g4 + 2] * scale, o[db][4 * g4 + 3] * scale));
        }
    }
    if (hi_ + 1 < HPW) {
      store(smem + ((hi_ + 1) & 1) * 2 * IMG);   // that buffer's last reads were head hi_ - 1's, before the barrier
      q_convert();
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------
// fp32 rows -> bf16 hi / lo planes (+ RMSNorm row scale): one wave per row, f32x4 per lane-step.
// F16: one fp16 plane (round to nearest even) -- the A operand of the fp16 single-pass Linears.  With a
// row_scale output the fp16 plane holds x * row_scale (the RMS-normalised row, |value| <= sqrt(K)), not the raw
// residual stream: a raw |x| > 65504 would round to inf in fp16, and the fp16 GEMMs then skip EP_RS.
template <bool F16>
__global__ void __launch_bounds__(256) tok_split_kernel(const float* __restrict__ x, int64_t x_ld, int64_t M, int K,
                                                        uint16_t* __restrict__ hi, uint16_t* __restrict__ lo,
                                                        int64_t p_ld, float* __restrict__ row_scale) {
  const int lane = threadIdx.x & 63;
  const int64_t m = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;
  const float* xr = x + m * x_ld;
  float ss = 0.f;
  if constexpr (F16) {
    float rs = 1.f;
    if (row_scale) {   // pass 1: the row's sum of squares (the second pass re-reads the row from L1 / L2)
      for (int k = lane * 4; k < K; k += 256) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(xr + k);
#pragma unroll
        for (int q = 0; q < 4; ++q) ss = fmaf(v[q], v[q], ss);
      }
#pragma unroll
      for (int s = 32; s >= 1; s >>= 1) ss += __shfl_xor(ss, s);
      rs = sqrtf((float)K) / fmaxf(sqrtf(ss), 1e-12f);
      if (lane == 0) row_scale[m] = rs;
    }
    for (int k = lane * 4; k < K; k += 256) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(xr + k);
      uint32_t w[2];
#pragma unroll
      for (int q = 0; q < 2; ++q)
        w[q] = (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)(v[2 * q] * rs)) |
               ((uint32_t)__builtin_bit_cast(uint16_t, (_Float16)(v[2 * q + 1] * rs)) << 16);
      *reinterpret_cast<uint2*>(hi + m * p_ld + k) = make_uint2(w[0], w[1]);
    }
    return;
  }
  for (int k = lane * 4; k < K; k += 256) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(xr + k);
    __bf16 h[4], l[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      ss = fmaf(v[q], v[q], ss);
      split_bf16(v[q], h[q], l[q]);
    }
    *reinterpret_cast<uint2*>(hi + m * p_ld + k) = make_uint2(pack2(h[0], h[1]), pack2(h[2], h[3]));
    if (lo) *reinterpret_cast<uint2*>(lo + m * p_ld + k) = make_uint2(pack2(l[0], l[1]), pack2(l[2], l[3]));
  }
  if (row_scale) {
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) ss += __shfl_xor(ss, s);
    if (lane == 0) row_scale[m] = sqrtf((float)K) / fmaxf(sqrtf(ss), 1e-12f);
  }
}

}  // namespace

int launch_tok_gemm(const TokGemmArgs& a, int x3, hipStream_t st) {
  SESA_REQUIRE(a.n_groups >= 1 && a.n_tiles_n >= 1 && a.M >= 0, SESA_ERR_INVALID, "tok_gemm: bad grid");
  SESA_REQUIRE(x3 != 2 || !a.a_hi || !a.conv, SESA_ERR_INVALID, "tok_gemm: fp16 conv gathers take fp32 input");
  SESA_REQUIRE(!(a.out_hi && a.residual) && (a.out_hi || a.out), SESA_ERR_INVALID,
               "tok_gemm: split epilogue takes no residual; an output is required");
  if (a.M == 0) return SESA_OK;
  const int64_t m_tiles = (a.M + 127) / 128;
  SESA_REQUIRE(m_tiles * a.n_tiles_n < (1ll << 31) && a.n_groups < 65536, SESA_ERR_INVALID, "tok_gemm: grid too large");
  dim3 grid((unsigned)(m_tiles * a.n_tiles_n), (unsigned)a.n_groups);
  // variant 0 (default): 256 threads, 128 x 128 tile (4 waves of 64 x 64), single stage, 2 WG / CU
  // variant 1: 512 threads, 256 x 128 tile (8 waves of 64 x 64), double-buffered, 1 WG / CU
  static const int variant = getenv("SESA_TOKGEMM_VARIANT") ? atoi(getenv("SESA_TOKGEMM_VARIANT")) : 0;
  if (a.conv) {
    const ConvGeo& c = a.geo;
    SESA_REQUIRE(a.n_groups == 1 && c.Cin > 0 && c.Cin % 4 == 0 && c.n_taps >= 1 && c.n_taps <= kMaxTaps &&
                     a.x_ld % 4 == 0 && c.P1 > 0 && c.P2 > 0 && c.Q1 > 0 && c.Q2 > 0 && c.phases >= 1 && !a.rope &&
                     !a.rownorm && (int64_t)c.P1 * c.P2 > 0 && (c.phases == 1 || !a.glu),
                 SESA_ERR_INVALID, "tok_gemm conv: bad geometry");
    SESA_REQUIRE((c.phases == 1 && c.oq1 == 0) || c.O1 > 0, SESA_ERR_INVALID, "tok_gemm conv: output rows need O1");
    SESA_REQUIRE(!c.o_fmajor || c.oq1 > 0, SESA_ERR_INVALID, "tok_gemm conv: axis-2-major output needs oq1");
    SESA_REQUIRE(c.xq1 == 0 || (c.x_row0 >= 0 && c.x_row0 + c.Q1 <= c.xq1), SESA_ERR_INVALID,
                 "tok_gemm conv: input sub-range [%d, %d) outside %d rows", c.x_row0, c.x_row0 + c.Q1, c.xq1);
    SESA_REQUIRE(c.oq1 == 0 || (c.o_row0 >= 0 && c.o_row0 + c.O1 <= c.oq1), SESA_ERR_INVALID,
                 "tok_gemm conv: output sub-range [%d, %d) outside %d rows", c.o_row0, c.o_row0 + c.O1, c.oq1);
    SESA_REQUIRE(!a.a_hi, SESA_ERR_INVALID, "tok_gemm conv: pre-split A is for token rows");
    // SESA_HCONV_VARIANT=1: the double-buffered 512-thread 256 x 128 tile for the implicit-GEMM convs (A/B)
    static const int hv = getenv("SESA_HCONV_VARIANT") ? atoi(getenv("SESA_HCONV_VARIANT")) : 0;
    // SESA_HCONV_PD = 1 | 2 | 3: register prefetch depth of the fp16 conv gathers (A/B).  Deeper is slower: same
    // box, HTDemucs hconv 804 / 802 ms per step (PD 1) -> 938 (2) -> 1052 (3) (profiles/r04_hconv_pd_ab_*.json)
    static const int pd = getenv("SESA_HCONV_PD") ? atoi(getenv("SESA_HCONV_PD")) : 1;
    if (x3 == 2 && pd == 2) {
      if (a.bn64)
        hipLaunchKernelGGL((tok_gemm_kernel<false, 256, 128, 2, 2, 1, false, true, false, 64, true, 2>), grid, dim3(256),
                           0, st, a);
      else
        hipLaunchKernelGGL((tok_gemm_kernel<false, 256, 128, 2, 2, 2, false, true, false, 128, true, 2>), grid,
                           dim3(256), 0, st, a);
    } else if (x3 == 2 && pd == 3) {
      if (a.bn64)
        hipLaunchKernelGGL((tok_gemm_kernel<false, 256, 128, 2, 2, 1, false, true, false, 64, true, 3>), grid, dim3(256),
                           0, st, a);
      else
        hipLaunchKernelGGL((tok_gemm_kernel<false, 256, 128, 2, 2, 2, false, true, false, 128, true, 3>), grid,
                           dim3(256), 0, st, a);
    } else if (x3 == 2) {
      // fp16 single pass (fp16 weight images): 64- or 128-column tiles
      if (a.bn64)
        hipLaunchKernelGGL((tok_gemm_kernel<false, 256, 128, 2, 2, 1, false, true, false, 64, true>), grid, dim3(256), 0,
                           st, a);
      else if (hv == 1)
        hipLaunchKernelGGL((tok_gemm_kernel<false, 512, 256, 2, 2, 2, true, true, false, 128, true>),
                           dim3((unsigned)(((a.M + 255) / 256) * a.n_tiles_n)), dim3(512), 0, st, a);
      else
        hipLaunchKernelGGL((tok_gemm_kernel<false, 256, 128, 2, 2, 2, false, true, false, 128, true>), grid, dim3(256),
                           0, st, a);
    } else if (a.bn64) {
      // 64-column tiles (the caller asked for them and counted n_tiles_n in 64-column units)
      if (x3) hipLaunchKernelGGL((tok_gemm_kernel<true, 256, 128, 2, 2, 1, false, true, false, 64>), grid, dim3(256), 0, st, a);
      else hipLaunchKernelGGL((tok_gemm_kernel<false, 256, 128, 2, 2, 1, false, true, false, 64>), grid, dim3(256), 0, st, a);
    } else if (hv == 1) {
      const dim3 g2((unsigned)(((a.M + 255) / 256) * a.n_tiles_n));
      if (x3) hipLaunchKernelGGL((tok_gemm_kernel<true, 512, 256, 2, 2, 2, true, true, false>), g2, dim3(512), 0, st, a);
      else hipLaunchKernelGGL((tok_gemm_kernel<false, 512, 256, 2, 2, 2, true, true, false>), g2, dim3(512), 0, st, a);
    } else if (x3) {
      hipLaunchKernelGGL((tok_gemm_kernel<true, 256, 128, 2, 2, 2, false, true, false>), grid, dim3(256), 0, st, a);
    } else {
      hipLaunchKernelGGL((tok_gemm_kernel<false, 256, 128, 2, 2, 2, false, true, false>), grid, dim3(256), 0, st, a);
    }
  } else if (a.a_hi) {
    SESA_REQUIRE(a.a_ld % 4 == 0 && (x3 != 1 || a.a_lo) && (!a.rownorm || a.row_scale), SESA_ERR_INVALID,
                 "tok_gemm: pre-split A needs a_ld %% 4 == 0, the lo plane for bf16x3, row_scale for rownorm");
    // LDS-DMA kernel for the bf16x3 transformer Linears (every group's K % 8 == 0, epilogue one of
    // the specialised forms); SESA_TOKGEMM_GLDS=0 selects the register-staged kernel for A/B runs
    static const int glds = getenv("SESA_TOKGEMM_GLDS") ? atoi(getenv("SESA_TOKGEMM_GLDS")) : 1;
    int ep = -1;
    // x3 == 2: fp16 A planes x fp16 weight images, one pass (SESA_PREC_F16 Linears; LDS-DMA kernel only).
    // A rownorm fp16 A plane is already row-scaled by tok_split_kernel<true>, so those epilogues skip EP_RS.
    const bool f16 = x3 == 2;
    if ((glds || f16) && x3 && a.k8 && a.a_ld % 8 == 0 && !a.glu && !a.conv && a.o_ld % 4 == 0 &&
        (a.act == TOK_ACT_NONE || a.act == TOK_ACT_GELU) && (!a.rope || (a.dim_head == 64 && !a.residual)) &&
        (!a.out_hi || a.out_lo || f16) && (!a.residual || a.n4)) {
      ep = (a.rownorm && !f16 ? EP_RS : 0) | (a.rope ? EP_ROPE : 0) | (a.act == TOK_ACT_GELU ? EP_GELU : 0) |
           (a.residual ? EP_RES : 0) | (a.out_hi ? EP_SPLIT : 0) | (f16 ? EP_F16 : 0);
    }
    const dim3 gbig((unsigned)(((a.M + 255) / 256) * ((a.n_tiles_n + 1) / 2)), (unsigned)a.n_groups);
    static const int m16 = getenv("SESA_TOKGEMM_M16") ? atoi(getenv("SESA_TOKGEMM_M16")) : 1;
#define SESA_GLDS(EPV)                                                                                 \
  if (m16) hipLaunchKernelGGL((tok_gemm_glds_kernel<EPV, true>), gbig, dim3(512), 0, st, a);            \
  else hipLaunchKernelGGL((tok_gemm_glds_kernel<EPV, false>), gbig, dim3(512), 0, st, a);
    // fp16: the compact-stage ring, DEPTH - 1 chunks in flight (SESA_TOKGEMM_DEPTH = 2 | 3 | 4; 16x16x32 only).
    // Depth 3 by default: same box, BS-Roformer 189.2x (2) -> 194.0x (3), 192.2x (4); outputs bit-identical
    // (profiles/r04_tokgemm_bench_f16.txt, r04_bsr_depth_*.json)
    static const int depth = [] {
      const int d = getenv("SESA_TOKGEMM_DEPTH") ? atoi(getenv("SESA_TOKGEMM_DEPTH")) : 3;
      return d == 3 || d == 4 ? d : 2;
    }();
    // the half tile (256 x 128, 256 threads, two workgroups per CU) on a depth-3 ring, by default: same box,
    // BS-Roformer 193.0 / 193.0x -> 195.3 / 194.8x, and 190.3 / 190.3x -> 195.0 / 195.7x with the LDS-staged FF1
    // output (profiles/r04_bsr_halftile_ab_*.json, r04_bsr_ff1stage_ab_*.json); SESA_TOKGEMM_HT=0: 256 x 256
    static const bool ht = !(getenv("SESA_TOKGEMM_HT") && std::string(getenv("SESA_TOKGEMM_HT")) == "0");
    const dim3 ght((unsigned)(((a.M + 255) / 256) * a.n_tiles_n), (unsigned)a.n_groups);
    // SESA_TOKGEMM_PERS=1: the half tile as a persistent grid of two workgroups per CU, the second slot delayed by
    // SESA_TOKGEMM_STAGGER x 8128 cycles (tok_gemm_glds_kernel<PERS>; A/B)
    static const bool pers = getenv("SESA_TOKGEMM_PERS") && std::string(getenv("SESA_TOKGEMM_PERS")) == "1";
    static const int stagger = getenv("SESA_TOKGEMM_STAGGER") ? atoi(getenv("SESA_TOKGEMM_STAGGER")) : 1;
    static const int n_cu = [] {
      int d = 0, n = 0;
      (void)hipGetDevice(&d);
      (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d);
      return n > 0 ? n : 256;
    }();
    TokGemmArgs ap = a;
    const bool use_pers = pers && ght.x > 2u * (unsigned)n_cu && (2 * n_cu) % 8 == 0;
    const dim3 gpers((unsigned)(2 * n_cu), (unsigned)a.n_groups);
    if (use_pers) {
      ap.pers_tiles = (int)ght.x;
      ap.stagger = stagger;
    }
#define SESA_GLDS16(EPV)                                                                                   \
  if (m16 && ht && use_pers) hipLaunchKernelGGL((tok_gemm_glds_kernel<EPV, true, 3, true, true>), gpers, dim3(256), 0, st, ap); \
  else if (m16 && ht) hipLaunchKernelGGL((tok_gemm_glds_kernel<EPV, true, 3, true>), ght, dim3(256), 0, st, a);    \
  else if (m16 && depth == 4) hipLaunchKernelGGL((tok_gemm_glds_kernel<EPV, true, 4>), gbig, dim3(512), 0, st, a); \
  else if (m16 && depth == 3) hipLaunchKernelGGL((tok_gemm_glds_kernel<EPV, true, 3>), gbig, dim3(512), 0, st, a); \
  else SESA_GLDS(EPV)
    switch (ep) {
      case 0: SESA_GLDS(0) break;
      case EP_RS | EP_ROPE: SESA_GLDS(EP_RS | EP_ROPE) break;
      case EP_RES: SESA_GLDS(EP_RES) break;
      case EP_RS | EP_GELU | EP_SPLIT: SESA_GLDS(EP_RS | EP_GELU | EP_SPLIT) break;
      case EP_GELU | EP_SPLIT: SESA_GLDS(EP_GELU | EP_SPLIT) break;
      case EP_SPLIT: SESA_GLDS(EP_SPLIT) break;                       // q / k / v planes for attention
      case EP_RS | EP_ROPE | EP_SPLIT: SESA_GLDS(EP_RS | EP_ROPE | EP_SPLIT) break;
      case EP_F16 | EP_GELU | EP_SPLIT: SESA_GLDS16(EP_F16 | EP_GELU | EP_SPLIT) break;  // FF1 (A pre-scaled)
      case EP_F16 | EP_RES: SESA_GLDS16(EP_F16 | EP_RES) break;                                         // FF2
      case EP_F16 | EP_ROPE: SESA_GLDS16(EP_F16 | EP_ROPE) break;                       // QKV (A pre-scaled)
      case EP_F16 | EP_ROPE | EP_SPLIT: SESA_GLDS16(EP_F16 | EP_ROPE | EP_SPLIT) break;   // QKV -> fp16 plane
      case EP_F16: SESA_GLDS16(EP_F16) break;                                   // fp32 rows out
      case EP_F16 | EP_SPLIT: SESA_GLDS16(EP_F16 | EP_SPLIT) break;             // HTDemucs q / kv -> fp16 planes
      default: ep = -1;
    }
    SESA_REQUIRE(!f16 || ep >= 0, SESA_ERR_INVALID, "tok_gemm: no fp16 kernel for this epilogue / shape");
#undef SESA_GLDS16
#undef SESA_GLDS
    if (ep >= 0) {
      SESA_CHECK_LAUNCH();
      return SESA_OK;
    }
    if (x3) hipLaunchKernelGGL((tok_gemm_kernel<true, 256, 128, 2, 2, 2, false, false, true>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((tok_gemm_kernel<false, 256, 128, 2, 2, 2, false, false, true>), grid, dim3(256), 0, st, a);
  } else if (x3 == 2) {
    // fp32 rows rounded once to fp16 in the staging, fp16 weight images, one pass
    hipLaunchKernelGGL((tok_gemm_kernel<false, 256, 128, 2, 2, 2, false, false, false, 128, true>), grid, dim3(256), 0,
                       st, a);
  } else if (variant == 1) {
    const int64_t mt = (a.M + 255) / 256;
    dim3 g1((unsigned)(mt * a.n_tiles_n), (unsigned)a.n_groups);
    if (x3) hipLaunchKernelGGL((tok_gemm_kernel<true, 512, 256, 2, 2, 2, true, false, false>), g1, dim3(512), 0, st, a);
    else hipLaunchKernelGGL((tok_gemm_kernel<false, 512, 256, 2, 2, 2, true, false, false>), g1, dim3(512), 0, st, a);
  } else {
    if (x3) hipLaunchKernelGGL((tok_gemm_kernel<true, 256, 128, 2, 2, 2, false, false, false>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((tok_gemm_kernel<false, 256, 128, 2, 2, 2, false, false, false>), grid, dim3(256), 0, st, a);
  }
  SESA_CHECK_LAUNCH();
  return SESA_OK;
}

int launch_tok_split(const float* x, int64_t x_ld, int64_t M, int K, uint16_t* hi, uint16_t* lo, int64_t p_ld,
                     float* row_scale, hipStream_t st) {
  SESA_REQUIRE(x && hi && M >= 0 && K > 0 && K % 4 == 0 && x_ld % 4 == 0 && p_ld % 4 == 0 && p_ld >= K &&
                   (M + 3) / 4 < (1ll << 31),
               SESA_ERR_INVALID, "tok_split: bad shape");
  if (M == 0) return SESA_OK;
  hipLaunchKernelGGL(tok_split_kernel<false>, dim3((unsigned)((M + 3) / 4)), dim3(256), 0, st, x, x_ld, M, K, hi, lo,
                     p_ld, row_scale);
  SESA_CHECK_LAUNCH();
  return SESA_OK;
}

int launch_tok_split_f16(const float* x, int64_t x_ld, int64_t M, int K, uint16_t* hi, int64_t p_ld, float* row_scale,
                         hipStream_t st) {
  SESA_REQUIRE(x && hi && M >= 0 && K > 0 && K % 4 == 0 && x_ld % 4 == 0 && p_ld % 4 == 0 && p_ld >= K &&
                   (M + 3) / 4 < (1ll << 31),
               SESA_ERR_INVALID, "tok_split_f16: bad shape");
  if (M == 0) return SESA_OK;
  hipLaunchKernelGGL(tok_split_kernel<true>, dim3((unsigned)((M + 3) / 4)), dim3(256), 0, st, x, x_ld, M, K, hi,
                     nullptr, p_ld, row_scale);
  SESA_CHECK_LAUNCH();
  return SESA_OK;
}

int launch_attention(const AttnArgs& a, int x3, hipStream_t st) {
  SESA_REQUIRE(a.L >= 1 && a.n_seq >= 1 && a.heads >= 1 && a.sdiv >= 1 && a.Lk >= 0 && a.dh >= 0 && a.dh <= kHD &&
                   a.dh % 4 == 0 && (!a.kv || a.kv_ld % 4 == 0) && (!a.out_hi || a.o_ld % 4 == 0),
               SESA_ERR_INVALID, "attention: bad shape");
  SESA_REQUIRE(a.n_seq < 65536 * 4 && a.heads < 65536, SESA_ERR_INVALID, "attention: grid too large");
  dim3 grid((unsigned)((a.L + 127) / 128), (unsigned)a.heads, (unsigned)a.n_seq);
  const bool pre = a.qkv_hi != nullptr;
  SESA_REQUIRE(!pre || ((!a.kv || a.kv_hi) && (a.dh == 0 || a.dh % 8 == 0) && a.ld % 8 == 0 && a.k_off % 4 == 0 &&
                        a.v_off % 4 == 0 && (!x3 || (a.qkv_lo && (!a.kv || a.kv_lo)))),
               SESA_ERR_INVALID, "attention: pre-split planes need dh %% 8, 8-B aligned offsets and the lo planes");
  // x3 == 2: QK^T and PV on one fp16 pass (fp32 QKV rows; SESA_PREC_F16 of BS- / Mel-Band-Roformer)
  SESA_REQUIRE(x3 != 2 || !pre, SESA_ERR_INVALID, "attention: the fp16 kernel reads fp32 q / k / v rows");
  SESA_REQUIRE(!a.out_f16 || (a.out_hi && x3 == 2), SESA_ERR_INVALID, "attention: fp16 output plane from the fp16 kernel");
  SESA_REQUIRE(!a.qkv16 || (x3 == 2 && (!a.kv || (a.kv16 && a.kv_ld % 4 == 0)) && (a.dh == 0 || a.dh % 8 == 0) &&
                            a.ld % 4 == 0 && a.k_off % 4 == 0 && a.v_off % 4 == 0),
               SESA_ERR_INVALID, "attention: fp16 q / k / v planes (fp16 kernel; cross attention needs kv16), dh %% 8, "
               "8-B aligned");
  if (x3 == 2) {
    const dim3 g64((unsigned)((a.L + 63) / 64), (unsigned)a.heads, (unsigned)a.n_seq);
    // band attention (single key block): heads looped per workgroup, SESA_ATTN_BAND_HPW = 1 (off) | 2 | 4 | 8.
    // Same box, attention class 171.1 (1) -> 165.9 (2) / 167.2-168.3 (4) / 169.6 (8) ms per step, output
    // bit-identical (profiles/r04_attn_band_hpw*.json)
    static const int hpw = [] {
      const int v = getenv("SESA_ATTN_BAND_HPW") ? atoi(getenv("SESA_ATTN_BAND_HPW")) : 2;
      return v == 2 || v == 4 || v == 8 ? v : 1;
    }();
    if (hpw > 1 && a.qkv16 && !a.kv && a.L <= kKB && (a.Lk == 0 || a.Lk == a.L) && (a.dh == 0 || a.dh == kHD) &&
        a.out_hi && a.out_f16 && a.heads % hpw == 0) {
      const dim3 gb(1u, (unsigned)(a.heads / hpw), (unsigned)a.n_seq);
      if (hpw == 2) hipLaunchKernelGGL(attn_f16_band_kernel<2>, gb, dim3(128), 0, st, a);
      else if (hpw == 4) hipLaunchKernelGGL(attn_f16_band_kernel<4>, gb, dim3(128), 0, st, a);
      else hipLaunchKernelGGL(attn_f16_band_kernel<8>, gb, dim3(128), 0, st, a);
    } else if (a.qkv16) {
      if (a.L <= 64) hipLaunchKernelGGL((attn_f16_kernel<2, true>), g64, dim3(128), 0, st, a);
      else hipLaunchKernelGGL((attn_f16_kernel<4, true>), grid, dim3(kThreads), 0, st, a);
    } else if (a.L <= 64) {
      hipLaunchKernelGGL(attn_f16_kernel<2>, g64, dim3(128), 0, st, a);
    } else {
      hipLaunchKernelGGL(attn_f16_kernel<4>, grid, dim3(kThreads), 0, st, a);
    }
  } else if (pre) {
    if (x3) hipLaunchKernelGGL((attn_kernel<true, true>), grid, dim3(kThreads), 0, st, a);
    else hipLaunchKernelGGL((attn_kernel<false, true>), grid, dim3(kThreads), 0, st, a);
  } else if (x3) {
    hipLaunchKernelGGL((attn_kernel<true, false>), grid, dim3(kThreads), 0, st, a);
  } else {
    hipLaunchKernelGGL((attn_kernel<false, false>), grid, dim3(kThreads), 0, st, a);
  }
  SESA_CHECK_LAUNCH();
  return SESA_OK;
}

}  // namespace sesa
