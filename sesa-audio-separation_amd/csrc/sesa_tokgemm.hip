// Token-major MFMA contractions for the transformer models (BS-Roformer) on gfx950.
//
// tok_gemm_kernel -- Y[m, n] = epi( sum_k X[m, k] * W[n, k] ) for the Linear layers of
//   bs_roformer.py: BandSplit (:222-249, grouped over the 62 bands), Attention.to_qkv + to_gates
//   (:97-99, one GEMM, rotary applied to q/k in the epilogue, :111-113), to_out (:101-104, +
//   residual :214), FeedForward (:55-74, GELU / + residual :215), MaskEstimator MLPs (:277-310,
//   grouped, Tanh and GLU in the epilogues).  RMSNorm (:43-50) is fused: gamma is folded into W at
//   pack time and the row scale sqrt(K)/max(||x||, 1e-12) is computed from the staged A values.
//   Workgroup tile 256 tokens x 256 columns, 8 waves of 64x128 (2x4 blocks of 32x32), K chunks of
//   32 staged fp32 -> bf16 hi/lo in double-buffered LDS; weights arrive pre-split and pre-swizzled.
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

// ---------------------------------------------------------------------------------------------
// 512 threads (8 waves: 4 along M x 2 along N, 64x128 each), tile 256 tokens x 256 columns, LDS
// double-buffered (2 x 64 KB) with ONE barrier per 32-wide K chunk (48 MFMAs per wave per barrier): iteration k runs the MFMAs of
// stage k&1, writes chunk k+1 (already in registers) to the other stage and issues the global loads
// of chunk k+2.  The body is straight-line (clamped addresses, validity applied at store time).
template <bool X3, int NT, int BM, int WN, int MI, int NI, bool DB, bool CONV>
__global__ void __launch_bounds__(NT, DB ? 1 : 2) tok_gemm_kernel(TokGemmArgs a) {
  constexpr int BN = kTokBN, BK = kTokBK;
  static_assert((NT / 64) == (BM / (32 * MI)) * WN && BN == WN * NI * 32, "tile");
  constexpr int ROWB = BK * 2;                 // 64 B per image row (32 bf16)
  constexpr int A_BYTES = BM * ROWB;
  constexpr int W_BYTES = BN * ROWB;
  constexpr int STAGE = 2 * A_BYTES + 2 * W_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[(DB ? 2 : 1) * STAGE];
  __shared__ float rs[BM];
  __shared__ int orow_base[CONV ? BM : 1], orow_i1[CONV ? BM : 1];  // transposed-conv output rows

  const TokGroup g = a.groups[blockIdx.y];
  const int n_tile = blockIdx.x % a.n_tiles_n;
  const int m_tile = blockIdx.x / a.n_tiles_n;
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
  f32x4 areg[AI];
  f32x4 a2reg[CONV ? AI : 1];
  float ss[AI];
  const float* xrow[AI];
  bool rok[AI];
  // CONV: per-row input grid origin (b Q1, i1 s1, i2 s2) and per-chunk validity
  int rb1[CONV ? AI : 1], ri1[CONV ? AI : 1], ri2[CONV ? AI : 1];
  bool aval[CONV ? AI : 1];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    ss[i] = 0.f;
    const int m = m0 + arow0 + RS * i;
    rok[i] = m < a.M;
    xrow[i] = a.x + (int64_t)(rok[i] ? m : a.M - 1) * a.x_ld + g.x_off;
    if constexpr (CONV) {
      const int mm = rok[i] ? m : 0;
      const int i2 = mm % a.geo.P2, t = mm / a.geo.P2;
      const int i1 = t % a.geo.P1, b = t / a.geo.P1;
      rb1[i] = b * a.geo.Q1;
      ri1[i] = i1 * a.geo.s1;
      ri2[i] = i2 * a.geo.s2;
      aval[i] = false;
    }
  }
  bool kok = true;
  constexpr int W16 = (X3 ? 2 : 1) * W_BYTES / 16;
  constexpr int W_ITEMS = (W16 + NT - 1) / NT;
  u32x4 wreg[W_ITEMS];
  const uint16_t* wblk = a.w + g.w_off + (int64_t)n_tile * n_chunks * (2 * W_BYTES / 2);

  auto load_chunk = [&](int kc) {
    const u32x4* s4 = reinterpret_cast<const u32x4*>(wblk + (int64_t)kc * (2 * W_BYTES / 2));
    Unroll<0, W_ITEMS>::run([&](auto I) {
      const int e = tid + I * NT;
      wreg[I] = s4[e < W16 ? e : W16 - 1];
    });
    const int k = kc * BK + akq;
    kok = k < g.K;  // K % 4 == 0 (host check): a quad is wholly in or out
    const int kc_ = kok ? k : 0;
    if constexpr (CONV) {
      // Cin % 4 == 0 (host check): a quad lies inside one tap
      const int tap = kc_ / a.geo.Cin, c = kc_ - tap * a.geo.Cin;
      const int d1 = a.geo.d1[tap], d2 = a.geo.d2[tap];
#pragma unroll
      for (int i = 0; i < AI; ++i) {
        const int j1 = ri1[i] + d1, j2 = ri2[i] + d2;
        aval[i] = rok[i] && kok && j1 >= 0 && j1 < a.geo.Q1 && j2 >= 0 && j2 < a.geo.Q2;
        const int64_t off = aval[i] ? ((int64_t)(rb1[i] + j1) * a.geo.Q2 + j2) * a.x_ld + g.x_off + c : 0;
        areg[i] = *reinterpret_cast<const f32x4*>(a.x + off);
        if (a.geo.x2) a2reg[i] = *reinterpret_cast<const f32x4*>(a.geo.x2 + off);
      }
    } else {
#pragma unroll
      for (int i = 0; i < AI; ++i) areg[i] = *reinterpret_cast<const f32x4*>(xrow[i] + kc_);
    }
  };
  // count: 1 when this store is a real chunk (0 for the clamped repeat past the end: no RMS sum)
  auto store_chunk = [&](char* stg, float count) {
    char* Ahi = stg;
    char* Alo = stg + A_BYTES;
    u32x4* d4 = reinterpret_cast<u32x4*>(stg + 2 * A_BYTES);
    Unroll<0, W_ITEMS>::run([&](auto I) {
      const int e = min(tid + I * NT, W16 - 1);  // duplicates write identical values
      d4[e] = wreg[I];
    });
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int row = arow0 + RS * i;
      bool ok = rok[i] && kok;
      if constexpr (CONV) ok = aval[i];
      __bf16 hi[4], lo[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float v = ok ? areg[i][q] : 0.f;
        if constexpr (CONV) {
          if (a.geo.x2 && ok) v += a2reg[i][q];
        }
        ss[i] = fmaf(v * count, v, ss[i]);
        split_bf16(v, hi[q], lo[q]);
      }
      const int off = row * ROWB + ((((akq >> 3) ^ ((row >> 2) & 3))) << 4) + ((akq & 4) << 1);
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
        acc[i][j] = mfma32(ah[i], bh[j], acc[i][j]);
      }
  };

  if (DB) {
    load_chunk(0);
    store_chunk(smem, 1.f);
    load_chunk(min(1, n_chunks - 1));
    __syncthreads();
    for (int kc = 0; kc < n_chunks; ++kc) {
      const char* cur = smem + (kc & 1) * STAGE;
      char* nxt = smem + ((kc + 1) & 1) * STAGE;
      kstep(cur, 0);
      store_chunk(nxt, kc + 1 < n_chunks ? 1.f : 0.f);
      load_chunk(min(kc + 2, n_chunks - 1));
      kstep(cur, 1);
      __syncthreads();
    }
  } else {
    // single stage, two barriers per chunk, register prefetch of the next chunk under the MFMAs;
    // two workgroups per CU overlap one's staging / epilogue with the other's MFMAs
    load_chunk(0);
    for (int kc = 0; kc < n_chunks; ++kc) {
      __syncthreads();
      store_chunk(smem, 1.f);
      __syncthreads();
      load_chunk(min(kc + 1, n_chunks - 1));
      kstep(smem, 0);
      kstep(smem, 1);
    }
  }

  // ---- RMSNorm row scales: 8 threads share a row ----
  if (a.rownorm) {
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

  const bool tconv = CONV && a.geo.phases > 1;
  if constexpr (CONV) {
    if (a.geo.phases > 1) {
      for (int r = tid; r < BM; r += NT) {
        const int m = min(m0 + r, a.M - 1);
        const int i2 = m % a.geo.P2, t = m / a.geo.P2;
        const int i1 = t % a.geo.P1, b = t / a.geo.P1;
        orow_i1[r] = i1 * a.geo.phases - a.geo.opad;
        orow_base[r] = (b * a.geo.O1 + orow_i1[r]) * a.geo.P2 + i2;
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
        return (int64_t)orow_base[ml] + (int64_t)ph * a.geo.P2;
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
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          bool ok;
          const int64_t m = orow(r, ok);
          if (ok) a.out[m * a.o_ld + g.o_off + nc] = v[r];
        }
      }
    });
  });
}

// ---------------------------------------------------------------------------------------------
// Flash attention, head dim 64, 4 waves x 32 queries per workgroup, 64-key blocks.
// LDS images per block (bf16 hi / lo): K [64 key][64 d] and V^T [64 d][64 key'], 128-B rows with
// the 16-B chunk index XOR-swizzled by ((row >> 1) & 7) (conflict-free ds_read_b128 groups).
// key' permutes each 16-key group so the P^T registers of one lane are 8 consecutive key' slots:
//   key_local = (j & 3) + 8 (j >> 2) + 4 hl  <->  key' = 8 hl + j.
constexpr int kHD = 64;
constexpr int kKB = 64;

__device__ __forceinline__ int swz(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }

template <bool X3>
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
  {
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

  // staging: 64 keys x 64 d of K and of V (fp32) = 2 x 1024 f32x4; 8 per thread
  f32x4 kreg[4], vreg[4];
  auto load_block = [&](int kb) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + i * kThreads;  // (key, 4-d quad): 64 keys x 16 quads
      const int key = e >> 4, dq = (e & 15) * 4;
      const int p = kb * kKB + key;
      const bool ok = p < Lk && dq < dh;
      const float* row = kvb + ktoken(ok ? p : 0) * kv_ld + head * dh + (ok ? dq : 0);
      kreg[i] = ok ? *reinterpret_cast<const f32x4*>(row + a.k_off) : f32x4{0.f, 0.f, 0.f, 0.f};
      vreg[i] = ok ? *reinterpret_cast<const f32x4*>(row + a.v_off) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto store_block = [&]() {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + i * kThreads;
      const int key = e >> 4, dq = (e & 15) * 4;
      __bf16 hi[4], lo[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) split_bf16(kreg[i][q], hi[q], lo[q]);
      const int off = swz(key, dq >> 3) + ((dq & 4) << 1);
      *reinterpret_cast<uint2*>(Khi + off) = make_uint2(pack2(hi[0], hi[1]), pack2(hi[2], hi[3]));
      if (X3) *reinterpret_cast<uint2*>(Klo + off) = make_uint2(pack2(lo[0], lo[1]), pack2(lo[2], lo[3]));
      // V^T[d][key'] (2-byte scattered stores)
      const int kl = key & 15;
      const int kp = (key & ~15) + 8 * ((kl >> 2) & 1) + (kl & 3) + 4 * (kl >> 3);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        __bf16 vh, vl;
        split_bf16(vreg[i][q], vh, vl);
        const int d = dq + q;
        const int voff = swz(d, kp >> 3) + ((kp & 7) << 1);
        *reinterpret_cast<__bf16*>(Vhi + voff) = vh;
        if (X3) *reinterpret_cast<__bf16*>(Vlo + voff) = vl;
      }
    }
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
        const int d = db * 32 + l32;
        const int off = swz(d, 2 * ks + hl);
        const bf16x8 vh = *reinterpret_cast<const bf16x8*>(Vhi + off);
        if (X3) {
          const bf16x8 vl = *reinterpret_cast<const bf16x8*>(Vlo + off);
          o[db] = mfma32(vl, ph, o[db]);
          o[db] = mfma32(vh, pl, o[db]);
        }
        o[db] = mfma32(vh, ph, o[db]);
      }
    }
  }

  if (!q_ok) return;
  const int64_t tq = token(q_pos);
  const float gate = a.g_off >= 0 ? sigmoidf_(a.qkv[tq * a.ld + a.g_off + head]) : 1.f;
  const float scale = gate / l_run;
  float* op = a.out + tq * a.o_ld + head * dh;
#pragma unroll
  for (int db = 0; db < 2; ++db)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const int d = db * 32 + 8 * g4 + 4 * hl;
      if (d >= dh) continue;
      f32x4 v;
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = o[db][4 * g4 + q] * scale;
      *reinterpret_cast<f32x4*>(op + d) = v;
    }
}

}  // namespace

int launch_tok_gemm(const TokGemmArgs& a, int x3, hipStream_t st) {
  SESA_REQUIRE(a.n_groups >= 1 && a.n_tiles_n >= 1 && a.M >= 0, SESA_ERR_INVALID, "tok_gemm: bad grid");
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
    if (x3) hipLaunchKernelGGL((tok_gemm_kernel<true, 256, 128, 2, 2, 2, false, true>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((tok_gemm_kernel<false, 256, 128, 2, 2, 2, false, true>), grid, dim3(256), 0, st, a);
  } else if (variant == 1) {
    const int64_t mt = (a.M + 255) / 256;
    dim3 g1((unsigned)(mt * a.n_tiles_n), (unsigned)a.n_groups);
    if (x3) hipLaunchKernelGGL((tok_gemm_kernel<true, 512, 256, 2, 2, 2, true, false>), g1, dim3(512), 0, st, a);
    else hipLaunchKernelGGL((tok_gemm_kernel<false, 512, 256, 2, 2, 2, true, false>), g1, dim3(512), 0, st, a);
  } else {
    if (x3) hipLaunchKernelGGL((tok_gemm_kernel<true, 256, 128, 2, 2, 2, false, false>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((tok_gemm_kernel<false, 256, 128, 2, 2, 2, false, false>), grid, dim3(256), 0, st, a);
  }
  SESA_CHECK_LAUNCH();
  return SESA_OK;
}

int launch_attention(const AttnArgs& a, int x3, hipStream_t st) {
  SESA_REQUIRE(a.L >= 1 && a.n_seq >= 1 && a.heads >= 1 && a.sdiv >= 1 && a.Lk >= 0 && a.dh >= 0 && a.dh <= kHD &&
                   a.dh % 4 == 0 && (!a.kv || a.kv_ld % 4 == 0),
               SESA_ERR_INVALID, "attention: bad shape");
  SESA_REQUIRE(a.n_seq < 65536 * 4 && a.heads < 65536, SESA_ERR_INVALID, "attention: grid too large");
  dim3 grid((unsigned)((a.L + 127) / 128), (unsigned)a.heads, (unsigned)a.n_seq);
  if (x3) hipLaunchKernelGGL(attn_kernel<true>, grid, dim3(kThreads), 0, st, a);
  else hipLaunchKernelGGL(attn_kernel<false>, grid, dim3(kThreads), 0, st, a);
  SESA_CHECK_LAUNCH();
  return SESA_OK;
}

}  // namespace sesa
