// MFMA contraction kernels for the MDX23C TFC-TDF network (gfx950, wave64).
//
// Layout: every activation is NHWC fp32 [B][T][F][C] (channels innermost), so both GEMM operands
// of a convolution are K-contiguous (K = input channel) and MFMA fragments are single 16-byte
// LDS reads.  Precision: fp32 activations in HBM; operands are split in-register into bf16
// hi + lo and contracted with 3 MFMA passes (hi*hi + hi*lo + lo*hi, fp32 accumulate) -- the
// parity mode -- or with one bf16 pass (X3 = false).
//
// tap_gemm_kernel -- implicit-GEMM convolution over (T, F) with KHxKW taps and stride S
//   (nn.Conv2d 3x3 p1 / 1x1, Downscale 2x2 s2, and the ConvTranspose2d 2x2 s2 of Upscale as a
//   1x1 GEMM with N = 4*C_out and a scattering epilogue), mdx23c_tfc_tdf_v3.py:74-138, 161, 183-187.
//   Workgroup tile: TM rows x 32 columns of output positions x BN output channels; 4 waves.
//   Per 16-channel K chunk the halo tile is loaded ONCE from HBM/L2, the consumer's
//   InstanceNorm-affine + exact GELU (or the x*first_conv_out product) is applied in the
//   prologue, split to bf16 hi/lo and stored to LDS; all KH*KW taps then read shifted windows.
//   Epilogue: optional residual add (x + s, :137) and output GELU, fp32 store, and per-channel
//   sum / sum-of-squares for the NEXT InstanceNorm (double atomics), so no norm kernel and no
//   extra pass over the activation exists anywhere.
// tdf_kernel -- the TDF nn.Linear over the frequency axis (:113-120), per (b, t):
//   out[f', c] = sum_f W[f', f] * act(x)[f, c] (+ residual), same prologue / epilogue fusion.
//
// MFMA: v_mfma_f32_32x32x16_bf16.  Lane l holds A[m = l&31][k = 8(l>>5)+j] and
// B[k = 8(l>>5)+j][n = l&31]; D: column n = l&31, row (r&3) + 8(r>>2) + 4(l>>5).
// LDS images store 16-byte halves swizzled by (row>>3)&1 (conv) / (row>>2)&3 (TDF) so the
// ds_read_b128 lane groups are bank-conflict free.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "sesa_common.hpp"
#include "sesa_tapgemm.hpp"

namespace sesa {
namespace {

constexpr int kThreads = 256;
constexpr int kMaxCin = 1536;

// Compile-time unrolled loop: f(std::integral_constant<int, I>) for I in [0, N).  Array indices become
// frontend constants, so SROA keeps staging arrays in registers (a pragma-unrolled loop left the
// 9-entry weight staging array in scratch).
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

// Select source 0/1 without runtime-indexing the kernel-argument struct (which would go to scratch).
__device__ __forceinline__ Src pick_src(const GemmIn& in, int s) {
  Src r;
  r.ptr = s ? in.src[1].ptr : in.src[0].ptr;
  r.stats = s ? in.src[1].stats : in.src[0].stats;
  r.mul = s ? in.src[1].mul : in.src[0].mul;
  r.C = s ? in.src[1].C : in.src[0].C;
  r.mode = s ? in.src[1].mode : in.src[0].mode;
  r.hi = s ? in.src[1].hi : in.src[0].hi;
  r.lo = s ? in.src[1].lo : in.src[0].lo;
  return r;
}

// Per-channel affine (scale, shift) of the consumer's InstanceNorm, from the producer's sums.
__device__ void build_affine(const GemmIn& in, int b, float* sc, float* sh) {
  for (int c = threadIdx.x; c < in.C_in; c += kThreads) {
    const int s = c < in.C_split ? 0 : 1;
    const Src src = pick_src(in, s);
    const int cl = c - (s ? in.C_split : 0);
    float scale = 1.f, shift = 0.f;
    if (src.mode == SRC_NORM_GELU) {
      const double* st = src.stats + ((int64_t)b * src.C + cl) * 2;
      const double mean = st[0] * in.inv_count;
      double var = st[1] * in.inv_count - mean * mean;
      if (var < 0) var = 0;
      const float rstd = (float)(1.0 / sqrt(var + 1e-5));
      const float g = in.gamma ? in.gamma[c] : 1.f;
      const float be = in.beta ? in.beta[c] : 0.f;
      scale = g * rstd;
      shift = be - (float)mean * scale;
    }
    sc[c] = scale;
    sh[c] = shift;
  }
}

__device__ __forceinline__ void transform4(float (&v)[4], int mode, const float* sc, const float* sh, int c,
                                           const float* mulp) {
  if (mode == SRC_NORM_GELU) {
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = gelu_erf(v[q] * sc[c + q] + sh[c + q]);
  } else if (mode == SRC_MUL) {
    const float4 m = *reinterpret_cast<const float4*>(mulp);
    v[0] *= m.x; v[1] *= m.y; v[2] *= m.z; v[3] *= m.w;
  }
}

// ---------------------------------------------------------------------------------------------
// K is walked in 16-channel chunks: first the n_chunks chunks of the main (normalised) input over
// all KH*KW taps, then x_chunks chunks of an optional RAW extra input over the centre tap only --
// the 1x1 shortcut of TFC_TDF (mdx23c_tfc_tdf_v3.py:126, :132, :137) fused into tfc2's conv as
// extra K, so `s` never round-trips through HBM.
template <int KH, int KW, int S, int PAD, int TM, int BN, int WM, bool X3, bool UPS, bool XTRA, bool PRE>
__global__ void __launch_bounds__(kThreads, 2) tap_gemm_kernel(ConvArgs a) {
  constexpr int WN = 4 / WM;
  constexpr int MI = TM / WM;                 // 32-position MFMA row blocks per wave
  constexpr int NI = BN / WN / 32;            // 32-channel MFMA column blocks per wave
  constexpr int HT = (TM - 1) * S + KH;       // halo rows
  constexpr int HW = (kTF - 1) * S + KW;      // halo cols
  constexpr int NPOS = HT * HW;
  constexpr int TAPS = KH * KW;
  constexpr int CTAP = (KH / 2) * KW + KW / 2;  // centre tap (the 1x1 shortcut's alignment, PAD = 1)
  constexpr int A_BYTES = NPOS * 32;          // one (hi or lo) image: 16 bf16 per position
  constexpr int W_BYTES = TAPS * BN * 32;
  constexpr int W1_BYTES = BN * 32;           // one-tap image of an extra (shortcut) chunk
  static_assert(MI >= 1 && NI >= 1, "tile");

  __shared__ __attribute__((aligned(16))) char smem[2 * A_BYTES + 2 * W_BYTES + 2 * kMaxCin * 4];
  char* A_hi = smem;
  char* A_lo = smem + A_BYTES;
  char* W_hi = smem + 2 * A_BYTES;
  float* sc = reinterpret_cast<float*>(W_hi + 2 * W_BYTES);
  float* sh = sc + kMaxCin;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int l32 = lane & 31, h = lane >> 5;

  // XCD-aware block order (1-D grid over tiles x output-channel blocks): the NB channel blocks of a
  // spatial tile get ids 8 apart inside a window of 8*NB consecutive ids, so they run at the same
  // time on the SAME XCD and its L2 serves the shared input halo (the dispatcher deals ids
  // round-robin over the 8 XCDs; speed only, never correctness).  Requires n_tiles % 8 == 0 for the
  // full grouping; the tail falls back to the plain order.
  const int tiles_f = a.F_out / kTF;
  const int NB = (a.n_cols + BN - 1) / BN;
  const int n_tiles = ((a.T_out + TM - 1) / TM) * tiles_f;
  int tile, nb;
  {
    const int id = blockIdx.x;
    const int full = (n_tiles / 8) * 8 * NB;
    if (id < full) {
      const int g = id / (8 * NB), r = id - g * 8 * NB;
      tile = g * 8 + (r & 7);
      nb = r >> 3;
    } else {
      const int r = id - full;
      tile = (n_tiles / 8) * 8 + r / NB;
      nb = r % NB;
    }
  }
  const int t0 = (tile / tiles_f) * TM;
  const int f0 = (tile % tiles_f) * kTF;
  const int b = blockIdx.z;
  const int t_in0 = t0 * S - PAD, f_in0 = f0 * S - PAD;
  const int n_total = a.n_chunks + (XTRA ? a.x_chunks : 0);

  build_affine(a.in, b, sc, sh);

  f32x16 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // per-nb weight block: [n_chunks x (hi,lo) TAPS-tap images][x_chunks x (hi,lo) 1-tap images]
  const uint16_t* wblk = a.w + (int64_t)nb * (a.n_chunks * W_BYTES + (XTRA ? a.x_chunks * W1_BYTES : 0));

  // Register-staged software pipeline: the global loads of chunk k+1 are issued before the MFMAs
  // of chunk k and land while they run; transform + LDS write happen between two barriers.
  constexpr int A_ITEMS = (NPOS * 4 + kThreads - 1) / kThreads;
  constexpr int W16 = (X3 ? 2 : 1) * W_BYTES / 16;
  constexpr int W_ITEMS = (W16 + kThreads - 1) / kThreads;
  static_assert(A_ITEMS <= 32, "valid mask");
  f32x4 areg[A_ITEMS];  // native vectors: HIP's float4/uint4 structs copy via memcpy and defeat SROA
  u32x4 wreg[W_ITEMS];
  uint32_t avalid = 0;

  // source of chunk kc: (src, local channel offset, first concatenated channel, is-extra)
  auto chunk_src = [&](int kc, Src& src, int& cl0, int& k0, bool& ext) {
    ext = XTRA && kc >= a.n_chunks;
    k0 = (ext ? kc - a.n_chunks : kc) * kConvBK;
    const GemmIn& g = ext ? a.xin : a.in;
    const int s = k0 < g.C_split ? 0 : 1;
    src = pick_src(g, s);
    cl0 = k0 - (s ? g.C_split : 0);
  };

  auto load_chunk = [&](int kc) {
    Src src;
    int cl0, k0;
    bool ext;
    chunk_src(kc, src, cl0, k0, ext);
    const int w16 = ext ? (X3 ? 2 : 1) * W1_BYTES / 16 : W16;
    const u32x4* wsrc = reinterpret_cast<const u32x4*>(
        wblk + (ext ? (int64_t)a.n_chunks * W_BYTES + (int64_t)(kc - a.n_chunks) * W1_BYTES
                    : (int64_t)kc * W_BYTES));
    Unroll<0, W_ITEMS>::run([&](auto I) {
      const int e = tid + I * kThreads;
      wreg[I] = wsrc[e < w16 ? e : w16 - 1];  // unconditional (clamped) so wreg stays in VGPRs
    });
    avalid = 0;
    if (PRE && !ext) {
      // pre-activated planes: item = (position, 8-channel half): 16 B of hi + 16 B of lo
      constexpr int P_ITEMS = (NPOS * 2 + kThreads - 1) / kThreads;
      static_assert(2 * P_ITEMS <= A_ITEMS, "PRE staging registers");
      Unroll<0, P_ITEMS>::run([&](auto I) {
        constexpr int i = decltype(I)::value;
        const int e = tid + i * kThreads;
        const int p = e >> 1, hf = e & 1;
        const int hr = p / HW, hc = p - hr * HW;
        const int ti = t_in0 + hr, fi = f_in0 + hc;
        const bool ok = (e < NPOS * 2) && ti >= 0 && ti < a.T_in && fi >= 0 && fi < a.F_in;
        if (ok) {
          const int64_t idx = (((int64_t)b * a.T_in + ti) * a.F_in + fi) * src.C + cl0 + 8 * hf;
          areg[2 * i] = *reinterpret_cast<const f32x4*>(src.hi + idx);
          areg[2 * i + 1] = *reinterpret_cast<const f32x4*>(src.lo + idx);
        } else {
          areg[2 * i] = f32x4{0.f, 0.f, 0.f, 0.f};
          areg[2 * i + 1] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      });
      return;
    }
    Unroll<0, A_ITEMS>::run([&](auto I) {
      constexpr int i = decltype(I)::value;
      const int e = tid + i * kThreads;
      const int p = e >> 2, g = e & 3;
      const int hr = p / HW, hc = p - hr * HW;
      const int ti = t_in0 + hr, fi = f_in0 + hc;
      const bool ok = (e < NPOS * 4) && ti >= 0 && ti < a.T_in && fi >= 0 && fi < a.F_in;
      if (ok) {
        const int64_t idx = (((int64_t)b * a.T_in + ti) * a.F_in + fi) * src.C + cl0 + 4 * g;
        areg[i] = *reinterpret_cast<const f32x4*>(src.ptr + idx);
        avalid |= 1u << i;
      } else {
        areg[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    });
  };

  auto store_chunk = [&](int kc) {
    Src src;
    int cl0, k0;
    bool ext;
    chunk_src(kc, src, cl0, k0, ext);
    const int w16 = ext ? (X3 ? 2 : 1) * W1_BYTES / 16 : W16;
    u32x4* wdst = reinterpret_cast<u32x4*>(W_hi);
    Unroll<0, W_ITEMS>::run([&](auto I) {
      const int e = tid + I * kThreads;
      if (e < w16) wdst[e] = wreg[I];
    });
    if (PRE && !ext) {  // straight copies (zeros for out-of-bounds positions are already in areg)
      constexpr int P_ITEMS = (NPOS * 2 + kThreads - 1) / kThreads;
      Unroll<0, P_ITEMS>::run([&](auto I) {
        constexpr int i = decltype(I)::value;
        const int e = tid + i * kThreads;
        if (NPOS * 2 % kThreads != 0 && e >= NPOS * 2) return;
        const int p = e >> 1, hf = e & 1;
        const int off = p * 32 + ((hf ^ ((p >> 3) & 1)) << 4);
        *reinterpret_cast<f32x4*>(A_hi + off) = areg[2 * i];
        if (X3) *reinterpret_cast<f32x4*>(A_lo + off) = areg[2 * i + 1];
      });
      return;
    }
    Unroll<0, A_ITEMS>::run([&](auto I) {
      constexpr int i = decltype(I)::value;
      const int e = tid + i * kThreads;
      if (NPOS * 4 % kThreads != 0 && e >= NPOS * 4) return;
      const int p = e >> 2, g = e & 3;
      const int off = p * 32 + ((((g >> 1) ^ ((p >> 3) & 1))) << 4) + ((g & 1) << 3);
      float v[4] = {areg[i][0], areg[i][1], areg[i][2], areg[i][3]};
      if (!ext && (avalid & (1u << i))) {
        const float* mulp = nullptr;
        if (src.mode == SRC_MUL) {
          const int hr = p / HW, hc = p - hr * HW;
          const int64_t idx = (((int64_t)b * a.T_in + t_in0 + hr) * a.F_in + f_in0 + hc) * src.C + cl0 + 4 * g;
          mulp = src.mul + idx;
        }
        transform4(v, src.mode, sc, sh, k0 + 4 * g, mulp);
      }
      __bf16 hi[4], lo[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) split_bf16(v[q], hi[q], lo[q]);
      *reinterpret_cast<uint2*>(A_hi + off) = make_uint2(pack2(hi[0], hi[1]), pack2(hi[2], hi[3]));
      if (X3) *reinterpret_cast<uint2*>(A_lo + off) = make_uint2(pack2(lo[0], lo[1]), pack2(lo[2], lo[3]));
    });
  };

  // one tap: A window shifted by (dy, dx), W image tap `wt` of a (hi, lo) image pair `wimg` bytes apart
  auto mfma_tap = [&](int dy, int dx, int wt, int wimg) {
    bf16x8 ah[MI], al[MI], bh[NI], bl[NI];
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int row = wm * MI + i;
      const int p = (row * S + dy) * HW + l32 * S + dx;
      const int off = p * 32 + ((h ^ ((p >> 3) & 1)) << 4);
      ah[i] = *reinterpret_cast<const bf16x8*>(A_hi + off);
      if (X3) al[i] = *reinterpret_cast<const bf16x8*>(A_lo + off);
    }
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int p = wt * BN + (wn * NI + j) * 32 + l32;
      const int off = p * 32 + ((h ^ ((p >> 3) & 1)) << 4);
      bh[j] = *reinterpret_cast<const bf16x8*>(W_hi + off);
      if (X3) bl[j] = *reinterpret_cast<const bf16x8*>(W_hi + wimg + off);
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

  load_chunk(0);
  for (int kc = 0; kc < n_total; ++kc) {
    __syncthreads();  // previous chunk's fragment reads are done (and sc/sh are built)
    store_chunk(kc);
    __syncthreads();
    if (kc + 1 < n_total) load_chunk(kc + 1);
    if (!XTRA || kc < a.n_chunks) {
      constexpr int TU = XTRA ? 3 : TAPS;  // the fused-shortcut variant needs the registers
#pragma unroll TU
      for (int tap = 0; tap < TAPS; ++tap) mfma_tap(tap / KW, tap % KW, tap, W_BYTES);
    } else {
      mfma_tap(CTAP / KW, CTAP % KW, 0, W1_BYTES);
    }
  }

  // ---- epilogue ----
  float ssum[NI], ssq[NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) { ssum[j] = 0.f; ssq[j] = 0.f; }
  const int C_out = a.out.C_out;
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int ncol = nb * BN + (wn * NI + j) * 32 + l32;  // GEMM column
    int co = ncol, dy = 0, dx = 0;
    if (UPS) {
      const int tap = ncol / C_out;
      co = ncol - tap * C_out;
      dy = tap >> 1;
      dx = tap & 1;
    }
    const bool col_ok = UPS ? (ncol < a.n_cols) : (co < C_out);
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int t = t0 + wm * MI + i;
      if (t >= a.T_out || !col_ok) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int f = f0 + (r & 3) + 8 * (r >> 2) + 4 * h;
        int64_t idx;
        if (UPS) {
          const int T2 = a.T_out * 2, F2 = a.F_out * 2;
          idx = (((int64_t)b * T2 + 2 * t + dy) * F2 + 2 * f + dx) * C_out + co;
        } else {
          idx = (((int64_t)b * a.T_out + t) * a.F_out + f) * C_out + co;
        }
        float v = acc[i][j][r];
        if (a.out.residual) v += a.out.residual[idx];
        if (a.out.gelu) v = gelu_erf(v);
        a.out.ptr[idx] = v;
        ssum[j] += v;
        ssq[j] += v * v;
      }
    }
  }
  if (a.out.stats) {
    // reduce over the two lane halves, then over the WM waves sharing these columns (LDS)
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);  // [WM][BN][2]
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      ssum[j] += __shfl_xor(ssum[j], 32);
      ssq[j] += __shfl_xor(ssq[j], 32);
      if (h == 0) {
        const int n = (wn * NI + j) * 32 + l32;
        red[(wm * BN + n) * 2 + 0] = ssum[j];
        red[(wm * BN + n) * 2 + 1] = ssq[j];
      }
    }
    __syncthreads();
    for (int n = tid; n < BN; n += kThreads) {
      float s0 = 0.f, s1 = 0.f;
#pragma unroll
      for (int w = 0; w < WM; ++w) {
        s0 += red[(w * BN + n) * 2 + 0];
        s1 += red[(w * BN + n) * 2 + 1];
      }
      const int ncol = nb * BN + n;
      const int co = UPS ? ncol % C_out : ncol;
      if ((UPS ? ncol < a.n_cols : co < C_out)) {
        double* st = a.out.stats + ((int64_t)b * C_out + co) * 2;
        atomicAdd(st + 0, (double)s0);
        atomicAdd(st + 1, (double)s1);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// TDF linear: per (b, t), D[m = f_out][n = c] = sum_k W[m][k] * act(x[b][t][k][c]).
// One workgroup covers BM = 128*MI output rows (all of M for the TDF's first Linear, so every
// input element is normalised + GELU'd once) x BN = 64 channels; 4 waves stacked along M.
// BK_CONTIG: the input is the transposed U^T [b][t][c][k] written by the first Linear (k
//   contiguous -> two 16-B loads per 8 k); otherwise NHWC [b][t][k][c] (lanes walk c).
// OUT_T: write the output transposed as U^T [b][t][c][m] (16-B stores of 4 consecutive rows).
template <int MI, bool X3, bool BK_CONTIG, bool OUT_T>
__global__ void __launch_bounds__(kThreads, 2) tdf_kernel(TdfArgs a) {
  constexpr int BN = 64;
  constexpr int WM = 4;
  constexpr int NI = BN / 32;
  constexpr int BM = WM * MI * 32;
  constexpr int ROWB = kTdfBK * 2;            // 64 B per image row (32 bf16)
  constexpr int AW_BYTES = BM * ROWB;
  constexpr int B_BYTES = BN * ROWB;
  __shared__ __attribute__((aligned(16))) char smem[2 * AW_BYTES + 2 * B_BYTES + 2 * kMaxCin * 4];
  char* Whi = smem;
  char* Wlo = smem + AW_BYTES;
  char* Bhi = smem + 2 * AW_BYTES;
  char* Blo = Bhi + B_BYTES;
  float* sc = reinterpret_cast<float*>(Blo + B_BYTES);
  float* sh = sc + kMaxCin;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wm = tid >> 6;
  const int l32 = lane & 31, h = lane >> 5;
  const int mb = blockIdx.x, c0 = blockIdx.y * BN;
  const int bt = blockIdx.z;
  const int b = bt / a.T;
  const Src src = pick_src(a.in, 0);
  const int C = src.C;

  build_affine(a.in, b, sc, sh);

  f32x16 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const float* xin = src.ptr + (int64_t)bt * a.K * C;  // this (b, t) slice, either layout
  const uint16_t* wblk = a.w + (int64_t)mb * a.n_chunks * (2 * AW_BYTES / 2);

  constexpr int N16 = (X3 ? 2 : 1) * AW_BYTES / 16;
  constexpr int W_ITEMS = (N16 + kThreads - 1) / kThreads;
  constexpr int B_ITEMS = (BN * 4 + kThreads - 1) / kThreads;
  u32x4 wreg[W_ITEMS];
  f32x4 breg[B_ITEMS][2];

  auto load_chunk = [&](int kc) {
    const u32x4* s4 = reinterpret_cast<const u32x4*>(wblk + (int64_t)kc * (2 * AW_BYTES / 2));
    Unroll<0, W_ITEMS>::run([&](auto I) {
      const int e = tid + I * kThreads;
      wreg[I] = s4[e < N16 ? e : N16 - 1];
    });
    const int k0 = kc * kTdfBK;
    Unroll<0, B_ITEMS>::run([&](auto I) {
      const int e = tid + I * kThreads;
      const int n = e % BN, g = e / BN;
      const int c = c0 + n;
      const int k = k0 + 8 * g;
      const bool ok = (e < BN * 4) && c < C && k < a.K;
      if (BK_CONTIG) {
        // k-contiguous: K is a multiple of 8, so a group of 8 is wholly in or out
        const f32x4* p4 = reinterpret_cast<const f32x4*>(xin + (int64_t)(ok ? c : 0) * a.K + (ok ? k : 0));
        breg[I][0] = ok ? p4[0] : f32x4{0.f, 0.f, 0.f, 0.f};
        breg[I][1] = ok ? p4[1] : f32x4{0.f, 0.f, 0.f, 0.f};
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const bool okj = ok && k + j < a.K;
          breg[I][j >> 2][j & 3] = okj ? xin[(int64_t)(k + j) * C + c] : 0.f;
        }
      }
    });
  };

  load_chunk(0);
  for (int kc = 0; kc < a.n_chunks; ++kc) {
    __syncthreads();
    {
      u32x4* d4 = reinterpret_cast<u32x4*>(Whi);
      Unroll<0, W_ITEMS>::run([&](auto I) {
        const int e = tid + I * kThreads;
        if (N16 % kThreads == 0 || e < N16) d4[e] = wreg[I];
      });
      const int k0 = kc * kTdfBK;
      Unroll<0, B_ITEMS>::run([&](auto I) {
        const int e = tid + I * kThreads;
        if (BN * 4 % kThreads != 0 && e >= BN * 4) return;
        const int n = e % BN, g = e / BN;
        const int c = c0 + n;
        const bool ok = c < C && k0 + 8 * g < a.K;
        const float scale = ok ? sc[c] : 1.f, shift = ok ? sh[c] : 0.f;
        __bf16 hi[8], lo[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float x = breg[I][j >> 2][j & 3];
          if (src.mode == SRC_NORM_GELU && ok && k0 + 8 * g + j < a.K) x = gelu_erf(x * scale + shift);
          split_bf16(x, hi[j], lo[j]);
        }
        const int off = n * ROWB + ((g ^ ((n >> 2) & 3)) << 4);
        *reinterpret_cast<uint4*>(Bhi + off) =
            make_uint4(pack2(hi[0], hi[1]), pack2(hi[2], hi[3]), pack2(hi[4], hi[5]), pack2(hi[6], hi[7]));
        if (X3)
          *reinterpret_cast<uint4*>(Blo + off) =
              make_uint4(pack2(lo[0], lo[1]), pack2(lo[2], lo[3]), pack2(lo[4], lo[5]), pack2(lo[6], lo[7]));
      });
    }
    __syncthreads();
    if (kc + 1 < a.n_chunks) load_chunk(kc + 1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 ah[MI], al[MI], bh[NI], bl[NI];
      const int q = ks * 2 + h;
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int row = (wm * MI + i) * 32 + l32;
        const int off = row * ROWB + ((q ^ ((row >> 2) & 3)) << 4);
        ah[i] = *reinterpret_cast<const bf16x8*>(Whi + off);
        if (X3) al[i] = *reinterpret_cast<const bf16x8*>(Wlo + off);
      }
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int n = j * 32 + l32;
        const int off = n * ROWB + ((q ^ ((n >> 2) & 3)) << 4);
        bh[j] = *reinterpret_cast<const bf16x8*>(Bhi + off);
        if (X3) bl[j] = *reinterpret_cast<const bf16x8*>(Blo + off);
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
    }
  }

  float ssum[NI], ssq[NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) { ssum[j] = 0.f; ssq[j] = 0.f; }
  const int Cout = a.out.C_out;
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int c = c0 + j * 32 + l32;
    if (c >= Cout) continue;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int m0 = mb * BM + (wm * MI + i) * 32 + 8 * g4 + 4 * h;  // rows m0 .. m0+3 in regs 4*g4 ..
        if (OUT_T) {
          // U^T [b][t][c][m]; M is a multiple of 4 here (F / bottleneck_factor, checked on the host)
          if (m0 >= a.M) continue;
          f32x4 v4;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float v = acc[i][j][4 * g4 + q];
            v4[q] = v;
            ssum[j] += v;
            ssq[j] += v * v;
          }
          *reinterpret_cast<f32x4*>(a.out.ptr + ((int64_t)bt * Cout + c) * a.M + m0) = v4;
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int m = m0 + q;
            if (m >= a.M) continue;
            const int64_t idx = ((int64_t)bt * a.M + m) * Cout + c;
            float v = acc[i][j][4 * g4 + q];
            if (a.out.residual) v += a.out.residual[idx];
            a.out.ptr[idx] = v;
            ssum[j] += v;
            ssq[j] += v * v;
          }
        }
      }
    }
  }
  if (a.out.stats) {
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);  // [WM][BN][2]
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      ssum[j] += __shfl_xor(ssum[j], 32);
      ssq[j] += __shfl_xor(ssq[j], 32);
      if (h == 0) {
        const int n = j * 32 + l32;
        red[(wm * BN + n) * 2 + 0] = ssum[j];
        red[(wm * BN + n) * 2 + 1] = ssq[j];
      }
    }
    __syncthreads();
    for (int n = tid; n < BN; n += kThreads) {
      const int c = c0 + n;
      if (c >= Cout) continue;
      float s0 = 0.f, s1 = 0.f;
#pragma unroll
      for (int w = 0; w < WM; ++w) {
        s0 += red[(w * BN + n) * 2 + 0];
        s1 += red[(w * BN + n) * 2 + 1];
      }
      double* st = a.out.stats + ((int64_t)b * Cout + c) * 2;
      atomicAdd(st + 0, (double)s0);
      atomicAdd(st + 1, (double)s1);
    }
  }
}


// ---------------------------------------------------------------------------------------------
// act_split: one pass over a normalised tensor, writing the bf16 hi/lo operand planes of its
// consumer (InstanceNorm affine + exact GELU applied once per element instead of once per
// consuming tile).  HBM-bound: reads 4 B, writes 2 + 2 B per element.
__global__ void __launch_bounds__(kThreads) act_split_kernel(GemmIn in, int64_t n_pos, int pos_per_block,
                                                             uint16_t* __restrict__ hi, uint16_t* __restrict__ lo) {
  __shared__ float sc[kMaxCin], sh[kMaxCin];
  const int b = blockIdx.y;
  build_affine(in, b, sc, sh);
  __syncthreads();
  const int C = in.C_in;
  const int groups = C / 8;  // 8 channels per thread-item (C % 16 == 0)
  const int64_t p0 = (int64_t)blockIdx.x * pos_per_block;
  const int64_t np = (n_pos - p0) < pos_per_block ? (n_pos - p0) : pos_per_block;
  const int64_t items = np * groups;
  for (int64_t e = threadIdx.x; e < items; e += kThreads) {
    const int64_t p = p0 + e / groups;
    const int c = (int)(e % groups) * 8;
    const int s = c < in.C_split ? 0 : 1;
    const Src src = pick_src(in, s);
    const int cl = c - (s ? in.C_split : 0);
    const f32x4* xp = reinterpret_cast<const f32x4*>(src.ptr + ((int64_t)b * n_pos + p) * src.C + cl);
    const f32x4 x0 = xp[0], x1 = xp[1];
    float v[8] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
    __bf16 h8[8], l8[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float y = src.mode == SRC_NORM_GELU ? gelu_erf(v[q] * sc[c + q] + sh[c + q]) : v[q];
      split_bf16(y, h8[q], l8[q]);
    }
    const int64_t o = ((int64_t)b * n_pos + p) * C + c;
    *reinterpret_cast<uint4*>(hi + o) =
        make_uint4(pack2(h8[0], h8[1]), pack2(h8[2], h8[3]), pack2(h8[4], h8[5]), pack2(h8[6], h8[7]));
    *reinterpret_cast<uint4*>(lo + o) =
        make_uint4(pack2(l8[0], l8[1]), pack2(l8[2], l8[3]), pack2(l8[4], l8[5]), pack2(l8[6], l8[7]));
  }
}

template <int KH, int KW, int S, int PAD, int TM, int BN, int WM, bool UPS, bool XTRA, bool PRE>
int launch_conv_t(int x3, const ConvArgs& a, int batch, hipStream_t st) {
  // PRE kernels read only the bf16 planes of the main input
  SESA_REQUIRE(!PRE || (a.in.src[0].mode == SRC_PRE && a.in.src[0].hi && a.in.src[0].lo && a.in.C_split == a.in.C_in),
               SESA_ERR_INVALID, "conv: this kernel needs a single pre-activated (act_split) input");
  SESA_REQUIRE(PRE || (a.in.src[0].mode != SRC_PRE && a.in.src[1].mode != SRC_PRE), SESA_ERR_INVALID,
               "conv: pre-activated input given to a transforming kernel");
  dim3 grid((unsigned)(((a.T_out + TM - 1) / TM) * (a.F_out / kTF) * ((a.n_cols + BN - 1) / BN)), 1u,
            (unsigned)batch);
  if (x3)
    hipLaunchKernelGGL((tap_gemm_kernel<KH, KW, S, PAD, TM, BN, WM, true, UPS, XTRA, PRE>), grid, dim3(kThreads), 0, st, a);
  else
    hipLaunchKernelGGL((tap_gemm_kernel<KH, KW, S, PAD, TM, BN, WM, false, UPS, XTRA, PRE>), grid, dim3(kThreads), 0, st, a);
  SESA_CHECK_LAUNCH();
  return SESA_OK;
}

}  // namespace

// Tile choices per kind (BN = 64 unless the GEMM N is <= 32).
int launch_conv(int kind, int bn, int x3, const ConvArgs& a, int batch, hipStream_t st) {
  SESA_REQUIRE(a.F_out % kTF == 0, SESA_ERR_INVALID, "conv: F_out %d not a multiple of %d", a.F_out, kTF);
  SESA_REQUIRE(a.in.C_in % kConvBK == 0 && a.in.C_split % kConvBK == 0 && a.in.C_in <= kMaxCin, SESA_ERR_INVALID,
               "conv: C_in %d / split %d must be multiples of %d (<= %d)", a.in.C_in, a.in.C_split, kConvBK,
               kMaxCin);
  switch (kind) {
    case CONV3X3:
      if (a.x_chunks > 0) {
        SESA_REQUIRE(a.xin.C_in % kConvBK == 0 && a.xin.C_split % kConvBK == 0, SESA_ERR_INVALID,
                     "conv: fused shortcut C_in %d must be a multiple of %d", a.xin.C_in, kConvBK);
        return launch_conv_t<3, 3, 1, 1, 8, 64, 4, false, true, true>(x3, a, batch, st);
      }
      return launch_conv_t<3, 3, 1, 1, 8, 64, 4, false, false, true>(x3, a, batch, st);
    case CONV1X1:
      if (bn == 32) return launch_conv_t<1, 1, 1, 0, 8, 32, 4, false, false, false>(x3, a, batch, st);
      return launch_conv_t<1, 1, 1, 0, 8, 64, 4, false, false, false>(x3, a, batch, st);
    case CONV2X2S2:
      return launch_conv_t<2, 2, 2, 0, 4, 64, 4, false, false, true>(x3, a, batch, st);
    case DECONV2X2S2:
      return launch_conv_t<1, 1, 1, 0, 8, 64, 4, true, false, true>(x3, a, batch, st);
  }
  set_error("conv: unknown kind %d", kind);
  return SESA_ERR_INVALID;
}

template <int MI, bool BKC, bool OT>
int launch_tdf_t(int x3, const TdfArgs& a, int batch, hipStream_t st) {
  constexpr int BM = 4 * MI * 32;
  dim3 grid((unsigned)((a.M + BM - 1) / BM), (unsigned)((a.out.C_out + 63) / 64), (unsigned)(batch * a.T));
  if (x3) hipLaunchKernelGGL((tdf_kernel<MI, true, BKC, OT>), grid, dim3(kThreads), 0, st, a);
  else hipLaunchKernelGGL((tdf_kernel<MI, false, BKC, OT>), grid, dim3(kThreads), 0, st, a);
  SESA_CHECK_LAUNCH();
  return SESA_OK;
}

int tdf_block_rows(int M) { return M > 128 ? 256 : 128; }

int launch_act_split(const GemmIn& in, int64_t n_pos, int batch, uint16_t* hi, uint16_t* lo, hipStream_t st) {
  SESA_REQUIRE(in.C_in % 16 == 0 && in.C_split % 8 == 0 && in.C_in <= kMaxCin, SESA_ERR_INVALID,
               "act_split: C %d must be a multiple of 16 (<= %d)", in.C_in, kMaxCin);
  const int ppb = (int)((16384 + in.C_in - 1) / in.C_in);  // ~16K elements per block
  dim3 grid((unsigned)((n_pos + ppb - 1) / ppb), (unsigned)batch);
  hipLaunchKernelGGL(act_split_kernel, grid, dim3(kThreads), 0, st, in, n_pos, ppb, hi, lo);
  SESA_CHECK_LAUNCH();
  return SESA_OK;
}

// transposed_io: 0 = first Linear (NHWC in, U^T out), 1 = second Linear (U^T in, NHWC out)
int launch_tdf(int x3, const TdfArgs& a, int batch, hipStream_t st, int transposed_io) {
  SESA_REQUIRE(a.in.C_in <= kMaxCin, SESA_ERR_INVALID, "tdf: C %d > %d", a.in.C_in, kMaxCin);
  if (transposed_io == 0) {
    SESA_REQUIRE(a.M % 4 == 0, SESA_ERR_INVALID, "tdf: M %d must be a multiple of 4", a.M);
    return tdf_block_rows(a.M) == 256 ? launch_tdf_t<2, false, true>(x3, a, batch, st)
                                      : launch_tdf_t<1, false, true>(x3, a, batch, st);
  }
  SESA_REQUIRE(a.K % 8 == 0, SESA_ERR_INVALID, "tdf: K %d must be a multiple of 8", a.K);
  return tdf_block_rows(a.M) == 256 ? launch_tdf_t<2, true, false>(x3, a, batch, st)
                                    : launch_tdf_t<1, true, false>(x3, a, batch, st);
}

}  // namespace sesa
