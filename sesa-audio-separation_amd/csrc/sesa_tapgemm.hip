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

#include <algorithm>
#include <atomic>
#include <cstdlib>
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

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
// fp16 operands (SESA_PREC_F16 / F16W2 TFC convs): the same 8 x 16-bit fragment registers, read as fp16
__device__ __forceinline__ f32x16 mfma32h(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                0);
}
__device__ __forceinline__ uint32_t pack2h(float a, float b) {  // round-to-nearest-even fp16 pair
  return (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)a) | ((uint32_t)__builtin_bit_cast(uint16_t, (_Float16)b) << 16);
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
  for (int c = threadIdx.x; c < in.C_in; c += blockDim.x) {  // (act_split launches < kThreads threads)
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
// F16 (PRE, no XTRA, X3 = false): the fp16 plane of act_f16 against the fp16 weight image, one
// v_mfma_f32_32x32x16_f16 pass (the transposed up-convs of MDX23C's fp16mix)
template <int KH, int KW, int S, int PAD, int TM, int BN, int WM, bool X3, bool UPS, bool XTRA, bool PRE,
          bool F16 = false>
__global__ void __launch_bounds__(kThreads, 2) tap_gemm_kernel(ConvArgs a) {
  static_assert(!F16 || (PRE && !XTRA && !X3), "fp16: a pre-activated fp16 plane, no shortcut");
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
  constexpr int W1_ITEMS = ((X3 ? 2 : 1) * W1_BYTES / 16 + kThreads - 1) / kThreads;
  static_assert(A_ITEMS <= 32, "valid mask");
  f32x4 areg[A_ITEMS];  // native vectors: HIP's float4/uint4 structs copy via memcpy and defeat SROA
  u32x4 wreg[W_ITEMS];
  uint32_t avalid = 0;

  // source of chunk kc: (src, local channel offset, first concatenated channel, is-extra)
  auto chunk_src = [&](int kc, auto EXT, Src& src, int& cl0, int& k0) {
    constexpr bool ext = decltype(EXT)::value;
    k0 = (ext ? kc - a.n_chunks : kc) * kConvBK;
    const GemmIn& g = ext ? a.xin : a.in;
    const int s = k0 < g.C_split ? 0 : 1;
    src = pick_src(g, s);
    cl0 = k0 - (s ? g.C_split : 0);
  };

  auto load_chunk = [&](int kc, auto EXT) {
    constexpr bool ext = decltype(EXT)::value;
    Src src;
    int cl0, k0;
    chunk_src(kc, EXT, src, cl0, k0);
    const int w16 = ext ? (X3 ? 2 : 1) * W1_BYTES / 16 : W16;
    const u32x4* wsrc = reinterpret_cast<const u32x4*>(
        wblk + (ext ? (int64_t)a.n_chunks * W_BYTES + (int64_t)(kc - a.n_chunks) * W1_BYTES
                    : (int64_t)kc * W_BYTES));
    constexpr int WI = ext ? W1_ITEMS : W_ITEMS;
    Unroll<0, WI>::run([&](auto I) {
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
          if constexpr (!F16) areg[2 * i + 1] = *reinterpret_cast<const f32x4*>(src.lo + idx);
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

  auto store_chunk = [&](int kc, auto EXT) {
    constexpr bool ext = decltype(EXT)::value;
    Src src;
    int cl0, k0;
    chunk_src(kc, EXT, src, cl0, k0);
    const int w16 = ext ? (X3 ? 2 : 1) * W1_BYTES / 16 : W16;
    u32x4* wdst = reinterpret_cast<u32x4*>(W_hi);
    constexpr int WI = ext ? W1_ITEMS : W_ITEMS;
    Unroll<0, WI>::run([&](auto I) {
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
        if constexpr (F16) acc[i][j] = mfma32h(ah[i], bh[j], acc[i][j]);
        else acc[i][j] = mfma32(ah[i], bh[j], acc[i][j]);
      }
  };

  // Main K loop over the normalised input (all taps, fully unrolled), then -- XTRA only -- a
  // separate loop over the raw shortcut chunks (centre tap), so neither loop body carries the
  // other's code and register pressure.
  using kMain = std::false_type;
  using kExt = std::integral_constant<bool, XTRA>;
  load_chunk(0, kMain{});
  for (int kc = 0; kc < a.n_chunks; ++kc) {
    __syncthreads();  // previous chunk's fragment reads are done (and sc/sh are built)
    store_chunk(kc, kMain{});
    __syncthreads();
    if (kc + 1 < a.n_chunks) load_chunk(kc + 1, kMain{});
    else if (XTRA && n_total > a.n_chunks) load_chunk(kc + 1, kExt{});
#pragma unroll
    for (int tap = 0; tap < TAPS; ++tap) mfma_tap(tap / KW, tap % KW, tap, W_BYTES);
  }
  if (XTRA) {
    for (int kc = a.n_chunks; kc < n_total; ++kc) {
      __syncthreads();
      store_chunk(kc, kExt{});
      __syncthreads();
      if (kc + 1 < n_total) load_chunk(kc + 1, kExt{});
      mfma_tap(CTAP / KW, CTAP % KW, 0, W1_BYTES);
    }
  }

  // ---- epilogue ----
  // InstanceNorm statistics in fp64 from the first add on: E[x^2] - E[x]^2 is formed in double at the
  // consumer, so channels whose |mean| >> std (large norm beta, DC offsets) keep their precision
  double ssum[NI], ssq[NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) { ssum[j] = 0.0; ssq[j] = 0.0; }
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
        ssum[j] += (double)v;
        ssq[j] = fma((double)v, (double)v, ssq[j]);
      }
    }
  }
  if (a.out.stats) {
    // reduce over the two lane halves, then over the WM waves sharing these columns (LDS)
    __syncthreads();
    double* red = reinterpret_cast<double*>(smem);  // [WM][BN][2]
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
      double s0 = 0.0, s1 = 0.0;
#pragma unroll
      for (int w = 0; w < WM; ++w) {
        s0 += red[(w * BN + n) * 2 + 0];
        s1 += red[(w * BN + n) * 2 + 1];
      }
      const int ncol = nb * BN + n;
      const int co = UPS ? ncol % C_out : ncol;
      if ((UPS ? ncol < a.n_cols : co < C_out)) {
        double* st = a.out.stats + ((int64_t)b * C_out + co) * 2;
        atomicAdd(st + 0, s0);
        atomicAdd(st + 1, s1);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// conv3x3_db_kernel: the TFC 3x3 convolutions (mdx23c_tfc_tdf_v3.py:104-112, 121-129) on the
// pre-activated bf16 hi/lo planes of act_split, with LDS DOUBLE-BUFFERING and one barrier per K
// chunk.  512 threads (8 waves, 2 per SIMD, one workgroup per CU): tile 16 rows (t) x 32 columns
// (f) x 64 output channels, wave w owns output rows 2w, 2w+1 (MI = 2) x 64 channels (NI = 2).
// Per 16-channel chunk one stage holds the 18x34 input halo (hi + lo, 39 KB) and the 9-tap weight
// image (hi + lo, 36 KB); two stages = 152 KB.  Iteration k: MFMAs on stage k&1 while the
// registers holding chunk k+1 (loaded during iteration k-1) are written to stage (k+1)&1, then
// chunk k+2 is loaded to registers, then one barrier.  Twice the positions per workgroup of
// tap_gemm_kernel halves the weight traffic per FLOP.
// XTRA: the raw block input rides along as extra K over the centre tap (the 1x1 shortcut, :126,
// :137): its chunks load only the 16x32 inner positions (fp32, split in registers).
// Weight image and A-image layouts are exactly tap_gemm_kernel's (same host packing).
// EPI (ablation knob for tools/conv_bench.hip; the product uses 0): 1 = store without statistics,
// 2 = no epilogue.
// ACT: the main input is the RAW fp32 producer output (one or two channel-concatenated sources, mode
// SRC_NORM_GELU) and the consumer's InstanceNorm affine + exact GELU + bf16 hi/lo split run in the
// staging step (same arithmetic as act_split_kernel, so the operands are bit-identical), instead of a
// separate act_split pass over HBM (8 B per element).  The per-channel affine of this batch item is
// built once per workgroup into LDS (kActMaxC channels).  Each thread stages a fixed 8-channel half of
// every chunk (tid & 1), so its 8 (scale, shift) pairs are two ds_read_b128 per chunk.
// F16 (SESA_PREC_F16 / SESA_PREC_F16W2, X3 = true): the main chunks run on v_mfma_f32_32x32x16_f16 with
// the activation rounded once to fp16 (one A image: act_split's fp16 plane, or the fused staging's fp16
// pack) against the fp16 weight image (F16 = 1, one pass) or its fp16 hi + lo pair (F16 = 2, two
// passes: the weights to ~2^-22); the fused 1x1 shortcut chunks stay bf16x3.
// MI4 (F16 = 1, pre-activated input): 32-row tiles, each wave 4 output rows x 64 channels (128
// accumulators), main loop dx-major -- per dx the MI + 2 = 6 halo-row A fragments are read once and serve
// the 3 dy taps (4 x 2 MFMAs each) -- so 0.5 LDS fragment reads per MFMA instead of 1.  A stage then
// holds only the images the mode reads (one A, one W: 55 KB); the shortcut stages keep their bf16 hi / lo
// layout (78 KB), so a stage is the larger of the two.
constexpr int kActMaxC = 1024;
// MDMA (MI4 only): the main chunks are staged by LDS-DMA (buffer_load ... lds) instead of through VGPRs: each lane's
// source offset for its halo slot is computed ONCE per tile (out-of-image halo slots get an offset past num_records,
// so the hardware writes zeros -- no clamping, masking or select per chunk), the chunk advance is folded into the
// buffer resource base (SALU), and one counted wait + barrier per chunk replaces the register staging
// (load_item / store_main: ~200 VALU and 7 ds_write_b128 per thread per chunk).  The A image is padded to whole
// 1-KiB DMA pieces (37 KiB), so a stage is 55 KiB and two stages sit in the same LDS as before.
// SCR = 3 (MDMA only): the fused 1x1 shortcut INTERLEAVED with the main chunks -- shortcut chunk kc rides in main
// iteration kc: its W1 image (hi + lo, 4 KiB) is DMA'd into the main stage beside W, and each lane loads its own
// A fragments (4 rows x 32 B of the raw fp32 block input, 32 VGPRs) one iteration ahead, so the HBM stream of the
// raw input runs under the MFMA-bound main loop instead of in a phase of its own after it (where it was bound by
// the bytes a CU keeps in flight).  Shortcut chunks beyond n_main (decoder blocks: the block input has 2 C
// channels) run on the per-wave DMA ring afterwards, as SCR = 2.
template <bool X3, bool XTRA, int EPI = 0, bool ACT = false, int F16 = 0, bool MI4 = false, int SCR = 0,
          int SCD = 2, bool ORD = false, int MDMA = 0>
__global__ void __launch_bounds__(512, 1) conv3x3_db_kernel(ConvArgs a) {
  static_assert(F16 == 0 || X3, "the fp16 modes keep the shortcut chunks bf16x3");
  static_assert(!MDMA || (MI4 && F16 == 1 && !ACT), "MDMA: the fp16 32-row tile on pre-activated planes");
  static_assert(!MI4 || (F16 == 1 && !ACT), "MI4: fp16 single pass on pre-activated planes");
  static_assert(!SCR || (XTRA && X3), "SCR: the bf16x3 fused shortcut from registers / per-wave LDS-DMA");
  static_assert(SCR < 2 || MI4, "SCR 2 / 3: the 32-row tile (one wave = 4 rows of 32 positions)");
  static_assert(SCR != 3 || MDMA, "SCR 3: the interleaved shortcut rides the LDS-DMA main loop");
  constexpr bool SCI = SCR == 3;
  constexpr bool ALO = X3 && F16 == 0;  // main chunks read an A lo image
  constexpr bool WLO = X3 && F16 != 1;  // main chunks read a W lo image
  constexpr int NT = 512;
  constexpr int MI = MI4 ? 4 : 2;
  constexpr int TM = 8 * MI, WM = 8, NI = 2, BN = 64;
  constexpr int HT = TM + 2, HW = kTF + 2, NPOS = HT * HW;
  constexpr int A_BYTES = NPOS * 32;           // one (hi or lo) image
  constexpr int W_BYTES = 9 * BN * 32;
  constexpr int W1_BYTES = BN * 32;
  // main stage: [A hi][A lo if ALO][W hi][W lo if WLO]; shortcut stage: [A hi][A lo][W1 hi][W1 lo]
  constexpr int A_IMG_M = MDMA ? (A_BYTES + 1023) / 1024 * 1024 : A_BYTES;   // MDMA: whole 1-KiB pieces
  constexpr int WOFF_M = MDMA ? A_IMG_M : (ALO ? 2 : 1) * A_BYTES;
  constexpr int WOFF_X = 2 * A_BYTES;
  constexpr int W1OFF_M = WOFF_M + (WLO ? 2 : 1) * W_BYTES;   // SCI: the shortcut chunk's W1 image (hi + lo)
  constexpr int STAGE_M = W1OFF_M + (SCI ? 2 * W1_BYTES : 0);
  constexpr int STAGE_X = XTRA ? WOFF_X + 2 * W1_BYTES : 0;
  constexpr int STAGE = MI4 ? (STAGE_M > STAGE_X ? STAGE_M : STAGE_X) : 2 * A_BYTES + 2 * W_BYTES;
  // (one LDS array: the ACT affine table sits past the two stages)
  // SCR 2: the shortcut phase's per-wave rings take the whole 160 KiB (8 waves x kScrWave)
  constexpr int kScrWave = 2 * 8192 + 4096;
  constexpr int SMEM_B = 2 * STAGE + (ACT ? 2 * kActMaxC * 4 : 0);
  __shared__ __attribute__((aligned(16))) char smem[SCR >= 2 && 8 * kScrWave > SMEM_B ? 8 * kScrWave : SMEM_B];
  float* act_sc = reinterpret_cast<float*>(smem + 2 * STAGE);
  float* act_sh = act_sc + kActMaxC;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wm = tid >> 6;
  const int l32 = lane & 31, h = lane >> 5;

  // XCD-aware block order, as tap_gemm_kernel: the NB channel blocks of a tile run together
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
  const int t_in0 = t0 - 1, f_in0 = f0 - 1;
  const int n_main = a.n_chunks;
  const uint16_t* wblk = a.w + (int64_t)nb * (n_main * W_BYTES + (XTRA ? a.x_chunks * W1_BYTES : 0));
  const Src src = pick_src(a.in, 0);
  const int C = src.C;
  if constexpr (ACT) build_affine(a.in, b, act_sc, act_sh);   // ordered before use by the first barrier

  f32x16 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  constexpr int P_ITEMS = (NPOS * 2 + NT - 1) / NT;           // (position, 8-ch half): 16 B hi + 16 B lo
  constexpr int W16 = (WLO ? 2 : 1) * W_BYTES / 16;
  constexpr int W_ITEMS = (W16 + NT - 1) / NT;
  constexpr int X_ITEMS = TM * kTF * 4 / NT;                 // ext: (inner position, 4-ch group) fp32
  constexpr int W1_16 = (X3 ? 2 : 1) * W1_BYTES / 16;
  static_assert(2 * P_ITEMS >= X_ITEMS && W_ITEMS >= 1 && W1_16 <= NT, "staging");
  f32x4 areg[2 * P_ITEMS];
  u32x4 wreg[W_ITEMS];
  uint32_t avalid = 0;  // per staging item: inside the input image (else stored as zeros)

  auto load_w = [&](int kc) {
    const u32x4* wsrc = reinterpret_cast<const u32x4*>(wblk + (int64_t)kc * W_BYTES);
    Unroll<0, W_ITEMS>::run([&](auto I) {
      const int e = tid + I * NT;
      wreg[I] = wsrc[e < W16 ? e : W16 - 1];
    });
  };
  auto store_w = [&](char* stg) {
    u32x4* wdst = reinterpret_cast<u32x4*>(stg + (MI4 ? WOFF_M : 2 * A_BYTES));
    Unroll<0, W_ITEMS>::run([&](auto I) {
      const int e = min(tid + I * NT, W16 - 1);  // duplicates write identical values
      wdst[e] = wreg[I];
    });
  };
  // Staging item i of chunk kc: (halo position, 8-channel half).  Straight-line (no branches, so the
  // scheduler can spread it under the MFMAs): surplus threads repeat the last item; out-of-image halo
  // positions load a clamped address and are zeroed at store time (nothing waits on the load here).
  auto load_item = [&](auto I, int kc) {
    constexpr int i = decltype(I)::value;
    const int cl0 = kc * kConvBK;
    const int e = min(tid + i * NT, NPOS * 2 - 1);
    const int p = e >> 1, hf = e & 1;
    const int hr = p / HW, hc = p - hr * HW;
    const int ti = t_in0 + hr, fi = f_in0 + hc;
    const bool ok = ti >= 0 && ti < a.T_in && fi >= 0 && fi < a.F_in;
    const int tc = min(max(ti, 0), a.T_in - 1), fc = min(max(fi, 0), a.F_in - 1);
    if constexpr (ACT) {
      // raw fp32: 8 channels = 32 contiguous bytes (the same 4 B per element as the hi + lo planes); the
      // chunk's source (chunks never straddle the concatenation: C_split % 16 == 0)
      const int s1 = cl0 >= a.in.C_split;
      const float* xp = s1 ? a.in.src[1].ptr : a.in.src[0].ptr;
      const int xc = s1 ? a.in.src[1].C : a.in.src[0].C;
      const int xl0 = cl0 - (s1 ? a.in.C_split : 0);
      const f32x4* xq =
          reinterpret_cast<const f32x4*>(xp + (((int64_t)b * a.T_in + tc) * a.F_in + fc) * xc + xl0 + 8 * hf);
      areg[2 * i] = xq[0];
      areg[2 * i + 1] = xq[1];
    } else {
      const int64_t idx = (((int64_t)b * a.T_in + tc) * a.F_in + fc) * C + cl0 + 8 * hf;
      areg[2 * i] = *reinterpret_cast<const f32x4*>(src.hi + idx);
      if constexpr (ALO) areg[2 * i + 1] = *reinterpret_cast<const f32x4*>(src.lo + idx);
    }
    avalid = (avalid & ~(1u << i)) | ((uint32_t)ok << i);
  };
  auto load_main = [&](int kc) {
    load_w(kc);
    Unroll<0, P_ITEMS>::run([&](auto I) { load_item(I, kc); });
  };
  // ACT: the (scale, shift) pairs of this thread's 8 channels of chunk kc (LDS table)
  f32x4 aff[4];
  auto load_aff = [&](int kc) {
    const int c = kc * kConvBK + 8 * (tid & 1);
    aff[0] = *reinterpret_cast<const f32x4*>(act_sc + c);
    aff[1] = *reinterpret_cast<const f32x4*>(act_sc + c + 4);
    aff[2] = *reinterpret_cast<const f32x4*>(act_sh + c);
    aff[3] = *reinterpret_cast<const f32x4*>(act_sh + c + 4);
  };
  // ACT: pair q (channels 2q, 2q+1) of item i -> packed bf16 hi / lo words.  act_split_kernel's
  // arithmetic, y = GELU(fma(x, scale, shift)), then hi / lo; scalar f32 ops (packed v_pk_* f32 VALU
  // beside MFMAs costs extra issue cycles, MI355X_MICROARCH.md constants table; the file is built with
  // -fno-slp-vectorize so they stay scalar) -- per component the same operations as gelu_erf2, so the
  // operands are bit-identical to act_split's.  Branch-free: the out-of-image mask is ANDed into the
  // packed words (a select compiled to an exec-masked branch around the GELU).
  uint32_t hw[P_ITEMS][4], lw[P_ITEMS][4];
  auto xform_pair = [&](auto I, auto Q) {
    constexpr int i = decltype(I)::value, q = decltype(Q)::value;
    const uint32_t keep = 0u - ((avalid >> i) & 1u);
    const f32x4 xv = areg[2 * i + (q >> 1)];
    const float x0 = xv[(q & 1) * 2], x1 = xv[(q & 1) * 2 + 1];
    const float s0 = aff[q >> 1][(q & 1) * 2], s1 = aff[q >> 1][(q & 1) * 2 + 1];
    const float h0_ = aff[2 + (q >> 1)][(q & 1) * 2], h1_ = aff[2 + (q >> 1)][(q & 1) * 2 + 1];
    const float y0 = gelu_erf(fmaf(x0, s0, h0_));
    const float y1 = gelu_erf(fmaf(x1, s1, h1_));
    if constexpr (F16 != 0) {
      hw[i][q] = pack2h(y0, y1) & keep;
    } else {
      __bf16 h0, l0, h1, l1;
      split_bf16(y0, h0, l0);
      split_bf16(y1, h1, l1);
      hw[i][q] = pack2(h0, h1) & keep;
      lw[i][q] = pack2(l0, l1) & keep;
    }
  };
  auto item_off = [&](int i) {
    const int e = min(tid + i * NT, NPOS * 2 - 1);
    const int p = e >> 1, hf = e & 1;
    return p * 32 + ((hf ^ ((p >> 3) & 1)) << 4);
  };
  auto write_item = [&](auto I, char* stg) {
    constexpr int i = decltype(I)::value;
    const int off = item_off(i);
    *reinterpret_cast<u32x4*>(stg + off) = u32x4{hw[i][0], hw[i][1], hw[i][2], hw[i][3]};
    if (ALO) *reinterpret_cast<u32x4*>(stg + A_BYTES + off) = u32x4{lw[i][0], lw[i][1], lw[i][2], lw[i][3]};
  };
  auto store_main = [&](char* stg, int kc) {
    store_w(stg);
    if constexpr (ACT) {
      load_aff(kc);
      Unroll<0, P_ITEMS>::run([&](auto I) {
        Unroll<0, 4>::run([&](auto Q) { xform_pair(I, Q); });
        write_item(I, stg);
      });
    } else {
      Unroll<0, P_ITEMS>::run([&](auto I) {
        constexpr int i = decltype(I)::value;
        const int off = item_off(i);
        const bool ok = (avalid >> i) & 1u;
        const f32x4 z = {0.f, 0.f, 0.f, 0.f};
        *reinterpret_cast<f32x4*>(stg + off) = ok ? areg[2 * i] : z;
        if (ALO) *reinterpret_cast<f32x4*>(stg + A_BYTES + off) = ok ? areg[2 * i + 1] : z;
      });
    }
  };
  // ext chunk kx (0-based over the shortcut input's channels): raw fp32, inner positions only
  auto load_ext = [&](int kx) {
    const u32x4* wsrc =
        reinterpret_cast<const u32x4*>(wblk + (int64_t)n_main * W_BYTES + (int64_t)kx * W1_BYTES);
    wreg[0] = wsrc[tid < W1_16 ? tid : W1_16 - 1];
    const int k0 = kx * kConvBK;
    const int s = k0 < a.xin.C_split ? 0 : 1;
    const Src xs = pick_src(a.xin, s);
    const int cl0 = k0 - (s ? a.xin.C_split : 0);
    Unroll<0, X_ITEMS>::run([&](auto I) {
      constexpr int i = decltype(I)::value;
      const int e = tid + i * NT;
      const int p = e >> 2, g = e & 3;
      const int r = p / kTF, cc = p - r * kTF;
      const int ti = t0 + r, fi = f0 + cc;
      const int tc = min(ti, a.T_in - 1);
      areg[i] = *reinterpret_cast<const f32x4*>(xs.ptr + (((int64_t)b * a.T_in + tc) * a.F_in + fi) * xs.C +
                                                  cl0 + 4 * g);
      if (i == 0) avalid = 0;
      avalid |= (uint32_t)(ti < a.T_in) << i;
    });
  };
  auto store_ext = [&](char* stg) {
    char* A_hi = stg;
    char* A_lo = stg + A_BYTES;
    u32x4* wdst = reinterpret_cast<u32x4*>(stg + WOFF_X);
    wdst[min(tid, W1_16 - 1)] = wreg[0];
    Unroll<0, X_ITEMS>::run([&](auto I) {
      constexpr int i = decltype(I)::value;
      const int e = tid + i * NT;
      const int pi = e >> 2, g = e & 3;
      const int r = pi / kTF, cc = pi - r * kTF;
      const int p = (r + 1) * HW + cc + 1;  // halo coordinates of the centre-tap window
      const int off = p * 32 + ((((g >> 1) ^ ((p >> 3) & 1))) << 4) + ((g & 1) << 3);
      const bool ok = (avalid >> i) & 1u;
      __bf16 hi[4], lo[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) split_bf16(ok ? areg[i][q] : 0.f, hi[q], lo[q]);
      *reinterpret_cast<uint2*>(A_hi + off) = make_uint2(pack2(hi[0], hi[1]), pack2(hi[2], hi[3]));
      if (X3) *reinterpret_cast<uint2*>(A_lo + off) = make_uint2(pack2(lo[0], lo[1]), pack2(lo[2], lo[3]));
    });
  };
  // Fragment registers are double-buffered across taps: the LDS reads of tap t+1 are issued before
  // the MFMAs of tap t, so only the first tap of a chunk waits on LDS latency.
  struct Frags {
    bf16x8 ah[MI], al[MI], bh[NI], bl[NI];
  };
  // EXT: a shortcut chunk (bf16x3 in every mode); else a main chunk (ALO / WLO)
  auto read_frags = [&](Frags& fr, const char* stg, int dy, int dx, int wt, int wimg, auto EXT) {
    constexpr bool rd_al = decltype(EXT)::value ? X3 : ALO;
    constexpr bool rd_bl = decltype(EXT)::value ? X3 : WLO;
    const char* A_hi = stg;
    const char* A_lo = stg + A_BYTES;
    const char* W_hi = stg + (decltype(EXT)::value || !MI4 ? 2 * A_BYTES : WOFF_M);
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int row = wm * MI + i;
      const int p = (row + dy) * HW + l32 + dx;
      const int off = p * 32 + ((h ^ ((p >> 3) & 1)) << 4);
      fr.ah[i] = *reinterpret_cast<const bf16x8*>(A_hi + off);
      if (rd_al) fr.al[i] = *reinterpret_cast<const bf16x8*>(A_lo + off);
    }
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int p = wt * BN + j * 32 + l32;
      const int off = p * 32 + ((h ^ ((p >> 3) & 1)) << 4);
      fr.bh[j] = *reinterpret_cast<const bf16x8*>(W_hi + off);
      if (rd_bl) fr.bl[j] = *reinterpret_cast<const bf16x8*>(W_hi + wimg + off);
    }
  };
  auto mfma_group = [&](const Frags& fr, int i, int j, auto EXT) {
    if constexpr (F16 != 0 && !decltype(EXT)::value) {
      if constexpr (F16 == 2) acc[i][j] = mfma32h(fr.ah[i], fr.bl[j], acc[i][j]);
      acc[i][j] = mfma32h(fr.ah[i], fr.bh[j], acc[i][j]);
    } else {
      if (X3) {
        acc[i][j] = mfma32(fr.al[i], fr.bh[j], acc[i][j]);
        acc[i][j] = mfma32(fr.ah[i], fr.bl[j], acc[i][j]);
      }
      acc[i][j] = mfma32(fr.ah[i], fr.bh[j], acc[i][j]);
    }
  };
  auto mfmas = [&](const Frags& fr, auto EXT) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) mfma_group(fr, i, j, EXT);
  };
  constexpr std::false_type kMain{};
  constexpr std::true_type kExt{};

  // ---- main chunks: straight-line pipelined body, clamped (redundant) prefetch at the tail ----
  // MDMA: this wave's DMA pieces per chunk (A pieces first, then the W image's), wave-uniform piece index
  constexpr int MD_A_PC = A_IMG_M / 1024, MD_W_END = MD_A_PC + W_BYTES / 1024;
  constexpr int MD_PC = MD_W_END + (SCI ? 2 * W1_BYTES / 1024 : 0), MD_PPW = (MD_PC + 7) / 8;
  uint32_t mdo[MDMA ? MD_PPW : 1];   // per-lane source byte offsets (A: from the chunk-0 plane base; W / W1: image)
  const int wv = __builtin_amdgcn_readfirstlane(wm);
  // SCI: shortcut chunks 0 .. n_sci - 1 interleaved with the main chunks, the rest on the ring afterwards
  const int n_sci = SCI ? min(a.x_chunks, n_main) : 0;
  auto md_issue = [&](int kc, char* stg) {
    if constexpr (MDMA) {
      const uint32_t plane_bytes = (uint32_t)((int64_t)a.T_in * a.F_in * C * 2);
      const char* abase = reinterpret_cast<const char*>(src.hi + (int64_t)b * a.T_in * a.F_in * C) + kc * 32;
      const char* wbase = reinterpret_cast<const char*>(wblk) + (int64_t)kc * 2 * W_BYTES;
      const __amdgpu_buffer_rsrc_t ra =
          __builtin_amdgcn_make_buffer_rsrc((void*)const_cast<char*>(abase), (short)0, (int)(plane_bytes - kc * 32), 0x00020000);
      const __amdgpu_buffer_rsrc_t rw =
          __builtin_amdgcn_make_buffer_rsrc((void*)const_cast<char*>(wbase), (short)0, W_BYTES, 0x00020000);
      // SCI: shortcut chunk kc's W1 image (hi + lo), stored after the main chunks' images
      const char* w1base = reinterpret_cast<const char*>(wblk + (int64_t)n_main * W_BYTES) + (int64_t)kc * 2 * W1_BYTES;
      const __amdgpu_buffer_rsrc_t rw1 =
          __builtin_amdgcn_make_buffer_rsrc((void*)const_cast<char*>(w1base), (short)0, 2 * W1_BYTES, 0x00020000);
#pragma unroll
      for (int i = 0; i < MD_PPW; ++i) {
        // (the voffset as int: an unsigned lvalue here made the host pass silently drop this kernel's launch stub)
        const int pc = wv + 8 * i;
        if (pc < MD_A_PC)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (__attribute__((address_space(3))) void*)(stg + pc * 1024), 16,
                                                   (int)mdo[i], 0, 0, 0);
        else if (pc < MD_W_END)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(
              rw, (__attribute__((address_space(3))) void*)(stg + WOFF_M + (pc - MD_A_PC) * 1024), 16, (int)mdo[i], 0, 0, 0);
        else if (pc < MD_PC && kc < n_sci)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(
              rw1, (__attribute__((address_space(3))) void*)(stg + W1OFF_M + (pc - MD_W_END) * 1024), 16, (int)mdo[i], 0, 0,
              0);
      }
    }
  };
  // SCI: this lane's A fragments of shortcut chunk kx -- rows wm MI + i, position f0 + l32, channels 8 h .. 8 h + 7
  // of the chunk (32 contiguous bytes of the raw fp32 input; rows past T_in clamped here, zeroed at the split)
  f32x4 xa[SCI ? MI : 1][2];
  auto sci_load = [&](int kx) {
    if constexpr (SCI) {
      const int k0 = kx * kConvBK;
      const int sx = k0 < a.xin.C_split ? 0 : 1;
      const Src xs = pick_src(a.xin, sx);
      const int cl0 = k0 - (sx ? a.xin.C_split : 0) + 8 * h;
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int t = min(t0 + wm * MI + i, a.T_in - 1);
        const f32x4* q =
            reinterpret_cast<const f32x4*>(xs.ptr + (((int64_t)b * a.T_in + t) * a.F_in + f0 + l32) * xs.C + cl0);
        xa[i][0] = q[0];
        xa[i][1] = q[1];
      }
    }
  };
  // SCI: the bf16x3 MFMAs of the shortcut chunk in xa against the W1 image of stage stg (the ring's arithmetic)
  auto sci_mma = [&](const char* stg) {
    if constexpr (SCI) {
      const char* wimg = stg + W1OFF_M;
      bf16x8 bh[NI], bl[NI];
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int p = j * 32 + l32;
        const int off = p * 32 + ((h ^ ((p >> 3) & 1)) << 4);
        bh[j] = *reinterpret_cast<const bf16x8*>(wimg + off);
        bl[j] = *reinterpret_cast<const bf16x8*>(wimg + W1_BYTES + off);
      }
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const bool ok = t0 + wm * MI + i < a.T_in;
        __bf16 hv[8], lv[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) split_bf16(ok ? xa[i][q >> 2][q & 3] : 0.f, hv[q], lv[q]);
        const bf16x8 ah = bf16x8{hv[0], hv[1], hv[2], hv[3], hv[4], hv[5], hv[6], hv[7]};
        const bf16x8 al = bf16x8{lv[0], lv[1], lv[2], lv[3], lv[4], lv[5], lv[6], lv[7]};
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          acc[i][j] = mfma32(al, bh[j], acc[i][j]);
          acc[i][j] = mfma32(ah, bl[j], acc[i][j]);
          acc[i][j] = mfma32(ah, bh[j], acc[i][j]);
        }
      }
    }
  };
  auto main_phase = [&]() __attribute__((always_inline)) {
    if constexpr (MDMA) {
      // halo slot of lane l in A piece pc: position p = 32 pc + l / 2, LDS half-slot l & 1, which holds channel half
      // (l & 1) ^ ((p >> 3) & 1) (the fragment reads' swizzle)
      constexpr uint32_t kOOB = 0x80000000u;
#pragma unroll
      for (int i = 0; i < MD_PPW; ++i) {
        const int pc = wv + 8 * i;
        uint32_t v = kOOB;
        if (pc < MD_A_PC) {
          const int p = pc * 32 + (lane >> 1);
          const int hr = p / HW, hc = p - hr * HW;
          const int ti = t_in0 + hr, fi = f_in0 + hc;
          const int hf = (lane & 1) ^ ((p >> 3) & 1);
          if (p < NPOS && ti >= 0 && ti < a.T_in && fi >= 0 && fi < a.F_in)
            v = (uint32_t)((((int64_t)ti * a.F_in + fi) * C + 8 * hf) * 2);
        } else if (pc < MD_W_END) {
          v = (uint32_t)((pc - MD_A_PC) * 1024 + lane * 16);
        } else if (pc < MD_PC) {
          v = (uint32_t)((pc - MD_W_END) * 1024 + lane * 16);
        }
        mdo[i] = v;
      }
      md_issue(0, smem);
      if (SCI && n_sci > 0) sci_load(0);
    } else {
      load_main(0);
      if constexpr (ACT) __syncthreads();   // the LDS affine table, before the first staging step reads it
      store_main(smem, 0);
      load_main(min(1, n_main - 1));
      __syncthreads();
    }
    for (int kc = 0; kc < n_main; ++kc) {
      char* cur = smem + (kc & 1) * STAGE;
      char* nxt = smem + ((kc + 1) & 1) * STAGE;
      if constexpr (MDMA) {
        // chunk kc landed for every wave (each waits for its own pieces; the barrier joins them), and every wave's
        // fragment reads of the other stage (chunk kc - 1) retired -- chunk kc + 1 goes there
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        // SCI: shortcut chunk kc (its fragments landed with the wait above) before the next DMA is in flight, so a
        // compiler-inserted wait for xa cannot hold up on chunk kc + 1's pieces; then its successor's loads
        if (SCI && kc < n_sci) sci_mma(cur);
        if (kc + 1 < n_main) md_issue(kc + 1, nxt);
        if (SCI && kc + 1 < n_sci) sci_load(kc + 1);
      }
      Frags fr[2];
      if constexpr (MI4) {
        // dx-major: the 6 halo-row A fragments of column shift dx, then the 3 dy taps (B double-buffered)
        const char* Wm = cur + WOFF_M;
        auto read_b = [&](bf16x8* bq, int tap) __attribute__((always_inline)) {
  #pragma unroll
          for (int j = 0; j < NI; ++j) {
            const int p = tap * BN + j * 32 + l32;
            bq[j] = *reinterpret_cast<const bf16x8*>(Wm + p * 32 + ((h ^ ((p >> 3) & 1)) << 4));
          }
        };
        bf16x8 bq[2][NI];
        read_b(bq[0], 0);
        Unroll<0, 3>::run([&](auto DX) {
          constexpr int dx = decltype(DX)::value;
          bf16x8 ar[MI + 2];
  #pragma unroll
          for (int r = 0; r < MI + 2; ++r) {
            const int p = (wm * MI + r) * HW + l32 + dx;
            ar[r] = *reinterpret_cast<const bf16x8*>(cur + p * 32 + ((h ^ ((p >> 3) & 1)) << 4));
          }
          Unroll<0, 3>::run([&](auto DY) {
            constexpr int dy = decltype(DY)::value, q = dx * 3 + dy;  // q: order of this tap
            constexpr int nq = q + 1, ntap = (nq % 3) * 3 + nq / 3;   // the next tap in dx-major order
            if (nq < 9) read_b(bq[nq & 1], ntap);
  #pragma unroll
            for (int i = 0; i < MI; ++i)
  #pragma unroll
              for (int j = 0; j < NI; ++j) acc[i][j] = mfma32h(ar[i + dy], bq[q & 1][j], acc[i][j]);
            if constexpr (!MDMA) {
              if (q == 1) {
                store_main(nxt, min(kc + 1, n_main - 1));
                load_main(min(kc + 2, n_main - 1));
              }
            }
          });
        });
        if constexpr (MDMA) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // reads of `cur` retired
        else __syncthreads();
        continue;
      }
      read_frags(fr[0], cur, 0, 0, 0, W_BYTES, kMain);
      if constexpr (!ACT) {
        Unroll<0, 9>::run([&](auto T) {
          constexpr int tap = decltype(T)::value;
          if (tap + 1 < 9) read_frags(fr[(tap + 1) & 1], cur, (tap + 1) / 3, (tap + 1) % 3, tap + 1, W_BYTES, kMain);
          mfmas(fr[tap & 1], kMain);
          if (tap == 1) {
            // stage chunk kc+1 (in registers since the previous iteration) under the MFMAs, then start
            // loading chunk kc+2; past the end both are harmless repeats of the last chunk
            store_main(nxt, min(kc + 1, n_main - 1));
            load_main(min(kc + 2, n_main - 1));
          }
        });
      } else {
        // ACT: the staging of chunk kc+1 is VALU-heavy (~27 VALU per element, ~6 per MFMA), and left to
        // the scheduler it clumps after one tap, idling the matrix pipe while both waves of a SIMD do it
        // together.  So it is cut into 12 slices -- one (item, channel pair) each, ~54 VALU -- pinned by
        // sched_barrier between the 36 three-MFMA accumulator groups of the iteration (one slice after
        // every third group); an item's LDS write and its reload with chunk kc+2 follow its last pair.
        const int ks = min(kc + 1, n_main - 1), kl = min(kc + 2, n_main - 1);
        load_aff(ks);
        Unroll<0, 9>::run([&](auto T) {
          constexpr int tap = decltype(T)::value;
          if (tap + 1 < 9) read_frags(fr[(tap + 1) & 1], cur, (tap + 1) / 3, (tap + 1) % 3, tap + 1, W_BYTES, kMain);
          Unroll<0, MI * NI>::run([&](auto G) {
            constexpr int g = decltype(G)::value, gi = 4 * tap + g;
            mfma_group(fr[tap & 1], g / NI, g % NI, kMain);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (gi == 0) {
              store_w(nxt);
              load_w(kl);
            }
            if constexpr (gi % 3 == 1 && gi / 3 < 4 * P_ITEMS) {
              constexpr int sl = gi / 3, it = sl / 4, q = sl % 4;
              xform_pair(std::integral_constant<int, it>{}, std::integral_constant<int, q>{});
              if constexpr (q == 3) {
                write_item(std::integral_constant<int, it>{}, nxt);
                load_item(std::integral_constant<int, it>{}, kl);
              }
            }
            __builtin_amdgcn_sched_barrier(0);
          });
        });
      }
      __syncthreads();
    }
    if constexpr (MDMA) {
      __builtin_amdgcn_s_barrier();   // every wave's reads of the last stage retired (the shortcut ring reuses it)
      asm volatile("" ::: "memory");
    }
  };
  // ---- fused 1x1 shortcut chunks (centre tap) ----
  auto shortcut_phase = [&]() __attribute__((always_inline)) {
    if constexpr (XTRA && (SCR == 2 || SCR == 3)) {
      // Per-wave LDS-DMA ring: each wave streams only its own 4 rows x 32 positions x 16 channels of the raw
      // fp32 block input (8 KiB = eight 1-KiB buffer_load ... lds pieces per chunk) into a private 2-slot ring
      // and the chunk's W1 image (hi + lo, 4 KiB = four pieces) into a private slot: 20 KiB per wave, the whole
      // 160 KiB LDS.  No barrier and no VGPR staging: a CU keeps two chunks of the input (128 KiB) in flight
      // where the LDS-staged form keeps one (64 KiB) behind one barrier per chunk.  Every transfer is a DMA, so
      // the compiler tracks no register loads here and the counted waits below are the only ones.
      // x image per slot: position p = 32 row + f holds 16 channels in 64 B, its 16-B quads permuted by
      // (f >> 2) & 3 (conflict-free ds_read_b128 groups).
      const int nx = a.x_chunks;
      const int kb = n_sci;   // SCR 3: the chunks the main loop did not take (nx - kb even: host check)
      const char* w1 = reinterpret_cast<const char*>(wblk + (int64_t)n_main * W_BYTES);
      char* ring = smem + wm * kScrWave;
      char* wimg = ring + 2 * 8192;
      const __amdgpu_buffer_rsrc_t rw =
          __builtin_amdgcn_make_buffer_rsrc((void*)const_cast<char*>(w1), (short)0, nx * 2 * W1_BYTES, 0x00020000);
      auto issue_x = [&](int kx, int slot) {
        const int k0 = kx * kConvBK;
        const int sx = k0 < a.xin.C_split ? 0 : 1;
        const Src xs = pick_src(a.xin, sx);
        const int cl0 = k0 - (sx ? a.xin.C_split : 0);
        const int fl = lane >> 2, qs = lane & 3;   // this lane's LDS slot: position fl of the piece, quad qs
        // buffer resource over this batch item's image (32-bit offsets)
        const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
            (void*)const_cast<float*>(xs.ptr + (int64_t)b * a.T_in * a.F_in * xs.C), (short)0,
            (int)((int64_t)a.T_in * a.F_in * xs.C * 4), 0x00020000);
#pragma unroll
        for (int pc = 0; pc < 8; ++pc) {
          const int i = pc >> 1, f = (pc & 1) * 16 + fl;
          const int t = min(t0 + wm * MI + i, a.T_in - 1);
          const int q = qs ^ ((f >> 2) & 3);        // the channel quad stored in slot qs
          const uint32_t voff = (uint32_t)((((int64_t)t * a.F_in + f0 + f) * xs.C + cl0 + 4 * q) * 4);
          __builtin_amdgcn_raw_ptr_buffer_load_lds(
              rx, (__attribute__((address_space(3))) void*)(ring + slot * 8192 + pc * 1024), 16, voff, 0, 0, 0);
        }
      };
      auto issue_w = [&](int kx) {
#pragma unroll
        for (int pc = 0; pc < 4; ++pc)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (__attribute__((address_space(3))) void*)(wimg + pc * 1024), 16,
                                                   (uint32_t)(kx * 2 * W1_BYTES + pc * 1024 + lane * 16), 0, 0, 0);
      };
      // the main phase's last barrier retired every wave's reads of the stages this ring overwrites.
      // Straight-line loop unrolled by the two slots; every step issues its refills (clamped to the last chunk
      // at the tail: harmless repeats), so the count of transfers behind a chunk's is the same on every path:
      // issue order x(k) W1(k) x(k+1) | W1(k+1) x(k+2) | ..., and chunk k is complete once only x(k+1)'s 8
      // pieces remain.  nx - kb is even (host check).
      if (kb < nx) {
      issue_x(kb, 0);
      issue_w(kb);
      issue_x(min(kb + 1, nx - 1), 1);
      for (int kx0 = kb; kx0 < nx; kx0 += 2) {
        Unroll<0, 2>::run([&](auto S) {
          constexpr int slot = decltype(S)::value;
          const int kx = kx0 + slot;
          asm volatile("s_waitcnt vmcnt(8)" ::: "memory");    // x(kx) and W1(kx) landed
          bf16x8 bh[NI], bl[NI];
#pragma unroll
          for (int j = 0; j < NI; ++j) {
            const int p = j * 32 + l32;
            const int off = p * 32 + ((h ^ ((p >> 3) & 1)) << 4);
            bh[j] = *reinterpret_cast<const bf16x8*>(wimg + off);
            bl[j] = *reinterpret_cast<const bf16x8*>(wimg + W1_BYTES + off);
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // W1(kx) in registers: its slot is free
          issue_w(min(kx + 1, nx - 1));
          const char* img = ring + slot * 8192;
#pragma unroll
          for (int i = 0; i < MI; ++i) {
            const bool ok = t0 + wm * MI + i < a.T_in;
            const int pb = (i * 32 + l32) * 64;
            const int sw = (l32 >> 2) & 3;
            const f32x4 x0 = *reinterpret_cast<const f32x4*>(img + pb + (((2 * h) ^ sw) << 4));
            const f32x4 x1 = *reinterpret_cast<const f32x4*>(img + pb + (((2 * h + 1) ^ sw) << 4));
            __bf16 hv[8], lv[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) split_bf16(ok ? (q < 4 ? x0[q] : x1[q - 4]) : 0.f, hv[q], lv[q]);
            const bf16x8 ah = bf16x8{hv[0], hv[1], hv[2], hv[3], hv[4], hv[5], hv[6], hv[7]};
            const bf16x8 al = bf16x8{lv[0], lv[1], lv[2], lv[3], lv[4], lv[5], lv[6], lv[7]};
#pragma unroll
            for (int j = 0; j < NI; ++j) {
              acc[i][j] = mfma32(al, bh[j], acc[i][j]);
              acc[i][j] = mfma32(ah, bl[j], acc[i][j]);
              acc[i][j] = mfma32(ah, bh[j], acc[i][j]);
            }
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this slot's reads done before the refill
          issue_x(min(kx + 2, nx - 1), slot);
        });
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");         // the tail's repeat refills landed
      }
      __syncthreads();   // the epilogue's statistics reduction reuses the LDS
    } else if constexpr (XTRA && SCR == 1) {
      // Register-direct form: every lane loads its own A fragments straight from the raw fp32 block input
      // (inner position (t0 + row, f0 + l32), channels 8h..8h+7 of the chunk: 32 contiguous bytes, the
      // MFMA's row / k layout) and its B fragments from the packed W1 image (same byte layout as the LDS copy),
      // splits A into bf16 hi / lo in registers and runs the bf16x3 MFMAs in the same order as the LDS form
      // (bit-identical results).  No LDS and no barrier: each wave streams its own rows with SCD chunks in
      // flight, so the phase is bounded by bytes in flight per CU, not by one chunk's latency per barrier.
      const int nx = a.x_chunks;
      const char* w1 = reinterpret_cast<const char*>(wblk + (int64_t)n_main * W_BYTES);
      // the W1 images (hi + lo, 4 KiB per chunk) of up to kScrPiece chunks at a time live in LDS (free once the
      // main loop's last barrier has passed): copied by LDS-DMA, one barrier per piece, then ds_read_b128 per
      // fragment -- registers stay for the x stream
      constexpr int kScrPiece = (2 * STAGE) / (2 * W1_BYTES) < 32 ? (2 * STAGE) / (2 * W1_BYTES) : 32;
      auto copy_w1 = [&](int k0, int k1) {
        const int pieces = (k1 - k0) * (2 * W1_BYTES / 1024);
        for (int q = wm; q < pieces; q += 8)
          __builtin_amdgcn_global_load_lds(w1 + (int64_t)k0 * 2 * W1_BYTES + q * 1024 + lane * 16,
                                           (__attribute__((address_space(3))) void*)(smem + q * 1024), 16, 0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      };
      f32x4 xa[SCD][MI][2];
      auto ld_row = [&](int s, int i, int kx) {
        const int k0 = kx * kConvBK;
        const int sx = k0 < a.xin.C_split ? 0 : 1;
        const Src xs = pick_src(a.xin, sx);
        const int cl0 = k0 - (sx ? a.xin.C_split : 0) + 8 * h;
        const int t = min(t0 + wm * MI + i, a.T_in - 1);
        const f32x4* q =
            reinterpret_cast<const f32x4*>(xs.ptr + (((int64_t)b * a.T_in + t) * a.F_in + f0 + l32) * xs.C + cl0);
        xa[s][i][0] = q[0];
        xa[s][i][1] = q[1];
      };
      int piece0 = 0, piece1 = min(nx, kScrPiece);
      copy_w1(piece0, piece1);
      Unroll<0, SCD>::run([&](auto S) {
        constexpr int s = decltype(S)::value;
  #pragma unroll
        for (int i = 0; i < MI; ++i) ld_row(s, i, min(s, nx - 1));
      });
      for (int kx0 = 0; kx0 < nx; kx0 += SCD) {
        Unroll<0, SCD>::run([&](auto S) {
          constexpr int s = decltype(S)::value;
          const int kx = kx0 + s;
          if (kx < nx) {
            if (kx == piece1) {   // next piece of W1 images (every wave reaches this with the same kx)
              __syncthreads();    // all reads of the previous piece are done
              piece0 = piece1;
              piece1 = min(nx, piece1 + kScrPiece);
              copy_w1(piece0, piece1);
            }
            const char* wl = smem + (kx - piece0) * 2 * W1_BYTES;
            bf16x8 bh[NI], bl[NI];
  #pragma unroll
            for (int j = 0; j < NI; ++j) {
              const int p = j * 32 + l32;
              const int off = p * 32 + ((h ^ ((p >> 3) & 1)) << 4);
              bh[j] = *reinterpret_cast<const bf16x8*>(wl + off);
              bl[j] = *reinterpret_cast<const bf16x8*>(wl + W1_BYTES + off);
            }
            const bool refill = kx + SCD < nx;
            // row by row: split row i, refill its registers with chunk kx + SCD, then its MFMAs -- so only one
            // row's hi / lo fragments are live beside the in-flight loads
  #pragma unroll
            for (int i = 0; i < MI; ++i) {
              const bool ok = t0 + wm * MI + i < a.T_in;
              __bf16 hv[8], lv[8];
  #pragma unroll
              for (int q = 0; q < 8; ++q) split_bf16(ok ? xa[s][i][q >> 2][q & 3] : 0.f, hv[q], lv[q]);
              const bf16x8 ah = bf16x8{hv[0], hv[1], hv[2], hv[3], hv[4], hv[5], hv[6], hv[7]};
              const bf16x8 al = bf16x8{lv[0], lv[1], lv[2], lv[3], lv[4], lv[5], lv[6], lv[7]};
              if (refill) ld_row(s, i, kx + SCD);
  #pragma unroll
              for (int j = 0; j < NI; ++j) {
                acc[i][j] = mfma32(al, bh[j], acc[i][j]);
                acc[i][j] = mfma32(ah, bl[j], acc[i][j]);
                acc[i][j] = mfma32(ah, bh[j], acc[i][j]);
              }
            }
          }
        });
      }
      __syncthreads();   // the epilogue's statistics reduction reuses the LDS
    } else if (XTRA && a.x_chunks > 0) {
      const int nx = a.x_chunks;
      load_ext(0);
      store_ext(smem);
      load_ext(min(1, nx - 1));
      __syncthreads();
      for (int kx = 0; kx < nx; ++kx) {
        char* cur = smem + (kx & 1) * STAGE;
        char* nxt = smem + ((kx + 1) & 1) * STAGE;
        Frags fr;
        read_frags(fr, cur, 1, 1, 0, W1_BYTES, kExt);
        mfmas(fr, kExt);
        store_ext(nxt);
        load_ext(min(kx + 2, nx - 1));
        __syncthreads();
      }
    }
  };
  // ORD: with a fused shortcut, every other group of 8 workgroups runs the shortcut phase (HBM-bound: the
  // raw block input, 4 B per channel) BEFORE the main phase (MFMA-bound).  At one workgroup per CU the grid's
  // workgroups otherwise move through the two phases in lockstep -- the whole chip MFMA-bound, then the whole
  // chip HBM-bound; split orders keep half the CUs in each.  (Only the fp32 summation order of the two
  // phases' contributions differs between the orders.)
  if (ORD && XTRA && ((blockIdx.x >> 3) & 1)) {
    shortcut_phase();
    main_phase();
  } else {
    main_phase();
    shortcut_phase();
  }

  if constexpr (EPI == 2) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) asm volatile("" ::"v"(acc[i][j]));
    return;
  }
  // ---- epilogue: fp32 store + per-channel sum / sum-of-squares for the next InstanceNorm ----
  // Statistics: fp32 partial sums over each lane's 16-value runs (relative error ~ a few ulp of a
  // 16-term sum), fp64 from there on -- E[x^2] - E[x]^2 is formed in double at the consumer, so channels
  // whose |mean| >> std (large norm beta, DC offsets) keep their precision (stress golden
  // mdx23c_small_stress.npz).  (Per-value fp64 accumulation cost ~3 % of the level-0 conv.)
  double ssum[NI], ssq[NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) { ssum[j] = 0.0; ssq[j] = 0.0; }
  const int C_out = a.out.C_out;
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int co = nb * BN + j * 32 + l32;
    if (co >= C_out) continue;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int t = t0 + wm * MI + i;
      if (t >= a.T_out) continue;
      float ps = 0.f, pq = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int f = f0 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int64_t idx = (((int64_t)b * a.T_out + t) * a.F_out + f) * C_out + co;
        const float v = acc[i][j][r];
        __builtin_nontemporal_store(v, a.out.ptr + idx);  // streamed: 7.6 GB per level-0 launch
        ps += v;
        pq = fmaf(v, v, pq);
      }
      if constexpr (EPI == 1) continue;
      ssum[j] += (double)ps;
      ssq[j] += (double)pq;
    }
  }
  if (EPI == 0 && a.out.stats) {
    double* red = reinterpret_cast<double*>(smem);  // [WM][BN][2] (the last barrier retired all LDS reads)
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
    for (int n = tid; n < BN; n += NT) {
      double s0 = 0.0, s1 = 0.0;
#pragma unroll
      for (int w = 0; w < WM; ++w) {
        s0 += red[(w * BN + n) * 2 + 0];
        s1 += red[(w * BN + n) * 2 + 1];
      }
      const int co = nb * BN + n;
      if (co < C_out) {
        double* st = a.out.stats + ((int64_t)b * C_out + co) * 2;
        atomicAdd(st + 0, s0);
        atomicAdd(st + 1, s1);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// conv3x3_wino_kernel: the TFC 3x3 convolutions (mdx23c_tfc_tdf_v3.py:104-112, 121-129) as Winograd
// F(2, 3) along the frequency axis -- per output pair (f = 2j, 2j + 1) and input row r of the 3-row
// window, the 4-tap input transform
//     d_i = x[r][2j - 1 + i]  (i = 0..3, zero padding),   V0 = d0 - d2, V1 = d1 + d2, V2 = d2 - d1, V3 = d1 - d3,
// the weight transform (per dy, host, fp64: U0 = w0, U1 = (w0 + w1 + w2) / 2, U2 = (w0 - w1 + w2) / 2,
// U3 = w2) and the output transform y(2j) = M0 + M1 + M2, y(2j + 1) = M1 - M2 - M3 with
//     M_p[pair][co] = sum_{dy, ci} V_p[row + dy][pair][ci] U_p[dy][ci][co]
// -- 12 MFMA taps per output pair where the direct form has 18 (2/3 of the MFMA work).  Each M_p is
// a bf16x3 contraction like the direct kernel's; the transforms are fp32 adds (V) and fp64 (U), so the
// result is the direct convolution to fp32 rounding (summation order differs).
//   * Input: the consumer's activation GELU(InstanceNorm(x)) as fp32 (act_split's SRC_ACT32 output).
//   * 512 threads (8 waves, one workgroup per CU), tile 16 rows (t) x 32 columns (f = 16 pairs) x 64
//     output channels; wave w owns rows 2w, 2w + 1 as ONE 32-row MFMA block (row = m >> 4, pair =
//     m & 15) x 64 channels x 4 points: acc[4][2] = 128 registers, and the output transform is in-lane.
//   * Stages: each 16-channel chunk is two stages, points {0, 1} then {2, 3}; a stage holds V for its
//     2 points over the 18 halo rows (hi + lo, 36 KB) and the 6-tap (2 points x 3 dy) weight image (24 KB);
//     two stages (120 KB) double-buffered with one barrier per stage, exactly the staging pipeline of
//     conv3x3_db_kernel (registers hold stage s + 2 while stage s + 1 is written under stage s's MFMAs).
//     A stage item is (halo row, pair, 8-channel half): 3 input positions -> 2 V values per channel.
//   * XTRA (the fused 1x1 shortcut, :126, :137): the centre-tap-only kernel transforms to U1 = w / 2,
//     U2 = -w / 2, so each 16-channel chunk of the raw block input is one more stage with V1 = x(2j) +
//     x(2j + 1), V2 = x(2j + 1) - x(2j) on the 16 inner rows (2 k-steps into acc[1], acc[2]).
//   * Epilogue: output transform, fp32 stores (non-temporal), per-channel sums for the next
//     InstanceNorm (fp32 over each lane's 32-value runs, fp64 beyond), as conv3x3_db_kernel.
constexpr int kWinoRows = 18;                             // halo rows of a 16-row tile
constexpr int kWinoVPlane = 2 * kWinoRows * 16 * 32;      // 2 points x 18 rows x 16 pairs x 16 ch bf16
constexpr int kWinoWPlane = 6 * 64 * 32;                  // 6 taps (2 points x 3 dy) x 64 co x 16 ci bf16
constexpr int kWinoXPlane = 2 * 64 * 32;                  // shortcut stage: 2 taps (points 1, 2)
constexpr int kWinoStage = 2 * kWinoVPlane + 2 * kWinoWPlane;
constexpr int kWinoWImg = kWinoWPlane;                    // uint16 per main-stage weight image (hi + lo)
constexpr int kWinoXImg = kWinoXPlane;                    // uint16 per shortcut-stage image (hi + lo)
// raw input of halo rows 16, 17 (fp32 [2][34][16] = 4352 B), one buffer per chunk parity; each LDS-DMA
// wave-instruction writes a whole 1 KiB, so a buffer spans the 5 pieces (5 KiB) -- the last piece's
// surplus lanes must not land in the other chunk's rows
constexpr int kWinoRawRows = 5 * 1024;
static_assert(kWinoWImg == kWinoMainImg && kWinoXImg == kWinoShortImg, "host packing (sesa_tapgemm.hpp)");

// FRDB: fragment registers double-buffered across k-steps (the next k-step's LDS reads issued before
// this one's MFMAs); else read just before use (24 registers fewer).
// ABL (ablation knob for tools/conv_bench.hip; the product uses 0): 1 = no V split / LDS writes,
// 2 = no weight DMA, 3 = no staging at all (MFMAs, fragment reads and barriers only), 4 = no halo rows
// 16, 17 (wave 0's second items).
// SLC: the staging of the next stage sliced between the k-steps (else all of it after k-step 1).
template <bool X3, bool XTRA, int EPI = 0, bool FRDB = false, int ABL = 0, bool SLC = false>
__global__ void __launch_bounds__(512, 1) conv3x3_wino_kernel(ConvArgs a) {
  constexpr int NT = 512, TM = 16, BN = 64, NI = 2;
  // two stages, then the raw input of halo rows 16, 17 for two chunks ([2 rows][34 positions][16 ch] fp32)
  __shared__ __attribute__((aligned(16))) char smem[2 * kWinoStage + 2 * kWinoRawRows];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wm = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, h = lane >> 5;

  // XCD-aware block order, as conv3x3_db_kernel: the NB channel blocks of a tile run together
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
  const int n_main = a.n_chunks;
  const int n_x = XTRA ? a.x_chunks : 0;
  const int n_stage = 2 * n_main + n_x;
  const uint16_t* wblk = a.w + (int64_t)nb * ((int64_t)n_main * 2 * kWinoWImg + (int64_t)n_x * kWinoXImg);
  const float* X = a.in.src[0].ptr;
  const int C = a.in.C_in;
  // shortcut sources as plain values (a select between fields of the kernel-argument struct can become a
  // select of their addresses, which puts the whole struct in scratch and every derived load on flat)
  const float* const xs_p0 = a.xin.src[0].ptr;
  const float* const xs_p1 = a.xin.src[1].ptr;
  const int xs_c0 = a.xin.src[0].C, xs_c1 = a.xin.src[1].C, xs_split = a.xin.C_split;

  f32x16 acc[4][NI];
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[p][j][r] = 0.f;

  // ---- staging: registers hold the next stage's inputs (3 positions x 8 channels per item, halo rows
  // 0..15); the 64 items of halo rows 16, 17 are wave 0's second items, staged from a raw copy of those
  // two rows that wave 0 brings into LDS by DMA one chunk ahead (registers for a second item would
  // spill; spreading those items over all waves as one channel per lane measured slower) ----
  f32x4 areg[1][6];
  uint32_t aval = 0;  // bit 3 * item + position: inside the input image (else zero)
  // weight images go global -> LDS by LDS-DMA (buffer resource over this block's images, 32-bit offsets;
  // the packed image is the LDS image, 1 KiB per wave-instruction: 3 pieces per wave for a main stage,
  // 1 for a shortcut stage)
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(wblk), (short)0, (int)(((int64_t)n_main * 2 * kWinoWImg + (int64_t)n_x * kWinoXImg) * 2),
      0x00020000);
  auto dma_w = [&](char* stg, int s) __attribute__((always_inline)) {
    char* wdst = stg + 2 * kWinoVPlane;
    if (!XTRA || s < 2 * n_main) {
      const uint32_t base = (uint32_t)(s * kWinoWImg * 2);
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const int pc = wm + 8 * i;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (__attribute__((address_space(3))) void*)(wdst + pc * 1024), 16,
                                                 base + pc * 1024 + lane * 16, 0, 0, 0);
      }
    } else {
      const uint32_t base = (uint32_t)((2 * n_main * kWinoWImg + (s - 2 * n_main) * kWinoXImg) * 2);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (__attribute__((address_space(3))) void*)(wdst + wm * 1024), 16,
                                               base + wm * 1024 + lane * 16, 0, 0, 0);
    }
  };
  auto item_geom = [&](int it, int& hr, int& pair, int& hh) __attribute__((always_inline)) {
    const int e = it ? NT + (tid & 63) : tid;
    hr = e >> 5;
    pair = (e >> 1) & 15;
    hh = e & 1;
  };
  auto load_stage = [&](int s) __attribute__((always_inline)) {
    if (!XTRA || s < 2 * n_main) {
      const int kc = s >> 1, pp = s & 1;
      aval = 0;
      Unroll<0, 1>::run([&](auto IT) {
        constexpr int it = decltype(IT)::value;
        int hr, pair, hh;
        item_geom(it, hr, pair, hh);
        const int ti = t0 - 1 + hr;
        const int tc = min(max(ti, 0), a.T_in - 1);
        Unroll<0, 3>::run([&](auto Q) {
          constexpr int q = decltype(Q)::value;
          const int fi = f0 + 2 * pair - 1 + pp + q;
          const bool ok = ti >= 0 && ti < a.T_in && fi >= 0 && fi < a.F_in;
          const int fc = min(max(fi, 0), a.F_in - 1);
          const f32x4* xp =
              reinterpret_cast<const f32x4*>(X + (((int64_t)b * a.T_in + tc) * a.F_in + fc) * C + kc * kConvBK + 8 * hh);
          areg[it][2 * q] = xp[0];
          areg[it][2 * q + 1] = xp[1];
          aval |= (uint32_t)ok << (3 * it + q);
        });
      });
    } else {
      const int kx = s - 2 * n_main;
      const int k0 = kx * kConvBK;
      const bool s1 = k0 >= xs_split;
      const float* xp0 = s1 ? xs_p1 : xs_p0;
      const int xc = s1 ? xs_c1 : xs_c0;
      const int cl0 = k0 - (s1 ? xs_split : 0);
      const int r = tid >> 5, pair = (tid >> 1) & 15, hh = tid & 1;
      const int ti = t0 + r;
      const int tc = min(ti, a.T_in - 1);
      aval = 0;
      Unroll<0, 2>::run([&](auto Q) {
        constexpr int q = decltype(Q)::value;
        const int fi = f0 + 2 * pair + q;
        const f32x4* xp = reinterpret_cast<const f32x4*>(xp0 + (((int64_t)b * a.T_in + tc) * a.F_in + fi) * xc + cl0 + 8 * hh);
        areg[0][2 * q] = xp[0];
        areg[0][2 * q + 1] = xp[1];
        aval |= (uint32_t)(ti < a.T_in) << q;
      });
    }
  };
  // V byte offset of (point slot pl, halo row hr, pair, channel half hh) within a plane
  auto v_off = [](int pl, int hr, int pair, int hh) __attribute__((always_inline)) {
    return ((pl * kWinoRows + hr) * 16 + pair) * 32 + ((hh ^ ((pair >> 3) & 1)) << 4);
  };
  auto put8 = [&](char* stg, int off, const float (&v)[8]) __attribute__((always_inline)) {
    uint32_t hw[4], lw[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      __bf16 h0, l0, h1, l1;
      split_bf16(v[2 * q], h0, l0);
      split_bf16(v[2 * q + 1], h1, l1);
      hw[q] = pack2(h0, h1);
      lw[q] = pack2(l0, l1);
    }
    *reinterpret_cast<u32x4*>(stg + off) = u32x4{hw[0], hw[1], hw[2], hw[3]};
    if (X3) *reinterpret_cast<u32x4*>(stg + kWinoVPlane + off) = u32x4{lw[0], lw[1], lw[2], lw[3]};
  };
  // V values of one staging item of stage s: it 0 = this thread's item (registers), it 1 = wave 0's item
  // of halo rows 16, 17 (the LDS raw rows); returns the two V slots' LDS offsets
  auto v_item = [&](auto IT, int s, float (&va)[8], float (&vb)[8], int& o0, int& o1) __attribute__((always_inline)) {
    constexpr int it = decltype(IT)::value;
    if (XTRA && s >= 2 * n_main) {  // shortcut stage: V1 = x(2j) + x(2j + 1), V2 = x(2j + 1) - x(2j)
      const int r = tid >> 5, pair = (tid >> 1) & 15, hh = tid & 1;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const float e0 = (aval & 1u) ? areg[0][c >> 2][c & 3] : 0.f;
        const float e1 = ((aval >> 1) & 1u) ? areg[0][2 + (c >> 2)][c & 3] : 0.f;
        va[c] = e0 + e1;
        vb[c] = e1 - e0;
      }
      o0 = v_off(0, r + 1, pair, hh);
      o1 = v_off(1, r + 1, pair, hh);
      return;
    }
    const int pp = s & 1;
    int hr, pair, hh;
    item_geom(it, hr, pair, hh);
    f32x4 xq[6];
    uint32_t okb;
    if constexpr (it == 0) {
#pragma unroll
      for (int i = 0; i < 6; ++i) xq[i] = areg[0][i];
      okb = aval;
    } else {
      // halo rows 16, 17 from the raw rows wave 0 copied for this chunk
      const char* raw = smem + 2 * kWinoStage + ((s >> 1) & 1) * kWinoRawRows;
      const int ti = t0 - 1 + hr;
      okb = 0;
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int pos = 2 * pair + pp + q;  // relative to f0 - 1
        const int fi = f0 - 1 + pos;
        const f32x4* rp = reinterpret_cast<const f32x4*>(raw + (((hr - 16) * 34 + pos) * 16 + 8 * hh) * 4);
        xq[2 * q] = rp[0];
        xq[2 * q + 1] = rp[1];
        okb |= (uint32_t)(ti < a.T_in && fi >= 0 && fi < a.F_in) << q;
      }
    }
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const float q0 = (okb >> 0) & 1u ? xq[c >> 2][c & 3] : 0.f;
      const float q1 = (okb >> 1) & 1u ? xq[2 + (c >> 2)][c & 3] : 0.f;
      const float q2 = (okb >> 2) & 1u ? xq[4 + (c >> 2)][c & 3] : 0.f;
      // pp 0: (q0, q1, q2) = (d0, d1, d2) -> V0 = d0 - d2, V1 = d1 + d2
      // pp 1: (q0, q1, q2) = (d1, d2, d3) -> V2 = d2 - d1, V3 = d1 - d3
      va[c] = pp ? q1 - q0 : q0 - q2;
      vb[c] = pp ? q0 - q2 : q1 + q2;
    }
    o0 = v_off(0, hr, pair, hh);
    o1 = v_off(1, hr, pair, hh);
  };
  auto store_stage = [&](char* stg, int s) __attribute__((always_inline)) {
    float va[8], vb[8];
    int o0, o1;
    v_item(std::integral_constant<int, 0>{}, s, va, vb, o0, o1);
    put8(stg, o0, va);
    put8(stg, o1, vb);
    if (wm == 0 && (!XTRA || s < 2 * n_main)) {
      v_item(std::integral_constant<int, 1>{}, s, va, vb, o0, o1);
      put8(stg, o0, va);
      put8(stg, o1, vb);
    }
  };

  struct Frags {
    bf16x8 ah, al, bh[NI], bl[NI];
  };
  // k-step (point slot pl, dy) of a stage: A = V_pl at halo row 2 wm + (m >> 4) + dy, B = weight tap
  auto read_frags = [&](Frags& fr, const char* stg, int pl, int dy, int tap, int wplane) __attribute__((always_inline)) {
    const int pair = l32 & 15;
    const int off = v_off(pl, 2 * wm + (l32 >> 4) + dy, pair, h);
    fr.ah = *reinterpret_cast<const bf16x8*>(stg + off);
    if (X3) fr.al = *reinterpret_cast<const bf16x8*>(stg + kWinoVPlane + off);
    const char* W = stg + 2 * kWinoVPlane;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int p = tap * BN + j * 32 + l32;
      const int o = p * 32 + ((h ^ ((p >> 3) & 1)) << 4);
      fr.bh[j] = *reinterpret_cast<const bf16x8*>(W + o);
      if (X3) fr.bl[j] = *reinterpret_cast<const bf16x8*>(W + wplane + o);
    }
  };
  auto mfmas = [&](const Frags& fr, auto P) __attribute__((always_inline)) {
    constexpr int p = decltype(P)::value;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      if (X3) {
        acc[p][j] = mfma32(fr.al, fr.bh[j], acc[p][j]);
        acc[p][j] = mfma32(fr.ah, fr.bl[j], acc[p][j]);
      }
      acc[p][j] = mfma32(fr.ah, fr.bh[j], acc[p][j]);
    }
  };

  // wave 0: the raw input of halo rows 16, 17 (t0 + 15, t0 + 16) of chunk kc into its LDS copy
  // ([row][34 positions from f0 - 1][16 ch], lane-linear 16-B pieces; clamped addresses, the
  // out-of-image positions are masked when staged)
  auto dma_rows = [&](int kc) __attribute__((always_inline)) {
    char* raw = smem + 2 * kWinoStage + (kc & 1) * kWinoRawRows;
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(X) + (int64_t)b * a.T_in * a.F_in * C, (short)0,
        (int)((int64_t)a.T_in * a.F_in * C * 4), 0x00020000);
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const int e = min(lane + 64 * i, 2 * 34 * 4 - 1);
      const int r = e / 136, rem = e - r * 136, pos = rem >> 2, c4 = rem & 3;
      const int tc = min(t0 + 15 + r, a.T_in - 1);
      const int fc = min(max(f0 - 1 + pos, 0), a.F_in - 1);
      const uint32_t voff = (uint32_t)((((int64_t)tc * a.F_in + fc) * C + kc * kConvBK + 4 * c4) * 4);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (__attribute__((address_space(3))) void*)(raw + i * 1024), 16,
                                               voff, 0, 0, 0);
    }
  };
  // Wait for this wave's DMAs (weights of the next stage, wave 0's raw rows) while the raw loads issued
  // after them (for the stage after that) stay in flight: vmcnt counts in issue order, and the memory
  // clobbers keep the DMAs ahead of those loads.  Raw loads per stage: 6 (main), 4 (shortcut).
  auto wait_dma = [&](int s_loaded) __attribute__((always_inline)) {
    if (XTRA && s_loaded >= 2 * n_main) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  };
  // Producing stage s + 1 into `nxt` while stage s's MFMAs run, in slices pinned between the k-steps
  // (sched_barrier) so the two waves of a SIMD do not both stall their MFMA stream on one clump of VALU:
  //   k 0: weight DMA (+ wave 0's raw rows of a new chunk)   k 1: V of this thread's item, then the raw
  //   loads of stage s + 2 (registers free again: the longest lead)   k 2 / k 3: split + LDS writes of
  //   the two V slots   k 4: wave 0's item of halo rows 16, 17.
  struct Prod {
    int s1, s2;
    float va[8], vb[8];
    int o0, o1;
  };
  auto slice = [&](auto K, Prod& pr, char* nxt, int s) __attribute__((always_inline)) {
    constexpr int k = decltype(K)::value;
    if constexpr (ABL == 3) {
      if constexpr (k == 0) pr.s1 = pr.s2 = 2 * n_main + n_x;  // (wait_dma: vmcnt(6) / (4) still harmless)
      return;
    }
    if constexpr (ABL == 1 && k >= 2) return;
    if constexpr (ABL == 4 && k == 4) return;
    if constexpr (ABL == 2 && k == 0) {
      pr.s1 = min(s + 1, n_stage - 1);
      pr.s2 = min(s + 2, n_stage - 1);
      return;
    }
    if constexpr (k == 0) {
      pr.s1 = min(s + 1, n_stage - 1);
      pr.s2 = min(s + 2, n_stage - 1);
      // a new chunk's first stage: its rows 16, 17 (read from the next iteration on; that copy last
      // served chunk kc - 2)
      if (wm == 0 && pr.s2 < 2 * n_main && (pr.s2 & 1) == 0 && pr.s2 > s) dma_rows(pr.s2 >> 1);
      dma_w(nxt, pr.s1);
      asm volatile("" ::: "memory");
    } else if constexpr (k == 1) {
      v_item(std::integral_constant<int, 0>{}, pr.s1, pr.va, pr.vb, pr.o0, pr.o1);
      load_stage(pr.s2);
    } else if constexpr (k == 2) {
      put8(nxt, pr.o0, pr.va);
    } else if constexpr (k == 3) {
      put8(nxt, pr.o1, pr.vb);
    } else if constexpr (k == 4) {
      if (wm == 0 && (!XTRA || pr.s1 < 2 * n_main)) {
        float va[8], vb[8];
        int o0, o1;
        v_item(std::integral_constant<int, 1>{}, pr.s1, va, vb, o0, o1);
        put8(nxt, o0, va);
        put8(nxt, o1, vb);
      }
    }
  };

  if (wm == 0) {
    dma_rows(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  load_stage(0);
  store_stage(smem, 0);
  dma_w(smem, 0);
  asm volatile("" ::: "memory");
  load_stage(min(1, n_stage - 1));
  wait_dma(min(1, n_stage - 1));
  __syncthreads();
  for (int kc = 0; kc < n_main; ++kc) {
    Unroll<0, 2>::run([&](auto PP) {
      constexpr int pp = decltype(PP)::value;
      const int s = 2 * kc + pp;
      char* cur = smem + pp * kWinoStage;
      char* nxt = smem + (1 - pp) * kWinoStage;
      Prod pr;
      Frags fr[FRDB ? 2 : 1];
      if constexpr (FRDB) read_frags(fr[0], cur, 0, 0, 0, kWinoWPlane);
      Unroll<0, 6>::run([&](auto K) {
        constexpr int k = decltype(K)::value;
        if constexpr (FRDB) {
          if constexpr (k + 1 < 6)
            read_frags(fr[(k + 1) & 1], cur, (k + 1) / 3, (k + 1) % 3, k + 1, kWinoWPlane);
          mfmas(fr[k & 1], std::integral_constant<int, 2 * pp + k / 3>{});
        } else {
          read_frags(fr[0], cur, k / 3, k % 3, k, kWinoWPlane);
          mfmas(fr[0], std::integral_constant<int, 2 * pp + k / 3>{});
        }
        if constexpr (SLC) {
          __builtin_amdgcn_sched_barrier(0);
          slice(K, pr, nxt, s);
          __builtin_amdgcn_sched_barrier(0);
        } else if constexpr (k == 1) {
          Unroll<0, 5>::run([&](auto J) { slice(J, pr, nxt, s); });
        }
      });
      wait_dma(pr.s2);
      __syncthreads();
    });
  }
  if constexpr (XTRA) {
    for (int kx = 0; kx < n_x; ++kx) {
      const int s = 2 * n_main + kx;
      char* cur = smem + (kx & 1) * kWinoStage;
      char* nxt = smem + ((kx + 1) & 1) * kWinoStage;
      Prod pr;
      Frags fr[2];
      read_frags(fr[0], cur, 0, 1, 0, kWinoXPlane);
      read_frags(fr[1], cur, 1, 1, 1, kWinoXPlane);
      mfmas(fr[0], std::integral_constant<int, 1>{});
      slice(std::integral_constant<int, 0>{}, pr, nxt, s);
      slice(std::integral_constant<int, 1>{}, pr, nxt, s);
      mfmas(fr[1], std::integral_constant<int, 2>{});
      slice(std::integral_constant<int, 2>{}, pr, nxt, s);
      slice(std::integral_constant<int, 3>{}, pr, nxt, s);
      wait_dma(pr.s2);
      __syncthreads();
    }
  }

  if constexpr (EPI == 2) {
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
      for (int j = 0; j < NI; ++j) asm volatile("" ::"v"(acc[p][j]));
    return;
  }
  // ---- epilogue: output transform, fp32 stores, per-channel statistics ----
  double ssum[NI], ssq[NI];
  const int C_out = a.out.C_out;
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    ssum[j] = 0.0;
    ssq[j] = 0.0;
    const int co = nb * BN + j * 32 + l32;
    if (co >= C_out) continue;
#pragma unroll
    for (int hb = 0; hb < 2; ++hb) {  // r in [8 hb, 8 hb + 8): output row 2 wm + hb
      const int t = t0 + 2 * wm + hb;
      if (t >= a.T_out) continue;
      float ps = 0.f, pq = 0.f;
#pragma unroll
      for (int rr = 0; rr < 8; ++rr) {
        const int r = 8 * hb + rr;
        const int pair = ((r & 3) + 8 * (r >> 2) + 4 * h) & 15;
        const float m0 = acc[0][j][r], m1 = acc[1][j][r], m2 = acc[2][j][r], m3 = acc[3][j][r];
        const float ye = m0 + m1 + m2;
        const float yo = m1 - m2 - m3;
        const int64_t idx = (((int64_t)b * a.T_out + t) * a.F_out + f0 + 2 * pair) * C_out + co;
        __builtin_nontemporal_store(ye, a.out.ptr + idx);
        __builtin_nontemporal_store(yo, a.out.ptr + idx + C_out);
        ps += ye + yo;
        pq = fmaf(ye, ye, fmaf(yo, yo, pq));
      }
      ssum[j] += (double)ps;
      ssq[j] += (double)pq;
    }
  }
  if (EPI == 0 && a.out.stats) {
    double* red = reinterpret_cast<double*>(smem);  // [8 waves][BN][2] (the last barrier retired all LDS reads)
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
    for (int n = tid; n < BN; n += NT) {
      double s0 = 0.0, s1 = 0.0;
#pragma unroll
      for (int w = 0; w < 8; ++w) {
        s0 += red[(w * BN + n) * 2 + 0];
        s1 += red[(w * BN + n) * 2 + 1];
      }
      const int co = nb * BN + n;
      if (co < C_out) {
        double* st = a.out.stats + ((int64_t)b * C_out + co) * 2;
        atomicAdd(st + 0, s0);
        atomicAdd(st + 1, s1);
      }
    }
  }
}

// Sum of a double over the 16 lanes of each DPP row (every lane of the row gets the sum): xor 1 and
// xor 2 by quad_perm, then row_half_mirror (i <-> 7 - i) and row_mirror (i <-> 15 - i), each applied to
// both 32-bit halves.
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double x) {
  const uint64_t u = __builtin_bit_cast(uint64_t, x);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, CTRL, 0xF, 0xF, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), CTRL, 0xF, 0xF, false);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ double row16_sum(double x) {
  x += dpp_f64<0xB1>(x);   // quad_perm [1, 0, 3, 2]
  x += dpp_f64<0x4E>(x);   // quad_perm [2, 3, 0, 1]
  x += dpp_f64<0x141>(x);  // row_half_mirror
  x += dpp_f64<0x140>(x);  // row_mirror
  return x;
}

// ---------------------------------------------------------------------------------------------
// conv3x3_m16_kernel: the TFC 3x3 convolutions (mdx23c_tfc_tdf_v3.py:104-112, 121-129) on
// v_mfma_f32_16x16x32_bf16 -- the same cycles per FLOP as 32x32x16 but ~1.12x its FLOP/s under the
// power limit (MI355X_MICROARCH.md, DVFS) -- as a PERSISTENT kernel with LDS-DMA staging.
//   * Tile 16 rows (t) x 32 columns (f) x 64 output channels, 512 threads; wave w owns rows 2w, 2w+1:
//     4 position blocks (row, 16-column half) x 4 channel blocks of 16x16.
//   * K chunk = 16 input channels x 9 taps = 4.5 k-steps of 32: k-step s pairs taps 2s (lanes 0-31)
//     and 2s+1 (lanes 32-63); tap 8 of an even chunk is read into registers by lanes 0-31 and paired
//     with tap 8 of the next (odd) chunk, read by lanes 32-63 -- 9 full k-steps per chunk pair.
//   * Each stage (halo 18x34 hi + lo, 9-tap weight image hi + lo = 76 KiB) is filled by
//     global_load_lds_dwordx4 (lane-linear LDS destination; the host weight swizzle is undone in the
//     per-lane source offset; out-of-image halo lanes read zeros past the buffer range), two stages,
//     one counted wait + barrier per step.  Unswizzled 32-B position rows are conflict-free for the 16x16x32
//     fragment pattern (lane groups of ds_read_b128 see 8 distinct positions x both halves).
//   * Persistent: one workgroup per CU walks work items (b, tile, channel block) with stride
//     gridDim.x; the DMA of the next item's first chunk is issued under the current item's last
//     step, so no per-tile prologue is exposed, and the epilogue's stores drain under the next tile.
//   * XTRA: the 1x1 shortcut (:126, :137) as extra K over the centre tap, read from bf16 hi / lo
//     planes of the raw block input (act_split's second output), 32 channels per step.
// EPI (ablation knob for tools/conv_bench.hip; the product uses 0): 1 = no statistics, 2 = no epilogue.

template <bool X3, bool XTRA, int EPI = 0>
__global__ void __launch_bounds__(512, 1) conv3x3_m16_kernel(ConvArgs a, int n_work) {
  constexpr int TM = 16, BN = 64, HW = kTF + 2, NPOS = (TM + 2) * HW;
  constexpr int A_IMG = ((NPOS * 32 + 1023) / 1024) * 1024;  // 20 KiB per plane (612 x 32 B, padded)
  constexpr int W_IMG = 9 * BN * 32;                          // 18 KiB per plane
  constexpr int STAGE = 2 * A_IMG + 2 * W_IMG;                // 76 KiB
  constexpr int XA_IMG = TM * kTF * 64;                       // ext: 512 positions x 32 ch (32 KiB)
  constexpr int XW_IMG = BN * 64;                             // ext: 64 channels x 32 ch (4 KiB)
  constexpr int RED = 8 * BN * 2 * 8;                         // [wave][channel][sum, sumsq] fp64
  static_assert(2 * XA_IMG + 2 * XW_IMG <= STAGE && 2 * STAGE + RED <= 163840, "LDS budget");
  constexpr int NPL = X3 ? 2 : 1;                             // planes staged
  constexpr int A_PC = A_IMG / 1024, W_PC = W_IMG / 1024, XA_PC = XA_IMG / 1024, XW_PC = XW_IMG / 1024;
  constexpr int MAIN_PC = NPL * (A_PC + W_PC), EXT_PC = NPL * (XA_PC + XW_PC);
  constexpr int W_CHUNK = 2 * 9 * BN * 16;                    // uint16 per packed (hi, lo) chunk image
  constexpr int W1_CHUNK = 2 * BN * 16;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE + RED];
  double* red = reinterpret_cast<double*>(smem + 2 * STAGE);

  const int tid = threadIdx.x;
  int lane = tid & 63;  // re-materialised per step (below): keeps lane-derived addresses out of the hoisted set
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: piece loops and descriptors in SGPRs
  int fr = lane & 15, q = lane >> 4;
  const int tiles_f = a.F_out / kTF;
  const int NB = (a.n_cols + BN - 1) / BN;
  const int n_tiles = ((a.T_out + TM - 1) / TM) * tiles_f;
  const int per_b = n_tiles * NB;
  const int n_main = a.n_chunks;
  const int n_ext = XTRA ? a.x_chunks / 2 : 0;
  const int S = n_main + n_ext;
  const Src src = pick_src(a.in, 0);
  const int C = src.C;
  const int64_t w_nb = (int64_t)n_main * W_CHUNK + (XTRA ? (int64_t)a.x_chunks * W1_CHUNK : 0);

  struct Item {
    int b, t0, f0, nb;
  };
  // XCD-aware order within a batch item (as tap_gemm_kernel): ids 8g + x .. share XCD x, and the NB
  // channel blocks of a tile are 8 ids apart (same XCD, same round), so their input is read from L2
  auto decode = [&](int w) {
    Item it;
    it.b = w / per_b;
    const int id = w - it.b * per_b;
    const int full = (n_tiles / 8) * 8 * NB;
    int tile;
    if (id < full) {
      const int g = id / (8 * NB), r = id - g * 8 * NB;
      tile = g * 8 + (r & 7);
      it.nb = r >> 3;
    } else {
      const int r = id - full;
      tile = (n_tiles / 8) * 8 + r / NB;
      it.nb = r % NB;
    }
    it.t0 = (tile / tiles_f) * TM;
    it.f0 = (tile % tiles_f) * kTF;
    return it;
  };

  // ---- LDS-DMA issue of step s of item `it` into stage `stg` (wave-uniform piece loop) ----
  // buffer_load ... lds through per-item buffer resources: 32-bit per-lane offsets, and an offset past
  // num_records (out-of-image halo lanes) returns zeros, so padding costs no extra load or branch
  constexpr uint32_t kOOB = 0x80000000u;
  constexpr int kRsrcW3 = 0x00020000;  // raw buffer, gfx9 data format word
  auto rsrc = [](const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, kRsrcW3);
  };
  auto dma = [](__amdgpu_buffer_rsrc_t r, char* lds, uint32_t voff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, 0, 0, 0);
  };
  const uint32_t w_bytes = (uint32_t)(w_nb * 2);
  auto issue = [&](const Item& it, int s, char* stg) {
    const __amdgpu_buffer_rsrc_t rw = rsrc(a.w + (int64_t)it.nb * w_nb, w_bytes);
    if (!XTRA || s < n_main) {
      const int kc = s;
      const int64_t item = (int64_t)it.b * a.T_in * a.F_in * C;
      const uint32_t plane_bytes = (uint32_t)((int64_t)a.T_in * a.F_in * C * 2);
      const __amdgpu_buffer_rsrc_t rh = rsrc(src.hi + item, plane_bytes);
      const __amdgpu_buffer_rsrc_t rl = rsrc(src.lo + item, plane_bytes);
#pragma unroll
      for (int i = 0; i < (MAIN_PC + 7) / 8; ++i) {
        const int pc = wave + 8 * i;
        if (pc >= MAIN_PC) break;
        if (pc < NPL * A_PC) {
          const int plane = pc / A_PC, qq = pc - plane * A_PC;
          const int u = qq * 64 + lane, p = u >> 1, hf = u & 1;
          const int hr = p / HW, hc = p - hr * HW;
          const int ti = it.t0 - 1 + hr, fi = it.f0 - 1 + hc;
          const bool ok = p < NPOS && ti >= 0 && ti < a.T_in && fi >= 0 && fi < a.F_in;
          const uint32_t voff = ok ? (uint32_t)(((ti * a.F_in + fi) * C + kc * kConvBK + 8 * hf) * 2) : kOOB;
          dma(plane ? rl : rh, stg + plane * A_IMG + qq * 1024, voff);
        } else {
          const int pw = pc - NPL * A_PC;
          const int plane = pw / W_PC, qq = pw - plane * W_PC;
          const int u = qq * 64 + lane, e = u >> 1, hf = u & 1;
          dma(rw, stg + 2 * A_IMG + plane * W_IMG + qq * 1024,
              (uint32_t)((kc * W_CHUNK + plane * (W_CHUNK / 2) + 8 * (2 * e + (hf ^ ((e >> 3) & 1)))) * 2));
        }
      }
    } else {
      const int kx = s - n_main;  // 32-channel ext step over the shortcut planes
      const int Cx = a.xin.C_in;
      const int64_t item = (int64_t)it.b * a.T_in * a.F_in * Cx;
      const uint32_t plane_bytes = (uint32_t)((int64_t)a.T_in * a.F_in * Cx * 2);
      const __amdgpu_buffer_rsrc_t rh = rsrc(a.xin.src[0].hi + item, plane_bytes);
      const __amdgpu_buffer_rsrc_t rl = rsrc(a.xin.src[0].lo + item, plane_bytes);
#pragma unroll
      for (int i = 0; i < (EXT_PC + 7) / 8; ++i) {
        const int pc = wave + 8 * i;
        if (pc >= EXT_PC) break;
        if (pc < NPL * XA_PC) {
          const int plane = pc / XA_PC, qq = pc - plane * XA_PC;
          const int u = qq * 64 + lane, p = u >> 2, c16 = u & 3;
          const int kq = c16 ^ (((p >> 3) & 1) << 1);  // 64-B rows: 16-B unit swizzle for 16x16x32 reads
          const int ti = it.t0 + (p >> 5), fi = it.f0 + (p & 31);
          const uint32_t voff = ti < a.T_in ? (uint32_t)(((ti * a.F_in + fi) * Cx + kx * 32 + 8 * kq) * 2) : kOOB;
          dma(plane ? rl : rh, stg + plane * XA_IMG + qq * 1024, voff);
        } else {
          const int pw = pc - NPL * XA_PC;
          const int plane = pw / XW_PC, qq = pw - plane * XW_PC;
          const int u = qq * 64 + lane, n = u >> 2, c16 = u & 3;
          const int kq = c16 ^ (((n >> 3) & 1) << 1);
          const int hf = kq & 1;
          dma(rw, stg + 2 * XA_IMG + plane * XW_IMG + qq * 1024,
              (uint32_t)((n_main * W_CHUNK + (2 * kx + (kq >> 1)) * W1_CHUNK + plane * (W1_CHUNK / 2) +
                          8 * (2 * n + (hf ^ ((n >> 3) & 1)))) *
                         2));
        }
      }
    }
  };

  f32x4 acc[4][4];
  struct Frags {
    bf16x8 ah[4], al[4], bh[4], bl[4];
  };
  // main-chunk fragments of tap `tap` (per lane) from stage stg
  auto read_main = [&](Frags& f, const char* stg, int tap) {
    const int dy = tap / 3, dx = tap - 3 * (tap / 3);
    const int hf = q & 1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wave * 2 + (i >> 1), col = (i & 1) * 16 + fr;
      const int off = ((row + dy) * HW + col + dx) * 32 + hf * 16;
      f.ah[i] = *reinterpret_cast<const bf16x8*>(stg + off);
      if (X3) f.al[i] = *reinterpret_cast<const bf16x8*>(stg + A_IMG + off);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int off = 2 * A_IMG + (tap * BN + j * 16 + fr) * 32 + hf * 16;
      f.bh[j] = *reinterpret_cast<const bf16x8*>(stg + off);
      if (X3) f.bl[j] = *reinterpret_cast<const bf16x8*>(stg + W_IMG + off);
    }
  };
  auto read_ext = [&](Frags& f, const char* stg) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int p = (wave * 2 + (i >> 1)) * 32 + (i & 1) * 16 + fr;
      const int off = p * 64 + ((q ^ (((p >> 3) & 1) << 1)) << 4);
      f.ah[i] = *reinterpret_cast<const bf16x8*>(stg + off);
      if (X3) f.al[i] = *reinterpret_cast<const bf16x8*>(stg + XA_IMG + off);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = j * 16 + fr;
      const int off = 2 * XA_IMG + n * 64 + ((q ^ (((n >> 3) & 1) << 1)) << 4);
      f.bh[j] = *reinterpret_cast<const bf16x8*>(stg + off);
      if (X3) f.bl[j] = *reinterpret_cast<const bf16x8*>(stg + XW_IMG + off);
    }
  };
  // D = W x act^T: output channels are the MFMA rows, positions the columns, so lane l's 4 registers
  // of block (i, j) are 4 consecutive channels (4 (l >> 4) .. + 3 of block j) at position l & 15 of
  // block i -- one 16-byte store each in the epilogue
  auto mfmas = [&](const Frags& f) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (X3) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.bh[j], f.al[i], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.bl[j], f.ah[i], acc[i][j], 0, 0, 0);
        }
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.bh[j], f.ah[i], acc[i][j], 0, 0, 0);
      }
  };

  int w = blockIdx.x;
  if (w >= n_work) return;  // (uniform per workgroup)
  Item cur = decode(w);
  issue(cur, 0, smem);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  int g = 0;  // global step counter: stage parity
  for (;;) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int w_next = w + (int)gridDim.x;
    for (int s = 0; s < S; ++s, ++g) {
      lane = tid & 63;
      asm volatile("" : "+v"(lane));
      fr = lane & 15;
      q = lane >> 4;
      char* stg = smem + (g & 1) * STAGE;
      char* oth = smem + ((g + 1) & 1) * STAGE;
      const bool main_step = !XTRA || s < n_main;
      if (main_step && (s & 1)) {
        // the tap-8 k-step of the chunk pair (s - 1, s): lanes 0-31 read the even chunk, still in the
        // other stage, lanes 32-63 this one; then one barrier before that stage is overwritten
        Frags f;
        read_main(f, (q >> 1) ? stg : oth, 8);
        mfmas(f);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
      // next step's DMA into the other stage (its last reads are retired by the barrier above, or for
      // an even step by the previous step's wait + barrier)
      {
        const bool last = s + 1 >= S;  // (one issue site: it inlines to a lot of code)
        if (!last || w_next < n_work) issue(last ? decode(w_next) : cur, last ? 0 : s + 1, oth);
      }
      if (main_step) {
        Unroll<0, 4>::run([&](auto KS) {
          constexpr int ks = decltype(KS)::value;
          Frags f;
          read_main(f, stg, 2 * ks + (q >> 1));
          mfmas(f);
        });
      } else {
        Frags f;
        read_ext(f, stg);
        mfmas(f);
      }
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }

    if constexpr (EPI == 2) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(acc[i][j]));
    } else {
      // ---- epilogue: fp32 store (16 B per lane) + fp64 per-channel sum / sum-of-squares ----
      const int C_out = a.out.C_out;
      double ssum[4][4], ssq[4][4];  // [channel block j][channel 4 (l >> 4) + r]
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int co = cur.nb * BN + j * 16 + 4 * q;  // C_out % 16 == 0 (conv3x3_m16_selected)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          ssum[j][r] = 0.0;
          ssq[j][r] = 0.0;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int t = cur.t0 + wave * 2 + (i >> 1);
          const int f = cur.f0 + (i & 1) * 16 + fr;
          if (co >= C_out || t >= a.T_out) continue;
          *reinterpret_cast<f32x4*>(a.out.ptr + (((int64_t)cur.b * a.T_out + t) * a.F_out + f) * C_out + co) =
              acc[i][j];
          if constexpr (EPI == 1) continue;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const double v = (double)acc[i][j][r];
            ssum[j][r] += v;
            ssq[j][r] = fma(v, v, ssq[j][r]);
          }
        }
      }
      if (EPI == 0 && a.out.stats) {
        // sum over the 16 positions (lanes l & 15) of each lane group: DPP within rows of 16
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            ssum[j][r] = row16_sum(ssum[j][r]);
            ssq[j][r] = row16_sum(ssq[j][r]);
          }
        if (fr == 0) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int n = j * 16 + 4 * q + r;
              red[(wave * BN + n) * 2 + 0] = ssum[j][r];
              red[(wave * BN + n) * 2 + 1] = ssq[j][r];
            }
        }
        __syncthreads();
        if (tid < BN) {
          double s0 = 0.0, s1 = 0.0;
#pragma unroll
          for (int wv = 0; wv < 8; ++wv) {
            s0 += red[(wv * BN + tid) * 2 + 0];
            s1 += red[(wv * BN + tid) * 2 + 1];
          }
          const int co = cur.nb * BN + tid;
          if (co < C_out) {
            double* st = a.out.stats + ((int64_t)cur.b * C_out + co) * 2;
            atomicAdd(st + 0, s0);
            atomicAdd(st + 1, s1);
          }
        }
        // red is rewritten only after the next item's step barriers
      }
    }
    w = w_next;
    if (w >= n_work) break;
    cur = decode(w);
  }
}

// ---------------------------------------------------------------------------------------------
// TDF linear (mdx23c_tfc_tdf_v3.py:113-120) as one GEMM per launch over all (b, t):
//   D[m][n] = sum_k W[m][k] * act(X[k][n]),  n = (b, t, c) flattened over the whole batch.
// The weight (M x K, <= 1 MB as hi+lo) is the small operand and stays L2-resident; the workgroup
// tile is BM rows x BN = 128 columns (per-column norm affines computed once in the prologue),
// 4 waves of MI x NI 32x32 blocks, 2 workgroups per CU so one workgroup's staging overlaps the
// other's MFMAs.  Every thread stages 4 consecutive columns x 4 k rows of X per K chunk.
// U (the bottleneck activation between the two Linears) is stored k-major TILED:
//   [n / 128][ceil(M / 32)][32 m][128 n] fp32 (tdf_u_floats() gives the padded size), so the first
//   Linear stores full 128-B lines straight from the MFMA layout and each K chunk the second
//   Linear stages is one contiguous 16 KB block.
// U_IN:  X is tiled U; else NHWC [(b,t)][k][c].
// U_OUT: D is written as tiled U; else NHWC [(b,t)][m][c] (+ in-place residual, x + tdf(x), :136),
//   transposed through LDS so every thread moves 16 B of a row (residual load, add, store).
//   Epilogue: per-column sum / sum-of-squares for the next InstanceNorm (fp64 atomics per (b, c)).
template <int WM, int WN, int MI, int NI, bool X3, bool U_IN, bool U_OUT>
__global__ void __launch_bounds__(64 * WM * WN, 2) tdf_kernel(TdfArgs a) {
  constexpr int NT = 64 * WM * WN;
  constexpr int BN = WN * NI * 32;
  constexpr int BM = WM * MI * 32;
  static_assert(BN == 128, "U tiling and the epilogue assume 128-column tiles");
  constexpr int ROWB = kTdfBK * 2;            // 64 B per image row (32 bf16)
  constexpr int AW_BYTES = BM * ROWB;
  constexpr int B_BYTES = BN * ROWB;
  constexpr int EPI_ROWS = 32;                // rows per epilogue pass through LDS
  constexpr int EPI_BYTES = EPI_ROWS * BN * 4;
  constexpr int MAIN_BYTES = 2 * AW_BYTES + 2 * B_BYTES;
  constexpr int SM_BYTES = MAIN_BYTES > EPI_BYTES ? MAIN_BYTES : EPI_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[SM_BYTES + 3 * BN * 4];
  char* Whi = smem;
  char* Wlo = smem + AW_BYTES;
  char* Bhi = smem + 2 * AW_BYTES;
  char* Blo = Bhi + B_BYTES;
  float* csc = reinterpret_cast<float*>(smem + SM_BYTES);  // per-column affine
  float* csh = csc + BN;
  int* cvalid = reinterpret_cast<int*>(csh + BN);

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int l32 = lane & 31, h = lane >> 5;
  const int n_mb = (a.M + BM - 1) / BM;
  const int mb = blockIdx.x % n_mb;
  const int64_t n0 = (int64_t)(blockIdx.x / n_mb) * BN;
  const Src src = pick_src(a.in, 0);
  const int C = src.C;
  const int64_t n_total = (int64_t)a.batch * a.T * C;

  // per-column InstanceNorm affine of the consumer (norm over (T, K) per (b, c), :113/:117)
  for (int j = tid; j < BN; j += NT) {
    const int64_t n = n0 + j;
    float scale = 1.f, shift = 0.f;
    const int ok = n < n_total;
    if (ok && src.mode == SRC_NORM_GELU) {
      const int c = (int)(n % C);
      const int b = (int)(n / ((int64_t)a.T * C));
      const double* st = src.stats + ((int64_t)b * C + c) * 2;
      const double mean = st[0] * a.in.inv_count;
      double var = st[1] * a.in.inv_count - mean * mean;
      if (var < 0) var = 0;
      const float rstd = (float)(1.0 / sqrt(var + 1e-5));
      const float g = a.in.gamma ? a.in.gamma[c] : 1.f;
      const float be = a.in.beta ? a.in.beta[c] : 0.f;
      scale = g * rstd;
      shift = be - (float)mean * scale;
    }
    csc[j] = scale;
    csh[j] = shift;
    cvalid[j] = ok;
  }

  f32x16 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const uint16_t* wblk = a.w + (int64_t)mb * a.n_chunks * (2 * AW_BYTES / 2);

  constexpr int N16 = (X3 ? 2 : 1) * AW_BYTES / 16;
  constexpr int W_ITEMS = (N16 + NT - 1) / NT;
  constexpr int B_ITEMS_ALL = BN * 2;  // (4 columns, 4 k) items per 32-k chunk
  constexpr int B_ITEMS = (B_ITEMS_ALL + NT - 1) / NT;
  u32x4 wreg[W_ITEMS];
  f32x4 breg[B_ITEMS][4];

  auto load_chunk = [&](int kc) {
    const u32x4* s4 = reinterpret_cast<const u32x4*>(wblk + (int64_t)kc * (2 * AW_BYTES / 2));
    Unroll<0, W_ITEMS>::run([&](auto I) {
      const int e = tid + I * NT;
      wreg[I] = s4[e < N16 ? e : N16 - 1];
    });
    const int k0 = kc * kTdfBK;
    Unroll<0, B_ITEMS>::run([&](auto I) {
      const int e = tid + I * NT;
      const int j = (e % (BN / 4)) * 4, g = e / (BN / 4);  // 4 columns, k = k0 + 4g .. +3
      const int64_t n = n0 + j;
      const bool okn = (e < B_ITEMS_ALL) && n < n_total;  // n_total % 4 == 0 (C % 4 == 0)
      if (U_IN) {
        const float* blk = src.ptr + (((n0 >> 7) * a.n_chunks + kc) << 12) + j;  // contiguous [32 k][128 n]
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const bool ok = okn && k0 + 4 * g + q < a.K;
          breg[I][q] = ok ? *reinterpret_cast<const f32x4*>(blk + (4 * g + q) * 128) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
      } else {
        const int64_t bt = n / C;
        const int c = (int)(n - bt * C);  // C % 4 == 0: the 4 columns share (b, t)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int k = k0 + 4 * g + q;
          const bool ok = okn && k < a.K;
          breg[I][q] = ok ? *reinterpret_cast<const f32x4*>(src.ptr + (bt * a.K + k) * C + c)
                          : f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
    });
  };

  auto store_chunk = [&](int kc) {
    u32x4* d4 = reinterpret_cast<u32x4*>(Whi);
    Unroll<0, W_ITEMS>::run([&](auto I) {
      const int e = tid + I * NT;
      if (N16 % NT == 0 || e < N16) d4[e] = wreg[I];
    });
    const int k0 = kc * kTdfBK;
    Unroll<0, B_ITEMS>::run([&](auto I) {
      const int e = tid + I * NT;
      if (B_ITEMS_ALL % NT != 0 && e >= B_ITEMS_ALL) return;
      const int j0 = (e % (BN / 4)) * 4, g = e / (BN / 4);
#pragma unroll
      for (int cc = 0; cc < 4; ++cc) {
        const int j = j0 + cc;
        const float scale = csc[j], shift = csh[j];
        const bool okc = cvalid[j];
        __bf16 hi[4], lo[4];
        float xv[4] = {breg[I][0][cc], breg[I][1][cc], breg[I][2][cc], breg[I][3][cc]};
        if (src.mode == SRC_NORM_GELU) {
          // packed pairs (v_pk_fma_f32): this staging is VALU-issue-bound and not overlapped with the
          // workgroup's own MFMAs
#pragma unroll
          for (int q = 0; q < 4; q += 2) {
            const f32x2 y = gelu_erf2(__builtin_elementwise_fma(f32x2{xv[q], xv[q + 1]}, f32x2{scale, scale},
                                                                f32x2{shift, shift}));
            xv[q] = (okc && k0 + 4 * g + q < a.K) ? y[0] : 0.f;
            xv[q + 1] = (okc && k0 + 4 * g + q + 1 < a.K) ? y[1] : 0.f;
          }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) split_bf16(xv[q], hi[q], lo[q]);
        const int off = j * ROWB + ((((g >> 1) ^ ((j >> 2) & 3))) << 4) + ((g & 1) << 3);
        *reinterpret_cast<uint2*>(Bhi + off) = make_uint2(pack2(hi[0], hi[1]), pack2(hi[2], hi[3]));
        if (X3) *reinterpret_cast<uint2*>(Blo + off) = make_uint2(pack2(lo[0], lo[1]), pack2(lo[2], lo[3]));
      }
    });
  };

  load_chunk(0);
  for (int kc = 0; kc < a.n_chunks; ++kc) {
    __syncthreads();  // previous chunk's fragment reads done (and the column affines are built)
    store_chunk(kc);
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
        const int n = (wn * NI + j) * 32 + l32;
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

  // ---- epilogue ----
  // Each thread ends up owning column partial sums for 4 consecutive columns (cs4 = tid % 32).
  double ssum[4] = {0.0, 0.0, 0.0, 0.0}, ssq[4] = {0.0, 0.0, 0.0, 0.0};   // fp64 norm statistics
  const int cs4 = (tid % (BN / 4)) * 4;
  if (U_OUT) {
    // tiled U: for each register, lanes 0-31 / 32-63 store two full 128-B rows (32 consecutive n)
    const int mchunks = (a.M + 31) >> 5;
    float* ublk = a.out.ptr + (((n0 >> 7) * mchunks) << 12);
    double* red2 = reinterpret_cast<double*>(smem);  // [WM][BN][2] (main-loop LDS is dead)
    static_assert(WM * BN * 2 * 8 <= SM_BYTES, "fp64 reduction fits the dead main-loop LDS");
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int jl = (wn * NI + j) * 32 + l32;
      const bool nok = n0 + jl < n_total;
      double s0 = 0.0, s1 = 0.0;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = mb * BM + (wm * MI + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          if (!nok || m >= a.M) continue;
          const float v = acc[i][j][r];
          ublk[((m >> 5) << 12) + (m & 31) * 128 + jl] = v;
          s0 += (double)v;
          s1 = fma((double)v, (double)v, s1);
        }
      s0 += __shfl_xor(s0, 32);
      s1 += __shfl_xor(s1, 32);
      if (h == 0) {
        red2[(wm * BN + jl) * 2 + 0] = s0;
        red2[(wm * BN + jl) * 2 + 1] = s1;
      }
    }
    __syncthreads();
    if (a.out.stats) {
      for (int jl = tid; jl < BN; jl += NT) {
        const int64_t n = n0 + jl;
        if (n >= n_total) continue;
        double s0 = 0.0, s1 = 0.0;
#pragma unroll
        for (int w = 0; w < WM; ++w) {
          s0 += red2[(w * BN + jl) * 2 + 0];
          s1 += red2[(w * BN + jl) * 2 + 1];
        }
        const int c = (int)(n % C);
        const int b = (int)(n / ((int64_t)a.T * C));
        double* st = a.out.stats + ((int64_t)b * C + c) * 2;
        atomicAdd(st + 0, s0);
        atomicAdd(st + 1, s1);
      }
    }
    return;
  }

  // NHWC output through LDS, EPI_ROWS rows per pass.  A 128-column tile lies in one (b, t) when
  // C % 128 == 0 (every real config); otherwise each 4-column group computes its own (b, t).
  float* stage = reinterpret_cast<float*>(smem);  // [EPI_ROWS][BN] fp32, row-swizzled by 16-B groups
  constexpr int ITEMS = EPI_ROWS * BN / 4 / NT;   // f32x4 items per thread per pass
  static_assert(EPI_ROWS * BN / 4 % NT == 0, "epilogue items");
  const int64_t ncol = n0 + cs4;
  const bool col_ok = ncol < n_total;
  const int64_t bt = ncol / C;
  const int c = (int)(ncol - bt * C);
  // residual rows of pass p (they alias the output: each pass's rows are loaded before that pass's
  // stores; pass p + 1's are issued right after pass p's stores, in flight over its LDS staging)
  auto load_res = [&](f32x4 (&res)[ITEMS], int p) {
    const int row0 = mb * BM + p * EPI_ROWS;
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {
      const int rl = (tid + it * NT) / (BN / 4);
      const int m = row0 + rl;
      res[it] = (a.out.residual && col_ok && m < a.M)
                    ? *reinterpret_cast<const f32x4*>(a.out.residual + (bt * a.M + m) * C + c)
                    : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  f32x4 res[ITEMS];
  load_res(res, 0);
  Unroll<0, BM / EPI_ROWS>::run([&](auto P) {
    constexpr int p = decltype(P)::value;
    const int row0 = mb * BM + p * EPI_ROWS;
    __syncthreads();  // previous pass's stage reads (and the main loop's LDS reads) are done
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int rb = (wm * MI + i) * 32;  // tile-local row block of this MFMA block
      if (rb < p * EPI_ROWS || rb >= (p + 1) * EPI_ROWS) continue;
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int jl = (wn * NI + j) * 32 + l32;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rl = rb - p * EPI_ROWS + (r & 3) + 8 * (r >> 2) + 4 * h;
          stage[rl * BN + (((jl >> 2) ^ (rl & 31)) << 2) + (jl & 3)] = acc[i][j][r];
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {
      const int rl = (tid + it * NT) / (BN / 4);
      const int m = row0 + rl;
      if (!col_ok || m >= a.M) continue;
      f32x4 v = *reinterpret_cast<const f32x4*>(stage + rl * BN + (((cs4 >> 2) ^ (rl & 31)) << 2));
      v += res[it];
      *reinterpret_cast<f32x4*>(a.out.ptr + (bt * a.M + m) * C + c) = v;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        ssum[q] += (double)v[q];
        ssq[q] = fma((double)v[q], (double)v[q], ssq[q]);
      }
    }
    if constexpr (p + 1 < BM / EPI_ROWS) load_res(res, p + 1);  // in flight over the next pass's staging
  });
  if (a.out.stats) {
    // threads tid, tid + 32, ... own the same 4 columns: reduce through LDS in fp64 (the stage
    // region, dead once every thread has passed the barrier below)
    static_assert(2 * NT * 4 * 8 <= SM_BYTES, "fp64 reduction fits the stage region");
    double* r8 = reinterpret_cast<double*>(smem);
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      r8[q * NT + tid] = ssum[q];
      r8[(4 + q) * NT + tid] = ssq[q];
    }
    __syncthreads();
    if (tid < BN / 4 && col_ok) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        double s0 = 0.0, s1 = 0.0;
        for (int t = tid; t < NT; t += BN / 4) {
          s0 += r8[q * NT + t];
          s1 += r8[(4 + q) * NT + t];
        }
        const int64_t n = ncol + q;
        const int cq = (int)(n % C);
        const int b = (int)(n / ((int64_t)a.T * C));
        double* st = a.out.stats + ((int64_t)b * C + cq) * 2;
        atomicAdd(st + 0, s0);
        atomicAdd(st + 1, s1);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// tdf_u_split_kernel: act(U) of the second TDF Linear (InstanceNorm affine of tdf[3], exact GELU, bf16
// hi / lo) once per element, written as the B images tdf_dma_kernel<.., PRE> copies by LDS-DMA
// ([column tile][chunk][hi: 128 n x 32 k][lo], the image swizzle included).  Without it the second
// Linear converts every U element once per 256-row block of its output (4x at level 0), and its
// staging is VALU-issue-bound.  One workgroup per (column tile, chunk); thread = column x 8 k.
template <bool F16 = false>
__global__ void __launch_bounds__(512) tdf_u_split_kernel(TdfArgs a) {
  constexpr int BN = 128, ROWB = kTdfBK * 2;
  const int64_t ntile = blockIdx.x;
  const int kc = blockIdx.y;
  const Src src = pick_src(a.in, 0);
  const int C = src.C;
  const int n = threadIdx.x & (BN - 1), kq = threadIdx.x >> 7;
  const int64_t col = ntile * BN + n;
  const int64_t bt = col / C;
  const int c = (int)(col - bt * C), b = (int)(bt / a.T);
  float csc = 1.f, csh = 0.f;
  const bool act = src.mode == SRC_NORM_GELU;
  if (act) {
    const double* st = src.stats + ((int64_t)b * C + c) * 2;
    const double mean = st[0] * a.in.inv_count;
    double var = st[1] * a.in.inv_count - mean * mean;
    if (var < 0) var = 0;
    const float rstd = (float)(1.0 / sqrt(var + 1e-5));
    const float gm = a.in.gamma ? a.in.gamma[c] : 1.f;
    const float be = a.in.beta ? a.in.beta[c] : 0.f;
    csc = gm * rstd;
    csh = be - (float)mean * csc;
  }
  const int64_t blk = ntile * a.n_chunks + kc;
  const float* u = src.ptr + blk * (kTdfBK * BN);
  float v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = __builtin_nontemporal_load(u + (8 * kq + e) * BN + n);
  if (act) {
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      const f32x2 y = gelu_erf2(__builtin_elementwise_fma(f32x2{v[e], v[e + 1]}, f32x2{csc, csc}, f32x2{csh, csh}));
      v[e] = y[0];
      v[e + 1] = y[1];
    }
  }
  uint32_t hw[4], lw[4];
#pragma unroll
  for (int e = 0; e < 8; e += 2) {
    if constexpr (F16) {   // one fp16 image (the lo image is not read by the fp16 GEMM)
      hw[e / 2] = pack2h(v[e], v[e + 1]);
      continue;
    }
    __bf16 h0, l0, h1, l1;
    split_bf16(v[e], h0, l0);
    split_bf16(v[e + 1], h1, l1);
    hw[e / 2] = pack2(h0, h1);
    lw[e / 2] = pack2(l0, l1);
  }
  char* dst = reinterpret_cast<char*>(a.u_planes) + blk * (kTdfBK * BN * 4);
  const int off = n * ROWB + ((kq ^ ((n >> 2) & 3)) << 4);
  *reinterpret_cast<uint4*>(dst + off) = make_uint4(hw[0], hw[1], hw[2], hw[3]);
  if constexpr (!F16) *reinterpret_cast<uint4*>(dst + BN * ROWB + off) = make_uint4(lw[0], lw[1], lw[2], lw[3]);
}

// An LDS store hipcc's waitcnt pass does not see: it treats every plain store into a __shared__ array that an LDS-DMA
// (buffer_load ... lds) also writes as possibly aliasing the DMA and waits vmcnt(0) before it (profiles/r06_isa_audit.txt).
// The caller orders it: the store's data registers are ordinary compiler-tracked values, and its readers sit behind an
// explicit lgkmcnt(0) + barrier.
__device__ __forceinline__ void ds_write_b128_untracked(char* p, u32x4 v) {
  const uint32_t a = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)p;
  asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(v) : "memory");
}

// ---------------------------------------------------------------------------------------------
// tdf_dma_kernel: the TDF Linears (mdx23c_tfc_tdf_v3.py:113-120) with every operand staged by LDS-DMA
// so each chunk's HBM latency is covered by several chunks of MFMAs (tdf_kernel covers it with one).
//   * 512 threads (8 waves, WM x WN), tile BM rows x 128 columns (one (b, t) x 128 channels; C % 128 == 0),
//     wave tile 64 rows x (128 / WN) columns of 32x32x16 blocks.
//   * per 32-deep K chunk: W (BM x 32, hi + lo, the packed image verbatim) into a 2-stage ring, one
//     chunk ahead, and X as raw fp32 [32 k][128 n] (one contiguous 512-B row per k for NHWC input, one
//     16 KiB block for tiled U) into a 4-stage ring, three chunks ahead (one counted s_waitcnt per chunk).
//     Chunk kc + 1 is converted -- each thread one column x 8 k: 8 conflict-free ds_read_b32, InstanceNorm
//     affine of its column from registers, packed GELU, hi / lo, one ds_write_b128 per plane (a
//     4-column x 2-k item put every ds_write_b32 of a wave on 4 banks) -- into the second B image while
//     chunk kc's MFMAs run: one barrier per chunk.
//   * epilogue without LDS transposes: the 32x32 D layout has consecutive lanes on consecutive columns
//     (channels), so U rows (U_OUT) and NHWC rows (+ the residual, prefetched into registers under the
//     last chunk) are written as full 128-B lines; per-column statistics (fp32 over 16-value runs, fp64
//     beyond) reduced through LDS.
// F16 (X3 = false): W and B images in fp16, one v_mfma_f32_32x32x16_f16 pass (SESA_PREC_F16MIX TDF plan).
// DEEP (F16 only; round 5): the fp16 images free LDS for deeper rings -- W two chunks ahead (3 stages), X five ahead
// (6 stages, 96 KiB of the input in flight per CU instead of 48) -- and the PRE input DMAs only the fp16 image of each
// 16-KiB block (tdf_u_split_kernel<F16> writes no lo image: the plain ring fetched 8 KiB of unwritten bytes per chunk).
template <bool X3, bool U_IN, bool U_OUT, int BM, bool PRE = false, bool F16 = false, bool DEEP = false>
__global__ void __launch_bounds__(512, 1) tdf_dma_kernel(TdfArgs a) {
  static_assert(!PRE || U_IN, "pre-split B images exist for the tiled U input only");
  static_assert(!F16 || !X3, "fp16: one pass");
  static_assert(!DEEP || F16, "deep rings: the fp16 images");
  constexpr int BN = 128;
  constexpr int WM = BM / 64, WN = 8 / WM;
  constexpr int MI = 2, NI = BN / WN / 32;
  static_assert(WM * WN == 8 && NI >= 1, "wave grid");
  constexpr int ROWB = kTdfBK * 2;                 // 64 B per image row (32 bf16)
  constexpr int W_PLANE = BM * ROWB;
  constexpr int W_STAGE = (X3 ? 2 : 1) * W_PLANE;
  constexpr int X_STAGE = kTdfBK * BN * 4;         // 16 KiB fp32
  constexpr int B_PLANE = BN * ROWB;                // 8 KiB
  constexpr int NWS = DEEP ? 3 : 2, NXS = DEEP ? 6 : 4;   // W ring (one / two chunks ahead), X ring (three / five)
  constexpr int W_OFF = 0, X_OFF = NWS * W_STAGE, B_OFF = X_OFF + NXS * X_STAGE;
  constexpr int B_IMG = (X3 ? 2 : 1) * B_PLANE;      // two B images: chunk kc's MFMAs / chunk kc+1's conversion
  constexpr int SMEM = B_OFF + 2 * B_IMG;
  static_assert(SMEM <= 163840 && WM * BN * 2 * 8 <= SMEM, "LDS budget");
  constexpr int X_DMA = DEEP && PRE ? X_STAGE / 2 : X_STAGE;   // bytes DMA'd per X chunk
  constexpr int W_PC = W_STAGE / 1024, X_PC = X_DMA / 1024;
  static_assert(W_PC % 8 == 0 && X_PC % 8 == 0, "uniform DMA pieces per wave");
  // s_waitcnt: all but the X_PC / 8 youngest vector-memory ops (the X DMA issued last), lgkmcnt(0)
  constexpr int VMN = X_PC / 8, WPW = W_PC / 8;
  constexpr int WAIT_ONE = (VMN & 15) | ((VMN >> 4) << 14) | (7 << 4);
  // DEEP: vmcnt(n) (expcnt not waited, lgkmcnt(0))
  constexpr int WAIT_D2 = ((2 * VMN + WPW) & 15) | (((2 * VMN + WPW) >> 4) << 14) | (7 << 4);
  constexpr int WAIT_D1 = ((VMN + WPW) & 15) | (((VMN + WPW) >> 4) << 14) | (7 << 4);
  constexpr int WAIT_D0 = (WPW & 15) | ((WPW >> 4) << 14) | (7 << 4);
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int l32 = lane & 31, h = lane >> 5;
  const Src src = pick_src(a.in, 0);
  const int C = src.C;
  const int n_mb = (a.M + BM - 1) / BM;
  // XCD-aware order: ids 8 apart share an XCD; the n_mb row blocks of a column tile are 8 ids apart
  int ntile, mb;
  {
    const int id = blockIdx.x;
    const int x = id & 7, rest = id >> 3;
    mb = rest % n_mb;
    ntile = (rest / n_mb) * 8 + x;
  }
  const int64_t n0 = (int64_t)ntile * BN;
  const int64_t n_total = (int64_t)a.batch * a.T * C;
  if (n0 >= n_total) return;  // (uniform; the grid is rounded up to 8 column tiles)
  const int64_t bt = n0 / C;
  const int c0 = (int)(n0 - bt * C);
  const int b = (int)(bt / a.T);
  const int nk = a.n_chunks;

  // ---- LDS-DMA issue (buffer resources: 32-bit offsets) ----
  auto rsrc = [](const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
  };
  auto dma = [](__amdgpu_buffer_rsrc_t r, char* lds, uint32_t voff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, 0, 0, 0);
  };
  const uint16_t* wblk = a.w + (int64_t)mb * nk * (2 * W_PLANE / 2);
  const __amdgpu_buffer_rsrc_t rw = rsrc(wblk, (uint32_t)((int64_t)nk * 2 * W_PLANE));
  // PRE: the X ring carries the B images tdf_u_split_kernel wrote (same 16 KiB per chunk as fp32 U)
  const float* xbase = PRE    ? reinterpret_cast<const float*>(a.u_planes) + (n0 >> 7) * (int64_t)nk * (kTdfBK * BN)
                       : U_IN ? src.ptr + (n0 >> 7) * (int64_t)nk * (kTdfBK * BN)
                              : src.ptr + bt * (int64_t)a.K * C + c0;
  const __amdgpu_buffer_rsrc_t rx =
      rsrc(xbase, U_IN ? (uint32_t)(nk * X_STAGE) : (uint32_t)(((int64_t)(a.K - 1) * C + BN) * 4));
  auto issue_w = [&](int kc) {
    char* stg = smem + W_OFF + (kc % NWS) * W_STAGE;
#pragma unroll
    for (int i = 0; i < (W_PC + 7) / 8; ++i) {
      const int pc = wave + 8 * i;
      if (pc < W_PC) dma(rw, stg + pc * 1024, (uint32_t)(kc * 2 * W_PLANE + pc * 1024 + lane * 16));
    }
  };
  auto issue_x = [&](int kc) {
    char* stg = smem + X_OFF + (kc % NXS) * X_STAGE;
#pragma unroll
    for (int i = 0; i < X_PC / 8; ++i) {
      const int pc = wave + 8 * i;                 // piece = k rows 2 pc, 2 pc + 1 (512 B each)
      uint32_t voff;
      if (U_IN) voff = (uint32_t)(kc * X_STAGE + pc * 1024 + lane * 16);
      else {
        const int k = kc * kTdfBK + 2 * pc + (lane >> 5);
        voff = (uint32_t)(((int64_t)k * C + (lane & 31) * 4) * 4);
      }
      dma(rx, stg + pc * 1024, voff);
    }
  };

  // ---- this thread's staging item: column ncol of the tile, k = 8 kq .. 8 kq + 7 of the chunk ----
  // (X reads: consecutive lanes on consecutive columns of a 512-B fp32 row; B writes: one 16-B unit of
  // hi and of lo per thread, conflict-free under the image swizzle)
  const int ncol = tid & (BN - 1), kq = tid >> 7;  // kq 0..3
  const bool act = src.mode == SRC_NORM_GELU;
  float csc = 1.f, csh = 0.f;
  if (act) {
    const int c = c0 + ncol;
    const double* st = src.stats + ((int64_t)b * C + c) * 2;
    const double mean = st[0] * a.in.inv_count;
    double var = st[1] * a.in.inv_count - mean * mean;
    if (var < 0) var = 0;
    const float rstd = (float)(1.0 / sqrt(var + 1e-5));
    const float gm = a.in.gamma ? a.in.gamma[c] : 1.f;
    const float be = a.in.beta ? a.in.beta[c] : 0.f;
    csc = gm * rstd;
    csh = be - (float)mean * csc;
  }
  const int b_off = ncol * ROWB + ((kq ^ ((ncol >> 2) & 3)) << 4);
  auto convert = [&](int kc) {
    if constexpr (PRE) return;
    const float* xs = reinterpret_cast<const float*>(smem + X_OFF + (kc % NXS) * X_STAGE);
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = xs[(8 * kq + e) * BN + ncol];
    if (act) {
      // scalar f32 (not v_pk_*): this conversion runs beside the MFMAs, where packed f32 VALU costs
      // extra issue cycles (MI355X_MICROARCH.md constants table)
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = gelu_erf(fmaf(v[e], csc, csh));
    }
    uint32_t hw[4], lw[4];
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      if constexpr (F16) {
        hw[e / 2] = pack2h(v[e], v[e + 1]);
        continue;
      }
      __bf16 h0, l0, h1, l1;
      split_bf16(v[e], h0, l0);
      split_bf16(v[e + 1], h1, l1);
      hw[e / 2] = pack2(h0, h1);
      lw[e / 2] = pack2(l0, l1);
    }
    char* Bhi = smem + B_OFF + (kc & 1) * B_IMG;
    // (inline-asm stores: hipcc treats a plain LDS store into this array as possibly aliasing the in-flight LDS-DMA
    // and drains vmcnt(0) before it -- every chunk in flight, i.e. the whole ring -- each iteration; the B images are
    // disjoint from the DMA rings, and the loop's lgkmcnt(0) + barrier orders these stores before their readers)
    ds_write_b128_untracked(Bhi + b_off, u32x4{hw[0], hw[1], hw[2], hw[3]});
    if (X3) ds_write_b128_untracked(Bhi + B_PLANE + b_off, u32x4{lw[0], lw[1], lw[2], lw[3]});
  };

  f32x16 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // residual rows (NHWC, may alias the output): prefetched under the last chunk
  float res[U_OUT ? 1 : MI][U_OUT ? 1 : NI][U_OUT ? 1 : 16];
  auto load_res = [&]() {
    if constexpr (!U_OUT) {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          const int jl = (wn * NI + j) * 32 + l32;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int m = mb * BM + (wm * MI + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            res[i][j][r] = (a.out.residual && m < a.M) ? a.out.residual[(bt * a.M + m) * C + c0 + jl] : 0.f;
          }
        }
    }
  };

  // prologue: W(0) (DEEP: and W(1)), X(0 .. NXS - 2) landed; chunk 0 converted
  issue_w(0);
  if (DEEP && nk > 1) issue_w(1);
#pragma unroll
  for (int d = 0; d < NXS - 1; ++d)
    if (d < nk) issue_x(d);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  convert(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  // iteration kc: MFMAs of chunk kc (B image kc & 1, W stage kc % 2) with chunk kc + 1 converted into the
  // other B image in between; W(kc + 1) and X(kc + 3) issued at the top into stages whose last readers
  // (iteration kc - 1's MFMAs, iteration kc - 2's conversion) are behind a barrier; one barrier per chunk
  for (int kc = 0; kc < nk; ++kc) {
    const bool more_w = kc + 1 < nk, more_x = kc + NXS - 1 < nk;
    if (DEEP) {
      if (kc + 2 < nk) issue_w(kc + 2);
    } else if (more_w) {
      issue_w(kc + 1);
    }
    if (more_x) issue_x(kc + NXS - 1);
    if (!U_OUT && kc + 1 == nk) load_res();
    const char* W = smem + W_OFF + (kc % NWS) * W_STAGE;
    const char* Bh = PRE ? smem + X_OFF + (kc % NXS) * X_STAGE : smem + B_OFF + (kc & 1) * B_IMG;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 ah[MI], al[MI], bh[NI], bl[NI];
      const int q = ks * 2 + h;
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int row = (wm * MI + i) * 32 + l32;
        const int off = row * ROWB + ((q ^ ((row >> 2) & 3)) << 4);
        ah[i] = *reinterpret_cast<const bf16x8*>(W + off);
        if (X3) al[i] = *reinterpret_cast<const bf16x8*>(W + W_PLANE + off);
      }
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int n = (wn * NI + j) * 32 + l32;
        const int off = n * ROWB + ((q ^ ((n >> 2) & 3)) << 4);
        bh[j] = *reinterpret_cast<const bf16x8*>(Bh + off);
        if (X3) bl[j] = *reinterpret_cast<const bf16x8*>(Bh + B_PLANE + off);
      }
      if (!PRE && ks == 0 && more_w) convert(kc + 1);  // VALU / LDS work between this chunk's MFMAs
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          if (X3) {
            acc[i][j] = mfma32(al[i], bh[j], acc[i][j]);
            acc[i][j] = mfma32(ah[i], bl[j], acc[i][j]);
          }
          if constexpr (F16) acc[i][j] = mfma32h(ah[i], bh[j], acc[i][j]);
          else acc[i][j] = mfma32(ah[i], bh[j], acc[i][j]);
        }
    }
    // W(kc + 1) and X(kc + 2) landed (only X(kc + 3), issued last, may stay in flight; the residual
    // prefetch of the last iteration is waited for at its use).  DEEP: the ops younger than W(kc + 1) -- X(kc + 4),
    // W(kc + 2), X(kc + 5), as far as they were issued -- may stay in flight
    if (DEEP) {
      if (kc + 5 < nk) __builtin_amdgcn_s_waitcnt(WAIT_D2);
      else if (kc + 4 < nk) __builtin_amdgcn_s_waitcnt(WAIT_D1);
      else if (kc + 2 < nk) __builtin_amdgcn_s_waitcnt(WAIT_D0);
      else if (more_w) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    } else if (more_x) __builtin_amdgcn_s_waitcnt(WAIT_ONE);
    else if (more_w) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }

  // ---- epilogue: output rows (full 128-B lines) + per-column statistics ----
  double* red = reinterpret_cast<double*>(smem);  // [WM][BN][2] (every LDS read retired by the last barrier)
  const int64_t u_base = U_OUT ? (int64_t)ntile * ((a.M + 31) >> 5) * 4096 : 0;
  // full row blocks (M % BM == 0 for every real shape): no per-element guards, 32-bit offsets from a
  // uniform tile base (the guarded form compiled to ~100 exec-mask branches and 64-bit math per store)
  auto epilogue = [&](auto FULLT) {
    constexpr bool FULL = decltype(FULLT)::value;
    float* obase = U_OUT ? a.out.ptr + u_base + (int64_t)((mb * BM) >> 5) * 4096
                         : a.out.ptr + (bt * a.M + mb * BM) * C + c0;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int jl = (wn * NI + j) * 32 + l32;
      double s0 = 0.0, s1 = 0.0;  // fp32 partial sums over each 16-value run, fp64 from there
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        float ps = 0.f, pq = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int ml = (wm * MI + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;  // row within the block
          if (!FULL && mb * BM + ml >= a.M) continue;
          float v = acc[i][j][r];
          if constexpr (U_OUT) {
            obase[((ml >> 5) << 12) + (ml & 31) * 128 + jl] = v;
          } else {
            v += res[i][j][r];
            obase[ml * C + jl] = v;
          }
          ps += v;
          pq = fmaf(v, v, pq);
        }
        s0 += (double)ps;
        s1 += (double)pq;
      }
      s0 += __shfl_xor(s0, 32);
      s1 += __shfl_xor(s1, 32);
      if (h == 0) {
        red[(wm * BN + jl) * 2 + 0] = s0;
        red[(wm * BN + jl) * 2 + 1] = s1;
      }
    }
  };
  if ((mb + 1) * BM <= a.M) epilogue(std::true_type{});
  else epilogue(std::false_type{});
  if (a.out.stats) {
    __syncthreads();
    if (tid < BN) {
      double s0 = 0.0, s1 = 0.0;
#pragma unroll
      for (int w = 0; w < WM; ++w) {
        s0 += red[(w * BN + tid) * 2 + 0];
        s1 += red[(w * BN + tid) * 2 + 1];
      }
      double* st = a.out.stats + ((int64_t)b * C + c0 + tid) * 2;
      atomicAdd(st + 0, s0);
      atomicAdd(st + 1, s1);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// act_split: one pass over a normalised tensor, writing the bf16 hi/lo operand planes of its
// consumer (InstanceNorm affine + exact GELU applied once per element instead of once per
// consuming tile).  HBM-bound: reads 4 B, writes 2 + 2 B per element.
// Thread layout: blockDim = groups * lanes_pos (groups = C / 8); thread (pl, g) owns the fixed
// 8-channel group g, so its 8 (scale, shift) pairs live in registers, and walks positions
// pl, pl + lanes_pos, ... of the block's range -- consecutive threads still cover consecutive
// 32-B pieces of a row (coalesced), with no per-item index division or LDS affine reads.  Four
// positions' loads are issued before any is transformed; the GELU runs on packed float2 pairs.
constexpr int kActUnroll = 4;
// rhi / rlo (nullable): the raw (untransformed) input split to bf16 planes as well -- the fused 1x1
// shortcut operand of conv3x3_m16_kernel, written while the input is in registers anyway.
// F32OUT: the activation itself as fp32 (hi = the fp32 output, lo / rhi / rlo unused) -- the SRC_ACT32 input of
// conv3x3_wino_kernel, whose Winograd input transform needs the unsplit value.
// F16OUT (lo == nullptr): the activation rounded once to fp16 into `hi` -- the A plane of the fp16 TFC convs.
template <bool F32OUT, bool F16OUT = false>
__global__ void __launch_bounds__(kThreads) act_split_kernel(GemmIn in, int64_t n_pos, int pos_per_block,
                                                             uint16_t* __restrict__ hi, uint16_t* __restrict__ lo,
                                                             uint16_t* __restrict__ rhi, uint16_t* __restrict__ rlo) {
  __shared__ float sc_s[kMaxCin], sh_s[kMaxCin];
  const int b = blockIdx.y;
  build_affine(in, b, sc_s, sh_s);
  __syncthreads();
  const int C = in.C_in;
  const int groups = C >> 3;  // 8 channels per thread (C % 16 == 0)
  const int lanes_pos = (int)blockDim.x / groups;
  const int g = (int)threadIdx.x % groups;
  const int pl = (int)threadIdx.x / groups;
  if (pl >= lanes_pos) return;
  const int c = g * 8;
  const int s = c < in.C_split ? 0 : 1;
  const Src src = pick_src(in, s);
  const int cl = c - (s ? in.C_split : 0);
  const bool act = src.mode == SRC_NORM_GELU;
  f32x2 sc[4], sh[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    sc[q] = f32x2{sc_s[c + 2 * q], sc_s[c + 2 * q + 1]};
    sh[q] = f32x2{sh_s[c + 2 * q], sh_s[c + 2 * q + 1]};
  }
  const int64_t p_begin = (int64_t)blockIdx.x * pos_per_block + pl;
  const int64_t p_end = (int64_t)(blockIdx.x + 1) * pos_per_block < n_pos ? (int64_t)(blockIdx.x + 1) * pos_per_block
                                                                           : n_pos;
  const float* xbase = src.ptr + (int64_t)b * n_pos * src.C + cl;
  const int64_t obase = (int64_t)b * n_pos * C + c;
  for (int64_t p0 = p_begin; p0 < p_end; p0 += (int64_t)kActUnroll * lanes_pos) {
    f32x4 x[kActUnroll][2];
#pragma unroll
    for (int u = 0; u < kActUnroll; ++u) {
      const int64_t p = p0 + (int64_t)u * lanes_pos;
      if (p < p_end) {
        const f32x4* xp = reinterpret_cast<const f32x4*>(xbase + p * src.C);
        x[u][0] = __builtin_nontemporal_load(xp);
        x[u][1] = __builtin_nontemporal_load(xp + 1);
      }
    }
#pragma unroll
    for (int u = 0; u < kActUnroll; ++u) {
      const int64_t p = p0 + (int64_t)u * lanes_pos;
      if (p >= p_end) continue;
      f32x2 v[4] = {f32x2{x[u][0][0], x[u][0][1]}, f32x2{x[u][0][2], x[u][0][3]}, f32x2{x[u][1][0], x[u][1][1]},
                    f32x2{x[u][1][2], x[u][1][3]}};
      uint32_t hw[4], lw[4];
      const int64_t o = obase + p * C;
      if constexpr (F32OUT) {
        f32x2 y[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) y[q] = act ? gelu_erf2(__builtin_elementwise_fma(v[q], sc[q], sh[q])) : v[q];
        f32x4* op = reinterpret_cast<f32x4*>(reinterpret_cast<float*>(hi) + o);
        __builtin_nontemporal_store(f32x4{y[0][0], y[0][1], y[1][0], y[1][1]}, op);
        __builtin_nontemporal_store(f32x4{y[2][0], y[2][1], y[3][0], y[3][1]}, op + 1);
        continue;
      }
      if constexpr (F16OUT) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x2 y = act ? gelu_erf2(__builtin_elementwise_fma(v[q], sc[q], sh[q])) : v[q];
          hw[q] = pack2h(y[0], y[1]);
        }
        *reinterpret_cast<uint4*>(hi + o) = make_uint4(hw[0], hw[1], hw[2], hw[3]);
        continue;
      }
      if (rhi) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          __bf16 h0, l0, h1, l1;
          split_bf16(v[q][0], h0, l0);
          split_bf16(v[q][1], h1, l1);
          hw[q] = pack2(h0, h1);
          lw[q] = pack2(l0, l1);
        }
        *reinterpret_cast<uint4*>(rhi + o) = make_uint4(hw[0], hw[1], hw[2], hw[3]);
        *reinterpret_cast<uint4*>(rlo + o) = make_uint4(lw[0], lw[1], lw[2], lw[3]);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x2 y = act ? gelu_erf2(__builtin_elementwise_fma(v[q], sc[q], sh[q])) : v[q];
        __bf16 h0, l0, h1, l1;
        split_bf16(y[0], h0, l0);
        split_bf16(y[1], h1, l1);
        hw[q] = pack2(h0, h1);
        lw[q] = pack2(l0, l1);
      }
      *reinterpret_cast<uint4*>(hi + o) = make_uint4(hw[0], hw[1], hw[2], hw[3]);
      *reinterpret_cast<uint4*>(lo + o) = make_uint4(lw[0], lw[1], lw[2], lw[3]);
    }
  }
}

template <int KH, int KW, int S, int PAD, int TM, int BN, int WM, bool UPS, bool XTRA, bool PRE>
int launch_conv_t(int x3, const ConvArgs& a, int batch, hipStream_t st) {
  // PRE kernels read only the bf16 planes of the main input (x3 == 3: the one fp16 plane of act_f16)
  SESA_REQUIRE(!PRE || (a.in.src[0].mode == SRC_PRE && a.in.src[0].hi && (x3 == 3 || a.in.src[0].lo) &&
                        a.in.C_split == a.in.C_in),
               SESA_ERR_INVALID, "conv: this kernel needs a single pre-activated (act_split) input");
  SESA_REQUIRE(x3 != 3 || (PRE && !XTRA), SESA_ERR_INVALID, "conv: fp16 tap kernel takes a pre-activated plane only");
  SESA_REQUIRE(PRE || (a.in.src[0].mode != SRC_PRE && a.in.src[1].mode != SRC_PRE), SESA_ERR_INVALID,
               "conv: pre-activated input given to a transforming kernel");
  dim3 grid((unsigned)(((a.T_out + TM - 1) / TM) * (a.F_out / kTF) * ((a.n_cols + BN - 1) / BN)), 1u,
            (unsigned)batch);
  if constexpr (PRE && !XTRA) {
    if (x3 == 3) {
      hipLaunchKernelGGL((tap_gemm_kernel<KH, KW, S, PAD, TM, BN, WM, false, UPS, XTRA, PRE, true>), grid,
                         dim3(kThreads), 0, st, a);
      SESA_CHECK_LAUNCH();
      return SESA_OK;
    }
  }
  if (x3)
    hipLaunchKernelGGL((tap_gemm_kernel<KH, KW, S, PAD, TM, BN, WM, true, UPS, XTRA, PRE>), grid, dim3(kThreads), 0, st, a);
  else
    hipLaunchKernelGGL((tap_gemm_kernel<KH, KW, S, PAD, TM, BN, WM, false, UPS, XTRA, PRE>), grid, dim3(kThreads), 0, st, a);
  SESA_CHECK_LAUNCH();
  return SESA_OK;
}

}  // namespace

namespace {
int cu_count() {
  static int n[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (n[dev] == 0) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    n[dev] = v;
  }
  return n[dev];
}
// SESA_CONV_VARIANT=m16 selects conv3x3_m16_kernel (measured on par with conv3x3_db_kernel -- see
// DESIGN.md 4a -- while its shortcut operand costs act_split an extra plane write); default: db.
std::atomic<int> g_conv_variant{-1};
int conv_variant() {
  int v = g_conv_variant.load(std::memory_order_relaxed);
  if (v < 0) {
    v = getenv("SESA_CONV_VARIANT") && std::string(getenv("SESA_CONV_VARIANT")) == "m16" ? 1 : 0;
    int expect = -1;
    g_conv_variant.compare_exchange_strong(expect, v);
    v = g_conv_variant.load(std::memory_order_relaxed);
  }
  return v;
}
}  // namespace

int set_conv3x3_variant(int v) {
  const int prev = conv_variant();
  g_conv_variant.store(v == 1 ? 1 : 0);
  return prev;
}

// SESA_CONV_MI4=0: the fp16 single-pass TFC convs on the 16-row tile (A/B of conv3x3_db_kernel<MI4>)
bool conv3x3_mi4_enabled() {
  static const bool v = !(getenv("SESA_CONV_MI4") && std::string(getenv("SESA_CONV_MI4")) == "0");
  return v;
}

// SESA_CONV_ORD=1: every other group of 8 workgroups of a conv with a fused shortcut runs the shortcut phase
// first (conv3x3_db_kernel<ORD>).  Off: measured slower -- conv_bench 57 f16 L0 7.37 -> 8.11 ms, the headline
// 249.0x -> 246.9x same box (profiles/r04_ord_*): the shortcut phase is bound by the bytes one CU keeps in
// flight, not by the chip's HBM bandwidth, so desynchronising the phases buys nothing.
bool conv3x3_ord_enabled() {
  static const bool v = getenv("SESA_CONV_ORD") && std::string(getenv("SESA_CONV_ORD")) == "1";
  return v;
}

// The fused 1x1 shortcut of the fp16 MI4 conv3x3 on the per-wave LDS-DMA ring (SCR = 2): measured
// 4-17 % faster per level than the LDS-staged phase and bit-identical to it (profiles/
// r04_conv_bench_f16_dmaring.txt).  SESA_CONV_SCR=0 restores the LDS-staged phase (A/B).
bool conv3x3_scr_ring_enabled() {
  static const bool v = !(getenv("SESA_CONV_SCR") && std::string(getenv("SESA_CONV_SCR")) == "0");
  return v;
}

// The fp16 MI4 conv3x3's main chunks staged by LDS-DMA with per-tile precomputed halo offsets (conv3x3_db_kernel<MDMA>)
// instead of through VGPRs: measured bit-identical and 3-4 % faster per level without the shortcut, ~1 % with it
// (tools/conv_bench 57 mdma, profiles/r05_conv_bench_mdma.txt), +0.4 % end to end on one box.  SESA_CONV_MDMA=0: the
// register-staged main phase (A/B).
bool conv3x3_mdma_enabled() {
  static const bool v = !(getenv("SESA_CONV_MDMA") && std::string(getenv("SESA_CONV_MDMA")) == "0");
  return v;
}

// The fused 1x1 shortcut interleaved with the LDS-DMA main loop (conv3x3_db_kernel<SCR = 3>), opt-in SESA_CONV_SCI=1:
// measured SLOWER than the ring after the main loop -- per level +0 (L1 enc) ... +37 % (L3 enc), the headline 270.5 ->
// 266.8x same box (profiles/r05_u_*): the main loop does not leave the raw-input stream idle issue slots to hide in,
// the shortcut's MFMAs, splits and loads simply add to it.
bool conv3x3_sci_enabled() {
  static const bool v = getenv("SESA_CONV_SCI") && std::string(getenv("SESA_CONV_SCI")) == "1";
  return v;
}

bool tap_bn128_enabled() {
  static const bool v = !(getenv("SESA_TAP_BN128") && std::string(getenv("SESA_TAP_BN128")) == "0");
  return v;
}

// conv3x3_db_kernel<ACT>: the consumer's norm + GELU + split fused into the staging (no act_split pass).
// Each workgroup stages (and so transforms) every input element of its halo once per 64-channel output
// block, i.e. ~1.2 x C_out / 64 times per element, where act_split transforms it once: measured on
// MI355X (tools/conv_bench act, profiles/r03_conv_act_*.txt) the fusion wins only with <= 2 output
// blocks (level 0, C_out = 128) -- the main loop runs at the power-limited MFMA plateau, so the
// staging VALU is not free even when interleaved with the MFMAs.  SESA_CONV_FUSED_ACT=0: never;
// =all: at every T >= 32 level (A/B).
bool conv3x3_fused_act_ok(int T_out, int C_in, int C_out) {
  static const int mode = [] {
    const char* e = getenv("SESA_CONV_FUSED_ACT");
    return !e ? 1 : std::string(e) == "0" ? 0 : std::string(e) == "all" ? 2 : 1;
  }();
  return mode > 0 && conv_variant() == 0 && T_out >= 32 && C_in <= kActMaxC && C_in % kConvBK == 0 &&
         (mode == 2 || C_out <= 128);
}

// Winograd F(2, 3) TFC convs (conv3x3_wino_kernel), opt-in: measured on MI355X at parity with the direct
// kernel end to end (profiles/r03_wino_*): its main loop alone runs 1.6x the direct
// kernel's effective rate, but staging V (bf16 split + LDS writes, 2 V values per input element) and the
// shortcut stages give it back.  SESA_CONV_WINO / sesa_mdx23c_set_wino: 0 (default) never; 1 = T_out in
// [32, 128] (levels 1-3, whose inputs pass through act_split anyway); all / 2 = every T >= 32 level (level
// 0 then trades its fused activation for an act_split fp32 pass).  Read when a model is finalized.
std::atomic<int> g_wino_mode{-1};
int wino_mode() {
  int v = g_wino_mode.load(std::memory_order_relaxed);
  if (v < 0) {
    const char* e = getenv("SESA_CONV_WINO");
    v = !e ? 0 : std::string(e) == "all" || std::string(e) == "2" ? 2 : std::string(e) == "1" ? 1 : 0;
    int expect = -1;
    g_wino_mode.compare_exchange_strong(expect, v);
    v = g_wino_mode.load(std::memory_order_relaxed);
  }
  return v;
}
int set_conv3x3_wino(int mode) {
  const int prev = wino_mode();
  g_wino_mode.store(mode >= 0 && mode <= 2 ? mode : 0);
  return prev;
}
bool conv3x3_wino_selected(int T_out, int C_in, int C_out) {
  const int mode = wino_mode();
  return mode > 0 && conv_variant() == 0 && T_out >= 32 && (mode == 2 || T_out <= 128) && C_in % kConvBK == 0 &&
         C_in <= kMaxCin && C_out % 16 == 0;
}

bool conv3x3_m16_selected(int T_out, int C_in, int C_out, int C_shortcut) {
  return conv_variant() == 1 && T_out >= 32 && C_in % 32 == 0 && C_out % 16 == 0 && C_shortcut % 32 == 0;
}

// Tile choices per kind (BN = 64 unless the GEMM N is <= 32).
// x3: 0 = bf16, 1 = bf16x3; 2 / 3 = the fp16 TFC-conv modes (SESA_PREC_F16W2 / SESA_PREC_F16), accepted only
// for the direct double-buffered 3x3 kernel (the host packs those convs' main chunks as fp16 hi / lo).
int launch_conv(int kind, int bn, int x3, const ConvArgs& a, int batch, hipStream_t st) {
  SESA_REQUIRE(a.F_out % kTF == 0, SESA_ERR_INVALID, "conv: F_out %d not a multiple of %d", a.F_out, kTF);
  const int xmode = x3;
  x3 = x3 != 0 ? 1 : 0;
  const bool db3 = kind == CONV3X3 && a.in.src[0].mode != SRC_ACT32 && a.T_out >= 32 && a.out.residual == nullptr &&
                   a.out.gelu == 0 && !conv3x3_m16_selected(a.T_out, a.in.C_in, a.out.C_out, a.x_chunks > 0 ? a.xin.C_in : 0);
  SESA_REQUIRE(xmode >= 0 && xmode <= 3 && (xmode < 2 || db3 || (xmode == 3 && kind == DECONV2X2S2)), SESA_ERR_INVALID,
               "conv: fp16 mode %d only for the direct 3x3 kernel and the transposed up-convs", xmode);
  SESA_REQUIRE(a.in.C_in % kConvBK == 0 && a.in.C_split % kConvBK == 0 && a.in.C_in <= kMaxCin, SESA_ERR_INVALID,
               "conv: C_in %d / split %d must be multiples of %d (<= %d)", a.in.C_in, a.in.C_split, kConvBK,
               kMaxCin);
  switch (kind) {
    case CONV3X3:
      if (a.in.src[0].mode == SRC_ACT32) {
        SESA_REQUIRE(a.in.src[0].ptr && a.in.C_split == a.in.C_in && a.in.src[0].C == a.in.C_in &&
                         a.out.residual == nullptr && a.out.gelu == 0 && a.T_in == a.T_out && a.F_in == a.F_out &&
                         a.n_chunks * kConvBK == a.in.C_in && a.out.C_out % 16 == 0,
                     SESA_ERR_INVALID, "conv3x3 (Winograd): needs one pre-activated fp32 input, same-size conv");
        if (a.x_chunks > 0)
          SESA_REQUIRE(a.xin.C_in % kConvBK == 0 && a.xin.C_split % kConvBK == 0 && a.x_chunks * kConvBK == a.xin.C_in &&
                           a.xin.src[0].mode == SRC_RAW && a.xin.src[1].mode == SRC_RAW && a.xin.src[0].C % 8 == 0 &&
                           a.xin.src[1].C % 8 == 0,
                       SESA_ERR_INVALID, "conv3x3 (Winograd): fused shortcut must be a raw input, C_in multiple of %d",
                       kConvBK);
        const int64_t nblk = (int64_t)((a.T_out + 15) / 16) * (a.F_out / kTF) * ((a.n_cols + 63) / 64);
        SESA_REQUIRE(nblk < (1ll << 31) && batch < 65536, SESA_ERR_INVALID, "conv3x3 (Winograd): grid too large");
        dim3 grid((unsigned)nblk, 1u, (unsigned)batch);
        if (a.x_chunks > 0) {
          if (x3) hipLaunchKernelGGL((conv3x3_wino_kernel<true, true>), grid, dim3(512), 0, st, a);
          else hipLaunchKernelGGL((conv3x3_wino_kernel<false, true>), grid, dim3(512), 0, st, a);
        } else {
          if (x3) hipLaunchKernelGGL((conv3x3_wino_kernel<true, false>), grid, dim3(512), 0, st, a);
          else hipLaunchKernelGGL((conv3x3_wino_kernel<false, false>), grid, dim3(512), 0, st, a);
        }
        SESA_CHECK_LAUNCH();
        return SESA_OK;
      }
      if (a.out.residual == nullptr && a.out.gelu == 0 &&
          conv3x3_m16_selected(a.T_out, a.in.C_in, a.out.C_out, a.x_chunks > 0 ? a.xin.C_in : 0)) {
        SESA_REQUIRE(a.in.src[0].mode == SRC_PRE && a.in.src[0].hi && a.in.src[0].lo && a.in.C_split == a.in.C_in,
                     SESA_ERR_INVALID, "conv3x3: needs a single pre-activated (act_split) input");
        SESA_REQUIRE(a.x_chunks == 0 || (a.xin.src[0].mode == SRC_PRE && a.xin.src[0].hi && a.xin.src[0].lo &&
                                         a.xin.C_split == a.xin.C_in && a.x_chunks * kConvBK == a.xin.C_in),
                     SESA_ERR_INVALID, "conv3x3: the fused shortcut must be given as act_split raw planes");
        SESA_REQUIRE(a.T_in == a.T_out && a.F_in == a.F_out && a.n_chunks * kConvBK == a.in.C_in, SESA_ERR_INVALID,
                     "conv3x3: same-size convolution expected");
        const int64_t n_work =
            (int64_t)batch * ((a.T_out + 15) / 16) * (a.F_out / kTF) * ((a.n_cols + 63) / 64);
        SESA_REQUIRE(n_work < (1ll << 31), SESA_ERR_INVALID, "conv3x3: too many work items");
        const dim3 grid((unsigned)std::min<int64_t>(n_work, cu_count()));
        if (a.x_chunks > 0) {
          if (x3) hipLaunchKernelGGL((conv3x3_m16_kernel<true, true>), grid, dim3(512), 0, st, a, (int)n_work);
          else hipLaunchKernelGGL((conv3x3_m16_kernel<false, true>), grid, dim3(512), 0, st, a, (int)n_work);
        } else {
          if (x3) hipLaunchKernelGGL((conv3x3_m16_kernel<true, false>), grid, dim3(512), 0, st, a, (int)n_work);
          else hipLaunchKernelGGL((conv3x3_m16_kernel<false, false>), grid, dim3(512), 0, st, a, (int)n_work);
        }
        SESA_CHECK_LAUNCH();
        return SESA_OK;
      }
      if (a.T_out >= 32 && a.out.residual == nullptr && a.out.gelu == 0) {
        // double-buffered 16-row tile (levels with T >= 32); tile rows past T_out are masked
        const bool act = a.in.src[0].mode == SRC_NORM_GELU;
        if (act) {
          SESA_REQUIRE(conv3x3_fused_act_ok(a.T_out, a.in.C_in, a.out.C_out) && a.in.src[0].ptr && a.in.src[0].stats &&
                           (a.in.C_split == a.in.C_in ||
                            (a.in.src[1].mode == SRC_NORM_GELU && a.in.src[1].ptr && a.in.src[1].stats)) &&
                           a.in.src[0].C % 8 == 0 && (a.in.C_split == a.in.C_in || a.in.src[1].C % 8 == 0),
                       SESA_ERR_INVALID, "conv3x3: fused-activation input must be normalised fp32 sources, C <= %d",
                       kActMaxC);
        } else {
          SESA_REQUIRE(a.in.src[0].mode == SRC_PRE && a.in.src[0].hi && (xmode >= 2 || a.in.src[0].lo) &&
                           a.in.C_split == a.in.C_in,
                       SESA_ERR_INVALID, "conv3x3: needs a single pre-activated (act_split) input");
        }
        dim3 grid((unsigned)(((a.T_out + 15) / 16) * (a.F_out / kTF) * ((a.n_cols + 63) / 64)), 1u, (unsigned)batch);
        if (a.x_chunks > 0)
          SESA_REQUIRE(a.xin.C_in % kConvBK == 0 && a.xin.C_split % kConvBK == 0 && a.xin.src[0].mode == SRC_RAW &&
                           a.xin.src[1].mode == SRC_RAW,
                       SESA_ERR_INVALID, "conv3x3: fused shortcut must be a raw input, C_in multiple of %d", kConvBK);
        const bool ord = conv3x3_ord_enabled();
#define SESA_DB(X3V, XTRAV, F16V)                                                                                     \
  do {                                                                                                               \
    if (act) hipLaunchKernelGGL((conv3x3_db_kernel<X3V, XTRAV, 0, true, F16V>), grid, dim3(512), 0, st, a);           \
    else if (XTRAV && ord)                                                                                           \
      hipLaunchKernelGGL((conv3x3_db_kernel<X3V, XTRAV, 0, false, F16V, false, false, 2, true>), grid, dim3(512), 0, \
                         st, a);                                                                                     \
    else hipLaunchKernelGGL((conv3x3_db_kernel<X3V, XTRAV, 0, false, F16V>), grid, dim3(512), 0, st, a);              \
  } while (0)
        // xmode 2 = fp16 x fp16 hi/lo weights (F16 = 2), 3 = fp16 single pass (F16 = 1; on pre-activated
        // planes the 32-row MI4 tile unless SESA_CONV_MI4=0)
        if (xmode == 3 && !act && conv3x3_mi4_enabled()) {
          const dim3 g32((unsigned)(((a.T_out + 31) / 32) * (a.F_out / kTF) * ((a.n_cols + 63) / 64)), 1u,
                         (unsigned)batch);
          // the DMA ring walks chunk pairs and addresses each batch item's shortcut image with 32-bit offsets
          const bool ring = a.x_chunks > 0 && !ord && conv3x3_scr_ring_enabled() && a.x_chunks % 2 == 0 &&
                            (int64_t)a.T_in * a.F_in * std::max(a.xin.src[0].C, a.xin.src[1].C) * 4 < (1ll << 31);
          // MDMA: the batch item's fp16 plane addressed with 32-bit offsets
          const bool mdma = conv3x3_mdma_enabled() && (int64_t)a.T_in * a.F_in * a.in.src[0].C * 2 < (1ll << 31);
          // SCI: the shortcut chunks past the main loop's (a.x_chunks - a.n_chunks of them) go to the ring in pairs
          const bool sci = ring && mdma && conv3x3_sci_enabled() &&
                           (a.x_chunks - std::min(a.x_chunks, a.n_chunks)) % 2 == 0;
          if (sci)
            hipLaunchKernelGGL((conv3x3_db_kernel<true, true, 0, false, 1, true, 3, 2, false, 1>), g32, dim3(512), 0, st,
                               a);
          else if (ring && mdma)
            hipLaunchKernelGGL((conv3x3_db_kernel<true, true, 0, false, 1, true, 2, 2, false, 1>), g32, dim3(512), 0, st,
                               a);
          else if (ring)
            hipLaunchKernelGGL((conv3x3_db_kernel<true, true, 0, false, 1, true, 2>), g32, dim3(512), 0, st, a);
          else if (a.x_chunks == 0 && mdma)
            hipLaunchKernelGGL((conv3x3_db_kernel<true, false, 0, false, 1, true, 0, 2, false, 1>), g32, dim3(512), 0, st,
                               a);
          else if (a.x_chunks > 0 && ord)
            hipLaunchKernelGGL((conv3x3_db_kernel<true, true, 0, false, 1, true, false, 2, true>), g32, dim3(512), 0, st, a);
          else if (a.x_chunks > 0)
            hipLaunchKernelGGL((conv3x3_db_kernel<true, true, 0, false, 1, true>), g32, dim3(512), 0, st, a);
          else hipLaunchKernelGGL((conv3x3_db_kernel<true, false, 0, false, 1, true>), g32, dim3(512), 0, st, a);
        } else if (a.x_chunks > 0) {
          if (xmode == 3) SESA_DB(true, true, 1);
          else if (xmode == 2) SESA_DB(true, true, 2);
          else if (x3) SESA_DB(true, true, 0);
          else SESA_DB(false, true, 0);
        } else {
          if (xmode == 3) SESA_DB(true, false, 1);
          else if (xmode == 2) SESA_DB(true, false, 2);
          else if (x3) SESA_DB(true, false, 0);
          else SESA_DB(false, false, 0);
        }
#undef SESA_DB
        SESA_CHECK_LAUNCH();
        return SESA_OK;
      }
      if (a.x_chunks > 0) {
        SESA_REQUIRE(a.xin.C_in % kConvBK == 0 && a.xin.C_split % kConvBK == 0, SESA_ERR_INVALID,
                     "conv: fused shortcut C_in %d must be a multiple of %d", a.xin.C_in, kConvBK);
        return launch_conv_t<3, 3, 1, 1, 8, 64, 4, false, true, true>(x3, a, batch, st);
      }
      return launch_conv_t<3, 3, 1, 1, 8, 64, 4, false, false, true>(x3, a, batch, st);
    case CONV1X1:
      if (bn == 32) return launch_conv_t<1, 1, 1, 0, 8, 32, 4, false, false, false>(x3, a, batch, st);
      if (bn == 128) return launch_conv_t<1, 1, 1, 0, 8, 128, 4, false, false, false>(x3, a, batch, st);
      return launch_conv_t<1, 1, 1, 0, 8, 64, 4, false, false, false>(x3, a, batch, st);
    case CONV2X2S2:
      if (bn == 128) return launch_conv_t<2, 2, 2, 0, 4, 128, 4, false, false, true>(x3, a, batch, st);
      return launch_conv_t<2, 2, 2, 0, 4, 64, 4, false, false, true>(x3, a, batch, st);
    case DECONV2X2S2:   // (xmode 3: the fp16 plane x fp16 image kernel)
      if (bn == 128) return launch_conv_t<1, 1, 1, 0, 8, 128, 4, true, false, true>(xmode == 3 ? 3 : x3, a, batch, st);
      return launch_conv_t<1, 1, 1, 0, 8, 64, 4, true, false, true>(xmode == 3 ? 3 : x3, a, batch, st);
  }
  set_error("conv: unknown kind %d", kind);
  return SESA_ERR_INVALID;
}

template <int WM, int WN, int MI, int NI, bool KC, bool OT>
int launch_tdf_t(int x3, const TdfArgs& a, hipStream_t st) {
  constexpr int BM = WM * MI * 32, BN = WN * NI * 32, NT = 64 * WM * WN;
  const int64_t n_total = (int64_t)a.batch * a.T * a.in.src[0].C;
  const int64_t blocks = ((a.M + BM - 1) / BM) * ((n_total + BN - 1) / BN);
  SESA_REQUIRE(blocks < (1ll << 31), SESA_ERR_INVALID, "tdf: grid too large");
  if (x3) hipLaunchKernelGGL((tdf_kernel<WM, WN, MI, NI, true, KC, OT>), dim3((unsigned)blocks), dim3(NT), 0, st, a);
  else hipLaunchKernelGGL((tdf_kernel<WM, WN, MI, NI, false, KC, OT>), dim3((unsigned)blocks), dim3(NT), 0, st, a);
  SESA_CHECK_LAUNCH();
  return SESA_OK;
}

// BN = 128 columns; BM from the row count (weights are packed per BM-row block to match)
template <bool KC, bool OT>
int launch_tdf_bm(int x3, const TdfArgs& a, hipStream_t st) {
  switch (tdf_block_rows(a.M)) {
    case 256: return launch_tdf_t<4, 1, 2, 4, KC, OT>(x3, a, st);
    case 128: return launch_tdf_t<2, 2, 2, 2, KC, OT>(x3, a, st);
    case 64: return launch_tdf_t<1, 4, 2, 1, KC, OT>(x3, a, st);
    default: return launch_tdf_t<1, 4, 1, 1, KC, OT>(x3, a, st);
  }
}

int64_t tdf_u_floats(int64_t n_cols, int M) { return ((n_cols + 127) / 128) * 128 * (int64_t)((M + 31) / 32 * 32); }

int tdf_block_rows(int M) { return M > 128 ? 256 : M > 64 ? 128 : M > 32 ? 64 : 32; }


int launch_act_split(const GemmIn& in, int64_t n_pos, int batch, uint16_t* hi, uint16_t* lo, hipStream_t st,
                     uint16_t* raw_hi, uint16_t* raw_lo) {
  SESA_REQUIRE(in.C_in % 16 == 0 && in.C_split % 8 == 0 && in.C_in <= kMaxCin, SESA_ERR_INVALID,
               "act_split: C %d must be a multiple of 16 (<= %d)", in.C_in, kMaxCin);
  SESA_REQUIRE((raw_hi == nullptr) == (raw_lo == nullptr), SESA_ERR_INVALID, "act_split: raw planes come in pairs");
  // blockDim = groups * lanes_pos (every thread owns one 8-channel group); ~32 positions per thread
  const int groups = in.C_in / 8;
  const int lanes_pos = groups >= kThreads ? 1 : kThreads / groups;
  const int ppb = lanes_pos * 32;
  dim3 grid((unsigned)((n_pos + ppb - 1) / ppb), (unsigned)batch);
  hipLaunchKernelGGL(act_split_kernel<false>, grid, dim3((unsigned)(groups * lanes_pos)), 0, st, in, n_pos, ppb, hi,
                     lo, raw_hi, raw_lo);
  SESA_CHECK_LAUNCH();
  return SESA_OK;
}

int launch_act_f16(const GemmIn& in, int64_t n_pos, int batch, uint16_t* out, hipStream_t st) {
  SESA_REQUIRE(in.C_in % 16 == 0 && in.C_split % 8 == 0 && in.C_in <= kMaxCin, SESA_ERR_INVALID,
               "act_f16: C %d must be a multiple of 16 (<= %d)", in.C_in, kMaxCin);
  const int groups = in.C_in / 8;
  const int lanes_pos = groups >= kThreads ? 1 : kThreads / groups;
  const int ppb = lanes_pos * 32;
  dim3 grid((unsigned)((n_pos + ppb - 1) / ppb), (unsigned)batch);
  hipLaunchKernelGGL((act_split_kernel<false, true>), grid, dim3((unsigned)(groups * lanes_pos)), 0, st, in, n_pos,
                     ppb, out, nullptr, nullptr, nullptr);
  SESA_CHECK_LAUNCH();
  return SESA_OK;
}

int launch_act_f32(const GemmIn& in, int64_t n_pos, int batch, float* out, hipStream_t st) {
  SESA_REQUIRE(in.C_in % 16 == 0 && in.C_split % 8 == 0 && in.C_in <= kMaxCin, SESA_ERR_INVALID,
               "act_f32: C %d must be a multiple of 16 (<= %d)", in.C_in, kMaxCin);
  const int groups = in.C_in / 8;
  const int lanes_pos = groups >= kThreads ? 1 : kThreads / groups;
  const int ppb = lanes_pos * 32;
  dim3 grid((unsigned)((n_pos + ppb - 1) / ppb), (unsigned)batch);
  hipLaunchKernelGGL(act_split_kernel<true>, grid, dim3((unsigned)(groups * lanes_pos)), 0, st, in, n_pos, ppb,
                     reinterpret_cast<uint16_t*>(out), nullptr, nullptr, nullptr);
  SESA_CHECK_LAUNCH();
  return SESA_OK;
}

// transposed_io: 0 = first Linear (NHWC in, U^T out), 1 = second Linear (U^T in, NHWC out)
namespace {
int tdf_variant() {  // SESA_TDF_VARIANT=old: the round-1 register-staged tdf_kernel everywhere (A/B)
  static const int v = getenv("SESA_TDF_VARIANT") && std::string(getenv("SESA_TDF_VARIANT")) == "old" ? 1 : 0;
  return v;
}
}  // namespace

// The fp16 TDF Linears on the deep rings (tdf_dma_kernel<..., DEEP>): the pre-split second Linear 3.61 -> 3.21 ms at
// level 0, the tdf class 142 -> 138 ms per step, configs[1] 270.5 -> 272.6x same box, bit-identical output
// (profiles/r05_w_*).  SESA_TDF_DEEP=0: the round-4 rings (A/B).
bool tdf_deep_enabled() {
  static const bool v = !(getenv("SESA_TDF_DEEP") && std::string(getenv("SESA_TDF_DEEP")) == "0");
  return v;
}

// the LDS-DMA TDF kernel takes this Linear (and so may run it in fp16, x3 == 2; the host packs those
// weights as fp16 images): C % 128 == 0, K % 32 == 0, 128 or 256 row blocks, one normalised / raw source
bool tdf_dma_eligible(int C, int K, int M) {
  const int bm = tdf_block_rows(M);
  return tdf_variant() == 0 && C % 128 == 0 && K % kTdfBK == 0 && (bm == 256 || bm == 128);
}

int launch_tdf(int x3, const TdfArgs& a, int batch, hipStream_t st, int transposed_io) {
  TdfArgs b = a;
  b.batch = batch;
  SESA_REQUIRE(a.in.src[0].C % 4 == 0, SESA_ERR_INVALID, "tdf: C %d must be a multiple of 4", a.in.src[0].C);
  {
    const int C = a.in.src[0].C;
    const int bm = tdf_block_rows(a.M);
    const int mode = a.in.src[0].mode;
    const bool dma_ok = tdf_dma_eligible(C, a.K, a.M) && (mode == SRC_NORM_GELU || mode == SRC_RAW) &&
                        a.in.C_split == a.in.C_in && a.in.C_in == C;
    SESA_REQUIRE(x3 != 2 || dma_ok, SESA_ERR_INVALID, "tdf: the fp16 mode needs the LDS-DMA kernel's shapes");
    if (dma_ok) {
      const int64_t n_tiles = (int64_t)batch * a.T * C / 128;
      const int64_t grid = (n_tiles + 7) / 8 * 8 * ((a.M + bm - 1) / bm);
      SESA_REQUIRE(grid < (1ll << 31), SESA_ERR_INVALID, "tdf: grid too large");
      const dim3 g((unsigned)grid), blk(512);
      const bool deep = tdf_deep_enabled();
#define SESA_TDF_DMA(UI, UO, BMV)                                                                     \
  do {                                                                                                \
    if (x3 == 2 && deep) hipLaunchKernelGGL((tdf_dma_kernel<false, UI, UO, BMV, false, true, true>), g, blk, 0, st, b); \
    else if (x3 == 2) hipLaunchKernelGGL((tdf_dma_kernel<false, UI, UO, BMV, false, true>), g, blk, 0, st, b); \
    else if (x3) hipLaunchKernelGGL((tdf_dma_kernel<true, UI, UO, BMV>), g, blk, 0, st, b);            \
    else hipLaunchKernelGGL((tdf_dma_kernel<false, UI, UO, BMV>), g, blk, 0, st, b);                  \
  } while (0)
      if (transposed_io == 0) {
        if (bm == 256) SESA_TDF_DMA(false, true, 256);
        else SESA_TDF_DMA(false, true, 128);
      } else if (b.u_planes && (a.M + bm - 1) / bm >= 3) {
        // act(U) once per element, then the GEMM copies B images (measured: a win where the in-kernel
        // conversion would run >= 3x per element -- level 0 -- neutral at 2x, a loss at 1x)
        if (x3 == 2)
          hipLaunchKernelGGL(tdf_u_split_kernel<true>, dim3((unsigned)n_tiles, (unsigned)a.n_chunks), dim3(512), 0, st, b);
        else
          hipLaunchKernelGGL(tdf_u_split_kernel<false>, dim3((unsigned)n_tiles, (unsigned)a.n_chunks), dim3(512), 0, st, b);
        SESA_CHECK_LAUNCH();
#define SESA_TDF_PRE(BMV)                                                                               \
  do {                                                                                                  \
    if (x3 == 2 && deep) hipLaunchKernelGGL((tdf_dma_kernel<false, true, false, BMV, true, true, true>), g, blk, 0, st, b); \
    else if (x3 == 2) hipLaunchKernelGGL((tdf_dma_kernel<false, true, false, BMV, true, true>), g, blk, 0, st, b); \
    else if (x3) hipLaunchKernelGGL((tdf_dma_kernel<true, true, false, BMV, true>), g, blk, 0, st, b);        \
    else hipLaunchKernelGGL((tdf_dma_kernel<false, true, false, BMV, true>), g, blk, 0, st, b);              \
  } while (0)
        if (bm == 256) SESA_TDF_PRE(256);
        else SESA_TDF_PRE(128);
#undef SESA_TDF_PRE
      } else {
        if (bm == 256) SESA_TDF_DMA(true, false, 256);
        else SESA_TDF_DMA(true, false, 128);
      }
#undef SESA_TDF_DMA
      SESA_CHECK_LAUNCH();
      return SESA_OK;
    }
  }
  if (transposed_io == 0) {
    SESA_REQUIRE(a.M % 4 == 0, SESA_ERR_INVALID, "tdf: M %d must be a multiple of 4", a.M);
    return launch_tdf_bm<false, true>(x3, b, st);
  }
  SESA_REQUIRE(a.K % 8 == 0, SESA_ERR_INVALID, "tdf: K %d must be a multiple of 8", a.K);
  return launch_tdf_bm<true, false>(x3, b, st);
}

}  // namespace sesa
