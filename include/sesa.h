/*
 * libsesa -- MI355X-native chunked source-separation hot path (C ABI).
 *
 * Drop-in boundary for the reference's separation hot path
 * (test4373/SESA-Audio-Separation).  Plain pointers and sizes, no torch
 * types.  All tensors are DEVICE pointers owned by the caller; `stream` is a hipStream_t
 * (NULL = default stream).  Every entry point is asynchronous on `stream`, never synchronises
 * the host, never allocates inside a launch function (safe under hipGraph capture), and
 * returns 0 on success or a negative SESA_ERR_* code with a thread-local message available
 * from sesa_last_error().
 *
 * Concurrency: functions are re-entrant per stream.  The network forwards (sesa_mdx23c_forward, sesa_bsr_forward,
 * sesa_scnet_forward, sesa_htdemucs_forward) take all mutable state from the caller's workspace -- measured independent
 * of its prior contents and writing nothing outside their buffers (tools/ws_guard.py) -- and read the handle's packed
 * weights only, so forwards of one handle may run on several streams of one device at once, each with its own
 * workspace, input and output; the results are bit-identical to running them one after another
 * (tests/test_gpu_parity.py::test_side_streams_bit_identical, tests/test_bsr.py::test_full_size_4min_properties;
 * full-size 4-min tracks at two streams: all four networks 0 differing samples, tools/streams_check.py).  Rounds 4-6
 * saw them differ, from two gfx950 behaviours under another kernel's waves on the same CU: (1) packed-fp32 VALU ops
 * with a source op_sel (v_pk_add_f32 / v_pk_mul_f32, SLP-emitted in the FFT kernels) returned wrong values beside
 * MFMA work (profiles/r06_pk_opsel_hazard.txt) -- libsesa is built without them, tools/isa_guard.py fails the build
 * otherwise; (2) an s_barrier reached with the wave's own LDS writes in flight (the compiler omits the lgkmcnt wait
 * of __syncthreads where its fence needs no cross-address-space ordering) let other waves read the previous FFT
 * stage -- every such barrier now waits first (sesa_sync), tools/barrier_scan.py fails the build otherwise
 * (profiles/r06_sync_ab.txt).  The other entry points (STFT / iSTFT / gather / OLA / blend) are plain streaming
 * kernels without shared state.  Only sesa_*_set_param / _finalize / _destroy mutate a handle and must not overlap
 * its forwards.
 *
 * Compute is fp32 in / fp32 out.  The MDX23C network runs its contractions on MFMA in one of
 * two precisions (sesa_mdx23c_config.precision):
 *   SESA_PREC_BF16X3 -- hi/lo bf16 split, 3 MFMA passes, fp32 accumulate (parity mode:
 *                       ~1.4e-6 RMS vs the fp32 reference on the vocals config)
 *   SESA_PREC_BF16   -- single bf16 pass (throughput mode; ~6e-4 RMS, outside the 1e-4 gate)
 *   SESA_PREC_F16W2 / SESA_PREC_F16 -- the TFC 3x3 convolutions of the T >= 32 levels (~70 % of the
 *                       MDX23C FLOPs) on fp16 MFMA: the activation rounded once to fp16 (2^-11) against
 *                       the fp16 hi + lo weights (2 passes) or the fp16 weights (1 pass); every other
 *                       contraction bf16x3 (MDX23C only; the other models accept BF16X3 / BF16)
 *   SESA_PREC_F16MIX -- MDX23C: those convs per level as the plan of sesa_mdx23c_set_f16_plan says
 *                       (default: one fp16 pass everywhere except the encoder level-1 convs, bf16x3 --
 *                       they carry ~70 % of the fp16 rounding error at the stems), the decoder TDF Linears fp16;
 *                       HTDemucs: the cross-transformer attention (QK^T, PV; fp32 softmax statistics),
 *                       the implicit-GEMM convs, 1x1 rewrites and the transformer / channel Linears on one fp16
 *                       pass (norms and DConv statistics fp32 / fp64);
 *                       SCNet: the token GEMMs (3x3 convs, LSTM input projections, Linears) on one fp16
 *                       pass, the LSTM recurrence bf16x3
 */
#ifndef SESA_H_
#define SESA_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SESA_OK 0
#define SESA_ERR_INVALID (-1)   /* bad argument / unsupported configuration              */
#define SESA_ERR_HIP (-2)       /* HIP runtime error                                      */
#define SESA_ERR_STATE (-3)     /* object used in the wrong state (e.g. params missing)    */
#define SESA_ERR_NOMEM (-4)     /* device allocation failed (create/finalize only)         */

#define SESA_PREC_BF16X3 0
#define SESA_PREC_BF16 1
#define SESA_PREC_F16W2 2 /* MDX23C: TFC 3x3 convs (T >= 32) fp16 activations x fp16 hi/lo weights, 2 passes */
#define SESA_PREC_F16 3   /* MDX23C: TFC 3x3 convs (T >= 32) single fp16 pass; BS- / Mel-Band-Roformer: the
                             QKV / FF Linears single fp16 pass; the rest bf16x3                           */
#define SESA_PREC_F16MIX 4 /* MDX23C: per-level plan of the T >= 32 TFC 3x3 convs (sesa_mdx23c_set_f16_plan);
                              HTDemucs: fp16 attention + convs; SCNet: fp16 token GEMMs */

int sesa_version(void);
const char* sesa_last_error(void);

/* ---------------------------------------------------------------------------------------
 * Spectral front/back end.
 * Replaces models/mdx23c_tfc_tdf_v3.py:14-30 (STFT.__call__ -> torch.stft, center=True,
 * reflect pad, periodic Hann, onesided, un-normalised, cropped to dim_f bins).
 *   x   [n_sig, len]                 fp32
 *   out [n_sig, 2 (re,im), dim_f, frames]  frames = 1 + len / hop
 * (for n_sig = B*c this is exactly the reference's [B, 2c, dim_f, frames] output).
 * Supported: n_fft == 8192, len % hop == 0, len > n_fft/2.
 */
int sesa_stft_f32(const float* x, int n_sig, int len, int n_fft, int hop, int dim_f, float* out,
                  void* stream);

/* Replaces models/mdx23c_tfc_tdf_v3.py:32-44 (STFT.inverse: zero-pad bins dim_f..n_fft/2,
 * torch.istft center=True without `length`).
 *   spec [n_sig, 2 (re,im), dim_f, frames] fp32
 *   out  [n_sig, hop * (frames - 1)]       fp32
 * `frame_ws` is caller-owned scratch of sesa_istft_workspace_size(...) bytes.
 */
size_t sesa_istft_workspace_size(int n_sig, int frames, int n_fft);
int sesa_istft_f32(const float* spec, int n_sig, int dim_f, int frames, int n_fft, int hop,
                   float* out, void* frame_ws, void* stream);

/* ---------------------------------------------------------------------------------------
 * Chunker / windowed overlap-add (inference_pytorch.py:55-186 == utils.py:330-477 generic).
 *
 * sesa_chunk_gather_f32 -- inference_pytorch.py:102-103 + :125-138: builds the batch
 *   out[j] = pad_C( reflect_pad_border(mix)[:, starts[j] : starts[j]+C] ) for j < n_chunks,
 *   where the border reflect pad is applied iff `border` > 0 (caller passes 0 when the
 *   reference would not pad) and a short chunk is padded with reflect if its length > C/2
 *   else with zeros.
 *   mix [n_ch, L] (unpadded), starts (host int64 array, padded coordinates), out [n_chunks, n_ch, C]
 */
int sesa_chunk_gather_f32(const float* mix, int n_ch, int64_t L, int64_t border,
                          const int64_t* starts, int n_chunks, int chunk, float* out, void* stream);

/* sesa_chunk_gather_constant_f32 -- utils.py:371-380 + :413-418 (utils.demix demucs mode, model_type
 *   'htdemucs'): out[j] = zero_pad_C( mix[:, starts[j] : starts[j]+C] ) -- no border pad, and every
 *   short chunk is padded with zeros ('constant') whatever its length.  Same layouts as above.
 */
int sesa_chunk_gather_constant_f32(const float* mix, int n_ch, int64_t L, const int64_t* starts,
                                   int n_chunks, int chunk, float* out, void* stream);

/* sesa_ola_accumulate_f32 -- inference_pytorch.py:151-159.  For chunk j (in order):
 *   result[:, s_j : s_j+n_j] += y[j, :, :n_j] * window[:n_j];  counter[s_j : s_j+n_j] += window[:n_j]
 * with fp32 multiply-then-add rounding and chunk-order summation exactly as the reference.
 *   y [n_chunks, n_out_ch, C] (n_out_ch = n_instr * 2), window [C] (device, the batch's window
 *   after the first/last fade fix-ups), result [n_out_ch, L_pad], counter [L_pad].
 *   starts / seg_lens are host arrays (the chunk plan is host-side control).
 *   n_out_ch == 0 (y and result may be NULL) accumulates the counter only.
 */
int sesa_ola_accumulate_f32(const float* y, int n_chunks, int n_out_ch, int chunk,
                            const int64_t* starts, const int64_t* seg_lens, const float* window,
                            float* result, float* counter, int64_t L_pad, void* stream);

/* sesa_ola_finalize_f32 -- inference_pytorch.py:174-180: out = nan_to_num(result / counter,
 * nan=0) cropped to [border, L_pad - border).  out [n_out_ch, L_pad - 2*border]. */
int sesa_ola_finalize_f32(const float* result, const float* counter, int n_out_ch, int64_t L_pad,
                          int64_t border, float* out, void* stream);

/* ---------------------------------------------------------------------------------------
 * MDX23C TFC-TDF-v3 network (models/mdx23c_tfc_tdf_v3.py:141-242, TFC_TDF_net).
 * Only norm == InstanceNorm and act == gelu are supported (the released configs).
 */
typedef struct sesa_mdx23c_config {
  int chunk_size, dim_f, dim_t, hop_length, n_fft, audio_channels;   /* audio.*            */
  int num_subbands, num_scales, num_blocks_per_scale, num_channels;  /* model.*            */
  int growth, bottleneck_factor, scale_t, scale_f;
  int num_instruments;                                               /* prefer_target_instrument */
  int precision;                                                     /* SESA_PREC_*        */
} sesa_mdx23c_config;

typedef struct sesa_mdx23c sesa_mdx23c;

/* Build the network plan on the current HIP device. */
int sesa_mdx23c_create(const sesa_mdx23c_config* cfg, sesa_mdx23c** out);
/* Number of parameters and the i-th (name, numel) in the reference named_parameters() order. */
int sesa_mdx23c_num_params(const sesa_mdx23c* m);
int sesa_mdx23c_param_info(const sesa_mdx23c* m, int i, const char** name, int64_t* numel);
/* Copy one parameter (HOST fp32, reference state_dict layout) by its reference name
 * (load_state_dict semantics; unknown names return SESA_ERR_INVALID). */
int sesa_mdx23c_set_param(sesa_mdx23c* m, const char* name, const float* host, int64_t numel);
/* Pack weights into the MFMA layouts on the device (after every parameter was set). */
int sesa_mdx23c_finalize(sesa_mdx23c* m, void* stream);
size_t sesa_mdx23c_workspace_size(const sesa_mdx23c* m, int batch);
/* x [batch, audio_channels, chunk_size] -> out [batch, num_instruments, audio_channels, chunk_size] */
int sesa_mdx23c_forward(sesa_mdx23c* m, const float* x, int batch, float* out, void* workspace,
                        size_t workspace_bytes, void* stream);
int sesa_mdx23c_destroy(sesa_mdx23c* m);

/* Kernel choice for the TFC 3x3 convolutions at T >= 32 (process-wide; returns the previous value):
 * 0 = conv3x3_db_kernel (default; v_mfma_f32_32x32x16_bf16, register-staged double buffer),
 * 1 = conv3x3_m16_kernel (v_mfma_f32_16x16x32_bf16, persistent, LDS-DMA; measured on par).
 * Initialised from SESA_CONV_VARIANT=m16.  A forward picks it up at its next call. */
int sesa_mdx23c_set_conv_variant(int variant);
/* Winograd F(2, 3) TFC 3x3 convolutions (conv3x3_wino_kernel; process-wide, returns the previous value):
 * 0 = off (default), 1 = levels with 32 <= T <= 128, 2 = every level with T >= 32.  Initialised from
 * SESA_CONV_WINO; decided per convolution when a model is finalized (the weights are packed for it). */
int sesa_mdx23c_set_wino(int mode);
/* SESA_PREC_F16MIX plan (read when a model is finalized): 16 digits, encoder levels 0..7 then decoder
 * levels 0..7, '1' = fp16, '2' = fp16 x fp16 hi/lo weights, '3' = bf16x3; NULL plan = query only.  The
 * previous plan is copied to prev (17 bytes) when prev is not NULL.  Default "1311111111111111"
 * (env SESA_F16_PLAN overrides it at first use). */
int sesa_mdx23c_set_f16_plan(const char* plan, char* prev);
/* SESA_PREC_F16MIX plan of the TDF Linears (same layout; '1' = one fp16 pass, '3' = bf16x3; only Linears of
 * the LDS-DMA kernel's shapes run fp16).  Default "1333111111111111": encoder levels 1-3 bf16x3, the other stacks
 * in fp16 (env SESA_TDF_PLAN overrides it at first use).  In fp16mix the transposed up-convs also run one fp16
 * pass (env SESA_MDX_UP16=0: bf16x3). */
int sesa_mdx23c_set_tdf_plan(const char* plan, char* prev);

/* ---------------------------------------------------------------------------------------
 * BS-Roformer (models/bs_roformer/bs_roformer.py:327-587, BSRoformer)
 * and Mel-Band-Roformer (same engine, `mel` fields below).
 * STFT n_fft = win = 2048 (any hop dividing chunk_size), stereo or mono, dim_head 64,
 * mask_estimator_depth 2, linear_transformer_depth 0, skip_connection False (released configs).
 * Parameters are the reference state_dict() keys (incl. layers.*.rotary_embed.freqs).
 */
typedef struct sesa_bsr_config {
  int chunk_size, audio_channels, n_fft, hop_length, win_length;
  int dim, depth, heads, dim_head, time_transformer_depth, freq_transformer_depth;
  int num_stems, mask_estimator_depth, mlp_expansion_factor;
  int n_bands;
  const int* freqs_per_bands;   /* host array [n_bands] (frequencies per band), copied by create */
  int precision;                /* SESA_PREC_*                                       */
  /* Mel-Band-Roformer (models/bs_roformer/mel_band_roformer.py:324-620) when mel != 0:
   * overlapping bands gathered by freq_indices ((f, s) rows, reference buffer `freq_indices`,
   * :431-437), RMSNorm after every Transformer (norm_output, :218), no final_norm, mask MLPs of
   * mask_estimator_depth + 1 Linear layers (:261-283), masks scatter-averaged (:596-606). */
  int mel;
  int n_freq_indices;
  const int* freq_indices;      /* host array [n_freq_indices], copied by create (mel only) */
} sesa_bsr_config;

typedef struct sesa_bsr sesa_bsr;

int sesa_bsr_create(const sesa_bsr_config* cfg, sesa_bsr** out);
int sesa_bsr_num_params(const sesa_bsr* m);
int sesa_bsr_param_info(const sesa_bsr* m, int i, const char** name, int64_t* numel);
int sesa_bsr_set_param(sesa_bsr* m, const char* name, const float* host, int64_t numel);
int sesa_bsr_finalize(sesa_bsr* m, void* stream);
size_t sesa_bsr_workspace_size(const sesa_bsr* m, int batch);
/* x [batch, audio_channels, chunk_size] -> out [batch, num_stems, audio_channels, chunk_size] */
int sesa_bsr_forward(sesa_bsr* m, const float* x, int batch, float* out, void* workspace,
                     size_t workspace_bytes, void* stream);
int sesa_bsr_destroy(sesa_bsr* m);

/* ---------------------------------------------------------------------------------------
 * SCNet (models/scnet/scnet.py:239-373 SCNet + models/scnet/separation.py).
 * n_fft = win_size = 4096, conv_kernel 3, even num_dplayer, LSTM hidden (dims[-1] * expand, x2 on
 * the odd dual-path layers) in {32, 64, 128, 256}.  Parameters are the reference state_dict() keys.
 * band_sr is double so the split points match the reference's math.ceil(Fr * SR) (scnet.py:117-122).
 */
typedef struct sesa_scnet_config {
  int chunk_size, audio_channels, n_sources;
  int n_fft, hop_size, win_size, normalized;
  int n_dims;
  const int* dims;              /* host array [n_dims] (model.dims), copied by create          */
  double band_sr[3];
  int band_stride[3], band_kernel[3], conv_depths[3];
  int compress, conv_kernel, num_dplayer, expand;
  int precision;                /* SESA_PREC_*: the MFMA token GEMMs (LSTM input / output Linears) */
} sesa_scnet_config;

typedef struct sesa_scnet sesa_scnet;

int sesa_scnet_create(const sesa_scnet_config* cfg, sesa_scnet** out);
int sesa_scnet_num_params(const sesa_scnet* m);
int sesa_scnet_param_info(const sesa_scnet* m, int i, const char** name, int64_t* numel);
int sesa_scnet_set_param(sesa_scnet* m, const char* name, const float* host, int64_t numel);
int sesa_scnet_finalize(sesa_scnet* m, void* stream);
size_t sesa_scnet_workspace_size(const sesa_scnet* m, int batch);
/* x [batch, audio_channels, chunk_size] -> out [batch, n_sources, audio_channels, chunk_size] */
int sesa_scnet_forward(sesa_scnet* m, const float* x, int batch, float* out, void* workspace,
                       size_t workspace_bytes, void* stream);
int sesa_scnet_destroy(sesa_scnet* m);

/* ---------------------------------------------------------------------------------------
 * HTDemucs (models/demucs4ht.py:28-693 HTDemucs, cac), the hybrid
 * time / frequency U-Net with the cross-domain transformer.  Replaces HTDemucs.forward
 * (:548-693) for use_train_segment=False: _spec (:427-446), _magnitude (:459-468), the branch
 * normalisation, HEncLayer / HDecLayer / DConv (third-party demucs.hdemucs / demucs.demucs,
 * restated), the CrossTransformerEncoder (demucs.transformer, restated), _mask (:470-481) and
 * _ispec (:448-457).  Supported: stereo, cac, num_subbands 1, no multi_freqs, wiener_iters 0,
 * nfft 4096, kernel 8 / stride 4, rewrite, no GroupNorm in the U-Net layers (norm_starts >=
 * depth), every encoder level a frequency level (no branch merge), sinusoidal embeddings,
 * dense attention, norm_first + norm_out + LayerScale (the released htdemucs configs).
 * Parameters are the reference state_dict() keys.
 */
typedef struct sesa_htdemucs_config {
  int chunk_size;                       /* samples per forward item (samplerate * segment)       */
  int audio_channels, n_sources;
  int channels, channels_time, growth, nfft, depth;
  int kernel_size, stride, context, context_enc;
  int norm_starts, rewrite, cac, num_subbands;
  int dconv_mode, dconv_depth, dconv_comp;
  int bottom_channels;
  int t_layers, t_heads, t_norm_in, t_norm_first, t_norm_out, t_layer_scale, t_gelu, t_cross_first;
  double t_hidden_scale, freq_emb, emb_scale, t_max_period, t_weight_pos_embed;
  int precision;                        /* SESA_PREC_*: the MFMA GEMMs (convs, transformer)      */
} sesa_htdemucs_config;

typedef struct sesa_htdemucs sesa_htdemucs;

int sesa_htdemucs_create(const sesa_htdemucs_config* cfg, sesa_htdemucs** out);
int sesa_htdemucs_num_params(const sesa_htdemucs* m);
int sesa_htdemucs_param_info(const sesa_htdemucs* m, int i, const char** name, int64_t* numel);
/* Shape of the i-th parameter: writes ndim (<= 4) and dims[0 .. ndim). */
int sesa_htdemucs_param_shape(const sesa_htdemucs* m, int i, int64_t* dims, int* ndim);
int sesa_htdemucs_set_param(sesa_htdemucs* m, const char* name, const float* host, int64_t numel);
int sesa_htdemucs_finalize(sesa_htdemucs* m, void* stream);
size_t sesa_htdemucs_workspace_size(const sesa_htdemucs* m, int batch);
/* x [batch, audio_channels, chunk_size] -> out [batch, n_sources, audio_channels, chunk_size] */
int sesa_htdemucs_forward(sesa_htdemucs* m, const float* x, int batch, float* out, void* workspace,
                          size_t workspace_bytes, void* stream);
int sesa_htdemucs_destroy(sesa_htdemucs* m);

/* ---------------------------------------------------------------------------------------
 * Ensemble blend (ensemble.py:172-407, AudioEnsembleEngine.process_waveform / process_spectral /
 * run_ensemble's buffer loop).  Methods in the reference's --type order.
 *   x   [n_files][n_ch][L] fp32 (device; the inputs cut to the shortest, ensemble.py:304-306)
 *   out [n_ch][L] float64 (device; written as PCM_24 by the caller, :311)
 *   weights: host float[n_files] or NULL (normalised in float32 exactly as :288-293)
 * Spectral methods process independent `buffer`-sample pieces (scipy stft/istft per piece,
 * nperseg = min(1024, piece)); pieces < 256 samples use avg_wave (:355-357).  They need a
 * caller-owned workspace of sesa_blend_workspace_size_n(n_files, n_ch, buffer) bytes
 * (sesa_blend_workspace_size(n_ch, buffer) covers n_files <= 8).  1 <= n_files <= 64.  NaN
 * propagates through max / min / median as in numpy.
 */
#define SESA_BLEND_AVG_WAVE 0
#define SESA_BLEND_MEDIAN_WAVE 1
#define SESA_BLEND_MAX_WAVE 2
#define SESA_BLEND_MIN_WAVE 3
#define SESA_BLEND_MAX_FFT 4
#define SESA_BLEND_MIN_FFT 5
#define SESA_BLEND_MEDIAN_FFT 6
size_t sesa_blend_workspace_size(int n_ch, int64_t buffer);
size_t sesa_blend_workspace_size_n(int n_files, int n_ch, int64_t buffer);
int sesa_blend_f32(const float* x, int n_files, int n_ch, int64_t L, int64_t buffer, int method,
                   const float* weights, double* out, void* workspace, size_t workspace_bytes,
                   void* stream);

/* ---------------------------------------------------------------------------------------
 * FLAC codec (HOST memory; the CLI's audio I/O: inference_pytorch.py:213 librosa.load of FLAC
 * inputs, :262-272 sf.write(<name>_<instr>.flac, subtype=PCM_16 / PCM_24)).  Decoded samples are
 * scaled like libsndfile's float read (int / 2^(bits-1)); the encoder quantises like libsndfile's
 * float write (x * (2^(bits-1) - 1), round half to even), clipped to the bit depth.
 *   out / in: interleaved float [frames][channels]
 */
int sesa_flac_info(const uint8_t* data, size_t n, int* channels, int* sample_rate, int* bits, int64_t* frames);
int sesa_flac_decode(const uint8_t* data, size_t n, float* out, int64_t max_frames, int64_t* frames_out);
size_t sesa_flac_encode_bound(int64_t frames, int channels, int bits);
int sesa_flac_encode(const float* in, int64_t frames, int channels, int sample_rate, int bits, uint8_t* out,
                     size_t cap, size_t* written);

/* ---------------------------------------------------------------------------------------
 * Kernel timing (measurement support for bench.py; not part of the reference surface).
 * While enabled, every launch issued by libsesa is bracketed by a hipEvent pair on its own
 * stream and tagged with its kernel class and ALGORITHMIC work (reference FLOPs for the
 * contractions -- not the 3x MFMA work of the bf16x3 split -- or HBM bytes for streaming
 * kernels).  sesa_profile_read synchronises on the recorded events.
 */
#define SESA_KCLASS_CONV3X3 0
#define SESA_KCLASS_CONV1X1 1
#define SESA_KCLASS_DOWN 2
#define SESA_KCLASS_UP 3
#define SESA_KCLASS_TDF 4
#define SESA_KCLASS_STFT 5
#define SESA_KCLASS_ISTFT 6
#define SESA_KCLASS_ACT 7     /* act_split: norm + GELU + bf16 split pass (work = HBM bytes) */
#define SESA_KCLASS_TOKGEMM 8 /* token-major Linear layers (transformer models)           */
#define SESA_KCLASS_ATTN 9    /* flash attention (work = 4 L^2 d FLOP per sequence-head)    */
#define SESA_KCLASS_LSTM 10   /* SCNet bi-LSTM recurrence (work = h W_hh^T FLOP)            */
#define SESA_KCLASS_SIMT 11   /* fp32 VALU kernels: SCNet convolutions / feature-conversion DFTs, HTDemucs DConv */
#define SESA_KCLASS_OLA 12    /* chunk gather / overlap-add / finalize (work = HBM bytes)     */
#define SESA_KCLASS_HCONV 13  /* HTDemucs implicit-GEMM convolutions (tok_gemm conv mode)    */
#define SESA_KCLASS_CONV3X3_X3 14 /* MDX23C fp16 modes: the TFC 3x3 convs that stay bf16x3 (plan '3', T < 32) */
#define SESA_KCLASS_DFT 15    /* SCNet feature-conversion DFTs over T on MFMA (work = 2 M K N GEMM FLOP) */
#define SESA_KCLASS_COUNT 16
int sesa_profile_enable(int enable);   /* 1: start recording (clears previous records), 0: stop */
int sesa_profile_read(int kclass, double* total_ms, int64_t* launches, double* total_work);
/* as sesa_profile_read, plus the class's ALGORITHMIC HBM bytes (each operand read once, each result written once,
 * in the storage type the launch actually reads / writes) for the compute classes -- the bytes the roofline's
 * HBM floor is priced on (0 for a launch that states none) */
int sesa_profile_read2(int kclass, double* total_ms, int64_t* launches, double* total_work, double* total_bytes);
/* sum over the class's launches of max(work / (peak_tflops 1e12), bytes / (peak_gbs 1e9)) in ms: the class's time at
 * the roofline bound of each launch's own arithmetic intensity */
int sesa_profile_floor(int kclass, double peak_tflops, double peak_gbs, double* floor_ms);

/* Diagnostics (tools/streams_trace.py): while a trace is open on the calling host thread, every instrumented launch of
 * the network forwards is followed, on its own stream, by a kernel that adds a 64-bit checksum of that launch's output
 * bytes into the next slot of `buf` (device memory, `cap` zeroed uint64 slots), so two runs can be compared launch by
 * launch.  sesa_debug_trace_end closes the trace, copies each traced launch's kernel class into `classes` (up to cap)
 * and returns the number of traced launches. */
int sesa_debug_trace_begin(void* buf, int cap);
int sesa_debug_trace_end(int* classes, int cap);

#ifdef __cplusplus
}
#endif
#endif /* SESA_H_ */
