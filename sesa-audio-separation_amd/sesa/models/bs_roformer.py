"""BS-Roformer on the native MI355X forward (libsesa ``sesa_bsr_*``).

Drop-in for ``models/bs_roformer/bs_roformer.py:327-587`` (``BSRoformer``): constructed from
``**config.model`` exactly like the reference registry does (``utils.py:104-106``), same
``state_dict`` keys / shapes (incl. ``layers.*.rotary_embed.freqs``, so released checkpoints load
unchanged), same call ``model(x[B, ch, C]) -> [B, ch, C]`` for one stem (``[B, stems, ch, C]``
otherwise, :579-582).  The forward runs entirely in libsesa on the current HIP stream: STFT,
band split, the depth x (time, freq) rotary transformers, mask estimators, complex mask and
iSTFT (sesa_bsroformer.hip, kernels in sesa_tokgemm.hip).  No CPU fallback.
"""
import ctypes

import torch

from .. import _native as N
from .native import NativeModule

DEFAULT_FREQS_PER_BANDS = (2,) * 24 + (4,) * 12 + (12,) * 8 + (24,) * 8 + (48,) * 8 + (128, 129)


def _freqs(dim_head, theta=10000.0):
    return (1.0 / (theta ** (torch.arange(0, dim_head, 2)[: dim_head // 2].float() / dim_head))).numpy()


class BSRoformer(NativeModule):
    """Reference-compatible BS-Roformer module (torch.nn.Module) backed by the native HIP forward."""
    # round 6: two forwards in flight differed from one stream in 500-4600 of the 4-min track's 21 M samples until the
    # iSTFT's FFT stage barrier waited for the wave's own LDS writes (sesa_sync); now 0 differing
    # (tools/streams_check.py, profiles/r06_sync_ab.txt), so the NativeModule default (multi-stream) holds


    _prefix = "bsr"
    # fp16: the QKV / FF Linears on one fp16 MFMA pass (include/sesa.h SESA_PREC_F16; 7e-6 emulated on the
    # full vocals chunk); the band split, attention, out-projection and mask MLPs stay bf16x3
    _precisions = ("bf16x3", "bf16", "fp16")
    _amp_precision = "fp16"  # --enable_amp (the reference's AMP is fp16 autocast)
    _prec_codes = {"bf16x3": N.SESA_PREC_BF16X3, "bf16": N.SESA_PREC_BF16, "fp16": N.SESA_PREC_F16}

    def __init__(self, dim, *, depth, stereo=False, num_stems=1, time_transformer_depth=2, freq_transformer_depth=2,
                 linear_transformer_depth=0, freqs_per_bands=DEFAULT_FREQS_PER_BANDS, dim_head=64, heads=8,
                 attn_dropout=0.0, ff_dropout=0.0, flash_attn=True, dim_freqs_in=1025, stft_n_fft=2048,
                 stft_hop_length=512, stft_win_length=2048, stft_normalized=False, stft_window_fn=None,
                 mask_estimator_depth=2, multi_stft_resolution_loss_weight=1.0,
                 multi_stft_resolutions_window_sizes=(4096, 2048, 1024, 512, 256), multi_stft_hop_size=147,
                 multi_stft_normalized=False, multi_stft_window_fn=None, mlp_expansion_factor=4,
                 use_torch_checkpoint=False, skip_connection=False, chunk_size=None, precision="bf16x3"):
        super().__init__(precision)
        if linear_transformer_depth or skip_connection or stft_normalized or stft_window_fn is not None:
            raise N.SesaError("BSRoformer: linear attention, skip connections, normalized or custom STFT windows "
                              "have no native implementation")
        self.stereo = bool(stereo)
        self.audio_channels = 2 if stereo else 1
        self.num_stems = int(num_stems)
        self.freqs_per_bands = tuple(int(f) for f in freqs_per_bands)
        if sum(self.freqs_per_bands) != stft_n_fft // 2 + 1:
            raise AssertionError(f"the number of freqs in the bands must equal {stft_n_fft // 2 + 1} based on the "
                                 f"STFT settings, but got {sum(self.freqs_per_bands)}")
        self.chunk_size = chunk_size
        self._kw = dict(audio_channels=self.audio_channels, n_fft=int(stft_n_fft), hop_length=int(stft_hop_length),
                        win_length=int(stft_win_length), dim=int(dim), depth=int(depth), heads=int(heads),
                        dim_head=int(dim_head), time_transformer_depth=int(time_transformer_depth),
                        freq_transformer_depth=int(freq_transformer_depth), num_stems=self.num_stems,
                        mask_estimator_depth=int(mask_estimator_depth),
                        mlp_expansion_factor=int(mlp_expansion_factor))
        self._register_params(self._shapes(), self._init_value)

    def _init_value(self, name, shape):
        if name.endswith("rotary_embed.freqs"):
            return torch.from_numpy(_freqs(self._kw["dim_head"]))
        if name.endswith("gamma"):
            return torch.ones(shape)
        return torch.zeros(shape)

    # ---- parameter registry (reference state_dict order, bs_roformer.py:372-433) ----
    def band_dims(self):
        return [2 * f * self.audio_channels for f in self.freqs_per_bands]

    def _shapes(self):
        k = self._kw
        dim, heads, dh = k["dim"], k["heads"], k["dim_head"]
        inner, ff, hid = heads * dh, dim * 4, dim * k["mlp_expansion_factor"]
        out = []
        for i in range(k["depth"]):
            for j, dep in ((0, k["time_transformer_depth"]), (1, k["freq_transformer_depth"])):
                for l in range(dep):
                    p = f"layers.{i}.{j}.layers.{l}"
                    out += [(f"{p}.0.rotary_embed.freqs", (dh // 2,)), (f"{p}.0.norm.gamma", (dim,)),
                            (f"{p}.0.to_qkv.weight", (3 * inner, dim)), (f"{p}.0.to_gates.weight", (heads, dim)),
                            (f"{p}.0.to_gates.bias", (heads,)), (f"{p}.0.to_out.0.weight", (dim, inner)),
                            (f"{p}.1.net.0.gamma", (dim,)), (f"{p}.1.net.1.weight", (ff, dim)),
                            (f"{p}.1.net.1.bias", (ff,)), (f"{p}.1.net.4.weight", (dim, ff)),
                            (f"{p}.1.net.4.bias", (dim,))]
        out.append(("final_norm.gamma", (dim,)))
        dims = self.band_dims()
        for b, d in enumerate(dims):
            out += [(f"band_split.to_features.{b}.0.gamma", (d,)), (f"band_split.to_features.{b}.1.weight", (dim, d)),
                    (f"band_split.to_features.{b}.1.bias", (dim,))]
        for n in range(self.num_stems):
            for b, d in enumerate(dims):
                p = f"mask_estimators.{n}.to_freqs.{b}.0"
                out += [(f"{p}.0.weight", (hid, dim)), (f"{p}.0.bias", (hid,)), (f"{p}.2.weight", (2 * d, hid)),
                        (f"{p}.2.bias", (2 * d,))]
        return out

    # ---- native handles ----
    _mel = False
    _freq_indices = ()

    def _config(self, chunk):
        fpb = (ctypes.c_int * len(self.freqs_per_bands))(*self.freqs_per_bands)
        fidx = (ctypes.c_int * max(1, len(self._freq_indices)))(*self._freq_indices)
        c = N.SesaBsrConfig(chunk_size=int(chunk), n_bands=len(self.freqs_per_bands), freqs_per_bands=fpb,
                            precision=self._prec_codes[self.precision],
                            mel=1 if self._mel else 0, n_freq_indices=len(self._freq_indices), freq_indices=fidx,
                            **self._kw)
        self._keep = (fpb, fidx)   # ctypes arrays must outlive the create call
        return c

    def _out_shape(self, B, ch, C):
        return (B, self.num_stems, ch, C)

    def _post(self, out):
        return out[:, 0] if self.num_stems == 1 else out

    @torch.no_grad()
    def forward(self, raw_audio, target=None):
        if target is not None:
            raise N.SesaError("BSRoformer: the training loss branch is not part of the native inference path")
        if not isinstance(raw_audio, torch.Tensor) or not raw_audio.is_cuda:
            raise N.SesaError(f"{type(self).__name__}.forward: input must be a HIP device tensor (no CPU fallback)")
        x = raw_audio
        if x.ndim == 2:
            x = x[:, None]
        if x.shape[1] != self.audio_channels:
            raise AssertionError("stereo needs to be set to True if passing in audio signal that is stereo")
        return super().forward(x)
