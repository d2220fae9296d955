"""Mel-Band-Roformer on the native MI355X forward (libsesa ``sesa_bsr_*`` with ``mel = 1``).

Drop-in for ``models/bs_roformer/mel_band_roformer.py:324-620`` (``MelBandRoformer``): built from
``**config.model`` (``utils.py:101-103``), same state_dict keys / shapes, same call
``model(x[B, ch, C]) -> [B, ch, C]`` (one stem) or ``[B, stems, ch, C]``.  The band layout is the
reference's: the librosa Slaney mel filterbank (restated below with numpy -- librosa is absent),
entries [0][0] and [-1][-1] forced to 1, bands = its support, overlapping; the masks of
frequencies shared by several bands are averaged (:596-606).  Everything else -- STFT, gather,
band split, rotary transformers with output RMSNorm, (depth+1)-layer mask MLPs, scatter-average,
complex mask, iSTFT -- runs in libsesa (sesa_bsroformer.hip).
"""
import numpy as np
import torch

from .. import _native as N
from .bs_roformer import BSRoformer
from .native import NativeModule


def _hz_to_mel(f):
    f = np.asanyarray(f, dtype=np.float64)
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, np.log(6.4) / 27.0
    m = f / f_sp
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-30) / min_log_hz) / logstep, m)


def _mel_to_hz(m):
    m = np.asanyarray(m, dtype=np.float64)
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, np.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), f_sp * m)


def mel_filter_bank(sr, n_fft, n_mels):
    """librosa.filters.mel(sr=sr, n_fft=n_fft, n_mels=n_mels) (Slaney scale and norm, float32)."""
    w = np.zeros((n_mels, 1 + n_fft // 2), dtype=np.float32)
    fftfreqs = np.fft.rfftfreq(n=n_fft, d=1.0 / sr)
    mel_f = _mel_to_hz(np.linspace(_hz_to_mel(0.0), _hz_to_mel(sr / 2.0), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = np.subtract.outer(mel_f, fftfreqs)
    for i in range(n_mels):
        w[i] = np.maximum(0, np.minimum(-ramps[i] / fdiff[i], ramps[i + 2] / fdiff[i + 1]))
    w *= (2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels]))[:, None]
    return w


def mel_bands(sample_rate, n_fft, num_bands, stereo):
    """(num_freqs_per_band, freq_indices over (f s)) -- mel_band_roformer.py:400-441."""
    fb = mel_filter_bank(sample_rate, n_fft, num_bands)
    fb[0][0] = 1.0
    fb[-1, -1] = 1.0
    fpb = fb > 0
    if not fpb.any(axis=0).all():
        raise AssertionError("all frequencies need to be covered by all bands for now")
    idx = np.tile(np.arange(fpb.shape[1]), (num_bands, 1))[fpb]
    if stereo:
        idx = (idx[:, None] * 2 + np.arange(2)).reshape(-1)
    return tuple(int(n) for n in fpb.sum(axis=1)), tuple(int(i) for i in idx)


class MelBandRoformer(BSRoformer):
    _mel = True

    def __init__(self, dim, *, depth, stereo=False, num_stems=1, time_transformer_depth=2, freq_transformer_depth=2,
                 linear_transformer_depth=0, num_bands=60, dim_head=64, heads=8, attn_dropout=0.1, ff_dropout=0.1,
                 flash_attn=True, dim_freqs_in=1025, sample_rate=44100, stft_n_fft=2048, stft_hop_length=512,
                 stft_win_length=2048, stft_normalized=False, stft_window_fn=None, mask_estimator_depth=1,
                 multi_stft_resolution_loss_weight=1.0,
                 multi_stft_resolutions_window_sizes=(4096, 2048, 1024, 512, 256), multi_stft_hop_size=147,
                 multi_stft_normalized=False, multi_stft_window_fn=None, match_input_audio_length=False,
                 mlp_expansion_factor=4, use_torch_checkpoint=False, skip_connection=False, precision="bf16x3"):
        NativeModule.__init__(self, precision)
        if linear_transformer_depth or skip_connection or stft_normalized or stft_window_fn is not None:
            raise N.SesaError("MelBandRoformer: linear attention, skip connections, normalized or custom STFT "
                              "windows have no native implementation")
        fpb, idx = mel_bands(sample_rate, stft_n_fft, num_bands, stereo)
        self._freq_indices = idx
        self.match_input_audio_length = match_input_audio_length
        self.stereo = bool(stereo)
        self.audio_channels = 2 if stereo else 1
        self.num_stems = int(num_stems)
        self.freqs_per_bands = fpb
        self.chunk_size = None
        self._kw = dict(audio_channels=self.audio_channels, n_fft=int(stft_n_fft), hop_length=int(stft_hop_length),
                        win_length=int(stft_win_length), dim=int(dim), depth=int(depth), heads=int(heads),
                        dim_head=int(dim_head), time_transformer_depth=int(time_transformer_depth),
                        freq_transformer_depth=int(freq_transformer_depth), num_stems=self.num_stems,
                        mask_estimator_depth=int(mask_estimator_depth),
                        mlp_expansion_factor=int(mlp_expansion_factor))
        self._register_params(self._shapes(), self._init_value)
        self.register_buffer("freq_indices", torch.tensor(idx), persistent=False)

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
                out.append((f"layers.{i}.{j}.norm.gamma", (dim,)))
        dims = self.band_dims()
        for b, d in enumerate(dims):
            out += [(f"band_split.to_features.{b}.0.gamma", (d,)), (f"band_split.to_features.{b}.1.weight", (dim, d)),
                    (f"band_split.to_features.{b}.1.bias", (dim,))]
        nl = k["mask_estimator_depth"] + 1
        for n in range(self.num_stems):
            for b, d in enumerate(dims):
                p = f"mask_estimators.{n}.to_freqs.{b}.0"
                ins = [dim] + [hid] * (nl - 1)
                outs = [hid] * (nl - 1) + [2 * d]
                for li in range(nl):
                    out += [(f"{p}.{2 * li}.weight", (outs[li], ins[li])), (f"{p}.{2 * li}.bias", (outs[li],))]
        return out
