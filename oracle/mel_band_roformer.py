"""Functional PyTorch-CPU fp32 restatement of Mel-Band-Roformer.  TEST INFRASTRUCTURE.

Restates ``/root/reference/models/bs_roformer/mel_band_roformer.py`` (inference branch):

* band layout (:400-445) -- librosa Slaney mel filterbank (restated in oracle/_stubs/librosa),
  entries [0][0] and [-1][-1] forced to 1, bands = support (> 0), overlapping; ``freq_indices``
  gathers the (f, s) rows of every band in ascending order; ``num_bands_per_freq`` averages.
* ``Transformer`` (:187-228) ends with RMSNorm (norm_output=True); no final_norm.
* ``MLP`` (:261-283) has ``depth + 1`` Linear layers (Tanh between).
* ``forward`` (:480-620): STFT, gather, band split, depth x (time, freq) transformers, mask
  estimators, scatter_add of the masks over the gathered frequencies / num_bands_per_freq,
  complex multiply, iSTFT(length = input length if match_input_audio_length else default).
Shares RMSNorm / Attention / FeedForward / rotary with oracle/bs_roformer.py (identical code in
the reference: bs_roformer.py:43-121 == mel_band_roformer.py:52-130).
"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

from . import bs_roformer as ob

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "_stubs"))
from librosa import filters  # noqa: E402  (restated)
from rotary_embedding_torch import inv_freqs  # noqa: E402

load_cfg = ob.load_cfg


def model_kwargs(cfg):
    m = dict(cfg["model"])
    d = dict(stereo=False, num_stems=1, time_transformer_depth=2, freq_transformer_depth=2,
             linear_transformer_depth=0, num_bands=60, dim_head=64, heads=8, sample_rate=44100, stft_n_fft=2048,
             stft_hop_length=512, stft_win_length=2048, stft_normalized=False, mask_estimator_depth=1,
             match_input_audio_length=False, mlp_expansion_factor=4, skip_connection=False)
    d.update(m)
    return d


def bands(k):
    """(freqs_per_band bool [nb, F], freq_indices (f s) int64, num_bands_per_freq [F])."""
    fb = torch.from_numpy(filters.mel(sr=k["sample_rate"], n_fft=k["stft_n_fft"], n_mels=k["num_bands"]))
    fb[0][0] = 1.0
    fb[-1, -1] = 1.0
    fpb = fb > 0
    assert fpb.any(dim=0).all()
    nfreq = fpb.shape[1]
    idx = torch.arange(nfreq).repeat(k["num_bands"], 1)[fpb]
    if k["stereo"]:
        idx = (idx[:, None] * 2 + torch.arange(2)).reshape(-1)
    return fpb, idx, fpb.sum(dim=0)


def band_dims(k):
    ch = 2 if k["stereo"] else 1
    fpb, _, _ = bands(k)
    return [2 * int(n) * ch for n in fpb.sum(dim=1).tolist()]


def param_names(cfg):
    k = model_kwargs(cfg)
    dim, heads, dh = k["dim"], k["heads"], k["dim_head"]
    inner, ff = heads * dh, dim * 4
    out = []
    for i in range(k["depth"]):
        for j, dep in ((0, k["time_transformer_depth"]), (1, k["freq_transformer_depth"])):
            for l in range(dep):
                p = f"layers.{i}.{j}.layers.{l}"
                out += [(f"{p}.0.rotary_embed.freqs", (dh // 2,)), (f"{p}.0.norm.gamma", (dim,)),
                        (f"{p}.0.to_qkv.weight", (3 * inner, dim)), (f"{p}.0.to_gates.weight", (heads, dim)),
                        (f"{p}.0.to_gates.bias", (heads,)), (f"{p}.0.to_out.0.weight", (dim, inner)),
                        (f"{p}.1.net.0.gamma", (dim,)), (f"{p}.1.net.1.weight", (ff, dim)),
                        (f"{p}.1.net.1.bias", (ff,)), (f"{p}.1.net.4.weight", (dim, ff)), (f"{p}.1.net.4.bias", (dim,))]
            out.append((f"layers.{i}.{j}.norm.gamma", (dim,)))
    dims = band_dims(k)
    for b, din in enumerate(dims):
        out += [(f"band_split.to_features.{b}.0.gamma", (din,)), (f"band_split.to_features.{b}.1.weight", (dim, din)),
                (f"band_split.to_features.{b}.1.bias", (dim,))]
    hid = dim * k["mlp_expansion_factor"]
    nl = k["mask_estimator_depth"] + 1
    for n in range(k["num_stems"]):
        for b, din in enumerate(dims):
            p = f"mask_estimators.{n}.to_freqs.{b}.0"
            ins = [dim] + [hid] * (nl - 1)
            outs = [hid] * (nl - 1) + [2 * din]
            for li in range(nl):
                out += [(f"{p}.{2 * li}.weight", (outs[li], ins[li])), (f"{p}.{2 * li}.bias", (outs[li],))]
    return out


def synth_params(cfg, affine="random"):
    from .weights import param_rng, synth_param
    import math
    k = model_kwargs(cfg)
    names = param_names(cfg)
    shapes = dict(names)
    out = {}
    for name, shape in names:
        if name.endswith("rotary_embed.freqs"):
            out[name] = inv_freqs(k["dim_head"]).numpy().astype(np.float32)
        elif name.endswith(".bias") and affine == "random":
            b = 1.0 / math.sqrt(shapes[name[:-5] + ".weight"][1])
            out[name] = param_rng(name).uniform(-b, b, size=shape).astype(np.float32)
        elif name.endswith(".bias"):
            out[name] = np.zeros(shape, np.float32)
        else:
            out[name] = synth_param(name, shape, affine)
    return out


def transformer(P, prefix, depth, x, heads):
    x = ob.transformer(P, prefix, depth, x, heads)
    return ob.rmsnorm(x, P[f"{prefix}.norm.gamma"])


def forward(P, cfg, raw_audio):
    k = model_kwargs(cfg)
    heads = k["heads"]
    if raw_audio.ndim == 2:
        raw_audio = raw_audio[:, None]
    b, s, t = raw_audio.shape
    win = torch.hann_window(k["stft_win_length"])
    skw = dict(n_fft=k["stft_n_fft"], hop_length=k["stft_hop_length"], win_length=k["stft_win_length"],
               normalized=k["stft_normalized"])
    spec = torch.view_as_real(torch.stft(raw_audio.reshape(b * s, t), **skw, window=win, return_complex=True))
    f_bins, T = spec.shape[1], spec.shape[2]
    spec = spec.reshape(b, s, f_bins, T, 2).permute(0, 2, 1, 3, 4).reshape(b, f_bins * s, T, 2)  # b (f s) t c
    fpb, idx, nbpf = bands(k)
    x = spec[:, idx]                                                   # b f' t c
    x = x.permute(0, 2, 1, 3).reshape(b, T, -1)                        # b t (f' c)
    dims = band_dims(k)
    feats, off = [], 0
    for j, din in enumerate(dims):
        pj = f"band_split.to_features.{j}"
        feats.append(ob.rmsnorm(x[..., off:off + din], P[f"{pj}.0.gamma"]) @ P[f"{pj}.1.weight"].T + P[f"{pj}.1.bias"])
        off += din
    x = torch.stack(feats, dim=-2)
    nb = x.shape[2]
    for i in range(k["depth"]):
        x = x.permute(0, 2, 1, 3).reshape(b * nb, T, -1)
        x = transformer(P, f"layers.{i}.0", k["time_transformer_depth"], x, heads)
        x = x.reshape(b, nb, T, -1).permute(0, 2, 1, 3).reshape(b * T, nb, -1)
        x = transformer(P, f"layers.{i}.1", k["freq_transformer_depth"], x, heads)
        x = x.reshape(b, T, nb, -1)
    nl = k["mask_estimator_depth"] + 1
    masks = []
    for n in range(k["num_stems"]):
        outs = []
        for j, din in enumerate(dims):
            p = f"mask_estimators.{n}.to_freqs.{j}.0"
            h = x[:, :, j]
            for li in range(nl):
                h = h @ P[f"{p}.{2 * li}.weight"].T + P[f"{p}.{2 * li}.bias"]
                if li < nl - 1:
                    h = torch.tanh(h)
            outs.append(F.glu(h, dim=-1))
        masks.append(torch.cat(outs, dim=-1))
    masks = torch.stack(masks, dim=1)                                   # b n t (f' c)
    ns = k["num_stems"]
    masks = masks.reshape(b, ns, T, -1, 2).permute(0, 1, 3, 2, 4)      # b n f' t c
    sr = torch.view_as_complex(spec.contiguous()).unsqueeze(1)         # b 1 (f s) t
    m = torch.view_as_complex(masks.contiguous())
    scatter_idx = idx.view(1, 1, -1, 1).expand(b, ns, -1, T)
    summed = torch.zeros(b, ns, sr.shape[2], T, dtype=sr.dtype).scatter_add_(2, scatter_idx, m)
    denom = nbpf.repeat_interleave(s).view(-1, 1)
    sr = sr * (summed / denom.clamp(min=1e-8))
    sr = sr.reshape(b, ns, f_bins, s, T).permute(0, 1, 3, 2, 4).reshape(b * ns * s, f_bins, T)
    length = t if k["match_input_audio_length"] else None
    recon = torch.istft(sr, **skw, window=win, return_complex=False, length=length)
    recon = recon.reshape(b, ns, s, -1)
    return recon[:, 0] if ns == 1 else recon


class OracleModel:
    def __init__(self, cfg, params):
        self.cfg = cfg
        self.P = ob.to_torch(params)

    def __call__(self, x):
        with torch.inference_mode():
            return forward(self.P, self.cfg, torch.as_tensor(x))
