"""HTDemucs restatement on the restated demucs layers.  TEST INFRASTRUCTURE.

Restates ``/root/reference/models/demucs4ht.py`` (HTDemucs, cac configurations) as functions over a
module tree built from ``oracle/_stubs/demucs`` (the restatement of the third-party ``demucs``
layers, UNPINNED -- see that package's docstring):

* ``build`` -- the layer geometry of ``HTDemucs.__init__`` (:247-420): per depth index the freq /
  time encoder (HEncLayer), decoder (HDecLayer, inserted in reverse), the ``last_freq`` merge rule,
  the frequency embedding after layer 0, the bottom 1x1 channel resamplers and the
  CrossTransformerEncoder; module names equal the reference ``state_dict`` keys.
* ``forward`` -- ``HTDemucs.forward`` (:548-693) for ``use_train_segment=False``, ``cac=True``:
  ``_spec`` (:427-446: reflect pad 3*hop/2 each side + to a multiple of hop, normalized Hann STFT,
  drop the Nyquist bin, crop 2 frames each side), ``_magnitude`` (complex as channels, :459-468),
  mean / std normalisation of both branches, encoder with time -> frequency injection, transformer,
  decoder with the branch split, ``_mask`` (:470-481) and ``_ispec`` (:448-457), sum of branches.

Pinned by tests/golden/make_golden_htdemucs.py, which runs the reference class itself on the same
restated layers: this file is checked against the reference's HTDemucs-level code; the layer
boundary stays unpinned (no demucs package, no reference fixture).
"""
import math

import numpy as np
import torch
import torch.nn.functional as F
import yaml
from einops import rearrange
from torch import nn


def load_cfg(path):
    with open(path) as f:
        return yaml.safe_load(f)


def _kw(cfg):
    k = dict(cfg["htdemucs"])
    k.update(sources=list(cfg["training"]["instruments"]), audio_channels=int(cfg["training"]["channels"]))
    if not k.get("cac", True) or k.get("num_subbands", 1) != 1 or k.get("multi_freqs"):
        raise NotImplementedError("oracle restates the cac, single-band, no-multi_freqs HTDemucs only")
    return k


def build(cfg):
    """Module tree with the reference's names (demucs4ht.py:247-420), weights uninitialised."""
    import sys
    import os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "_stubs"))
    from demucs.hdemucs import HDecLayer, HEncLayer, ScaledEmbedding
    from demucs.transformer import CrossTransformerEncoder
    k = _kw(cfg)
    root = nn.Module()
    root.encoder, root.decoder, root.tencoder, root.tdecoder = (nn.ModuleList() for _ in range(4))
    ach, nsrc = k["audio_channels"], len(k["sources"])
    chin, chin_z = ach, 2 * ach
    chout = k.get("channels_time") or k["channels"]
    chout_z = k["channels"]
    freqs = k["nfft"] // 2
    dkw = {"depth": k["dconv_depth"], "compress": k["dconv_comp"], "init": k["dconv_init"], "gelu": True}
    for index in range(k["depth"]):
        freq = freqs > 1
        ker, stri = k["kernel_size"], k["stride"]
        if not freq:
            ker, stri = k["time_stride"] * 2, k["time_stride"]
        pad, last_freq = True, False
        if freq and freqs <= k["kernel_size"]:
            ker, pad, last_freq = freqs, False, True
        kw = dict(kernel_size=ker, stride=stri, freq=freq, pad=pad, norm=index >= k["norm_starts"],
                  rewrite=k["rewrite"], norm_groups=k["norm_groups"], dconv_kw=dkw)
        kwt = dict(kw, freq=0, kernel_size=k["kernel_size"], stride=k["stride"], pad=True)
        if last_freq:
            chout_z = max(chout, chout_z)
            chout = chout_z
        root.encoder.append(HEncLayer(chin_z, chout_z, dconv=k["dconv_mode"] & 1, context=k["context_enc"], **kw))
        if freq:
            root.tencoder.append(HEncLayer(chin, chout, dconv=k["dconv_mode"] & 1, context=k["context_enc"],
                                           empty=last_freq, **kwt))
        if index == 0:
            chin = ach * nsrc
            chin_z = 2 * chin
        root.decoder.insert(0, HDecLayer(chout_z, chin_z, dconv=k["dconv_mode"] & 2, last=index == 0,
                                         context=k["context"], **kw))
        if freq:
            root.tdecoder.insert(0, HDecLayer(chout, chin, dconv=k["dconv_mode"] & 2, empty=last_freq,
                                              last=index == 0, context=k["context"], **kwt))
        chin, chin_z = chout, chout_z
        chout, chout_z = int(k["growth"] * chout), int(k["growth"] * chout_z)
        if freq:
            freqs = 1 if freqs <= k["kernel_size"] else freqs // k["stride"]
        if index == 0 and k["freq_emb"]:
            root.freq_emb = ScaledEmbedding(freqs, chin_z, smooth=k["emb_smooth"], scale=k["emb_scale"])
    tc = k["channels"] * k["growth"] ** (k["depth"] - 1)
    if k["bottom_channels"]:
        b = k["bottom_channels"]
        root.channel_upsampler = nn.Conv1d(tc, b, 1)
        root.channel_downsampler = nn.Conv1d(b, tc, 1)
        root.channel_upsampler_t = nn.Conv1d(tc, b, 1)
        root.channel_downsampler_t = nn.Conv1d(b, tc, 1)
        tc = b
    if k["t_layers"] > 0:
        root.crosstransformer = CrossTransformerEncoder(
            dim=tc, emb=k["t_emb"], hidden_scale=k["t_hidden_scale"], num_heads=k["t_heads"], num_layers=k["t_layers"],
            cross_first=k["t_cross_first"], dropout=k["t_dropout"], max_positions=k["t_max_positions"],
            norm_in=k["t_norm_in"], norm_in_group=k["t_norm_in_group"], group_norm=k["t_group_norm"],
            norm_first=k["t_norm_first"], norm_out=k["t_norm_out"], max_period=k["t_max_period"],
            layer_scale=k["t_layer_scale"], gelu=k["t_gelu"], sin_random_shift=k["t_sin_random_shift"],
            weight_pos_embed=k["t_weight_pos_embed"], sparse_self_attn=k["t_sparse_self_attn"],
            sparse_cross_attn=k["t_sparse_cross_attn"])
    return root.eval()


def param_names(cfg):
    return [(n, tuple(t.shape)) for n, t in build(cfg).state_dict().items()]


def load(cfg, params):
    m = build(cfg)
    m.load_state_dict({n: torch.as_tensor(np.asarray(v)) for n, v in params.items()}, strict=True)
    return m


def _spec(x, nfft):
    """HTDemucs._spec (demucs4ht.py:427-446)."""
    from demucs.hdemucs import pad1d
    from demucs.spec import spectro
    hl = nfft // 4
    le = int(math.ceil(x.shape[-1] / hl))
    pad = hl // 2 * 3
    x = pad1d(x, (pad, pad + le * hl - x.shape[-1]), mode="reflect")
    z = spectro(x, nfft, hl)[..., :-1, :]
    return z[..., 2:2 + le]


def _ispec(z, nfft, length):
    """HTDemucs._ispec (demucs4ht.py:448-457), scale 0."""
    from demucs.spec import ispectro
    hl = nfft // 4
    z = F.pad(F.pad(z, (0, 0, 0, 1)), (2, 2))
    pad = hl // 2 * 3
    le = hl * int(math.ceil(length / hl)) + 2 * pad
    x = ispectro(z, hl, length=le)
    return x[..., pad:pad + length]


@torch.inference_mode()
def forward(m, cfg, mix):
    """HTDemucs.forward (demucs4ht.py:548-693): mix [B, ch, L] -> [B, sources, ch, L]."""
    k = _kw(cfg)
    length = mix.shape[-1]
    z = _spec(mix, k["nfft"])
    B, C, Fr, T = z.shape
    x = torch.view_as_real(z).permute(0, 1, 4, 2, 3).reshape(B, C * 2, Fr, T)   # _magnitude, cac
    mean = x.mean(dim=(1, 2, 3), keepdim=True)
    std = x.std(dim=(1, 2, 3), keepdim=True)
    x = (x - mean) / (1e-5 + std)
    xt = mix
    meant = xt.mean(dim=(1, 2), keepdim=True)
    stdt = xt.std(dim=(1, 2), keepdim=True)
    xt = (xt - meant) / (1e-5 + stdt)
    saved, saved_t, lengths, lengths_t = [], [], [], []
    for idx, encode in enumerate(m.encoder):
        lengths.append(x.shape[-1])
        inject = None
        if idx < len(m.tencoder):
            lengths_t.append(xt.shape[-1])
            tenc = m.tencoder[idx]
            xt = tenc(xt)
            if not tenc.empty:
                saved_t.append(xt)
            else:
                inject = xt
        x = encode(x, inject)
        if idx == 0 and hasattr(m, "freq_emb"):
            frs = torch.arange(x.shape[-2], device=x.device)
            x = x + k["freq_emb"] * m.freq_emb(frs).t()[None, :, :, None].expand_as(x)
        saved.append(x)
    if hasattr(m, "crosstransformer"):
        if k["bottom_channels"]:
            f = x.shape[2]
            x = rearrange(m.channel_upsampler(rearrange(x, "b c f t -> b c (f t)")), "b c (f t) -> b c f t", f=f)
            xt = m.channel_upsampler_t(xt)
        x, xt = m.crosstransformer(x, xt)
        if k["bottom_channels"]:
            x = rearrange(m.channel_downsampler(rearrange(x, "b c f t -> b c (f t)")), "b c (f t) -> b c f t", f=f)
            xt = m.channel_downsampler_t(xt)
    offset = k["depth"] - len(m.tdecoder)
    for idx, decode in enumerate(m.decoder):
        x, pre = decode(x, saved.pop(-1), lengths.pop(-1))
        if idx >= offset:
            tdec = m.tdecoder[idx - offset]
            length_t = lengths_t.pop(-1)
            if tdec.empty:
                xt, _ = tdec(pre[:, :, 0], None, length_t)
            else:
                xt, _ = tdec(xt, saved_t.pop(-1), length_t)
    S = len(k["sources"])
    x = x.view(B, S, -1, Fr, T) * std[:, None] + mean[:, None]
    zout = torch.view_as_complex(x.view(B, S, -1, 2, Fr, T).permute(0, 1, 2, 4, 5, 3).contiguous())   # _mask, cac
    x = _ispec(zout, k["nfft"], length)
    xt = xt.view(B, S, -1, length) * stdt[:, None] + meant[:, None]
    return xt + x
