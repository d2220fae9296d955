"""Functional PyTorch-CPU fp32 restatement of BS-Roformer.  TEST INFRASTRUCTURE.

Restates ``/root/reference/models/bs_roformer/bs_roformer.py`` (inference branch):

* ``RMSNorm`` (:43-50)           -- ``F.normalize(x, dim=-1) * sqrt(dim) * gamma``
* ``FeedForward`` (:55-74)       -- RMSNorm, Linear(+b), GELU, Linear(+b)
* ``Attention`` (:77-121)        -- RMSNorm, to_qkv (no bias), rotary q/k, SDPA (scale d^-1/2),
                                    sigmoid(to_gates(x)) per head, to_out (no bias)
* ``Transformer`` (:178-217)     -- x = attn(x) + x; x = ff(x) + x  (norm_output=False)
* ``BandSplit`` (:222-249)       -- per band RMSNorm + Linear(+b), stacked on dim -2
* ``MaskEstimator`` (:277-310)   -- per band MLP(dim -> hidden, Tanh, -> 2*dim_in) + GLU
* ``BSRoformer.forward`` (:447-587) -- STFT, band split, depth x (time, freq) transformers,
                                    final norm, mask, complex multiply, iSTFT(length=...)
* ``param_names`` -- the reference ``state_dict()`` keys / shapes (rotary ``freqs`` per layer,
  as stored in released checkpoints).

The rotary embedding is the restatement in ``oracle/_stubs/rotary_embedding_torch`` (third-party,
unpinned: parity at that boundary is unpinned).  ``params`` maps state_dict names to fp32 tensors.
"""
import math
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "_stubs"))
from rotary_embedding_torch import angles, apply_rotary_emb, inv_freqs  # noqa: E402

DEFAULT_FREQS_PER_BANDS = (2,) * 24 + (4,) * 12 + (12,) * 8 + (24,) * 8 + (48,) * 8 + (128, 129)


def load_cfg(path):
    """YAML with the !!python/tuple tag of the released configs (SafeLoader otherwise)."""
    import yaml

    class _L(yaml.SafeLoader):
        pass

    _L.add_constructor("tag:yaml.org,2002:python/tuple", lambda ld, node: tuple(ld.construct_sequence(node)))
    with open(path) as f:
        return yaml.load(f, Loader=_L)


def model_kwargs(cfg):
    """BSRoformer(**config.model) with the constructor defaults (bs_roformer.py:329-363)."""
    m = dict(cfg["model"])
    d = dict(stereo=False, num_stems=1, time_transformer_depth=2, freq_transformer_depth=2,
             linear_transformer_depth=0, freqs_per_bands=DEFAULT_FREQS_PER_BANDS, dim_head=64, heads=8,
             stft_n_fft=2048, stft_hop_length=512, stft_win_length=2048, stft_normalized=False,
             mask_estimator_depth=2, mlp_expansion_factor=4, skip_connection=False)
    d.update(m)
    d["freqs_per_bands"] = tuple(int(f) for f in d["freqs_per_bands"])
    return d


def band_dims(k):
    ch = 2 if k["stereo"] else 1
    return [2 * f * ch for f in k["freqs_per_bands"]]


def param_names(cfg):
    """(name, shape) of the reference state_dict, in registration order."""
    k = model_kwargs(cfg)
    dim, heads, dh = k["dim"], k["heads"], k["dim_head"]
    inner = heads * dh
    ff = dim * 4
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
    out.append(("final_norm.gamma", (dim,)))
    dims = band_dims(k)
    for b, din in enumerate(dims):
        out += [(f"band_split.to_features.{b}.0.gamma", (din,)), (f"band_split.to_features.{b}.1.weight", (dim, din)),
                (f"band_split.to_features.{b}.1.bias", (dim,))]
    hid = dim * k["mlp_expansion_factor"]
    if k["mask_estimator_depth"] != 2:
        raise NotImplementedError("oracle: mask_estimator_depth 2 only (the released configs)")
    for n in range(k["num_stems"]):
        for b, din in enumerate(dims):
            p = f"mask_estimators.{n}.to_freqs.{b}.0"
            out += [(f"{p}.0.weight", (hid, dim)), (f"{p}.0.bias", (hid,)), (f"{p}.2.weight", (2 * din, hid)),
                    (f"{p}.2.bias", (2 * din,))]
    return out


def synth_params(cfg, affine="random", seed=0):
    """Name-keyed synthetic weights (oracle/weights.py scheme); rotary freqs are the real ones;
    Linear biases U(+-1/sqrt(fan_in)) of their weight (affine='random') or 0; gammas U(0.5,1.5) or 1."""
    from .weights import param_rng, synth_param
    k = model_kwargs(cfg)
    names = param_names(cfg)
    shapes = dict(names)
    out = {}
    for name, shape in names:
        if name.endswith("rotary_embed.freqs"):
            out[name] = inv_freqs(k["dim_head"]).numpy().astype(np.float32)
        elif name.endswith(".bias") and (name[:-5] + ".weight") in shapes and affine == "random":
            fan_in = shapes[name[:-5] + ".weight"][1]
            b = 1.0 / math.sqrt(fan_in)
            out[name] = param_rng(name, seed).uniform(-b, b, size=shape).astype(np.float32)
        elif name.endswith(".bias"):
            out[name] = np.zeros(shape, np.float32)
        else:
            out[name] = synth_param(name, shape, affine, seed)
    return out


def to_torch(params):
    return {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in params.items()}


def rmsnorm(x, gamma):
    return F.normalize(x, dim=-1) * (x.shape[-1] ** 0.5) * gamma


def attention(P, p, x, freqs, heads):
    b, n, _ = x.shape
    x = rmsnorm(x, P[f"{p}.norm.gamma"])
    qkv = x @ P[f"{p}.to_qkv.weight"].T
    q, k, v = qkv.reshape(b, n, 3, heads, -1).permute(2, 0, 3, 1, 4)  # 'b n (qkv h d) -> qkv b h n d'
    ang = angles(freqs, n)
    q = apply_rotary_emb(ang, q)
    k = apply_rotary_emb(ang, k)
    out = F.scaled_dot_product_attention(q, k, v)
    gates = x @ P[f"{p}.to_gates.weight"].T + P[f"{p}.to_gates.bias"]
    out = out * gates.permute(0, 2, 1).unsqueeze(-1).sigmoid()
    out = out.permute(0, 2, 1, 3).reshape(b, n, -1)
    return out @ P[f"{p}.to_out.0.weight"].T


def feedforward(P, p, x):
    x = rmsnorm(x, P[f"{p}.net.0.gamma"])
    x = F.gelu(x @ P[f"{p}.net.1.weight"].T + P[f"{p}.net.1.bias"])
    return x @ P[f"{p}.net.4.weight"].T + P[f"{p}.net.4.bias"]


def transformer(P, prefix, depth, x, heads):
    for l in range(depth):
        p = f"{prefix}.layers.{l}"
        x = attention(P, f"{p}.0", x, P[f"{p}.0.rotary_embed.freqs"], heads) + x
        x = feedforward(P, f"{p}.1", x) + x
    return x


def stft_window(k):
    return torch.hann_window(k["stft_win_length"])


def forward(P, cfg, raw_audio):
    """BSRoformer.forward (bs_roformer.py:447-587), inference branch.  raw_audio [b, s, t]."""
    k = model_kwargs(cfg)
    heads = k["heads"]
    if raw_audio.ndim == 2:
        raw_audio = raw_audio[:, None]
    b, s, t = raw_audio.shape
    win = stft_window(k)
    skw = dict(n_fft=k["stft_n_fft"], hop_length=k["stft_hop_length"], win_length=k["stft_win_length"],
               normalized=k["stft_normalized"])
    spec = torch.stft(raw_audio.reshape(b * s, t), **skw, window=win, return_complex=True)
    spec = torch.view_as_real(spec)                                   # [b*s, f, T, 2]
    f_bins, T = spec.shape[1], spec.shape[2]
    spec = spec.reshape(b, s, f_bins, T, 2).permute(0, 2, 1, 3, 4).reshape(b, f_bins * s, T, 2)  # b (f s) t c
    x = spec.permute(0, 2, 1, 3).reshape(b, T, -1)                   # b t (f c)
    dims = band_dims(k)
    feats, off = [], 0
    for j, din in enumerate(dims):
        xb = x[..., off:off + din]
        off += din
        pj = f"band_split.to_features.{j}"
        feats.append(rmsnorm(xb, P[f"{pj}.0.gamma"]) @ P[f"{pj}.1.weight"].T + P[f"{pj}.1.bias"])
    x = torch.stack(feats, dim=-2)                                    # [b, T, F, d]
    nb = x.shape[2]
    for i in range(k["depth"]):
        x = x.permute(0, 2, 1, 3).reshape(b * nb, T, -1)             # b t f d -> (b f) t d
        x = transformer(P, f"layers.{i}.0", k["time_transformer_depth"], x, heads)
        x = x.reshape(b, nb, T, -1).permute(0, 2, 1, 3).reshape(b * T, nb, -1)  # -> (b t) f d
        x = transformer(P, f"layers.{i}.1", k["freq_transformer_depth"], x, heads)
        x = x.reshape(b, T, nb, -1)
    x = rmsnorm(x, P["final_norm.gamma"])
    masks = []
    for n in range(k["num_stems"]):
        outs = []
        for j, din in enumerate(dims):
            p = f"mask_estimators.{n}.to_freqs.{j}.0"
            h = torch.tanh(x[:, :, j] @ P[f"{p}.0.weight"].T + P[f"{p}.0.bias"])
            y = h @ P[f"{p}.2.weight"].T + P[f"{p}.2.bias"]
            outs.append(F.glu(y, dim=-1))
        masks.append(torch.cat(outs, dim=-1))
    mask = torch.stack(masks, dim=1)                                  # b n t (f c)
    mask = mask.reshape(b, k["num_stems"], T, -1, 2).permute(0, 1, 3, 2, 4)  # b n f t c
    sr = torch.view_as_complex(spec.unsqueeze(1).contiguous())        # b 1 f t
    m = torch.view_as_complex(mask.contiguous())
    sr = sr * m
    sr = sr.reshape(b, k["num_stems"], f_bins, s, T).permute(0, 1, 3, 2, 4).reshape(b * k["num_stems"] * s, f_bins, T)
    recon = torch.istft(sr, **skw, window=win, return_complex=False, length=t)
    recon = recon.reshape(b, k["num_stems"], s, t)
    return recon[:, 0] if k["num_stems"] == 1 else recon


class OracleModel:
    """Callable [B,2,C] -> [B,2,C] (1 stem) for oracle/demix.py."""

    def __init__(self, cfg, params):
        self.cfg = cfg
        self.P = to_torch(params)

    def __call__(self, x):
        with torch.inference_mode():
            return forward(self.P, self.cfg, torch.as_tensor(x))
