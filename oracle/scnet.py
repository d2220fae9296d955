"""Functional PyTorch-CPU fp32 restatement of SCNet.  TEST INFRASTRUCTURE.

Restates ``/root/reference/models/scnet/scnet.py`` and ``separation.py`` (inference forward):

* ``SCNet.forward`` (scnet.py:325-373)   -- right zero-pad so the frame count is even, normalized
                                           rectangular-window STFT (n_fft 4096, center, reflect),
                                           encoder, separation net, decoder, iSTFT, crop
* ``SDlayer`` (:86-148)                  -- 3 frequency bands (ceil(F * SR) split points), each a
                                           Conv2d (k, 1) stride (s, 1) over F after zero padding
* ``ConvolutionModule`` (:15-52)         -- per (b, f) row over T: x += 1x1(Swish(GN(dw3(GLU(
                                           conv3(GN(x)))))))   (GN = GroupNorm(1, .), eps 1e-5)
* ``SDblock`` (:199-236)                 -- GELU(conv_module(band)), bands concatenated over F
                                           (= skip), then the 3x3 ``globalconv``
* ``FusionLayer`` (:55-83)               -- x += skip; GLU(conv3x3(x.repeat(1, 2, 1, 1)))
* ``SUlayer`` (:151-196)                 -- per band ConvTranspose2d (k, 1) stride (s, 1), trimmed
                                           symmetrically to the original band length
* ``DualPathRNN`` (separation.py:37-86)  -- freq path then time path: GN, bi-LSTM (PyTorch gate
                                           order i, f, g, o), Linear(2H -> d), residual
* ``FeatureConversion`` (:6-34)          -- rfft / irfft over T, norm="ortho", real|imag on C

The LSTM recurrence is written out (not nn.LSTM) so this file states the algorithm the HIP kernel
implements.  ``params`` maps reference state_dict names to fp32 tensors.
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

BAND_KEYS = ("low", "mid", "high")


def load_cfg(path):
    import yaml
    with open(path) as f:
        return yaml.safe_load(f)


def model_kwargs(cfg):
    """SCNet(**config.model) with the constructor defaults (scnet.py:260-279)."""
    d = dict(sources=["drums", "bass", "other", "vocals"], audio_channels=2, dims=[4, 32, 64, 128], nfft=4096,
             hop_size=1024, win_size=4096, normalized=True, band_SR=[0.175, 0.392, 0.433], band_stride=[1, 4, 16],
             band_kernel=[3, 4, 16], conv_depths=[3, 2, 1], compress=4, conv_kernel=3, num_dplayer=6, expand=1)
    d.update(dict(cfg["model"]))
    return d


def param_names(cfg):
    """Reference state_dict() (name, shape) in registration order (scnet.py:280-323)."""
    k = model_kwargs(cfg)
    dims, nsrc, kern = k["dims"], len(k["sources"]), k["conv_kernel"]
    out = []
    for i in range(len(dims) - 1):
        cin, cout = dims[i], dims[i + 1]
        p = f"encoder.{i}"
        for b in range(3):
            kk = k["band_kernel"][b]
            out += [(f"{p}.SDlayer.convs.{b}.weight", (cout, cin, kk, 1)), (f"{p}.SDlayer.convs.{b}.bias", (cout,))]
        hid = int(cout / k["compress"])
        for b, depth in enumerate(k["conv_depths"]):
            for l in range(abs(depth)):
                q = f"{p}.conv_modules.{b}.layers.{l}"
                out += [(f"{q}.0.weight", (cout,)), (f"{q}.0.bias", (cout,)),
                        (f"{q}.1.weight", (2 * hid, cout, kern)), (f"{q}.1.bias", (2 * hid,)),
                        (f"{q}.3.weight", (hid, 1, kern)), (f"{q}.3.bias", (hid,)),
                        (f"{q}.4.weight", (hid,)), (f"{q}.4.bias", (hid,)),
                        (f"{q}.6.weight", (cout, hid, 1)), (f"{q}.6.bias", (cout,))]
        out += [(f"{p}.globalconv.weight", (cout, cout, 3, 3)), (f"{p}.globalconv.bias", (cout,))]
    n_lv = len(dims) - 1
    for j in range(n_lv):
        i = n_lv - 1 - j  # decoder.insert(0, ...) (:315)
        c = dims[i + 1]
        co = dims[i] if i != 0 else dims[i] * nsrc
        p = f"decoder.{j}"
        out += [(f"{p}.0.conv.weight", (2 * c, 2 * c, 3, 3)), (f"{p}.0.conv.bias", (2 * c,))]
        for b in range(3):
            kk = k["band_kernel"][b]
            out += [(f"{p}.1.convtrs.{b}.weight", (c, co, kk, 1)), (f"{p}.1.convtrs.{b}.bias", (co,))]
    for i in range(k["num_dplayer"]):
        d = dims[-1] * (2 if i % 2 == 1 else 1)
        H = d * k["expand"]
        p = f"separation_net.dp_modules.{i}"
        for l in range(2):
            for sfx in ("", "_reverse"):
                out += [(f"{p}.lstm_layers.{l}.weight_ih_l0{sfx}", (4 * H, d)),
                        (f"{p}.lstm_layers.{l}.weight_hh_l0{sfx}", (4 * H, H)),
                        (f"{p}.lstm_layers.{l}.bias_ih_l0{sfx}", (4 * H,)),
                        (f"{p}.lstm_layers.{l}.bias_hh_l0{sfx}", (4 * H,))]
        for l in range(2):
            out += [(f"{p}.linear_layers.{l}.weight", (d, 2 * H)), (f"{p}.linear_layers.{l}.bias", (d,))]
        for l in range(2):
            out += [(f"{p}.norm_layers.{l}.weight", (d,)), (f"{p}.norm_layers.{l}.bias", (d,))]
    return out


def synth_params(cfg, affine="random", seed=0):
    """Name-keyed synthetic weights (oracle/weights.py scheme).  Conv/Linear/LSTM weights
    U(+-1/sqrt(prod(shape[1:]))); their biases U(+-1/sqrt(fan_in of the weight)) (affine='random')
    or 0; GroupNorm gamma U(0.5, 1.5) / beta U(-0.2, 0.2) (affine='random') or 1 / 0."""
    from .weights import param_rng, synth_param
    names = param_names(cfg)
    shapes = dict(names)
    out = {}
    for name, shape in names:
        wname = name[:-5] + ".weight" if name.endswith(".bias") else name.replace("bias_", "weight_")
        if "bias" in name and wname in shapes and len(shapes[wname]) >= 2:
            fan_in = int(np.prod(shapes[wname][1:]))
            if affine == "random":
                b = 1.0 / math.sqrt(fan_in)
                out[name] = param_rng(name, seed).uniform(-b, b, size=shape).astype(np.float32)
            else:
                out[name] = np.zeros(shape, np.float32)
        else:
            out[name] = synth_param(name, shape, affine, seed)
    return out


def to_torch(params):
    return {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in params.items()}


def band_splits(Fr, band_SR):
    """SDlayer split points (scnet.py:117-122)."""
    a = math.ceil(Fr * band_SR[0])
    b = math.ceil(Fr * (band_SR[0] + band_SR[1]))
    return [(0, a), (a, b), (b, Fr)]


def sd_layer(P, p, x, k):
    """scnet.py:114-148: per band zero pad over F and Conv2d (kernel, 1) stride (stride, 1)."""
    outs, lens = [], []
    for b, (s, e) in enumerate(band_splits(x.shape[2], k["band_SR"])):
        stride, kern = k["band_stride"][b], k["band_kernel"][b]
        ext = x[:, :, s:e, :]
        n = e - s
        lens.append(n)
        tot = kern - stride if stride == 1 else (stride - n % stride) % stride
        ext = F.pad(ext, (0, 0, tot // 2, tot - tot // 2))
        outs.append(F.conv2d(ext, P[f"{p}.convs.{b}.weight"], P[f"{p}.convs.{b}.bias"], stride=(stride, 1)))
    return outs, lens


def conv_module(P, p, x, depth, kern):
    """ConvolutionModule.forward (scnet.py:49-52) on x [N, C, T]."""
    for l in range(abs(depth)):
        q = f"{p}.layers.{l}"
        y = F.group_norm(x, 1, P[f"{q}.0.weight"], P[f"{q}.0.bias"], 1e-5)
        y = F.conv1d(y, P[f"{q}.1.weight"], P[f"{q}.1.bias"], padding=kern // 2)
        y = F.glu(y, 1)
        y = F.conv1d(y, P[f"{q}.3.weight"], P[f"{q}.3.bias"], padding=kern // 2, groups=y.shape[1])
        y = F.group_norm(y, 1, P[f"{q}.4.weight"], P[f"{q}.4.bias"], 1e-5)
        y = y * y.sigmoid()
        y = F.conv1d(y, P[f"{q}.6.weight"], P[f"{q}.6.bias"])
        x = x + y
    return x


def sd_block(P, p, x, k):
    """SDblock.forward (scnet.py:223-236)."""
    bands, orig = sd_layer(P, f"{p}.SDlayer", x, k)
    outs = []
    for b, band in enumerate(bands):
        B, C, f, T = band.shape
        y = conv_module(P, f"{p}.conv_modules.{b}", band.permute(0, 2, 1, 3).reshape(-1, C, T),
                        k["conv_depths"][b], k["conv_kernel"])
        outs.append(F.gelu(y.view(B, f, C, T).permute(0, 2, 1, 3)))
    lengths = [o.shape[-2] for o in outs]
    full = torch.cat(outs, 2)
    return F.conv2d(full, P[f"{p}.globalconv.weight"], P[f"{p}.globalconv.bias"], padding=1), full, lengths, orig


def fusion(P, p, x, skip):
    """FusionLayer.forward (scnet.py:78-83)."""
    x = x + skip
    x = x.repeat(1, 2, 1, 1)
    return F.glu(F.conv2d(x, P[f"{p}.conv.weight"], P[f"{p}.conv.bias"], padding=1), 1)


def su_layer(P, p, x, lengths, orig, k):
    """SUlayer.forward (scnet.py:171-196)."""
    s0, s1 = lengths[0], lengths[0] + lengths[1]
    outs = []
    for b, (s, e) in enumerate(((0, s0), (s0, s1), (s1, x.shape[2]))):
        o = F.conv_transpose2d(x[:, :, s:e, :], P[f"{p}.convtrs.{b}.weight"], P[f"{p}.convtrs.{b}.bias"],
                               stride=(k["band_stride"][b], 1))
        dist = abs(orig[b] - o.shape[2]) // 2
        outs.append(o[:, :, dist:dist + orig[b], :])
    return torch.cat(outs, 2)


def lstm_dir(x, w_ih, w_hh, b_ih, b_hh, reverse):
    """One direction of torch.nn.LSTM (batch_first, 1 layer): gates = x W_ih^T + b_ih + h W_hh^T + b_hh,
    (i, f, g, o) = (sigma, sigma, tanh, sigma); c = f c + i g; h = o tanh(c).  x [N, L, I] -> [N, L, H]."""
    N, L, _ = x.shape
    H = w_hh.shape[1]
    gx = x @ w_ih.t() + (b_ih + b_hh)
    h = x.new_zeros(N, H)
    c = x.new_zeros(N, H)
    out = x.new_empty(N, L, H)
    for s in (range(L - 1, -1, -1) if reverse else range(L)):
        g = gx[:, s] + h @ w_hh.t()
        i, f, gg, o = g.split(H, 1)
        c = f.sigmoid() * c + i.sigmoid() * gg.tanh()
        h = o.sigmoid() * c.tanh()
        out[:, s] = h
    return out


def bilstm(P, p, x):
    f = lstm_dir(x, P[f"{p}.weight_ih_l0"], P[f"{p}.weight_hh_l0"], P[f"{p}.bias_ih_l0"], P[f"{p}.bias_hh_l0"], False)
    r = lstm_dir(x, P[f"{p}.weight_ih_l0_reverse"], P[f"{p}.weight_hh_l0_reverse"], P[f"{p}.bias_ih_l0_reverse"],
                 P[f"{p}.bias_hh_l0_reverse"], True)
    return torch.cat([f, r], 2)


def dual_path(P, p, x):
    """DualPathRNN.forward (separation.py:62-86)."""
    B, C, Fr, T = x.shape
    res = x
    y = F.group_norm(x, 1, P[f"{p}.norm_layers.0.weight"], P[f"{p}.norm_layers.0.bias"], 1e-5)
    y = y.transpose(1, 3).reshape(B * T, Fr, C)
    y = bilstm(P, f"{p}.lstm_layers.0", y)
    y = F.linear(y, P[f"{p}.linear_layers.0.weight"], P[f"{p}.linear_layers.0.bias"])
    x = y.view(B, T, Fr, C).transpose(1, 3) + res
    res = x
    y = F.group_norm(x, 1, P[f"{p}.norm_layers.1.weight"], P[f"{p}.norm_layers.1.bias"], 1e-5)
    y = y.transpose(1, 2).reshape(B * Fr, C, T).transpose(1, 2)
    y = bilstm(P, f"{p}.lstm_layers.1", y)
    y = F.linear(y, P[f"{p}.linear_layers.1.weight"], P[f"{p}.linear_layers.1.bias"])
    return y.transpose(1, 2).reshape(B, Fr, C, T).transpose(1, 2) + res


def feature_conversion(x, inverse):
    """FeatureConversion.forward (separation.py:20-34)."""
    if inverse:
        C = x.shape[1] // 2
        return torch.fft.irfft(torch.complex(x[:, :C], x[:, C:]), dim=3, norm="ortho")
    z = torch.fft.rfft(x, dim=3, norm="ortho")
    return torch.cat([z.real, z.imag], 1)


def pad_amount(L, hop):
    """scnet.py:330-333."""
    padding = hop - L % hop
    if (L + padding) // hop % 2 == 0:
        padding += hop
    return padding


def forward(P, cfg, x):
    """SCNet.forward (scnet.py:325-373): x [B, ch, L] -> [B, n_sources, ch, L]."""
    k = model_kwargs(cfg)
    B, ach = x.shape[0], k["audio_channels"]
    hop = k["hop_size"]
    padding = pad_amount(x.shape[-1], hop)
    x = F.pad(x, (0, padding))
    L = x.shape[-1]
    # window=None in the reference means a rectangular window of win_length (torch.stft docs)
    stft = dict(n_fft=k["nfft"], hop_length=hop, win_length=k["win_size"], center=True, normalized=k["normalized"],
                window=torch.ones(k["win_size"]))
    z = torch.view_as_real(torch.stft(x.reshape(-1, L), **stft, return_complex=True))
    z = z.permute(0, 3, 1, 2).reshape(z.shape[0] // ach, z.shape[3] * ach, z.shape[1], z.shape[2])
    _, _, Fr, T = z.shape
    skips, lens, origs = [], [], []
    h = z
    for i in range(len(k["dims"]) - 1):
        h, skip, ln, og = sd_block(P, f"encoder.{i}", h, k)
        skips.append(skip)
        lens.append(ln)
        origs.append(og)
    for i in range(k["num_dplayer"]):
        h = dual_path(P, f"separation_net.dp_modules.{i}", h)
        h = feature_conversion(h, inverse=(i % 2 == 1))
    for j in range(len(k["dims"]) - 1):
        h = fusion(P, f"decoder.{j}.0", h, skips.pop())
        h = su_layer(P, f"decoder.{j}.1", h, lens.pop(), origs.pop(), k)
    n = k["dims"][0]
    h = h.view(B, n, -1, Fr, T).reshape(-1, 2, Fr, T).permute(0, 2, 3, 1)
    y = torch.istft(torch.view_as_complex(h.contiguous()), **stft)
    y = y.reshape(B, len(k["sources"]), ach, -1)
    return y[:, :, :, :-padding]


class Model:
    """Callable wrapper (backend-shaped): x [B, ch, C] -> [B, n_sources, ch, C]."""

    def __init__(self, cfg, params):
        self.cfg = cfg
        self.P = params

    def __call__(self, x):
        with torch.inference_mode():
            return forward(self.P, self.cfg, x)
