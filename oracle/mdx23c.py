"""Functional PyTorch-CPU fp32 restatement of MDX23C (TFC-TDF-v3).  TEST INFRASTRUCTURE.

Restates ``/root/reference/models/mdx23c_tfc_tdf_v3.py``:

* ``stft`` / ``istft``   -- ``STFT.__call__`` (:14-30) / ``STFT.inverse`` (:32-44)
* ``tfc_tdf``            -- ``TFC_TDF.forward`` (:131-138); block layout (:100-129)
* ``forward``            -- ``TFC_TDF_net.forward`` (:205-242), ``cac2cws``/``cws2cac`` (:191-203)
* ``param_shapes``       -- ``TFC_TDF_net.__init__`` (:141-189) parameter names / shapes,
  the keys of the reference ``state_dict`` (so real checkpoints load by name).

``params`` is a dict name -> torch.Tensor (float32, CPU).  The network runs in
the reference's own NCHW layout with the reference's torch CPU ops, so this is
the "reference CPU path" the product is measured against.
"""
import torch
import torch.nn.functional as F


def _num_instruments(cfg):
    # utils.prefer_target_instrument (utils.py:480-499)
    t = cfg["training"].get("target_instrument")
    return 1 if t else len(cfg["training"]["instruments"])


def param_shapes(cfg):
    """(name, shape) in the reference's named_parameters() order (mdx23c_tfc_tdf_v3.py:141-189)."""
    m, a = cfg["model"], cfg["audio"]
    k = m["num_subbands"]
    dim_c = k * a["num_channels"] * 2
    n, l, c, g, bn = m["num_scales"], m["num_blocks_per_scale"], m["num_channels"], m["growth"], m["bottleneck_factor"]
    sc = m["scale"]
    f = a["dim_f"] // k
    out = [("first_conv.weight", (c, dim_c, 1, 1))]

    def tfc_tdf(prefix, in_c, c, f):
        for i in range(l):
            p = f"{prefix}.blocks.{i}"
            out.extend([
                (f"{p}.tfc1.0.weight", (in_c,)), (f"{p}.tfc1.0.bias", (in_c,)),
                (f"{p}.tfc1.2.weight", (c, in_c, 3, 3)),
                (f"{p}.tdf.0.weight", (c,)), (f"{p}.tdf.0.bias", (c,)),
                (f"{p}.tdf.2.weight", (f // bn, f)),
                (f"{p}.tdf.3.weight", (c,)), (f"{p}.tdf.3.bias", (c,)),
                (f"{p}.tdf.5.weight", (f, f // bn)),
                (f"{p}.tfc2.0.weight", (c,)), (f"{p}.tfc2.0.bias", (c,)),
                (f"{p}.tfc2.2.weight", (c, c, 3, 3)),
                (f"{p}.shortcut.weight", (c, in_c, 1, 1)),
            ])
            in_c = c

    for i in range(n):
        tfc_tdf(f"encoder_blocks.{i}.tfc_tdf", c, c, f)
        out.extend([(f"encoder_blocks.{i}.downscale.conv.0.weight", (c,)),
                    (f"encoder_blocks.{i}.downscale.conv.0.bias", (c,)),
                    (f"encoder_blocks.{i}.downscale.conv.2.weight", (c + g, c, sc[0], sc[1]))])
        f = f // sc[1]
        c += g
    tfc_tdf("bottleneck_block", c, c, f)
    for i in range(n):
        out.extend([(f"decoder_blocks.{i}.upscale.conv.0.weight", (c,)),
                    (f"decoder_blocks.{i}.upscale.conv.0.bias", (c,)),
                    (f"decoder_blocks.{i}.upscale.conv.2.weight", (c, c - g, sc[0], sc[1]))])
        f = f * sc[1]
        c -= g
        tfc_tdf(f"decoder_blocks.{i}.tfc_tdf", 2 * c, c, f)
    out.append(("final_conv.0.weight", (c, c + dim_c, 1, 1)))
    out.append(("final_conv.2.weight", (_num_instruments(cfg) * dim_c, c, 1, 1)))
    return out


def hann(n_fft):
    return torch.hann_window(n_fft, periodic=True)


def stft(x, a):
    """STFT.__call__ (mdx23c_tfc_tdf_v3.py:14-30): [..., c, t] -> [..., 2c, dim_f, frames]."""
    batch_dims = x.shape[:-2]
    c, t = x.shape[-2:]
    x = x.reshape(-1, t)
    X = torch.stft(x, n_fft=a["n_fft"], hop_length=a["hop_length"], window=hann(a["n_fft"]),
                   center=True, return_complex=True)
    X = torch.view_as_real(X).permute(0, 3, 1, 2)
    X = X.reshape(*batch_dims, c * 2, -1, X.shape[-1])
    return X[..., :a["dim_f"], :]


def istft(x, a):
    """STFT.inverse (mdx23c_tfc_tdf_v3.py:32-44): zero Nyquist pad, complex, torch.istft (no length)."""
    batch_dims = x.shape[:-3]
    c, f, t = x.shape[-3:]
    n = a["n_fft"] // 2 + 1
    x = torch.cat([x, torch.zeros(*batch_dims, c, n - f, t)], -2)
    x = x.reshape(-1, 2, n, t).permute(0, 2, 3, 1)
    x = torch.complex(x[..., 0].contiguous(), x[..., 1].contiguous())
    y = torch.istft(x, n_fft=a["n_fft"], hop_length=a["hop_length"], window=hann(a["n_fft"]), center=True)
    return y.reshape(*batch_dims, 2, -1)


def _in_gelu(x, p, name):
    # get_norm('InstanceNorm') + get_act('gelu') (:47-71): InstanceNorm2d(affine=True, eps=1e-5), exact GELU
    x = F.instance_norm(x, weight=p[name + ".weight"], bias=p[name + ".bias"], eps=1e-5)
    return F.gelu(x)


def tfc_tdf(x, p, prefix, n_blocks):
    """TFC_TDF.forward (mdx23c_tfc_tdf_v3.py:131-138)."""
    for i in range(n_blocks):
        q = f"{prefix}.blocks.{i}"
        s = F.conv2d(x, p[q + ".shortcut.weight"])
        x = F.conv2d(_in_gelu(x, p, q + ".tfc1.0"), p[q + ".tfc1.2.weight"], padding=1)
        t = F.linear(_in_gelu(x, p, q + ".tdf.0"), p[q + ".tdf.2.weight"])
        t = F.linear(_in_gelu(t, p, q + ".tdf.3"), p[q + ".tdf.5.weight"])
        x = x + t
        x = F.conv2d(_in_gelu(x, p, q + ".tfc2.0"), p[q + ".tfc2.2.weight"], padding=1)
        x = x + s
    return x


def forward(params, cfg, x):
    """TFC_TDF_net.forward (mdx23c_tfc_tdf_v3.py:205-242): [B,2,C] -> [B,n_instr,2,C] (or [B,2,C])."""
    m, a = cfg["model"], cfg["audio"]
    p = params
    k = m["num_subbands"]
    n, l, sc = m["num_scales"], m["num_blocks_per_scale"], m["scale"]
    X = stft(x, a)
    b, c, f, t = X.shape
    mix = X = X.reshape(b, c * k, f // k, t)                       # cac2cws (:191-196)
    first = X = F.conv2d(X, p["first_conv.weight"])
    X = X.transpose(-1, -2)
    skips = []
    for i in range(n):
        X = tfc_tdf(X, p, f"encoder_blocks.{i}.tfc_tdf", l)
        skips.append(X)
        X = F.conv2d(_in_gelu(X, p, f"encoder_blocks.{i}.downscale.conv.0"),
                     p[f"encoder_blocks.{i}.downscale.conv.2.weight"], stride=tuple(sc))
    X = tfc_tdf(X, p, "bottleneck_block", l)
    for i in range(n):
        X = F.conv_transpose2d(_in_gelu(X, p, f"decoder_blocks.{i}.upscale.conv.0"),
                               p[f"decoder_blocks.{i}.upscale.conv.2.weight"], stride=tuple(sc))
        X = torch.cat([X, skips.pop()], 1)
        X = tfc_tdf(X, p, f"decoder_blocks.{i}.tfc_tdf", l)
    X = X.transpose(-1, -2)
    X = X * first
    X = torch.cat([mix, X], 1)
    X = F.conv2d(F.gelu(F.conv2d(X, p["final_conv.0.weight"])), p["final_conv.2.weight"])
    b, c, f, t = X.shape
    X = X.reshape(b, c // k, f * k, t)                              # cws2cac (:198-203)
    ni = _num_instruments(cfg)
    if ni > 1:
        X = X.reshape(b, ni, -1, f * k, t)
    return istft(X, a)


def to_torch_params(np_params):
    return {k: torch.from_numpy(v) for k, v in np_params.items()}


class OracleModel:
    """Callable model wrapper (the ``backend(x)`` role of pytorch_backend.py:284-314) on CPU fp32."""

    def __init__(self, cfg, params):
        self.cfg = cfg
        self.params = to_torch_params(params) if not isinstance(next(iter(params.values())), torch.Tensor) else params

    @torch.inference_mode()
    def __call__(self, x):
        return forward(self.params, self.cfg, x.float())
