"""demucs.demucs restated (see package docstring): DConv, LayerScale, rescale_module; ``Demucs`` is a
placeholder (imported by models/demucs4ht.py:10 but only instantiated by ``get_model`` for
``model: demucs``, which the HTDemucs path never selects)."""
import torch
from torch import nn


class LayerScale(nn.Module):
    """Per-channel scale, initialised to ``init`` (rescales a residual branch)."""

    def __init__(self, channels: int, init: float = 0, channel_last=False):
        super().__init__()
        self.channel_last = channel_last
        self.scale = nn.Parameter(torch.zeros(channels, requires_grad=True))
        self.scale.data[:] = init

    def forward(self, x):
        if self.channel_last:
            return self.scale * x
        return self.scale[:, None] * x


class DConv(nn.Module):
    """Residual branch of dilated 1-D convs: per layer d, x += LayerScale(GLU(GN(conv1x1(GELU(GN(
    conv_k(x, dilation 2^d)))))))."""

    def __init__(self, channels: int, compress: float = 4, depth: int = 2, init: float = 1e-4, norm=True,
                 attn=False, heads=4, ndecay=4, lstm=False, gelu=True, kernel=3, dilate=True):
        super().__init__()
        assert kernel % 2 == 1
        if attn or lstm:
            raise NotImplementedError("DConv attn / lstm branches are not used by HTDemucs")
        self.channels = channels
        self.compress = compress
        self.depth = abs(depth)
        dilate = depth > 0
        norm_fn = (lambda d: nn.GroupNorm(1, d)) if norm else (lambda d: nn.Identity())
        hidden = int(channels / compress)
        act = nn.GELU if gelu else nn.ReLU
        self.layers = nn.ModuleList([])
        for d in range(self.depth):
            dilation = 2 ** d if dilate else 1
            padding = dilation * (kernel // 2)
            mods = [nn.Conv1d(channels, hidden, kernel, dilation=dilation, padding=padding), norm_fn(hidden), act(),
                    nn.Conv1d(hidden, 2 * channels, 1), norm_fn(2 * channels), nn.GLU(1),
                    LayerScale(channels, init)]
            self.layers.append(nn.Sequential(*mods))

    def forward(self, x):
        for layer in self.layers:
            x = x + layer(x)
        return x


def rescale_conv(conv, reference):
    std = conv.weight.std().detach()
    scale = (std / reference) ** 0.5
    conv.weight.data /= scale
    if conv.bias is not None:
        conv.bias.data /= scale


def rescale_module(module, reference):
    for sub in module.modules():
        if isinstance(sub, (nn.Conv1d, nn.ConvTranspose1d, nn.Conv2d, nn.ConvTranspose2d)):
            rescale_conv(sub, reference)


class Demucs(nn.Module):
    def __init__(self, *args, **kwargs):
        raise NotImplementedError("demucs.demucs.Demucs is not restated (only HTDemucs is on the path)")
