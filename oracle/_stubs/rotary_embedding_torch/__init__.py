"""Restatement of the third-party ``rotary_embedding_torch`` pieces BS-Roformer uses.  TEST
INFRASTRUCTURE ONLY (oracle/): never imported by the product path.

The package is an UNPINNED dependency of the reference (``requirements.txt:33``), not vendored and
not installed here, so its published algorithm is restated:

* ``RotaryEmbedding(dim)``: ``freqs = 1 / theta ** (arange(0, dim, 2)[:dim//2] / dim)``, theta 10000,
  held as ``nn.Parameter(freqs, requires_grad=False)`` (so it appears in ``state_dict`` as
  ``...rotary_embed.freqs``, as in released checkpoints).
* ``rotate_queries_or_keys(t)``: positions ``arange(seq_len)`` along dim -2, angles
  ``pos * freqs`` repeated pairwise ``'... n -> ... (n r)', r=2``, then
  ``t * cos + rotate_half(t) * sin`` with ``rotate_half`` on interleaved pairs
  ``(x1, x2) -> (-x2, x1)``.

Parity at this boundary is UNPINNED by any reference test (the reference has none); it is the
algorithm as published.  Used (a) by tests/golden/make_golden_bsr.py to import the reference
model, and (b) by oracle/bs_roformer.py.
"""
import torch
from torch import nn


def rotate_half(x):
    x = x.reshape(*x.shape[:-1], -1, 2)
    x1, x2 = x.unbind(dim=-1)
    return torch.stack((-x2, x1), dim=-1).reshape(*x.shape[:-2], -1)


def apply_rotary_emb(freqs, t, start_index=0, scale=1.0):
    rot_dim = freqs.shape[-1]
    end_index = start_index + rot_dim
    t_left, t_mid, t_right = t[..., :start_index], t[..., start_index:end_index], t[..., end_index:]
    t_mid = (t_mid * freqs.cos() * scale) + (rotate_half(t_mid) * freqs.sin() * scale)
    return torch.cat((t_left, t_mid, t_right), dim=-1)


def inv_freqs(dim, theta=10000.0):
    return 1.0 / (theta ** (torch.arange(0, dim, 2)[: (dim // 2)].float() / dim))


def angles(freqs, seq_len):
    """[seq_len, 2*len(freqs)] fp32 angles, pairwise repeated (the library's forward())."""
    seq = torch.arange(seq_len, dtype=torch.float32)
    f = torch.einsum("i,f->if", seq.type(freqs.dtype), freqs)
    return f.repeat_interleave(2, dim=-1)


class RotaryEmbedding(nn.Module):
    def __init__(self, dim, theta=10000, learned_freq=False, interpolate_factor=1.0, **_ignored):
        super().__init__()
        self.freqs = nn.Parameter(inv_freqs(dim, float(theta)), requires_grad=learned_freq)
        self.interpolate_factor = interpolate_factor

    def rotate_queries_or_keys(self, t, seq_dim=-2, offset=0):
        seq_len = t.shape[seq_dim]
        seq = (torch.arange(seq_len, device=t.device, dtype=t.dtype) + offset) / self.interpolate_factor
        f = torch.einsum("i,f->if", seq.type(self.freqs.dtype), self.freqs).repeat_interleave(2, dim=-1)
        return apply_rotary_emb(f, t)
