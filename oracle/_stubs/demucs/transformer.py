"""demucs.transformer restated (see package docstring): the cross-domain transformer of HTDemucs.

Only the configuration HTDemucs uses is restated: sinusoidal embeddings (``emb='sin'``), dense
attention (no sparse masks), LayerNorm / MyGroupNorm norms, LayerScale, ``batch_first=True``."""
import math
import random

import torch
import torch.nn.functional as F
from einops import rearrange
from torch import nn


def create_sin_embedding(length: int, dim: int, shift: int = 0, device="cpu", max_period=10000):
    assert dim % 2 == 0
    pos = shift + torch.arange(length, device=device).view(-1, 1, 1)
    half_dim = dim // 2
    adim = torch.arange(dim // 2, device=device).view(1, 1, -1)
    phase = pos / (max_period ** (adim / (half_dim - 1)))
    return torch.cat([torch.cos(phase), torch.sin(phase)], dim=-1)


def create_2d_sin_embedding(d_model, height, width, device="cpu", max_period=10000):
    if d_model % 4 != 0:
        raise ValueError(f"Cannot use sin/cos positional encoding with odd dimension (got dim={d_model})")
    pe = torch.zeros(d_model, height, width)
    d_model = int(d_model / 2)
    div_term = torch.exp(torch.arange(0.0, d_model, 2) * -(math.log(max_period) / d_model))
    pos_w = torch.arange(0.0, width).unsqueeze(1)
    pos_h = torch.arange(0.0, height).unsqueeze(1)
    pe[0:d_model:2, :, :] = torch.sin(pos_w * div_term).transpose(0, 1).unsqueeze(1).repeat(1, height, 1)
    pe[1:d_model:2, :, :] = torch.cos(pos_w * div_term).transpose(0, 1).unsqueeze(1).repeat(1, height, 1)
    pe[d_model::2, :, :] = torch.sin(pos_h * div_term).transpose(0, 1).unsqueeze(2).repeat(1, 1, width)
    pe[d_model + 1::2, :, :] = torch.cos(pos_h * div_term).transpose(0, 1).unsqueeze(2).repeat(1, 1, width)
    return pe[None, :].to(device)


class MyGroupNorm(nn.GroupNorm):
    """GroupNorm over (T, C) for (B, T, C) inputs."""

    def forward(self, x):
        x = x.transpose(1, 2)
        return super().forward(x).transpose(1, 2)


class LayerScale(nn.Module):
    def __init__(self, channels: int, init: float = 0, channel_last=False):
        super().__init__()
        self.channel_last = channel_last
        self.scale = nn.Parameter(torch.zeros(channels, requires_grad=True))
        self.scale.data[:] = init

    def forward(self, x):
        if self.channel_last:
            return self.scale * x
        return self.scale[:, None] * x


class MyTransformerEncoderLayer(nn.TransformerEncoderLayer):
    def __init__(self, d_model, nhead, dim_feedforward=2048, dropout=0.1, activation=F.relu, group_norm=0,
                 norm_first=False, norm_out=False, layer_norm_eps=1e-5, layer_scale=False, init_values=1e-4,
                 device=None, dtype=None, sparse=False, mask_type="diag", mask_random_seed=42,
                 sparse_attn_window=500, global_window=50, auto_sparsity=False, sparsity=0.95, batch_first=False):
        if sparse:
            raise NotImplementedError("sparse attention is not used by the released HTDemucs configs")
        factory_kwargs = {"device": device, "dtype": dtype}
        super().__init__(d_model=d_model, nhead=nhead, dim_feedforward=dim_feedforward, dropout=dropout,
                         activation=activation, layer_norm_eps=layer_norm_eps, batch_first=batch_first,
                         norm_first=norm_first, device=device, dtype=dtype)
        self.sparse = sparse
        self.auto_sparsity = auto_sparsity
        if group_norm:
            self.norm1 = MyGroupNorm(int(group_norm), d_model, eps=layer_norm_eps, **factory_kwargs)
            self.norm2 = MyGroupNorm(int(group_norm), d_model, eps=layer_norm_eps, **factory_kwargs)
        self.norm_out = None
        if self.norm_first & norm_out:
            self.norm_out = MyGroupNorm(num_groups=int(norm_out), num_channels=d_model)
        self.gamma_1 = LayerScale(d_model, init_values, True) if layer_scale else nn.Identity()
        self.gamma_2 = LayerScale(d_model, init_values, True) if layer_scale else nn.Identity()

    def forward(self, src, src_mask=None, src_key_padding_mask=None):
        x = src
        if self.norm_first:
            x = x + self.gamma_1(self._sa_block(self.norm1(x), src_mask, src_key_padding_mask))
            x = x + self.gamma_2(self._ff_block(self.norm2(x)))
            if self.norm_out:
                x = self.norm_out(x)
        else:
            x = self.norm1(x + self.gamma_1(self._sa_block(x, src_mask, src_key_padding_mask)))
            x = self.norm2(x + self.gamma_2(self._ff_block(x)))
        return x


class CrossTransformerEncoderLayer(nn.Module):
    def __init__(self, d_model: int, nhead: int, dim_feedforward: int = 2048, dropout: float = 0.1,
                 activation=F.relu, layer_norm_eps: float = 1e-5, layer_scale: bool = False,
                 init_values: float = 1e-4, norm_first: bool = False, group_norm: bool = False,
                 norm_out: bool = False, sparse=False, mask_type="diag", mask_random_seed=42,
                 sparse_attn_window=500, global_window=50, sparsity=0.95, auto_sparsity=None, device=None,
                 dtype=None, batch_first=False):
        if sparse:
            raise NotImplementedError("sparse attention is not used by the released HTDemucs configs")
        factory_kwargs = {"device": device, "dtype": dtype}
        super().__init__()
        self.sparse = sparse
        self.auto_sparsity = auto_sparsity
        self.cross_attn = nn.MultiheadAttention(d_model, nhead, dropout=dropout, batch_first=batch_first)
        self.linear1 = nn.Linear(d_model, dim_feedforward, **factory_kwargs)
        self.dropout = nn.Dropout(dropout)
        self.linear2 = nn.Linear(dim_feedforward, d_model, **factory_kwargs)
        self.norm_first = norm_first
        if group_norm:
            self.norm1 = MyGroupNorm(int(group_norm), d_model, eps=layer_norm_eps, **factory_kwargs)
            self.norm2 = MyGroupNorm(int(group_norm), d_model, eps=layer_norm_eps, **factory_kwargs)
            self.norm3 = MyGroupNorm(int(group_norm), d_model, eps=layer_norm_eps, **factory_kwargs)
        else:
            self.norm1 = nn.LayerNorm(d_model, eps=layer_norm_eps, **factory_kwargs)
            self.norm2 = nn.LayerNorm(d_model, eps=layer_norm_eps, **factory_kwargs)
            self.norm3 = nn.LayerNorm(d_model, eps=layer_norm_eps, **factory_kwargs)
        self.norm_out = None
        if self.norm_first & norm_out:
            self.norm_out = MyGroupNorm(num_groups=int(norm_out), num_channels=d_model)
        self.gamma_1 = LayerScale(d_model, init_values, True) if layer_scale else nn.Identity()
        self.gamma_2 = LayerScale(d_model, init_values, True) if layer_scale else nn.Identity()
        self.dropout1 = nn.Dropout(dropout)
        self.dropout2 = nn.Dropout(dropout)
        self.activation = activation

    def forward(self, q, k, mask=None):
        if self.norm_first:
            x = q + self.gamma_1(self._ca_block(self.norm1(q), self.norm2(k), mask))
            x = x + self.gamma_2(self._ff_block(self.norm3(x)))
            if self.norm_out:
                x = self.norm_out(x)
        else:
            x = self.norm1(q + self.gamma_1(self._ca_block(q, k, mask)))
            x = self.norm2(x + self.gamma_2(self._ff_block(x)))
        return x

    def _ca_block(self, q, k, attn_mask=None):
        x = self.cross_attn(q, k, k, attn_mask=attn_mask, need_weights=False)[0]
        return self.dropout1(x)

    def _ff_block(self, x):
        x = self.linear2(self.dropout(self.activation(self.linear1(x))))
        return self.dropout2(x)


class CrossTransformerEncoder(nn.Module):
    def __init__(self, dim: int, emb: str = "sin", hidden_scale: float = 4.0, num_heads: int = 8, num_layers: int = 6,
                 cross_first: bool = False, dropout: float = 0.0, max_positions: int = 1000, norm_in: bool = True,
                 norm_in_group: bool = False, group_norm: int = False, norm_first: bool = False,
                 norm_out: bool = False, max_period: float = 10000.0, weight_decay: float = 0.0, lr=None,
                 layer_scale: bool = False, gelu: bool = True, sin_random_shift: int = 0,
                 weight_pos_embed: float = 1.0, cape_mean_normalize: bool = True, cape_augment: bool = True,
                 cape_glob_loc_scale: list = [5000.0, 1.0, 1.4], sparse_self_attn: bool = False,
                 sparse_cross_attn: bool = False, mask_type: str = "diag", mask_random_seed: int = 42,
                 sparse_attn_window: int = 500, global_window: int = 50, auto_sparsity: bool = False,
                 sparsity: float = 0.95):
        super().__init__()
        assert dim % num_heads == 0
        if emb != "sin":
            raise NotImplementedError("only the sinusoidal embedding of the released HTDemucs configs is restated")
        hidden_dim = int(dim * hidden_scale)
        self.num_layers = num_layers
        self.classic_parity = 1 if cross_first else 0
        self.emb = emb
        self.max_period = max_period
        self.weight_decay = weight_decay
        self.weight_pos_embed = weight_pos_embed
        self.sin_random_shift = sin_random_shift
        self.lr = lr
        activation = F.gelu if gelu else F.relu
        if norm_in:
            self.norm_in = nn.LayerNorm(dim)
            self.norm_in_t = nn.LayerNorm(dim)
        elif norm_in_group:
            self.norm_in = MyGroupNorm(int(norm_in_group), dim)
            self.norm_in_t = MyGroupNorm(int(norm_in_group), dim)
        else:
            self.norm_in = nn.Identity()
            self.norm_in_t = nn.Identity()
        self.layers = nn.ModuleList()
        self.layers_t = nn.ModuleList()
        kw = {"d_model": dim, "nhead": num_heads, "dim_feedforward": hidden_dim, "dropout": dropout,
              "activation": activation, "group_norm": group_norm, "norm_first": norm_first, "norm_out": norm_out,
              "layer_scale": layer_scale, "mask_type": mask_type, "mask_random_seed": mask_random_seed,
              "sparse_attn_window": sparse_attn_window, "global_window": global_window, "sparsity": sparsity,
              "auto_sparsity": auto_sparsity, "batch_first": True}
        for idx in range(num_layers):
            if idx % 2 == self.classic_parity:
                self.layers.append(MyTransformerEncoderLayer(**kw, sparse=sparse_self_attn))
                self.layers_t.append(MyTransformerEncoderLayer(**kw, sparse=sparse_self_attn))
            else:
                self.layers.append(CrossTransformerEncoderLayer(**kw, sparse=sparse_cross_attn))
                self.layers_t.append(CrossTransformerEncoderLayer(**kw, sparse=sparse_cross_attn))

    def forward(self, x, xt):
        B, C, Fr, T1 = x.shape
        pos_emb_2d = create_2d_sin_embedding(C, Fr, T1, x.device, self.max_period)
        pos_emb_2d = rearrange(pos_emb_2d, "b c fr t1 -> b (t1 fr) c")
        x = rearrange(x, "b c fr t1 -> b (t1 fr) c")
        x = self.norm_in(x)
        x = x + self.weight_pos_embed * pos_emb_2d
        B, C, T2 = xt.shape
        xt = rearrange(xt, "b c t2 -> b t2 c")
        pos_emb = self._get_pos_embedding(T2, B, C, x.device)
        pos_emb = rearrange(pos_emb, "t2 b c -> b t2 c")
        xt = self.norm_in_t(xt)
        xt = xt + self.weight_pos_embed * pos_emb
        for idx in range(self.num_layers):
            if idx % 2 == self.classic_parity:
                x = self.layers[idx](x)
                xt = self.layers_t[idx](xt)
            else:
                old_x = x
                x = self.layers[idx](x, xt)
                xt = self.layers_t[idx](xt, old_x)
        x = rearrange(x, "b (t1 fr) c -> b c fr t1", t1=T1)
        xt = rearrange(xt, "b t2 c -> b c t2")
        return x, xt

    def _get_pos_embedding(self, T, B, C, device):
        shift = random.randrange(self.sin_random_shift + 1)
        return create_sin_embedding(T, C, shift=shift, device=device, max_period=self.max_period)
