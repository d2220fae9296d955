"""HTDemucs on the native MI355X forward (libsesa ``sesa_htdemucs_*``).

Drop-in for ``models/demucs4ht.py:28-693`` (``HTDemucs``) as built by the reference registry
(``get_model``, :696-711: ``HTDemucs(sources=training.instruments, audio_channels=training.channels,
samplerate=training.samplerate, segment=training.segment, **config.htdemucs)``): same ``state_dict``
keys / shapes, same call ``model(mix[B, 2, L]) -> [B, n_sources, 2, L]``.  The whole forward --
``_spec``, both U-Net branches with their DConv residual branches, the cross-domain transformer,
``_mask`` / ``_ispec`` and the branch sum -- runs in libsesa (sesa_htdemucs.hip) on the current HIP
stream.  Configurations outside the released htdemucs structure are refused with a message.
"""
from .. import _native as N
from .native import NativeModule

import ctypes

import torch

_DEFAULTS = dict(channels=48, channels_time=None, growth=2, nfft=4096, num_subbands=1, wiener_iters=0, end_iters=0,
                 wiener_residual=False, cac=True, depth=4, rewrite=True, multi_freqs=None, multi_freqs_depth=3,
                 freq_emb=0.2, emb_scale=10, emb_smooth=True, kernel_size=8, time_stride=2, stride=4, context=1,
                 context_enc=0, norm_starts=4, norm_groups=4, dconv_mode=1, dconv_depth=2, dconv_comp=8,
                 dconv_init=1e-3, bottom_channels=0, t_layers=5, t_emb="sin", t_hidden_scale=4.0, t_heads=8,
                 t_dropout=0.0, t_max_positions=10000, t_norm_in=True, t_norm_in_group=False, t_group_norm=False,
                 t_norm_first=True, t_norm_out=True, t_max_period=10000.0, t_weight_decay=0.0, t_lr=None,
                 t_layer_scale=True, t_gelu=True, t_weight_pos_embed=1.0, t_sin_random_shift=0,
                 t_cape_mean_normalize=True, t_cape_augment=True, t_cape_glob_loc_scale=(5000.0, 1.0, 1.4),
                 t_sparse_self_attn=False, t_sparse_cross_attn=False, t_mask_type="diag", t_mask_random_seed=42,
                 t_sparse_attn_window=500, t_global_window=100, t_sparsity=0.95, t_auto_sparsity=False,
                 t_cross_first=False, rescale=0.1, use_train_segment=False)


class HTDemucs(NativeModule):
    """Reference-compatible HTDemucs backed by the native HIP forward."""

    _prefix = "htdemucs"
    # fp16mix: the cross-transformer attention (fp32 softmax statistics), the implicit-GEMM convs, the 1x1
    # rewrites and the transformer / channel Linears on one fp16 MFMA pass (SESA_HTD_PRESPLIT=0 keeps the Linears
    # bf16x3); norms and the DConv statistics fp32 / fp64
    _precisions = ("bf16x3", "bf16", "fp16mix")
    _amp_precision = "fp16mix"  # --enable_amp (the reference's AMP is fp16 autocast): 5.9e-6 full segment

    def __init__(self, sources, audio_channels=2, samplerate=44100, segment=10, precision="bf16x3", **kw):
        super().__init__(precision)
        unknown = set(kw) - set(_DEFAULTS)
        if unknown:
            raise TypeError(f"HTDemucs: unexpected arguments {sorted(unknown)}")
        k = dict(_DEFAULTS, **kw)
        refuse = []
        if k["multi_freqs"]:
            refuse.append("multi_freqs")
        if k["wiener_iters"] or k["end_iters"]:
            refuse.append("wiener filtering (wiener_iters > 0)")
        if k["t_emb"] != "sin":
            refuse.append(f"t_emb={k['t_emb']!r}")
        if k["t_sparse_self_attn"] or k["t_sparse_cross_attn"]:
            refuse.append("sparse attention")
        if k["t_norm_in_group"] or k["t_group_norm"]:
            refuse.append("group-norm transformer variants")
        if refuse:
            raise NotImplementedError("HTDemucs native engine: unsupported configuration: " + ", ".join(refuse))
        if not k["t_gelu"]:
            # the native fp16mix transformer writes its FF1 output through a GELU-only fp16 epilogue: a ReLU
            # transformer (t_gelu=False) runs bf16x3 / bf16 only, and --enable_amp maps it to bf16x3
            self._precisions = ("bf16x3", "bf16")
            self._amp_precision = "bf16x3"
            if self.precision == "fp16mix":
                raise ValueError("HTDemucs: precision 'fp16mix' needs t_gelu=True (the fp16 FF1 epilogue is GELU "
                                 "only); use 'bf16x3'")
        self.sources = list(sources)
        self.audio_channels = int(audio_channels)
        self.samplerate = samplerate
        self.segment = segment
        self._k = k
        h = self._create(int(samplerate * segment))
        try:
            shapes = []
            for i in range(N.lib().sesa_htdemucs_num_params(h)):
                nm = ctypes.c_char_p()
                N.check(N.lib().sesa_htdemucs_param_info(h, i, ctypes.byref(nm), None))
                dims = (ctypes.c_int64 * 4)()
                nd = ctypes.c_int()
                N.check(N.lib().sesa_htdemucs_param_shape(h, i, dims, ctypes.byref(nd)))
                shapes.append((nm.value.decode(), tuple(dims[d] for d in range(nd.value))))
        finally:
            N.lib().sesa_htdemucs_destroy(h)
        self._register_params(shapes, self._init_value)

    def _init_value(self, name, shape):
        """Defaults of the reference modules before a checkpoint is loaded: norm gammas 1, LayerScale
        at its init value, everything else 0 (a checkpoint is expected)."""
        last = name.rsplit(".", 1)[-1]
        if last == "scale":
            return torch.full(shape, 1e-4 if name.startswith("crosstransformer") else float(self._k["dconv_init"]))
        if last == "weight" and len(shape) == 1:
            return torch.ones(shape)
        return torch.zeros(shape)

    def _config(self, chunk):
        k = self._k
        return N.SesaHtdemucsConfig(
            chunk_size=int(chunk), audio_channels=self.audio_channels, n_sources=len(self.sources),
            channels=int(k["channels"]), channels_time=int(k["channels_time"] or 0), growth=int(k["growth"]),
            nfft=int(k["nfft"]), depth=int(k["depth"]), kernel_size=int(k["kernel_size"]), stride=int(k["stride"]),
            context=int(k["context"]), context_enc=int(k["context_enc"]), norm_starts=int(k["norm_starts"]),
            rewrite=int(bool(k["rewrite"])), cac=int(bool(k["cac"])), num_subbands=int(k["num_subbands"]),
            dconv_mode=int(k["dconv_mode"]), dconv_depth=int(k["dconv_depth"]), dconv_comp=int(k["dconv_comp"]),
            bottom_channels=int(k["bottom_channels"] or 0), t_layers=int(k["t_layers"]), t_heads=int(k["t_heads"]),
            t_norm_in=int(bool(k["t_norm_in"])), t_norm_first=int(bool(k["t_norm_first"])),
            t_norm_out=int(bool(k["t_norm_out"])), t_layer_scale=int(bool(k["t_layer_scale"])),
            t_gelu=int(bool(k["t_gelu"])), t_cross_first=int(bool(k["t_cross_first"])),
            t_hidden_scale=float(k["t_hidden_scale"]), freq_emb=float(k["freq_emb"] or 0.0),
            emb_scale=float(k["emb_scale"]), t_max_period=float(k["t_max_period"]),
            t_weight_pos_embed=float(k["t_weight_pos_embed"]),
            precision={"bf16x3": N.SESA_PREC_BF16X3, "bf16": N.SESA_PREC_BF16,
                       "fp16mix": N.SESA_PREC_F16MIX}[self.precision])

    def _out_shape(self, B, ch, L):
        return (B, len(self.sources), ch, L)

    @torch.no_grad()
    def forward(self, mix):
        """HTDemucs.forward (:548-693).  use_train_segment (eval): a shorter mix is zero-padded to the
        training length and the output cropped back (:551-560, :691-692)."""
        L = mix.shape[-1]
        if self._k["use_train_segment"]:
            tl = int(self.segment * self.samplerate)
            if L < tl:
                return super().forward(torch.nn.functional.pad(mix, (0, tl - L)))[..., :L]
        return super().forward(mix)


def get_model(config, precision="bf16x3"):
    """models/demucs4ht.py:696-711 get_model (htdemucs only)."""
    if config.model != "htdemucs":
        raise NotImplementedError(f"model '{config.model}' (demucs / hdemucs) has no MI355X-native engine")
    extra = dict(sources=list(config.training.instruments), audio_channels=config.training.channels,
                 samplerate=config.training.samplerate, segment=config.training.segment)
    return HTDemucs(**extra, **dict(config.htdemucs), precision=precision)
