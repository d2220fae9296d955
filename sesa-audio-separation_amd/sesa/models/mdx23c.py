"""MDX23C TFC-TDF-v3 on the native MI355X forward (libsesa ``sesa_mdx23c_*``).

Drop-in for ``models/mdx23c_tfc_tdf_v3.py:141-242`` (``TFC_TDF_net``): same constructor
argument (the model config), same parameter names/shapes (``named_parameters`` /
``state_dict`` / ``load_state_dict`` keyed exactly like the reference, so released checkpoints
load unchanged), same call signature ``model(x[B,2,C]) -> [B,n_instr,2,C]`` (``[B,2,C]`` for a
single target instrument, :236-240); a ``torch.nn.Module`` (sesa/models/native.py).  The forward
runs entirely in libsesa on the current HIP stream; weights are packed once per device on first use
and repacked when a parameter changes.
"""
import torch

from .. import _native as N
from ..config import prefer_target_instrument
from .native import NativeModule


def _cfg_get(cfg, *path, default=None):
    cur = cfg
    for p in path:
        if cur is None:
            return default
        cur = cur[p] if isinstance(cur, dict) and p in cur else getattr(cur, p, None)
    return default if cur is None else cur


class TFC_TDF_net(NativeModule):
    """Reference-compatible MDX23C module (torch.nn.Module) backed by the native HIP forward."""

    _prefix = "mdx23c"
    # fp16 / fp16w2: the TFC 3x3 convs of the T >= 32 levels on fp16 MFMA (include/sesa.h SESA_PREC_F16*);
    # fp16mix: per level as sesa_mdx23c_set_f16_plan says (default: fp16 except the encoder level-1 convs)
    _precisions = ("bf16x3", "bf16", "fp16w2", "fp16", "fp16mix")
    _amp_precision = "fp16mix"  # --enable_amp: fp16 TFC convs except the encoder level-1 ones (every fixture <= 1e-4)
    _prec_codes = {"bf16x3": N.SESA_PREC_BF16X3, "bf16": N.SESA_PREC_BF16, "fp16w2": N.SESA_PREC_F16W2,
                   "fp16": N.SESA_PREC_F16, "fp16mix": N.SESA_PREC_F16MIX}

    def __init__(self, config, precision="bf16x3"):
        super().__init__(precision)
        self.config = config
        m, a = config.model, config.audio
        if str(m.norm) != "InstanceNorm" or str(m.act) != "gelu":
            raise N.SesaError(f"mdx23c: only norm=InstanceNorm, act=gelu are implemented "
                              f"(got {m.norm}, {m.act})")
        self.num_target_instruments = len(prefer_target_instrument(config))
        self.num_subbands = m.num_subbands
        sc = list(m.scale)
        self._ccfg = dict(
            chunk_size=int(a.chunk_size), dim_f=int(a.dim_f), dim_t=int(a.dim_t), hop_length=int(a.hop_length),
            n_fft=int(a.n_fft), audio_channels=int(a.num_channels), num_subbands=int(m.num_subbands),
            num_scales=int(m.num_scales), num_blocks_per_scale=int(m.num_blocks_per_scale),
            num_channels=int(m.num_channels), growth=int(m.growth), bottleneck_factor=int(m.bottleneck_factor),
            scale_t=int(sc[0]), scale_f=int(sc[1]), num_instruments=self.num_target_instruments)
        from .mdx23c_shapes import param_shapes
        shapes = dict(param_shapes(self._ccfg))
        h = self._create(self._ccfg["chunk_size"])
        try:
            names = [n for n, _ in self._native_registry(h)]
        finally:
            self._fn("destroy")(h)
        self._register_params([(n, shapes[n]) for n in names])

    def _config(self, chunk):
        return N.SesaMdx23cConfig(**self._ccfg,
                                  precision=self._prec_codes[self.precision])

    def workspace_bytes(self, batch, chunk=None):
        # not cached: the size depends on the precision (bf16x3 adds lo planes) and on the process-wide
        # conv3x3 variant as well as on the batch; the host-side dry run costs well under a millisecond
        return super().workspace_bytes(batch, self._ccfg["chunk_size"])

    def _out_shape(self, B, ch, C):
        return (B, self.num_target_instruments, ch, C)

    def _post(self, out):
        return out if self.num_target_instruments > 1 else out[:, 0]

    @torch.no_grad()
    def forward(self, x):
        if isinstance(x, torch.Tensor) and x.is_cuda:
            B, ch, C = x.shape
            if C != self._ccfg["chunk_size"] or ch != self._ccfg["audio_channels"]:
                raise N.SesaError(f"TFC_TDF_net.forward: expected [B,{self._ccfg['audio_channels']},"
                                  f"{self._ccfg['chunk_size']}], got {list(x.shape)}")
        return super().forward(x)
