"""SCNet on the native MI355X forward (libsesa ``sesa_scnet_*``).

Drop-in for ``models/scnet/scnet.py:239-373`` (``SCNet``): constructed from ``**config.model``
exactly like the reference registry (``utils.py:119-121``), same ``state_dict`` keys / shapes, same
call ``model(x[B, ch, L]) -> [B, n_sources, ch, L]``.  The whole forward -- normalized STFT, the
sparse down-sampling encoder (band convs, ConvolutionModules, global 3x3 convs), the dual-path
bi-LSTM separation net with its rfft/irfft feature conversions, the fusion / sparse up-sampling
decoder and the iSTFT -- runs in libsesa (sesa_scnet.hip) on the current HIP stream.  No CPU
fallback.
"""
import ctypes

import torch

from .. import _native as N
from .native import NativeModule


class SCNet(NativeModule):
    """Reference-compatible SCNet module (torch.nn.Module) backed by the native HIP forward."""

    _prefix = "scnet"
    # fp16mix: the token GEMMs (3x3 convs, LSTM input projections, dual-path Linears) on one fp16 MFMA pass;
    # the LSTM recurrence bf16x3, the VALU kernels fp32
    _precisions = ("bf16x3", "bf16", "fp16mix")
    _amp_precision = "fp16mix"  # --enable_amp (the reference's AMP is fp16 autocast): 9.7e-6 full chunk

    def __init__(self, sources=("drums", "bass", "other", "vocals"), audio_channels=2, dims=(4, 32, 64, 128),
                 nfft=4096, hop_size=1024, win_size=4096, normalized=True, band_SR=(0.175, 0.392, 0.433),
                 band_stride=(1, 4, 16), band_kernel=(3, 4, 16), conv_depths=(3, 2, 1), compress=4, conv_kernel=3,
                 num_dplayer=6, expand=1, precision="bf16x3"):
        super().__init__(precision)
        self.sources = list(sources)
        self.audio_channels = int(audio_channels)
        self.dims = [int(d) for d in dims]
        self.hop_length = int(hop_size)
        self._kw = dict(n_fft=int(nfft), hop_size=int(hop_size), win_size=int(win_size), normalized=bool(normalized),
                        band_SR=[float(v) for v in band_SR], band_stride=[int(v) for v in band_stride],
                        band_kernel=[int(v) for v in band_kernel], conv_depths=[int(v) for v in conv_depths],
                        compress=compress, conv_kernel=int(conv_kernel), num_dplayer=int(num_dplayer),
                        expand=int(expand))
        # GroupNorm gammas (the only 1-D weights) default to 1
        self._register_params(self._shapes(), lambda n, s: torch.ones(s) if len(s) == 1 and n.endswith("weight")
                              else torch.zeros(s))

    # ---- parameter registry (reference state_dict order, scnet.py:280-323) ----
    def _shapes(self):
        k, dims, nsrc = self._kw, self.dims, len(self.sources)
        kern = k["conv_kernel"]
        out = []
        for i in range(len(dims) - 1):
            cin, cout = dims[i], dims[i + 1]
            p = f"encoder.{i}"
            for b in range(3):
                out += [(f"{p}.SDlayer.convs.{b}.weight", (cout, cin, k["band_kernel"][b], 1)),
                        (f"{p}.SDlayer.convs.{b}.bias", (cout,))]
            hid = int(cout / k["compress"])
            for b, depth in enumerate(k["conv_depths"]):
                for li in range(abs(depth)):
                    q = f"{p}.conv_modules.{b}.layers.{li}"
                    out += [(f"{q}.0.weight", (cout,)), (f"{q}.0.bias", (cout,)),
                            (f"{q}.1.weight", (2 * hid, cout, kern)), (f"{q}.1.bias", (2 * hid,)),
                            (f"{q}.3.weight", (hid, 1, kern)), (f"{q}.3.bias", (hid,)),
                            (f"{q}.4.weight", (hid,)), (f"{q}.4.bias", (hid,)),
                            (f"{q}.6.weight", (cout, hid, 1)), (f"{q}.6.bias", (cout,))]
            out += [(f"{p}.globalconv.weight", (cout, cout, 3, 3)), (f"{p}.globalconv.bias", (cout,))]
        n_lv = len(dims) - 1
        for j in range(n_lv):
            i = n_lv - 1 - j
            c = dims[i + 1]
            co = dims[i] if i != 0 else dims[i] * nsrc
            p = f"decoder.{j}"
            out += [(f"{p}.0.conv.weight", (2 * c, 2 * c, 3, 3)), (f"{p}.0.conv.bias", (2 * c,))]
            for b in range(3):
                out += [(f"{p}.1.convtrs.{b}.weight", (c, co, k["band_kernel"][b], 1)),
                        (f"{p}.1.convtrs.{b}.bias", (co,))]
        for i in range(k["num_dplayer"]):
            d = dims[-1] * (2 if i % 2 == 1 else 1)
            H = d * k["expand"]
            p = f"separation_net.dp_modules.{i}"
            for li in range(2):
                for sfx in ("", "_reverse"):
                    q = f"{p}.lstm_layers.{li}"
                    out += [(f"{q}.weight_ih_l0{sfx}", (4 * H, d)), (f"{q}.weight_hh_l0{sfx}", (4 * H, H)),
                            (f"{q}.bias_ih_l0{sfx}", (4 * H,)), (f"{q}.bias_hh_l0{sfx}", (4 * H,))]
            for li in range(2):
                out += [(f"{p}.linear_layers.{li}.weight", (d, 2 * H)), (f"{p}.linear_layers.{li}.bias", (d,))]
            for li in range(2):
                out += [(f"{p}.norm_layers.{li}.weight", (d,)), (f"{p}.norm_layers.{li}.bias", (d,))]
        return out

    # ---- native config ----
    def _config(self, chunk):
        k = self._kw
        self._keep = (ctypes.c_int * len(self.dims))(*self.dims)
        return N.SesaScnetConfig(
            chunk_size=int(chunk), audio_channels=self.audio_channels, n_sources=len(self.sources), n_fft=k["n_fft"],
            hop_size=k["hop_size"], win_size=k["win_size"], normalized=int(k["normalized"]), n_dims=len(self.dims),
            dims=self._keep, band_sr=(ctypes.c_double * 3)(*k["band_SR"]),
            band_stride=(ctypes.c_int * 3)(*k["band_stride"]), band_kernel=(ctypes.c_int * 3)(*k["band_kernel"]),
            conv_depths=(ctypes.c_int * 3)(*k["conv_depths"]), compress=int(k["compress"]),
            conv_kernel=k["conv_kernel"], num_dplayer=k["num_dplayer"], expand=k["expand"],
            precision={"bf16x3": N.SESA_PREC_BF16X3, "bf16": N.SESA_PREC_BF16,
                       "fp16mix": N.SESA_PREC_F16MIX}[self.precision])

    def _out_shape(self, B, ch, L):
        if ch != self.audio_channels:
            raise AssertionError(f"SCNet expects {self.audio_channels} audio channels, got {ch}")
        return (B, len(self.sources), ch, L)
