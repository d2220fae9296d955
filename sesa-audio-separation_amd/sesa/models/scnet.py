"""SCNet on the native MI355X forward (libsesa ``sesa_scnet_*``).

Drop-in for ``models/scnet/scnet.py:239-373`` (``SCNet``): constructed from ``**config.model``
exactly like the reference registry (``utils.py:119-121``), same ``state_dict`` keys / shapes, same
call ``model(x[B, ch, L]) -> [B, n_sources, ch, L]``.  The whole forward -- normalized STFT, the
sparse down-sampling encoder (band convs, ConvolutionModules, global 3x3 convs), the dual-path
bi-LSTM separation net with its rfft/irfft feature conversions, the fusion / sparse up-sampling
decoder and the iSTFT -- runs in libsesa (sesa_scnet.hip) on the current HIP stream.  No CPU
fallback.
"""
import collections
import ctypes

import numpy as np
import torch

from .. import _native as N


class SCNet:
    """Reference-compatible SCNet module backed by the native HIP forward."""

    def __init__(self, sources=("drums", "bass", "other", "vocals"), audio_channels=2, dims=(4, 32, 64, 128),
                 nfft=4096, hop_size=1024, win_size=4096, normalized=True, band_SR=(0.175, 0.392, 0.433),
                 band_stride=(1, 4, 16), band_kernel=(3, 4, 16), conv_depths=(3, 2, 1), compress=4, conv_kernel=3,
                 num_dplayer=6, expand=1, precision="bf16x3"):
        self.sources = list(sources)
        self.audio_channels = int(audio_channels)
        self.dims = [int(d) for d in dims]
        self.hop_length = int(hop_size)
        self.precision = precision
        self._kw = dict(n_fft=int(nfft), hop_size=int(hop_size), win_size=int(win_size), normalized=bool(normalized),
                        band_SR=[float(v) for v in band_SR], band_stride=[int(v) for v in band_stride],
                        band_kernel=[int(v) for v in band_kernel], conv_depths=[int(v) for v in conv_depths],
                        compress=compress, conv_kernel=int(conv_kernel), num_dplayer=int(num_dplayer),
                        expand=int(expand))
        self._params = collections.OrderedDict((n, torch.zeros(s, dtype=torch.float32))
                                               for n, s in self.param_shapes())
        for n, t in self._params.items():  # GroupNorm gammas (the only 1-D weights) default to 1
            if t.ndim == 1 and n.endswith("weight"):
                t.fill_(1.0)
        self._handles, self._ws = {}, {}
        self._hchunk = None
        self._dirty = True
        self.training = False

    # ---- parameter registry (reference state_dict order, scnet.py:280-323) ----
    def param_shapes(self):
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

    # ---- native handle (one per device, rebuilt when weights / chunk size / precision change) ----
    def _create(self, chunk):
        k = self._kw
        dims = (ctypes.c_int * len(self.dims))(*self.dims)
        cfg = N.SesaScnetConfig(
            chunk_size=int(chunk), audio_channels=self.audio_channels, n_sources=len(self.sources), n_fft=k["n_fft"],
            hop_size=k["hop_size"], win_size=k["win_size"], normalized=int(k["normalized"]), n_dims=len(self.dims),
            dims=dims, band_sr=(ctypes.c_double * 3)(*k["band_SR"]), band_stride=(ctypes.c_int * 3)(*k["band_stride"]),
            band_kernel=(ctypes.c_int * 3)(*k["band_kernel"]), conv_depths=(ctypes.c_int * 3)(*k["conv_depths"]),
            compress=int(k["compress"]), conv_kernel=k["conv_kernel"], num_dplayer=k["num_dplayer"],
            expand=k["expand"], precision=N.SESA_PREC_BF16X3 if self.precision == "bf16x3" else N.SESA_PREC_BF16)
        h = ctypes.c_void_p()
        N.check(N.lib().sesa_scnet_create(ctypes.byref(cfg), ctypes.byref(h)), "sesa_scnet_create")
        return h

    def _handle(self, device, chunk):
        idx = device.index
        if self._dirty or self._hchunk != chunk:
            for hd in self._handles.values():
                N.lib().sesa_scnet_destroy(hd)
            self._handles.clear()
            self._dirty = False
            self._hchunk = chunk
        if idx not in self._handles:
            with torch.cuda.device(idx):
                h = self._create(chunk)
                names = []
                for i in range(N.lib().sesa_scnet_num_params(h)):
                    nm = ctypes.c_char_p()
                    N.check(N.lib().sesa_scnet_param_info(h, i, ctypes.byref(nm), None))
                    names.append(nm.value.decode())
                if names != list(self._params):
                    raise N.SesaError("SCNet: native parameter registry differs from the Python one")
                for name, t in self._params.items():
                    arr = np.ascontiguousarray(t.detach().to("cpu", torch.float32).numpy())
                    N.check(N.lib().sesa_scnet_set_param(h, name.encode(), arr.ctypes.data, arr.size),
                            f"set_param {name}")
                N.check(N.lib().sesa_scnet_finalize(h, torch.cuda.current_stream().cuda_stream), "sesa_scnet_finalize")
            self._handles[idx] = h
        return self._handles[idx]

    def set_precision(self, precision):
        if precision not in ("bf16x3", "bf16"):
            raise ValueError(precision)
        if precision != self.precision:
            self.precision = precision
            self._dirty = True
        return self

    def workspace(self, device, h, batch):
        need = N.lib().sesa_scnet_workspace_size(h, batch)
        ws = self._ws.get(device.index)
        if ws is None or ws.numel() < need:
            self._ws.pop(device.index, None)
            self._ws[device.index] = ws = torch.empty(need, dtype=torch.uint8, device=device)
        return ws

    # ---- nn.Module-like surface ----
    def named_parameters(self):
        return iter(self._params.items())

    def parameters(self):
        return iter(self._params.values())

    def state_dict(self):
        return collections.OrderedDict((k, v.clone()) for k, v in self._params.items())

    def load_state_dict(self, state_dict, strict=True):
        missing = [k for k in self._params if k not in state_dict]
        unexpected = [k for k in state_dict if k not in self._params]
        if strict and (missing or unexpected):
            raise RuntimeError(f"Error(s) in loading state_dict for SCNet: missing={missing} unexpected={unexpected}")
        for k, v in state_dict.items():
            if k in self._params:
                v = torch.as_tensor(v).to(torch.float32)
                if tuple(v.shape) != tuple(self._params[k].shape):
                    raise RuntimeError(f"size mismatch for {k}: copying a param with shape {tuple(v.shape)}, "
                                       f"the shape in current model is {tuple(self._params[k].shape)}")
                self._params[k] = v.detach().cpu().clone()
        self._dirty = True
        return collections.namedtuple("IncompatibleKeys", "missing_keys unexpected_keys")(missing, unexpected)

    def eval(self):
        return self

    def train(self, mode=True):
        return self

    def to(self, *args, **kwargs):
        return self

    def requires_grad_(self, flag=False):
        return self

    def __call__(self, x):
        return self.forward(x)

    @torch.no_grad()
    def forward(self, x):
        if not isinstance(x, torch.Tensor) or not x.is_cuda:
            raise N.SesaError("SCNet.forward: input must be a HIP device tensor (no CPU fallback)")
        x = x.to(torch.float32).contiguous()
        B, ch, L = x.shape
        if ch != self.audio_channels:
            raise AssertionError(f"SCNet expects {self.audio_channels} audio channels, got {ch}")
        h = self._handle(x.device, L)
        out = torch.empty(B, len(self.sources), ch, L, device=x.device, dtype=torch.float32)
        ws = self.workspace(x.device, h, B)
        N.check(N.lib().sesa_scnet_forward(h, x.data_ptr(), B, out.data_ptr(), ws.data_ptr(), ws.numel(),
                                           torch.cuda.current_stream(x.device).cuda_stream), "sesa_scnet_forward")
        return out

    def __del__(self):
        try:
            for hd in self._handles.values():
                N.lib().sesa_scnet_destroy(hd)
        except Exception:
            pass
