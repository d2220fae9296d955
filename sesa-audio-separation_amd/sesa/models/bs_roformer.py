"""BS-Roformer on the native MI355X forward (libsesa ``sesa_bsr_*``).

Drop-in for ``models/bs_roformer/bs_roformer.py:327-587`` (``BSRoformer``): constructed from
``**config.model`` exactly like the reference registry does (``utils.py:104-106``), same
``state_dict`` keys / shapes (incl. ``layers.*.rotary_embed.freqs``, so released checkpoints load
unchanged), same call ``model(x[B, ch, C]) -> [B, ch, C]`` for one stem (``[B, stems, ch, C]``
otherwise, :579-582).  The forward runs entirely in libsesa on the current HIP stream: STFT,
band split, the depth x (time, freq) rotary transformers, mask estimators, complex mask and
iSTFT (sesa_bsroformer.hip, kernels in sesa_tokgemm.hip).  No CPU fallback.
"""
import collections
import ctypes

import numpy as np
import torch

from .. import _native as N

DEFAULT_FREQS_PER_BANDS = (2,) * 24 + (4,) * 12 + (12,) * 8 + (24,) * 8 + (48,) * 8 + (128, 129)


def _freqs(dim_head, theta=10000.0):
    return (1.0 / (theta ** (torch.arange(0, dim_head, 2)[: dim_head // 2].float() / dim_head))).numpy()


class BSRoformer:
    """Reference-compatible BS-Roformer module backed by the native HIP forward."""

    def __init__(self, dim, *, depth, stereo=False, num_stems=1, time_transformer_depth=2, freq_transformer_depth=2,
                 linear_transformer_depth=0, freqs_per_bands=DEFAULT_FREQS_PER_BANDS, dim_head=64, heads=8,
                 attn_dropout=0.0, ff_dropout=0.0, flash_attn=True, dim_freqs_in=1025, stft_n_fft=2048,
                 stft_hop_length=512, stft_win_length=2048, stft_normalized=False, stft_window_fn=None,
                 mask_estimator_depth=2, multi_stft_resolution_loss_weight=1.0,
                 multi_stft_resolutions_window_sizes=(4096, 2048, 1024, 512, 256), multi_stft_hop_size=147,
                 multi_stft_normalized=False, multi_stft_window_fn=None, mlp_expansion_factor=4,
                 use_torch_checkpoint=False, skip_connection=False, chunk_size=None, precision="bf16x3"):
        if linear_transformer_depth or skip_connection or stft_normalized or stft_window_fn is not None:
            raise N.SesaError("BSRoformer: linear attention, skip connections, normalized or custom STFT windows "
                              "have no native implementation")
        self.stereo = bool(stereo)
        self.audio_channels = 2 if stereo else 1
        self.num_stems = int(num_stems)
        self.freqs_per_bands = tuple(int(f) for f in freqs_per_bands)
        if sum(self.freqs_per_bands) != stft_n_fft // 2 + 1:
            raise AssertionError(f"the number of freqs in the bands must equal {stft_n_fft // 2 + 1} based on the "
                                 f"STFT settings, but got {sum(self.freqs_per_bands)}")
        self.chunk_size = chunk_size
        self.precision = precision
        self._kw = dict(audio_channels=self.audio_channels, n_fft=int(stft_n_fft), hop_length=int(stft_hop_length),
                        win_length=int(stft_win_length), dim=int(dim), depth=int(depth), heads=int(heads),
                        dim_head=int(dim_head), time_transformer_depth=int(time_transformer_depth),
                        freq_transformer_depth=int(freq_transformer_depth), num_stems=self.num_stems,
                        mask_estimator_depth=int(mask_estimator_depth),
                        mlp_expansion_factor=int(mlp_expansion_factor))
        self._params = collections.OrderedDict((n, torch.zeros(s, dtype=torch.float32))
                                               for n, s in self.param_shapes())
        for n, t in self._params.items():
            if n.endswith("rotary_embed.freqs"):
                t.copy_(torch.from_numpy(_freqs(dim_head)))
            elif n.endswith("gamma"):
                t.fill_(1.0)
        self._handles, self._ws, self._ws_bytes = {}, {}, {}
        self._hchunk = None
        self._dirty = True
        self.training = False

    # ---- parameter registry (reference state_dict order, bs_roformer.py:372-433) ----
    def band_dims(self):
        return [2 * f * self.audio_channels for f in self.freqs_per_bands]

    def param_shapes(self):
        k = self._kw
        dim, heads, dh = k["dim"], k["heads"], k["dim_head"]
        inner, ff, hid = heads * dh, dim * 4, dim * k["mlp_expansion_factor"]
        out = []
        for i in range(k["depth"]):
            for j, dep in ((0, k["time_transformer_depth"]), (1, k["freq_transformer_depth"])):
                for l in range(dep):
                    p = f"layers.{i}.{j}.layers.{l}"
                    out += [(f"{p}.0.rotary_embed.freqs", (dh // 2,)), (f"{p}.0.norm.gamma", (dim,)),
                            (f"{p}.0.to_qkv.weight", (3 * inner, dim)), (f"{p}.0.to_gates.weight", (heads, dim)),
                            (f"{p}.0.to_gates.bias", (heads,)), (f"{p}.0.to_out.0.weight", (dim, inner)),
                            (f"{p}.1.net.0.gamma", (dim,)), (f"{p}.1.net.1.weight", (ff, dim)),
                            (f"{p}.1.net.1.bias", (ff,)), (f"{p}.1.net.4.weight", (dim, ff)),
                            (f"{p}.1.net.4.bias", (dim,))]
        out.append(("final_norm.gamma", (dim,)))
        dims = self.band_dims()
        for b, d in enumerate(dims):
            out += [(f"band_split.to_features.{b}.0.gamma", (d,)), (f"band_split.to_features.{b}.1.weight", (dim, d)),
                    (f"band_split.to_features.{b}.1.bias", (dim,))]
        for n in range(self.num_stems):
            for b, d in enumerate(dims):
                p = f"mask_estimators.{n}.to_freqs.{b}.0"
                out += [(f"{p}.0.weight", (hid, dim)), (f"{p}.0.bias", (hid,)), (f"{p}.2.weight", (2 * d, hid)),
                        (f"{p}.2.bias", (2 * d,))]
        return out

    # ---- native handles ----
    _mel = False
    _freq_indices = ()

    def _config(self, chunk):
        fpb = (ctypes.c_int * len(self.freqs_per_bands))(*self.freqs_per_bands)
        fidx = (ctypes.c_int * max(1, len(self._freq_indices)))(*self._freq_indices)
        c = N.SesaBsrConfig(chunk_size=int(chunk), n_bands=len(self.freqs_per_bands), freqs_per_bands=fpb,
                            precision=N.SESA_PREC_BF16 if self.precision == "bf16" else N.SESA_PREC_BF16X3,
                            mel=1 if self._mel else 0, n_freq_indices=len(self._freq_indices), freq_indices=fidx,
                            **self._kw)
        self._keep = (fpb, fidx)   # ctypes arrays must outlive the create call
        return c, fpb

    def _create(self, chunk):
        c, _fpb = self._config(chunk)
        h = ctypes.c_void_p()
        N.check(N.lib().sesa_bsr_create(ctypes.byref(c), ctypes.byref(h)), "sesa_bsr_create")
        return h

    def _handle(self, device, chunk):
        idx = device.index if device.index is not None else torch.cuda.current_device()
        if self._dirty or self._hchunk != chunk:
            for hd in self._handles.values():
                N.lib().sesa_bsr_destroy(hd)
            self._handles.clear()
            self._ws_bytes.clear()
            self._dirty = False
            self._hchunk = chunk
        if idx not in self._handles:
            with torch.cuda.device(idx):
                h = self._create(chunk)
                names = []
                for i in range(N.lib().sesa_bsr_num_params(h)):
                    nm = ctypes.c_char_p()
                    N.check(N.lib().sesa_bsr_param_info(h, i, ctypes.byref(nm), None))
                    names.append(nm.value.decode())
                if names != list(self._params):
                    raise N.SesaError("BSRoformer: native parameter registry differs from the Python one")
                for name, t in self._params.items():
                    arr = np.ascontiguousarray(t.detach().to("cpu", torch.float32).numpy())
                    N.check(N.lib().sesa_bsr_set_param(h, name.encode(), arr.ctypes.data, arr.size), f"set_param {name}")
                N.check(N.lib().sesa_bsr_finalize(h, torch.cuda.current_stream().cuda_stream), "sesa_bsr_finalize")
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
        need = N.lib().sesa_bsr_workspace_size(h, batch)
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
            raise RuntimeError(f"Error(s) in loading state_dict for BSRoformer: missing={missing} "
                               f"unexpected={unexpected}")
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

    def __call__(self, x, target=None):
        return self.forward(x, target)

    @torch.no_grad()
    def forward(self, raw_audio, target=None):
        if target is not None:
            raise N.SesaError("BSRoformer: the training loss branch is not part of the native inference path")
        if not isinstance(raw_audio, torch.Tensor) or not raw_audio.is_cuda:
            raise N.SesaError("BSRoformer.forward: input must be a HIP device tensor (no CPU fallback)")
        x = raw_audio.to(torch.float32)
        if x.ndim == 2:
            x = x[:, None]
        x = x.contiguous()
        B, ch, C = x.shape
        if ch != self.audio_channels:
            raise AssertionError("stereo needs to be set to True if passing in audio signal that is stereo")
        h = self._handle(x.device, C)
        out = torch.empty(B, self.num_stems, ch, C, device=x.device, dtype=torch.float32)
        ws = self.workspace(x.device, h, B)
        N.check(N.lib().sesa_bsr_forward(h, x.data_ptr(), B, out.data_ptr(), ws.data_ptr(), ws.numel(),
                                         torch.cuda.current_stream(x.device).cuda_stream), "sesa_bsr_forward")
        return out[:, 0] if self.num_stems == 1 else out

    def __del__(self):
        try:
            for hd in self._handles.values():
                N.lib().sesa_bsr_destroy(hd)
        except Exception:
            pass
