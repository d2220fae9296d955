"""MDX23C TFC-TDF-v3 on the native MI355X forward (libsesa ``sesa_mdx23c_*``).

Drop-in for ``models/mdx23c_tfc_tdf_v3.py:141-242`` (``TFC_TDF_net``): same constructor
argument (the model config), same parameter names/shapes (``named_parameters`` /
``state_dict`` / ``load_state_dict`` keyed exactly like the reference, so released checkpoints
load unchanged), same call signature ``model(x[B,2,C]) -> [B,n_instr,2,C]`` (``[B,2,C]`` for a
single target instrument, :236-240).  The forward runs entirely in libsesa on the current HIP
stream; weights are packed once per device on first use.
"""
import collections
import ctypes

import numpy as np
import torch

from .. import _native as N
from ..config import prefer_target_instrument


def _cfg_get(cfg, *path, default=None):
    cur = cfg
    for p in path:
        if cur is None:
            return default
        cur = cur[p] if isinstance(cur, dict) and p in cur else getattr(cur, p, None)
    return default if cur is None else cur


class TFC_TDF_net:
    """Reference-compatible MDX23C module backed by the native HIP forward."""

    def __init__(self, config, precision="bf16x3"):
        self.config = config
        m, a = config.model, config.audio
        if str(m.norm) != "InstanceNorm" or str(m.act) != "gelu":
            raise N.SesaError(f"mdx23c: only norm=InstanceNorm, act=gelu are implemented "
                              f"(got {m.norm}, {m.act})")
        self.num_target_instruments = len(prefer_target_instrument(config))
        self.num_subbands = m.num_subbands
        self.precision = precision
        sc = list(m.scale)
        self._ccfg = dict(
            chunk_size=int(a.chunk_size), dim_f=int(a.dim_f), dim_t=int(a.dim_t), hop_length=int(a.hop_length),
            n_fft=int(a.n_fft), audio_channels=int(a.num_channels), num_subbands=int(m.num_subbands),
            num_scales=int(m.num_scales), num_blocks_per_scale=int(m.num_blocks_per_scale),
            num_channels=int(m.num_channels), growth=int(m.growth), bottleneck_factor=int(m.bottleneck_factor),
            scale_t=int(sc[0]), scale_f=int(sc[1]), num_instruments=self.num_target_instruments)
        self._params = collections.OrderedDict()
        h = self._create_handle(precision)
        try:
            n = N.lib().sesa_mdx23c_num_params(h)
            for i in range(n):
                name = ctypes.c_char_p()
                numel = ctypes.c_int64()
                N.check(N.lib().sesa_mdx23c_param_info(h, i, ctypes.byref(name), ctypes.byref(numel)))
                self._params[name.value.decode()] = None
        finally:
            N.lib().sesa_mdx23c_destroy(h)
        from .mdx23c_shapes import param_shapes
        shapes = dict(param_shapes(self._ccfg))
        for k in self._params:
            self._params[k] = torch.zeros(shapes[k], dtype=torch.float32)
        self._handles = {}      # device index -> native handle
        self._ws = {}           # device index -> workspace tensor (largest batch seen)
        self._ws_bytes = {}     # batch -> bytes
        self._dirty = True
        self.training = False

    # ---- native handle management ----
    def _create_handle(self, precision):
        c = N.SesaMdx23cConfig(**self._ccfg, precision=N.SESA_PREC_BF16 if precision == "bf16" else N.SESA_PREC_BF16X3)
        h = ctypes.c_void_p()
        N.check(N.lib().sesa_mdx23c_create(ctypes.byref(c), ctypes.byref(h)), "sesa_mdx23c_create")
        return h

    def _handle(self, device):
        idx = device.index if device.index is not None else torch.cuda.current_device()
        if self._dirty:
            for hd in self._handles.values():
                N.lib().sesa_mdx23c_destroy(hd)
            self._handles.clear()
            self._dirty = False
        if idx not in self._handles:
            with torch.cuda.device(idx):
                h = self._create_handle(self.precision)
                for name, t in self._params.items():
                    arr = np.ascontiguousarray(t.detach().to("cpu", torch.float32).numpy())
                    N.check(N.lib().sesa_mdx23c_set_param(h, name.encode(), arr.ctypes.data, arr.size),
                            f"set_param {name}")
                N.check(N.lib().sesa_mdx23c_finalize(h, torch.cuda.current_stream().cuda_stream),
                        "sesa_mdx23c_finalize")
            self._handles[idx] = h
        return self._handles[idx]

    def set_precision(self, precision):
        if precision not in ("bf16x3", "bf16"):
            raise ValueError(precision)
        if precision != self.precision:
            self.precision = precision
            self._dirty = True
        return self

    def workspace_bytes(self, batch):
        if batch not in self._ws_bytes:
            h = self._create_handle(self.precision)
            try:
                self._ws_bytes[batch] = N.lib().sesa_mdx23c_workspace_size(h, batch)
            finally:
                N.lib().sesa_mdx23c_destroy(h)
        return self._ws_bytes[batch]

    # ---- nn.Module-like surface used by the reference callers ----
    def named_parameters(self):
        return iter(self._params.items())

    def parameters(self):
        return iter(self._params.values())

    def state_dict(self):
        return collections.OrderedDict((k, v.clone()) for k, v in self._params.items())

    def load_state_dict(self, state_dict, strict=True):
        """torch load_state_dict semantics (reference uses strict=False, inference_pytorch.py:368)."""
        missing = [k for k in self._params if k not in state_dict]
        unexpected = [k for k in state_dict if k not in self._params]
        if strict and (missing or unexpected):
            raise RuntimeError(f"Error(s) in loading state_dict for TFC_TDF_net: missing={missing} "
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

    # ---- forward ----
    def workspace(self, device, batch):
        """One workspace per device, grown to the largest batch seen and reused for smaller ones
        (the requirement is monotone in batch), so a track's short last group never reallocates."""
        idx = device.index
        need = self.workspace_bytes(batch)
        ws = self._ws.get(idx)
        if ws is None or ws.numel() < need:
            self._ws.pop(idx, None)
            self._ws[idx] = ws = torch.empty(need, dtype=torch.uint8, device=device)
        return ws

    def __call__(self, x):
        return self.forward(x)

    @torch.no_grad()
    def forward(self, x):
        if not isinstance(x, torch.Tensor) or not x.is_cuda:
            raise N.SesaError("TFC_TDF_net.forward: input must be a HIP device tensor (no CPU fallback)")
        x = x.to(torch.float32).contiguous()
        B, ch, C = x.shape
        if C != self._ccfg["chunk_size"] or ch != self._ccfg["audio_channels"]:
            raise N.SesaError(f"TFC_TDF_net.forward: expected [B,{self._ccfg['audio_channels']},"
                              f"{self._ccfg['chunk_size']}], got {list(x.shape)}")
        h = self._handle(x.device)
        ni = self.num_target_instruments
        out = torch.empty(B, ni, ch, C, device=x.device, dtype=torch.float32)
        ws = self.workspace(x.device, B)
        N.check(N.lib().sesa_mdx23c_forward(h, x.data_ptr(), B, out.data_ptr(), ws.data_ptr(), ws.numel(),
                                            torch.cuda.current_stream(x.device).cuda_stream), "sesa_mdx23c_forward")
        return out if ni > 1 else out[:, 0]

    def __del__(self):
        try:
            for hd in self._handles.values():
                N.lib().sesa_mdx23c_destroy(hd)
        except Exception:
            pass
