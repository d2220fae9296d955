"""``torch.nn.Module`` shell over a libsesa network handle.

The reference models are ``nn.Module`` s (``models/*.py``): callers use ``state_dict`` /
``load_state_dict(strict=...)``, ``named_parameters``, ``.to(device)``, ``.eval()``,
``requires_grad_(False)`` and wrap them in ``nn.DataParallel`` (inference.py:202-210,
pytorch_backend.py:103-108).  ``NativeModule`` registers every parameter under its reference
``state_dict`` name as a real ``nn.Parameter`` (a module tree mirrors the dotted names), so all of
that is plain PyTorch behaviour; ``forward`` runs the native HIP network.

The packed device weights of a native handle are rebuilt whenever a parameter's storage or
version counter changes (``load_state_dict`` copies in place and bumps ``_version``; ``.to()``
swaps storages), when the precision changes, or for a new input length.  There is no CPU
fallback: ``forward`` on a CPU tensor raises.
"""
import ctypes

import numpy as np
import torch

from .. import _native as N
from .. import ops as _ops  # noqa: F401  (registers the sesa::<net>_forward custom ops)


class _Node(torch.nn.Module):
    """Intermediate node of the parameter tree; ``node[i]`` indexes numbered children like the
    reference's ModuleList / Sequential (``model.encoder[0].conv.weight``)."""

    def __getitem__(self, i):
        return self._modules[str(i)]

    def __len__(self):
        return len(self._modules)


class NativeModule(torch.nn.Module):
    """Base of the native model faces.  Subclasses set ``_prefix`` (``sesa_<prefix>_*`` entry
    points) and implement ``_config(chunk)`` (the ctypes config struct) and ``_out_shape``."""
    # forwards of one handle on several streams at once (sesa.parallel streams > 1): bit-identical to one stream for
    # this model at full size (tools/streams_check.py).  A model that is not sets it False and the
    # multi-stream loops run it on one stream.
    multi_stream_ok = True


    _prefix = None
    _precisions = ("bf16x3", "bf16")
    _amp_precision = "bf16"  # --enable_amp (sesa.backend)

    def __init__(self, precision="bf16x3"):
        super().__init__()
        self.precision = precision
        self._handles = {}
        self._ws = {}
        self._sig = None

    # ---- parameter tree -------------------------------------------------------------------
    def _register_params(self, shapes, init=None):
        """shapes: [(dotted_name, shape)] in reference state_dict order; init(name, shape) -> tensor."""
        for name, shape in shapes:
            mod = self
            parts = name.split(".")
            for p in parts[:-1]:
                if p not in mod._modules:
                    mod.add_module(p, _Node())
                mod = mod._modules[p]
            t = init(name, shape) if init else torch.zeros(shape)
            mod.register_parameter(parts[-1], torch.nn.Parameter(t.to(torch.float32), requires_grad=False))

    def param_shapes(self):
        return [(n, tuple(p.shape)) for n, p in self.named_parameters()]

    # ---- native handle ----------------------------------------------------------------------
    def _fn(self, name):
        return getattr(N.lib(), f"sesa_{self._prefix}_{name}")

    def _create(self, chunk):
        cfg = self._config(chunk)
        h = ctypes.c_void_p()
        N.check(self._fn("create")(ctypes.byref(cfg), ctypes.byref(h)), f"sesa_{self._prefix}_create")
        return h

    def _native_registry(self, h):
        out = []
        for i in range(self._fn("num_params")(h)):
            nm, numel = ctypes.c_char_p(), ctypes.c_int64()
            N.check(self._fn("param_info")(h, i, ctypes.byref(nm), ctypes.byref(numel)))
            out.append((nm.value.decode(), numel.value))
        return out

    def _signature(self, chunk):
        return (self.precision, chunk,
                tuple((p.data_ptr(), p._version) for p in self.parameters()))

    def _release(self):
        for h in self._handles.values():
            self._fn("destroy")(h)
        self._handles.clear()
        self._ws.clear()

    def _handle(self, device, chunk):
        sig = self._signature(chunk)
        if sig != self._sig:
            self._release()
            self._sig = sig
        idx = device.index
        if idx not in self._handles:
            with torch.cuda.device(idx):
                h = self._create(chunk)
                if [n for n, _ in self._native_registry(h)] != [n for n, _ in self.named_parameters()]:
                    self._fn("destroy")(h)
                    raise N.SesaError(f"{type(self).__name__}: native parameter registry differs from the module's")
                for name, t in self.named_parameters():
                    arr = np.ascontiguousarray(t.detach().to("cpu", torch.float32).numpy())
                    N.check(self._fn("set_param")(h, name.encode(), arr.ctypes.data, arr.size), f"set_param {name}")
                N.check(self._fn("finalize")(h, torch.cuda.current_stream(device).cuda_stream),
                        f"sesa_{self._prefix}_finalize")
            self._handles[idx] = h
        return self._handles[idx]

    def set_precision(self, precision):
        if precision not in self._precisions:
            raise ValueError(f"{type(self).__name__}: precision {precision!r} not in {self._precisions}")
        self.precision = precision
        return self

    def workspace(self, device, h, batch):
        """Per (device, stream) workspace: forwards enqueued on different streams may run concurrently."""
        need = self._fn("workspace_size")(h, batch)
        key = (device.index, torch.cuda.current_stream(device).cuda_stream)
        ws = self._ws.get(key)
        if ws is None or ws.numel() < need:
            self._ws.pop(key, None)
            self._ws[key] = ws = torch.empty(need, dtype=torch.uint8, device=device)
        return ws

    def workspace_bytes(self, batch, chunk):
        """Workspace of one forward of `batch` items of length `chunk` (host-side plan only)."""
        h = self._create(chunk)
        try:
            return int(self._fn("workspace_size")(h, batch))
        finally:
            self._fn("destroy")(h)

    @torch.no_grad()
    def forward(self, x):
        if not isinstance(x, torch.Tensor) or not x.is_cuda:
            raise N.SesaError(f"{type(self).__name__}.forward: input must be a HIP device tensor (no CPU fallback)")
        x = x.to(torch.float32).contiguous()
        B, ch, L = x.shape
        h = self._handle(x.device, L)
        ws = self.workspace(x.device, h, B)
        out = getattr(torch.ops.sesa, f"{self._prefix}_forward")(h.value, x, ws, list(self._out_shape(B, ch, L)))
        return self._post(out)

    def _post(self, out):
        return out

    def __del__(self):
        try:
            self._release()
        except Exception:
            pass
