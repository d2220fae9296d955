"""Inference backend: drop-in for ``pytorch_backend.py`` (PyTorchBackend :19-332,
create_inference_session :492-536).

The reference backend wraps an nn.Module with device flags, fp16 autocast and torch.compile /
jit / channels_last modes.  Here the model is a native libsesa network; the optimisation modes
are accepted for CLI compatibility and map onto what exists on MI355X:

* ``enable_amp``  -> the model's throughput precision (``_amp_precision``) instead of the default
  3-pass bf16x3 parity precision: MDX23C ``fp16mix`` (its TFC 3x3 convs on one fp16 MFMA pass except the
  encoder level-1 ones: <= 5.3e-5 RMS on every full-chunk golden up to 0.3-RMS input -- the reference's AMP
  is fp16 autocast, :308-311, 1.35e-4 RMS), BS- / Mel-Band-Roformer ``fp16`` (QKV / out / FF Linears and
  attention on fp16 MFMA), SCNet / HTDemucs ``fp16mix`` (SCNet: 3x3 convs, LSTM input projections and Linears
  on one fp16 pass, the LSTM recurrence bf16x3; HTDemucs: implicit-GEMM convs, 1x1 rewrites, transformer /
  channel Linears and attention on one fp16 pass, norms and DConv fp32 / fp64); each gated at 1e-4 on the
  model's full-width golden by tests/test_amp_precision.py.
* ``optimize_mode`` ('channels_last' | 'compile' | 'jit' | 'default') -> no effect: the native
  forward already runs channels-last with fused prologues/epilogues, and there is no tracing
  compiler in the path.
* ``enable_tf32`` / ``enable_cudnn_benchmark`` -> no effect (no TF32 on gfx950, no cuDNN).

Unlike the reference there is NO CPU fallback: a device that is not a HIP GPU is an error.
"""
import torch

from ._native import SesaError


class HipBackend:
    """PyTorchBackend-compatible callable: ``backend(x[B,2,C]) -> model(x)``."""

    def __init__(self, device="cuda:0", optimize_mode="channels_last", exec_batch=None):
        if isinstance(device, torch.device):
            device = str(device)
        if not str(device).startswith("cuda"):
            raise SesaError(f"HipBackend: device {device!r} is not a HIP device; the MI355X path has no CPU fallback")
        if not torch.cuda.is_available():
            raise SesaError("HipBackend: no HIP device visible")
        self.device = device
        self.optimize_mode = optimize_mode
        self.model = None
        self.compiled_model = None
        self.use_amp = False
        self.exec_batch = exec_batch

    def optimize_model(self, model, example_input=None, use_amp=False, use_channels_last=True):
        self.model = model.eval()
        self.use_amp = bool(use_amp)
        if hasattr(model, "set_precision"):
            model.set_precision(getattr(model, "_amp_precision", "bf16") if self.use_amp else "bf16x3")
        self.compiled_model = self.model
        return self.compiled_model

    def __call__(self, x):
        if self.compiled_model is None:
            raise RuntimeError("No model has been optimized yet")
        if not x.is_cuda:
            x = x.to(self.device)
        with torch.no_grad():
            return self.compiled_model(x)


PyTorchBackend = HipBackend


def create_inference_session(model, device="cuda:0", optimize_mode="default", enable_amp=False, enable_tf32=True,
                             enable_cudnn_benchmark=True, exec_batch=None):
    """pytorch_backend.create_inference_session (:492-536).  NOTE: the default of ``enable_amp``
    is False here (parity precision); the reference CLI also passes False unless --enable_amp.
    ``exec_batch`` None: planned per track (sesa.demix.plan_exec_batch)."""
    be = HipBackend(device=device, optimize_mode=optimize_mode, exec_batch=exec_batch)
    be.optimize_model(model, use_amp=enable_amp)
    return be
