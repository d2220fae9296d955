"""CPU emulation of fp16 attention (and fp16 Linears) in BS-Roformer (test infrastructure: oracle/bs_roformer.py
with operands rounded in torch), against the reference full-chunk golden.
  lin16  -- every Linear's activation and weight rounded to fp16 (as emulate_bsr_fp16.py a16w16)
  attn16 -- attention QK^T and PV on fp16 operands: q (pre-scaled by 1/8, exact), k, v rounded to fp16; the
            flash kernel's P = exp(s - m) rounded to fp16 before PV, the row sum l in fp32 of the unrounded P
  all16  -- both
Usage: python tests/emulation/emulate_bsr_attn16.py lin16 attn16 all16 [--fixture bsr_full_chunk.npz] [--mel]"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F
from torch.overrides import TorchFunctionMode

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
torch.set_num_threads(os.cpu_count())
mel = "--mel" in sys.argv
if mel:
    import oracle.mel_band_roformer as ob
    CFG = "config_mel_band_roformer_vocals.yaml"
    FX = "mbr_full_chunk.npz"
else:
    import oracle.bs_roformer as ob
    CFG = "config_bs_roformer_vocals.yaml"
    FX = "bsr_full_chunk.npz"
if "--fixture" in sys.argv:
    FX = sys.argv[sys.argv.index("--fixture") + 1]
g = np.load(os.path.join(REPO, "tests", "golden", FX))
cfg = ob.load_cfg(os.path.join(REPO, "sesa-audio-separation_amd", "sesa", "configs", CFG))
P = ob.to_torch(ob.synth_params(cfg, str(g["affine"])))


def h(t):
    return t.half().float()


def sdpa16(q, k, v, *a, **kw):
    s = (h(q * 0.125) @ h(k).transpose(-1, -2))
    m = s.amax(-1, keepdim=True)
    p = torch.exp(s - m)
    return (h(p) @ h(v)) / p.sum(-1, keepdim=True)


class Mode(TorchFunctionMode):
    def __init__(self, lin):
        super().__init__()
        self.lin = lin

    def __torch_function__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if self.lin and getattr(func, "__name__", "") in ("matmul", "__matmul__") and len(args) == 2 and args[1].dim() == 2:
            return func(h(args[0]), h(args[1]), **kwargs)
        return func(*args, **kwargs)


for mode in [m for m in sys.argv[1:] if m in ("none", "lin16", "attn16", "all16")]:
    x = torch.from_numpy(g["x"])
    orig = F.scaled_dot_product_attention
    try:
        if mode in ("attn16", "all16"):
            F.scaled_dot_product_attention = sdpa16
        with torch.inference_mode(), Mode(mode in ("lin16", "all16")):
            y = ob.forward(P, cfg, x).numpy()
    finally:
        F.scaled_dot_product_attention = orig
    d = y.astype(np.float64) - g["y"]
    r = float(np.sqrt(np.mean(d ** 2)))
    print(f"{FX} {mode}: rms {r:.3e} rel {r / float(np.sqrt(np.mean(g['y'].astype(np.float64) ** 2))):.3e} "
          f"max {np.abs(d).max():.3e}", flush=True)
