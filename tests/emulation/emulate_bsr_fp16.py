"""CPU emulation of fp16 Linears in BS-Roformer (test infrastructure; oracle/bs_roformer.py with every
activation x weight matmul's activation rounded to fp16, weights exact (a16w32) or fp16 (a16w16)), against
the reference full-chunk golden.  Results: a16w32 4.5e-6, a16w16 7.0e-6."""
import os, sys, numpy as np, torch
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import oracle.bs_roformer as ob
from torch.overrides import TorchFunctionMode
torch.set_num_threads(8)
g = np.load(REPO + '/tests/golden/bsr_full_chunk.npz')
cfg = ob.load_cfg(REPO + '/sesa-audio-separation_amd/sesa/configs/config_bs_roformer_vocals.yaml')
P = ob.to_torch(ob.synth_params(cfg, str(g["affine"])))
class Mode(TorchFunctionMode):
    def __init__(self, wround): super().__init__(); self.wround = wround
    def __torch_function__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if getattr(func, "__name__", "") in ("matmul", "__matmul__") and len(args) == 2 and args[1].dim() == 2:
            a, w = args
            a = a.half().float()
            if self.wround: w = w.half().float()
            return func(a, w, **kwargs)
        return func(*args, **kwargs)
for mode in sys.argv[1:]:
    x = torch.from_numpy(g["x"])
    with torch.inference_mode():
        if mode == 'none':
            y = ob.forward(P, cfg, x).numpy()
        else:
            with Mode(mode == 'a16w16'):
                y = ob.forward(P, cfg, x).numpy()
    print(mode, f"{float(np.sqrt(np.mean((y.astype(np.float64) - g['y']) ** 2))):.3e}", 'ref rms', f"{float(np.sqrt(np.mean(g['y'].astype(np.float64)**2))):.3e}", flush=True)
