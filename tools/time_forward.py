"""Quick timing of the native MDX23C forward at a given batch (diagnostic, not the bench)."""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "sesa-audio-separation_amd"))
import torch  # noqa: E402

from sesa.utils import get_model_from_config  # noqa: E402
from sesa.weights import synth_state_dict  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=4)
ap.add_argument("--iters", type=int, default=5)
ap.add_argument("--precision", default="bf16x3")
ap.add_argument("--config", default="config_vocals_mdx23c.yaml")
a = ap.parse_args()
m, c = get_model_from_config("mdx23c", os.path.join(REPO, "sesa-audio-separation_amd/sesa/configs", a.config))
m.load_state_dict(synth_state_dict(m), strict=True)
m.set_precision(a.precision)
x = 0.1 * torch.randn(a.batch, 2, c.audio.chunk_size, device="cuda")
m(x)
torch.cuda.synchronize()
t = time.time()
for _ in range(a.iters):
    m(x)
torch.cuda.synchronize()
dt = (time.time() - t) / a.iters
flop = 2.4341e12 * a.batch
print(f"batch {a.batch} {a.precision}: {dt*1e3:.1f} ms/forward, {dt/a.batch*1e3:.1f} ms/chunk, "
      f"{flop/dt/1e12:.1f} TFLOP/s algorithmic, RTF(ov4) {a.batch*65280/44100/dt:.1f}x")
