"""Diagnostic: is a native forward enqueued on a side stream identical to the same forward on the current
stream?  (tests/test_gpu_parity.py::test_side_streams_* found streams = 2 differing by ~1 %.)"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "sesa-audio-separation_amd"), os.path.join(REPO, "tests")]
from conftest import CONFIGS  # noqa: E402
from sesa.utils import get_model_from_config  # noqa: E402
from sesa.weights import synth_state_dict  # noqa: E402

dev = torch.device("cuda:0")
m, c = get_model_from_config("mdx23c", os.path.join(CONFIGS, "config_mdx23c_small.yaml"))
m.load_state_dict(synth_state_dict(m, affine="random"), strict=True)
x = torch.from_numpy((0.1 * np.random.default_rng(3).standard_normal((3, 2, c.audio.chunk_size))).astype(np.float32)).to(dev)
y0 = m(x)
y0b = m(x)
torch.cuda.synchronize()
print("main vs main:", float((y0 - y0b).abs().max()))
side = torch.cuda.Stream(dev)
side.wait_stream(torch.cuda.current_stream(dev))
with torch.cuda.stream(side):
    y1 = m(x)
torch.cuda.synchronize()
print("side vs main:", float((y1 - y0).abs().max()), "max", float(y0.abs().max()), "ws keys", len(m._ws))
# concurrent: main and side at once
with torch.cuda.stream(side):
    y2 = m(x)
y3 = m(x)
torch.cuda.synchronize()
print("concurrent side vs main:", float((y2 - y0).abs().max()), float((y3 - y0).abs().max()))
