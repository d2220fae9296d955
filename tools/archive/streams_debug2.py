"""Diagnostic 2: demix_sharded(streams=2) vs streams=1 -- where do the outputs differ?"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "sesa-audio-separation_amd"), os.path.join(REPO, "tests")]
from conftest import CONFIGS  # noqa: E402
from sesa.config import load_config  # noqa: E402
from sesa.parallel import local_accumulate_device, shard_plan  # noqa: E402
from sesa.utils import get_model_from_config  # noqa: E402
from sesa.weights import synth_state_dict  # noqa: E402

dev = torch.device("cuda:0")
m, c = get_model_from_config("mdx23c", os.path.join(CONFIGS, "config_mdx23c_small.yaml"))
m.load_state_dict(synth_state_dict(m, affine="random"), strict=True)
rng = np.random.default_rng(2)
mix = torch.from_numpy((0.1 * rng.standard_normal((2, 400000))).astype(np.float32)).to(dev)
plan = shard_plan(c, 400000, 1)
rows = 4
l1 = local_accumulate_device(c, m, mix, plan, 0, rows, 3, 1)
l1b = local_accumulate_device(c, m, mix, plan, 0, rows, 3, 1)
torch.cuda.synchronize()
print("streams1 vs streams1:", float((l1 - l1b).abs().max()))
for s in (2, 3):
    l2 = local_accumulate_device(c, m, mix, plan, 0, rows, 3, s)
    torch.cuda.synchronize()
    d = (l1 - l2).abs().amax(0)
    bad = torch.nonzero(d > 1e-6).flatten()
    print(f"streams {s}: max diff {float(d.max()):.3e}; differing samples {bad.numel()}",
          "first/last", bad[:5].tolist(), bad[-5:].tolist() if bad.numel() else [])
    starts = [g[0] for g in plan["flat"]]
    print("chunk starts", starts[:12], "C", plan["chunk"])
