"""Round 6: does a full-size track separate bit-identically with forwards on two streams?  (tests/test_bsr.py's 4-min
fp16 case differed once demix_device ran two streams.)  Runs demix_device on the 4-min track at streams 1, 1 again
(run-to-run determinism), 2, and 2 with every per-stream workspace zeroed before each forward (stale-workspace
reads), and prints the max |diff| / differing samples of each against the first run.

  python tools/streams_check.py MODEL PRECISION [EXEC_BATCH]
"""
import contextlib
import io
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "sesa-audio-separation_amd"), os.path.join(REPO, "tests")]
from conftest import CONFIGS  # noqa: E402
from sesa.demix import demix_device  # noqa: E402
from sesa.models import native as nat  # noqa: E402
from sesa.utils import get_model_from_config  # noqa: E402
from sesa.weights import synth_model_state, synth_state_dict  # noqa: E402

CFG = {"mdx23c": "config_vocals_mdx23c.yaml", "bs_roformer": "config_bs_roformer_vocals.yaml",
       "htdemucs": "config_musdb18_htdemucs.yaml", "scnet": "config_musdb18_scnet.yaml"}
kind, prec = sys.argv[1], sys.argv[2]
eb = int(sys.argv[3]) if len(sys.argv) > 3 else 4
dev = torch.device("cuda:0")
m, c = get_model_from_config(kind, os.path.join(CONFIGS, CFG[kind]))
m.load_state_dict(synth_state_dict(m) if kind == "mdx23c" else synth_model_state(m, affine="random"), strict=True)
m.set_precision(prec)
m.multi_stream_ok = True   # measure the raw behaviour (the product loops clamp a model that sets it False to one stream)
L = 240 * 44100
mix = torch.from_numpy((0.1 * np.random.default_rng(0).standard_normal((2, L))).astype(np.float32)).to(dev)
_orig_ws = nat.NativeModule.workspace


def zeroed_ws(self, device, h, batch):
    ws = _orig_ws(self, device, h, batch)
    ws.zero_()
    return ws


def run(streams, zero=False):
    nat.NativeModule.workspace = zeroed_ws if zero else _orig_ws
    with contextlib.redirect_stdout(io.StringIO()):
        y = demix_device(c, m, mix, dev, exec_batch=eb, streams=streams)
    torch.cuda.synchronize()
    nat.NativeModule.workspace = _orig_ws
    return y


ref = run(1)
for name, kw in (("streams1_again", dict(streams=1)), ("streams2", dict(streams=2)),
                 ("streams2_zeroed_ws", dict(streams=2, zero=True)), ("streams1_zeroed_ws", dict(streams=1, zero=True)),
                 ("streams2_again", dict(streams=2))):
    y = run(**kw)
    d = (y - ref).abs()
    print(f"RESULT {kind} {prec} eb {eb} {name}: max|diff| {d.max().item():.3e}, differing samples "
          f"{int((d > 0).sum().item())} of {d.numel()}", flush=True)
