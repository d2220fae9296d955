"""Generate SCNet golden fixtures by running the REAL reference model on CPU.

Run here (not on the GPU box):  python tests/golden/make_golden_scnet.py [--full]

Imports /root/reference/models/scnet (torch only; the reference's utils-level third-party imports
are stubbed by make_golden.install_stubs()).  Weights: oracle.scnet.synth_params (name-keyed,
deterministic).  Fixtures are data only (inputs and expected outputs).

Fixtures:
  params_scnet_<tag>.json  reference state_dict() (name, shape) list
  scnet_small.npz          SCNet.forward, reduced config, batch 2 x 1 s, random GroupNorm affines
  demix_scnet_small.npz    inference_pytorch.demix_pytorch_optimized on the reduced model (2.5 s mix)
  scnet_full_chunk.npz     (--full) one 485100-sample chunk through the musdb18 config
  scnet_large_small.npz    SCNet.forward at the SCNet-large widths (dims [4, 64, 128, 256], LSTM H 256 / 512)
  scnet_wide_small.npz     SCNet.forward at dims [4, 48, 96, 192] (CM hidden 48, LSTM H 192 / 384)
"""
import argparse
import contextlib
import io
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)

import make_golden as mg  # noqa: E402
from oracle import scnet as osc  # noqa: E402


def _cfg(name):
    return osc.load_cfg(os.path.join(mg.CFG_DIR, name))


def build_ref(cfg, affine, seed=0):
    from models.scnet import SCNet
    model = SCNet(**osc.model_kwargs(cfg)).eval()
    sd = osc.synth_params(cfg, affine, seed)
    ref_keys = [(k, tuple(v.shape)) for k, v in model.state_dict().items()]
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    return model, ref_keys


def gen_params(cfg_name, tag):
    _, keys = build_ref(_cfg(cfg_name), "unit")
    with open(os.path.join(HERE, f"params_scnet_{tag}.json"), "w") as f:
        json.dump([[n, list(s)] for n, s in keys], f)


@torch.inference_mode()
def gen_forward(cfg_name, out_name, batch, seed, affine):
    cfg = _cfg(cfg_name)
    model, _ = build_ref(cfg, affine)
    C = cfg["audio"]["chunk_size"]
    x = np.stack([mg.mix_signal(seed + b, C) for b in range(batch)])
    y = model(torch.from_numpy(x)).numpy()
    mg.save(out_name, x=x, y=y, affine=np.array(affine))


@torch.inference_mode()
def gen_demix():
    import inference_pytorch as ip
    from pytorch_backend import PyTorchBackend
    cfg = _cfg("config_scnet_small.yaml")
    model, _ = build_ref(cfg, "random")
    be = PyTorchBackend(device="cpu", optimize_mode="default")
    be.compiled_model = model
    be.model = model
    be.use_amp = False
    c = mg.to_attr(json.loads(json.dumps(cfg)))
    mix = mg.mix_signal(11, 110000)
    with contextlib.redirect_stdout(io.StringIO()) as out:
        res = ip.demix_pytorch_optimized(c, be, mix, "cpu")
    prog = [ln for ln in out.getvalue().splitlines() if ln.startswith("[SESA_PROGRESS]")]
    mg.save("demix_scnet_small.npz", mix=mix, progress=np.array(prog),
            **{f"stem_{k}": v for k, v in res.items()})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--full", action="store_true")
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    mg.install_stubs()
    torch.set_num_threads(os.cpu_count())
    todo = args.only.split(",") if args.only else ["params", "fwd", "demix", "wide"]
    if "params" in todo:
        gen_params("config_musdb18_scnet.yaml", "musdb")
        gen_params("config_scnet_small.yaml", "small")
        gen_params("config_scnet_large_small.yaml", "large_small")
    if "fwd" in todo:
        gen_forward("config_scnet_small.yaml", "scnet_small.npz", 2, 61, "random")
    if "wide" in todo:
        gen_forward("config_scnet_large_small.yaml", "scnet_large_small.npz", 1, 71, "random")
        gen_forward("config_scnet_wide_small.yaml", "scnet_wide_small.npz", 2, 81, "random")
    if "demix" in todo:
        gen_demix()
    if args.full or "full" in todo:
        gen_forward("config_musdb18_scnet.yaml", "scnet_full_chunk.npz", 1, 0, "random")


if __name__ == "__main__":
    main()
