"""Generate HTDemucs golden fixtures by running the REAL reference model class on CPU.

Run here (not on the GPU box):  python tests/golden/make_golden_htdemucs.py [--full]

Imports /root/reference/models/demucs4ht.py (HTDemucs: _spec / _magnitude / encoder-decoder loop /
_mask / _ispec as the reference wrote them).  Its third-party imports are absent here: ``demucs``
(unpinned) is replaced by the restatement in oracle/_stubs/demucs (layers, cross transformer,
spectro) and ``openunmix`` by a placeholder that is never called for cac configs -- parity at that
layer boundary is UNPINNED.  Weights: name-keyed synthetic (below).

Fixtures:
  params_htdemucs_<tag>.json   reference state_dict() (name, shape) list
  htdemucs_small.npz           HTDemucs.forward, reduced config, batch 2 x 2 s segment
  htdemucs_full_segment.npz    (--full) one 485100-sample segment through the musdb18 config
"""
import argparse
import json
import math
import os
import sys

import numpy as np
import torch
import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle", "_stubs"))

import make_golden as mg  # noqa: E402


def _cfg(name):
    with open(os.path.join(mg.CFG_DIR, name)) as f:
        return yaml.safe_load(f)


def synth_params(shapes, affine="random"):
    """Name-keyed weights (oracle/weights.py scheme): >=2-D tensors U(+-1/sqrt(prod(shape[1:]))),
    biases U(+-1/sqrt(fan_in of their weight)), norm gammas U(0.5, 1.5) / betas U(-0.2, 0.2),
    LayerScale ``scale`` U(0.1, 0.3) (so the residual branches matter in the fixtures).
    ``shapes``: dict name -> shape in state_dict order."""
    from oracle.weights import param_rng, synth_param
    out = {}
    for name, shape in shapes.items():
        head, _, last = name.rpartition(".")
        wname = f"{head}.{last.replace('bias', 'weight')}" if "bias" in last else None
        if last == "scale":
            out[name] = param_rng(name).uniform(0.1, 0.3, size=shape).astype(np.float32)
        elif wname and wname in shapes and len(shapes[wname]) >= 2:
            b = 1.0 / math.sqrt(int(np.prod(shapes[wname][1:])))
            out[name] = param_rng(name).uniform(-b, b, size=shape).astype(np.float32)
        else:
            out[name] = synth_param(name, shape, affine)
    return out


def build_ref(cfg, affine):
    from models.demucs4ht import HTDemucs
    extra = dict(sources=cfg["training"]["instruments"], audio_channels=cfg["training"]["channels"],
                 samplerate=cfg["training"]["samplerate"], segment=cfg["training"]["segment"])
    model = HTDemucs(**extra, **cfg["htdemucs"]).eval()   # models/demucs4ht.py:696-711 get_model
    keys = [(k, tuple(v.shape)) for k, v in model.state_dict().items()]
    sd = synth_params(dict(keys), affine)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    return model, keys


def gen_params(cfg_name, tag):
    _, keys = build_ref(_cfg(cfg_name), "unit")
    with open(os.path.join(HERE, f"params_htdemucs_{tag}.json"), "w") as f:
        json.dump([[n, list(s)] for n, s in keys], f)


@torch.inference_mode()
def gen_forward(cfg_name, out_name, batch, seed):
    cfg = _cfg(cfg_name)
    model, _ = build_ref(cfg, "random")
    L = int(cfg["training"]["samplerate"] * cfg["training"]["segment"])
    x = np.stack([mg.mix_signal(seed + b, L) for b in range(batch)])
    y = model(torch.from_numpy(x)).numpy()
    mg.save(out_name, x=x, y=y, affine=np.array("random"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--full", action="store_true")
    args = ap.parse_args()
    mg.install_stubs()
    om = sys.modules["omegaconf"]
    om.OmegaConf = type("OmegaConf", (), {"to_container": staticmethod(lambda c, resolve=True: dict(c))})
    torch.set_num_threads(os.cpu_count())
    gen_params("config_musdb18_htdemucs.yaml", "musdb")
    gen_params("config_htdemucs_small.yaml", "small")
    gen_forward("config_htdemucs_small.yaml", "htdemucs_small.npz", 2, 71)
    if args.full:
        gen_forward("config_musdb18_htdemucs.yaml", "htdemucs_full_segment.npz", 1, 0)


if __name__ == "__main__":
    main()
