"""Generate BS-Roformer golden fixtures by running the REAL reference model on CPU.

Run here (not on the GPU box):  python tests/golden/make_golden_bsr.py [--full]

Imports /root/reference/models/bs_roformer with the third-party modules the reference needs but
this image lacks stubbed (make_golden.install_stubs(): ml_collections, omegaconf, loralib,
soundfile, librosa; plus oracle/_stubs: beartype (decorator only) and the restated
rotary_embedding_torch -- parity at the rotary boundary is therefore unpinned).
Weights: oracle.bs_roformer.synth_params (name-keyed, deterministic).  Fixtures are data only.

Fixtures:
  params_bsr_<tag>.json   reference state_dict() (name, shape) list
  bsr_small.npz           BSRoformer.forward, reduced config, batch 2 x 1 s
  demix_bsr_small.npz     inference_pytorch.demix_pytorch_optimized on the reduced model (3.3 s mix)
  bsr_full_chunk.npz      (--full) one 352800-sample chunk through the vocals config
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
sys.path.insert(0, os.path.join(REPO, "oracle", "_stubs"))

import make_golden as mg  # noqa: E402
from oracle import bs_roformer as ob  # noqa: E402


def _cfg(name):
    return ob.load_cfg(os.path.join(mg.CFG_DIR, name))


def build_ref(cfg, affine, seed=0):
    from models.bs_roformer import BSRoformer
    model = BSRoformer(**ob.model_kwargs(cfg)).eval()
    sd = ob.synth_params(cfg, affine, seed)
    ref_keys = [(k, tuple(v.shape)) for k, v in model.state_dict().items()]
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    return model, ref_keys


def install_librosa_stub():
    """The reference mel_band_roformer does `from librosa import filters`: use the restated mel."""
    import importlib
    sys.modules.pop("librosa", None)
    sys.modules["librosa"] = importlib.import_module("librosa")   # oracle/_stubs/librosa


def build_ref_mel(cfg, affine):
    from models.bs_roformer.mel_band_roformer import MelBandRoformer
    from oracle import mel_band_roformer as om
    model = MelBandRoformer(**om.model_kwargs(cfg)).eval()
    sd = om.synth_params(cfg, affine)
    ref_keys = [(k, tuple(v.shape)) for k, v in model.state_dict().items()]
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    return model, ref_keys


@torch.inference_mode()
def gen_mel():
    from oracle import mel_band_roformer as om
    for name, tag in (("config_mel_band_roformer_vocals.yaml", "vocals"), ("config_mel_band_roformer_small.yaml", "small")):
        cfg = _cfg(name)
        model, keys = build_ref_mel(cfg, "unit")
        with open(os.path.join(HERE, f"params_mbr_{tag}.json"), "w") as f:
            json.dump([[n, list(s)] for n, s in keys], f)
        k = om.model_kwargs(cfg)
        fpb, idx, nbpf = om.bands(k)
        assert torch.equal(model.freq_indices, idx) and torch.equal(model.num_bands_per_freq, nbpf)
    cfg = _cfg("config_mel_band_roformer_small.yaml")
    model, _ = build_ref_mel(cfg, "random")
    C = cfg["audio"]["chunk_size"]
    x = np.stack([mg.mix_signal(51 + b, C) for b in range(2)])
    mg.save("mbr_small.npz", x=x, y=model(torch.from_numpy(x)).numpy(), affine=np.array("random"),
            freq_indices=model.freq_indices.numpy(), num_bands_per_freq=model.num_bands_per_freq.numpy())


@torch.inference_mode()
def gen_mel_full():
    cfg = _cfg("config_mel_band_roformer_vocals.yaml")
    model, _ = build_ref_mel(cfg, "random")
    x = mg.mix_signal(0, cfg["audio"]["chunk_size"])[None]
    mg.save("mbr_full_chunk.npz", x=x, y=model(torch.from_numpy(x)).numpy(), affine=np.array("random"))


def gen_params(cfg_name, tag):
    cfg = _cfg(cfg_name)
    _, keys = build_ref(cfg, "unit")
    with open(os.path.join(HERE, f"params_bsr_{tag}.json"), "w") as f:
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
    cfg = _cfg("config_bs_roformer_small.yaml")
    model, _ = build_ref(cfg, "random")
    be = PyTorchBackend(device="cpu", optimize_mode="default")
    be.compiled_model = model
    be.model = model
    be.use_amp = False
    c = mg.to_attr(json.loads(json.dumps(cfg)))
    mix = mg.mix_signal(9, 145000)
    with contextlib.redirect_stdout(io.StringIO()) as out:
        res = ip.demix_pytorch_optimized(c, be, mix, "cpu")
    prog = [ln for ln in out.getvalue().splitlines() if ln.startswith("[SESA_PROGRESS]")]
    mg.save("demix_bsr_small.npz", mix=mix, vocals=res["vocals"], progress=np.array(prog))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--full", action="store_true")
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    mg.install_stubs()
    install_librosa_stub()
    torch.set_num_threads(os.cpu_count())
    todo = args.only.split(",") if args.only else ["params", "fwd", "demix", "mel"]
    if "params" in todo:
        gen_params("config_bs_roformer_vocals.yaml", "vocals")
        gen_params("config_bs_roformer_small.yaml", "small")
    if "fwd" in todo:
        gen_forward("config_bs_roformer_small.yaml", "bsr_small.npz", 2, 41, "random")
    if "demix" in todo:
        gen_demix()
    if "mel" in todo:
        gen_mel()
    if "melfull" in todo:
        gen_mel_full()
    if args.full or "full" in todo:
        gen_forward("config_bs_roformer_vocals.yaml", "bsr_full_chunk.npz", 1, 0, "random")


if __name__ == "__main__":
    main()
