#!/usr/bin/env python3
"""BASELINE configs[4] at FULL width on a short mix, from the REAL reference (build container only).

Usage:  python tests/golden/make_golden_ensemble_full.py

Members as the configs[4] bench line runs them: MDX23C vocals (unit-affine name-keyed weights, as
mdx23c_full_chunk.npz), BS-Roformer vocals (viperx 1297 widths) and SCNet musdb18 (oracle synth_params
'random', as bsr_full_chunk.npz / scnet_full_chunk.npz).  Each member goes through the reference
``inference_pytorch.demix_pytorch_optimized`` (:55-186) with its reference model class on CPU fp32; the
vocals stems are blended by the reference ``AudioEnsembleEngine.process_waveform`` / ``process_spectral``
over run_ensemble's 32768-frame buffers (ensemble.py:258-407; weights normalised as :288-293).  The mix is
3 s (132 300 samples, seed 13): 3 MDX23C chunks, 1 BS-Roformer chunk, 2 SCNet chunks.  ~2 min of CPU.

Fixtures (round 5 adds two variants, and every blend method in each):
  ensemble_full.npz         0.1-RMS mix, MDX23C unit affine, BS-Roformer / SCNet random affine, weight seed 0
  ensemble_full_loud.npz    --variant loud:   the same mix scaled to 0.3 RMS
  ensemble_full_wseed2.npz  --variant wseed2: 0.1-RMS mix, every member on weight seed 2 (random affine)
Each holds mix, weights, vocals_<member>, blend_<method> for avg_wave (weights 0.5/0.3/0.2), median_wave,
max_wave, min_wave, max_fft, min_fft, median_fft, plus mix_scale / weight_seed / affine_<member>.
"""
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

L = 132300
WEIGHTS = np.array([0.5, 0.3, 0.2], np.float32)


_BE = []


@torch.inference_mode()
def demix_ref(model, cfg, mix):
    import inference_pytorch as ip
    be = _BE[0]                   # one backend: its constructor sets the interop threads (once per process)
    be.compiled_model = model
    be.model = model
    be.use_amp = False
    c = mg.to_attr(json.loads(json.dumps(cfg)))
    with contextlib.redirect_stdout(io.StringIO()):
        return ip.demix_pytorch_optimized(c, be, mix, "cpu")


def blend_ref(waves, method, weights=None, buffer=32768):
    import ensemble as ens
    eng = ens.AudioEnsembleEngine()
    eng.log_file = os.path.join("/tmp", "sesa_golden_ensemble_full.log")
    w = None if weights is None else weights / weights.sum()
    n, ch, n_s = waves.shape
    out = np.zeros((ch, n_s))
    for pos in range(0, n_s, buffer):
        chunk = waves[:, :, pos:pos + buffer]
        res = eng.process_spectral(chunk, method) if method.endswith("_fft") else eng.process_waveform(chunk, method, w)
        if res is None:
            res = eng.process_waveform(chunk, "avg_wave", w)
        out[:, pos:pos + chunk.shape[2]] = res
    return out


METHODS = ("avg_wave", "median_wave", "max_wave", "min_wave", "max_fft", "min_fft", "median_fft")
VARIANTS = {"base": ("ensemble_full.npz", 1.0, 0), "loud": ("ensemble_full_loud.npz", 3.0, 0),
            "wseed2": ("ensemble_full_wseed2.npz", 1.0, 2)}


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", default="base", choices=sorted(VARIANTS))
    args = ap.parse_args()
    out_name, scale, seed = VARIANTS[args.variant]
    mdx_affine = "unit" if seed == 0 else "random"
    mg.install_stubs()
    import make_golden_bsr as mgb
    import make_golden_scnet as mgs
    mgb.install_librosa_stub()
    from pytorch_backend import PyTorchBackend
    _BE.append(PyTorchBackend(device="cpu", optimize_mode="default"))
    torch.set_num_threads(os.cpu_count())
    mix = (mg.mix_signal(13, L) * np.float32(scale)).astype(np.float32)
    stems = {}
    cfg = mg.load_cfg("config_vocals_mdx23c.yaml")
    model, _ = mg.build_ref_model(cfg, mdx_affine, seed=seed)
    stems["mdx23c"] = demix_ref(model, cfg, mix)["vocals"]
    print("mdx23c done", flush=True)
    cfg = mgb._cfg("config_bs_roformer_vocals.yaml")
    model, _ = mgb.build_ref(cfg, "random", seed)
    stems["bs_roformer"] = demix_ref(model, cfg, mix)["vocals"]
    print("bs_roformer done", flush=True)
    cfg = mgs._cfg("config_musdb18_scnet.yaml")
    model, _ = mgs.build_ref(cfg, "random", seed)
    stems["scnet"] = demix_ref(model, cfg, mix)["vocals"]
    print("scnet done", flush=True)
    waves = np.stack([stems[k] for k in ("mdx23c", "bs_roformer", "scnet")]).astype(np.float64)
    # the reference blends are float64; stored as float32 (<= 1e-9 absolute here, against an 8e-5 RMS gate) to keep
    # the three fixtures small
    blends = {f"blend_{m}": blend_ref(waves, m, WEIGHTS if m == "avg_wave" else None).astype(np.float32)
              for m in METHODS}
    mg.save(out_name, mix=mix, weights=WEIGHTS, **{f"vocals_{k}": v for k, v in stems.items()}, **blends,
            mix_scale=np.float32(scale), weight_seed=np.array(seed), affine_mdx23c=np.array(mdx_affine),
            affine_bs_roformer=np.array("random"), affine_scnet=np.array("random"))


if __name__ == "__main__":
    main()
