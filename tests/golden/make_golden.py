#!/usr/bin/env python3
"""Generate golden vectors by running the REAL reference code on CPU (build container only).

Usage:  python tests/golden/make_golden.py [--full]

Imports /root/reference with its absent third-party modules stubbed (SURVEY.md §8(c) recipe:
ml_collections.ConfigDict -> attr-dict, omegaconf/loralib/soundfile/librosa -> empty modules),
loads the name-keyed synthetic weights (oracle/weights.py) into the reference ``TFC_TDF_net`` and
records inputs/outputs as .npz fixtures next to this script.  Nothing here runs on the GPU box and
no reference source is copied: the fixtures are data (inputs and expected outputs).

Fixtures:
  params_<cfg>.json       reference named_parameters() (name, shape) list
  stft_istft.npz          STFT.__call__ / STFT.inverse on a 16384-sample stereo signal
  mdx23c_small.npz        TFC_TDF_net.forward, reduced config, random affine norms
  mdx23c_small_vocals.npz TFC_TDF_net.forward, single-target reduced config
  demix_small_*.npz       inference_pytorch.demix_pytorch_optimized on the reduced model
  mdx23c_full_chunk.npz   (--full) one 261120-sample chunk through the full vocals config
  mdx23c_full_{sines,loud,wseed2}.npz  (--only full_levels) the same model on the §8(d) sines signal,
                          on 0.3-RMS white noise, and a second weight draw
  ensemble.npz            ensemble.AudioEnsembleEngine.process_waveform/process_spectral
  demix_full_10s.npz      (--only demix_full) BASELINE configs[0]: demix_pytorch_optimized, full vocals
                          config, 10 s mix, 13 chunks
"""
import argparse
import io
import json
import os
import sys
import types
import contextlib

import numpy as np
import torch
import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
CFG_DIR = os.path.join(REPO, "sesa-audio-separation_amd", "sesa", "configs")
sys.path.insert(0, REPO)

from oracle.weights import synth_state_dict  # noqa: E402


class AttrDict(dict):
    """Minimal ml_collections.ConfigDict stand-in: attribute access over a dict."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v


def to_attr(o):
    if isinstance(o, dict):
        return AttrDict({k: to_attr(v) for k, v in o.items()})
    if isinstance(o, list):
        return [to_attr(v) for v in o]
    return o


def install_stubs():
    ml = types.ModuleType("ml_collections")
    ml.ConfigDict = lambda d=None: to_attr(d or {})
    sys.modules["ml_collections"] = ml
    om = types.ModuleType("omegaconf")
    om.OmegaConf = object
    sys.modules["omegaconf"] = om
    for name in ("loralib", "soundfile"):
        sys.modules[name] = types.ModuleType(name)
    lb = types.ModuleType("librosa")
    lb.filters = None
    sys.modules["librosa"] = lb
    sys.path.insert(0, REF)


def load_cfg(name):
    with open(os.path.join(CFG_DIR, name)) as f:
        return yaml.safe_load(f)


def build_ref_model(cfg_dict, affine, seed=0):
    from models.mdx23c_tfc_tdf_v3 import TFC_TDF_net
    model = TFC_TDF_net(to_attr(cfg_dict)).eval()
    shapes = [(n, tuple(p.shape)) for n, p in model.named_parameters()]
    sd = synth_state_dict(shapes, affine=affine, seed=seed)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    return model, shapes


def mix_signal(seed, n):
    rng = np.random.default_rng(seed)
    return (0.1 * rng.standard_normal((2, n))).astype(np.float32)


def sines_signal(seed, n, sr=44100):
    """SURVEY §8(d)'s second synthetic signal: per channel, 20 sines at amplitude 0.02 with log-uniform
    random frequencies in [40 Hz, 16 kHz] and uniform random phases, plus 0.05-std white noise (seed 1);
    a non-white spectrum with tonal peaks."""
    rng = np.random.default_rng(seed)
    t = np.arange(n, dtype=np.float64) / sr
    out = np.empty((2, n), np.float64)
    for c in range(2):
        f = np.exp(rng.uniform(np.log(40.0), np.log(16000.0), 20))
        ph = rng.uniform(0.0, 2 * np.pi, 20)
        out[c] = (0.02 * np.sin(2 * np.pi * f[:, None] * t[None] + ph[:, None])).sum(0)
        out[c] += 0.05 * rng.standard_normal(n)
    return out.astype(np.float32)


def save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez(path, **arrays)
    print(f"wrote {path} ({os.path.getsize(path) / 1e6:.2f} MB)")


def gen_params(cfg_name, tag):
    cfg = load_cfg(cfg_name)
    _, shapes = build_ref_model(cfg, "unit")
    with open(os.path.join(HERE, f"params_{tag}.json"), "w") as f:
        json.dump([[n, list(s)] for n, s in shapes], f)


def gen_stft():
    from models.mdx23c_tfc_tdf_v3 import STFT
    a = to_attr(load_cfg("config_vocals_mdx23c.yaml")["audio"])
    st = STFT(a)
    x = torch.from_numpy(mix_signal(3, 16384))[None]            # [1,2,16384]
    X = st(x)                                                    # [1,4,4096,17]
    rng = np.random.default_rng(4)
    spec = (rng.standard_normal((1, 2, 4, 4096, 17))).astype(np.float32)   # 2 instruments
    y = st.inverse(torch.from_numpy(spec))                       # [1,2,2,16384]
    save("stft_istft.npz", x=x.numpy(), X=X.numpy(), spec=spec, y=y.numpy())


@torch.inference_mode()
def gen_forward(cfg_name, out_name, batch, seed, affine):
    cfg = load_cfg(cfg_name)
    model, _ = build_ref_model(cfg, affine)
    C = cfg["audio"]["chunk_size"]
    x = np.stack([mix_signal(seed + b, C) for b in range(batch)])
    y = model(torch.from_numpy(x)).numpy()
    save(out_name, x=x, y=y, affine=np.array(affine))


@torch.inference_mode()
def gen_full_levels():
    """Full-width MDX23C vocals chunk beyond the quiet white-noise golden: the §8(d)
    seed-1 sines + noise signal, white noise at 0.3 RMS (seed 5, about -10 dBFS), and the 0.1-RMS seed-0
    chunk through an independent second weight draw (seed 2, random norm affine)."""
    cfg = load_cfg("config_vocals_mdx23c.yaml")
    C = cfg["audio"]["chunk_size"]
    model, _ = build_ref_model(cfg, "unit")
    for name, x in (("mdx23c_full_sines.npz", sines_signal(1, C)),
                    ("mdx23c_full_loud.npz", (0.3 * np.random.default_rng(5).standard_normal((2, C))).astype(np.float32))):
        y = model(torch.from_numpy(x[None])).numpy()
        save(name, x=x[None], y=y, affine=np.array("unit"), weight_seed=np.array(0))
    model, _ = build_ref_model(cfg, "random", seed=2)
    x = mix_signal(0, C)[None]
    y = model(torch.from_numpy(x)).numpy()
    save("mdx23c_full_wseed2.npz", x=x, y=y, affine=np.array("random"), weight_seed=np.array(2))


@torch.inference_mode()
def gen_demix():
    import inference_pytorch as ip
    cfg = load_cfg("config_mdx23c_small.yaml")
    model, _ = build_ref_model(cfg, "random")
    from pytorch_backend import PyTorchBackend
    be = PyTorchBackend(device="cpu", optimize_mode="default")
    be.compiled_model = model
    be.model = model
    be.use_amp = False
    cases = [("unpadded", 40000, 1), ("unpadded", 40000, 2), ("padded", 110250, 1),
             ("padded", 110250, 3), ("short", 20000, 1)]
    for kind, L, bs in cases:
        c = to_attr(json.loads(json.dumps(cfg)))
        c.inference.batch_size = bs
        mix = mix_signal(7, L)
        with contextlib.redirect_stdout(io.StringIO()) as out:
            res = ip.demix_pytorch_optimized(c, be, mix, "cpu")
        prog = [ln for ln in out.getvalue().splitlines() if ln.startswith("[SESA_PROGRESS]")]
        save(f"demix_small_{kind}_L{L}_bs{bs}.npz", mix=mix, L=np.array(L), batch_size=np.array(bs),
             vocals=res["vocals"], other=res["other"], progress=np.array(prog))


@torch.inference_mode()
def gen_stress():
    """InstanceNorm precision stress: reduced MDX23C, norm beta ~ U(2, 4) (every
    normalised channel far from zero mean downstream) and a mix with a DC offset of 0.4."""
    cfg = load_cfg("config_mdx23c_small.yaml")
    model, _ = build_ref_model(cfg, "stress")
    C = cfg["audio"]["chunk_size"]
    x = np.stack([mix_signal(51 + b, C) + np.float32(0.4) for b in range(2)]).astype(np.float32)
    y = model(torch.from_numpy(x)).numpy()
    save("mdx23c_small_stress.npz", x=x, y=y, affine=np.array("stress"))


@torch.inference_mode()
def gen_demix_full():
    """BASELINE configs[0]: the REAL demix_pytorch_optimized on the full MDX23C vocals config, 10 s of
    44.1 kHz stereo (seed 0, 441000 samples -> 13 chunks at overlap 4), inference.batch_size 1,
    unit-affine weights (as mdx23c_full_chunk.npz).  ~75 s of CPU."""
    import inference_pytorch as ip
    from pytorch_backend import PyTorchBackend
    cfg = load_cfg("config_vocals_mdx23c.yaml")
    model, _ = build_ref_model(cfg, "unit")
    be = PyTorchBackend(device="cpu", optimize_mode="default")
    be.compiled_model = model
    be.model = model
    be.use_amp = False
    c = to_attr(json.loads(json.dumps(cfg)))
    mix = mix_signal(0, 441000)
    with contextlib.redirect_stdout(io.StringIO()) as out:
        res = ip.demix_pytorch_optimized(c, be, mix, "cpu")
    prog = [ln for ln in out.getvalue().splitlines() if ln.startswith("[SESA_PROGRESS]")]
    save("demix_full_10s.npz", mix=mix, vocals=res["vocals"], other=res["other"], progress=np.array(prog))


def gen_ensemble():
    import ensemble as ens
    eng = ens.AudioEnsembleEngine()
    eng.log_file = os.path.join("/tmp", "sesa_golden_ensemble.log")
    rng = np.random.default_rng(11)
    waves = (0.1 * rng.standard_normal((3, 2, 4096))).astype(np.float64)   # [files, ch, samples]
    weights = np.array([0.5, 0.3, 0.2], np.float32)
    weights /= weights.sum()                                               # ensemble.py:288-293
    out = {"waves": waves, "weights": weights}
    for m in ("avg_wave", "median_wave", "max_wave", "min_wave"):
        out[m] = eng.process_waveform(waves, m, weights)
    out["avg_wave_unweighted"] = eng.process_waveform(waves, "avg_wave", None)
    for m in ("max_fft", "min_fft", "median_fft"):
        out[m] = eng.process_spectral(waves, m)
    odd = waves[:, :, :1500]                                               # nperseg 1024, ragged tail
    out["odd"] = odd
    out["median_fft_odd"] = eng.process_spectral(odd, "median_fft")
    small = waves[:, :, :600]                                              # nperseg = min(1024, 600)
    out["small"] = small
    out["max_fft_small"] = eng.process_spectral(small, "max_fft")
    out["short_is_none"] = np.array(eng.process_spectral(waves[:, :, :200], "max_fft") is None)
    save("ensemble.npz", **out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--full", action="store_true", help="also the full-width vocals chunk (~10 s CPU)")
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    install_stubs()
    torch.set_num_threads(os.cpu_count())
    todo = args.only.split(",") if args.only else ["params", "stft", "fwd", "demix", "ensemble"]
    if "params" in todo:
        gen_params("config_vocals_mdx23c.yaml", "vocals")
        gen_params("config_mdx23c_small.yaml", "small")
    if "stft" in todo:
        gen_stft()
    if "fwd" in todo:
        gen_forward("config_mdx23c_small.yaml", "mdx23c_small.npz", 2, 21, "random")
        gen_forward("config_mdx23c_small_vocals.yaml", "mdx23c_small_vocals.npz", 1, 31, "random")
    if "demix" in todo:
        gen_demix()
    if "ensemble" in todo:
        gen_ensemble()
    if "stress" in todo:
        gen_stress()
    if "demix_full" in todo:
        gen_demix_full()
    if "full_levels" in todo:
        gen_full_levels()
    if args.full or "full" in todo:
        gen_forward("config_vocals_mdx23c.yaml", "mdx23c_full_chunk.npz", 1, 0, "unit")


if __name__ == "__main__":
    main()
