"""Pin the BS-Roformer CPU oracle (oracle/bs_roformer.py) against golden vectors produced by the
real reference model (tests/golden/make_golden_bsr.py).  CPU only."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import CONFIGS, GOLDEN, rms
from oracle import bs_roformer as ob
from oracle import demix as odemix


def cfg(name):
    return ob.load_cfg(os.path.join(CONFIGS, name))


@pytest.mark.parametrize("cfg_name,tag", [("config_bs_roformer_vocals.yaml", "vocals"),
                                          ("config_bs_roformer_small.yaml", "small")])
def test_param_names_match_reference_state_dict(cfg_name, tag):
    with open(os.path.join(GOLDEN, f"params_bsr_{tag}.json")) as f:
        ref = [(n, tuple(s)) for n, s in json.load(f)]
    assert ob.param_names(cfg(cfg_name)) == ref


def test_band_layout_vocals():
    k = ob.model_kwargs(cfg("config_bs_roformer_vocals.yaml"))
    dims = ob.band_dims(k)
    assert len(dims) == 62 and sum(dims) == 4100
    assert sum(k["freqs_per_bands"]) == 1025


def test_forward_small(golden):
    g = golden("bsr_small.npz")
    c = cfg("config_bs_roformer_small.yaml")
    P = ob.to_torch(ob.synth_params(c, str(g["affine"])))
    with torch.inference_mode():
        y = ob.forward(P, c, torch.from_numpy(g["x"])).numpy()
    assert y.shape == g["y"].shape
    assert rms(y, g["y"]) < 1e-6


def test_demix_small(golden):
    g = golden("demix_bsr_small.npz")
    c = cfg("config_bs_roformer_small.yaml")
    model = ob.OracleModel(c, ob.synth_params(c, "random"))
    out = odemix.demix(c, model, g["mix"], batch_size=int(c["inference"]["batch_size"]))
    assert out["vocals"].shape == g["vocals"].shape
    assert rms(out["vocals"], g["vocals"]) < 1e-6


# ---- Mel-Band-Roformer (oracle/mel_band_roformer.py vs the reference, make_golden_bsr.py --only mel) ----
from oracle import mel_band_roformer as om  # noqa: E402


@pytest.mark.parametrize("cfg_name,tag", [("config_mel_band_roformer_vocals.yaml", "vocals"),
                                          ("config_mel_band_roformer_small.yaml", "small")])
def test_mel_param_names_match_reference_state_dict(cfg_name, tag):
    with open(os.path.join(GOLDEN, f"params_mbr_{tag}.json")) as f:
        ref = [(n, tuple(s)) for n, s in json.load(f)]
    assert om.param_names(cfg(cfg_name)) == ref


def test_mel_bands_and_forward_small(golden):
    g = golden("mbr_small.npz")
    c = cfg("config_mel_band_roformer_small.yaml")
    k = om.model_kwargs(c)
    _, idx, nbpf = om.bands(k)
    assert np.array_equal(idx.numpy(), g["freq_indices"]) and np.array_equal(nbpf.numpy(), g["num_bands_per_freq"])
    P = ob.to_torch(om.synth_params(c, str(g["affine"])))
    with torch.inference_mode():
        y = om.forward(P, c, torch.from_numpy(g["x"])).numpy()
    assert y.shape == g["y"].shape
    assert rms(y, g["y"]) < 1e-6
