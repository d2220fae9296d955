"""Pin the CPU oracle (oracle/) against golden vectors produced by the real reference
(tests/golden/make_golden.py).  CPU only."""
import glob
import json
import os

import numpy as np
import pytest
import torch
import yaml

from conftest import CONFIGS, GOLDEN, rms
from oracle import demix as odemix
from oracle import mdx23c as om
from oracle.weights import synth_state_dict


def cfg(name):
    with open(os.path.join(CONFIGS, name)) as f:
        return yaml.safe_load(f)


@pytest.mark.parametrize("cfg_name,tag", [("config_vocals_mdx23c.yaml", "vocals"),
                                          ("config_mdx23c_small.yaml", "small")])
def test_param_names_match_reference(cfg_name, tag):
    with open(os.path.join(GOLDEN, f"params_{tag}.json")) as f:
        ref = [(n, tuple(s)) for n, s in json.load(f)]
    assert om.param_shapes(cfg(cfg_name)) == ref


def test_stft_istft(golden):
    g = golden("stft_istft.npz")
    a = cfg("config_vocals_mdx23c.yaml")["audio"]
    X = om.stft(torch.from_numpy(g["x"]), a).numpy()
    assert X.shape == g["X"].shape
    assert np.abs(X - g["X"]).max() < 1e-5
    y = om.istft(torch.from_numpy(g["spec"]), a).numpy()
    assert y.shape == g["y"].shape
    assert np.abs(y - g["y"]).max() < 1e-6


@pytest.mark.parametrize("fixture,cfg_name", [("mdx23c_small.npz", "config_mdx23c_small.yaml"),
                                              ("mdx23c_small_vocals.npz", "config_mdx23c_small_vocals.yaml"),
                                              ("mdx23c_small_stress.npz", "config_mdx23c_small.yaml")])
def test_forward_small(golden, fixture, cfg_name):
    g = golden(fixture)
    c = cfg(cfg_name)
    params = om.to_torch_params(synth_state_dict(om.param_shapes(c), affine=str(g["affine"])))
    with torch.inference_mode():
        y = om.forward(params, c, torch.from_numpy(g["x"])).numpy()
    assert y.shape == g["y"].shape
    assert rms(y, g["y"]) < 1e-6


@pytest.mark.slow
def test_forward_full_chunk(golden):
    g = golden("mdx23c_full_chunk.npz")
    c = cfg("config_vocals_mdx23c.yaml")
    params = om.to_torch_params(synth_state_dict(om.param_shapes(c)))
    with torch.inference_mode():
        y = om.forward(params, c, torch.from_numpy(g["x"])).numpy()
    assert rms(y, g["y"]) < 1e-6


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "demix_small_*.npz"))),
                         ids=lambda p: os.path.basename(p))
def test_demix_matches_reference(path):
    g = np.load(path)
    c = cfg("config_mdx23c_small.yaml")
    params = synth_state_dict(om.param_shapes(c), affine="random")
    model = om.OracleModel(c, params)
    out = odemix.demix(c, model, g["mix"], batch_size=int(g["batch_size"]))
    for k in ("vocals", "other"):
        assert out[k].shape == g[k].shape
        assert rms(out[k], g[k]) < 1e-6, k


def test_chunk_plan_counts():
    # 10 s -> 13 chunks, 4-min at ov4 -> 169
    for L, n in ((441000, 13), (10584000, 169)):
        _, _, _, batches = odemix.chunk_plan(L, 261120, 4, 1)
        assert sum(len(b[0]) for b in batches) == n
