"""HTDemucs oracle (no native engine yet).

oracle/htdemucs.py restates models/demucs4ht.py's HTDemucs on the restated third-party demucs layers
(oracle/_stubs/demucs).  tests/golden/make_golden_htdemucs.py ran the REFERENCE HTDemucs class on
the same restated layers, so these tests pin the oracle to the reference's HTDemucs-level code
(spec/ispec padding, cac magnitude / mask, branch normalisation, injection, transformer plumbing,
decoder split).  The layer boundary is parity-unpinned: the demucs package is absent.
"""
import json
import os

import numpy as np
import pytest
import torch

from conftest import CONFIGS, GOLDEN, rms

torch.set_num_threads(min(8, os.cpu_count() or 1))


def _synth(cfg):
    import importlib.util
    spec = importlib.util.spec_from_file_location("mgh", os.path.join(GOLDEN, "make_golden_htdemucs.py"))
    mgh = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mgh)
    from oracle import htdemucs as oh
    return mgh.synth_params(dict(oh.param_names(cfg)), "random")


@pytest.mark.parametrize("cfg_name,tag", [("config_musdb18_htdemucs.yaml", "musdb"),
                                          ("config_htdemucs_small.yaml", "small")])
def test_param_names_match_reference(cfg_name, tag):
    from oracle import htdemucs as oh
    cfg = oh.load_cfg(os.path.join(CONFIGS, cfg_name))
    with open(os.path.join(GOLDEN, f"params_htdemucs_{tag}.json")) as f:
        ref = [(n, tuple(s)) for n, s in json.load(f)]
    assert oh.param_names(cfg) == ref


@pytest.mark.parametrize("cfg_name,fx", [("config_htdemucs_small.yaml", "htdemucs_small.npz"),
                                         ("config_musdb18_htdemucs.yaml", "htdemucs_full_segment.npz")])
def test_oracle_matches_reference_class(cfg_name, fx, golden):
    from oracle import htdemucs as oh
    cfg = oh.load_cfg(os.path.join(CONFIGS, cfg_name))
    g = golden(fx)
    m = oh.load(cfg, _synth(cfg))
    y = oh.forward(m, cfg, torch.from_numpy(g["x"])).numpy()
    assert y.shape == g["y"].shape
    assert rms(y, g["y"]) <= 1e-6
