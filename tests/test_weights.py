"""sesa.weights.synth_model_state (bench.py's parity leg rebuilds the golden fixtures' models with it, without
the oracle) reproduces exactly the weights each fixture generator loaded into the reference: oracle
synth_params (BS-/Mel-Band-Roformer, SCNet) and tests/golden/make_golden_htdemucs.synth_params; and
synth_state_dict's second weight draw (seed 2) matches oracle/weights.py's.  CPU only."""
import importlib.util
import os

import numpy as np
import pytest
import torch

from conftest import CONFIGS, GOLDEN


def _check(model, ref):
    from sesa.weights import synth_model_state
    sd = synth_model_state(model, "random")
    assert list(sd) == list(ref)
    for k, v in ref.items():
        np.testing.assert_array_equal(sd[k].numpy(), np.asarray(v, np.float32), err_msg=k)


@pytest.mark.parametrize("model_type,oracle_mod,cfg_name", [
    ("bs_roformer", "bs_roformer", "config_bs_roformer_vocals.yaml"),
    ("mel_band_roformer", "mel_band_roformer", "config_mel_band_roformer_small.yaml"),
    ("scnet", "scnet", "config_musdb18_scnet.yaml")])
def test_synth_model_state_matches_oracle_scheme(model_type, oracle_mod, cfg_name):
    import importlib
    from sesa.utils import get_model_from_config
    o = importlib.import_module(f"oracle.{oracle_mod}")
    m, _ = get_model_from_config(model_type, os.path.join(CONFIGS, cfg_name))
    _check(m, o.synth_params(o.load_cfg(os.path.join(CONFIGS, cfg_name)), "random"))


def test_synth_model_state_matches_htdemucs_fixture_scheme():
    from oracle import htdemucs as oh
    from sesa.utils import get_model_from_config
    spec = importlib.util.spec_from_file_location("mgh", os.path.join(GOLDEN, "make_golden_htdemucs.py"))
    mgh = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mgh)
    cfg_name = "config_musdb18_htdemucs.yaml"
    m, _ = get_model_from_config("htdemucs", os.path.join(CONFIGS, cfg_name))
    _check(m, mgh.synth_params(dict(oh.param_names(oh.load_cfg(os.path.join(CONFIGS, cfg_name)))), "random"))


def test_second_weight_draw_matches_oracle():
    from oracle import mdx23c as om
    from oracle.weights import synth_state_dict as oracle_sd
    from sesa.utils import get_model_from_config
    from sesa.weights import synth_state_dict
    import yaml
    m, _ = get_model_from_config("mdx23c", os.path.join(CONFIGS, "config_mdx23c_small.yaml"))
    with open(os.path.join(CONFIGS, "config_mdx23c_small.yaml")) as f:
        cfg = yaml.safe_load(f)
    ref = oracle_sd(om.param_shapes(cfg), affine="random", seed=2)
    sd = synth_state_dict(m, affine="random", seed=2)
    assert list(sd) == list(ref)
    for k in ref:
        np.testing.assert_array_equal(sd[k].numpy(), ref[k], err_msg=k)
    base = synth_state_dict(m, affine="random")
    assert not torch.equal(base["first_conv.weight"], sd["first_conv.weight"])
