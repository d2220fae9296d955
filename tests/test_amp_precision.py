"""--enable_amp is what the GUI always passes (/root/reference/processing.py:207, 292-293); the backend maps it
to each model's throughput precision (sesa/backend.py, pytorch_backend.py:308-311 is fp16 autocast in the
reference).  Every precision that mapping selects must hold north_star's 1e-4 per-sample RMS gate on the
model's full-width reference golden: here each native model type goes through create_inference_session(
enable_amp=True) exactly as the CLI builds it, and runs its full-chunk fixture.  GPU only."""
import os

import numpy as np
import pytest
import torch

from conftest import CONFIGS, rms

pytestmark = pytest.mark.gpu
RMS_GATE = 1e-4

CASES = [("mdx23c", "config_vocals_mdx23c.yaml", "mdx23c_full_loud.npz"),
         ("mdx23c", "config_vocals_mdx23c.yaml", "mdx23c_full_wseed2.npz"),
         ("bs_roformer", "config_bs_roformer_vocals.yaml", "bsr_full_chunk.npz"),
         ("mel_band_roformer", "config_mel_band_roformer_vocals.yaml", "mbr_full_chunk.npz"),
         ("scnet", "config_musdb18_scnet.yaml", "scnet_full_chunk.npz"),
         ("htdemucs", "config_musdb18_htdemucs.yaml", "htdemucs_full_segment.npz")]


@pytest.mark.parametrize("model_type,cfg_name,fixture", CASES, ids=[f"{c[0]}-{c[2]}" for c in CASES])
def test_enable_amp_precision_holds_the_gate(golden, model_type, cfg_name, fixture):
    from sesa.backend import create_inference_session
    from sesa.utils import get_model_from_config
    from sesa.weights import synth_model_state, synth_state_dict
    assert torch.cuda.is_available()
    g = golden(fixture)
    affine = str(g["affine"]) if "affine" in g.files else "random"
    seed = int(g["weight_seed"]) if "weight_seed" in g.files else 0
    m, _ = get_model_from_config(model_type, os.path.join(CONFIGS, cfg_name))
    m.load_state_dict(synth_state_dict(m, affine=affine, seed=seed) if model_type == "mdx23c" else
                      synth_model_state(m, affine=affine, seed=seed), strict=True)
    be = create_inference_session(m, device="cuda:0", enable_amp=True)
    assert m.precision == m._amp_precision
    y = be(torch.from_numpy(g["x"]).to("cuda:0")).cpu().numpy()
    err = rms(y, g["y"])
    print(f"{model_type} {fixture} --enable_amp -> {m.precision}: rms {err:.3e} (ref rms {rms(g['y'], 0):.3e})")
    assert y.shape == g["y"].shape and np.isfinite(y).all() and err <= RMS_GATE
