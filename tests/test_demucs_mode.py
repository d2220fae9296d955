"""utils.demix demucs mode (model_type 'htdemucs', reference utils.py:371-380, :408-477).

Fixture tests/golden/demix_demucs_mode.npz = the REAL reference utils.demix run on CPU with a fixed
position-dependent toy model (tests/golden/make_golden_demucs_mode.py): ragged tails, a track
shorter than one chunk, overlap 2 and 4, batch sizes 1/2/3, and the single-instrument bare-array
return.  CPU: the oracle restatement against the fixture.  GPU: the device chunker
(sesa_chunk_gather_constant_f32 + OLA kernels) through sesa.utils.demix against the fixture.
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import demix as odemix

# (tag, L, samplerate, segment, num_overlap, batch_size, n_instruments) -- as the generating script
CASES = [
    ("ragged_bs1", 10500, 1000, 4, 4, 1, 2),
    ("ragged_bs3", 10500, 1000, 4, 4, 3, 2),
    ("short", 2500, 1000, 4, 4, 2, 2),
    ("exact_ov2", 8000, 1000, 4, 2, 2, 2),
    ("single", 9100, 1000, 4, 4, 2, 1),
]


def toy_model(n_instr):
    def f(x):
        a = 0.5 * x + 0.25 * torch.flip(x, dims=[-1])
        if n_instr == 1:
            return a
        b = torch.roll(x, 7, dims=-1) - 0.1 * x
        return torch.stack([a, b], dim=1)
    return f


def cfg_for(sr, seg, ov, bs, ni):
    return {"training": {"samplerate": sr, "segment": seg, "instruments": ["vocals", "other"][:ni],
                         "use_amp": False},
            "inference": {"num_overlap": ov, "batch_size": bs}}


@pytest.fixture(scope="module")
def fx():
    return np.load(os.path.join(GOLDEN, "demix_demucs_mode.npz"))


def _stack(res, instruments):
    return np.stack([res[k] for k in instruments]) if isinstance(res, dict) else res


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_oracle_demucs_mode_matches_reference(fx, case):
    tag, L, sr, seg, ov, bs, ni = case
    cfg = cfg_for(sr, seg, ov, bs, ni)
    res = odemix.demix_demucs_mode(cfg, toy_model(ni), fx[f"{tag}_mix"])
    assert isinstance(res, dict) == bool(fx[f"{tag}_is_dict"])
    np.testing.assert_array_equal(_stack(res, cfg["training"]["instruments"]), fx[f"{tag}_est"])


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_device_demucs_mode_matches_reference(fx, case):
    from sesa.config import wrap
    from sesa.utils import demix
    tag, L, sr, seg, ov, bs, ni = case
    cfg = wrap(cfg_for(sr, seg, ov, bs, ni))
    res = demix(cfg, toy_model(ni), fx[f"{tag}_mix"], "cuda:0", model_type="htdemucs")
    assert isinstance(res, dict) == bool(fx[f"{tag}_is_dict"])
    got = _stack(res, list(cfg.training.instruments))
    # integer-free fp32 path, same operation order as the reference: bit-exact expected; the
    # tolerance only absorbs a possible 1-ulp difference of the toy model's GPU elementwise ops
    assert got.shape == fx[f"{tag}_est"].shape
    assert np.max(np.abs(got - fx[f"{tag}_est"])) <= 1e-6
