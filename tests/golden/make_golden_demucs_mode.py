#!/usr/bin/env python3
"""Golden vectors for utils.demix demucs mode (model_type 'htdemucs', utils.py:371-380, :408-477),
made by running the REAL reference ``utils.demix`` on CPU (build container only; stub recipe of
make_golden.py / SURVEY.md §8(c)).

The chunker is model-agnostic, so the model is a fixed position-dependent toy map (toy_model below,
also used by the tests) -- the fixture pins the chunk plan, zero-padded tails, batch grouping,
counter and the single-instrument bare-array return, not a network.

Usage:  python tests/golden/make_golden_demucs_mode.py   -> tests/golden/demix_demucs_mode.npz
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import make_golden as mg  # noqa: E402

# (tag, L, samplerate, segment, num_overlap, batch_size, n_instruments)
CASES = [
    ("ragged_bs1", 10500, 1000, 4, 4, 1, 2),
    ("ragged_bs3", 10500, 1000, 4, 4, 3, 2),
    ("short", 2500, 1000, 4, 4, 2, 2),
    ("exact_ov2", 8000, 1000, 4, 2, 2, 2),
    ("single", 9100, 1000, 4, 4, 2, 1),
]


def toy_model(n_instr):
    """[B, 2, C] -> [B, n, 2, C] (n > 1) or [B, 2, C]: depends on the position inside the chunk."""
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


def main():
    mg.install_stubs()
    sys.path.insert(0, mg.REF)
    import utils as ref_utils  # the reference's utils.py
    out = {}
    for tag, L, sr, seg, ov, bs, ni in CASES:
        rng = np.random.default_rng(len(tag) * 1000 + L)
        mix = (0.1 * rng.standard_normal((2, L))).astype(np.float32)
        cfg = mg.to_attr(cfg_for(sr, seg, ov, bs, ni))
        res = ref_utils.demix(cfg, toy_model(ni), mix, "cpu", model_type="htdemucs")
        est = np.stack([res[k] for k in cfg.training.instruments]) if isinstance(res, dict) else res
        out[f"{tag}_mix"] = mix
        out[f"{tag}_est"] = est.astype(np.float32)
        out[f"{tag}_is_dict"] = np.array(isinstance(res, dict))
    np.savez_compressed(os.path.join(HERE, "demix_demucs_mode.npz"), **out)
    print("wrote demix_demucs_mode.npz", {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
