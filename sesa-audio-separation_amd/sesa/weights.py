"""Synthetic weights of a given architecture (no checkpoints offline): the name-keyed PCG64
definition of SURVEY.md §8(d) -- per parameter PCG64(crc32(name) ^ 0x5E5A); conv/linear
U(+-1/sqrt(fan_in)); norm gamma=1, beta=0 (or random / "stress" (beta U(2, 4)) affine for tests)."""
import zlib

import numpy as np
import torch


def synth_state_dict(model, affine="unit"):
    sd = {}
    for name, t in model.named_parameters():
        rng = np.random.Generator(np.random.PCG64(zlib.crc32(name.encode()) ^ 0x5E5A))
        shape = tuple(t.shape)
        if len(shape) >= 2:
            bound = 1.0 / np.sqrt(int(np.prod(shape[1:])))
            v = rng.uniform(-bound, bound, size=shape)
        elif name.endswith("bias"):
            v = (rng.uniform(-0.2, 0.2, size=shape) if affine == "random" else
                 rng.uniform(2.0, 4.0, size=shape) if affine == "stress" else np.zeros(shape))
        else:
            v = rng.uniform(0.5, 1.5, size=shape) if affine in ("random", "stress") else np.ones(shape)
        sd[name] = torch.from_numpy(v.astype(np.float32))
    return sd
