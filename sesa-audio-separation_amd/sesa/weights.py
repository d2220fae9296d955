"""Synthetic weights of a given architecture (no checkpoints offline): the name-keyed PCG64
definition of SURVEY.md §8(d) -- per parameter PCG64(crc32(name) ^ 0x5E5A); conv/linear
U(+-1/sqrt(fan_in)); norm gamma=1, beta=0 (or random / "stress" (beta U(2, 4)) affine for tests)."""
import zlib

import numpy as np
import torch


def synth_state_dict(model, affine="unit", seed=0):
    """seed 0: the §8(d) draw; seed k > 0: PCG64([crc32(name) ^ 0x5E5A, k]), an independent second draw."""
    sd = {}
    for name, t in model.named_parameters():
        key = zlib.crc32(name.encode()) ^ 0x5E5A
        rng = np.random.Generator(np.random.PCG64(key if seed == 0 else [key, int(seed)]))
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


def synth_model_state(model, affine="random", seed=0):
    """Name-keyed synthetic weights for any native model (the BS-/Mel-Roformer, SCNet and HTDemucs golden
    fixtures' scheme, tests/golden/make_golden_*.py): >= 2-D tensors U(+-1/sqrt(prod(shape[1:]))); a bias
    (``x.bias``, LSTM ``bias_ih_l0`` ...) of such a weight U(+-1/sqrt(fan_in of the weight)) with
    affine="random", else 0; LayerScale ``scale`` U(0.1, 0.3); rotary ``freqs`` keep the module's own
    (the real inverse frequencies); other 1-D tensors (norm gammas / betas) as synth_state_dict.  Used by
    bench.py's parity leg to rebuild the fixtures' models without the oracle."""
    shapes = {n: tuple(t.shape) for n, t in model.named_parameters()}
    cur = dict(model.named_parameters())
    sd = {}
    for name, shape in shapes.items():
        key = zlib.crc32(name.encode()) ^ 0x5E5A
        rng = np.random.Generator(np.random.PCG64(key if seed == 0 else [key, int(seed)]))
        head, _, last = name.rpartition(".")
        wname = f"{head}.{last.replace('bias', 'weight')}" if "bias" in last else None
        if name.endswith("rotary_embed.freqs"):
            sd[name] = cur[name].detach().to("cpu", torch.float32).clone()
            continue
        if last == "scale":
            v = rng.uniform(0.1, 0.3, size=shape)
        elif wname and wname in shapes and len(shapes[wname]) >= 2:
            b = 1.0 / np.sqrt(int(np.prod(shapes[wname][1:])))
            v = rng.uniform(-b, b, size=shape) if affine == "random" else np.zeros(shape)
        elif len(shape) >= 2:
            b = 1.0 / np.sqrt(int(np.prod(shape[1:])))
            v = rng.uniform(-b, b, size=shape)
        elif name.endswith("bias"):
            v = (rng.uniform(-0.2, 0.2, size=shape) if affine == "random" else
                 rng.uniform(2.0, 4.0, size=shape) if affine == "stress" else np.zeros(shape))
        else:
            v = rng.uniform(0.5, 1.5, size=shape) if affine in ("random", "stress") else np.ones(shape)
        sd[name] = torch.from_numpy(np.asarray(v, np.float64).astype(np.float32))
    return sd
