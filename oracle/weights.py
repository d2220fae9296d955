"""Name-keyed deterministic synthetic weights.  TEST INFRASTRUCTURE.

For every parameter, in ``named_parameters()`` order, a PCG64 generator is
seeded with ``zlib.crc32(name) ^ 0x5E5A``.  Conv / Linear weights are drawn
from U(-1/sqrt(fan_in), +1/sqrt(fan_in)) with fan_in = prod(shape[1:]) (torch's
``_calculate_fan_in_and_fan_out`` convention, the bound of torch's default
init).  Norm affine weights are 1 and biases 0 -- or, with
``affine="random"``, gamma ~ U(0.5, 1.5) and beta ~ U(-0.2, 0.2) so that tests
exercise the affine path; ``affine="stress"``: beta ~ U(2, 4), so every normalised channel has
|mean| >> std downstream (InstanceNorm statistics precision).
"""
import zlib

import numpy as np

SEED_XOR = 0x5E5A


def param_rng(name: str, seed: int = 0) -> np.random.Generator:
    """seed 0: PCG64(crc32(name) ^ 0x5E5A); seed k > 0: a second, independent weight
    draw for the same architecture, PCG64([crc32(name) ^ 0x5E5A, k])."""
    key = zlib.crc32(name.encode()) ^ SEED_XOR
    return np.random.Generator(np.random.PCG64(key if seed == 0 else [key, int(seed)]))


def synth_param(name: str, shape, affine: str = "unit", seed: int = 0) -> np.ndarray:
    rng = param_rng(name, seed)
    shape = tuple(int(s) for s in shape)
    if len(shape) >= 2:
        fan_in = int(np.prod(shape[1:]))
        bound = 1.0 / np.sqrt(fan_in)
        return rng.uniform(-bound, bound, size=shape).astype(np.float32)
    # 1-D: norm affine parameters (MDX23C has no conv/linear biases)
    if name.endswith("bias"):
        if affine == "random":
            return rng.uniform(-0.2, 0.2, size=shape).astype(np.float32)
        if affine == "stress":
            return rng.uniform(2.0, 4.0, size=shape).astype(np.float32)
        return np.zeros(shape, np.float32)
    if affine in ("random", "stress"):
        return rng.uniform(0.5, 1.5, size=shape).astype(np.float32)
    return np.ones(shape, np.float32)


def synth_state_dict(shapes, affine: str = "unit", seed: int = 0):
    """shapes: iterable of (name, shape) in named_parameters() order."""
    return {name: synth_param(name, shape, affine, seed) for name, shape in shapes}
