"""Round 5: workspace hygiene of every native forward (the streams > 1 discrepancy).

tools/streams_debug3.py showed the MDX23C forward OUTPUT of group 0 differing (x identical) when it ran beside
forwards on other streams -- and which stream count fails changed between boxes, i.e. it depends on what the
main stream's workspace held BEFORE the forward.  Hypotheses: (a) a kernel reads workspace bytes that this
forward never wrote (stale data of an earlier forward), (b) a kernel writes outside the buffers it was given.

For each model / config / precision / batch this calls sesa_<net>_forward directly with
  * the workspace pre-filled with 0x00, 0xFF (NaN in f32 / f64 / f16 / bf16) and random bytes -- outputs must be
    bit-identical and finite (a difference pins (a));
  * 1 MiB guard bands of 0xA5 before and after the workspace, the input and the output -- they must survive (b).
"""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "sesa-audio-separation_amd"), os.path.join(REPO, "tests")]
from conftest import CONFIGS  # noqa: E402
from sesa import _native as N  # noqa: E402
from sesa.utils import get_model_from_config  # noqa: E402
from sesa.weights import synth_model_state, synth_state_dict  # noqa: E402

dev = torch.device("cuda:0")
G = 1 << 20


def guarded(nbytes, fill):
    big = torch.full((nbytes + 2 * G,), 0xA5, dtype=torch.uint8, device=dev)
    mid = big[G:G + nbytes]
    if fill == "rand":
        mid.copy_(torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device=dev))
    else:
        mid.fill_(fill)
    return big, mid


def guards_ok(big, nbytes):
    return bool((big[:G] == 0xA5).all()) and bool((big[G + nbytes:] == 0xA5).all())


def first_bad(big, nbytes):
    lo = torch.nonzero(big[:G] != 0xA5).flatten()
    hi = torch.nonzero(big[G + nbytes:] != 0xA5).flatten()
    return (int(lo[0]) - G if lo.numel() else None, int(hi[0]) if hi.numel() else None,
            int(lo.numel()) + int(hi.numel()))


def run(kind, cfg_name, precision, batch, seed=3):
    m, c = get_model_from_config(kind, os.path.join(CONFIGS, cfg_name))
    m.load_state_dict(synth_state_dict(m, affine="random") if kind == "mdx23c" else
                      synth_model_state(m, affine="random"), strict=True)
    m.set_precision(precision)
    L = int(c.training.samplerate * c.training.segment) if kind == "htdemucs" else int(c.audio.chunk_size)
    h = m._handle(dev, L)
    need = int(m._fn("workspace_size")(h, batch))
    rng = np.random.default_rng(seed)
    x = torch.from_numpy((0.1 * rng.standard_normal((batch, 2, L))).astype(np.float32)).to(dev)
    out_shape = list(m._out_shape(batch, 2, L))
    n_out = int(np.prod(out_shape)) * 4
    outs, msgs = {}, []
    st = torch.cuda.current_stream(dev).cuda_stream
    for fill in (0x00, 0xFF, "rand", 0xFF):
        wbig, ws = guarded(need, fill)
        xbig, xm = guarded(x.numel() * 4, 0)
        xm.view(torch.float32).copy_(x.flatten())
        obig, om = guarded(n_out, 0x5A)
        N.check(m._fn("forward")(h, xm.data_ptr(), batch, om.data_ptr(), ws.data_ptr(), need, st), "forward")
        torch.cuda.synchronize()
        y = om.view(torch.float32).clone()
        outs[str(fill)] = y
        for nm, big, nb in (("workspace", wbig, need), ("input", xbig, x.numel() * 4), ("output", obig, n_out)):
            if not guards_ok(big, nb):
                msgs.append(f"{nm} guard overwritten (fill {fill}): first before/after offsets, count {first_bad(big, nb)}")
        if not bool(torch.isfinite(y).all()):
            msgs.append(f"non-finite output with workspace fill {fill}: {int((~torch.isfinite(y)).sum())} values")
    ref = outs["0"]
    for k, y in outs.items():
        d = float((y - ref).abs().max()) if torch.isfinite(y).all() else float("nan")
        if not torch.equal(y, ref):
            diff = (y != ref).view(batch, -1)
            msgs.append(f"fill {k} vs 0x00: max diff {d:.3e}, differing per item {diff.sum(1).tolist()}")
    print(f"{kind:12s} {cfg_name:34s} {precision:8s} B={batch}: ws {need / 2**20:.1f} MiB  "
          + ("OK" if not msgs else "PROBLEM\n    " + "\n    ".join(msgs)), flush=True)
    m._release()
    return not msgs


CASES = [("mdx23c", "config_mdx23c_small.yaml", p, b) for p in ("bf16x3", "fp16mix", "fp16") for b in (1, 3)] + [
    ("mdx23c", "config_vocals_mdx23c.yaml", p, 2) for p in ("bf16x3", "fp16mix")] + [
    ("bs_roformer", "config_bs_roformer_small.yaml", p, 2) for p in ("bf16x3", "fp16")] + [
    ("mel_band_roformer", "config_mel_band_roformer_small.yaml", "fp16", 2),
    ("bs_roformer", "config_bs_roformer_vocals.yaml", "fp16", 2),
    ("scnet", "config_scnet_small.yaml", "bf16x3", 2), ("scnet", "config_scnet_small.yaml", "fp16mix", 3),
    ("scnet", "config_musdb18_scnet.yaml", "fp16mix", 2),
    ("htdemucs", "config_htdemucs_small.yaml", "bf16x3", 2), ("htdemucs", "config_htdemucs_small.yaml", "fp16mix", 3),
    ("htdemucs", "config_musdb18_htdemucs.yaml", "fp16mix", 2)]

if __name__ == "__main__":
    only = sys.argv[1] if len(sys.argv) > 1 else None
    bad = [c for c in CASES if (only is None or c[0] == only) and not run(*c)]
    print(f"{len(bad)} case(s) with problems")
