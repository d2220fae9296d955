"""Round 5: configs[4] blend parity per member precision (which MDX23C plan holds every blend <= 8e-5?).

For each full-width ensemble fixture (tests/golden/ensemble_full{,_loud,_wseed2}.npz) the BS-Roformer (fp16) and
SCNet (fp16mix) stems are computed once; the MDX23C stem in each candidate precision / fp16mix plan; then every
blend method against the reference blend.  Prints one line per (fixture, candidate, method) and a summary of the
worst blend per candidate.
"""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "sesa-audio-separation_amd"), os.path.join(REPO, "tests")]
from conftest import CONFIGS  # noqa: E402
from sesa import _native  # noqa: E402
from sesa.ensemble import blend_device  # noqa: E402
from sesa.parallel import demix_sharded  # noqa: E402
from sesa.utils import get_model_from_config  # noqa: E402
from sesa.weights import synth_model_state, synth_state_dict  # noqa: E402

FIX = ("ensemble_full.npz", "ensemble_full_loud.npz", "ensemble_full_wseed2.npz")
METHODS = ("avg_wave", "median_wave", "max_wave", "min_wave", "max_fft", "min_fft", "median_fft")
# (label, precision, fp16mix conv plan or None)
CANDS = [("fp16mix", "fp16mix", None), ("bf16x3", "bf16x3", None), ("fp16w2", "fp16w2", None),
         ("plan1321", "fp16mix", "1321111111111111"), ("plan1331", "fp16mix", "1331111111111111"),
         ("plan2322", "fp16mix", "2322222222222222"), ("plan1311dec2", "fp16mix", "1311111122222222"),
         ("plan3311", "fp16mix", "3311111111111111")]
dev = torch.device("cuda:0")


def rms(a, b):
    return float(np.sqrt(np.mean((np.asarray(a, np.float64) - np.asarray(b, np.float64)) ** 2)))


def stem(kind, cfg_name, g, prec, plan=None):
    seed = int(g["weight_seed"])
    affine = str(g[f"affine_{kind}"])
    m, c = get_model_from_config(kind, os.path.join(CONFIGS, cfg_name))
    m.load_state_dict(synth_state_dict(m, affine=affine, seed=seed) if kind == "mdx23c" else
                      synth_model_state(m, affine=affine, seed=seed), strict=True)
    m.set_precision(prec)
    prev = ctypes.create_string_buffer(17)
    if plan:
        _native.check(_native.lib().sesa_mdx23c_set_f16_plan(plan.encode(), prev))
    try:
        est = demix_sharded(c, m, torch.from_numpy(g["mix"]).to(dev), dev, rank=0, world=1, exec_batch=2)
    finally:
        if plan:
            _native.check(_native.lib().sesa_mdx23c_set_f16_plan(prev.value, None))
    from sesa.config import prefer_target_instrument
    return est[prefer_target_instrument(c).index("vocals")].clone()


def main():
    worst = {}
    for fx in FIX:
        g = np.load(os.path.join(REPO, "tests", "golden", fx), allow_pickle=False)
        bsr = stem("bs_roformer", "config_bs_roformer_vocals.yaml", g, "fp16")
        scn = stem("scnet", "config_musdb18_scnet.yaml", g, "fp16mix")
        print(f"{fx}: bsr fp16 {rms(bsr.cpu(), g['vocals_bs_roformer']):.3e}  "
              f"scnet fp16mix {rms(scn.cpu(), g['vocals_scnet']):.3e}", flush=True)
        for label, prec, plan in CANDS:
            mdx = stem("mdx23c", "config_vocals_mdx23c.yaml", g, prec, plan)
            x = torch.stack([mdx, bsr, scn])
            errs = {}
            for meth in METHODS:
                y = blend_device(x, meth, list(g["weights"]) if meth == "avg_wave" else None)
                errs[meth] = rms(y.cpu(), g[f"blend_{meth}"])
            w = max(errs.values())
            worst[label] = max(worst.get(label, 0.0), w)
            print(f"  {label:13s} mdx {rms(mdx.cpu(), g['vocals_mdx23c']):.3e}  "
                  + " ".join(f"{k} {v:.2e}" for k, v in errs.items()), flush=True)
    print("worst blend per candidate:", {k: f"{v:.3e}" for k, v in worst.items()})


if __name__ == "__main__":
    main()
