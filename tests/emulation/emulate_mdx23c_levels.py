"""CPU emulation of the fp16 TFC-conv precisions on every full-chunk MDX23C golden (test infrastructure:
oracle/mdx23c.py with the direct 3x3 conv operands rounded in torch), and a per-conv sensitivity scan.

The direct TFC 3x3 convs (T >= 32, levels 0-3 of encoder and decoder, 32 convs) are the ones the fp16
precisions put on fp16 MFMA (sesa_mdx23c.hip); everything else stays ~fp32 (bf16x3).

Usage:
  python tests/emulation/emulate_mdx23c_levels.py modes  [fixture ...]   # fp32 / fp16 / fp16w2 / mixes
  python tests/emulation/emulate_mdx23c_levels.py scan   fixture [lo:hi]  # fp16 on one conv at a time
MODES may also name a libsesa SESA_PREC_F16MIX plan as plan:<16 digits>.  Per-conv modes are written as a 32-character string over {3: bf16x3/fp32, 2: fp16w2, 1: fp16,
4: fp16 weights x the activation as fp16 hi + lo (two passes)}, conv order =
call order (encoder L0 block0 tfc1, tfc2, block1 tfc1, tfc2, L1 ..., decoder L3 ... L0).
"""
import os
import sys
import types

import numpy as np
import torch
import torch.nn.functional as F
import yaml

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import oracle.mdx23c as om  # noqa: E402
from oracle.weights import synth_state_dict  # noqa: E402

torch.set_num_threads(os.cpu_count())
CFG = yaml.safe_load(open(REPO + "/sesa-audio-separation_amd/sesa/configs/config_vocals_mdx23c.yaml"))
OTHER = set(filter(None, os.environ.get("OTHER", "").split(",")))
FIXTURES = ["mdx23c_full_chunk.npz", "mdx23c_full_sines.npz", "mdx23c_full_loud.npz", "mdx23c_full_wseed2.npz"]


def f16(t):
    return t.half().float()


def w_f16x2(w):
    hi = w.half().float()
    return hi + (w - hi).half().float()


def make(per_conv, tdf=None):
    """tdf: None, or a set of TDF stack indices (call order: encoder L0..L4, bottleneck, decoder L4..L0 = 0..10)
    whose two Linears run with fp16 activations and weights."""
    ns = types.SimpleNamespace(**{k: getattr(F, k) for k in dir(F) if not k.startswith("_")})
    idx = [0]
    lin = [0]

    def linear(inp, w, *a, **k):
        stack = lin[0] // 4          # 2 blocks x 2 Linears per TFC_TDF stack
        lin[0] += 1
        if tdf and stack in tdf:
            return F.linear(f16(inp), f16(w), *a, **k)
        return F.linear(inp, w, *a, **k)

    ns.linear = linear

    def conv2d(inp, w, *a, **k):
        # OTHER (env, comma list): also round these operands to fp16 -- down (2x2 s2 downscale), sc (fused 1x1
        # shortcuts, every level), scw (the T >= 32 shortcuts' weights only), sca (their
        # activation only), c33 (3x3 convs of the T < 32 levels)
        if w.shape[-1] == 2 and "down" in OTHER:
            return F.conv2d(f16(inp), f16(w), *a, **k)
        if w.shape[-1] == 1 and w.shape[0] != w.shape[1] and "sc" in OTHER and inp.shape[1] > 4:
            return F.conv2d(f16(inp), f16(w), *a, **k)
        if w.shape[-1] == 1 and w.shape[0] != w.shape[1] and "scw" in OTHER and inp.shape[1] > 4 and inp.shape[2] >= 32:
            return F.conv2d(inp, f16(w), *a, **k)   # shortcut of the fp16 convs: fp16 weights x exact activation
        if w.shape[-1] == 1 and w.shape[0] != w.shape[1] and "sca" in OTHER and inp.shape[1] > 4 and inp.shape[2] >= 32:
            return F.conv2d(f16(inp), w_f16x2(w), *a, **k)   # fp16 activation x fp16 hi + lo weights
        if w.shape[-1] == 3 and inp.shape[2] < 32 and "c33" in OTHER:
            return F.conv2d(f16(inp), f16(w), *a, **k)
        if w.shape[-1] == 3 and inp.shape[2] >= 32:
            m = per_conv[idx[0]]
            idx[0] += 1
            if m == "1":
                return F.conv2d(f16(inp), f16(w), *a, **k)
            if m == "2":
                return F.conv2d(f16(inp), w_f16x2(w), *a, **k)
            if m == "4":   # activation as fp16 hi + lo (~exact), fp16 weights: two passes
                return F.conv2d(inp, f16(w), *a, **k)
        return F.conv2d(inp, w, *a, **k)

    ns.conv2d = conv2d

    def conv_transpose2d(inp, w, *a, **k):
        if "up" in OTHER:
            return F.conv_transpose2d(f16(inp), f16(w), *a, **k)
        return F.conv_transpose2d(inp, w, *a, **k)

    ns.conv_transpose2d = conv_transpose2d
    return ns, idx


_cache = {}


def load(fixture):
    if fixture not in _cache:
        g = np.load(os.path.join(REPO, "tests", "golden", fixture))
        seed = int(g["weight_seed"]) if "weight_seed" in g.files else 0
        params = om.to_torch_params(synth_state_dict(om.param_shapes(CFG), affine=str(g["affine"]), seed=seed))
        _cache[fixture] = (params, torch.from_numpy(g["x"]), g["y"].astype(np.float64))
    return _cache[fixture]


def run(fixture, per_conv, tdf=None):
    params, x, ref = load(fixture)
    om.F, idx = make(per_conv, tdf)
    try:
        with torch.inference_mode():
            y = om.forward(params, CFG, x).numpy().astype(np.float64)
    finally:
        om.F = F
    assert per_conv == "3" * 32 or idx[0] == 32, idx
    d = y - ref
    rms = float(np.sqrt(np.mean(d ** 2)))
    ref_rms = float(np.sqrt(np.mean(ref ** 2)))
    return rms, rms / ref_rms, float(np.abs(d).max()), ref_rms


NAMED = {"fp32": "3" * 32, "fp16": "1" * 32, "fp16w2": "2" * 32,
         "fp16_L0w2": "2" * 4 + "1" * 24 + "2" * 4,            # level-0 encoder + decoder convs fp16w2
         "fp16_L01w2": "2" * 8 + "1" * 16 + "2" * 8}


def plan_to_convs(plan16):
    """libsesa SESA_PREC_F16MIX plan (encoder levels 0..7, decoder levels 0..7) -> 32 per-conv digits in call
    order (encoder L0..L3, decoder L3..L0, 4 convs per level)."""
    return "".join(plan16[lv] * 4 for lv in range(4)) + "".join(plan16[8 + lv] * 4 for lv in (3, 2, 1, 0))


def main():
    what = sys.argv[1]
    if what == "modes":
        fixtures = sys.argv[2:] or FIXTURES
        modes = os.environ.get("MODES", "fp32,fp16,fp16w2").split(",")
        # TDF=...: those TDF stacks' Linears in fp16 too (the fp16mix default: stacks 5-10)
        # (comma-separated stacks or lo-hi ranges, e.g. 0,4-10)
        tdf = None
        if os.environ.get("TDF"):
            tdf = set()
            for part in os.environ["TDF"].split(","):
                lo, _, hi = part.partition("-")
                tdf |= set(range(int(lo), int(hi or lo) + 1))
        for fx in fixtures:
            for m in modes:
                pc = NAMED.get(m, plan_to_convs(m[5:]) if m.startswith("plan:") else m)
                r, rel, mx, rr = run(fx, pc, tdf)
                print(f"{fx:28s} {m:12s} rms {r:.3e} rel {rel:.3e} max {mx:.3e} (ref rms {rr:.3e})", flush=True)
    elif what == "tdfscan":   # fp16 TDF Linears of one stack at a time, on top of a conv plan
        fx = sys.argv[2]
        pc = plan_to_convs(sys.argv[3]) if len(sys.argv) > 3 else "3" * 32
        base = run(fx, pc)[0]
        print(f"conv plan alone: rms {base:.3e}", flush=True)
        for st in range(11):
            r = run(fx, pc, {st})[0]
            print(f"tdf stack {st:2d} fp16: rms {r:.3e} (added {max(r * r - base * base, 0) ** 0.5:.3e})", flush=True)
        r = run(fx, pc, set(range(6, 11)))[0]
        print(f"decoder TDF stacks (6-10) fp16: rms {r:.3e}", flush=True)
    elif what == "scan":
        fx = sys.argv[2]
        lo, hi = (int(v) for v in (sys.argv[3] if len(sys.argv) > 3 else "0:32").split(":"))
        for i in range(lo, hi):
            pc = "3" * i + "1" + "3" * (31 - i)
            r, rel, mx, _ = run(fx, pc)
            print(f"conv {i:2d} fp16 alone: rms {r:.3e}", flush=True)


if __name__ == "__main__":
    main()
