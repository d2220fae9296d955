"""Round 5: which kernel class makes concurrent forwards on several streams disagree with one stream?

tools/ws_guard.py showed every native forward independent of its workspace's prior contents and writing nothing
outside its buffers, yet tools/streams_debug3.py saw a main-stream forward's OUTPUT change when forwards ran on
other streams beside it (and which stream count failed varied between boxes).  libsesa's SESA_DEBUG_SYNC hook
(sesa_profile.hip) device-synchronises after launches: "all" serialises every launch; "except:<k>" leaves only
kernel class k free to overlap other streams' work.  Each configuration runs in a fresh process (the variable is
read once): the streams=1 reference, then REPS runs each of streams 2, 3 and 4, counting runs whose local OLA
buffer differs from the reference.

Usage: python tools/streams_bisect.py [model] [precision]    (child mode: --child <sync> <model> <precision>)
"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLASSES = {"conv3x3": 0, "conv1x1": 1, "down": 2, "up": 3, "tdf": 4, "stft": 5, "istft": 6, "act": 7, "ola": 12,
           "conv3x3_x3": 14, "tokgemm": 8, "attn": 9, "lstm": 10, "simt": 11, "hconv": 13, "dft": 15}
REPS = 3


def child(sync, model, precision):
    import numpy as np
    import torch
    sys.path[:0] = [REPO, os.path.join(REPO, "sesa-audio-separation_amd"), os.path.join(REPO, "tests")]
    from conftest import CONFIGS
    from sesa.parallel import local_accumulate_device, shard_plan
    import sesa.parallel as par
    from sesa.utils import get_model_from_config
    from sesa.weights import synth_model_state, synth_state_dict
    dev = torch.device("cuda:0")
    cfg = {"mdx23c": "config_mdx23c_small.yaml", "bs_roformer": "config_bs_roformer_small.yaml",
           "scnet": "config_scnet_small.yaml", "htdemucs": "config_htdemucs_small.yaml"}[model]
    m, c = get_model_from_config(model, os.path.join(CONFIGS, cfg))
    m.load_state_dict(synth_state_dict(m, affine="random") if model == "mdx23c" else
                      synth_model_state(m, affine="random"), strict=True)
    m.set_precision(precision)
    rng = np.random.default_rng(2)
    L = 400000
    mix = torch.from_numpy((0.1 * rng.standard_normal((2, L))).astype(np.float32)).to(dev)
    mode = "demucs" if model == "htdemucs" else "generic"
    plan = shard_plan(c, L, 1, mode)
    from sesa.config import prefer_target_instrument
    ni = len(c.training.instruments) if mode == "demucs" else len(prefer_target_instrument(c))
    rows = 2 * ni
    par._ALLOW_STREAMS = True
    ref = local_accumulate_device(c, m, mix, plan, 0, rows, 3, 1)
    torch.cuda.synchronize()
    bad = []
    for s in (2, 3, 4):
        for _ in range(REPS):
            out = local_accumulate_device(c, m, mix, plan, 0, rows, 3, s)
            torch.cuda.synchronize()
            d = float((out - ref).abs().max())
            if d != 0.0:
                bad.append((s, d))
    print(f"RESULT sync={sync} {model} {precision}: {len(bad)} of {3 * REPS} multi-stream runs differ "
          + (f"(streams, max diff) {bad}" if bad else ""), flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child(*sys.argv[2:5])
        return
    model = sys.argv[1] if len(sys.argv) > 1 else "mdx23c"
    precision = sys.argv[2] if len(sys.argv) > 2 else "bf16x3"
    kset = {"mdx23c": ["conv3x3", "conv1x1", "down", "up", "tdf", "stft", "istft", "act", "ola", "conv3x3_x3"],
            "bs_roformer": ["tokgemm", "attn", "act", "stft", "istft", "ola"],
            "scnet": ["tokgemm", "lstm", "simt", "dft", "act", "stft", "istft", "ola"],
            "htdemucs": ["tokgemm", "hconv", "attn", "simt", "stft", "istft", "ola"]}[model]
    configs = ["none", "all"] + [f"except:{CLASSES[k]}" for k in kset]
    for sync in configs:
        env = dict(os.environ)
        if sync != "none":
            env["SESA_DEBUG_SYNC"] = sync
        r = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), "--child", sync, model, precision],
                           env=env, capture_output=True, text=True, timeout=300)
        lines = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT")]
        name = sync if not sync.startswith("except:") else \
            "except " + [k for k, v in CLASSES.items() if v == int(sync[7:])][0]
        print(f"[{name}] " + (lines[0] if lines else f"rc={r.returncode} {r.stderr[-800:]}"), flush=True)
        if r.returncode != 0:
            break


if __name__ == "__main__":
    main()
