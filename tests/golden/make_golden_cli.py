"""Golden fixtures for the CLI per-file flow (reference inference_pytorch.run_folder_pytorch_optimized).

Run here (not on the GPU box):  python tests/golden/make_golden_cli.py

Imports /root/reference (stubs as make_golden.py) and runs the REAL
``run_folder_pytorch_optimized(backend, args, config, "cpu", model)`` (inference_pytorch.py:189-274)
on the reduced MDX23C with name-keyed weights: demix, TTA (utils.apply_tta, :241-292), demud
phase remix (:231-248), extract_instrumental (:250-254), normalize / denormalize (:221-223,
:257-260) and the output naming / subtype choice (:262-272).  ``librosa.load`` is replaced by a
lookup of fixed mixes and ``soundfile.write`` by a recorder, so the fixture holds exactly what the
reference would hand to soundfile: file name, float data [T, 2], rate and subtype.
"""
import argparse
import contextlib
import io
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402

# (tag, flags, normalize, mixes {file name: (seed, length)})
CASES = [
    ("tta_demud_instr", dict(use_tta=True, demud_phaseremix_inst=True, extract_instrumental=True), False,
     {"song one.wav": (41, 70000)}),
    ("normalize_pcm16_flac", dict(flac_file=True, pcm_type="PCM_16", extract_instrumental=True), True,
     {"b.wav": (42, 50000), "a_very_long_file_name_for_shortening_test.wav": (43, 30000)}),
]


_BE = []


def run_case(tag, flags, normalize, mixes):
    import inference_pytorch as ip
    from pytorch_backend import PyTorchBackend
    if not _BE:   # one backend: its __init__ sets the interop thread count, which torch allows once
        _BE.append(PyTorchBackend(device="cpu", optimize_mode="default"))
    cfg = mg.load_cfg("config_mdx23c_small.yaml")
    if normalize:
        cfg["inference"]["normalize"] = True
    model, _ = mg.build_ref_model(cfg, "random")
    be = _BE[0]
    be.compiled_model = model
    be.model = model
    be.use_amp = False
    config = mg.to_attr(json.loads(json.dumps(cfg)))
    written = {}
    arrays = {}
    sys.modules["librosa"].load = lambda path, sr=None, mono=False: (
        mg.mix_signal(*mixes[os.path.basename(path)]), sr)
    sys.modules["soundfile"].write = lambda path, data, sr, subtype=None: written.__setitem__(
        os.path.basename(path), (np.array(data, np.float32), sr, subtype))
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        inp = os.path.join(d, "in")
        os.makedirs(inp)
        for name in mixes:
            open(os.path.join(inp, name), "wb").close()
        base = dict(input_folder=inp, store_dir=os.path.join(d, "out"), disable_detailed_pbar=False,
                    use_tta=False, demud_phaseremix_inst=False, extract_instrumental=False, flac_file=False,
                    pcm_type="PCM_24", export_format="flac PCM_24", model_type="mdx23c")
        base.update(flags)
        args = argparse.Namespace(**base)
        with contextlib.redirect_stdout(io.StringIO()) as out:
            ip.run_folder_pytorch_optimized(be, args, config, "cpu", model=model)
    meta = {"tag": tag, "flags": flags, "normalize": normalize, "mixes": {k: list(v) for k, v in mixes.items()},
            "outputs": {}}
    for i, (fn, (data, sr, subtype)) in enumerate(sorted(written.items())):
        arrays[f"{tag}_out{i}"] = data
        meta["outputs"][fn] = {"key": f"{tag}_out{i}", "sr": sr, "subtype": subtype}
    meta["progress"] = [ln for ln in out.getvalue().splitlines() if ln.startswith("[SESA_PROGRESS]")]
    return meta, arrays


def main():
    mg.install_stubs()
    torch.set_num_threads(os.cpu_count())
    metas, arrays = [], {}
    with torch.inference_mode():
        for case in CASES:
            m, a = run_case(*case)
            metas.append(m)
            arrays.update(a)
            print(m["tag"], sorted(m["outputs"]))
    arrays["meta"] = np.array(json.dumps(metas))
    mg.save("cli_flow.npz", **arrays)


if __name__ == "__main__":
    main()
