"""The CLI drop-in end to end.

Golden: tests/golden/cli_flow.npz = what the REAL reference run_folder_pytorch_optimized
(inference_pytorch.py:189-274) handed to soundfile.write for each output file -- demix, TTA
(utils.apply_tta :241-292), demud phase remix (:231-248), extract_instrumental (:250-254),
normalize / denormalize (:221-223, :257-260), output naming and subtype (:262-272) -- on the reduced
MDX23C with name-keyed weights (tests/golden/make_golden_cli.py).

GPU: ``python -m sesa.inference``'s ``proc_folder`` on WAV inputs holding the same samples, with a
weights-only checkpoint file; every written file is read back (WAV FLOAT, or FLAC PCM_16 decoded by
libsesa's codec) and compared with the reference's data (quantised like libsndfile's float write for
PCM): per-sample RMS <= 1e-4 (north_star gate).  Also: the progress protocol lines, and a raw native
model passed to apply_tta keeps the precision its session set (ADVICE r1 finding).
"""
import contextlib
import io
import json
import os

import numpy as np
import pytest
import torch
import yaml

from conftest import CONFIGS, GOLDEN, rms

RMS_GATE = 1e-4


def _cases():
    g = np.load(os.path.join(GOLDEN, "cli_flow.npz"))
    return json.loads(str(g["meta"])), g


def _mix(seed, n):
    rng = np.random.default_rng(seed)
    return (0.1 * rng.standard_normal((2, n))).astype(np.float32)


def _setup(tmp_path, case):
    from sesa.audio_io import write_audio
    from sesa.utils import get_model_from_config
    from sesa.weights import synth_state_dict
    with open(os.path.join(CONFIGS, "config_mdx23c_small.yaml")) as f:
        cfg = yaml.safe_load(f)
    if case["normalize"]:
        cfg["inference"]["normalize"] = True
    cfg_path = tmp_path / "config.yaml"
    with open(cfg_path, "w") as f:
        yaml.safe_dump(cfg, f)
    model, _ = get_model_from_config("mdx23c", str(cfg_path))
    ckpt = tmp_path / "model.ckpt"
    torch.save({"state_dict": synth_state_dict(model, affine="random")}, str(ckpt))
    inp = tmp_path / "in"
    inp.mkdir()
    for name, (seed, n) in case["mixes"].items():
        write_audio(str(inp / name), _mix(seed, n).T, 44100, subtype="FLOAT")   # exact float32 samples
    return cfg_path, ckpt, inp


def _argv(case, cfg_path, ckpt, inp, out):
    argv = ["--model_type", "mdx23c", "--config_path", str(cfg_path), "--start_check_point", str(ckpt),
            "--input_folder", str(inp), "--store_dir", str(out)]
    fl = case["flags"]
    for k in ("use_tta", "demud_phaseremix_inst", "extract_instrumental", "flac_file"):
        if fl.get(k):
            argv.append(f"--{k}")
    if "pcm_type" in fl:
        argv += ["--pcm_type", fl["pcm_type"]]
    return argv


def test_cli_parser_defaults_follow_reference():
    from sesa.inference import build_parser, get_soundfile_subtype
    a = build_parser().parse_args(["--config_path", "c"])
    assert a.export_format == "flac PCM_24" and a.pcm_type == "PCM_24" and a.exec_batch == 0
    assert get_soundfile_subtype("PCM_16") == "PCM_16" and get_soundfile_subtype("PCM_16", True) == "FLOAT"
    assert get_soundfile_subtype("nope") == "FLOAT"


@pytest.mark.gpu
@pytest.mark.parametrize("idx", [0, 1])
def test_cli_flow_matches_reference(tmp_path, idx):
    from sesa.audio_io import quantize_pcm, read_any
    from sesa.inference import proc_folder
    metas, g = _cases()
    case = metas[idx]
    cfg_path, ckpt, inp = _setup(tmp_path, case)
    out = tmp_path / "out"
    with contextlib.redirect_stdout(io.StringIO()) as log:
        rc = proc_folder(_argv(case, cfg_path, ckpt, inp, out))
    assert rc == 0, log.getvalue()[-2000:]
    prog = [ln for ln in log.getvalue().splitlines() if ln.startswith("[SESA_PROGRESS]")]
    assert prog == case["progress"]
    assert sorted(os.listdir(out)) == sorted(case["outputs"])
    for fn, o in case["outputs"].items():
        ref = g[o["key"]]                                         # [T, 2] float, as passed to sf.write
        got, sr = read_any(str(out / fn))
        assert sr == o["sr"] and got.shape == ref.T.shape
        if o["subtype"] in ("PCM_16", "PCM_24"):
            bits = 16 if o["subtype"] == "PCM_16" else 24
            ref = (quantize_pcm(ref, bits, clip=True) / float(1 << (bits - 1))).astype(np.float32)
        err = rms(got.T, ref)
        print(f"{case['tag']} {fn}: rms {err:.3e}")
        assert err <= RMS_GATE


@pytest.mark.gpu
def test_raw_model_keeps_session_precision():
    """utils.apply_tta / demix on the raw model after an --enable_amp session (MDX23C: the fp16mix precision):
    the precision the session set must stay (inference_pytorch.py:229 passes the raw model)."""
    from sesa.backend import create_inference_session
    from sesa.utils import apply_tta, demix, get_model_from_config
    from sesa.weights import synth_state_dict
    model, cfg = get_model_from_config("mdx23c", os.path.join(CONFIGS, "config_mdx23c_small.yaml"))
    model.load_state_dict(synth_state_dict(model, affine="random"))
    create_inference_session(model, device="cuda:0", enable_amp=True)
    assert model.precision == "fp16mix" == model._amp_precision
    mix = _mix(3, 40000)
    w = demix(cfg, model, mix, "cuda:0", model_type="mdx23c")
    apply_tta(cfg, model, mix, w, "cuda:0", "mdx23c")
    assert model.precision == "fp16mix" == model._amp_precision


def test_flac_codec_roundtrip(tmp_path):
    """libsesa FLAC encoder / decoder (host code): lossless round trip of the PCM the writer
    quantised, every block-size edge, 16 and 24 bit, stereo and mono."""
    from sesa.audio_io import quantize_pcm, read_any, write_audio
    rng = np.random.default_rng(0)
    for n in (1, 15, 16, 17, 4095, 4096, 4097, 12000):
        for ch in (1, 2):
            for sub, bits in (("PCM_16", 16), ("PCM_24", 24)):
                x = np.clip(0.3 * rng.standard_normal((ch, n)), -1.2, 1.2).astype(np.float32)
                x[:, : n // 3] = 0.25   # a constant run (CONSTANT / low-order FIXED subframes)
                p = tmp_path / "x.flac"
                write_audio(str(p), x.T, 48000, subtype=sub)
                y, sr = read_any(str(p))
                q = quantize_pcm(x, bits, clip=True) / float(1 << (bits - 1))
                assert sr == 48000 and y.shape == x.shape
                assert np.array_equal(y, q.astype(np.float32)), (n, ch, sub)


def test_pcm_quantize_matches_libsndfile_rule():
    from sesa.audio_io import quantize_pcm
    x = np.array([0.0, 0.5, -0.5, 1.0, -1.0, 1.5 / 32767, 2.5 / 32767, 1.2], np.float32)
    q = quantize_pcm(x, 16)
    assert q[:5].tolist() == [0, 16384, -16384, 32767, -32767]   # lrintf(x * 0x7FFF), half to even
    assert q[5] == 2 and q[6] == 2
    assert q[7] == ((int(np.rint(np.float32(1.2) * np.float32(32767))) + 32768) % 65536) - 32768  # wraps


def test_flac_rejects_oversized_streaminfo_total(tmp_path):
    """A corrupt STREAMINFO total_samples (36-bit field) must not size the decode buffer: the reader
    bounds it by what the file's bytes can hold and raises before allocating."""
    from sesa.audio_io import flac_max_samples, read_any, write_audio
    x = np.full((2, 5000), 0.25, np.float32)
    p = tmp_path / "ok.flac"
    write_audio(str(p), x.T, 44100, subtype="PCM_16")
    data = bytearray(p.read_bytes())
    assert read_any(str(p))[0].shape == (2, 5000)
    # STREAMINFO body at byte 8; total_samples = low 4 bits of byte 21 + bytes 22..25
    data[21] = (data[21] & 0xF0) | 0x0F
    data[22:26] = b"\xff\xff\xff\xff"
    bad = tmp_path / "bad.flac"
    bad.write_bytes(bytes(data))
    assert flac_max_samples(bytes(data), 2) < (1 << 36) - 1
    with pytest.raises(Exception, match="corrupt header|STREAMINFO|FLAC"):
        read_any(str(bad))
