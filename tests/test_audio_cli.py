"""CPU tests: WAV codec (sesa/audio_io.py) and the CLI surface (sesa/inference.py)."""
import os

import numpy as np
import pytest


@pytest.mark.parametrize("subtype,tol", [("FLOAT", 0.0), ("PCM_16", 1 / 32768), ("PCM_24", 1 / 8388608)])
def test_wav_roundtrip(tmp_path, subtype, tol):
    from sesa.audio_io import read_audio, write_audio
    rng = np.random.default_rng(0)
    x = (0.1 * rng.standard_normal((2, 5000))).clip(-0.99, 0.99).astype(np.float32)
    p = tmp_path / "a.wav"
    write_audio(str(p), x.T, 44100, subtype=subtype)
    y, sr = read_audio(str(p), sr=44100)
    assert sr == 44100 and y.shape == x.shape
    assert np.abs(y - x).max() <= tol + 1e-7


def test_wav_resample(tmp_path):
    from sesa.audio_io import read_audio, write_audio
    t = np.arange(48000) / 48000.0
    x = np.stack([np.sin(2 * np.pi * 440 * t), np.cos(2 * np.pi * 440 * t)]).astype(np.float32)
    write_audio(str(tmp_path / "b.wav"), x.T, 48000, subtype="FLOAT")
    y, sr = read_audio(str(tmp_path / "b.wav"), sr=44100)
    assert sr == 44100 and abs(y.shape[1] - 44100) <= 1


def test_cli_flags_match_reference_and_reject_cpu(capsys):
    from sesa.inference import build_parser, proc_folder
    a = build_parser().parse_args(["--model_type", "mdx23c", "--config_path", "x", "--input_folder", "i",
                                   "--store_dir", "o", "--extract_instrumental", "--use_tta",
                                   "--export_format", "wav FLOAT", "--enable_amp"])
    assert a.extract_instrumental and a.use_tta and a.enable_amp and a.export_format == "wav FLOAT"
    assert proc_folder(["--force_cpu", "--config_path", "x"]) == 2
