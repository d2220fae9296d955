"""Ensemble blend.

CPU: the NumPy oracle (oracle/ensemble.py) against the reference's own process_waveform /
process_spectral outputs (tests/golden/ensemble.npz); the CLI surface.
GPU (``gpu``): libsesa ``sesa_blend_f32`` against the golden vectors and against the oracle's
buffer loop on ragged lengths.  Tolerance: float64 arithmetic on both sides -> 1e-12 absolute
(waveform methods are exact up to summation order; spectral ones differ by FFT rounding).
"""
import numpy as np
import pytest
import torch

from oracle import ensemble as oe

TOL = 1e-12


def test_oracle_matches_reference(golden):
    g = golden("ensemble.npz")
    w = g["waves"]
    for m in ("avg_wave", "median_wave", "max_wave", "min_wave"):
        assert np.abs(oe.process_waveform(w, m, g["weights"]) - g[m]).max() == 0.0
    assert np.abs(oe.process_waveform(w, "avg_wave") - g["avg_wave_unweighted"]).max() == 0.0
    for m in ("max_fft", "min_fft", "median_fft"):
        assert np.abs(oe.process_spectral(w, m) - g[m]).max() < 1e-15
    assert np.abs(oe.process_spectral(g["odd"], "median_fft") - g["median_fft_odd"]).max() < 1e-15
    assert np.abs(oe.process_spectral(g["small"], "max_fft") - g["max_fft_small"]).max() < 1e-15
    assert (oe.process_spectral(w[:, :, :200], "max_fft") is None) == bool(g["short_is_none"])


def test_cli_surface():
    from sesa.ensemble import build_parser
    a = build_parser().parse_args(["--files", "a.wav", "b.wav", "--type", "median_fft", "--weights", "1", "2",
                                   "--output", "o.wav"])
    assert a.files == ["a.wav", "b.wav"] and a.type == "median_fft" and a.weights == [1.0, 2.0] and a.buffer == 32768
    with pytest.raises(SystemExit):
        build_parser().parse_args(["--files", "a.wav", "--type", "bogus", "--output", "o"])


@pytest.mark.gpu
def test_device_blend_matches_reference(golden):
    from sesa.ensemble import AudioEnsembleEngine
    g = golden("ensemble.npz")
    eng = AudioEnsembleEngine()
    # The device blend takes float32 stems (what the separator writes); the fixture's waves are float64,
    # so the oracle is re-run on the same float32-rounded values (1e-12 below), and the reference's own
    # outputs bound the input rounding alone: |x - fp32(x)| <= 2^-24 |x| per sample, <= 1e-7 here.
    w = g["waves"].astype(np.float32)
    ref_w = w.astype(np.float64)
    assert np.abs(ref_w - g["waves"]).max() <= 2.0 ** -24 * np.abs(g["waves"]).max()
    for m in ("avg_wave", "median_wave", "max_wave", "min_wave", "max_fft", "min_fft", "median_fft"):
        got = eng.process_waveform(w, m, g["weights"]) if m.endswith("_wave") else eng.process_spectral(w, m)
        assert np.abs(got - g[m]).max() <= 1e-7, m
    for m in ("avg_wave", "median_wave", "max_wave", "min_wave"):
        exp = oe.process_waveform(ref_w, m, g["weights"])
        assert np.abs(eng.process_waveform(w, m, g["weights"]) - exp).max() <= TOL, m
    for m in ("max_fft", "min_fft", "median_fft"):
        exp = oe.process_spectral(ref_w, m)
        assert np.abs(eng.process_spectral(w, m) - exp).max() <= TOL, m
    odd = g["odd"].astype(np.float32)
    assert np.abs(eng.process_spectral(odd, "median_fft") - oe.process_spectral(odd.astype(np.float64), "median_fft")).max() <= TOL
    small = g["small"].astype(np.float32)
    assert np.abs(eng.process_spectral(small, "max_fft") - oe.process_spectral(small.astype(np.float64), "max_fft")).max() <= TOL
    assert eng.process_spectral(w[:, :, :200], "max_fft") is None


@pytest.mark.gpu
@pytest.mark.parametrize("L", [70000, 65636, 4000])
@pytest.mark.parametrize("method", ["avg_wave", "median_wave", "max_fft", "median_fft", "min_fft"])
def test_device_buffer_loop_matches_oracle(L, method):
    from sesa.ensemble import blend_device
    rng = np.random.default_rng(L)
    waves = (0.1 * rng.standard_normal((3, 2, L))).astype(np.float32)
    weights = [3.0, 1.0, 2.0]
    got = blend_device(waves, method, weights, buffer=32768).cpu().numpy()
    exp = oe.blend(waves.astype(np.float64), method, weights, buffer=32768)
    assert got.shape == exp.shape
    assert np.abs(got - exp).max() <= TOL


@pytest.mark.gpu
@pytest.mark.parametrize("n_files", [9, 13])
@pytest.mark.parametrize("method", ["avg_wave", "median_wave", "max_wave", "min_wave", "max_fft", "median_fft",
                                    "min_fft"])
def test_device_blend_many_files(n_files, method):
    """More than 8 inputs (ensemble.py has no file limit): every method against the oracle."""
    from sesa.ensemble import blend_device
    rng = np.random.default_rng(n_files)
    waves = (0.1 * rng.standard_normal((n_files, 2, 40000))).astype(np.float32)
    weights = list(rng.uniform(0.5, 2.0, n_files))
    got = blend_device(waves, method, weights, buffer=32768).cpu().numpy()
    exp = oe.blend(waves.astype(np.float64), method, weights, buffer=32768)
    assert np.abs(got - exp).max() <= TOL


@pytest.mark.gpu
@pytest.mark.parametrize("method", ["median_wave", "max_wave", "min_wave"])
def test_device_blend_nan_propagates(method):
    """np.max / np.min / np.median propagate NaN (fmax / fmin would drop it)."""
    from sesa.ensemble import blend_device
    waves = np.full((3, 1, 1000), 0.25, np.float32)
    waves[1, 0, 17] = np.nan
    got = blend_device(waves, method).cpu().numpy()
    assert np.isnan(got[0, 17]) and np.isfinite(np.delete(got[0], 17)).all()


@pytest.mark.gpu
def test_run_ensemble_writes_pcm24(tmp_path, capsys):
    from sesa.audio_io import quantize_pcm, read_wav, write_audio
    from sesa.ensemble import main
    rng = np.random.default_rng(5)
    files = []
    for i in range(3):
        x = (0.1 * rng.standard_normal((2, 50000 + 1000 * i))).astype(np.float32)
        p = tmp_path / f"in{i}.wav"
        write_audio(str(p), x.T, 44100, subtype="FLOAT")
        files.append(str(p))
    out = tmp_path / "out.wav"
    assert main(["--files", *files, "--type", "max_fft", "--output", str(out)]) == 0
    assert "[SESA_PROGRESS]100" in capsys.readouterr().out
    y, sr = read_wav(str(out))
    ins = np.stack([read_wav(f)[0][:, :50000] for f in files]).astype(np.float64)
    exp = oe.blend(ins, "max_fft")
    assert sr == 44100 and y.shape == (2, 50000)
    # soundfile's PCM_24 write (libsndfile: lrintf(x * 0x7FFFFF)) read back as int / 2^23
    exp_q = quantize_pcm(exp.astype(np.float32), 24) / 8388608.0
    assert np.abs(y - exp_q).max() <= 1.0 / 8388608 + 1e-9     # at most one PCM_24 step (rounding ties)
    assert main(["--files", files[0], "--type", "avg_wave", "--output", str(out)]) == 1   # < 2 files
