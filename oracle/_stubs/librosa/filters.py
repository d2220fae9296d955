"""Restatement of ``librosa.filters.mel`` (librosa's published Slaney mel filterbank; the library is
an unpinned reference dependency, requirements.txt, absent here).  TEST INFRASTRUCTURE.

mel(sr, n_fft, n_mels=128, fmin=0, fmax=sr/2, htk=False, norm='slaney', dtype=float32):
  fft bin centres linspace(0, sr/2, 1 + n_fft//2); n_mels + 2 mel-spaced edge frequencies
  (Slaney scale: linear below 1 kHz at 200/3 Hz per mel, logarithmic above with step
  log(6.4)/27); triangular weights max(0, min(lower, upper)) between neighbouring edges; Slaney
  area normalisation 2 / (f[i+2] - f[i]).  Computed in float64, stored as `dtype`.
Mel-Band-Roformer only uses the support pattern (weights > 0) plus two forced entries, so parity
at this boundary is exact for the pattern; the weights' last bits are unpinned.
"""
import numpy as np


def hz_to_mel(freqs, htk=False):
    freqs = np.asanyarray(freqs, dtype=np.float64)
    if htk:
        return 2595.0 * np.log10(1.0 + freqs / 700.0)
    f_min, f_sp = 0.0, 200.0 / 3
    mels = (freqs - f_min) / f_sp
    min_log_hz = 1000.0
    min_log_mel = (min_log_hz - f_min) / f_sp
    logstep = np.log(6.4) / 27.0
    if freqs.ndim:
        log_t = freqs >= min_log_hz
        mels[log_t] = min_log_mel + np.log(freqs[log_t] / min_log_hz) / logstep
    elif freqs >= min_log_hz:
        mels = min_log_mel + np.log(freqs / min_log_hz) / logstep
    return mels


def mel_to_hz(mels, htk=False):
    mels = np.asanyarray(mels, dtype=np.float64)
    if htk:
        return 700.0 * (10.0 ** (mels / 2595.0) - 1.0)
    f_min, f_sp = 0.0, 200.0 / 3
    freqs = f_min + f_sp * mels
    min_log_hz = 1000.0
    min_log_mel = (min_log_hz - f_min) / f_sp
    logstep = np.log(6.4) / 27.0
    if mels.ndim:
        log_t = mels >= min_log_mel
        freqs[log_t] = min_log_hz * np.exp(logstep * (mels[log_t] - min_log_mel))
    elif mels >= min_log_mel:
        freqs = min_log_hz * np.exp(logstep * (mels - min_log_mel))
    return freqs


def mel(*, sr, n_fft, n_mels=128, fmin=0.0, fmax=None, htk=False, norm="slaney", dtype=np.float32):
    if fmax is None:
        fmax = float(sr) / 2
    weights = np.zeros((n_mels, int(1 + n_fft // 2)), dtype=dtype)
    fftfreqs = np.fft.rfftfreq(n=n_fft, d=1.0 / sr)
    mel_f = mel_to_hz(np.linspace(hz_to_mel(fmin, htk=htk), hz_to_mel(fmax, htk=htk), n_mels + 2), htk=htk)
    fdiff = np.diff(mel_f)
    ramps = np.subtract.outer(mel_f, fftfreqs)
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        weights[i] = np.maximum(0, np.minimum(lower, upper))
    if norm == "slaney":
        enorm = 2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels])
        weights *= enorm[:, np.newaxis]
    return weights
