"""NumPy float64 restatement of the ensemble blend.  TEST INFRASTRUCTURE.

Restates ``/root/reference/ensemble.py``:

* ``process_waveform`` (:172-183) -- avg (np.average with normalised float32 weights, :288-293),
  median, max, min over the file axis.
* ``process_spectral`` (:185-256) -- per channel scipy.signal.stft(nperseg=min(1024, len),
  noverlap=nperseg//2, periodic Hann, boundary zeros, padded, scaling 'spectrum'), combined
  magnitude (max/min/median over files) with the phase of file 0, scipy.signal.istft, then
  truncate / zero-pad to the chunk length; None when the chunk is shorter than 256 samples.
* ``blend`` -- the buffer loop of ``run_ensemble`` (:319-372): independent ``buffer``-frame
  pieces, spectral failure -> avg_wave fallback with the weights.

scipy's STFT/ISTFT are restated explicitly (numpy rfft / irfft) so the arithmetic is visible;
both are pinned against the reference's own process_spectral outputs (tests/golden/ensemble.npz).
"""
import numpy as np


def process_waveform(chunks, method, weights=None):
    if method == "avg_wave":
        if weights is not None:
            return np.average(chunks, axis=0, weights=weights)
        return np.mean(chunks, axis=0)
    if method == "median_wave":
        return np.median(chunks, axis=0)
    if method == "max_wave":
        return np.max(chunks, axis=0)
    if method == "min_wave":
        return np.min(chunks, axis=0)
    raise ValueError(method)


def hann_periodic(n):
    return 0.5 - 0.5 * np.cos(2.0 * np.pi * np.arange(n) / n)


def stft(x, nperseg):
    """scipy.signal.stft(x, nperseg, noverlap=nperseg//2, window='hann') -> Z [freq, time]."""
    nstep = nperseg - nperseg // 2
    win = hann_periodic(nperseg)
    x = np.concatenate([np.zeros(nperseg // 2), x, np.zeros(nperseg // 2)])       # boundary='zeros'
    nadd = (-(x.shape[-1] - nperseg) % nstep) % nperseg                              # padded=True
    x = np.concatenate([x, np.zeros(nadd)])
    nseg = (x.shape[-1] - nperseg) // nstep + 1
    frames = np.stack([x[i * nstep:i * nstep + nperseg] for i in range(nseg)])
    Z = np.fft.rfft(frames * win, n=nperseg, axis=-1) / win.sum()                    # scaling='spectrum'
    return Z.T


def istft(Z, nperseg):
    """scipy.signal.istft(Z, nperseg, noverlap=nperseg//2, window='hann', boundary=True)."""
    nstep = nperseg - nperseg // 2
    win = hann_periodic(nperseg)
    nseg = Z.shape[-1]
    xsubs = np.fft.irfft(Z, n=nperseg, axis=0)[:nperseg] * win.sum()
    out_len = nperseg + (nseg - 1) * nstep
    x = np.zeros(out_len)
    norm = np.zeros(out_len)
    for i in range(nseg):
        x[i * nstep:i * nstep + nperseg] += xsubs[:, i] * win
        norm[i * nstep:i * nstep + nperseg] += win ** 2
    x = x[nperseg // 2:-(nperseg // 2)]
    norm = norm[nperseg // 2:-(nperseg // 2)]
    return x / np.where(norm > 1e-10, norm, 1.0)


def process_spectral(chunks, method):
    min_samples = min(c.shape[1] for c in chunks)
    nperseg = min(1024, min_samples)
    specs = []
    for c in chunks:
        c = c[:, :min_samples]
        if c.shape[1] < 256:
            return None
        specs.append(np.array([stft(c[ch], nperseg) for ch in range(c.shape[0])]))
    specs = np.array(specs)
    mag = np.abs(specs)
    if method == "max_fft":
        comb = np.max(mag, axis=0)
    elif method == "min_fft":
        comb = np.min(mag, axis=0)
    elif method == "median_fft":
        comb = np.median(mag, axis=0)
    else:
        raise ValueError(method)
    comb = comb * np.exp(1j * np.angle(specs[0]))
    L = chunks[0].shape[1]
    out = np.zeros((comb.shape[0], L))
    for ch in range(comb.shape[0]):
        xr = istft(comb[ch], nperseg)
        if xr.shape[0] < L:
            xr = np.pad(xr, (0, L - xr.shape[0]))
        out[ch] = xr[:L]
    return out


def blend(waves, method, weights=None, buffer=32768):
    """run_ensemble's buffer loop on [n_files, ch, L] float arrays -> [ch, L] float64."""
    waves = np.asarray(waves, np.float64)
    n, ch, L = waves.shape
    if weights is not None and len(weights) == n:
        weights = np.asarray(weights, np.float32)
        weights = weights / weights.sum()
    else:
        weights = None
    out = np.zeros((ch, L))
    for pos in range(0, L, buffer):
        cs = min(buffer, L - pos)
        chunks = waves[:, :, pos:pos + cs]
        res = process_spectral(chunks, method) if method.endswith("_fft") else process_waveform(chunks, method, weights)
        if res is None:
            res = process_waveform(chunks, "avg_wave", weights)
        out[:, pos:pos + cs] = res
    return out
