"""Index model of htd_istft_wave_kernel's one-wave inverse real FFT (diagnostic, not product): the same
lane / register / LDS-slot assignments as the HIP kernel, written with numpy over the 64 lanes, checked against
numpy's irfft.  Run: python tools/istft_wave_fft_model.py

Per frame (one signal, one wave of 64 lanes, 32 complex values per lane):
  load   lane L holds X[k] for k = L + 64 u + 256 r (u < 4, r < 8): exactly stage 1's butterfly inputs
  pack   A[k] = irfft_pack(X, k) (sesa_fft2048.hpp) with X[2048 - k] read back from the wave's LDS buffer
  stage1 radix 8, s = 1:   butterfly bf = L + 64 u (p = bf), inputs A[p + 256 r] from registers
  stage2 radix 8, s = 8:   bf = L + 64 u, q = bf % 8, p = bf / 8, inputs x[bf + 256 r]
  stage3 radix 8, s = 64:  q = L, p = u, inputs x[L + 64 u + 256 r]
  stage4 radix 4, s = 512: q = L + 64 u (u < 8), inputs x[q + 512 r]; outputs z[q + 512 j] stay in registers,
         so lane L owns complex positions k = L + 64 u + 512 j -- closed under the hop (512 complex = 1024 samples)
Stockham radix-R stage (n, s, m = n / R): y[q + s (R p + j)] = w^(j p s) sum_r x[q + s (p + m r)] e^(+2 pi i r j / R)
with w = exp(+2 pi i / 2048) (inverse transform).
"""
import numpy as np

NL = 64
N = 2048


def tw(e):
    return np.exp(2j * np.pi * (e % N) / N)


def radix(xs, R):
    """xs: list of R arrays (the butterfly inputs r = 0..R-1); returns the R DFT outputs (inverse sign)."""
    return [sum(xs[r] * np.exp(2j * np.pi * r * j / R) for r in range(R)) for j in range(R)]


def wave_irfft(X):
    """X: 2049 complex bins -> 4096 real samples (unnormalised inverse real FFT, like fft2048<true> + pack)."""
    L = np.arange(NL)
    # load: per lane 32 bins k = L + 64 u + 256 r
    reg = {(u, r): X[L + 64 * u + 256 * r] for u in range(4) for r in range(8)}
    # LDS buffer: X[k] at slot k; mirror read X[2048 - k] (k = 0: slot 2048 -> the Nyquist bin, kept in a register)
    lds = np.zeros(N + 1, complex)
    for (u, r), v in reg.items():
        lds[L + 64 * u + 256 * r] = v
    lds[N] = X[N]
    twN = np.exp(-2j * np.pi * np.arange(N + 1) / 4096)
    A = {}
    for (u, r), xk in reg.items():
        k = L + 64 * u + 256 * r
        xm = np.conj(lds[N - k])
        E = 0.5 * (xk + xm)
        D = xk - xm
        O = 0.5 * D * np.conj(twN[k])
        A[(u, r)] = E + 1j * O          # (E.x - O.y, E.y + O.x)
    # stage 1 (s = 1, m = 256): bf = L + 64 u, p = bf
    buf = np.zeros(N, complex)
    for u in range(4):
        p = L + 64 * u
        ys = radix([A[(u, r)] for r in range(8)], 8)
        for j in range(8):
            buf[8 * p + j] = ys[j] * tw(j * p)
    # stage 2 (s = 8, m = 32)
    out = np.zeros(N, complex)
    for u in range(4):
        bf = L + 64 * u
        q, p = bf % 8, bf // 8
        ys = radix([buf[bf + 256 * r] for r in range(8)], 8)
        for j in range(8):
            out[q + 8 * (8 * p + j)] = ys[j] * tw(j * p * 8)
    buf = out
    # stage 3 (s = 64, m = 4): q = L, p = u
    out = np.zeros(N, complex)
    for u in range(4):
        ys = radix([buf[L + 64 * u + 256 * r] for r in range(8)], 8)
        for j in range(8):
            out[L + 64 * (8 * u + j)] = ys[j] * tw(j * u * 64)
    buf = out
    # stage 4 (radix 4, s = 512, m = 1): q = L + 64 u, u < 8; outputs in registers z[(u, j)] = z[q + 512 j]
    z = np.zeros(N, complex)
    for u in range(8):
        q = L + 64 * u
        ys = radix([buf[q + 512 * r] for r in range(4)], 4)
        for j in range(4):
            z[q + 512 * j] = ys[j]
    x = np.empty(2 * N)
    x[0::2] = z.real
    x[1::2] = z.imag
    return x


def main():
    rng = np.random.default_rng(0)
    X = rng.standard_normal(N + 1) + 1j * rng.standard_normal(N + 1)
    X[0] = X[0].real
    X[N] = 0.0
    got = wave_irfft(X)
    ref = np.fft.irfft(X, 4096) * 4096 / 2   # fft2048<true> + irfft_pack: sum without 1/N, half-spectrum packing
    err = np.abs(got - ref).max() / np.abs(ref).max()
    print(f"wave irfft vs numpy: max rel err {err:.2e}")
    assert err < 1e-12, err


if __name__ == "__main__":
    main()
